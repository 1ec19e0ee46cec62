"""Whole-step hipGraph replay of Trainer.step (VERDICT r3 "take the host off the critical path").

The eager step issues ~950 launches from Python (engine ops, ctypes calls, torch allocations): about as
long on the host as the bf16 step takes on the GPU.  A step whose shapes repeat is captured ONCE into a
hipGraph (torch.cuda.CUDAGraph over the same launches: forward, backward, the per-block AdamW on its side
stream) and then replayed with one launch.

What changes between replays without re-capture:
* the batch: copied into the graph's static input tensors;
* the dropout / gumbel / negative-sampling seed: the captured launches carry the K3M_GRAPH_SEED marker and
  read the step's seed from the device word whose address they carry, refilled before each replay with
  the value the eager step would pass (K3MEngine.step_seed);
* the AdamW scalars (schedule lr, bias corrections): captured as k3m_adamw_ex_dev launches reading one
  row per run of a device table, refilled before each replay by k3m_adamw_scalars_n with exactly the
  fp32 values k3m_adamw_ex computes for (mult * lr(step), wd, step).
Host-side bookkeeping (step counters, NaN fail-fast, the label-count check) runs around each replay.

Eligible: one process (no DDP all-reduce), accum_steps == 1, the label-count hint present (no host sync
inside the step), the default warmup_linear schedule, the pretraining objective 2, the built-in AdamW.
A step is captured when the same key (batch shapes, dtypes, label counts, dropout / overlap mode) came
twice in a row; one graph is kept (a new key frees the old one), so a loader whose label counts change
every batch simply stays eager.  A replayed step returns copies of its small outputs (the loss and the
per-task losses), which outlive the next replay; larger outputs (logit-sized tensors) are the graph's static
tensors, overwritten by the next replay (clone what must outlive it).  A capture that fails (an op that
cannot be captured, a host sync on an untested path) is dropped with a warning and that key runs eagerly.
"""
import gc
import warnings

import numpy as np
import torch

from . import _lib as L


def _key(tr, batch):
    from . import ops
    parts = []
    for k in sorted(batch):
        v = batch[k]
        if torch.is_tensor(v):
            parts.append((k, tuple(v.shape), str(v.dtype), v.device.index))
        elif k == "_label_counts":
            parts.append((k, tuple(int(x) for x in v)))
    # the deterministic mode picks different backward kernels (ops.embed_bwd & co.): a graph captured in one mode
    # must not be replayed in the other (ops.set_deterministic can flip it at run time)
    return tuple(parts) + (tr.dropout, tr.overlap, tr.optimizer, bool(ops.DETERMINISTIC))


class AdamTable(object):
    """Device rows of (step_size, decay, 1/bc1, 1/bc2), one per captured AdamW launch, and the host side
    that refills them per replay (a small ring of pinned staging buffers, reused once its copy is done)."""

    RING = 3

    def __init__(self, device, rows=256):
        self.device = device
        self.mult, self.wd, self.flags = [], [], None
        self.dev = torch.zeros((max(int(rows), 1), 4), dtype=torch.float32, device=device)   # rows 16-B aligned
        self.host = None

    def row(self, mult, wd, flags):
        if self.flags is None:
            self.flags = flags
        assert (flags & ~L.ADAM_ZERO_GRAD) == (self.flags & ~L.ADAM_ZERO_GRAD), "one AdamW variant per graph"
        i = len(self.mult)
        if i == self.dev.shape[0]:
            raise RuntimeError("more than %d AdamW launches in one captured step" % i)
        self.mult.append(float(mult))
        self.wd.append(float(wd))
        return self.dev[i].data_ptr()

    def finalize(self):
        n = len(self.mult)
        self.mult_np = np.asarray(self.mult, dtype=np.float64)
        self.wd_np = np.ascontiguousarray(np.asarray(self.wd, dtype=np.float64))
        self.host = [torch.empty((max(n, 1), 4), dtype=torch.float32, pin_memory=True) for _ in range(self.RING)]
        self.events = [None] * self.RING
        self.slot = 0

    def upload(self, lr, step, beta1, beta2):
        n = len(self.mult)
        if n == 0:
            return
        s = self.slot
        self.slot = (s + 1) % self.RING
        if self.events[s] is not None:
            self.events[s].synchronize()   # the copy that last read this staging buffer is done
        lr_np = np.ascontiguousarray(self.mult_np * float(lr))   # the same double products run_lr forms
        h = self.host[s]
        L.call("k3m_adamw_scalars_n", n, lr_np.ctypes.data, self.wd_np.ctypes.data, beta1, beta2, int(step),
               int(self.flags), h.data_ptr())
        self.dev[:n].copy_(h[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[s] = ev


class StepGraph(object):
    """One captured step: static inputs, the graph, its outputs and the per-replay device scalars."""

    SMALL = 4096   # outputs up to this many elements are returned as copies (loss terms, counters)

    def __init__(self, tr, batch):
        eng = tr.engine
        dev = eng.fp.device
        self.tr = tr
        self.hint = tuple(int(x) for x in batch["_label_counts"])
        self.static = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in batch.items()}
        self.seed = torch.zeros((1,), dtype=torch.int64, device=dev)   # the step's seed word (outside the pool)
        # one row per AdamW launch the step can issue: the sweep's runs or the per-block runs of the overlap
        rows = max(len(tr.runs), sum(len(r) for r in getattr(tr, "block_runs", {}).values()))
        self.table = AdamTable(dev, rows)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        eng.graph_seed = self.seed.data_ptr()
        eng.capturing = True
        tr._adam_table = self.table
        # no automatic garbage collection while the stream captures: a collected cycle holding a HIP object (an
        # event of an earlier trainer, a stream) would run its destructor mid-capture, where HIP refuses the call
        # and the C++ destructor aborts the process (seen once in the full GPU suite, test_gpu_graph)
        gc.collect()
        gc_was = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode="relaxed"):
                self.out = tr._device_step(self.static)
        finally:
            if gc_was:
                gc.enable()
            eng.graph_seed = 0
            eng.capturing = False
            tr._adam_table = None
        self.counts = eng.captured_counts
        eng.captured_counts = None
        self.table.finalize()

    def replay(self, batch):
        tr, eng = self.tr, self.tr.engine
        for k, v in batch.items():
            if torch.is_tensor(v):
                dst = self.static[k]
                if v is not dst:
                    dst.copy_(v, non_blocking=True)
        eng.fp.refresh_shadow()   # a checkpoint load marks the bf16 shadow stale; the graph does not refresh it
        self.seed.fill_(eng.step_seed(tr.global_step))
        self.table.upload(tr.current_lr(), tr.global_step + 1, tr.beta1, tr.beta2)
        self.graph.replay()
        if self.counts is not None:
            eng._verify_hint(self.hint, self.counts)
        out = {k: (v.clone() if torch.is_tensor(v) and v.numel() <= self.SMALL else v) for k, v in self.out.items()}
        if tr.watch is not None:
            tr.watch.push(tr.global_step, out["loss"])
        tr.global_step += 1
        eng.step_count += 1
        return out


class StepGraphs(object):
    """Trainer.step's graph policy.  A key (batch shapes, label counts, modes) seen for the first time runs
    eagerly.  tr.graph True: the second consecutive sighting captures.  tr.graph "auto": the second sighting
    runs eagerly (from an idle queue) with HIP events around it, and the third decides — capture when the host
    needed more than HOST_SHARE of the step's GPU time to issue it (the step is launch-bound), else stay eager
    for that key: a replay costs 1.5-2 % more GPU time than the same launches queued from Python ahead of the
    GPU (replayed kernel nodes start later; profiles/r4b_ab_graph.txt), so it pays only when the host is the
    bottleneck.  One graph kept."""

    HOST_SHARE = 0.95

    def __init__(self, tr):
        self.tr = tr
        self.graph = None
        self.graph_key = None
        self.last_key = None
        self.decided = {}
        self.timing = None
        self.captures = 0
        self.replays = 0
        self.last_decision = None

    def eligible(self, batch):
        tr = self.tr
        return (tr.ddp is None and tr.accum_steps == 1 and tr.micro == 0 and tr.ADAMW is None
                and tr.lr_schedule == "warmup_linear" and tr.objective != 1 and batch.get("_label_counts") is not None
                and tr.engine.fp.data.is_cuda)

    def _capture(self, batch, key):
        self.tr.engine.check_hints()   # a completed label-count check that failed raises before any update
        self.graph = None              # one graph: free the previous one's pool first
        torch.cuda.empty_cache()
        try:
            g = StepGraph(self.tr, batch)
        except Exception as e:   # noqa: BLE001 - any capture failure falls back to the eager step
            # nothing captured ran on the device and the capture body changes no host counters (count=False),
            # so the eager step below is the step this call would have been
            self.tr.engine.captured_counts = None
            torch.cuda.synchronize()
            self.decided[key] = "eager"
            self.last_decision = {"mode": "eager", "capture_failed": "%s: %s" % (type(e).__name__, e)}
            warnings.warn("k3m: hipGraph capture of the step failed (%s: %s); this batch shape runs eagerly"
                          % (type(e).__name__, e))
            return None
        self.graph = g
        self.graph_key = key
        self.captures += 1
        self.replays += 1
        return self.graph.replay(batch)

    def _timed_eager(self, batch, key):
        import time
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()   # from an idle queue: a full launch queue would block the host and inflate host_ms
        e0.record()
        h0 = time.perf_counter()
        out = self.tr._eager_step(batch)
        host_ms = 1e3 * (time.perf_counter() - h0)
        e1.record()
        self.timing = (key, host_ms, e0, e1)
        return out

    def step(self, batch):
        """The step's outputs when this policy ran it (replayed, captured or timed), None for a plain eager step."""
        from . import debug
        if debug.ON or not self.eligible(batch):
            return None   # debug mode checks indices and synchronises per call: eager only
        key = _key(self.tr, batch)
        if self.graph is not None and key == self.graph_key:
            self.replays += 1
            return self.graph.replay(batch)
        dec = self.decided.get(key)
        if dec == "eager":
            return None
        seen, self.last_key = self.last_key, key
        if key != seen:
            return None   # first sighting: eager (lazy first-use initialisations happen outside any capture)
        if self.tr.graph is True or dec == "graph":
            return self._capture(batch, key)
        if self.timing is None or self.timing[0] != key:
            return self._timed_eager(batch, key)
        _, host_ms, e0, e1 = self.timing
        self.timing = None
        e1.synchronize()
        gpu_ms = e0.elapsed_time(e1)
        graph = host_ms > self.HOST_SHARE * gpu_ms
        self.decided[key] = "graph" if graph else "eager"
        self.last_decision = {"host_issue_ms": round(host_ms, 3), "gpu_ms": round(gpu_ms, 3),
                              "mode": "graph" if graph else "eager"}
        return self._capture(batch, key) if graph else None
