"""Data-parallel gradient exchange: one process per GPU, RCCL all-reduce over xGMI (torch
"nccl" backend on ROCm), overlapped with the backward pass.

Replaces apex.parallel.DistributedDataParallel (train_concap_struc.py:303-308).  Design for
MI355X:
* gradients live in ONE flat fp32 buffer (k3m_amd/params.py), so a bucket is a contiguous slice —
  no bucket copy in or out;
* buckets follow the real grad-ready order of the wide engine: heads / fusion / structure
  aggregator first, then each encoder block (text layer, image layer, co-attention block) as soon
  as its backward finishes, embeddings last (the word embedding also carries the tied MLM
  decoder gradient, so it is final only at the very end);
* the 86 never-grad tensors (frozen segment) are excluded — apex/torch DDP would wait on them;
* all-reduces run on a dedicated HIP stream that waits on an event recorded after the block's
  backward, so RCCL traffic overlaps the remaining backward kernels; averaging (1/world) is
  folded into the AdamW kernel's grad_scale;
* parameters are broadcast from rank 0 at start (DDP's initial sync);
* ``comm_dtype=torch.bfloat16`` (the bf16-encoder mode): each bucket is cast to a bf16 image on the comm
  stream, all-reduced in bf16 (0.85 GB instead of 1.69 GB per rank per step) and cast back into the
  fp32 gradient — the reduced-precision all-reduce of the reference's mixed-precision branches (apex DDP
  reduces the fp16 gradients, train_concap_struc.py:303-308, :397-433);
* every step records HIP events around each bucket on the comm stream plus one at the end of the
  backward on the compute stream: ``timing()`` reports the exposed all-reduce time (end of the last
  all-reduce minus end of the backward, 0 if hidden) and the comm stream's busy time, read after the
  timed region (no host sync inside the step);
* ``on_reduced`` (set by the Trainer): each block's AdamW is released from the comm stream as soon as the
  block's buckets are reduced, on the optimizer's side stream.
"""
import collections

import torch
import torch.distributed as dist

from .params import param_spec, segment_of


def _block_of(name):
    parts = name.split(".")
    if parts[0] == "encoder":
        kind = {"layer": "t", "v_layer": "v"}.get(parts[1], "c")
        return (kind, int(parts[2]))
    if parts[0] in ("embeddings", "v_embeddings"):
        return ("emb", 0)
    return ("head", 0)


class GradAllReducer(object):
    def __init__(self, fp, group=None, max_bucket_elems=32 * 1024 * 1024, comm_dtype=None):
        self.group = group
        assert comm_dtype in (None, torch.float32, torch.bfloat16)
        self.comm_dtype = None if comm_dtype == torch.float32 else comm_dtype
        self.comm = None
        self.record = True
        # per step: (backward-end event, comm-end event, [(start, end) per bucket]); the last 64 steps
        self.steps = collections.deque(maxlen=64)
        self.world = dist.get_world_size(group)
        self.fp = fp
        # contiguous ranges per readiness block
        ranges = {}
        for name, shape in fp.spec:
            if segment_of(name) == "frozen":
                continue
            blk = _block_of(name)
            o = fp.offsets[name]
            n = 1
            for s in shape:
                n *= s
            ranges.setdefault(blk, []).append((o, o + n))
        self.blocks = {}
        for blk, rs in ranges.items():
            rs.sort()
            merged = []
            for a, b in rs:
                # tensors of a block are adjacent up to 16-byte alignment padding
                if merged and a - merged[-1][1] < 4:
                    merged[-1] = (merged[-1][0], b)
                else:
                    merged.append((a, b))
            # split into buckets of at most max_bucket_elems
            out = []
            for a, b in merged:
                while b - a > max_bucket_elems:
                    out.append((a, a + max_bucket_elems))
                    a += max_bucket_elems
                out.append((a, b))
            self.blocks[blk] = out
        self.stream = None
        self.pending = []
        self.done = set()
        # on_reduced(blk): called on the comm stream right after the block's buckets are reduced (the Trainer
        # releases that block's AdamW there, overlapping the remaining backward and all-reduces)
        self.on_reduced = None

    def broadcast_params(self, fp):
        dist.broadcast(fp.data, src=0, group=self.group)
        fp.shadow_fresh = False

    def begin(self, engine):
        self.done = set()
        self.pending = []
        self.cur = []
        g = self.fp.grad
        if g.is_cuda and self.stream is None:
            self.stream = torch.cuda.Stream(device=g.device)
        if self.comm_dtype is not None and self.comm is None:
            if not g.is_cuda:
                raise RuntimeError("bf16 gradient buckets need HIP tensors (k3m_convert)")
            self.comm = torch.empty(g.numel(), dtype=self.comm_dtype, device=g.device)

    def _convert(self, src, sdt, dst, ddt, a, n):
        from . import _lib as L
        L.call("k3m_convert", src.data_ptr() + a * src.element_size(), sdt, dst.data_ptr() + a * dst.element_size(),
               ddt, n, 0, 1.0, L.stream())

    def _launch(self, blk):
        if blk in self.done or blk not in self.blocks:
            return
        self.done.add(blk)
        g = self.fp.grad
        if not g.is_cuda:
            for a, b in self.blocks[blk]:
                self.pending.append(dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
            return
        from . import _lib as L
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(g.device))
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            for a, b in self.blocks[blk]:
                t0 = torch.cuda.Event(enable_timing=True) if self.record else None
                if t0 is not None:
                    t0.record()
                if self.comm is not None:
                    n = b - a
                    self._convert(g, L.F32, self.comm, L.BF16, a, n)
                    w = dist.all_reduce(self.comm[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                    w.wait()   # orders the comm stream after the all-reduce (no host wait with RCCL)
                    self._convert(self.comm, L.BF16, g, L.F32, a, n)
                else:
                    w = dist.all_reduce(g[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
                    w.wait()
                self.pending.append(w)
                if t0 is not None:
                    t1 = torch.cuda.Event(enable_timing=True)
                    t1.record()
                    self.cur.append((t0, t1))
            if self.on_reduced is not None:
                self.on_reduced(blk)

    def grad_ready(self, kind, index):
        if kind in ("t", "v", "c"):
            self._launch(("head", 0))   # heads/fusion/struct grads are final before the encoder
            self._launch((kind, index))
        elif kind == "emb":
            self._launch(("head", 0))
            self._launch(("emb", 0))

    def finish(self):
        g = self.fp.grad
        bwd_end = None
        if g.is_cuda and self.record:
            bwd_end = torch.cuda.Event(enable_timing=True)
            bwd_end.record(torch.cuda.current_stream(g.device))
        for blk in list(self.blocks):
            self._launch(blk)
        for w in self.pending:
            w.wait()
        self.pending = []
        if g.is_cuda:
            if bwd_end is not None:
                comm_end = torch.cuda.Event(enable_timing=True)
                comm_end.record(self.stream)
                self.steps.append((bwd_end, comm_end, self.cur))
            torch.cuda.current_stream(g.device).wait_stream(self.stream)

    def timing(self, last=None):
        """{allreduce_exposed_ms, allreduce_busy_ms, buckets} averaged over the recorded steps (the last
        ``last`` ones); synchronises on the events, so call it after the timed region."""
        steps = list(self.steps)[-last:] if last else list(self.steps)
        if not steps:
            return None
        exp, busy = [], []
        for bwd_end, comm_end, cur in steps:
            comm_end.synchronize()
            exp.append(max(0.0, bwd_end.elapsed_time(comm_end)))
            busy.append(sum(a.elapsed_time(b) for a, b in cur))
        return {"allreduce_exposed_ms": sum(exp) / len(exp), "allreduce_busy_ms": sum(busy) / len(busy),
                "buckets_per_step": len(steps[-1][2]), "steps": len(steps),
                "comm_dtype": "bf16" if self.comm is not None else "fp32"}
