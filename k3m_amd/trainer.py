"""The pretraining step: forward + backward + (DDP all-reduce) + optimizer + LR schedule.

Mirrors the driver loop of train_concap_struc.py:466-589.

* Optimizer (A14).  Default: the fp32 branch (:434-448), pytorch_transformers AdamW(lr, eps=1e-8,
  betas=(0.9, 0.98)).  ``optimizer="fused_adam"``: the mixed-precision branches (:397-433), apex
  FusedAdam(bias_correction=False, betas (0.9, 0.999)); the per-group weight decay (0.01 / 0.0) of
  the parameter groups overrides FusedAdam's default 5e-4, as torch param groups do.
* Parameter groups (:352-389).  Weight decay 0.01 on every name without "bias" / "LayerNorm.bias" /
  "LayerNorm.weight".  With a pretrained model each tensor is its own group and the names of the
  BERT weight-name file run at lr x 0.1 (``lr_mult``: name -> multiplier; ``bert_lr_mult`` builds
  it with the driver's ``key[12:]`` rule).  ``frozen_names`` (``--freeze``, :243-260) are skipped.
  Tensors of equal (weight decay, multiplier) that are adjacent in the flat buffer are ONE launch.
* Schedule.  WarmupLinearSchedule stepped after the optimizer (:588), so step s runs at
  lr * lambda(s) and the first step at lr = 0.  ``lr_schedule="warmup_linear_fp16"``: the --fp16
  branch (:579-584), where only ``param_groups[0]`` is re-set to lr * warmup_linear(step / t_total,
  warmup_proportion) and every other group keeps the 0 that WarmupLinearSchedule's constructor
  assigned (reproduced as the reference runs; not the default).
* Gradient accumulation (:561-575): each micro-step back-propagates loss / accum_steps; the
  optimizer (and the DDP all-reduce) run on every accum_steps-th call.
* ``objective == 1`` label rewrite (:481-494) before the forward.
* loss = mlm_t + img * loss_img_weight + mlm_pv + lpm (:531-533), the optimised objective.
* NaN fail-fast: every step's loss is copied to pinned host memory behind an event and
  checked a step later, without a host synchronisation; a non-finite loss raises FloatingPointError.
"""
import collections
import math
import os

import torch

from . import _lib as L
from .engine import K3MEngine
from .params import param_spec, segment_of


def warmup_linear_lambda(step, warmup, t_total):
    """pytorch_transformers 1.1.0 WarmupLinearSchedule.lr_lambda."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(t_total - step) / float(max(1.0, t_total - warmup)))


def warmup_linear_fp16(x, warmup=0.002):
    """train_concap_struc.py:60-65 (the --fp16 branch's manual schedule, x = step / t_total)."""
    if x < warmup:
        return x / warmup
    return max((x - 1.) / (warmup - 1.), 0)


def bert_lr_mult(names, bert_weight_names, ddp=True, mult=0.1):
    """lr multipliers of the pretrained-model parameter groups (train_concap_struc.py:369-375): a
    parameter whose driver-side name ``key`` has ``key[12:]`` in the weight-name list runs at
    lr * 0.1.  Under (apex) DDP ``key`` is ``"module." + name``."""
    want = set(bert_weight_names)
    out = {}
    for n in names:
        key = ("module." + n) if ddp else n
        if key[12:] in want:
            out[n] = mult
    return out


def objective1_labels(batch):
    """objective == 1 (train_concap_struc.py:481-494): items whose text / PV / image were replaced
    (is_next + is_next_pv_v + is_next_pv_t != 0) lose their masked-LM and region labels; the rewrite
    multiplies by the keep flag and maps every 0 to -1 (a label id 0 too, as the reference)."""
    keep = ((batch["is_next"] + batch["is_next_pv_v"] + batch["is_next_pv_t"]) == 0).long().unsqueeze(1)
    out = dict(batch)
    for k in ("image_label", "lm_label_ids", "lm_label_ids_pv"):
        v = batch[k] * keep
        out[k] = torch.where(v == 0, torch.full_like(v, -1), v)
    out.pop("_label_counts", None)
    return out


def init_reference(fp, cfg, seed):
    """BertPreTrainedModel.init_weights (vilbert_k3m.py:1940-1951) on the device: N(0, 0.02) for
    Linear / Embedding weights, zero biases, LayerNorm weight 1 / bias 0."""
    g = torch.Generator(device=fp.device).manual_seed(int(seed))
    std = getattr(cfg, "initializer_range", 0.02)
    for name, _ in param_spec(cfg):
        t = fp.p[name]
        if "LayerNorm" in name:
            t.fill_(1.0 if name.endswith(".weight") else 0.0)
        elif name.endswith(".bias"):
            t.zero_()
        else:
            t.normal_(0.0, std, generator=g)
    fp.shadow_fresh = False


def optimizer_runs(fp, weight_decay=0.01, lr_mult=None, frozen_names=()):
    """[(offset, length, wd, lr_mult)] over the flat buffer: maximal runs of adjacent optimised
    tensors with equal (weight decay, multiplier).  Lengths are rounded up to 4 floats (16 B): the
    alignment padding between tensors is zero in p, g, m and v and stays zero under the update."""
    lr_mult = lr_mult or {}
    frozen_names = set(frozen_names)
    items = []
    for name, shape in fp.spec:
        seg = segment_of(name)
        if seg == "frozen" or name in frozen_names:
            continue
        o = fp.offsets[name]
        n = math.prod(shape)
        items.append((o, o + n, weight_decay if seg == "decay" else 0.0, float(lr_mult.get(name, 1.0))))
    items.sort()
    runs = []
    for a, b, wd, mu in items:
        if runs and runs[-1][2] == wd and runs[-1][3] == mu and a - runs[-1][1] < 4:
            runs[-1][1] = b
        else:
            runs.append([a, b, wd, mu])
    return [(a, (b - a + 3) // 4 * 4, wd, mu) for a, b, wd, mu in runs]


def block_runs(fp, weight_decay=0.01, lr_mult=None, frozen_names=()):
    """optimizer_runs() cut at the gradient-readiness blocks of the wide engine (k3m_amd.ddp._block_of:
    heads / fusion / structure, each encoder block, the embeddings): {block: [(offset, length, wd, lr_mult)]},
    so that a block's AdamW can run as soon as the backward has finished that block."""
    from .ddp import _block_of
    lr_mult = lr_mult or {}
    frozen_names = set(frozen_names)
    per = {}
    for name, shape in fp.spec:
        if segment_of(name) == "frozen" or name in frozen_names:
            continue
        o = fp.offsets[name]
        per.setdefault(_block_of(name), []).append(
            (o, o + math.prod(shape), weight_decay if segment_of(name) == "decay" else 0.0, float(lr_mult.get(name, 1.0))))
    out = {}
    for blk, items in per.items():
        items.sort()
        runs = []
        for a, b, wd, mu in items:
            if runs and runs[-1][2] == wd and runs[-1][3] == mu and a - runs[-1][1] < 4:
                runs[-1][1] = b
            else:
                runs.append([a, b, wd, mu])
        out[blk] = [(a, (b - a + 3) // 4 * 4, wd, mu) for a, b, wd, mu in runs]
    return out


# AdamW of each gradient block on a side stream as soon as the backward has finished that block (single
# process) or the block's gradient buckets are all-reduced (DDP), on the last micro-step: the HBM-bound sweep
# overlaps the rest of the backward instead of following it.  K3M_OPT_OVERLAP=0 restores the one sweep.
OPT_OVERLAP = os.environ.get("K3M_OPT_OVERLAP", "1") != "0"
# Replay a repeated step as one hipGraph (k3m_amd/graph.py): "auto" (default) when the eager step's host issue
# time is a large share of its GPU time, "1" always, "0" never (every launch issued from Python).
_g = os.environ.get("K3M_GRAPH", "auto")
GRAPH_STEP = "auto" if _g == "auto" else _g != "0"


class LossWatch(object):
    """Asynchronous NaN / inf fail-fast: the loss of each step is copied into pinned host memory
    behind an event; the copy is inspected once the event has completed (a later step), so the
    check never stalls the launch queue.  ``flush()`` (a sync) checks everything outstanding."""

    def __init__(self, lag=2):
        self.pending = collections.deque()
        self.lag = lag

    def push(self, step, loss):
        if not loss.is_cuda:
            v = float(loss.reshape(-1)[0])
            if not math.isfinite(v):
                raise FloatingPointError("non-finite loss %r at step %d" % (v, step))
            return
        host = torch.empty((1,), dtype=torch.float32, pin_memory=True)
        host.copy_(loss.detach().reshape(-1)[:1], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.pending.append((step, host, ev))
        self.poll()

    def poll(self, force=False):
        while self.pending and (force or len(self.pending) > self.lag or self.pending[0][2].query()):
            step, host, ev = self.pending.popleft()
            ev.synchronize()
            v = float(host[0])
            if not math.isfinite(v):
                self.pending.clear()
                raise FloatingPointError("non-finite loss %r at step %d (fail-fast, SURVEY §5)" % (v, step))

    def flush(self):
        self.poll(force=True)


def fp_is_cuda(eng):
    return eng.fp.data.is_cuda


class Trainer(object):
    ADAMW = None   # None: k3m_adamw_ex (pytorch_transformers AdamW / apex FusedAdam); else a legacy entry point

    def __init__(self, cfg, device, lr=1e-4, warmup_steps=0, total_steps=10000, seed=1234, ddp=None,
                 loss_img_weight=1.0, beta1=0.9, beta2=None, eps=1e-8, weight_decay=0.01, init=True, dtype="fp32",
                 optimizer="adamw", lr_schedule="warmup_linear", warmup_proportion=None, accum_steps=1,
                 lr_mult=None, frozen_names=(), objective=2, nan_check=True):
        assert optimizer in ("adamw", "fused_adam")
        assert lr_schedule in ("warmup_linear", "warmup_linear_fp16")
        self.engine = K3MEngine(cfg, device, seed=seed, dtype=dtype)
        fp = self.engine.fp
        if init:
            init_reference(fp, cfg, seed)
        if ddp is not None:
            ddp.broadcast_params(fp)
        self.ddp = ddp
        self.lr, self.warmup, self.t_total = lr, warmup_steps, total_steps
        self.warmup_proportion = (warmup_proportion if warmup_proportion is not None
                                  else float(warmup_steps) / max(1, total_steps))
        self.optimizer, self.lr_schedule = optimizer, lr_schedule
        if beta2 is None:   # pytorch_transformers AdamW (0.9, 0.98) as passed by the driver; FusedAdam default
            beta2 = 0.98 if optimizer == "adamw" else 0.999
        self.beta1, self.beta2, self.eps, self.wd = beta1, beta2, eps, weight_decay
        self.loss_img_weight = loss_img_weight
        self.accum_steps = int(accum_steps)
        assert self.accum_steps >= 1
        self.objective = objective
        self.global_step = 0
        self.micro = 0
        if lr_schedule == "warmup_linear_fp16" and lr_mult:
            raise NotImplementedError("the --fp16 schedule quirk is defined for the two-group optimizer only")
        self.runs = optimizer_runs(fp, weight_decay, lr_mult, frozen_names)
        # the reference's parameter-group layout (checkpoint interchange): per-tensor groups when a
        # pretrained model is loaded (lr_mult given, possibly empty), else the two AdamW groups
        self.lr_mult = dict(lr_mult) if lr_mult is not None else None
        self.frozen_names = tuple(frozen_names)
        self.excluded = sorted(set(frozen_names))
        nopt = max(a + n for a, n, _, _ in self.runs)
        assert nopt <= fp.segments["frozen"][0] + 4
        self.m = torch.zeros(nopt, dtype=torch.float32, device=fp.device)
        self.v = torch.zeros(nopt, dtype=torch.float32, device=fp.device)
        self.watch = LossWatch() if nan_check else None
        self.dropout = True   # False: the step runs without dropout (model.eval() forward; parity runs)
        self.block_runs = block_runs(fp, weight_decay, lr_mult, frozen_names)
        self.opt_stream = None
        self.overlap = OPT_OVERLAP
        self.graph = GRAPH_STEP
        self._graphs = None
        self._adam_table = None   # set while a hipGraph captures the step (k3m_amd/graph.py)

    def evaluate(self, batch, noise=None, ent_neg=None, val_neg=None):
        """The validation forward of train_concap_struc.py:612-688 (model.eval(), no gradients): returns
        the losses dict with ``loss`` = mlm_t + img * loss_img_weight + mlm_pv + lpm (:656-657)."""
        out, _ = self.engine.forward(batch, train=False, noise=noise, ent_neg=ent_neg, val_neg=val_neg,
                                     seed=self.global_step * self.accum_steps + self.micro)
        out["loss"] = out["masked_lm_loss"] + out["masked_lm_loss_pv"] + out["loss_lpm"] + \
            out["masked_img_loss"] * self.loss_img_weight
        return out

    # ---------------------------------------------------------------- schedule
    def current_lr(self):
        """lr of the next optimizer step for a multiplier-1 tensor of the first group."""
        if self.lr_schedule == "warmup_linear_fp16" and self.global_step > 0:
            return self.lr * warmup_linear_fp16(self.global_step / self.t_total, self.warmup_proportion)
        # LambdaLR: the constructor sets lr * lambda(0); scheduler.step() after each optimizer step
        return self.lr * warmup_linear_lambda(self.global_step, self.warmup, self.t_total)

    def run_lr(self, off, mult):
        """lr of the run starting at flat offset ``off``.  Under the --fp16 schedule only
        ``param_groups[0]`` — the decay group, i.e. the flat buffer's decay segment — is re-set
        (:584); every other group keeps lr * lambda(0) (two-group layout only, see __init__)."""
        if self.lr_schedule == "warmup_linear_fp16" and off >= self.engine.fp.segments["no_decay"][0]:
            return mult * self.lr * warmup_linear_lambda(0, self.warmup, self.t_total)
        return mult * self.current_lr()

    # ---------------------------------------------------------------- optimizer
    def _adamw(self, off, n, wd, mult, step, grad_scale, flags):
        """k3m_adamw_ex over one run; inside a hipGraph capture k3m_adamw_ex_dev with the run's row of the
        graph's scalar table (k3m_amd/graph.py refills it before each replay)."""
        fp = self.engine.fp
        # with a bf16 encoder the same launch refreshes the weight shadow from the new fp32 values
        sh = fp.data16[off:].data_ptr() if fp.data16 is not None else None
        if self._adam_table is not None:
            row = self._adam_table.row(mult, wd, flags)   # lr = mult * current_lr(): warmup_linear only
            L.call("k3m_adamw_ex_dev", fp.data[off:].data_ptr(), fp.grad[off:].data_ptr(), self.m[off:].data_ptr(),
                   self.v[off:].data_ptr(), sh, n, row, self.beta1, self.beta2, self.eps, grad_scale, flags, L.stream())
            return
        L.call("k3m_adamw_ex", fp.data[off:].data_ptr(), fp.grad[off:].data_ptr(), self.m[off:].data_ptr(),
               self.v[off:].data_ptr(), sh, n, self.run_lr(off, mult), self.beta1, self.beta2, self.eps, wd, step,
               grad_scale, flags, L.stream())

    def _adam_runs(self, runs, step, grad_scale, flags):
        for off, n, wd, mult in runs:
            if n:
                self._adamw(off, n, wd, mult, step, grad_scale, flags)

    def _overlap_begin(self, grad_scale=1.0):
        """State of an overlapped optimizer step: blocks still to update and the side stream."""
        dev = self.engine.fp.device
        if self.opt_stream is None:
            self.opt_stream = torch.cuda.Stream(device=dev)
        self._pending = set(self.block_runs)
        self._flags = L.ADAM_ZERO_GRAD | (L.ADAM_APEX if self.optimizer == "fused_adam" else 0)
        self._grad_scale = grad_scale

    def _overlap_block(self, blk):
        """The block's AdamW on the side stream, after everything issued so far on the CURRENT stream (the
        compute stream at a backward hand-off; the comm stream after the block's all-reduce under DDP)."""
        if blk not in self._pending:
            return
        self._pending.discard(blk)
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.opt_stream):
            self.opt_stream.wait_event(ev)
            self._adam_runs(self.block_runs[blk], self.global_step + 1, self._grad_scale, self._flags)

    def _overlap_hook(self, kind, index):
        # the heads / fusion / structure gradients are final before the first encoder block's (ddp.grad_ready)
        self._overlap_block(("head", 0))
        self._overlap_block((kind, index))

    def _overlap_finish(self, count=True):
        fp = self.engine.fp
        fresh = fp.shadow_fresh
        for blk in sorted(self._pending):
            self._overlap_block(blk)
        torch.cuda.current_stream(fp.device).wait_stream(self.opt_stream)
        for name in self.excluded:   # --freeze: gradients the optimizer skips are dropped as well
            fp.g[name].zero_()
        fp.shadow_fresh = fresh
        if count:
            self.global_step += 1

    def optimizer_step(self, grad_scale=1.0, zero_grad=True, count=True):
        """One optimizer step over every run; the gradient buffer is zeroed in the same sweep.
        count=False (a graph capture): the step counter is left to the replay."""
        fp = self.engine.fp
        step = self.global_step + 1
        fresh = fp.shadow_fresh
        flags = (L.ADAM_ZERO_GRAD if zero_grad else 0) | (L.ADAM_APEX if self.optimizer == "fused_adam" else 0)
        for off, n, wd, mult in self.runs:
            if n == 0:
                continue
            if self.ADAMW is not None:   # torch.optim.AdamW (fine-tuning); zeroing below
                sh = fp.data16[off:].data_ptr() if fp.data16 is not None else None
                L.call(self.ADAMW, fp.data[off:].data_ptr(), fp.grad[off:].data_ptr(), self.m[off:].data_ptr(),
                       self.v[off:].data_ptr(), sh, n, self.run_lr(off, mult), self.beta1, self.beta2, self.eps, wd,
                       step, grad_scale, L.stream())
                continue
            self._adamw(off, n, wd, mult, step, grad_scale, flags)
        if zero_grad and self.ADAMW is not None:
            fp.grad.zero_()
        elif zero_grad:
            for name in self.excluded:   # --freeze: gradients the optimizer skips are dropped as well
                fp.g[name].zero_()
        fp.shadow_fresh = fresh   # frozen tensors are not updated: the shadow stays as fresh as it was
        if count:
            self.global_step += 1

    def finish(self):
        """Synchronising end-of-run (or end-of-epoch) checks: every outstanding label-count hint and
        every outstanding loss fail-fast check."""
        self.engine.check_hints(wait=True)
        if self.watch is not None:
            self.watch.flush()

    # ---------------------------------------------------------------- checkpoints
    def save_checkpoint(self, tar_path=None, bin_path=None):
        """The reference driver's .tar / .bin files (train_concap_struc.py:691-705; k3m_amd/checkpoint.py)."""
        from .checkpoint import save_checkpoint
        save_checkpoint(self, tar_path=tar_path, bin_path=bin_path)

    def load_checkpoint(self, tar_path):
        """Resume from a reference-layout .tar (train_concap_struc.py:277-293)."""
        from .checkpoint import load_checkpoint
        return load_checkpoint(self, tar_path)

    # ---------------------------------------------------------------- the step
    def step(self, batch, noise=None, ent_neg=None, val_neg=None):
        """One micro-step (forward + backward); the optimizer runs every ``accum_steps`` calls.
        Returns the forward's outputs; ``out["loss"]`` is the optimised objective.

        With ``self.graph`` (K3M_GRAPH: True, or "auto" = when the step is host-bound) a step that a hipGraph can
        replay (k3m_amd/graph.py: one process, no accumulation, host label counts, the default schedule) runs as
        one graph launch once the same batch shapes repeat; its outputs are then the graph's static tensors,
        overwritten by the next replay."""
        if self.graph and noise is None and ent_neg is None and val_neg is None:
            if self._graphs is None:
                from .graph import StepGraphs
                self._graphs = StepGraphs(self)
            out = self._graphs.step(batch)
            if out is not None:
                return out
        return self._eager_step(batch, noise, ent_neg, val_neg)

    def _device_step(self, batch):
        """The device work of one optimizer step (forward, backward, AdamW) with no host-side bookkeeping:
        the body a hipGraph captures.  Preconditions: single process, accum_steps == 1, a label-count hint."""
        eng = self.engine
        if self.objective == 1:
            batch = objective1_labels(batch)
        out, ctx = eng.forward(batch, train=self.dropout, seed=self.global_step)
        out["loss"] = out["masked_lm_loss"] + out["masked_lm_loss_pv"] + out["loss_lpm"] + \
            out["masked_img_loss"] * self.loss_img_weight
        hook = None
        if self.overlap:
            self._overlap_begin()
            hook = self._overlap_hook
        eng.backward(ctx, w_mlm=1.0, w_img=self.loss_img_weight, w_lpm=1.0, grad_ready=hook)
        if self.overlap:
            self._overlap_finish(count=False)
        else:
            self.optimizer_step(count=False)
        return out

    def _eager_step(self, batch, noise=None, ent_neg=None, val_neg=None):
        eng = self.engine
        if self.objective == 1:
            batch = objective1_labels(batch)
        out, ctx = eng.forward(batch, train=self.dropout, noise=noise, ent_neg=ent_neg, val_neg=val_neg,
                               seed=self.global_step * self.accum_steps + self.micro)
        w = 1.0 / self.accum_steps
        out["loss"] = out["masked_lm_loss"] + out["masked_lm_loss_pv"] + out["loss_lpm"] + \
            out["masked_img_loss"] * self.loss_img_weight
        last = self.micro + 1 == self.accum_steps
        sync = self.ddp is not None and last
        overlap = self.overlap and last and self.ADAMW is None and fp_is_cuda(eng)
        hook = None
        if sync:
            self.ddp.begin(eng)
            hook = self.ddp.grad_ready
            if overlap:   # each block's AdamW (1/world folded in) as soon as its buckets are reduced
                eng.check_hints()
                self._overlap_begin(grad_scale=1.0 / self.ddp.world)
                self.ddp.on_reduced = self._overlap_block
        elif overlap:
            eng.check_hints()   # a completed label-count check that failed raises before any update
            self._overlap_begin()
            hook = self._overlap_hook
        eng.backward(ctx, w_mlm=w, w_img=self.loss_img_weight * w, w_lpm=w, grad_ready=hook)
        if self.watch is not None:
            self.watch.push(self.global_step, out["loss"])
        self.micro += 1
        if last:
            if overlap:
                if sync:
                    self.ddp.finish()
                    self.ddp.on_reduced = None
                self._overlap_finish()
            else:
                eng.check_hints()   # a completed label-count check that failed raises before the update
                scale = 1.0
                if sync:
                    self.ddp.finish()
                    scale = 1.0 / self.ddp.world
                self.optimizer_step(grad_scale=scale)
            self.micro = 0
            eng.step_count += 1
        return out
