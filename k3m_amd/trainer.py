"""The pretraining step: forward + backward + (DDP all-reduce) + AdamW + WarmupLinearSchedule.

Mirrors the driver loop of train_concap_struc.py:466-589 with the fp32 optimizer branch
(:434-448): pytorch_transformers AdamW(lr, eps=1e-8, betas=(0.9, 0.98)), weight decay 0.01 on
every parameter except names containing "bias"/"LayerNorm.bias"/"LayerNorm.weight" (:352-367),
WarmupLinearSchedule stepped after the optimizer (:588) so step s runs at lr * lambda(s) and the
first step at lr = 0.  loss = mlm_t + img * loss_img_weight + mlm_pv + lpm (:531-533).
"""
import math

import torch

from . import _lib as L
from .engine import K3MEngine
from .params import param_spec


def warmup_linear_lambda(step, warmup, t_total):
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(t_total - step) / float(max(1.0, t_total - warmup)))


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


class Trainer(object):
    ADAMW = "k3m_adamw"   # pytorch_transformers AdamW (train_concap_struc.py:436-441)

    def __init__(self, cfg, device, lr=1e-4, warmup_steps=0, total_steps=10000, seed=1234, ddp=None,
                 loss_img_weight=1.0, beta1=0.9, beta2=0.98, eps=1e-8, weight_decay=0.01, init=True, dtype="fp32"):
        self.engine = K3MEngine(cfg, device, seed=seed, dtype=dtype)
        fp = self.engine.fp
        if init:
            init_reference(fp, cfg, seed)
        if ddp is not None:
            ddp.broadcast_params(fp)
        self.ddp = ddp
        self.lr, self.warmup, self.t_total = lr, warmup_steps, total_steps
        self.beta1, self.beta2, self.eps, self.wd = beta1, beta2, eps, weight_decay
        self.loss_img_weight = loss_img_weight
        self.global_step = 0
        d0, d1 = fp.segments["decay"]
        n0, n1 = fp.segments["no_decay"]
        # segment lengths rounded up to 16 B: the padding between tensors is zero in p, g, m and v
        self.segs = [(d0, (d1 - d0 + 3) // 4 * 4, weight_decay), (n0, (n1 - n0 + 3) // 4 * 4, 0.0)]
        nopt = n0 + self.segs[1][1]
        assert nopt <= fp.segments["frozen"][0]
        self.m = torch.zeros(nopt, dtype=torch.float32, device=fp.device)
        self.v = torch.zeros(nopt, dtype=torch.float32, device=fp.device)

    def current_lr(self):
        return self.lr * warmup_linear_lambda(self.global_step, self.warmup, self.t_total)

    def optimizer_step(self, grad_scale=1.0):
        fp = self.engine.fp
        lr = self.current_lr()
        step = self.global_step + 1
        fresh = fp.shadow_fresh
        for off, n, wd in self.segs:
            if n == 0:
                continue
            # with a bf16 encoder the same launch refreshes the weight shadow from the new fp32 values
            sh = fp.data16[off:].data_ptr() if fp.data16 is not None else None
            L.call(self.ADAMW, fp.data[off:].data_ptr(), fp.grad[off:].data_ptr(), self.m[off:].data_ptr(),
                   self.v[off:].data_ptr(), sh, n, lr, self.beta1, self.beta2, self.eps, wd, step, grad_scale,
                   L.stream())
        fp.shadow_fresh = fresh   # frozen tensors are not updated: the shadow stays as fresh as it was
        fp.grad.zero_()
        self.global_step += 1

    def save_checkpoint(self, tar_path=None, bin_path=None):
        """The reference driver's .tar / .bin files (train_concap_struc.py:691-705; k3m_amd/checkpoint.py)."""
        from .checkpoint import save_checkpoint
        save_checkpoint(self, tar_path=tar_path, bin_path=bin_path)

    def load_checkpoint(self, tar_path):
        """Resume from a reference-layout .tar (train_concap_struc.py:277-293)."""
        from .checkpoint import load_checkpoint
        return load_checkpoint(self, tar_path)

    def step(self, batch, noise=None, ent_neg=None, val_neg=None):
        eng = self.engine
        out, ctx = eng.forward(batch, train=True, noise=noise, ent_neg=ent_neg, val_neg=val_neg,
                               seed=self.global_step)
        hook = self.ddp.grad_ready if self.ddp is not None else None
        if self.ddp is not None:
            self.ddp.begin(eng)
        eng.backward(ctx, w_mlm=1.0, w_img=self.loss_img_weight, w_lpm=1.0, grad_ready=hook)
        scale = 1.0
        if self.ddp is not None:
            self.ddp.finish()
            scale = 1.0 / self.ddp.world
        self.optimizer_step(grad_scale=scale)
        eng.step_count += 1
        return out
