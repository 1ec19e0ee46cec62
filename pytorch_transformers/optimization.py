"""``pytorch_transformers.optimization`` (1.1.0 API) for the offline build: ``AdamW`` and the LambdaLR
schedules the reference driver uses (train_concap_struc.py:23, :436-448).

``AdamW.step()`` runs the HIP kernel ``k3m_adamw`` (include/k3m_hip.h; the same update as
k3m_amd.trainer's fused launches) once per parameter tensor, with the published 1.1.0 semantics:
m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; p -= lr sqrt(1-b2^t)/(1-b1^t) m/(sqrt(v)+eps); then
p -= lr wd p.  There is no CPU path: parameters must be HIP (cuda) fp32 tensors, otherwise step()
raises.  For the whole-model step use ``k3m_amd.trainer.Trainer`` (one launch per segment).
"""
import math

import torch
from torch.optim.lr_scheduler import LambdaLR


class AdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0, correct_bias=True):
        if lr < 0.0:
            raise ValueError("Invalid learning rate: {} - should be >= 0.0".format(lr))
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameter: {}".format(betas))
        if not 0.0 <= eps:
            raise ValueError("Invalid epsilon value: {} - should be >= 0.0".format(eps))
        super(AdamW, self).__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                                 correct_bias=correct_bias))

    @torch.no_grad()
    def step(self, closure=None):
        from k3m_amd import _lib as L
        loss = closure() if closure is not None else None
        for group in self.param_groups:
            if not group["correct_bias"]:
                raise NotImplementedError("AdamW(correct_bias=False) is not on the k3m_adamw kernel")
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.grad.dtype == torch.float32):
                    raise RuntimeError("pytorch_transformers.AdamW (MI355X build) steps HIP fp32 tensors only; got %s %s"
                                       % (p.device, p.dtype))
                st = self.state[p]
                n = p.numel()
                npad = (n + 3) // 4 * 4
                if not st:
                    st["step"] = 0
                    # the reference layout: moments shaped like the parameter (state_dict interchange)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                m, v = st["exp_avg"], st["exp_avg_sq"]
                if m.shape != p.shape or v.shape != p.shape:
                    raise ValueError("AdamW state for a parameter of shape %s has moments of shape %s / %s"
                                     % (tuple(p.shape), tuple(m.shape), tuple(v.shape)))
                if not (m.is_cuda and v.is_cuda and m.dtype == torch.float32 and v.dtype == torch.float32):
                    raise RuntimeError("AdamW moments must be HIP fp32 tensors (got %s %s)" % (m.device, m.dtype))
                st["step"] += 1
                ts = (p.data, p.grad, m, v)
                direct = npad == n and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in ts)
                if direct:
                    pp, gg, mm, vv = ts
                else:
                    # the kernel runs on 16-B vectors: stage padded copies (pad 0) and write the results back
                    pp, gg, mm, vv = (torch.zeros(npad, dtype=torch.float32, device=p.device) for _ in range(4))
                    for dst, src in zip((pp, gg, mm, vv), ts):
                        dst[:n].copy_(src.reshape(-1))
                L.call("k3m_adamw", pp.data_ptr(), gg.data_ptr(), mm.data_ptr(), vv.data_ptr(),
                       None, npad, float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                       float(group["weight_decay"]), int(st["step"]), 1.0, L.stream())
                if not direct:
                    for dst, src in zip((p.data, m, v), (pp, mm, vv)):
                        dst.copy_(src[:n].view_as(dst))
        return loss


class ConstantLRSchedule(LambdaLR):
    def __init__(self, optimizer, last_epoch=-1):
        super(ConstantLRSchedule, self).__init__(optimizer, lambda _: 1.0, last_epoch=last_epoch)


class WarmupConstantSchedule(LambdaLR):
    def __init__(self, optimizer, warmup_steps, last_epoch=-1):
        self.warmup_steps = warmup_steps
        super(WarmupConstantSchedule, self).__init__(optimizer, self.lr_lambda, last_epoch=last_epoch)

    def lr_lambda(self, step):
        if step < self.warmup_steps:
            return float(step) / float(max(1.0, self.warmup_steps))
        return 1.0


class WarmupLinearSchedule(LambdaLR):
    """Linear warmup over ``warmup_steps`` then linear decay to 0 at ``t_total``."""

    def __init__(self, optimizer, warmup_steps, t_total, last_epoch=-1):
        self.warmup_steps = warmup_steps
        self.t_total = t_total
        super(WarmupLinearSchedule, self).__init__(optimizer, self.lr_lambda, last_epoch=last_epoch)

    def lr_lambda(self, step):
        if step < self.warmup_steps:
            return float(step) / float(max(1, self.warmup_steps))
        return max(0.0, float(self.t_total - step) / float(max(1.0, self.t_total - self.warmup_steps)))


class WarmupCosineSchedule(LambdaLR):
    def __init__(self, optimizer, warmup_steps, t_total, cycles=.5, last_epoch=-1):
        self.warmup_steps, self.t_total, self.cycles = warmup_steps, t_total, cycles
        super(WarmupCosineSchedule, self).__init__(optimizer, self.lr_lambda, last_epoch=last_epoch)

    def lr_lambda(self, step):
        if step < self.warmup_steps:
            return float(step) / float(max(1.0, self.warmup_steps))
        progress = float(step - self.warmup_steps) / float(max(1, self.t_total - self.warmup_steps))
        return max(0.0, 0.5 * (1. + math.cos(math.pi * float(self.cycles) * 2.0 * progress)))
