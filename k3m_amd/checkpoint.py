"""Checkpoint interchange with the reference driver.

The reference writes, per epoch (train_concap_struc.py:691-705):

* ``K3M_struc_presample-<p>_epoch-<e>.bin``: ``model.state_dict()`` — 999 keys, the 998 parameters
  of ``named_parameters()`` plus the tied ``cls.predictions.decoder.weight`` (vilbert_k3m.py:2266-2272);
* ``...tar``: ``{"model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "global_step"}``

and reads them back with ``module.`` stripped (:259-297).  The optimizer is pytorch_transformers'
AdamW over the two parameter groups of :352-367 (weights with decay 0.01 first, then the
"bias"/"LayerNorm.*" names with 0.0, each in ``named_parameters()`` order); its
``state_dict()`` is torch.optim.Optimizer's: parameters numbered consecutively across the groups,
per-parameter state ``{"step", "exp_avg", "exp_avg_sq"}`` only for parameters that received a
gradient (the 86 never-grad tensors have none).  The scheduler is WarmupLinearSchedule, a LambdaLR
(``warmup_steps``, ``t_total``, ``base_lrs``, ``last_epoch`` ...).

Here the parameters and the AdamW moments live in flat HBM buffers (k3m_amd/params.py,
trainer.py); this module maps between those buffers and the reference's per-tensor layout.
Files are read with ``torch.load(weights_only=True)`` (tensors and plain containers only).
"""
import torch

from .params import is_frozen, is_no_decay

DECODER_KEY = "cls.predictions.decoder.weight"
TIED_TO = "embeddings.word_embeddings.weight"


def reference_groups(names):
    """Parameter-name lists of the two AdamW groups (train_concap_struc.py:352-367)."""
    return [[n for n in names if not is_no_decay(n)], [n for n in names if is_no_decay(n)]]


def model_state_dict(fp):
    """CPU copy of the 999-key reference state_dict."""
    sd = {}
    for name, _ in fp.spec:
        sd[name] = fp.p[name].detach().to("cpu", copy=True)
    if "cls.predictions.bias" in fp.p:   # pretraining model: the tied MLM decoder
        sd[DECODER_KEY] = sd[TIED_TO]
    return sd


def load_model_state_dict(fp, sd, strict=True):
    """Copy a (reference or own) state_dict into the flat parameter buffer; strips ``module.``."""
    sd = {(k[7:] if k.startswith("module.") else k): v for k, v in sd.items()}
    missing = [n for n, _ in fp.spec if n not in sd]
    if strict and missing:
        raise KeyError("state_dict lacks %d parameters, e.g. %s" % (len(missing), missing[:4]))
    with torch.no_grad():
        for name, _ in fp.spec:
            if name in sd:
                t = sd[name]
                if tuple(t.shape) != tuple(fp.shapes[name]):
                    raise ValueError("%s: shape %s, expected %s" % (name, tuple(t.shape), fp.shapes[name]))
                fp.p[name].copy_(t.to(fp.p[name].device, torch.float32))
    fp.shadow_fresh = False
    return missing


def optimizer_state_dict(fp, m, v, step, lr_now, base_lr, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01):
    """torch.optim.Optimizer.state_dict() of the reference AdamW, from the flat moments m, v."""
    names = [n for n, _ in fp.spec]
    groups = reference_groups(names)
    state, pg, idx = {}, [], 0
    for gi, gnames in enumerate(groups):
        ids = []
        for n in gnames:
            if step > 0 and not is_frozen(n):
                o, k = fp.offsets[n], fp.p[n].numel()
                state[idx] = {"step": int(step), "exp_avg": m[o:o + k].view(fp.shapes[n]).to("cpu", copy=True),
                              "exp_avg_sq": v[o:o + k].view(fp.shapes[n]).to("cpu", copy=True)}
            ids.append(idx)
            idx += 1
        pg.append({"lr": float(lr_now), "betas": tuple(betas), "eps": float(eps),
                   "weight_decay": float(weight_decay if gi == 0 else 0.0), "correct_bias": True,
                   "initial_lr": float(base_lr), "params": ids})
    return {"state": state, "param_groups": pg}


def load_optimizer_state_dict(fp, m, v, osd):
    """Fill the flat moments from a reference-layout optimizer state_dict; returns its step."""
    names = [n for n, _ in fp.spec]
    order = [n for g in reference_groups(names) for n in g]
    nparams = sum(len(g["params"]) for g in osd["param_groups"])
    if nparams != len(order):
        raise ValueError("optimizer state covers %d parameters, expected %d" % (nparams, len(order)))
    step = 0
    with torch.no_grad():
        m.zero_()
        v.zero_()
        for g in osd["param_groups"]:
            for pid in g["params"]:
                st = osd["state"].get(pid, osd["state"].get(str(pid)))
                if not st:
                    continue
                n = order[pid]
                if is_frozen(n):
                    continue
                o, k = fp.offsets[n], fp.p[n].numel()
                m[o:o + k].copy_(st["exp_avg"].reshape(-1).to(m.device, torch.float32))
                v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1).to(v.device, torch.float32))
                s = st["step"]
                step = max(step, int(s.item() if torch.is_tensor(s) else s))
    return step


def scheduler_state_dict(warmup, t_total, base_lr, step, lr_now):
    """LambdaLR.state_dict() of WarmupLinearSchedule(optimizer, warmup_steps, t_total) after ``step``
    scheduler steps (two parameter groups)."""
    return {"warmup_steps": warmup, "t_total": t_total, "base_lrs": [float(base_lr)] * 2, "last_epoch": int(step),
            "_step_count": int(step) + 1, "_get_lr_called_within_step": False, "_last_lr": [float(lr_now)] * 2,
            "lr_lambdas": [None, None]}


def save_checkpoint(trainer, tar_path=None, bin_path=None):
    """Write the reference's .bin and/or .tar for a k3m_amd.trainer.Trainer."""
    fp = trainer.engine.fp
    sd = model_state_dict(fp)
    if bin_path:
        torch.save(sd, bin_path)
    if tar_path:
        lr_now = trainer.current_lr()
        torch.save({"model_state_dict": sd,
                    "optimizer_state_dict": optimizer_state_dict(fp, trainer.m, trainer.v, trainer.global_step, lr_now,
                                                                 trainer.lr, (trainer.beta1, trainer.beta2),
                                                                 trainer.eps, trainer.wd),
                    "scheduler_state_dict": scheduler_state_dict(trainer.warmup, trainer.t_total, trainer.lr,
                                                                 trainer.global_step, lr_now),
                    "global_step": int(trainer.global_step)}, tar_path)


def load_checkpoint(trainer, tar_path):
    """Resume a Trainer from a reference-layout .tar (train_concap_struc.py:277-293)."""
    ck = torch.load(tar_path, map_location="cpu", weights_only=True)
    fp = trainer.engine.fp
    load_model_state_dict(fp, ck["model_state_dict"])
    opt_step = load_optimizer_state_dict(fp, trainer.m, trainer.v, ck["optimizer_state_dict"])
    sch = ck.get("scheduler_state_dict") or {}
    if "warmup_steps" in sch:
        trainer.warmup = sch["warmup_steps"]
    if "t_total" in sch:
        trainer.t_total = sch["t_total"]
    if sch.get("base_lrs"):
        trainer.lr = float(sch["base_lrs"][0])
    trainer.global_step = int(ck.get("global_step", sch.get("last_epoch", opt_step)))
    trainer.engine.step_count = trainer.global_step
    fp.grad.zero_()
    return trainer.global_step
