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


def param_groups_of(fp, weight_decay=0.01, lr_mult=None, frozen_names=()):
    """[(names, weight_decay, lr multiplier)] in the reference's param_groups order.

    * No pretrained model (:352-367): two groups over ALL of ``named_parameters()`` (``--freeze``d
      tensors included: the list is not filtered by requires_grad) — decay, then no_decay.
    * Pretrained model (``lr_mult`` given, :368-385): one group per tensor with ``requires_grad``
      (the ``--freeze`` names are left out), in ``named_parameters()`` order, lr x multiplier and
      weight decay 0.01 / 0.0 by name."""
    names = [n for n, _ in fp.spec]
    if lr_mult is None:
        a, b = reference_groups(names)
        return [(a, weight_decay, 1.0), (b, 0.0, 1.0)]
    frozen = set(frozen_names)
    return [([n], 0.0 if is_no_decay(n) else 0.01, float(lr_mult.get(n, 1.0))) for n in names if n not in frozen]


def _groups_of_trainer(trainer):
    return param_groups_of(trainer.engine.fp, getattr(trainer, "wd", 0.01), getattr(trainer, "lr_mult", None),
                           getattr(trainer, "frozen_names", ()))


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


def optimizer_state_dict(fp, m, v, step, groups, group_lr, base_lr, betas=(0.9, 0.98), eps=1e-8,
                         optimizer="adamw"):
    """torch.optim.Optimizer.state_dict() of the reference optimizer, from the flat moments m, v.

    ``groups`` = param_groups_of(...); ``group_lr(i)`` = the current lr of group i.  ``optimizer``:
    "adamw" = pytorch_transformers AdamW (per-parameter ``step``, ``correct_bias``); "fused_adam" =
    apex FusedAdam as the --apex_fast branch holds it (:413-418: per-group ``step``,
    ``bias_correction=False``).  The --fp16 branch wraps FusedAdam in FP16_Optimizer, whose own
    state_dict (fp32 master copies, loss scaler) is not reproduced."""
    state, pg, idx = {}, [], 0
    for gi, (gnames, wd, mult) in enumerate(groups):
        ids = []
        for n in gnames:
            if step > 0 and not is_frozen(n):
                o, k = fp.offsets[n], fp.p[n].numel()
                st = {"exp_avg": m[o:o + k].view(fp.shapes[n]).to("cpu", copy=True),
                      "exp_avg_sq": v[o:o + k].view(fp.shapes[n]).to("cpu", copy=True)}
                if optimizer == "adamw":
                    st = dict(step=int(step), **st)
                state[idx] = st
            ids.append(idx)
            idx += 1
        g = {"lr": float(group_lr(gi)), "betas": tuple(betas), "eps": float(eps), "weight_decay": float(wd)}
        if optimizer == "adamw":
            g["correct_bias"] = True
        else:
            g["bias_correction"] = False
            g["step"] = int(step)
        g["initial_lr"] = float(base_lr * mult)
        g["params"] = ids
        pg.append(g)
    return {"state": state, "param_groups": pg}


def load_optimizer_state_dict(fp, m, v, osd, groups):
    """Fill the flat moments from a reference-layout optimizer state_dict; returns its step.
    ``groups`` = the layout this run's optimizer was built with (param_groups_of); a file of another
    layout (group count or sizes differ) is rejected instead of mapped onto the wrong tensors."""
    got = [len(g["params"]) for g in osd["param_groups"]]
    want = [len(g[0]) for g in groups]
    if got != want:
        raise ValueError("optimizer state has %d groups of sizes %s..., this optimizer %d groups of sizes %s... "
                         "(two-group vs per-tensor layout, or a different --freeze list)"
                         % (len(got), got[:4], len(want), want[:4]))
    pid_name = {}
    for g, (gnames, _, _) in zip(osd["param_groups"], groups):
        for pid, n in zip(g["params"], gnames):
            pid_name[pid] = n
    step = 0
    with torch.no_grad():
        m.zero_()
        v.zero_()
        for g in osd["param_groups"]:
            if "step" in g:   # apex FusedAdam keeps the step per group
                step = max(step, int(g["step"]))
            for pid in g["params"]:
                st = osd["state"].get(pid, osd["state"].get(str(pid)))
                if not st:
                    continue
                n = pid_name[pid]
                if is_frozen(n):
                    continue
                o, k = fp.offsets[n], fp.p[n].numel()
                if tuple(st["exp_avg"].shape) != tuple(fp.shapes[n]):
                    raise ValueError("%s: moment shape %s, expected %s" % (n, tuple(st["exp_avg"].shape),
                                                                          fp.shapes[n]))
                m[o:o + k].copy_(st["exp_avg"].reshape(-1).to(m.device, torch.float32))
                v[o:o + k].copy_(st["exp_avg_sq"].reshape(-1).to(v.device, torch.float32))
                if "step" in st:
                    s = st["step"]
                    step = max(step, int(s.item() if torch.is_tensor(s) else s))
    return step


def scheduler_state_dict(warmup, t_total, base_lrs, step, last_lrs):
    """LambdaLR.state_dict() of WarmupLinearSchedule(optimizer, warmup_steps, t_total) after ``step``
    scheduler steps (one base lr per parameter group)."""
    return {"warmup_steps": warmup, "t_total": t_total, "base_lrs": [float(x) for x in base_lrs],
            "last_epoch": int(step), "_step_count": int(step) + 1, "_get_lr_called_within_step": False,
            "_last_lr": [float(x) for x in last_lrs], "lr_lambdas": [None] * len(base_lrs)}


def _group_lrs(trainer, groups):
    """Current lr of every group (LambdaLR: initial_lr * lambda; the --fp16 quirk keeps every group
    but the first at lr * lambda(0))."""
    fp = trainer.engine.fp
    out = []
    for gi, (gnames, _, mult) in enumerate(groups):
        if hasattr(trainer, "run_lr"):
            out.append(trainer.run_lr(fp.offsets[gnames[0]] if gnames else 0, mult))
        else:
            out.append(mult * trainer.current_lr())
    return out


def save_checkpoint(trainer, tar_path=None, bin_path=None):
    """Write the reference's .bin and/or .tar for a k3m_amd.trainer.Trainer, with the optimizer and
    scheduler state in the parameter-group layout the Trainer was built with."""
    fp = trainer.engine.fp
    sd = model_state_dict(fp)
    if bin_path:
        torch.save(sd, bin_path)
    if tar_path:
        groups = _groups_of_trainer(trainer)
        lrs = _group_lrs(trainer, groups)
        base = [trainer.lr * mult for _, _, mult in groups]
        opt = getattr(trainer, "optimizer", "adamw")
        torch.save({"model_state_dict": sd,
                    "optimizer_state_dict": optimizer_state_dict(fp, trainer.m, trainer.v, trainer.global_step, groups,
                                                                 lambda i: lrs[i], trainer.lr,
                                                                 (trainer.beta1, trainer.beta2), trainer.eps, opt),
                    "scheduler_state_dict": scheduler_state_dict(trainer.warmup, trainer.t_total, base,
                                                                 trainer.global_step, lrs),
                    "global_step": int(trainer.global_step)}, tar_path)


def load_checkpoint(trainer, tar_path):
    """Resume a Trainer from a reference-layout .tar (train_concap_struc.py:277-293)."""
    ck = torch.load(tar_path, map_location="cpu", weights_only=True)
    fp = trainer.engine.fp
    load_model_state_dict(fp, ck["model_state_dict"])
    groups = _groups_of_trainer(trainer)
    opt_step = load_optimizer_state_dict(fp, trainer.m, trainer.v, ck["optimizer_state_dict"], groups)
    sch = ck.get("scheduler_state_dict") or {}
    if "warmup_steps" in sch:
        trainer.warmup = sch["warmup_steps"]
    if "t_total" in sch:
        trainer.t_total = sch["t_total"]
    if sch.get("base_lrs"):
        trainer.lr = float(sch["base_lrs"][0]) / groups[0][2]
    trainer.global_step = int(ck.get("global_step", sch.get("last_epoch", opt_step)))
    trainer.engine.step_count = trainer.global_step
    fp.grad.zero_()
    return trainer.global_step
