"""Drop-in import surface for the pretraining driver.

``train_concap_struc.py`` imports (train_concap_struc.py:26)::

    from vilbert_k3m.vilbert_k3m import BertConfig, BertForMultiModalPreTraining_tri_stru

and uses the model as an nn.Module: ``Model(config)`` / ``Model.from_pretrained(path, config=...,
default_gpu=...)`` (:231-236), ``.cuda()``, ``.train()``, ``named_parameters()`` (optimizer groups,
:352-389), ``state_dict()`` (:691-705), and the 10-tuple ``forward`` (:502-524) whose summed losses
are back-propagated with ``loss.backward()`` (:569).  This module provides the same class on top of
the MI355X engine (k3m_amd/engine.py): parameters are nn.Parameter views of the engine's flat HBM
buffer, forward runs the HIP kernels, and one autograd node routes ``loss.backward()`` into the
engine's explicit backward.  Reference: vilbert_k3m/vilbert_k3m.py:2186-2859, utils.py:756-1086.
"""
import torch
import torch.nn as nn

from .config import BertConfig  # noqa: F401  (re-exported: same config ABI)
from .engine import K3MEngine
from .trainer import init_reference

_OUT_KEYS = ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "next_sentence_loss", "c_initial",
             "c_final", "loss_lpm")


class _Step(torch.autograd.Function):
    @staticmethod
    def forward(fctx, anchor, model, batch, kw):
        out, ectx = model.engine.forward(batch, train=model.training, **kw)
        fctx.model, fctx.ectx = model, ectx
        return tuple(out[k].clone() for k in _OUT_KEYS)

    @staticmethod
    def backward(fctx, g_t, g_img, g_pv, g_nsp, g_ci, g_cf, g_lpm):
        model, ectx = fctx.model, fctx.ectx

        def val(g):
            return 0.0 if g is None else float(g.reshape(-1)[0])
        wt, wpv = val(g_t), val(g_pv)
        if g_ci is not None:
            ectx["d_c_initial"] = g_ci
        if g_cf is not None:
            ectx["d_c_final"] = g_cf
        model._prepare_grads()
        model.engine.backward(ectx, w_mlm=wt, w_img=val(g_img), w_lpm=val(g_lpm), w_mlm_pv=wpv)
        model._expose_grads()
        fctx.ectx = None
        return None, None, None, None


class BertForMultiModalPreTraining_tri_stru(nn.Module):
    """Same constructor / forward contract as the reference class (vilbert_k3m.py:2186)."""

    def __init__(self, config, device=None, seed=42, dtype="fp32"):
        super().__init__()
        self.config = config
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.engine = K3MEngine(config, dev, seed=seed, dtype=dtype)
        init_reference(self.engine.fp, config, seed)
        self._names = [n for n, _ in self.engine.fp.spec]
        for n in self._names:
            p = nn.Parameter(self.engine.fp.p[n], requires_grad=True)
            self.register_parameter(n.replace(".", "__"), p)
        self._anchor = torch.zeros(1, device=dev, requires_grad=True)

    # --- parameter naming identical to the reference
    def named_parameters(self, prefix="", recurse=True, remove_duplicate=True):
        for n in self._names:
            yield prefix + n, getattr(self, n.replace(".", "__"))

    def parameters(self, recurse=True):
        for _, p in self.named_parameters():
            yield p

    def state_dict(self, *args, **kwargs):
        sd = self.engine.fp.state_dict()
        return {k: v.detach() for k, v in sd.items()}

    def load_state_dict(self, state_dict, strict=True):
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in state_dict.items()}
        missing = [n for n in self._names if n not in sd]
        if strict and missing:
            raise KeyError("missing keys: %s" % missing[:8])
        with torch.no_grad():
            for n in self._names:
                if n in sd:
                    self.engine.fp.p[n].copy_(sd[n].to(self.engine.fp.p[n].device, torch.float32))
        return missing

    @classmethod
    def from_pretrained(cls, path, config=None, default_gpu=True, **kw):
        """Loads a reference checkpoint (.bin state_dict); renames gamma/beta and strips the
        ``bert.`` prefix like utils.py:999-1052.  Returns the model in eval mode (:1076)."""
        model = cls(config, **kw)
        sd = torch.load(path, map_location="cpu", weights_only=True)
        fixed = {}
        for k, v in sd.items():
            k2 = k.replace("gamma", "weight").replace("beta", "bias")
            if k2.startswith("bert."):
                k2 = k2[5:]
            fixed[k2] = v
        model.load_state_dict(fixed, strict=False)
        model.eval()
        return model

    def tie_weights(self):
        pass  # the decoder IS the word-embedding view of the flat buffer

    def half(self):
        """``model.half()`` of the --fp16 / --apex_fast branch (train_concap_struc.py:299-300, before the optimizer
        is built at :352-441).  The reference casts the weights to fp16 and apex keeps fp32 master copies; here the
        engine switches to its 16-bit mode (bf16 encoder GEMMs and attention — the MI355X 16-bit matrix format —
        fp32 master weights, heads and optimizer).  Parameter names, order and values are kept; the parameters
        become views of the new engine's buffer, so build the optimizer after this call, as the driver does.
        The driver's ``.half()`` inputs (:496-499) are accepted: forward reads them as fp32."""
        if self.engine.dtype == "bf16":
            return self
        old = self.engine
        eng = K3MEngine(self.config, old.device, seed=old.base_seed, dtype="bf16")
        with torch.no_grad():
            eng.fp.data.copy_(old.fp.data)
            eng.fp.grad.copy_(old.fp.grad)
        eng.fp.shadow_fresh = False
        eng.step_count = old.step_count
        self.engine = eng
        for n in self._names:
            key = n.replace(".", "__")
            old_p = getattr(self, key)
            grad = old_p.grad
            # keep the driver's --freeze choice (train_concap_struc.py:255-257 runs before .half() at :300): the
            # optimizer groups are built from requires_grad (:371), so that flag is what keeps a tensor frozen
            p = nn.Parameter(eng.fp.p[n], requires_grad=old_p.requires_grad)
            self._parameters[key] = p
            if grad is not None:
                p.grad = eng.fp.g[n]
        return self

    # --- gradients live in the engine's flat buffer
    def _prepare_grads(self):
        p0 = getattr(self, self._names[0].replace(".", "__"))
        if p0.grad is None:
            self.engine.fp.grad.zero_()   # zero_grad(set_to_none=True) happened

    def _expose_grads(self):
        for n in self._names:
            p = getattr(self, n.replace(".", "__"))
            if p.grad is None or p.grad.data_ptr() != self.engine.fp.g[n].data_ptr():
                p.grad = self.engine.fp.g[n]

    def forward(self, input_ids, image_feat, image_loc, token_type_ids=None, attention_mask=None,
                image_attention_mask=None, masked_lm_labels=None, image_label=None, image_target=None,
                next_sentence_label=None, output_all_attention_masks=False, input_ids_pv=None, token_type_ids_pv=None,
                attention_mask_pv=None, masked_lm_labels_pv=None, next_sentence_label_pv_v=None,
                next_sentence_label_pv_t=None, index_p=None, index_v=None, device=None, gumbel_noise=None,
                ent_neg=None, val_neg=None):
        dev = self.engine.device

        def d(t, like=None):
            if t is None:
                return torch.ones_like(like) if like is not None else None
            return torch.as_tensor(t).to(dev)
        ids = d(input_ids)
        batch = dict(
            input_ids=ids, input_mask=d(attention_mask, ids),
            segment_ids=d(token_type_ids) if token_type_ids is not None else torch.zeros_like(ids),
            lm_label_ids=d(masked_lm_labels), is_next=d(next_sentence_label),
            input_ids_pv=d(input_ids_pv), image_feat=d(image_feat).float(), image_loc=d(image_loc).float(),
            image_target=d(image_target).float(), image_label=d(image_label),
            lm_label_ids_pv=d(masked_lm_labels_pv), is_next_pv_v=d(next_sentence_label_pv_v),
            is_next_pv_t=d(next_sentence_label_pv_t), index_p=d(index_p), index_v=d(index_v))
        batch["input_mask_pv"] = d(attention_mask_pv, batch["input_ids_pv"])
        batch["segment_ids_pv"] = (d(token_type_ids_pv) if token_type_ids_pv is not None
                                   else torch.zeros_like(batch["input_ids_pv"]))
        B, R = batch["image_feat"].shape[:2]
        batch["image_mask"] = (d(image_attention_mask) if image_attention_mask is not None
                               else torch.ones((B, R), dtype=torch.int64, device=dev))
        # labelled-row counts attached by the loaders (k3m_amd/loaders.py): no device->host sync
        n_m = getattr(masked_lm_labels, "_k3m_n_labels", None)
        n_v = getattr(image_label, "_k3m_n_labels", None)
        if n_m is not None and n_v is not None:
            batch["_label_counts"] = (n_m, n_v)
        kw = {"noise": gumbel_noise, "ent_neg": ent_neg, "val_neg": val_neg}
        mlm_t, img, mlm_pv, nsp, c_init, c_final, lpm = _Step.apply(self._anchor, self, batch, kw)
        return (mlm_t, img, 0, mlm_pv, 0, 0, nsp, c_init, c_final, lpm)
