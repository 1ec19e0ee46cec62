"""Item-alignment fine-tuning: K3MForItemAlignment
(vilbert_k3m/vilbert_k3m.py:2862-3456) and the fp32 training loop of finetune.py:385-489.

MI355X layout: the two items of every pair go through the encoder as ONE stacked batch of 2B
items (item 1 rows, then item 2 rows) — the same wide lock-step passes as pretraining, with twice
the rows per GEMM — so a pair step costs one encoder forward/backward, not two.  The engine runs
in its "item_alignment" task (no MLM / region / NSP heads, no LPM; the structure aggregator's
zero-triple fallback stays inside each item group).  The pair heads are fused HIP kernels
(k3m_amd/csrc/align.hip): "ce" = ClassificationHead + CrossEntropyLoss, "cosine" =
CosineEmbeddingLoss(margin 0).  "inner" has no loss function in the reference (the constructor
only sets one for ce / cosine, :2925-2931) and is rejected here.

Optimizer: torch.optim.AdamW(lr, eps, betas=(0.9, 0.98)) over the same two weight-decay groups as
pretraining (finetune.py:254-361) — a different update rule from pytorch_transformers' AdamW
(decay before the step, eps after the bias correction): k3m_adamw_torch.  WarmupLinearSchedule
stepped after the optimizer.
"""
import torch

from . import _lib as L
from . import ops
from .engine import K3MEngine, Lin
from .trainer import Trainer

HEAD_OFFSET = 1 << 44   # dropout counter range of the pair head (far above the encoder's)

ARG_NAMES = ["labels", "input_ids_1", "token_type_ids_1", "attention_mask_1", "input_ids_pv_1", "token_type_ids_pv_1",
             "attention_mask_pv_1", "index_p_1", "index_v_1", "image_feat_1", "image_loc_1", "image_attention_mask_1",
             "input_ids_2", "token_type_ids_2", "attention_mask_2", "input_ids_pv_2", "token_type_ids_pv_2",
             "attention_mask_pv_2", "index_p_2", "index_v_2", "image_feat_2", "image_loc_2", "image_attention_mask_2"]
_ENGINE_NAMES = [("input_ids", "input_ids"), ("token_type_ids", "segment_ids"), ("attention_mask", "input_mask"),
                 ("input_ids_pv", "input_ids_pv"), ("token_type_ids_pv", "segment_ids_pv"),
                 ("attention_mask_pv", "input_mask_pv"), ("index_p", "index_p"), ("index_v", "index_v"),
                 ("image_feat", "image_feat"), ("image_loc", "image_loc"), ("image_attention_mask", "image_mask")]


def stack_pair(pair, device):
    """Pair batch (forward-argument names) -> the engine's stacked 2B batch."""
    out = {}
    for src, dst in _ENGINE_NAMES:
        a, b = pair[src + "_1"], pair[src + "_2"]
        if a.shape[1:] != b.shape[1:]:
            raise ValueError("%s: items 1 and 2 differ in shape (%s vs %s)" % (src, tuple(a.shape), tuple(b.shape)))
        out[dst] = torch.cat([a.to(device), b.to(device)]).contiguous()
    return out


class K3MForItemAlignment(object):
    """The fine-tuning model on one GPU.  ``forward`` takes the reference's arguments
    (vilbert_k3m.py:3379-3403) and returns its 4-tuple (item_embedding_1, item_embedding_2, probs,
    loss); ``backward()`` accumulates the gradients of that loss into ``engine.fp.grad``."""

    def __init__(self, cfg, device=None, seed=1234, dtype="fp32", engine=None):
        if getattr(cfg, "task", None) != "item_alignment":
            raise ValueError("config must come from k3m_amd.config.finetune_config (task 'item_alignment')")
        self.cfg = cfg
        self.loss_type = getattr(cfg, "loss_type", "ce")
        if self.loss_type not in ("ce", "cosine"):
            raise ValueError("loss_type %r: the reference defines a loss only for 'ce' and 'cosine'" % self.loss_type)
        self.engine = engine if engine is not None else K3MEngine(cfg, device, seed=seed, dtype=dtype)
        fp = self.engine.fp
        if self.loss_type == "ce":
            self.cls_dense = Lin(fp, "classifier.dense")
        self.p_h = cfg.hidden_dropout_prob
        self._ctx = None

    def __call__(self, *args, **kw):
        return self.forward(*args, **kw)

    def forward(self, *args, output_all_attention_masks=False, train=True, noise=None, seed=None, **kw):
        """Positional / keyword arguments as K3MForItemAlignment.forward.  noise: optional pair
        (noise_item1, noise_item2) of {v,t,pv} gumbel-noise dicts (explicit randomness for parity)."""
        pair = dict(zip(ARG_NAMES, args))
        pair.update({k: v for k, v in kw.items() if k in ARG_NAMES})
        missing = [k for k in ARG_NAMES if k not in pair]
        if missing:
            raise TypeError("missing arguments: %s" % missing)
        eng = self.engine
        dev = eng.device
        batch = stack_pair(pair, dev)
        B = pair["input_ids_1"].shape[0]
        nz = None
        if noise is not None:
            nz = {k: torch.cat([noise[0][k], noise[1][k]]) for k in noise[0]}
        out, ctx = eng.forward(batch, train=train, noise=nz, seed=seed, groups=2)
        cf = out["c_final"]
        H = cf.shape[1]
        labels = pair["labels"].to(device=dev, dtype=torch.float32).contiguous()
        p = self.p_h if train else 0.0
        loss = torch.empty((1,), dtype=torch.float32, device=dev)
        rows = torch.empty((B,), dtype=torch.float32, device=dev)
        fp = eng.fp
        if self.loss_type == "ce":
            x = torch.empty((B, 2 * H), dtype=torch.float32, device=dev)
            L.call("k3m_align_pair_cat", cf.data_ptr(), B, H, p, ctx["seed"], HEAD_OFFSET, x.data_ptr(), L.stream())
            u = self.cls_dense.fwd(x)
            logits = torch.empty((B, 2), dtype=torch.float32, device=dev)
            probs = torch.empty_like(logits)
            dlog = torch.empty_like(logits)
            du = torch.empty_like(u)
            gW = torch.zeros((2, H), dtype=torch.float32, device=dev)   # folded into fp.grad by backward()
            gb = torch.zeros((2,), dtype=torch.float32, device=dev)
            L.call("k3m_align_ce_fwd_bwd", u.data_ptr(), fp.p["classifier.out_proj.weight"].data_ptr(),
                   fp.p["classifier.out_proj.bias"].data_ptr(), labels.data_ptr(), B, H, p, ctx["seed"],
                   HEAD_OFFSET + 2 * B * H, logits.data_ptr(), probs.data_ptr(), dlog.data_ptr(), rows.data_ptr(),
                   loss.data_ptr(), du.data_ptr(), gW.data_ptr(), gb.data_ptr(), L.stream())
            ctx["head"] = ("ce", x, du, gW, gb, B, H, p)
            res = (probs[:, 0], probs[:, 1], probs[:, 1], loss)
        else:
            probs = torch.empty((B,), dtype=torch.float32, device=dev)
            de = torch.empty_like(cf)
            L.call("k3m_align_cosine_fwd_bwd", cf.data_ptr(), labels.data_ptr(), B, H, 0.0, loss.data_ptr(),
                   probs.data_ptr(), rows.data_ptr(), de.data_ptr(), L.stream())
            ctx["head"] = ("cosine", de)
            res = (cf[:B], cf[B:], probs, loss)
        self._ctx = ctx
        return res

    def backward(self, grad_ready=None):
        """Gradients of the last forward's loss, ACCUMULATED into engine.fp.grad."""
        ctx, self._ctx = self._ctx, None
        if ctx is None:
            raise RuntimeError("backward() without a preceding forward()")
        fp = self.engine.fp
        head = ctx["head"]
        if head[0] == "ce":
            _, x, du, gW, gb, B, H, p = head
            ops.add_(fp.g["classifier.out_proj.weight"], gW)
            ops.add_(fp.g["classifier.out_proj.bias"], gb)
            self.cls_dense.wgrad(du, x)
            dx = self.cls_dense.dgrad(du)
            dcf = torch.empty((2 * B, H), dtype=torch.float32, device=x.device)
            L.call("k3m_align_pair_cat_bwd", dx.data_ptr(), B, H, p, ctx["seed"], HEAD_OFFSET, dcf.data_ptr(),
                   L.stream())
        else:
            dcf = head[1]
        ctx["d_c_final"] = dcf
        self.engine.backward(ctx, grad_ready=grad_ready)


class ItemAlignmentTrainer(Trainer):
    """finetune.py's fp32 loop: forward, backward, (DDP all-reduce), torch.optim.AdamW step,
    WarmupLinearSchedule step (finetune.py:385-489)."""

    ADAMW = "k3m_adamw_torch"

    def __init__(self, cfg, device, lr=5e-5, warmup_steps=0, total_steps=10000, seed=42, ddp=None, beta1=0.9,
                 beta2=0.98, eps=1e-8, weight_decay=0.01, init=True, dtype="fp32"):
        super(ItemAlignmentTrainer, self).__init__(cfg, device, lr=lr, warmup_steps=warmup_steps,
                                                   total_steps=total_steps, seed=seed, ddp=ddp, beta1=beta1,
                                                   beta2=beta2, eps=eps, weight_decay=weight_decay, init=init,
                                                   dtype=dtype)
        self.model = K3MForItemAlignment(cfg, engine=self.engine)

    def step(self, pair, noise=None):
        """One optimisation step on a pair batch (dict with the forward's argument names)."""
        eng = self.engine
        e1, e2, probs, loss = self.model.forward(*[pair[k] for k in ARG_NAMES], train=True, noise=noise,
                                                 seed=self.global_step)
        hook = self.ddp.grad_ready if self.ddp is not None else None
        if self.ddp is not None:
            self.ddp.begin(eng)
        self.model.backward(grad_ready=hook)
        scale = 1.0
        if self.ddp is not None:
            self.ddp.finish()
            scale = 1.0 / self.ddp.world
        self.optimizer_step(grad_scale=scale)
        eng.step_count += 1
        return {"item_embedding_1": e1, "item_embedding_2": e2, "probs": probs, "loss": loss}


def evaluate(model, batches, thresholds=None):
    """finetune.py:519-617 evaluation: the pair model in eval mode over ``batches`` (dicts with the
    forward's argument names), probs collected on the host, precision / recall / F1 of
    ``probs >= threshold`` for thresholds 0.1 .. 0.9.  (The reference concatenates with
    ``np.concatenate(model_probs, probs)`` — the second argument is the axis, so it fails from the
    second batch on; here the batches are concatenated.)"""
    import numpy as np
    from sklearn.metrics import f1_score, precision_score, recall_score
    if thresholds is None:
        thresholds = np.arange(0.1, 1.0, 0.1)
    probs, labels = [], []
    for pair in batches:
        _, _, p, _ = model.forward(*[pair[k] for k in ARG_NAMES], train=False)
        model._ctx = None   # no backward in evaluation
        probs.append(p.detach().float().cpu().numpy())
        labels.append(pair["labels"].detach().float().cpu().numpy())
    probs = np.concatenate(probs) if probs else np.zeros(0)
    labels = np.concatenate(labels) if labels else np.zeros(0)
    out = []
    for t in thresholds:
        pred = probs >= t
        out.append({"threshold": float(t),
                    "precision": float(precision_score(labels, pred, zero_division=0)),
                    "recall": float(recall_score(labels, pred, zero_division=0)),
                    "f1": float(f1_score(labels, pred, zero_division=0))})
    return out, probs, labels


def save_model(model, path):
    """The per-epoch ``K3M_item_alignment-<p>_epoch-<e>.bin`` (finetune.py:618-621): state_dict()."""
    from .checkpoint import model_state_dict
    torch.save(model_state_dict(model.engine.fp), path)
