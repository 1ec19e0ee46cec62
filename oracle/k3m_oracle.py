"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU fp32 restatement (plain PyTorch on the host) of the K3M tri-modal pretraining step, written
from the reference's behaviour, used as the parity checker for the HIP path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module; the
product path (``k3m_amd``) never does.

Pinning: checked against golden vectors produced by the reference model itself
(``tests/golden/make_golden.py`` imports /root/reference/vilbert_k3m/vilbert_k3m.py in the build
container and records losses, c_initial/c_final and gradients) — see tests/test_oracle_golden.py.

Randomness is made explicit so parity is exact:
* gumbel noise of ``F.gumbel_softmax`` (vilbert_k3m.py:2364) is an input (``noise[mod]``, shape
  [B, L, 3, D]);
* the ``random.sample`` negative draws of the LPM loss (:2480, :2492) are inputs
  (``ent_neg`` / ``val_neg`` [B, NPV, 2] int64, -1 = no draw);
* dropout is off (eval-mode parity, as in the reference's ``model.eval()``).

Parameters are a dict {reference state_dict name: tensor}.
"""
import math

import torch
import torch.nn.functional as F


# ---------------------------------------------------------------- primitives

def layer_norm(x, w, b, eps=1e-12):
    """TF-style LayerNorm (vilbert_k3m.py:319-332): biased variance, eps inside the sqrt."""
    u = x.mean(-1, keepdim=True)
    s = (x - u).pow(2).mean(-1, keepdim=True)
    return w * ((x - u) / torch.sqrt(s + eps)) + b


def gelu(x):
    """erf GELU (vilbert_k3m.py:119-125)."""
    return x * 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0)))


def linear(P, name, x):
    y = x @ P[name + ".weight"].t()
    b = P.get(name + ".bias")
    return y + b if b is not None else y


def ext_mask(mask):
    """(1 - m) * -10000 additive key mask (vilbert_k3m.py:2547-2580) -> [B, 1, 1, L]."""
    return (1.0 - mask.to(torch.float32))[:, None, None, :] * -10000.0


def heads(x, nh):
    B, L, D = x.shape
    return x.view(B, L, nh, D // nh).permute(0, 2, 1, 3)


def _drop(x, drop, site):
    """Training-mode dropout with an explicit mask (0 or 1/(1-p) per element) — the oracle is fed the
    masks of the implementation under test (tests/test_gpu_train_mode_parity.py); eval mode (None)
    is the identity, as nn.Dropout in model.eval()."""
    if drop is None or drop.get(site) is None:
        return x
    return x * drop[site].to(x.dtype).reshape(x.shape)


def attend(q, k, v, mask_add, nh, drop=None, site="attn"):
    """softmax(q k^T / sqrt(d) + mask) v, heads split from the last dim (vilbert_k3m.py:439-475);
    dropout on the probabilities (:466)."""
    d = q.shape[-1] // nh
    qh, kh, vh = heads(q, nh), heads(k, nh), heads(v, nh)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(d) + mask_add
    p = _drop(torch.softmax(s, dim=-1), drop, site)
    ctx = (p @ vh).permute(0, 2, 1, 3).contiguous()
    return ctx.view(ctx.shape[0], ctx.shape[1], -1)


# ---------------------------------------------------------------- layers

def bert_layer(P, pre, x, mask_add, nh, drop=None):
    """BertLayer / BertImageLayer (vilbert_k3m.py:535-548, :696-709), post-LN.  ``drop`` (training
    mode): masks for "attn" (probabilities, :466), "attn_out" (BertSelfOutput :487) and "ffn_out"
    (BertOutput :530)."""
    q = linear(P, pre + ".attention.self.query", x)
    k = linear(P, pre + ".attention.self.key", x)
    v = linear(P, pre + ".attention.self.value", x)
    ctx = attend(q, k, v, mask_add, nh, drop, "attn")
    a = layer_norm(_drop(linear(P, pre + ".attention.output.dense", ctx), drop, "attn_out") + x,
                   P[pre + ".attention.output.LayerNorm.weight"], P[pre + ".attention.output.LayerNorm.bias"])
    f = gelu(linear(P, pre + ".intermediate.dense", a))
    return layer_norm(_drop(linear(P, pre + ".output.dense", f), drop, "ffn_out") + a,
                      P[pre + ".output.LayerNorm.weight"], P[pre + ".output.LayerNorm.bias"])


def connection_layer(P, pre, s1, m1, s2, m2, nh, drop=None):
    """BertConnectionLayer(_two_text) (vilbert_k3m.py:1030-1111) with BertBiAttention :753-838
    and BertBiOutput :986-996.  Stream 1 attends to stream 2 and vice versa.  ``drop`` (training
    mode): "attn1" / "attn2" (probabilities, :797 / :819), "out1" / "out2" (BiOutput :988 / :991),
    "ffn1" / "ffn2" (v_output / t_output)."""
    b = pre + ".biattention."
    q1, k1, v1 = linear(P, b + "query1", s1), linear(P, b + "key1", s1), linear(P, b + "value1", s1)
    q2, k2, v2 = linear(P, b + "query2", s2), linear(P, b + "key2", s2), linear(P, b + "value2", s2)
    ctx1 = attend(q2, k1, v1, m1, nh, drop, "attn1")   # stream-2 queries over stream-1 keys
    ctx2 = attend(q1, k2, v2, m2, nh, drop, "attn2")   # stream-1 queries over stream-2 keys
    o = pre + ".biOutput."
    h1 = layer_norm(_drop(linear(P, o + "dense1", ctx2), drop, "out1") + s1, P[o + "LayerNorm1.weight"],
                    P[o + "LayerNorm1.bias"])
    h2 = layer_norm(_drop(linear(P, o + "dense2", ctx1), drop, "out2") + s2, P[o + "LayerNorm2.weight"],
                    P[o + "LayerNorm2.bias"])
    f1 = gelu(linear(P, pre + ".v_intermediate.dense", h1))
    y1 = layer_norm(_drop(linear(P, pre + ".v_output.dense", f1), drop, "ffn1") + h1,
                    P[pre + ".v_output.LayerNorm.weight"], P[pre + ".v_output.LayerNorm.bias"])
    f2 = gelu(linear(P, pre + ".t_intermediate.dense", h2))
    y2 = layer_norm(_drop(linear(P, pre + ".t_output.dense", f2), drop, "ffn2") + h2,
                    P[pre + ".t_output.LayerNorm.weight"], P[pre + ".t_output.LayerNorm.bias"])
    return y1, y2


def run_pair(P, cfg, txt, tmask, other, omask, co_prefix, other_is_text):
    """One pair pass of BertEncoder (calculate_for_text_img :1154, calculate_for_pv_img :1332,
    calculate_for_two_text :1510).  ``other`` is the image stream (image layers) or, for the
    two-text pass, the PV stream (shared text layers)."""
    nh_t, nh_v, nh_b = cfg.num_attention_heads, cfg.v_num_attention_heads, cfg.bi_num_attention_heads
    v_ids = cfg.t_biattention_id if other_is_text else cfg.v_biattention_id
    t_start = v_start = 0
    for c, (v_end, t_end) in enumerate(zip(v_ids, cfg.t_biattention_id)):
        for i in range(t_start, t_end):
            txt = bert_layer(P, "encoder.layer.%d" % i, txt, tmask, nh_t)
        for i in range(v_start, v_end):
            if other_is_text:
                other = bert_layer(P, "encoder.layer.%d" % i, other, omask, nh_t)
            else:
                other = bert_layer(P, "encoder.v_layer.%d" % i, other, omask, nh_v)
        other, txt = connection_layer(P, "encoder.%s.%d" % (co_prefix, c), other, omask, txt, tmask, nh_b)
        v_start, t_start = v_end, t_end
    n_other = cfg.num_hidden_layers if other_is_text else cfg.v_num_hidden_layers
    for i in range(v_start, n_other):
        if other_is_text:
            other = bert_layer(P, "encoder.layer.%d" % i, other, omask, nh_t)
        else:
            other = bert_layer(P, "encoder.v_layer.%d" % i, other, omask, nh_v)
    for i in range(t_start, cfg.num_hidden_layers):
        txt = bert_layer(P, "encoder.layer.%d" % i, txt, tmask, nh_t)
    return txt, other


def embeddings(P, ids, tt):
    """BertEmbeddings (vilbert_k3m.py:361-382): word + position + type -> LN (dropout off).
    ``padding_idx=0`` (:343-345): the lookup adds no gradient to word row 0."""
    pos = torch.arange(ids.shape[1])
    e = (F.embedding(ids, P["embeddings.word_embeddings.weight"], padding_idx=0)
         + P["embeddings.position_embeddings.weight"][pos][None]
         + P["embeddings.token_type_embeddings.weight"][tt])
    return layer_norm(e, P["embeddings.LayerNorm.weight"], P["embeddings.LayerNorm.bias"])


def v_embeddings(P, feat, loc):
    """BertImageEmbeddings (vilbert_k3m.py:2153-2161)."""
    e = linear(P, "v_embeddings.image_embeddings", feat) + linear(P, "v_embeddings.image_location_embeddings", loc)
    return layer_norm(e, P["v_embeddings.LayerNorm.weight"], P["v_embeddings.LayerNorm.bias"])


def gumbel_hard(ak, g):
    """torch.nn.functional.gumbel_softmax(ak, tau=1, hard=True, dim=2) with explicit noise g
    (straight-through: forward one-hot of argmax(softmax(ak + g)), gradient of the soft sample)."""
    y = torch.softmax(ak + g, dim=2)
    idx = y.argmax(dim=2, keepdim=True)
    hard = torch.zeros_like(ak).scatter_(2, idx, 1.0)
    return hard - y.detach() + y


def fuse(P, mod, x0, x1, x2, noise, mode):
    """pre_sampling_sequence (vilbert_k3m.py:2331-2374) for if_pre_sampling==1, mean for 0 (:2388-2391)."""
    if mode == 0:
        return (x0 + x1 + x2) / 3
    x0, x1, x2 = F.relu(x0), F.relu(x1), F.relu(x2)
    c = torch.cat((x0, x1, x2), 2)
    a = [torch.sigmoid(linear(P, "score_%s_%s" % (k, mod), c)) for k in ("self", "cross1", "cross2")]
    ak = torch.stack(a, 2)
    sel = gumbel_hard(ak, noise)
    return x0 * sel[:, :, 0] + x1 * sel[:, :, 1] + x2 * sel[:, :, 2]


def structure_aggregator(P, c_init, seq_pv, index_p, index_v, ent_neg, val_neg, margin):
    """structure_aggregator (vilbert_k3m.py:2413-2505) with the negative draws as inputs.

    Quirks kept: p / v are the mean of the two ENDPOINT rows (:2443-2444); a zero-triple item
    reuses the most recent ``t`` (bare except :2452-2456); the margin ranking loss pushes the
    positive distance above the negative one (:2501-2502)."""
    B = seq_pv.shape[0]
    props, vals = [], []
    c_final = []
    t = None
    for i in range(B):
        props.append([])
        vals.append([])
        rows = []
        for j in range(index_p.shape[1]):
            if int(index_p[i, j, 0]) == 0:
                break
            p = seq_pv[i].index_select(0, index_p[i, j]).mean(0)
            v = seq_pv[i].index_select(0, index_v[i, j]).mean(0)
            props[i].append(p)
            vals[i].append(v)
            rows.append(linear(P, "struc_w1", torch.cat((c_init[i], p, v), 0)))
        if rows:
            t = torch.stack(rows, 0)
        elif t is None:
            t = c_init[i].unsqueeze(0)
        b = linear(P, "struc_w2", F.leaky_relu(t))
        att = torch.softmax(b, dim=0)
        c_final.append(c_init[i] + linear(P, "struc_w3", (att * t).sum(0)))
    c_final = torch.stack(c_final, 0)
    if ent_neg is None:   # item alignment: no LPM (vilbert_k3m.py:3288-3291)
        return c_final, None
    pos, neg = [], []
    for i in range(B):
        for j in range(len(props[i])):
            base = props[i][j] - vals[i][j]
            pn = torch.norm(c_final[i] + base)
            for k in ent_neg[i, j].tolist():
                if k >= 0:
                    pos.append(pn)
                    neg.append(torch.norm(c_final[k] + base))
            for k in val_neg[i, j].tolist():
                if k >= 0:
                    pos.append(pn)
                    neg.append(torch.norm(c_final[i] + props[i][j] - vals[i][k]))
    pos = torch.stack(pos) if pos else torch.zeros(0)
    neg = torch.stack(neg) if neg else torch.zeros(0)
    loss = torch.clamp(neg - pos + margin, min=0).mean()
    return c_final, loss


def encode(P, cfg, batch, noise=None):
    """Embeddings, the three co-attention pair encoders, the initial-interactive fusion, pooling
    and c_initial (bert_tri + get_sequence_pooled_output_final, vilbert_k3m.py:2376-2411, :2673-2725;
    identical in K3MForItemAlignment.item_embedding :3329-3371)."""
    ids, tmask_i, tt = batch["input_ids"], batch["input_mask"], batch["segment_ids"]
    pids, pmask_i, ptt = batch["input_ids_pv"], batch["input_mask_pv"], batch["segment_ids_pv"]
    feat, loc, imask_i = batch["image_feat"], batch["image_loc"], batch["image_mask"]
    tmask, pmask, imask = ext_mask(tmask_i), ext_mask(pmask_i), ext_mask(imask_i)
    mode = getattr(cfg, "if_pre_sampling", 1)

    ind_v = v_embeddings(P, feat, loc)
    ind_t = embeddings(P, ids, tt)
    ind_pv = embeddings(P, pids, ptt)

    t_v, v_t = run_pair(P, cfg, ind_t, tmask, ind_v, imask, "c_layer", False)
    pv_v, v_pv = run_pair(P, cfg, ind_pv, pmask, ind_v, imask, "c_layer_pv_v", False)
    t_pv, pv_t = run_pair(P, cfg, ind_t, tmask, ind_pv, pmask, "c_layer_pv_t", True)

    nz = noise or {}
    seq_v = fuse(P, "v", ind_v, v_t, v_pv, nz.get("v"), mode)
    seq_t = fuse(P, "t", ind_t, t_v, t_pv, nz.get("t"), mode)
    seq_pv = fuse(P, "pv", ind_pv, pv_v, pv_t, nz.get("pv"), mode)

    pooled_v = linear(P, "map_bi_to_individual", seq_v[:, 1:].mean(1))
    pooled_t = seq_t[:, 1:].mean(1)
    pooled_pv = seq_pv[:, 1:].mean(1)
    c_init = (pooled_v + pooled_t + pooled_pv) / 3
    return dict(seq_v=seq_v, seq_t=seq_t, seq_pv=seq_pv, pooled_v=pooled_v, pooled_t=pooled_t, pooled_pv=pooled_pv,
                c_init=c_init)


def forward(P, cfg, batch, noise=None, ent_neg=None, val_neg=None):
    """Full pretraining forward (vilbert_k3m.py:2673-2846).  Returns a dict of the 10-tuple items
    and the summed training loss of train_concap_struc.py:531-533 (loss_img_weight = 1)."""
    enc = encode(P, cfg, batch, noise)
    seq_v, seq_t, seq_pv = enc["seq_v"], enc["seq_t"], enc["seq_pv"]
    pooled_v, pooled_t, pooled_pv, c_init = enc["pooled_v"], enc["pooled_t"], enc["pooled_pv"], enc["c_init"]
    c_final, loss_lpm = structure_aggregator(P, c_init, seq_pv, batch["index_p"], batch["index_v"],
                                             ent_neg, val_neg, float(getattr(cfg, "margin", 1.0)))

    # heads (BertPreTrainingHeads :1875-1909); MLM on all T and P positions, tied decoder
    def mlm_logits(h):
        h = gelu(linear(P, "cls.predictions.transform.dense", h))
        h = layer_norm(h, P["cls.predictions.transform.LayerNorm.weight"], P["cls.predictions.transform.LayerNorm.bias"])
        return h @ P["embeddings.word_embeddings.weight"].t() + P["cls.predictions.bias"]

    lt = mlm_logits(seq_t)
    lpv = mlm_logits(seq_pv)
    hv = gelu(linear(P, "cls.imagePredictions.transform.dense", seq_v))
    hv = layer_norm(hv, P["cls.imagePredictions.transform.LayerNorm.weight"], P["cls.imagePredictions.transform.LayerNorm.bias"])
    lv = linear(P, "cls.imagePredictions.decoder", hv)
    nsp = linear(P, "cls.seq_relationship", pooled_t + pooled_pv + pooled_v)

    V = cfg.vocab_size
    loss_t = F.cross_entropy(lt.reshape(-1, V), batch["lm_label_ids"].reshape(-1), ignore_index=-1)
    loss_pv = F.cross_entropy(lpv.reshape(-1, V), batch["lm_label_ids_pv"].reshape(-1), ignore_index=-1)
    # region KL (visual_target 0, :2753-2760): sum over masked rows / number of masked rows
    logp = F.log_softmax(lv[:, 1:], dim=2)
    tgt = batch["image_target"]
    kl = torch.xlogy(tgt, tgt) - tgt * logp
    lab = (batch["image_label"] == 1)
    loss_img = (kl * lab.unsqueeze(2).float()).sum() / lab.sum()
    nsp_label = 1 - 1 * ((batch["is_next"] + batch["is_next_pv_v"] + batch["is_next_pv_t"]) == 0)
    loss_nsp = F.cross_entropy(nsp.view(-1, 2), nsp_label.view(-1), ignore_index=-1)
    total = loss_t + loss_img + loss_pv + loss_lpm
    return dict(loss=total, masked_lm_loss=loss_t, masked_img_loss=loss_img, masked_lm_loss_pv=loss_pv,
                next_sentence_loss=loss_nsp, loss_lpm=loss_lpm, c_initial=c_init, c_final=c_final,
                pooled_t=pooled_t, pooled_pv=pooled_pv, pooled_v=pooled_v,
                logits_t=lt, logits_pv=lpv, logits_v=lv)


# ---------------------------------------------------------------- item alignment (fine-tuning)

PAIR_KEYS = [("input_ids", "input_ids"), ("token_type_ids", "segment_ids"), ("attention_mask", "input_mask"),
             ("input_ids_pv", "input_ids_pv"), ("token_type_ids_pv", "segment_ids_pv"),
             ("attention_mask_pv", "input_mask_pv"), ("index_p", "index_p"), ("index_v", "index_v"),
             ("image_feat", "image_feat"), ("image_loc", "image_loc"), ("image_attention_mask", "image_mask")]


def item_batch(pair, k):
    """The engine-named batch of item k (1 or 2) of a pair batch named as the arguments of
    K3MForItemAlignment.forward (vilbert_k3m.py:3379-3403)."""
    return {dst: pair["%s_%d" % (src, k)] for src, dst in PAIR_KEYS}


def item_alignment_forward(P, cfg, pair, noise1=None, noise2=None):
    """K3MForItemAlignment.forward (vilbert_k3m.py:3379-3456), eval mode.  Returns
    (item_embedding_1, item_embedding_2, probs, loss) with the reference's quirks: for "ce" the
    first two outputs are probs[:, 0] / probs[:, 1]; for "cosine" probs compares item 1 with itself
    (:3443); "inner" has no loss function in the reference (AttributeError) and is rejected."""
    es = []
    for k, nz in ((1, noise1), (2, noise2)):
        b = item_batch(pair, k)
        enc = encode(P, cfg, b, nz)
        c_final, _ = structure_aggregator(P, enc["c_init"], enc["seq_pv"], b["index_p"], b["index_v"], None, None, 0.0)
        es.append(c_final)
    e1, e2 = es
    labels = pair["labels"]
    lt = getattr(cfg, "loss_type", "ce")
    if lt == "ce":
        h = torch.tanh(linear(P, "classifier.dense", torch.cat((e1, e2), 1)))
        logits = linear(P, "classifier.out_proj", h)
        probs = torch.softmax(logits, dim=1)
        loss = F.cross_entropy(logits.view(-1, 2), labels.view(-1).to(torch.long))
        return probs[:, 0], probs[:, 1], probs[:, 1], loss
    if lt == "cosine":
        loss = F.cosine_embedding_loss(e1, e2, 2 * labels - 1, margin=0.0)
        probs = (F.cosine_similarity(e1, e1) + 1) / 2
        return e1, e2, probs, loss
    raise ValueError("loss_type %r has no loss function in the reference" % lt)


def adamw_torch_step(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.98, eps=1e-8):
    """torch.optim.AdamW single-tensor math (finetune.py:356-361): decay first, bias-corrected denom."""
    p.mul_(1.0 - lr * wd)
    m.lerp_(g, 1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


# ---------------------------------------------------------------- optimizer

def warmup_linear_lambda(step, warmup, t_total):
    """pytorch_transformers 1.1.0 WarmupLinearSchedule multiplier (train_concap_struc.py:444-448)."""
    if step < warmup:
        return float(step) / float(max(1, warmup))
    return max(0.0, float(t_total - step) / float(max(1.0, t_total - warmup)))


def adamw_step(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.98, eps=1e-8):
    """pytorch_transformers 1.1.0 AdamW for one tensor (in place; ``step`` is the 1-based count
    after increment).  eps is added to sqrt(v) outside the bias correction; decoupled weight
    decay is applied AFTER the Adam update with the uncorrected lr."""
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    denom = v.sqrt().add_(eps)
    step_size = lr * math.sqrt(1.0 - beta2 ** step) / (1.0 - beta1 ** step)
    p.addcdiv_(m, denom, value=-step_size)
    if wd > 0.0:
        p.add_(p, alpha=-lr * wd)


def fused_adam_step(p, g, m, v, step, lr, wd, beta1=0.9, beta2=0.999, eps=1e-8, bias_correction=False):
    """apex FusedAdam, adam_w_mode (the optimizer of the mixed-precision driver branches,
    train_concap_struc.py:410-411, :426: bias_correction=False; per-group weight_decay 0.01 / 0.0
    overrides the constructor's 5e-4).  Restated from apex's multi_tensor_adam (ADAM_MODE_1):
    p -= lr * ((m / bc1) / (sqrt(v / bc2) + eps) + wd * p).  Unpinned: apex is not installed."""
    m.mul_(beta1).add_(g, alpha=1.0 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step if bias_correction else 1.0
    bc2 = 1.0 - beta2 ** step if bias_correction else 1.0
    denom = (v / bc2).sqrt().add_(eps)
    upd = (m / bc1) / denom + wd * p
    p.sub_(lr * upd)
