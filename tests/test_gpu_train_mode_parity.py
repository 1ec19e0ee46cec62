"""Training-mode (dropout on) parity of the HIP layer ops against the oracle fed the HIP's own
dropout masks.  Dropout masks are not reproducible across implementations (the
reference draws them from torch's RNG), so the masks the kernels applied are regenerated on the host
from their (seed, offset) counters (tests/dropmask.py restates k3m_amd/csrc/common.h) and handed to the
oracle's layer functions (oracle/k3m_oracle.py ``drop=``), in the reference's dropout placement and
with the reference's rate per site, read from the config (vilbert_k3m.py: attention probabilities
:466 / :797 / :819, BertSelfOutput :487, BertOutput :530, BertBiOutput :988-991, BertImageOutput
:690).  The rates are set to four different values so a site that drew from the wrong rate fails.

Checked, per layer kind (text BertLayer 12 heads x 64, image BertImageLayer 8 x 128, the 1024-bi
co-attention layer image x text (37 x 36) and image x PV (37 x 128), the two-text co-attention PV x text
(8 heads x 96, 128 x 36), each also through the lock-step path the engine runs (fwd_steps / bwd_steps
under engine._lockstep, grouped GEMM launches), and the text / image embeddings with their output
dropout): forward output, input gradient(s) and the parameter gradients against a float64 autograd
reference (fp32 kernels: 2e-4 of each tensor's scale)."""
import numpy as np
import pytest
import torch

from golden_util import CFG_PATH
import dropmask as DM

pytestmark = pytest.mark.gpu
RATES = dict(hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.15, v_hidden_dropout_prob=0.2,
             v_attention_probs_dropout_prob=0.25)
TOL = 2e-4


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd.config import pretrain_config
    from k3m_amd.engine import K3MEngine
    from k3m_amd.weights import param_values
    cfg = pretrain_config(CFG_PATH)
    for k, v in RATES.items():
        setattr(cfg, k, v)
    e = K3MEngine(cfg, torch.device("cuda"))
    e.fp.load(param_values(cfg, 31))
    e._vals = param_values(cfg, 31)
    return e


def _p64(eng, prefix):
    return {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in eng._vals.items()
            if k.startswith(prefix + ".")}


def _close(a, b, what, floor=0.0):
    """max |a - b| <= TOL * max|b| + floor (floor: gradients that are analytically ~0, e.g. the key bias —
    softmax is shift invariant — carry fp32 noise only)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = float((a - b).abs().max())
    scale = float(b.abs().max()) + 1e-12
    assert err <= TOL * scale + floor, (what, err, scale)


def _mask(m):
    return (1.0 - m.double())[:, None, None, :] * -10000.0


def _lengths_mask(nseq, L, g):
    lens = torch.randint(L // 2, L + 1, (nseq,), generator=g)
    return (torch.arange(L)[None, :] < lens[:, None]).long()


@pytest.mark.parametrize("kind", ["text", "image"])
def test_bert_layer_train_mode(eng, kind):
    from oracle import k3m_oracle as O
    from k3m_amd.engine import Rng, _ext_mask
    c = eng.cfg
    if kind == "text":
        op, pre, H, nh, L = eng.text[4], "encoder.layer.4", c.hidden_size, c.num_attention_heads, 36
        pa, ph = c.attention_probs_dropout_prob, c.hidden_dropout_prob
    else:
        op, pre, H, nh, L = eng.image[2], "encoder.v_layer.2", c.v_hidden_size, c.v_num_attention_heads, 37
        pa, ph = c.v_attention_probs_dropout_prob, c.v_hidden_dropout_prob
    nseq, seed = 5, 777
    g = torch.Generator().manual_seed(3)
    x = torch.randn(nseq * L, H, generator=g)
    m = _lengths_mask(nseq, L, g)
    dy = torch.randn(nseq * L, H, generator=g)
    dev = torch.device("cuda")
    eng.fp.grad.zero_()
    rng = Rng(seed)
    y, saved = op.fwd(x.to(dev), [(0, nseq, L, _ext_mask(m.to(dev)))], rng)
    dx = op.bwd(dy.to(dev), saved)
    torch.cuda.synchronize()
    # the layer's counters: attention probabilities, then the two residual tails (Rng.take order)
    na, nh_ = nseq * nh * L * L, nseq * L * H
    drop = {"attn": torch.from_numpy(DM.attn_keep_scale(rng.seed, 0, nseq * nh * L, L, pa)),
            "attn_out": torch.from_numpy(DM.keep_scale(rng.seed, na, nh_, ph)),
            "ffn_out": torch.from_numpy(DM.keep_scale(rng.seed, na + nh_, nh_, ph))}
    P = _p64(eng, pre)
    xr = x.double().view(nseq, L, H).requires_grad_(True)
    yr = O.bert_layer(P, pre, xr, _mask(m), nh, drop=drop)
    yr.backward(dy.double().view(nseq, L, H))
    _close(y, yr.reshape(-1, H), kind + " y")
    _close(dx, xr.grad.reshape(-1, H), kind + " dx")
    for n, p in P.items():
        _close(eng.fp.g[n], p.grad, kind + " grad " + n, floor=2e-6)
    # dropout was really on: the eval-mode layer differs
    ye = O.bert_layer(P, pre, x.double().view(nseq, L, H), _mask(m), nh)
    assert float((ye.reshape(-1, H) - yr.reshape(-1, H).detach()).abs().max()) > 1e-2


# per co-attention kind: (engine op list, prefix, stream-1 / stream-2 lengths and widths) and the reference's
# dropout rate per site: BertBiAttention(_two_text) probabilities :742-743 / :865-872, BertBiOutput(_two_txt)
# :974-981 / :1000-1008, v_output BertImageOutput :687 (1024-bi) or BertOutput (two-text), t_output BertOutput
CO_KINDS = {
    "tv": ("co_tv", "encoder.c_layer.2", 37, 36, "v", "t"),
    "pv": ("co_pv", "encoder.c_layer_pv_v.3", 37, 128, "v", "t"),
    "tt": ("co_tt", "encoder.c_layer_pv_t.1", 128, 36, "t", "t"),
}


def _co_rates(c, kind):
    ffn1 = c.v_hidden_dropout_prob if kind != "tt" else c.hidden_dropout_prob
    return [("attn1", c.v_attention_probs_dropout_prob), ("attn2", c.attention_probs_dropout_prob),
            ("out1", c.v_hidden_dropout_prob), ("out2", c.hidden_dropout_prob),
            ("ffn1", ffn1), ("ffn2", c.hidden_dropout_prob)]


@pytest.mark.parametrize("kind,lockstep", [("tv", False), ("tv", True), ("pv", True), ("tt", False), ("tt", True)])
def test_coattention_layer_train_mode(eng, kind, lockstep):
    from oracle import k3m_oracle as O
    from k3m_amd.engine import Rng, _ext_mask, _lockstep
    c = eng.cfg
    ops_name, pre, L1, L2, w1, w2 = CO_KINDS[kind]
    op = getattr(eng, ops_name)[int(pre.rsplit(".", 1)[1])]
    H1 = c.v_hidden_size if w1 == "v" else c.hidden_size
    H2 = c.hidden_size
    nb = c.bi_num_attention_heads
    nseq, seed = 3, 4242 + L1 + L2
    g = torch.Generator().manual_seed(9 + L2)
    s1, s2 = torch.randn(nseq * L1, H1, generator=g), torch.randn(nseq * L2, H2, generator=g)
    m1, m2 = _lengths_mask(nseq, L1, g), _lengths_mask(nseq, L2, g)
    dy1, dy2 = torch.randn(nseq * L1, H1, generator=g), torch.randn(nseq * L2, H2, generator=g)
    dev = torch.device("cuda")
    eng.fp.grad.zero_()
    rng = Rng(seed)
    o1 = torch.empty(nseq * L1, H1, device=dev)
    o2 = torch.empty(nseq * L2, H2, device=dev)
    ds1 = torch.empty(nseq * L1, H1, device=dev)
    ds2 = torch.empty(nseq * L2, H2, device=dev)
    args = (s1.to(dev), s2.to(dev), nseq, L1, L2, _ext_mask(m1.to(dev)), _ext_mask(m2.to(dev)), rng, o1, o2)
    if lockstep:
        res = []
        _lockstep([op.fwd_steps(*args, res)])
        saved = res[0]
        _lockstep([op.bwd_steps(dy1.to(dev), dy2.to(dev), saved, ds1, ds2)])
    else:
        saved = op.fwd(*args)
        op.bwd(dy1.to(dev), dy2.to(dev), saved, ds1, ds2)
    torch.cuda.synchronize()
    # counters in ConnectionOp order: probs1 (stream-2 queries over stream-1 keys), probs2, BiOutput tails
    # 1 and 2, stream-1 FFN tail, stream-2 FFN tail
    n12 = nseq * nb * L1 * L2
    sizes = dict(attn1=n12, attn2=n12, out1=nseq * L1 * H1, out2=nseq * L2 * H2, ffn1=nseq * L1 * H1,
                 ffn2=nseq * L2 * H2)
    # attention score blocks: probs1 = stream-2 queries (L2) over stream-1 keys (L1), probs2 the reverse
    attn_rows = dict(attn1=(nseq * nb * L2, L1), attn2=(nseq * nb * L1, L2))
    drop, off = {}, 0
    for site, p in _co_rates(c, kind):
        if site in attn_rows:
            drop[site] = torch.from_numpy(DM.attn_keep_scale(rng.seed, off, *attn_rows[site], p))
        else:
            drop[site] = torch.from_numpy(DM.keep_scale(rng.seed, off, sizes[site], p))
        off += sizes[site]
    P = _p64(eng, pre)
    r1 = s1.double().view(nseq, L1, H1).requires_grad_(True)
    r2 = s2.double().view(nseq, L2, H2).requires_grad_(True)
    y1, y2 = O.connection_layer(P, pre, r1, _mask(m1), r2, _mask(m2), nb, drop=drop)
    (y1 * dy1.double().view_as(y1)).sum().add((y2 * dy2.double().view_as(y2)).sum()).backward()
    tag = "co %s%s " % (kind, " lockstep" if lockstep else "")
    _close(o1, y1.reshape(-1, H1), tag + "y1")
    _close(o2, y2.reshape(-1, H2), tag + "y2")
    _close(ds1, r1.grad.reshape(-1, H1), tag + "ds1")
    _close(ds2, r2.grad.reshape(-1, H2), tag + "ds2")
    for n, p in P.items():
        if p.grad is None:   # q_dense1/2 of BertBiOutput are never used
            continue
        _close(eng.fp.g[n], p.grad, tag + "grad " + n, floor=2e-6)


def test_embeddings_train_mode(eng):
    """BertEmbeddings (vilbert_k3m.py:361-382) and BertImageEmbeddings (:2153-2161) with their output
    dropout (hidden_dropout_prob for both, :380 / :2150), through the engine's own calls (engine.py
    forward 'embeddings' block, backward 'embeddings' block): forward outputs and the gradients of the
    word / position / token-type tables, both LayerNorms and the two image-embedding Linears."""
    from oracle import k3m_oracle as O
    from k3m_amd import ops
    from k3m_amd.engine import Rng
    c = eng.cfg
    fp = eng.fp
    dev = torch.device("cuda")
    B, T, R, H, Hv = 4, 36, 37, c.hidden_size, c.v_hidden_size
    p = c.hidden_dropout_prob
    g = torch.Generator().manual_seed(21)
    ids = torch.randint(0, 200, (B, T), generator=g)
    ids[:, -3:] = 0                                # padding id 0 gets no word-table gradient
    tt = torch.randint(0, 2, (B, T), generator=g)
    feat = torch.randn(B * R, c.v_feature_size, generator=g)
    loc = torch.rand(B * R, 5, generator=g)
    dy_t = torch.randn(B * T, H, generator=g)
    dy_v = torch.randn(B * R, Hv, generator=g)
    eng.fp.grad.zero_()
    rng = Rng(99)
    # ---- forward, as K3MEngine.forward
    out = torch.empty(B * T, H, device=dev)
    c0, c1 = torch.empty_like(out), torch.empty_like(out)
    xh, rs = torch.empty_like(out), torch.empty(B * T, device=dev)
    off_t = rng.take(B * T * H)
    ops.embed_fwd(ids.to(dev), tt.to(dev), fp.p["embeddings.word_embeddings.weight"],
                  fp.p["embeddings.position_embeddings.weight"], fp.p["embeddings.token_type_embeddings.weight"],
                  eng.emb_ln.g, eng.emb_ln.b, out, c0, c1, xh, rs, p, rng.seed, off_t)
    img = eng.vemb_img.fwd(feat.to(dev))
    lce = eng.vemb_loc.fwd(loc.to(dev))
    ov = torch.empty(B * R, Hv, device=dev)
    xhv, rsv = torch.empty_like(ov), torch.empty(B * R, device=dev)
    off_v = rng.take(B * R * Hv)
    ops.ln_fwd(img, lce, eng.vemb_ln.g, eng.vemb_ln.b, ov, xhv, rsv, p_out=p, seed=rng.seed, off_out=off_v)
    # ---- backward, as K3MEngine._backward
    ds = torch.empty(B * T, H, device=dev)
    dyd = dy_t.to(dev)
    ops.ln_bwd(dyd, xh, rs, eng.emb_ln.g, ds, ds, eng.emb_ln.gg, eng.emb_ln.gb, p_out=p, seed=rng.seed, off_out=off_t)
    ops.embed_bwd(ids.to(dev).contiguous(), tt.to(dev).contiguous(), ds, fp.g["embeddings.word_embeddings.weight"],
                  fp.g["embeddings.position_embeddings.weight"], fp.g["embeddings.token_type_embeddings.weight"])
    dsv = torch.empty(B * R, Hv, device=dev)
    ops.ln_bwd(dy_v.to(dev), xhv, rsv, eng.vemb_ln.g, dsv, dsv, eng.vemb_ln.gg, eng.vemb_ln.gb, p_out=p,
               seed=rng.seed, off_out=off_v)
    eng.vemb_img.wgrad(dsv, feat.to(dev))
    eng.vemb_loc.wgrad(dsv, loc.to(dev))
    torch.cuda.synchronize()
    # ---- float64 reference with the kernels' masks
    mt = torch.from_numpy(DM.keep_scale(rng.seed, off_t, B * T * H, p)).double().view(B, T, H)
    mv = torch.from_numpy(DM.keep_scale(rng.seed, off_v, B * R * Hv, p)).double().view(B * R, Hv)
    P = {k: torch.from_numpy(v).double().requires_grad_(True) for k, v in eng._vals.items()
         if k.startswith("embeddings.") or k.startswith("v_embeddings.")}
    yt = O.embeddings(P, ids, tt) * mt
    yv = O.v_embeddings(P, feat.double(), loc.double()) * mv
    (yt * dy_t.double().view(B, T, H)).sum().add((yv * dy_v.double()).sum()).backward()
    _close(out, yt.reshape(-1, H), "emb y")
    _close(c0, yt.reshape(-1, H), "emb copy 0")
    _close(c1, yt.reshape(-1, H), "emb copy 1")
    _close(ov, yv, "v_emb y")
    for n, pr in P.items():
        _close(eng.fp.g[n], pr.grad, "emb grad " + n, floor=2e-6)
    assert float(eng.fp.g["embeddings.word_embeddings.weight"][0].abs().max()) == 0.0   # padding_idx=0
    # dropout really on: about p of the outputs are zero
    zf = float((out == 0).float().mean())
    assert abs(zf - p) < 0.02, zf
