"""Training-mode (dropout on) parity of the HIP layer ops against the oracle fed the HIP's own
dropout masks.  Dropout masks are not reproducible across implementations (the
reference draws them from torch's RNG), so the masks the kernels applied are regenerated on the host
from their (seed, offset) counters (tests/dropmask.py restates k3m_amd/csrc/common.h) and handed to the
oracle's layer functions (oracle/k3m_oracle.py ``drop=``), in the reference's dropout placement and
with the reference's rate per site, read from the config (vilbert_k3m.py: attention probabilities
:466 / :797 / :819, BertSelfOutput :487, BertOutput :530, BertBiOutput :988-991, BertImageOutput
:690).  The rates are set to four different values so a site that drew from the wrong rate fails.

Checked, per layer kind (text BertLayer 12 heads x 64, image BertImageLayer 8 x 128, the 1024-bi
co-attention layer image x text): forward output, input gradient(s) and the layer's parameter
gradients against a float64 autograd reference (fp32 kernels: 2e-4 of each tensor's scale)."""
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
    drop = {"attn": torch.from_numpy(DM.keep_scale(rng.seed, 0, na, pa)),
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


def test_coattention_layer_train_mode(eng):
    from oracle import k3m_oracle as O
    from k3m_amd.engine import Rng, _ext_mask
    c = eng.cfg
    op, pre = eng.co_tv[2], "encoder.c_layer.2"
    Hv, H, nb = c.v_hidden_size, c.hidden_size, c.bi_num_attention_heads
    nseq, R, T, seed = 4, 37, 36, 4242
    g = torch.Generator().manual_seed(9)
    s1, s2 = torch.randn(nseq * R, Hv, generator=g), torch.randn(nseq * T, H, generator=g)
    m1, m2 = _lengths_mask(nseq, R, g), _lengths_mask(nseq, T, g)
    dy1, dy2 = torch.randn(nseq * R, Hv, generator=g), torch.randn(nseq * T, H, generator=g)
    dev = torch.device("cuda")
    eng.fp.grad.zero_()
    rng = Rng(seed)
    o1 = torch.empty(nseq * R, Hv, device=dev)
    o2 = torch.empty(nseq * T, H, device=dev)
    saved = op.fwd(s1.to(dev), s2.to(dev), nseq, R, T, _ext_mask(m1.to(dev)), _ext_mask(m2.to(dev)), rng, o1, o2)
    ds1 = torch.empty(nseq * R, Hv, device=dev)
    ds2 = torch.empty(nseq * T, H, device=dev)
    op.bwd(dy1.to(dev), dy2.to(dev), saved, ds1, ds2)
    torch.cuda.synchronize()
    # counters in ConnectionOp.fwd order: probs1 (text queries over image keys), probs2, BiOutput tails
    # 1 and 2, image FFN tail, text FFN tail
    n1 = n2 = nseq * nb * T * R
    sizes = [("attn1", n1, c.v_attention_probs_dropout_prob), ("attn2", n2, c.attention_probs_dropout_prob),
             ("out1", nseq * R * Hv, c.v_hidden_dropout_prob), ("out2", nseq * T * H, c.hidden_dropout_prob),
             ("ffn1", nseq * R * Hv, c.v_hidden_dropout_prob), ("ffn2", nseq * T * H, c.hidden_dropout_prob)]
    drop, off = {}, 0
    for site, n, p in sizes:
        drop[site] = torch.from_numpy(DM.keep_scale(rng.seed, off, n, p))
        off += n
    P = _p64(eng, pre)
    r1 = s1.double().view(nseq, R, Hv).requires_grad_(True)
    r2 = s2.double().view(nseq, T, H).requires_grad_(True)
    y1, y2 = O.connection_layer(P, pre, r1, _mask(m1), r2, _mask(m2), nb, drop=drop)
    (y1 * dy1.double().view_as(y1)).sum().add((y2 * dy2.double().view_as(y2)).sum()).backward()
    _close(o1, y1.reshape(-1, Hv), "co y1")
    _close(o2, y2.reshape(-1, H), "co y2")
    _close(ds1, r1.grad.reshape(-1, Hv), "co ds1")
    _close(ds2, r2.grad.reshape(-1, H), "co ds2")
    for n, p in P.items():
        if p.grad is None:   # q_dense1/2 of BertBiOutput are never used
            continue
        _close(eng.fp.g[n], p.grad, "co grad " + n, floor=2e-6)
