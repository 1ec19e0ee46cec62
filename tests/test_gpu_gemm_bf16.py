"""bf16-operand MFMA GEMM (gemm_bf16.hip) against a plain PyTorch fp32 reference of the same op
on the bf16-rounded operands.  Accumulation is fp32 in both, so the fp32-C results agree to
summation-order rounding (rel 1e-5 of max|ref| x sqrt(k) headroom); bf16-C results additionally
carry one bf16 output rounding (rel 2^-8)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd import _lib
    _lib.load()
    return torch.device("cuda")


def _rel(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-12))


def _ops(m, n, k, at, bt, dev, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = torch.randn(m, k, generator=g).to(dev).bfloat16()
    Bm = torch.randn(k, n, generator=g).to(dev).bfloat16()
    a = A.t().contiguous() if at else A
    b = Bm.t().contiguous() if bt else Bm
    return A, Bm, a, b


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (300, 200, 100), (2368, 1024, 2048), (37, 1601, 1024),
                                   (64, 768, 5), (1000, 3072, 768), (20992 // 8, 768, 3072)])
@pytest.mark.parametrize("at,bt", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_bf16_layouts_f32c(dev, m, n, k, at, bt):
    from k3m_amd import ops
    A, Bm, a, b = _ops(m, n, k, at, bt, dev, m * 7 + n + k)
    c = torch.randn(m, n, device=dev)
    ref = 0.5 * (A.float() @ Bm.float()) + 0.25 * c
    ops.gemm(a, at, b, bt, c, m, n, k, alpha=0.5, beta=0.25)
    assert _rel(c, ref) < 1e-5


@pytest.mark.parametrize("m,n,k", [(300, 200, 100), (1000, 3072, 768), (37, 1601, 1024)])
@pytest.mark.parametrize("at,bt", [(0, 1), (0, 0)])
def test_gemm_bf16_layouts_bf16c(dev, m, n, k, at, bt):
    from k3m_amd import ops
    A, Bm, a, b = _ops(m, n, k, at, bt, dev, m + n * 3 + k)
    c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    ref = A.float() @ Bm.float()
    ops.gemm(a, at, b, bt, c, m, n, k)
    # one round-to-nearest of the fp32 sum: |err| <= 2^-9 |ref| elementwise
    err = (c.float() - ref).abs()
    assert bool((err <= ref.abs() * 2.0 ** -8 + 1e-6 * ref.abs().max()).all())


@pytest.mark.parametrize("splitk", [2, 5])
def test_gemm_bf16_splitk(dev, splitk):
    from k3m_amd import ops
    m, n, k = 768, 768, 20000
    A = torch.randn(k, m, device=dev).bfloat16()
    Bm = torch.randn(k, n, device=dev).bfloat16()
    c = torch.randn(m, n, device=dev)
    ref = A.float().t() @ Bm.float() + c
    ws = torch.empty(splitk * m * n, device=dev)
    ops.gemm(A, 1, Bm, 0, c, m, n, k, beta=1.0, splitk=splitk, ws=ws)
    assert _rel(c, ref) < 1e-5


def test_gemm_bf16_epilogues(dev):
    from k3m_amd import ops, _lib as L
    F = torch.nn.functional
    x = torch.randn(500, 768, device=dev).bfloat16()
    W = (torch.randn(3072, 768, device=dev) * 0.05).bfloat16()
    b = torch.randn(3072, device=dev)
    r = x.float() @ W.float().t() + b
    pre = torch.empty(500, 3072, device=dev, dtype=torch.bfloat16)
    y = torch.empty(500, 3072, device=dev, dtype=torch.bfloat16)
    ops.gemm(x, 0, W, 1, y, 500, 3072, 768, L.EPI_BIAS_GELU, b, pre)
    assert _rel(pre, r) < 2.0 ** -8
    assert _rel(y, F.gelu(pre.float())) < 2.0 ** -8
    s = torch.empty(500, 3072, device=dev)
    ops.gemm(x, 0, W, 1, s, 500, 3072, 768, L.EPI_BIAS_SIGMOID, b)
    assert _rel(s, torch.sigmoid(r)) < 1e-5
    dy = torch.randn(500, 3072, device=dev).bfloat16()
    pre2 = torch.randn(500, 768, device=dev).bfloat16()
    dx = torch.empty(500, 768, device=dev, dtype=torch.bfloat16)
    ops.gemm(dy, 0, W, 0, dx, 500, 768, 3072, L.EPI_DGELU, None, pre2)
    xr = pre2.float().requires_grad_(True)
    F.gelu(xr).backward(dy.float() @ W.float())
    assert _rel(dx, xr.grad) < 2.0 ** -7


# ---------------------------------------------------------------- bf16 storage in the other kernels
def _ln_ref(s, g, b):
    u = s.mean(-1, keepdim=True)
    v = (s - u).pow(2).mean(-1, keepdim=True)
    return g * (s - u) / torch.sqrt(v + 1e-12) + b


@pytest.mark.parametrize("cols,M", [(768, 999), (1024, 999),
                                    # the half-wave 16-B kernels (forward >= 4,096 rows, backward >= 16,384)
                                    (768, 5000), (768, 16500), (1024, 16400)])
def test_layernorm_bf16(dev, cols, M):
    """bf16 activations in/out, fp32 statistics and parameter gradients; reference = fp32 math on
    the bf16 inputs; tolerance = bf16 output rounding."""
    from k3m_amd import ops
    x = torch.randn(M, cols, device=dev).bfloat16()
    r = torch.randn(M, cols, device=dev).bfloat16()
    g = 1 + 0.1 * torch.randn(cols, device=dev)
    b = 0.1 * torch.randn(cols, device=dev)
    y = torch.empty_like(x)
    xh = torch.empty_like(x)
    rs = torch.empty(M, device=dev)
    ops.ln_fwd(x, r, g, b, y, xh, rs)
    xr, rr = x.float().requires_grad_(True), r.float().requires_grad_(True)
    gr, br = g.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = _ln_ref(xr + rr, gr, br)
    assert _rel(y, yr) < 2.0 ** -7
    dy = torch.randn(M, cols, device=dev).bfloat16()
    yr.backward(dy.float())
    dres = torch.empty_like(x)
    dg = torch.zeros(cols, device=dev)
    db = torch.zeros(cols, device=dev)
    ops.ln_bwd(dy, xh, rs, g, dres, dres, dg, db)
    assert _rel(dres, xr.grad) < 2.0 ** -6
    assert _rel(dg, gr.grad) < 1e-2
    assert _rel(db, br.grad) < 1e-4


@pytest.mark.parametrize("M", [999, 16500])
def test_layernorm_bf16_dropout_acc(dev, M):
    """bf16 LayerNorm with input dropout, an accumulated residual gradient and the fused dx column sums (the
    engine's post-LN tail): the backward regenerates the forward's mask; matches the fp32 kernels run on the
    same bf16 values within bf16 rounding."""
    from k3m_amd import ops
    cols = 768
    x = torch.randn(M, cols, device=dev).bfloat16()
    r = torch.randn(M, cols, device=dev).bfloat16()
    g = 1 + 0.1 * torch.randn(cols, device=dev)
    b = 0.1 * torch.randn(cols, device=dev)
    dy = torch.randn(M, cols, device=dev).bfloat16()
    acc0 = torch.randn(M, cols, device=dev).bfloat16()
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        xx, rr, dd = x.to(dt), r.to(dt), dy.to(dt)
        y, xh = torch.empty_like(xx), torch.empty_like(xx)
        rs = torch.empty(M, device=dev)
        ops.ln_fwd(xx, rr, g, b, y, xh, rs, p_in=0.1, seed=9, off_in=123)
        dres, dx = acc0.to(dt).clone(), torch.empty_like(xx)
        dg, db, xs = (torch.zeros(cols, device=dev) for _ in range(3))
        ops.ln_bwd(dd, xh.to(dt), rs, g, dres, dx, dg, db, p_in=0.1, seed=9, off_in=123, acc_res=True, dxsum=xs)
        out[dt] = [t.float() for t in (y, dres, dx, dg, db, xs)]
    for a, c in zip(out[torch.bfloat16][:3], out[torch.float32][:3]):
        assert _rel(a, c) < 2.0 ** -6
    assert torch.equal(out[torch.bfloat16][2] == 0, out[torch.float32][2] == 0)   # the same dropout mask
    for a, c in zip(out[torch.bfloat16][3:], out[torch.float32][3:]):
        assert _rel(a, c) < 2e-2


def test_colsum_bf16(dev):
    from k3m_amd import ops
    x = torch.randn(20992, 768, device=dev).bfloat16()
    out = torch.randn(768, device=dev)
    ref = out + x.float().sum(0)
    ops.colsum(x, out, accumulate=True)
    assert _rel(out, ref) < 1e-5


@pytest.mark.parametrize("lq,lk,nh,hd", [(36, 36, 12, 64), (128, 128, 12, 64), (37, 37, 8, 128), (36, 37, 8, 128),
                                         (128, 36, 8, 96)])
def test_attention_bf16(dev, lq, lk, nh, hd):
    """bf16 q/k/v/ctx (fp32 softmax and probabilities) against fp32 math on the same bf16 inputs."""
    import math
    from k3m_amd import ops
    B, D = 5, nh * hd
    qkv_q = torch.randn(B * lq, 3 * D, device=dev).bfloat16()
    qkv_k = torch.randn(B * lk, 3 * D, device=dev).bfloat16()
    q, k, v = qkv_q[:, :D], qkv_k[:, D:2 * D], qkv_k[:, 2 * D:]
    m = torch.ones(B, lk, device=dev)
    m[:, lk - 3:] = 0
    mask = ((1 - m) * -10000).contiguous()
    ctx = torch.empty(B * lq, D, device=dev, dtype=torch.bfloat16)
    probs = torch.empty(B * nh * lq * lk, device=dev)
    ops.attn_fwd(q, k, v, mask, ctx, probs, B, lq, lk, nh, hd, 1 / math.sqrt(hd), 0.0, 0, 0)
    qr, kr, vr = [t.float().reshape(B, -1, D).clone().requires_grad_(True) for t in (q, k, v)]
    qh = qr.view(B, lq, nh, hd).permute(0, 2, 1, 3)
    kh = kr.view(B, lk, nh, hd).permute(0, 2, 1, 3)
    vh = vr.view(B, lk, nh, hd).permute(0, 2, 1, 3)
    p = torch.softmax(qh @ kh.transpose(-1, -2) / math.sqrt(hd) + mask[:, None, None, :], -1)
    cr = (p @ vh).permute(0, 2, 1, 3).reshape(B, lq, D)
    assert _rel(probs.view(B, nh, lq, lk), p) < 1e-4
    assert _rel(ctx.view(B, lq, D), cr) < 2.0 ** -7
    dctx = torch.randn(B * lq, D, device=dev).bfloat16()
    cr.backward(dctx.float().view(B, lq, D))
    dq, dk, dv = [torch.empty(B * n_, D, device=dev, dtype=torch.bfloat16) for n_ in (lq, lk, lk)]
    ops.attn_bwd(dctx, ctx, q, k, v, probs, dq, dk, dv, B, lq, lk, nh, hd, 1 / math.sqrt(hd), 0.0, 0, 0)
    # dS uses the bf16-rounded ctx in D = rowdot(dO, O): a few bf16 ulps of slack
    assert _rel(dq.view(B, lq, D), qr.grad) < 2e-2
    assert _rel(dk.view(B, lk, D), kr.grad) < 2e-2
    assert _rel(dv.view(B, lk, D), vr.grad) < 2.0 ** -6


@pytest.mark.parametrize("lq,lk,nh,hd", [(36, 36, 12, 64), (128, 128, 12, 64), (37, 37, 8, 128), (36, 37, 8, 128),
                                         (128, 37, 8, 128), (37, 128, 8, 128), (128, 36, 8, 128), (20, 90, 4, 64),
                                         (128, 36, 8, 96), (36, 128, 8, 96),
                                         (1, 5, 2, 64), (128, 101, 8, 128), (128, 128, 8, 128), (96, 128, 12, 64),
                                         (65, 128, 4, 64), (128, 128, 8, 96), (33, 64, 3, 64), (64, 64, 5, 64), (40, 17, 7, 64),
                                         # L > 128: attention_flash_long.hip (the config-5 shapes
                                         # PV 320 self-attention, PV <-> title d = 96, PV <-> image d = 128), ragged
                                         # and multi-key-group heads, the 512 maximum, a single query
                                         (320, 320, 12, 64), (36, 320, 8, 96), (320, 36, 8, 96), (320, 37, 8, 128),
                                         (37, 320, 8, 128), (512, 512, 2, 64), (200, 450, 3, 128), (450, 200, 2, 96),
                                         (129, 129, 4, 64), (1, 300, 2, 64), (300, 7, 2, 128), (256, 50, 12, 64)])
def test_flash_attention_bf16(dev, lq, lk, nh, hd):
    """LSE-saving bf16 attention (attention_bf16.hip; attention_flash_long.hip past 128) against fp32 math on the
    same bf16 inputs, and, with dropout on, against the probability-saving kernel drawing the same mask."""
    import math
    from k3m_amd import ops
    B, D = 5, nh * hd
    g = torch.Generator(device="cpu").manual_seed(lq * 131 + lk)
    qkv_q = torch.randn(B * lq, 3 * D, generator=g).to(dev).bfloat16()
    qkv_k = torch.randn(B * lk, 3 * D, generator=g).to(dev).bfloat16()
    q, k, v = qkv_q[:, :D], qkv_k[:, D:2 * D], qkv_k[:, 2 * D:]
    m = torch.ones(B, lk, device=dev)
    m[:, max(1, lk - 3):] = 0
    mask = ((1 - m) * -10000).contiguous()
    sc = 1 / math.sqrt(hd)
    ctx = torch.empty(B * lq, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh * lq, device=dev)
    ops.flash_attn_fwd(q, k, v, mask, ctx, lse, B, lq, lk, nh, hd, sc, 0.0, 0, 0)
    qr, kr, vr = [t.float().reshape(B, -1, D).clone().requires_grad_(True) for t in (q, k, v)]
    qh = qr.view(B, lq, nh, hd).permute(0, 2, 1, 3)
    kh = kr.view(B, lk, nh, hd).permute(0, 2, 1, 3)
    vh = vr.view(B, lk, nh, hd).permute(0, 2, 1, 3)
    sco = qh @ kh.transpose(-1, -2) * sc + mask[:, None, None, :]
    p = torch.softmax(sco, -1)
    cr = (p @ vh).permute(0, 2, 1, 3).reshape(B, lq, D)
    assert _rel(lse.view(B, nh, lq), torch.logsumexp(sco, -1)) < 1e-4
    assert _rel(ctx.view(B, lq, D), cr) < 2e-2
    dctx = torch.randn(B * lq, D, generator=g).to(dev).bfloat16()
    cr.backward(dctx.float().view(B, lq, D))
    dq, dk, dv = [torch.empty(B * n_, D, device=dev, dtype=torch.bfloat16) for n_ in (lq, lk, lk)]
    ops.flash_attn_bwd(dctx, ctx, q, k, v, mask, lse, dq, dk, dv, B, lq, lk, nh, hd, sc, 0.0, 0, 0)
    # P and dS are rounded to bf16 before the dV / dK products (the rest is fp32-accumulated)
    assert _rel(dq.view(B, lq, D), qr.grad) < 3e-2
    assert _rel(dk.view(B, lk, D), kr.grad) < 3e-2
    assert _rel(dv.view(B, lk, D), vr.grad) < 2e-2
    # dropout: same counter-based mask as the probability-saving kernel
    c1 = torch.empty_like(ctx)
    c2 = torch.empty_like(ctx)
    probs = torch.empty(B * nh * lq * lk, device=dev)
    ops.flash_attn_fwd(q, k, v, mask, c1, lse, B, lq, lk, nh, hd, sc, 0.1, 11, 5)
    ops.attn_fwd(q, k, v, mask, c2, probs, B, lq, lk, nh, hd, sc, 0.1, 11, 5)
    assert _rel(c1, c2) < 2e-2
    g1 = [torch.empty_like(t) for t in (dq, dk, dv)]
    g2 = [torch.empty_like(t) for t in (dq, dk, dv)]
    ops.flash_attn_bwd(dctx, c1, q, k, v, mask, lse, *g1, B, lq, lk, nh, hd, sc, 0.1, 11, 5)
    ops.attn_bwd(dctx, c2, q, k, v, probs, *g2, B, lq, lk, nh, hd, sc, 0.1, 11, 5)
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 4e-2


@pytest.mark.parametrize("lq,lk,nh,hd", [(320, 320, 4, 64), (37, 320, 8, 128), (100, 512, 2, 96)])
def test_flash_long_backward_deterministic(dev, lq, lk, nh, hd):
    """attention_flash_long.hip's backward has no atomics: heads split into key groups reduce their fp32 dQ partials
    in group order, so two runs are bit-identical (dropout on)."""
    import math
    from k3m_amd import ops
    B, D = 3, nh * hd
    g = torch.Generator(device="cpu").manual_seed(7)
    q = torch.randn(B * lq, D, generator=g).to(dev).bfloat16()
    k = torch.randn(B * lk, D, generator=g).to(dev).bfloat16()
    v = torch.randn(B * lk, D, generator=g).to(dev).bfloat16()
    mask = torch.zeros(B, lk, device=dev)
    mask[:, lk - 5:] = -10000.0
    ctx = torch.empty(B * lq, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh * lq, device=dev)
    sc = 1 / math.sqrt(hd)
    ops.flash_attn_fwd(q, k, v, mask, ctx, lse, B, lq, lk, nh, hd, sc, 0.1, 3, 17)
    dctx = torch.randn(B * lq, D, generator=g).to(dev).bfloat16()
    outs = []
    for _ in range(2):
        gr = [torch.full((B * n_, D), float("nan"), device=dev, dtype=torch.bfloat16) for n_ in (lq, lk, lk)]
        ops.flash_attn_bwd(dctx, ctx, q, k, v, mask, lse, *gr, B, lq, lk, nh, hd, sc, 0.1, 3, 17)
        outs.append(gr)
    for a, b in zip(*outs):
        assert torch.isfinite(a.float()).all()
        assert torch.equal(a, b)


_B16_WALK_SCRIPT = r'''
import sys, torch
sys.path.insert(0, sys.argv[2])
from k3m_amd import ops, _lib as L
dev = torch.device("cuda")
out = {}
torch.manual_seed(7)
bf = torch.bfloat16
# 256x256 and 256x128 forwards (bias, bias+GELU, ragged M), input gradients with and without dGELU, split-K
# weight gradients and a grouped launch, all in bf16 (the persistent walk's layouts and both MFMA shapes)
x = torch.randn(5000, 768, device=dev).to(bf); w = (torch.randn(3072, 768, device=dev) * 0.05).to(bf)
b = torch.randn(3072, device=dev)
pre = torch.empty(5000, 3072, device=dev, dtype=bf)
out["fwd_gelu"] = ops.linear(x, w, b, epi=L.EPI_BIAS_GELU, aux=pre); out["pre"] = pre
out["fwd_bias"] = ops.linear(x, w, b)
x2 = torch.randn(2368, 1024, device=dev).to(bf); w2 = (torch.randn(1024, 1024, device=dev) * 0.05).to(bf)
out["fwd_t128"] = ops.linear(x2, w2, b[:1024])
dy = torch.randn(5000, 3072, device=dev).to(bf); aux = torch.randn(5000, 768, device=dev).to(bf)
out["dgrad_dgelu"] = ops.linear_dgrad(dy, w, dgelu_aux=aux)
out["dgrad"] = ops.linear_dgrad(dy, w)
gw = torch.ones(3072, 768, device=dev)
ops.linear_wgrad(dy, x, gw); out["wgrad"] = gw
with ops.grouped():
    g1 = ops.linear(x2, w2, b[:1024]); g2 = ops.linear(x[:2304], w[:1024], b[:1024])
out["g1"], out["g2"] = g1, g2
torch.cuda.synchronize()
torch.save({k: v.float().cpu() for k, v in out.items()}, sys.argv[1])
'''


def test_b16_walk_variants_bit_identical(tmp_path):
    """The bf16 large-tile GEMMs compute every tile identically on the one-workgroup-per-tile grid
    (K3M_B16_PERSIST=0), the persistent walk (default), the persistent walk with the ping-pong main loop on
    every tile (K3M_B16_PP=7) and without the two-workgroups-per-CU GELU/dGELU kernel (K3M_B16_DUAL=0):
    same MFMA order per accumulator, so bit-identical C, pre-activations, slabs and grouped outputs.  The
    knobs are read at library load, so each setting runs in its own process."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "b16_walk_case.py"
    script.write_text(_B16_WALK_SCRIPT)
    res = {}
    for name, knobs in (("tile", {"K3M_B16_PERSIST": "0", "K3M_B16_DUAL": "0"}),
                        ("walk", {"K3M_B16_PERSIST": "1", "K3M_B16_PP": "0", "K3M_B16_DUAL": "0"}),
                        ("pp", {"K3M_B16_PERSIST": "1", "K3M_B16_PP": "7", "K3M_B16_DUAL": "0"})):
        path = str(tmp_path / ("out_%s.pt" % name))
        env = dict(os.environ, **knobs)
        subprocess.run([sys.executable, str(script), path, repo], check=True, env=env, timeout=240)
        res[name] = torch.load(path, weights_only=True)
    for name in ("walk", "pp"):
        for k in res["tile"]:
            assert torch.equal(res["tile"][k], res[name][k]), (name, k)


@pytest.mark.parametrize("lq,lk", [(320, 36), (36, 320)])
def test_flash_long_d96_matches_fixed_seed_golden(dev, lq, lk):
    """a fixed-seed fixture of the ragged 320 x 36 / 36 x 320 head-dim-96 co-attention with dropout, from
    this repository's exact-fp32 kernels (tests/golden/make_flash_long_golden.py; parity unpinned upstream: the
    reference's dropout draws cannot be reproduced).  The bf16 flash kernels (attention_flash_long.hip for the
    320-long side) must stay within the bf16 bars of test_flash_attention_bf16 of it."""
    import math
    import os
    import numpy as np
    from k3m_amd import ops
    import importlib.util
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    spec = importlib.util.spec_from_file_location("mflg", os.path.join(here, "make_flash_long_golden.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    gold = np.load(os.path.join(here, "flash_long_d96.npz"))
    B, NH, HD = int(gold["B"]), int(gold["NH"]), int(gold["HD"])
    p, seed, off = float(gold["p_drop"]), int(gold["seed"]), int(gold["off"])
    q, k, v, dctx, mask = mk.inputs(lq, lk, dev)
    D = NH * HD
    sc = 1 / math.sqrt(HD)
    ctx = torch.empty(B * lq, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * NH * lq, device=dev)
    ops.flash_attn_fwd(q, k, v, mask.contiguous(), ctx, lse, B, lq, lk, NH, HD, sc, p, seed, off)
    dq, dk, dv = [torch.empty(B * n_, D, device=dev, dtype=torch.bfloat16) for n_ in (lq, lk, lk)]
    ops.flash_attn_bwd(dctx, ctx, q, k, v, mask.contiguous(), lse, dq, dk, dv, B, lq, lk, NH, HD, sc, p, seed, off)
    torch.cuda.synchronize()
    tag = "%dx%d" % (lq, lk)
    for name, t, bar in (("ctx", ctx, 2e-2), ("dq", dq, 4e-2), ("dk", dk, 4e-2), ("dv", dv, 4e-2)):
        ref = torch.from_numpy(gold["%s/%s" % (tag, name)].astype(np.float32)).to(dev)
        assert _rel(t, ref) < bar, (tag, name, _rel(t, ref))


_FLASH_LONG_SCRIPT = r'''
import sys, math, torch
sys.path.insert(0, sys.argv[2])
from k3m_amd import ops
dev = torch.device("cuda")
out = {}
for (lq, lk, nh, hd, B) in ((320, 320, 4, 64, 3), (320, 36, 4, 96, 3), (37, 320, 4, 128, 2), (200, 450, 3, 128, 2),
                            (450, 200, 2, 96, 2), (1, 300, 2, 64, 2), (300, 7, 2, 128, 2), (129, 129, 4, 64, 2),
                            (512, 512, 2, 64, 1)):
    D = nh * hd
    g = torch.Generator(device="cpu").manual_seed(lq * 7 + lk)
    q = torch.randn(B * lq, D, generator=g).to(dev).bfloat16()
    k = torch.randn(B * lk, D, generator=g).to(dev).bfloat16()
    v = torch.randn(B * lk, D, generator=g).to(dev).bfloat16()
    mask = torch.zeros(B, lk, device=dev)
    mask[:, max(1, lk - 5):] = -10000.0
    ctx = torch.empty(B * lq, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh * lq, device=dev)
    sc = 1 / math.sqrt(hd)
    ops.flash_attn_fwd(q, k, v, mask, ctx, lse, B, lq, lk, nh, hd, sc, 0.1, 3, 17)
    dctx = torch.randn(B * lq, D, generator=g).to(dev).bfloat16()
    gr = [torch.full((B * n_, D), float("nan"), device=dev, dtype=torch.bfloat16) for n_ in (lq, lk, lk)]
    ops.flash_attn_bwd(dctx, ctx, q, k, v, mask, lse, *gr, B, lq, lk, nh, hd, sc, 0.1, 3, 17)
    for name, t in zip(("dq", "dk", "dv", "ctx", "lse"), gr + [ctx, lse]):
        out["%dx%dx%d_%s" % (lq, lk, hd, name)] = t.float().cpu()
torch.cuda.synchronize()
torch.save(out, sys.argv[1])
'''


def test_flash_long_bwd_dma_bit_identical_to_register_form(tmp_path):
    """attention_flash_long.hip's LDS-DMA forward and backward (K3M_FLASH_LONG_FWD / _BWD = 2, default) against the
    register-staged ones (= 1): same arithmetic, rows past lq / lk staged as clamped copies whose scores carry the -inf
    mask (forward) or whose P, Pd and dS are exactly 0 (backward), so the context, the LSE, dQ, dK and dV are
    bit-identical — config-5 shapes, multi-group heads (d = 96 / 128 past 224 keys), ragged, a single query, the 512
    maximum, dropout on.  The knobs are read at library load: one process per setting."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "flash_long_case.py"
    script.write_text(_FLASH_LONG_SCRIPT)
    res = {}
    for fwd, bwd in (("1", "1"), ("2", "1"), ("2", "2")):
        path = str(tmp_path / ("out_%s%s.pt" % (fwd, bwd)))
        env = dict(os.environ, K3M_FLASH_LONG_FWD=fwd, K3M_FLASH_LONG_BWD=bwd)
        subprocess.run([sys.executable, str(script), path, repo], check=True, env=env, timeout=240)
        res[fwd + bwd] = torch.load(path, weights_only=True)
    bad = []
    for x, y in (("11", "21"), ("21", "22")):   # the forward alone, then the backward alone
        for k in res[x]:
            a, b = res[x][k], res[y][k]
            assert torch.isfinite(b).all(), (y, k)
            if not torch.equal(a, b):
                bad.append((x, y, k, float((a - b).abs().max()), int((a != b).sum()), a.numel()))
    assert not bad, bad
