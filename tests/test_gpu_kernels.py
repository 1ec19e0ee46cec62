"""Per-kernel numerics on the GPU against plain PyTorch fp32 references of the same op."""
import math

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
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("m,n,k", [(128, 128, 64), (300, 200, 100), (2368, 1024, 2048), (37, 1601, 1024),
                                   (64, 768, 5), (1000, 3072, 768)])
@pytest.mark.parametrize("at,bt", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_gemm_layouts(dev, m, n, k, at, bt):
    from k3m_amd import ops
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n + k)
    A = torch.randn(m, k, generator=g).to(dev)
    Bm = torch.randn(k, n, generator=g).to(dev)
    a = A.t().contiguous() if at else A
    b = Bm.t().contiguous() if bt else Bm
    c = torch.randn(m, n, device=dev)
    ref = 0.5 * (A @ Bm) + 0.25 * c
    ops.gemm(a, at, b, bt, c, m, n, k, alpha=0.5, beta=0.25)
    assert _rel(c, ref) < 1e-5


@pytest.mark.parametrize("splitk", [2, 5])
def test_gemm_splitk(dev, splitk):
    from k3m_amd import ops
    m, n, k = 768, 768, 20000
    A = torch.randn(k, m, device=dev)
    Bm = torch.randn(k, n, device=dev)
    c = torch.randn(m, n, device=dev)
    ref = A.t() @ Bm + c
    ws = torch.empty(splitk * m * n, device=dev)
    ops.gemm(A, 1, Bm, 0, c, m, n, k, beta=1.0, splitk=splitk, ws=ws)
    assert _rel(c, ref) < 1e-5


def test_gemm_epilogues(dev):
    from k3m_amd import ops, _lib as L
    x = torch.randn(500, 768, device=dev)
    W = torch.randn(3072, 768, device=dev) * 0.05
    b = torch.randn(3072, device=dev)
    pre = torch.empty(500, 3072, device=dev)
    y = ops.linear(x, W, b, epi=L.EPI_BIAS_GELU, aux=pre)
    r = x @ W.t() + b
    assert _rel(pre, r) < 1e-5
    assert _rel(y, torch.nn.functional.gelu(r)) < 1e-5
    s = ops.linear(x, W, b, epi=L.EPI_BIAS_SIGMOID)
    assert _rel(s, torch.sigmoid(r)) < 1e-5
    dy = torch.randn(500, 3072, device=dev)
    W2 = torch.randn(3072, 768, device=dev) * 0.05
    d = ops.linear_dgrad(dy, W2)
    assert _rel(d, dy @ W2) < 1e-5
    pre2 = torch.randn(500, 768, device=dev)
    dx = ops.linear_dgrad(dy, W, dgelu_aux=pre2)
    xr = pre2.clone().requires_grad_(True)
    torch.nn.functional.gelu(xr).backward(dy @ W)
    assert _rel(dx, xr.grad) < 1e-5


def test_gelu_accuracy_fp64(dev):
    """The branch-free erfc-form GELU / dGELU (common.h phi_cdf) against float64 erf over [-12, 12]: the
    epilogue GELU (a GEMM with an identity weight) and the elementwise dGELU kernel.  Bounds: absolute 5e-7
    everywhere, relative 2e-5 for |x| < 5 (the erff form's 1 + erf cancels to ~5 % relative in the left tail)."""
    from k3m_amd import ops, _lib as L
    x = torch.linspace(-12, 12, 64 * 1024, device=dev, dtype=torch.float64)
    xf = x.float().reshape(-1, 64).contiguous()
    eye = torch.eye(64, device=dev)
    pre = torch.empty_like(xf)
    y = ops.linear(xf, eye, torch.zeros(64, device=dev), epi=L.EPI_BIAS_GELU, aux=pre)
    assert _rel(pre, xf) < 1e-7
    x64 = pre.double()           # the epilogue's input, whatever the GEMM rounded
    cdf = 0.5 * (1 + torch.erf(x64 / math.sqrt(2)))
    ref_g = x64 * cdf
    ref_d = cdf + x64 * torch.exp(-0.5 * x64 * x64) / math.sqrt(2 * math.pi)
    xf = pre
    err = (y.double() - ref_g).abs()
    assert float(err.max()) < 5e-7
    mid = x64.abs() < 5
    assert float((err[mid] / ref_g[mid].abs().clamp_min(1e-30)).max()) < 2e-5
    d = torch.empty_like(xf)
    ops.dgelu(torch.ones_like(xf), xf, d)
    derr = (d.double() - ref_d).abs()
    assert float(derr.max()) < 5e-7


def test_wgrad_colsum(dev):
    from k3m_amd import ops
    dy = torch.randn(20992, 768, device=dev)
    x = torch.randn(20992, 3072, device=dev)
    gW = torch.randn(768, 3072, device=dev)
    gb = torch.randn(768, device=dev)
    rW = gW + dy.t() @ x
    rb = gb + dy.sum(0)
    ops.linear_wgrad(dy, x, gW, gb)
    assert _rel(gW, rW) < 1e-5
    assert _rel(gb, rb) < 1e-5


def _ln_ref(s, g, b):
    u = s.mean(-1, keepdim=True)
    v = (s - u).pow(2).mean(-1, keepdim=True)
    return g * (s - u) / torch.sqrt(v + 1e-12) + b


@pytest.mark.parametrize("cols", [768, 1024])
def test_layernorm(dev, cols):
    from k3m_amd import ops
    M = 999
    x = torch.randn(M, cols, device=dev)
    r = torch.randn(M, cols, device=dev)
    g = 1 + 0.1 * torch.randn(cols, device=dev)
    b = 0.1 * torch.randn(cols, device=dev)
    y = torch.empty_like(x)
    xh = torch.empty_like(x)
    rs = torch.empty(M, device=dev)
    ops.ln_fwd(x, r, g, b, y, xh, rs)
    xr, rr, gr, br = [t.clone().requires_grad_(True) for t in (x, r, g, b)]
    yr = _ln_ref(xr + rr, gr, br)
    assert _rel(y, yr) < 1e-5
    dy = torch.randn_like(y)
    yr.backward(dy)
    dres = torch.empty_like(x)
    dg = torch.zeros(cols, device=dev)
    db = torch.zeros(cols, device=dev)
    xs = torch.ones(cols, device=dev)
    ops.ln_bwd(dy, xh, rs, g, dres, dres, dg, db, dxsum=xs)
    assert _rel(dres, xr.grad) < 1e-4
    assert _rel(dg, gr.grad) < 1e-4
    assert _rel(db, br.grad) < 1e-4
    assert _rel(xs, 1 + xr.grad.sum(0)) < 1e-4   # fused bias gradient of the producing Linear


@pytest.mark.parametrize("cols,acc,alias", [(768, False, True), (768, True, False), (1024, True, False)])
def test_layernorm_bwd_bf16_long(dev, cols, acc, alias):
    """The software-pipelined half-wave bf16 backward (norm.hip ln_bwd_bf16_kernel, rows >= 16,384, LDS column
    partials) against the LayerNorm backward in fp32 torch on the same bf16 inputs; 20,003 rows leave a ragged
    last grid step.  Also reduced by the one-call k3m_ln_bwd (slab_batch_kernel)."""
    from k3m_amd import ops
    M = 20003
    gen = torch.Generator(device="cpu").manual_seed(cols + acc)
    dy = torch.randn(M, cols, generator=gen).to(dev).bfloat16()
    xh = torch.randn(M, cols, generator=gen).to(dev).bfloat16()
    rs = (0.5 + torch.rand(M, generator=gen)).to(dev)
    g = (1 + 0.1 * torch.randn(cols, generator=gen)).to(dev)
    old = torch.randn(M, cols, generator=gen).to(dev).bfloat16()
    dres = old.clone()
    dx = dres if alias else torch.empty_like(dres)
    dg = torch.zeros(cols, device=dev)
    db = torch.zeros(cols, device=dev)
    xs = torch.zeros(cols, device=dev)
    ops.ln_bwd(dy, xh, rs, g, dres, dx, dg, db, acc_res=acc, dxsum=xs)
    d, x = dy.float(), xh.float()
    dxh = d * g
    ds = (dxh - dxh.mean(1, keepdim=True) - x * (dxh * x).mean(1, keepdim=True)) * rs[:, None]
    ref = ds + old.float() if acc else ds
    # bf16 outputs: one rounding of the fp32 value (2^-8 relative) on top of fp32 summation-order differences
    assert _rel(dres.float(), ref) < 5e-3
    if not alias:
        assert _rel(dx.float(), ds) < 5e-3
    assert _rel(dg, (d * x).sum(0)) < 1e-5
    assert _rel(db, d.sum(0)) < 1e-5
    assert _rel(xs, dx.float().sum(0)) < 1e-5   # the sum of dx as stored


@pytest.mark.parametrize("nslab", [2, 7, 9, 20])
def test_slab_reduce_batch_orders(dev, nslab):
    """k3m_slab_reduce_batch's split-K (vec) path: out (+)= slab 0 + slab 1 + ... in that order, bit-exact
    against the same left-to-right fp32 sum, for the slab counts the weight gradients use."""
    import ctypes as C
    from k3m_amd import _lib as L
    cols = 768 * 3072 + 4
    gen = torch.Generator(device="cpu").manual_seed(nslab)
    ws = torch.randn(nslab, cols, generator=gen).to(dev)
    out0 = torch.randn(cols, generator=gen).to(dev)
    outs = [out0.clone(), torch.empty_like(out0)]
    for acc, out in zip((1, 0), outs):
        n = 1
        wsp = (C.c_void_p * n)(ws.data_ptr())
        op = (C.c_void_p * n)(out.data_ptr())
        ns = (C.c_int * n)(nslab)
        cs = (C.c_int * n)(cols)
        ac = (C.c_int * n)(acc)
        L.call("k3m_slab_reduce_batch", C.cast(wsp, C.c_void_p), C.cast(op, C.c_void_p), C.cast(ns, C.c_void_p),
               C.cast(cs, C.c_void_p), C.cast(ac, C.c_void_p), n, L.stream())
    torch.cuda.synchronize()
    ref = ws[0].clone()
    for k in range(1, nslab):
        ref += ws[k]
    assert torch.equal(outs[1], ref)
    assert torch.equal(outs[0], out0 + ref)


def test_dropout_ln_regenerates_mask(dev):
    from k3m_amd import ops
    M, cols = 512, 768
    x = torch.randn(M, cols, device=dev)
    g = torch.ones(cols, device=dev)
    b = torch.zeros(cols, device=dev)
    y, xh = torch.empty_like(x), torch.empty_like(x)
    rs = torch.empty(M, device=dev)
    ops.ln_fwd(x, None, g, b, y, xh, rs, p_in=0.1, seed=5, off_in=77)
    dx, dres = torch.empty_like(x), torch.empty_like(x)
    dg, db = torch.zeros(cols, device=dev), torch.zeros(cols, device=dev)
    xs = torch.zeros(cols, device=dev)
    ops.ln_bwd(torch.randn_like(x), xh, rs, g, dres, dx, dg, db, p_in=0.1, seed=5, off_in=77, dxsum=xs)
    assert _rel(xs, dx.sum(0)) < 1e-4
    frac = float((dx == 0).float().mean())
    assert 0.08 < frac < 0.12
    ratio = dx[dx != 0] / dres[dx != 0]
    assert torch.allclose(ratio, torch.full_like(ratio, 1 / 0.9), rtol=1e-5)
    # the forward used the same mask: dropped inputs did not reach the LN sum
    s_ref = x.clone()
    s_ref[dx == 0] = 0
    s_ref = s_ref / 0.9 * (dx != 0) + 0 * s_ref
    assert _rel(y, _ln_ref(s_ref, g, b)) < 1e-4


def _attn_ref(q, k, v, mask, nh):
    B, Lq, D = q.shape
    Lk = k.shape[1]
    hd = D // nh
    qh = q.view(B, Lq, nh, hd).permute(0, 2, 1, 3)
    kh = k.view(B, Lk, nh, hd).permute(0, 2, 1, 3)
    vh = v.view(B, Lk, nh, hd).permute(0, 2, 1, 3)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(hd) + mask[:, None, None, :]
    p = torch.softmax(s, -1)
    return (p @ vh).permute(0, 2, 1, 3).reshape(B, Lq, D), p


@pytest.mark.parametrize("lq,lk,nh,hd", [(36, 36, 12, 64), (128, 128, 12, 64), (37, 37, 8, 128), (36, 37, 8, 128),
                                         (37, 128, 8, 128), (128, 36, 8, 96), (36, 128, 8, 96),
                                         # ragged d = 64 shapes of the bf16x6 key-major backward (attn_bwd_x6km_kernel)
                                         (65, 65, 4, 64), (100, 128, 3, 64), (33, 50, 2, 64), (128, 40, 2, 64),
                                         # d = 128 with up to 128 keys on the two-pass x6 forward staging
                                         (64, 128, 2, 128), (60, 97, 3, 128), (96, 65, 2, 128)])
def test_attention(dev, lq, lk, nh, hd):
    from k3m_amd import ops
    B = 5
    D = nh * hd
    qkv_q = torch.randn(B * lq, 3 * D, device=dev)
    qkv_k = torch.randn(B * lk, 3 * D, device=dev)
    q, k, v = qkv_q[:, :D], qkv_k[:, D:2 * D], qkv_k[:, 2 * D:]
    m = torch.ones(B, lk, device=dev)
    m[:, lk - 3:] = 0
    mask = ((1 - m) * -10000).contiguous()
    ctx = torch.empty(B * lq, D, device=dev)
    probs = torch.empty(B * nh * lq * lk, device=dev)
    ops.attn_fwd(q, k, v, mask, ctx, probs, B, lq, lk, nh, hd, 1 / math.sqrt(hd), 0.0, 0, 0)
    qr, kr, vr = [t.reshape(B, -1, D).clone().requires_grad_(True) for t in (q, k, v)]
    cr, pr = _attn_ref(qr, kr, vr, mask, nh)
    assert _rel(ctx.view(B, lq, D), cr) < 1e-5
    assert _rel(probs.view(B, nh, lq, lk), pr) < 1e-5
    dctx = torch.randn(B * lq, D, device=dev)
    cr.backward(dctx.view(B, lq, D))
    dq = torch.empty(B * lq, D, device=dev)
    dk = torch.empty(B * lk, D, device=dev)
    dv = torch.empty(B * lk, D, device=dev)
    ops.attn_bwd(dctx, ctx, q, k, v, probs, dq, dk, dv, B, lq, lk, nh, hd, 1 / math.sqrt(hd), 0.0, 0, 0)
    assert _rel(dq.view(B, lq, D), qr.grad) < 1e-4
    assert _rel(dk.view(B, lk, D), kr.grad) < 1e-4
    assert _rel(dv.view(B, lk, D), vr.grad) < 1e-4


def test_embedding(dev):
    from k3m_amd import ops
    V, H, B, Lx = 1000, 768, 4, 36
    word = torch.randn(V, H, device=dev)
    pos = torch.randn(512, H, device=dev)
    typ = torch.randn(2, H, device=dev)
    g = 1 + 0.1 * torch.randn(H, device=dev)
    b = 0.1 * torch.randn(H, device=dev)
    ids = torch.randint(0, V, (B, Lx), device=dev)
    ids[:, -5:] = 0
    tt = torch.randint(0, 2, (B, Lx), device=dev)
    y0, y1, xh = [torch.empty(B * Lx, H, device=dev) for _ in range(3)]
    rs = torch.empty(B * Lx, device=dev)
    ops.embed_fwd(ids, tt, word, pos, typ, g, b, y0, y1, None, xh, rs, 0.0, 0, 0)
    wr, pr, tr = [t.clone().requires_grad_(True) for t in (word, pos, typ)]
    e = torch.nn.functional.embedding(ids, wr, padding_idx=0) + pr[:Lx][None] + tr[tt]
    ref = _ln_ref(e, g, b).reshape(B * Lx, H)
    assert _rel(y0, ref) < 1e-5 and torch.equal(y0, y1)
    dy = torch.randn_like(y0)
    ref.backward(dy)
    ds = torch.empty_like(dy)
    dg = torch.zeros(H, device=dev)
    db = torch.zeros(H, device=dev)
    ops.ln_bwd(dy, xh, rs, g, ds, ds, dg, db)
    dw = torch.zeros_like(word)
    dp = torch.zeros_like(pos)
    dt = torch.zeros_like(typ)
    ops.embed_bwd(ids, tt, ds, dw, dp, dt)
    assert _rel(dw, wr.grad) < 1e-4 and _rel(dp, pr.grad) < 1e-4 and _rel(dt, tr.grad) < 1e-4


def test_adamw_matches_pytorch_transformers_semantics(dev):
    from k3m_amd import _lib as L
    from oracle.k3m_oracle import adamw_step
    n = 4096
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.randn(n, device=dev).abs() * 0.01
    v = torch.rand(n, device=dev) * 0.01
    pc, gc, mc, vc = [t.cpu().clone() for t in (p, g, m, v)]
    L.call("k3m_adamw", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), None, n, 1e-4, 0.9, 0.98, 1e-8,
           0.01, 3, 1.0, L.stream())
    adamw_step(pc, gc, mc, vc, 3, 1e-4, 0.01)
    torch.cuda.synchronize()
    assert torch.allclose(p.cpu(), pc, rtol=1e-6, atol=1e-7)
    assert torch.allclose(m.cpu(), mc, rtol=1e-6, atol=1e-8)
    assert torch.allclose(v.cpu(), vc, rtol=1e-6, atol=1e-9)
