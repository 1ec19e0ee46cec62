"""fp32 GEMM accuracy: the default bf16x6 split kernels (include/k3m_hip.h K3M_F32_SPLIT_BF16X6) against
an fp64 GEMM of the same fp32 inputs, next to the exact-f32 MFMA kernels (K3M_F32_MFMA_F32).

The claim under test (k3m_amd/csrc/gemm_x6_tile.h): splitting each fp32 operand exactly into three
bf16 planes and accumulating the six leading partial products in fp32 gives fp32-level accuracy.
The bar: the split kernel's max and rms error vs fp64 are within 1.5x of the f32-MFMA kernel's
(in practice they are slightly SMALLER), on every layout, tile path, split-K and epilogue.
"""
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


def _errs(c, ref64):
    d = c.double().cpu() - ref64
    return float(d.abs().max()), float(d.pow(2).mean().sqrt())


def _case(dev, m, n, k, at, bt, splitk=1, seed=0):
    from k3m_amd import ops, _lib as L
    g = torch.Generator(device="cpu").manual_seed(seed + m + 3 * n + 7 * k)
    A = torch.rand(m, k, generator=g) * 2 - 1
    Bm = (torch.rand(k, n, generator=g) * 2 - 1) * 0.05
    ref = A.double() @ Bm.double()
    a = (A.t().contiguous() if at else A).to(dev)
    b = (Bm.t().contiguous() if bt else Bm).to(dev)
    out = {}
    for algo in (L.F32_SPLIT_BF16X6, L.F32_MFMA_F32):
        c = torch.zeros(m, n, device=dev)
        ws = torch.empty(splitk * m * n, device=dev) if splitk > 1 else None
        ops.gemm(a, at, b, bt, c, m, n, k, beta=1.0 if splitk > 1 else 0.0, splitk=splitk, ws=ws, f32_algo=algo)
        out[algo] = _errs(c, ref)
    scale = float(ref.abs().max())
    x6, f32 = out[L.F32_SPLIT_BF16X6], out[L.F32_MFMA_F32]
    assert x6[0] <= 1.5 * f32[0] + 1e-7 * scale, (x6, f32)
    assert x6[1] <= 1.5 * f32[1] + 1e-8 * scale, (x6, f32)
    assert x6[0] < 1e-5 * max(scale, 1.0)


@pytest.mark.parametrize("m,n,k", [(4096, 3072, 768),   # 256x256x16 tiles
                                   (4000, 3000, 772),   # 256x256x16, ragged M/N and a partial k-tile
                                   (20992, 768, 768),   # 256x256x16: one wave of 246 blocks instead of two of 256x128
                                   (2304, 2304, 768),   # 128x128x32 tiles
                                   (1024, 1024, 2048),  # 64x64x32 tiles
                                   (300, 200, 100)])    # ragged edges
@pytest.mark.parametrize("at,bt", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_x6_accuracy_vs_fp64(dev, m, n, k, at, bt):
    _case(dev, m, n, k, at, bt)


@pytest.mark.parametrize("splitk", [3, 5])
def test_x6_splitk_accuracy(dev, splitk):
    _case(dev, 768, 1024, 20000, 1, 0, splitk=splitk)


@pytest.mark.parametrize("at,bt", [(1, 0), (0, 0), (0, 1)])
def test_x6_splitk_256x256(dev, at, bt):
    # the weight-gradient shape (3072 x 768 over 20k rows, split 7) runs on 256x256x16 tiles
    _case(dev, 3072, 768, 20000, at, bt, splitk=7)


def test_x6_splitk_fill_rule(dev):
    """The image-stream weight gradient (1,024 x 1,024 over 4,736 rows) under ops._splitk's fill rule: 8 slices
    of 592 rows (the default minimum would give 4, half the CUs idle); the last slice shorter, none empty."""
    from k3m_amd import ops
    s = ops._splitk(1024, 1024, 4736, torch.float32)
    assert s == (8 if ops.SPLITK_FILL else 4)
    assert ops._splitk(1024, 1024, 4736, torch.float32, grouped=True) == 4
    _case(dev, 1024, 1024, 4736, 1, 0, splitk=s)


def test_x6_epilogues_match_torch(dev):
    from k3m_amd import ops, _lib as L
    x = torch.randn(2048, 768, device=dev)
    W = torch.randn(3072, 768, device=dev) * 0.05
    b = torch.randn(3072, device=dev)
    pre = torch.empty(2048, 3072, device=dev)
    y = ops.linear(x, W, b, epi=L.EPI_BIAS_GELU, aux=pre)
    r = (x.double() @ W.double().t() + b.double()).float()
    assert float((pre - r).abs().max()) < 1e-5 * float(r.abs().max())
    assert float((y - torch.nn.functional.gelu(r)).abs().max()) < 2e-5 * float(r.abs().max())
    dy = torch.randn(2048, 3072, device=dev)
    aux = torch.randn(2048, 768, device=dev)
    dx = ops.linear_dgrad(dy, W, dgelu_aux=aux)
    xr = aux.clone().requires_grad_(True)
    torch.nn.functional.gelu(xr).backward((dy.double() @ W.double()).float())
    assert float((dx - xr.grad).abs().max()) < 2e-5 * float(xr.grad.abs().max())


@pytest.mark.parametrize("m,n,k", [(4096, 3072, 768), (4000, 3000, 772), (20992, 768, 768), (8192, 3072, 768),
                                   (2304, 2304, 768), (1000, 3072, 768), (1024, 1024, 2048)])
@pytest.mark.parametrize("at,bt", [(0, 1), (0, 0), (1, 0), (1, 1)])
def test_x6_beta_all_tiles(dev, m, n, k, at, bt):
    """C = alpha*op(A)op(B) + beta*C on every x6 tile path (256x256, 256x128, 128x128, 64x64), repeated: the
    read-modify-write of C must see the old value in every lane (regression for a 64x64 BK=32 build)."""
    from k3m_amd import ops, _lib as L
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n + k)
    A = torch.randn(m, k, generator=g)
    Bm = torch.randn(k, n, generator=g)
    C0 = torch.randn(m, n, generator=g)
    ref = 0.5 * (A.double() @ Bm.double()) + 0.25 * C0.double()
    a = (A.t().contiguous() if at else A).to(dev)
    b = (Bm.t().contiguous() if bt else Bm).to(dev)
    c0 = C0.to(dev)
    for _ in range(5):
        c = c0.clone()
        ops.gemm(a, at, b, bt, c, m, n, k, alpha=0.5, beta=0.25, f32_algo=L.F32_SPLIT_BF16X6)
        err = float((c.double().cpu() - ref).abs().max())
        assert err < 2e-5 * float(ref.abs().max()), err


def test_grouped_matches_individual(monkeypatch):
    """k3m_gemm_grouped (one grid over several problems, in any problem order: K3M_GROUP_LPT) is bit-identical to
    launching each problem through k3m_gemm with the same split: same tile computation, split-K slabs and
    epilogues.  (ops._splitk's fill rule gives an UNgrouped under-filled weight gradient more k-slices than the
    grouped call, a different fp32 summation order; it is held off here.)"""
    import torch
    from k3m_amd import ops, _lib as L
    monkeypatch.setattr(ops, "SPLITK_FILL", False)
    monkeypatch.setattr(ops, "SMALL_SPLITK", False)   # grouped problems are never auto-split
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cases = [  # (m, n, k, epi) nt forward problems of the co-attention blocks, ragged edges included
        (2368, 3072, 1024, L.EPI_BIAS), (2304, 3072, 768, L.EPI_BIAS), (8192, 2304, 768, L.EPI_BIAS),
        (300, 200, 96, L.EPI_BIAS), (2304, 1024, 1024, L.EPI_BIAS)]
    for grouped in (False, True):
        outs = []
        torch.manual_seed(1)
        ins = [(torch.randn(m, k, device=dev), torch.randn(n, k, device=dev) * 0.05, torch.randn(n, device=dev))
               for m, n, k, _ in cases]
        if grouped:
            with ops.grouped():
                for (x, w, b), (m, n, k, epi) in zip(ins, cases):
                    outs.append(ops.linear(x, w, b))
        else:
            for (x, w, b), (m, n, k, epi) in zip(ins, cases):
                outs.append(ops.linear(x, w, b))
        torch.cuda.synchronize()
        if not grouped:
            ref = outs
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)
    # weight gradients (tn, split-K, beta = 1) and input gradients with the dGELU epilogue (nn)
    dys = [torch.randn(20992 if i == 0 else 2304, n, device=dev) for i, n in enumerate((768, 1024, 3072))]
    xs = [torch.randn(dy.shape[0], k, device=dev) for dy, k in zip(dys, (3072, 1024, 768))]
    res = {}
    for grouped in (False, True):
        torch.manual_seed(2)
        gws = [torch.ones(dy.shape[1], x.shape[1], device=dev) for dy, x in zip(dys, xs)]
        ws_ = [torch.randn(dy.shape[1], x.shape[1], device=dev) * 0.05 for dy, x in zip(dys, xs)]
        auxs = [torch.randn(dy.shape[0], x.shape[1], device=dev) for dy, x in zip(dys, xs)]
        if grouped:
            with ops.grouped():
                for dy, x, gw in zip(dys, xs, gws):
                    ops.linear_wgrad(dy, x, gw)
                dxs = [ops.linear_dgrad(dy, w, dgelu_aux=a) for dy, w, a in zip(dys, ws_, auxs)]
        else:
            for dy, x, gw in zip(dys, xs, gws):
                ops.linear_wgrad(dy, x, gw)
            dxs = [ops.linear_dgrad(dy, w, dgelu_aux=a) for dy, w, a in zip(dys, ws_, auxs)]
        torch.cuda.synchronize()
        res[grouped] = (gws, dxs)
    for a, b in zip(res[True][0] + res[True][1], res[False][0] + res[False][1]):
        assert torch.equal(a, b)


_PERSIST_SCRIPT = r'''
import sys, torch
sys.path.insert(0, sys.argv[2])
from k3m_amd import ops, _lib as L
dev = torch.device("cuda")
out = {}
torch.manual_seed(5)
# forward with bias+GELU (256x256 persistent walk, ragged M), dgrad with dGELU, split-K weight gradient,
# a 256x128 problem and a grouped launch
x = torch.randn(5000, 768, device=dev); w = torch.randn(3072, 768, device=dev) * 0.05; b = torch.randn(3072, device=dev)
pre = torch.empty(5000, 3072, device=dev)
out["fwd"] = ops.linear(x, w, b, epi=L.EPI_BIAS_GELU, aux=pre); out["pre"] = pre
dy = torch.randn(5000, 3072, device=dev); aux = torch.randn(5000, 768, device=dev)
out["dgrad"] = ops.linear_dgrad(dy, w, dgelu_aux=aux)
gw = torch.ones(3072, 768, device=dev)
ops.linear_wgrad(dy, x, gw); out["wgrad"] = gw
x2 = torch.randn(2368, 1024, device=dev); w2 = torch.randn(1024, 1024, device=dev) * 0.05; b2 = torch.randn(1024, device=dev)
out["t128"] = ops.linear(x2, w2, b2)
with ops.grouped():
    g1 = ops.linear(x2, w2, b2); g2 = ops.linear(x[:2304], w[:1024], b[:1024])
out["g1"], out["g2"] = g1, g2
# k not a multiple of the k-tile (a partial last k-tile on every layout), and a split-K slice edge
x3 = torch.randn(3000, 1000, device=dev); w3 = torch.randn(2304, 1000, device=dev) * 0.05
out["ktail_fwd"] = ops.linear(x3, w3, None)
dy3 = torch.randn(3000, 2304, device=dev)
out["ktail_dgrad"] = ops.linear_dgrad(dy3, w3)
gw3 = torch.zeros(2304, 1000, device=dev)
ops.linear_wgrad(dy3[:2996], x3[:2996], gw3); out["ktail_wgrad"] = gw3
x4 = torch.randn(2500, 776, device=dev); w4 = torch.randn(1024, 776, device=dev) * 0.05
out["ktail_t128"] = ops.linear(x4, w4, None)
torch.cuda.synchronize()
torch.save({k: v.cpu() for k, v in out.items()}, sys.argv[1])
'''


def test_persistent_walk_bit_identical(tmp_path):
    """The persistent x6 walk (gemm_x6p.hip, K3M_X6_PERSIST=1, default) computes every tile exactly as the
    one-workgroup-per-tile kernels (K3M_X6_PERSIST=0): bit-identical C, aux, split-K sums and grouped
    outputs, and so do the persistent walks with the ping-pong main loops (K3M_X6_PP=63: every layout and tile, the
    256x256 weight-gradient walk on the LDS-DMA-staged form; K3M_X6_PP=127: every 256x256 walk on it)
    and with it off (K3M_X6_PP=0).  The knobs are read at library load, so each setting runs in its own
    process."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "persist_case.py"
    script.write_text(_PERSIST_SCRIPT)
    res = {}
    for name, knobs in (("tile", {"K3M_X6_PERSIST": "0"}), ("walk", {"K3M_X6_PERSIST": "1", "K3M_X6_PP": "0"}),
                        ("pp", {"K3M_X6_PERSIST": "1", "K3M_X6_PP": "63"}),
                        ("ppd", {"K3M_X6_PERSIST": "1", "K3M_X6_PP": "127"})):
        path = str(tmp_path / ("out_%s.pt" % name))
        env = dict(os.environ, **knobs)
        subprocess.run([sys.executable, str(script), path, repo], check=True, env=env, timeout=240)
        res[name] = torch.load(path, weights_only=True)
    for name in ("walk", "pp", "ppd"):
        for k in res["tile"]:
            assert torch.equal(res["tile"][k], res[name][k]), (name, k)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("m,n,k", [(5000, 3072, 768),    # 256x256 persistent input-gradient walk, ragged M
                                   (20992, 768, 3072),   # the text FFN2 -> dGELU shape
                                   (2304, 1024, 3072),   # 256x128 / 128x128 tiles
                                   (700, 300, 200)])     # small tiles, ragged everything
def test_dgelu_colsum_slabs(dev, dtype, m, n, k):
    """K3M_GEMM_COLSUM_SLABS: the dGELU input gradient also leaves the column sums of its output as 32-row
    slabs (the bias gradient of the Linear it feeds): their sum equals the column sums of the stored C."""
    from k3m_amd import ops, _lib as L
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    dy = torch.randn(m, k, generator=g).to(dev).to(tdt)
    W = (torch.randn(k, n, generator=g) * 0.05).to(dev).to(tdt)
    aux = torch.randn(m, n, generator=g).to(dev).to(tdt)
    ns = (m + 31) // 32
    ws = torch.full((ns * n,), float("nan"), device=dev)
    c = torch.empty(m, n, device=dev, dtype=tdt)
    ops.gemm(dy, 0, W, 0, c, m, n, k, L.EPI_DGELU | L.GEMM_COLSUM_SLABS, None, aux, 1.0, 0.0, 1, ws)
    c_ref = torch.empty(m, n, device=dev, dtype=tdt)
    ops.gemm(dy, 0, W, 0, c_ref, m, n, k, L.EPI_DGELU, None, aux, 1.0, 0.0)
    torch.cuda.synchronize()
    assert torch.equal(c, c_ref)                       # the flag does not change C
    slabs = ws.view(ns, n)
    assert torch.isfinite(slabs).all()                 # every slab row written, including the ragged last one
    ref = c.double().sum(0)
    got = slabs.double().sum(0)
    assert float((got - ref).abs().max()) <= 1e-5 * float(ref.abs().max()) + 1e-6
    # per 32-row group
    grp = torch.nn.functional.pad(c.double(), (0, 0, 0, ns * 32 - m)).view(ns, 32, n).sum(1)
    assert float((slabs.double() - grp).abs().max()) <= 1e-5 * float(grp.abs().max()) + 1e-6


@pytest.mark.parametrize("m,n,k", [(64, 768, 768), (64, 1024, 1024), (389, 1024, 2048), (389, 1024, 1601),
                                   (100, 300, 2048), (1, 768, 640), (5, 300, 1500)])
@pytest.mark.parametrize("epi", ["none", "bias", "gelu", "dgelu", "sigmoid", "beta"])
def test_small_splitk_epilogues(dev, m, n, k, epi):
    """Small fp32 products split over k automatically (ops.small_splitk): the epilogue the caller
    asked for runs in the split-K reduction, with the unsplit kernel's element formulas; compared with the unsplit
    launch (K3M_SMALL_SPLITK off) and with fp64."""
    import math
    from k3m_amd import ops, _lib as L
    assert ops.small_splitk(m, n, k) > 1
    g = torch.Generator(device="cpu").manual_seed(m + n + k)
    A = (torch.rand(m, k, generator=g) * 2 - 1).to(dev)
    W = ((torch.rand(n, k, generator=g) * 2 - 1) * 0.05).to(dev)
    bias = (torch.rand(n, generator=g) - 0.5).to(dev)
    aux0 = torch.randn(m, n, generator=g).to(dev)
    c0 = torch.randn(m, n, generator=g).to(dev)
    E = {"none": L.EPI_NONE, "bias": L.EPI_BIAS, "gelu": L.EPI_BIAS_GELU, "dgelu": L.EPI_DGELU,
         "sigmoid": L.EPI_BIAS_SIGMOID, "beta": L.EPI_BIAS}[epi]
    alpha, beta = (0.7, 0.5) if epi == "beta" else (1.0, 0.0)

    def run(small):
        old = ops.SMALL_SPLITK
        ops.SMALL_SPLITK = small
        try:
            c = c0.clone()
            aux = aux0.clone()
            ops.gemm(A, 0, W, 1, c, m, n, k, E, bias if E in (L.EPI_BIAS, L.EPI_BIAS_GELU, L.EPI_BIAS_SIGMOID) else None,
                     aux if E in (L.EPI_BIAS_GELU, L.EPI_DGELU) else None, alpha, beta)
        finally:
            ops.SMALL_SPLITK = old
        torch.cuda.synchronize()
        return c.double().cpu(), aux.double().cpu()
    cs, auxs = run(True)
    cu, auxu = run(False)
    p = A.double().cpu() @ W.double().cpu().t()
    b64 = bias.double().cpu()
    erf = torch.special.erf
    if E == L.EPI_NONE:
        ref = p
    elif E == L.EPI_BIAS:
        ref = alpha * (p + b64) + beta * c0.double().cpu()
    elif E == L.EPI_BIAS_GELU:
        ref = 0.5 * (p + b64) * (1 + erf((p + b64) / math.sqrt(2)))
        assert float((auxs - (p + b64)).abs().max()) < 1e-5 * float((p + b64).abs().max())
    elif E == L.EPI_DGELU:
        x = aux0.double().cpu()
        ref = p * (0.5 * (1 + erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi))
    else:
        ref = torch.sigmoid(p + b64)
    scale = float(ref.abs().max())
    assert float((cs - ref).abs().max()) < 1e-5 * scale, epi
    assert float((cs - cu).abs().max()) < 1e-5 * scale, epi   # the split and the unsplit launch agree


@pytest.mark.parametrize("small", [True, False])
@pytest.mark.parametrize("at,bt", [(1, 0), (0, 0), (0, 1), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(1024, 5, 2368), (300, 8, 700), (77, 1, 256), (64, 3, 9000)])
def test_skinny_gemm(dev, m, n, k, at, bt, small, monkeypatch):
    """n <= 8 fp32 products (the image-location weight gradient, tn 1024 x 5 x 2,368) on the skinny kernel, whole
    and split over k into slabs (ops.small_splitk): exact fp32 FMAs against fp64, alpha / beta, run-to-run
    bit-identical."""
    from k3m_amd import ops
    monkeypatch.setattr(ops, "SMALL_SPLITK", small)
    g = torch.Generator(device="cpu").manual_seed(m * 7 + n)
    A = torch.rand(m, k, generator=g) * 2 - 1
    Bm = torch.rand(k, n, generator=g) * 2 - 1
    c0 = torch.randn(m, n, generator=g)
    a = (A.t().contiguous() if at else A).to(dev)
    b = (Bm.t().contiguous() if bt else Bm).to(dev)
    outs = []
    for _ in range(2):
        c = c0.clone().to(dev)
        ops.gemm(a, at, b, bt, c, m, n, k, alpha=0.5, beta=1.0)
        torch.cuda.synchronize()
        outs.append(c.cpu())
    ref = 0.5 * (A.double() @ Bm.double()) + c0.double()
    assert torch.equal(outs[0], outs[1])
    assert float((outs[0].double() - ref).abs().max()) < 1e-5 * float(ref.abs().max())


def test_skinny_split_epilogue(dev):
    """A split skinny product with the bias + GELU epilogue applied in the split-K reduction."""
    from k3m_amd import ops, _lib as L
    assert ops.small_splitk(1024, 5, 2368) > 1
    g = torch.Generator(device="cpu").manual_seed(5)
    x = (torch.rand(1024, 2368, generator=g) * 2 - 1).to(dev)
    W = (torch.rand(5, 2368, generator=g) * 0.1 - 0.05).to(dev)
    b = torch.randn(5, generator=g).to(dev)
    pre = torch.empty(1024, 5, device=dev)
    y = ops.linear(x, W, b, epi=L.EPI_BIAS_GELU, aux=pre)
    r = x.double() @ W.double().t() + b.double()
    assert float((pre.double() - r).abs().max()) < 1e-5 * float(r.abs().max())
    ref = torch.nn.functional.gelu(r)
    assert float((y.double() - ref).abs().max()) < 1e-5 * float(ref.abs().max())
