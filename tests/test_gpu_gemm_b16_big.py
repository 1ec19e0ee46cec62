"""The large-tile bf16 GEMM (csrc/gemm_b16_tile.h: 256x256 / 256x128 tiles, LDS-DMA staging,
v_mfma_f32_16x16x32_bf16) on the shapes of the bf16 encoder, every operand layout it takes, the
fused epilogues, split-K and the grouped launch — against a torch fp32 GEMM of the same bf16
operands.  Tolerances: fp32 C 2e-5 relative to the output scale (fp32 accumulation in a different
order); bf16 C 1e-2 (one bf16 rounding of the result)."""
import pytest
import torch

from k3m_amd import _lib as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _ref(a, at, b, bt):
    A = a.float().t() if at else a.float()
    B = b.float() if bt == 0 else b.float().t()
    return A @ B


def _check(got, ref, tol):
    err = float((got.float() - ref).abs().max())
    scale = float(ref.abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("m,n,k", [(20992, 3072, 768), (4736, 1000, 1024), (8192, 2304, 768), (2368, 3072, 1024)])
def test_forward_kc_kc(dev, m, n, k):
    from k3m_amd import ops
    g = torch.Generator(device=dev).manual_seed(m + n)
    x = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn((n, k), device=dev, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn((n,), device=dev, generator=g)
    ref = _ref(x, 0, w, 1) + bias
    y = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    pre = torch.empty_like(y)
    ops.gemm(x, 0, w, 1, y, m, n, k, L.EPI_BIAS_GELU, bias, pre)
    y32 = torch.empty((m, n), dtype=torch.float32, device=dev)
    ops.gemm(x, 0, w, 1, y32, m, n, k, L.EPI_BIAS, bias)
    torch.cuda.synchronize()
    _check(y32, ref, 2e-5)
    _check(pre, ref, 1e-2)
    _check(y, torch.nn.functional.gelu(pre.float()), 1e-2)


@pytest.mark.parametrize("m,n,k", [(20992, 768, 3072), (4736, 1024, 1024), (2304, 768, 1024)])
def test_dgrad_kc_mn(dev, m, n, k):
    """dx = dy . W (B MN-contiguous), plain and with the dGELU epilogue, beta = 1 accumulation."""
    from k3m_amd import ops
    g = torch.Generator(device=dev).manual_seed(m)
    dy = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn((k, n), device=dev, generator=g) * 0.05).to(torch.bfloat16)
    ref = _ref(dy, 0, w, 0)
    c0 = torch.randn((m, n), device=dev, generator=g).to(torch.bfloat16)
    c = c0.clone()
    ops.gemm(dy, 0, w, 0, c, m, n, k, L.EPI_NONE, None, None, 1.0, 1.0)
    aux = torch.randn((m, n), device=dev, generator=g).to(torch.bfloat16)
    d = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    ops.gemm(dy, 0, w, 0, d, m, n, k, L.EPI_DGELU, None, aux)
    torch.cuda.synchronize()
    _check(c, ref + c0.float(), 1e-2)
    x = aux.float()
    dg = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    _check(d, ref * dg, 1e-2)


@pytest.mark.parametrize("n,k,m,splitk", [(3072, 768, 20992, 1), (3072, 768, 20992, 7), (1024, 1024, 4736, 4),
                                          (1024, 1024, 4736, 7),   # ops._splitk fill rule: 256 x 128 tiles, last slice short
                                          (768, 768, 2304, 3)])
def test_wgrad_mn_mn(dev, n, k, m, splitk):
    """gW[n,k] += alpha dy^T x (both MN-contiguous), fp32 C, split-K slabs."""
    from k3m_amd import ops
    g = torch.Generator(device=dev).manual_seed(n + splitk)
    dy = torch.randn((m, n), device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
    gw0 = torch.randn((n, k), device=dev, generator=g)
    gw = gw0.clone()
    ws = torch.empty((splitk * n * k,), dtype=torch.float32, device=dev) if splitk > 1 else None
    ops.gemm(dy, 1, x, 0, gw, n, k, m, L.EPI_NONE, None, None, 0.5, 1.0, splitk, ws)
    torch.cuda.synchronize()
    _check(gw, 0.5 * _ref(dy, 1, x, 0) + gw0, 2e-5)


def test_grouped_launch(dev):
    """Co-attention stage shapes in one grouped grid (k3m_gemm_grouped), bf16 C with bias."""
    from k3m_amd import ops
    g = torch.Generator(device=dev).manual_seed(7)
    probs = [(2304, 1024, 768), (8192, 1024, 768), (2368, 3072, 1024), (2304, 2304, 768)]
    outs, refs = [], []
    with ops.grouped():
        for m, n, k in probs:
            x = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
            w = (torch.randn((n, k), device=dev, generator=g) * 0.05).to(torch.bfloat16)
            b = torch.randn((n,), device=dev, generator=g)
            y = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
            ops.gemm(x, 0, w, 1, y, m, n, k, L.EPI_BIAS, b)
            outs.append(y)
            refs.append(_ref(x, 0, w, 1) + b)
    torch.cuda.synchronize()
    for y, r in zip(outs, refs):
        _check(y, r, 1e-2)
