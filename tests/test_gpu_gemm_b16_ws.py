"""The epilogue-wave bf16 GEMM (csrc/gemm_b16_ws.h, K3M_B16_WS): MFMA waves hand each 256 x 128 tile to four
epilogue waves through an LDS image while they go on with the next tile.  Same products, same accumulation order
and one bf16 rounding of (accumulator + bias) as the one-role kernels (gemm_b16_tile.h), so C and the GELU
pre-activation must be bit-identical to them on every eligible shape: the full FFN1 forward, ragged M and N, the
smallest eligible K (17 k-steps), long K, alpha, a grouped launch of unequal problems and a grid smaller than the
CU count.  The knob is read at library load, so each setting runs in its own process.  Plus a torch fp32 check of the
new path in the test process."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

_SCRIPT = r'''
import sys, torch
sys.path.insert(0, sys.argv[2])
from k3m_amd import ops, _lib as L
dev = torch.device("cuda")
bf = torch.bfloat16
out = {}
g = torch.Generator(device="cpu").manual_seed(11)
def rnd(*s, scale=1.0):
    return (torch.randn(*s, generator=g) * scale).to(dev).to(bf)
x = rnd(20992, 768); w = rnd(3072, 768, scale=0.05); b = torch.randn(3072, generator=g).to(dev)
pre = torch.empty(20992, 3072, device=dev, dtype=bf)
out["ffn1_gelu"] = ops.linear(x, w, b, epi=L.EPI_BIAS_GELU, aux=pre); out["ffn1_pre"] = pre
out["ragged_bias"] = ops.linear(x[:5000], w[:2304], b[:2304])
y = torch.empty(3001, 1000, device=dev, dtype=bf)
ops.gemm(x[:3001], 0, w[:1000], 1, y, 3001, 1000, 768, L.EPI_NONE, None, None, 0.5, 0.0); out["none_alpha"] = y
xk = rnd(4736, 544); wk = rnd(1024, 544, scale=0.05)
pk = torch.empty(4736, 1024, device=dev, dtype=bf)
out["kmin_gelu"] = ops.linear(xk, wk, b[:1024], epi=L.EPI_BIAS_GELU, aux=pk); out["kmin_pre"] = pk
x2 = rnd(20992, 3072); w2 = rnd(768, 3072, scale=0.02)
out["ffn2_bias"] = ops.linear(x2, w2, b[:768])
out["small_grid"] = ops.linear(x[:100], w[:512], b[:512])
xa, xb, xc = rnd(2368, 1024), rnd(8192, 768), rnd(2304, 768)
wa, wb, wc = rnd(1024, 1024, scale=0.05), rnd(3072, 768, scale=0.05), rnd(3072, 768, scale=0.05)
pa_, pb_, pc_ = [torch.empty(r, c, device=dev, dtype=bf) for r, c in ((2368, 1024), (8192, 3072), (2304, 3072))]
with ops.grouped():
    ga = ops.linear(xa, wa, b[:1024], epi=L.EPI_BIAS_GELU, aux=pa_)
    gb = ops.linear(xb, wb, b, epi=L.EPI_BIAS_GELU, aux=pb_)
    gc = ops.linear(xc, wc, b, epi=L.EPI_BIAS_GELU, aux=pc_)
out.update(grp_a=ga, grp_b=gb, grp_c=gc, grp_pa=pa_, grp_pb=pb_, grp_pc=pc_)
torch.cuda.synchronize()
torch.save({k: v.float().cpu() for k, v in out.items()}, sys.argv[1])
'''


def test_ws_kernel_bit_identical_to_one_role_kernels(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "ws_case.py"
    script.write_text(_SCRIPT)
    res = {}
    for name, knobs in (("one_role", {"K3M_B16_WS": "0"}), ("ws", {"K3M_B16_WS": "3"})):
        path = str(tmp_path / ("out_%s.pt" % name))
        env = dict(os.environ, **knobs)
        subprocess.run([sys.executable, str(script), path, repo], check=True, env=env, timeout=240)
        res[name] = torch.load(path, weights_only=True)
    for k in res["one_role"]:
        a, b = res["one_role"][k], res["ws"][k]
        assert torch.isfinite(b).all(), k
        assert torch.equal(a, b), (k, float((a - b).abs().max()))


def test_ws_kernel_matches_torch():
    """The default-knob path of this process against torch fp32 (whichever kernel the library's knob selects)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd import ops, _lib as L
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    m, n, k = 6000, 2304, 1024
    x = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn((n, k), device=dev, generator=g) * 0.05).to(torch.bfloat16)
    bias = torch.randn((n,), device=dev, generator=g)
    pre = torch.empty((m, n), dtype=torch.bfloat16, device=dev)
    y = ops.linear(x, w, bias, epi=L.EPI_BIAS_GELU, aux=pre)
    ref = x.float() @ w.float().t() + bias
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((pre.float() - ref).abs().max()) <= 1e-2 * scale
    assert float((y.float() - torch.nn.functional.gelu(pre.float())).abs().max()) <= 1e-2 * scale
