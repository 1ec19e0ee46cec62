"""Debug: the test_gemm_layouts case with alpha/beta, against fp64 and against torch's own fp32 GEMM."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from k3m_amd import ops, _lib as L

L.load()
m, n, k, at, bt = [int(x) for x in sys.argv[1:6]]
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(m * 7 + n + k)
A = torch.randn(m, k, generator=g).to(dev)
Bm = torch.randn(k, n, generator=g).to(dev)
a = A.t().contiguous() if at else A
b = Bm.t().contiguous() if bt else Bm
c0 = torch.randn(m, n, device=dev)
ref64 = 0.5 * (A.double() @ Bm.double()) + 0.25 * c0.double()
reft = 0.5 * (A @ Bm) + 0.25 * c0
print("torch fp32 vs fp64: max err %.3e (max|ref| %.3e)" % (float((reft.double() - ref64).abs().max()), float(ref64.abs().max())))
for algo in (L.F32_SPLIT_BF16X6, L.F32_MFMA_F32):
    c = c0.clone()
    ops.gemm(a, at, b, bt, c, m, n, k, alpha=0.5, beta=0.25, f32_algo=algo)
    d = (c.double() - ref64).abs()
    bad = (d > 1e-4 * ref64.abs().max()).nonzero().cpu()
    print("algo", algo, "max err %.3e" % float(d.max()), "bad", bad.shape[0],
          "rows", sorted(set(bad[:, 0].tolist()))[:12], "cols", sorted(set(bad[:, 1].tolist()))[:12])
# same data, alpha=1, beta=0
ref1 = A.double() @ Bm.double()
for trial in range(3):
    c = torch.zeros(m, n, device=dev)
    ops.gemm(a, at, b, bt, c, m, n, k, f32_algo=L.F32_SPLIT_BF16X6)
    d = (c.double() - ref1).abs()
    bad = (d > 1e-4 * ref1.abs().max()).nonzero().cpu()
    print("beta0 trial", trial, "max err %.3e" % float(d.max()), "bad", bad.shape[0],
          "rows", sorted(set(bad[:, 0].tolist()))[:12], "cols", sorted(set(bad[:, 1].tolist()))[:12])
    if bad.shape[0]:
        i, j = bad[0].tolist()
        print("   example", i, j, float(c[i, j]), float(ref1[i, j]))
