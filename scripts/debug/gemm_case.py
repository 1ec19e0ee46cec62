"""Debug one GEMM case: error pattern of the fp32 paths against an fp64 reference."""
import sys
import os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from k3m_amd import ops, _lib as L

L.load()
m, n, k, at, bt = [int(x) for x in sys.argv[1:6]]
dev = torch.device("cuda")
g = torch.Generator(device="cpu").manual_seed(1)
A = torch.randn(m, k, generator=g)
Bm = torch.randn(k, n, generator=g)
ref = (A.double() @ Bm.double())
a = (A.t().contiguous() if at else A).to(dev)
b = (Bm.t().contiguous() if bt else Bm).to(dev)
for algo in (L.F32_SPLIT_BF16X6, L.F32_MFMA_F32):
    for rep in range(3):
        c = torch.zeros(m, n, device=dev)
        ops.gemm(a, at, b, bt, c, m, n, k, f32_algo=algo)
        torch.cuda.synchronize()
        d = (c.double().cpu() - ref).abs()
        bad = (d > 1e-3 * ref.abs().max()).nonzero()
        print("algo", algo, "rep", rep, "max err %.3e" % float(d.max()), "bad", bad.shape[0],
              "rows", sorted(set(bad[:, 0].tolist()))[:12], "cols", sorted(set(bad[:, 1].tolist()))[:12])
