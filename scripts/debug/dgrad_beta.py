"""Error map of the bf16 dgrad GEMM with beta = 1 (tests/test_gpu_gemm_b16_big.py::test_dgrad_kc_mn
[4736-1024-1024] failure): which row / column blocks are wrong, over repeated calls (debug)."""
import sys
import torch

sys.path.insert(0, ".")
from k3m_amd import ops, _lib as L  # noqa: E402

dev = torch.device("cuda")
m, n, k = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
g = torch.Generator(device=dev).manual_seed(m)
dy = torch.randn((m, k), device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn((k, n), device=dev, generator=g) * 0.05).to(torch.bfloat16)
ref = dy.float() @ w.float()
for rep in range(3):
    for beta, cdt in ((0.0, torch.float32), (1.0, torch.float32), (0.0, torch.bfloat16), (1.0, torch.bfloat16)):
        c0 = torch.randn((m, n), device=dev, generator=g).to(cdt)
        c = c0.clone()
        ops.gemm(dy, 0, w, 0, c, m, n, k, L.EPI_NONE, None, None, 1.0, beta)
        torch.cuda.synchronize()
        want = ref + beta * c0.float()
        bad = (c.float() - want).abs() > 0.02 * want.abs().max()
        nb = int(bad.sum())
        msg = "rep %d beta %g %s wrong %d" % (rep, beta, str(cdt)[6:], nb)
        if nb:
            r = bad.any(1).nonzero().flatten()
            cc = bad.any(0).nonzero().flatten()
            msg += " rows %d..%d (%d) cols %d..%d (%d)" % (int(r.min()), int(r.max()), len(r), int(cc.min()),
                                                         int(cc.max()), len(cc))
        print(msg, flush=True)
        for i, j in bad.nonzero()[:4].tolist():
            print("   [%d,%d] got %.4f ref %.4f c0 %.4f  (got-ref)/c0 %.3f" % (
                i, j, float(c[i, j]), float(ref[i, j]), float(c0[i, j]),
                (float(c[i, j]) - float(ref[i, j])) / float(c0[i, j])), flush=True)
