"""Probe the bf16 GEMM operand paths with permutation data (debug harness, not a test):
A[i, l] = 1 iff l == i % K, so C[i, :] must equal B[i % K, :].  B holds a code that names its k
row (first pass) or its column (second pass) modulo 256, so a fragment read from the wrong k-tile
stage or the wrong column shows up as a wrong code."""
import sys
import torch

sys.path.insert(0, ".")
from k3m_amd import ops  # noqa: E402


def probe(m, n, k, bt, what):
    dev = torch.device("cuda")
    a = torch.zeros((m, k), device=dev)
    a[torch.arange(m), torch.arange(m) % k] = 1
    a = a.to(torch.bfloat16)
    lk = torch.arange(k, device=dev)[:, None].expand(k, n)
    jn = torch.arange(n, device=dev)[None, :].expand(k, n)
    code = (lk % 256) if what == "k" else (jn % 256)
    B = code.float()                                  # logical [k, n]
    b = (B.t().contiguous() if bt else B.contiguous()).to(torch.bfloat16)
    c = torch.zeros((m, n), device=dev)
    ops.gemm(a, 0, b, bt, c, m, n, k)
    torch.cuda.synchronize()
    ref = B[torch.arange(m, device=dev) % k]
    bad = (c != ref)
    print("m n k bt code", m, n, k, bt, what, "wrong", int(bad.sum()), "of", m * n, flush=True)
    if bad.any():
        for i, j in bad.nonzero()[:8].tolist():
            print("  C[%d,%d] = %g want %g" % (i, j, float(c[i, j]), float(ref[i, j])))


if __name__ == "__main__":
    for shape in [(4736, 1024, 1024), (1000, 3072, 768), (20992, 768, 3072), (2368, 3072, 1024)]:
        for bt in (0, 1):
            for what in ("k", "n"):
                probe(*shape, bt, what)
