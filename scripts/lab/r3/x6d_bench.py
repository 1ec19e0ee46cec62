"""Pre-split (LDS-DMA) bf16x6 GEMM vs the in-kernel-split x6 kernels on the text-layer shapes: bit-identity
of the outputs and time per launch (HIP events, best of passes).
usage: python scripts/x6d_bench.py [reps] [shape substring] [x6|x6d|both]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import ops, _lib as L  # noqa: E402

M = 20992
SHAPES = [
    ("fwd ffn1 plain", "nt", M, 3072, 768, L.EPI_NONE),
    ("fwd ffn1 gelu", "nt", M, 3072, 768, L.EPI_BIAS_GELU),
    ("fwd qkv", "nt", M, 2304, 768, L.EPI_BIAS),
    ("fwd ffn2", "nt", M, 768, 3072, L.EPI_BIAS),
    ("dgrad ffn1", "nn", M, 768, 3072, L.EPI_NONE),
    ("dgrad ffn2->dgelu", "nn", M, 3072, 768, L.EPI_DGELU),
    ("wgrad ffn1", "tn", 3072, 768, M, L.EPI_NONE),
    ("wgrad ffn2", "tn", 768, 3072, M, L.EPI_NONE),
]


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e30
    for _ in range(3):
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


def main(reps=10, only=None, which="both"):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for name, kind, m, n, k, epi in SHAPES:
        if only and only not in name:
            continue
        if kind == "nt":
            a, b, at, bt = torch.randn(m, k, device=dev), torch.randn(n, k, device=dev) * 0.02, 0, 1
        elif kind == "nn":
            a, b, at, bt = torch.randn(m, k, device=dev), torch.randn(k, n, device=dev) * 0.02, 0, 0
        else:
            a, b, at, bt = torch.randn(k, m, device=dev), torch.randn(k, n, device=dev) * 0.02, 1, 0
        bias = torch.randn(n, device=dev) if epi in (L.EPI_BIAS, L.EPI_BIAS_GELU) else None
        aux0 = torch.randn(m, n, device=dev) if epi in (L.EPI_BIAS_GELU, L.EPI_DGELU) else None
        s = ops._splitk(m, n, k) if kind == "tn" else 1
        ws = torch.empty(s * m * n, device=dev) if s > 1 else None
        beta = 1.0 if kind == "tn" else 0.0
        c0 = torch.zeros(m, n, device=dev)
        c1 = torch.zeros(m, n, device=dev)
        aux1 = aux0.clone() if aux0 is not None else None
        ap, bp = ops.split3(a), ops.split3(b)
        ops.gemm(a, at, b, bt, c0, m, n, k, epi, bias, aux0, 1.0, beta, s, ws)
        ops.gemm_planes(ap, at, bp, bt, c1, m, n, k, epi, bias, aux1, 1.0, beta, s, ws)
        torch.cuda.synchronize()
        same = torch.equal(c0, c1) and (aux0 is None or torch.equal(aux0, aux1))
        maxd = (c0 - c1).abs().max().item()
        t0 = t1 = float("nan")
        if which in ("x6", "both"):
            t0 = timeit(lambda: ops.gemm(a, at, b, bt, c0, m, n, k, epi, bias, aux0, 1.0, beta, s, ws), reps)
        if which in ("x6d", "both"):
            t1 = timeit(lambda: ops.gemm_planes(ap, at, bp, bt, c1, m, n, k, epi, bias, aux1, 1.0, beta, s, ws), reps)
        tsa = timeit(lambda: ops.split3(a, ap), reps)
        fl = 2.0 * m * n * k
        print("%-20s m=%6d n=%5d k=%6d s=%d  x6 %.3f ms %6.1f TF/s | x6d %.3f ms %6.1f TF/s (%.3f of 416.7) | "
              "split(A) %.3f ms | bit-identical %s maxdiff %.3g" % (
                  name, m, n, k, s, t0, fl / t0 / 1e9, t1, fl / t1 / 1e9, fl / t1 / 1e9 / 416.7, tsa, same, maxd),
              flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10, sys.argv[2] if len(sys.argv) > 2 else None,
         sys.argv[3] if len(sys.argv) > 3 else "both")
