"""The vendor libraries on the step's GEMM shapes (torch.matmul -> hipBLASLt / rocBLAS), beside scripts/gemm_bench.py:
where the hand-written kernels stand against the library on the same box.  fp32 runs with TF32/XF32 off (exact f32).
usage: python scripts/torch_gemm_ref.py [fp32|bf16|both] [reps]"""
import sys

import torch

SHAPES = [  # name, kind, m, n, k  (C[m,n] = A . B, kind as scripts/gemm_bench.py)
    ("fwd ffn1", "nt", 20992, 3072, 768),
    ("fwd ffn2", "nt", 20992, 768, 3072),
    ("dgrad ffn1", "nn", 20992, 768, 3072),
    ("wgrad ffn1", "tn", 3072, 768, 20992),
    ("wgrad ffn2", "tn", 768, 3072, 20992),
    ("sq4k nt", "nt", 4096, 4096, 4096),
]


def run(name, kind, m, n, k, dtype, reps):
    dev = torch.device("cuda")
    if kind == "nt":
        a, b = torch.randn(m, k, device=dev, dtype=dtype), torch.randn(n, k, device=dev, dtype=dtype)
        f = lambda: torch.matmul(a, b.t())  # noqa: E731
    elif kind == "nn":
        a, b = torch.randn(m, k, device=dev, dtype=dtype), torch.randn(k, n, device=dev, dtype=dtype)
        f = lambda: torch.matmul(a, b)  # noqa: E731
    else:
        a, b = torch.randn(k, m, device=dev, dtype=dtype), torch.randn(k, n, device=dev, dtype=dtype)
        f = lambda: torch.matmul(a.t(), b)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print("%-12s %s %-8s m=%6d n=%5d k=%6d  %8.3f ms  %7.1f TF/s" % (name, kind, str(dtype)[6:], m, n, k, ms,
                                                                   2.0 * m * n * k / ms / 1e9), flush=True)


if __name__ == "__main__":
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dts = {"fp32": [torch.float32], "bf16": [torch.bfloat16], "both": [torch.float32, torch.bfloat16]}[which]
    for d in dts:
        for sh in SHAPES:
            run(*sh, dtype=d, reps=reps)
