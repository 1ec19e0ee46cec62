"""Microbenchmark of the libk3m_hip GEMM on the text-layer shapes of the wide engine (bs=64):
forward x.W^T, input-gradient dY.W and weight-gradient dY^T.X.  Prints TF/s per shape."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import ops, _lib as L  # noqa: E402

M = 20992
SHAPES = [
    ("fwd qkv", "nt", M, 2304, 768, L.EPI_BIAS),
    ("fwd out", "nt", M, 768, 768, L.EPI_BIAS),
    ("fwd ffn1 gelu", "nt", M, 3072, 768, L.EPI_BIAS_GELU),
    ("fwd ffn1 plain", "nt", M, 3072, 768, L.EPI_NONE),
    ("fwd ffn2", "nt", M, 768, 3072, L.EPI_BIAS),
    ("dgrad qkv", "nn", M, 768, 2304, L.EPI_NONE),
    ("dgrad ffn2->dgelu", "nn", M, 3072, 768, L.EPI_DGELU),
    ("dgrad ffn1", "nn", M, 768, 3072, L.EPI_NONE),
    ("wgrad ffn1", "tn", 3072, 768, M, L.EPI_NONE),
    ("wgrad ffn2", "tn", 768, 3072, M, L.EPI_NONE),
    ("wgrad qkv", "tn", 2304, 768, M, L.EPI_NONE),
    ("wgrad out", "tn", 768, 768, M, L.EPI_NONE),
    # co-attention (per-pass) shapes
    ("co txt ffn2", "nt", 2304, 768, 3072, L.EPI_BIAS),
    ("co img qkv", "nt", 2368, 3072, 1024, L.EPI_BIAS),
    ("co img dense", "nt", 2368, 1024, 1024, L.EPI_BIAS),
    ("co pv ffn1", "nt", 8192, 3072, 768, L.EPI_BIAS_GELU),
    ("co txt dgrad", "nn", 2304, 768, 3072, L.EPI_NONE),
    ("co img wgrad", "tn", 1024, 1024, 2368, L.EPI_NONE),
    # image-layer (4,736 rows) and small head shapes of the step (scripts/gemm_calls.py)
    ("img dgrad dgelu", "nn", 4736, 1024, 1024, L.EPI_DGELU),
    ("img dgrad plain", "nn", 4736, 1024, 1024, L.EPI_NONE),
    ("img fwd gelu", "nt", 4736, 1024, 1024, L.EPI_BIAS_GELU),
    ("img fwd bias", "nt", 4736, 1024, 1024, L.EPI_BIAS),
    ("loc wgrad", "tn", 1024, 5, 2368, L.EPI_NONE),
    ("mlm wgrad", "tn", 768, 768, 1552, L.EPI_NONE),
    # square reference shapes (the CDNA guide quotes its bf16 templates at 4096^3)
    ("sq4k nt", "nt", 4096, 4096, 4096, L.EPI_NONE),
    ("sq4k ffn1-k", "nt", 20992, 3072, 4096, L.EPI_NONE),
]


def run(name, kind, m, n, k, epi, reps=10, dtype=torch.float32):
    dev = torch.device("cuda")
    if kind == "nt":
        a, b = torch.randn(m, k, device=dev), torch.randn(n, k, device=dev) * 0.02
        at, bt = 0, 1
    elif kind == "nn":
        a, b = torch.randn(m, k, device=dev), torch.randn(k, n, device=dev) * 0.02
        at, bt = 0, 0
    else:
        a, b = torch.randn(k, m, device=dev), torch.randn(k, n, device=dev) * 0.02
        at, bt = 1, 0
    a, b = a.to(dtype), b.to(dtype)
    cdt = torch.float32 if kind == "tn" else dtype   # weight gradients accumulate into fp32
    c = torch.zeros(m, n, device=dev, dtype=cdt)
    bias = torch.zeros(n, device=dev)
    aux = torch.randn(m, n, device=dev, dtype=cdt) if epi in (L.EPI_BIAS_GELU, L.EPI_DGELU) else None
    beta = 1.0 if kind == "tn" else 0.0
    s = ops._splitk(m, n, k, dtype) if kind == "tn" else 1
    ws = torch.empty(s * m * n, device=dev) if s > 1 else None

    def go():
        ops.gemm(a, at, b, bt, c, m, n, k, epi, bias if epi in (L.EPI_BIAS, L.EPI_BIAS_GELU) else None, aux, 1.0,
                 beta, s, ws)
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2.0 * m * n * k / (ms * 1e-3) / 1e12
    print("%-20s %s %s m=%6d n=%5d k=%6d splitk=%2d  %8.3f ms  %7.1f TF/s" % (name, kind, str(dtype)[6:], m, n, k, s,
                                                                            ms, tf), flush=True)
    return tf


if __name__ == "__main__":
    L.load()
    only = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "all" else None
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dts = {"fp32": [torch.float32], "bf16": [torch.bfloat16], "both": [torch.float32, torch.bfloat16]}[
        sys.argv[3] if len(sys.argv) > 3 else "fp32"]
    for d in dts:
        for sh in SHAPES:
            if only is None or only in sh[0]:
                run(*sh, reps=reps, dtype=d)
