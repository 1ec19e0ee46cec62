"""Runs a fixed set of bf16 GEMMs (every layout, epilogue, split-K and a grouped launch) through k3m_gemm and
saves C (and the GELU pre-activation / colsum slabs) to a .pt file: tests/test_gpu_gemm_b16_dual.py runs it
under K3M_B16_DUAL=0 and =1 in child processes and requires bit-identical outputs.
usage: python scripts/b16_dump.py out.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import ops, _lib as L  # noqa: E402

CASES = [  # name, kind, m, n, k, epilogue, splitk
    ("fwd_bias", "nt", 4736, 2304, 768, L.EPI_BIAS, 1),
    ("fwd_gelu", "nt", 8192, 3072, 768, L.EPI_BIAS_GELU, 1),
    ("fwd_edge", "nt", 2368, 1000, 1024, L.EPI_BIAS, 1),
    ("fwd_sigmoid", "nt", 2304, 1024, 1024, L.EPI_BIAS_SIGMOID, 1),
    ("dgrad", "nn", 4736, 768, 3072, L.EPI_NONE, 1),
    ("dgrad_dgelu", "nn", 4096, 3072, 768, L.EPI_DGELU, 1),
    ("wgrad", "tn", 3072, 768, 8192, L.EPI_NONE, 1),
    ("wgrad_split", "tn", 1024, 1024, 20992, L.EPI_NONE, 5),
]


def main(out):
    L.load()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    res = {}
    for name, kind, m, n, k, epi, s in CASES:
        if kind == "nt":
            a, b, at, bt = torch.randn(m, k, device=dev, generator=g), torch.randn(n, k, device=dev, generator=g), 0, 1
        elif kind == "nn":
            a, b, at, bt = torch.randn(m, k, device=dev, generator=g), torch.randn(k, n, device=dev, generator=g), 0, 0
        else:
            a, b, at, bt = torch.randn(k, m, device=dev, generator=g), torch.randn(k, n, device=dev, generator=g), 1, 0
        a, b = a.bfloat16(), (b * 0.05).bfloat16()
        cdt = torch.float32 if kind == "tn" else torch.bfloat16
        c = torch.randn(m, n, device=dev, generator=g).to(cdt) if kind == "tn" else torch.empty(m, n, device=dev, dtype=cdt)
        bias = torch.randn(n, device=dev, generator=g)
        aux = (torch.empty(m, n, device=dev, dtype=cdt) if epi == L.EPI_BIAS_GELU else
               torch.randn(m, n, device=dev, generator=g).to(cdt) if epi == L.EPI_DGELU else None)
        ws = torch.empty(s * m * n, device=dev) if s > 1 else None
        ops.gemm(a, at, b, bt, c, m, n, k, epi, bias if epi in (L.EPI_BIAS, L.EPI_BIAS_GELU, L.EPI_BIAS_SIGMOID) else None,
                 aux, 1.0, 1.0 if kind == "tn" else 0.0, s, ws)
        res[name] = c.cpu()
        if epi == L.EPI_BIAS_GELU:
            res[name + "_aux"] = aux.cpu()
    # grouped launch (the co-attention stages): three problems of one template
    probs = []
    with ops.grouped():
        for i, (m, n, k) in enumerate([(2304, 3072, 1024), (2368, 3072, 1024), (8192, 3072, 768)]):
            a = torch.randn(m, k, device=dev, generator=g).bfloat16()
            b = (torch.randn(n, k, device=dev, generator=g) * 0.05).bfloat16()
            c = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
            bias = torch.randn(n, device=dev, generator=g)
            probs.append((a, b, c, bias))
            ops.gemm(a, 0, b, 1, c, m, n, k, L.EPI_BIAS, bias)
    for i, (_, _, c, _) in enumerate(probs):
        res["grouped%d" % i] = c.cpu()
    torch.cuda.synchronize()
    torch.save(res, out)


if __name__ == "__main__":
    main(sys.argv[1])
