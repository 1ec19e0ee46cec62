"""Lab: the image-layer dGELU input gradient (4,736 x 1,024 x 1,024, bf16 operands) under the step's variants:
C fp32 / bf16, with / without the fused column-sum slabs (K3M_GEMM_COLSUM_SLABS)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from k3m_amd import ops, _lib as L  # noqa: E402


def main():
    dev = torch.device("cuda")
    m, n, k = 4736, 1024, 1024
    a = torch.randn(m, k, device=dev).to(torch.bfloat16)
    b = (torch.randn(k, n, device=dev) * 0.02).to(torch.bfloat16)
    for cdt in (torch.bfloat16, torch.float32):
        for cs in (False, True):
            c = torch.zeros(m, n, device=dev, dtype=cdt)
            aux = torch.randn(m, n, device=dev, dtype=cdt)
            ws = torch.empty(((m + 31) // 32) * n, device=dev) if cs else None
            epi = L.EPI_DGELU | (L.GEMM_COLSUM_SLABS if cs else 0)

            def go():
                ops.gemm(a, 0, b, 0, c, m, n, k, epi, None, aux, 1.0, 0.0, 1, ws)
            for _ in range(3):
                go()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                go()
            e1.record()
            torch.cuda.synchronize()
            print("C %s colsum %d: %.3f ms" % (str(cdt)[6:], cs, e0.elapsed_time(e1) / 20), flush=True)


if __name__ == "__main__":
    main()
