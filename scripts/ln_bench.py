"""LayerNorm forward / backward (bf16 and fp32) on the step's shapes: time per launch and effective HBM rate,
and (bf16) the outputs of the current build for comparison across K3M_LN_BF16_VEC settings.
usage: python scripts/ln_bench.py [out.pt]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import ops  # noqa: E402

SHAPES = [(20992, 768), (8192, 768), (2304, 768), (2368, 1024), (45568, 768)]
P = float(os.environ.get("LN_P", "0.1"))   # the input dropout of the timed calls


def timeit(fn, reps=20):
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


def main(out=None):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    keep = {}
    for dtype in (torch.bfloat16, torch.float32):
        eb = 2 if dtype == torch.bfloat16 else 4
        for rows, cols in SHAPES:
            x = torch.randn(rows, cols, device=dev).to(dtype)
            r = torch.randn(rows, cols, device=dev).to(dtype)
            g, b = torch.rand(cols, device=dev) + 0.5, torch.randn(cols, device=dev)
            y, xh = torch.empty_like(x), torch.empty_like(x)
            rs = torch.empty(rows, device=dev)
            dy = torch.randn(rows, cols, device=dev).to(dtype)
            dres, dx = torch.empty_like(x), torch.empty_like(x)
            dg, db, xs = (torch.zeros(cols, device=dev) for _ in range(3))
            fwd = lambda: ops.ln_fwd(x, r, g, b, y, xh, rs, p_in=P, p_out=0.0, seed=3, off_in=11)  # noqa: E731
            bwd = lambda: ops.ln_bwd(dy, xh, rs, g, dres, dx, dg, db, p_in=P, seed=3, off_in=11, dxsum=xs)  # noqa: E731
            fwd()
            torch.cuda.synchronize()
            if dtype == torch.bfloat16:
                dg.zero_(), db.zero_(), xs.zero_()
                bwd()
                torch.cuda.synchronize()
                keep["%dx%d" % (rows, cols)] = [t[:512].float().cpu() for t in (y, xh, rs, dres, dx, dg, db, xs)]
            tf, tb = timeit(fwd), timeit(bwd)
            n = rows * cols
            print("%-5s %6d x %4d  ln_fwd %7.1f us %6.0f GB/s | ln_bwd %7.1f us %6.0f GB/s" % (
                "bf16" if eb == 2 else "fp32", rows, cols, tf * 1e3, 4 * n * eb / tf / 1e6, tb * 1e3,
                4 * n * eb / tb / 1e6), flush=True)
    if out:
        torch.save(keep, out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
