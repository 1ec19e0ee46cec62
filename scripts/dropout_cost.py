"""What the counter-based dropout hash costs: time the short attention kernels and the LayerNorm
forward/backward with p = 0 (no hash evaluated) and p = 0.1 on the wide engine's shapes (fp32).
Prints one line per kernel."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import _lib as L, ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / reps
        best = t if best is None else min(best, t)
    return best


def attn(nseq, lq, lk, nh, hd, p):
    dev = torch.device("cuda")
    D = nh * hd
    q, k, v = (torch.randn(nseq * n, D, device=dev) for n in (lq, lk, lk))
    mask = torch.zeros(nseq * lk, device=dev)
    ctx = torch.empty(nseq * lq, D, device=dev)
    probs = torch.empty(nseq * nh * lq * lk, device=dev)
    dctx = torch.randn_like(ctx)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    s = 1 / math.sqrt(hd)
    st = L.stream()

    def fwd():
        L.call("k3m_attn_fwd", q.data_ptr(), D, k.data_ptr(), D, v.data_ptr(), D, mask.data_ptr(), ctx.data_ptr(), D,
               probs.data_ptr(), nseq, lq, lk, nh, hd, s, p, 1, 0, L.F32, st)

    def bwd():
        L.call("k3m_attn_bwd", dctx.data_ptr(), D, ctx.data_ptr(), D, q.data_ptr(), D, k.data_ptr(), D, v.data_ptr(), D,
               probs.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), D, D, D, nseq, lq, lk, nh, hd, s, p, 1, 0,
               L.F32, st)
    return timed(fwd), timed(bwd)


def ln(rows, cols, p):
    dev = torch.device("cuda")
    x, res = torch.randn(rows, cols, device=dev), torch.randn(rows, cols, device=dev)
    g, b = torch.ones(cols, device=dev), torch.zeros(cols, device=dev)
    y, xhat = torch.empty_like(x), torch.empty_like(x)
    rstd = torch.empty(rows, device=dev)
    dy = torch.randn_like(x)
    dres, dx = torch.empty_like(x), torch.empty_like(x)
    dgs, dbs = torch.zeros(cols, device=dev), torch.zeros(cols, device=dev)
    f = timed(lambda: ops.ln_fwd(x, res, g, b, y, xhat, rstd, p_in=p, seed=1))
    bw = timed(lambda: ops.ln_bwd(dy, xhat, rstd, g, dres, dx, dgs, dbs, p_in=p, seed=1))
    return f, bw


def main():
    for shp in [(128, 128, 128, 12, 64), (128, 36, 36, 12, 64), (128, 37, 37, 8, 128), (64, 128, 37, 8, 128)]:
        a0, a1 = attn(*shp, 0.0), attn(*shp, 0.1)
        print("attn nseq=%3d lq=%3d lk=%3d nh=%2d d=%3d   p=0: fwd %7.1f bwd %7.1f us   p=0.1: fwd %7.1f bwd %7.1f us"
              % (shp + a0 + a1), flush=True)
    for rows, cols in [(20992, 768), (4736, 1024)]:
        l0, l1 = ln(rows, cols, 0.0), ln(rows, cols, 0.1)
        print("ln %5dx%4d   p=0: fwd %7.1f bwd %7.1f us   p=0.1: fwd %7.1f bwd %7.1f us" % ((rows, cols) + l0 + l1),
              flush=True)


if __name__ == "__main__":
    main()
