"""Time the whole-head attention kernels (attention.hip) against the blocked ones
(attention_long.hip) on the wide engine's shapes at bs=64 (fp32, dropout 0.1): which path each
(Lq, Lk, d) should take.  Prints one line per shape."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import _lib as L  # noqa: E402

SHAPES = [  # (nseq, lq, lk, nh, hd): text/PV self-attention, image, co-attention
    (128, 128, 128, 12, 64), (128, 36, 36, 12, 64), (128, 37, 37, 8, 128), (64, 36, 37, 8, 128), (64, 37, 36, 8, 128),
    (64, 128, 37, 8, 128), (64, 37, 128, 8, 128), (64, 128, 36, 8, 96), (64, 36, 128, 8, 96)]


def run(nseq, lq, lk, nh, hd, long_path, reps=20):
    dev = torch.device("cuda")
    D = nh * hd
    q = torch.randn(nseq * lq, D, device=dev)
    k = torch.randn(nseq * lk, D, device=dev)
    v = torch.randn(nseq * lk, D, device=dev)
    mask = torch.zeros(nseq * lk, device=dev)
    ctx = torch.empty(nseq * lq, D, device=dev)
    probs = torch.empty(nseq * nh * lq * lk, device=dev)
    dctx = torch.randn_like(ctx)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    ws = torch.empty_like(probs)
    s = 1 / math.sqrt(hd)
    st = L.stream()

    def fwd():
        L.call("k3m_attn_long_fwd" if long_path else "k3m_attn_fwd", q.data_ptr(), D, k.data_ptr(), D, v.data_ptr(), D,
               mask.data_ptr(), ctx.data_ptr(), D, probs.data_ptr(), nseq, lq, lk, nh, hd, s, 0.1, 1, 0, L.F32, st)

    def bwd():
        args = [dctx.data_ptr(), D, ctx.data_ptr(), D, q.data_ptr(), D, k.data_ptr(), D, v.data_ptr(), D, probs.data_ptr()]
        if long_path:
            args.append(ws.data_ptr())
        L.call("k3m_attn_long_bwd" if long_path else "k3m_attn_bwd", *args, dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
               D, D, D, nseq, lq, lk, nh, hd, s, 0.1, 1, 0, L.F32, st)

    out = []
    for fn in (fwd, bwd):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    return out


def main():
    # warm the clock
    a = torch.randn(8192, 8192, device="cuda")
    for _ in range(20):
        a @ a
    for shp in SHAPES:
        r = []
        for rep in range(2):
            r = [run(*shp, False), run(*shp, True)]
        (sf, sb), (lf, lb) = r
        print("nseq=%3d lq=%3d lk=%3d nh=%2d d=%3d   short fwd %7.1f bwd %7.1f us   blocked fwd %7.1f bwd %7.1f us"
              % (shp + (sf, sb, lf, lb)), flush=True)


if __name__ == "__main__":
    main()
