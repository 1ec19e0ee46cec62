"""Microbenchmark of the fused attention kernels on the step's shapes (bs=64): forward and
backward, fp32 and bf16.  Prints us per launch."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from k3m_amd import ops, _lib as L  # noqa: E402

B = 64
P_DROP = float(os.environ.get("ATTN_P", "0.1"))   # attention-probability dropout of the timed calls
SHAPES = [  # name, nseq, lq, lk, nh, hd
    ("text T", 2 * B, 36, 36, 12, 64),
    ("text P", 2 * B, 128, 128, 12, 64),
    ("image R", 2 * B, 37, 37, 8, 128),
    ("co txt->img", B, 36, 37, 8, 128),
    ("co pv->img", B, 128, 37, 8, 128),
    ("co img->pv", B, 37, 128, 8, 128),
    ("co pv->txt", B, 128, 36, 8, 128),
    ("co2 pv->txt", B, 128, 36, 8, 96),
    ("co2 txt->pv", B, 36, 128, 8, 96),
]
# BASELINE configs[4] (bs=128, PV 320): the shapes attention_flash_long.hip serves in bf16
SHAPES5 = [
    ("pv self", 256, 320, 320, 12, 64),
    ("co pv->img", 128, 320, 37, 8, 128),
    ("co img->pv", 128, 37, 320, 8, 128),
    ("co2 pv->txt", 128, 320, 36, 8, 96),
    ("co2 txt->pv", 128, 36, 320, 8, 96),
]


def run(name, nseq, lq, lk, nh, hd, dtype, reps=20):
    dev = torch.device("cuda")
    D = nh * hd
    qkv_q = torch.randn(nseq * lq, 3 * D, device=dev).to(dtype)
    qkv_k = torch.randn(nseq * lk, 3 * D, device=dev).to(dtype)
    q, k, v = qkv_q[:, :D], qkv_k[:, D:2 * D], qkv_k[:, 2 * D:]
    mask = torch.zeros(nseq, lk, device=dev)
    ctx = torch.empty(nseq * lq, D, device=dev, dtype=dtype)
    probs = torch.empty(nseq * nh * lq * lk, device=dev)
    dctx = torch.randn(nseq * lq, D, device=dev).to(dtype)
    dq = torch.empty(nseq * lq, D, device=dev, dtype=dtype)
    dk = torch.empty(nseq * lk, D, device=dev, dtype=dtype)
    dv = torch.empty(nseq * lk, D, device=dev, dtype=dtype)
    sc = 1 / math.sqrt(hd)

    flash = dtype == torch.bfloat16 and hd in (64, 96, 128) and FLASH
    lse = torch.empty(nseq * nh * lq, device=dev)

    def fwd():
        if flash:
            ops.flash_attn_fwd(q, k, v, mask, ctx, lse, nseq, lq, lk, nh, hd, sc, P_DROP, 7, 0)
        else:
            ops.attn_fwd(q, k, v, mask, ctx, probs, nseq, lq, lk, nh, hd, sc, P_DROP, 7, 0)

    def bwd():
        if flash:
            ops.flash_attn_bwd(dctx, ctx, q, k, v, mask, lse, dq, dk, dv, nseq, lq, lk, nh, hd, sc, P_DROP, 7, 0)
        else:
            ops.attn_bwd(dctx, ctx, q, k, v, probs, dq, dk, dv, nseq, lq, lk, nh, hd, sc, P_DROP, 7, 0)
    res = []
    for f in (fwd, bwd):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record()
        torch.cuda.synchronize()
        res.append(1000 * e0.elapsed_time(e1) / reps)
    print("%-12s %-8s %-5s nseq=%4d lq=%3d lk=%3d nh=%2d hd=%3d  fwd %8.1f us  bwd %8.1f us" % (
        name, str(dtype)[6:], "flash" if flash else "", nseq, lq, lk, nh, hd, res[0], res[1]), flush=True)


FLASH = True

if __name__ == "__main__":
    L.load()
    dts = {"fp32": [torch.float32], "bf16": [torch.bfloat16], "both": [torch.float32, torch.bfloat16]}[
        sys.argv[1] if len(sys.argv) > 1 else "both"]
    shapes = SHAPES5 if len(sys.argv) > 2 and sys.argv[2] == "cfg5" else SHAPES
    if len(sys.argv) > 3:   # one shape by name
        shapes = [sh for sh in shapes if sh[0] == sys.argv[3]]
    for d in dts:
        for sh in shapes:
            run(*sh, dtype=d)
    if torch.bfloat16 in dts:
        FLASH = False
        for sh in shapes:
            run(*sh, dtype=torch.bfloat16)
