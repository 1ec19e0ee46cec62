"""Regression fixture for the long-sequence co-attention: a ragged 320 x 36 and 36 x 320 head-dim-96
co-attention (the config-5 PV <-> title shape, c_layer_pv_t, vilbert_k3m.py:841-965) with dropout, computed by
THIS repository's exact-fp32 attention (attention_long.hip / attention.hip through ops.attn_fwd / attn_bwd) on
bf16-exact inputs.  Parity unpinned against upstream (the reference's dropout draws cannot be reproduced); the
fixture pins the bf16 flash-long kernels (attention_flash_long.hip) so a later layout change cannot move them
silently.  Inputs are regenerated from the seed in the test; outputs are stored as float16.

    python tests/golden/make_flash_long_golden.py      # on a GPU box; writes tests/golden/flash_long_d96.npz
"""
import math
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

CASES = [(320, 36), (36, 320)]
B, NH, HD, P_DROP, SEED, OFF = 2, 4, 96, 0.1, 1234567, 99


def inputs(lq, lk, dev):
    """bf16-exact q/k/v/dctx and a ragged key mask (item 0: all keys valid but the last 3; item 1: 60 % valid)."""
    D = NH * HD
    g = torch.Generator(device="cpu").manual_seed(lq * 1000 + lk)
    q = torch.randn(B * lq, D, generator=g).bfloat16()
    k = torch.randn(B * lk, D, generator=g).bfloat16()
    v = torch.randn(B * lk, D, generator=g).bfloat16()
    dctx = torch.randn(B * lq, D, generator=g).bfloat16()
    m = torch.ones(B, lk)
    m[0, lk - 3:] = 0
    m[1, int(0.6 * lk):] = 0
    mask = (1 - m) * -10000.0
    return [t.to(dev) for t in (q, k, v, dctx, mask)]


def main():
    from k3m_amd import ops
    dev = torch.device("cuda")
    out = {"B": B, "NH": NH, "HD": HD, "p_drop": P_DROP, "seed": SEED, "off": OFF}
    for lq, lk in CASES:
        q, k, v, dctx, mask = [t.float() if t.dtype == torch.bfloat16 else t for t in inputs(lq, lk, dev)]
        D = NH * HD
        sc = 1 / math.sqrt(HD)
        ctx = torch.empty(B * lq, D, device=dev)
        probs = torch.empty(B * NH * lq * lk, device=dev)
        ops.attn_fwd(q, k, v, mask.contiguous(), ctx, probs, B, lq, lk, NH, HD, sc, P_DROP, SEED, OFF)
        dq, dk, dv = [torch.empty(B * n_, D, device=dev) for n_ in (lq, lk, lk)]
        ops.attn_bwd(dctx, ctx, q, k, v, probs, dq, dk, dv, B, lq, lk, NH, HD, sc, P_DROP, SEED, OFF)
        torch.cuda.synchronize()
        tag = "%dx%d" % (lq, lk)
        for name, t in (("ctx", ctx), ("dq", dq), ("dk", dk), ("dv", dv)):
            out["%s/%s" % (tag, name)] = t.cpu().numpy().astype(np.float16)
    np.savez_compressed(os.path.join(HERE, "flash_long_d96.npz"), **out)
    print("wrote", os.path.join(HERE, "flash_long_d96.npz"))


if __name__ == "__main__":
    main()
