"""Per-kernel roofline at the config-2 (bs=64) shapes of the wide engine: every kernel family of the
step timed with HIP events (median of reps, warm L2/MALL) against its own roofline.

For each kernel: algorithmic FLOPs and bytes per launch (stated below), achieved FLOP/s and GB/s,
and the roofline time max(FLOPs / matrix peak, bytes / 8 TB/s); `frac` = roofline time / measured
time.  Writes profiles/<out>.json and prints a table.

    python scripts/kernel_roofline.py [out_name]
"""
import json
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from k3m_amd import ops, _lib as L  # noqa: E402

HBM = 8.0e12
PEAK = {"x6": 2.5e15 / 6, "f32": 157.3e12, "bf16": 2.5e15, "none": None}
B, T, P, R = 64, 36, 128, 37
ROWS_T = 2 * B * T + 2 * B * P       # wide text buffer rows (20,992)
ROWS_V = 2 * B * R                   # wide image buffer rows (4,736)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e-3)
    ts.sort()
    return ts[len(ts) // 2]


def row(name, ref, t, flops, nbytes, peak_key, note=""):
    peak = PEAK[peak_key]
    t_flop = flops / peak if peak and flops else 0.0
    t_mem = nbytes / HBM
    bound = "mfma" if t_flop >= t_mem else "hbm"
    roof = max(t_flop, t_mem)
    return {"kernel": name, "replaces": ref, "time_us": round(t * 1e6, 2), "gflop": round(flops / 1e9, 3),
            "mbytes": round(nbytes / 1e6, 2), "achieved_tflops": round(flops / t / 1e12, 2) if flops else None,
            "achieved_gbs": round(nbytes / t / 1e9, 1), "bound": bound,
            "peak": ("%.1f TFLOP/s" % (peak / 1e12)) if bound == "mfma" else "8000 GB/s",
            "roofline_us": round(roof * 1e6, 2), "frac": round(roof / t, 3), "note": note}


def main():
    out_name = sys.argv[1] if len(sys.argv) > 1 else "r1_kernel_roofline"
    L.load()
    dev = torch.device("cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    res = []
    f32 = torch.float32

    # ---- GEMMs (bf16x6 fp32 path)
    H, I = 768, 3072
    x = torch.randn(ROWS_T, H, device=dev, generator=g)
    W1 = torch.randn(I, H, device=dev, generator=g) * 0.02
    b1 = torch.zeros(I, device=dev)
    pre = torch.empty(ROWS_T, I, device=dev)
    y = torch.empty(ROWS_T, I, device=dev)
    t = timeit(lambda: ops.linear(x, W1, b1, out=y, epi=L.EPI_BIAS_GELU, aux=pre))
    fl = 2.0 * ROWS_T * I * H
    res.append(row("gemm_x6 FFN1 fwd +bias+GELU (20992x3072x768)", "BertIntermediate :504-518", t, fl,
                   4 * (ROWS_T * H + I * H + 2 * ROWS_T * I), "x6"))
    dy = torch.randn(ROWS_T, I, device=dev, generator=g)
    gW = torch.zeros(I, H, device=dev)
    t = timeit(lambda: ops.linear_wgrad(dy, x, gW, None))
    s = ops._splitk(I, H, ROWS_T)
    res.append(row("gemm_x6 FFN1 weight grad (3072x768x20992, split-K %d + reduce)" % s, "autograd of :504-518", t,
                   fl, 4 * (ROWS_T * H + ROWS_T * I + 2 * I * H), "x6"))
    del pre, y, dy

    # ---- attention (fp32): text layer on the PV rows (128 seqs x 12 heads, L=128, d=64) and image (128 x 8, L=37, d=128)
    for (nseq, lq, lk, nh, hd, tag, ref) in [(2 * B, P, P, 12, 64, "text/PV L=128 d=64", "BertSelfAttention :439-475"),
                                             (2 * B, T, T, 12, 64, "text L=36 d=64", "BertSelfAttention :439-475"),
                                             (2 * B, R, R, 8, 128, "image L=37 d=128", "BertImageSelfAttention :586-634"),
                                             (B, T, P, 8, 96, "two-text 36x128 d=96", "BertBiAttention_two_text :913-951")]:
        Dm = nh * hd
        q = torch.randn(nseq * lq, Dm, device=dev, generator=g)
        k = torch.randn(nseq * lk, Dm, device=dev, generator=g)
        v = torch.randn(nseq * lk, Dm, device=dev, generator=g)
        mask = torch.zeros(nseq * lk, device=dev)
        ctx = torch.empty_like(q)
        probs = torch.empty(nseq * nh * lq * lk, device=dev)
        sc = 1.0 / math.sqrt(hd)
        t = timeit(lambda: ops.attn_fwd(q, k, v, mask, ctx, probs, nseq, lq, lk, nh, hd, sc, 0.1, 1, 0))
        fl = 4.0 * lq * lk * hd * nseq * nh
        by = 4 * (2 * nseq * lq * Dm + 2 * nseq * lk * Dm + nseq * nh * lq * lk)
        res.append(row("attn_fwd f32 %s" % tag, ref, t, fl, by, "f32", "saves P for the backward"))
        dctx = torch.randn_like(q)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        t = timeit(lambda: ops.attn_bwd(dctx, ctx, q, k, v, probs, dq, dk, dv, nseq, lq, lk, nh, hd, sc, 0.1, 1, 0))
        by = 4 * (4 * nseq * lq * Dm + 4 * nseq * lk * Dm + 2 * nseq * nh * lq * lk)
        res.append(row("attn_bwd f32 %s" % tag, "autograd of " + ref, t, 2 * fl, by, "f32", "reads P twice"))
        del q, k, v, ctx, probs, dctx, dq, dk, dv

    # ---- LayerNorm tail (dropout + residual + LN), wide text buffer
    res_ = torch.randn(ROWS_T, H, device=dev, generator=g)
    gam, bet = torch.ones(H, device=dev), torch.zeros(H, device=dev)
    yy, xh = torch.empty(ROWS_T, H, device=dev), torch.empty(ROWS_T, H, device=dev)
    rs = torch.empty(ROWS_T, device=dev)
    t = timeit(lambda: ops.ln_fwd(x, res_, gam, bet, yy, xh, rs, p_in=0.1, seed=3, off_in=0))
    res.append(row("ln_fwd f32 dropout+residual+LN (20992x768)", "BertSelfOutput/BertOutput :485-489, :528-532", t, 0,
                   4 * (4 * ROWS_T * H + ROWS_T), "none"))
    dy = torch.randn(ROWS_T, H, device=dev, generator=g)
    dres, dx = torch.empty_like(dy), torch.empty_like(dy)
    dg, db, dxs = torch.zeros(H, device=dev), torch.zeros(H, device=dev), torch.zeros(H, device=dev)
    t = timeit(lambda: ops.ln_bwd(dy, xh, rs, gam, dres, dx, dg, db, p_in=0.1, seed=3, off_in=0, dxsum=dxs))
    res.append(row("ln_bwd f32 (+dgamma/dbeta/bias-grad slabs)", "autograd of BertLayerNorm :319-332", t, 0,
                   4 * (4 * ROWS_T * H + ROWS_T), "none"))
    del res_, yy, xh, dy, dres, dx

    # ---- embeddings (text + PV rows of the wide buffer: written to 2 destinations each)
    V = 21128
    word = torch.randn(V, H, device=dev, generator=g) * 0.02
    pos = torch.randn(512, H, device=dev, generator=g) * 0.02
    typ = torch.randn(2, H, device=dev, generator=g) * 0.02
    ids = torch.randint(1, V, (B, P), device=dev, generator=g)
    tt = torch.zeros(B, P, dtype=torch.int64, device=dev)
    ya, yb = torch.empty(B * P, H, device=dev), torch.empty(B * P, H, device=dev)
    xe, re_ = torch.empty(B * P, H, device=dev), torch.empty(B * P, device=dev)
    t = timeit(lambda: ops.embed_fwd(ids, tt, word, pos, typ, gam, bet, ya, yb, None, xe, re_, 0.1, 5, 0))
    res.append(row("embed_fwd f32 gather+LN+dropout (64x128 tokens, 2 outputs)", "BertEmbeddings :361-382", t, 0,
                   4 * B * P * H * 6 + 8 * B * P * 2, "none"))
    dword, dpos, dtyp = torch.zeros_like(word), torch.zeros_like(pos), torch.zeros_like(typ)
    t = timeit(lambda: ops.embed_bwd(ids, tt, ya, dword, dpos, dtyp))
    res.append(row("embed_bwd f32 scatter-add (64x128 tokens)", "autograd of :361-382", t, 0,
                   4 * B * P * H * 4 + 8 * B * P * 2, "none", "float atomics: 3 adds per element"))
    del word, dword

    # ---- MLM cross-entropy over the labelled rows (~24/sample at bs=64) x 21,128 vocab, in place
    nl = 24 * B
    logits = torch.randn(nl, V, device=dev, generator=g)
    labels = torch.randint(0, V, (nl,), device=dev, generator=g)
    rsc = torch.full((nl,), 1.0 / nl, device=dev)
    lrows = torch.empty(nl, device=dev)
    t = timeit(lambda: L.call("k3m_ce_fwd_bwd", logits.data_ptr(), V, labels.data_ptr(), rsc.data_ptr(), nl, V,
                              lrows.data_ptr(), L.stream()))
    res.append(row("ce_fwd_bwd fused log-softmax CE + grad (1536x21128)", "loss_mlm :2255, :2817-2826", t, 0,
                   4 * 2 * nl * V, "none"))
    del logits

    # ---- AdamW over 400M fp32 parameters (decay segment size order)
    n = 400_000_000
    p = torch.zeros(n, device=dev)
    gr = torch.zeros(n, device=dev)
    m = torch.zeros(n, device=dev)
    v2 = torch.zeros(n, device=dev)
    t = timeit(lambda: L.call("k3m_adamw", p.data_ptr(), gr.data_ptr(), m.data_ptr(), v2.data_ptr(), None, n, 1e-4,
                              0.9, 0.98, 1e-8, 0.01, 5, 1.0, L.stream()), reps=5)
    res.append(row("adamw f32 (400M params)", "pytorch_transformers AdamW (train_concap_struc.py:436-441)", t, 0,
                   28 * n, "none", "28 B/param: p,g,m,v read; p,m,v written"))
    del p, gr, m, v2

    # ---- column sums (bias gradients not fused into a LayerNorm backward)
    xx = torch.randn(ROWS_T, I, device=dev, generator=g)
    cs = torch.zeros(I, device=dev)
    t = timeit(lambda: ops.colsum(xx, cs))
    res.append(row("colsum f32 (20992x3072)", "bias grads of nn.Linear", t, 0, 4 * ROWS_T * I, "none"))

    out = {"config": "config 2 shapes, bs=64 (wide engine: %d text rows, %d image rows)" % (ROWS_T, ROWS_V),
           "method": "HIP events around each launch, median of 20 (5 for AdamW), warm caches; "
                     "roofline = max(FLOPs/peak, bytes/8 TB/s)", "rows": res}
    path = os.path.join(HERE, "profiles", out_name + ".json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("%-70s %9s %9s %9s %8s %6s" % ("kernel", "us", "TFLOP/s", "GB/s", "roof_us", "frac"))
    for r in res:
        print("%-70s %9.1f %9s %9.1f %8.1f %6.3f" % (r["kernel"][:70], r["time_us"], r["achieved_tflops"],
                                                   r["achieved_gbs"], r["roofline_us"], r["frac"]))


if __name__ == "__main__":
    main()
