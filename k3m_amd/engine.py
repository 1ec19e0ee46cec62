"""K3M tri-modal pretraining step on MI355X: forward + explicit backward over libk3m_hip kernels.

Reference: BertForMultiModalPreTraining_tri_stru (vilbert_k3m/vilbert_k3m.py:2186-2859) driven by
train_concap_struc.py:466-589.

MI355X-first organisation ("wide" passes)
-----------------------------------------
The reference runs three independent pair passes (calculate_for_text_img :1154,
calculate_for_pv_img :1332, calculate_for_two_text :1510) that each re-run the SHARED 12 text
layers and 6 image layers.  The layer index is in lock-step across the passes (every pass runs
text layers [t_start, t_end) and image layers [v_start, v_end) before co-attention block c), so
this engine stacks the streams of all passes row-wise and runs each shared layer ONCE per step:

    wide text buffer  [2B*T + 2B*P, 768] = [text(p1) | text(p3) | pv(p2) | pv(p3)]
    wide image buffer [2B*R, 1024]       = [img(p1)  | img(p2)]

One text-layer launch then covers 20,992 rows at bs=64 (4x fewer, 4x larger GEMMs than the
reference), and each weight gradient is one GEMM reducing over every use of the weight.
Co-attention block c applies the three pass-specific layers (c_layer, c_layer_pv_v,
c_layer_pv_t) to disjoint row slices.  Dropout masks are per row, so stacking is exact.

Parameters and gradients live in one flat fp32 buffer each (k3m_amd/params.py); weight
gradients are accumulated in place by the GEMM epilogue (beta = 1) and bias/LN gradients by the
reduction kernels, so there is no autograd bookkeeping on the hot path.
"""
import contextlib
import math
import os

import torch

from . import debug
from . import _lib as L
from . import ops
from .params import flat_layout

EPS = 1e-12


class Rng(object):
    """Counter-based RNG bookkeeping: each random site gets (seed, offset) and the backward pass
    regenerates its draws from the same pair."""

    def __init__(self, seed):
        self.seed = int(seed) & ((1 << 63) - 1)
        self.off = 0

    def take(self, n):
        o = self.off
        self.off += int(n)
        return o


class FlatParams(object):
    """All parameters (and their gradients) as views into single contiguous fp32 buffers, plus an
    optional bf16 shadow of the parameters (the operand copy for a bf16 encoder; fp32 stays the
    master copy that AdamW updates)."""

    def __init__(self, cfg, device, bf16_shadow=False):
        self.spec, self.offsets, self.segments, self.total, self.shapes = flat_layout(cfg)
        self.device = device
        self.data = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.data16 = torch.zeros(self.total, dtype=torch.bfloat16, device=device) if bf16_shadow else None
        self.shadow_fresh = False
        self.p, self.g = {}, {}
        for name, shape in self.spec:
            o = self.offsets[name]
            n = math.prod(shape)
            self.p[name] = self.data[o:o + n].view(shape)
            self.g[name] = self.grad[o:o + n].view(shape)

    def fused(self, names, grad=False, bf16=False):
        """Contiguous view spanning adjacent tensors (e.g. query|key|value weights -> [3H, H])."""
        buf = self.grad if grad else (self.data16 if bf16 else self.data)
        o = self.offsets[names[0]]
        n = 0
        for nm in names:
            assert self.offsets[nm] == o + n, "tensors are not adjacent: %s" % nm
            n += math.prod(self.shapes[nm])
        sh0 = self.shapes[names[0]]
        rows = sum(self.shapes[nm][0] for nm in names)
        return buf[o:o + n].view((rows,) + tuple(sh0[1:]))

    def load(self, values):
        for name, _ in self.spec:
            v = values[name]
            t = torch.as_tensor(v) if not isinstance(v, torch.Tensor) else v
            self.p[name].copy_(t.to(torch.float32).reshape(self.shapes[name]))
        self.shadow_fresh = False

    def p16(self, name):
        """bf16 shadow view of one parameter (bf16 mode only)."""
        o = self.offsets[name]
        return self.data16[o:o + math.prod(self.shapes[name])].view(self.shapes[name])

    def refresh_shadow(self):
        """bf16 shadow <- fp32 parameters (after loads / external optimizers; the Trainer's AdamW
        writes the shadow itself)."""
        if self.data16 is not None and not self.shadow_fresh:
            ops.convert(self.data, self.data16)
        self.shadow_fresh = True

    def state_dict(self):
        sd = {}
        for name, _ in self.spec:
            sd[name] = self.p[name]
        if "cls.predictions.bias" in self.p:   # the tied MLM decoder of the pretraining model
            sd["cls.predictions.decoder.weight"] = self.p["embeddings.word_embeddings.weight"]
        return sd


class Lin(object):
    """A (possibly fused) Linear: weight [N,K] / bias [N] views + gradient views."""

    def __init__(self, fp, prefixes):
        if isinstance(prefixes, str):
            prefixes = [prefixes]
        w = [p + ".weight" for p in prefixes]
        b = [p + ".bias" for p in prefixes]
        self.W, self.gW = fp.fused(w), fp.fused(w, True)
        self.b, self.gb = fp.fused(b), fp.fused(b, True)
        self.W16 = fp.fused(w, bf16=True) if fp.data16 is not None else None

    def _w(self, x):
        # operands share a dtype: a bf16 activation multiplies the bf16 weight shadow
        return self.W16 if x.dtype == torch.bfloat16 else self.W

    def fwd(self, x, out=None, epi=None, aux=None, alpha=1.0, beta=0.0, out_dtype=None):
        return ops.linear(x, self._w(x), self.b, out=out, epi=epi, aux=aux, alpha=alpha, beta=beta,
                          out_dtype=out_dtype)

    def wgrad(self, dy, x, alpha=1.0, bias_done=False):
        """bias_done: the bias gradient was already accumulated by dy's producer (k3m_ln_bwd dxsum)."""
        ops.linear_wgrad(dy, x, self.gW, None if bias_done else self.gb, alpha=alpha)

    def dgrad(self, dy, dx=None, beta=0.0, dgelu_aux=None, alpha=1.0, colsum_out=None):
        return ops.linear_dgrad(dy, self._w(dy), dx=dx, beta=beta, dgelu_aux=dgelu_aux, alpha=alpha,
                                colsum_out=colsum_out)


class LN(object):
    def __init__(self, fp, prefix):
        self.g, self.b = fp.p[prefix + ".weight"], fp.p[prefix + ".bias"]
        self.gg, self.gb = fp.g[prefix + ".weight"], fp.g[prefix + ".bias"]


# ---------------------------------------------------------------- sub-blocks

class AddLN(object):
    """y = LN(dropout(x) + res) (BertSelfOutput / BertOutput / BertBiOutput tails)."""

    def __init__(self, ln, p):
        self.ln, self.p = ln, p

    def fwd(self, x, res, rng, out=None):
        M, H = x.shape
        y = out if out is not None else torch.empty_like(x)
        xhat = torch.empty((M, H), dtype=x.dtype, device=x.device)
        rstd = torch.empty((M,), dtype=torch.float32, device=x.device)
        off = rng.take(M * H) if self.p > 0 else 0
        ops.ln_fwd(x, res, self.ln.g, self.ln.b, y, xhat, rstd, p_in=self.p, seed=rng.seed, off_in=off)
        return y, (xhat, rstd, rng.seed, off)

    def bwd(self, dy, saved, dres, dxsum=None):
        """writes d(res) into dres; returns d(x) (aliases dres when dropout is off).  dxsum: fp32
        [H] accumulating colsum(d(x)) — the bias gradient of the Linear that produced x."""
        xhat, rstd, seed, off = saved
        dx = dres if self.p == 0 else torch.empty_like(dres)
        ops.ln_bwd(dy, xhat, rstd, self.ln.g, dres, dx, self.ln.gg, self.ln.gb, p_in=self.p, seed=seed, off_in=off,
                   dxsum=dxsum)
        return dx


class FFN(object):
    """BertIntermediate(gelu) + BertOutput (post-LN), vilbert_k3m.py:504-532 / :665-693."""

    def __init__(self, fp, inter, outp, p):
        self.i = Lin(fp, inter + ".dense")
        self.o = Lin(fp, outp + ".dense")
        self.tail = AddLN(LN(fp, outp + ".LayerNorm"), p)

    def fwd(self, h, rng, out=None):
        M = h.shape[0]
        I = self.i.W.shape[0]
        u = torch.empty((M, I), dtype=h.dtype, device=h.device)
        f = self.i.fwd(h, epi=L.EPI_BIAS_GELU, aux=u)
        o = self.o.fwd(f)
        y, tsv = self.tail.fwd(o, h, rng, out=out)
        return y, (h, u, f, tsv)

    def bwd(self, dy, saved, dh_out=None):
        h, u, f, tsv = saved
        dh = dh_out if dh_out is not None else torch.empty_like(h)
        do = self.tail.bwd(dy, tsv, dh, dxsum=self.o.gb)
        self.o.wgrad(do, f, bias_done=True)
        du = self.o.dgrad(do, dgelu_aux=u, colsum_out=self.i.gb)   # + intermediate bias gradient
        self.i.wgrad(du, h, bias_done=True)
        self.i.dgrad(du, dx=dh, beta=1.0)
        return dh


def _flash(q, hd, lq, lk):
    # bf16 encoder: the LSE-saving bf16 kernels (attention_bf16.hip for whole heads of L <= 128,
    # attention_flash_long.hip up to L = 512); fp32: the exact-fp32 kernels (attention.hip, attention_long.hip)
    return q.dtype == torch.bfloat16 and (ops.flash_fits(lq, lk, hd) or ops.flash_long_fits(lq, lk, hd))


def _attn_fwd(q, k, v, mask, nseq, lq, lk, nh, p, rng, out=None):
    hd = q.shape[1] // nh
    ctx = out if out is not None else torch.empty((nseq * lq, q.shape[1]), dtype=q.dtype, device=q.device)
    off = rng.take(nseq * nh * lq * lk) if p > 0 else 0
    if _flash(q, hd, lq, lk):
        stat = torch.empty((nseq * nh * lq,), dtype=torch.float32, device=q.device)   # row LSE
        ops.flash_attn_fwd(q, k, v, mask, ctx, stat, nseq, lq, lk, nh, hd, 1.0 / math.sqrt(hd), p, rng.seed, off)
    else:
        stat = torch.empty((nseq * nh * lq * lk,), dtype=torch.float32, device=q.device)   # probabilities
        ops.attn_fwd(q, k, v, mask, ctx, stat, nseq, lq, lk, nh, hd, 1.0 / math.sqrt(hd), p, rng.seed, off)
    return ctx, (stat, mask, nseq, lq, lk, nh, hd, p, rng.seed, off)


def _attn_bwd(dctx, o, q, k, v, saved, dq, dk, dv):
    stat, mask, nseq, lq, lk, nh, hd, p, seed, off = saved
    if _flash(q, hd, lq, lk):
        ops.flash_attn_bwd(dctx, o, q, k, v, mask, stat, dq, dk, dv, nseq, lq, lk, nh, hd, 1.0 / math.sqrt(hd), p,
                           seed, off)
    else:
        ops.attn_bwd(dctx, o, q, k, v, stat, dq, dk, dv, nseq, lq, lk, nh, hd, 1.0 / math.sqrt(hd), p, seed, off)


class BertLayerOp(object):
    """BertLayer / BertImageLayer (vilbert_k3m.py:535-548, :696-709) over a wide buffer whose rows
    hold several sequence segments [(row0, nseq, L, mask)]."""

    def __init__(self, fp, prefix, nh, p_attn, p_hidden):
        self.qkv = Lin(fp, [prefix + ".attention.self.query", prefix + ".attention.self.key",
                            prefix + ".attention.self.value"])
        self.o = Lin(fp, prefix + ".attention.output.dense")
        self.tail = AddLN(LN(fp, prefix + ".attention.output.LayerNorm"), p_hidden)
        self.ffn = FFN(fp, prefix + ".intermediate", prefix + ".output", p_hidden)
        self.nh, self.p_attn = nh, p_attn

    def fwd(self, x, segs, rng):
        M, H = x.shape
        qkv = self.qkv.fwd(x)
        ctx = torch.empty((M, H), dtype=x.dtype, device=x.device)
        asv = []
        with ops.branches():   # the sequence segments (text 36, PV 128) are independent launches
            for (r0, nseq, ln, mask) in segs:
                r1 = r0 + nseq * ln
                _, s = ops.branch(_attn_fwd, qkv[r0:r1, 0:H], qkv[r0:r1, H:2 * H], qkv[r0:r1, 2 * H:], mask, nseq, ln,
                                  ln, self.nh, self.p_attn, rng, out=ctx[r0:r1])
                asv.append(s)
        a = self.o.fwd(ctx)
        h1, tsv = self.tail.fwd(a, x, rng)
        y, fsv = self.ffn.fwd(h1, rng)
        return y, (x, qkv, ctx, asv, tsv, fsv, segs)

    def bwd(self, dy, saved):
        x, qkv, ctx, asv, tsv, fsv, segs = saved
        M, H = x.shape
        dh1 = self.ffn.bwd(dy, fsv)
        dx = torch.empty_like(x)
        da = self.tail.bwd(dh1, tsv, dx, dxsum=self.o.gb)
        self.o.wgrad(da, ctx, bias_done=True)
        dctx = self.o.dgrad(da)
        dqkv = torch.empty_like(qkv)
        with ops.branches():
            for (r0, nseq, ln, mask), s in zip(segs, asv):
                r1 = r0 + nseq * ln
                ops.branch(_attn_bwd, dctx[r0:r1], ctx[r0:r1], qkv[r0:r1, 0:H], qkv[r0:r1, H:2 * H], qkv[r0:r1, 2 * H:],
                           s, dqkv[r0:r1, 0:H], dqkv[r0:r1, H:2 * H], dqkv[r0:r1, 2 * H:])
        self.qkv.wgrad(dqkv, x)
        self.qkv.dgrad(dqkv, dx=dx, beta=1.0)
        return dx


    # lock-step form (see ConnectionOp.fwd_steps): segments end at the GEMM stages
    def fwd_steps(self, x, segs, rng, res):
        M, H = x.shape
        qkv = self.qkv.fwd(x)
        yield
        ctx = torch.empty((M, H), dtype=x.dtype, device=x.device)
        asv = []
        for (r0, nseq, ln, mask) in segs:
            r1 = r0 + nseq * ln
            _, sv = _attn_fwd(qkv[r0:r1, 0:H], qkv[r0:r1, H:2 * H], qkv[r0:r1, 2 * H:], mask, nseq, ln, ln, self.nh,
                              self.p_attn, rng, out=ctx[r0:r1])
            asv.append(sv)
        a = self.o.fwd(ctx)
        yield
        h1, tsv = self.tail.fwd(a, x, rng)
        u = torch.empty((M, self.ffn.i.W.shape[0]), dtype=h1.dtype, device=h1.device)
        f = self.ffn.i.fwd(h1, epi=L.EPI_BIAS_GELU, aux=u)
        yield
        o = self.ffn.o.fwd(f)
        yield
        y, ts2 = self.ffn.tail.fwd(o, h1, rng)
        res.append((y, (x, qkv, ctx, asv, tsv, (h1, u, f, ts2), segs)))

    def bwd_steps(self, dy, saved, res):
        x, qkv, ctx, asv, tsv, fsv, segs = saved
        M, H = x.shape
        h1, u, f, ts2 = fsv
        dh1 = torch.empty_like(h1)
        do = self.ffn.tail.bwd(dy, ts2, dh1, dxsum=self.ffn.o.gb)
        self.ffn.o.wgrad(do, f, bias_done=True)
        du = self.ffn.o.dgrad(do, dgelu_aux=u, colsum_out=self.ffn.i.gb)
        yield
        self.ffn.i.wgrad(du, h1, bias_done=True)
        self.ffn.i.dgrad(du, dx=dh1, beta=1.0)
        yield
        dx = torch.empty_like(x)
        da = self.tail.bwd(dh1, tsv, dx, dxsum=self.o.gb)
        self.o.wgrad(da, ctx, bias_done=True)
        dctx = self.o.dgrad(da)
        yield
        dqkv = torch.empty_like(qkv)
        for (r0, nseq, ln, mask), sv in zip(segs, asv):
            r1 = r0 + nseq * ln
            _attn_bwd(dctx[r0:r1], ctx[r0:r1], qkv[r0:r1, 0:H], qkv[r0:r1, H:2 * H], qkv[r0:r1, 2 * H:], sv,
                      dqkv[r0:r1, 0:H], dqkv[r0:r1, H:2 * H], dqkv[r0:r1, 2 * H:])
        self.qkv.wgrad(dqkv, x)
        self.qkv.dgrad(dqkv, dx=dx, beta=1.0)
        res.append(dx)


class ConnectionOp(object):
    """BertConnectionLayer / BertConnectionLayer_two_text (vilbert_k3m.py:1030-1111):
    bi-directional attention between stream 1 (image or PV) and stream 2 (text or PV)."""

    def __init__(self, fp, prefix, nh, p_attn1, p_attn2, p_h1, p_h2, p_ffn1, p_ffn2):
        b = prefix + ".biattention."
        self.qkv1 = Lin(fp, [b + "query1", b + "key1", b + "value1"])
        self.qkv2 = Lin(fp, [b + "query2", b + "key2", b + "value2"])
        o = prefix + ".biOutput."
        self.d1, self.d2 = Lin(fp, o + "dense1"), Lin(fp, o + "dense2")
        self.t1 = AddLN(LN(fp, o + "LayerNorm1"), p_h1)
        self.t2 = AddLN(LN(fp, o + "LayerNorm2"), p_h2)
        self.f1 = FFN(fp, prefix + ".v_intermediate", prefix + ".v_output", p_ffn1)
        self.f2 = FFN(fp, prefix + ".t_intermediate", prefix + ".t_output", p_ffn2)
        self.nh, self.pa1, self.pa2 = nh, p_attn1, p_attn2

    def fwd(self, s1, s2, nseq, l1, l2, mask1, mask2, rng, out1, out2):
        Hb = self.qkv1.W.shape[0] // 3
        q1 = self.qkv1.fwd(s1)
        q2 = self.qkv2.fwd(s2)
        # ctx1: stream-2 queries over stream-1 keys (+ stream-1 mask); ctx2 the converse (:786-824)
        ctx1, a1s = _attn_fwd(q2[:, 0:Hb], q1[:, Hb:2 * Hb], q1[:, 2 * Hb:], mask1, nseq, l2, l1, self.nh, self.pa1, rng)
        ctx2, a2s = _attn_fwd(q1[:, 0:Hb], q2[:, Hb:2 * Hb], q2[:, 2 * Hb:], mask2, nseq, l1, l2, self.nh, self.pa2, rng)
        h1, t1s = self.t1.fwd(self.d1.fwd(ctx2), s1, rng)
        h2, t2s = self.t2.fwd(self.d2.fwd(ctx1), s2, rng)
        _, f1s = self.f1.fwd(h1, rng, out=out1)
        _, f2s = self.f2.fwd(h2, rng, out=out2)
        return (s1, s2, q1, q2, ctx1, ctx2, a1s, a2s, t1s, t2s, f1s, f2s, Hb)

    def bwd(self, dy1, dy2, saved, ds1, ds2):
        s1, s2, q1, q2, ctx1, ctx2, a1s, a2s, t1s, t2s, f1s, f2s, Hb = saved
        dh1 = self.f1.bwd(dy1, f1s)
        dh2 = self.f2.bwd(dy2, f2s)
        da1 = self.t1.bwd(dh1, t1s, ds1, dxsum=self.d1.gb)
        da2 = self.t2.bwd(dh2, t2s, ds2, dxsum=self.d2.gb)
        self.d1.wgrad(da1, ctx2, bias_done=True)
        dctx2 = self.d1.dgrad(da1)
        self.d2.wgrad(da2, ctx1, bias_done=True)
        dctx1 = self.d2.dgrad(da2)
        dq1 = torch.empty_like(q1)
        dq2 = torch.empty_like(q2)
        _attn_bwd(dctx1, ctx1, q2[:, 0:Hb], q1[:, Hb:2 * Hb], q1[:, 2 * Hb:], a1s, dq2[:, 0:Hb], dq1[:, Hb:2 * Hb],
                  dq1[:, 2 * Hb:])
        _attn_bwd(dctx2, ctx2, q1[:, 0:Hb], q2[:, Hb:2 * Hb], q2[:, 2 * Hb:], a2s, dq1[:, 0:Hb], dq2[:, Hb:2 * Hb],
                  dq2[:, 2 * Hb:])
        self.qkv1.wgrad(dq1, s1)
        self.qkv1.dgrad(dq1, dx=ds1, beta=1.0)
        self.qkv2.wgrad(dq2, s2)
        self.qkv2.dgrad(dq2, dx=ds2, beta=1.0)


    # ---- lock-step form: the same computation as fwd / bwd cut into segments at the GEMM stages, so
    # the three co-attention blocks of one schedule step issue their (independent) GEMMs together and
    # each stage runs as one grouped launch (_lockstep).  Inside a segment no op reads a GEMM output
    # of the same segment.
    def fwd_steps(self, s1, s2, nseq, l1, l2, mask1, mask2, rng, out1, out2, res):
        Hb = self.qkv1.W.shape[0] // 3
        q1 = self.qkv1.fwd(s1)
        q2 = self.qkv2.fwd(s2)
        yield
        ctx1, a1s = ops.branch(_attn_fwd, q2[:, 0:Hb], q1[:, Hb:2 * Hb], q1[:, 2 * Hb:], mask1, nseq, l2, l1, self.nh,
                               self.pa1, rng)
        ctx2, a2s = ops.branch(_attn_fwd, q1[:, 0:Hb], q2[:, Hb:2 * Hb], q2[:, 2 * Hb:], mask2, nseq, l1, l2, self.nh,
                               self.pa2, rng)
        x1 = self.d1.fwd(ctx2)
        x2 = self.d2.fwd(ctx1)
        yield
        h1, t1s = self.t1.fwd(x1, s1, rng)
        h2, t2s = self.t2.fwd(x2, s2, rng)
        u1 = torch.empty((h1.shape[0], self.f1.i.W.shape[0]), dtype=h1.dtype, device=h1.device)
        u2 = torch.empty((h2.shape[0], self.f2.i.W.shape[0]), dtype=h2.dtype, device=h2.device)
        g1 = self.f1.i.fwd(h1, epi=L.EPI_BIAS_GELU, aux=u1)
        g2 = self.f2.i.fwd(h2, epi=L.EPI_BIAS_GELU, aux=u2)
        yield
        o1 = self.f1.o.fwd(g1)
        o2 = self.f2.o.fwd(g2)
        yield
        _, ts1 = self.f1.tail.fwd(o1, h1, rng, out=out1)
        _, ts2 = self.f2.tail.fwd(o2, h2, rng, out=out2)
        res.append((s1, s2, q1, q2, ctx1, ctx2, a1s, a2s, t1s, t2s, (h1, u1, g1, ts1), (h2, u2, g2, ts2), Hb))

    def bwd_steps(self, dy1, dy2, saved, ds1, ds2):
        s1, s2, q1, q2, ctx1, ctx2, a1s, a2s, t1s, t2s, f1s, f2s, Hb = saved
        (h1, u1, g1, ts1), (h2, u2, g2, ts2) = f1s, f2s
        dh1, dh2 = torch.empty_like(h1), torch.empty_like(h2)
        do1 = self.f1.tail.bwd(dy1, ts1, dh1, dxsum=self.f1.o.gb)
        do2 = self.f2.tail.bwd(dy2, ts2, dh2, dxsum=self.f2.o.gb)
        self.f1.o.wgrad(do1, g1, bias_done=True)
        self.f2.o.wgrad(do2, g2, bias_done=True)
        du1 = self.f1.o.dgrad(do1, dgelu_aux=u1, colsum_out=self.f1.i.gb)
        du2 = self.f2.o.dgrad(do2, dgelu_aux=u2, colsum_out=self.f2.i.gb)
        yield
        self.f1.i.wgrad(du1, h1, bias_done=True)
        self.f2.i.wgrad(du2, h2, bias_done=True)
        self.f1.i.dgrad(du1, dx=dh1, beta=1.0)
        self.f2.i.dgrad(du2, dx=dh2, beta=1.0)
        yield
        da1 = self.t1.bwd(dh1, t1s, ds1, dxsum=self.d1.gb)
        da2 = self.t2.bwd(dh2, t2s, ds2, dxsum=self.d2.gb)
        self.d1.wgrad(da1, ctx2, bias_done=True)
        self.d2.wgrad(da2, ctx1, bias_done=True)
        dctx2 = self.d1.dgrad(da1)
        dctx1 = self.d2.dgrad(da2)
        yield
        dq1 = torch.empty_like(q1)
        dq2 = torch.empty_like(q2)
        ops.branch(_attn_bwd, dctx1, ctx1, q2[:, 0:Hb], q1[:, Hb:2 * Hb], q1[:, 2 * Hb:], a1s, dq2[:, 0:Hb],
                   dq1[:, Hb:2 * Hb], dq1[:, 2 * Hb:])
        ops.branch(_attn_bwd, dctx2, ctx2, q1[:, 0:Hb], q2[:, Hb:2 * Hb], q2[:, 2 * Hb:], a2s, dq1[:, 0:Hb],
                   dq2[:, Hb:2 * Hb], dq2[:, 2 * Hb:])
        self.qkv1.wgrad(dq1, s1)
        self.qkv2.wgrad(dq2, s2)
        self.qkv1.dgrad(dq1, dx=ds1, beta=1.0)
        self.qkv2.dgrad(dq2, dx=ds2, beta=1.0)


GROUPED = os.environ.get("K3M_GROUPED", "1") != "0"
# text + image layer lock step: off by default — the text layers' GEMMs already fill the chip and the
# mixed group measured 2.3 % slower (434.5 vs 444.6 samples/s, same box, A/B/A/B)
GROUP_GATE = GROUPED and os.environ.get("K3M_GROUP_GATE", "1") != "0"   # the three fusion-gate GEMMs
GROUP_TV = GROUPED and os.environ.get("K3M_GROUP_TV", "0") == "1"


def _lockstep(gens):
    """Run generators segment by segment; each round's GEMMs are issued under one ops.grouped()."""
    live = list(gens)
    while live:
        nxt = []
        with ops.grouped():
            with ops.branches():   # closes (main waits for the side streams) before the GEMM flush
                for g in live:
                    try:
                        next(g)
                        nxt.append(g)
                    except StopIteration:
                        pass
        live = nxt


def label_counts(batch):
    """(masked-LM labels of text + PV, masked regions): the row counts of the labelled-row heads.
    A loader that builds the batch on the host stores them as batch["_label_counts"] so the forward
    needs no device->host sync; this helper computes them from a batch (one sync)."""
    n_m = int((batch["lm_label_ids"] >= 0).sum()) + int((batch["lm_label_ids_pv"] >= 0).sum())
    n_v = int((batch["image_label"] >= 1).sum())
    return (n_m, n_v)


def _ext_mask(m):
    # (1 - mask) * -10000 additive key mask (vilbert_k3m.py:2547-2580); input marshalling
    return ((1.0 - m.to(torch.float32)) * -10000.0).contiguous()


class K3MEngine(object):
    """One replica of the model on one GPU (one process per GPU; DDP in k3m_amd/ddp.py)."""

    def __init__(self, cfg, device=None, seed=1234, dtype="fp32"):
        """dtype: "fp32" (everything fp32) or "bf16" (mixed precision: the encoder — text, image and
        co-attention layers, >95% of the FLOPs — keeps activations and activation gradients in bf16
        and multiplies the bf16 weight shadow on the bf16 MFMA; embeddings, fusion, heads, losses,
        parameter gradients and AdamW stay fp32)."""
        self.cfg = cfg
        self.device = torch.device(device if device is not None else "cuda")
        L.load()
        assert dtype in ("fp32", "bf16")
        self.dtype = dtype
        self.enc_dtype = torch.bfloat16 if dtype == "bf16" else torch.float32
        fp = self.fp = FlatParams(cfg, self.device, bf16_shadow=(dtype == "bf16"))
        self.base_seed = int(seed)
        self.step_count = 0
        # hipGraph capture (k3m_amd/graph.py): graph_seed = device address of the seed word the replay refills;
        # launches then pass K3M_GRAPH_SEED | address and draw with that word's value.  The label-count check
        # is left to the replay (no host work inside a capture).
        self.graph_seed = 0
        self.capturing = False
        self.captured_counts = None
        # tests: keep copies of the labelled-row MLM logits and masked-region logits of each forward
        # (out["mlm_logits"] rows in compaction order — text rows, then PV rows, row-major; out["img_logits"])
        self.capture_logits = False
        c = cfg
        assert getattr(c, "fixed_t_layer", 0) == 0 and getattr(c, "fixed_v_layer", 0) == 0
        assert not getattr(c, "in_batch_pairs", False) and not getattr(c, "fast_mode", False)
        assert not getattr(c, "dynamic_attention", False) and getattr(c, "model", "bert") in ("bert", "roberta")
        assert getattr(c, "use_image", True) and c.with_coattention
        assert getattr(c, "visual_target", 0) == 0
        self.H, self.Hv, self.Hb = c.hidden_size, c.v_hidden_size, c.bi_hidden_size
        self.p_h = c.hidden_dropout_prob
        self.p_a = c.attention_probs_dropout_prob
        self.p_vh = c.v_hidden_dropout_prob
        self.p_va = c.v_attention_probs_dropout_prob
        self.text = [BertLayerOp(fp, "encoder.layer.%d" % i, c.num_attention_heads, self.p_a, self.p_h)
                     for i in range(c.num_hidden_layers)]
        self.image = [BertLayerOp(fp, "encoder.v_layer.%d" % i, c.v_num_attention_heads, self.p_va, self.p_vh)
                      for i in range(c.v_num_hidden_layers)]
        nco = len(c.v_biattention_id)
        nb = c.bi_num_attention_heads
        self.co_tv = [ConnectionOp(fp, "encoder.c_layer.%d" % i, nb, self.p_va, self.p_a, self.p_vh, self.p_h,
                                   self.p_vh, self.p_h) for i in range(nco)]
        self.co_pv = [ConnectionOp(fp, "encoder.c_layer_pv_v.%d" % i, nb, self.p_va, self.p_a, self.p_vh, self.p_h,
                                   self.p_vh, self.p_h) for i in range(nco)]
        self.co_tt = [ConnectionOp(fp, "encoder.c_layer_pv_t.%d" % i, nb, self.p_va, self.p_a, self.p_vh, self.p_h,
                                   self.p_h, self.p_h) for i in range(nco)]
        self.emb_ln = LN(fp, "embeddings.LayerNorm")
        self.vemb_img = Lin(fp, "v_embeddings.image_embeddings")
        self.vemb_loc = Lin(fp, "v_embeddings.image_location_embeddings")
        self.vemb_ln = LN(fp, "v_embeddings.LayerNorm")
        self.gate = {m: Lin(fp, ["score_self_%s" % m, "score_cross1_%s" % m, "score_cross2_%s" % m])
                     for m in ("v", "t", "pv")}
        self.map_b2i = Lin(fp, "map_bi_to_individual")
        # "pretrain": the pretraining heads + LPM; "item_alignment": the encoder up to c_final only
        # (K3MForItemAlignment.item_embedding, vilbert_k3m.py:3329-3377; its pair head is k3m_amd.finetune)
        self.task = getattr(c, "task", "pretrain")
        if self.task == "pretrain":
            self.mlm_t = Lin(fp, "cls.predictions.transform.dense")
            self.mlm_ln = LN(fp, "cls.predictions.transform.LayerNorm")
            self.img_t = Lin(fp, "cls.imagePredictions.transform.dense")
            self.img_ln = LN(fp, "cls.imagePredictions.transform.LayerNorm")
            self.img_dec = Lin(fp, "cls.imagePredictions.decoder")
        self.sw1, self.sw3 = Lin(fp, "struc_w1"), Lin(fp, "struc_w3")
        self.schedule = self._schedule()

    def _lo(self, x):
        """bf16 operand copy of an fp32 activation for the large fp32-region GEMMs (fusion gates, tied
        MLM decoder) in bf16 mode; the activation itself stays fp32.  Identity in fp32 mode."""
        if self.dtype != "bf16":
            return x
        return ops.convert(x.contiguous(), torch.empty(x.shape, dtype=torch.bfloat16, device=x.device))

    # ------------------------------------------------------------ encoder schedule
    def _schedule(self):
        """[(kind, index)] in lock-step order: ('t', i) text layer on all four text/PV streams,
        ('v', i) image layer on both image streams, ('c', i) co-attention block i."""
        c = self.cfg
        sch = []
        t0 = v0 = 0
        for i, (v1, t1) in enumerate(zip(c.v_biattention_id, c.t_biattention_id)):
            sch += [("t", k) for k in range(t0, t1)]
            sch += [("v", k) for k in range(v0, v1)]
            sch.append(("c", i))
            t0, v0 = t1, v1
        sch += [("v", k) for k in range(v0, c.v_num_hidden_layers)]
        sch += [("t", k) for k in range(t0, c.num_hidden_layers)]
        return sch

    # ------------------------------------------------------------ forward
    def _verify_hint(self, hint, cnt):
        """Check a host-side label-count hint against the device count without blocking: the count is
        copied to pinned memory behind an event and compared once the event has completed (a later
        forward, or check_hints(wait=True)); a mismatch raises — the head buffers were sized wrong."""
        host = torch.empty((2,), dtype=torch.int32, pin_memory=True)
        host.copy_(cnt, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        if not hasattr(self, "_hint_checks"):
            self._hint_checks = []
        self._hint_checks.append((tuple(hint), host, ev))
        self.check_hints()

    def step_seed(self, seed):
        """The 63-bit seed forward(seed=seed) draws with (the word a graph replay writes)."""
        return Rng(self.base_seed * 1000003 + seed).seed

    def check_hints(self, wait=False):
        pend = getattr(self, "_hint_checks", [])
        while pend and (wait or pend[0][2].query()):
            hint, host, ev = pend.pop(0)
            ev.synchronize()
            got = (int(host[0]), int(host[1]))
            if got != hint:
                pend.clear()
                raise RuntimeError("stale labelled-row count hint %s: the labels hold %s (labels edited after "
                                   "collation, or a hand-built _label_counts)" % (hint, got))

    def forward(self, batch, train=True, noise=None, ent_neg=None, val_neg=None, seed=None, groups=1):
        """Runs the forward of the step; returns (losses dict of device tensors, ctx for backward).

        batch: dict of device tensors with the reference names (A0 in SURVEY.md §8(a)).
        noise: optional {v,t,pv: [B, L, 3, D]} gumbel noise; ent_neg/val_neg optional [B,NPV,2].
        groups: the batch is that many independent model calls stacked along dim 0 (the item
        alignment pair: item 1 rows then item 2 rows); only the structure aggregator's
        zero-triple fallback crosses items, and it is kept inside each group."""
        c = self.cfg
        fp = self.fp
        if debug.ON:
            debug.check_batch(batch, c, ent_neg, val_neg)
        fp.refresh_shadow()
        dev = self.device
        H, Hv = self.H, self.Hv
        ED = self.enc_dtype
        ids, tt, mt = batch["input_ids"], batch["segment_ids"], batch["input_mask"]
        pids, ptt, mp = batch["input_ids_pv"], batch["segment_ids_pv"], batch["input_mask_pv"]
        feat, loc, mv = batch["image_feat"], batch["image_loc"], batch["image_mask"]
        B, T = ids.shape
        P = pids.shape[1]
        R = feat.shape[1]
        BT, BP, BR = B * T, B * P, B * R
        rng = Rng(self.base_seed * 1000003 + (seed if seed is not None else self.step_count))
        if self.graph_seed:
            rng.seed = L.GRAPH_SEED | int(self.graph_seed)
        ph = self.p_h if train else 0.0
        pvh = self.p_vh if train else 0.0
        ctx = {"B": B, "T": T, "P": P, "R": R, "train": train, "seed": rng.seed}

        mask_t, mask_p, mask_v = _ext_mask(mt), _ext_mask(mp), _ext_mask(mv)
        mask_t2 = torch.cat([mask_t, mask_t]).contiguous()
        mask_p2 = torch.cat([mask_p, mask_p]).contiguous()
        mask_v2 = torch.cat([mask_v, mask_v]).contiguous()

        # ---- embeddings (BertEmbeddings x2, BertImageEmbeddings)
        Nt = 2 * BT + 2 * BP
        XT = torch.empty((Nt, H), dtype=torch.float32, device=dev)
        ind_t = torch.empty((BT, H), dtype=torch.float32, device=dev)
        ind_pv = torch.empty((BP, H), dtype=torch.float32, device=dev)
        xh_t = torch.empty_like(ind_t)
        rs_t = torch.empty((BT,), dtype=torch.float32, device=dev)
        xh_p = torch.empty_like(ind_pv)
        rs_p = torch.empty((BP,), dtype=torch.float32, device=dev)
        off_t = rng.take(BT * H) if ph > 0 else 0
        ops.embed_fwd(ids, tt, fp.p["embeddings.word_embeddings.weight"], fp.p["embeddings.position_embeddings.weight"],
                      fp.p["embeddings.token_type_embeddings.weight"], self.emb_ln.g, self.emb_ln.b, ind_t, XT[0:BT],
                      XT[BT:2 * BT], xh_t, rs_t, ph, rng.seed, off_t)
        off_p = rng.take(BP * H) if ph > 0 else 0
        ops.embed_fwd(pids, ptt, fp.p["embeddings.word_embeddings.weight"], fp.p["embeddings.position_embeddings.weight"],
                      fp.p["embeddings.token_type_embeddings.weight"], self.emb_ln.g, self.emb_ln.b, ind_pv,
                      XT[2 * BT:2 * BT + BP], XT[2 * BT + BP:], xh_p, rs_p, ph, rng.seed, off_p)
        ctx["emb"] = (xh_t, rs_t, off_t, xh_p, rs_p, off_p)

        feat2 = feat.reshape(BR, feat.shape[2])
        loc2 = loc.reshape(BR, loc.shape[2])
        img = self.vemb_img.fwd(feat2)
        lce = self.vemb_loc.fwd(loc2)
        ind_v = torch.empty((BR, Hv), dtype=torch.float32, device=dev)
        xh_v = torch.empty_like(ind_v)
        rs_v = torch.empty((BR,), dtype=torch.float32, device=dev)
        off_v = rng.take(BR * Hv) if ph > 0 else 0
        ops.ln_fwd(img, lce, self.vemb_ln.g, self.vemb_ln.b, ind_v, xh_v, rs_v, p_out=ph, seed=rng.seed, off_out=off_v)
        XV = torch.empty((2 * BR, Hv), dtype=ED, device=dev)
        ops.convert(ind_v, XV[0:BR])
        ops.convert(ind_v, XV[BR:])
        if ED != torch.float32:
            XT = ops.convert(XT, torch.empty((Nt, H), dtype=ED, device=dev))
        ctx["vemb"] = (feat2, loc2, xh_v, rs_v, off_v)

        # ---- encoder, lock-step wide passes
        tsegs = [(0, 2 * B, T, mask_t2), (2 * BT, 2 * B, P, mask_p2)]
        vsegs = [(0, 2 * B, R, mask_v2)]
        enc = []
        sched = list(self.schedule)
        si = 0
        while si < len(sched):
            kind, i = sched[si]
            nxt = sched[si + 1] if si + 1 < len(sched) else None
            if GROUP_TV and nxt is not None and {kind, nxt[0]} == {"t", "v"}:
                # a text layer and an image layer at the same schedule position are independent:
                # run them in lock step so their GEMM stages share grouped launches
                pair = [(kind, i), nxt]
                gens, outs = [], []
                for k_, j_ in pair:
                    op = self.text[j_] if k_ == "t" else self.image[j_]
                    if not train:
                        op = _eval_view(op)
                    r = []
                    outs.append(r)
                    gens.append(op.fwd_steps(XT if k_ == "t" else XV, tsegs if k_ == "t" else vsegs, rng, r))
                _lockstep(gens)
                for (k_, j_), r in zip(pair, outs):
                    y, sv = r[0]
                    if k_ == "t":
                        XT = y
                    else:
                        XV = y
                    enc.append((k_, j_, sv))
                si += 2
                continue
            si += 1
            if kind == "t":
                op = self.text[i]
                if not train:
                    op = _eval_view(op)
                XT, sv = op.fwd(XT, tsegs, rng)
                enc.append((kind, i, sv))
            elif kind == "v":
                op = self.image[i]
                if not train:
                    op = _eval_view(op)
                XV, sv = op.fwd(XV, vsegs, rng)
                enc.append((kind, i, sv))
            else:
                XT2 = torch.empty_like(XT)
                XV2 = torch.empty_like(XV)
                ops_ = [self.co_tv[i], self.co_pv[i], self.co_tt[i]]
                if not train:
                    ops_ = [_eval_view(o) for o in ops_]
                args = [(XV[0:BR], XT[0:BT], B, R, T, mask_v, mask_t, rng, XV2[0:BR], XT2[0:BT]),
                        (XV[BR:], XT[2 * BT:2 * BT + BP], B, R, P, mask_v, mask_p, rng, XV2[BR:],
                         XT2[2 * BT:2 * BT + BP]),
                        (XT[2 * BT + BP:], XT[BT:2 * BT], B, P, T, mask_p, mask_t, rng, XT2[2 * BT + BP:],
                         XT2[BT:2 * BT])]
                if GROUPED:
                    res = [[], [], []]
                    _lockstep([o.fwd_steps(*a, res=r) for o, a, r in zip(ops_, args, res)])
                    s_tv, s_pv, s_tt = res[0][0], res[1][0], res[2][0]
                else:
                    s_tv, s_pv, s_tt = [o.fwd(*a) for o, a in zip(ops_, args)]
                enc.append((kind, i, (s_tv, s_pv, s_tt, ops_)))
                XT, XV = XT2, XV2
        ctx["enc"] = enc
        if ED != torch.float32:   # encoder -> fp32 fusion / heads
            XT = ops.convert(XT, torch.empty((Nt, H), dtype=torch.float32, device=dev))
            XV = ops.convert(XV, torch.empty((2 * BR, Hv), dtype=torch.float32, device=dev))
        ctx["XT"], ctx["XV"] = XT, XV

        # ---- initial-interactive fusion (get_sequence_pooled_output_final :2376-2411)
        mode = getattr(c, "if_pre_sampling", 1)
        seq_tp = torch.empty((BT + BP, H), dtype=torch.float32, device=dev)
        seq_v = torch.empty((BR, Hv), dtype=torch.float32, device=dev)
        streams = {
            "v": (ind_v, XV[0:BR], XV[BR:], seq_v, Hv),
            "t": (ind_t, XT[0:BT], XT[BT:2 * BT], seq_tp[0:BT], H),
            "pv": (ind_pv, XT[2 * BT:2 * BT + BP], XT[2 * BT + BP:], seq_tp[BT:], H),
        }
        fus = {}
        gate_a = {}
        if mode == 1:   # the three modalities' gate GEMMs are independent: one grouped launch (GROUP_GATE)
            ccs = {}
            for m in ("v", "t", "pv"):
                x0, x1, x2, out, D = streams[m]
                rows = x0.shape[0]
                cc = torch.empty((rows, 3 * D), dtype=torch.float32, device=dev)
                L.call("k3m_relu_cat3", x0.data_ptr(), x1.data_ptr(), x2.data_ptr(), cc.data_ptr(), rows, D, L.F32,
                       L.stream())
                ccs[m] = (cc, self._lo(cc))
            with (ops.grouped() if GROUP_GATE else contextlib.nullcontext()):
                for m in ("v", "t", "pv"):
                    gate_a[m] = self.gate[m].fwd(ccs[m][1], epi=L.EPI_BIAS_SIGMOID, out_dtype=torch.float32)
        for m in ("v", "t", "pv"):
            x0, x1, x2, out, D = streams[m]
            rows = x0.shape[0]
            if mode == 1:
                cc = ccs[m][0]
                a = gate_a[m]
                ys = torch.empty_like(a)
                idx = torch.empty((rows * D,), dtype=torch.uint8, device=dev)
                nz = None
                off_g = 0
                if noise is not None:
                    nz = noise[m].reshape(rows * 3 * D).to(device=dev, dtype=torch.float32).contiguous()
                else:
                    off_g = rng.take(rows * 3 * D)
                L.call("k3m_gate_fwd", a.data_ptr(), cc.data_ptr(), L.ptr(nz), ys.data_ptr(), idx.data_ptr(),
                       out.data_ptr(), rows, D, rng.seed, off_g, L.F32, L.stream())
                fus[m] = (cc, a, ys, idx)
            elif mode == 0:
                L.call("k3m_mean3", x0.data_ptr(), x1.data_ptr(), x2.data_ptr(), out.data_ptr(), out.numel(), L.F32,
                       L.stream())
                fus[m] = None
            else:
                raise NotImplementedError("if_pre_sampling=%s" % mode)
        ctx["fus"] = (fus, streams, mode)
        ctx["seq_tp"], ctx["seq_v"] = seq_tp, seq_v

        # ---- pooled outputs and c_initial (:2404-2409, :2722-2725)
        mean_v = torch.empty((B, Hv), dtype=torch.float32, device=dev)
        pooled_t = torch.empty((B, H), dtype=torch.float32, device=dev)
        pooled_pv = torch.empty((B, H), dtype=torch.float32, device=dev)
        L.call("k3m_seq_mean", seq_v.data_ptr(), B, R, 1, Hv, 1.0, mean_v.data_ptr(), 0, L.F32, L.stream())
        L.call("k3m_seq_mean", seq_tp.data_ptr(), B, T, 1, H, 1.0, pooled_t.data_ptr(), 0, L.F32, L.stream())
        L.call("k3m_seq_mean", seq_tp[BT:].data_ptr(), B, P, 1, H, 1.0, pooled_pv.data_ptr(), 0, L.F32, L.stream())
        pooled_v = self.map_b2i.fwd(mean_v)
        c_init = torch.empty((B, H), dtype=torch.float32, device=dev)
        L.call("k3m_mean3", pooled_v.data_ptr(), pooled_t.data_ptr(), pooled_pv.data_ptr(), c_init.data_ptr(),
               c_init.numel(), L.F32, L.stream())
        ctx["pool"] = (mean_v,)

        # ---- structure aggregator + LPM (:2413-2505)
        index_p, index_v = batch["index_p"].contiguous(), batch["index_v"].contiguous()
        NPV = index_p.shape[1]
        X = torch.empty((B * NPV, 3 * H), dtype=torch.float32, device=dev)
        nvalid = torch.empty((B,), dtype=torch.int32, device=dev)
        src = torch.empty((B,), dtype=torch.int32, device=dev)
        assert B % groups == 0
        Bg = B // groups
        for gi in range(groups):   # src (zero-triple fallback) is group-relative
            r0 = gi * Bg
            L.call("k3m_sa_gather", seq_tp[BT + r0 * P:].data_ptr(), index_p[r0:].data_ptr(), index_v[r0:].data_ptr(),
                   c_init[r0:].data_ptr(), X[r0 * NPV:].data_ptr(), nvalid[r0:].data_ptr(), src[r0:].data_ptr(), Bg, P,
                   NPV, H, L.F32, L.stream())
        Tm = self.sw1.fwd(X)
        att = torch.empty((B, NPV), dtype=torch.float32, device=dev)
        agg = torch.empty((B, H), dtype=torch.float32, device=dev)
        for gi in range(groups):
            r0 = gi * Bg
            L.call("k3m_sa_attn_fwd", Tm[r0 * NPV:].data_ptr(), nvalid[r0:].data_ptr(), src[r0:].data_ptr(),
                   fp.p["struc_w2.weight"].data_ptr(), fp.p["struc_w2.bias"].data_ptr(), c_init[r0:].data_ptr(),
                   att[r0:].data_ptr(), agg[r0:].data_ptr(), Bg, NPV, H, L.stream())
        c_final = c_init.clone()
        self.sw3.fwd(agg, out=c_final, beta=1.0)
        if self.task != "pretrain":
            ctx["struct"] = (X, nvalid, src, Tm, att, agg, c_init, c_final, None, None, None, index_p, index_v, NPV,
                             None)
            ctx["groups"] = groups
            ctx["batch"] = batch
            return {"c_initial": c_init, "c_final": c_final, "pooled_t": pooled_t, "pooled_pv": pooled_pv,
                    "pooled_v": pooled_v}, ctx
        assert groups == 1
        nneg = int(getattr(c, "num_negative_pv", 4))
        if ent_neg is None:
            ke, kv = nneg // 2, nneg - nneg // 2   # vilbert_k3m.py:2476, :2488
            ent_neg = torch.empty((B, NPV, ke), dtype=torch.int64, device=dev)
            val_neg = torch.empty((B, NPV, kv), dtype=torch.int64, device=dev)
            L.call("k3m_lpm_sample", nvalid.data_ptr(), B, NPV, ke, kv, rng.seed, rng.take(B * NPV * (ke + kv)),
                   L.ptr(ent_neg), L.ptr(val_neg), L.stream())
        else:
            ent_neg = ent_neg.to(device=dev, dtype=torch.int64).contiguous()
            val_neg = val_neg.to(device=dev, dtype=torch.int64).contiguous()
            ke, kv = ent_neg.shape[2], val_neg.shape[2]
        lpm = torch.empty((1,), dtype=torch.float32, device=dev)
        lws = torch.empty((B * NPV * (2 * (ke + kv) + 1) + 2,), dtype=torch.float32, device=dev)
        margin = float(getattr(c, "margin", 1.0))
        L.call("k3m_lpm_fwd", c_final.data_ptr(), X.data_ptr(), nvalid.data_ptr(), L.ptr(ent_neg), L.ptr(val_neg), B, NPV,
               H, ke, kv, margin, lpm.data_ptr(), lws.data_ptr(), L.stream())
        ctx["struct"] = (X, nvalid, src, Tm, att, agg, c_init, c_final, ent_neg, val_neg, lws, index_p, index_v, NPV,
                         margin)

        # ---- heads on labelled rows only (unlabelled logits do not reach the loss or the gradients)
        losses = torch.zeros((4,), dtype=torch.float32, device=dev)   # mlm_t, mlm_pv, img, -
        nmax = BT + BP
        # zero-filled: rows past the device count (a hint larger than the true count) gather row 0 with
        # row_scale 0 and add nothing to any loss or gradient; a smaller hint is caught by check_hints
        idx_m = torch.zeros((nmax,), dtype=torch.int32, device=dev)
        lab_m = torch.zeros((nmax,), dtype=torch.int64, device=dev)
        sc_m = torch.zeros((nmax,), dtype=torch.float32, device=dev)
        sl_m = torch.zeros((nmax,), dtype=torch.int32, device=dev)
        cnt = torch.zeros((2,), dtype=torch.int32, device=dev)
        L.call("k3m_compact_labels_ex", batch["lm_label_ids"].contiguous().data_ptr(), BT, 0, T, T, 0, 0,
               idx_m.data_ptr(), lab_m.data_ptr(), None, sc_m.data_ptr(), sl_m.data_ptr(), cnt.data_ptr(), L.stream())
        L.call("k3m_compact_labels_ex", batch["lm_label_ids_pv"].contiguous().data_ptr(), BP, 0, P, P, BT, 1,
               idx_m.data_ptr(), lab_m.data_ptr(), None, sc_m.data_ptr(), sl_m.data_ptr(), cnt.data_ptr(), L.stream())
        R1 = R - 1
        idx_v = torch.zeros((B * R1,), dtype=torch.int32, device=dev)
        src_v = torch.zeros((B * R1,), dtype=torch.int32, device=dev)
        sc_v = torch.zeros((B * R1,), dtype=torch.float32, device=dev)
        sl_v = torch.zeros((B * R1,), dtype=torch.int32, device=dev)
        cnt_v = cnt[1:2]
        L.call("k3m_compact_labels_ex", batch["image_label"].contiguous().data_ptr(), B * R1, 1, R1, R, 1, 2,
               idx_v.data_ptr(), None, src_v.data_ptr(), sc_v.data_ptr(), sl_v.data_ptr(), cnt_v.data_ptr(),
               L.stream())
        hint = batch.get("_label_counts")
        if hint is not None:   # counted on the host when the batch was built (label_counts): no sync
            n_m, n_v = int(hint[0]), int(hint[1])
            if self.capturing:
                self.captured_counts = cnt   # checked by the graph after each replay
            else:
                self._verify_hint((n_m, n_v), cnt)
        else:
            n_m, n_v = [int(x) for x in cnt.tolist()]   # host sync (labelled-row counts)

        V = c.vocab_size
        hm = torch.empty((n_m, H), dtype=torch.float32, device=dev)
        ops.gather_rows(seq_tp, idx_m, n_m, hm)
        pre_m = torch.empty_like(hm)
        hm1 = self.mlm_t.fwd(hm, epi=L.EPI_BIAS_GELU, aux=pre_m)
        hl = torch.empty_like(hm)
        xh_m = torch.empty_like(hm)
        rs_m = torch.empty((n_m,), dtype=torch.float32, device=dev)
        if n_m:
            ops.ln_fwd(hm1, None, self.mlm_ln.g, self.mlm_ln.b, hl, xh_m, rs_m)
        E = fp.p["embeddings.word_embeddings.weight"] if self.dtype != "bf16" else fp.p16(
            "embeddings.word_embeddings.weight")
        logits = ops.linear(self._lo(hl), E, fp.p["cls.predictions.bias"], out_dtype=torch.float32)
        if self.capture_logits:   # the CE kernel overwrites the logits with their gradient
            captured = {"mlm_logits": logits.clone()}
        lr_m = torch.empty((n_m,), dtype=torch.float32, device=dev)
        L.call("k3m_ce_fwd_bwd", logits.data_ptr(), V, lab_m.data_ptr(), sc_m.data_ptr(), n_m, V, lr_m.data_ptr(),
               L.stream())
        if n_m:
            L.call("k3m_loss_reduce", lr_m.data_ptr(), sc_m.data_ptr(), sl_m.data_ptr(), n_m, losses.data_ptr(),
                   L.stream())
        ctx["mlm"] = (idx_m, n_m, hm, pre_m, hl, xh_m, rs_m, logits)
        ctx["mlm_slot"] = sl_m   # 0: text row, 1: PV row (k3m_scale_rows_by_slot)

        Cv = c.v_target_size
        hv = torch.empty((n_v, Hv), dtype=torch.float32, device=dev)
        ops.gather_rows(seq_v, idx_v, n_v, hv)
        pre_v = torch.empty_like(hv)
        hv1 = self.img_t.fwd(hv, epi=L.EPI_BIAS_GELU, aux=pre_v)
        hlv = torch.empty_like(hv)
        xh_iv = torch.empty_like(hv)
        rs_iv = torch.empty((n_v,), dtype=torch.float32, device=dev)
        if n_v:
            ops.ln_fwd(hv1, None, self.img_ln.g, self.img_ln.b, hlv, xh_iv, rs_iv)
        lv = self.img_dec.fwd(hlv)
        if self.capture_logits:
            captured["img_logits"] = lv.clone()
        tgt = batch["image_target"].reshape(B * R1, Cv).contiguous()
        lr_v = torch.empty((n_v,), dtype=torch.float32, device=dev)
        L.call("k3m_kl_fwd_bwd", lv.data_ptr(), Cv, tgt.data_ptr(), Cv, src_v.data_ptr(), sc_v.data_ptr(), n_v, Cv,
               lr_v.data_ptr(), L.stream())
        if n_v:
            L.call("k3m_loss_reduce", lr_v.data_ptr(), sc_v.data_ptr(), sl_v.data_ptr(), n_v, losses.data_ptr(),
                   L.stream())
        else:
            losses[2] = float("nan")   # 0/0 as in the reference (:2758-2760)
        ctx["img"] = (idx_v, n_v, hv, pre_v, hlv, xh_iv, rs_iv, lv)

        nsp = torch.empty((1,), dtype=torch.float32, device=dev)
        L.call("k3m_nsp_loss", pooled_t.data_ptr(), pooled_pv.data_ptr(), pooled_v.data_ptr(),
               fp.p["cls.seq_relationship.weight"].data_ptr(), fp.p["cls.seq_relationship.bias"].data_ptr(),
               batch["is_next"].contiguous().data_ptr(), batch["is_next_pv_v"].contiguous().data_ptr(),
               batch["is_next_pv_t"].contiguous().data_ptr(), B, H, nsp.data_ptr(), L.stream())
        out = {
            "masked_lm_loss": losses[0:1], "masked_lm_loss_pv": losses[1:2], "masked_img_loss": losses[2:3],
            "loss_lpm": lpm, "next_sentence_loss": nsp, "c_initial": c_init, "c_final": c_final,
            "pooled_t": pooled_t, "pooled_pv": pooled_pv, "pooled_v": pooled_v,
        }
        out["loss"] = losses[0:1] + losses[1:2] + losses[2:3] + lpm
        if self.capture_logits:
            out.update(captured)
        ctx["batch"] = batch
        return out, ctx

    # ------------------------------------------------------------ backward
    def backward(self, ctx, w_mlm=1.0, w_img=1.0, w_lpm=1.0, grad_ready=None, w_mlm_pv=None):
        """Backward of  w_mlm*(mlm_t + mlm_pv) + w_img*img + w_lpm*lpm  (train_concap_struc.py:533); with
        w_mlm_pv given, of  w_mlm*mlm_t + w_mlm_pv*mlm_pv + ...  (a caller weighting the two MLM losses apart).
        Parameter gradients are ACCUMULATED into self.fp.grad.  grad_ready(kind, index) is called as
        soon as the gradients of an encoder block are final (DDP bucket hook).

        The LayerNorm / bias-gradient slab reductions are batched (ops.deferred_reductions): flushed
        right before each grad_ready hand-off (so the all-reduce sees final gradients) and at the end."""
        with ops.deferred_reductions() as dr:
            # flushed at every block boundary, with or without DDP: the slab workspaces of one block are
            # all that is alive at a time, and they are read back soon after they were written
            def hook(kind, index):
                dr.flush()
                if grad_ready is not None:
                    grad_ready(kind, index)
            self._backward(ctx, w_mlm, w_img, w_lpm, hook, w_mlm_pv)

    def _backward(self, ctx, w_mlm=1.0, w_img=1.0, w_lpm=1.0, grad_ready=None, w_mlm_pv=None):
        c = self.cfg
        fp = self.fp
        dev = self.device
        H, Hv = self.H, self.Hv
        B, T, P, R = ctx["B"], ctx["T"], ctx["P"], ctx["R"]
        BT, BP, BR = B * T, B * P, B * R
        batch = ctx["batch"]
        seq_tp, seq_v = ctx["seq_tp"], ctx["seq_v"]
        dseq_tp = torch.zeros_like(seq_tp)
        dseq_v = torch.zeros_like(seq_v)

        # ---- MLM head (dlogits already in place from the forward CE kernel)
        idx_m, n_m, hm, pre_m, hl, xh_m, rs_m, dlog = ctx["mlm"] if "mlm" in ctx else (None, 0) + (None,) * 6
        if n_m and w_mlm_pv is not None and w_mlm_pv != w_mlm:
            # text and PV rows of the shared decoder carry different upstream weights: fold them into the rows
            L.call("k3m_scale_rows_by_slot", dlog.data_ptr(), dlog.shape[1], ctx["mlm_slot"].data_ptr(), n_m,
                   dlog.shape[1], w_mlm, w_mlm_pv, L.stream())
            w_mlm = 1.0
        if n_m:
            bf = self.dtype == "bf16"
            E = fp.p16("embeddings.word_embeddings.weight") if bf else fp.p["embeddings.word_embeddings.weight"]
            gE = fp.g["embeddings.word_embeddings.weight"]
            dlo = self._lo(dlog)
            dhl = ops.linear_dgrad(dlo, E, dx=torch.empty(hl.shape, dtype=torch.float32, device=dev), alpha=w_mlm)
            ops.linear_wgrad(dlo, self._lo(hl), gE, None, alpha=w_mlm)
            ops.colsum(dlog, fp.g["cls.predictions.bias"], accumulate=True, alpha=w_mlm)
            dh1 = torch.empty_like(hl)
            ops.ln_bwd(dhl, xh_m, rs_m, self.mlm_ln.g, dh1, dh1, self.mlm_ln.gg, self.mlm_ln.gb)
            du = torch.empty_like(hl)
            ops.dgelu(dh1, pre_m, du)
            self.mlm_t.wgrad(du, hm)
            dhm = self.mlm_t.dgrad(du)
            ops.scatter_add_rows(dhm, idx_m, n_m, dseq_tp)
        idx_v, n_v, hv, pre_v, hlv, xh_iv, rs_iv, dlv = ctx["img"] if "img" in ctx else (None, 0) + (None,) * 6
        if n_v:
            dhlv = self.img_dec.dgrad(dlv, alpha=w_img)
            self.img_dec.wgrad(dlv, hlv, alpha=w_img)
            dh1v = torch.empty_like(hlv)
            ops.ln_bwd(dhlv, xh_iv, rs_iv, self.img_ln.g, dh1v, dh1v, self.img_ln.gg, self.img_ln.gb)
            duv = torch.empty_like(hlv)
            ops.dgelu(dh1v, pre_v, duv)
            self.img_t.wgrad(duv, hv)
            dhv = self.img_t.dgrad(duv)
            ops.scatter_add_rows(dhv, idx_v, n_v, dseq_v)

        # ---- structure aggregator + LPM
        (X, nvalid, src, Tm, att, agg, c_init, c_final, ent_neg, val_neg, lws, index_p, index_v, NPV,
         margin) = ctx["struct"]
        dcf = torch.zeros_like(c_final)
        dX = torch.zeros_like(X)
        det = ops.DETERMINISTIC   # fixed-order forms of the three kernels below (no float atomics)
        if lws is not None:
            if det:
                L.call("k3m_lpm_bwd_det", c_final.data_ptr(), X.data_ptr(), nvalid.data_ptr(), L.ptr(ent_neg),
                       L.ptr(val_neg), B, NPV, H, ent_neg.shape[2], val_neg.shape[2], lws.data_ptr(), dcf.data_ptr(),
                       dX.data_ptr(), L.stream())
            else:
                L.call("k3m_lpm_bwd", c_final.data_ptr(), X.data_ptr(), nvalid.data_ptr(), L.ptr(ent_neg),
                       L.ptr(val_neg), B, NPV, H, ent_neg.shape[2], val_neg.shape[2], margin, lws.data_ptr(),
                       dcf.data_ptr(), dX.data_ptr(), L.stream())
            if w_lpm != 1.0:
                ops.add_(dcf, dcf.clone(), w_lpm - 1.0)
                ops.add_(dX, dX.clone(), w_lpm - 1.0)
        if "d_c_final" in ctx:
            ops.add_(dcf, ctx["d_c_final"].contiguous())
        dagg = self.sw3.dgrad(dcf)
        self.sw3.wgrad(dcf, agg)
        dci = dcf.clone()                                   # c_final = c_init + ...
        if "d_c_initial" in ctx:
            ops.add_(dci, ctx["d_c_initial"].contiguous())
        dT = torch.zeros_like(Tm)
        groups = ctx.get("groups", 1)
        Bg = B // groups
        sa_ws = torch.empty((Bg * (H + 1),), dtype=torch.float32, device=dev) if det else None
        for gi in range(groups):
            r0 = gi * Bg
            if det:
                L.call("k3m_sa_attn_bwd_det", dagg[r0:].data_ptr(), Tm[r0 * NPV:].data_ptr(), att[r0:].data_ptr(),
                       nvalid[r0:].data_ptr(), src[r0:].data_ptr(), fp.p["struc_w2.weight"].data_ptr(),
                       dT[r0 * NPV:].data_ptr(), fp.g["struc_w2.weight"].data_ptr(), fp.g["struc_w2.bias"].data_ptr(),
                       dci[r0:].data_ptr(), sa_ws.data_ptr(), Bg, NPV, H, L.stream())
            else:
                L.call("k3m_sa_attn_bwd", dagg[r0:].data_ptr(), Tm[r0 * NPV:].data_ptr(), att[r0:].data_ptr(),
                       nvalid[r0:].data_ptr(), src[r0:].data_ptr(), fp.p["struc_w2.weight"].data_ptr(),
                       dT[r0 * NPV:].data_ptr(), fp.g["struc_w2.weight"].data_ptr(), fp.g["struc_w2.bias"].data_ptr(),
                       dci[r0:].data_ptr(), Bg, NPV, H, L.stream())
        self.sw1.wgrad(dT, X)
        self.sw1.dgrad(dT, dx=dX, beta=1.0)
        L.call("k3m_sa_gather_bwd_det" if det else "k3m_sa_gather_bwd", dX.data_ptr(), index_p.data_ptr(),
               index_v.data_ptr(), nvalid.data_ptr(), dseq_tp[BT:].data_ptr(), dci.data_ptr(), B, P, NPV, H, L.F32,
               L.stream())

        # ---- pooled outputs
        (mean_v,) = ctx["pool"]
        dpv = torch.empty((B, H), dtype=torch.float32, device=dev)
        dpt = torch.empty_like(dpv)
        dppv = torch.empty_like(dpv)
        L.call("k3m_mean3_bwd", dci.data_ptr(), dpv.data_ptr(), dpt.data_ptr(), dppv.data_ptr(), dci.numel(), 0, L.F32,
               L.stream())
        dmean_v = self.map_b2i.dgrad(dpv)
        self.map_b2i.wgrad(dpv, mean_v)
        L.call("k3m_seq_mean_bwd", dmean_v.data_ptr(), B, R, 1, Hv, 1.0, dseq_v.data_ptr(), L.F32, L.stream())
        L.call("k3m_seq_mean_bwd", dpt.data_ptr(), B, T, 1, H, 1.0, dseq_tp.data_ptr(), L.F32, L.stream())
        L.call("k3m_seq_mean_bwd", dppv.data_ptr(), B, P, 1, H, 1.0, dseq_tp[BT:].data_ptr(), L.F32, L.stream())

        # ---- fusion
        fus, streams, mode = ctx["fus"]
        XT, XV = ctx["XT"], ctx["XV"]
        dXT = torch.empty_like(XT)
        dXV = torch.empty_like(XV)
        d_ind = {}
        dslices = {
            "v": (dXV[0:BR], dXV[BR:], dseq_v),
            "t": (dXT[0:BT], dXT[BT:2 * BT], dseq_tp[0:BT]),
            "pv": (dXT[2 * BT:2 * BT + BP], dXT[2 * BT + BP:], dseq_tp[BT:]),
        }
        gb = {}
        if mode == 1:   # gate backward: elementwise part, then the three modalities' GEMMs grouped
            for m in ("v", "t", "pv"):
                rows, D = streams[m][0].shape[0], streams[m][4]
                cc, a, ys, idx = fus[m]
                dc = torch.empty_like(cc)
                dpre = torch.empty_like(cc)
                L.call("k3m_gate_bwd", dslices[m][2].data_ptr(), a.data_ptr(), cc.data_ptr(), ys.data_ptr(),
                       idx.data_ptr(), dc.data_ptr(), dpre.data_ptr(), rows, D, L.F32, L.stream())
                ops.colsum(dpre, self.gate[m].gb, accumulate=True)
                gb[m] = (dc, dpre, self._lo(dpre), self._lo(cc))
            with (ops.grouped() if GROUP_GATE else contextlib.nullcontext()):
                for m in ("v", "t", "pv"):
                    dc, dpre, dlo, clo = gb[m]
                    self.gate[m].dgrad(dlo, dx=dc, beta=1.0)
                    self.gate[m].wgrad(dlo, clo, bias_done=True)
        for m in ("v", "t", "pv"):
            x0 = streams[m][0]
            D = streams[m][4]
            rows = x0.shape[0]
            d1, d2, dout = dslices[m]
            d0 = torch.empty_like(x0)
            if mode == 1:
                cc = fus[m][0]
                dc = gb[m][0]
                L.call("k3m_relu_split3_bwd", dc.data_ptr(), cc.data_ptr(), d0.data_ptr(), d1.data_ptr(), d2.data_ptr(),
                       rows, D, 0, L.F32, L.stream())
            else:
                L.call("k3m_mean3_bwd", dout.data_ptr(), d0.data_ptr(), d1.data_ptr(), d2.data_ptr(), dout.numel(), 0,
                       L.F32, L.stream())
            d_ind[m] = d0

        # ---- encoder (reverse lock-step)
        if self.enc_dtype != torch.float32:
            dXT = ops.convert(dXT, torch.empty(dXT.shape, dtype=self.enc_dtype, device=dev))
            dXV = ops.convert(dXV, torch.empty(dXV.shape, dtype=self.enc_dtype, device=dev))
        renc = list(reversed(ctx["enc"]))
        ei = 0
        while ei < len(renc):
            kind, i, sv = renc[ei]
            nxt = renc[ei + 1] if ei + 1 < len(renc) else None
            if GROUP_TV and nxt is not None and {kind, nxt[0]} == {"t", "v"}:
                gens, outs = [], []
                for k_, j_, sv_ in (renc[ei], nxt):
                    op = self.text[j_] if k_ == "t" else self.image[j_]
                    if not ctx["train"]:
                        op = _eval_view(op)
                    r = []
                    outs.append(r)
                    gens.append(op.bwd_steps(dXT if k_ == "t" else dXV, sv_, r))
                _lockstep(gens)
                for (k_, j_, _), r in zip((renc[ei], nxt), outs):
                    if k_ == "t":
                        dXT = r[0]
                    else:
                        dXV = r[0]
                    if grad_ready is not None:
                        grad_ready(k_, j_)
                ei += 2
                continue
            ei += 1
            if kind == "t":
                op = self.text[i] if ctx["train"] else _eval_view(self.text[i])
                dXT = op.bwd(dXT, sv)
            elif kind == "v":
                op = self.image[i] if ctx["train"] else _eval_view(self.image[i])
                dXV = op.bwd(dXV, sv)
            else:
                s_tv, s_pv, s_tt, ops_ = sv
                dXT2 = torch.empty_like(dXT)
                dXV2 = torch.empty_like(dXV)
                bargs = [(dXV[0:BR], dXT[0:BT], s_tv, dXV2[0:BR], dXT2[0:BT]),
                         (dXV[BR:], dXT[2 * BT:2 * BT + BP], s_pv, dXV2[BR:], dXT2[2 * BT:2 * BT + BP]),
                         (dXT[2 * BT + BP:], dXT[BT:2 * BT], s_tt, dXT2[2 * BT + BP:], dXT2[BT:2 * BT])]
                if GROUPED:
                    _lockstep([o.bwd_steps(*a) for o, a in zip(ops_, bargs)])
                else:
                    for o, a in zip(ops_, bargs):
                        o.bwd(*a)
                dXT, dXV = dXT2, dXV2
            if grad_ready is not None:
                grad_ready(kind, i)

        # ---- embeddings
        ph = self.p_h if ctx["train"] else 0.0
        dt_ = d_ind["t"]
        ops.convert(dXT[0:BT], dt_, accumulate=True)
        ops.convert(dXT[BT:2 * BT], dt_, accumulate=True)
        dp_ = d_ind["pv"]
        ops.convert(dXT[2 * BT:2 * BT + BP], dp_, accumulate=True)
        ops.convert(dXT[2 * BT + BP:], dp_, accumulate=True)
        dv_ = d_ind["v"]
        ops.convert(dXV[0:BR], dv_, accumulate=True)
        ops.convert(dXV[BR:], dv_, accumulate=True)
        xh_t, rs_t, off_t, xh_p, rs_p, off_p = ctx["emb"]
        gword = fp.g["embeddings.word_embeddings.weight"]
        gpos = fp.g["embeddings.position_embeddings.weight"]
        gtyp = fp.g["embeddings.token_type_embeddings.weight"]
        for dy, xh, rs, off, ids, tt in ((dt_, xh_t, rs_t, off_t, batch["input_ids"], batch["segment_ids"]),
                                         (dp_, xh_p, rs_p, off_p, batch["input_ids_pv"], batch["segment_ids_pv"])):
            ds = torch.empty_like(dy)
            ops.ln_bwd(dy, xh, rs, self.emb_ln.g, ds, ds, self.emb_ln.gg, self.emb_ln.gb, p_out=ph,
                       seed=ctx["seed"], off_out=off)
            ops.embed_bwd(ids.contiguous(), tt.contiguous(), ds, gword, gpos, gtyp)
        feat2, loc2, xh_v, rs_v, off_v = ctx["vemb"]
        dsv = torch.empty_like(dv_)
        ops.ln_bwd(dv_, xh_v, rs_v, self.vemb_ln.g, dsv, dsv, self.vemb_ln.gg, self.vemb_ln.gb, p_out=ph,
                   seed=ctx["seed"], off_out=off_v)
        self.vemb_img.wgrad(dsv, feat2)
        self.vemb_loc.wgrad(dsv, loc2)
        if grad_ready is not None:
            grad_ready("emb", 0)


def _eval_view(op):
    """Same op with every dropout probability set to zero (model.eval())."""
    import copy
    o = copy.copy(op)
    for k, v in list(vars(o).items()):
        if isinstance(v, AddLN):
            setattr(o, k, AddLN(v.ln, 0.0))
        elif isinstance(v, FFN):
            f = copy.copy(v)
            f.tail = AddLN(v.tail.ln, 0.0)
            setattr(o, k, f)
        elif k in ("p_attn", "pa1", "pa2"):
            setattr(o, k, 0.0)
    return o
