"""Long-sequence attention (attention_long.hip, L > 128: fine-tuning PV text 256, config 5 P = 320)
against a plain PyTorch fp32 reference of the same op (probabilities, context, dQ/dK/dV; 1e-5 /
1e-4 relative), and against the whole-head kernel of attention.hip at L <= 128 with dropout on (same
counters, so the two paths must agree)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _ref(q, k, v, mask, nh):
    B, Lq, D = q.shape
    Lk = k.shape[1]
    hd = D // nh
    qh = q.view(B, Lq, nh, hd).permute(0, 2, 1, 3)
    kh = k.view(B, Lk, nh, hd).permute(0, 2, 1, 3)
    vh = v.view(B, Lk, nh, hd).permute(0, 2, 1, 3)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(hd) + mask[:, None, None, :]
    p = torch.softmax(s, -1)
    return (p @ vh).permute(0, 2, 1, 3).reshape(B, Lq, D), p


def _inputs(dev, B, lq, lk, nh, hd, pad=5):
    D = nh * hd
    qkv_q = torch.randn(B * lq, 3 * D, device=dev)
    qkv_k = torch.randn(B * lk, 3 * D, device=dev)
    q, k, v = qkv_q[:, :D], qkv_k[:, D:2 * D], qkv_k[:, 2 * D:]
    m = torch.ones(B, lk, device=dev)
    m[:, lk - pad:] = 0
    return q, k, v, ((1 - m) * -10000).contiguous()


def _call(name, *a):
    from k3m_amd import _lib as L
    L.call(name, *a)


@pytest.mark.parametrize("lq,lk,nh,hd", [(256, 256, 12, 64), (320, 320, 12, 64), (50, 256, 8, 96), (256, 50, 8, 96),
                                         (256, 37, 8, 128), (130, 200, 12, 64), (36, 36, 12, 64)])
def test_long_attention_matches_torch(dev, lq, lk, nh, hd):
    from k3m_amd import _lib as L
    B = 3
    D = nh * hd
    q, k, v, mask = _inputs(dev, B, lq, lk, nh, hd)
    ctx = torch.empty(B * lq, D, device=dev)
    probs = torch.empty(B * nh * lq * lk, device=dev)
    s = 1 / math.sqrt(hd)
    _call("k3m_attn_long_fwd", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
          mask.data_ptr(), ctx.data_ptr(), D, probs.data_ptr(), B, lq, lk, nh, hd, s, 0.0, 0, 0, L.F32, L.stream())
    qr, kr, vr = [t.reshape(B, -1, D).clone().requires_grad_(True) for t in (q, k, v)]
    cr, pr = _ref(qr, kr, vr, mask, nh)
    assert _rel(ctx.view(B, lq, D), cr) < 1e-5
    assert _rel(probs.view(B, nh, lq, lk), pr) < 1e-5
    dctx = torch.randn(B * lq, D, device=dev)
    cr.backward(dctx.view(B, lq, D))
    dq = torch.empty(B * lq, D, device=dev)
    dk = torch.empty(B * lk, D, device=dev)
    dv = torch.empty(B * lk, D, device=dev)
    ws = torch.empty_like(probs)
    _call("k3m_attn_long_bwd", dctx.data_ptr(), D, ctx.data_ptr(), D, q.data_ptr(), q.stride(0), k.data_ptr(),
          k.stride(0), v.data_ptr(), v.stride(0), probs.data_ptr(), ws.data_ptr(), dq.data_ptr(), dk.data_ptr(),
          dv.data_ptr(), D, D, D, B, lq, lk, nh, hd, s, 0.0, 0, 0, L.F32, L.stream())
    assert _rel(dq.view(B, lq, D), qr.grad) < 1e-4
    assert _rel(dk.view(B, lk, D), kr.grad) < 1e-4
    assert _rel(dv.view(B, lk, D), vr.grad) < 1e-4


@pytest.mark.parametrize("lq,lk,nh,hd", [(128, 128, 12, 64), (37, 37, 8, 128), (36, 128, 8, 96)])
def test_long_matches_short_with_dropout(dev, lq, lk, nh, hd):
    """Same dropout counters: the long path reproduces the whole-head kernel, dropout included."""
    from k3m_amd import _lib as L
    B = 4
    D = nh * hd
    q, k, v, mask = _inputs(dev, B, lq, lk, nh, hd)
    s, p, seed, off = 1 / math.sqrt(hd), 0.1, 1234, 777
    outs = {}
    for name in ("short", "long"):
        ctx = torch.empty(B * lq, D, device=dev)
        probs = torch.empty(B * nh * lq * lk, device=dev)
        fwd = "k3m_attn_fwd" if name == "short" else "k3m_attn_long_fwd"
        _call(fwd, q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0), mask.data_ptr(),
              ctx.data_ptr(), D, probs.data_ptr(), B, lq, lk, nh, hd, s, p, seed, off, L.F32, L.stream())
        dctx = torch.ones(B * lq, D, device=dev) * 0.01 + torch.linspace(-1, 1, B * lq * D, device=dev).view(B * lq, D)
        dq = torch.empty(B * lq, D, device=dev)
        dk = torch.empty(B * lk, D, device=dev)
        dv = torch.empty(B * lk, D, device=dev)
        args = [dctx.data_ptr(), D, ctx.data_ptr(), D, q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0),
                v.data_ptr(), v.stride(0), probs.data_ptr()]
        if name == "long":
            args.append(torch.empty_like(probs).data_ptr())
        _call("k3m_attn_bwd" if name == "short" else "k3m_attn_long_bwd", *args, dq.data_ptr(), dk.data_ptr(),
              dv.data_ptr(), D, D, D, B, lq, lk, nh, hd, s, p, seed, off, L.F32, L.stream())
        torch.cuda.synchronize()
        outs[name] = (ctx, probs, dq, dk, dv)
    for a, b in zip(outs["long"], outs["short"]):
        assert _rel(a, b) < 1e-5
