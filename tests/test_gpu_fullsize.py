"""Size-independent properties of the step at BASELINE.json's full size (config 2: bs=64, T=36,
P=128, R=37, 10 triples), where the CPU oracle is too slow to compare against directly.

* the default fp32 path (bf16x6 GEMMs) and the exact-f32 MFMA path compute the same step: every
  loss within 1e-4 relative, c_final within 1e-3 (but for rare near-tie flips of the hard gumbel
  gate), total gradient norm within 1e-4 and every parameter's gradient norm within 1e-3 relative
  (+ a floor for ~0 gradients);
* the step is reproducible: two eval-mode steps on the same inputs give bitwise-identical losses and
  forward outputs, and gradients equal to fp32 rounding (float atomics in two backward kernels);
* a train-mode full-size step (dropout, device gumbel noise and negatives, AdamW) is finite.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B = 64


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd.config import pretrain_config
    from k3m_amd.engine import K3MEngine
    from k3m_amd.weights import param_values
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    from golden_util import CFG_PATH
    dev = torch.device("cuda")
    cfg = pretrain_config(CFG_PATH)
    eng = K3MEngine(cfg, dev)
    eng.fp.load(param_values(cfg, 11))
    batch = {k: v.to(dev) for k, v in synthetic_batch(cfg, B, "cpu", seed=21).items()}
    noise = {k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=22).items()}
    NPV = batch["index_p"].shape[1]
    ent = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    for i in range(B):
        for j in range(10):
            ent[i, j, 0] = (i + 1) % B
            ent[i, j, 1] = (i + 7) % B
            val[i, j, 0] = (j + 1) % 10
            val[i, j, 1] = (j + 3) % 10
    return cfg, eng, batch, noise, ent, val


LOSSES = ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm", "next_sentence_loss", "loss")


def _run(setup, algo):
    from k3m_amd import ops
    cfg, eng, batch, noise, ent, val = setup
    old = ops.F32_ALGO
    ops.F32_ALGO = algo
    try:
        eng.fp.grad.zero_()
        out, ctx = eng.forward(batch, train=False, noise=noise, ent_neg=ent, val_neg=val)
        eng.backward(ctx)
        torch.cuda.synchronize()
    finally:
        ops.F32_ALGO = old
    losses = np.array([float(out[k]) for k in LOSSES])
    _run.gates = gate_choices(ctx)
    return losses, out["c_final"].detach().clone(), eng.fp.grad.detach().clone()


def gate_choices(ctx):
    """The hard gumbel gate's choice per (row, channel) of each modality (k3m_gate_fwd's idx: 0 self, 1 cross1,
    2 cross2; the argmax of vilbert_k3m.py:2363-2372)."""
    fus = ctx["fus"][0]
    return {m: fus[m][3].detach().clone() for m in ("v", "t", "pv") if fus.get(m) is not None}


def flip_rate(ga, gb):
    """Fraction of gate choices that differ between two runs, per modality and overall."""
    out, nd, nt = {}, 0, 0
    for m in ga:
        d = int((ga[m] != gb[m]).sum())
        out[m] = d / ga[m].numel()
        nd, nt = nd + d, nt + ga[m].numel()
    out["all"] = nd / max(nt, 1)
    out["flips"], out["choices"] = nd, nt
    return out


def test_fullsize_x6_matches_exact_f32(setup):
    from k3m_amd import _lib as L
    l6, c6, g6 = _run(setup, L.F32_SPLIT_BF16X6)
    q6 = _run.gates
    lf, cf, gf = _run(setup, L.F32_MFMA_F32)
    fr = flip_rate(q6, _run.gates)
    # the hard gate's flip rate between the two fp32 GEMM algorithms at full size (a flip needs
    # two gate logits within the GEMMs' rounding difference of a tie)
    print("full-size hard-gate flips x6 vs exact f32: %s" % fr)
    assert fr["all"] <= 1.0 / 2000, fr
    assert np.all(np.isfinite(l6)), l6
    np.testing.assert_allclose(l6, lf, rtol=1e-4, atol=1e-6)
    # c_final comes out of the hard (argmax) gumbel gate: where two gate logits are within the
    # GEMMs' rounding difference of a tie, the two algorithms may pick different sources for that
    # channel.  Such flips must stay rare; every other element agrees to 1e-3.
    bad = ~torch.isclose(c6, cf, rtol=1e-3, atol=1e-4)
    assert int(bad.sum()) <= max(8, c6.numel() // 2000), (int(bad.sum()), c6.numel())
    n6, nf = float(g6.double().norm()), float(gf.double().norm())
    assert abs(n6 - nf) <= 1e-4 * nf, (n6, nf)
    eng = setup[1]
    worst = 0.0
    for name, _ in eng.fp.spec:
        o, n = eng.fp.offsets[name], eng.fp.g[name].numel()
        a, b = float(g6[o:o + n].double().norm()), float(gf[o:o + n].double().norm())
        rel = abs(a - b) / max(b, 1e-30)
        if b > 1e-6:
            worst = max(worst, rel)
            assert rel <= 1e-3 or abs(a - b) <= 1e-6 * nf, (name, a, b)
    print("full-size x6 vs f32: losses", l6, lf, "worst per-tensor grad-norm rel %.2e" % worst)


def test_fullsize_losses_match_cpu_oracle(setup):
    """VERDICT r5 item 3 / north_star "loss parity <= 1e-3 vs CPU reference" at the metric's config (bs=64, T=36,
    P=128, R=37, 10 triples), not only on the bs <= 3 goldens: the default fp32 engine (bf16x6 GEMMs) against the
    CPU oracle (oracle/k3m_oracle.py, pinned to the reference goldens by test_oracle_golden.py) on the same weights,
    batch, gumbel noise and LPM negatives, eval mode.  Every loss within 1e-3 relative; c_initial within 1e-3."""
    import os
    from k3m_amd import _lib as L
    from k3m_amd.weights import param_values
    from oracle import k3m_oracle as O
    cfg, eng, batch, noise, ent, val = setup
    l6, _, _ = _run(setup, L.F32_SPLIT_BF16X6)
    out_gpu, _ = eng.forward(batch, train=False, noise=noise, ent_neg=ent, val_neg=val)
    ci_gpu = out_gpu["c_initial"].detach().cpu().numpy()
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    P = {k: torch.from_numpy(v) for k, v in param_values(cfg, 11).items()}
    with torch.no_grad():
        ref = O.forward(P, cfg, {k: v.cpu() for k, v in batch.items()}, {k: v.cpu() for k, v in noise.items()}, ent,
                        val)
    lo = np.array([float(ref[k]) for k in LOSSES])
    rel = np.abs(l6 - lo) / np.maximum(np.abs(lo), 1e-3)
    print("full-size HIP vs CPU oracle: losses", l6, lo, "rel", rel)
    assert (rel <= 1e-3).all(), (l6, lo, rel)
    np.testing.assert_allclose(ci_gpu, ref["c_initial"].numpy(), rtol=1e-3, atol=1e-4)


def test_fullsize_step_is_deterministic(setup):
    """Forward outputs are bitwise reproducible.  Gradients are reproducible to fp32 rounding: the
    embedding scatter-add and the structure-aggregator backward accumulate with float atomics (as the
    reference's CUDA index_add / autograd do), so their summation order — and everything upstream of
    them in the backward — may differ in the last bits between runs."""
    from k3m_amd import _lib as L
    l1, c1, g1 = _run(setup, L.F32_SPLIT_BF16X6)
    l2, c2, g2 = _run(setup, L.F32_SPLIT_BF16X6)
    assert np.array_equal(l1, l2), (l1, l2)
    assert torch.equal(c1, c2)
    eng = setup[1]
    tot = float(g1.double().norm())
    worst = 0.0
    for name, _ in eng.fp.spec:
        o, n = eng.fp.offsets[name], eng.fp.g[name].numel()
        d = float((g1[o:o + n].double() - g2[o:o + n].double()).norm())
        ref = float(g1[o:o + n].double().norm())
        worst = max(worst, d / max(ref, 1e-30) if ref > 1e-6 else 0.0)
        assert d <= 1e-5 * ref + 1e-7 * tot, (name, d, ref)
    print("run-to-run gradient difference: worst per-tensor relative %.2e" % worst)


def test_fullsize_train_step_finite():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from golden_util import CFG_PATH
    dev = torch.device("cuda")
    cfg = pretrain_config(CFG_PATH)
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=1, total_steps=10, seed=4)
    batch = synthetic_batch(cfg, B, dev, seed=6)
    for _ in range(3):
        out = tr.step(batch)
        assert np.isfinite(float(out["loss"]))
    assert torch.isfinite(tr.engine.fp.data).all()
