"""Full-step parity of the HIP engine (libk3m_hip through the C ABI) against the golden vectors
recorded from the reference model (tests/golden) and against the CPU oracle.  Eval mode (no
dropout), explicit gumbel noise and LPM negatives -> deterministic comparison.
Tolerance: 1e-3 relative on every loss (BASELINE.json north_star), c_initial / c_final 1e-3."""
import numpy as np
import pytest
import torch

from golden_util import CASES, load_case, case_config, case_batch, case_noise, check_logits, check_img_logits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


_ENG = {}


def engine_for(cfg, seed, dev, dtype="fp32"):
    from k3m_amd.engine import K3MEngine
    from k3m_amd.weights import param_values
    key = (cfg.if_pre_sampling, seed, dtype)
    if key not in _ENG:
        _ENG.clear()
        e = K3MEngine(cfg, dev, dtype=dtype)
        e.fp.load(param_values(cfg, seed))
        _ENG[key] = e
    e = _ENG[key]
    e.fp.grad.zero_()
    return e


@pytest.mark.parametrize("case", CASES)
def test_engine_matches_reference_golden(dev, case):
    g = load_case(case)
    cfg = case_config(g)
    eng = engine_for(cfg, int(g["weight_seed"]), dev)
    batch = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    eng.capture_logits = True
    try:
        out, ctx = eng.forward(batch, train=False, noise=noise, ent_neg=torch.from_numpy(g["ent_neg"]),
                               val_neg=torch.from_numpy(g["val_neg"]))
    finally:
        eng.capture_logits = False
    eng.backward(ctx)
    torch.cuda.synchronize()
    got = np.array([float(out[k]) for k in ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm",
                                           "next_sentence_loss", "loss")])
    np.testing.assert_allclose(got, g["losses"], rtol=1e-3, atol=1e-4)
    # logits of the labelled MLM rows and the masked regions (north_star "logits ... within 1e-3")
    check_logits(g, out["mlm_logits"].cpu().numpy(), g["logit/img_rows"], 1e-3, case)
    check_img_logits(g, out["img_logits"].cpu().numpy(), 1e-3, case)
    np.testing.assert_allclose(out["c_initial"].cpu().numpy(), g["c_initial"], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(out["c_final"].cpu().numpy(), g["c_final"], rtol=1e-3, atol=1e-4)
    G = eng.fp.g
    for k in g:
        if k.startswith("grad_full/") or k.startswith("grad_slice/"):
            n = k.split("/", 1)[1]
            gr = G[n]
            if k.startswith("grad_slice/"):
                gr = gr[:4] if gr.dim() == 2 else gr[:256]
            ref = g[k]
            # relative to the tensor's scale; absolute floor for gradients that are analytically ~0
            # (e.g. struc_w2.bias: a softmax is shift invariant, so its true gradient is 0)
            err = np.abs(gr.cpu().numpy() - ref).max()
            assert err <= 5e-3 * np.abs(ref).max() + 1e-6, (n, err, np.abs(ref).max())
    for n, ref in zip(list(g["grad_norm_names"]), g["grad_norms"]):
        gn = float(G[n].double().norm())
        if np.isnan(ref):
            assert gn == 0.0, n
        else:
            assert abs(gn - ref) <= 5e-3 * ref + 1e-6, (n, gn, ref)


def test_train_mode_step_is_finite_and_learns(dev):
    """Dropout on, device-side gumbel noise and negatives, AdamW: losses finite and the summed
    loss goes down over a few steps on a fixed small batch."""
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from golden_util import CFG_PATH
    cfg = pretrain_config(CFG_PATH)
    tr = Trainer(cfg, dev, lr=2e-4, warmup_steps=0, total_steps=100, seed=3)
    batch = synthetic_batch(cfg, 8, dev, seed=5)
    losses = []
    for _ in range(6):
        out = tr.step(batch)
        losses.append(float(out["loss"]))
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses


# ---------------------------------------------------------------- bf16 encoder (configs[2] precision)
# The bf16 mode rounds encoder activations and weights to bf16 (8 significant bits), so it is
# compared with the reference's fp32 golden values at mixed-precision tolerances: losses within
# BF16_LOSS_RTOL; every recorded gradient tensor with cosine similarity >= BF16_GRAD_COS and norm
# within BF16_GRAD_NORM_RTOL of the fp32 reference (small bias gradients that are sums of
# cancelling terms carry the most relative bf16 noise, hence the per-tensor cosine bar), and all
# recorded gradients together with cosine >= BF16_GLOBAL_COS.
# Measured over the five goldens (round 5, profiles/r5c/bf16_golden_parity.txt): loss relative error <= 3.5e-3
# (the NSP loss of bs3_zero_triple; the others <= 2.7e-3), worst per-tensor gradient cosine 0.9961, worst norm
# relative 0.0096, global cosine >= 0.9973.  Bars about 2x above those (round 4: 1e-2 / 0.98 / 3e-2).
BF16_LOSS_RTOL = 7e-3
BF16_GRAD_COS = 0.99
BF16_GRAD_NORM_RTOL = 2e-2
BF16_GLOBAL_COS = 0.995
# bf16 logit bars, set from the measured error distribution over the five goldens
# (profiles/r4_bf16_logit_errors.json, scripts/bf16_logit_errors.py; error = |bf16 - ref| / row max |ref|):
# worst element 0.218 (cfg5), worst 99th percentile 0.063 (cfg4), worst per-column mean 0.0147 (region head,
# bs2_hard), worst mean 0.0067, worst logsumexp error 1.0e-3 absolute.  A systematic error in a few vocabulary
# or region columns shows in the per-column mean, not in the max or the global mean.
BF16_LOGIT_RTOL = 0.25
BF16_LOGIT_MEAN = 1e-2
BF16_LOGIT_P99 = 0.08
BF16_LOGIT_COLMEAN = 0.02
BF16_LSE_ATOL = 5e-3


@pytest.mark.parametrize("case", CASES)
def test_bf16_engine_close_to_reference_golden(dev, case):
    g = load_case(case)
    cfg = case_config(g)
    eng = engine_for(cfg, int(g["weight_seed"]), dev, dtype="bf16")
    batch = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    eng.capture_logits = True
    try:
        out, ctx = eng.forward(batch, train=False, noise=noise, ent_neg=torch.from_numpy(g["ent_neg"]),
                               val_neg=torch.from_numpy(g["val_neg"]))
    finally:
        eng.capture_logits = False
    eng.backward(ctx)
    torch.cuda.synchronize()
    # bf16 encoder: every logit within BF16_LOGIT_RTOL of its row's max |logit|, mean error BF16_LOGIT_MEAN
    check_logits(g, out["mlm_logits"].cpu().numpy(), g["logit/img_rows"], BF16_LOGIT_RTOL, case + " bf16",
                 mean_rtol=BF16_LOGIT_MEAN, p99=BF16_LOGIT_P99, col_mean=BF16_LOGIT_COLMEAN, lse_atol=BF16_LSE_ATOL)
    check_img_logits(g, out["img_logits"].cpu().numpy(), BF16_LOGIT_RTOL, case + " bf16", mean_rtol=BF16_LOGIT_MEAN,
                     p99=BF16_LOGIT_P99, col_mean=BF16_LOGIT_COLMEAN)
    got = np.array([float(out[k]) for k in ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm",
                                           "next_sentence_loss", "loss")])
    rel = np.abs(got - g["losses"]) / np.maximum(np.abs(g["losses"]), 1e-3)
    print("bf16 loss rel err", case, rel)
    assert (rel <= BF16_LOSS_RTOL).all(), (got, g["losses"])
    G = eng.fp.g
    worst_cos, worst_norm = 1.0, 0.0
    dot = na = nb2 = 0.0
    for k in g:
        if k.startswith("grad_full/"):
            n = k.split("/", 1)[1]
            a = G[n].double().cpu().numpy().ravel()
            b = g[k].astype(np.float64).ravel()
            nb = np.linalg.norm(b)
            if nb < 1e-6:
                continue
            cos = float(a @ b / (np.linalg.norm(a) * nb + 1e-30))
            nr = abs(np.linalg.norm(a) - nb) / nb
            dot, na, nb2 = dot + float(a @ b), na + float(a @ a), nb2 + float(b @ b)
            worst_cos, worst_norm = min(worst_cos, cos), max(worst_norm, nr)
            assert cos >= BF16_GRAD_COS and nr <= BF16_GRAD_NORM_RTOL, (n, cos, nr)
    gcos = dot / np.sqrt(na * nb2)
    print("bf16 grads: worst cos %.5f worst norm rel %.4f global cos %.6f" % (worst_cos, worst_norm, gcos))
    assert gcos >= BF16_GLOBAL_COS, gcos


def test_bf16_train_mode_learns(dev):
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from golden_util import CFG_PATH
    cfg = pretrain_config(CFG_PATH)
    tr = Trainer(cfg, dev, lr=2e-4, warmup_steps=0, total_steps=100, seed=3, dtype="bf16")
    batch = synthetic_batch(cfg, 8, dev, seed=5)
    losses = []
    for _ in range(6):
        out = tr.step(batch)
        losses.append(float(out["loss"]))
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses
