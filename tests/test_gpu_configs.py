"""BASELINE.json configs[2..4] at full size (the reference cannot run these shapes on CPU in any
reasonable time; bs=2 slices of configs[3]/[4] are pinned against reference goldens in
test_gpu_parity.py: cfg4_bs2, cfg5_bs2).  Size-independent properties:

* configs[2] (bf16, bs=64): the bf16 step computes the same step as the fp32 step on the same
  inputs and weights: losses within 2e-3, total gradient cosine >= 0.995 and norm within 1e-2
  (bars about 10x / 2x / 4x above the measured values; test_bf16_matches_fp32_step, also for configs 4 and 5);
* configs[3] (12/6/6 layers, seq_len 128, 100 boxes, bf16, bs=256) and configs[4] (50 PV triples in
  a 320-token PV sequence, bf16, bs=128): two train-mode Trainer steps (dropout, device gumbel noise
  and LPM negatives, AdamW) are finite and the peak device memory of the step is reported and fits
  the 288 GB HBM of one MI355X with room for the 7 other data-parallel ranks' buffers being absent
  (each rank owns its GPU).
"""
import numpy as np
import pytest
import torch

from test_gpu_fullsize import gate_choices, flip_rate

pytestmark = pytest.mark.gpu

LOSSES = ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm", "next_sentence_loss", "loss")
HBM_BYTES = 288e9


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


def _tables(B, NPV, n):
    ent = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    for i in range(B):
        for j in range(n):
            ent[i, j, 0], ent[i, j, 1] = (i + 1) % B, (i + 5) % B
            val[i, j, 0], val[i, j, 1] = (j + 1) % n, (j + 2) % n
    return ent, val


# full-size shapes of BASELINE.json configs[2..4]: bs, T, P, boxes, triples, NPV
CMP = {
    "config3_bs64": dict(B=64, T=36, P=128, nbox=36, n_triples=10, npv=20),
    "config4_seq128_100boxes_bs256": dict(B=256, T=128, P=128, nbox=100, n_triples=10, npv=20),
    "config5_50triples_bs128": dict(B=128, T=36, P=320, nbox=36, n_triples=50, npv=50),
}


@pytest.mark.parametrize("name", sorted(CMP))
def test_bf16_matches_fp32_step(dev, name):
    """The bf16 step against the fp32 step on the same inputs and weights at each bf16 config's full size (VERDICT r4
    item 5b: configs 4 and 5 were only checked for finiteness): losses within 2e-3 relative, total gradient cosine
    >= 0.995, norm within 1e-2.  Config 5's PV attention runs attention_flash_long.hip in bf16 and the exact-fp32
    attention_long.hip in fp32.  Bars from the measured values (profiles/r5b_cfg_bf16_vs_fp32.txt: loss rel
    <= 1.6e-4, cosine >= 0.9972, norm rel <= 2.8e-3), about 10x / 2x / 4x above them (round 4's 1e-2 / 0.99 / 5e-2
    were the mixed-precision defaults)."""
    from golden_util import CFG_PATH
    from k3m_amd.config import pretrain_config
    from k3m_amd.engine import K3MEngine
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    from k3m_amd.weights import param_values
    cfg = pretrain_config(CFG_PATH)
    c = CMP[name]
    B = c["B"]
    vals = param_values(cfg, 17)
    batch = {k: v.to(dev) for k, v in synthetic_batch(cfg, B, "cpu", seed=31, T=c["T"], P=c["P"], n_boxes=c["nbox"],
                                                         n_triples=c["n_triples"], npv=c["npv"]).items()}
    noise = {k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=32, T=c["T"], P=c["P"], R=c["nbox"] + 1).items()}
    ent, val = _tables(B, batch["index_p"].shape[1], c["n_triples"] - 1)
    res = {}
    for dt in ("fp32", "bf16"):
        eng = K3MEngine(cfg, dev, dtype=dt)
        eng.fp.load(vals)
        eng.fp.grad.zero_()
        out, ctx = eng.forward(batch, train=False, noise=noise, ent_neg=ent, val_neg=val)
        eng.backward(ctx)
        torch.cuda.synchronize()
        res[dt] = (np.array([float(out[k]) for k in LOSSES]), eng.fp.grad.detach().double().clone(),
                   gate_choices(ctx))
        del eng, out, ctx
        torch.cuda.empty_cache()
    lf, gf, qf = res["fp32"]
    lb, gb, qb = res["bf16"]
    fr = flip_rate(qf, qb)
    # how often the bf16 encoder changes the hard gumbel gate's choice (vilbert_k3m.py:2363-2372)
    print("bf16 vs fp32 %s: hard-gate flips %s" % (name, fr))
    assert fr["all"] <= 2e-3, fr   # measured 4.5e-4 to 4.7e-4 (profiles/r6/gate_flip_rate.json)
    assert np.all(np.isfinite(lb)), lb
    rel = np.abs(lb - lf) / np.maximum(np.abs(lf), 1e-3)
    cos = float(gf @ gb / (gf.norm() * gb.norm()))
    nrel = abs(float(gb.norm()) - float(gf.norm())) / float(gf.norm())
    print("bf16 vs fp32 %s: loss rel" % name, rel, "grad cos %.6f norm rel %.3e" % (cos, nrel))
    assert (rel <= 2e-3).all(), (lb, lf)
    assert cos >= 0.995 and nrel <= 1e-2, (cos, nrel)


# bs, T, P, boxes, triples, NPV per BASELINE.json configs
FULL = {
    "config4_seq128_100boxes_bs256": dict(B=256, T=128, P=128, nbox=100, n_triples=10, npv=20),
    "config5_50triples_bs128": dict(B=128, T=36, P=320, nbox=36, n_triples=50, npv=50),
}


@pytest.mark.parametrize("name", sorted(FULL))
def test_fullsize_config_train_steps(dev, name):
    from golden_util import CFG_PATH
    from k3m_amd.config import pretrain_config
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.trainer import Trainer
    s = FULL[name]
    cfg = pretrain_config(CFG_PATH)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=1, total_steps=10, seed=4, dtype="bf16")
    batch = synthetic_batch(cfg, s["B"], dev, seed=6, T=s["T"], P=s["P"], n_boxes=s["nbox"],
                            n_triples=s["n_triples"], npv=s["npv"])
    assert batch["input_ids"].shape == (s["B"], s["T"]) and batch["image_feat"].shape[1] == s["nbox"] + 1
    assert batch["index_p"].shape[1] == s["npv"] and int((batch["index_p"][:, :, 0] != 0).sum(1).min()) >= s["n_triples"] - 1
    losses = []
    for _ in range(2):
        out = tr.step(batch)
        losses.append([float(out[k]) for k in LOSSES])
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated()
    print("%s: losses %s peak device memory %.1f GB" % (name, losses, peak / 1e9))
    assert np.all(np.isfinite(losses)), losses
    assert float(out["loss_lpm"]) > 0
    assert torch.isfinite(tr.engine.fp.data).all()
    assert peak < 0.9 * HBM_BYTES, peak
    del tr, batch, out
    torch.cuda.empty_cache()
