"""Helpers to load the committed golden fixtures (tests/golden/golden_*.npz)."""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CASES = ["bs2_hard", "bs3_zero_triple", "bs2_mean", "cfg4_bs2", "cfg5_bs2"]
CFG_PATH = os.path.join(REPO, "configs", "bert_base_6layer_6conect.json")


def load_case(name):
    d = np.load(os.path.join(HERE, "golden", "golden_%s.npz" % name), allow_pickle=False)
    return {k: d[k] for k in d.files}


def case_config(g):
    from k3m_amd.config import pretrain_config
    return pretrain_config(CFG_PATH, if_pre_sampling=int(g["mode"]))


def case_batch(g):
    return {k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("in/")}


def case_noise(g):
    """Regenerate the gumbel noise the fixture generator fed to F.gumbel_softmax."""
    b = case_batch(g)
    B, T = b["input_ids"].shape
    P = b["input_ids_pv"].shape[1]
    R = b["image_feat"].shape[1]
    rng = np.random.default_rng(int(g["noise_seed"]))
    shapes = [("v", (B, R, 3, 1024)), ("t", (B, T, 3, 768)), ("pv", (B, P, 3, 768))]
    return {k: torch.from_numpy((-np.log(rng.standard_exponential(s))).astype(np.float32)) for k, s in shapes}


# ---------------------------------------------------------------- item alignment (fine-tuning)
FT_CASES = ["ce", "cosine"]


def load_ft_case(name):
    d = np.load(os.path.join(HERE, "golden", "golden_ft_%s.npz" % name), allow_pickle=False)
    return {k: d[k] for k in d.files}


def ft_config(g):
    from k3m_amd.config import finetune_config
    return finetune_config(CFG_PATH, loss_type=str(g["loss_type"]), if_pre_sampling=int(g["mode"]))


def ft_pair(g):
    """Pair batch named as K3MForItemAlignment.forward's arguments (vilbert_k3m.py:3379-3403)."""
    t = lambda k: torch.from_numpy(np.ascontiguousarray(g["out/" + k]))  # noqa: E731
    pair = {"labels": t("labels")}
    for k in (1, 2):
        pair.update({"input_ids_%d" % k: t("input_ids_%d" % k), "token_type_ids_%d" % k: t("segment_ids_%d" % k),
                     "attention_mask_%d" % k: t("input_mask_%d" % k), "input_ids_pv_%d" % k: t("input_ids_pv_%d" % k),
                     "token_type_ids_pv_%d" % k: t("segment_ids_pv_%d" % k),
                     "attention_mask_pv_%d" % k: t("input_mask_pv_%d" % k), "index_p_%d" % k: t("index_p_%d" % k),
                     "index_v_%d" % k: t("index_v_%d" % k), "image_feat_%d" % k: t("coll_image_feat_%d" % k),
                     "image_loc_%d" % k: t("coll_image_loc_%d" % k),
                     "image_attention_mask_%d" % k: t("coll_image_mask_%d" % k)})
    return pair


def ft_noise(g):
    """Gumbel noise per item (make_finetune_golden.py: noise_seed for item 1, noise_seed + 1 for item 2)."""
    pair = ft_pair(g)
    B, T = pair["input_ids_1"].shape
    P = pair["input_ids_pv_1"].shape[1]
    R = pair["image_feat_1"].shape[1]
    out = []
    for s in (int(g["noise_seed"]), int(g["noise_seed"]) + 1):
        rng = np.random.default_rng(s)
        shapes = [("v", (B, R, 3, 1024)), ("t", (B, T, 3, 768)), ("pv", (B, P, 3, 768))]
        out.append({k: torch.from_numpy((-np.log(rng.standard_exponential(sh))).astype(np.float32)) for k, sh in shapes})
    return out


# ---------------------------------------------------------------- logits (north_star "logits")
def check_logits(g, mlm_rows, img_rows, rtol, what="", mean_rtol=None, p99=None, col_mean=None, lse_atol=None):
    """Compare labelled-row MLM logits (text rows then PV rows, row-major; [n, V]) and masked-region logits
    ([n_v, Cv]) with the fixture's logit record (make_golden.py): the 256 recorded vocabulary columns,
    each row's label logit and logsumexp, and every region class.  Tolerance: rtol of each row's
    max |logit| (absolute per row)."""
    mlm_rows = np.asarray(mlm_rows, np.float64)
    img_rows = np.asarray(img_rows, np.float64)
    assert mlm_rows.shape[0] == g["logit/mlm_rows"].shape[0], (what, mlm_rows.shape, g["logit/mlm_rows"].shape)
    assert img_rows.shape == g["logit/img_rows"].shape, (what, img_rows.shape, g["logit/img_rows"].shape)
    cols = g["logit/mlm_cols"]
    scale = np.abs(g["logit/mlm_rows"]).max(1, keepdims=True) + 1e-6
    d = np.abs(mlm_rows[:, cols] - g["logit/mlm_rows"]) / scale
    np.testing.assert_array_less(d, rtol, err_msg=what + " mlm")
    _dist_bars(d, what + " mlm", mean_rtol, p99, col_mean)
    m = mlm_rows.max(1)
    lse = m + np.log(np.exp(mlm_rows - m[:, None]).sum(1))
    if lse_atol is not None:
        np.testing.assert_allclose(lse, g["logit/mlm_lse"], rtol=0, atol=lse_atol, err_msg=what + " lse")
    else:
        np.testing.assert_allclose(lse, g["logit/mlm_lse"], rtol=rtol, atol=rtol, err_msg=what + " lse")
    return img_rows, scale


def _dist_bars(d, what, mean_rtol, p99, col_mean):
    """Distribution bars on the per-element errors d [rows, cols]: the mean, the 99th percentile and the
    per-COLUMN mean over the rows (a systematic error confined to a few columns passes the global bars but
    not this one)."""
    if mean_rtol is not None:
        assert d.mean() < mean_rtol, (what, float(d.mean()))
    if p99 is not None:
        assert np.quantile(d, 0.99) < p99, (what, float(np.quantile(d, 0.99)))
    if col_mean is not None:
        assert d.mean(0).max() < col_mean, (what, float(d.mean(0).max()), int(d.mean(0).argmax()))


def check_img_logits(g, img_rows, rtol, what="", mean_rtol=None, p99=None, col_mean=None):
    sc = np.abs(g["logit/img_rows"]).max(1, keepdims=True) + 1e-6
    d = np.abs(np.asarray(img_rows, np.float64) - g["logit/img_rows"]) / sc
    np.testing.assert_array_less(d, rtol, err_msg=what + " img")
    _dist_bars(d, what + " img", mean_rtol, p99, col_mean)
