"""Helpers to load the committed golden fixtures (tests/golden/golden_*.npz)."""
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CASES = ["bs2_hard", "bs3_zero_triple", "bs2_mean"]
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
