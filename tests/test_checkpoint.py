"""Checkpoint interchange with the reference driver (k3m_amd/checkpoint.py; train_concap_struc.py:259-297,
:691-705).  CPU tests: the saved state_dict has exactly the reference's 999 keys and shapes
(tests/golden/param_inventory.json, recorded from the reference model), the optimizer / scheduler
state_dicts follow the reference's AdamW grouping (:352-367) and torch layouts, and a save -> load
round trip restores parameters, moments and step bit for bit.  The GPU test resumes training from a
.tar and checks it continues like the uninterrupted run."""
import json
import os
import types

import numpy as np
import pytest
import torch

from golden_util import CFG_PATH, HERE


def _full_cfg():
    from k3m_amd.config import pretrain_config
    return pretrain_config(CFG_PATH)


def test_state_dict_keys_match_reference_inventory():
    from k3m_amd.params import param_spec
    from k3m_amd.checkpoint import DECODER_KEY, TIED_TO
    inv = json.load(open(os.path.join(HERE, "golden", "param_inventory.json")))["params"]
    spec = param_spec(_full_cfg())
    assert [(n, list(s)) for n, s in spec] == [(n, list(s)) for n, s in inv]   # names, order, shapes
    shapes = dict(spec)
    assert DECODER_KEY not in shapes and shapes[TIED_TO] == (21128, 768)


def _tiny_cfg():
    cfg = _full_cfg()
    cfg.num_hidden_layers, cfg.v_num_hidden_layers = 2, 1
    cfg.v_biattention_id, cfg.t_biattention_id = [0], [1]
    cfg.vocab_size, cfg.hidden_size, cfg.intermediate_size = 97, 64, 128
    cfg.v_hidden_size = cfg.bi_hidden_size = cfg.v_intermediate_size = 64
    cfg.v_feature_size, cfg.v_target_size, cfg.max_position_embeddings = 32, 17, 40
    return cfg


def _fake_trainer(cfg, seed, step):
    from k3m_amd.engine import FlatParams
    fp = FlatParams(cfg, torch.device("cpu"))
    g = torch.Generator().manual_seed(seed)
    fp.data.copy_(torch.randn(fp.total, generator=g))
    nopt = fp.segments["frozen"][0]
    t = types.SimpleNamespace(engine=types.SimpleNamespace(fp=fp, step_count=step), global_step=step,
                              m=torch.randn(nopt, generator=g), v=torch.rand(nopt, generator=g),
                              lr=1e-4, warmup=10, t_total=1000, beta1=0.9, beta2=0.98, eps=1e-8, wd=0.01)
    t.current_lr = lambda: t.lr * min(1.0, t.global_step / t.warmup)
    return t


def test_checkpoint_layout_and_round_trip(tmp_path):
    from k3m_amd import checkpoint as C
    from k3m_amd.params import is_frozen, is_no_decay
    cfg = _tiny_cfg()
    src = _fake_trainer(cfg, 1, step=7)
    tar, binp = str(tmp_path / "k.tar"), str(tmp_path / "k.bin")
    C.save_checkpoint(src, tar_path=tar, bin_path=binp)

    ck = torch.load(tar, map_location="cpu", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "scheduler_state_dict", "global_step"}
    names = [n for n, _ in src.engine.fp.spec]
    sd = ck["model_state_dict"]
    assert list(sd) == names + [C.DECODER_KEY]
    assert torch.equal(sd[C.DECODER_KEY], sd[C.TIED_TO])
    assert list(torch.load(binp, weights_only=True)) == list(sd)
    osd = ck["optimizer_state_dict"]
    g0, g1 = osd["param_groups"]
    assert (g0["weight_decay"], g1["weight_decay"]) == (0.01, 0.0)
    order = [n for n in names if not is_no_decay(n)] + [n for n in names if is_no_decay(n)]
    assert g0["params"] + g1["params"] == list(range(len(names)))
    assert set(osd["state"]) == {i for i, n in enumerate(order) if not is_frozen(n)}
    st = next(iter(osd["state"].values()))
    assert set(st) == {"step", "exp_avg", "exp_avg_sq"} and st["step"] == 7
    assert ck["scheduler_state_dict"]["last_epoch"] == 7 and ck["global_step"] == 7

    dst = _fake_trainer(cfg, 2, step=0)
    dst.engine.fp.grad = torch.zeros_like(dst.engine.fp.data)
    assert C.load_checkpoint(dst, tar) == 7
    fs, fd = src.engine.fp, dst.engine.fp
    for n in names:
        assert torch.equal(fs.p[n], fd.p[n]), n
        if not is_frozen(n):
            o, k = fs.offsets[n], fs.p[n].numel()
            assert torch.equal(src.m[o:o + k], dst.m[o:o + k]) and torch.equal(src.v[o:o + k], dst.v[o:o + k]), n
    assert (dst.global_step, dst.warmup, dst.t_total, dst.lr) == (7, 10, 1000, 1e-4)


def test_load_strips_module_prefix():
    from k3m_amd import checkpoint as C
    cfg = _tiny_cfg()
    a, b = _fake_trainer(cfg, 3, 0), _fake_trainer(cfg, 4, 0)
    sd = {"module." + k: v for k, v in C.model_state_dict(a.engine.fp).items()}
    C.load_model_state_dict(b.engine.fp, sd)
    for n, _ in a.engine.fp.spec:
        assert torch.equal(a.engine.fp.p[n], b.engine.fp.p[n]), n


@pytest.mark.gpu
def test_resume_from_tar_continues_training(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd import checkpoint as C
    dev = torch.device("cuda")
    cfg = _full_cfg()
    batch = synthetic_batch(cfg, 8, dev, seed=9)
    tr = Trainer(cfg, dev, lr=2e-4, warmup_steps=2, total_steps=50, seed=5)
    for _ in range(3):
        tr.step(batch)
    tar = str(tmp_path / "resume.tar")
    C.save_checkpoint(tr, tar_path=tar)
    ref = [float(tr.step(batch)["loss"]) for _ in range(2)]
    ref_p = tr.engine.fp.data.clone()
    del tr
    torch.cuda.empty_cache()
    tr2 = Trainer(cfg, dev, lr=1.0, warmup_steps=0, total_steps=1, seed=5, init=False)
    assert C.load_checkpoint(tr2, tar) == 3
    got = [float(tr2.step(batch)["loss"]) for _ in range(2)]
    np.testing.assert_allclose(got, ref, rtol=1e-5)
    d = float((tr2.engine.fp.data - ref_p).norm() / ref_p.norm())
    assert d < 1e-5, d


def test_checkpoint_per_tensor_groups_round_trip(tmp_path):
    """Pretrained-model layout (train_concap_struc.py:368-385): one group per requires_grad tensor in
    named_parameters() order, lr x multiplier, --freeze names left out; moments land on the same
    tensors after a round trip, and a two-group file is rejected instead of mis-mapped."""
    from k3m_amd import checkpoint as C
    from k3m_amd.params import is_frozen, is_no_decay
    cfg = _tiny_cfg()
    src = _fake_trainer(cfg, 5, step=3)
    names = [n for n, _ in src.engine.fp.spec]
    frozen = [names[3], names[10]]
    src.lr_mult = {names[0]: 0.1, names[7]: 0.1}
    src.frozen_names = tuple(frozen)
    tar = str(tmp_path / "pt.tar")
    C.save_checkpoint(src, tar_path=tar)
    ck = torch.load(tar, map_location="cpu", weights_only=True)
    pg = ck["optimizer_state_dict"]["param_groups"]
    kept = [n for n in names if n not in frozen]
    assert len(pg) == len(kept)
    assert [g["params"] for g in pg] == [[i] for i in range(len(kept))]
    for g, n in zip(pg, kept):
        assert g["weight_decay"] == (0.0 if is_no_decay(n) else 0.01), n
        assert abs(g["initial_lr"] - src.lr * src.lr_mult.get(n, 1.0)) < 1e-15, n
    assert len(ck["scheduler_state_dict"]["base_lrs"]) == len(kept)
    assert set(ck["optimizer_state_dict"]["state"]) == {i for i, n in enumerate(kept) if not is_frozen(n)}

    dst = _fake_trainer(cfg, 6, step=0)
    dst.lr_mult, dst.frozen_names = dict(src.lr_mult), tuple(frozen)
    dst.engine.fp.grad = torch.zeros_like(dst.engine.fp.data)
    assert C.load_checkpoint(dst, tar) == 3
    fs, fd = src.engine.fp, dst.engine.fp
    for n in kept:
        if not is_frozen(n):
            o, k = fs.offsets[n], fs.p[n].numel()
            assert torch.equal(src.m[o:o + k], dst.m[o:o + k]), n
    assert dst.lr == src.lr

    two = _fake_trainer(cfg, 7, step=0)   # two-group optimizer cannot take the per-tensor file
    two.engine.fp.grad = torch.zeros_like(two.engine.fp.data)
    with pytest.raises(ValueError):
        C.load_checkpoint(two, tar)


def test_checkpoint_fused_adam_layout(tmp_path):
    """--apex_fast branch (:413-418): apex FusedAdam state_dict — per-group step and
    bias_correction=False, per-parameter exp_avg / exp_avg_sq only."""
    from k3m_amd import checkpoint as C
    cfg = _tiny_cfg()
    src = _fake_trainer(cfg, 8, step=4)
    src.optimizer = "fused_adam"
    tar = str(tmp_path / "fa.tar")
    C.save_checkpoint(src, tar_path=tar)
    osd = torch.load(tar, map_location="cpu", weights_only=True)["optimizer_state_dict"]
    assert all(g["step"] == 4 and g["bias_correction"] is False for g in osd["param_groups"])
    assert set(next(iter(osd["state"].values()))) == {"exp_avg", "exp_avg_sq"}
    dst = _fake_trainer(cfg, 9, step=0)
    dst.optimizer = "fused_adam"
    dst.engine.fp.grad = torch.zeros_like(dst.engine.fp.data)
    assert C.load_checkpoint(dst, tar) == 4
    from k3m_amd.params import is_frozen
    fs = src.engine.fp
    for n, _ in fs.spec:
        if not is_frozen(n):
            o, k = fs.offsets[n], fs.p[n].numel()
            assert torch.equal(src.m[o:o + k], dst.m[o:o + k]) and torch.equal(src.v[o:o + k], dst.v[o:o + k]), n
