"""Host-side logic of the training step (no GPU): optimizer runs over the flat buffer and the
parameter groups of train_concap_struc.py:352-389, the LR schedules (:392-448, :579-588), the
objective == 1 label rewrite (:481-494), the asynchronous NaN fail-fast, the apex FusedAdam
restatement, and the drop-in import surface (vilbert_k3m shim package, loaders' constructor)."""
import math
import types

import numpy as np
import pytest
import torch

from golden_util import CFG_PATH


def _fp(cfg):
    from k3m_amd.params import flat_layout
    spec, offsets, segments, total, shapes = flat_layout(cfg)
    return types.SimpleNamespace(spec=spec, offsets=offsets, segments=segments, total=total, shapes=shapes)


def _cfg():
    from k3m_amd.config import pretrain_config
    return pretrain_config(CFG_PATH)


def test_optimizer_runs_two_groups():
    """No pretrained model: two groups (decay 0.01 / no_decay 0.0) -> two contiguous runs that cover
    every tensor receiving a gradient exactly once and skip the 86 never-grad tensors."""
    from k3m_amd.params import segment_of
    from k3m_amd.trainer import optimizer_runs
    fp = _fp(_cfg())
    runs = optimizer_runs(fp)
    assert [(wd, mu) for _, _, wd, mu in runs] == [(0.01, 1.0), (0.0, 1.0)]
    cover = np.zeros(fp.total, np.int8)
    for a, n, _, _ in runs:
        assert a % 4 == 0 and n % 4 == 0
        cover[a:a + n] += 1
    for name, shape in fp.spec:
        o, k = fp.offsets[name], math.prod(shape)
        want = 0 if segment_of(name) == "frozen" else 1
        assert (cover[o:o + k] == want).all(), name
    n_frozen = sum(1 for n, _ in fp.spec if segment_of(n) == "frozen")
    assert n_frozen == 86


def test_optimizer_runs_lr_mult_and_freeze():
    """Pretrained model: per-tensor groups with lr x 0.1 for the BERT weight names
    (train_concap_struc.py:369-385); --freeze names are skipped (:243-260)."""
    from k3m_amd.trainer import optimizer_runs, bert_lr_mult
    fp = _fp(_cfg())
    names = [n for n, _ in fp.spec]
    # the weight-name file as a DDP run would match it: "module." + name, first 12 characters dropped
    bert_names = [("module." + n)[12:] for n in names if n.startswith("embeddings.") or n.startswith("encoder.layer.")]
    mult = bert_lr_mult(names, bert_names, ddp=True)
    assert all(n.startswith("embeddings.") or n.startswith("encoder.layer.") for n in mult)
    assert len(mult) == 5 + 12 * 16
    frozen = ["encoder.layer.0.attention.self.query.weight"]
    runs = optimizer_runs(fp, lr_mult=mult, frozen_names=frozen)
    got = {}
    for name, shape in fp.spec:
        o = fp.offsets[name]
        hit = [r for r in runs if r[0] <= o < r[0] + r[1]]
        got[name] = hit
    assert got[frozen[0]] == []
    assert got["embeddings.word_embeddings.weight"][0][3] == 0.1
    assert got["encoder.layer.3.output.dense.weight"][0][3] == 0.1
    assert got["encoder.v_layer.0.output.dense.weight"][0][3] == 1.0
    assert got["encoder.layer.3.output.dense.bias"][0][2] == 0.0
    # without DDP the driver's key[12:] applies to the bare name
    assert bert_lr_mult(["encoder.layer.0.output.dense.weight"], ["r.0.output.dense.weight"], ddp=False)


def test_schedules():
    from k3m_amd.trainer import warmup_linear_lambda, warmup_linear_fp16
    assert warmup_linear_lambda(0, 10, 100) == 0.0       # the first step runs at lr = 0
    assert warmup_linear_lambda(5, 10, 100) == 0.5
    assert warmup_linear_lambda(10, 10, 100) == 1.0
    assert abs(warmup_linear_lambda(55, 10, 100) - 0.5) < 1e-12
    assert warmup_linear_lambda(200, 10, 100) == 0.0
    assert warmup_linear_fp16(0.05, 0.1) == 0.5            # train_concap_struc.py:60-65
    assert abs(warmup_linear_fp16(0.55, 0.1) - 0.5) < 1e-12
    assert warmup_linear_fp16(1.5, 0.1) == 0


def test_objective1_label_rewrite():
    from k3m_amd.trainer import objective1_labels
    b = {"is_next": torch.tensor([0, 1, 0]), "is_next_pv_v": torch.tensor([0, 0, 0]),
         "is_next_pv_t": torch.tensor([0, 0, 1]),
         "lm_label_ids": torch.tensor([[5, -1, 0], [7, 8, -1], [9, -1, 3]]),
         "lm_label_ids_pv": torch.tensor([[-1, 4], [6, -1], [2, 2]]),
         "image_label": torch.tensor([[1, -1], [1, 1], [-1, 1]]), "_label_counts": (1, 1)}
    o = objective1_labels(b)
    # kept rows unchanged except that a label id 0 becomes -1 (the reference's `== 0 -> -1`)
    assert o["lm_label_ids"].tolist() == [[5, -1, -1], [-1, -1, -1], [-1, -1, -1]]
    assert o["lm_label_ids_pv"].tolist() == [[-1, 4], [-1, -1], [-1, -1]]
    assert o["image_label"].tolist() == [[1, -1], [-1, -1], [-1, -1]]
    assert "_label_counts" not in o
    assert b["lm_label_ids"].tolist()[0] == [5, -1, 0]   # the caller's batch is untouched


def test_loss_watch_fail_fast_cpu():
    from k3m_amd.trainer import LossWatch
    w = LossWatch()
    w.push(0, torch.tensor([1.5]))
    with pytest.raises(FloatingPointError):
        w.push(1, torch.tensor([float("nan")]))


def test_fused_adam_restatement_known_answer():
    """apex FusedAdam(adam_w_mode, bias_correction=False) one step by hand."""
    from oracle.k3m_oracle import fused_adam_step
    p = torch.tensor([1.0, -2.0], dtype=torch.float64)
    g = torch.tensor([0.5, 0.25], dtype=torch.float64)
    m, v = torch.zeros(2, dtype=torch.float64), torch.zeros(2, dtype=torch.float64)
    fused_adam_step(p, g, m, v, 1, lr=0.1, wd=0.01, beta1=0.9, beta2=0.999, eps=1e-8, bias_correction=False)
    m_ = 0.1 * np.array([0.5, 0.25])
    v_ = 0.001 * np.array([0.25, 0.0625])
    p_ = np.array([1.0, -2.0]) - 0.1 * (m_ / (np.sqrt(v_) + 1e-8) + 0.01 * np.array([1.0, -2.0]))
    np.testing.assert_allclose(p.numpy(), p_, rtol=1e-12)
    np.testing.assert_allclose(m.numpy(), m_, rtol=1e-12)


def test_dropin_import_surface():
    """The driver's import lines (train_concap_struc.py:25-26) resolve to this build, unchanged."""
    from vilbert_k3m.datasets import ConceptCapLoaderTrain_struc, ConceptCapLoaderVal_struc  # noqa: F401
    from vilbert_k3m.vilbert_k3m import BertConfig, BertForMultiModalPreTraining_tri_stru
    from k3m_amd.vilbert_k3m import BertForMultiModalPreTraining_tri_stru as Impl
    assert BertForMultiModalPreTraining_tri_stru is Impl
    cfg = BertConfig.from_json_file(CFG_PATH)
    assert cfg.num_hidden_layers == 12 and cfg.v_biattention_id == [0, 1, 2, 3, 4, 5]
    import inspect
    sig = inspect.signature(ConceptCapLoaderTrain_struc.__init__)
    for kw in ("max_seq_len", "max_seq_len_pv", "max_num_pv", "max_region_len", "batch_size", "visual_target",
               "v_target_size", "num_workers", "local_rank", "objective", "cache", "serializer"):
        assert kw in sig.parameters, kw
    sig = inspect.signature(ConceptCapLoaderVal_struc.__init__)
    for kw in ("max_seq_len", "max_seq_len_pv", "max_num_pv", "max_region_len", "batch_size", "visual_target",
               "v_target_size", "objective", "serializer"):
        assert kw in sig.parameters, kw


def test_raw_tsv_records(tmp_path):
    """Raw product rows -> the records data_prepare.py writes for items without an image."""
    from k3m_amd.loaders import read_raw_tsv, write_records, RecordDir
    p = tmp_path / "rows.tsv"
    p.write_text("1\ttitle one\thttp://x\ta#:#b#;#c#:#d\tcat\n2\tt2\thttp://y\tk#:#v\tcat\n", encoding="utf-8")
    recs = read_raw_tsv(str(p))
    assert [r[2] for r in recs] == ["a:b;c:d;", "k:v;"]          # '#' stripped, trailing ';' (:333-336)
    assert recs[0][4:7] == (800, 800, 1)
    write_records(str(tmp_path / "rec"), recs)
    rd = RecordDir(str(tmp_path / "rec"))
    assert len(rd) == 2
    r = rd[1]
    assert r[0] == "2" and r[2] == "k:v;" and r[6] == 1 and r[7].shape == (1, 4) and r[8].shape == (1, 2048)
    np.testing.assert_allclose(r[7][0], [0.1, 0.1, 799.9, 799.9], rtol=1e-6)


def test_fp16_schedule_first_group_is_the_decay_segment():
    """--fp16 schedule quirk (train_concap_struc.py:579-584): only param_groups[0] — the decay group —
    follows warmup_linear; identified by the flat-buffer segment, so weight_decay=0 still trains."""
    from k3m_amd.trainer import Trainer
    fp = _fp(_cfg())
    t = types.SimpleNamespace(lr_schedule="warmup_linear_fp16", lr=1e-3, warmup=10, t_total=100,
                              warmup_proportion=0.1, global_step=50, engine=types.SimpleNamespace(fp=fp))
    t.current_lr = lambda: Trainer.current_lr(t)
    dec, nod = fp.segments["decay"][0], fp.segments["no_decay"][0]
    assert Trainer.run_lr(t, dec, 1.0) > 0            # group 0: re-set every step
    assert Trainer.run_lr(t, nod, 1.0) == 0.0         # other groups keep lr * lambda(0) = 0
