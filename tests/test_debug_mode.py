"""Debug mode (k3m_amd/debug.py): index checks against the reference input contract, on the host.
The serialized-launch half and the engine integration run on the GPU (tests/test_gpu_debug_mode.py)."""
import os

import pytest
import torch

from k3m_amd import debug
from k3m_amd.config import pretrain_config
from k3m_amd.synthetic import synthetic_batch

CFG_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                        "bert_base_6layer_6conect.json")


def test_check_range_bounds_and_ignore():
    debug.check_range(torch.tensor([0, 5, 9]), 0, 10, "x")
    debug.check_range(torch.tensor([-1, 3, -1]), 0, 10, "labels", ignore=-1)
    debug.check_range(torch.tensor([-1, -1]), 0, 10, "labels", ignore=-1)
    debug.check_range(torch.empty(0, dtype=torch.int64), 0, 1, "empty")
    with pytest.raises(debug.K3mIndexError, match=r"x: index 10 out of range \[0, 10\)"):
        debug.check_range(torch.tensor([0, 10]), 0, 10, "x")
    with pytest.raises(debug.K3mIndexError, match="index -2"):
        debug.check_range(torch.tensor([-2, 3]), 0, 10, "labels", ignore=-1)
    assert issubclass(debug.K3mIndexError, IndexError)   # what torch's nn.Embedding raises on the CPU


def test_check_batch_accepts_the_synthetic_contract():
    cfg = pretrain_config(CFG_PATH)
    b = synthetic_batch(cfg, 3, torch.device("cpu"), seed=4)
    debug.check_batch(b, cfg)


@pytest.mark.parametrize("field,value,msg", [
    ("input_ids", 21128, "input_ids: index 21128"),
    ("input_ids_pv", -5, "input_ids_pv: index -5"),
    ("segment_ids", 2, "segment_ids: index 2"),
    ("lm_label_ids", 30000, "lm_label_ids: index 30000"),
    ("is_next", 3, "is_next: index 3"),
    ("index_p", 128, "index_p: index 128"),
    ("index_v", -3, "index_v: index -3"),
])
def test_check_batch_names_the_bad_field(field, value, msg):
    cfg = pretrain_config(CFG_PATH)
    b = synthetic_batch(cfg, 2, torch.device("cpu"), seed=5)
    t = b[field].clone()
    t.view(-1)[1] = value
    b[field] = t
    with pytest.raises(debug.K3mIndexError, match=msg):
        debug.check_batch(b, cfg)


def test_check_batch_negatives_and_lengths():
    cfg = pretrain_config(CFG_PATH)
    b = synthetic_batch(cfg, 2, torch.device("cpu"), seed=6)
    npv = b["index_p"].shape[1]
    ent = torch.full((2, npv, 2), -1, dtype=torch.int64)
    val = torch.full((2, npv, 2), -1, dtype=torch.int64)
    n = int(debug.item_triples(b["index_p"])[1])   # 10 triples, padded to npv = 20 pairs
    assert n == 10 < npv
    ent[0, 0, 0], val[1, 0, 1] = 1, n - 1
    debug.check_batch(b, cfg, ent, val)
    # a value negative naming a padding pair (n <= k < npv) is refused too -- LPM would read an unset row
    val[1, 0, 1] = n
    with pytest.raises(debug.K3mIndexError, match="triple count"):
        debug.check_batch(b, cfg, ent, val)
    val[1, n, 1] = npv - 1   # pairs j >= n are not scored: their table entries are not checked
    val[1, 0, 1] = n - 1
    debug.check_batch(b, cfg, ent, val)
    ent[0, 0, 1] = 2   # only 2 items in the batch
    with pytest.raises(debug.K3mIndexError, match="ent_neg"):
        debug.check_batch(b, cfg, ent, val)
    ent[0, 0, 1] = -1
    val[0, 1, 0] = npv
    with pytest.raises(debug.K3mIndexError, match="val_neg"):
        debug.check_batch(b, cfg, ent, val)
    with pytest.raises(debug.K3mIndexError, match="exceeds max_position_embeddings"):
        debug.check_len(513, cfg.max_position_embeddings, "text length")
