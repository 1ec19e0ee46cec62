"""Debug mode on the GPU (k3m_amd/debug.py): serialized launches give the same losses as the release
path, and a batch outside the reference input contract is refused before any kernel reads it."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

CFG_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                        "bert_base_6layer_6conect.json")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from k3m_amd import _lib
    _lib.load()
    return torch.device("cuda")


@pytest.fixture
def debug_on():
    from k3m_amd import debug
    old = debug.ON
    debug.set_debug(True)
    yield debug
    debug.set_debug(old)


def _cfg():
    from k3m_amd.config import pretrain_config
    return pretrain_config(CFG_PATH)


def _losses(tr, b):
    out, _ = tr.engine.forward(b, train=False, seed=7)
    return {k: float(v) for k, v in out.items() if torch.is_tensor(v) and v.numel() == 1}


def test_debug_forward_matches_release(dev, debug_on):
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    cfg = _cfg()
    tr = Trainer(cfg, dev, seed=11)
    b = synthetic_batch(cfg, 2, dev, seed=12)
    dbg = _losses(tr, b)
    debug_on.set_debug(False)
    rel = _losses(tr, b)
    assert dbg and dbg == rel


def test_debug_refuses_out_of_range_batch(dev, debug_on):
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    cfg = _cfg()
    tr = Trainer(cfg, dev, seed=13)
    b = synthetic_batch(cfg, 2, dev, seed=14)
    bad = dict(b)
    bad["input_ids"] = b["input_ids"].clone()
    bad["input_ids"][1, 3] = cfg.vocab_size + 7
    with pytest.raises(debug_on.K3mIndexError, match="input_ids: index %d" % (cfg.vocab_size + 7)):
        tr.engine.forward(bad, train=False)
    bad = dict(b)
    bad["index_v"] = b["index_v"].clone()
    bad["index_v"][0, 0, 1] = b["input_ids_pv"].shape[1]
    with pytest.raises(debug_on.K3mIndexError, match="index_v"):
        tr.engine.forward(bad, train=False)
    _losses(tr, b)   # the engine is still usable: nothing bad reached the device


def test_debug_row_gather_checked(dev, debug_on):
    from k3m_amd import ops
    src = torch.randn(10, 64, device=dev)
    out = torch.empty(4, 64, device=dev)
    idx = torch.tensor([0, 3, 9, 2], device=dev, dtype=torch.int32)
    ops.gather_rows(src, idx, 4, out)
    assert torch.equal(out, src[idx.long()])
    with pytest.raises(debug_on.K3mIndexError, match="gather_rows index: index 10"):
        ops.gather_rows(src, torch.tensor([0, 10, 1, 2], device=dev, dtype=torch.int32), 4, out)
    dst = torch.zeros(3, 64, device=dev)
    with pytest.raises(debug_on.K3mIndexError, match="scatter_add_rows index: index 3"):
        ops.scatter_add_rows(out, torch.tensor([0, 1, 3, 2], device=dev, dtype=torch.int32), 4, dst)
