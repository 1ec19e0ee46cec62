"""Data path on the GPU: the region collation kernel
(k3m_collate_regions through RegionCollator) against the reference's collation recorded in
tests/golden/golden_data.npz, bit for bit; at the driver's full size (B=64, 36 x 2048 features)
against the numpy restatement (oracle/data_oracle.py); and records -> loader -> one training step."""
import os

import numpy as np
import pytest
import torch

from k3m_amd import data as D
from oracle import data_oracle as DO
from tests.test_data import CASES, D_FIELDS, case, char_tokenizer, preprocessor, records

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def gold():
    z = np.load(os.path.join(HERE, "golden", "golden_data.npz"))
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name", CASES)
def test_collator_matches_reference(gold, name):
    c = case(gold, name)
    pre = preprocessor(c, D.RandomStreams(int(c["cfg/seed"])))
    samples = [pre.prepare(r) for r in records(c)]
    col = D.RegionCollator("cuda", pre.max_region_len, pre.v_feature_size, pre.v_target_size, pre.visual_target)
    batch, ids = col(samples)
    torch.cuda.synchronize()
    assert ids == [str(x) for x in c["in/item_id"]]
    assert np.array_equal(batch["image_feat"].cpu().numpy(), c["coll/image_feat"])
    assert np.array_equal(batch["image_loc"].cpu().numpy(), c["coll/image_loc"])
    assert np.array_equal(batch["image_mask"].cpu().numpy(), c["coll/image_mask"])
    for f in D_FIELDS[1:]:
        if f in ("image_feat", "image_loc", "image_mask", "masked_label"):
            continue
        got = batch[f].cpu().numpy()
        want = c["out/" + f]
        assert np.array_equal(got, want.reshape(got.shape)), f


@pytest.mark.parametrize("B,R,F,p_zero,p_mask", [(64, 36, 2048, 0.15, 0.3), (3, 36, 2048, 1.0, 1.0),
                                                 (1, 1, 4, 0.0, 0.0), (7, 10, 1604, 0.5, 0.9)])
def test_collate_kernel_full_size(B, R, F, p_zero, p_mask):
    from k3m_amd import _lib
    rng = np.random.default_rng(B * 1000 + F)
    feat = (rng.standard_normal((B, R, F)) * rng.uniform(0.1, 100, (B, R, 1))).astype(np.float32)
    zero = (rng.random((B, R)) < p_zero).astype(np.uint8)
    mlab = ((rng.random((B, R)) < p_mask) | zero.astype(bool)).astype(np.uint8)
    want = DO.collate_regions(feat, zero, mlab)
    fd = torch.from_numpy(feat).cuda()
    out = torch.full((B, R + 1, F), float("nan"), device="cuda")
    zd, md = torch.from_numpy(zero).cuda(), torch.from_numpy(mlab).cuda()   # kept alive across the launch
    _lib.call("k3m_collate_regions", fd.data_ptr(), R * F, zd.data_ptr(), md.data_ptr(), None, B, R, F, out.data_ptr(),
              _lib.stream())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)


def test_loader_feeds_training_step():
    """records -> K3mPretrainLoader (native prep + GPU collation) -> one Trainer step."""
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    cfg = pretrain_config(os.path.join(os.path.dirname(HERE), "configs", "bert_base_6layer_6conect.json"))
    rng = np.random.default_rng(0)
    titles = ["女装上衣%d号新款加绒打底衫" % i for i in range(4)]
    pvs = ["颜色#:#红色#;#尺码#:#大#;#材质#:#棉", "产地#:#中国#;#款式#:#带护网", "no-properties", "品名#:#请填写"]
    recs = []
    for i in range(4):
        nb = [36, 12, 0, 5][i]
        x1 = rng.uniform(0, 500, max(nb, 1))
        y1 = rng.uniform(0, 400, max(nb, 1))
        boxes = np.stack([x1, y1, x1 + 100, y1 + 80], 1).astype(np.float32)[:nb]
        recs.append(("id%d" % i, titles[i], pvs[i], "", 600, 800, nb, boxes,
                     np.abs(rng.standard_normal((nb, 2048))).astype(np.float32),
                     rng.dirichlet(np.ones(1601), nb).astype(np.float32)))
    loader = D.K3mPretrainLoader(recs, char_tokenizer(), "cuda", batch_size=4, streams=D.RandomStreams(7),
                                 max_seq_len=36, max_seq_len_pv=128, max_num_pv=20, max_region_len=36)
    batches = list(loader)
    assert len(batches) == 1
    batch, ids = batches[0]
    assert batch["image_feat"].shape == (4, 37, 2048) and ids == ["id0", "id1", "id2", "id3"]
    tr = Trainer(cfg, torch.device("cuda", 0), lr=1e-4, warmup_steps=0, total_steps=10, seed=1)
    out = tr.step(batch)
    loss = float(out["loss"] if isinstance(out, dict) else out)
    assert np.isfinite(loss) and loss > 0
