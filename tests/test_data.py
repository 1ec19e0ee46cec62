"""Data path on the CPU: the native per-sample preprocessing
(libk3m_data.so via k3m_amd.data) against the reference's own BertPreprocessBatch outputs recorded
in tests/golden/golden_data.npz (make_data_golden.py), bit for bit; the random streams against
CPython's `random` and numpy's legacy RandomState; the collation restatement against the reference's
collation."""
import os
import random

import numpy as np
import pytest

from k3m_amd import data as D
from oracle import data_oracle as DO

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "golden_data.npz")
CASES = ["base", "short", "vis", "vt1"]


@pytest.fixture(scope="module")
def gold():
    z = np.load(GOLD)
    return {k: z[k] for k in z.files}


def char_tokenizer():
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_golden import CharTokenizer
    return CharTokenizer()


def case(gold, name):
    return {k[len(name) + 1:]: v for k, v in gold.items() if k.startswith(name + "/")}


def records(c):
    out = []
    for b in range(len(c["in/item_id"])):
        nb = int(c["in/num_boxes"][b])
        h, w = c["in/image_hw"][b]
        out.append((str(c["in/item_id"][b]), str(c["in/caption"][b]), str(c["in/pv"][b]), "", h, w, nb,
                    c["in/boxes"][b, :nb], c["in/feat"][b, :nb], c["in/target"][b, :nb]))
    return out


def preprocessor(c, streams):
    kw = {k[4:]: v.item() for k, v in c.items() if k.startswith("cfg/") and k != "cfg/seed"}
    return D.BertPreprocessBatch(char_tokenizer(), streams=streams, **kw)


def test_data_lib_exports():
    assert sorted(D.data_exported_symbols()) == sorted(D.DATA_SIGNATURES)


@pytest.mark.parametrize("seed", [0, 1, 5, 2 ** 31 + 7, 2 ** 45 + 11])
def test_streams_match_python_and_numpy(seed):
    rs = D.RandomStreams(seed, seed % 2 ** 32)
    random.seed(seed)
    np.random.seed(seed % 2 ** 32)
    assert [random.random() for _ in range(3000)] == [rs.random() for _ in range(3000)]
    for high in (1, 2, 5, 21128, 30522, 2 ** 31 - 1, 2 ** 32):
        assert [np.random.randint(high) for _ in range(200)] == [rs.randint(high) for _ in range(200)]


@pytest.mark.parametrize("name", CASES)
def test_preprocess_matches_reference(gold, name):
    c = case(gold, name)
    pre = preprocessor(c, D.RandomStreams(int(c["cfg/seed"])))
    outs = [pre(r) for r in records(c)]
    for j, field in enumerate(D_FIELDS[1:], 1):
        got = [o[j] for o in outs]
        if field == "masked_label":
            assert [g.dtype == np.bool_ for g in got] == list(c["out/masked_label_is_bool"])
            got = [np.asarray(g, np.float64) for g in got]
        got = np.stack(got)
        want = c["out/" + field]
        assert got.dtype == want.dtype, field
        assert got.shape == want.shape, field
        assert np.array_equal(got, want), "%s/%s differs at %s" % (name, field, np.argwhere(got != want)[:5])


def test_cases_cover_edges(gold):
    """The fixture exercises what it claims: random replacements, masked regions with overlap
    chains, default boxes, truncation, zero-triple PV, full region windows."""
    b = case(gold, "base")
    s = case(gold, "short")
    ids, lm = b["out/input_ids"], b["out/lm_label_ids"]
    assert ((lm >= 0) & (ids != 103) & (ids != lm)).any()              # 10% random token
    assert ((lm >= 0) & (ids == lm)).any()                              # 10% kept
    ml, lab = b["out/masked_label"], b["out/image_label"]
    assert (ml.sum(1) > (lab == 1).sum(1)).any()                        # IoU > 0.4 chains
    assert (b["in/num_boxes"] == 0).any() and (s["in/num_boxes"] == 10).any()
    assert (s["out/input_mask"].sum(1) == 16).any() and (s["out/input_mask_pv"].sum(1) == 24).any()
    assert (s["out/index_p"][:, 0, 1] == 0).any()                       # no triple
    v = case(gold, "vis")
    assert (v["out/lm_label_ids"] == -1).all() and (v["out/image_label"] == -1).all()


@pytest.mark.parametrize("name", CASES)
def test_collation_restatement_matches_reference(gold, name):
    c = case(gold, name)
    pre = preprocessor(c, D.RandomStreams(int(c["cfg/seed"])))
    samples = [pre.prepare(r) for r in records(c)]
    R, F = pre.max_region_len, pre.v_feature_size
    feat = np.zeros((len(samples), R, F), np.float32)
    for b, s in enumerate(samples):
        feat[b, :s.num_boxes] = s.feat
    zero = np.stack([s.zero_feat for s in samples])
    mlab = np.stack([s.masked_label for s in samples])
    got = DO.collate_regions(feat, zero, mlab)
    assert np.array_equal(got, c["coll/image_feat"])
    loc, mask = DO.collate_locations(np.stack([s.image_loc for s in samples]), np.stack([s.image_mask for s in samples]))
    assert np.array_equal(loc, c["coll/image_loc"]) and np.array_equal(mask, c["coll/image_mask"])


def test_prepare_rejects_bad_records():
    pre = D.BertPreprocessBatch(char_tokenizer(), max_region_len=4, v_feature_size=8, v_target_size=4)
    bx = np.zeros((5, 4), np.float32)
    with pytest.raises(ValueError):
        pre.prepare(("x", "a", "b", "", 10, 10, 5, bx, np.zeros((5, 8)), np.zeros((5, 4))))


D_FIELDS = ["item_id", "input_ids", "input_mask", "segment_ids", "lm_label_ids", "is_next", "input_ids_pv",
            "input_mask_pv", "segment_ids_pv", "lm_label_ids_pv", "is_next_pv_v", "is_next_pv_t", "index_p", "index_v",
            "image_feat", "image_loc", "image_target", "image_label", "image_mask", "masked_label"]


# ---------------------------------------------------------------- fine-tuning pairs
@pytest.fixture(scope="module")
def ft_gold():
    z = np.load(os.path.join(HERE, "golden", "golden_ft_data.npz"))
    return {k: z[k] for k in z.files}


def ft_records(g):
    recs = []
    for b in range(len(g["in/label"])):
        rec = [int(g["in/label"][b])]
        for k in (1, 2):
            nb = int(g["in/num_boxes_%d" % k][b])
            h, w = g["in/image_hw_%d" % k][b]
            rec += [str(g["in/item_id_%d" % k][b]), str(g["in/caption_%d" % k][b]), str(g["in/pv_%d" % k][b]), "", h, w,
                    nb, g["in/boxes_%d" % k][b, :nb], g["in/feat_%d" % k][b, :nb], g["in/target_%d" % k][b, :nb]]
        recs.append(tuple(rec))
    return recs


def ft_preprocessor(g):
    return D.K3MPreprocessBatch(char_tokenizer(), max_seq_len=int(g["cfg/max_seq_len"]),
                                max_seq_len_pv=int(g["cfg/max_seq_len_pv"]), max_num_pv=int(g["cfg/max_num_pv"]),
                                max_region_len=int(g["cfg/max_region_len"]), v_feature_size=int(g["cfg/v_feature_size"]),
                                v_target_size=int(g["cfg/v_target_size"]))


def test_finetune_preprocess_matches_reference(ft_gold):
    g = ft_gold
    pre = ft_preprocessor(g)
    outs = [pre(r) for r in ft_records(g)]
    for j, field in enumerate(D.PAIR_TUPLE):
        if field.startswith("item_id"):
            assert [o[j] for o in outs] == [str(x) for x in g["in/" + field]]
            continue
        got = np.stack([np.asarray(o[j]) for o in outs])
        want = g["out/" + field]
        assert got.shape == want.shape and np.array_equal(got, want), field
    assert (g["in/num_boxes_1"] == 0).any() or (g["in/num_boxes_2"] == 0).any()


def test_finetune_collation_restatement_matches_reference(ft_gold):
    g = ft_gold
    for k in (1, 2):
        f, l, m = DO.collate_pair_item(g["out/image_feat_%d" % k], g["out/num_boxes_%d" % k], g["out/image_loc_%d" % k],
                                       g["out/image_mask_%d" % k])
        assert np.array_equal(f, g["out/coll_image_feat_%d" % k], equal_nan=True)
        assert np.array_equal(l, g["out/coll_image_loc_%d" % k]) and np.array_equal(m, g["out/coll_image_mask_%d" % k])
