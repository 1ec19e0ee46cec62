"""Golden vectors for the data path — run in the BUILD container only.

Records built from rows of data/raw_multidata_of_product_preatrain.small_train (titles and
property-value strings) plus seeded synthetic regions (no images are bundled) are pushed through the
reference's own BertPreprocessBatch.__call__ (vilbert_k3m/datasets/concept_cap_dataset_struc.py
:564-648, imported with the stubs of make_golden.py and its character tokenizer) and the global-region
collation of ConceptCapLoaderTrain_struc.__iter__ (:381-397), under ``random.seed(s);
np.random.seed(s)``.  Edge cases: truncated titles and PV strings, no / one / unterminated /
malformed property-value triples, more triples than max_num_pv, empty title, num_boxes = 0 (default
region), num_boxes < and = max_region_len, clustered boxes (IoU > 0.4 chains), visualization=True,
visual_target=1.  Features are small (F=64, C=40) so the fixture stays small; only inputs and
outputs are committed (golden_data.npz).

Usage:  python tests/golden/make_data_golden.py
"""
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF, CharTokenizer, _stub_imports  # noqa: E402

FIELDS = ["item_id", "input_ids", "input_mask", "segment_ids", "lm_label_ids", "is_next", "input_ids_pv",
          "input_mask_pv", "segment_ids_pv", "lm_label_ids_pv", "is_next_pv_v", "is_next_pv_t", "index_p", "index_v",
          "image_feat", "image_loc", "image_target", "image_label", "image_mask", "masked_label"]


def regions(rng, nbox, F, C, clustered=False):
    h, w = float(rng.integers(300, 1000)), float(rng.integers(300, 1000))
    if clustered:   # a few boxes jittered around two centres: many IoU > 0.4 pairs
        cx = rng.choice([0.3 * w, 0.6 * w], nbox) + rng.normal(0, 6, nbox)
        cy = rng.choice([0.4 * h, 0.5 * h], nbox) + rng.normal(0, 6, nbox)
        bw, bh = rng.uniform(80, 120, nbox), rng.uniform(80, 120, nbox)
        x1, y1, x2, y2 = cx - bw / 2, cy - bh / 2, cx + bw / 2, cy + bh / 2
    else:
        x1 = rng.uniform(0, w * 0.7, nbox)
        y1 = rng.uniform(0, h * 0.7, nbox)
        x2 = np.minimum(w, x1 + rng.uniform(20, w * 0.3, nbox))
        y2 = np.minimum(h, y1 + rng.uniform(20, h * 0.3, nbox))
    boxes = np.stack([x1, y1, x2, y2], 1).astype(np.float32)
    if nbox > 1:
        boxes[-1] = boxes[0]          # an exact duplicate box (IoU 1)
    f = (np.abs(rng.standard_normal((nbox, F))) * 0.5).astype(np.float32)
    p = rng.random((nbox, C)).astype(np.float32)
    return h, w, boxes, f, p


PV_EDGE = [
    "no-properties-here",                       # zero triples
    "颜色#:#红色",                               # one triple, no trailing ';'
    "颜色#:#红色#;#",                            # one triple
    "颜色#:#红色#;#尺码#:#大",                    # last triple unterminated
    ";#颜色#:#红色#:#蓝色",                       # malformed: ';' before ':' and two ':'
    "#;#".join("属性%d#:#值%d" % (i, i) for i in range(30)),   # more triples than max_num_pv
    "",
]


def make_case(name, rows, pre_kw, seed, nboxes, F=64, C=40, clustered=(), edit=None):
    from vilbert_k3m.datasets.concept_cap_dataset_struc import BertPreprocessBatch
    tok = CharTokenizer()
    pre = BertPreprocessBatch(tok, v_feature_size=F, v_target_size=C, **pre_kw)
    R = pre.max_region_len
    rng = np.random.default_rng(1000 + seed)
    recs = []
    for i, r in enumerate(rows):
        item_id, title, _url, pv, cate = r
        if edit:
            title, pv = edit(i, title, pv)
        nb = nboxes[i % len(nboxes)]
        h, w, boxes, f, p = regions(rng, max(nb, 1), F, C, clustered=i in clustered)
        if nb == 0:
            boxes, f, p = boxes[:0], f[:0], p[:0]
        recs.append((item_id, title, pv, cate, h, w, nb, boxes, f, p))
    random.seed(seed)
    np.random.seed(seed)
    outs = [pre((rid, t, pv, c, h, w, nb, bx.copy(), f.copy(), p.copy())) for (rid, t, pv, c, h, w, nb, bx, f, p) in recs]
    res = {}
    B = len(recs)
    res["in/item_id"] = np.array([r[0] for r in recs])
    res["in/caption"] = np.array([r[1] for r in recs])
    res["in/pv"] = np.array([r[2] for r in recs])
    res["in/image_hw"] = np.array([[r[4], r[5]] for r in recs], np.float64)
    res["in/num_boxes"] = np.array([r[6] for r in recs], np.int64)
    res["in/boxes"] = np.zeros((B, R, 4), np.float32)
    res["in/feat"] = np.zeros((B, R, F), np.float32)
    res["in/target"] = np.zeros((B, R, C), np.float32)
    for b, r in enumerate(recs):
        n = r[6]
        res["in/boxes"][b, :n] = r[7]
        res["in/feat"][b, :n] = r[8]
        res["in/target"][b, :n] = r[9]
    for k, v in pre_kw.items():
        res["cfg/" + k] = np.array(v)
    res["cfg/seed"] = np.array(seed)
    res["cfg/v_feature_size"] = np.array(F)
    res["cfg/v_target_size"] = np.array(C)
    for j, name_ in enumerate(FIELDS[1:], 1):
        vals = [o[j] for o in outs]
        if name_ == "masked_label":
            res["out/masked_label_is_bool"] = np.array([v.dtype == np.bool_ for v in vals])
            vals = [np.asarray(v, np.float64) for v in vals]
        res["out/" + name_] = np.stack(vals)
    # collation (ConceptCapLoaderTrain_struc.__iter__, dataset:381-397)
    image_feat, image_loc = res["out/image_feat"], res["out/image_loc"]
    masked_label, image_mask = res["out/masked_label"], res["out/image_mask"]
    cnt = np.sum(masked_label == 0, axis=1, keepdims=True)
    cnt[cnt == 0] = 1
    g = np.sum(image_feat, axis=1) / cnt
    res["coll/image_feat"] = np.array(np.concatenate([np.expand_dims(g, 1), image_feat], 1), dtype=np.float32)
    gl = np.repeat(np.array([[0, 0, 1, 1, 1]], dtype=np.float32), B, axis=0)
    res["coll/image_loc"] = np.array(np.concatenate([np.expand_dims(gl, 1), image_loc], 1), dtype=np.float32)
    res["coll/image_mask"] = np.concatenate([np.repeat(np.array([[1]]), B, axis=0), image_mask], 1)
    return {name + "/" + k: v for k, v in res.items()}


def main():
    _stub_imports()
    rows = [l.rstrip("\n").split("\t") for l in open(os.path.join(REF, "data/raw_multidata_of_product_preatrain.small_train"),
                                                        encoding="utf-8")]
    out = {}
    # A: default geometry of the driver (T=36, P=128, 20 PV slots, 36 regions), 24 rows
    out.update(make_case("base", rows[:24], dict(max_seq_len=36, max_seq_len_pv=128, max_num_pv=20, max_region_len=36),
                         seed=5, nboxes=[36, 20, 10, 0, 1, 36, 35, 7], clustered=(0, 2, 5)))

    # B: short windows (truncation), few PV slots, num_boxes == max_region_len, PV edge strings
    def edit_b(i, title, pv):
        if i < len(PV_EDGE):
            pv = PV_EDGE[i]
        if i == len(PV_EDGE):
            title = ""
        return title, pv
    out.update(make_case("short", rows[30:44], dict(max_seq_len=16, max_seq_len_pv=24, max_num_pv=3, max_region_len=10),
                         seed=11, nboxes=[10, 10, 3, 0, 10], clustered=(0, 1, 4, 9), edit=edit_b))
    # C: visualization=True (draws kept, nothing masked)
    out.update(make_case("vis", rows[50:56], dict(max_seq_len=36, max_seq_len_pv=64, max_num_pv=8, max_region_len=12,
                                                  visualization=True), seed=3, nboxes=[12, 5, 0]))
    # D: visual_target=1 (targets are the unmasked features)
    out.update(make_case("vt1", rows[60:68], dict(max_seq_len=36, max_seq_len_pv=64, max_num_pv=8, max_region_len=12,
                                                  visual_target=1), seed=21, nboxes=[12, 9, 0, 4], clustered=(1,)))
    path = os.path.join(HERE, "golden_data.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path) // 1024, "KiB")


if __name__ == "__main__":
    main()
