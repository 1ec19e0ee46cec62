"""Golden vectors for item-alignment fine-tuning — BUILD container only.

Imports the reference K3MForItemAlignment (vilbert_k3m/vilbert_k3m.py:2862-3456) and its data path
(K3MPreprocessBatch, dataset:936-1263; K3MDataLoader.post_process, :265-292) with the stubs and the
character tokenizer of make_golden.py, under the fine-tuning driver's config mutations
(finetune.py:1307-1322: model "roberta", use_image, loss_type).  Records:

* ``param_inventory_finetune.json``: named_parameters() names/shapes for loss_type ce and cosine;
* ``golden_ft_<case>.npz``: a pair batch built by the reference's own preprocessing (rows of
  data/raw_multidata_of_product_preatrain.small_train + seeded synthetic regions), weights from
  k3m_amd.weights.param_values, explicit gumbel noise per item, model.eval(); outputs
  (item_embedding_1, item_embedding_2, probs, loss) and gradients of the loss;
* ``golden_ft_data.npz``: the preprocessing alone on edge cases (num_boxes = 0, truncation,
  unterminated / absent property-value triples) — no model.

Usage:  python tests/golden/make_finetune_golden.py
"""
import json
import os
import re
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
from make_golden import REF, CharTokenizer, _stub_imports, gumbel_noise  # noqa: E402
from make_data_golden import PV_EDGE, regions  # noqa: E402

PAIR_FIELDS = ["label", "item_id_1", "input_ids_1", "input_mask_1", "segment_ids_1", "input_ids_pv_1",
               "input_mask_pv_1", "segment_ids_pv_1", "index_p_1", "index_v_1", "num_boxes_1", "image_feat_1",
               "image_loc_1", "image_target_1", "image_mask_1", "item_id_2", "input_ids_2", "input_mask_2",
               "segment_ids_2", "input_ids_pv_2", "input_mask_pv_2", "segment_ids_pv_2", "index_p_2", "index_v_2",
               "num_boxes_2", "image_feat_2", "image_loc_2", "image_target_2", "image_mask_2"]


def rows():
    return [l.rstrip("\n").split("\t") for l in open(os.path.join(REF, "data/raw_multidata_of_product_preatrain.small_train"),
                                                      encoding="utf-8")]


def ref_cfg(loss_type, mode):
    import vilbert_k3m.vilbert_k3m as K
    from k3m_amd.config import finetune_config
    path = os.path.join(REPO, "configs/bert_base_6layer_6conect.json")
    cfg = finetune_config(path, loss_type=loss_type, if_pre_sampling=mode)
    rcfg = K.BertConfig.from_json_file(path)
    for k in ("v_target_size", "visual_target", "model", "use_image", "with_coattention", "dynamic_attention",
              "if_pre_sampling", "num_negative_image", "loss_type"):
        setattr(rcfg, k, getattr(cfg, k))
    return cfg, rcfg


def build_pairs(pre, rs, labels, nboxes, F, C, seed, edit=None):
    """records -> K3MPreprocessBatch.__call__ -> stacked columns -> K3MDataLoader.__iter__ collation."""
    from vilbert_k3m.datasets.concept_cap_dataset_struc import K3MDataLoader
    rng = np.random.default_rng(seed)
    recs, raw = [], []
    for i in range(len(labels)):
        items = []
        for k in range(2):
            item_id, title, _url, pv, cate = rs[2 * i + k]
            if edit:
                title, pv = edit(2 * i + k, title, pv)
            nb = nboxes[(2 * i + k) % len(nboxes)]
            h, w, boxes, f, p = regions(rng, max(nb, 1), F, C, clustered=False)
            if nb == 0:
                boxes, f, p = boxes[:0], f[:0], p[:0]
            items.append((item_id, title, pv, cate, h, w, nb, boxes, f, p))
        raw.append(items)
        recs.append((labels[i],) + items[0] + items[1])
    outs = [pre(r) for r in recs]
    cols = {n: np.stack([o[j] for o in outs]) for j, n in enumerate(PAIR_FIELDS)}
    res = {}
    for k in (1, 2):
        f, l, m = K3MDataLoader.post_process(None, cols["input_ids_%d" % k], cols["num_boxes_%d" % k],
                                             cols["image_feat_%d" % k], cols["image_loc_%d" % k],
                                             cols["image_mask_%d" % k])
        cols["coll_image_feat_%d" % k], cols["coll_image_loc_%d" % k], cols["coll_image_mask_%d" % k] = f, l, m
    cols["labels"] = cols["label"].astype(np.float32)
    R = pre.max_region_len
    for k in (1, 2):
        res["in/caption_%d" % k] = np.array([it[k - 1][1] for it in raw])
        res["in/pv_%d" % k] = np.array([it[k - 1][2] for it in raw])
        res["in/item_id_%d" % k] = np.array([it[k - 1][0] for it in raw])
        res["in/image_hw_%d" % k] = np.array([[it[k - 1][4], it[k - 1][5]] for it in raw], np.float64)
        res["in/num_boxes_%d" % k] = np.array([it[k - 1][6] for it in raw], np.int64)
        bx = np.zeros((len(raw), R, 4), np.float32)
        fe = np.zeros((len(raw), R, F), np.float32)
        tg = np.zeros((len(raw), R, C), np.float32)
        for b, it in enumerate(raw):
            n = it[k - 1][6]
            bx[b, :n], fe[b, :n], tg[b, :n] = it[k - 1][7], it[k - 1][8], it[k - 1][9]
        res["in/boxes_%d" % k], res["in/feat_%d" % k], res["in/target_%d" % k] = bx, fe, tg
    res["in/label"] = np.array(labels, np.int64)
    for n, v in cols.items():
        if n.startswith("item_id"):
            continue
        res["out/" + n] = np.asarray(v)
    return res, cols


def data_case():
    from vilbert_k3m.datasets.concept_cap_dataset_struc import K3MPreprocessBatch
    F, C = 64, 40
    pre = K3MPreprocessBatch(CharTokenizer(), max_seq_len=16, max_seq_len_pv=24, max_num_pv=3, max_region_len=10,
                             v_feature_size=F, v_target_size=C)

    def edit(i, title, pv):
        if i < len(PV_EDGE):
            pv = PV_EDGE[i]
        return title, pv
    rs = rows()[100:112]
    res, _ = build_pairs(pre, rs, [1, 0, 1, 0, 1, 0], [10, 3, 0, 7, 1, 10], F, C, seed=77, edit=edit)
    res["cfg/max_seq_len"], res["cfg/max_seq_len_pv"], res["cfg/max_num_pv"] = np.array(16), np.array(24), np.array(3)
    res["cfg/max_region_len"], res["cfg/v_feature_size"], res["cfg/v_target_size"] = np.array(10), np.array(F), np.array(C)
    path = os.path.join(HERE, "golden_ft_data.npz")
    np.savez_compressed(path, **res)
    print("data ->", path, os.path.getsize(path) // 1024, "KiB")


def model_case(name, loss_type, mode, row0, labels, weight_seed, noise_seed, T=36, P=128, NPV=20):
    import vilbert_k3m.vilbert_k3m as K
    from vilbert_k3m.datasets.concept_cap_dataset_struc import K3MPreprocessBatch
    from k3m_amd.weights import param_values
    cfg, rcfg = ref_cfg(loss_type, mode)
    pre = K3MPreprocessBatch(CharTokenizer(), max_seq_len=T, max_seq_len_pv=P, max_num_pv=NPV, max_region_len=36)
    B = len(labels)
    res, cols = build_pairs(pre, rows()[row0:row0 + 2 * B], labels, [36, 20, 9, 36], 2048, 1601, seed=row0)
    torch.manual_seed(0)
    model = K.K3MForItemAlignment(rcfg)
    vals = param_values(cfg, weight_seed)
    sd = {k: torch.from_numpy(v) for k, v in vals.items()}
    missing, unexpected = model.load_state_dict(sd, strict=True), None
    model.eval()
    shapes = [("v", (B, 37, 3, 1024)), ("t", (B, T, 3, 768)), ("pv", (B, P, 3, 768))]
    n1 = {k: torch.from_numpy(v) for k, v in gumbel_noise(noise_seed, shapes).items()}
    n2 = {k: torch.from_numpy(v) for k, v in gumbel_noise(noise_seed + 1, shapes).items()}
    calls = []

    def fake_gumbel(logits, tau=1.0, hard=False, eps=1e-10, dim=-1):
        L = logits.shape[1]
        key = "v" if logits.shape[-1] == 1024 else ("t" if L == T else "pv")
        nz = n1 if len(calls) < 3 else n2
        calls.append(key)
        y = ((logits + nz[key]) / tau).softmax(dim)
        idx = y.max(dim, keepdim=True)[1]
        hardv = torch.zeros_like(logits).scatter_(dim, idx, 1.0)
        return hardv - y.detach() + y

    K.F.gumbel_softmax = fake_gumbel
    tb = lambda k: torch.from_numpy(np.ascontiguousarray(cols[k]))  # noqa: E731
    args = [tb("labels")]
    for k in (1, 2):
        args += [tb("input_ids_%d" % k), tb("segment_ids_%d" % k), tb("input_mask_%d" % k), tb("input_ids_pv_%d" % k),
                 tb("segment_ids_pv_%d" % k), tb("input_mask_pv_%d" % k), tb("index_p_%d" % k), tb("index_v_%d" % k),
                 tb("coll_image_feat_%d" % k), tb("coll_image_loc_%d" % k), tb("coll_image_mask_%d" % k)]
    e1, e2, probs, loss = model(*args)
    loss.backward()
    assert calls == ["v", "t", "pv", "v", "t", "pv"] or mode != 1, calls
    res["out/e1"], res["out/e2"] = e1.detach().numpy(), e2.detach().numpy()
    res["out/probs"], res["out/loss"] = probs.detach().numpy(), np.array(float(loss))
    res["noise_seed"], res["weight_seed"] = np.array(noise_seed), np.array(weight_seed)
    res["mode"], res["loss_type"] = np.array(mode), np.array(loss_type)
    gn_names, gn = [], []
    for n, p in model.named_parameters():
        gn_names.append(n)
        gn.append(np.nan if p.grad is None else float(p.grad.double().norm()))
    res["grad_norm_names"] = np.array(gn_names)
    res["grad_norms"] = np.array(gn, np.float64)
    params = dict(model.named_parameters())
    for n in ["struc_w2.weight", "struc_w3.bias", "map_bi_to_individual.bias", "embeddings.LayerNorm.weight",
              "encoder.layer.11.output.dense.bias", "encoder.c_layer_pv_t.5.biOutput.dense2.bias",
              "v_embeddings.LayerNorm.bias"] + (["classifier.out_proj.weight", "classifier.out_proj.bias",
                                                  "classifier.dense.bias"] if loss_type == "ce" else []):
        g = params[n].grad
        res["grad_full/" + n] = np.zeros(tuple(params[n].shape), np.float32) if g is None else g.numpy()
    # the model fixture keeps only what the model consumes (the preprocessing is pinned by golden_ft_data)
    res = {k: v for k, v in res.items() if not k.startswith("in/")
           and not re.match(r"out/image_(feat|target|loc|mask)_\d", k)}
    path = os.path.join(HERE, "golden_ft_%s.npz" % name)
    np.savez_compressed(path, **res)
    print(name, "loss", float(loss), "->", path, os.path.getsize(path) // 1024, "KiB")


def inventory():
    import vilbert_k3m.vilbert_k3m as K
    out = {}
    for lt in ("ce", "cosine"):
        _, rcfg = ref_cfg(lt, 1)
        m = K.K3MForItemAlignment(rcfg)
        out[lt] = [[n, list(p.shape)] for n, p in m.named_parameters()]
        out[lt + "_state_dict_keys"] = list(m.state_dict().keys())
    path = os.path.join(HERE, "param_inventory_finetune.json")
    json.dump(out, open(path, "w"))
    print("inventory ->", path, {k: len(v) for k, v in out.items()})


if __name__ == "__main__":
    _stub_imports()
    torch.set_num_threads(8)
    inventory()
    data_case()
    model_case("ce", "ce", 1, row0=140, labels=[1, 0], weight_seed=31, noise_seed=5)
    model_case("cosine", "cosine", 0, row0=150, labels=[0, 1], weight_seed=32, noise_seed=6)
