"""The driver-facing pretraining loaders: ``ConceptCapLoaderTrain_struc`` / ``ConceptCapLoaderVal_struc``
(vilbert_k3m/datasets/concept_cap_dataset_struc.py:297-530) with the constructor the driver calls
(train_concap_struc.py:315-348, including ``local_rank=``, which the reference constructor rejects)
and the same iterator contract: each item is ``(16 tensors ..., index_p, index_v, item_id)``
(dataset:413), the 16 tensors in the driver's unpacking order (train_concap_struc.py:477-479).

MI355X-first: records are preprocessed by the native ``BertPreprocessBatch`` (k3m_amd/data.py,
libk3m_data.so) and collated on the GPU (``RegionCollator``), so the 16 tensors are already device
tensors when ``device`` is a GPU (the driver's ``.cuda(non_blocking=True)`` is then a no-op), and
the labelled-row counts ride along on the label tensors (``_k3m_n_labels``) so the model's
forward needs no device->host sync for its head buffers.

Record sources (``os.path.join(corpus_path, file_name)``):

* a record directory written by ``write_records`` — the 10 fields of the reference's LMDB rows
  (data_prepare.py:365: item_id, title, pvs, cate, image_h, image_w, num_boxes, boxes, features,
  cls_prob) as plain ``.npy`` arrays, memory-mapped (nothing is unpickled);
* a raw product TSV (data/README.md: id, title, image url, KG, category; e.g.
  data/raw_multidata_of_product_preatrain.small_train): the KG string is normalised as
  data_prepare.py:333-336 does ('#' removed, trailing ';'), and each item gets the record
  data_prepare.py:340-345 writes for an item without an image (one 800x800 box, zero features and
  class probabilities) — or seeded synthetic regions with ``synthetic_regions=seed``;
* ``records=``: any iterable of 10-field records.

The tensorpack LMDB container itself is not read (its storage engine is outside the hot path;
convert with ``write_records``).
"""
import os
import random

import numpy as np

from .data import BertPreprocessBatch, RandomStreams, RegionCollator

FIELDS = ("item_id", "title", "pvs", "cate", "image_h", "image_w", "num_boxes", "boxes", "features", "cls_prob")


def write_records(path, records, max_boxes=36, v_feature_size=2048, v_target_size=1601):
    """Store 10-field records (data_prepare.py:365) as a memory-mappable directory of .npy files."""
    recs = list(records)
    n = len(recs)
    os.makedirs(path, exist_ok=True)
    ids = np.array([str(r[0]) for r in recs])
    np.save(os.path.join(path, "item_id.npy"), ids)
    np.save(os.path.join(path, "title.npy"), np.array([str(r[1]) for r in recs]))
    np.save(os.path.join(path, "pvs.npy"), np.array([str(r[2]) for r in recs]))
    np.save(os.path.join(path, "cate.npy"), np.array([str(r[3]) for r in recs]))
    np.save(os.path.join(path, "image_hw.npy"), np.array([[float(r[4]), float(r[5])] for r in recs], np.float64))
    nb = np.array([int(r[6]) for r in recs], np.int32)
    np.save(os.path.join(path, "num_boxes.npy"), nb)
    boxes = np.zeros((n, max_boxes, 4), np.float32)
    feats = np.lib.format.open_memmap(os.path.join(path, "features.npy"), "w+", np.float32, (n, max_boxes, v_feature_size))
    probs = np.lib.format.open_memmap(os.path.join(path, "cls_prob.npy"), "w+", np.float32, (n, max_boxes, v_target_size))
    for i, r in enumerate(recs):
        k = int(r[6])
        if k > max_boxes:
            raise ValueError("record %d has %d boxes > %d" % (i, k, max_boxes))
        if k:
            boxes[i, :k] = np.asarray(r[7], np.float32).reshape(k, 4)
            feats[i, :k] = np.asarray(r[8], np.float32).reshape(k, v_feature_size)
            probs[i, :k] = np.asarray(r[9], np.float32).reshape(k, v_target_size)
    np.save(os.path.join(path, "boxes.npy"), boxes)
    feats.flush()
    probs.flush()
    del feats, probs


class CharTokenizer(object):
    """Offline stand-in for BertTokenizer(bert-base-chinese) when no vocab.txt exists: one id per
    character (whitespace skipped, '#' removed), the KG separators on the ids the reference
    hard-codes (':' -> 131, ';' -> 132; dataset:785-840), [CLS] 101 / [SEP] 102 / [MASK] 103.  The
    golden fixtures (tests/golden/make_golden.py) were recorded with the same mapping."""
    mask_token = "[MASK]"

    def encode(self, text):
        out = []
        for ch in text.replace("#", ""):
            if ch == ":":
                out.append(131)
            elif ch == ";":
                out.append(132)
            elif ch.isspace():
                continue
            else:
                out.append(200 + (ord(ch) * 7919) % (21128 - 200))
        return out

    def convert_tokens_to_ids(self, tok):
        return {"[MASK]": 103, "[CLS]": 101, "[SEP]": 102, "[PAD]": 0}[tok]

    def add_special_tokens_single_sentence(self, ids):
        return [101] + list(ids) + [102]

    def __len__(self):
        return 21128


class RecordDir(object):
    """Random access to a write_records directory (features memory-mapped)."""

    def __init__(self, path):
        ld = lambda f, mm=None: np.load(os.path.join(path, f + ".npy"), mmap_mode=mm, allow_pickle=False)
        self.item_id, self.title, self.pvs, self.cate = ld("item_id"), ld("title"), ld("pvs"), ld("cate")
        self.hw, self.nb, self.boxes = ld("image_hw"), ld("num_boxes"), ld("boxes")
        self.feat, self.prob = ld("features", "r"), ld("cls_prob", "r")

    def __len__(self):
        return len(self.item_id)

    def __getitem__(self, i):
        k = int(self.nb[i])
        return (str(self.item_id[i]), str(self.title[i]), str(self.pvs[i]), str(self.cate[i]), float(self.hw[i, 0]),
                float(self.hw[i, 1]), k, self.boxes[i, :k], self.feat[i, :k], self.prob[i, :k])


def _no_image_region(v_feature_size, v_target_size):
    # data_prepare.py:340-345: the record of an item whose image is missing
    h = w = 800
    return (h, w, 1, np.array([[0.1, 0.1, w - 0.1, h - 0.1]], np.float32), np.zeros((1, v_feature_size), np.float32),
            np.zeros((1, v_target_size), np.float32))


def _synthetic_region(rng, nbox, v_feature_size, v_target_size):
    h, w = 600.0, 800.0
    x1 = rng.uniform(0, w * 0.7, nbox)
    y1 = rng.uniform(0, h * 0.7, nbox)
    x2 = np.minimum(w, x1 + rng.uniform(20, w * 0.3, nbox))
    y2 = np.minimum(h, y1 + rng.uniform(20, h * 0.3, nbox))
    boxes = np.stack([x1, y1, x2, y2], 1).astype(np.float32)
    f = np.abs(rng.standard_normal((nbox, v_feature_size))).astype(np.float32) * 0.5
    lg = rng.standard_normal((nbox, v_target_size)).astype(np.float32) * 2
    p = np.exp(lg - lg.max(1, keepdims=True))
    return h, w, nbox, boxes, f, (p / p.sum(1, keepdims=True)).astype(np.float32)


def read_raw_tsv(path, v_feature_size=2048, v_target_size=1601, synthetic_regions=None, nbox=36):
    """Records from a raw product TSV (data/README.md)."""
    rng = np.random.default_rng(synthetic_regions) if synthetic_regions is not None else None
    out = []
    with open(path, encoding="utf-8") as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) < 4:
                continue
            item_id, title, _url, pvs = parts[:4]
            cate = parts[4] if len(parts) > 4 else ""
            pvs = pvs.replace("#", "")
            if not pvs.endswith(";"):
                pvs += ";"
            reg = (_synthetic_region(rng, nbox, v_feature_size, v_target_size) if rng is not None
                   else _no_image_region(v_feature_size, v_target_size))
            out.append((item_id, title, pvs, cate) + reg)
    return out


def open_records(corpus_path, file_name, **kw):
    path = os.path.join(corpus_path, file_name) if corpus_path else file_name
    if os.path.isdir(path) and os.path.exists(os.path.join(path, "item_id.npy")):
        return RecordDir(path)
    if os.path.isfile(path):
        with open(path, "rb") as f:
            head = f.read(4096)
        if b"\t" in head:
            return read_raw_tsv(path, **kw)
    raise NotImplementedError(
        "%s: not a k3m record directory (k3m_amd.loaders.write_records) or a raw product TSV; the tensorpack "
        "LMDB container is not read by this build — convert its records with write_records" % path)


def _device_of(device, local_rank):
    import torch
    if device is not None:
        return torch.device(device)
    if torch.cuda.is_available():
        return torch.device("cuda", max(0, int(local_rank)) % max(1, torch.cuda.device_count()))
    raise RuntimeError("the K3M loaders collate on the GPU (no CPU fallback)")


class _LoaderBase(object):
    def __init__(self, corpus_path, file_name, tokenizer, max_seq_len=32, max_seq_len_pv=32, max_num_pv=20,
                 max_region_len=36, v_feature_size=2048, v_target_size=1601, v_loc_size=5, visual_target=0,
                 batch_size=512, objective=0, visualization=False, shuffle=True, seed=None, device=None,
                 local_rank=-1, records=None, synthetic_regions=None):
        self.records = records if records is not None else open_records(
            corpus_path, file_name, v_feature_size=v_feature_size, v_target_size=v_target_size,
            synthetic_regions=synthetic_regions)
        self.num_dataset = len(self.records)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self._order_rng = random.Random(seed)
        self.pre = BertPreprocessBatch(tokenizer, max_seq_len=max_seq_len, max_seq_len_pv=max_seq_len_pv,
                                       max_num_pv=max_num_pv, max_region_len=max_region_len,
                                       v_feature_size=v_feature_size, v_target_size=v_target_size,
                                       v_loc_size=v_loc_size, visual_target=visual_target, visualization=visualization,
                                       objective=objective, streams=RandomStreams(0 if seed is None else seed))
        self.collate = RegionCollator(_device_of(device, local_rank), max_region_len, v_feature_size, v_target_size,
                                      visual_target)

    def __len__(self):
        return (self.num_dataset + self.batch_size - 1) // self.batch_size

    def batches(self):
        """(batch dict for k3m_amd.engine, item ids) per batch — the engine-facing form."""
        order = list(range(self.num_dataset))
        if self.shuffle:
            self._order_rng.shuffle(order)
        for s in range(0, len(order), self.batch_size):
            yield self.collate([self.pre.prepare(self.records[i]) for i in order[s:s + self.batch_size]])

    def __iter__(self):
        for batch, ids in self.batches():
            n_m, n_v = batch.pop("_label_counts")
            # the head-buffer sizes travel with the label tensors (read by the model's forward)
            batch["lm_label_ids"]._k3m_n_labels = n_m
            batch["image_label"]._k3m_n_labels = n_v
            t = tuple(batch[k] for k in ("input_ids", "input_mask", "segment_ids", "lm_label_ids", "is_next",
                                         "input_ids_pv", "input_mask_pv", "segment_ids_pv", "lm_label_ids_pv",
                                         "is_next_pv_v", "is_next_pv_t", "image_feat", "image_loc", "image_target",
                                         "image_label", "image_mask"))
            index_p, index_v = batch.pop("_index_host")   # built on the host by the collator: no sync
            yield t + (index_p, index_v, ids)


class ConceptCapLoaderTrain_struc(_LoaderBase):
    """Drop-in for the reference training loader (dataset:297-416); shuffles every epoch
    (LMDBSerializer.load(shuffle=True), :350).  ``rank`` / ``local_rank`` pick the device; like the
    reference, every rank reads the whole corpus (no sharding, :340-343) with its own order."""

    def __init__(self, corpus_path, file_name, tokenizer, max_seq_len=32, max_seq_len_pv=32, max_num_pv=20,
                 max_region_len=36, v_feature_size=2048, v_target_size=1601, v_loc_size=5, visual_target=0,
                 batch_size=512, num_workers=25, cache=10000, rank=-1, local_rank=-1, objective=0,
                 visualization=False, serializer=None, seed=None, device=None, records=None, synthetic_regions=None):
        super(ConceptCapLoaderTrain_struc, self).__init__(
            corpus_path, file_name, tokenizer, max_seq_len, max_seq_len_pv, max_num_pv, max_region_len,
            v_feature_size, v_target_size, v_loc_size, visual_target, batch_size, objective, visualization,
            shuffle=True, seed=seed, device=device, local_rank=local_rank if local_rank != -1 else rank,
            records=records, synthetic_regions=synthetic_regions)
        self.num_workers, self.cache = num_workers, cache


class ConceptCapLoaderVal_struc(_LoaderBase):
    """Drop-in for the reference validation loader (dataset:419-530): fixed order."""

    def __init__(self, corpus_path, file_name, tokenizer, max_seq_len=32, max_seq_len_pv=32, max_num_pv=20,
                 max_region_len=36, v_feature_size=2048, v_target_size=1601, v_loc_size=5, visual_target=0,
                 batch_size=512, objective=0, visualization=False, serializer=None, seed=None, device=None,
                 local_rank=-1, records=None, synthetic_regions=None):
        super(ConceptCapLoaderVal_struc, self).__init__(
            corpus_path, file_name, tokenizer, max_seq_len, max_seq_len_pv, max_num_pv, max_region_len,
            v_feature_size, v_target_size, v_loc_size, visual_target, batch_size, objective, visualization,
            shuffle=False, seed=seed, device=device, local_rank=local_rank, records=records,
            synthetic_regions=synthetic_regions)
