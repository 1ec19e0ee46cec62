"""K3M pretraining data path: the per-sample preprocessing of
``BertPreprocessBatch`` (vilbert_k3m/datasets/concept_cap_dataset_struc.py:532-933) and the batch
collation of ``ConceptCapLoaderTrain_struc.__iter__`` (:372-410), re-homed for MI355X:

* per sample, on the host: tokenisation by the caller's tokenizer (as the reference), then
  truncation, word masking, property-value masking/indexing, box IoU, location normalisation and
  region masking in C++ (libk3m_data.so, include/k3m_data.h) with random streams that reproduce
  the reference's Python ``random`` and numpy legacy ``np.random`` draws bit for bit;
* per batch, on the GPU: the feature rows (the only bulky data: 36 x 2048 fp32 per sample) are
  copied to HBM once, raw; masked rows are zeroed and the global-region mean row is prepended by
  one HBM-bound kernel (k3m_collate_regions, include/k3m_hip.h), bit-identical to the reference's
  numpy.

The reference draws from the process-global ``random`` / ``np.random``; here the two streams are an
explicit ``RandomStreams`` object.  ``RandomStreams(seed)`` is the state after
``random.seed(seed); np.random.seed(seed)``.

There is no Python fallback: the native libraries must be built (``python -m k3m_amd.build_lib``).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
DATA_LIB_PATH = os.path.join(HERE, "libk3m_data.so")


class K3mRng(C.Structure):
    _fields_ = [("mt", C.c_uint32 * 624), ("mti", C.c_int32)]


_vp, _i32, _i64, _f32 = C.c_void_p, C.c_int32, C.c_int64, C.c_float
_R = C.POINTER(K3mRng)
DATA_SIGNATURES = {
    "k3m_rng_seed_python": (None, [_R, C.c_uint64]),
    "k3m_rng_seed_numpy": (None, [_R, C.c_uint32]),
    "k3m_rng_uint32": (C.c_uint32, [_R]),
    "k3m_rng_random": (C.c_double, [_R]),
    "k3m_rng_randint_numpy": (C.c_int64, [_R, C.c_int64]),
    "k3m_prep_text": (C.c_int, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _R, _R, _vp, _vp, _vp, _vp]),
    "k3m_prep_pv": (C.c_int, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp,
                              _vp]),
    "k3m_prep_regions": (C.c_int, [_vp, _i32, _f32, _f32, _i32, _i32, _R, _vp, _vp, _vp, _vp, _vp, _vp]),
}

_dl = None


def load_data_lib(path=DATA_LIB_PATH):
    global _dl
    if _dl is not None:
        return _dl
    if not os.path.exists(path):
        raise RuntimeError("libk3m_data.so not found at %s — build it with `python -m k3m_amd.build_lib`" % path)
    lib = C.CDLL(path)
    for name, (res, args) in DATA_SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _dl = lib
    return lib


def data_exported_symbols(path=DATA_LIB_PATH):
    lib = C.CDLL(path)
    return [n for n in DATA_SIGNATURES if hasattr(lib, n)]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class RandomStreams(object):
    """The reference's two random streams as owned MT19937 states: ``py`` (Python ``random``:
    mask_word / mask_region draws) and ``np`` (numpy legacy ``np.random``: random replacement
    tokens)."""

    def __init__(self, seed=None, np_seed=None):
        self.py = K3mRng()
        self.np = K3mRng()
        self.seed(0 if seed is None else seed, np_seed)

    def seed(self, seed, np_seed=None):
        dl = load_data_lib()
        seed = abs(int(seed))          # random.seed(int) seeds with |n|
        if seed >= 1 << 64:
            raise ValueError("seeds must be below 2**64")
        np_seed = seed if np_seed is None else int(np_seed)
        if not 0 <= np_seed < 1 << 32:
            raise ValueError("np.random.seed must be between 0 and 2**32 - 1")
        dl.k3m_rng_seed_python(C.byref(self.py), seed)
        dl.k3m_rng_seed_numpy(C.byref(self.np), np_seed)

    def random(self):
        """random.random()"""
        return load_data_lib().k3m_rng_random(C.byref(self.py))

    def randint(self, high):
        """np.random.randint(high)"""
        return load_data_lib().k3m_rng_randint_numpy(C.byref(self.np), int(high))


class PreparedSample(object):
    """One preprocessed record, features not yet masked (zero_feat marks the rows the reference
    zeroes) so the batch collation can do it on the GPU."""
    __slots__ = ("item_id", "text", "pv", "index_p", "index_v", "image_loc", "image_label", "image_mask",
                 "zero_feat", "masked_label", "num_boxes", "feat", "target")


class BertPreprocessBatch(object):
    """Drop-in for the reference's ``BertPreprocessBatch`` (dataset:532-933): same constructor
    arguments, ``__call__(data)`` returns the same 20-tuple of numpy arrays for a record
    ``(item_id, caption, pv, category, image_h, image_w, num_boxes, boxes, features, targets)``.
    ``streams`` replaces the process-global random state (default: a RandomStreams(0))."""

    def __init__(self, tokenizer, max_seq_len=32, max_seq_len_pv=32, max_num_pv=20, max_region_len=36,
                 v_feature_size=2048, v_target_size=1601, v_loc_size=5, visual_target=0, visualization=False,
                 objective=0, streams=None):
        if v_loc_size != 5:
            raise ValueError("v_loc_size must be 5 (the reference's location layout)")
        self.max_seq_len = max_seq_len
        self.max_seq_len_pv = max_seq_len_pv
        self.max_num_pv = max_num_pv
        self.max_region_len = max_region_len
        self.v_feature_size = v_feature_size
        self.v_target_size = v_target_size
        self.v_loc_size = v_loc_size
        self.visual_target = visual_target
        self.visualization = bool(visualization)
        self.objective = objective
        self.tokenizer = tokenizer
        self.streams = streams if streams is not None else RandomStreams(0)
        self.mask_id = int(tokenizer.convert_tokens_to_ids(tokenizer.mask_token))
        sp = list(tokenizer.add_special_tokens_single_sentence([]))
        if len(sp) != 2:
            raise ValueError("tokenizer must wrap a sentence as [CLS] ids [SEP]")
        self.cls_id, self.sep_id = int(sp[0]), int(sp[1])
        self.vocab = len(tokenizer)
        self._dl = load_data_lib()

    # -- per-record work ------------------------------------------------------------------------
    def prepare(self, data):
        """Everything of __call__ except writing the masked feature rows: returns a PreparedSample."""
        item_id, caption, pv, _category, image_h, image_w, num_boxes, boxes, feats, targets = data
        dl, R = self._dl, self.max_region_len
        s = PreparedSample()
        s.item_id = item_id
        # text first, then regions: the order of the reference's random draws (:666-716)
        tok = np.ascontiguousarray(self.tokenizer.encode(caption), dtype=np.int32)
        T = self.max_seq_len
        out = np.empty((4, T), np.int64)
        rc = dl.k3m_prep_text(_p(tok), tok.size, T, self.mask_id, self.cls_id, self.sep_id, self.vocab,
                              int(self.visualization), C.byref(self.streams.py), C.byref(self.streams.np),
                              _p(out[0]), _p(out[1]), _p(out[2]), _p(out[3]))
        if rc:
            raise ValueError("k3m_prep_text: bad arguments")
        s.text = out
        tokp = np.ascontiguousarray(self.tokenizer.encode(pv), dtype=np.int32)
        P, NPV = self.max_seq_len_pv, self.max_num_pv
        outp = np.empty((4, P), np.int64)
        ip = np.empty((NPV, 2), np.int64)
        iv = np.empty((NPV, 2), np.int64)
        rc = dl.k3m_prep_pv(_p(tokp), tokp.size, P, NPV, 1, self.mask_id, self.cls_id, self.sep_id, 131, 132,
                            _p(outp[0]), _p(outp[1]), _p(outp[2]), _p(outp[3]), _p(ip), _p(iv))
        if rc:
            raise ValueError("k3m_prep_pv: bad arguments")
        s.pv, s.index_p, s.index_v = outp, ip, iv

        nb = int(num_boxes)
        if nb > R:
            raise ValueError("num_boxes %d exceeds max_region_len %d" % (nb, R))
        bx = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 4) if nb > 0 else np.zeros((0, 4), np.float32)
        if nb > 0 and bx.shape[0] != nb:
            raise ValueError("boxes hold %d rows for num_boxes %d" % (bx.shape[0], nb))
        s.image_loc = np.empty((R, 5), np.float32)
        s.image_label = np.empty(R, np.int64)
        s.image_mask = np.empty(R, np.int64)
        s.zero_feat = np.empty(R, np.uint8)
        s.masked_label = np.empty(R, np.uint8)
        nbo = C.c_int(0)
        rc = dl.k3m_prep_regions(_p(bx), nb, float(image_h), float(image_w), R, int(self.visualization),
                                 C.byref(self.streams.py), _p(s.image_loc), _p(s.image_label), _p(s.image_mask),
                                 _p(s.zero_feat), _p(s.masked_label), C.byref(nbo))
        if rc:
            raise ValueError("k3m_prep_regions: bad arguments")
        s.num_boxes = nbo.value
        if nb > 0:
            s.feat = np.asarray(feats, dtype=np.float32).reshape(nb, self.v_feature_size)
            s.target = np.asarray(targets, dtype=np.float32).reshape(nb, self.v_target_size)
        else:   # the reference's default region has zero features and targets (:578-583)
            s.feat = np.zeros((1, self.v_feature_size), np.float32)
            s.target = np.zeros((1, self.v_target_size), np.float32)
        return s

    def __call__(self, data):
        """The reference's 20-tuple (dataset:623-648), masked feature rows zeroed on the host."""
        s = self.prepare(data)
        R, nb = self.max_region_len, s.num_boxes
        feat = np.zeros((R, self.v_feature_size), np.float32)
        feat[:nb] = s.feat
        if self.visual_target == 0:
            target = np.zeros((R, self.v_target_size), np.float32)
            target[:nb] = s.target
        else:
            target = feat.copy()
        feat[s.zero_feat.astype(bool)] = 0
        ml = s.masked_label.astype(bool) if s.masked_label.any() else np.zeros(R)
        z = np.array(0)
        return (s.item_id, s.text[0], s.text[1], s.text[2], s.text[3], z, s.pv[0], s.pv[1], s.pv[2], s.pv[3],
                z.copy(), z.copy(), s.index_p, s.index_v, feat, s.image_loc, target, s.image_label, s.image_mask, ml)


class RegionCollator(object):
    """Batch collation of ConceptCapLoaderTrain_struc.__iter__ (dataset:372-410) with the feature
    work on the GPU: returns the driver's batch dict (the 16 tensors + index_p / index_v, the names
    k3m_amd.engine consumes) on ``device`` plus the item ids."""

    def __init__(self, device, max_region_len=36, v_feature_size=2048, v_target_size=1601, visual_target=0):
        import torch
        self.torch = torch
        self.device = torch.device(device)
        self.R, self.F, self.Ct = max_region_len, v_feature_size, v_target_size
        self.visual_target = visual_target
        if self.F % 4:
            raise ValueError("v_feature_size must be a multiple of 4")
        self._stage = None
        self._copied = None

    def _staging(self, B):
        t = self.torch
        if self._copied is not None:
            # the previous batch's host->device copies read this staging buffer: they must have
            # landed before it is overwritten (a loader running ahead of the GPU would otherwise
            # hand the previous batch the next batch's features)
            self._copied.synchronize()
            self._copied = None
        if self._stage is None or self._stage[0].shape[0] < B:
            pin = self.device.type == "cuda"
            ct = self.F if self.visual_target else self.Ct
            self._stage = (t.empty((B, self.R, self.F), dtype=t.float32, pin_memory=pin),
                           t.empty((B, self.R, ct), dtype=t.float32, pin_memory=pin))
        return self._stage[0][:B], self._stage[1][:B]

    def __call__(self, samples):
        from . import _lib
        t = self.torch
        B, R, F = len(samples), self.R, self.F
        feat_h, tgt_h = self._staging(B)
        fh, th = feat_h.numpy(), tgt_h.numpy()
        for b, s in enumerate(samples):
            nb = s.num_boxes
            fh[b, :nb] = s.feat
            fh[b, nb:] = 0
            if self.visual_target == 0:
                th[b, :nb] = s.target
                th[b, nb:] = 0
        dev = self.device
        nbk = dev.type == "cuda"
        feat_d = feat_h.to(dev, non_blocking=nbk)
        if self.visual_target:
            tgt = feat_d.clone()        # image_target = unmasked features (dataset:594-596)
        else:
            tgt = tgt_h.to(dev, non_blocking=nbk)
        if nbk:
            self._copied = t.cuda.Event()
            self._copied.record()
        zero = t.from_numpy(np.stack([s.zero_feat for s in samples])).to(dev, non_blocking=nbk)
        mlab = t.from_numpy(np.stack([s.masked_label for s in samples])).to(dev, non_blocking=nbk)
        image_feat = t.empty((B, R + 1, F), dtype=t.float32, device=dev)
        if dev.type != "cuda":
            raise RuntimeError("RegionCollator runs the collation on the GPU (no CPU fallback)")
        _lib.call("k3m_collate_regions", feat_d.data_ptr(), R * F, zero.data_ptr(), mlab.data_ptr(), None, B, R, F,
                  image_feat.data_ptr(), _lib.stream())
        loc = np.empty((B, R + 1, 5), np.float32)
        loc[:, 0] = (0, 0, 1, 1, 1)
        loc[:, 1:] = np.stack([s.image_loc for s in samples])
        imask = np.ones((B, R + 1), np.int64)
        imask[:, 1:] = np.stack([s.image_mask for s in samples])
        text = np.stack([s.text for s in samples])          # [B, 4, T]
        pv = np.stack([s.pv for s in samples])
        z = np.zeros(B, np.int64)

        def d(a):
            return t.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=nbk)

        batch = dict(input_ids=d(text[:, 0]), input_mask=d(text[:, 1]), segment_ids=d(text[:, 2]),
                     lm_label_ids=d(text[:, 3]), is_next=d(z), input_ids_pv=d(pv[:, 0]), input_mask_pv=d(pv[:, 1]),
                     segment_ids_pv=d(pv[:, 2]), lm_label_ids_pv=d(pv[:, 3]), is_next_pv_v=d(z), is_next_pv_t=d(z),
                     image_feat=image_feat, image_loc=d(loc), image_target=tgt,
                     image_label=d(np.stack([s.image_label for s in samples])), image_mask=d(imask),
                     index_p=d(np.stack([s.index_p for s in samples])),
                     index_v=d(np.stack([s.index_v for s in samples])))
        # labelled-row counts of the heads, known here on the host (engine.label_counts): the
        # forward then sizes its compacted head buffers without a device->host sync
        batch["_label_counts"] = (int((text[:, 3] >= 0).sum()) + int((pv[:, 3] >= 0).sum()),
                                  int(sum(int((s.image_label >= 1).sum()) for s in samples)))
        # host copies of the PV spans: the driver-facing iterator yields these (no device->host copy)
        batch["_index_host"] = (np.stack([s.index_p for s in samples]), np.stack([s.index_v for s in samples]))
        return batch, [s.item_id for s in samples]


class K3mPretrainLoader(object):
    """Iterator over batches of records (the role of ConceptCapLoaderTrain_struc, dataset:293-414):
    records -> BertPreprocessBatch.prepare -> RegionCollator.  ``records`` is any iterable of the
    10-field tuples the reference's LMDB rows deserialize to."""

    def __init__(self, records, tokenizer, device, batch_size=64, streams=None, **kw):
        self.records = records
        self.batch_size = batch_size
        self.pre = BertPreprocessBatch(tokenizer, streams=streams, **kw)
        self.collate = RegionCollator(device, self.pre.max_region_len, self.pre.v_feature_size,
                                      self.pre.v_target_size, self.pre.visual_target)

    def __iter__(self):
        buf = []
        for r in self.records:
            buf.append(self.pre.prepare(r))
            if len(buf) == self.batch_size:
                yield self.collate(buf)
                buf = []
        if buf:
            yield self.collate(buf)


# ------------------------------------------------------------------------------------------------
# Fine-tuning pairs: K3MPreprocessBatch (dataset:936-1263) and the
# K3MDataLoader collation (:255-292).  Nothing is masked or drawn at random; the global region is
# the sum of the region rows divided by the RAW num_boxes (0 -> inf / nan, as the reference).

PAIR_TUPLE = ["label", "item_id_1", "input_ids_1", "input_mask_1", "segment_ids_1", "input_ids_pv_1",
              "input_mask_pv_1", "segment_ids_pv_1", "index_p_1", "index_v_1", "num_boxes_1", "image_feat_1",
              "image_loc_1", "image_target_1", "image_mask_1", "item_id_2", "input_ids_2", "input_mask_2",
              "segment_ids_2", "input_ids_pv_2", "input_mask_pv_2", "segment_ids_pv_2", "index_p_2", "index_v_2",
              "num_boxes_2", "image_feat_2", "image_loc_2", "image_target_2", "image_mask_2"]


class PreparedItem(object):
    __slots__ = ("item_id", "text", "pv", "index_p", "index_v", "image_loc", "image_mask", "num_boxes", "nb", "feat",
                 "target")


class K3MPreprocessBatch(object):
    """Drop-in for the reference's fine-tuning ``K3MPreprocessBatch`` (dataset:936-1263): a record
    ``(label, item 1: item_id, caption, pv, category, image_h, image_w, num_boxes, boxes, features,
    targets, item 2: ...)`` -> the reference's 29-tuple of numpy arrays."""

    def __init__(self, tokenizer, max_seq_len=32, max_seq_len_pv=32, max_num_pv=20, max_region_len=36,
                 v_feature_size=2048, v_target_size=1601, v_loc_size=5, visual_target=0):
        if v_loc_size != 5:
            raise ValueError("v_loc_size must be 5 (the reference's location layout)")
        self.max_seq_len, self.max_seq_len_pv, self.max_num_pv = max_seq_len, max_seq_len_pv, max_num_pv
        self.max_region_len, self.v_feature_size, self.v_target_size = max_region_len, v_feature_size, v_target_size
        self.v_loc_size, self.visual_target, self.tokenizer = v_loc_size, visual_target, tokenizer
        self.mask_id = int(tokenizer.convert_tokens_to_ids(tokenizer.mask_token))
        sp = list(tokenizer.add_special_tokens_single_sentence([]))
        if len(sp) != 2:
            raise ValueError("tokenizer must wrap a sentence as [CLS] ids [SEP]")
        self.cls_id, self.sep_id = int(sp[0]), int(sp[1])
        self._dl = load_data_lib()

    def prepare_item(self, item):
        item_id, caption, pv, _category, image_h, image_w, num_boxes, boxes, feats, targets = item
        dl, R = self._dl, self.max_region_len
        s = PreparedItem()
        s.item_id = item_id
        tok = np.ascontiguousarray(self.tokenizer.encode(caption), dtype=np.int32)
        T, P, NPV = self.max_seq_len, self.max_seq_len_pv, self.max_num_pv
        s.text = np.empty((3, T), np.int64)
        lab = np.empty(T, np.int64)
        if dl.k3m_prep_text(_p(tok), tok.size, T, self.mask_id, self.cls_id, self.sep_id, 0, 0, None, None,
                            _p(s.text[0]), _p(s.text[1]), _p(s.text[2]), _p(lab)):
            raise ValueError("k3m_prep_text: bad arguments")
        tokp = np.ascontiguousarray(self.tokenizer.encode(pv), dtype=np.int32)
        s.pv = np.empty((3, P), np.int64)
        labp = np.empty(P, np.int64)
        s.index_p = np.empty((NPV, 2), np.int64)
        s.index_v = np.empty((NPV, 2), np.int64)
        if dl.k3m_prep_pv(_p(tokp), tokp.size, P, NPV, 0, self.mask_id, self.cls_id, self.sep_id, 131, 132,
                          _p(s.pv[0]), _p(s.pv[1]), _p(s.pv[2]), _p(labp), _p(s.index_p), _p(s.index_v)):
            raise ValueError("k3m_prep_pv: bad arguments")
        nb = int(num_boxes)
        if nb > R:
            raise ValueError("num_boxes %d exceeds max_region_len %d" % (nb, R))
        bx = np.ascontiguousarray(boxes, dtype=np.float32).reshape(-1, 4) if nb > 0 else np.zeros((0, 4), np.float32)
        s.image_loc = np.empty((R, 5), np.float32)
        il, im = np.empty(R, np.int64), np.empty(R, np.int64)
        zf, ml = np.empty(R, np.uint8), np.empty(R, np.uint8)
        nbo = C.c_int(0)
        if dl.k3m_prep_regions(_p(bx), nb, float(image_h), float(image_w), R, 0, None, _p(s.image_loc), _p(il),
                               _p(im), _p(zf), _p(ml), C.byref(nbo)):
            raise ValueError("k3m_prep_regions: bad arguments")
        s.num_boxes = num_boxes                      # raw, as InputExample(num_boxes=...) keeps it
        s.nb = nbo.value
        s.image_mask = (np.arange(R) < nb).astype(np.int64)   # [1] * num_boxes (raw) padded (:1148)
        if nb > 0:
            s.feat = np.asarray(feats, dtype=np.float32).reshape(nb, self.v_feature_size)
            s.target = np.asarray(targets, dtype=np.float32).reshape(nb, self.v_target_size)
        else:
            s.feat = np.zeros((1, self.v_feature_size), np.float32)
            s.target = np.zeros((1, self.v_target_size), np.float32)
        return s

    def prepare(self, data):
        return data[0], self.prepare_item(data[1:11]), self.prepare_item(data[11:21])

    def _item_tuple(self, s):
        R = self.max_region_len
        feat = np.zeros((R, self.v_feature_size), np.float32)
        feat[:s.nb] = s.feat
        if self.visual_target == 0:
            target = np.zeros((R, self.v_target_size), np.float32)
            target[:s.nb] = s.target
        else:
            target = feat.copy()
        return (s.item_id, s.text[0], s.text[1], s.text[2], s.pv[0], s.pv[1], s.pv[2], s.index_p, s.index_v,
                s.num_boxes, feat, s.image_loc, target, s.image_mask)

    def __call__(self, data):
        label, a, b = self.prepare(data)
        return (label,) + self._item_tuple(a) + self._item_tuple(b)


class PairCollator(object):
    """K3MDataLoader.__iter__ collation (dataset:255-263, post_process :265-292) with the feature
    rows collated on the GPU: returns the K3MForItemAlignment.forward arguments as a dict (plus
    image_target_1/2, as the reference's batch carries them) and the item-id lists."""

    def __init__(self, device, max_region_len=36, v_feature_size=2048, v_target_size=1601, visual_target=0):
        import torch
        self.torch = torch
        self.device = torch.device(device)
        self.R, self.F, self.Ct = max_region_len, v_feature_size, v_target_size
        self.visual_target = visual_target

    def _item(self, items):
        from . import _lib
        t = self.torch
        B, R, F = len(items), self.R, self.F
        if self.device.type != "cuda":
            raise RuntimeError("PairCollator runs the collation on the GPU (no CPU fallback)")
        pin = True
        fh = t.zeros((B, R, F), dtype=t.float32, pin_memory=pin)
        ct = F if self.visual_target else self.Ct
        th = t.zeros((B, R, ct), dtype=t.float32, pin_memory=pin)
        fn, tn = fh.numpy(), th.numpy()
        for b, s in enumerate(items):
            fn[b, :s.nb] = s.feat
            if self.visual_target == 0:
                tn[b, :s.nb] = s.target
        dev = self.device
        feat_d = fh.to(dev, non_blocking=True)
        tgt = feat_d.clone() if self.visual_target else th.to(dev, non_blocking=True)
        div = t.from_numpy(np.array([int(s.num_boxes) for s in items], np.int32)).to(dev, non_blocking=True)
        out = t.empty((B, R + 1, F), dtype=t.float32, device=dev)
        _lib.call("k3m_collate_regions", feat_d.data_ptr(), R * F, None, None, div.data_ptr(), B, R, F, out.data_ptr(),
                  _lib.stream())
        loc = np.empty((B, R + 1, 5), np.float32)
        loc[:, 0] = (0, 0, 1, 1, 1)
        loc[:, 1:] = np.stack([s.image_loc for s in items])
        mask = np.ones((B, R + 1), np.int64)
        mask[:, 1:] = np.stack([s.image_mask for s in items])
        text = np.stack([s.text for s in items])
        pv = np.stack([s.pv for s in items])

        def d(a):
            return t.from_numpy(np.ascontiguousarray(a)).to(dev, non_blocking=True)

        return dict(input_ids=d(text[:, 0]), attention_mask=d(text[:, 1]), token_type_ids=d(text[:, 2]),
                    input_ids_pv=d(pv[:, 0]), attention_mask_pv=d(pv[:, 1]), token_type_ids_pv=d(pv[:, 2]),
                    index_p=d(np.stack([s.index_p for s in items])), index_v=d(np.stack([s.index_v for s in items])),
                    image_feat=out, image_loc=d(loc), image_attention_mask=d(mask), image_target=tgt), \
            [s.item_id for s in items], (feat_d, div)

    def __call__(self, prepared):
        t = self.torch
        labels = t.tensor(np.array([float(p[0]) for p in prepared], np.float32)).to(self.device)
        out = {"labels": labels}
        ids = []
        keep = []
        for k in (1, 2):
            d, iid, hold = self._item([p[k] for p in prepared])
            out.update({"%s_%d" % (n, k): v for n, v in d.items()})
            ids.append(iid)
            keep.append(hold)
        self._hold = keep          # staging buffers stay alive until the next call
        return out, ids[0], ids[1]
