"""Parameter inventory of ``BertForMultiModalPreTraining_tri_stru`` and its flat HBM layout.

The names, shapes and order reproduce ``named_parameters()`` of the reference model
(module registration order: vilbert_k3m.py:2190-2264; per-module layouts :335-1152, :1753-1924,
:2141-2161), so ``state_dict()`` files interchange (999 keys incl. the tied
``cls.predictions.decoder.weight``).

MI355X layout: every parameter is a view into ONE contiguous fp32 buffer (``FlatParams``), and so
is every gradient (a second buffer of the same size).  Consequences:

* fused projections are free views: ``query|key|value`` (and the three fusion-gate scorers)
  are stored back to back, so the QKV weight is one ``[3H, H]`` matrix and the QKV GEMM is one
  launch;
* the optimizer is ONE elementwise AdamW launch per weight-decay segment over the buffer;
* gradient buckets for the RCCL all-reduce are contiguous slices of the gradient buffer.

Segments, in buffer order: ``decay`` (weight decay 0.01), ``no_decay`` (0.0; names containing
"bias" / "LayerNorm.bias" / "LayerNorm.weight" — train_concap_struc.py:244, :352-367) and
``frozen`` (the 86 tensors that never receive a gradient because their outputs are unused:
``q_dense{1,2}`` :976-984/:1007-1015, the poolers :2620-2631, ``seq_relationship`` whose NSP loss
is excluded from the total (train_concap_struc.py:533), ``map_individual_to_bi`` and ``soft_*``
:2223-2250).  ``pytorch_transformers.AdamW`` skips parameters whose ``.grad`` is None, so the
frozen segment is never touched by the optimizer — exactly the reference's behaviour.
"""
import re

NO_DECAY = ("bias", "LayerNorm.bias", "LayerNorm.weight")


def _lin(prefix, out_f, in_f, bias=True):
    r = [(prefix + ".weight", (out_f, in_f))]
    if bias:
        r.append((prefix + ".bias", (out_f,)))
    return r


def _ln(prefix, n):
    return [(prefix + ".weight", (n,)), (prefix + ".bias", (n,))]


def _bert_layer(p, H, I):
    return (_lin(p + ".attention.self.query", H, H) + _lin(p + ".attention.self.key", H, H)
            + _lin(p + ".attention.self.value", H, H) + _lin(p + ".attention.output.dense", H, H)
            + _ln(p + ".attention.output.LayerNorm", H) + _lin(p + ".intermediate.dense", I, H)
            + _lin(p + ".output.dense", H, I) + _ln(p + ".output.LayerNorm", H))


def _conn_layer(p, H1, H2, Hb, I1, I2):
    """BertConnectionLayer (stream1 width H1, stream2 width H2, bi width Hb)."""
    s = []
    s += _lin(p + ".biattention.query1", Hb, H1) + _lin(p + ".biattention.key1", Hb, H1)
    s += _lin(p + ".biattention.value1", Hb, H1)
    s += _lin(p + ".biattention.query2", Hb, H2) + _lin(p + ".biattention.key2", Hb, H2)
    s += _lin(p + ".biattention.value2", Hb, H2)
    s += _lin(p + ".biOutput.dense1", H1, Hb) + _ln(p + ".biOutput.LayerNorm1", H1)
    s += _lin(p + ".biOutput.q_dense1", H1, Hb)
    s += _lin(p + ".biOutput.dense2", H2, Hb) + _ln(p + ".biOutput.LayerNorm2", H2)
    s += _lin(p + ".biOutput.q_dense2", H2, Hb)
    s += _lin(p + ".v_intermediate.dense", I1, H1) + _lin(p + ".v_output.dense", H1, I1)
    s += _ln(p + ".v_output.LayerNorm", H1)
    s += _lin(p + ".t_intermediate.dense", I2, H2) + _lin(p + ".t_output.dense", H2, I2)
    s += _ln(p + ".t_output.LayerNorm", H2)
    return s


def param_spec(cfg):
    """Ordered [(name, shape)] exactly as the reference ``named_parameters()``; ``cfg.task``
    selects the model: "pretrain" (BertForMultiModalPreTraining_tri_stru, default) or
    "item_alignment" (K3MForItemAlignment, vilbert_k3m.py:2862-2950)."""
    if getattr(cfg, "task", "pretrain") == "item_alignment":
        return item_alignment_spec(cfg)
    H, I, V = cfg.hidden_size, cfg.intermediate_size, cfg.vocab_size
    Hv, Iv, Hb = cfg.v_hidden_size, cfg.v_intermediate_size, cfg.bi_hidden_size
    use_image = getattr(cfg, "use_image", True)
    nco = len(cfg.v_biattention_id)
    s = [("embeddings.word_embeddings.weight", (V, H)),
         ("embeddings.position_embeddings.weight", (cfg.max_position_embeddings, H)),
         ("embeddings.token_type_embeddings.weight", (cfg.type_vocab_size, H))]
    s += _ln("embeddings.LayerNorm", H)
    for i in range(cfg.num_hidden_layers):
        s += _bert_layer("encoder.layer.%d" % i, H, I)
    if use_image:
        for i in range(cfg.v_num_hidden_layers):
            s += _bert_layer("encoder.v_layer.%d" % i, Hv, Iv)
    if cfg.with_coattention:
        if use_image:
            for i in range(nco):
                s += _conn_layer("encoder.c_layer.%d" % i, Hv, H, Hb, Iv, I)
            for i in range(nco):
                s += _conn_layer("encoder.c_layer_pv_v.%d" % i, Hv, H, Hb, Iv, I)
        for i in range(nco):
            s += _conn_layer("encoder.c_layer_pv_t.%d" % i, H, H, H, I, I)
    s += _lin("t_pooler.dense", Hb, H)
    if use_image:
        s += _lin("v_embeddings.image_embeddings", Hv, cfg.v_feature_size)
        s += _lin("v_embeddings.image_location_embeddings", Hv, 5)
        s += _ln("v_embeddings.LayerNorm", Hv)
        s += _lin("v_pooler.dense", Hb, Hv)
    # own parameters precede sub-module parameters in named_parameters()
    s += [("cls.predictions.bias", (V,))]
    s += _lin("cls.predictions.transform.dense", H, H)
    s += _ln("cls.predictions.transform.LayerNorm", H)
    s += _lin("cls.seq_relationship", 2, H)
    if use_image:
        s += _lin("cls.imagePredictions.transform.dense", Hv, Hv)
        s += _ln("cls.imagePredictions.transform.LayerNorm", Hv)
        s += _lin("cls.imagePredictions.decoder", cfg.v_target_size, Hv)
        s += _lin("map_individual_to_bi", Hb, H)
        s += _lin("map_bi_to_individual", H, Hb)
        for n in ("score_self_v", "score_cross1_v", "score_cross2_v", "soft_v"):
            s += _lin(n, Hb, 3 * Hb)
    nm = 3 if use_image else 2
    for n in ("score_self_t", "score_cross1_t", "score_cross2_t", "soft_t",
              "score_self_pv", "score_cross1_pv", "score_cross2_pv", "soft_pv"):
        s += _lin(n, H, nm * H)
    s += _lin("struc_w1", H, 3 * H) + _lin("struc_w2", 1, H) + _lin("struc_w3", H, H)
    return s


def _encoder_spec(cfg):
    H, I = cfg.hidden_size, cfg.intermediate_size
    Hv, Iv, Hb = cfg.v_hidden_size, cfg.v_intermediate_size, cfg.bi_hidden_size
    nco = len(cfg.v_biattention_id)
    s = []
    for i in range(cfg.num_hidden_layers):
        s += _bert_layer("encoder.layer.%d" % i, H, I)
    for i in range(cfg.v_num_hidden_layers):
        s += _bert_layer("encoder.v_layer.%d" % i, Hv, Iv)
    if cfg.with_coattention:
        for i in range(nco):
            s += _conn_layer("encoder.c_layer.%d" % i, Hv, H, Hb, Iv, I)
        for i in range(nco):
            s += _conn_layer("encoder.c_layer_pv_v.%d" % i, Hv, H, Hb, Iv, I)
        for i in range(nco):
            s += _conn_layer("encoder.c_layer_pv_t.%d" % i, H, H, H, I, I)
    return s


def item_alignment_spec(cfg):
    """K3MForItemAlignment.named_parameters() (vilbert_k3m.py:2866-2950, use_image=True): module
    registration order embeddings, v_embeddings, v_pooler, encoder, t_pooler, the fusion maps and
    gates, classifier (loss_type "ce": ClassificationHead :2164-2183), struc_w1..3."""
    if not getattr(cfg, "use_image", True):
        raise NotImplementedError("item alignment without the image modality (use_image=False)")
    H, V = cfg.hidden_size, cfg.vocab_size
    Hv, Hb = cfg.v_hidden_size, cfg.bi_hidden_size
    s = [("embeddings.word_embeddings.weight", (V, H)),
         ("embeddings.position_embeddings.weight", (cfg.max_position_embeddings, H)),
         ("embeddings.token_type_embeddings.weight", (cfg.type_vocab_size, H))]
    s += _ln("embeddings.LayerNorm", H)
    s += _lin("v_embeddings.image_embeddings", Hv, cfg.v_feature_size)
    s += _lin("v_embeddings.image_location_embeddings", Hv, 5)
    s += _ln("v_embeddings.LayerNorm", Hv)
    s += _lin("v_pooler.dense", Hb, Hv)
    s += _encoder_spec(cfg)
    s += _lin("t_pooler.dense", Hb, H)
    s += _lin("map_individual_to_bi", Hb, H)
    s += _lin("map_bi_to_individual", H, Hb)
    for n in ("score_self_v", "score_cross1_v", "score_cross2_v", "soft_v"):
        s += _lin(n, Hb, 3 * Hb)
    for n in ("score_self_t", "score_cross1_t", "score_cross2_t", "soft_t",
              "score_self_pv", "score_cross1_pv", "score_cross2_pv", "soft_pv"):
        s += _lin(n, H, 3 * H)
    if getattr(cfg, "loss_type", "ce") == "ce":
        s += _lin("classifier.dense", H, 2 * H) + _lin("classifier.out_proj", 2, H)
    s += _lin("struc_w1", H, 3 * H) + _lin("struc_w2", 1, H) + _lin("struc_w3", H, H)
    return s


_FROZEN_RE = re.compile(r"(\.q_dense[12]\.|^t_pooler\.|^v_pooler\.|^cls\.seq_relationship\.|"
                        r"^map_individual_to_bi\.|^soft_(v|t|pv)\.)")


def is_frozen(name):
    """True for the tensors that never get a gradient in the pretraining step (and, the same set
    minus the absent NSP head, in the item-alignment step: its poolers, q_dense*,
    map_individual_to_bi and soft_* outputs are unused too, vilbert_k3m.py:3183-3376)."""
    return bool(_FROZEN_RE.search(name))


def is_no_decay(name):
    return any(nd in name for nd in NO_DECAY)


def segment_of(name):
    if is_frozen(name):
        return "frozen"
    return "no_decay" if is_no_decay(name) else "decay"


# Groups of parameters that must be adjacent in the flat buffer so that the fused operand is a
# single contiguous view.  Each entry: list of names in physical order (weights and biases are
# adjacent separately).
def fused_groups(cfg):
    groups = []
    qkv = ("query", "key", "value")

    def add(prefix, subs):
        groups.append([prefix + s + ".weight" for s in subs])
        groups.append([prefix + s + ".bias" for s in subs])

    for i in range(cfg.num_hidden_layers):
        add("encoder.layer.%d.attention.self." % i, qkv)
    if getattr(cfg, "use_image", True):
        for i in range(cfg.v_num_hidden_layers):
            add("encoder.v_layer.%d.attention.self." % i, qkv)
    if cfg.with_coattention:
        kinds = (["c_layer", "c_layer_pv_v"] if getattr(cfg, "use_image", True) else []) + ["c_layer_pv_t"]
        for k in kinds:
            for i in range(len(cfg.v_biattention_id)):
                add("encoder.%s.%d.biattention." % (k, i), ("query1", "key1", "value1"))
                add("encoder.%s.%d.biattention." % (k, i), ("query2", "key2", "value2"))
    mods = (["v"] if getattr(cfg, "use_image", True) else []) + ["t", "pv"]
    for m in mods:
        add("", ["score_self_%s" % m, "score_cross1_%s" % m, "score_cross2_%s" % m])
    return groups


def flat_layout(cfg, align=64):
    """Return (spec, offsets, seg_bounds, total).

    ``offsets[name]`` is the element offset in the flat buffer; members of a fused group are
    contiguous; each segment starts on an ``align``-element boundary; every tensor starts on a
    4-element (16-byte) boundary so vector loads stay aligned (fused-group members keep exact
    adjacency — all their sizes are multiples of 4).
    """
    spec = param_spec(cfg)
    shapes = dict(spec)
    numel = {n: int(_prod(s)) for n, s in spec}
    group_of = {}
    for g in fused_groups(cfg):
        for n in g:
            group_of[n] = g
    offsets = {}
    seg_bounds = {}
    pos = 0
    for seg in ("decay", "no_decay", "frozen"):
        pos = (pos + align - 1) // align * align
        start = pos
        for n, _ in spec:
            if segment_of(n) != seg or n in offsets:
                continue
            members = group_of.get(n, [n])
            for m in members:
                assert segment_of(m) == seg, (m, seg)
                pos = (pos + 3) // 4 * 4
                offsets[m] = pos
                pos += numel[m]
        seg_bounds[seg] = (start, pos)
    total = (pos + align - 1) // align * align
    assert len(offsets) == len(spec)
    return spec, offsets, seg_bounds, total, shapes


def _prod(s):
    p = 1
    for x in s:
        p *= x
    return p
