"""Debug mode ("HIP_LAUNCH_BLOCKING / AMD_SERIALIZE_KERNEL debug mode; bounds-checked debug build").

K3M_DEBUG=1 (or ``set_debug(True)``) turns on, for every library call:
* serialized launches: ``_lib.call`` waits for the device after each entry point, so an asynchronous fault or a
  non-finite result is attributed to the call that caused it, not to a later synchronisation;
* bounds checks of every data-dependent index before the kernel that uses it runs: token / segment ids against the
  embedding tables, label ids against the classifier widths (-1 = ignore, as the reference's CrossEntropyLoss
  ``ignore_index=-1``, vilbert_k3m.py:2271), structure triples against the PV sequence (index_p / index_v,
  :2441-2444), LPM negatives against the batch and the item's pairs, and the row indices of gather / scatter.
  The reference's own failure on such input is torch's "index out of range" (nn.Embedding, :2141) -- here an
  IndexError naming the field, the offending value and the bound, raised on the host before any kernel reads the
  index, so a bad batch never reaches a GPU memory access.

Release runs (the default) pay nothing: every check is behind ``ON``.
"""
import os

import torch

ON = os.environ.get("K3M_DEBUG", "0") not in ("", "0")


def set_debug(on=True):
    global ON
    ON = bool(on)


class K3mIndexError(IndexError):
    pass


def check_range(t, lo, hi, what, ignore=None):
    """Every element of t in [lo, hi) (or equal to ``ignore``); raises K3mIndexError otherwise."""
    if t is None or t.numel() == 0:
        return
    x = t.detach()
    if ignore is not None:
        x = x[x != ignore]
        if x.numel() == 0:
            return
    mn, mx = int(x.min()), int(x.max())
    if mn < lo or mx >= hi:
        bad = mn if mn < lo else mx
        raise K3mIndexError("%s: index %d out of range [%d, %d)%s" % (
            what, bad, lo, hi, "" if ignore is None else " (ignore value %d)" % ignore))


def check_len(n, limit, what):
    """A sequence length against the position table (position ids 0 .. n-1)."""
    if n > limit:
        raise K3mIndexError("%s %d exceeds max_position_embeddings %d" % (what, n, limit))


def check_batch(batch, cfg, ent_neg=None, val_neg=None):
    """The reference input contract of one step's batch, checked before the forward."""
    V, TV = cfg.vocab_size, cfg.type_vocab_size
    check_range(batch.get("input_ids"), 0, V, "input_ids")
    check_range(batch.get("input_ids_pv"), 0, V, "input_ids_pv")
    check_range(batch.get("segment_ids"), 0, TV, "segment_ids")
    check_range(batch.get("segment_ids_pv"), 0, TV, "segment_ids_pv")
    check_range(batch.get("lm_label_ids"), 0, V, "lm_label_ids", ignore=-1)
    check_range(batch.get("lm_label_ids_pv"), 0, V, "lm_label_ids_pv", ignore=-1)
    for k in ("is_next", "is_next_pv_v", "is_next_pv_t"):
        check_range(batch.get(k), 0, 2, k, ignore=-1)
    ids = batch.get("input_ids")
    if ids is not None and ids.dim() == 2:
        check_len(ids.shape[1], cfg.max_position_embeddings, "text length")
    pv = batch.get("input_ids_pv")
    if pv is not None and pv.dim() == 2:
        P = pv.shape[1]
        check_len(P, cfg.max_position_embeddings, "PV length")
        check_range(batch.get("index_p"), 0, P, "index_p")
        check_range(batch.get("index_v"), 0, P, "index_v")
        B = pv.shape[0]
        ip = batch.get("index_p")
        npv = ip.shape[1] if ip is not None and ip.dim() >= 2 else None
        # negatives: entity ones name another item of the batch, value ones another pair of the same item (< 0: none)
        if ent_neg is not None:
            check_range(ent_neg[ent_neg >= 0], 0, B, "ent_neg")
        if val_neg is not None and npv is not None:
            check_range(val_neg[val_neg >= 0], 0, npv, "val_neg")
            check_val_neg(ip, val_neg)


def item_triples(index_p):
    """Per-item triple count: triples stop at the first j with index_p[i, j, 0] == 0 (vilbert_k3m.py:2441; the
    rule of struct.hip count_valid)."""
    z = (index_p[..., 0] == 0)
    npv = index_p.shape[1]
    first = torch.where(z.any(dim=1), z.int().argmax(dim=1), torch.full_like(z[:, 0], npv, dtype=torch.int64))
    return first


def check_val_neg(index_p, val_neg):
    """A value negative of pair (i, j) names another pair of the SAME item, so it must be below that item's own triple
    count, not only below the padded width: a negative pointing at a padding pair would make LPM read an unset row
    (the reference samples from range(len(property_vecs[i])), vilbert_k3m.py:2489-2494).  Only the pairs LPM
    scores (j < n) are checked."""
    if index_p is None or val_neg.numel() == 0:
        return
    n = item_triples(index_p.detach().to(val_neg.device)).view(-1, 1, 1)   # [B, 1, 1]
    j = torch.arange(val_neg.shape[1], device=val_neg.device).view(1, -1, 1)
    scored = (j < n) & (val_neg >= 0)
    bad = scored & (val_neg >= n)
    if bool(bad.any()):
        i, jj, e = [int(x) for x in bad.nonzero()[0]]
        raise K3mIndexError("val_neg: index %d of item %d pair %d out of range [0, %d) (the item's triple count)"
                            % (int(val_neg[i, jj, e]), i, jj, int(n.view(-1)[i])))


def sync(name):
    """Serialized-launch mode: wait for the call's kernels; a device fault surfaces here, naming the call."""
    try:
        torch.cuda.synchronize()
    except RuntimeError as e:
        raise RuntimeError("%s: device error after the call (K3M_DEBUG serialized mode): %s" % (name, e)) from e
