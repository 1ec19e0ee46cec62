"""Seeded synthetic pretraining batches with the reference's input contract (SURVEY.md §8(a) A0,
§8(d)); generated directly in HBM.

Token / index layout mirrors BertPreprocessBatch (vilbert_k3m/datasets/concept_cap_dataset_struc.py
:654-747): [CLS]=101 ... [SEP]=102, PV triples "p p : v v ;" (':'=131, ';'=132) from position 1,
index_p = [begin, ':' pos], index_v = [':'+1, ';' pos] (index_pv :785-813), value tokens of
triples 2..n masked with [MASK]=103 and labelled (mask_word_pv :815-840); the image rows get the
global region first (row 0 = mean feature, loc [0,0,1,1,1]; dataset:381-397).
"""
import torch


def synthetic_batch(cfg, batch_size, device, seed=1234, T=36, P=128, n_boxes=36, n_triples=10, npv=20):
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    B = batch_size
    V = cfg.vocab_size
    R = n_boxes + 1
    ids = torch.randint(200, V, (B, T), generator=g)
    ids[:, 0] = 101
    ids[:, -1] = 102
    lm = torch.full((B, T), -1, dtype=torch.int64)
    pick = torch.rand((B, T), generator=g) < 0.15
    pick[:, 0] = False
    pick[:, -1] = False
    pick[torch.arange(B), torch.randint(1, T - 1, (B,), generator=g)] = True   # >= 1 label per item
    lm[pick] = ids[pick]
    ids = torch.where(pick, torch.full_like(ids, 103), ids)

    pids = torch.zeros((B, P), dtype=torch.int64)
    pmask = torch.zeros((B, P), dtype=torch.int64)
    lmp = torch.full((B, P), -1, dtype=torch.int64)
    index_p = torch.zeros((B, npv, 2), dtype=torch.int64)
    index_v = torch.zeros((B, npv, 2), dtype=torch.int64)
    toks = torch.randint(200, V, (B, n_triples, 4), generator=g)
    pids[:, 0] = 101
    for j in range(n_triples):
        s = 1 + 6 * j
        pids[:, s] = toks[:, j, 0]
        pids[:, s + 1] = toks[:, j, 1]
        pids[:, s + 2] = 131
        pids[:, s + 3] = toks[:, j, 2]
        pids[:, s + 4] = toks[:, j, 3]
        pids[:, s + 5] = 132
        index_p[:, j, 0], index_p[:, j, 1] = s, s + 2
        index_v[:, j, 0], index_v[:, j, 1] = s + 3, s + 5
        if j >= 1:
            lmp[:, s + 3] = pids[:, s + 3]
            lmp[:, s + 4] = pids[:, s + 4]
            pids[:, s + 3] = 103
            pids[:, s + 4] = 103
    end = 1 + 6 * n_triples
    pids[:, end] = 102
    pmask[:, :end + 1] = 1

    feat = torch.randn((B, n_boxes, cfg.v_feature_size), generator=g).abs()
    feat = torch.cat([feat.mean(1, keepdim=True), feat], 1)
    xy = torch.rand((B, n_boxes, 2, 2), generator=g).sort(dim=2).values
    x1, x2 = xy[:, :, 0, 0], xy[:, :, 1, 0]
    y1, y2 = xy[:, :, 0, 1], xy[:, :, 1, 1]
    loc = torch.stack([x1, y1, x2, y2, (x2 - x1) * (y2 - y1)], 2)
    loc = torch.cat([torch.tensor([0.0, 0.0, 1.0, 1.0, 1.0]).expand(B, 1, 5), loc], 1)
    tgt = torch.softmax(torch.randn((B, n_boxes, cfg.v_target_size), generator=g), -1)
    lab = torch.full((B, n_boxes), -1, dtype=torch.int64)
    pk = torch.rand((B, n_boxes), generator=g) < 0.15
    pk[torch.arange(B), torch.randint(0, n_boxes, (B,), generator=g)] = True
    lab[pk] = 1
    z = torch.zeros((B,), dtype=torch.int64)
    batch = dict(
        input_ids=ids, input_mask=torch.ones((B, T), dtype=torch.int64), segment_ids=torch.zeros((B, T), dtype=torch.int64),
        lm_label_ids=lm, is_next=z, input_ids_pv=pids, input_mask_pv=pmask,
        segment_ids_pv=torch.zeros((B, P), dtype=torch.int64), lm_label_ids_pv=lmp, is_next_pv_v=z.clone(),
        is_next_pv_t=z.clone(), image_feat=feat.float(), image_loc=loc.float(), image_target=tgt.float(),
        image_label=lab, image_mask=torch.ones((B, R), dtype=torch.int64), index_p=index_p, index_v=index_v)
    return {k: v.contiguous().to(device) for k, v in batch.items()}


def synthetic_noise(cfg, batch_size, seed=0, T=36, P=128, R=37):
    """Explicit gumbel noise (for deterministic comparisons)."""
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    out = {}
    for k, L, D in (("v", R, cfg.bi_hidden_size), ("t", T, cfg.hidden_size), ("pv", P, cfg.hidden_size)):
        e = torch.empty((batch_size, L, 3, D)).exponential_(generator=g)
        out[k] = -e.log()
    return out
