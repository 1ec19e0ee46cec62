"""CPU restatement of the data path's batch collation — TEST INFRASTRUCTURE ONLY (imported by
tests/ and bench cpu_baseline legs, never by the product path).

collate_regions follows ConceptCapLoaderTrain_struc.__iter__
(vilbert_k3m/datasets/concept_cap_dataset_struc.py:381-397) plus mask_region's feature zeroing
(:913-915).  Pinned against the reference's own outputs in tests/golden/golden_data.npz
(make_data_golden.py runs the reference's BertPreprocessBatch and collation).
"""
import numpy as np


def collate_regions(feat, zero_feat, masked_label):
    """feat fp32 [B][R][F] (raw), zero_feat / masked_label [B][R] -> (image_feat [B][R+1][F],
    the collated location prefix [0,0,1,1,1] is added by the caller)."""
    f = np.array(feat, dtype=np.float32, copy=True)
    f[np.asarray(zero_feat).astype(bool)] = 0                       # image_feat[i] = 0 (:913-915)
    cnt = np.sum(np.asarray(masked_label) == 0, axis=1, keepdims=True)   # :383-384
    cnt[cnt == 0] = 1
    g = np.sum(f, axis=1) / cnt                                         # fp32 sum, float64 divide
    return np.array(np.concatenate([np.expand_dims(g, 1), f], 1), dtype=np.float32)


def collate_locations(image_loc, image_mask):
    """image_loc [B][R][5], image_mask [B][R] -> the loader's [B][R+1] forms (:389-397)."""
    B = image_loc.shape[0]
    gl = np.repeat(np.array([[0, 0, 1, 1, 1]], dtype=np.float32), B, axis=0)
    loc = np.array(np.concatenate([np.expand_dims(gl, 1), image_loc], 1), dtype=np.float32)
    mask = np.concatenate([np.repeat(np.array([[1]]), B, axis=0), image_mask], 1)
    return loc, mask


def collate_pair_item(feat, num_boxes, image_loc, image_mask):
    """K3MDataLoader.post_process (dataset:265-292): global row = sum of the region rows / RAW
    num_boxes (no zero guard), location prefix [0,0,1,1,1], mask prefix 1."""
    cnt = np.expand_dims(np.asarray(num_boxes), 1)
    with np.errstate(divide="ignore", invalid="ignore"):
        g = np.sum(feat, axis=1) / cnt
    f = np.array(np.concatenate([np.expand_dims(g, 1), feat], 1), dtype=np.float32)
    loc, mask = collate_locations(image_loc, image_mask)
    return f, loc, mask
