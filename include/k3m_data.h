/* libk3m_data — native host side of the K3M data path: the per-sample
 * preprocessing of BertPreprocessBatch (vilbert_k3m/datasets/concept_cap_dataset_struc.py:532-933)
 * in C++, with random streams that reproduce the reference's Python `random` and numpy legacy
 * `np.random` draws bit for bit, so a seeded run masks exactly the tokens and regions the reference
 * masks.  The heavy region-feature collation runs on the GPU (k3m_collate_regions, k3m_hip.h).
 *
 * Conventions: plain host pointers and sizes, int status (0 ok, 1 bad argument), no allocation,
 * no global state (every random stream is a caller-owned K3mRng).
 */
#ifndef K3M_DATA_H
#define K3M_DATA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MT19937 state (624 words + position), shared by both seeding conventions. */
typedef struct K3mRng {
  uint32_t mt[624];
  int32_t mti;
} K3mRng;

/* random.seed(n) of CPython (init_by_array over the 32-bit words of |n|). */
void k3m_rng_seed_python(K3mRng* r, uint64_t seed);
/* np.random.seed(n) of numpy's legacy RandomState (init_genrand(n), 0 <= n < 2^32). */
void k3m_rng_seed_numpy(K3mRng* r, uint32_t seed);
uint32_t k3m_rng_uint32(K3mRng* r);
/* random.random(): 53-bit double in [0, 1). */
double k3m_rng_random(K3mRng* r);
/* np.random.randint(high) (legacy masked rejection on 32-bit draws), 0 <= result < high <= 2^32. */
int64_t k3m_rng_randint_numpy(K3mRng* r, int64_t high);

/* Title text of one sample (BertPreprocessBatch.convert_example_to_features, dataset:650-700 with
 * mask_word :763-783): truncate the token ids to max_len-2, mask 15% of them (80% -> mask_id,
 * 10% -> np.random.randint(vocab), 10% kept; one py draw per token, an np draw for the 10% case),
 * add [CLS]=cls_id ... [SEP]=sep_id, pad to max_len.  Outputs are int64 [max_len].  visualization != 0
 * keeps the draws but masks nothing (the reference's visualization flag).  py == NULL: no draws and
 * no masking (the fine-tuning K3MPreprocessBatch, dataset:1035-1038; np_rng may then be NULL). */
int k3m_prep_text(const int32_t* tok, int ntok, int max_len, int mask_id, int cls_id, int sep_id, int vocab,
                  int visualization, K3mRng* py, K3mRng* np_rng, int64_t* input_ids, int64_t* input_mask, int64_t* segment_ids,
                  int64_t* lm_label_ids);

/* Property-value text of one sample (mask_word_pv :815-840, index_pv :785-813): truncate to
 * max_len-2, mask every value token of triples 2..n (':'=colon_id ... ';'=semi_id) when
 * mask_values != 0 (pretraining; 0 for fine-tuning, dataset:1036), add [CLS]/[SEP], pad;
 * index_p/index_v int64 [max_num_pv][2] ([begin, ':' pos], [':' pos + 1, ';' pos]), padded with
 * [0, 0].  Deterministic. */
int k3m_prep_pv(const int32_t* tok, int ntok, int max_len, int max_num_pv, int mask_values, int mask_id, int cls_id,
                int sep_id, int colon_id, int semi_id, int64_t* input_ids, int64_t* input_mask, int64_t* segment_ids,
                int64_t* lm_label_ids, int64_t* index_p, int64_t* index_v);

/* Regions of one sample (__call__ :575-610 + mask_region :898-933): box IoU, location
 * normalisation [x1/w, y1/h, x2/w, y2/h, area/(w h)] (fp32, reference op order), 15% of the boxes
 * masked (one py draw per box; 90% of them get their features zeroed: zero_feat[i] = 1), the
 * masked boxes and every box overlapping one by IoU > 0.4 flagged in masked_label (they leave the
 * global-region mean).  num_boxes <= 0 takes the reference's default box.  Outputs over
 * max_region rows: image_loc fp32 [max_region][5], image_label / image_mask int64, zero_feat /
 * masked_label uint8.  The effective num_boxes is returned through nb_out.  py == NULL: no region
 * masking (K3MPreprocessBatch.image_processing, dataset:1180-1216). */
int k3m_prep_regions(const float* boxes, int num_boxes, float image_h, float image_w, int max_region,
                     int visualization, K3mRng* py,
                     float* image_loc, int64_t* image_label, int64_t* image_mask, uint8_t* zero_feat,
                     uint8_t* masked_label, int* nb_out);

#ifdef __cplusplus
}
#endif

#endif
