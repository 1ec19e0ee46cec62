// Native host side of the K3M data path: BertPreprocessBatch (concept_cap_dataset_struc.py:532-933)
// per-sample work with reference-exact random streams.  Built with -ffp-contract=off so every fp32
// expression rounds exactly like the numpy float32 array expression it restates.
#include <cmath>
#include <cstring>

#include "../../include/k3m_data.h"

namespace {

constexpr int N = 624, M = 397;
constexpr uint32_t MATRIX_A = 0x9908b0dfu, UPPER = 0x80000000u, LOWER = 0x7fffffffu;

void init_genrand(K3mRng* r, uint32_t s) {
  r->mt[0] = s;
  for (int i = 1; i < N; ++i) r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
  r->mti = N;
}

// MT19937 init_by_array (Matsumoto & Nishimura 2002), as CPython's random_seed uses it
void init_by_array(K3mRng* r, const uint32_t* key, int klen) {
  init_genrand(r, 19650218u);
  int i = 1, j = 0;
  for (int k = (N > klen ? N : klen); k; --k) {
    r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    ++i;
    ++j;
    if (i >= N) {
      r->mt[0] = r->mt[N - 1];
      i = 1;
    }
    if (j >= klen) j = 0;
  }
  for (int k = N - 1; k; --k) {
    r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    ++i;
    if (i >= N) {
      r->mt[0] = r->mt[N - 1];
      i = 1;
    }
  }
  r->mt[0] = 0x80000000u;
  r->mti = N;
}

// IoU of two boxes with the +1 pixel convention of iou() (dataset:40-77), numpy float32 op order
float box_iou(const float* a, const float* b) {
  const float area_b = (b[2] - b[0] + 1.0f) * (b[3] - b[1] + 1.0f);
  const float area_a = (a[2] - a[0] + 1.0f) * (a[3] - a[1] + 1.0f);
  float iw = std::fmin(a[2], b[2]) - std::fmax(a[0], b[0]) + 1.0f;
  if (iw < 0.0f) iw = 0.0f;
  float ih = std::fmin(a[3], b[3]) - std::fmax(a[1], b[1]) + 1.0f;
  if (ih < 0.0f) ih = 0.0f;
  const float inter = iw * ih;
  const float ua = area_a + area_b - inter;
  return inter / ua;
}

}  // namespace

extern "C" {

void k3m_rng_seed_python(K3mRng* r, uint64_t seed) {
  uint32_t key[2] = {(uint32_t)(seed & 0xffffffffu), (uint32_t)(seed >> 32)};
  init_by_array(r, key, key[1] ? 2 : 1);
}

void k3m_rng_seed_numpy(K3mRng* r, uint32_t seed) { init_genrand(r, seed); }

uint32_t k3m_rng_uint32(K3mRng* r) {
  static const uint32_t mag01[2] = {0u, MATRIX_A};
  if (r->mti >= N) {
    int kk = 0;
    for (; kk < N - M; ++kk) {
      const uint32_t y = (r->mt[kk] & UPPER) | (r->mt[kk + 1] & LOWER);
      r->mt[kk] = r->mt[kk + M] ^ (y >> 1) ^ mag01[y & 1u];
    }
    for (; kk < N - 1; ++kk) {
      const uint32_t y = (r->mt[kk] & UPPER) | (r->mt[kk + 1] & LOWER);
      r->mt[kk] = r->mt[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 1u];
    }
    const uint32_t y = (r->mt[N - 1] & UPPER) | (r->mt[0] & LOWER);
    r->mt[N - 1] = r->mt[M - 1] ^ (y >> 1) ^ mag01[y & 1u];
    r->mti = 0;
  }
  uint32_t y = r->mt[r->mti++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

double k3m_rng_random(K3mRng* r) {
  const uint32_t a = k3m_rng_uint32(r) >> 5, b = k3m_rng_uint32(r) >> 6;
  return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
}

int64_t k3m_rng_randint_numpy(K3mRng* r, int64_t high) {
  if (high <= 1) return 0;
  const uint64_t rng = (uint64_t)(high - 1);
  uint64_t mask = rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t v;
  while ((v = k3m_rng_uint32(r) & (uint32_t)mask) > rng) {
  }
  return (int64_t)v;
}

int k3m_prep_text(const int32_t* tok, int ntok, int max_len, int mask_id, int cls_id, int sep_id, int vocab,
                  int visualization, K3mRng* py, K3mRng* np_rng, int64_t* input_ids, int64_t* input_mask, int64_t* segment_ids,
                  int64_t* lm_label_ids) {
  if (max_len < 2 || ntok < 0 || (ntok > 0 && !tok) || (py && !np_rng)) return 1;
  const int n = ntok < max_len - 2 ? ntok : max_len - 2;   // _truncate_seq_pair (:741-753)
  input_ids[0] = cls_id;
  lm_label_ids[0] = -1;
  for (int i = 0; i < n; ++i) {                            // mask_word (:763-783)
    const int32_t t = tok[i];
    int64_t out = t, lab = -1;
    double prob = py ? k3m_rng_random(py) : 1.0;   // no stream: no masking (K3MPreprocessBatch)
    if (prob < 0.15 && !visualization) {
      prob /= 0.15;
      if (prob < 0.8) out = mask_id;
      else if (prob < 0.9) out = k3m_rng_randint_numpy(np_rng, vocab);
      lab = t;
    }
    input_ids[1 + i] = out;
    lm_label_ids[1 + i] = lab;
  }
  input_ids[1 + n] = sep_id;
  lm_label_ids[1 + n] = -1;
  for (int i = 0; i < max_len; ++i) {
    input_mask[i] = i < n + 2 ? 1 : 0;
    segment_ids[i] = 0;
    if (i >= n + 2) {
      input_ids[i] = 0;
      lm_label_ids[i] = -1;
    }
  }
  return 0;
}

int k3m_prep_pv(const int32_t* tok, int ntok, int max_len, int max_num_pv, int mask_values, int mask_id, int cls_id,
                int sep_id, int colon_id, int semi_id, int64_t* input_ids, int64_t* input_mask, int64_t* segment_ids,
                int64_t* lm_label_ids, int64_t* index_p, int64_t* index_v) {
  if (max_len < 2 || max_len > 4096 || ntok < 0 || (ntok > 0 && !tok) || max_num_pv < 0) return 1;
  const int n = ntok < max_len - 2 ? ntok : max_len - 2;
  // mask_word_pv (:815-840) on the truncated tokens
  int i131[4096], i132[4096], n131 = 0, n132 = 0;
  for (int i = 0; i < n; ++i) {
    if (tok[i] == colon_id) i131[n131++] = i;
    if (tok[i] == semi_id) i132[n132++] = i;
  }
  if (n132 == n131 - 1) i132[n132++] = n;
  int off = 0;
  if (n132 > 1) off = 1;   // values of triples 2..n (with <= 1 triple the first one is masked)
  for (int i = 0; i < n; ++i) {
    input_ids[1 + i] = tok[i];
    lm_label_ids[1 + i] = -1;
  }
  const int npair = !mask_values ? 0 : (n131 - off) < (n132 - off) ? (n131 - off) : (n132 - off);
  for (int p = 0; p < npair; ++p) {
    const int beg = i131[p + off], end = i132[p + off];
    for (int i = beg + 1; i < end; ++i) {
      lm_label_ids[1 + i] = input_ids[1 + i];   // in place, as the reference (overlapping ranges)
      input_ids[1 + i] = mask_id;
    }
  }
  input_ids[0] = cls_id;
  lm_label_ids[0] = -1;
  input_ids[1 + n] = sep_id;
  lm_label_ids[1 + n] = -1;
  // index_pv (:785-813) on [CLS] + tokens + [SEP]
  n131 = n132 = 0;
  for (int i = 0; i < n + 2; ++i) {
    if (input_ids[i] == colon_id) i131[n131++] = i;
    if (input_ids[i] == semi_id) i132[n132++] = i;
  }
  if (n132 == n131) {
  } else if (n132 == n131 - 1) {
    --n131;
  } else {
    n131 = n132 = 0;
  }
  int npv = 0, begin = 1;
  const int np2 = n131 < n132 ? n131 : n132;
  for (int p = 0; p < np2 && npv < max_num_pv; ++p) {
    index_p[2 * npv] = begin;
    index_p[2 * npv + 1] = i131[p];
    index_v[2 * npv] = i131[p] + 1;
    index_v[2 * npv + 1] = i132[p];
    begin = i132[p] + 1;
    ++npv;
  }
  for (int p = npv; p < max_num_pv; ++p) index_p[2 * p] = index_p[2 * p + 1] = index_v[2 * p] = index_v[2 * p + 1] = 0;
  for (int i = 0; i < max_len; ++i) {
    input_mask[i] = i < n + 2 ? 1 : 0;
    segment_ids[i] = 0;
    if (i >= n + 2) {
      input_ids[i] = 0;
      lm_label_ids[i] = -1;
    }
  }
  return 0;
}

int k3m_prep_regions(const float* boxes, int num_boxes, float image_h, float image_w, int max_region,
                     int visualization, K3mRng* py,
                     float* image_loc, int64_t* image_label, int64_t* image_mask, uint8_t* zero_feat,
                     uint8_t* masked_label, int* nb_out) {
  if (max_region <= 0 || (num_boxes > 0 && !boxes) || num_boxes > max_region) return 1;
  const float defbox[4] = {0.1f, 0.1f, (float)(800.0 - 0.1), (float)(800.0 - 0.1)};
  const float* b = boxes;
  int nb = num_boxes;
  double h = image_h, w = image_w;
  if (nb <= 0) {   // no boxes: the reference's default region (:578-583)
    h = 800.0;
    w = 800.0;
    nb = 1;
    b = defbox;
  }
  const float fw = (float)w, fh = (float)h, fwh = (float)(w * h);
  for (int i = 0; i < max_region; ++i) {
    float x0 = 0.f, y0 = 0.f, x1 = 0.f, y1 = 0.f;
    if (i < nb) {
      x0 = b[4 * i];
      y0 = b[4 * i + 1];
      x1 = b[4 * i + 2];
      y1 = b[4 * i + 3];
    }
    image_loc[5 * i + 4] = (y1 - y0) * (x1 - x0) / fwh;
    image_loc[5 * i + 0] = x0 / fw;
    image_loc[5 * i + 1] = y0 / fh;
    image_loc[5 * i + 2] = x1 / fw;
    image_loc[5 * i + 3] = y1 / fh;
    zero_feat[i] = 0;
    masked_label[i] = 0;
    image_label[i] = -1;
    image_mask[i] = i < nb ? 1 : 0;
  }
  for (int i = 0; py && i < nb; ++i) {   // mask_region (:898-933); no stream: no masking
    double prob = k3m_rng_random(py);
    if (prob < 0.15 && !visualization) {
      prob /= 0.15;
      if (prob < 0.9) zero_feat[i] = 1;
      // overlaps[i] > 0.4: the reference zero-pads overlaps to float64 when nb < max_region
      // (np.column_stack, :902-904) and compares in float64; otherwise in float32
      for (int k = 0; k < nb; ++k) {
        const float o = box_iou(b + 4 * i, b + 4 * k);
        if (nb < max_region ? (double)o > 0.4 : o > 0.4f) masked_label[k] = 1;
      }
      image_label[i] = 1;
    }
  }
  if (nb_out) *nb_out = nb;
  return 0;
}

}  // extern "C"
