// Structure aggregator + link-prediction (LPM) loss, vectorised over a padded [B, NPV] triple
// layout (reference: structure_aggregator, vilbert_k3m.py:2413-2505, a Python loop with one host
// sync per triple).  Every item's triples are independent workgroups; the data-dependent parts
// (number of valid triples, zero-triple items, negative draws) are index tables on the device.
//
// Semantics kept from the reference:
//  * p_ij / v_ij = mean of the two ENDPOINT rows index_p[i,j] / index_v[i,j] (:2443-2444);
//  * triples stop at the first j with index_p[i,j,0] == 0 (:2441);
//  * an item without triples reuses the `t` of the latest earlier item that had triples, or
//    [c_initial_0] if none did (bare except, :2452-2456)  -> src[i];
//  * c_final_i = c_init_i + W3 (sum_j att_j t_j) + b3, att = softmax_j(w2.leaky_relu(t_j) + b2);
//  * LPM: MarginRankingLoss(margin)(pos, neg, y=+1) = mean(max(0, neg - pos + margin)) (:2501).
#include "common.h"

namespace {

constexpr int NT = 256;

__device__ __forceinline__ int count_valid(const int64_t* index_p, int i, int npv) {
  int n = npv;
  for (int j = 0; j < npv; ++j)
    if (index_p[((long long)i * npv + j) * 2] == 0) {
      n = j;
      break;
    }
  return n;
}

// nvalid[i] and src[i] (the latest item k <= i with triples, -1 if none) for every item: one
// 1024-thread workgroup, one item per thread, an inclusive max-scan per 1024-item chunk carried
// across chunks (was a single serial thread: 101 us per step at B = 64).
constexpr int CNT_NT = 1024;
__global__ __launch_bounds__(CNT_NT) void sa_count_kernel(const int64_t* index_p, int batch, int npv, int32_t* nvalid,
                                                          int32_t* src) {
  __shared__ int scan[CNT_NT];
  int carry = -1;
  for (int base = 0; base < batch; base += CNT_NT) {
    const int i = base + (int)threadIdx.x;
    int n = 0;
    if (i < batch) {
      n = count_valid(index_p, i, npv);
      nvalid[i] = n;
    }
    scan[threadIdx.x] = (i < batch && n > 0) ? i : -1;
    __syncthreads();
    for (int d = 1; d < CNT_NT; d <<= 1) {
      const int o = threadIdx.x >= (unsigned)d ? scan[threadIdx.x - d] : -1;
      __syncthreads();
      scan[threadIdx.x] = max(scan[threadIdx.x], o);
      __syncthreads();
    }
    if (i < batch) src[i] = max(carry, scan[threadIdx.x]);   // -1 -> c_initial[0]
    carry = max(carry, scan[CNT_NT - 1]);
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(NT) void sa_gather_kernel(const T* seq, const int64_t* index_p, const int64_t* index_v,
                                                       const float* c_init, float* X, const int32_t* nvalid, int len,
                                                       int npv, int h) {
  const int i = blockIdx.x / npv, j = blockIdx.x % npv;
  float* x = X + (long long)blockIdx.x * 3 * h;
  const bool ok = j < nvalid[i];
  const long long ip = ((long long)i * npv + j) * 2;
  const long long pa = ok ? index_p[ip] : 0, pb = ok ? index_p[ip + 1] : 0;
  const long long va = ok ? index_v[ip] : 0, vb = ok ? index_v[ip + 1] : 0;
  const T* s = seq + (long long)i * len * h;
  for (int c = threadIdx.x; c < h; c += NT) {
    if (ok) {
      x[c] = c_init[(long long)i * h + c];
      x[h + c] = (to_f(s[pa * h + c]) + to_f(s[pb * h + c])) * 0.5f;
      x[2 * h + c] = (to_f(s[va * h + c]) + to_f(s[vb * h + c])) * 0.5f;
    } else {
      x[c] = 0.f;
      x[h + c] = 0.f;
      x[2 * h + c] = 0.f;
    }
  }
}

__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : 0.01f * x; }

// one workgroup per item; npv <= 64
__global__ __launch_bounds__(NT) void sa_attn_fwd_kernel(const float* T, const int32_t* nvalid, const int32_t* src,
                                                         const float* w2, const float* b2, const float* c_init,
                                                         float* att, float* agg, int npv, int h) {
  __shared__ float red[4];
  __shared__ float beta_s[64];
  const int i = blockIdx.x;
  const int s = src[i];
  float* ag = agg + (long long)i * h;
  float* at = att + (long long)i * npv;
  if (s < 0) {
    for (int c = threadIdx.x; c < h; c += NT) ag[c] = c_init[c];
    for (int j = threadIdx.x; j < npv; j += NT) at[j] = j == 0 ? 1.f : 0.f;
    return;
  }
  const int n = nvalid[s];
  for (int j = 0; j < n; ++j) {
    const float* t = T + ((long long)s * npv + j) * h;
    float a = 0.f;
    for (int c = threadIdx.x; c < h; c += NT) a += w2[c] * lrelu(t[c]);
    a = block_sum<4>(a, red);
    if (threadIdx.x == 0) beta_s[j] = a + b2[0];
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int j = 0; j < n; ++j) mx = fmaxf(mx, beta_s[j]);
  float sum = 0.f;
  for (int j = 0; j < n; ++j) sum += expf(beta_s[j] - mx);
  for (int j = threadIdx.x; j < npv; j += NT) at[j] = j < n ? expf(beta_s[j] - mx) / sum : 0.f;
  for (int c = threadIdx.x; c < h; c += NT) {
    float a = 0.f;
    for (int j = 0; j < n; ++j) a += (expf(beta_s[j] - mx) / sum) * T[((long long)s * npv + j) * h + c];
    ag[c] = a;
  }
}

__global__ __launch_bounds__(NT) void sa_attn_bwd_kernel(const float* dagg, const float* T, const float* att,
                                                         const int32_t* nvalid, const int32_t* src, const float* w2,
                                                         float* dT, float* dw2, float* db2, float* dc_init, int npv,
                                                         int h) {
  __shared__ float red[4];
  __shared__ float datt[64];
  const int i = blockIdx.x;
  const int s = src[i];
  const float* dg = dagg + (long long)i * h;
  if (s < 0) {
    for (int c = threadIdx.x; c < h; c += NT) atomicAdd(dc_init + c, dg[c]);
    return;
  }
  const int n = nvalid[s];
  const float* at = att + (long long)i * npv;
  for (int j = 0; j < n; ++j) {
    const float* t = T + ((long long)s * npv + j) * h;
    float a = 0.f;
    for (int c = threadIdx.x; c < h; c += NT) a += dg[c] * t[c];
    a = block_sum<4>(a, red);
    if (threadIdx.x == 0) datt[j] = a;
  }
  __syncthreads();
  float dot = 0.f;
  for (int j = 0; j < n; ++j) dot += at[j] * datt[j];
  float db = 0.f;
  for (int j = 0; j < n; ++j) {
    const float dbeta = at[j] * (datt[j] - dot);
    db += dbeta;
    const float* t = T + ((long long)s * npv + j) * h;
    float* dt = dT + ((long long)s * npv + j) * h;
    for (int c = threadIdx.x; c < h; c += NT) {
      const float tv = t[c];
      const float g = at[j] * dg[c] + dbeta * w2[c] * (tv > 0.f ? 1.f : 0.01f);
      atomicAdd(dt + c, g);
      atomicAdd(dw2 + c, dbeta * lrelu(tv));
    }
  }
  if (threadIdx.x == 0) atomicAdd(db2, db);
}

// negative e of triple ij: e < ke entity negatives (ent[ij*ke + e]), then kv value negatives
constexpr int LPM_KMAX = 16;
__device__ __forceinline__ bool pair_neg(const int64_t* ent, const int64_t* val, long long ij, int e, int ke, int kv,
                                         int& k) {
  const long long v = e < ke ? ent[ij * ke + e] : val[ij * kv + (e - ke)];
  k = (int)v;
  return v >= 0;
}

// ws layout (K = ke + kv): [B*npv*K] hinge (-1 = no pair), [B*npv] pos norm, [B*npv*K] neg norm,
// [2] (count, sum)
__global__ __launch_bounds__(NT) void lpm_fwd_kernel(const float* cf, const float* X, const int32_t* nvalid,
                                                     const int64_t* ent, const int64_t* val, int npv, int h, int ke,
                                                     int kv, float margin, float* ws, int total) {
  __shared__ float red[4];
  const int K = ke + kv;
  const int i = blockIdx.x / npv, j = blockIdx.x % npv;
  const long long ij = blockIdx.x;
  float* hinge = ws;
  float* posn = ws + (long long)total * K;
  float* negn = posn + total;
  if (j >= nvalid[i]) {
    if ((int)threadIdx.x < K) hinge[ij * K + threadIdx.x] = -1.f;
    return;
  }
  const float* x = X + ij * 3 * h;
  float a = 0.f;
  for (int c = threadIdx.x; c < h; c += NT) {
    const float u = cf[(long long)i * h + c] + x[h + c] - x[2 * h + c];
    a += u * u;
  }
  const float pn = sqrtf(block_sum<4>(a, red));
  if (threadIdx.x == 0) posn[ij] = pn;
  for (int e = 0; e < K; ++e) {
    int k;
    const bool has = pair_neg(ent, val, ij, e, ke, kv, k);
    if (!has) {
      if (threadIdx.x == 0) hinge[ij * K + e] = -1.f;
      continue;
    }
    float b = 0.f;
    for (int c = threadIdx.x; c < h; c += NT) {
      float u;
      if (e < ke) u = cf[(long long)k * h + c] + x[h + c] - x[2 * h + c];
      else u = cf[(long long)i * h + c] + x[h + c] - X[((long long)i * npv + k) * 3 * h + 2 * h + c];
      b += u * u;
    }
    const float nn = sqrtf(block_sum<4>(b, red));
    if (threadIdx.x == 0) {
      negn[ij * K + e] = nn;
      hinge[ij * K + e] = fmaxf(0.f, nn - pn + margin);
    }
  }
}

__global__ __launch_bounds__(NT) void lpm_reduce_kernel(float* ws, int total, int K, float* loss) {
  __shared__ float red[4];
  float cnt = 0.f, sum = 0.f;
  for (int p = threadIdx.x; p < total * K; p += NT) {
    const float hv = ws[p];
    if (hv >= 0.f) {
      cnt += 1.f;
      sum += hv;
    }
  }
  cnt = block_sum<4>(cnt, red);
  sum = block_sum<4>(sum, red);
  if (threadIdx.x == 0) {
    float* tail = ws + (long long)total * (2 * K + 1);
    tail[0] = cnt;
    tail[1] = sum;
    loss[0] = cnt > 0.f ? sum / cnt : NAN;  // mean of an empty tensor is NaN, as in the reference
  }
}

__global__ __launch_bounds__(NT) void lpm_bwd_kernel(const float* cf, const float* X, const int32_t* nvalid,
                                                     const int64_t* ent, const int64_t* val, int npv, int h, int ke,
                                                     int kv, const float* ws, int total, float* dcf, float* dX) {
  const int K = ke + kv;
  const int i = blockIdx.x / npv, j = blockIdx.x % npv;
  const long long ij = blockIdx.x;
  if (j >= nvalid[i]) return;
  const float* hinge = ws;
  const float* posn = ws + (long long)total * K;
  const float* negn = posn + total;
  const float cnt = ws[(long long)total * (2 * K + 1)];
  const float w = 1.f / cnt;
  const float* x = X + ij * 3 * h;
  float* dx = dX + ij * 3 * h;
  // coefficient of the positive norm: -w per active pair
  float cpos = 0.f;
  float cneg[LPM_KMAX];
  int kk[LPM_KMAX];
#pragma unroll
  for (int e = 0; e < LPM_KMAX; ++e) {
    cneg[e] = 0.f;
    kk[e] = -1;
    int k;
    if (e < K && pair_neg(ent, val, ij, e, ke, kv, k) && hinge[ij * K + e] > 0.f) {
      cpos -= w;
      cneg[e] = w / fmaxf(negn[ij * K + e], 1e-30f);
      kk[e] = k;
    }
  }
  const float cp = cpos / fmaxf(posn[ij], 1e-30f);
  for (int c = threadIdx.x; c < h; c += NT) {
    const float p = x[h + c], v = x[2 * h + c];
    const float up = cf[(long long)i * h + c] + p - v;
    float gci = cp * up, gp = cp * up, gv = -cp * up;
#pragma unroll
    for (int e = 0; e < LPM_KMAX; ++e) {
      if (kk[e] < 0) continue;
      if (e < ke) {
        const float u = cf[(long long)kk[e] * h + c] + p - v;
        const float g = cneg[e] * u;
        atomicAdd(dcf + (long long)kk[e] * h + c, g);
        gp += g;
        gv -= g;
      } else {
        const long long ik = (long long)i * npv + kk[e];
        const float u = cf[(long long)i * h + c] + p - X[ik * 3 * h + 2 * h + c];
        const float g = cneg[e] * u;
        gci += g;
        gp += g;
        atomicAdd(dX + ik * 3 * h + 2 * h + c, -g);
      }
    }
    atomicAdd(dcf + (long long)i * h + c, gci);
    atomicAdd(dx + h + c, gp);
    atomicAdd(dx + 2 * h + c, gv);
  }
}

// random.sample(range(nc), take) semantics: `take` distinct ranks drawn uniformly without replacement
// (draw q picks uniformly among the nc - q ranks not drawn yet: the r-th free rank, found by stepping
// over the earlier draws in ascending order), then rank -> index skipping `self`.
__device__ __forceinline__ void sample_distinct(uint64_t seed, uint64_t base, int nc, int take, int self,
                                                int64_t* out) {
  int drawn[LPM_KMAX];   // ascending
  for (int q = 0; q < take; ++q) {
    int r = (int)(k3m_hash(seed, base + q) % (uint32_t)(nc - q));
    int pos = 0;
    for (; pos < q; ++pos) {
      if (r >= drawn[pos]) ++r;
      else break;
    }
    for (int s = q; s > pos; --s) drawn[s] = drawn[s - 1];
    drawn[pos] = r;
    out[q] = r >= self ? r + 1 : r;
  }
}

__global__ void lpm_sample_kernel(const int32_t* nvalid, int batch, int npv, int n_ent, int n_val, uint64_t seed,
                                  uint64_t off, int64_t* ent, int64_t* val) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= batch * npv) return;
  const int i = t / npv, j = t % npv;
  for (int q = 0; q < n_ent; ++q) ent[(long long)t * n_ent + q] = -1;
  for (int q = 0; q < n_val; ++q) val[(long long)t * n_val + q] = -1;
  const int n = nvalid[i];
  if (j >= n) return;
  const uint64_t base = off + (uint64_t)t * (n_ent + n_val);
  // entity candidates: all k != i (vilbert_k3m.py:2476-2480); value candidates: j' != j (:2488-2492)
  sample_distinct(seed, base, batch - 1, min(batch - 1, n_ent), i, ent + (long long)t * n_ent);
  sample_distinct(seed, base + n_ent, n - 1, min(n - 1, n_val), j, val + (long long)t * n_val);
}

template <typename T>
__global__ __launch_bounds__(NT) void sa_gather_bwd_kernel(const float* dX, const int64_t* index_p,
                                                           const int64_t* index_v, const int32_t* nvalid, T* dseq,
                                                           float* dc_init, int len, int npv, int h) {
  const int i = blockIdx.x / npv, j = blockIdx.x % npv;
  if (j >= nvalid[i]) return;
  const long long ip = ((long long)i * npv + j) * 2;
  const long long pa = index_p[ip], pb = index_p[ip + 1], va = index_v[ip], vb = index_v[ip + 1];
  const float* dx = dX + (long long)blockIdx.x * 3 * h;
  T* ds = dseq + (long long)i * len * h;
  for (int c = threadIdx.x; c < h; c += NT) {
    atomicAdd(dc_init + (long long)i * h + c, dx[c]);
    const float gp = 0.5f * dx[h + c], gv = 0.5f * dx[2 * h + c];
    atomicAdd(reinterpret_cast<float*>(ds) + pa * h + c, gp);
    atomicAdd(reinterpret_cast<float*>(ds) + pb * h + c, gp);
    atomicAdd(reinterpret_cast<float*>(ds) + va * h + c, gv);
    atomicAdd(reinterpret_cast<float*>(ds) + vb * h + c, gv);
  }
}

// ---------------------------------------------------------------- deterministic mode (K3M_DETERMINISTIC)
// The same backward with every sum in a fixed order (no float atomics): a destination row has one owning
// workgroup, which adds its contributions in item / triple order; sums over the whole batch (dw2, db2) go
// through per-item partials reduced in item order.

constexpr int SA_CPT = 8;   // columns per thread (hidden <= 2048)

// sa_attn_bwd_kernel's contribution of item i (triples of src s >= 0) to dT[s] (plain read-modify-write: the
// caller owns s), to this thread's dw2 columns (acc) and to db (returned, thread 0)
__device__ __forceinline__ float sa_item_bwd(const float* dagg, const float* T, const float* att, const float* w2, float* dT,
                             int i, int s, int n, int npv, int h, float* acc, float* red, float* datt) {
  const float* dg = dagg + (long long)i * h;
  const float* at = att + (long long)i * npv;
  for (int j = 0; j < n; ++j) {
    const float* t = T + ((long long)s * npv + j) * h;
    float a = 0.f;
    for (int c = threadIdx.x; c < h; c += NT) a += dg[c] * t[c];
    a = block_sum<4>(a, red);
    if (threadIdx.x == 0) datt[j] = a;
  }
  __syncthreads();
  float dot = 0.f;
  for (int j = 0; j < n; ++j) dot += at[j] * datt[j];
  float db = 0.f;
  for (int j = 0; j < n; ++j) {
    const float dbeta = at[j] * (datt[j] - dot);
    db += dbeta;
    const float* t = T + ((long long)s * npv + j) * h;
    float* dt = dT + ((long long)s * npv + j) * h;
#pragma unroll
    for (int q = 0; q < SA_CPT; ++q) {
      const int c = threadIdx.x + q * NT;
      if (c >= h) break;
      const float tv = t[c];
      dt[c] += at[j] * dg[c] + dbeta * w2[c] * (tv > 0.f ? 1.f : 0.01f);
      acc[q] += dbeta * lrelu(tv);
    }
  }
  __syncthreads();   // datt is reused by the next item
  return db;
}

// block b owns dT[b] (when item b has triples) and handles the items that read b's triples (b itself and the
// zero-triple items after it: src is a running max, so they follow b contiguously); block 0 also adds the
// leading zero-triple items (src = -1) to c_initial row 0.  Partial dw2 / db2 -> ws[b][0 .. h].
__global__ __launch_bounds__(NT) void sa_attn_bwd_det_kernel(const float* dagg, const float* T, const float* att,
                                                             const int32_t* nvalid, const int32_t* src,
                                                             const float* w2, float* dT, float* dc_init, float* ws,
                                                             int batch, int npv, int h) {
  __shared__ float red[4];
  __shared__ float datt[64];
  const int b = blockIdx.x;
  float acc[SA_CPT];
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q) acc[q] = 0.f;
  float db = 0.f;
  if (b == 0) {
    for (int i = 0; i < batch && src[i] < 0; ++i)
      for (int c = threadIdx.x; c < h; c += NT) dc_init[c] += dagg[(long long)i * h + c];
  }
  const int n = nvalid[b];
  if (n > 0)
    for (int i = b; i < batch && src[i] == b; ++i) db += sa_item_bwd(dagg, T, att, w2, dT, i, b, n, npv, h, acc, red, datt);
  float* wb = ws + (long long)b * (h + 1);
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q)
    if (threadIdx.x + q * NT < h) wb[threadIdx.x + q * NT] = acc[q];
  if (threadIdx.x == 0) wb[h] = db;
}
__global__ __launch_bounds__(NT) void sa_w2_reduce_kernel(const float* ws, float* dw2, float* db2, int batch, int h) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c > h) return;
  float a = 0.f;
  for (int b = 0; b < batch; ++b) a += ws[(long long)b * (h + 1) + c];
  if (c < h) dw2[c] += a;
  else db2[0] += a;
}

// LPM backward, own-item part: block i walks its triples in order; its own X rows (p, v and the value
// negatives, all rows of item i) and c_final[i] get plain read-modify-writes.  The entity negatives' terms
// on other items' c_final rows are lpm_bwd_ent_det_kernel's.
__global__ __launch_bounds__(NT) void lpm_bwd_item_det_kernel(const float* cf, const float* X, const int32_t* nvalid,
                                                              const int64_t* ent, const int64_t* val, int npv, int h,
                                                              int ke, int kv, const float* ws, int total, float* dcf,
                                                              float* dX) {
  const int K = ke + kv;
  const int i = blockIdx.x;
  const float* hinge = ws;
  const float* posn = ws + (long long)total * K;
  const float* negn = posn + total;
  const float w = 1.f / ws[(long long)total * (2 * K + 1)];
  float gci_acc[SA_CPT];
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q) gci_acc[q] = 0.f;
  const int n = nvalid[i];
  for (int j = 0; j < n; ++j) {
    const long long ij = (long long)i * npv + j;
    const float* x = X + ij * 3 * h;
    float* dx = dX + ij * 3 * h;
    float cpos = 0.f;
    float cneg[LPM_KMAX];
    int kk[LPM_KMAX];
#pragma unroll
    for (int e = 0; e < LPM_KMAX; ++e) {
      cneg[e] = 0.f;
      kk[e] = -1;
      int k;
      if (e < K && pair_neg(ent, val, ij, e, ke, kv, k) && hinge[ij * K + e] > 0.f) {
        cpos -= w;
        cneg[e] = w / fmaxf(negn[ij * K + e], 1e-30f);
        kk[e] = k;
      }
    }
    const float cp = cpos / fmaxf(posn[ij], 1e-30f);
#pragma unroll
    for (int q = 0; q < SA_CPT; ++q) {
      const int c = threadIdx.x + q * NT;
      if (c >= h) break;
      const float p = x[h + c], v = x[2 * h + c];
      const float up = cf[(long long)i * h + c] + p - v;
      float gci = cp * up, gp = cp * up, gv = -cp * up;
#pragma unroll
      for (int e = 0; e < LPM_KMAX; ++e) {
        if (kk[e] < 0) continue;
        if (e < ke) {
          const float g = cneg[e] * (cf[(long long)kk[e] * h + c] + p - v);
          gp += g;
          gv -= g;
        } else {
          const long long ik = (long long)i * npv + kk[e];
          const float g = cneg[e] * (cf[(long long)i * h + c] + p - X[ik * 3 * h + 2 * h + c]);
          gci += g;
          gp += g;
          dX[ik * 3 * h + 2 * h + c] -= g;
        }
      }
      gci_acc[q] += gci;
      dx[h + c] += gp;
      dx[2 * h + c] += gv;
    }
  }
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q)
    if (threadIdx.x + q * NT < h) dcf[(long long)i * h + threadIdx.x + q * NT] += gci_acc[q];
}

// entity-negative terms on c_final[k]: block k scans every triple (item, triple, negative order) for the
// active pairs whose entity negative is k
__global__ __launch_bounds__(NT) void lpm_bwd_ent_det_kernel(const float* cf, const float* X, const int32_t* nvalid,
                                                             const int64_t* ent, int batch, int npv, int h, int ke,
                                                             int kv, const float* ws, int total, float* dcf) {
  const int K = ke + kv;
  const int k = blockIdx.x;
  const float* hinge = ws;
  const float* negn = ws + (long long)total * K + total;
  const float w = 1.f / ws[(long long)total * (2 * K + 1)];
  float acc[SA_CPT];
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q) acc[q] = 0.f;
  for (int i = 0; i < batch; ++i) {
    const int n = nvalid[i];
    for (int j = 0; j < n; ++j) {
      const long long ij = (long long)i * npv + j;
      for (int e = 0; e < ke; ++e) {
        if (ent[ij * ke + e] != k || !(hinge[ij * K + e] > 0.f)) continue;
        const float cn = w / fmaxf(negn[ij * K + e], 1e-30f);
        const float* x = X + ij * 3 * h;
#pragma unroll
        for (int q = 0; q < SA_CPT; ++q) {
          const int c = threadIdx.x + q * NT;
          if (c < h) acc[q] += cn * (cf[(long long)k * h + c] + x[h + c] - x[2 * h + c]);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q)
    if (threadIdx.x + q * NT < h) dcf[(long long)k * h + threadIdx.x + q * NT] += acc[q];
}

// sa_gather_bwd_kernel with one workgroup per item walking its triples in order (every row it writes -- the
// item's sequence rows and c_initial[i] -- belongs to that item)
__global__ __launch_bounds__(NT) void sa_gather_bwd_det_kernel(const float* dX, const int64_t* index_p,
                                                               const int64_t* index_v, const int32_t* nvalid,
                                                               float* dseq, float* dc_init, int len, int npv, int h) {
  const int i = blockIdx.x;
  const int n = nvalid[i];
  float* ds = dseq + (long long)i * len * h;
  float acc[SA_CPT];
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q) acc[q] = 0.f;
  for (int j = 0; j < n; ++j) {
    const long long ip = ((long long)i * npv + j) * 2;
    const long long pa = index_p[ip], pb = index_p[ip + 1], va = index_v[ip], vb = index_v[ip + 1];
    const float* dx = dX + ((long long)i * npv + j) * 3 * h;
#pragma unroll
    for (int q = 0; q < SA_CPT; ++q) {
      const int c = threadIdx.x + q * NT;
      if (c >= h) break;
      acc[q] += dx[c];
      const float gp = 0.5f * dx[h + c], gv = 0.5f * dx[2 * h + c];
      ds[pa * h + c] += gp;
      ds[pb * h + c] += gp;
      ds[va * h + c] += gv;
      ds[vb * h + c] += gv;
    }
  }
#pragma unroll
  for (int q = 0; q < SA_CPT; ++q)
    if (threadIdx.x + q * NT < h) dc_init[(long long)i * h + threadIdx.x + q * NT] += acc[q];
}

}  // namespace

extern "C" int k3m_sa_gather(const void* seq, const int64_t* index_p, const int64_t* index_v, const float* c_init,
                             float* X, int32_t* nvalid, int32_t* src, int batch, int len, int npv, int hidden,
                             int dtype, hipStream_t st) {
  K3M_ARG(seq && index_p && index_v && c_init && X && nvalid && src && npv > 0 && npv <= 64);
  K3M_ARG(dtype == K3M_F32);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_count_kernel, dim3(1), dim3(CNT_NT), 0, st, index_p, batch, npv, nvalid, src);
  hipLaunchKernelGGL(sa_gather_kernel<float>, dim3(batch * npv), dim3(NT), 0, st, (const float*)seq, index_p, index_v,
                     c_init, X, nvalid, len, npv, hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_sa_attn_fwd(const float* T, const int32_t* nvalid, const int32_t* src, const float* w2,
                               const float* b2, const float* c_init, float* att, float* agg, int batch, int npv,
                               int hidden, hipStream_t st) {
  K3M_ARG(T && nvalid && src && w2 && b2 && c_init && att && agg && npv <= 64);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_attn_fwd_kernel, dim3(batch), dim3(NT), 0, st, T, nvalid, src, w2, b2, c_init, att, agg, npv,
                     hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_sa_attn_bwd(const float* dagg, const float* T, const float* att, const int32_t* nvalid,
                               const int32_t* src, const float* w2, float* dT, float* dw2, float* db2, float* dc_init,
                               int batch, int npv, int hidden, hipStream_t st) {
  K3M_ARG(dagg && T && att && nvalid && src && w2 && dT && dw2 && db2 && dc_init && npv <= 64);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_attn_bwd_kernel, dim3(batch), dim3(NT), 0, st, dagg, T, att, nvalid, src, w2, dT, dw2, db2,
                     dc_init, npv, hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_lpm_fwd(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                           const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val, float margin,
                           float* loss, float* ws, hipStream_t st) {
  K3M_ARG(c_final && X && nvalid && loss && ws && n_ent >= 0 && n_val >= 0 && n_ent + n_val <= LPM_KMAX);
  K3M_ARG((ent_neg || n_ent == 0) && (val_neg || n_val == 0));
  const int total = batch * npv;
  if (total == 0) return 0;
  hipLaunchKernelGGL(lpm_fwd_kernel, dim3(total), dim3(NT), 0, st, c_final, X, nvalid, ent_neg, val_neg, npv, hidden,
                     n_ent, n_val, margin, ws, total);
  hipLaunchKernelGGL(lpm_reduce_kernel, dim3(1), dim3(NT), 0, st, ws, total, n_ent + n_val, loss);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_lpm_bwd(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                           const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val, float margin,
                           const float* ws, float* dc_final, float* dX, hipStream_t st) {
  K3M_ARG(c_final && X && nvalid && ws && dc_final && dX && n_ent >= 0 && n_val >= 0 && n_ent + n_val <= LPM_KMAX);
  K3M_ARG((ent_neg || n_ent == 0) && (val_neg || n_val == 0));
  (void)margin;
  const int total = batch * npv;
  if (total == 0) return 0;
  hipLaunchKernelGGL(lpm_bwd_kernel, dim3(total), dim3(NT), 0, st, c_final, X, nvalid, ent_neg, val_neg, npv, hidden,
                     n_ent, n_val, ws, total, dc_final, dX);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_lpm_sample(const int32_t* nvalid, int batch, int npv, int n_ent, int n_val, uint64_t seed,
                              uint64_t off, int64_t* ent_neg, int64_t* val_neg, hipStream_t st) {
  K3M_ARG(nvalid && n_ent >= 0 && n_val >= 0 && n_ent + n_val <= LPM_KMAX);
  K3M_ARG((ent_neg || n_ent == 0) && (val_neg || n_val == 0));
  const int total = batch * npv;
  if (total == 0) return 0;
  hipLaunchKernelGGL(lpm_sample_kernel, dim3(k3m_cdiv(total, 256)), dim3(256), 0, st, nvalid, batch, npv, n_ent, n_val,
                     seed, off, ent_neg, val_neg);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_sa_gather_bwd(const float* dX, const int64_t* index_p, const int64_t* index_v,
                                 const int32_t* nvalid, void* dseq, float* dc_init, int batch, int len, int npv,
                                 int hidden, int dtype, hipStream_t st) {
  K3M_ARG(dX && index_p && index_v && nvalid && dseq && dc_init);
  K3M_ARG(dtype == K3M_F32);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_gather_bwd_kernel<float>, dim3(batch * npv), dim3(NT), 0, st, dX, index_p, index_v, nvalid,
                     (float*)dseq, dc_init, len, npv, hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- deterministic-mode entry points
extern "C" int k3m_sa_attn_bwd_det(const float* dagg, const float* T, const float* att, const int32_t* nvalid,
                                   const int32_t* src, const float* w2, float* dT, float* dw2, float* db2,
                                   float* dc_init, float* ws, int batch, int npv, int hidden, hipStream_t st) {
  K3M_ARG(dagg && T && att && nvalid && src && w2 && dT && dw2 && db2 && dc_init && ws && npv <= 64);
  K3M_ARG(hidden <= SA_CPT * NT);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_attn_bwd_det_kernel, dim3(batch), dim3(NT), 0, st, dagg, T, att, nvalid, src, w2, dT, dc_init,
                     ws, batch, npv, hidden);
  hipLaunchKernelGGL(sa_w2_reduce_kernel, dim3(k3m_cdiv(hidden + 1, NT)), dim3(NT), 0, st, ws, dw2, db2, batch, hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_lpm_bwd_det(const float* c_final, const float* X, const int32_t* nvalid, const int64_t* ent_neg,
                               const int64_t* val_neg, int batch, int npv, int hidden, int n_ent, int n_val,
                               const float* ws, float* dc_final, float* dX, hipStream_t st) {
  K3M_ARG(c_final && X && nvalid && ws && dc_final && dX && n_ent >= 0 && n_val >= 0 && n_ent + n_val <= LPM_KMAX);
  K3M_ARG((ent_neg || n_ent == 0) && (val_neg || n_val == 0) && hidden <= SA_CPT * NT);
  const int total = batch * npv;
  if (total == 0) return 0;
  hipLaunchKernelGGL(lpm_bwd_item_det_kernel, dim3(batch), dim3(NT), 0, st, c_final, X, nvalid, ent_neg, val_neg, npv,
                     hidden, n_ent, n_val, ws, total, dc_final, dX);
  if (n_ent > 0)
    hipLaunchKernelGGL(lpm_bwd_ent_det_kernel, dim3(batch), dim3(NT), 0, st, c_final, X, nvalid, ent_neg, batch, npv,
                       hidden, n_ent, n_val, ws, total, dc_final);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_sa_gather_bwd_det(const float* dX, const int64_t* index_p, const int64_t* index_v,
                                     const int32_t* nvalid, void* dseq, float* dc_init, int batch, int len, int npv,
                                     int hidden, int dtype, hipStream_t st) {
  K3M_ARG(dX && index_p && index_v && nvalid && dseq && dc_init && hidden <= SA_CPT * NT);
  K3M_ARG(dtype == K3M_F32);
  if (batch == 0) return 0;
  hipLaunchKernelGGL(sa_gather_bwd_det_kernel, dim3(batch), dim3(NT), 0, st, dX, index_p, index_v, nvalid,
                     (float*)dseq, dc_init, len, npv, hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}
