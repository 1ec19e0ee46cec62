// Loss kernels of the pretraining heads: label compaction, masked-LM cross-entropy and region KL
// (forward and gradient in one pass over the logits row), per-task loss reduction, NSP forward.
#include "common.h"

namespace {

// --- label compaction (single workgroup, order preserving) -----------------------------------
__global__ __launch_bounds__(1024) void compact_kernel(const int64_t* __restrict__ labels, int n, int64_t thresh,
                                                       int inner, int outer, int base, int slot_id,
                                                       int32_t* __restrict__ idx, int64_t* __restrict__ lab,
                                                       int32_t* __restrict__ src, float* __restrict__ scale,
                                                       int32_t* __restrict__ slot, int32_t* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ int total;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int start = count[0];
  int run = 0;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int r = c0 + tid;
    const bool f = r < n && labels[r] >= thresh;
    const unsigned long long bal = __ballot(f);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int off = 0;
    for (int k = 0; k < w; ++k) off += wsum[k];
    int tot = 0;
    for (int k = 0; k < 16; ++k) tot += wsum[k];
    if (f) {
      const int pos = start + run + off + before;
      idx[pos] = (r / inner) * outer + (r % inner) + base;
      if (lab) lab[pos] = labels[r];
      if (src) src[pos] = r;
      if (slot) slot[pos] = slot_id;
    }
    run += tot;
    __syncthreads();
  }
  if (tid == 0) total = run;
  __syncthreads();
  const float inv = run > 0 ? 1.0f / (float)run : 0.f;
  for (int k = tid; k < run; k += 1024)
    if (scale) scale[start + k] = inv;
  __syncthreads();
  if (tid == 0) count[0] = start + total;
}

// --- cross-entropy over the vocabulary: one workgroup per row -------------------------------
__global__ __launch_bounds__(256) void ce_kernel(float* __restrict__ logits, long long ld,
                                                 const int64_t* __restrict__ labels, const float* __restrict__ rscale,
                                                 int vocab, float* __restrict__ loss_rows) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  float* x = logits + (long long)r * ld;
  float mx = -INFINITY;
  for (int c = threadIdx.x * 4; c < vocab; c += 1024) {
    if (c + 3 < vocab) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(x + c);
      mx = fmaxf(mx, fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3])));
    } else {
      for (int q = c; q < vocab; ++q) mx = fmaxf(mx, x[q]);
    }
  }
  mx = block_max<4>(mx, red);
  float s = 0.f;
  for (int c = threadIdx.x; c < vocab; c += 256) s += expf(x[c] - mx);
  s = block_sum<4>(s, red);
  const float lse = mx + logf(s);
  const int64_t lb = labels[r];
  const float sc = rscale[r];
  if (threadIdx.x == 0) loss_rows[r] = lse - x[lb];
  __syncthreads();
  const float invs = 1.f / s;
  for (int c = threadIdx.x; c < vocab; c += 256) {
    const float p = expf(x[c] - mx) * invs;
    x[c] = sc * (p - (c == lb ? 1.f : 0.f));
  }
}

// --- region KL: sum_c xlogy(t,t) - t*logsoftmax(x) --------------------------------------------
__global__ __launch_bounds__(256) void kl_kernel(float* __restrict__ logits, long long ld, const float* __restrict__ tgt,
                                                 long long ldt, const int32_t* __restrict__ trow,
                                                 const float* __restrict__ rscale, int ncls,
                                                 float* __restrict__ loss_rows) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  float* x = logits + (long long)r * ld;
  const float* t = tgt + (long long)trow[r] * ldt;
  float mx = -INFINITY;
  for (int c = threadIdx.x; c < ncls; c += 256) mx = fmaxf(mx, x[c]);
  mx = block_max<4>(mx, red);
  float s = 0.f, st = 0.f, xt = 0.f, tlt = 0.f;
  for (int c = threadIdx.x; c < ncls; c += 256) {
    const float xv = x[c], tv = t[c];
    s += expf(xv - mx);
    st += tv;
    xt += tv * xv;
    tlt += tv > 0.f ? tv * logf(tv) : 0.f;
  }
  s = block_sum<4>(s, red);
  st = block_sum<4>(st, red);
  xt = block_sum<4>(xt, red);
  tlt = block_sum<4>(tlt, red);
  const float lse = mx + logf(s);
  if (threadIdx.x == 0) loss_rows[r] = tlt - (xt - st * lse);
  __syncthreads();
  const float sc = rscale[r], invs = 1.f / s;
  for (int c = threadIdx.x; c < ncls; c += 256) {
    const float p = expf(x[c] - mx) * invs;
    x[c] = sc * (p * st - t[c]);
  }
}

// gradient rows of the text / PV MLM heads (slot 0 / 1 of the shared decoder's labelled rows) weighted by their
// losses' upstream gradients, which differ only when a caller weights mlm_t and mlm_pv differently
__global__ __launch_bounds__(256) void scale_rows_slot_kernel(float* __restrict__ x, long long ld,
                                                              const int32_t* __restrict__ slot, int cols, float w0,
                                                              float w1) {
  const int r = blockIdx.x;
  const float w = slot[r] == 0 ? w0 : w1;
  float* row = x + (long long)r * ld;
  for (int c = threadIdx.x; c < cols; c += 256) row[c] *= w;
}

__global__ __launch_bounds__(256) void loss_reduce_kernel(const float* __restrict__ lr, const float* __restrict__ sc,
                                                          const int32_t* __restrict__ slot, int rows,
                                                          float* __restrict__ out) {
  __shared__ float red[4];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int r = threadIdx.x; r < rows; r += 256) {
    const int k = slot[r];
    const float v = lr[r] * sc[r];
    acc[0] += k == 0 ? v : 0.f;
    acc[1] += k == 1 ? v : 0.f;
    acc[2] += k == 2 ? v : 0.f;
    acc[3] += k == 3 ? v : 0.f;
  }
  for (int k = 0; k < 4; ++k) {
    const float t = block_sum<4>(acc[k], red);
    if (threadIdx.x == 0) out[k] += t;
  }
}

__global__ __launch_bounds__(256) void nsp_kernel(const float* pt, const float* ppv, const float* pv, const float* w,
                                                  const float* b, const int64_t* l0, const int64_t* l1,
                                                  const int64_t* l2, int batch, int hidden, float* out) {
  __shared__ float red[4];
  float tot = 0.f;
  for (int i = 0; i < batch; ++i) {
    float z0 = 0.f, z1 = 0.f;
    for (int c = threadIdx.x; c < hidden; c += 256) {
      const float x = pt[(long long)i * hidden + c] + ppv[(long long)i * hidden + c] + pv[(long long)i * hidden + c];
      z0 += x * w[c];
      z1 += x * w[hidden + c];
    }
    z0 = block_sum<4>(z0, red) + b[0];
    z1 = block_sum<4>(z1, red) + b[1];
    const int lab = (l0[i] + l1[i] + l2[i]) == 0 ? 0 : 1;
    const float m = fmaxf(z0, z1);
    const float lse = m + logf(expf(z0 - m) + expf(z1 - m));
    tot += lse - (lab ? z1 : z0);
  }
  if (threadIdx.x == 0) out[0] = tot / batch;
}

}  // namespace

extern "C" int k3m_compact_labels_ex(const int64_t* labels, int n, int64_t thresh, int inner, int outer, int base,
                                     int slot_id, int32_t* idx, int64_t* out_labels, int32_t* src, float* row_scale,
                                     int32_t* slot, int32_t* count, hipStream_t st) {
  K3M_ARG(labels && idx && count && n >= 0 && inner > 0);
  hipLaunchKernelGGL(compact_kernel, dim3(1), dim3(1024), 0, st, labels, n, thresh, inner, outer, base, slot_id, idx,
                     out_labels, src, row_scale, slot, count);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_ce_fwd_bwd(float* logits, long long ld, const int64_t* labels, const float* row_scale, int rows,
                              int vocab, float* loss_rows, hipStream_t st) {
  if (rows == 0) return 0;
  K3M_ARG(logits && labels && row_scale && loss_rows && rows >= 0 && vocab > 0);
  if (rows == 0) return 0;
  K3M_ARG(ld % 4 == 0);
  hipLaunchKernelGGL(ce_kernel, dim3(rows), dim3(256), 0, st, logits, ld, labels, row_scale, vocab, loss_rows);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_kl_fwd_bwd(float* logits, long long ld, const float* target, long long ldt, const int32_t* trow,
                              const float* row_scale, int rows, int ncls, float* loss_rows, hipStream_t st) {
  if (rows == 0) return 0;
  K3M_ARG(logits && target && trow && row_scale && loss_rows && rows >= 0);
  if (rows == 0) return 0;
  hipLaunchKernelGGL(kl_kernel, dim3(rows), dim3(256), 0, st, logits, ld, target, ldt, trow, row_scale, ncls,
                     loss_rows);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_scale_rows_by_slot(float* x, long long ld, const int32_t* slot, int rows, int cols, float w0,
                                      float w1, hipStream_t st) {
  if (rows == 0) return 0;
  K3M_ARG(x && slot && rows > 0 && cols > 0 && ld >= cols);
  hipLaunchKernelGGL(scale_rows_slot_kernel, dim3(rows), dim3(256), 0, st, x, ld, slot, cols, w0, w1);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_loss_reduce(const float* loss_rows, const float* row_scale, const int32_t* slot, int rows,
                               float* out, hipStream_t st) {
  K3M_ARG(loss_rows && row_scale && slot && out);
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, st, loss_rows, row_scale, slot, rows, out);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_nsp_loss(const float* pt, const float* ppv, const float* pv, const float* w, const float* b,
                            const int64_t* l0, const int64_t* l1, const int64_t* l2, int batch, int hidden, float* out,
                            hipStream_t st) {
  K3M_ARG(pt && ppv && pv && w && b && l0 && l1 && l2 && out && batch > 0);
  hipLaunchKernelGGL(nsp_kernel, dim3(1), dim3(256), 0, st, pt, ppv, pv, w, b, l0, l1, l2, batch, hidden, out);
  K3M_CHECK_LAUNCH();
  return 0;
}
