// Item-alignment pair heads (K3MForItemAlignment.forward, vilbert_k3m.py:3379-3456; SURVEY.md §8(f)
// rank 3).  The two items of a pair run through the encoder as ONE stacked batch, so their final
// item embeddings arrive as e = c_final [2B][H] (item 1 rows 0..B-1, item 2 rows B..2B-1).
//
//  "ce"     ClassificationHead (:2164-2183): x = dropout([e1 ; e2]); u = dense(x) (k3m_gemm);
//           logits = out_proj(dropout(tanh(u))); probs = softmax(logits, dim 1);
//           loss = CrossEntropyLoss(logits, labels.long()) (mean).
//  "cosine" loss = CosineEmbeddingLoss(margin)(e1, e2, 2*labels - 1) (mean);
//           probs = (cosine_similarity(e1, e1) + 1) / 2 (the reference compares e1 with ITSELF, :3443).
//
// Forward and backward of each head are fused (the loss is the end of the graph), deterministic
// (no atomics: per-row kernels, then one reduction kernel).  Tiny: B x H elements.
#include "common.h"

namespace {

constexpr int NT = 256;
constexpr int NW = NT / 64;

__global__ __launch_bounds__(NT) void pair_cat_kernel(const float* __restrict__ e, int B, int H, float p, uint64_t seed,
                                                      uint64_t off, float* __restrict__ x) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < 2 * H; c += NT) {
    const float v = c < H ? e[(long long)b * H + c] : e[(long long)(B + b) * H + (c - H)];
    x[(long long)b * 2 * H + c] = v * k3m_dropout_scale(seed, off + (uint64_t)b * 2 * H + c, p);
  }
}

__global__ __launch_bounds__(NT) void pair_cat_bwd_kernel(const float* __restrict__ dx, int B, int H, float p,
                                                          uint64_t seed, uint64_t off, float* __restrict__ de) {
  const int b = blockIdx.x;
  for (int c = threadIdx.x; c < 2 * H; c += NT) {
    const float g = dx[(long long)b * 2 * H + c] * k3m_dropout_scale(seed, off + (uint64_t)b * 2 * H + c, p);
    if (c < H)
      de[(long long)b * H + c] = g;
    else
      de[(long long)(B + b) * H + (c - H)] = g;
  }
}

// one workgroup per pair row: tanh, dropout, the two logits, softmax, CE row loss, dlogits, du
__global__ __launch_bounds__(NT) void ce_rows_kernel(const float* __restrict__ u, const float* __restrict__ W,
                                                     const float* __restrict__ bias, const float* __restrict__ labels,
                                                     int B, int H, float p, uint64_t seed, uint64_t off,
                                                     float* __restrict__ logits, float* __restrict__ probs,
                                                     float* __restrict__ dlogits, float* __restrict__ loss_rows,
                                                     float* __restrict__ du) {
  __shared__ float red[NW];
  const int b = blockIdx.x;
  const float* ub = u + (long long)b * H;
  float a0 = 0.f, a1 = 0.f;
  for (int c = threadIdx.x; c < H; c += NT) {
    const float h = tanhf(ub[c]) * k3m_dropout_scale(seed, off + (uint64_t)b * H + c, p);
    a0 += h * W[c];
    a1 += h * W[H + c];
  }
  a0 = block_sum<NW>(a0, red);
  a1 = block_sum<NW>(a1, red);
  const float l0 = a0 + bias[0], l1 = a1 + bias[1];
  const float mx = fmaxf(l0, l1);
  const float lse = mx + logf(expf(l0 - mx) + expf(l1 - mx));
  const float p0 = expf(l0 - lse), p1 = expf(l1 - lse);
  const long long y = (long long)labels[b];   // labels.to(torch.long): truncation toward zero
  const bool ok = y == 0 || y == 1;
  const float inv_b = 1.f / (float)B;
  const float d0 = ok ? (p0 - (y == 0 ? 1.f : 0.f)) * inv_b : NAN;
  const float d1 = ok ? (p1 - (y == 1 ? 1.f : 0.f)) * inv_b : NAN;
  if (threadIdx.x == 0) {
    logits[2 * b] = l0;
    logits[2 * b + 1] = l1;
    probs[2 * b] = p0;
    probs[2 * b + 1] = p1;
    dlogits[2 * b] = d0;
    dlogits[2 * b + 1] = d1;
    loss_rows[b] = ok ? lse - (y == 0 ? l0 : l1) : NAN;
  }
  for (int c = threadIdx.x; c < H; c += NT) {
    const float t = tanhf(ub[c]);
    const float keep = k3m_dropout_scale(seed, off + (uint64_t)b * H + c, p);
    du[(long long)b * H + c] = (d0 * W[c] + d1 * W[H + c]) * keep * (1.f - t * t);
  }
}

// out_proj weight/bias gradients (accumulated) and the mean loss; one thread per hidden column
__global__ __launch_bounds__(NT) void ce_reduce_kernel(const float* __restrict__ u, const float* __restrict__ dlogits,
                                                       const float* __restrict__ loss_rows, int B, int H, float p,
                                                       uint64_t seed, uint64_t off, float* __restrict__ loss,
                                                       float* __restrict__ gW, float* __restrict__ gb) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c < H) {
    float g0 = 0.f, g1 = 0.f;
    for (int b = 0; b < B; ++b) {
      const float h = tanhf(u[(long long)b * H + c]) * k3m_dropout_scale(seed, off + (uint64_t)b * H + c, p);
      g0 += dlogits[2 * b] * h;
      g1 += dlogits[2 * b + 1] * h;
    }
    gW[c] += g0;
    gW[H + c] += g1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float s = 0.f, s0 = 0.f, s1 = 0.f;
    for (int b = 0; b < B; ++b) {
      s += loss_rows[b];
      s0 += dlogits[2 * b];
      s1 += dlogits[2 * b + 1];
    }
    loss[0] = s / (float)B;
    gb[0] += s0;
    gb[1] += s1;
  }
}

// CosineEmbeddingLoss (ATen cosine_embedding_loss: EPSILON 1e-12 added to the squared norms) and
// its gradient for both items; probs from cosine_similarity(e1, e1) (norms clamped at 1e-8)
__global__ __launch_bounds__(NT) void cosine_rows_kernel(const float* __restrict__ e, const float* __restrict__ labels,
                                                         int B, int H, float margin, float* __restrict__ probs,
                                                         float* __restrict__ loss_rows, float* __restrict__ de) {
  __shared__ float red[NW];
  const int b = blockIdx.x;
  const float* x1 = e + (long long)b * H;
  const float* x2 = e + (long long)(B + b) * H;
  float s12 = 0.f, s11 = 0.f, s22 = 0.f;
  for (int c = threadIdx.x; c < H; c += NT) {
    s12 += x1[c] * x2[c];
    s11 += x1[c] * x1[c];
    s22 += x2[c] * x2[c];
  }
  s12 = block_sum<NW>(s12, red);
  s11 = block_sum<NW>(s11, red);
  s22 = block_sum<NW>(s22, red);
  const float m1 = s11 + 1e-12f, m2 = s22 + 1e-12f;
  const float denom = sqrtf(m1 * m2);
  const float cs = s12 / denom;
  const float y = 2.f * labels[b] - 1.f;
  float l = 0.f, dl = 0.f;
  if (y == 1.f) {
    l = 1.f - cs;
    dl = -1.f;
  } else if (y == -1.f) {
    l = fmaxf(cs - margin, 0.f);
    dl = cs >= margin ? 1.f : 0.f;   // clamp_min passes the gradient at the boundary
  }
  dl *= 1.f / (float)B;
  const float n1 = fmaxf(sqrtf(s11), 1e-8f);
  if (threadIdx.x == 0) {
    loss_rows[b] = l;
    probs[b] = (s11 / (n1 * n1) + 1.f) * 0.5f;
  }
  for (int c = threadIdx.x; c < H; c += NT) {
    de[(long long)b * H + c] = dl * (x2[c] / denom - cs * x1[c] / m1);
    de[(long long)(B + b) * H + c] = dl * (x1[c] / denom - cs * x2[c] / m2);
  }
}

__global__ void mean_kernel(const float* __restrict__ rows, int n, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s += rows[i];
  out[0] = s / (float)n;
}

}  // namespace

extern "C" int k3m_align_pair_cat(const float* e, int B, int H, float p, uint64_t seed, uint64_t off, float* x,
                                  hipStream_t st) {
  K3M_ARG(e && x && B >= 0 && H > 0 && p >= 0.f && p < 1.f);
  if (B == 0) return 0;
  hipLaunchKernelGGL(pair_cat_kernel, dim3(B), dim3(NT), 0, st, e, B, H, p, seed, off, x);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_align_pair_cat_bwd(const float* dx, int B, int H, float p, uint64_t seed, uint64_t off, float* de,
                                      hipStream_t st) {
  K3M_ARG(dx && de && B >= 0 && H > 0 && p >= 0.f && p < 1.f);
  if (B == 0) return 0;
  hipLaunchKernelGGL(pair_cat_bwd_kernel, dim3(B), dim3(NT), 0, st, dx, B, H, p, seed, off, de);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_align_ce_fwd_bwd(const float* u, const float* W, const float* bias, const float* labels, int B,
                                    int H, float p, uint64_t seed, uint64_t off, float* logits, float* probs,
                                    float* dlogits, float* loss_rows, float* loss, float* du, float* gW, float* gb,
                                    hipStream_t st) {
  K3M_ARG(u && W && bias && labels && logits && probs && dlogits && loss_rows && loss && du && gW && gb);
  K3M_ARG(B > 0 && H > 0 && p >= 0.f && p < 1.f);
  hipLaunchKernelGGL(ce_rows_kernel, dim3(B), dim3(NT), 0, st, u, W, bias, labels, B, H, p, seed, off, logits, probs,
                     dlogits, loss_rows, du);
  K3M_CHECK_LAUNCH();
  hipLaunchKernelGGL(ce_reduce_kernel, dim3((H + NT - 1) / NT), dim3(NT), 0, st, u, dlogits, loss_rows, B, H, p, seed,
                     off, loss, gW, gb);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_align_cosine_fwd_bwd(const float* e, const float* labels, int B, int H, float margin, float* loss,
                                        float* probs, float* loss_rows, float* de, hipStream_t st) {
  K3M_ARG(e && labels && loss && probs && loss_rows && de && B > 0 && H > 0);
  hipLaunchKernelGGL(cosine_rows_kernel, dim3(B), dim3(NT), 0, st, e, labels, B, H, margin, probs, loss_rows, de);
  K3M_CHECK_LAUNCH();
  hipLaunchKernelGGL(mean_kernel, dim3(1), dim3(64), 0, st, loss_rows, B, loss);
  K3M_CHECK_LAUNCH();
  return 0;
}
