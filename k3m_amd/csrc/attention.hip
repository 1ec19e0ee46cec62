// Fused multi-head attention for the short K3M sequences (L <= 128): one workgroup per
// (sequence, head); the head's K and V live in LDS for the whole workgroup, each wave owns query
// rows, the softmax row stays in registers (lane = key) and P.V runs with lane = head channel.
// Scores never touch HBM except the softmax probabilities saved for the backward pass.
//
// Reference semantics (vilbert_k3m.py:449-464, :608-623, :786-824): scores = q.k^T * scale + mask,
// softmax over keys, dropout on the probabilities, context = P.V, heads concatenated along the
// hidden dimension.
#include "common.h"

namespace {

constexpr int MAXL = 128;  // keys per sequence (2 per lane)
constexpr int MAXD = 128;  // head dim (2 per lane)

template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const T* __restrict__ q, long long ldq, const T* __restrict__ k,
                                                       long long ldk, const T* __restrict__ v, long long ldv,
                                                       const float* __restrict__ kmask, T* __restrict__ ctx,
                                                       long long ldc, float* __restrict__ probs, int lq, int lk,
                                                       int nh, int hd, float scale, float p_drop, uint64_t seed,
                                                       uint64_t off) {
  extern __shared__ float smem[];
  const int sh = blockIdx.x;
  const int s = sh / nh, h = sh % nh;
  const int hp = hd + 1;
  float* Ks = smem;                 // [lk][hd+1]
  float* Vs = Ks + lk * hp;         // [lk][hd]
  float* Ms = Vs + lk * hd;         // [lk]
  float* Qs = Ms + MAXL;            // [4][MAXD]
  float* Ps = Qs + 4 * MAXD;        // [4][MAXL]
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int e = tid; e < lk * hd; e += 256) {
    const int j = e / hd, d = e % hd;
    Ks[j * hp + d] = to_f(k[((long long)s * lk + j) * ldk + h * hd + d]);
    Vs[j * hd + d] = to_f(v[((long long)s * lk + j) * ldv + h * hd + d]);
  }
  for (int j = tid; j < lk; j += 256) Ms[j] = kmask ? kmask[(long long)s * lk + j] : 0.f;
  __syncthreads();
  float* qs = Qs + w * MAXD;
  float* ps = Ps + w * MAXL;
  for (int i0 = 0; i0 < lq; i0 += 4) {  // block-uniform trip count (barriers inside)
    const int i = i0 + w;
    const bool act = i < lq;
    const long long qrow = ((long long)s * lq + (act ? i : 0));
    if (act)
      for (int d = lane; d < hd; d += 64) qs[d] = to_f(q[qrow * ldq + h * hd + d]) * scale;
    __syncthreads();
    float sc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = lane + 64 * t;
      float a = -INFINITY;
      if (j < lk) {
        a = 0.f;
        const float* kr = Ks + j * hp;
        for (int d = 0; d < hd; ++d) a += qs[d] * kr[d];
        a += Ms[j];
      }
      sc[t] = a;
    }
    const float mx = wave_max(fmaxf(sc[0], sc[1]));
    float e0 = (lane < lk) ? expf(sc[0] - mx) : 0.f;
    float e1 = (lane + 64 < lk) ? expf(sc[1] - mx) : 0.f;
    const float inv = 1.f / wave_sum(e0 + e1);
    e0 *= inv;
    e1 *= inv;
    const long long prow = (((long long)s * nh + h) * lq + i) * lk;
    if (act && lane < lk) {
      probs[prow + lane] = e0;
      ps[lane] = e0 * k3m_dropout_scale(seed, off + prow + lane, p_drop);
    }
    if (act && lane + 64 < lk) {
      probs[prow + lane + 64] = e1;
      ps[lane + 64] = e1 * k3m_dropout_scale(seed, off + prow + lane + 64, p_drop);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int d = lane + 64 * t;
      if (act && d < hd) {
        float a = 0.f;
        for (int j = 0; j < lk; ++j) a += ps[j] * Vs[j * hd + d];
        ctx[qrow * ldc + h * hd + d] = from_f<T>(a);
      }
    }
    __syncthreads();
  }
}

// Backward.  Pass 1 (wave per query row i): dPd_ij = dctx_i.V_j; dP = dPd*dropmask;
// dS_ij = P_ij (dP_ij - sum_j P_ij dP_ij); dQ_i = scale * sum_j dS_ij K_j; dS kept in LDS.
// Pass 2 (wave per key row j): dK_j = scale * sum_i dS_ij Q_i; dV_j = sum_i Pd_ij dctx_i.
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const T* __restrict__ dctx, long long ldc, const T* __restrict__ q,
                                                       long long ldq, const T* __restrict__ k, long long ldk,
                                                       const T* __restrict__ v, long long ldv,
                                                       const float* __restrict__ probs, T* __restrict__ dq,
                                                       T* __restrict__ dk, T* __restrict__ dv, long long lddq,
                                                       long long lddk, long long lddv, int lq, int lk, int nh, int hd,
                                                       float scale, float p_drop, uint64_t seed, uint64_t off) {
  extern __shared__ float smem[];
  const int sh = blockIdx.x;
  const int s = sh / nh, h = sh % nh;
  const int hp = hd + 1, lkp = lk + 1;
  float* Vs = smem;                  // [lk][hd+1]
  float* dS = Vs + lk * hp;          // [lq][lk+1]
  float* Gs = dS + lq * lkp;         // [4][MAXD] dctx row scratch
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  for (int e = tid; e < lk * hd; e += 256) {
    const int j = e / hd, d = e % hd;
    Vs[j * hp + d] = to_f(v[((long long)s * lk + j) * ldv + h * hd + d]);
  }
  __syncthreads();
  float* gs = Gs + w * MAXD;
  for (int i0 = 0; i0 < lq; i0 += 4) {  // block-uniform trip count (barriers inside)
    const int i = i0 + w;
    const bool act = i < lq;
    const long long qrow = (long long)s * lq + (act ? i : 0);
    if (act)
      for (int d = lane; d < hd; d += 64) gs[d] = to_f(dctx[qrow * ldc + h * hd + d]);
    __syncthreads();
    const long long prow = (((long long)s * nh + h) * lq + i) * lk;
    float pv[2], dp[2];
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = lane + 64 * t;
      pv[t] = 0.f;
      dp[t] = 0.f;
      if (act && j < lk) {
        float a = 0.f;
        const float* vr = Vs + j * hp;
        for (int d = 0; d < hd; ++d) a += gs[d] * vr[d];
        a *= k3m_dropout_scale(seed, off + prow + j, p_drop);
        pv[t] = probs[prow + j];
        dp[t] = a;
        dot += pv[t] * a;
      }
    }
    dot = wave_sum(dot);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int j = lane + 64 * t;
      if (act && j < lk) dS[i * lkp + j] = pv[t] * (dp[t] - dot);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int d = lane + 64 * t;
      if (act && d < hd) {
        float a = 0.f;
        for (int j = 0; j < lk; ++j) a += dS[i * lkp + j] * to_f(k[((long long)s * lk + j) * ldk + h * hd + d]);
        dq[qrow * lddq + h * hd + d] = from_f<T>(a * scale);
      }
    }
    __syncthreads();
  }
  __syncthreads();
  for (int j = w; j < lk; j += 4) {
    float ak[2] = {0.f, 0.f}, av[2] = {0.f, 0.f};
    for (int i = 0; i < lq; ++i) {
      const long long qrow = (long long)s * lq + i;
      const long long pidx = (((long long)s * nh + h) * lq + i) * lk + j;
      const float ds = dS[i * lkp + j];
      const float pd = probs[pidx] * k3m_dropout_scale(seed, off + pidx, p_drop);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int d = lane + 64 * t;
        if (d < hd) {
          ak[t] += ds * to_f(q[qrow * ldq + h * hd + d]);
          av[t] += pd * to_f(dctx[qrow * ldc + h * hd + d]);
        }
      }
    }
    const long long krow = (long long)s * lk + j;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int d = lane + 64 * t;
      if (d < hd) {
        dk[krow * lddk + h * hd + d] = from_f<T>(ak[t] * scale);
        dv[krow * lddv + h * hd + d] = from_f<T>(av[t]);
      }
    }
  }
}

size_t fwd_lds(int lk, int hd) { return sizeof(float) * ((size_t)lk * (hd + 1) + (size_t)lk * hd + MAXL + 4 * MAXD + 4 * MAXL); }
size_t bwd_lds(int lq, int lk, int hd) { return sizeof(float) * ((size_t)lk * (hd + 1) + (size_t)lq * (lk + 1) + 4 * MAXD); }

template <typename T>
void set_lds_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    done = true;
  }
}

}  // namespace

extern "C" int k3m_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                            const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk,
                            int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype,
                            hipStream_t st) {
  K3M_ARG(q && k && v && ctx && probs);
  K3M_ARG(lq > 0 && lk > 0 && lk <= MAXL && hd > 0 && hd <= MAXD && nh > 0);
  if (nseq == 0) return 0;
  const size_t lds = fwd_lds(lk, hd);
  K3M_ARG(lds <= 160 * 1024);
  if (dtype == K3M_F32) {
    set_lds_attr<float>();
    hipLaunchKernelGGL(attn_fwd_kernel<float>, dim3(nseq * nh), dim3(256), lds, st, (const float*)q, ldq,
                       (const float*)k, ldk, (const float*)v, ldv, kmask, (float*)ctx, ldc, probs, lq, lk, nh, hd,
                       scale, p_drop, seed, off);
  } else if (dtype == K3M_BF16) {
    set_lds_attr<bf16_t>();
    hipLaunchKernelGGL(attn_fwd_kernel<bf16_t>, dim3(nseq * nh), dim3(256), lds, st, (const bf16_t*)q, ldq,
                       (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, kmask, (bf16_t*)ctx, ldc, probs, lq, lk, nh, hd,
                       scale, p_drop, seed, off);
  } else {
    return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_attn_bwd(const void* dctx, long long ldc, const void* q, long long ldq, const void* k, long long ldk,
                            const void* v, long long ldv, const float* probs, void* dq, void* dk, void* dv,
                            long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk, int nh, int hd,
                            float scale, float p_drop, uint64_t seed, uint64_t off, int dtype, hipStream_t st) {
  K3M_ARG(dctx && q && k && v && probs && dq && dk && dv);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && hd > 0 && hd <= MAXD && nh > 0);
  if (nseq == 0) return 0;
  const size_t lds = bwd_lds(lq, lk, hd);
  K3M_ARG(lds <= 160 * 1024);
  if (dtype == K3M_F32) {
    set_lds_attr<float>();
    hipLaunchKernelGGL(attn_bwd_kernel<float>, dim3(nseq * nh), dim3(256), lds, st, (const float*)dctx, ldc,
                       (const float*)q, ldq, (const float*)k, ldk, (const float*)v, ldv, probs, (float*)dq, (float*)dk,
                       (float*)dv, lddq, lddk, lddv, lq, lk, nh, hd, scale, p_drop, seed, off);
  } else if (dtype == K3M_BF16) {
    set_lds_attr<bf16_t>();
    hipLaunchKernelGGL(attn_bwd_kernel<bf16_t>, dim3(nseq * nh), dim3(256), lds, st, (const bf16_t*)dctx, ldc,
                       (const bf16_t*)q, ldq, (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, probs, (bf16_t*)dq,
                       (bf16_t*)dk, (bf16_t*)dv, lddq, lddk, lddv, lq, lk, nh, hd, scale, p_drop, seed, off);
  } else {
    return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}
