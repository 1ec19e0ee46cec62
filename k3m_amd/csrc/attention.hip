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

// Backward on the matrix cores (v_mfma_f32_32x32x2_f32), one workgroup per (sequence, head),
// every operand LDS-resident, sequence lengths padded to multiples of 32 with zeros:
//   D_i  = dO_i . O_i                      (= sum_j P_ij dP_ij, no cross-key reduction needed)
//   dS   = P * (dropmask * (dO V^T) - D)   phase 1, kept in LDS
//   dQ   = scale * dS K                    phase 2
//   dK   = scale * dS^T Q ; dV = Pd^T dO   phase 3 (Pd = P * dropmask read straight from HBM)
// 32x32x2 operand maps: lane l holds A[l&31][kk + (l>>5)] and B[kk + (l>>5)][l&31]; the 16
// accumulators of lane l sit at row (r&3) + 8(r>>2) + 4(l>>5), column l&31.
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const T* __restrict__ dctx, long long ldc,
                                                       const T* __restrict__ o, long long ldo,
                                                       const T* __restrict__ q, long long ldq, const T* __restrict__ k,
                                                       long long ldk, const T* __restrict__ v, long long ldv,
                                                       const float* __restrict__ probs, T* __restrict__ dq,
                                                       T* __restrict__ dk, T* __restrict__ dv, long long lddq,
                                                       long long lddk, long long lddv, int lq, int lk, int nh, int hd,
                                                       float scale, float p_drop, uint64_t seed, uint64_t off) {
  extern __shared__ float smem[];
  const int sh = blockIdx.x;
  const int s = sh / nh, h = sh % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const int hp = hd + 1, lkp = LK + 1;
  const bool q_in_lds = LQ <= LK;
  float* dOs = smem;                    // [LQ][hd+1]
  float* Xs = dOs + LQ * hp;            // [LK][hd+1]: V, then K, then Q (if LQ <= LK)
  float* dS = Xs + LK * hp;             // [LQ][LK+1]
  float* Ds = dS + LQ * lkp;            // [LQ]
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int cl = lane & 31, kl = lane >> 5;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * hd;

  // phase 0: stage dO and V, D_i = dO_i . O_i
  for (int e = tid; e < LQ * hd; e += 256) {
    const int i = e / hd, d = e % hd;
    dOs[i * hp + d] = i < lq ? to_f(dctx[(qrow0 + i) * ldc + hoff + d]) : 0.f;
  }
  for (int e = tid; e < LK * hd; e += 256) {
    const int j = e / hd, d = e % hd;
    Xs[j * hp + d] = j < lk ? to_f(v[(krow0 + j) * ldv + hoff + d]) : 0.f;
  }
  for (int i = w; i < LQ; i += 4) {
    float a = 0.f;
    if (i < lq)
      for (int d = lane; d < hd; d += 64) a += to_f(dctx[(qrow0 + i) * ldc + hoff + d]) * to_f(o[(qrow0 + i) * ldo + hoff + d]);
    a = wave_sum(a);
    if (lane == 0) Ds[i] = a;
  }
  __syncthreads();

  // phase 1: dS tiles [32 x 32] over (LQ/32) x (LK/32)
  {
    const int tq = LQ >> 5, tk = LK >> 5;
    for (int t = w; t < tq * tk; t += 4) {
      const int i0 = (t / tk) * 32, j0 = (t % tk) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      for (int kk = 0; kk < hd; kk += 2) {
        const float a = dOs[(i0 + cl) * hp + kk + kl];
        const float b = Xs[(j0 + cl) * hp + kk + kl];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
      const int j = j0 + cl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        float ds = 0.f;
        if (i < lq && j < lk) {
          const long long pidx = pbase + (long long)i * lk + j;
          ds = probs[pidx] * (acc[r] * k3m_dropout_scale(seed, off + pidx, p_drop) - Ds[i]);
        }
        dS[i * lkp + j] = ds;
      }
    }
  }
  __syncthreads();
  // phase 2: K -> Xs; dQ = scale * dS K
  for (int e = tid; e < LK * hd; e += 256) {
    const int j = e / hd, d = e % hd;
    Xs[j * hp + d] = j < lk ? to_f(k[(krow0 + j) * ldk + hoff + d]) : 0.f;
  }
  __syncthreads();
  {
    const int tq = LQ >> 5, td = hd >> 5;
    for (int t = w; t < tq * td; t += 4) {
      const int i0 = (t / td) * 32, d0 = (t % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      for (int kk = 0; kk < LK; kk += 2) {
        const float a = dS[(i0 + cl) * lkp + kk + kl];
        const float b = Xs[(kk + kl) * hp + d0 + cl];
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (i < lq) dq[(qrow0 + i) * lddq + hoff + d0 + cl] = from_f<T>(acc[r] * scale);
      }
    }
  }
  __syncthreads();
  // phase 3: Q -> Xs (when it fits); dK = scale * dS^T Q ; dV = Pd^T dO
  if (q_in_lds) {
    for (int e = tid; e < LQ * hd; e += 256) {
      const int i = e / hd, d = e % hd;
      Xs[i * hp + d] = i < lq ? to_f(q[(qrow0 + i) * ldq + hoff + d]) : 0.f;
    }
  }
  __syncthreads();
  {
    const int tk = LK >> 5, td = hd >> 5;
    for (int t = w; t < 2 * tk * td; t += 4) {
      const bool is_v = t >= tk * td;
      const int tt = is_v ? t - tk * td : t;
      const int j0 = (tt / td) * 32, d0 = (tt % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int j = j0 + cl;
      for (int kk = 0; kk < LQ; kk += 2) {
        const int i = kk + kl;
        float a, b;
        if (!is_v) {
          a = dS[i * lkp + j];
          if (q_in_lds) b = Xs[i * hp + d0 + cl];
          else b = i < lq ? to_f(q[(qrow0 + i) * ldq + hoff + d0 + cl]) : 0.f;
        } else {
          a = 0.f;
          if (i < lq && j < lk) {
            const long long pidx = pbase + (long long)i * lk + j;
            a = probs[pidx] * k3m_dropout_scale(seed, off + pidx, p_drop);
          }
          b = dOs[i * hp + d0 + cl];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jr = j0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (jr < lk) {
          if (is_v) dv[(krow0 + jr) * lddv + hoff + d0 + cl] = from_f<T>(acc[r]);
          else dk[(krow0 + jr) * lddk + hoff + d0 + cl] = from_f<T>(acc[r] * scale);
        }
      }
    }
  }
}

size_t fwd_lds(int lk, int hd) { return sizeof(float) * ((size_t)lk * (hd + 1) + (size_t)lk * hd + MAXL + 4 * MAXD + 4 * MAXL); }
size_t bwd_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  return sizeof(float) * (LQ * (hd + 1) + LK * (hd + 1) + LQ * (LK + 1) + LQ);
}

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

extern "C" int k3m_attn_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                            const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq,
                            void* dk, void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk,
                            int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype,
                            hipStream_t st) {
  K3M_ARG(dctx && o && q && k && v && probs && dq && dk && dv);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && hd > 0 && hd <= MAXD && hd % 32 == 0 && nh > 0);
  if (nseq == 0) return 0;
  const size_t lds = bwd_lds(lq, lk, hd);
  K3M_ARG(lds <= 160 * 1024);
  if (dtype == K3M_F32) {
    set_lds_attr<float>();
    hipLaunchKernelGGL(attn_bwd_kernel<float>, dim3(nseq * nh), dim3(256), lds, st, (const float*)dctx, ldc,
                       (const float*)o, ldo, (const float*)q, ldq, (const float*)k, ldk, (const float*)v, ldv, probs,
                       (float*)dq, (float*)dk, (float*)dv, lddq, lddk, lddv, lq, lk, nh, hd, scale, p_drop, seed, off);
  } else if (dtype == K3M_BF16) {
    set_lds_attr<bf16_t>();
    hipLaunchKernelGGL(attn_bwd_kernel<bf16_t>, dim3(nseq * nh), dim3(256), lds, st, (const bf16_t*)dctx, ldc,
                       (const bf16_t*)o, ldo, (const bf16_t*)q, ldq, (const bf16_t*)k, ldk, (const bf16_t*)v, ldv,
                       probs, (bf16_t*)dq, (bf16_t*)dk, (bf16_t*)dv, lddq, lddk, lddv, lq, lk, nh, hd, scale, p_drop,
                       seed, off);
  } else {
    return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}
