// Exact-fp32 attention for sequences longer than 128 (the fine-tuning PV text: max_seq_length_pv
// 256, finetune.py:1275 / run_finetune_item_alignment.sh; SURVEY §8(d) config 5: P = 320), up to
// 512 keys and head dim 128.  The whole-head-in-LDS kernels of attention.hip stop at 128 rows; here
// the query rows are blocked and K / V stream through LDS in 128-row chunks.
//
//   forward      workgroup per (sequence, head, 32 query rows): S = Q K^T (chunks) -> softmax ->
//                probabilities saved -> dropout -> O = Pd V (chunks)
//   backward A   workgroup per (sequence, head, 32 query rows): D = rowsum(dO * O),
//                dS = P * (drop * (dO V^T) - D) (chunks; dS also written to a workspace),
//                dQ = scale * dS K (chunks)
//   backward B   workgroup per (sequence, head, 64 key rows): dV = Pd^T dO, dK = scale * dS^T Q,
//                streaming the query rows in 128-row chunks
//
// Same semantics, dropout counters (element (s, h, i, j) at off + ((s*nh + h)*lq + i)*lk + j) and
// probability layout as attention.hip, so the two paths are interchangeable.  MFMA: 32x32x2 f32;
// LDS images use attention.hip's swizzle (element (i, c) at i*cols + (c ^ (i & 31))).
#include "common.h"

namespace {

constexpr int NT = 256;          // 4 waves
constexpr int NW = NT / 64;
constexpr int QB = 32;           // query rows per forward / backward-A workgroup
constexpr int KB = 64;           // key rows per backward-B workgroup
constexpr int CH = 128;          // rows per streamed chunk
constexpr int MAXLK = 512;
constexpr int MAXD = 128;

__device__ __forceinline__ int sw(int i, int c, int cols) { return i * cols + (c ^ (i & 31)); }

// rows [row0, row0 + nrows) of a [*, ld] matrix, columns [coff, coff + cols) -> swizzled fp32 image;
// rows >= nvalid are zero.  16-B vector loads (4 fp32 / 8 bf16).
template <typename T>
__device__ __forceinline__ void stage(float* __restrict__ dst, const T* __restrict__ src, long long row0, long long ld,
                                      int coff, int nrows, int nvalid, int cols) {
  constexpr int VE = 16 / sizeof(T);
  const int cpr = cols / VE, nch = nrows * cpr;
  for (int e = threadIdx.x; e < nch; e += NT) {
    const int i = e / cpr, c = (e - i * cpr) * VE;
    uint4 r = make_uint4(0u, 0u, 0u, 0u);
    if (i < nvalid) r = *reinterpret_cast<const uint4*>(src + (row0 + i) * ld + coff + c);
    const uint32_t w4[4] = {r.x, r.y, r.z, r.w};
    if constexpr (VE == 8) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        dst[sw(i, c + 2 * q, cols)] = __uint_as_float(w4[q] << 16);
        dst[sw(i, c + 2 * q + 1, cols)] = __uint_as_float(w4[q] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[sw(i, c + q, cols)] = __uint_as_float(w4[q]);
    }
  }
}

__device__ __forceinline__ int acc_row(int r, int kl) { return (r & 3) + 8 * (r >> 2) + 4 * kl; }

// ------------------------------------------------------------------ forward
template <typename T>
__global__ __launch_bounds__(NT) void long_fwd_kernel(const T* __restrict__ q, long long ldq, const T* __restrict__ k,
                                                      long long ldk, const T* __restrict__ v, long long ldv,
                                                      const float* __restrict__ kmask, T* __restrict__ ctx, long long ldc,
                                                      float* __restrict__ probs, int lq, int lk, int nh, int hd,
                                                      float scale, float p_drop, uint64_t seed, uint64_t off) {
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh, i0 = blockIdx.y * QB;
  const int LKP = (lk + CH - 1) / CH * CH;
  float* Qs = smem;                 // [QB][hd]
  float* Cs = Qs + QB * hd;         // [CH][hd]  K or V chunk
  float* Ss = Cs + CH * hd;         // [QB][LKP]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq + i0, krow0 = (long long)s * lk;
  const int hoff = h * hd, nq = min(QB, lq - i0);
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  stage<T>(Qs, q, qrow0, ldq, hoff, QB, nq, hd);
  for (int c0 = 0; c0 < LKP; c0 += CH) {
    __syncthreads();
    stage<T>(Cs, k, krow0 + c0, ldk, hoff, CH, min(CH, lk - c0), hd);
    __syncthreads();
    {  // wave w: key tile w of the chunk
      const int j0 = 32 * w;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      for (int kk = 0; kk < hd; kk += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Qs[sw(cl, kk + kl, hd)], Cs[sw(j0 + cl, kk + kl, hd)], acc, 0, 0, 0);
      const int j = c0 + j0 + cl;
      const float mj = j < lk ? (kmask ? kmask[krow0 + j] : 0.f) : -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) Ss[sw(acc_row(r, kl), j, LKP)] = acc[r] * scale + mj;
    }
  }
  __syncthreads();
  // softmax: a wave per row, lanes over the keys (<= 8 per lane)
  for (int i = w; i < QB; i += NW) {
    float x[MAXLK / 64];
    float mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < MAXLK / 64; ++u) {
      const int j = lane + 64 * u;
      x[u] = j < LKP ? Ss[sw(i, j, LKP)] : -INFINITY;
      mx = fmaxf(mx, x[u]);
    }
    mx = wave_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int u = 0; u < MAXLK / 64; ++u) {
      const int j = lane + 64 * u;
      x[u] = j < lk ? expf(x[u] - mx) : 0.f;
      sum += x[u];
    }
    const float inv = 1.f / wave_sum(sum);
    const bool act = i < nq;
    const long long prow = pbase + (long long)(i0 + i) * lk;
#pragma unroll
    for (int u = 0; u < MAXLK / 64; ++u) {
      const int j = lane + 64 * u;
      if (j < LKP) {
        float pd = 0.f;
        if (act && j < lk) {
          const float p = x[u] * inv;
          probs[prow + j] = p;
          pd = p * k3m_attn_dropout_scale(seed, p_drop, off, rbase + i0 + i, lk, j);
        }
        Ss[sw(i, j, LKP)] = pd;
      }
    }
  }
  // O = Pd V: wave w owns output column tile w (hd / 32 tiles)
  floatx16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  const int d0 = 32 * w;
  for (int c0 = 0; c0 < LKP; c0 += CH) {
    __syncthreads();
    stage<T>(Cs, v, krow0 + c0, ldv, hoff, CH, min(CH, lk - c0), hd);
    __syncthreads();
    if (d0 < hd)
      for (int kk = 0; kk < CH; kk += 2)
        o = __builtin_amdgcn_mfma_f32_32x32x2f32(Ss[sw(cl, c0 + kk + kl, LKP)], Cs[sw(kk + kl, d0 + cl, hd)], o, 0, 0, 0);
  }
  if (d0 < hd) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, kl);
      if (i < nq) ctx[(qrow0 + i) * ldc + hoff + d0 + cl] = from_f<T>(o[r]);
    }
  }
}

// ------------------------------------------------------------------ backward A: dS, dQ
template <typename T>
__global__ __launch_bounds__(NT) void long_bwd_q_kernel(const T* __restrict__ dctx, long long ldc,
                                                        const T* __restrict__ o, long long ldo, const T* __restrict__ k,
                                                        long long ldk, const T* __restrict__ v, long long ldv,
                                                        const float* __restrict__ probs, float* __restrict__ ds_ws,
                                                        T* __restrict__ dq, long long lddq, int lq, int lk, int nh,
                                                        int hd, float scale, float p_drop, uint64_t seed, uint64_t off) {
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh, i0 = blockIdx.y * QB;
  const int LKP = (lk + CH - 1) / CH * CH;
  float* R1 = smem;                 // [QB][hd] dO
  float* Cs = R1 + QB * hd;         // [CH][hd] V / K chunk
  float* Ss = Cs + CH * hd;         // [QB][LKP] dS
  float* Ds = Ss + QB * LKP;        // [QB] rowsum(dO * O)  (dynamic: the kernel has no static LDS)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq + i0, krow0 = (long long)s * lk;
  const int hoff = h * hd, nq = min(QB, lq - i0);
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  stage<T>(R1, dctx, qrow0, ldc, hoff, QB, nq, hd);
  for (int i = w; i < QB; i += NW) {   // D_i = dO_i . O_i
    float a = 0.f;
    if (i < nq)
      for (int d = lane; d < hd; d += 64) a += to_f(dctx[(qrow0 + i) * ldc + hoff + d]) * to_f(o[(qrow0 + i) * ldo + hoff + d]);
    a = wave_sum(a);
    if (lane == 0) Ds[i] = a;
  }
  for (int c0 = 0; c0 < LKP; c0 += CH) {
    __syncthreads();
    stage<T>(Cs, v, krow0 + c0, ldv, hoff, CH, min(CH, lk - c0), hd);
    __syncthreads();
    const int j0 = 32 * w;
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    for (int kk = 0; kk < hd; kk += 2)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(R1[sw(cl, kk + kl, hd)], Cs[sw(j0 + cl, kk + kl, hd)], acc, 0, 0, 0);
    const int j = c0 + j0 + cl;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, kl);
      float ds = 0.f;
      if (i < nq && j < lk) {
        const long long pidx = pbase + (long long)(i0 + i) * lk + j;
        ds = probs[pidx] * (acc[r] * k3m_attn_dropout_scale(seed, p_drop, off, rbase + i0 + i, lk, j) - Ds[i]);
        ds_ws[pidx] = ds;
      }
      Ss[sw(i, j, LKP)] = ds;
    }
  }
  floatx16 g;
#pragma unroll
  for (int r = 0; r < 16; ++r) g[r] = 0.f;
  const int d0 = 32 * w;
  for (int c0 = 0; c0 < LKP; c0 += CH) {
    __syncthreads();
    stage<T>(Cs, k, krow0 + c0, ldk, hoff, CH, min(CH, lk - c0), hd);
    __syncthreads();
    if (d0 < hd)
      for (int kk = 0; kk < CH; kk += 2)
        g = __builtin_amdgcn_mfma_f32_32x32x2f32(Ss[sw(cl, c0 + kk + kl, LKP)], Cs[sw(kk + kl, d0 + cl, hd)], g, 0, 0, 0);
  }
  if (d0 < hd) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, kl);
      if (i < nq) dq[(qrow0 + i) * lddq + hoff + d0 + cl] = from_f<T>(g[r] * scale);
    }
  }
}

// ------------------------------------------------------------------ backward B: dV, dK
// Ps [CH q][KB k] (dropped probabilities, then dS), Xs [CH][hd] (dO, then Q); acc tiles: the KB x hd
// output in 32x32 tiles, wave w takes tiles w, w + 4, ...
template <typename T>
__global__ __launch_bounds__(NT) void long_bwd_kv_kernel(const T* __restrict__ dctx, long long ldc,
                                                         const T* __restrict__ q, long long ldq,
                                                         const float* __restrict__ probs,
                                                         const float* __restrict__ ds_ws, T* __restrict__ dk,
                                                         T* __restrict__ dv, long long lddk, long long lddv, int lq,
                                                         int lk, int nh, int hd, float scale, float p_drop,
                                                         uint64_t seed, uint64_t off) {
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh, j0b = blockIdx.y * KB;
  float* Ps = smem;              // [CH][KB]
  float* Xs = Ps + CH * KB;      // [CH][hd]
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow = (long long)s * lq, krow0 = (long long)s * lk + j0b;
  const int hoff = h * hd, nk = min(KB, lk - j0b);
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const int ntile = (KB / 32) * (hd / 32);   // <= 8: at most two per wave
  for (int pass = 0; pass < 2; ++pass) {     // 0: dV = Pd^T dO   1: dK = scale dS^T Q
    floatx16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    for (int c0 = 0; c0 < lq; c0 += CH) {
      const int nrow = min(CH, lq - c0);
      __syncthreads();
      stage<T>(Xs, pass == 0 ? dctx : q, qrow + c0, pass == 0 ? ldc : ldq, hoff, CH, nrow, hd);
      for (int e = threadIdx.x; e < CH * KB; e += NT) {
        const int i = e / KB, j = e - i * KB;
        float x = 0.f;
        if (i < nrow && j < nk) {
          const long long pidx = pbase + (long long)(c0 + i) * lk + j0b + j;
          x = pass == 0 ? probs[pidx] * k3m_attn_dropout_scale(seed, p_drop, off, rbase + c0 + i, lk, j0b + j) : ds_ws[pidx];
        }
        Ps[sw(i, j, KB)] = x;
      }
      __syncthreads();
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int tile = w + NW * t;
        if (tile < ntile) {
          const int jt = (tile / (hd / 32)) * 32, dt = (tile % (hd / 32)) * 32;
          for (int kk = 0; kk < CH; kk += 2)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(Ps[sw(kk + kl, jt + cl, KB)], Xs[sw(kk + kl, dt + cl, hd)],
                                                          acc[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int tile = w + NW * t;
      if (tile < ntile) {
        const int jt = (tile / (hd / 32)) * 32, dt = (tile % (hd / 32)) * 32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = jt + acc_row(r, kl);
          if (j < nk) {
            if (pass == 0) dv[(krow0 + j) * lddv + hoff + dt + cl] = from_f<T>(acc[t][r]);
            else dk[(krow0 + j) * lddk + hoff + dt + cl] = from_f<T>(acc[t][r] * scale);
          }
        }
      }
    }
  }
}

size_t lds_q(int lk, int hd) {
  const size_t LKP = (lk + CH - 1) / CH * CH;
  return sizeof(float) * (QB * hd + CH * hd + QB * LKP);
}
size_t lds_kv(int hd) { return sizeof(float) * (CH * KB + CH * hd); }

bool vec_ok(const void* p, long long ld, int dtype) {
  const int ve = dtype == K3M_BF16 ? 8 : 4;
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % ve == 0;
}

template <typename T>
void set_attrs() {
  static bool done = false;
  if (!done) {
    const int mx = 160 * 1024;
    (void)hipFuncSetAttribute((const void*)long_fwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void*)long_bwd_q_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void*)long_bwd_kv_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    done = true;
  }
}

}  // namespace

extern "C" int k3m_attn_long_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                                 long long ldv, const float* kmask, void* ctx, long long ldc, float* probs, int nseq,
                                 int lq, int lk, int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off,
                                 int dtype, hipStream_t st) {
  K3M_ARG(q && k && v && ctx && probs && nh > 0 && nseq >= 0);
  K3M_ARG(lq > 0 && lk > 0 && lk <= MAXLK && hd > 0 && hd <= MAXD && hd % 32 == 0);
  K3M_ARG(dtype == K3M_F32 || dtype == K3M_BF16);
  K3M_ARG(vec_ok(q, ldq, dtype) && vec_ok(k, ldk, dtype) && vec_ok(v, ldv, dtype));
  if (nseq == 0) return 0;
  const dim3 grid(nseq * nh, (lq + QB - 1) / QB);
  const size_t lds = lds_q(lk, hd);
  if (dtype == K3M_F32) {
    set_attrs<float>();
    hipLaunchKernelGGL(long_fwd_kernel<float>, grid, dim3(NT), lds, st, (const float*)q, ldq, (const float*)k, ldk,
                       (const float*)v, ldv, kmask, (float*)ctx, ldc, probs, lq, lk, nh, hd, scale, p_drop, seed, off);
  } else {
    set_attrs<bf16_t>();
    hipLaunchKernelGGL(long_fwd_kernel<bf16_t>, grid, dim3(NT), lds, st, (const bf16_t*)q, ldq, (const bf16_t*)k, ldk,
                       (const bf16_t*)v, ldv, kmask, (bf16_t*)ctx, ldc, probs, lq, lk, nh, hd, scale, p_drop, seed,
                       off);
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_attn_long_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q,
                                 long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                                 const float* probs, float* ds_ws, void* dq, void* dk, void* dv, long long lddq,
                                 long long lddk, long long lddv, int nseq, int lq, int lk, int nh, int hd, float scale,
                                 float p_drop, uint64_t seed, uint64_t off, int dtype, hipStream_t st) {
  K3M_ARG(dctx && o && q && k && v && probs && ds_ws && dq && dk && dv && nh > 0 && nseq >= 0);
  K3M_ARG(lq > 0 && lk > 0 && lk <= MAXLK && hd > 0 && hd <= MAXD && hd % 32 == 0);
  K3M_ARG(dtype == K3M_F32 || dtype == K3M_BF16);
  K3M_ARG(vec_ok(q, ldq, dtype) && vec_ok(k, ldk, dtype) && vec_ok(v, ldv, dtype) && vec_ok(dctx, ldc, dtype));
  if (nseq == 0) return 0;
  const dim3 gq(nseq * nh, (lq + QB - 1) / QB), gk(nseq * nh, (lk + KB - 1) / KB);
  if (dtype == K3M_F32) {
    set_attrs<float>();
    hipLaunchKernelGGL(long_bwd_q_kernel<float>, gq, dim3(NT), lds_q(lk, hd) + QB * sizeof(float), st, (const float*)dctx, ldc,
                       (const float*)o, ldo, (const float*)k, ldk, (const float*)v, ldv, probs, ds_ws, (float*)dq, lddq,
                       lq, lk, nh, hd, scale, p_drop, seed, off);
    K3M_CHECK_LAUNCH();
    hipLaunchKernelGGL(long_bwd_kv_kernel<float>, gk, dim3(NT), lds_kv(hd), st, (const float*)dctx, ldc,
                       (const float*)q, ldq, probs, ds_ws, (float*)dk, (float*)dv, lddk, lddv, lq, lk, nh, hd, scale,
                       p_drop, seed, off);
  } else {
    set_attrs<bf16_t>();
    hipLaunchKernelGGL(long_bwd_q_kernel<bf16_t>, gq, dim3(NT), lds_q(lk, hd) + QB * sizeof(float), st, (const bf16_t*)dctx, ldc,
                       (const bf16_t*)o, ldo, (const bf16_t*)k, ldk, (const bf16_t*)v, ldv, probs, ds_ws, (bf16_t*)dq,
                       lddq, lq, lk, nh, hd, scale, p_drop, seed, off);
    K3M_CHECK_LAUNCH();
    hipLaunchKernelGGL(long_bwd_kv_kernel<bf16_t>, gk, dim3(NT), lds_kv(hd), st, (const bf16_t*)dctx, ldc,
                       (const bf16_t*)q, ldq, probs, ds_ws, (bf16_t*)dk, (bf16_t*)dv, lddk, lddv, lq, lk, nh, hd, scale,
                       p_drop, seed, off);
  }
  K3M_CHECK_LAUNCH();
  return 0;
}
