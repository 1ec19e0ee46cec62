// Fused multi-head attention for the short K3M sequences (L <= 128) on the matrix cores.
//
// One workgroup (8 waves) per (sequence, head).  Everything the head needs lives in LDS for the
// whole workgroup; sequence lengths are zero-padded to multiples of 32 and every product is a
// set of 32x32 tiles of v_mfma_f32_32x32x2_f32 (exact fp32).  Operand maps: lane l holds
// A[l&31][kk + (l>>5)] and B[kk + (l>>5)][l&31]; accumulator r of lane l is row
// (r&3) + 8(r>>2) + 4(l>>5), column l&31.
//
// LDS images are unpadded [rows][cols] with an XOR swizzle of the column by (row & 31):
// element (i, c) lives at i*cols + (c ^ (i & 31)).  Reads of 32 different rows at one column
// (A operands) and of 32 consecutive columns of one row (B operands, stores) are both
// conflict-free, and the largest case (L=128, d=64 backward: three 64 KiB images) fits in
// 160 KiB.
//
// Reference semantics (vilbert_k3m.py:449-464, :608-623, :786-824, :913-951): scores =
// q.k^T / sqrt(d) + additive key mask, softmax over keys, dropout on the probabilities,
// context = P.V, heads concatenated along the hidden dimension.
#include "common.h"

#include <cstdlib>

namespace {

constexpr int MAXL = 128;
constexpr int MAXD = 128;
constexpr float LOG2E = 1.4426950408889634f;
// Two builds of each kernel: (ML = 128, 8 waves) for any sequence up to 128, and (ML = 64, 4 waves)
// for sequences up to 64 (the text, image and text<->image co-attention cases: L = 36/37).  The
// short build's register arrays are sized for 64 rows, so it holds ~half the VGPRs and, with its
// <= 80 KB of LDS, two or three workgroups share a CU — the L <= 64 cases are latency-bound, and
// one 8-wave workgroup per CU left most of each block's global-load and barrier waits exposed.

__device__ __forceinline__ int sw(int i, int c, int cols) { return i * cols + (c ^ (i & 31)); }

// acc += sum_k A(k) B(k) over k in [0, K) for one 32x32 tile, K a multiple of 16: lane operands
// come from LDS through fa(k) / fb(k) (k already includes the lane's kl offset).  The next 16-wide
// k slice's eight A and eight B reads are issued before the current slice's eight MFMAs, so the
// LDS latency hides behind the matrix core instead of stalling every step.
template <int S = 8, typename FA, typename FB>
__device__ __forceinline__ void mfma_tile(floatx16& acc, int K, FA fa, FB fb) {
  static_assert(S == 4 || S == 8, "slice of 4 or 8 MFMA steps (K is a multiple of 16)");
  float a[S], b[S];
#pragma unroll
  for (int u = 0; u < S; ++u) {
    a[u] = fa(2 * u);
    b[u] = fb(2 * u);
  }
  for (int k0 = 0; k0 < K; k0 += 2 * S) {
    float an[S], bn[S];
    const int kn = k0 + 2 * S < K ? k0 + 2 * S : k0;  // last slice re-reads itself (unused, no branch)
#pragma unroll
    for (int u = 0; u < S; ++u) {
      an[u] = fa(kn + 2 * u);
      bn[u] = fb(kn + 2 * u);
    }
#pragma unroll
    for (int u = 0; u < S; ++u) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], b[u], acc, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < S; ++u) {
      a[u] = an[u];
      b[u] = bn[u];
    }
  }
}

// Phase timestamps for the lab build only (scripts/lab/attn_stamps.hip defines K3M_ATTN_STAMPS):
// wave 0 of each workgroup records the 100 MHz wall clock at the phase boundaries.
#ifdef K3M_ATTN_STAMPS
__device__ unsigned long long k3m_attn_stamps[K3M_ATTN_STAMPS * 8];
#define ATT_STAMP(n)                                                     \
  do {                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < K3M_ATTN_STAMPS)                \
      k3m_attn_stamps[blockIdx.x * 8 + (n)] = wall_clock64();            \
  } while (0)
#define ATT_STAMP_END(n) \
  do {                   \
    __syncthreads();     \
    ATT_STAMP(n);        \
  } while (0)
#else
#define ATT_STAMP(n) \
  do {               \
  } while (0)
#define ATT_STAMP_END(n) \
  do {                   \
  } while (0)
#endif

// Staging HBM -> LDS in two halves so the loads of the next operand can be issued before the
// current phase's MFMAs and written after its barrier: every thread loads its 16-byte chunks
// (8 bf16 / 4 fp32 of one row) into registers first — one HBM latency per operand, not one per
// element — then converts and writes them into the swizzled fp32 image (rows >= nvalid are zero).
template <typename T, int ML, int NTH>
struct Chunks {
  static constexpr int VE = 16 / sizeof(T);
  static constexpr int N = ML * MAXD / VE / NTH;  // chunks per thread for the largest tile
  uint4 r[N];
};

template <typename T, int ML, int NTH>
__device__ __forceinline__ void stage_load(Chunks<T, ML, NTH>& ch, const T* __restrict__ src, long long row0, long long ld,
                                           int coff, int nrows, int nvalid, int cols) {
  constexpr int VE = Chunks<T, ML, NTH>::VE;
  const int cpr = cols / VE, nch = nrows * cpr;
#pragma unroll
  for (int u = 0; u < Chunks<T, ML, NTH>::N; ++u) {
    const int e = threadIdx.x + u * NTH;
    ch.r[u] = make_uint4(0u, 0u, 0u, 0u);
    if (e < nch) {
      const int i = e / cpr, c = (e - i * cpr) * VE;
      if (i < nvalid) ch.r[u] = *reinterpret_cast<const uint4*>(src + (row0 + i) * ld + coff + c);
    }
  }
}

template <typename T, int ML, int NTH>
__device__ __forceinline__ void stage_store(float* __restrict__ dst, const Chunks<T, ML, NTH>& ch, int nrows, int cols) {
  constexpr int VE = Chunks<T, ML, NTH>::VE;
  const int cpr = cols / VE, nch = nrows * cpr;
#pragma unroll
  for (int u = 0; u < Chunks<T, ML, NTH>::N; ++u) {
    const int e = threadIdx.x + u * NTH;
    if (e < nch) {
      const int i = e / cpr, c = (e - i * cpr) * VE;
      const uint32_t w4[4] = {ch.r[u].x, ch.r[u].y, ch.r[u].z, ch.r[u].w};
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
}

template <typename T, int ML, int NTH>
__device__ __forceinline__ void stage(float* __restrict__ dst, const T* __restrict__ src, long long row0, long long ld,
                                      int coff, int nrows, int nvalid, int cols) {
  Chunks<T, ML, NTH> ch;
  stage_load(ch, src, row0, ld, coff, nrows, nvalid, cols);
  stage_store(dst, ch, nrows, cols);
}

// dst[e] = <chunk e of a, chunk e of b> for every staged chunk e (row-major, cols/VE per row)
template <typename T, int ML, int NTH>
__device__ __forceinline__ void chunk_dots(float* __restrict__ dst, const Chunks<T, ML, NTH>& a,
                                           const Chunks<T, ML, NTH>& b, int nrows, int cols) {
  constexpr int VE = Chunks<T, ML, NTH>::VE;
  const int nch = nrows * (cols / VE);
#pragma unroll
  for (int u = 0; u < Chunks<T, ML, NTH>::N; ++u) {
    const int e = threadIdx.x + u * NTH;
    if (e < nch) {
      const uint32_t wa[4] = {a.r[u].x, a.r[u].y, a.r[u].z, a.r[u].w};
      const uint32_t wb[4] = {b.r[u].x, b.r[u].y, b.r[u].z, b.r[u].w};
      float acc = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if constexpr (VE == 8) {
          acc += __uint_as_float(wa[q] << 16) * __uint_as_float(wb[q] << 16);
          acc += __uint_as_float(wa[q] & 0xffff0000u) * __uint_as_float(wb[q] & 0xffff0000u);
        } else {
          acc += __uint_as_float(wa[q]) * __uint_as_float(wb[q]);
        }
      }
      dst[e] = acc;
    }
  }
}

// ------------------------------------------------------------------ forward
template <typename T, int ML, int NW>
__global__ __launch_bounds__(NW * 64, ML == 64 ? 3 : 1) void attn_fwd_kernel(const T* __restrict__ q, long long ldq, const T* __restrict__ k,
                                                       long long ldk, const T* __restrict__ v, long long ldv,
                                                       const float* __restrict__ kmask, T* __restrict__ ctx,
                                                       long long ldc, float* __restrict__ probs, int lq, int lk,
                                                       int nh, int hd, float scale, float p_drop, uint64_t seed,
                                                       uint64_t off) {
  constexpr int NTH = NW * 64;
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  float* Qs = smem;              // [LQ][hd]
  float* KVs = Qs + LQ * hd;     // [LK][hd]  K, then V
  float* Ss = KVs + LK * hd;     // [LQ][LK]  scores, then dropped probabilities
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row math on the scalar unit
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * hd;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  ATT_STAMP(0);

  // additive key mask of the lane's key column in each 32-column tile (-inf on padding columns),
  // loaded with Q and K: a load after the MFMAs would make the S phase wait for V's loads too
  // (clamped addresses and no use before the S phase: the loads are issued unconditionally)
  float mk[ML / 32];
#pragma unroll
  for (int t = 0; t < ML / 32; ++t) mk[t] = 0.f;
  if (kmask) {
#pragma unroll
    for (int t = 0; t < ML / 32; ++t) mk[t] = kmask[krow0 + min(32 * t + cl, lk - 1)];
  }
  {  // Q's and K's loads are issued together: one exposed global latency, not two
    Chunks<T, ML, NTH> qch, kch;
    stage_load(qch, q, qrow0, ldq, hoff, LQ, lq, hd);
    stage_load(kch, k, krow0, ldk, hoff, LK, lk, hd);
    stage_store(Qs, qch, LQ, hd);
    stage_store(KVs, kch, LK, hd);
  }
  __syncthreads();
  ATT_STAMP(1);
  Chunks<T, ML, NTH> vch;  // V's loads fly while S is computed
  stage_load(vch, v, krow0, ldv, hoff, LK, lk, hd);
  // S = scale * Q K^T + mask
  {
    const int tq = LQ >> 5, tk = LK >> 5;
    for (int t = w; t < tq * tk; t += NW) {
      const int i0 = (t / tk) * 32, j0 = (t % tk) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile(acc, hd, [&](int kk) { return Qs[sw(i0 + cl, kk + kl, hd)]; },
                [&](int kk) { return KVs[sw(j0 + cl, kk + kl, hd)]; });
      const int j = j0 + cl;
      const float mj = j < lk ? mk[j0 >> 5] * LOG2E : -INFINITY;
      const float sl = scale * LOG2E;   // scores kept in log2 units: softmax uses exp2
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        Ss[sw(i, j, LK)] = acc[r] * sl + mj;
      }
    }
  }
  __syncthreads();
  ATT_STAMP(2);
  stage_store(KVs, vch, LK, hd);  // K no longer needed
  // softmax rows (wave per row, lanes over keys), dropout, save P.  A wave takes its rows in
  // groups of G: the G reductions are independent shuffle chains that overlap.  Rows >= lq (the
  // zero-padded queries) are skipped: their S rows stay as they are, and the PV rows they feed
  // are never stored.
  ATT_STAMP(3);
  {
    constexpr int RW = ML / NW, G = 4;
    constexpr bool TWO = ML > 64;   // keys lane + 64 exist only in the 128-row build
    const K3mDrop dr = k3m_drop_init(seed, p_drop);
    for (int g = 0; g < RW; g += G) {
      if (w + g * NW >= lq) break;   // wave-uniform
      float x0[G], x1[G], mx[G], sm[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int i = min(w + (g + u) * NW, LQ - 1);   // rows past lq: computed, never stored
        x0[u] = lane < LK ? Ss[sw(i, lane, LK)] : -INFINITY;
        x1[u] = TWO && lane + 64 < LK ? Ss[sw(i, lane + 64, LK)] : -INFINITY;
        mx[u] = fmaxf(x0[u], x1[u]);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int u = 0; u < G; ++u) mx[u] = fmaxf(mx[u], __shfl_xor(mx[u], o, 64));
#pragma unroll
      for (int u = 0; u < G; ++u) {
        x0[u] = lane < lk ? exp2f(x0[u] - mx[u]) : 0.f;
        x1[u] = TWO && lane + 64 < lk ? exp2f(x1[u] - mx[u]) : 0.f;
        sm[u] = x0[u] + x1[u];
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int u = 0; u < G; ++u) sm[u] += __shfl_xor(sm[u], o, 64);
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int i = w + (g + u) * NW;   // wave-uniform
        if (i >= lq) break;
        const float inv = __builtin_amdgcn_rcpf(sm[u]);
        const long long prow = pbase + (long long)i * lk;
        // values computed unconditionally; only the stores are predicated
        const float e0 = x0[u] * inv;
        const bool ok0 = lane < lk;
        const float pd0 = ok0 ? e0 * k3m_attn_drop(dr, off, rbase + i, lk, lane) : 0.f;
        if (ok0) probs[prow + lane] = e0;
        if (lane < LK) Ss[sw(i, lane, LK)] = pd0;
        if (TWO) {
          const float e1 = x1[u] * inv;
          const bool ok1 = lane + 64 < lk;
          const float pd1 = ok1 ? e1 * k3m_attn_drop(dr, off, rbase + i, lk, lane + 64) : 0.f;
          if (ok1) probs[prow + lane + 64] = e1;
          if (lane + 64 < LK) Ss[sw(i, lane + 64, LK)] = pd1;
        }
      }
    }
  }
  __syncthreads();
  ATT_STAMP(4);
  // O = Pd V
  {
    const int tq = LQ >> 5, td = hd >> 5;
    for (int t = w; t < tq * td; t += NW) {
      const int i0 = (t / td) * 32, d0 = (t % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile(acc, LK, [&](int kk) { return Ss[sw(i0 + cl, kk + kl, LK)]; },
                [&](int kk) { return KVs[sw(kk + kl, d0 + cl, hd)]; });
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (i < lq) ctx[(qrow0 + i) * ldc + hoff + d0 + cl] = from_f<T>(acc[r]);
      }
    }
  }
  ATT_STAMP_END(5);
}

// ------------------------------------------------------------------ backward
//   D_i  = dO_i . O_i                       (= sum_j P_ij dP_ij)
//   dS   = P * (dropmask * (dO V^T) - D)    phase 1  -> R3
//   dQ   = scale * dS K                     phase 2  (R2 <- K)
//   dV   = Pd^T dO                          phase 3  (R2 <- Pd)
//   dK   = scale * dS^T Q                   phase 4  (R1 <- Q)
template <typename T, int ML, int NW>
__global__ __launch_bounds__(NW * 64, ML == 64 ? 3 : 1) void attn_bwd_kernel(const T* __restrict__ dctx, long long ldc,
                                                       const T* __restrict__ o, long long ldo,
                                                       const T* __restrict__ q, long long ldq, const T* __restrict__ k,
                                                       long long ldk, const T* __restrict__ v, long long ldv,
                                                       const float* __restrict__ probs, T* __restrict__ dq,
                                                       T* __restrict__ dk, T* __restrict__ dv, long long lddq,
                                                       long long lddk, long long lddv, int lq, int lk, int nh, int hd,
                                                       float scale, float p_drop, uint64_t seed, uint64_t off) {
  constexpr int NTH = NW * 64;
  constexpr int BS = 4;   // MFMA slice depth of the backward's products (register budget)
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const int r2n = max(LK * hd, LQ * LK);
  float* R1 = smem;                 // [LQ][hd]: dO, later Q
  float* R2 = R1 + LQ * hd;         // V -> K -> Pd
  float* R3 = R2 + r2n;             // [LQ][LK]: dS
  // D_i is needed only until phase 1 ends, while R2 still holds V: keep it in R2's spare tail
  // when there is one (the L=128, d=64 case uses exactly 160 KiB that way)
  float* Ds = (LK * hd + LQ <= r2n) ? R2 + LK * hd : R3 + LQ * LK;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: row math on the scalar unit
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * hd;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  ATT_STAMP(0);

  // D_i = dO_i . O_i.  dO's, V's and O's 16-byte chunks are loaded together (one exposed global
  // latency); each thread writes the dot product of its dO and O chunks into R3 (free until
  // phase 1), then one thread per row adds its row's chunk dots in a fixed order.
  {
    Chunks<T, ML, NTH> c1, c2, c3;
    stage_load(c1, dctx, qrow0, ldc, hoff, LQ, lq, hd);
    stage_load(c2, v, krow0, ldv, hoff, LK, lk, hd);
    stage_load(c3, o, qrow0, ldo, hoff, LQ, lq, hd);
    stage_store(R1, c1, LQ, hd);
    stage_store(R2, c2, LK, hd);
    chunk_dots<T, ML, NTH>(R3, c1, c3, LQ, hd);
  }
  __syncthreads();
  {
    const int cpr = hd / Chunks<T, ML, NTH>::VE;
    if (threadIdx.x < LQ) {
      float a = 0.f;
      for (int c = 0; c < cpr; ++c) a += R3[threadIdx.x * cpr + c];
      Ds[threadIdx.x] = a;
    }
  }
  __syncthreads();
  ATT_STAMP(1);
  Chunks<T, ML, NTH> nch;  // K's loads fly during phase 1
  stage_load(nch, k, krow0, ldk, hoff, LK, lk, hd);
  // phase 1: dS
  {
    const int tq = LQ >> 5, tk = LK >> 5;
    for (int t = w; t < tq * tk; t += NW) {
      const int i0 = (t / tk) * 32, j0 = (t % tk) * 32;
      const int j = j0 + cl;
      float pr[16];   // this tile's probabilities: loaded before the MFMAs, which cover their latency
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        pr[r] = (i < lq && j < lk) ? probs[pbase + (long long)i * lk + j] : 0.f;
      }
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile<BS>(acc, hd, [&](int kk) { return R1[sw(i0 + cl, kk + kl, hd)]; },
                [&](int kk) { return R2[sw(j0 + cl, kk + kl, hd)]; });
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const float ds = pr[r] * (acc[r] * k3m_attn_drop(dr, off, rbase + i, lk, j) - Ds[i]);
        R3[sw(i, j, LK)] = (i < lq && j < lk) ? ds : 0.f;
      }
    }
  }
  __syncthreads();
  ATT_STAMP(2);
  stage_store(R2, nch, LK, hd);
  __syncthreads();
  stage_load(nch, q, qrow0, ldq, hoff, LQ, lq, hd);  // Q's loads fly during phases 2-3
  constexpr int U = ML * ML / NTH;
  float pv[U];   // phase 3's probabilities, loaded now: phase 2's MFMAs cover their latency
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = threadIdx.x + u * NTH;
    const int i = e / LK, j = e - i * LK;
    pv[u] = (e < LQ * LK && i < lq && j < lk) ? probs[pbase + (long long)i * lk + j] : 0.f;
  }
  // phase 2: dQ = scale * dS K
  {
    const int tq = LQ >> 5, td = hd >> 5;
    for (int t = w; t < tq * td; t += NW) {
      const int i0 = (t / td) * 32, d0 = (t % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile<BS>(acc, LK, [&](int kk) { return R3[sw(i0 + cl, kk + kl, LK)]; },
                [&](int kk) { return R2[sw(kk + kl, d0 + cl, hd)]; });
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (i < lq) dq[(qrow0 + i) * lddq + hoff + d0 + cl] = from_f<T>(acc[r] * scale);
      }
    }
  }
  __syncthreads();
  ATT_STAMP(3);
  // phase 3: R2 <- Pd [LQ][LK]; dV = Pd^T dO
  {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH;
      if (e < LQ * LK) {
        const int i = e / LK, j = e - i * LK;
        R2[sw(i, j, LK)] = pv[u] * k3m_attn_drop(dr, off, rbase + i, lk, j);
      }
    }
  }
  __syncthreads();
  {
    const int tk = LK >> 5, td = hd >> 5;
    for (int t = w; t < tk * td; t += NW) {
      const int j0 = (t / td) * 32, d0 = (t % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile<BS>(acc, LQ, [&](int kk) { return R2[sw(kk + kl, j0 + cl, LK)]; },    // A[j][i] = Pd[i][j]
                [&](int kk) { return R1[sw(kk + kl, d0 + cl, hd)]; });          // dO[i][d]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (j < lk) dv[(krow0 + j) * lddv + hoff + d0 + cl] = from_f<T>(acc[r]);
      }
    }
  }
  __syncthreads();
  ATT_STAMP(4);
  // phase 4: R1 <- Q; dK = scale * dS^T Q
  stage_store(R1, nch, LQ, hd);
  __syncthreads();
  {
    const int tk = LK >> 5, td = hd >> 5;
    for (int t = w; t < tk * td; t += NW) {
      const int j0 = (t / td) * 32, d0 = (t % td) * 32;
      floatx16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      mfma_tile<BS>(acc, LQ, [&](int kk) { return R3[sw(kk + kl, j0 + cl, LK)]; },    // A[j][i] = dS[i][j]
                [&](int kk) { return R1[sw(kk + kl, d0 + cl, hd)]; });          // Q[i][d]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (j < lk) dk[(krow0 + j) * lddk + hoff + d0 + cl] = from_f<T>(acc[r] * scale);
      }
    }
  }
  ATT_STAMP_END(5);
}

// x where ok, zeros elsewhere, per 32-bit word: a whole-float4 ?: select under a per-lane condition was lowered
// to a scratch store + indexed reload (or a branch + vmcnt(0) around the load); loads stay unconditional from
// clamped (valid) addresses
__device__ __forceinline__ float4 keep4(bool ok, float4 x) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_float4(__uint_as_float(__float_as_uint(x.x) & m), __uint_as_float(__float_as_uint(x.y) & m),
                     __uint_as_float(__float_as_uint(x.z) & m), __uint_as_float(__float_as_uint(x.w) & m));
}

// ------------------------------------------------------------------ forward, probabilities in registers
// fp32, lq, lk <= 128, K and V of the head in LDS (<= 80 KB: two or more workgroups per CU).  One
// wave per 32-query block, the queries on the MFMA lanes:
//   S^T = K Q^T    A = K from LDS (16-byte reads; lane half kl takes head dims [kl*HD/2, (kl+1)*HD/2)
//                  — the k order of a dot product is free), B = this wave's Q block held in
//                  registers (prescaled by scale*log2e), accumulators started at the key mask;
//   softmax        in the accumulators: lane (query q, half kl) holds keys 32kt + crow(r, kl), so a
//                  query's max and sum are 64 in-lane operations plus one exchange with lane ^ 32;
//   O^T = V^T P^T  B = the dropped probabilities straight from the accumulators (step s of key tile
//                  kt takes key 32kt + crow(s, kl) on both operands), A = V from LDS at
//                  compile-time offsets;
//   ctx            lane (q, kl) holds O[q][32dt + crow(r, kl)]: 16-byte stores.
// No S or P image in LDS, one barrier per workgroup.  crow(r, kl) = (r & 3) + 8 (r >> 2) + 4 kl.
template <int HD>
__global__ __launch_bounds__(256, 2) void attn_fwd_reg_kernel(const float* __restrict__ q, long long ldq,
                                                              const float* __restrict__ k, long long ldk,
                                                              const float* __restrict__ v, long long ldv,
                                                              const float* __restrict__ kmask, float* __restrict__ ctx,
                                                              long long ldc, float* __restrict__ probs, int lq, int lk,
                                                              int nh, float scale, float p_drop, uint64_t seed,
                                                              uint64_t off) {
  constexpr int NTH = 256, HH = HD / 2, NCH = HD / 4;
  constexpr int SWZ = (HD % 64 == 0) ? 15 : 7;   // XOR of the 16-byte chunk index by the key row
  constexpr int U = 8192 / 4 / NTH;               // staging chunks per thread and operand (LK*HD <= 8192)
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LK = (lk + 31) & ~31, nkt = LK >> 5;
  float* Ks = smem;              // [LK][HD], chunk c of row j stored at chunk c ^ (j & SWZ)
  float* Vs = Ks + LK * HD;      // [LK][HD]
  float* mk = Vs + LK * HD;      // [LK]: key mask in log2 units, -inf on padding keys
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const int qi = 32 * w + cl;    // this lane's query
  ATT_STAMP(0);

  // staging: K, V chunks and the mask (all loads first), and the wave's Q block into registers
  {
    float4 kc[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, j = e / NCH, c = e % NCH;
      const bool ok = e < LK * NCH && j < lk;
      const long long row = krow0 + min(j, lk - 1);
      kc[u] = keep4(ok, *reinterpret_cast<const float4*>(k + row * ldk + hoff + 4 * c));
      vc[u] = keep4(ok, *reinterpret_cast<const float4*>(v + row * ldv + hoff + 4 * c));
    }
    float mv = 0.f;
    if (threadIdx.x < LK && kmask) mv = kmask[krow0 + min((int)threadIdx.x, lk - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, j = e / NCH, c = e % NCH;
      if (e < LK * NCH) {
        *reinterpret_cast<float4*>(Ks + j * HD + 4 * (c ^ (j & SWZ))) = kc[u];
        *reinterpret_cast<float4*>(Vs + j * HD + 4 * c) = vc[u];
      }
    }
    if (threadIdx.x < LK) mk[threadIdx.x] = (int)threadIdx.x < lk ? mv * LOG2E : -INFINITY;
  }
  float qr[HH];
  {
    const float sl = scale * LOG2E;
    const bool ok = qi < lq;
    const float* src = q + (qrow0 + (ok ? qi : 0)) * ldq + hoff + kl * HH;
#pragma unroll
    for (int c = 0; c < HH / 4; ++c) {
      const float4 t = keep4(ok, *reinterpret_cast<const float4*>(src + 4 * c));
      qr[4 * c] = t.x * sl;
      qr[4 * c + 1] = t.y * sl;
      qr[4 * c + 2] = t.z * sl;
      qr[4 * c + 3] = t.w * sl;
    }
  }
  __syncthreads();
  ATT_STAMP(1);
  if (32 * w >= lq) return;   // no queries for this wave (no barrier follows)

  // S^T tiles, started at the key mask
  floatx16 acc[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const float4 m4 = *reinterpret_cast<const float4*>(mk + 32 * kt + 8 * a + 4 * kl);
        acc[kt][4 * a] = m4.x;
        acc[kt][4 * a + 1] = m4.y;
        acc[kt][4 * a + 2] = m4.z;
        acc[kt][4 * a + 3] = m4.w;
      }
      const int key = 32 * kt + cl;
      const float* krow = Ks + key * HD;
      const int sw = key & SWZ;
#pragma unroll
      for (int m = 0; m < HH; m += 4) {
        const float4 a4 = *reinterpret_cast<const float4*>(krow + 4 * (((kl * HH + m) >> 2) ^ sw));
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, qr[m], acc[kt], 0, 0, 0);
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, qr[m + 1], acc[kt], 0, 0, 0);
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, qr[m + 2], acc[kt], 0, 0, 0);
        acc[kt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, qr[m + 3], acc[kt], 0, 0, 0);
      }
    }
  }
  ATT_STAMP(2);

  // softmax over the keys of query qi, in the accumulators
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
    if (kt < nkt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, acc[kt][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sm = 0.f;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
    if (kt < nkt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[kt][r] = exp2f(acc[kt][r] - mx);
        sm += acc[kt][r];
      }
  sm += __shfl_xor(sm, 32, 64);
  {
    const float inv = __builtin_amdgcn_rcpf(sm);
    const K3mDrop dr = k3m_drop_init(seed, p_drop);
    const bool qok = qi < lq;
    const long long prow = pbase + (long long)(qok ? qi : 0) * lk;
    const K3mPairRow prr = k3m_pair_row(dr, off, rbase + (qok ? qi : 0), lk, 4 * kl);
    const bool vec = (lk & 3) == 0;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int j0 = 32 * kt + 8 * a + 4 * kl;
          // keys j0 .. j0 + 3: two pair draws (k3m_attn_drop); all ones when p = 0
          const uint32_t h01 = dr.thr != 0u ? k3m_pair_draw(prr, 16 * kt + 4 * a) : 0xffffffffu;
          const uint32_t h23 = dr.thr != 0u ? k3m_pair_draw(prr, 16 * kt + 4 * a + 1) : 0xffffffffu;
          float p4[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int j = j0 + b;
            p4[b] = acc[kt][4 * a + b] * inv;
            const float dm = k3m_attn_half(b < 2 ? h01 : h23, b) >= dr.thr16 ? dr.scale : 0.f;
            acc[kt][4 * a + b] = j < lk ? p4[b] * dm : 0.f;
          }
#ifdef K3M_LAB_NO_PSTORE   // lab only (scripts/lab/lab_build.sh): the forward without its probability stores
          if (false) {
#else
          if (qok) {
#endif
            if (vec && j0 < lk) {
              *reinterpret_cast<float4*>(probs + prow + j0) = make_float4(p4[0], p4[1], p4[2], p4[3]);
            } else if (!vec) {
#pragma unroll
              for (int b = 0; b < 4; ++b)
                if (j0 + b < lk) probs[prow + j0 + b] = p4[b];
            }
          }
        }
      }
    }
  }
  ATT_STAMP(3);

  // O^T = V^T P^T
  floatx16 o[HD / 32];
#pragma unroll
  for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
  const float* vbase = Vs + 4 * kl * HD + cl;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const int key = 32 * kt + (st & 3) + 8 * (st >> 2);   // + 4 kl, in vbase
#pragma unroll
        for (int dt = 0; dt < HD / 32; ++dt)
          o[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(vbase[key * HD + 32 * dt], acc[kt][st], o[dt], 0, 0, 0);
      }
    }
  }
  if (qi < lq) {
    float* dst = ctx + (qrow0 + qi) * ldc + hoff + 4 * kl;
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a)
        *reinterpret_cast<float4*>(dst + 32 * dt + 8 * a) =
            make_float4(o[dt][4 * a], o[dt][4 * a + 1], o[dt][4 * a + 2], o[dt][4 * a + 3]);
  }
  ATT_STAMP(4);
}

size_t fwd_reg_lds(int lk, int hd) {
  const size_t LK = (lk + 31) & ~31;
  return sizeof(float) * (2 * LK * hd + LK);
}

// ------------------------------------------------------------------ forward on the bf16 matrix cores
// The register-softmax forward with both products in the bf16x6 form of gemm_x6_tile.h (fp32 operands
// split exactly into three bf16 planes, the six leading partial products accumulated in fp32 on
// v_mfma_f32_32x32x16_bf16: 2.67x the f32-MFMA rate at fp32 accuracy).  Structure as attn_fwd_reg_kernel:
//   S^T = K Q^T    A = K rows from LDS (two 16-B reads per 8 head dims, split in registers), B = this
//                  wave's Q block (prescaled, split once when it fits the register budget);
//   softmax        unchanged (the 32x32x16 bf16 MFMA has the accumulator layout of the f32 one);
//   O^T = V^T P^T  B = the dropped probabilities of one 16-key step straight from the accumulators,
//                  split; A = V^T from a transposed LDS image [HD][LKP] (key chunk c of row d at
//                  c ^ (d & (LKP/4 - 1))), whose 8 keys per lane half — the accumulator order
//                  32kt + 16s + 8(e>>2) + 4h + (e&3) — are two 16-B reads.
typedef __bf16 x6bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t x6u32x4 __attribute__((ext_vector_type(4)));
typedef float x6float2 __attribute__((ext_vector_type(2)));
typedef __bf16 x6bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t x6_pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((x6float2{a, b}), x6bf16x2));
}
// x = h + m + l exactly (8 floats -> three packed bf16x8 planes)
__device__ __forceinline__ void x6_split8(const float (&x)[8], x6bf16x8& h, x6bf16x8& m, x6bf16x8& l) {
  x6u32x4 H, Mm, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t hh = x6_pk(a, b);
    const float r1a = a - __uint_as_float(hh << 16), r1b = b - __uint_as_float(hh & 0xffff0000u);
    const uint32_t mm = x6_pk(r1a, r1b);
    const float r2a = r1a - __uint_as_float(mm << 16), r2b = r1b - __uint_as_float(mm & 0xffff0000u);
    H[p] = hh;
    Mm[p] = mm;
    L[p] = x6_pk(r2a, r2b);
  }
  h = __builtin_bit_cast(x6bf16x8, H);
  m = __builtin_bit_cast(x6bf16x8, Mm);
  l = __builtin_bit_cast(x6bf16x8, L);
}
// acc += a.b over the six leading plane products, smallest first
__device__ __forceinline__ void x6_mma(floatx16& acc, const x6bf16x8& ah, const x6bf16x8& am, const x6bf16x8& al,
                                       const x6bf16x8& bh, const x6bf16x8& bm, const x6bf16x8& bl) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
}

__host__ __device__ constexpr int x6_lkp(int LK) { return LK <= 32 ? 32 : LK <= 64 ? 64 : 128; }

template <int HD>
__global__ __launch_bounds__(256, 2) void attn_fwd_x6_kernel(const float* __restrict__ q, long long ldq,
                                                             const float* __restrict__ k, long long ldk,
                                                             const float* __restrict__ v, long long ldv,
                                                             const float* __restrict__ kmask, float* __restrict__ ctx,
                                                             long long ldc, float* __restrict__ probs, int lq, int lk,
                                                             int nh, float scale, float p_drop, uint64_t seed,
                                                             uint64_t off) {
  constexpr int NTH = 256, HH = HD / 2, NCH = HD / 4, NS = HH / 8;
  constexpr int SWZ = (HD % 64 == 0) ? 15 : 7;    // K image: 16-byte chunk index XOR (key & SWZ)
  constexpr int U = 8192 / 4 / NTH;               // staging chunks per thread and operand (LK*HD <= 8192)
  constexpr bool QSPLIT = HD <= 96;               // Q planes held in registers (else split per use)
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LK = (lk + 31) & ~31, nkt = LK >> 5;
  const int LKP = x6_lkp(LK), VM = LKP / 4 - 1;
  float* Ks = smem;              // [LK][HD]
  float* Vt = Ks + LK * HD;      // [HD][LKP]
  float* mk = Vt + HD * LKP;     // [LK] key mask in log2 units, -inf on padding keys
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const int qi = 32 * w + cl;

  // staging: K row-major (chunk-swizzled), V transposed (keys of one d contiguous), the mask
  {
    float4 kc[U], vc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH;
      const int j = e / NCH, c = e % NCH;                 // K: row-major chunks (coalesced)
      const bool ok = e < LK * NCH && j < lk;
      kc[u] = keep4(ok, *reinterpret_cast<const float4*>(k + (krow0 + min(j, lk - 1)) * ldk + hoff + 4 * (c % NCH)));
      const int jv = e % LK, cv = e / LK;                 // V: 64 consecutive keys per wave instruction
      const bool okv = e < LK * NCH && jv < lk;
      vc[u] = keep4(okv, *reinterpret_cast<const float4*>(v + (krow0 + min(jv, lk - 1)) * ldv + hoff +
                                                           4 * min(cv, NCH - 1)));
    }
    float mv = 0.f;
    if (threadIdx.x < LK && kmask) mv = kmask[krow0 + min((int)threadIdx.x, lk - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH;
      if (e < LK * NCH) {
        const int j = e / NCH, c = e % NCH;
        *reinterpret_cast<float4*>(Ks + j * HD + 4 * (c ^ (j & SWZ))) = kc[u];
        const int jv = e % LK, cv = e / LK;
        const float vv[4] = {vc[u].x, vc[u].y, vc[u].z, vc[u].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int d = 4 * cv + i;
          Vt[d * LKP + 4 * ((jv >> 2) ^ (d & VM)) + (jv & 3)] = vv[i];
        }
      }
    }
    if (threadIdx.x < LK) mk[threadIdx.x] = (int)threadIdx.x < lk ? mv * LOG2E : -INFINITY;
  }
  float qr[HH];
  {
    const float sl = scale * LOG2E;
    const bool ok = qi < lq;
    const float* src = q + (qrow0 + (ok ? qi : 0)) * ldq + hoff + kl * HH;
#pragma unroll
    for (int c = 0; c < HH / 4; ++c) {
      const float4 t = keep4(ok, *reinterpret_cast<const float4*>(src + 4 * c));
      qr[4 * c] = t.x * sl;
      qr[4 * c + 1] = t.y * sl;
      qr[4 * c + 2] = t.z * sl;
      qr[4 * c + 3] = t.w * sl;
    }
  }
  x6bf16x8 qh[QSPLIT ? NS : 1], qm[QSPLIT ? NS : 1], ql[QSPLIT ? NS : 1];
  if constexpr (QSPLIT) {
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      float t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = qr[8 * st + e];
      x6_split8(t, qh[st], qm[st], ql[st]);
    }
  }
  __syncthreads();
  if (32 * w >= lq) return;   // no queries for this wave (no barrier follows)

  // S^T tiles, started at the key mask: head dims kl*HH + 8st + e on both operands
  floatx16 acc[4];
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const float4 m4 = *reinterpret_cast<const float4*>(mk + 32 * kt + 8 * a + 4 * kl);
        acc[kt][4 * a] = m4.x;
        acc[kt][4 * a + 1] = m4.y;
        acc[kt][4 * a + 2] = m4.z;
        acc[kt][4 * a + 3] = m4.w;
      }
      const int key = 32 * kt + cl;
      const float* krow = Ks + key * HD;
      const int sw = key & SWZ;
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const int c0 = (kl * HH + 8 * st) >> 2;
        const float4 a0 = *reinterpret_cast<const float4*>(krow + 4 * (c0 ^ sw));
        const float4 a1 = *reinterpret_cast<const float4*>(krow + 4 * ((c0 + 1) ^ sw));
        const float ka[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        x6bf16x8 ah, am, al;
        x6_split8(ka, ah, am, al);
        if constexpr (QSPLIT) {
          x6_mma(acc[kt], ah, am, al, qh[st], qm[st], ql[st]);
        } else {
          float t[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] = qr[8 * st + e];
          x6bf16x8 bh, bm, bl;
          x6_split8(t, bh, bm, bl);
          x6_mma(acc[kt], ah, am, al, bh, bm, bl);
        }
      }
    }
  }

  // softmax over the keys of query qi, in the accumulators (as attn_fwd_reg_kernel)
  float mx = -INFINITY;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
    if (kt < nkt)
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, acc[kt][r]);
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sm = 0.f;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
    if (kt < nkt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[kt][r] = exp2f(acc[kt][r] - mx);
        sm += acc[kt][r];
      }
  sm += __shfl_xor(sm, 32, 64);
  {
    const float inv = __builtin_amdgcn_rcpf(sm);
    const K3mDrop dr = k3m_drop_init(seed, p_drop);
    const bool qok = qi < lq;
    const long long prow = pbase + (long long)(qok ? qi : 0) * lk;
    const K3mPairRow prr = k3m_pair_row(dr, off, rbase + (qok ? qi : 0), lk, 4 * kl);
    const bool vec = (lk & 3) == 0;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int j0 = 32 * kt + 8 * a + 4 * kl;
          // keys j0 .. j0 + 3: two pair draws (k3m_attn_drop); all ones when p = 0
          const uint32_t h01 = dr.thr != 0u ? k3m_pair_draw(prr, 16 * kt + 4 * a) : 0xffffffffu;
          const uint32_t h23 = dr.thr != 0u ? k3m_pair_draw(prr, 16 * kt + 4 * a + 1) : 0xffffffffu;
          float p4[4];
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int j = j0 + b;
            p4[b] = acc[kt][4 * a + b] * inv;
            const float dm = k3m_attn_half(b < 2 ? h01 : h23, b) >= dr.thr16 ? dr.scale : 0.f;
            acc[kt][4 * a + b] = j < lk ? p4[b] * dm : 0.f;
          }
#ifdef K3M_LAB_NO_PSTORE   // lab only (scripts/lab/lab_build.sh): the forward without its probability stores
          if (false) {
#else
          if (qok) {
#endif
            if (vec && j0 < lk) {
              *reinterpret_cast<float4*>(probs + prow + j0) = make_float4(p4[0], p4[1], p4[2], p4[3]);
            } else if (!vec) {
#pragma unroll
              for (int b = 0; b < 4; ++b)
                if (j0 + b < lk) probs[prow + j0 + b] = p4[b];
            }
          }
        }
      }
    }
  }

  // O^T = V^T P^T: 16-key steps (kt, s2); lane half kl carries keys 32kt + 16 s2 + 8(e>>2) + 4kl + (e&3)
  floatx16 o[HD / 32];
#pragma unroll
  for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[dt][r] = 0.f;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt < nkt) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) pv[e] = acc[kt][8 * s2 + e];
        x6bf16x8 ph, pm, pl;
        x6_split8(pv, ph, pm, pl);
        const int ch = 8 * kt + 4 * s2 + kl;   // key chunk of e = 0..3 (e = 4..7: ch + 2)
#pragma unroll
        for (int dt = 0; dt < HD / 32; ++dt) {
          const int d = 32 * dt + cl;
          const float* vrow = Vt + d * LKP;
          const float4 v0 = *reinterpret_cast<const float4*>(vrow + 4 * (ch ^ (d & VM)));
          const float4 v1 = *reinterpret_cast<const float4*>(vrow + 4 * ((ch + 2) ^ (d & VM)));
          const float va[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          x6bf16x8 vh, vm, vl;
          x6_split8(va, vh, vm, vl);
          x6_mma(o[dt], vh, vm, vl, ph, pm, pl);
        }
      }
    }
  }
  if (qi < lq) {
    float* dst = ctx + (qrow0 + qi) * ldc + hoff + 4 * kl;
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a)
        *reinterpret_cast<float4*>(dst + 32 * dt + 8 * a) =
            make_float4(o[dt][4 * a], o[dt][4 * a + 1], o[dt][4 * a + 2], o[dt][4 * a + 3]);
  }
}

size_t fwd_x6_lds(int lk, int hd) {
  const int LK = (lk + 31) & ~31;
  return sizeof(float) * ((size_t)LK * hd + (size_t)hd * x6_lkp(LK) + LK);
}

// 16-byte global -> LDS copy (global_load_lds_dwordx4): the LDS destination is the wave-uniform base
// plus 16 * lane
__device__ __forceinline__ void glds16(const float* g, float* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// ------------------------------------------------------------------ backward, keys on the lanes
// fp32 partner of attn_fwd_reg_kernel (LQ*HD <= 8192).  Workgroup per (sequence, head), 4 waves:
//   key phase   wave w owns keys 32w..32w+31 (on the MFMA lanes; V rows in registers):
//               dPd = dO V^T (A = dO rows from a swizzled LDS image, 16-byte reads), then per element
//               dS = P (dPd m - D), Pd = P m (P prefetched from the forward, m the regenerated dropout
//               scale), both kept in accumulators; dV^T = dO^T Pd and dK^T = scale Q^T dS take them as
//               B operands (k = query crow(s, kl)), A from LDS at per-step offsets; 16-byte stores
//   dS image    written once to LDS (over dO / Q), then
//   query phase wave w owns queries 32w..: dQ = scale dS K (A = dS rows, 16-byte reads; B = K rows).
// D = rowsum(dO o O) from dot products of the staged 16-byte chunks.
template <int HD>
__global__ __launch_bounds__(256, 1) void attn_bwd_reg_kernel(
    const float* __restrict__ dctx, long long ldc, const float* __restrict__ o, long long ldo,
    const float* __restrict__ q, long long ldq, const float* __restrict__ k, long long ldk,
    const float* __restrict__ v, long long ldv, const float* __restrict__ probs, float* __restrict__ dq,
    float* __restrict__ dk, float* __restrict__ dv, long long lddq, long long lddk, long long lddv, int lq, int lk,
    int nh, float scale, float p_drop, uint64_t seed, uint64_t off) {
  constexpr int NTH = 256, HH = HD / 2, NCH = HD / 4;
  constexpr int SWZ = (HD % 64 == 0) ? 15 : 7;
  constexpr int UQ = 8192 / 4 / NTH;     // chunks per thread of a [LQ][HD] operand (LQ*HD <= 8192)
  constexpr int UK = 128 * NCH / NTH;    // chunks per thread of K (LK <= 128)
  extern __shared__ float smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  float* dOs = smem;              // [LQ][HD], chunk c of row i at chunk c ^ (i & SWZ)
  float* Qs = dOs + LQ * HD;      // [LQ][HD]
  float* Ks = Qs + LQ * HD;       // [LK][HD]
  float* Ds = Ks + LK * HD;       // [LQ]
  float* scr = Ds + LQ;           // [LQ][NCH] chunk dots of dO and O
  float* dSs = smem;              // [LQ][LK] over dOs / Qs after the key phase, chunk c of row i at c ^ (i & sws)
  const int sws = (LK % 64 == 0) ? 15 : 7;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  ATT_STAMP(0);

  {  // staging of dO (+ the D partials): every load first
    float4 cdo[UQ], co[UQ];
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCH, c = e % NCH;
      const bool ok = e < LQ * NCH && i < lq;
      const long long row = qrow0 + (ok ? i : 0);
      cdo[u] = keep4(ok, *reinterpret_cast<const float4*>(dctx + row * ldc + hoff + 4 * c));
      co[u] = keep4(ok, *reinterpret_cast<const float4*>(o + row * ldo + hoff + 4 * c));
    }
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCH, c = e % NCH;
      if (e < LQ * NCH) {
        *reinterpret_cast<float4*>(dOs + i * HD + 4 * (c ^ (i & SWZ))) = cdo[u];
        scr[e] = cdo[u].x * co[u].x + cdo[u].y * co[u].y + cdo[u].z * co[u].z + cdo[u].w * co[u].w;
      }
    }
  }
  const int key = 32 * w + cl;      // this lane's key in the key phase
  const bool kw = 32 * w < LK;      // wave-uniform
  float vr[HH];                     // V[key][kl*HH + m]
  {
    const bool ok = kw && key < lk;
    const float* src = v + (krow0 + (ok ? key : 0)) * ldv + hoff + kl * HH;
#pragma unroll
    for (int c = 0; c < HH / 4; ++c) {
      const float4 t = keep4(ok, *reinterpret_cast<const float4*>(src + 4 * c));
      vr[4 * c] = t.x;
      vr[4 * c + 1] = t.y;
      vr[4 * c + 2] = t.z;
      vr[4 * c + 3] = t.w;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < LQ) {
    float a = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) a += scr[threadIdx.x * NCH + c];
    Ds[threadIdx.x] = a;
  }
  __syncthreads();
  ATT_STAMP(1);
  // Q and K are needed from the dV/dK phase on: global -> LDS copies (no registers) that fly during
  // the dPd MFMAs.  A wave-instruction writes 64 consecutive 16-byte chunks (the plain row-major
  // images); chunks of padding rows are zeroed with ordinary stores instead.
#pragma unroll
  for (int u = 0; u < UQ; ++u) {
    const int e = threadIdx.x + u * NTH, i = e / NCH, c = e % NCH;
    if (e < LQ * NCH) {   // wave-uniform (LQ*NCH is a multiple of 512)
      if (i < lq) glds16(q + (qrow0 + i) * ldq + hoff + 4 * c, Qs + 4 * (u * NTH + 64 * w));
      else *reinterpret_cast<float4*>(Qs + 4 * e) = z4;
    }
  }
#pragma unroll
  for (int u = 0; u < UK; ++u) {
    const int e = threadIdx.x + u * NTH, j = e / NCH, c = e % NCH;
    if (e < LK * NCH) {
      if (j < lk) glds16(k + (krow0 + j) * ldk + hoff + 4 * c, Ks + 4 * (u * NTH + 64 * w));
      else *reinterpret_cast<float4*>(Ks + 4 * e) = z4;
    }
  }

  const int nqt = LQ >> 5;
  floatx16 acc[4], pdv[4];   // rows: queries 32qt + crow(r, kl); lanes: keys
  if (kw) {
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {   // the forward's probabilities, ahead of the MFMAs
      if (qt < nqt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * kl;
          pdv[qt][r] = (qr < lq && key < lk) ? probs[pbase + (long long)qr * lk + key] : 0.f;
        }
      }
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {   // dPd = dO V^T
      if (qt < nqt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[qt][r] = 0.f;
        const int ar = 32 * qt + cl;
        const float* arow = dOs + ar * HD;
        const int sw = ar & SWZ;
#pragma unroll
        for (int m = 0; m < HH; m += 4) {
          const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * (((kl * HH + m) >> 2) ^ sw));
          acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, vr[m], acc[qt], 0, 0, 0);
          acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, vr[m + 1], acc[qt], 0, 0, 0);
          acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, vr[m + 2], acc[qt], 0, 0, 0);
          acc[qt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, vr[m + 3], acc[qt], 0, 0, 0);
        }
      }
    }
    ATT_STAMP(2);
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {   // dS, Pd
      if (qt < nqt) {
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const float4 d4 = *reinterpret_cast<const float4*>(Ds + 32 * qt + 8 * a + 4 * kl);
          const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            const int r = 4 * a + b, qr = 32 * qt + 8 * a + 4 * kl + b;
            const bool ok = qr < lq && key < lk;
            const float m = k3m_attn_drop(dr, off, rbase + (ok ? qr : 0), lk, ok ? key : 0);
            const float p = pdv[qt][r];
            acc[qt][r] = ok ? p * (acc[qt][r] * m - dd[b]) : 0.f;
            pdv[qt][r] = p * m;
          }
        }
      }
    }
  }
  __syncthreads();   // Q and K copies landed (the barrier waits for this wave's copies first)
  if (kw) {
    // dV^T = dO^T Pd, dK^T = Q^T dS (B operands from the accumulators)
    floatx16 ov[HD / 32], ok_[HD / 32];
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        ov[dt][r] = 0.f;
        ok_[dt][r] = 0.f;
      }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      if (qt < nqt) {
#pragma unroll
        for (int st = 0; st < 16; ++st) {
          const int row = 32 * qt + (st & 3) + 8 * (st >> 2) + 4 * kl;
          const int sw = row & SWZ;
#pragma unroll
          for (int dt = 0; dt < HD / 32; ++dt) {
            const int d = 32 * dt + cl;
            const float a_do = dOs[row * HD + 4 * ((d >> 2) ^ sw) + (d & 3)];
            const float a_q = Qs[row * HD + d];
            ov[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_do, pdv[qt][st], ov[dt], 0, 0, 0);
            ok_[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_q, acc[qt][st], ok_[dt], 0, 0, 0);
          }
        }
      }
    }
    if (key < lk) {
      float* pv = dv + (krow0 + key) * lddv + hoff + 4 * kl;
      float* pk = dk + (krow0 + key) * lddk + hoff + 4 * kl;
#pragma unroll
      for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          *reinterpret_cast<float4*>(pv + 32 * dt + 8 * a) =
              make_float4(ov[dt][4 * a], ov[dt][4 * a + 1], ov[dt][4 * a + 2], ov[dt][4 * a + 3]);
          *reinterpret_cast<float4*>(pk + 32 * dt + 8 * a) =
              make_float4(ok_[dt][4 * a] * scale, ok_[dt][4 * a + 1] * scale, ok_[dt][4 * a + 2] * scale,
                          ok_[dt][4 * a + 3] * scale);
        }
    }
  }
  __syncthreads();   // every wave is done with dOs / Qs
  ATT_STAMP(3);
  if (kw) {
#pragma unroll
    for (int qt = 0; qt < 4; ++qt)
      if (qt < nqt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = 32 * qt + (r & 3) + 8 * (r >> 2) + 4 * kl;
          dSs[qr * LK + 4 * ((key >> 2) ^ (qr & sws)) + (key & 3)] = acc[qt][r];
        }
  }
  __syncthreads();
  if (32 * w < LQ) {   // dQ = scale dS K for queries 32w..32w+31
    floatx16 oq[HD / 32];
#pragma unroll
    for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) oq[dt][r] = 0.f;
    const int ar = 32 * w + cl, LH = LK >> 1;
    const float* arow = dSs + ar * LK;
    const int sw = ar & sws;
    const float* kb = Ks + kl * LH * HD + cl;
    for (int m = 0; m < LH; m += 4) {
      const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * (((kl * LH + m) >> 2) ^ sw));
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int dt = 0; dt < HD / 32; ++dt)
          oq[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], kb[(m + i) * HD + 32 * dt], oq[dt], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qr = 32 * w + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (qr < lq) {
        float* dst = dq + (qrow0 + qr) * lddq + hoff + cl;
#pragma unroll
        for (int dt = 0; dt < HD / 32; ++dt) dst[32 * dt] = oq[dt][r] * scale;
      }
    }
  }
  ATT_STAMP_END(4);
}

// ------------------------------------------------------------------ backward on the bf16 matrix cores, keys on lanes
// fp32 backward with every product in the bf16x6 form (gemm_x6_tile.h; the forward's attn_fwd_x6_kernel), laid out
// like attention_bf16.hip's key-major kernel:
//   staging     Q, dO and K split exactly into three bf16 planes each, stored as [rows][HD] bf16 images (16-B chunk
//               c of row r at c ^ swz(r)), so row fragments (ds_read_b128) and transposed fragments
//               (ds_read_b64_tr_b16) of every plane are conflict-free; D = rowsum(dO o O) from fp32 chunk dots;
//   key phase   wave w owns keys 32w..32w+31 on the MFMA lanes (its V rows split into B fragments in registers);
//               per 32-query tile dPd = dO V^T, then with P from the forward's probabilities and m the regenerated
//               dropout scale: Pd = P m, dS = P (dPd m - D) in the accumulators; dV^T += dO^T Pd and
//               dK^T += Q^T dS take Pd / dS split straight from the accumulators (accumulator k order) as B operands,
//               A = transposed plane reads; dS is kept in fp32 registers;
//   dS^T        three planes written once over the Q / dO images;
//   query phase dQ = scale dS K (A = dS^T planes, B = K planes, both transposed reads).
// ML: rows staged (>= LQ, LK), NW = ML / 32 waves.  Same semantics and dropout counters as attn_bwd_reg_kernel.
typedef short k6short4 __attribute__((ext_vector_type(4)));
typedef short k6short8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) k6short4 k6lds_short4;

template <int NC>
__device__ __forceinline__ int k6_ioff(int r, int c) {   // element offset of 8-bf16 chunk c of row r
  if constexpr (NC == 16) return r * 128 + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 3);
  else if constexpr (NC == 8) return r * 64 + ((c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) << 3);
  else return r * 32 + (c << 3);
}
__device__ __forceinline__ int k6_ioff_n(int nc, int r, int c) {
  return nc == 4 ? k6_ioff<4>(r, c) : nc == 8 ? k6_ioff<8>(r, c) : k6_ioff<16>(r, c);
}
// row fragment: X[rbase + (lane&31)][16 ks + 8 (lane>>5) .. +7]
template <int NC>
__device__ __forceinline__ x6bf16x8 k6_row(const uint16_t* img, int rbase, int ks, int lane) {
  return *reinterpret_cast<const x6bf16x8*>(img + k6_ioff<NC>(rbase + (lane & 31), 2 * ks + (lane >> 5)));
}
// transposed fragment (attention_bf16.hip trfrag): element e of lane l = X[row(e)][cbase + (l&31)],
// PERM = false: row(e) = rbase + 8h + e; PERM = true: row(e) = rbase + 8(e>>2) + 4h + (e&3)
template <int NC, bool PERM>
__device__ __forceinline__ x6bf16x8 k6_tr(const uint16_t* img, int rbase, int cbase, int lane) {
  const int g = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3, h = lane >> 5;
  const int ch = ((cbase + 16 * (g & 1)) >> 3) + (p >> 1);
  const int r0 = PERM ? rbase + 4 * h + qq : rbase + 8 * h + qq;
  const int r1 = PERM ? r0 + 8 : r0 + 4;
  const k6short4 x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((k6lds_short4*)(img + k6_ioff<NC>(r0, ch) + 4 * (p & 1)));
  const k6short4 x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((k6lds_short4*)(img + k6_ioff<NC>(r1, ch) + 4 * (p & 1)));
  const k6short8 vv = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(x6bf16x8, vv);
}
__device__ __forceinline__ x6bf16x8 k6_tr_n(const uint16_t* img, int nc, int rbase, int cbase, int lane) {
  if (nc == 4) return k6_tr<4, false>(img, rbase, cbase, lane);
  if (nc == 8) return k6_tr<8, false>(img, rbase, cbase, lane);
  return k6_tr<16, false>(img, rbase, cbase, lane);
}
// x = h + m + l exactly for 4 floats -> three packed bf16 quads
__device__ __forceinline__ void k6_split4(const float4 v, uint2& hq, uint2& mq, uint2& lq) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  uint32_t H[2], Mm[2], Lw[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float a = x[2 * p], b = x[2 * p + 1];
    const uint32_t hh = x6_pk(a, b);
    const float r1a = a - __uint_as_float(hh << 16), r1b = b - __uint_as_float(hh & 0xffff0000u);
    const uint32_t mm = x6_pk(r1a, r1b);
    const float r2a = r1a - __uint_as_float(mm << 16), r2b = r1b - __uint_as_float(mm & 0xffff0000u);
    H[p] = hh;
    Mm[p] = mm;
    Lw[p] = x6_pk(r2a, r2b);
  }
  hq = make_uint2(H[0], H[1]);
  mq = make_uint2(Mm[0], Mm[1]);
  lq = make_uint2(Lw[0], Lw[1]);
}
// accumulator registers 8s..8s+7 split into three bf16 operand fragments
__device__ __forceinline__ void k6_accsplit(const floatx16& a, int s, x6bf16x8& h, x6bf16x8& m, x6bf16x8& l) {
  float t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = a[8 * s + e];
  x6_split8(t, h, m, l);
}

template <int HD, int ML>
__global__ __launch_bounds__(ML * 2, 1) void attn_bwd_x6km_kernel(
    const float* __restrict__ dctx, long long ldc, const float* __restrict__ o, long long ldo,
    const float* __restrict__ q, long long ldq, const float* __restrict__ k, long long ldk,
    const float* __restrict__ v, long long ldv, const float* __restrict__ probs, float* __restrict__ dq,
    float* __restrict__ dk, float* __restrict__ dv, long long lddq, long long lddk, long long lddv, int lq, int lk,
    int nh, float scale, float p_drop, uint64_t seed, uint64_t off) {
  constexpr int NW = ML / 32, NTH = NW * 64;
  constexpr int NC = HD / 8, HW = HD, KS = HD / 16, DT = HD / 32, NCH = HD / 4;
  extern __shared__ float smem_f[];   // (the file's other kernels declare the dynamic LDS as float[])
  uint16_t* smem = reinterpret_cast<uint16_t*>(smem_f);
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const int QW = LQ == 96 ? 128 : LQ, QNC = QW / 8;   // dS^T image [LK][QW] per plane
  const int PQ = LQ * HW, PK = LK * HW, PS = LK * QW;   // bf16 elements per plane
  const int RQ = max(6 * PQ, 3 * PS);                  // Q | dO planes, later the dS^T planes
  uint16_t* Qs = smem;
  uint16_t* dOs = smem + 3 * PQ;
  uint16_t* dSt = smem;
  uint16_t* Ks = smem + RQ;
  float* Ds = reinterpret_cast<float*>(Ks + 3 * PK);
  float* scr = Ds + LQ;   // [LQ][NCH] chunk dots of dO and O
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long pbase = ((long long)s * nh + h) * lq * lk;
  const long long rbase = ((long long)s * nh + h) * lq;   // first score row (attention dropout counters)
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const int NQT = LQ >> 5;
  const int j = 32 * w + cl;     // this lane's key in the key phase
  const bool kw = 32 * w < LK;   // wave-uniform

  // this wave's V rows split into B-operand fragments (lane -> key j, dims 16 ks + 8 kl .. +7)
  x6bf16x8 vh[KS], vm[KS], vl[KS];
  {
    const bool okv = kw && j < lk;
    const float* vp = v + (krow0 + min(j, lk - 1)) * ldv + hoff + 8 * kl;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const float4 a = keep4(okv, *reinterpret_cast<const float4*>(vp + 16 * ks));
      const float4 b = keep4(okv, *reinterpret_cast<const float4*>(vp + 16 * ks + 4));
      const float t[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      x6_split8(t, vh[ks], vm[ks], vl[ks]);
    }
  }
  {
    // staging: every global load (Q, dO, O, K float4 chunks) issued before the first LDS write
    constexpr int U = ML * NCH / NTH;
    float4 rq[U], rdo[U], ro[U], rk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCH, c = e % NCH;
      const long long qo = qrow0 + min(i, lq - 1), ko = krow0 + min(i, lk - 1);
      rq[u] = keep4(i < lq, *reinterpret_cast<const float4*>(q + qo * ldq + hoff + 4 * c));
      rdo[u] = keep4(i < lq, *reinterpret_cast<const float4*>(dctx + qo * ldc + hoff + 4 * c));
      ro[u] = keep4(i < lq, *reinterpret_cast<const float4*>(o + qo * ldo + hoff + 4 * c));
      rk[u] = keep4(i < lk, *reinterpret_cast<const float4*>(k + ko * ldk + hoff + 4 * c));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCH, c = e % NCH;
      const int eo = 4 * (c & 1);
      if (i < LQ) {
        const int io = k6_ioff<NC>(i, c >> 1) + eo;
        uint2 a, b, cc;
        k6_split4(rq[u], a, b, cc);
        *reinterpret_cast<uint2*>(Qs + io) = a;
        *reinterpret_cast<uint2*>(Qs + PQ + io) = b;
        *reinterpret_cast<uint2*>(Qs + 2 * PQ + io) = cc;
        k6_split4(rdo[u], a, b, cc);
        *reinterpret_cast<uint2*>(dOs + io) = a;
        *reinterpret_cast<uint2*>(dOs + PQ + io) = b;
        *reinterpret_cast<uint2*>(dOs + 2 * PQ + io) = cc;
        scr[e] = rdo[u].x * ro[u].x + rdo[u].y * ro[u].y + rdo[u].z * ro[u].z + rdo[u].w * ro[u].w;
      }
      if (i < LK) {
        const int io = k6_ioff<NC>(i, c >> 1) + eo;
        uint2 a, b, cc;
        k6_split4(rk[u], a, b, cc);
        *reinterpret_cast<uint2*>(Ks + io) = a;
        *reinterpret_cast<uint2*>(Ks + PK + io) = b;
        *reinterpret_cast<uint2*>(Ks + 2 * PK + io) = cc;
      }
    }
    __syncthreads();
    if ((int)threadIdx.x < LQ) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc += scr[threadIdx.x * NCH + c];
      Ds[threadIdx.x] = acc;
    }
  }
  __syncthreads();

  floatx16 dsv[ML / 32];   // dS of each query tile (fp32; rows: queries 32 it + crow, lane: key j)
  if (kw) {
    floatx16 dV[DT], dK[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        dV[dt][r] = 0.f;
        dK[dt][r] = 0.f;
      }
    const int jc = min(j, lk - 1);
    const bool jok = j < lk;
#pragma unroll
    for (int it = 0; it < ML / 32; ++it) {
      if (it >= NQT) break;
      // the forward's probabilities of this tile, issued ahead of the dP MFMAs (unconditional, clamped)
      float p[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = 32 * it + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const float pv = probs[pbase + (long long)min(i, lq - 1) * lk + jc];
        p[r] = (i < lq && jok) ? pv : 0.f;
      }
      floatx16 dP;
#pragma unroll
      for (int r = 0; r < 16; ++r) dP[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        x6_mma(dP, k6_row<NC>(dOs, 32 * it, ks, lane), k6_row<NC>(dOs + PQ, 32 * it, ks, lane),
               k6_row<NC>(dOs + 2 * PQ, 32 * it, ks, lane), vh[ks], vm[ks], vl[ks]);
      // keep bits of this lane's key for the tile's 16 rows (padding rows / keys: P = 0 above)
      const uint32_t keep = dr.thr != 0u ? k3m_attn_keep_km16(dr, off, rbase + 32 * it, 4 * kl, lk, j) : 0xffffu;
      floatx16 Pd;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int i0 = 32 * it + 8 * a + 4 * kl;
        const float4 d4 = *reinterpret_cast<const float4*>(Ds + i0);
        const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int r = 4 * a + b;
          const float m = k3m_keep_f(keep, r, __float_as_uint(dr.scale));
          Pd[r] = p[r] * m;
          dP[r] = p[r] * (dP[r] * m - dd[b]);   // dS
        }
      }
      dsv[it] = dP;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        x6bf16x8 ph, pm, pl, sh, sm, sl;
        k6_accsplit(Pd, s2, ph, pm, pl);
        k6_accsplit(dP, s2, sh, sm, sl);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const int rb = 32 * it + 16 * s2, cb = 32 * dt;
          x6_mma(dV[dt], k6_tr<NC, true>(dOs, rb, cb, lane), k6_tr<NC, true>(dOs + PQ, rb, cb, lane),
                 k6_tr<NC, true>(dOs + 2 * PQ, rb, cb, lane), ph, pm, pl);
          x6_mma(dK[dt], k6_tr<NC, true>(Qs, rb, cb, lane), k6_tr<NC, true>(Qs + PQ, rb, cb, lane),
                 k6_tr<NC, true>(Qs + 2 * PQ, rb, cb, lane), sh, sm, sl);
        }
      }
    }
    // dV^T / dK^T: lane -> key j, register r -> d = 32 dt + 8 (r >> 2) + 4 kl + (r & 3): 16-B stores
    if (jok) {
      float* pv = dv + (krow0 + j) * lddv + hoff + 4 * kl;
      float* pk = dk + (krow0 + j) * lddk + hoff + 4 * kl;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          *reinterpret_cast<float4*>(pv + 32 * dt + 8 * a) =
              make_float4(dV[dt][4 * a], dV[dt][4 * a + 1], dV[dt][4 * a + 2], dV[dt][4 * a + 3]);
          *reinterpret_cast<float4*>(pk + 32 * dt + 8 * a) =
              make_float4(dK[dt][4 * a] * scale, dK[dt][4 * a + 1] * scale, dK[dt][4 * a + 2] * scale,
                          dK[dt][4 * a + 3] * scale);
        }
    }
  }
  __syncthreads();   // every wave is past its last read of Q / dO
  if (kw) {
    // dS^T[j][i] planes: registers 4a..4a+3 of tile it are queries 32 it + 8 a + 4 kl .. +3 (8 bytes per plane)
#pragma unroll
    for (int it = 0; it < ML / 32; ++it) {
      if (it >= NQT) break;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        uint2 x, y, z;
        k6_split4(make_float4(dsv[it][4 * a], dsv[it][4 * a + 1], dsv[it][4 * a + 2], dsv[it][4 * a + 3]), x, y, z);
        const int io = k6_ioff_n(QNC, j, 4 * it + a) + 4 * kl;
        *reinterpret_cast<uint2*>(dSt + io) = x;
        *reinterpret_cast<uint2*>(dSt + PS + io) = y;
        *reinterpret_cast<uint2*>(dSt + 2 * PS + io) = z;
      }
    }
  }
  __syncthreads();
  // query phase: dQ = scale dS K, tile it of 32 queries per wave (lane -> d, registers -> queries)
  for (int it = w; it < NQT; it += NW) {
    floatx16 oq[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) oq[dt][r] = 0.f;
    for (int kk = 0; kk < LK / 16; ++kk) {
      const x6bf16x8 ah = k6_tr_n(dSt, QNC, 16 * kk, 32 * it, lane);
      const x6bf16x8 am = k6_tr_n(dSt + PS, QNC, 16 * kk, 32 * it, lane);
      const x6bf16x8 al = k6_tr_n(dSt + 2 * PS, QNC, 16 * kk, 32 * it, lane);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        x6_mma(oq[dt], ah, am, al, k6_tr<NC, false>(Ks, 16 * kk, 32 * dt, lane),
               k6_tr<NC, false>(Ks + PK, 16 * kk, 32 * dt, lane), k6_tr<NC, false>(Ks + 2 * PK, 16 * kk, 32 * dt, lane));
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ii = 32 * it + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (ii < lq) {
        float* dst = dq + (qrow0 + ii) * lddq + hoff + cl;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) dst[32 * dt] = oq[dt][r] * scale;
      }
    }
  }
}

size_t bwd_x6km_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const size_t QW = LQ == 96 ? 128 : LQ;
  return 2 * (std::max(6 * LQ * hd, 3 * LK * QW) + 3 * LK * hd) + 4 * (LQ + LQ * (hd / 4));
}

size_t bwd_reg_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  return sizeof(float) * (2 * LQ * hd + LK * hd + LQ + LQ * (hd / 4));
}

size_t fwd_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  return sizeof(float) * (LQ * hd + LK * hd + LQ * LK);
}
size_t bwd_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const size_t r2n = std::max(LK * hd, LQ * LK);
  return sizeof(float) * (LQ * hd + r2n + LQ * LK + ((LK * hd + LQ <= r2n) ? 0 : LQ));
}

constexpr int LDS_MAX = 160 * 1024;

// the staging loads are 16-byte vectors along each row's head slice
bool vec_ok(const void* p, long long ld, int dtype) {
  const int ve = dtype == K3M_BF16 ? 8 : 4;
  return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % ve == 0;
}

template <typename T, int ML, int NW>
void set_lds_attr() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_kernel<T, ML, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)attn_bwd_kernel<T, ML, NW>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    done = true;
  }
}

template <typename T, int ML, int NW>
void launch_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk, int nh, int hd,
                float scale, float p_drop, uint64_t seed, uint64_t off, size_t lds, hipStream_t st) {
  set_lds_attr<T, ML, NW>();
  hipLaunchKernelGGL((attn_fwd_kernel<T, ML, NW>), dim3(nseq * nh), dim3(NW * 64), lds, st, (const T*)q, ldq,
                     (const T*)k, ldk, (const T*)v, ldv, kmask, (T*)ctx, ldc, probs, lq, lk, nh, hd, scale, p_drop,
                     seed, off);
}

template <typename T, int ML, int NW>
void launch_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq, void* dk,
                void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk, int nh, int hd,
                float scale, float p_drop, uint64_t seed, uint64_t off, size_t lds, hipStream_t st) {
  set_lds_attr<T, ML, NW>();
  hipLaunchKernelGGL((attn_bwd_kernel<T, ML, NW>), dim3(nseq * nh), dim3(NW * 64), lds, st, (const T*)dctx, ldc,
                     (const T*)o, ldo, (const T*)q, ldq, (const T*)k, ldk, (const T*)v, ldv, probs, (T*)dq, (T*)dk,
                     (T*)dv, lddq, lddk, lddv, lq, lk, nh, hd, scale, p_drop, seed, off);
}

}  // namespace

// the register-softmax forward serves fp32 heads whose K and V fit 2 workgroups per CU
static const bool kAttnFwdReg = k3m_env_flag("K3M_ATTN_FWD_REG", true);

// the forward's two products on the bf16 matrix cores (bf16x6, attn_fwd_x6_kernel); K3M_ATTN_X6=0 keeps
// the f32-MFMA register kernel
static const bool kAttnX6 = k3m_env_flag("K3M_ATTN_X6", true);

template <int HD>
void launch_fwd_reg(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                    const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk, int nh,
                    float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_fwd_reg_kernel<HD>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)attn_fwd_x6_kernel<HD>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    done = true;
  }
  if (kAttnX6) {
    hipLaunchKernelGGL(attn_fwd_x6_kernel<HD>, dim3(nseq * nh), dim3(256), fwd_x6_lds(lk, HD), st, (const float*)q,
                       ldq, (const float*)k, ldk, (const float*)v, ldv, kmask, (float*)ctx, ldc, probs, lq, lk, nh, scale,
                       p_drop, seed, off);
    return;
  }
  hipLaunchKernelGGL(attn_fwd_reg_kernel<HD>, dim3(nseq * nh), dim3(256), fwd_reg_lds(lk, HD), st, (const float*)q, ldq,
                     (const float*)k, ldk, (const float*)v, ldv, kmask, (float*)ctx, ldc, probs, lq, lk, nh, scale, p_drop,
                     seed, off);
}

extern "C" int k3m_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                            const float* kmask, void* ctx, long long ldc, float* probs, int nseq, int lq, int lk,
                            int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype,
                            hipStream_t st) {
  K3M_ARG(q && k && v && ctx && probs);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && hd > 0 && hd <= MAXD && hd % 32 == 0 && nh > 0);
  if (nseq == 0) return 0;
  K3M_ARG(vec_ok(q, ldq, dtype) && vec_ok(k, ldk, dtype) && vec_ok(v, ldv, dtype));
  K3M_ARG(dtype == K3M_F32 || dtype == K3M_BF16);
  const size_t lds = fwd_lds(lq, lk, hd);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  const bool small = false;   // the forward gains nothing from the short build (measured)
  const int LK = (lk + 31) & ~31;
  if (dtype == K3M_F32 && kAttnFwdReg && (hd == 64 || hd == 96 || hd == 128) && LK * hd <= 8192 &&
      vec_ok(ctx, ldc, dtype) && (reinterpret_cast<uintptr_t>(probs) & 15) == 0) {
    if (hd == 64) launch_fwd_reg<64>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    else if (hd == 96) launch_fwd_reg<96>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    else launch_fwd_reg<128>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    K3M_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == K3M_F32) {
    if (small) launch_fwd<float, 64, 4>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
    else launch_fwd<float, 128, 8>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
  } else {
    if (small) launch_fwd<bf16_t, 64, 4>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
    else launch_fwd<bf16_t, 128, 8>(q, ldq, k, ldk, v, ldv, kmask, ctx, ldc, probs, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

static const bool kAttnBwdReg = k3m_env_flag("K3M_ATTN_BWD_REG", true);
// the fp32 backward's products on the bf16 matrix cores (attn_bwd_x6km_kernel, d = 64): L = 128 260 -> 215 us,
// L = 36 84 -> 68 us per launch, fp32 step +0.6-0.9 % (profiles/r4b_ab_attn_bwd_x6.txt); K3M_ATTN_BWD_X6=0 keeps the
// f32-MFMA kernels
static const bool kAttnBwdX6 = k3m_env_flag("K3M_ATTN_BWD_X6", true);

// d = 128 heads of <= 64 queries and keys (image self-attention, text<->image co-attention) too (A/B knob)
static const bool kAttnBwdX6D128 = k3m_env_flag("K3M_ATTN_BWD_X6_D128", true);

template <int HD, int ML>
void launch_bwd_x6km(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                     const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq, void* dk,
                     void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk, int nh,
                     float scale, float p_drop, uint64_t seed, uint64_t off, size_t lds, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_x6km_kernel<HD, ML>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    done = true;
  }
  hipLaunchKernelGGL((attn_bwd_x6km_kernel<HD, ML>), dim3(nseq * nh), dim3(ML * 2), lds, st, (const float*)dctx, ldc,
                     (const float*)o, ldo, (const float*)q, ldq, (const float*)k, ldk, (const float*)v, ldv, probs,
                     (float*)dq, (float*)dk, (float*)dv, lddq, lddk, lddv, lq, lk, nh, scale, p_drop, seed, off);
}

template <int HD>
void launch_bwd_reg(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                    const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq, void* dk,
                    void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk, int nh,
                    float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t st) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_reg_kernel<HD>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    done = true;
  }
  hipLaunchKernelGGL(attn_bwd_reg_kernel<HD>, dim3(nseq * nh), dim3(256), bwd_reg_lds(lq, lk, HD), st,
                     (const float*)dctx, ldc, (const float*)o, ldo, (const float*)q, ldq, (const float*)k, ldk,
                     (const float*)v, ldv, probs, (float*)dq, (float*)dk, (float*)dv, lddq, lddk, lddv, lq, lk, nh, scale,
                     p_drop, seed, off);
}

extern "C" int k3m_attn_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q, long long ldq,
                            const void* k, long long ldk, const void* v, long long ldv, const float* probs, void* dq,
                            void* dk, void* dv, long long lddq, long long lddk, long long lddv, int nseq, int lq, int lk,
                            int nh, int hd, float scale, float p_drop, uint64_t seed, uint64_t off, int dtype,
                            hipStream_t st) {
  K3M_ARG(dctx && o && q && k && v && probs && dq && dk && dv);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && hd > 0 && hd <= MAXD && hd % 32 == 0 && nh > 0);
  if (nseq == 0) return 0;
  K3M_ARG(vec_ok(q, ldq, dtype) && vec_ok(k, ldk, dtype) && vec_ok(v, ldv, dtype) && vec_ok(dctx, ldc, dtype));
  K3M_ARG(dtype == K3M_F32 || dtype == K3M_BF16);
  const size_t lds = bwd_lds(lq, lk, hd);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  const bool small = lq <= 64 && lk <= 64 && hd <= 64;   // d = 128 runs better as one 8-wave block
  const int LQ = (lq + 31) & ~31;
  const bool x6d128 = kAttnBwdX6D128 && hd == 128 && lq <= 64 && lk <= 64;
  if (dtype == K3M_F32 && kAttnBwdX6 && (hd == 64 || x6d128) && bwd_x6km_lds(lq, lk, hd) <= (size_t)LDS_MAX &&
      vec_ok(o, ldo, dtype) && vec_ok(dk, lddk, dtype) && vec_ok(dv, lddv, dtype)) {
    const size_t xl = bwd_x6km_lds(lq, lk, hd);
    if (hd == 128)
      launch_bwd_x6km<128, 64>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq,
                               lk, nh, scale, p_drop, seed, off, xl, st);
    else if (small)
      launch_bwd_x6km<64, 64>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq,
                              lk, nh, scale, p_drop, seed, off, xl, st);
    else
      launch_bwd_x6km<64, 128>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq,
                               lk, nh, scale, p_drop, seed, off, xl, st);
    K3M_CHECK_LAUNCH();
    return 0;
  }
  // (for LK <= 64 the 64-row LDS kernel is faster: three workgroups per CU against one)
  if (dtype == K3M_F32 && kAttnBwdReg && (hd == 64 || hd == 96 || hd == 128) && LQ * hd <= 8192 && lk > 64 &&
      bwd_reg_lds(lq, lk, hd) <= (size_t)LDS_MAX && vec_ok(o, ldo, dtype) && vec_ok(dk, lddk, dtype) &&
      vec_ok(dv, lddv, dtype)) {
    if (hd == 64) launch_bwd_reg<64>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    else if (hd == 96) launch_bwd_reg<96>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    else launch_bwd_reg<128>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, scale, p_drop, seed, off, st);
    K3M_CHECK_LAUNCH();
    return 0;
  }
  if (dtype == K3M_F32) {
    if (small) launch_bwd<float, 64, 4>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
    else launch_bwd<float, 128, 8>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
  } else {
    if (small) launch_bwd<bf16_t, 64, 4>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
    else launch_bwd<bf16_t, 128, 8>(dctx, ldc, o, ldo, q, ldq, k, ldk, v, ldv, probs, dq, dk, dv, lddq, lddk, lddv, nseq, lq, lk, nh, hd, scale, p_drop, seed, off, lds, st);
  }
  K3M_CHECK_LAUNCH();
  return 0;
}
