// bf16 fused attention for the short K3M sequences (L <= 128, head dim 64, 96 or 128) on
// v_mfma_f32_32x32x16_bf16 — the mixed-precision encoder's attention.
//
// One workgroup (4 waves) per (sequence, head); Q, K, V (and dO) live in LDS as bf16 row-major
// images, 16-B chunk c of row r stored at slot c ^ swz(r) so that both kinds of operand read are
// bank-conflict-free: ds_read_b128 row reads (32 rows x one chunk) and gfx950's transposing
// ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group).
//
// Forward, wave w owns query tile i in [32w, 32w+32):
//   S^T = K Q^T  (A = K rows, B = Q rows; the tile has keys j on the registers and the query i
//                 on the lane, so the softmax over j is in-register + one lane-half exchange)
//   P   = softmax_j(scale S + mask), dropout, row log-sum-exp saved (no L x L probabilities in HBM)
//   O   = P V    (the bf16-converted P registers ARE the A operand — k order permuted as the
//                 accumulator map dictates — and V's B fragments come from transposed reads)
// Backward, wave w first owns query tile i (phase A), then key tile j (phase B):
//   A: recompute S^T and P from the saved LSE, dP^T = V dO^T, dS = P (mask dP - D), write
//      P_drop and dS as bf16 [i][j] images; dQ = scale dS K from registers (as in the forward).
//   B: dV = P_drop^T dO and dK = scale dS^T Q with both operands read transposed from LDS.
// Semantics are those of attention.hip (vilbert_k3m.py:449-464 etc.) with the same dropout counter
// (seed, off + ((s nh + h) lq + i) lk + j), so a mask drawn by one kernel is the other's mask.
#include "flash_frag.h"

#include <algorithm>

namespace {

using namespace k3m_flash;

constexpr int NW = 4, NT = NW * 64;
constexpr int MAXL = 128;
constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;

// stage rows [row0, row0 + nrows) x [coff, coff + 8 NC) of a bf16 matrix into an image
// (rows >= nvalid zero); all loads issued before the LDS writes
template <int NC, int NCI>
__device__ __forceinline__ void stage(uint16_t* img, const uint16_t* __restrict__ src, long long row0, long long ld,
                                      int coff, int nrows, int nvalid) {
  // NC chunks per source row, written into an image laid out with NCI chunks per row
  constexpr int U = MAXL * NC / NT;
  uint4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = threadIdx.x + u * NT;
    const int i = e / NC, c = e % NC;
    // unconditional load from a clamped row, zeroed after it (no per-element branch + vmcnt(0))
    const uint4 x = *reinterpret_cast<const uint4*>(src + (row0 + min(i, nvalid - 1)) * ld + coff + 8 * c);
    r[u] = keep_if(i < nvalid, x);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = threadIdx.x + u * NT;
    const int i = e / NC, c = e % NC;
    if (i < nrows) *reinterpret_cast<uint4*>(img + ioff<NCI>(i, c)) = r[u];
  }
}

// ------------------------------------------------------------------ forward
// PAIR (lq, lk <= 64: the 36-token text, 37-region image and text<->image heads): two heads per workgroup,
// waves 0-1 on head 2p, waves 2-3 on head 2p + 1, so every wave has queries and a workgroup's one memory round
// trip stages two heads (one head per workgroup left two of its four waves idle and doubled the number of
// latency-bound workgroups).  Image row 64 hh + r holds row r of head hh; the key mask is the sequence's, shared.
template <int HD, bool PAIR = false>
__global__ __launch_bounds__(NT, 2) void flash_fwd_kernel(const uint16_t* __restrict__ q, long long ldq,
                                                          const uint16_t* __restrict__ k, long long ldk,
                                                          const uint16_t* __restrict__ v, long long ldv,
                                                          const float* __restrict__ kmask, uint16_t* __restrict__ ctx,
                                                          long long ldc, float* __restrict__ lse, int lq, int lk,
                                                          int nh, float scale, float p_drop, uint64_t seed,
                                                          uint64_t off) {
  // head dim 96 rows are stored 128 wide (the 16-chunk swizzle) and only 12 chunks are used
  constexpr int NCL = HD / 8, NC = HD == 96 ? 16 : HD / 8, DT = HD / 32, KS = HD / 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int nhw = PAIR ? (nh + 1) >> 1 : nh;
  const int s = blockIdx.x / nhw, h0 = PAIR ? 2 * (blockIdx.x % nhw) : blockIdx.x % nhw;
  const int LQh = (lq + 31) & ~31, LKh = (lk + 31) & ~31;     // one head's padded rows
  const int LQ = PAIR ? MAXL : LQh, LK = PAIR ? MAXL : LKh;   // image rows
  uint16_t* Qs = smem;
  constexpr int HW = NC * 8;   // image row width
  uint16_t* Ks = Qs + LQ * HW;
  uint16_t* Vs = Ks + LK * HW;
  float* msk = reinterpret_cast<float*>(Vs + LK * HW);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;

  {
    // every global load (Q, K, V chunks, mask) issued before the first LDS write: one memory round trip
    constexpr int U = MAXL * NCL / NT;
    uint4 rq[U], rk[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NT, i = e / NCL, c = e % NCL;
      const int hh = PAIR ? i >> 6 : 0, li = PAIR ? i & 63 : i;
      const bool hok = !PAIR || h0 + hh < nh;
      const int ho = min(h0 + hh, nh - 1) * HD;
      // unconditional loads from clamped rows, zeroed after the load: a load under a per-element runtime
      // condition makes hipcc branch around it with a vmcnt(0) inside (every load one round trip)
      const bool qv = hok && li < lq, kv = hok && li < lk;
      const long long qo = qrow0 + min(li, lq - 1), ko = krow0 + min(li, lk - 1);
      const uint4 a = *reinterpret_cast<const uint4*>(q + qo * ldq + ho + 8 * c);
      const uint4 b = *reinterpret_cast<const uint4*>(k + ko * ldk + ho + 8 * c);
      const uint4 d = *reinterpret_cast<const uint4*>(v + ko * ldv + ho + 8 * c);
      rq[u] = keep_if(qv, a);
      rk[u] = keep_if(kv, b);
      rv[u] = keep_if(kv, d);
    }
    const int t = threadIdx.x;
    float mv = 0.f;
    if (t < LKh) mv = t < lk ? (kmask ? kmask[krow0 + t] * kLog2e : 0.f) : -INFINITY;   // exp2 domain
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NT, i = e / NCL, c = e % NCL;
      if (i < LQ) *reinterpret_cast<uint4*>(Qs + ioff<NC>(i, c)) = rq[u];
      if (i < LK) {
        *reinterpret_cast<uint4*>(Ks + ioff<NC>(i, c)) = rk[u];
        *reinterpret_cast<uint4*>(Vs + ioff<NC>(i, c)) = rv[u];
      }
    }
    if (t < LKh) msk[t] = mv;
  }
  __syncthreads();
  const int hh = PAIR ? w >> 1 : 0, h = h0 + hh;
  const int rb = 64 * hh;                       // image row of this wave's head's row 0
  const int i0 = 32 * (PAIR ? (w & 1) : w);     // the wave's query tile (head-local)
  if (h >= nh || i0 >= LQh) return;
  const int hoff = h * HD;
  const int NJT = LKh / 32;
  floatx16 S[MAXL / 32];
#pragma unroll
  for (int jt = 0; jt < MAXL / 32; ++jt) {
    if (jt < NJT) {
      floatx16 a = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Ks, rb + 32 * jt, ks, lane),
                                                     rowfrag<NC>(Qs, rb + i0, ks, lane), a, 0, 0, 0);
      S[jt] = a;
    }
  }
  // softmax over j (registers x lane halves) for query i = i0 + cl, in the exp2 domain (scores and mask pre-scaled
  // by log2 e: one multiply per score less than exp(x - max))
  const int i = i0 + cl;
  const float sl2 = scale * kLog2e;
  float mx = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < MAXL / 32; ++jt)
    if (jt < NJT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const float x = fmaf(S[jt][r], sl2, msk[j]);
        S[jt][r] = x;
        mx = fmaxf(mx, x);
      }
    }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int jt = 0; jt < MAXL / 32; ++jt)
    if (jt < NJT) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __builtin_amdgcn_exp2f(S[jt][r] - mx);
        S[jt][r] = e;
        sum += e;
      }
    }
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  const long long prow = ((long long)s * nh + h) * lq + i;   // row of the [nseq, nh, lq] LSE
  if (kl == 0 && i < lq) lse[prow] = mx * kLn2 + __logf(sum);
  if (p_drop > 0.f) {
    // registers 4 q + b of tile jt are keys 32 jt + 8 q + 4 kl + b: pairs (b = 0, 1), (2, 3) share one draw, pair
    // counter pb + 16 jt + 4 q + b / 2 (k3m_attn_drop), the high word mixed once (and once more for a carry)
    const K3mDrop dr = k3m_drop_init(seed, p_drop);
    const uint64_t pb = off + (uint64_t)prow * (uint64_t)((lk + 1) >> 1) + (uint64_t)(2 * kl);
    uint32_t lo = (uint32_t)pb, pre0 = k3m_pair_pre(dr.key, pb), pre1 = k3m_pair_pre(dr.key, pb + (1ull << 32));
    asm volatile("" : "+v"(lo), "+v"(pre0), "+v"(pre1));   // (the high-word multiply stays out of the pair loop)
    // padding keys carry P = 0 (their mask is -inf) and padding query rows are never stored: no per-score bounds test
    const float invs = inv * dr.scale;
#pragma unroll
    for (int jt = 0; jt < MAXL / 32; ++jt)
      if (jt < NJT) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int hb = 0; hb < 2; ++hb) {
            const uint32_t x = lo + (uint32_t)(16 * jt + 4 * q + hb);
            const uint32_t hh = k3m_mix32(x ^ (x < lo ? pre1 : pre0));
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2) {
              const int r = 4 * q + 2 * hb + b2;
              S[jt][r] = k3m_attn_half(hh, b2) >= dr.thr16 ? S[jt][r] * invs : 0.f;
            }
          }
      }
  } else {
#pragma unroll
    for (int jt = 0; jt < MAXL / 32; ++jt)
      if (jt < NJT) {
#pragma unroll
        for (int r = 0; r < 16; ++r) S[jt][r] *= inv;
      }
  }
  // O = P V
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    floatx16 o = zero16();
#pragma unroll
    for (int jt = 0; jt < MAXL / 32; ++jt)
      if (jt < NJT) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(accfrag(S[jt], s2),
                                                       trfrag<NC, true>(Vs, rb + 32 * jt + 16 * s2, 32 * dt, lane),
                                                       o, 0, 0, 0);
      }
    // o[r] = O[i0 + (r&3) + 8(r>>2) + 4kl][32 dt + cl]
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ii = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (ii < lq) ctx[(qrow0 + ii) * ldc + hoff + 32 * dt + cl] = bf_bits(o[r]);
    }
  }
}

// ------------------------------------------------------------------ backward
template <int HD>
__global__ __launch_bounds__(NT, 1) void flash_bwd_kernel(const uint16_t* __restrict__ dctx, long long ldc,
                                                          const uint16_t* __restrict__ o, long long ldo,
                                                          const uint16_t* __restrict__ q, long long ldq,
                                                          const uint16_t* __restrict__ k, long long ldk,
                                                          const uint16_t* __restrict__ v, long long ldv,
                                                          const float* __restrict__ kmask, const float* __restrict__ lse,
                                                          uint16_t* __restrict__ dq, uint16_t* __restrict__ dk,
                                                          uint16_t* __restrict__ dv, long long lddq, long long lddk,
                                                          long long lddv, int lq, int lk, int nh, float scale,
                                                          float p_drop, uint64_t seed, uint64_t off) {
  // head dim 96 rows are stored 128 wide (the 16-chunk swizzle) and only 12 chunks are used
  constexpr int NCL = HD / 8, NC = HD == 96 ? 16 : HD / 8, DT = HD / 32, KS = HD / 16;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const int PW = LK == 96 ? 128 : LK;          // row width of the P / dS images (NC 4, 8 or 16)
  uint16_t* Qs = smem;
  constexpr int HW = NC * 8;   // image row width
  uint16_t* dOs = Qs + LQ * HW;
  uint16_t* Ks = dOs + LQ * HW;
  uint16_t* Vs = Ks + LK * HW;
  uint16_t* Ps = Vs + LK * HW;                 // [LQ][PW] P_drop
  uint16_t* dSs = Ps + LQ * PW;                // [LQ][PW] dS
  float* msk = reinterpret_cast<float*>(dSs + LQ * PW);
  float* Ls = msk + LK;
  float* Ds = Ls + LQ;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long lrow0 = ((long long)s * nh + h) * lq;

  stage<NCL, NC>(Qs, q, qrow0, ldq, hoff, LQ, lq);
  stage<NCL, NC>(dOs, dctx, qrow0, ldc, hoff, LQ, lq);
  stage<NCL, NC>(Ks, k, krow0, ldk, hoff, LK, lk);
  stage<NCL, NC>(Vs, v, krow0, ldv, hoff, LK, lk);
  for (int j = threadIdx.x; j < LK; j += NT) msk[j] = j < lk ? (kmask ? kmask[krow0 + j] : 0.f) : -INFINITY;
  {
    // D_i = dO_i . O_i: two threads per row, each over half of the head dimension (16-B loads)
    const int ii = threadIdx.x >> 1, half = threadIdx.x & 1;
    float acc = 0.f;
    if (ii < lq) {
      const uint16_t* pd = dctx + (qrow0 + ii) * ldc + hoff + half * (HD / 2);
      const uint16_t* po = o + (qrow0 + ii) * ldo + hoff + half * (HD / 2);
      uint4 a[HD / 16], b[HD / 16];
#pragma unroll
      for (int c = 0; c < HD / 16; ++c) {
        a[c] = *reinterpret_cast<const uint4*>(pd + 8 * c);
        b[c] = *reinterpret_cast<const uint4*>(po + 8 * c);
      }
#pragma unroll
      for (int c = 0; c < HD / 16; ++c) {
        const uint32_t wa[4] = {a[c].x, a[c].y, a[c].z, a[c].w}, wb[4] = {b[c].x, b[c].y, b[c].z, b[c].w};
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc += __uint_as_float(wa[t] << 16) * __uint_as_float(wb[t] << 16) +
                 __uint_as_float(wa[t] & 0xffff0000u) * __uint_as_float(wb[t] & 0xffff0000u);
      }
    }
    acc += __shfl_xor(acc, 1, 64);
    if (half == 0 && ii < LQ) {
      Ds[ii] = acc;
      Ls[ii] = ii < lq ? lse[lrow0 + ii] : 0.f;
    }
  }
  __syncthreads();

  const int NJT = LK / 32;
  // ---- phase A: wave w owns query tile i0 = 32 w
  const int i0 = 32 * w;
  if (i0 < LQ) {
    const int i = i0 + cl;
    const float li = Ls[i], di = Ds[i];
    const bool iv = i < lq;
    floatx16 dQ[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dQ[dt] = zero16();
#pragma unroll
    for (int jt = 0; jt < MAXL / 32; ++jt) {
      if (jt >= NJT) break;
      floatx16 St = zero16(), dP = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        St = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Ks, 32 * jt, ks, lane), rowfrag<NC>(Qs, i0, ks, lane),
                                                      St, 0, 0, 0);
        dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Vs, 32 * jt, ks, lane), rowfrag<NC>(dOs, i0, ks, lane),
                                                      dP, 0, 0, 0);
      }
      floatx16 pd, ds;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * kl;
        const float p = iv ? __expf(St[r] * scale + msk[j] - li) : 0.f;
        const float dm = (p_drop > 0.f && iv && j < lk) ? k3m_attn_dropout_scale(seed, p_drop, off, lrow0 + i, lk, j) : 1.f;
        pd[r] = p * dm;
        ds[r] = p * (dP[r] * dm - di);
      }
      // P_drop and dS -> [i][j] images: registers 4g..4g+3 are 4 consecutive keys (8 bytes)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 4 * jt + g;   // chunk of keys 32 jt + 8 g .. +7; this lane half holds 4 kl .. 4 kl + 3
        uint2 wp, wd;
        wp.x = bf_bits(pd[4 * g]) | ((uint32_t)bf_bits(pd[4 * g + 1]) << 16);
        wp.y = bf_bits(pd[4 * g + 2]) | ((uint32_t)bf_bits(pd[4 * g + 3]) << 16);
        wd.x = bf_bits(ds[4 * g]) | ((uint32_t)bf_bits(ds[4 * g + 1]) << 16);
        wd.y = bf_bits(ds[4 * g + 2]) | ((uint32_t)bf_bits(ds[4 * g + 3]) << 16);
        int po;
        if (PW == 128) po = ioff<16>(i, c);
        else if (PW == 64) po = ioff<8>(i, c);
        else po = ioff<4>(i, c);
        *reinterpret_cast<uint2*>(Ps + po + 4 * kl) = wp;
        *reinterpret_cast<uint2*>(dSs + po + 4 * kl) = wd;
      }
      // dQ += dS K (dS registers as the A operand, K transposed)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 a = accfrag(ds, s2);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
          dQ[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, trfrag<NC, true>(Ks, 32 * jt + 16 * s2, 32 * dt, lane),
                                                            dQ[dt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ii = i0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (ii < lq) dq[(qrow0 + ii) * lddq + hoff + 32 * dt + cl] = bf_bits(dQ[dt][r] * scale);
      }
  }
  __syncthreads();
  // ---- phase B: wave w owns key tile j0 = 32 w: dV = P_drop^T dO, dK = scale dS^T Q
  const int j0 = 32 * w;
  if (j0 >= LK) return;
  floatx16 dV[DT], dK[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dV[dt] = zero16();
    dK[dt] = zero16();
  }
  for (int ik = 0; ik < LQ / 16; ++ik) {
    bf16x8 ap, as;
    if (PW == 128) {
      ap = trfrag<16, false>(Ps, 16 * ik, j0, lane);
      as = trfrag<16, false>(dSs, 16 * ik, j0, lane);
    } else if (PW == 64) {
      ap = trfrag<8, false>(Ps, 16 * ik, j0, lane);
      as = trfrag<8, false>(dSs, 16 * ik, j0, lane);
    } else {
      ap = trfrag<4, false>(Ps, 16 * ik, j0, lane);
      as = trfrag<4, false>(dSs, 16 * ik, j0, lane);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dV[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ap, trfrag<NC, false>(dOs, 16 * ik, 32 * dt, lane), dV[dt], 0, 0, 0);
      dK[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as, trfrag<NC, false>(Qs, 16 * ik, 32 * dt, lane), dK[dt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int j = j0 + (r & 3) + 8 * (r >> 2) + 4 * kl;
      if (j < lk) {
        dv[(krow0 + j) * lddv + hoff + 32 * dt + cl] = bf_bits(dV[dt][r]);
        dk[(krow0 + j) * lddk + hoff + 32 * dt + cl] = bf_bits(dK[dt][r] * scale);
      }
    }
}

// ------------------------------------------------------------------ backward, keys on the lanes
// The default backward (flash_bwd_kernel above holds P and dS as two [LQ][LK] LDS images: 132 KB at
// L = 128, one 4-wave workgroup per CU).  Here the probabilities never leave the registers:
//   key phase   wave w owns keys j0 = 32 w .. +31 on the MFMA lanes (its K and V rows are B-operand
//               fragments in registers, loaded straight from global); per 32-query tile
//                 S = Q K^T, dP = dO V^T            (A = Q / dO rows from LDS, 16-B reads)
//                 P = exp(scale S + mask - LSE), Pd = P m, dS = P (dP m - D)     (in accumulators)
//                 dV^T += dO^T Pd, dK^T += Q^T dS   (A = transposed LDS reads in the accumulator k
//                                                    order, B = the accumulators themselves)
//               and dS stays packed (bf16) in registers;
//   dS^T image  written once to LDS over the Q / dO images (every wave is past its last read);
//   query phase dQ = scale dS K per 32-query tile (A = dS from the transposed image, B = K from LDS).
// LDS at L = 128, d = 64: Q + dO + K = 48 KB (+ 1.5 KB vectors): two or three workgroups per CU instead
// of one.  Same semantics and dropout counters as flash_bwd_kernel / the forward.
template <int NC>
__device__ __forceinline__ bf16x8 trfrag_n(const uint16_t* img, int nc, int rbase, int cbase, int lane) {
  if (nc == 4) return trfrag<4, false>(img, rbase, cbase, lane);
  if (nc == 8) return trfrag<8, false>(img, rbase, cbase, lane);
  return trfrag<16, false>(img, rbase, cbase, lane);
}
__device__ __forceinline__ int ioff_n(int nc, int r, int c) {
  return nc == 4 ? ioff<4>(r, c) : nc == 8 ? ioff<8>(r, c) : ioff<16>(r, c);
}

template <int HD>
constexpr int km_occupancy() { return HD == 64 ? 2 : 1; }

template <int HD, int NW>
__global__ __launch_bounds__(NW * 64, km_occupancy<HD>()) void flash_bwd_km_kernel(
    const uint16_t* __restrict__ dctx, long long ldc, const uint16_t* __restrict__ o, long long ldo,
    const uint16_t* __restrict__ q, long long ldq, const uint16_t* __restrict__ k, long long ldk,
    const uint16_t* __restrict__ v, long long ldv, const float* __restrict__ kmask, const float* __restrict__ lse,
    uint16_t* __restrict__ dq, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, long long lddq, long long lddk,
    long long lddv, int lq, int lk, int nh, float scale, float p_drop, uint64_t seed, uint64_t off) {
  constexpr int NTH = NW * 64;
  constexpr int NCL = HD / 8, NC = HD == 96 ? 16 : HD / 8, DT = HD / 32, KS = HD / 16;
  constexpr int HW = NC * 8;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  const int QW = LQ == 96 ? 128 : LQ, QNC = QW / 8;      // dS^T image [LK][QW]
  const int RQ = max(2 * LQ * HW, LK * QW);               // the region shared by Q | dO and dS^T
  uint16_t* Qs = smem;
  uint16_t* dOs = Qs + LQ * HW;
  uint16_t* dSt = smem;
  uint16_t* Ks = smem + RQ;
  float* msk = reinterpret_cast<float*>(Ks + LK * HW);
  float* Ls = msk + LK;
  float* Ds = Ls + LQ;
  float* scr = Ds + LQ;   // [LQ][NCL] chunk dot products of dO and O
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long lrow0 = ((long long)s * nh + h) * lq;
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const int NQT = LQ >> 5;

  // this wave's key tile: K and V rows as B-operand fragments (lane -> key j, 8 consecutive d)
  const int j = 32 * w + cl;
  const bool kw = 32 * w < LK;   // wave-uniform
  bf16x8 kf[KS], vf[KS];
  {
    const bool ok = kw && j < lk;
    const uint16_t* kp = k + (krow0 + min(j, lk - 1)) * ldk + hoff + 8 * kl;
    const uint16_t* vp = v + (krow0 + min(j, lk - 1)) * ldv + hoff + 8 * kl;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const uint4 a = *reinterpret_cast<const uint4*>(kp + 16 * ks);
      const uint4 b = *reinterpret_cast<const uint4*>(vp + 16 * ks);
      kf[ks] = __builtin_bit_cast(bf16x8, keep_if(ok, a));
      vf[ks] = __builtin_bit_cast(bf16x8, keep_if(ok, b));
    }
  }
  {
    // prologue: every global load (Q, dO, O, K chunks; mask; LSE) issued before the first LDS write, so
    // the workgroup waits for one memory round trip, not four.  Thread t takes chunks e = t + u NTH
    // (row e / NCL, chunk e % NCL); D_i = dO_i . O_i from per-chunk dot products summed over the row.
    constexpr int U = (MAXL * NCL + NTH - 1) / NTH;
    uint4 rq[U], rdo[U], ro[U], rk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCL, c = e % NCL;
      // unconditional loads from clamped rows, zeroed after the load (see flash_fwd_kernel)
      const bool qv = i < lq, kv = i < lk;
      const long long qo = qrow0 + min(i, lq - 1), ko = krow0 + min(i, lk - 1);
      const uint4 a = *reinterpret_cast<const uint4*>(q + qo * ldq + hoff + 8 * c);
      const uint4 b = *reinterpret_cast<const uint4*>(dctx + qo * ldc + hoff + 8 * c);
      const uint4 d = *reinterpret_cast<const uint4*>(o + qo * ldo + hoff + 8 * c);
      const uint4 f = *reinterpret_cast<const uint4*>(k + ko * ldk + hoff + 8 * c);
      rq[u] = keep_if(qv, a);
      rdo[u] = keep_if(qv, b);
      ro[u] = keep_if(qv, d);
      rk[u] = keep_if(kv, f);
    }
    float mv = 0.f, lv = 0.f;
    const int t = threadIdx.x;
    if (t < LK) mv = t < lk ? (kmask ? kmask[krow0 + t] : 0.f) : -INFINITY;
    if (t < LQ) lv = t < lq ? lse[lrow0 + t] : INFINITY;   // padding query rows: P = exp(-inf) = 0
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * NTH, i = e / NCL, c = e % NCL;
      if (i < LQ) {
        *reinterpret_cast<uint4*>(Qs + ioff<NC>(i, c)) = rq[u];
        *reinterpret_cast<uint4*>(dOs + ioff<NC>(i, c)) = rdo[u];
        const uint32_t wa[4] = {rdo[u].x, rdo[u].y, rdo[u].z, rdo[u].w}, wb[4] = {ro[u].x, ro[u].y, ro[u].z, ro[u].w};
        float acc = 0.f;
#pragma unroll
        for (int t2 = 0; t2 < 4; ++t2)
          acc += __uint_as_float(wa[t2] << 16) * __uint_as_float(wb[t2] << 16) +
                 __uint_as_float(wa[t2] & 0xffff0000u) * __uint_as_float(wb[t2] & 0xffff0000u);
        scr[e] = acc;
      }
      if (i < LK) *reinterpret_cast<uint4*>(Ks + ioff<NC>(i, c)) = rk[u];
    }
    if (t < LK) msk[t] = mv;
    __syncthreads();
    if (t < LQ) {
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < NCL; ++c) acc += scr[t * NCL + c];
      Ds[t] = acc;
      Ls[t] = lv;
    }
  }
  __syncthreads();

  uint32_t dsp[MAXL / 32][8];   // dS of each query tile, bf16 pairs (registers 2t, 2t + 1)
  if (kw) {
    const float mj = msk[j];
    floatx16 dV[DT], dK[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      dV[dt] = zero16();
      dK[dt] = zero16();
    }
#pragma unroll
    for (int it = 0; it < MAXL / 32; ++it) {
      if (it >= NQT) break;
      // dropout keep bits of this lane's key for the tile's 16 query rows (register r), drawn before the products;
      // padding rows and keys draw unused values (P = 0 there)
      const uint32_t keep = dr.thr != 0u ? k3m_attn_keep_km16(dr, off, lrow0 + 32 * it, 4 * kl, lk, j) : 0xffffu;
      floatx16 S = zero16(), dP = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Qs, 32 * it, ks, lane), kf[ks], S, 0, 0, 0);
        dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(dOs, 32 * it, ks, lane), vf[ks], dP, 0, 0, 0);
      }
      // accumulator r holds query i = 32 it + 8 (r >> 2) + 4 kl + (r & 3), key j
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int i0 = 32 * it + 8 * a + 4 * kl;
        const float4 l4 = *reinterpret_cast<const float4*>(Ls + i0);
        const float4 d4 = *reinterpret_cast<const float4*>(Ds + i0);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int r = 4 * a + b;
          const float p = __expf(S[r] * scale + mj - lv[b]);
          const float dm = k3m_keep_f(keep, r, __float_as_uint(dr.scale));
          S[r] = p * dm;                          // P_drop
          dP[r] = p * (dP[r] * dm - dv4[b]);      // dS
        }
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) dsp[it][t] = (uint32_t)bf_bits(dP[2 * t]) | ((uint32_t)bf_bits(dP[2 * t + 1]) << 16);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 bp = accfrag(S, s2), bs = accfrag(dP, s2);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dV[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(dOs, 32 * it + 16 * s2, 32 * dt, lane), bp,
                                                            dV[dt], 0, 0, 0);
          dK[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(Qs, 32 * it + 16 * s2, 32 * dt, lane), bs,
                                                            dK[dt], 0, 0, 0);
        }
      }
    }
    // dV^T / dK^T: lane -> key j, register r -> d = 32 dt + 8 (r >> 2) + 4 kl + (r & 3): 8-B stores
    if (j < lk) {
      uint16_t* pv = dv + (krow0 + j) * lddv + hoff + 4 * kl;
      uint16_t* pk = dk + (krow0 + j) * lddk + hoff + 4 * kl;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          uint2 wv, wk;
          wv.x = bf_bits(dV[dt][4 * a]) | ((uint32_t)bf_bits(dV[dt][4 * a + 1]) << 16);
          wv.y = bf_bits(dV[dt][4 * a + 2]) | ((uint32_t)bf_bits(dV[dt][4 * a + 3]) << 16);
          wk.x = bf_bits(dK[dt][4 * a] * scale) | ((uint32_t)bf_bits(dK[dt][4 * a + 1] * scale) << 16);
          wk.y = bf_bits(dK[dt][4 * a + 2] * scale) | ((uint32_t)bf_bits(dK[dt][4 * a + 3] * scale) << 16);
          *reinterpret_cast<uint2*>(pv + 32 * dt + 8 * a) = wv;
          *reinterpret_cast<uint2*>(pk + 32 * dt + 8 * a) = wk;
        }
    }
  }
  __syncthreads();   // every wave is past its last read of Q / dO
  if (kw) {
    // dS^T[j][i]: registers 4a..4a+3 of query tile it are queries 32 it + 8 a + 4 kl .. +3 (8 bytes)
#pragma unroll
    for (int it = 0; it < MAXL / 32; ++it) {
      if (it >= NQT) break;
#pragma unroll
      for (int a = 0; a < 4; ++a)
        *reinterpret_cast<uint2*>(dSt + ioff_n(QNC, j, 4 * it + a) + 4 * kl) = make_uint2(dsp[it][2 * a], dsp[it][2 * a + 1]);
    }
  }
  __syncthreads();
  // query phase: dQ = scale dS K, tile it of 32 queries per wave (lane -> d, registers -> queries)
  for (int it = w; it < NQT; it += NW) {
    floatx16 dQ[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dQ[dt] = zero16();
    for (int kk = 0; kk < LK / 16; ++kk) {
      const bf16x8 a = trfrag_n<NC>(dSt, QNC, 16 * kk, 32 * it, lane);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        dQ[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, trfrag<NC, false>(Ks, 16 * kk, 32 * dt, lane), dQ[dt], 0, 0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ii = 32 * it + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (ii < lq) dq[(qrow0 + ii) * lddq + hoff + 32 * dt + cl] = bf_bits(dQ[dt][r] * scale);
      }
  }
}

size_t bwd_km_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  if (hd == 96) hd = 128;
  const size_t QW = LQ == 96 ? 128 : LQ;
  return 2 * (std::max(2 * LQ * hd, LK * QW) + LK * hd) + 4 * (LK + 2 * LQ) + 4 * LQ * (hd / 8);
}

size_t fwd_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  if (hd == 96) hd = 128;
  return 2 * (LQ * hd + 2 * LK * hd) + 4 * LK;
}
size_t bwd_lds(int lq, int lk, int hd) {
  const size_t LQ = (lq + 31) & ~31, LK = (lk + 31) & ~31;
  if (hd == 96) hd = 128;
  const size_t PW = LK == 96 ? 128 : LK;
  return 2 * (2 * LQ * hd + 2 * LK * hd + 2 * LQ * PW) + 4 * (LK + 2 * LQ);
}

constexpr int LDS_MAX = 160 * 1024;

void set_attrs() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)flash_fwd_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_fwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_fwd_kernel<96>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_fwd_kernel<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_kernel<96>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<64, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<64, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<96, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<96, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<128, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_bwd_km_kernel<128, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    done = true;
  }
}

bool vec_ok(const void* p, long long ld) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 8 == 0; }

}  // namespace

// two heads per forward workgroup for lq, lk <= 64 (flash_fwd_kernel PAIR); K3M_FLASH_PAIR=0 keeps one (A/B knob)
static const bool kFlashPair = k3m_env_flag("K3M_FLASH_PAIR", true);

// the key-major backward (flash_bwd_km_kernel); K3M_FLASH_BWD_KM=0 keeps the P / dS image kernel
static const bool kFlashBwdKM = k3m_env_flag("K3M_FLASH_BWD_KM", true);

extern "C" int k3m_flash_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                                  long long ldv, const float* kmask, void* ctx, long long ldc, float* lse, int nseq,
                                  int lq, int lk, int nh, int hd, float scale, float p_drop, uint64_t seed,
                                  uint64_t off, hipStream_t st) {
  K3M_ARG(q && k && v && ctx && lse);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && (hd == 64 || hd == 96 || hd == 128) && nh > 0 && nseq >= 0);
  K3M_ARG(vec_ok(q, ldq) && vec_ok(k, ldk) && vec_ok(v, ldv));
  if (nseq == 0) return 0;
  // (d = 64 only: a d = 128 pair needs 98 KB of LDS, one workgroup per CU = 2 heads, against 3 single-head
  // workgroups of 49 KB)
  const bool pair = kFlashPair && hd == 64 && lq <= 64 && lk <= 64 && nh > 1;
  const size_t lds = pair ? fwd_lds(MAXL, MAXL, hd) : fwd_lds(lq, lk, hd);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  set_attrs();
  const int nblk = nseq * (pair ? (nh + 1) / 2 : nh);
#define K3M_FLASH_FWD(HD_, P_)                                                                                   \
  hipLaunchKernelGGL((flash_fwd_kernel<HD_, P_>), dim3(nblk), dim3(NT), lds, st, (const uint16_t*)q, ldq,           \
                     (const uint16_t*)k, ldk, (const uint16_t*)v, ldv, kmask, (uint16_t*)ctx, ldc, lse, lq, lk, nh, \
                     scale, p_drop, seed, off)
  if (hd == 96) K3M_FLASH_FWD(96, false);
  else if (hd == 64) {
    if (pair) K3M_FLASH_FWD(64, true); else K3M_FLASH_FWD(64, false);
  } else K3M_FLASH_FWD(128, false);
#undef K3M_FLASH_FWD
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_flash_attn_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q,
                                  long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                                  const float* kmask, const float* lse, void* dq, void* dk, void* dv, long long lddq,
                                  long long lddk, long long lddv, int nseq, int lq, int lk, int nh, int hd,
                                  float scale, float p_drop, uint64_t seed, uint64_t off, hipStream_t st) {
  K3M_ARG(dctx && o && q && k && v && lse && dq && dk && dv);
  K3M_ARG(lq > 0 && lq <= MAXL && lk > 0 && lk <= MAXL && (hd == 64 || hd == 96 || hd == 128) && nh > 0 && nseq >= 0);
  K3M_ARG(vec_ok(q, ldq) && vec_ok(k, ldk) && vec_ok(v, ldv) && vec_ok(dctx, ldc) && vec_ok(o, ldo));
  if (nseq == 0) return 0;
  set_attrs();
  if (kFlashBwdKM && vec_ok(dk, lddk) && vec_ok(dv, lddv)) {
    const size_t lk_lds = bwd_km_lds(lq, lk, hd);
    K3M_ARG(lk_lds <= (size_t)LDS_MAX);
#define K3M_FLASH_BWD_KM(HD_, NW_)                                                                                     \
  hipLaunchKernelGGL((flash_bwd_km_kernel<HD_, NW_>), dim3(nseq * nh), dim3(NW_ * 64), lk_lds, st, (const uint16_t*)dctx, \
                     ldc, (const uint16_t*)o, ldo, (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v, \
                     ldv, kmask, lse, (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, lq, lk, nh, scale,   \
                     p_drop, seed, off)
    const bool two = lk <= 64;   // two waves own the key tiles of a short head: smaller workgroups, more per CU
    if (hd == 64) {
      if (two) K3M_FLASH_BWD_KM(64, 2); else K3M_FLASH_BWD_KM(64, 4);
    } else if (hd == 96) {
      if (two) K3M_FLASH_BWD_KM(96, 2); else K3M_FLASH_BWD_KM(96, 4);
    } else {
      if (two) K3M_FLASH_BWD_KM(128, 2); else K3M_FLASH_BWD_KM(128, 4);
    }
#undef K3M_FLASH_BWD_KM
    K3M_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = bwd_lds(lq, lk, hd);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  if (hd == 96)
    hipLaunchKernelGGL(flash_bwd_kernel<96>, dim3(nseq * nh), dim3(NT), lds, st, (const uint16_t*)dctx, ldc,
                       (const uint16_t*)o, ldo, (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v,
                       ldv, kmask, lse, (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, lq, lk, nh,
                       scale, p_drop, seed, off);
  else if (hd == 64)
    hipLaunchKernelGGL(flash_bwd_kernel<64>, dim3(nseq * nh), dim3(NT), lds, st, (const uint16_t*)dctx, ldc,
                       (const uint16_t*)o, ldo, (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v,
                       ldv, kmask, lse, (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, lq, lk, nh,
                       scale, p_drop, seed, off);
  else
    hipLaunchKernelGGL(flash_bwd_kernel<128>, dim3(nseq * nh), dim3(NT), lds, st, (const uint16_t*)dctx, ldc,
                       (const uint16_t*)o, ldo, (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v,
                       ldv, kmask, lse, (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, lq, lk, nh,
                       scale, p_drop, seed, off);
  K3M_CHECK_LAUNCH();
  return 0;
}
