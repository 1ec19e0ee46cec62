// bf16 flash attention for sequences longer than 128, up to max_position_embeddings = 512
// (config/bert_base_6layer_6conect.json:8) — the mixed-precision encoder's attention wherever a side of
// the score matrix exceeds the whole-head kernels of attention_bf16.hip: the 320-token PV stream of
// BASELINE configs[4] in its self-attention (320 x 320, d = 64), its co-attention with the image (320 x 37 /
// 37 x 320, d = 128) and with the title (320 x 36 / 36 x 320, d = 96), and the fine-tuning PV 256.
// Reference semantics: BertSelfAttention vilbert_k3m.py:439-475, BertBiAttention :753-838,
// BertBiAttention_two_text :904-965 — scores = QK^T / sqrt(d) + mask, softmax, dropout, context = P V.
//
// Nothing of size L x L is written to HBM (the exact-fp32 attention_long.hip saves the fp32 probabilities:
// 629 MB per PV self-attention at config 5); the forward saves the row log-sum-exp, the backward
// recomputes P from it.  Same dropout counters as every other attention kernel:
// u(seed, off + ((s nh + h) lq + i) lk + j), so a mask drawn here is the mask of attention.hip.
//
// Forward (flash_long_fwd_kernel): workgroup = (sequence, head, block of 128 queries), 4 waves; wave w
// keeps its 32 queries on the MFMA lanes (Q fragments in registers) and streams the keys in chunks of
// 64 through a double-buffered LDS ring (register prefetch of chunk c+1 while chunk c computes):
//   S^T = K Q^T           keys on the accumulator registers, the query on the lane
//   online softmax        running max / sum per lane (one lane-half exchange per chunk, exp2 domain)
//   O^T = V^T P^T         A = transposed reads of the V image, B = the bf16 P registers themselves;
//                         queries stay on the lanes, so the rescale exp2(m_old - m_new) is a per-lane scalar.
// Backward (flash_long_bwd_kernel): workgroup = (sequence, head, group of key tiles), wave w owns 32 keys
// (their K / V rows in the group's LDS images, dK^T / dV^T accumulators in registers), and the queries stream
// through LDS in chunks of 32 together with their LSE and D = rowsum(dO o O) (flash_long_prep_kernel):
//   key phase   S = Q K^T, dP = dO V^T, P = exp2(S' + mask' - LSE'), Pd = P m, dS = P (dP m - D),
//               dV^T += dO^T Pd, dK^T += Q^T dS (as flash_bwd_km_kernel), dS^T tile -> LDS image
//   dQ phase    dQ[chunk] = dS K over the group's keys: 16x16x32 MFMA tiles dealt to the waves
//               (A = dS from the dS^T image, B = K from the group's K image, both transposing reads)
// A head whose keys exceed one workgroup's register budget is split into key groups; each group then
// writes an fp32 dQ partial and flash_long_dq_reduce_kernel sums them in group order (deterministic).
#include "flash_frag.h"

#include <algorithm>

namespace {

using namespace k3m_flash;

constexpr int LMAX = 512;
constexpr int FKC = 64;     // keys per forward LDS chunk
constexpr int FNT = 256;    // forward threads (4 waves x 32 queries)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

template <int HD> struct Geo {
  static constexpr int NCL = HD / 8;                  // 16-B chunks of a head row
  static constexpr int NC = HD == 96 ? 16 : HD / 8;   // chunk slots of an image row (96 stored 128 wide)
  static constexpr int HW = NC * 8;                   // image row width (bf16)
  static constexpr int DT = HD / 32, KS = HD / 16;
};

// ------------------------------------------------------------------ forward
template <int HD>
__global__ __launch_bounds__(FNT, 2) void flash_long_fwd_kernel(const uint16_t* __restrict__ q, long long ldq,
                                                                const uint16_t* __restrict__ k, long long ldk,
                                                                const uint16_t* __restrict__ v, long long ldv,
                                                                const float* __restrict__ kmask,
                                                                uint16_t* __restrict__ ctx, long long ldc,
                                                                float* __restrict__ lse, int lq, int lk, int nh,
                                                                float scale, float p_drop, uint64_t seed,
                                                                uint64_t off) {
  using G = Geo<HD>;
  constexpr int NCL = G::NCL, NC = G::NC, HW = G::HW, DT = G::DT, KS = G::KS;
  constexpr int U = (FKC * NCL + FNT - 1) / FNT;   // 16-B chunks per thread per operand and key chunk
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Ks = smem;                              // [2][FKC][HW]
  uint16_t* Vs = Ks + 2 * FKC * HW;                 // [2][FKC][HW]
  float* msk = reinterpret_cast<float*>(Vs + 2 * FKC * HW);   // [LKP] mask * log2 e, -inf past lk
  const int s = blockIdx.x / nh, h = blockIdx.x % nh;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const int nkc = (lk + FKC - 1) / FKC, LKP = nkc * FKC;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const int qw0 = blockIdx.y * (FNT / 2) + 32 * w;  // first query of this wave
  const bool wact = qw0 < lq;                       // wave-uniform
  const int i = qw0 + cl;
  const bool iv = i < lq;
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const float sl2 = scale * LOG2E;
  const long long prow = ((long long)s * nh + h) * lq + min(i, lq - 1);   // row of the [nseq, nh, lq] LSE

  // Q fragments (B operand of S^T = K Q^T): lane -> query i, k = head dims 16 ks + 8 kl .. +7
  bf16x8 qf[KS];
  {
    const uint16_t* qp = q + (qrow0 + min(i, lq - 1)) * ldq + hoff + 8 * kl;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, keep_if(iv, *reinterpret_cast<const uint4*>(qp + 16 * ks)));
  }
  uint4 rk[U], rv[U];
  auto load = [&](int c) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * FNT, r = e / NCL, cc = e % NCL;
      const int j = c * FKC + r;
      // unconditional loads from clamped rows, zeroed after the load (no branch + vmcnt(0) per element)
      const long long ko = krow0 + min(j, lk - 1);
      const bool ok = j < lk && (FKC * NCL % FNT == 0 || e < FKC * NCL);
      rk[u] = keep_if(ok, *reinterpret_cast<const uint4*>(k + ko * ldk + hoff + 8 * cc));
      rv[u] = keep_if(ok, *reinterpret_cast<const uint4*>(v + ko * ldv + hoff + 8 * cc));
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = threadIdx.x + u * FNT, r = e / NCL, cc = e % NCL;
      if (FKC * NCL % FNT == 0 || e < FKC * NCL) {
        *reinterpret_cast<uint4*>(Ks + buf * FKC * HW + ioff<NC>(r, cc)) = rk[u];
        *reinterpret_cast<uint4*>(Vs + buf * FKC * HW + ioff<NC>(r, cc)) = rv[u];
      }
    }
  };
  load(0);
  for (int t = threadIdx.x; t < LKP; t += FNT)
    msk[t] = t < lk ? (kmask ? kmask[krow0 + t] * LOG2E : 0.f) : -INFINITY;
  store(0);
  __syncthreads();

  floatx16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = zero16();
  float m2 = -INFINITY, lp = 0.f;   // running max (log2 units, shared by the lane pair) and this lane's partial sum
  for (int c = 0; c < nkc; ++c) {
    if (c + 1 < nkc) load(c + 1);
    if (wact) {
      const uint16_t* Kb = Ks + (c & 1) * FKC * HW;
      const uint16_t* Vb = Vs + (c & 1) * FKC * HW;
      floatx16 S[FKC / 32];
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt) {
        floatx16 a = zero16();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Kb, 32 * jt, ks, lane), qf[ks], a, 0, 0, 0);
        S[jt] = a;
      }
      // S^T register r of tile jt: key j = c FKC + 32 jt + (r & 3) + 8 (r >> 2) + 4 kl, query i = this lane
      float mc = -INFINITY;
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = c * FKC + 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * kl;
          const float x = fmaf(S[jt][r], sl2, msk[j]);
          S[jt][r] = x;
          mc = fmaxf(mc, x);
        }
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m2, mc);
      const float mref = mn == -INFINITY ? 0.f : mn;   // a row with every key so far at -inf: keep exp2 finite
      const float alpha = __builtin_amdgcn_exp2f(m2 - mref);
      m2 = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      // keys past lk draw an unused value (p = 0 there)
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f(S[jt][r] - mref);
          lp = jt == 0 && r == 0 ? fmaf(lp, alpha, p) : lp + p;   // the rescale fused explicitly (fwd2 does the same)
          S[jt][r] = p * k3m_attn_drop(dr, off, prow, lk, c * FKC + 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * kl);
        }
      // O^T += V^T P^T: A = V image read transposed in the accumulator k order, B = P from the registers
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 b = accfrag(S[jt], s2);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(Vb, 32 * jt + 16 * s2, 32 * dt, lane), b,
                                                             o[dt], 0, 0, 0);
        }
    }
    if (c + 1 < nkc) store((c + 1) & 1);
    __syncthreads();
  }
  if (!wact) return;
  const float lt = lp + __shfl_xor(lp, 32, 64);
  const float inv = 1.f / lt;
  if (kl == 0 && iv) lse[prow] = m2 * LN2 + __logf(lt);
  if (iv) {
    // O^T register r of tile dt: head dim 32 dt + (r & 3) + 8 (r >> 2) + 4 kl -> 4 consecutive dims per 8-B store
    uint16_t* op = ctx + (qrow0 + i) * ldc + hoff + 4 * kl;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        uint2 wv;
        wv.x = bf_bits(o[dt][4 * a] * inv) | ((uint32_t)bf_bits(o[dt][4 * a + 1] * inv) << 16);
        wv.y = bf_bits(o[dt][4 * a + 2] * inv) | ((uint32_t)bf_bits(o[dt][4 * a + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + 32 * dt + 8 * a) = wv;
      }
  }
}

// ------------------------------------------------------------------ backward
// D[(s nh + h) lq + i] = dO_i . O_i over the head's dims (the bf16 O the forward wrote): LPH lanes per (row, head)
// (8 at d = 64, 16 at d = 96 / 128), lane c loading the head's 16-B chunk c, so a wave's loads are whole head rows
// of consecutive heads.  32-bit index arithmetic (rows x heads < 2^31, checked by the caller): the 64-bit
// divisions of the first form cost more than the loads (config 5: 145 us per launch for 252 MB).
template <int LPH>
__global__ __launch_bounds__(256) void flash_long_prep_kernel(const uint16_t* __restrict__ dctx, long long ldc,
                                                              const uint16_t* __restrict__ o, long long ldo,
                                                              float* __restrict__ dvec, int nseq, int lq, int nh,
                                                              int hd) {
  const unsigned total = (unsigned)nseq * (unsigned)lq * (unsigned)nh;
  const unsigned idx = (blockIdx.x * 256u + threadIdx.x) / LPH;   // (row, head)
  const int c = threadIdx.x & (LPH - 1);
  const bool live = idx < total;
  const unsigned id = live ? idx : 0u;
  const unsigned row = id / (unsigned)nh, h = id - row * (unsigned)nh;   // sequence row s lq + i
  float acc = 0.f;
  if (live && c < hd / 8) {
    const uint4 a = *reinterpret_cast<const uint4*>(dctx + (long long)row * ldc + (long long)h * hd + 8 * c);
    const uint4 b = *reinterpret_cast<const uint4*>(o + (long long)row * ldo + (long long)h * hd + 8 * c);
    const uint32_t wa[4] = {a.x, a.y, a.z, a.w}, wb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int t = 0; t < 4; ++t)
      acc += __uint_as_float(wa[t] << 16) * __uint_as_float(wb[t] << 16) +
             __uint_as_float(wa[t] & 0xffff0000u) * __uint_as_float(wb[t] & 0xffff0000u);
  }
#pragma unroll
  for (int m = LPH / 2; m > 0; m >>= 1) acc += __shfl_xor(acc, m, 64);
  if (live && c == 0) {
    const unsigned s = row / (unsigned)lq, i = row - s * (unsigned)lq;
    dvec[((long long)s * nh + h) * lq + i] = acc;
  }
}

// waves per backward workgroup (key tiles of 32): 12 at d = 64 (3 waves per SIMD, 131 KB of LDS), 7 at
// d = 96 / 128 (2 waves per SIMD; the K and V images of 7 tiles take 112 KB of the 160)
template <int HD> constexpr int bwd_max_waves() { return HD == 64 ? 12 : 7; }
constexpr int BQC = 32;   // queries per backward chunk
constexpr int BMIN_W = 4;  // at least 4 waves: they stage the query chunks and share the dQ tiles

template <int HD>
__global__ __launch_bounds__(bwd_max_waves<HD>() * 64, 1) void flash_long_bwd_kernel(
    const uint16_t* __restrict__ dctx, long long ldc, const uint16_t* __restrict__ q, long long ldq,
    const uint16_t* __restrict__ k, long long ldk, const uint16_t* __restrict__ v, long long ldv,
    const float* __restrict__ kmask, const float* __restrict__ lse, const float* __restrict__ dvec,
    uint16_t* __restrict__ dq, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, long long lddq, long long lddk,
    long long lddv, float* __restrict__ dq_ws, int lq, int lk, int nh, int tpg, float scale, float p_drop,
    uint64_t seed, uint64_t off) {
  using G = Geo<HD>;
  constexpr int NCL = G::NCL, NC = G::NC, HW = G::HW, DT = G::DT, KS = G::KS;
  constexpr int UQ = (BQC * NCL + BMIN_W * 64 - 1) / (BMIN_W * 64);   // 16-B chunks per thread per operand
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int nw = blockDim.x >> 6, nth = blockDim.x;
  const int GK = 32 * nw;
  uint16_t* Kimg = smem;                     // [GK][HW] the group's K rows
  uint16_t* Vimg = Kimg + GK * HW;           // [GK][HW] the group's V rows
  uint16_t* Qc = Vimg + GK * HW;             // [BQC][HW]
  uint16_t* dOc = Qc + BQC * HW;             // [BQC][HW]
  uint16_t* dSt = dOc + BQC * HW;            // [GK][BQC] dS^T of the chunk (64-B rows)
  float* Lc = reinterpret_cast<float*>(dSt + GK * BQC);   // [BQC] LSE * log2 e (+inf on padding rows)
  float* Dc = Lc + BQC;                                      // [BQC]
  const int s = blockIdx.x / nh, h = blockIdx.x % nh, grp = blockIdx.y, ngrp = gridDim.y;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long lrow0 = ((long long)s * nh + h) * lq;
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const float sl2 = scale * LOG2E;
  const int NKT = (lk + 31) >> 5;
  const int kt0 = grp * tpg, nkt = min(tpg, NKT - kt0);   // this group's key tiles
  const int kg0 = 32 * kt0;                                // first key of the group
  const int NQC = (lq + BQC - 1) / BQC;

  // this wave's 32 keys (lane -> key j); their K and V rows are read as B-operand fragments from the group's
  // K / V images (registers would push the d = 128 kernel past 256 VGPRs and the d = 64 one past the 168 of
  // three waves per SIMD)
  const bool kw = w < nkt;   // wave-uniform
  const int jl = 32 * w + cl, j = kg0 + jl;
  const bool jv = kw && j < lk;
  const float mj2 = jv ? (kmask ? kmask[krow0 + j] * LOG2E : 0.f) : -INFINITY;
  // the group's K and V images (rows past lk or past the group zero)
  for (int e = threadIdx.x; e < GK * NCL; e += nth) {
    const int r = e / NCL, cc = e % NCL, jj = kg0 + r;
    const bool ok = r < 32 * nkt && jj < lk;
    const long long ko = krow0 + min(jj, lk - 1);
    const uint4 x = *reinterpret_cast<const uint4*>(k + ko * ldk + hoff + 8 * cc);
    const uint4 y = *reinterpret_cast<const uint4*>(v + ko * ldv + hoff + 8 * cc);
    *reinterpret_cast<uint4*>(Kimg + ioff<NC>(r, cc)) = keep_if(ok, x);
    *reinterpret_cast<uint4*>(Vimg + ioff<NC>(r, cc)) = keep_if(ok, y);
  }
  // query chunk c -> registers (Q, dO rows; LSE, D) -> LDS
  uint4 rq[UQ], rd[UQ];
  float lv = 0.f, dv0 = 0.f;
  auto load = [&](int c) {
    const int q0 = c * BQC;
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = threadIdx.x + u * nth, r = e / NCL, cc = e % NCL, ii = q0 + r;
      const bool ok = e < BQC * NCL && ii < lq;
      const long long qo = qrow0 + min(ii, lq - 1);
      rq[u] = keep_if(ok, *reinterpret_cast<const uint4*>(q + qo * ldq + hoff + 8 * cc));
      rd[u] = keep_if(ok, *reinterpret_cast<const uint4*>(dctx + qo * ldc + hoff + 8 * cc));
    }
    const int t = threadIdx.x, ii = q0 + t;
    if (t < BQC) {
      const long long lr = lrow0 + min(ii, lq - 1);
      lv = ii < lq ? lse[lr] * LOG2E : INFINITY;   // padding query rows: P = exp2(-inf) = 0
      dv0 = ii < lq ? dvec[lr] : 0.f;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int u = 0; u < UQ; ++u) {
      const int e = threadIdx.x + u * nth, r = e / NCL, cc = e % NCL;
      if (e < BQC * NCL) {
        *reinterpret_cast<uint4*>(Qc + ioff<NC>(r, cc)) = rq[u];
        *reinterpret_cast<uint4*>(dOc + ioff<NC>(r, cc)) = rd[u];
      }
    }
    if (threadIdx.x < BQC) {
      Lc[threadIdx.x] = lv;
      Dc[threadIdx.x] = dv0;
    }
  };
  load(0);
  store();
  __syncthreads();

  floatx16 dV[DT], dK[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dV[dt] = zero16();
    dK[dt] = zero16();
  }
  constexpr int NT16 = 2 * (HD / 16);   // 16 x 16 dQ tiles of a 32-query chunk
  for (int c = 0; c < NQC; ++c) {
    const int q0 = c * BQC;
    if (c + 1 < NQC) load(c + 1);
    // ---- key phase
    if (kw) {
      // this lane's dropout keep bits for the chunk (register r = 4 a + b <-> query q0 + 8 a + 4 kl + b), drawn
      // before the products so the hash temporaries are not live beside the S / dP accumulators; query rows past lq
      // and keys past lk draw unused values (p = 0 there)
      const uint32_t keep = dr.thr != 0u ? k3m_attn_keep_km16(dr, off, lrow0 + q0, 4 * kl, lk, j) : 0xffffu;
      floatx16 S = zero16(), dP = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Qc, 0, ks, lane), rowfrag<NC>(Kimg, 32 * w, ks, lane), S,
                                                    0, 0, 0);
        dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(dOc, 0, ks, lane), rowfrag<NC>(Vimg, 32 * w, ks, lane),
                                                     dP, 0, 0, 0);
      }
      // accumulator r: query q0 + 8 (r >> 2) + 4 kl + (r & 3), key j = this lane
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int i0 = 8 * a + 4 * kl;
        const float4 l4 = *reinterpret_cast<const float4*>(Lc + i0);
        const float4 d4 = *reinterpret_cast<const float4*>(Dc + i0);
        const float lvv[4] = {l4.x, l4.y, l4.z, l4.w}, dvv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int r = 4 * a + b;
          const float p = __builtin_amdgcn_exp2f(fmaf(S[r], sl2, mj2) - lvv[b]);
          const float dm = k3m_keep_f(keep, r, __float_as_uint(dr.scale));
          S[r] = p * dm;                         // P_drop
          dP[r] = p * (dP[r] * dm - dvv[b]);     // dS
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 bp = accfrag(S, s2), bs = accfrag(dP, s2);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dV[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(dOc, 16 * s2, 32 * dt, lane), bp, dV[dt], 0, 0, 0);
          dK[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(Qc, 16 * s2, 32 * dt, lane), bs, dK[dt], 0, 0, 0);
        }
      }
      // dS^T tile -> LDS: registers 4a .. 4a+3 are queries 8 a + 4 kl .. +3 of key row jl (8 bytes)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        uint2 wd;
        wd.x = bf_bits(dP[4 * a]) | ((uint32_t)bf_bits(dP[4 * a + 1]) << 16);
        wd.y = bf_bits(dP[4 * a + 2]) | ((uint32_t)bf_bits(dP[4 * a + 3]) << 16);
        *reinterpret_cast<uint2*>(dSt + ioff<4>(jl, a) + 4 * kl) = wd;
      }
    } else {
      // a wave without keys (the group's last tiles, or fewer than 4 tiles): zero dS^T rows it owns
#pragma unroll
      for (int a = 0; a < 4; ++a) *reinterpret_cast<uint2*>(dSt + ioff<4>(jl, a) + 4 * kl) = make_uint2(0u, 0u);
    }
    __syncthreads();
    // ---- dQ phase: dQ[q0 .. q0+31][:] = dS K over the group's keys, 16 x 16 tiles dealt to the waves
    for (int t = w; t < NT16; t += nw) {
      const int qt = t & 1, d16 = t >> 1;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      int kt = 0;
      for (; kt + 1 < nkt; kt += 2) {   // two k-steps' reads in flight per MFMA pair
        const bf16x8 a0 = trfrag16<4>(dSt, 32 * kt, 16 * qt, lane), b0 = trfrag16<NC>(Kimg, 32 * kt, 16 * d16, lane);
        const bf16x8 a1 = trfrag16<4>(dSt, 32 * kt + 32, 16 * qt, lane);
        const bf16x8 b1 = trfrag16<NC>(Kimg, 32 * kt + 32, 16 * d16, lane);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
      }
      if (kt < nkt)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(trfrag16<4>(dSt, 32 * kt, 16 * qt, lane),
                                                      trfrag16<NC>(Kimg, 32 * kt, 16 * d16, lane), acc, 0, 0, 0);
      // acc[r]: query q0 + 16 qt + 4 (lane >> 4) + r, head dim 16 d16 + (lane & 15)
      const int dd = 16 * d16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = q0 + 16 * qt + 4 * (lane >> 4) + r;
        if (ii < lq) {
          if (ngrp == 1) dq[(qrow0 + ii) * lddq + hoff + dd] = bf_bits(acc[r] * scale);
          else dq_ws[(((long long)grp * gridDim.x + blockIdx.x) * lq + ii) * HD + dd] = acc[r];
        }
      }
    }
    __syncthreads();   // every read of the chunk's images is done
    if (c + 1 < NQC) {
      store();
      __syncthreads();
    }
  }
  // dV^T / dK^T: lane -> key j, register r -> head dim 32 dt + 8 (r >> 2) + 4 kl + (r & 3): 8-B stores
  if (jv) {
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

// ------------------------------------------------------------------ backward, LDS-DMA form (K3M_FLASH_LONG_BWD=2)
// The same workgroup decomposition and arithmetic as flash_long_bwd_kernel, with every operand staged by LDS-DMA
// (global_load_lds: no staging registers, no ds_write; the images' chunk swizzle goes into the per-lane source
// address, the XOR being an involution):
//  * K and V images of the group: one DMA burst in the prologue (the register form waited for one HBM round trip
//    per 640-thread pass);
//  * query chunks (Q rows, dO rows, raw LSE and D) in a ring of NQB slots, the DMA of chunk c + NQB issued as soon
//    as chunk c's key phase has read its slot: NQB - 1 chunks in flight instead of one register-prefetched chunk;
//  * rows past lq / lk are clamped copies of valid rows instead of zeros: their P (LSE = +inf, key mask -inf) and
//    hence Pd and dS are exactly 0, so every sum is unchanged (bit-identical to the register form);
//  * dQ leaves by buffer stores (rows past lq dropped by the descriptor), so each wave's vector-memory count per
//    chunk is fixed and the DMA waits are counted (vmcnt), two barriers per chunk instead of three.
template <int NC>
__device__ __forceinline__ int swz_of(int r) {
  if constexpr (NC == 16) return ((r & 3) << 2) | ((r >> 2) & 3);
  else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);   // NC == 8
}

// One LDS-DMA wave instruction as inline asm (as gemm_x6p.hip PPDLoop): issued through the builtin, the compiler's
// waitcnt pass cannot tell the ring slots from the K / V / dS^T images and puts a vmcnt(0) before every later LDS
// access, i.e. drains the chunks meant to stay in flight.  Hidden from it, the DMAs are ordered only by the counted
// vmcnt waits below (its own vmcnt counts for other loads stay conservative).  M0 = the wave-uniform LDS destination;
// s_nop 0: the M0 write -> LDS-DMA hazard.
__device__ __forceinline__ uint32_t lds_addr(const void* lds) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
}
__device__ __forceinline__ void lds_dma16(const void* g, void* lds) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(lds_addr(lds)) : "memory");
}
__device__ __forceinline__ void lds_dma4(const void* g, void* lds) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "{m0}"(lds_addr(lds)) : "memory");
}

// vmcnt(n), n wave-uniform (a scalar switch over the immediate forms)
template <int N>
__device__ __forceinline__ void vmwait() {
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void vmwait_n(int n) {
  switch (n < 0 ? 0 : n) {
#define K3M_FL_W(N) case N: vmwait<N>(); break;
    K3M_FL_W(0) K3M_FL_W(1) K3M_FL_W(2) K3M_FL_W(3) K3M_FL_W(4) K3M_FL_W(5) K3M_FL_W(6) K3M_FL_W(7)
    K3M_FL_W(8) K3M_FL_W(9) K3M_FL_W(10) K3M_FL_W(11) K3M_FL_W(12) K3M_FL_W(13) K3M_FL_W(14) K3M_FL_W(15)
    K3M_FL_W(16) K3M_FL_W(17) K3M_FL_W(18) K3M_FL_W(19) K3M_FL_W(20) K3M_FL_W(21) K3M_FL_W(22) K3M_FL_W(23)
    K3M_FL_W(24) K3M_FL_W(25) K3M_FL_W(26) K3M_FL_W(27) K3M_FL_W(28) K3M_FL_W(29) K3M_FL_W(30) K3M_FL_W(31)
    K3M_FL_W(32) K3M_FL_W(33) K3M_FL_W(34) K3M_FL_W(35) K3M_FL_W(36) K3M_FL_W(37) K3M_FL_W(38) K3M_FL_W(39)
    K3M_FL_W(40) K3M_FL_W(41) K3M_FL_W(42) K3M_FL_W(43) K3M_FL_W(44) K3M_FL_W(45) K3M_FL_W(46) K3M_FL_W(47)
#undef K3M_FL_W
    default: vmwait<0>(); break;
  }
}

// one DMA instruction (1 KiB: 1024 / (2 HW) rows) of an [rows][HW] image at rows r0 .. : lane -> (row, slot), the
// chunk stored in that slot read from row min(row, nvalid - 1) of the global operand (chunks past the head: clamped,
// never read).  saddr + 32-bit voffset form: the wave-uniform 64-bit base (the operand's row 0 + head offset) stays
// in SGPRs and each lane keeps one offset register (64-bit per-lane pointers had the forward spill in its loop).
template <int NC, int NCL>
__device__ __forceinline__ void dma_rows(uint16_t* img, int r0, const uint16_t* __restrict__ g, long long ld,
                                         long long row0, int nvalid, int hoff, int lane) {
  const int rr = lane / NC, slot = lane % NC, r = r0 + rr;   // 64 / NC rows per instruction
  const int c = min(slot ^ swz_of<NC>(r), NCL - 1);
  const uint16_t* base = g + row0 * ld + hoff;
  const uint64_t b = (uint64_t)(uintptr_t)base;
  // (readfirstlane returns int: through uint32_t, or the low word's sign would spread into the high word)
  const uint64_t bu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t voff = (uint32_t)(((long long)min(r, nvalid - 1) * ld + 8 * c) * 2);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(bu), "{m0}"(lds_addr(img + r0 * NC * 8))
               : "memory");
}

__device__ float k3m_inf_word = INFINITY;   // LDS-DMA source of the padding rows' LSE

template <int HD, bool DQ2>
__global__ __launch_bounds__(bwd_max_waves<HD>() * 64, 1) void flash_long_bwd2_kernel(
    const uint16_t* __restrict__ dctx, long long ldc, const uint16_t* __restrict__ q, long long ldq,
    const uint16_t* __restrict__ k, long long ldk, const uint16_t* __restrict__ v, long long ldv,
    const float* __restrict__ kmask, const float* __restrict__ lse, const float* __restrict__ dvec,
    uint16_t* __restrict__ dq, uint16_t* __restrict__ dk, uint16_t* __restrict__ dv, long long lddq, long long lddk,
    long long lddv, float* __restrict__ dq_ws, int lq, int lk, int nh, int tpg, int nqb, float scale, float p_drop,
    uint64_t seed, uint64_t off) {
  using G = Geo<HD>;
  constexpr int NCL = G::NCL, NC = G::NC, HW = G::HW, DT = G::DT, KS = G::KS;
  constexpr int RPI = 64 / NC;                 // image rows per DMA instruction
  constexpr int NQI = BQC / RPI;               // DMA instructions per chunk operand (Q or dO)
  constexpr int NCI = 2 * NQI + 1;             // per chunk, + one dword instruction for (LSE, D)
  constexpr int SL = 2 * BQC * HW + 128;       // bf16 elements per ring slot (+ 64 floats)
  constexpr int NT16 = 2 * (HD / 16);          // 16 x 16 dQ tiles of a 32-query chunk
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int nw = blockDim.x >> 6;
  const int GK = 32 * nw;
  uint16_t* Kimg = smem;                       // [GK][HW]
  uint16_t* Vimg = Kimg + GK * HW;             // [GK][HW]
  uint16_t* dSt = Vimg + GK * HW;              // [GK][BQC]
  uint16_t* ring = dSt + (DQ2 ? 2 : 1) * GK * BQC;   // nqb x {Q [BQC][HW], dO [BQC][HW], LSE [32] f32, D [32] f32}
  const int s = blockIdx.x / nh, h = blockIdx.x % nh, grp = blockIdx.y, ngrp = gridDim.y;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const long long lrow0 = ((long long)s * nh + h) * lq;
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const float sl2 = scale * LOG2E;
  const int NKT = (lk + 31) >> 5;
  const int kt0 = grp * tpg, nkt = min(tpg, NKT - kt0);
  const int kg0 = 32 * kt0;
  const int NQC = (lq + BQC - 1) / BQC;
  const bool kw = w < nkt;
  const int jl = 32 * w + cl, j = kg0 + jl;
  const bool jv = kw && j < lk;
  const float mj2 = jv ? (kmask ? kmask[krow0 + j] * LOG2E : 0.f) : -INFINITY;
  // this wave's share of every chunk's DMA (instruction i by wave i % nw) and of the dQ tiles (tile t by t % nw)
  const int n_w = w < NCI ? (NCI - 1 - w) / nw + 1 : 0;
  const int t_w = w < NT16 ? (NT16 - 1 - w) / nw + 1 : 0;
  const int st_w = 4 * t_w;   // dQ buffer stores per chunk
  auto dma_chunk = [&](int c) {
    uint16_t* sl = ring + (c % nqb) * SL;
    const int q0 = c * BQC;
    // the lane index made opaque here: per-lane offsets hoisted out of the chunk loop spilled at d = 64, and the
    // reload's vmcnt(0) drained the DMA ring at every chunk
    int ln = lane;
    asm volatile("" : "+v"(ln));
    for (int i = w; i < NCI; i += nw) {
      if (i < NQI) dma_rows<NC, NCL>(sl, i * RPI, q, ldq, qrow0 + q0, lq - q0, hoff, ln);
      else if (i < 2 * NQI) dma_rows<NC, NCL>(sl + BQC * HW, (i - NQI) * RPI, dctx, ldc, qrow0 + q0, lq - q0, hoff, ln);
      else {   // raw LSE (lanes 0-31; +inf for rows past lq, so P = 0 there) and D (lanes 32-63) of the chunk's rows
        const int kh = ln >> 5, ch = ln & 31;
        const long long lr = lrow0 + min(q0 + ch, lq - 1);
        lds_dma4(kh ? dvec + lr : (q0 + ch < lq ? lse + lr : &k3m_inf_word), sl + 2 * BQC * HW);
      }
    }
  };
  // prologue: the group's K and V images (rows past lk or past the group: clamped copies), then the first chunks
  {
    const int kv_inst = GK / RPI;   // per image; a multiple of nw
    for (int i = w; i < kv_inst; i += nw) {
      dma_rows<NC, NCL>(Kimg, i * RPI, k, ldk, krow0 + kg0, lk - kg0, hoff, lane);
      dma_rows<NC, NCL>(Vimg, i * RPI, v, ldv, krow0 + kg0, lk - kg0, hoff, lane);
    }
  }
  const int npre = min(nqb, NQC);
  for (int c = 0; c < npre; ++c) dma_chunk(c);
  vmwait_n(n_w * (npre - 1));   // K, V and chunk 0 landed (raw barrier: __syncthreads would drain every DMA)
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  floatx16 dV[DT], dK[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    dV[dt] = zero16();
    dK[dt] = zero16();
  }
  const long long dqbytes = ngrp == 1 ? ((long long)(gridDim.x / nh) * lq - 1) * lddq * 2 + (long long)nh * HD * 2
                                      : (long long)ngrp * gridDim.x * lq * HD * 4;
  const __amdgpu_buffer_rsrc_t rdq = __builtin_amdgcn_make_buffer_rsrc(
      ngrp == 1 ? (void*)dq : (void*)dq_ws, (short)0, (int)min(dqbytes, 0x7ffffff0LL), 0x00020000);
  // key phase of chunk c (ring slot c % nqb): P and dS of this wave's 32 keys -> dV, dK; dS^T into the image dS
  auto key_phase = [&](int c, uint16_t* dS) __attribute__((always_inline)) {
    const int q0 = c * BQC;
    const uint16_t* Qc = ring + (c % nqb) * SL;
    const uint16_t* dOc = Qc + BQC * HW;
    const float* Lc = reinterpret_cast<const float*>(dOc + BQC * HW);
    const float* Dc = Lc + BQC;
    // ---- key phase (as flash_long_bwd_kernel; LSE scaled and padding rows set to +inf here)
    if (kw) {
      const uint32_t keep = dr.thr != 0u ? k3m_attn_keep_km16(dr, off, lrow0 + q0, 4 * kl, lk, j) : 0xffffu;
      floatx16 S = zero16(), dP = zero16();
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Qc, 0, ks, lane), rowfrag<NC>(Kimg, 32 * w, ks, lane), S,
                                                    0, 0, 0);
        dP = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(dOc, 0, ks, lane), rowfrag<NC>(Vimg, 32 * w, ks, lane),
                                                     dP, 0, 0, 0);
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int i0 = 8 * a + 4 * kl;
        const float4 l4 = *reinterpret_cast<const float4*>(Lc + i0);
        const float4 d4 = *reinterpret_cast<const float4*>(Dc + i0);
        const float lraw[4] = {l4.x, l4.y, l4.z, l4.w}, dvv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int r = 4 * a + b;
          float lvb;   // padding query rows: +inf (the DMA above), P = 0
          {
#pragma clang fp contract(off)
            lvb = lraw[b] * LOG2E;   // rounded on its own, as the register form's pre-scaled LDS copy
          }
          const float p = __builtin_amdgcn_exp2f(fmaf(S[r], sl2, mj2) - lvb);
          const float dm = k3m_keep_f(keep, r, __float_as_uint(dr.scale));
          S[r] = p * dm;
          dP[r] = p * (dP[r] * dm - dvv[b]);
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 bp = accfrag(S, s2), bs = accfrag(dP, s2);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dV[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(dOc, 16 * s2, 32 * dt, lane), bp, dV[dt], 0, 0, 0);
          dK[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(Qc, 16 * s2, 32 * dt, lane), bs, dK[dt], 0, 0, 0);
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        uint2 wd;
        wd.x = bf_bits(dP[4 * a]) | ((uint32_t)bf_bits(dP[4 * a + 1]) << 16);
        wd.y = bf_bits(dP[4 * a + 2]) | ((uint32_t)bf_bits(dP[4 * a + 3]) << 16);
        *reinterpret_cast<uint2*>(dS + ioff<4>(jl, a) + 4 * kl) = wd;
      }
    } else {
#pragma unroll
      for (int a = 0; a < 4; ++a) *reinterpret_cast<uint2*>(dS + ioff<4>(jl, a) + 4 * kl) = make_uint2(0u, 0u);
    }
  };
  // dQ of chunk cq from its dS^T image dS
  auto dq_phase = [&](const uint16_t* dS, int cq) __attribute__((always_inline)) {
    const int q0 = cq * BQC;
    // ---- dQ phase: 16 x 16 tiles dealt to the waves; 4 buffer stores per tile, rows past lq dropped
    for (int t = w; t < NT16; t += nw) {
      const int qt = t & 1, d16 = t >> 1;
      floatx4 acc = {0.f, 0.f, 0.f, 0.f};
      int kt = 0;
      for (; kt + 1 < nkt; kt += 2) {
        const bf16x8 a0 = trfrag16<4>(dS, 32 * kt, 16 * qt, lane), b0 = trfrag16<NC>(Kimg, 32 * kt, 16 * d16, lane);
        const bf16x8 a1 = trfrag16<4>(dS, 32 * kt + 32, 16 * qt, lane);
        const bf16x8 b1 = trfrag16<NC>(Kimg, 32 * kt + 32, 16 * d16, lane);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc, 0, 0, 0);
      }
      if (kt < nkt)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(trfrag16<4>(dS, 32 * kt, 16 * qt, lane),
                                                      trfrag16<NC>(Kimg, 32 * kt, 16 * d16, lane), acc, 0, 0, 0);
      const int dd = 16 * d16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = q0 + 16 * qt + 4 * (lane >> 4) + r;
        if (ngrp == 1) {
          const int o = ii < lq ? (int)(((qrow0 + ii) * lddq + hoff + dd) * 2) : 0x7fffffff;
          __builtin_amdgcn_raw_buffer_store_b16(bf_bits(acc[r] * scale), rdq, o, 0, 0);
        } else {
          const int o = ii < lq ? (int)(((((long long)grp * gridDim.x + blockIdx.x) * lq + ii) * HD + dd) * 4)
                                : 0x7fffffff;
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r]), rdq, o, 0, 0);
        }
      }
    }
  };
  if constexpr (!DQ2) {
    for (int c = 0; c < NQC; ++c) {
      key_phase(c, dSt);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // dS^T complete; every read of this chunk's slot done
      __builtin_amdgcn_sched_barrier(0);
      dq_phase(dSt, c);
      // ---- the next chunks: chunk c + nqb into this chunk's slot; chunk c + 1 must have landed before the barrier
      const bool more = c + nqb < NQC;
      if (more) dma_chunk(c + nqb);
      if (c + 1 < NQC) {
        // vector-memory operations this wave issued after chunk c + 1's DMA: chunks x in [c + 2 - nqb, c] each
        // stored st_w dQ values and issued n_w DMAs when x + nqb < NQC; a prologue DMA also has the later prologue
        // chunks after it
        int younger = 0;
        const int x0 = c + 2 - nqb;
        for (int x = x0 < 0 ? 0 : x0; x <= c; ++x) younger += st_w + (x + nqb < NQC ? n_w : 0);
        if (c + 1 < nqb) younger += n_w * (npre - 1 - (c + 1));
        vmwait_n(younger);
      }
      __builtin_amdgcn_s_barrier();   // chunk c + 1 visible; dS^T free
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    // DQ2: two dS^T images.  Iteration c: (after the barrier that retired chunk c - 1's slot) DMA chunk c - 1 + nqb
    // into it, the key phase of chunk c into image c & 1, the dQ phase of chunk c - 1 from image (c - 1) & 1, then
    // one barrier (chunk c + 1 landed, image c & 1 complete, image (c - 1) & 1 free).  A wave whose key phase ends
    // early goes on to its dQ tiles instead of waiting at a second barrier.
    for (int c = 0; c < NQC; ++c) {
      if (c >= 1 && c - 1 + nqb < NQC) dma_chunk(c - 1 + nqb);
      key_phase(c, dSt + (c & 1) * GK * BQC);
      if (c >= 1) dq_phase(dSt + ((c - 1) & 1) * GK * BQC, c - 1);
      if (c + 1 < NQC) {
        // vector-memory operations this wave issued after chunk c + 1's DMA (issued in iteration i0, or in the
        // prologue when i0 <= 0): iteration i0's dQ stores, then per iteration x its DMA (if any) and dQ stores
        int younger = 0;
        const int i0 = c + 2 - nqb;
        if (i0 >= 1) younger += st_w;
        else younger += n_w * (npre - 1 - (c + 1));
        for (int x = i0 + 1 < 1 ? 1 : i0 + 1; x <= c; ++x) younger += (x - 1 + nqb < NQC ? n_w : 0) + st_w;
        vmwait_n(younger);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    dq_phase(dSt + ((NQC - 1) & 1) * GK * BQC, NQC - 1);
  }
  if (jv) {
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

// ------------------------------------------------------------------ forward, LDS-DMA form (K3M_FLASH_LONG_FWD=2)
// flash_long_fwd_kernel with the K / V chunks staged by LDS-DMA into a ring of NKB slots (chunk c + NKB - 1 issued
// right after the barrier that retires chunk c - 1's slot, so NKB - 1 chunks are in flight instead of one
// register-prefetched chunk, and no staging registers: at d = 64 three workgroups fit a CU instead of two).  Keys
// past lk are clamped copies instead of zeros; their scores carry the -inf key mask either way, so P, the running
// max / sum and the context are bit-identical.
template <int HD> constexpr int fwd2_nkb() { return HD == 64 ? 3 : 2; }
template <int HD> constexpr int fwd2_occ() { return HD == 64 ? 3 : 2; }

// DROP: the p > 0 form (a template parameter rather than a wave-uniform branch around two element loops: the d = 64
// dropout form needs 150 VGPRs instead of the whole 168 of three waves per SIMD)
template <int HD, bool DROP>
__global__ __launch_bounds__(FNT, fwd2_occ<HD>()) void flash_long_fwd2_kernel(
    const uint16_t* __restrict__ q, long long ldq, const uint16_t* __restrict__ k, long long ldk,
    const uint16_t* __restrict__ v, long long ldv, const float* __restrict__ kmask, uint16_t* __restrict__ ctx,
    long long ldc, float* __restrict__ lse, int lq, int lk, int nh, float scale, float p_drop, uint64_t seed,
    uint64_t off, int xcdmap) {
  using G = Geo<HD>;
  constexpr int NCL = G::NCL, NC = G::NC, HW = G::HW, DT = G::DT, KS = G::KS;
  constexpr int NKB = fwd2_nkb<HD>();
  constexpr int RPI = 64 / NC;                 // image rows per DMA instruction
  constexpr int CI = FKC / RPI;                // DMA instructions per chunk and operand
  constexpr int NWF = FNT / 64;                // 4 waves
  constexpr int N_W = 2 * CI / NWF;            // DMA instructions per wave per chunk
  static_assert((2 * CI) % NWF == 0, "chunk DMA must split over the waves");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* ring = smem;                                            // NKB x {K [FKC][HW], V [FKC][HW]}
  float* msk = reinterpret_cast<float*>(ring + NKB * 2 * FKC * HW);   // [LKP] mask * log2 e, -inf past lk
  // workgroup -> (sequence x head, query block).  xcdmap (the head count a multiple of 8): the query blocks of one
  // head get consecutive ids on ONE XCD (ids n, n + 8, ...; workgroups are dealt to the 8 XCDs round-robin), so they
  // run together and read that head's K / V rows through the same L2 instead of once each from HBM
  int hx = blockIdx.x, qb = blockIdx.y;
  if (xcdmap) {
    const int n = blockIdx.x + gridDim.x * blockIdx.y, loc = n >> 3;
    hx = (loc / (int)gridDim.y) * 8 + (n & 7);
    qb = loc % (int)gridDim.y;
  }
  const int s = hx / nh, h = hx % nh;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, cl = lane & 31, kl = lane >> 5;
  const int nkc = (lk + FKC - 1) / FKC, LKP = nkc * FKC;
  const long long qrow0 = (long long)s * lq, krow0 = (long long)s * lk;
  const int hoff = h * HD;
  const int qw0 = qb * (FNT / 2) + 32 * w;
  const bool wact = qw0 < lq;
  const int i = qw0 + cl;
  const bool iv = i < lq;
  const K3mDrop dr = k3m_drop_init(seed, p_drop);
  const float sl2 = scale * LOG2E;
  const long long prow = ((long long)s * nh + h) * lq + min(i, lq - 1);
  auto dma_chunk = [&](int c) {   // K and V rows c FKC .. + FKC - 1 (clamped) into slot c % NKB
    uint16_t* Kb = ring + (c % NKB) * 2 * FKC * HW;
    int ln = lane;   // opaque: the per-lane offsets are recomputed here instead of hoisted (and spilled) by the loop
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int t = 0; t < N_W; ++t) {
      const int inst = w + NWF * t;   // 0 .. 2 CI - 1: K first, then V
      if (inst < CI) dma_rows<NC, NCL>(Kb, inst * RPI, k, ldk, krow0 + c * FKC, lk - c * FKC, hoff, ln);
      else dma_rows<NC, NCL>(Kb + FKC * HW, (inst - CI) * RPI, v, ldv, krow0 + c * FKC, lk - c * FKC, hoff, ln);
    }
  };
  const int npre = min(NKB - 1, nkc);
  for (int c = 0; c < npre; ++c) dma_chunk(c);
  bf16x8 qf[KS];
  {
    const uint16_t* qp = q + (qrow0 + min(i, lq - 1)) * ldq + hoff + 8 * kl;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = __builtin_bit_cast(bf16x8, keep_if(iv, *reinterpret_cast<const uint4*>(qp + 16 * ks)));
  }
  for (int t = threadIdx.x; t < LKP; t += FNT)
    msk[t] = t < lk ? (kmask ? kmask[krow0 + t] * LOG2E : 0.f) : -INFINITY;

  floatx16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = zero16();
  float m2 = -INFINITY, lp = 0.f;
  for (int c = 0; c < nkc; ++c) {
    // chunk c landed (chunks c + 1 .. c + NKB - 2 may stay in flight), then the barrier that also retires every
    // read of chunk c - 1's slot, which chunk c + NKB - 1 then refills
    vmwait_n(N_W * max(0, min(NKB - 2, nkc - 1 - c)));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (c + NKB - 1 < nkc) dma_chunk(c + NKB - 1);
    if (wact) {
      const uint16_t* Kb = ring + (c % NKB) * 2 * FKC * HW;
      const uint16_t* Vb = Kb + FKC * HW;
      floatx16 S[FKC / 32];
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt) {
        floatx16 a = zero16();
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(rowfrag<NC>(Kb, 32 * jt, ks, lane), qf[ks], a, 0, 0, 0);
        S[jt] = a;
      }
      float mc = -INFINITY;
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = c * FKC + 32 * jt + (r & 3) + 8 * (r >> 2) + 4 * kl;
          const float x = fmaf(S[jt][r], sl2, msk[j]);
          S[jt][r] = x;
          mc = fmaxf(mc, x);
        }
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m2, mc);
      const float mref = mn == -INFINITY ? 0.f : mn;
      const float alpha = __builtin_amdgcn_exp2f(m2 - mref);
      m2 = mn;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      // the p = 0 test hoisted out of the element loop.  Registers 4 q + b of tile jt are keys
      // c FKC + 32 jt + 8 q + 4 kl + b: pairs (b = 0, 1) and (2, 3) of one draw each, pair counters
      // pb + 16 jt + 4 q + b / 2 from this lane's first pair pb; the high word is mixed once per chunk, for pb's high
      // word and for the next one (a pair whose low word carried)
      if constexpr (DROP) {
        const uint64_t pb = off + (uint64_t)prow * (uint64_t)((lk + 1) >> 1) + (uint64_t)(c * (FKC / 2) + 2 * kl);
        uint32_t lo = (uint32_t)pb, pre0 = k3m_pair_pre(dr.key, pb), pre1 = k3m_pair_pre(dr.key, pb + (1ull << 32));
        // opaque: otherwise the compiler sinks the high-word multiply below the carry select, one more 32-bit
        // multiply per pair
        asm volatile("" : "+v"(lo), "+v"(pre0), "+v"(pre1));
#pragma unroll
        for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
          for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int hb = 0; hb < 2; ++hb) {
              const uint32_t x = lo + (uint32_t)(16 * jt + 4 * q + hb);
              const uint32_t hh = k3m_mix32(x ^ (x < lo ? pre1 : pre0));
#pragma unroll
              for (int b2 = 0; b2 < 2; ++b2) {
                const int r = 4 * q + 2 * hb + b2;
                const float p = __builtin_amdgcn_exp2f(S[jt][r] - mref);
                lp = jt == 0 && r == 0 ? fmaf(lp, alpha, p) : lp + p;
                S[jt][r] = p * (k3m_attn_half(hh, b2) >= dr.thr16 ? dr.scale : 0.f);
              }
            }
      } else {
#pragma unroll
        for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float p = __builtin_amdgcn_exp2f(S[jt][r] - mref);
            lp = jt == 0 && r == 0 ? fmaf(lp, alpha, p) : lp + p;
            S[jt][r] = p;
          }
      }
#pragma unroll
      for (int jt = 0; jt < FKC / 32; ++jt)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 b = accfrag(S[jt], s2);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
            o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(trfrag<NC, true>(Vb, 32 * jt + 16 * s2, 32 * dt, lane), b,
                                                             o[dt], 0, 0, 0);
        }
    }
  }
  if (!wact) return;
  const float lt = lp + __shfl_xor(lp, 32, 64);
  const float inv = 1.f / lt;
  if (kl == 0 && iv) lse[prow] = m2 * LN2 + __logf(lt);
  if (iv) {
    uint16_t* op = ctx + (qrow0 + i) * ldc + hoff + 4 * kl;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        uint2 wv;
        wv.x = bf_bits(o[dt][4 * a] * inv) | ((uint32_t)bf_bits(o[dt][4 * a + 1] * inv) << 16);
        wv.y = bf_bits(o[dt][4 * a + 2] * inv) | ((uint32_t)bf_bits(o[dt][4 * a + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + 32 * dt + 8 * a) = wv;
      }
  }
}

// dq = bf16(scale * sum_g ws[g]), summed in group order; one thread per 4 head dims of a query row
__global__ __launch_bounds__(256) void flash_long_dq_reduce_kernel(const float* __restrict__ ws, uint16_t* __restrict__ dq,
                                                                   long long lddq, int nseq, int lq, int nh, int hd,
                                                                   int ngrp, float scale) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const int q4 = hd / 4;
  const long long per = (long long)nseq * nh * lq * hd;   // floats of one group's partial
  if (idx >= per / 4) return;
  const int d4 = (int)(idx % q4);
  const long long prow = idx / q4;             // (s nh + h) lq + i
  const int i = (int)(prow % lq);
  const long long sh = prow / lq;
  const int h = (int)(sh % nh), s = (int)(sh / nh);
  float4 acc = *reinterpret_cast<const float4*>(ws + prow * hd + 4 * d4);
  for (int g = 1; g < ngrp; ++g) {
    const float4 x = *reinterpret_cast<const float4*>(ws + g * per + prow * hd + 4 * d4);
    acc.x += x.x;
    acc.y += x.y;
    acc.z += x.z;
    acc.w += x.w;
  }
  uint2 o;
  o.x = bf_bits(acc.x * scale) | ((uint32_t)bf_bits(acc.y * scale) << 16);
  o.y = bf_bits(acc.z * scale) | ((uint32_t)bf_bits(acc.w * scale) << 16);
  *reinterpret_cast<uint2*>(dq + ((long long)s * lq + i) * lddq + (long long)h * hd + 4 * d4) = o;
}

constexpr int LDS_MAX = 160 * 1024;

size_t fwd_lds(int lk, int hd) {
  const size_t HW = hd == 96 ? 128 : hd;
  const size_t LKP = (lk + FKC - 1) / FKC * FKC;
  return 2 * (4 * FKC * HW) + 4 * LKP;
}

size_t fwd2_lds(int lk, int hd) {
  const size_t HW = hd == 96 ? 128 : hd;
  const size_t LKP = (lk + FKC - 1) / FKC * FKC;
  const size_t nkb = hd == 64 ? 3 : 2;
  return nkb * 2 * FKC * HW * 2 + 4 * LKP;
}
// K3M_FLASH_LONG_FWD: 2 (default) the LDS-DMA forward (flash_long_fwd2_kernel), 1 the register-staged one
const int kFlashLongFwd = k3m_env_int("K3M_FLASH_LONG_FWD", 2);
// K3M_FLASH_LONG_XCD: 1 (default) the LDS-DMA forward deals the query blocks of a head to one XCD (flash_long_fwd2_kernel)
const int kFlashLongXcd = k3m_env_int("K3M_FLASH_LONG_XCD", 1);

// key tiles per group and groups of a head's backward
// K3M_FLASH_LONG_TPG (lab A/B): at most this many 32-key tiles per backward workgroup (0: as many as fit)
const int kFlashLongTpg = k3m_env_int("K3M_FLASH_LONG_TPG", 0);

void bwd_groups(int lk, int hd, int& tpg, int& ngrp, int& nw) {
  const int nkt = (lk + 31) / 32;
  int cap = hd == 64 ? bwd_max_waves<64>() : bwd_max_waves<128>();
  if (kFlashLongTpg > 0) cap = std::min(cap, kFlashLongTpg);
  ngrp = (nkt + cap - 1) / cap;
  tpg = (nkt + ngrp - 1) / ngrp;
  nw = std::max(tpg, BMIN_W);
}

// LDS bytes of flash_long_bwd2_kernel with nqb ring slots
size_t bwd2_lds(int hd, int nw, int nqb, bool dq2) {
  const size_t HW = hd == 96 ? 128 : hd, GK = 32 * (size_t)nw;
  return 2 * (2 * GK * HW + (dq2 ? 2 : 1) * GK * BQC) + (size_t)nqb * 2 * (2 * BQC * HW + 128);
}

// K3M_FLASH_LONG_DQ2: 1 (default) two dS^T images in the LDS-DMA backward where they fit (one barrier per query chunk,
// the dQ tiles of chunk c - 1 beside the key phase of chunk c), 0 one image (two barriers per chunk)
const int kFlashLongDq2 = k3m_env_int("K3M_FLASH_LONG_DQ2", 1);

// K3M_FLASH_LONG_BWD: 2 (default) the LDS-DMA backward (flash_long_bwd2_kernel), 1 the register-staged one
const int kFlashLongBwd = k3m_env_int("K3M_FLASH_LONG_BWD", 2);

size_t bwd_lds(int hd, int nw) {
  const size_t HW = hd == 96 ? 128 : hd, GK = 32 * (size_t)nw;
  return 2 * (2 * GK * HW + 2 * BQC * HW + GK * BQC) + 4 * 2 * BQC;
}

void set_attrs() {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)flash_long_fwd_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd_kernel<96>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd_kernel<96>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd_kernel<128>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<96, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<96, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<128, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_fwd2_kernel<128, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<96, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<96, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<128, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    (void)hipFuncSetAttribute((const void*)flash_long_bwd2_kernel<128, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
    done = true;
  }
}

bool vec_ok(const void* p, long long ld) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 8 == 0; }

}  // namespace

extern "C" int k3m_flash_attn_long_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                                       long long ldv, const float* kmask, void* ctx, long long ldc, float* lse, int nseq,
                                       int lq, int lk, int nh, int hd, float scale, float p_drop, uint64_t seed,
                                       uint64_t off, hipStream_t st) {
  K3M_ARG(q && k && v && ctx && lse);
  K3M_ARG(lq > 0 && lq <= LMAX && lk > 0 && lk <= LMAX && (hd == 64 || hd == 96 || hd == 128) && nh > 0 && nseq >= 0);
  K3M_ARG(vec_ok(q, ldq) && vec_ok(k, ldk) && vec_ok(v, ldv) && vec_ok(ctx, ldc));
  if (nseq == 0) return 0;
  const size_t lds = fwd_lds(lk, hd);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  set_attrs();
  const dim3 grid(nseq * nh, (lq + FNT / 2 - 1) / (FNT / 2));
  if (kFlashLongFwd == 2 && fwd2_lds(lk, hd) <= (size_t)LDS_MAX) {
    const size_t lds2 = fwd2_lds(lk, hd);
    const bool drop = p_drop > 0.f;   // k3m_drop_init: thr != 0 iff p > 0
    const int xcdmap = kFlashLongXcd && (nseq * nh) % 8 == 0 ? 1 : 0;
#define K3M_FL_FWD2(HD_, DR_)                                                                                     \
    hipLaunchKernelGGL((flash_long_fwd2_kernel<HD_, DR_>), grid, dim3(FNT), lds2, st, (const uint16_t*)q, ldq,   \
                       (const uint16_t*)k, ldk, (const uint16_t*)v, ldv, kmask, (uint16_t*)ctx, ldc, lse, lq, lk, nh, \
                       scale, p_drop, seed, off, xcdmap)
    if (hd == 64) { if (drop) K3M_FL_FWD2(64, true); else K3M_FL_FWD2(64, false); }
    else if (hd == 96) { if (drop) K3M_FL_FWD2(96, true); else K3M_FL_FWD2(96, false); }
    else { if (drop) K3M_FL_FWD2(128, true); else K3M_FL_FWD2(128, false); }
#undef K3M_FL_FWD2
    K3M_CHECK_LAUNCH();
    return 0;
  }
#define K3M_FL_FWD(HD_)                                                                                           \
  hipLaunchKernelGGL(flash_long_fwd_kernel<HD_>, grid, dim3(FNT), lds, st, (const uint16_t*)q, ldq,                \
                     (const uint16_t*)k, ldk, (const uint16_t*)v, ldv, kmask, (uint16_t*)ctx, ldc, lse, lq, lk, nh, \
                     scale, p_drop, seed, off)
  if (hd == 64) K3M_FL_FWD(64);
  else if (hd == 96) K3M_FL_FWD(96);
  else K3M_FL_FWD(128);
#undef K3M_FL_FWD
  K3M_CHECK_LAUNCH();
  return 0;
}

namespace {
long long long_ws_bytes(int nseq, int lq, int lk, int nh, int hd) {
  int tpg, ngrp, nw;
  bwd_groups(lk, hd, tpg, ngrp, nw);
  const long long rows = (long long)nseq * nh * lq;
  long long b = (rows + 63) / 64 * 64 * 4;             // D
  if (ngrp > 1) b += (long long)ngrp * rows * hd * 4;  // fp32 dQ partials
  return b;
}
}  // namespace

extern "C" int k3m_flash_attn_long_ws_bytes(int nseq, int lq, int lk, int nh, int hd, long long* bytes) {
  K3M_ARG(bytes && nseq >= 0 && lq > 0 && lq <= LMAX && lk > 0 && lk <= LMAX && nh > 0 &&
          (hd == 64 || hd == 96 || hd == 128));
  *bytes = long_ws_bytes(nseq, lq, lk, nh, hd);
  return 0;
}

extern "C" int k3m_flash_attn_long_bwd(const void* dctx, long long ldc, const void* o, long long ldo, const void* q,
                                       long long ldq, const void* k, long long ldk, const void* v, long long ldv,
                                       const float* kmask, const float* lse, void* dq, void* dk, void* dv,
                                       long long lddq, long long lddk, long long lddv, void* ws, long long ws_bytes,
                                       int nseq, int lq, int lk, int nh, int hd, float scale, float p_drop,
                                       uint64_t seed, uint64_t off, hipStream_t st) {
  K3M_ARG(dctx && o && q && k && v && lse && dq && dk && dv && ws);
  K3M_ARG(lq > 0 && lq <= LMAX && lk > 0 && lk <= LMAX && (hd == 64 || hd == 96 || hd == 128) && nh > 0 && nseq >= 0);
  K3M_ARG(vec_ok(q, ldq) && vec_ok(k, ldk) && vec_ok(v, ldv) && vec_ok(dctx, ldc) && vec_ok(o, ldo));
  K3M_ARG(vec_ok(dk, lddk) && vec_ok(dv, lddv) && (lddq % 4 == 0) && ((reinterpret_cast<uintptr_t>(dq) & 7) == 0));
  K3M_ARG((reinterpret_cast<uintptr_t>(ws) & 15) == 0);
  if (nseq == 0) return 0;
  K3M_ARG(ws_bytes >= long_ws_bytes(nseq, lq, lk, nh, hd));
  int tpg, ngrp, nw;
  bwd_groups(lk, hd, tpg, ngrp, nw);
  const size_t lds = bwd_lds(hd, nw);
  K3M_ARG(lds <= (size_t)LDS_MAX);
  set_attrs();
  const long long rows = (long long)nseq * nh * lq;
  float* dvec = static_cast<float*>(ws);
  float* dq_ws = dvec + (rows + 63) / 64 * 64;
  K3M_ARG(rows * 16 < (1LL << 31));
  if (hd == 64)
    hipLaunchKernelGGL(flash_long_prep_kernel<8>, dim3(k3m_cdiv(rows * 8, 256)), dim3(256), 0, st,
                       (const uint16_t*)dctx, ldc, (const uint16_t*)o, ldo, dvec, nseq, lq, nh, hd);
  else
    hipLaunchKernelGGL(flash_long_prep_kernel<16>, dim3(k3m_cdiv(rows * 16, 256)), dim3(256), 0, st,
                       (const uint16_t*)dctx, ldc, (const uint16_t*)o, ldo, dvec, nseq, lq, nh, hd);
  const dim3 grid(nseq * nh, ngrp);
  if (kFlashLongBwd == 2) {
    const bool dq2 = kFlashLongDq2 != 0 && bwd2_lds(hd, nw, 2, true) <= (size_t)LDS_MAX;
    const int nqb = bwd2_lds(hd, nw, 3, dq2) <= (size_t)LDS_MAX ? 3 : 2;
    const size_t lds2 = bwd2_lds(hd, nw, nqb, dq2);
    K3M_ARG(lds2 <= (size_t)LDS_MAX);
    // 32-bit byte offsets of the dQ buffer stores
    K3M_ARG(ngrp > 1 ? (long long)ngrp * rows * hd * 4 < 0x7ffffff0LL
                     : ((long long)nseq * lq) * lddq * 2 < 0x7ffffff0LL);
#define K3M_FL_BWD2(HD_, DQ_)                                                                                     \
    hipLaunchKernelGGL((flash_long_bwd2_kernel<HD_, DQ_>), grid, dim3(64 * nw), lds2, st, (const uint16_t*)dctx, ldc, \
                       (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v, ldv, kmask, lse, dvec, \
                       (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, dq_ws, lq, lk, nh, tpg, nqb,    \
                       scale, p_drop, seed, off)
    if (dq2) {
      if (hd == 64) K3M_FL_BWD2(64, true);
      else if (hd == 96) K3M_FL_BWD2(96, true);
      else K3M_FL_BWD2(128, true);
    } else {
      if (hd == 64) K3M_FL_BWD2(64, false);
      else if (hd == 96) K3M_FL_BWD2(96, false);
      else K3M_FL_BWD2(128, false);
    }
#undef K3M_FL_BWD2
  } else {
#define K3M_FL_BWD(HD_)                                                                                          \
  hipLaunchKernelGGL(flash_long_bwd_kernel<HD_>, grid, dim3(64 * nw), lds, st, (const uint16_t*)dctx, ldc,        \
                     (const uint16_t*)q, ldq, (const uint16_t*)k, ldk, (const uint16_t*)v, ldv, kmask, lse, dvec, \
                     (uint16_t*)dq, (uint16_t*)dk, (uint16_t*)dv, lddq, lddk, lddv, dq_ws, lq, lk, nh, tpg, scale,  \
                     p_drop, seed, off)
  if (hd == 64) K3M_FL_BWD(64);
  else if (hd == 96) K3M_FL_BWD(96);
  else K3M_FL_BWD(128);
#undef K3M_FL_BWD
  }
  K3M_CHECK_LAUNCH();
  if (ngrp > 1) {
    hipLaunchKernelGGL(flash_long_dq_reduce_kernel, dim3(k3m_cdiv(rows * hd / 4, 256)), dim3(256), 0, st, dq_ws,
                       (uint16_t*)dq, lddq, nseq, lq, nh, hd, ngrp, scale);
    K3M_CHECK_LAUNCH();
  }
  return 0;
}
