// fp32 GEMM on the bf16 matrix cores: the "bf16x6" split (Henry, Tang & Heinecke, "Leveraging the
// bfloat16 Artificial Intelligence Datatype For Higher-Precision Computations", ARITH 2019).
//
// Why: gfx950's f32-input MFMA runs at 1/16 of the bf16 rate (157 vs 2,500 TF/s).  Every fp32
// operand x is split EXACTLY into three bf16 values x = h + m + l (h = rne(x), m = rne(x - h),
// l = x - h - m; each residual has <= 16 resp. <= 8 significant bits, so no information is lost),
// and a.b is accumulated in fp32 from the six partial products whose magnitude is >= 2^-16 of
// a.b:  hh + (hm + mh) + (hl + mm + lh).  Each bf16 x bf16 product is exact in the fp32 MFMA
// accumulator; the three dropped products (ml, lm, ll) are below 2^-24 |a.b| (the fp32 unit
// roundoff), so the result carries fp32 accuracy (tests/test_gpu_gemm_x6.py measures the error
// against an fp64 GEMM next to the exact-f32 MFMA kernel's).  Cost: 6 bf16 MFMAs per 32x32x16
// step (192 cycles) instead of 8 f32 MFMAs (512 cycles): a 2.67x higher fp32 roofline
// (2,500 / 6 = 416.7 TF/s).
//
// Structure: block tile TBM x TBN x BK (BK = 16 or 32 fp32), WM x WN waves of (TBM/WM) x (TBN/WN),
// v_mfma_f32_32x32x16_bf16.  Operands are split while being staged (register prefetch of the next
// k-tile, one barrier per k-tile, two LDS stages) into three bf16 planes per operand, each a
// k-contiguous [TILE][BK] image whose 16-B chunk c of row r sits at slot c ^ ((r >> SH) & (BK/8-1))
// (conflict-free ds_read_b128 fragments for the gfx950 16-lane read groups).  The fp32 C
// epilogue is k3m_f32::epilogue (same 32x32 accumulator layout).
#pragma once
#include "gemm_f32_tile.h"

namespace k3m_x6 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int BK>
__device__ __forceinline__ int slot_off(int r, int c) {
  // element offset of 8-bf16 chunk c of row r in a [TILE][BK] plane
  constexpr int CPR = BK / 8, SH = BK == 32 ? 2 : 3;
  return r * BK + ((c ^ ((r >> SH) & (CPR - 1))) << 3);
}

// exact three-way split of 4 floats into bf16 planes (round-to-nearest-even at each level)
__device__ __forceinline__ void split4(const floatx4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 hb = (__bf16)v[e];
    const float r1 = v[e] - (float)hb;
    const __bf16 mb = (__bf16)r1;
    const float r2 = r1 - (float)mb;
    h[e] = hb;
    m[e] = mb;
    l[e] = (__bf16)r2;
  }
}

template <bool KC, int TILE, int BK, int NT>
struct Stage {
  // KC: TILE*BK/4 float4; MN: (BK/4)*(TILE/4) blocks of 4(k) x 4(mn) = 4 float4 each
  static constexpr int NV = KC ? TILE * BK / 4 : BK * TILE / 16;
  static constexpr int NB = (NV + NT - 1) / NT;
  static constexpr int NR = KC ? NB : 4 * NB;
  floatx4 r[NR];
};

template <bool KC, bool VEC, int TILE, int BK, int NT>
__device__ __forceinline__ void load_tile(const float* __restrict__ p, long long ld, int mn0, int k0, int MN, int K,
                                          Stage<KC, TILE, BK, NT>& s) {
  const int t = threadIdx.x;
  constexpr int NV = Stage<KC, TILE, BK, NT>::NV;
  if constexpr (KC) {
    constexpr int QR = BK / 4;  // float4 per row
#pragma unroll
    for (int it = 0; it < Stage<KC, TILE, BK, NT>::NB; ++it) {
      const int idx = t + NT * it;
      if (NV % NT != 0 && idx >= NV) break;
      const int row = idx / QR, q = idx % QR;
      const int gm = mn0 + row, gk = k0 + 4 * q;
      if constexpr (VEC) {
        s.r[it] = (gm < MN && gk < K) ? *reinterpret_cast<const floatx4*>(p + (long long)gm * ld + gk)
                                      : floatx4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) s.r[it][e] = (gm < MN && gk + e < K) ? p[(long long)gm * ld + gk + e] : 0.f;
      }
    }
  } else {
    constexpr int Q = TILE / 4;
#pragma unroll
    for (int b = 0; b < Stage<KC, TILE, BK, NT>::NB; ++b) {
      const int idx = t + NT * b;
      if (NV % NT != 0 && idx >= NV) break;
      const int qm = idx % Q, g4 = idx / Q;
      const int gm = mn0 + 4 * qm;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int gk = k0 + 4 * g4 + kk;
        if constexpr (VEC) {
          s.r[4 * b + kk] = (gk < K && gm < MN) ? *reinterpret_cast<const floatx4*>(p + (long long)gk * ld + gm)
                                                : floatx4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            s.r[4 * b + kk][e] = (gk < K && gm + e < MN) ? p[(long long)gk * ld + gm + e] : 0.f;
        }
      }
    }
  }
}

// split + store: planes at lds, lds + TILE*BK, lds + 2*TILE*BK (bf16 elements)
template <bool KC, int TILE, int BK, int NT>
__device__ __forceinline__ void store_tile(__bf16* __restrict__ lds, const Stage<KC, TILE, BK, NT>& s) {
  const int t = threadIdx.x;
  constexpr int NV = Stage<KC, TILE, BK, NT>::NV, PL = TILE * BK;
  if constexpr (KC) {
    constexpr int QR = BK / 4;
#pragma unroll
    for (int it = 0; it < Stage<KC, TILE, BK, NT>::NB; ++it) {
      const int idx = t + NT * it;
      if (NV % NT != 0 && idx >= NV) break;
      const int row = idx / QR, q = idx % QR;
      const int off = slot_off<BK>(row, q >> 1) + 4 * (q & 1);
      bf16x4 h, m, l;
      split4(s.r[it], h, m, l);
      *reinterpret_cast<bf16x4*>(lds + off) = h;
      *reinterpret_cast<bf16x4*>(lds + PL + off) = m;
      *reinterpret_cast<bf16x4*>(lds + 2 * PL + off) = l;
    }
  } else {
    constexpr int Q = TILE / 4;
#pragma unroll
    for (int b = 0; b < Stage<KC, TILE, BK, NT>::NB; ++b) {
      const int idx = t + NT * b;
      if (NV % NT != 0 && idx >= NV) break;
      const int qm = idx % Q, g4 = idx / Q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const floatx4 v = {s.r[4 * b][e], s.r[4 * b + 1][e], s.r[4 * b + 2][e], s.r[4 * b + 3][e]};
        const int off = slot_off<BK>(4 * qm + e, g4 >> 1) + 4 * (g4 & 1);
        bf16x4 h, m, l;
        split4(v, h, m, l);
        *reinterpret_cast<bf16x4*>(lds + off) = h;
        *reinterpret_cast<bf16x4*>(lds + PL + off) = m;
        *reinterpret_cast<bf16x4*>(lds + 2 * PL + off) = l;
      }
    }
  }
}

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool VEC>
__device__ __forceinline__ void mainloop(const float* __restrict__ A, long long lda, const float* __restrict__ B,
                                         long long ldb, int M, int N, int m0, int n0, int kbeg, int kend,
                                         __bf16* smem, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int NT = 64 * WM * WN;
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int BUF = 3 * (TBM + TBN) * BK;  // bf16 elements per stage
  constexpr int PA = TBM * BK, PB = TBN * BK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stage<AK, TBM, BK, NT> ra;
  Stage<BK_, TBN, BK, NT> rb;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile<AK, VEC, TBM, BK, NT>(A, lda, m0, kbeg, M, kend, ra);
    load_tile<BK_, VEC, TBN, BK, NT>(B, ldb, n0, kbeg, N, kend, rb);
    store_tile<AK, TBM, BK, NT>(smem, ra);
    store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
  }
  __syncthreads();
  const int h = lane >> 5, cl = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<AK, VEC, TBM, BK, NT>(A, lda, m0, k0, M, kend, ra);
      load_tile<BK_, VEC, TBN, BK, NT>(B, ldb, n0, k0, N, kend, rb);
    }
    const __bf16* as = smem + cur * BUF;
    const __bf16* bs = as + 3 * PA;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[3][FM], b[3][FN];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[pl][i] = *reinterpret_cast<const bf16x8*>(as + pl * PA + slot_off<BK>(wm + 32 * i + cl, 2 * ks + h));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[pl][j] = *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, 2 * ks + h));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          // smallest terms first: (hl + mm + lh), (hm + mh), hh
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        }
    }
    if (more) {
      store_tile<AK, TBM, BK, NT>(smem + (cur ^ 1) * BUF, ra);
      store_tile<BK_, TBN, BK, NT>(smem + (cur ^ 1) * BUF + 3 * PA, rb);
    }
    __syncthreads();
  }
}

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool VEC, int EPI, int OCC>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_x6_kernel(K3mGemm g) {
  constexpr int LDS_BF16 = 2 * 3 * (TBM + TBN) * BK;
  constexpr int EPI_F32 = WM * WN * 32 * (TBN / WN + 8);
  constexpr int WORDS = (LDS_BF16 / 2 > EPI_F32 ? LDS_BF16 / 2 : EPI_F32);
  __shared__ __attribute__((aligned(16))) float smem[WORDS];
  int m0, n0;
  k3m_f32::tile_coords(g.m, g.n, TBM, TBN, m0, n0);
  int kbeg = 0, kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = blockIdx.y * per;
    kend = min(g.k, kbeg + per);
  }
  floatx16 acc[TBM / WM / 32][TBN / WN / 32];
  mainloop<TBM, TBN, WM, WN, BK, AK, BK_, VEC>(static_cast<const float*>(g.a), g.lda, static_cast<const float*>(g.b),
                                               g.ldb, g.m, g.n, m0, n0, kbeg, kend, reinterpret_cast<__bf16*>(smem), acc);
  k3m_f32::epilogue<TBM, TBN, WM, WN, EPI, WORDS>(g, m0, n0, smem, acc);
}

}  // namespace k3m_x6
