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

#ifndef K3M_X6_NS
#define K3M_X6_NS k3m_x6
#endif

namespace K3M_X6_NS {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

template <int BK>
__device__ __forceinline__ int slot_off(int r, int c) {
  // element offset of 8-bf16 chunk c of row r in a [TILE][BK] plane
  constexpr int CPR = BK / 8, SH = BK == 32 ? 2 : 3;
  return r * BK + ((c ^ ((r >> SH) & (CPR - 1))) << 3);
}

typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));

// two floats -> packed bf16 pair, round-to-nearest-even (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((float2v{a, b}), bf16x2v));
}

// MN-contiguous operand image: a [BK k][TILE mn] bf16 plane (rows of TILE/8 16-B chunks), chunk ch of
// row k at slot ch ^ swz(k).  The staging writes of 16 lanes are 128 contiguous bytes of one row
// (conflict-free), and the transposing fragment reads (ds_read_b64_tr_b16: per 16-lane group 4 rows
// x 16 columns) put the 4 rows x 4 chunks of a 32-lane half on 16 distinct bank quads.
template <int TILE>
__device__ __forceinline__ int mn_off(int k, int ch) {
  if constexpr (TILE >= 128) return k * TILE + ((ch ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 3);
  else return k * TILE + ((ch ^ (((k >> 1) & 1) << 2)) << 3);
}

typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short4v lds_short4v;

// MFMA operand fragment of an MN image: element e of lane l = X[16 ks + 8 (l>>5) + e][mn_base + (l&31)]
// (the same k order as the k-contiguous fragments), from two transposing reads.
template <int TILE>
__device__ __forceinline__ bf16x8 mn_frag(const __bf16* img, int mn_base, int ks, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, h = lane >> 5;
  const int ch = ((mn_base + 16 * (g & 1)) >> 3) + (p >> 1);
  const int r0 = 16 * ks + 8 * h + q;
  const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0, ch) + 4 * (p & 1)));
  const short4v x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0 + 4, ch) + 4 * (p & 1)));
  const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// exact three-way split of a float pair into packed bf16 planes h, m, l (a = h + m + l exactly):
// per pair 3 conversions, 2 x (unpack lo/hi + subtract) = ~4.5 VALU per element
__device__ __forceinline__ void split2(float a, float b, uint32_t& h, uint32_t& m, uint32_t& l) {
#ifdef K3M_X6_LAB_NO_SPLIT   // lab only (scripts/lab): the cost of the main loop without the split VALU
  h = pk_bf16(a, b);
  m = h;
  l = h;
  return;
#endif
  h = pk_bf16(a, b);
  const float r1a = a - __uint_as_float(h << 16), r1b = b - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(r1a, r1b);
  const float r2a = r1a - __uint_as_float(m << 16), r2b = r1b - __uint_as_float(m & 0xffff0000u);
  l = pk_bf16(r2a, r2b);
}

__device__ __forceinline__ void split4(const floatx4 v, u32x2v& h, u32x2v& m, u32x2v& l) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split2(v[0], v[1], h0, m0, l0);
  split2(v[2], v[3], h1, m1, l1);
  h = u32x2v{h0, h1};
  m = u32x2v{m0, m1};
  l = u32x2v{l0, l1};
}

template <bool KC, int TILE, int BK, int NT>
struct Stage {
  // TILE*BK/4 float4 per k-tile, spread over every thread of the block: KC = 4 consecutive k of one
  // row, MN = 4 consecutive mn of one k row.  (Round 4 and earlier staged MN operands as 4(k) x 4(mn)
  // blocks, which left half the threads of a 256-wide tile idle: those waves split nothing while their
  // SIMD partners split twice their share, and the extra 8 staging VGPRs per set made the input-gradient
  // walk spill inside its main loop.)
  static constexpr int NV = TILE * BK / 4;
  static constexpr int NB = (NV + NT - 1) / NT;
  static constexpr int NR = NB;
  floatx4 r[NR];
};

// Per-thread global source pointers of one operand tile, computed once per block and advanced by
// one k-tile per step.  Rows / column groups past the M or N edge are clamped to a valid address:
// what they load only reaches C rows / columns the epilogue never stores, so the steady-state loads
// carry no masks or branches.  Only a partial last k-tile (K % BK != 0) is masked (load_tail).
template <bool KC, int TILE, int BK, int NT>
struct Src {
  static constexpr int NB = Stage<KC, TILE, BK, NT>::NB;
  const float* p[NB];
  int kq[NB];    // k offset of the thread's first element inside the k-tile

  __device__ __forceinline__ void init(const float* __restrict__ base, long long ld, int mn0, int kbeg, int MN) {
    const int t = threadIdx.x;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int idx = t + NT * b;
      if constexpr (KC) {
        const int row = idx / (BK / 4), q = idx % (BK / 4);
        kq[b] = 4 * q;
        p[b] = base + (long long)min(mn0 + row, MN - 1) * ld + kbeg + 4 * q;
      } else {
        const int qm = idx % (TILE / 4), kr = idx / (TILE / 4);
        kq[b] = kr;
        p[b] = base + (long long)(kbeg + kr) * ld + max(0, min(mn0 + 4 * qm, MN - 4));
      }
    }
  }
  __device__ __forceinline__ void advance(long long ld);
};

template <bool KC, int TILE, int BK, int NT>
__device__ __forceinline__ void Src<KC, TILE, BK, NT>::advance(long long ld) {
#pragma unroll
  for (int b = 0; b < NB; ++b) p[b] += KC ? BK : BK * ld;
}

// Load the next full k-tile and advance the source pointers by one k-tile (16-B vectors; K % 4 == 0).
template <bool KC, int TILE, int BK, int NT>
__device__ __forceinline__ void load_full(Src<KC, TILE, BK, NT>& src, long long ld, Stage<KC, TILE, BK, NT>& s,
                                          bool adv = true) {
  constexpr int NB = Stage<KC, TILE, BK, NT>::NB, NV = Stage<KC, TILE, BK, NT>::NV;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (NV % NT != 0 && (int)threadIdx.x + NT * b >= NV) break;
    if constexpr (KC) {
      s.r[b] = *reinterpret_cast<const floatx4*>(src.p[b]);
      src.p[b] += adv ? BK : 0;
    } else {
      s.r[b] = *reinterpret_cast<const floatx4*>(src.p[b]);
      src.p[b] += adv ? BK * ld : 0;
    }
  }
}

// The partial last k-tile (pointers already advanced to it): krem (< BK, multiple of 4) k values
// remain; the rest load as zeros.
template <bool KC, int TILE, int BK, int NT>
__device__ __forceinline__ void load_tail(const Src<KC, TILE, BK, NT>& src, long long ld, int krem,
                                          Stage<KC, TILE, BK, NT>& s) {
  constexpr int NB = Stage<KC, TILE, BK, NT>::NB, NV = Stage<KC, TILE, BK, NT>::NV;
  const floatx4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (NV % NT != 0 && (int)threadIdx.x + NT * b >= NV) break;
    if constexpr (KC) {
      s.r[b] = src.kq[b] < krem ? *reinterpret_cast<const floatx4*>(src.p[b]) : z;
    } else {
      s.r[b] = src.kq[b] < krem ? *reinterpret_cast<const floatx4*>(src.p[b]) : z;
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
      u32x2v h, m, l;
      split4(s.r[it], h, m, l);
      *reinterpret_cast<u32x2v*>(lds + off) = h;
      *reinterpret_cast<u32x2v*>(lds + PL + off) = m;
      *reinterpret_cast<u32x2v*>(lds + 2 * PL + off) = l;
    }
  } else {
    constexpr int Q = TILE / 4;
#pragma unroll
    for (int b = 0; b < Stage<KC, TILE, BK, NT>::NB; ++b) {
      const int idx = t + NT * b;
      if (NV % NT != 0 && idx >= NV) break;
      const int qm = idx % Q, kr = idx / Q;   // k row kr, columns 4 qm .. 4 qm + 3
      const int off = mn_off<TILE>(kr, qm >> 1) + 4 * (qm & 1);
      u32x2v h, m, l;
      split4(s.r[b], h, m, l);
      *reinterpret_cast<u32x2v*>(lds + off) = h;
      *reinterpret_cast<u32x2v*>(lds + PL + off) = m;
      *reinterpret_cast<u32x2v*>(lds + 2 * PL + off) = l;
    }
  }
}

// VAR (tuning bits, lab-selectable): 1 = pin the next tile's global loads at the top of each step
// (sched_barrier), 2 = static s_setprio 1 for the second half of the waves (MI355X_MICROARCH.md,
// "Two waves per SIMD" item 4), 4 = pin the split+store after the MFMAs, 8 = s_setprio 1 for the
// first half instead.
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool VEC, bool PIPE = true, int VAR = 0>
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
  Src<AK, TBM, BK, NT> sa;
  Src<BK_, TBN, BK, NT> sb;
  sa.init(A, lda, m0, kbeg, M);
  sb.init(B, ldb, n0, kbeg, N);
  const int klen = kend - kbeg;
  const int nkf = klen > 0 ? klen / BK : 0;            // full k-tiles
  const int krem = klen > 0 ? klen - nkf * BK : 0;     // k values of a partial last tile
  const int h = lane >> 5, cl = lane & 31;
  auto compute = [&](int cur) {
    const __bf16* as = smem + cur * BUF;
    const __bf16* bs = as + 3 * PA;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[3][FM], b[3][FN];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[pl][i] = AK ? *reinterpret_cast<const bf16x8*>(as + pl * PA + slot_off<BK>(wm + 32 * i + cl, 2 * ks + h))
                        : mn_frag<TBM>(as + pl * PA, wm + 32 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[pl][j] = BK_ ? *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, 2 * ks + h))
                         : mn_frag<TBN>(bs + pl * PB, wn + 32 * j, ks, lane);
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
  };
  if constexpr ((VAR & 2) != 0) {
    if (w >= WM * WN / 2) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr ((VAR & 8) != 0) {
    if (w < WM * WN / 2) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (!PIPE) {
    // one register set: prefetch tile kt+1 while computing tile kt, write it after the MFMAs
    // (fewer VGPRs: lets two 8-wave blocks share a CU)
    if (nkf > 0) {
      load_full<AK, TBM, BK, NT>(sa, lda, ra, nkf > 1);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb, nkf > 1);
      store_tile<AK, TBM, BK, NT>(smem, ra);
      store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nkf; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nkf;
      if (more) {
        load_full<AK, TBM, BK, NT>(sa, lda, ra, kt + 2 < nkf);
        load_full<BK_, TBN, BK, NT>(sb, ldb, rb, kt + 2 < nkf);
      }
      compute(cur);
      if (more) {
        store_tile<AK, TBM, BK, NT>(smem + (cur ^ 1) * BUF, ra);
        store_tile<BK_, TBN, BK, NT>(smem + (cur ^ 1) * BUF + 3 * PA, rb);
      }
      __syncthreads();
    }
  } else {
    // Software pipeline, two register sets (unrolled by 2): during k-tile kt the LDS stage kt&1 is
    // consumed by the MFMAs while the registers of tile kt+1 (loaded one iteration earlier, so their
    // global latency is covered by a whole iteration) are split and written to the other stage in
    // the same basic block, where the scheduler interleaves that VALU work with the MFMAs; tile
    // kt+2 is loaded into the register set tile kt vacated.  Past the last full tile the loads
    // re-read that tile (pointers stop advancing) and the spare stores hit an unread stage, so the
    // steady state has no branches.
    Stage<AK, TBM, BK, NT> ra1;
    Stage<BK_, TBN, BK, NT> rb1;
    if (nkf > 0) {
      load_full<AK, TBM, BK, NT>(sa, lda, ra, nkf > 1);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb, nkf > 1);
      load_full<AK, TBM, BK, NT>(sa, lda, ra1, nkf > 2);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb1, nkf > 2);
      store_tile<AK, TBM, BK, NT>(smem, ra);
      store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
    }
    __syncthreads();
    for (int kt = 0; kt < nkf; kt += 2) {
      // even step: compute stage 0 | split ra1/rb1 (tile kt+1) -> stage 1 | load tile kt+2 -> ra/rb
      load_full<AK, TBM, BK, NT>(sa, lda, ra, kt + 3 < nkf);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb, kt + 3 < nkf);
      if constexpr ((VAR & 1) != 0) __builtin_amdgcn_sched_barrier(0);
      compute(0);
      if constexpr ((VAR & 4) != 0) __builtin_amdgcn_sched_barrier(0);
      store_tile<AK, TBM, BK, NT>(smem + BUF, ra1);
      store_tile<BK_, TBN, BK, NT>(smem + BUF + 3 * PA, rb1);
      __syncthreads();
      if (kt + 1 >= nkf) break;
      // odd step: compute stage 1 | split ra/rb (tile kt+2) -> stage 0 | load tile kt+3 -> ra1/rb1
      load_full<AK, TBM, BK, NT>(sa, lda, ra1, kt + 4 < nkf);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb1, kt + 4 < nkf);
      if constexpr ((VAR & 1) != 0) __builtin_amdgcn_sched_barrier(0);
      compute(1);
      if constexpr ((VAR & 4) != 0) __builtin_amdgcn_sched_barrier(0);
      store_tile<AK, TBM, BK, NT>(smem, ra);
      store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
      __syncthreads();
    }

  }
  if constexpr ((VAR & 10) != 0) __builtin_amdgcn_s_setprio(0);
  if (krem > 0) {  // peeled partial k-tile (masked loads); the pointers rest on the last full tile
    const int cur = nkf & 1;
    if (nkf > 0) {
      sa.advance(lda);
      sb.advance(ldb);
    }
    load_tail<AK, TBM, BK, NT>(sa, lda, krem, ra);
    load_tail<BK_, TBN, BK, NT>(sb, ldb, krem, rb);
    store_tile<AK, TBM, BK, NT>(smem + cur * BUF, ra);
    store_tile<BK_, TBN, BK, NT>(smem + cur * BUF + 3 * PA, rb);
    __syncthreads();
    compute(cur);
    __syncthreads();
  }
}

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool VEC, int EPI, int OCC, bool PIPE = true,
          int VAR = 0>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_x6_kernel(K3mGemm g) {
  constexpr int LDS_BF16 = 2 * 3 * (TBM + TBN) * BK;
  constexpr int EPI_F32 = WM * WN * 32 * (TBN / WN + 8);
  constexpr int WORDS = (LDS_BF16 / 2 > EPI_F32 ? LDS_BF16 / 2 : EPI_F32);
  __shared__ __attribute__((aligned(16))) float smem[WORDS];
  int m0, n0;
  // VAR bits 16 / 32 (lab): 4 / 2 row-tiles per N walk instead of 8
  K3M_F32_NS::tile_coords<(VAR & 16) ? 4 : (VAR & 32) ? 2 : 8>(g.m, g.n, TBM, TBN, m0, n0);
  int kbeg = 0, kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = blockIdx.y * per;
    kend = min(g.k, kbeg + per);
  }
  floatx16 acc[TBM / WM / 32][TBN / WN / 32];
  mainloop<TBM, TBN, WM, WN, BK, AK, BK_, VEC, PIPE, VAR>(static_cast<const float*>(g.a), g.lda, static_cast<const float*>(g.b),
                                               g.ldb, g.m, g.n, m0, n0, kbeg, kend, reinterpret_cast<__bf16*>(smem), acc);
  K3M_F32_NS::epilogue<TBM, TBN, WM, WN, EPI, WORDS>(g, m0, n0, smem, acc);
}

// Grouped launch: several independent problems that share the kernel template (layout,
// epilogue) in ONE grid — the co-attention blocks' GEMMs (three blocks x two streams, each only
// 2,304-8,192 rows) fill the 256 CUs together where each alone leaves CUs idle or falls back to a
// small tile.  blocks [start[p], start[p+1]) belong to problem p, split-major (slice, tile).
constexpr int GROUP_MAX = 8;
struct GemmGroup {
  K3mGemm g[GROUP_MAX];
  int start[GROUP_MAX + 1];
  int count;
};

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool VEC, int EPI, int OCC, bool PIPE = true>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_x6_grouped_kernel(GemmGroup grp) {
  constexpr int LDS_BF16 = 2 * 3 * (TBM + TBN) * BK;
  constexpr int EPI_F32 = WM * WN * 32 * (TBN / WN + 8);
  constexpr int WORDS = (LDS_BF16 / 2 > EPI_F32 ? LDS_BF16 / 2 : EPI_F32);
  __shared__ __attribute__((aligned(16))) float smem[WORDS];
  const int id = K3M_F32_NS::xcd_remap(blockIdx.x, grp.start[grp.count]);
  int p = 0;
  while (p + 1 < grp.count && id >= grp.start[p + 1]) ++p;
  const K3mGemm& g = grp.g[p];
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN, tiles = tm * tn;
  const int local = id - grp.start[p], slice = local / tiles, t = local - slice * tiles;
  constexpr int GROUP = 8;   // tile order inside a problem: GROUP row-tiles walk N together
  const int group_sz = GROUP * tn, first_m = (t / group_sz) * GROUP, gm_sz = min(tm - first_m, GROUP);
  const int m0 = (first_m + (t % group_sz) % gm_sz) * TBM, n0 = ((t % group_sz) / gm_sz) * TBN;
  int kbeg = 0, kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = slice * per;
    kend = min(g.k, kbeg + per);
  }
  floatx16 acc[TBM / WM / 32][TBN / WN / 32];
  mainloop<TBM, TBN, WM, WN, BK, AK, BK_, VEC, PIPE>(static_cast<const float*>(g.a), g.lda,
                                                     static_cast<const float*>(g.b), g.ldb, g.m, g.n, m0, n0, kbeg,
                                                     kend, reinterpret_cast<__bf16*>(smem), acc);
  K3M_F32_NS::epilogue<TBM, TBN, WM, WN, EPI, WORDS>(g, m0, n0, smem, acc, slice);
}

}  // namespace K3M_X6_NS
