// Large-tile bf16 GEMM for gfx950 (the bf16 encoder of the mixed-precision step, configs 3-5):
// bf16 operands, fp32 accumulation, fp32 or bf16 C with the fused epilogues of k3m_gemm.
//
// Structure (MI355X_MICROARCH.md / cdna_hip_programming.md §5):
//  * block tile TBM x TBN x 64 (256x256 or 256x128), 8 waves of 512 threads, one block per CU,
//    each wave a (TBM/WM) x (TBN/WN) slab of v_mfma_f32_16x16x32_bf16 tiles (the 16x16x32 shape
//    holds a higher clock than 32x32x16 on random data at equal cycles per FLOP);
//  * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction):
//    no staging registers, no VALU, no ds_write; two LDS stages, the next k-tile's DMA in flight
//    while the current one feeds the MFMAs, one vmcnt(0) + barrier per k-tile;
//  * LDS images are lane-linear per DMA instruction, so the bank-conflict swizzles live in the
//    per-lane SOURCE address and the fragment read applies the same XOR (an involution):
//      K-contiguous operand: [TILE][64] bf16, chunk c of row r at slot c ^ ((r >> 1) & 7)
//        (fragments by ds_read_b128, conflict-free for the 16-lane read groups);
//      MN-contiguous operand (W in input gradients, dY^T and X in weight gradients): [64][TILE],
//        chunk ch of k-row k at slot ch ^ (((k & 3) << 2) | ((k >> 2) & 3)), fragments by the
//        transposing ds_read_b64_tr_b16 (no register transpose);
//  * edge rows / columns: source addresses clamped into the operand (their products reach only C
//    entries the epilogue does not store); K must be a multiple of 64 (callers fall back otherwise);
//  * XCD-aware bijective block remap, 8 row-tiles walking N together;
//  * epilogue through LDS: row-contiguous 16-B stores, bias / bias+GELU (+pre-activation) / dGELU /
//    bias+sigmoid / alpha, beta; split-K writes raw fp32 slabs reduced by the caller.
#pragma once
#include "common.h"
#include "gemm_f32_tile.h"

#include <type_traits>

namespace k3m_b16 {

constexpr int BK = 64;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;

__device__ __forceinline__ int kc_off(int r, int c) { return r * BK + ((c ^ ((r >> 1) & 7)) << 3); }
template <int TILE>
__device__ __forceinline__ int mn_off(int k, int ch) {
  return k * TILE + ((ch ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 3);
}

__device__ __forceinline__ void glds16(const uint16_t* g, uint16_t* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// LDS-DMA sources of one operand tile (TILE rows/columns x 64 k): a wave-uniform (SGPR) running base
// that advances by one k-tile per issue, plus per-lane 32-bit element offsets (the instruction's
// saddr + voffset form: no 64-bit per-lane pointers to keep or advance).  Callers guarantee the
// offsets fit (k3m_gemm_bf16_impl checks the operand extents).
template <bool KC, int TILE, int NT>
struct Loader {
  static constexpr int INSTS = TILE * BK * 2 / 1024;   // wave instructions per k-tile
  static constexpr int NW = NT / 64;
  static constexpr int NI = INSTS / NW;                 // per wave
  static_assert(INSTS % NW == 0, "tile must split evenly over the waves");
  const uint16_t* base;   // wave-uniform
  long long step;         // elements per k-tile
  uint32_t off[NI];
  int lds0;               // wave-uniform element offset of the wave's first instruction in the image

  __device__ __forceinline__ void init(const uint16_t* __restrict__ a, long long ld, int mn0, int kbeg, int MN) {
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lds0 = w * 512;
    base = a + (KC ? (long long)kbeg : (long long)kbeg * ld);
    step = KC ? BK : BK * ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int inst = w + NW * i;
      if constexpr (KC) {
        const int row = inst * 8 + (l >> 3), slot = l & 7;
        const int ch = slot ^ ((row >> 1) & 7);
        off[i] = (uint32_t)((long long)min(mn0 + row, MN - 1) * ld + ch * 8);
      } else {
        constexpr int CPR = TILE / 8, RPI = 64 / CPR;   // 16-B chunks per k-row, k-rows per instruction
        const int kr = inst * RPI + l / CPR, slot = l % CPR;
        const int ch = slot ^ (((kr & 3) << 2) | ((kr >> 2) & 3));
        off[i] = (uint32_t)((long long)kr * ld + max(0, min(mn0 + ch * 8, MN - 8)));
      }
    }
  }
  __device__ __forceinline__ void issue(uint16_t* img) {
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(base + off[i], img + lds0 + i * NW * 512);
    base += step;
  }
};

// 16x16x32 operand fragment: lane l gets X[mnb + (l & 15)][32 s + 8 (l >> 4) + e], e = 0..7
template <bool KC, int TILE>
__device__ __forceinline__ bf16x8 frag(const uint16_t* img, int mnb, int s, int lane) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8*>(img + kc_off(mnb + (lane & 15), 4 * s + (lane >> 4)));
  } else {
    // two transposed 4(k) x 16(mn) block reads per 16-lane group g = lane >> 4: k-rows 32s + 8g + q
    // (+4); lane 4q+p addresses row q, columns 4p..4p+3 (ds_read_b64_tr_b16)
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int ch = (mnb >> 3) + (p >> 1);
    const int r0 = 32 * s + 8 * (lane >> 4) + q;
    const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0, ch) + 4 * (p & 1)));
    const short4v x1 =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0 + 4, ch) + 4 * (p & 1)));
    const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <int TBM, int TBN, int WM, int WN>
struct Shape {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int FM = TBM / WM / 16, FN = TBN / WN / 16;
  static constexpr int STAGE = (TBM + TBN) * BK;          // bf16 elements per stage
  static constexpr int LDS = 2 * STAGE;                   // bf16 elements
};

// Accumulators of one wave's (WTM x WTN) output slab for the two MFMA shapes, and how a 32-row group
// of them is staged into the epilogue's LDS image ([32][WS] fp32, row-major).
template <int MF, int WTM, int WTN> struct Acc;
template <int WTM, int WTN> struct Acc<16, WTM, WTN> {   // v_mfma_f32_16x16x32_bf16
  static constexpr int FM = WTM / 16, FN = WTN / 16;
  // staging row stride = columns + PAD floats: the 4 row groups of one 16-lane write (rows 4g + r) land on
  // 4 distinct 16-bank quarters (4 * PAD = 16 mod 64), and the 8-float row reads of the store pass (8 lanes per
  // row) interleave two rows on the 64 banks — both conflict-free (PAD 8 put rows 4 apart on the same banks)
  static constexpr int PAD = 4;
  floatx4 v[FM][FN];
  __device__ __forceinline__ void stage(int grp, float* wl, int ws, int lane) const {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) wl[(16 * ii + 4 * (lane >> 4) + r) * ws + 16 * j + (lane & 15)] = v[2 * grp + ii][j][r];
  }
};
template <int WTM, int WTN> struct Acc<32, WTM, WTN> {   // v_mfma_f32_32x32x16_bf16
  static constexpr int FM = WTM / 32, FN = WTN / 32;
  static constexpr int PAD = 8;   // the two 32-lane halves of a write (rows 4 apart) on opposite bank halves
  floatx16 v[FM][FN];
  __device__ __forceinline__ void stage(int grp, float* wl, int ws, int lane) const {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) wl[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * ws + 32 * j + (lane & 31)] = v[grp][j][r];
  }
};

// 32x32x16 operand fragment: lane l gets X[mnb + (l & 31)][16 s + 8 (l >> 5) + e], e = 0..7 (s = 0..3)
template <bool KC, int TILE>
__device__ __forceinline__ bf16x8 frag32(const uint16_t* img, int mnb, int s, int lane) {
  if constexpr (KC) {
    return *reinterpret_cast<const bf16x8*>(img + kc_off(mnb + (lane & 31), 2 * s + (lane >> 5)));
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, h = lane >> 5;
    const int ch = ((mnb + 16 * (g & 1)) >> 3) + (p >> 1);
    const int r0 = 16 * s + 8 * h + q;
    const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0, ch) + 4 * (p & 1)));
    const short4v x1 =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + mn_off<TILE>(r0 + 4, ch) + 4 * (p & 1)));
    const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

template <bool AK, bool BK_, int TBM, int TBN, int FM, int FN>
__device__ __forceinline__ void read_frags(const uint16_t* stage, int wm, int wn, int s, int lane, bf16x8 (&a)[FM],
                                           bf16x8 (&b)[FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i) a[i] = frag<AK, TBM>(stage, wm + 16 * i, s, lane);
#pragma unroll
  for (int j = 0; j < FN; ++j) b[j] = frag<BK_, TBN>(stage + TBM * BK, wn + 16 * j, s, lane);
}

template <int FM, int FN>
__device__ __forceinline__ void mfmas(floatx4 (&acc)[FM][FN], const bf16x8 (&a)[FM], const bf16x8 (&b)[FN]) {
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

// acc[i][j] += A[m0 + wm + 16 i .., kbeg:kend] . B[n0 + wn + 16 j .., kbeg:kend]^T;  (kend - kbeg) % 64 == 0
//
// Software pipeline (two LDS stages, two register fragment sets F0 / F1 = k-substeps 0 / 1 of a
// 64-deep k-tile), per k-tile kt:
//   read F1(kt) | MFMA F0(kt)                      (the reads of F1 fly under 32 MFMAs)
//   wait lgkmcnt(0) vmcnt(0); barrier              (tile kt+1 landed; every read of stage kt done)
//   DMA tile kt+2 -> stage kt & 1 | read F0(kt+1) | MFMA F1(kt)
// so each tile's DMA has a whole tile of MFMAs (64 per wave) to land, the fragment reads of one
// substep always overlap the MFMAs of the other, and no LDS read is in flight across a barrier
// (the DMA that follows a barrier overwrites the stage just read).  sched_barrier pins the order.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void mainloop(const uint16_t* __restrict__ A, long long lda, const uint16_t* __restrict__ B,
                                         long long ldb, int M, int N, int m0, int n0, int kbeg, int kend,
                                         uint16_t* smem, Acc<16, TBM / WM, TBN / WN>& accs, bool pre = false) {
  using S = Shape<TBM, TBN, WM, WN>;
  constexpr int FM = S::FM, FN = S::FN;
  auto& acc = accs.v;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  Loader<AK, TBM, S::NT> la;
  Loader<BK_, TBN, S::NT> lb;
  la.init(A, lda, m0, kbeg, M);
  lb.init(B, ldb, n0, kbeg, N);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  if (pre) {   // k-tile 0 already in flight to stage 0 (issued by the previous tile's epilogue)
    la.base += la.step;
    lb.base += lb.step;
  } else {
    la.issue(smem);
    lb.issue(smem + TBM * BK);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nk > 1) {
    la.issue(smem + S::STAGE);
    lb.issue(smem + S::STAGE + TBM * BK);
  }
  bf16x8 a0[FM], b0[FN], a1[FM], b1[FN];
  read_frags<AK, BK_, TBM, TBN, FM, FN>(smem, wm, wn, 0, lane, a0, b0);
  for (int kt = 0; kt < nk; ++kt) {
    uint16_t* cur = smem + (kt & 1) * S::STAGE;
    uint16_t* nxt = smem + ((kt + 1) & 1) * S::STAGE;
    read_frags<AK, BK_, TBM, TBN, FM, FN>(cur, wm, wn, 1, lane, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfmas<FM, FN>(acc, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) {
      la.issue(cur);
      lb.issue(cur + TBM * BK);
    }
    // unconditional (past the last tile it reads a stale stage nobody uses): a branch here would
    // make the wait before MFMA F0 a conservative lgkmcnt(0) instead of a counted one
    read_frags<AK, BK_, TBM, TBN, FM, FN>(nxt, wm, wn, 0, lane, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mfmas<FM, FN>(acc, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();   // the epilogue reuses the stages
}

// The same pipeline with v_mfma_f32_32x32x16_bf16 and four 16-deep k-substeps per tile (fragment sets
// Fa / Fb alternate): for the weight gradients, whose two MN-contiguous operands take two transposing
// reads per fragment — 12 reads per substep keep every substep's reads inside the 15 outstanding LDS
// operations a wave can count (the 24 of a 16x16x32 substep serialised the reads and the MFMAs).
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void mainloop32(const uint16_t* __restrict__ A, long long lda,
                                           const uint16_t* __restrict__ B, long long ldb, int M, int N, int m0,
                                           int n0, int kbeg, int kend, uint16_t* smem,
                                           Acc<32, TBM / WM, TBN / WN>& accs, bool pre = false) {
  using S = Shape<TBM, TBN, WM, WN>;
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  auto& acc = accs.v;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  Loader<AK, TBM, S::NT> la;
  Loader<BK_, TBN, S::NT> lb;
  la.init(A, lda, m0, kbeg, M);
  lb.init(B, ldb, n0, kbeg, N);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  if (pre) {   // k-tile 0 already in flight to stage 0 (issued by the previous tile's epilogue)
    la.base += la.step;
    lb.base += lb.step;
  } else {
    la.issue(smem);
    lb.issue(smem + TBM * BK);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nk > 1) {
    la.issue(smem + S::STAGE);
    lb.issue(smem + S::STAGE + TBM * BK);
  }
  bf16x8 fa[FM], fb[FN], ga[FM], gb[FN];
  auto rd = [&](const uint16_t* st, int sub, bf16x8(&a)[FM], bf16x8(&b)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i) a[i] = frag32<AK, TBM>(st, wm + 32 * i, sub, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[j] = frag32<BK_, TBN>(st + TBM * BK, wn + 32 * j, sub, lane);
  };
  auto mm = [&](const bf16x8(&a)[FM], const bf16x8(&b)[FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  };
  rd(smem, 0, fa, fb);
  for (int kt = 0; kt < nk; ++kt) {
    uint16_t* cur = smem + (kt & 1) * S::STAGE;
    uint16_t* nxt = smem + ((kt + 1) & 1) * S::STAGE;
    rd(cur, 1, ga, gb);
    __builtin_amdgcn_sched_barrier(0);
    mm(fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    rd(cur, 2, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    mm(ga, gb);
    __builtin_amdgcn_sched_barrier(0);
    rd(cur, 3, ga, gb);
    __builtin_amdgcn_sched_barrier(0);
    mm(fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) {
      la.issue(cur);
      lb.issue(cur + TBM * BK);
    }
    rd(nxt, 0, fa, fb);   // unconditional, as in mainloop
    __builtin_amdgcn_sched_barrier(0);
    mm(ga, gb);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------------
// Ping-pong main loop (K3M_B16_PP): the two waves of each SIMD (w and w + 4) run one phase apart, one
// issuing MFMAs while the other reads its fragments (same rationale and phase table as PPLoop in
// gemm_x6p.hip).  Per k-tile t (64 deep, stage t & 1), waves 0-3 run M(t) in phase 2t and C(t) in 2t+1,
// waves 4-7 one phase later.  M(t): all fragments of k-tile t into registers.  C(t): the k-tile's MFMAs.
// LDS-DMA: both groups issue their half of k-tile t+2 into stage t & 1 in phase 2t+2 (waves 0-3 at the
// head of M(t+1), waves 4-7 at the head of C(t)), after the last read of k-tile t (phase 2t+1), and
// both wait for it (vmcnt(0)) at the end of phase 2t+3, before its first read in phase 2t+4.
template <bool KC, int TILE>
struct HalfLoader {   // the DMA instructions of one half of an operand tile, spread over 4 waves
  static constexpr int INSTS = TILE * BK * 2 / 1024;
  static constexpr int NI = INSTS / 8;   // per wave
  static_assert(INSTS % 8 == 0, "half tile must split evenly over 4 waves");
  const uint16_t* base;
  long long step;
  uint32_t off[NI];
  int lds0;

  __device__ __forceinline__ void init(const uint16_t* __restrict__ a, long long ld, int mn0, int kbeg, int MN) {
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int first = (w >> 2) * (INSTS / 2) + (w & 3);   // instruction i of this wave: first + 4 i
    lds0 = first * 512;
    base = a + (KC ? (long long)kbeg : (long long)kbeg * ld);
    step = KC ? BK : BK * ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int inst = first + 4 * i;
      if constexpr (KC) {
        const int row = inst * 8 + (l >> 3), slot = l & 7;
        const int ch = slot ^ ((row >> 1) & 7);
        off[i] = (uint32_t)((long long)min(mn0 + row, MN - 1) * ld + ch * 8);
      } else {
        constexpr int CPR = TILE / 8, RPI = 64 / CPR;
        const int kr = inst * RPI + l / CPR, slot = l % CPR;
        const int ch = slot ^ (((kr & 3) << 2) | ((kr >> 2) & 3));
        off[i] = (uint32_t)((long long)kr * ld + max(0, min(mn0 + ch * 8, MN - 8)));
      }
    }
  }
  __device__ __forceinline__ void issue(uint16_t* img) {
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(base + off[i], img + lds0 + i * 4 * 512);
    base += step;
  }
};

__device__ __forceinline__ void pp_sync(bool vm) {
  __builtin_amdgcn_sched_barrier(0);
  if (vm) __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
  else __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// PH > 1 cuts each k-tile into PH M/C phase pairs of SUB / PH substeps (the 256 x 256 tile: 96 fragment
// registers of a whole k-tile beside 128 accumulators spill); the DMA rules hold per k-tile: waves 0-3 issue
// in the first M phase of k-tile kt and wait at the end of its last C phase, waves 4-7 issue in the last C
// phase of k-tile kt and wait at the end of the last M phase of k-tile kt + 1.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int MF>
__device__ __forceinline__ void mainloop_pp(const uint16_t* __restrict__ A, long long lda,
                                            const uint16_t* __restrict__ B, long long ldb, int M, int N, int m0,
                                            int n0, int kbeg, int kend, uint16_t* smem,
                                            Acc<MF, TBM / WM, TBN / WN>& accs) {
  static_assert(WM * WN == 8, "ping-pong pairs waves w and w + 4");
  using S = Shape<TBM, TBN, WM, WN>;
  constexpr int FM = TBM / WM / MF, FN = TBN / WN / MF;
  constexpr int SUB = MF == 16 ? BK / 32 : BK / 16;   // k-substeps per k-tile
  constexpr int PH = (TBM / WM) * (TBN / WN) >= 128 * 64 ? 2 : 1;
  constexpr int SP = SUB / PH;                         // substeps per phase
  auto& acc = accs.v;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      if constexpr (MF == 16) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      else
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    }
  HalfLoader<AK, TBM> la;
  HalfLoader<BK_, TBN> lb;
  la.init(A, lda, m0, kbeg, M);
  lb.init(B, ldb, n0, kbeg, N);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  const bool late = __builtin_amdgcn_readfirstlane(threadIdx.x >> 8) != 0;   // waves 4-7
  la.issue(smem);
  lb.issue(smem + TBM * BK);
  if (nk > 1) {
    la.issue(smem + S::STAGE);
    lb.issue(smem + S::STAGE + TBM * BK);
  }
  pp_sync(true);
  if (late) pp_sync(false);
  bf16x8 a[SP][FM], b[SP][FN];
  auto rd = [&](const uint16_t* st, int ph) {
#pragma unroll
    for (int q = 0; q < SP; ++q) {
      const int s = ph * SP + q;
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[q][i] = MF == 16 ? frag<AK, TBM>(st, wm + 16 * i, s, lane) : frag32<AK, TBM>(st, wm + 32 * i, s, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[q][j] = MF == 16 ? frag<BK_, TBN>(st + TBM * BK, wn + 16 * j, s, lane)
                           : frag32<BK_, TBN>(st + TBM * BK, wn + 32 * j, s, lane);
    }
  };
  auto mm = [&]() {
#pragma unroll
    for (int q = 0; q < SP; ++q)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (MF == 16) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[q][i], b[q][j], acc[i][j], 0, 0, 0);
          else acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q][i], b[q][j], acc[i][j], 0, 0, 0);
        }
  };
#pragma nounroll
  for (int kt = 0; kt < nk; ++kt) {
    uint16_t* cur = smem + (kt & 1) * S::STAGE;
    if (!late) {
#pragma unroll
      for (int ph = 0; ph < PH; ++ph) {
        if (ph == 0 && kt >= 1 && kt + 1 < nk) {   // k-tile kt+1 into the stage k-tile kt-1 left
          uint16_t* nxt = smem + ((kt + 1) & 1) * S::STAGE;
          la.issue(nxt);
          lb.issue(nxt + TBM * BK);
        }
        rd(cur, ph);
        pp_sync(false);
        mm();
        pp_sync(ph == PH - 1);
      }
    } else {
#pragma unroll
      for (int ph = 0; ph < PH; ++ph) {
        rd(cur, ph);
        pp_sync(ph == PH - 1);
        if (ph == PH - 1 && kt + 2 < nk) {         // k-tile kt+2 into the stage just read
          la.issue(cur);
          lb.issue(cur + TBM * BK);
        }
        mm();
        pp_sync(false);
      }
    }
  }
  if (!late) pp_sync(false);
}

__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p), b = *reinterpret_cast<const floatx4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __uint_as_float(a[q] << 16);
    v[2 * q + 1] = __uint_as_float(a[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
  *reinterpret_cast<floatx4*>(p) = floatx4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<floatx4*>(p + 4) = floatx4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  u32x4 a;
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = (uint32_t)from_f<bf16_t>(v[2 * q]).x | ((uint32_t)from_f<bf16_t>(v[2 * q + 1]).x << 16);
  *reinterpret_cast<u32x4*>(p) = a;
}
// non-temporal forms (lab: K3M_B16_LAB bit 2)
__device__ __forceinline__ void store8_nt(float* p, const float (&v)[8]) {
  __builtin_nontemporal_store(floatx4{v[0], v[1], v[2], v[3]}, reinterpret_cast<floatx4*>(p));
  __builtin_nontemporal_store(floatx4{v[4], v[5], v[6], v[7]}, reinterpret_cast<floatx4*>(p + 4));
}
__device__ __forceinline__ void store8_nt(bf16_t* p, const float (&v)[8]) {
  u32x4 a;
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = (uint32_t)from_f<bf16_t>(v[2 * q]).x | ((uint32_t)from_f<bf16_t>(v[2 * q + 1]).x << 16);
  __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(p));
}

// 8 consecutive C / aux elements as raw registers (prefetched before they are needed)
template <typename CT> struct Raw8;
template <> struct Raw8<bf16_t> {
  u32x4 r;
  __device__ __forceinline__ void load(const bf16_t* p) { r = *reinterpret_cast<const u32x4*>(p); }
  __device__ __forceinline__ void get(float (&v)[8]) const {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __uint_as_float(r[q] << 16);
      v[2 * q + 1] = __uint_as_float(r[q] & 0xffff0000u);
    }
  }
};
template <> struct Raw8<float> {
  floatx4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const floatx4*>(p);
    b = *reinterpret_cast<const floatx4*>(p + 4);
  }
  __device__ __forceinline__ void get(float (&v)[8]) const {
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
};

template <int EPI>
__device__ __forceinline__ void epi_math8(const float (&v)[8], const float (&bb)[8], const float (&ax)[8],
                                          const float (&old)[8], float alpha, float beta, bool rd_old,
                                          float (&o)[8], float (&pa)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (EPI == K3M_EPI_NONE) {
      o[e] = alpha * v[e];
    } else if constexpr (EPI == K3M_EPI_BIAS) {
      o[e] = alpha * (v[e] + bb[e]);
    } else if constexpr (EPI == K3M_EPI_BIAS_GELU) {
      pa[e] = v[e] + bb[e];
      o[e] = gelu_fast(to_f(from_f<bf16_t>(pa[e])));  // gelu of the stored pre-activation the backward sees
    } else if constexpr (EPI == K3M_EPI_DGELU) {
      o[e] = alpha * v[e] * dgelu_fast(ax[e]);
    } else {
      o[e] = sigmoid_f(v[e] + bb[e]);
    }
    if (rd_old) o[e] = fmaf(beta, old[e], o[e]);
  }
}

// Epilogue through LDS (the stages are free after the main loop): per pass each wave stages 32 rows
// x (TBN/WN) columns of its fp32 accumulators (row stride TBN/WN + 8 floats), then every lane
// handles 8 consecutive columns of one row: epilogue math, 16-B (bf16) / 32-B (fp32) stores.
// vmcnt counts loads and stores in issue order, so a load issued after a store cannot be waited for
// without draining that store.  Hence: the lane's 8 bias values (the same columns in every pass) are
// loaded once with vector loads and waited for before the first store, and interior tiles (inside C,
// 16-B aligned rows) run a branch-free pass sequence whose per-pass loads (dGELU pre-activation, old C
// for beta != 0) are issued RING passes ahead — the compiler can then count its waits instead of
// falling back to vmcnt(0) (which had drained every store of a pass before the next one).  Edge tiles
// keep the guarded per-element path.
// 16x16 accumulator layout: acc[i][j][r] = C[wm + 16 i + 4 (lane >> 4) + r][wn + 16 j + (lane & 15)].
struct NoHookB {
  __device__ __forceinline__ void operator()() const {}
};

// hook(): called once, after the first accumulator group is in LDS and before any global store of C (the
// persistent walk issues the next tile's first LDS-DMA there; the staging image then must not overlap stage 0).
template <int TBM, int TBN, int WM, int WN, int EPI, typename CT, typename AccT, class Hook = NoHookB>
__device__ __forceinline__ void epilogue(const K3mGemm& g, int m0, int n0, uint16_t* smem_u16, const AccT& acc,
                                         int slice, Hook hook = Hook(), bool nostore = false, bool ntstore = false) {
  using S = Shape<TBM, TBN, WM, WN>;
  constexpr int WNC = TBN / WN, WS = WNC + AccT::PAD, LPR = WNC / 8, RPP = 64 / LPR, NPS = 32 / RPP, NG = TBM / WM / 32;
  constexpr int RING = sizeof(CT) == 2 ? 2 : 1;   // passes the per-pass loads run ahead (register budget)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * WNC;
  float* wl = reinterpret_cast<float*>(smem_u16) + w * 32 * WS;
  const int M = g.m, N = g.n;
  const bool split = g.splitk > 1;
  CT* C = split ? reinterpret_cast<CT*>(g.ws + (long long)slice * M * N) : static_cast<CT*>(g.c);
  const long long ldc = split ? N : g.ldc;
  const float alpha = split ? 1.f : g.alpha, beta = split ? 0.f : g.beta;
  CT* aux = static_cast<CT*>(g.aux);
  const float* bias = g.bias;
  constexpr bool HAS_AUX = EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_DGELU;
  constexpr bool HAS_BIAS = EPI == K3M_EPI_BIAS || EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_BIAS_SIGMOID;
  constexpr bool CAN_OLD = EPI == K3M_EPI_NONE || EPI == K3M_EPI_BIAS || EPI == K3M_EPI_DGELU;
  const bool cvec = (ldc % 8 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                    (!HAS_AUX || ((g.ldaux % 8 == 0) && ((reinterpret_cast<uintptr_t>(aux) & 15) == 0)));
  const int lr = lane / LPR, lc = (lane % LPR) * 8;
  const int col = n0 + wn + lc;
  float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (HAS_BIAS) {
    if (((reinterpret_cast<uintptr_t>(bias) & 15) == 0) && col + 8 <= N) {
      load8(bias + col, bb);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = col + e < N ? bias[col + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(bb[e]));   // waited for here, before any store
  }
  const bool rd_old = CAN_OLD && beta != 0.f;
  auto row_of = [&](int grp, int ps) { return m0 + wm + 32 * grp + ps * RPP + lr; };
  // K3M_GEMM_COLSUM_SLABS (dGELU only, as in k3m_f32::epilogue_r): column sums of the STORED values of C
  constexpr bool CSUM = EPI == K3M_EPI_DGELU;
  float* const cws = (CSUM && !split) ? g.ws : nullptr;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (cvec && m0 + TBM <= M && n0 + TBN <= N) {
    auto body = [&](auto old_tag) {
      constexpr bool OLD = decltype(old_tag)::value;
      constexpr bool LOADS = OLD || EPI == K3M_EPI_DGELU;
      constexpr int NQ = NG * NPS;
      Raw8<CT> rax[EPI == K3M_EPI_DGELU ? RING : 1], rold[OLD ? RING : 1];
      auto issue = [&](int q, int slot) {
        if constexpr (LOADS) {
          const long long r = row_of(q / NPS, q % NPS);
          if constexpr (EPI == K3M_EPI_DGELU) rax[slot].load(aux + r * g.ldaux + col);
          if constexpr (OLD) rold[slot].load(C + r * ldc + col);
        }
      };
#pragma unroll
      for (int q = 0; q < RING; ++q)
        if (q < NQ) issue(q, q);
#pragma unroll
      for (int grp = 0; grp < NG; ++grp) {
        acc.stage(grp, wl, WS, lane);
        __syncthreads();
        if (grp == 0) hook();
#pragma unroll
        for (int ps = 0; ps < NPS; ++ps) {
          const int q = grp * NPS + ps, slot = q % RING;
          const int rr = ps * RPP + lr;
          const long long row = row_of(grp, ps);
          const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
          const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
          const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          float ax[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, old[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
          if constexpr (EPI == K3M_EPI_DGELU) rax[slot].get(ax);
          if constexpr (OLD) rold[slot].get(old);
          if (q + RING < NQ) issue(q + RING, slot);
          float o[8], pa[8];
          epi_math8<EPI>(v, bb, ax, old, alpha, beta, OLD, o, pa);
          if (nostore) {   // lab timing (K3M_B16_LAB bit 0): the math stays live, nothing is written
#pragma unroll
            for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(o[e]), "v"(pa[e]));
          } else if (ntstore) {
            store8_nt(C + row * ldc + col, o);
            if constexpr (EPI == K3M_EPI_BIAS_GELU) store8_nt(aux + row * g.ldaux + col, pa);
          } else {
            store8(C + row * ldc + col, o);
            if constexpr (EPI == K3M_EPI_BIAS_GELU) store8(aux + row * g.ldaux + col, pa);
          }
          if constexpr (CSUM) {
            if (cws)
#pragma unroll
              for (int e = 0; e < 8; ++e) cs[e] += to_f(from_f<CT>(o[e]));
          }
        }
        if constexpr (CSUM) {
          if (cws) K3M_F32_NS::colsum_flush<LPR>(cs, cws, (m0 + wm + 32 * grp) >> 5, N, col, lane, true);
        }
        __syncthreads();
      }
    };
    if (rd_old) body(std::integral_constant<bool, true>());
    else body(std::integral_constant<bool, false>());
    return;
  }
  // edge tiles: guarded per-element accesses (rolled pass loop: small code, few registers)
#pragma unroll
  for (int grp = 0; grp < NG; ++grp) {
    acc.stage(grp, wl, WS, lane);
    __syncthreads();
    if (grp == 0) hook();
#pragma unroll 1
    for (int ps = 0; ps < NPS; ++ps) {
      const int rr = ps * RPP + lr;
      const int row = row_of(grp, ps);
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
      if (row >= M || col >= N) continue;
      const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const bool full = cvec && col + 8 <= N;
      CT* cp = C + (long long)row * ldc + col;
      CT* ap = HAS_AUX ? aux + (long long)row * g.ldaux + col : nullptr;
      float old[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ax[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == K3M_EPI_DGELU) {
        if (full) load8(ap, ax);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) ax[e] = col + e < N ? to_f(ap[e]) : 0.f;
      }
      if (rd_old) {
        if (full) load8(cp, old);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = col + e < N ? to_f(cp[e]) : 0.f;
      }
      float o[8], pa[8];
      epi_math8<EPI>(v, bb, ax, old, alpha, beta, rd_old, o, pa);
      if constexpr (CSUM) {
        if (cws)
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += col + e < N ? to_f(from_f<CT>(o[e])) : 0.f;
      }
      if (full) {
        store8(cp, o);
        if constexpr (EPI == K3M_EPI_BIAS_GELU) store8(ap, pa);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < N) {
            cp[e] = from_f<CT>(o[e]);
            if constexpr (EPI == K3M_EPI_BIAS_GELU) ap[e] = from_f<CT>(pa[e]);
          }
      }
    }
    if constexpr (CSUM) {
      if (cws) K3M_F32_NS::colsum_flush<LPR>(cs, cws, (m0 + wm + 32 * grp) >> 5, N, col, lane, m0 + wm + 32 * grp < M);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ int xcd_remap(int id, int nblk) {
  const int xcd = id & 7, q = nblk >> 3, rr = nblk & 7;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + (id >> 3);
}

// tile (m0, n0) and split slice of block `id` of one problem (8 row-tiles walk N together)
__device__ __forceinline__ void coords(int local, int M, int N, int TBM, int TBN, int& m0, int& n0, int& slice) {
  const int tm = (M + TBM - 1) / TBM, tn = (N + TBN - 1) / TBN, tiles = tm * tn;
  slice = local / tiles;
  const int t = local - slice * tiles;
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tn, first_m = (t / group_sz) * GROUP, gm_sz = min(tm - first_m, GROUP);
  m0 = (first_m + (t % group_sz) % gm_sz) * TBM;
  n0 = ((t % group_sz) / gm_sz) * TBN;
}

__device__ __forceinline__ void k_range(const K3mGemm& g, int slice, int& kbeg, int& kend) {
  kbeg = 0;
  kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = slice * per;
    kend = min(g.k, kbeg + per);
  }
}

constexpr int GROUP_MAX = 8;
struct GemmGroup {
  K3mGemm g[GROUP_MAX];
  int start[GROUP_MAX + 1];
  int count;
  int lab;       // lab knob K3M_B16_LAB (timing experiments only): bit 0 = no C / aux stores, bit 1 = staggered start
  int stagger;   // bit 1: workgroup b waits (b & 3) * stagger ticks of the 100 MHz clock before its first tile
};

// one output tile on MF x MF x (512 / MF) MFMAs (MF = 16 or 32)
template <int TBM, int TBN, int WM, int WN>
struct EpiLds {   // bf16 elements of the epilogue's fp32 staging image (8 waves x 32 rows x (TBN/WN + 8))
  static constexpr int E = Shape<TBM, TBN, WM, WN>::NT / 64 * 32 * (TBN / WN + 8) * 2;
};

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
__device__ __forceinline__ void run_tile(const K3mGemm& g, int m0, int n0, int kbeg, int kend, int slice,
                                         uint16_t* smem) {
  static_assert(EpiLds<TBM, TBN, WM, WN>::E <= Shape<TBM, TBN, WM, WN>::LDS, "epilogue staging exceeds the LDS stages");
  Acc<MF, TBM / WM, TBN / WN> acc;
  if constexpr (MF == 32)
    mainloop32<TBM, TBN, WM, WN, AK, BK_>(static_cast<const uint16_t*>(g.a), g.lda, static_cast<const uint16_t*>(g.b),
                                          g.ldb, g.m, g.n, m0, n0, kbeg, kend, smem, acc);
  else
    mainloop<TBM, TBN, WM, WN, AK, BK_>(static_cast<const uint16_t*>(g.a), g.lda, static_cast<const uint16_t*>(g.b),
                                        g.ldb, g.m, g.n, m0, n0, kbeg, kend, smem, acc);
  epilogue<TBM, TBN, WM, WN, EPI, CT>(g, m0, n0, smem, acc, slice);
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_kernel(K3mGemm g) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[Shape<TBM, TBN, WM, WN>::LDS];
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  const int nsl = g.splitk > 1 ? g.splitk : 1;
  const int id = xcd_remap(blockIdx.x, tm * tn * nsl);
  int m0, n0, slice, kbeg, kend;
  coords(id, g.m, g.n, TBM, TBN, m0, n0, slice);
  k_range(g, slice, kbeg, kend);
  run_tile<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF>(g, m0, n0, kbeg, kend, slice, smem);
}

// several independent problems sharing the template in one grid: blocks [start[p], start[p+1]) are
// problem p (split-major: slice, tile)
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_grouped_kernel(GemmGroup grp) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[Shape<TBM, TBN, WM, WN>::LDS];
  const int id = xcd_remap(blockIdx.x, grp.start[grp.count]);
  int p = 0;
  while (p + 1 < grp.count && id >= grp.start[p + 1]) ++p;
  const K3mGemm& g = grp.g[p];
  int m0, n0, slice, kbeg, kend;
  coords(id - grp.start[p], g.m, g.n, TBM, TBN, m0, n0, slice);
  k_range(g, slice, kbeg, kend);
  run_tile<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF>(g, m0, n0, kbeg, kend, slice, smem);
}

// Persistent walk (K3M_B16_PERSIST): min(units, CUs) workgroups, each running units u, u + gridDim.x, ...
// of the group (problem, split slice, tile), the units of one "wave" (u / gridDim.x) remapped XCD-aware as in
// the one-unit-per-workgroup grid.  Same tiles, same arithmetic: bit-identical C.  PRE (K3M_B16_PREFETCH): the
// epilogue stages through an image placed after stage 0, and issues the next unit's first k-tile of LDS-DMA
// into stage 0 before its first store, so that load overlaps this tile's epilogue.
template <int TBM, int TBN, int WM, int WN>
struct PUnit {
  int p, m0, n0, slice, kbeg, kend;
  __device__ __forceinline__ void decode(const GemmGroup& grp, int u) {
    const int total = grp.start[grp.count];
    const int P = gridDim.x;
    const int base = (u / P) * P, cnt = min(P, total - base);
    const int id = base + xcd_remap(u - base, cnt);
    p = 0;
    while (p + 1 < grp.count && id >= grp.start[p + 1]) ++p;
    p = __builtin_amdgcn_readfirstlane(p);
    const K3mGemm& g = grp.g[p];
    coords(id - grp.start[p], g.m, g.n, TBM, TBN, m0, n0, slice);
    k_range(g, slice, kbeg, kend);
  }
};

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF, bool PRE, bool PP = false>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_persist_kernel(GemmGroup grp) {
  using S = Shape<TBM, TBN, WM, WN>;
  constexpr int EOFF = PRE ? TBM * BK + TBN * BK : 0;   // the epilogue image after stage 0 when prefetching
  constexpr int WORDS = (EOFF + EpiLds<TBM, TBN, WM, WN>::E > S::LDS) ? EOFF + EpiLds<TBM, TBN, WM, WN>::E : S::LDS;
  __shared__ __attribute__((aligned(16))) uint16_t smem[WORDS];
  const int total = grp.start[grp.count];
  int u = blockIdx.x;
  if (u >= total) return;
  if (grp.lab & 2) {   // lab: staggered start (bounded wait on the 100 MHz real-time clock)
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    const uint64_t until = t0 + (uint64_t)(blockIdx.x & 3) * (uint64_t)grp.stagger;
    while (__builtin_amdgcn_s_memrealtime() < until) __builtin_amdgcn_s_sleep(8);
  }
  const bool nostore = (grp.lab & 1) != 0, ntstore = (grp.lab & 4) != 0;
  PUnit<TBM, TBN, WM, WN> cur;
  cur.decode(grp, u);
  bool pre = false;
  for (;;) {   // uniform over the workgroup: every wave leaves together
    const K3mGemm& g = grp.g[cur.p];
    Acc<MF, TBM / WM, TBN / WN> acc;
    if constexpr (PP && !PRE)
      mainloop_pp<TBM, TBN, WM, WN, AK, BK_, MF>(static_cast<const uint16_t*>(g.a), g.lda,
                                                 static_cast<const uint16_t*>(g.b), g.ldb, g.m, g.n, cur.m0, cur.n0,
                                                 cur.kbeg, cur.kend, smem, acc);
    else if constexpr (MF == 32)
      mainloop32<TBM, TBN, WM, WN, AK, BK_>(static_cast<const uint16_t*>(g.a), g.lda, static_cast<const uint16_t*>(g.b),
                                            g.ldb, g.m, g.n, cur.m0, cur.n0, cur.kbeg, cur.kend, smem, acc, pre);
    else
      mainloop<TBM, TBN, WM, WN, AK, BK_>(static_cast<const uint16_t*>(g.a), g.lda, static_cast<const uint16_t*>(g.b),
                                          g.ldb, g.m, g.n, cur.m0, cur.n0, cur.kbeg, cur.kend, smem, acc, pre);
    const int nu = u + gridDim.x;
    const bool more = nu < total;
    PUnit<TBM, TBN, WM, WN> nxt = cur;
    if (more) nxt.decode(grp, nu);
    bool next_pre = false;
    if constexpr (PRE) {
      const bool issue = more && (nxt.kend - nxt.kbeg) / BK > 0;
      auto hook = [&]() {
        if (issue) {
          const K3mGemm& gn = grp.g[nxt.p];
          Loader<AK, TBM, S::NT> la;
          Loader<BK_, TBN, S::NT> lb;
          la.init(static_cast<const uint16_t*>(gn.a), gn.lda, nxt.m0, nxt.kbeg, gn.m);
          lb.init(static_cast<const uint16_t*>(gn.b), gn.ldb, nxt.n0, nxt.kbeg, gn.n);
          la.issue(smem);
          lb.issue(smem + TBM * BK);
        }
      };
      epilogue<TBM, TBN, WM, WN, EPI, CT>(g, cur.m0, cur.n0, smem + EOFF, acc, cur.slice, hook, nostore, ntstore);
      next_pre = issue;
    } else {
      epilogue<TBM, TBN, WM, WN, EPI, CT>(g, cur.m0, cur.n0, smem, acc, cur.slice, NoHookB(), nostore, ntstore);
    }
    if (!more) break;
    u = nu;
    cur = nxt;
    pre = next_pre;
  }
}


// ====================================================================== two workgroups per CU
// The 256x256 walk above runs ONE 8-wave workgroup per CU (128 KB of LDS stages): while it runs its
// epilogue (the bias / GELU / dGELU VALU and the C stores: a third of a K = 768 GEMM) no MFMA issues on
// that CU, and the lab timings (profiles/r4a_ab_flash_km_and_b16_lab.txt: stores off -13 %, epilogue
// math ~ -25 % on FFN1) put most of the K = 768 GEMMs' loss there.  The dual form fits TWO workgroups
// on a CU so one's epilogue overlaps the other's main loop (MFMA and VALU are separate pipes; vmcnt is
// per wave, so one workgroup's stores never hold the other's DMA waits):
//  * tile 256 x 128 x 32, 4 waves (2 x 2, each 128 x 64 — the same per-wave tile and accumulators);
//  * THREE LDS stages of 24 KB (72 KB per workgroup, 144 KB for the pair); operands by LDS-DMA with the
//    DMA of k-tile t+4 issued at iteration t into the stage just read, two k-tiles in flight across each
//    barrier (counted vmcnt), fragment reads of tile t+1 under the MFMAs of tile t;
//  * K-contiguous images [TILE][32] (64-B rows): chunk c of row r at slot c ^ g((r >> 2) & 3) with
//    g = {0, 2, 3, 1}, conflict-free for the ds_read_b128 lane groups of both MFMA shapes;
//    MN-contiguous images [32][TILE] as above (mn_off), transposing reads;
//  * persistent walk over 2 x CUs workgroups; epilogue through LDS exactly as the 8-wave kernel (same
//    arithmetic per element: bit-identical C).
constexpr int BKD = 32;

__device__ __forceinline__ int swz4(int r) { return (0x1320 >> (((r >> 2) & 3) << 2)) & 3; }
__device__ __forceinline__ int kc4_off(int r, int c) { return r * BKD + ((c ^ swz4(r)) << 3); }

template <bool KC, int TILE, int NT>
struct LoaderD {
  static constexpr int INSTS = TILE * BKD * 2 / 1024;   // wave instructions per k-tile
  static constexpr int NW = NT / 64;
  static constexpr int NI = INSTS / NW;                  // per wave
  static_assert(INSTS % NW == 0, "tile must split evenly over the waves");
  const uint16_t* base;
  long long step;
  uint32_t off[NI];
  int lds0;
  __device__ __forceinline__ void init(const uint16_t* __restrict__ a, long long ld, int mn0, int kbeg, int MN) {
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lds0 = w * 512;
    base = a + (KC ? (long long)kbeg : (long long)kbeg * ld);
    step = KC ? BKD : BKD * ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int inst = w + NW * i;
      if constexpr (KC) {   // 16 rows x 4 chunks per instruction
        const int row = inst * 16 + (l >> 2), slot = l & 3;
        const int ch = slot ^ swz4(row);
        off[i] = (uint32_t)((long long)min(mn0 + row, MN - 1) * ld + ch * 8);
      } else {
        constexpr int CPR = TILE / 8, RPI = 64 / CPR;
        const int kr = inst * RPI + l / CPR, slot = l % CPR;
        const int ch = slot ^ (((kr & 3) << 2) | ((kr >> 2) & 3));
        off[i] = (uint32_t)((long long)kr * ld + max(0, min(mn0 + ch * 8, MN - 8)));
      }
    }
  }
  __device__ __forceinline__ void issue(uint16_t* img) {
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(base + off[i], img + lds0 + i * NW * 512);
    base += step;
  }
};

// s_waitcnt vmcnt(N) only (expcnt, lgkmcnt at their maxima: not waited for)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Fragments of a wave's 128 x 64 slab: 16x16x32 — one set is a whole 32-deep k-tile (8 A x 4 B);
// 32x32x16 — one set is one 16-deep substep (4 A x 2 B), two per k-tile (the transposing reads of
// MN-contiguous operands take two ds_read_b64_tr_b16 per fragment: whole-tile sets spilled)
template <int MF, bool AK, bool BK_, int TBM, int TBN>
struct FragsD;
template <bool AK, bool BK_, int TBM, int TBN>
struct FragsD<16, AK, BK_, TBM, TBN> {
  bf16x8 a[8], b[4];
  __device__ __forceinline__ void read(const uint16_t* st, int, int wm, int wn, int lane) {
    const uint16_t* sb = st + TBM * BKD;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (AK) a[i] = *reinterpret_cast<const bf16x8*>(st + kc4_off(wm + 16 * i + (lane & 15), lane >> 4));
      else a[i] = frag<false, TBM>(st, wm + 16 * i, 0, lane);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (BK_) b[j] = *reinterpret_cast<const bf16x8*>(sb + kc4_off(wn + 16 * j + (lane & 15), lane >> 4));
      else b[j] = frag<false, TBN>(sb, wn + 16 * j, 0, lane);
    }
  }
  template <typename AccT>
  __device__ __forceinline__ void mfma(AccT& acc) const {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc.v[i][j], 0, 0, 0);
  }
};
template <bool AK, bool BK_, int TBM, int TBN>
struct FragsD<32, AK, BK_, TBM, TBN> {
  bf16x8 a[4], b[2];
  __device__ __forceinline__ void read(const uint16_t* st, int s, int wm, int wn, int lane) {
    const uint16_t* sb = st + TBM * BKD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (AK) a[i] = *reinterpret_cast<const bf16x8*>(st + kc4_off(wm + 32 * i + (lane & 31), 2 * s + (lane >> 5)));
      else a[i] = frag32<false, TBM>(st, wm + 32 * i, s, lane);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if constexpr (BK_) b[j] = *reinterpret_cast<const bf16x8*>(sb + kc4_off(wn + 32 * j + (lane & 31), 2 * s + (lane >> 5)));
      else b[j] = frag32<false, TBN>(sb, wn + 32 * j, s, lane);
    }
  }
  template <typename AccT>
  __device__ __forceinline__ void mfma(AccT& acc) const {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc.v[i][j], 0, 0, 0);
  }
};

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int MF>
__device__ __forceinline__ void mainloop_d(const uint16_t* __restrict__ A, long long lda,
                                           const uint16_t* __restrict__ B, long long ldb, int M, int N, int m0,
                                           int n0, int kbeg, int kend, uint16_t* smem,
                                           Acc<MF, TBM / WM, TBN / WN>& acc) {
  constexpr int NT = 64 * WM * WN, STAGE = (TBM + TBN) * BKD;
  static_assert(TBM / WM == 128 && TBN / WN == 64, "per-wave slab 128 x 64");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.v[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc.v[i][j][r] = 0.f;
  }
  LoaderD<AK, TBM, NT> la;
  LoaderD<BK_, TBN, NT> lb;
  la.init(A, lda, m0, kbeg, M);
  lb.init(B, ldb, n0, kbeg, N);
  constexpr int NI = LoaderD<AK, TBM, NT>::NI + LoaderD<BK_, TBN, NT>::NI;   // DMA instructions per k-tile
  const int nk = kend > kbeg ? (kend - kbeg) / BKD : 0;
  if (nk == 0) return;
  auto issue = [&](int stg) {
    la.issue(smem + stg * STAGE);
    lb.issue(smem + stg * STAGE + TBM * BKD);
  };
  issue(0);
  if (nk > 1) issue(1);
  if (nk > 2) issue(2);
  if (nk > 2) wait_vm<2 * NI>();
  else if (nk > 1) wait_vm<NI>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  FragsD<MF, AK, BK_, TBM, TBN> F, G;
  F.read(smem, 0, wm, wn, lane);
  if constexpr (MF == 16) {
    // iteration t: tile t+1 -> the other set under the MFMAs of tile t; wait for tile t+2 (tile t+3 may stay
    // in flight), barrier, DMA tile t+4 into the stage just read
    if (nk > 2) wait_vm<NI>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (nk > 3) issue(0);   // tile 3 -> the stage of tile 0 (already in F)
    int rs = 1;              // stage of tile t+1
    auto step = [&](FragsD<MF, AK, BK_, TBM, TBN>& cur, FragsD<MF, AK, BK_, TBM, TBN>& nxt, int t) {
      nxt.read(smem + rs * STAGE, 0, wm, wn, lane);   // past the last tile: a stale stage nobody uses
      __builtin_amdgcn_sched_barrier(0);
      cur.mfma(acc);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 3 < nk) wait_vm<NI>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 4 < nk) issue(rs);
      rs = rs == 2 ? 0 : rs + 1;
    };
    int t = 0;
    for (; t + 1 < nk; t += 2) {
      step(F, G, t);
      step(G, F, t + 1);
    }
    if (t < nk) step(F, G, t);
  } else {
    // iteration t: substep 1 of tile t -> G under the MFMAs of substep 0 (F); wait for tile t+1 (tile t+2 may
    // stay in flight), barrier, DMA tile t+3 into tile t's stage (both substeps read), substep 0 of tile
    // t+1 -> F under the MFMAs of G
    int cs = 0;   // stage of tile t
    for (int t = 0; t < nk; ++t) {
      const int ns = cs == 2 ? 0 : cs + 1;
      G.read(smem + cs * STAGE, 1, wm, wn, lane);
      __builtin_amdgcn_sched_barrier(0);
      F.mfma(acc);
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (t + 2 < nk) wait_vm<NI>();
      else wait_vm<0>();
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (t + 3 < nk) issue(cs);
      F.read(smem + ns * STAGE, 0, wm, wn, lane);   // past the last tile: a stale stage nobody uses
      __builtin_amdgcn_sched_barrier(0);
      G.mfma(acc);
      __builtin_amdgcn_sched_barrier(0);
      cs = ns;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();   // the epilogue reuses the stages
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
__global__ __launch_bounds__(64 * WM * WN, 2) void gemm_dual_kernel(GemmGroup grp) {
  constexpr int WORDS = 3 * (TBM + TBN) * BKD;
  static_assert(EpiLds<TBM, TBN, WM, WN>::E <= WORDS, "epilogue staging exceeds the LDS stages");
  __shared__ __attribute__((aligned(16))) uint16_t smem[WORDS];
  const int total = grp.start[grp.count];
  int u = blockIdx.x;
  if (u >= total) return;
  for (;;) {   // uniform over the workgroup: every wave leaves together
    PUnit<TBM, TBN, WM, WN> cur;
    cur.decode(grp, u);
    const K3mGemm& g = grp.g[cur.p];
    Acc<MF, TBM / WM, TBN / WN> acc;
    mainloop_d<TBM, TBN, WM, WN, AK, BK_, MF>(static_cast<const uint16_t*>(g.a), g.lda,
                                              static_cast<const uint16_t*>(g.b), g.ldb, g.m, g.n, cur.m0, cur.n0,
                                              cur.kbeg, cur.kend, smem, acc);
    epilogue<TBM, TBN, WM, WN, EPI, CT>(g, cur.m0, cur.n0, smem, acc, cur.slice);
    u += gridDim.x;
    if (u >= total) break;
  }
}

}  // namespace k3m_b16
