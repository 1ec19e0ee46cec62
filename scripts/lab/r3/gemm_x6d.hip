// fp32 GEMM on the bf16 matrix cores from PRE-SPLIT operands ("x6d"): the bf16x6 products of
// gemm_x6_tile.h, with both operands handed over as their three exact bf16 planes (h, m, l:
// x = h + m + l, k3m_split3 below) and staged global -> LDS by LDS-DMA.
//
// Why: in the x6 kernels every workgroup loads fp32 tiles into registers, splits them (~4.5 VALU per
// element) and writes three planes to LDS, once per tile that reads the operand (the FFN1 activation
// panel is split again by each of its 12 column tiles).  The staging registers, the split VALU and
// the ds_write pass sit in the main loop beside the MFMAs; the PMC profile
// (profiles/r3_pmc_x6_ffn1_fwd.json) shows the matrix pipe idle half the cycles.  Split once per
// operand instead (an HBM pass of 4 B read + 6 B written per element, or fused into the producer),
// and the main loop is the bf16 LDS-DMA loop of gemm_b16_tile.h with three planes per operand:
// no staging registers, no VALU, no ds_write.
//
// Structure: 256x128x16 tiles, 4 waves of 128x64, TWO workgroups per CU (72 KiB of LDS each: two stages
// of 3 x (256 + 128) x 16 bf16), so that one workgroup's barrier waits, fragment reads and epilogue
// stores (a 256x128 fp32 tile is 128 KiB of stores, ~1/3 of its MFMA time at K = 768 at the CU's
// share of HBM bandwidth) run under the other's MFMAs.  The LDS images
// are those of the x6 kernel (k3m_x6::slot_off / mn_off, the swizzle moved to the per-lane DMA
// source), the fragment reads and the six MFMAs per (i, j) in the same order, the epilogue is
// k3m_f32::epilogue: the result is bit-identical to the 256x256 x6 kernel on the same operands.
#include "gemm_x6_tile.h"

namespace k3m_x6d {

using k3m_x6::bf16x8;
using k3m_x6::mn_frag;
using k3m_x6::slot_off;

constexpr int BK = 16;      // k per stage: one 32x32x16 MFMA step

__device__ __forceinline__ void glds16(const uint16_t* g, __bf16* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// chunk swizzle of the MN-contiguous image row k (the XOR of k3m_x6::mn_off; an involution)
template <int TILE>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (TILE >= 128) return ((k & 3) << 2) | ((k >> 2) & 3);
  else return ((k >> 1) & 1) << 2;
}

// LDS-DMA sources of one operand's three planes for one k-tile.  The image of plane p is
// [TILE][16] (K-contiguous) or [16][TILE] (MN-contiguous) bf16, TILE*32 bytes = SEG 1-KiB segments;
// one wave instruction fills one segment lane-linearly (lane l -> bytes 16 l), so the swizzle is
// applied to the lane's SOURCE chunk.  Instruction i of wave w fills segment (w + NW i) of the
// operand's 3*SEG segments.  Rows / column chunks past the M or N edge are clamped to valid
// addresses: their products reach only C entries the epilogue does not store.
template <bool KC, int TILE, int NT>
struct PLoader {
  static constexpr int SEG = TILE * BK * 2 / 1024;
  static constexpr int NW = NT / 64;
  static constexpr int NI = 3 * SEG / NW;
  static_assert((3 * SEG) % NW == 0, "the planes' segments must split evenly over the waves");
  const uint16_t* src[NI];   // wave-uniform running bases (plane + k-tile)
  uint32_t off[NI];          // per-lane element offsets
  int dst[NI];               // wave-uniform element offsets in the operand's stage image
  long long step;

  __device__ __forceinline__ void init(const uint16_t* a, long long ld, long long pstride, int mn0, int kbeg, int MN) {
    const int l = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    step = KC ? BK : BK * ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int id = w + NW * i, pl = id / SEG, sub = id % SEG;
      src[i] = a + pl * pstride + (KC ? (long long)kbeg : (long long)kbeg * ld);
      dst[i] = pl * TILE * BK + sub * 512;
      if constexpr (KC) {
        const int row = sub * 32 + (l >> 1), c = (l & 1) ^ ((row >> 3) & 1);
        off[i] = (uint32_t)((long long)min(mn0 + row, MN - 1) * ld + 8 * c);
      } else {
        constexpr int CPR = TILE / 8, RPS = 64 / CPR;
        const int kr = sub * RPS + l / CPR, ch = (l % CPR) ^ mn_swz<TILE>(kr);
        off[i] = (uint32_t)((long long)kr * ld + max(0, min(mn0 + 8 * ch, MN - 8)));
      }
    }
  }
  __device__ __forceinline__ void issue(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      glds16(src[i] + off[i], img + dst[i]);
      src[i] += step;
    }
  }
};

// acc = A[m0.., kbeg:kend] . B[n0.., kbeg:kend]^T over (kend - kbeg) / 16 k-tiles ((kend - kbeg) % 16 == 0).
// Two LDS stages, per k-tile kt: wait for this wave's DMA of kt, barrier (every wave's DMA of kt landed,
// every wave done reading stage (kt+1)&1), fragment reads of kt, THEN the DMA of kt+1 into the other
// stage (issued after the reads, so the compiler's LDS-DMA hazard check before them finds nothing in
// flight), then the 48 MFMAs of kt.  Two workgroups share a CU: one's barrier waits, fragment reads
// and epilogue stores run under the other's MFMAs.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void mainloop2(const K3mGemm& g, long long pa, long long pb, int m0, int n0, int kbeg,
                                         int kend, __bf16* img, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int NT = 64 * WM * WN, FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int STAGE = 3 * (TBM + TBN) * BK, PA = TBM * BK, PB = TBN * BK;
  using LA = PLoader<AK, TBM, NT>;
  using LB = PLoader<BK_, TBN, NT>;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  const int h = lane >> 5, cl = lane & 31;
  LA la;
  LB lb;
  la.init(static_cast<const uint16_t*>(g.a), g.lda, pa, m0, kbeg, g.m);
  lb.init(static_cast<const uint16_t*>(g.b), g.ldb, pb, n0, kbeg, g.n);
  la.issue(img);
  lb.issue(img + 3 * PA);
  for (int kt = 0; kt < nk; ++kt) {
    __bf16* cur = img + (kt & 1) * STAGE;
    __bf16* nxt = img + ((kt + 1) & 1) * STAGE;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const __bf16* as = cur;
    const __bf16* bs = cur + 3 * PA;
    bf16x8 a[3][FM], b[3][FN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[pl][i] = AK ? *reinterpret_cast<const bf16x8*>(as + pl * PA + slot_off<BK>(wm + 32 * i + cl, h))
                      : mn_frag<TBM>(as + pl * PA, wm + 32 * i, 0, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[pl][j] = BK_ ? *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, h))
                       : mn_frag<TBN>(bs + pl * PB, wn + 32 * j, 0, lane);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 1 < nk) {
      la.issue(nxt);
      lb.issue(nxt + 3 * PA);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        // the x6 kernels' order: smallest terms first, (hl + mm + lh), (hm + mh), hh
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();   // the epilogue reuses the stages
}

// Fragments + MFMAs of one k-tile from a stage image (the x6 kernels' order per accumulator).
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void compute(const __bf16* stage, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32, PA = TBM * BK, PB = TBN * BK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  const int h = lane >> 5, cl = lane & 31;
  const __bf16* as = stage;
  const __bf16* bs = stage + 3 * PA;
  bf16x8 a[3][FM], b[3][FN];
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
      a[pl][i] = AK ? *reinterpret_cast<const bf16x8*>(as + pl * PA + slot_off<BK>(wm + 32 * i + cl, h))
                    : mn_frag<TBM>(as + pl * PA, wm + 32 * i, 0, lane);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b[pl][j] = BK_ ? *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, h))
                     : mn_frag<TBN>(bs + pl * PB, wn + 32 * j, 0, lane);
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
    }
}

// Three LDS stages, one workgroup per CU (256x256, 8 waves): per k-tile kt wait for this wave's DMA of kt
// (vmcnt counts the one younger k-tile in flight), barrier (every wave's DMA of kt landed; every wave done
// reading stage (kt-1)%3), DMA of kt+2 into that stage, fragments + MFMAs of kt.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void mainloop3(const K3mGemm& g, long long pa, long long pb, int m0, int n0, int kbeg,
                                          int kend, __bf16* img, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int NT = 64 * WM * WN, FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int STAGE = 3 * (TBM + TBN) * BK;
  using LA = PLoader<AK, TBM, NT>;
  using LB = PLoader<BK_, TBN, NT>;
  constexpr int VMC = LA::NI + LB::NI;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  LA la;
  LB lb;
  la.init(static_cast<const uint16_t*>(g.a), g.lda, pa, m0, kbeg, g.m);
  lb.init(static_cast<const uint16_t*>(g.b), g.ldb, pb, n0, kbeg, g.n);
  la.issue(img);
  lb.issue(img + 3 * TBM * BK);
  if (nk > 1) {
    la.issue(img + STAGE);
    lb.issue(img + STAGE + 3 * TBM * BK);
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 2 < nk) {
      const int nxt = cur == 0 ? 2 : cur - 1;
      la.issue(img + nxt * STAGE);
      lb.issue(img + nxt * STAGE + 3 * TBM * BK);
    }
    compute<TBM, TBN, WM, WN, AK, BK_>(img + cur * STAGE, acc);
    __builtin_amdgcn_sched_barrier(0);
    cur = cur == 2 ? 0 : cur + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// mainloop3 with the fragment reads of k-tile kt+1 interleaved with the MFMAs of kt (lab, K3M_X6D_VARIANT=2):
// F(kt) is in registers when iteration kt starts; after its barrier (DMA of kt+1 landed everywhere, stage kt
// free) the DMA of kt+3 goes to stage kt%3, the A fragments of kt+1 are read into spare registers, and each
// column group j of MFMAs is followed by the reads of kt+1's B fragments j, whose registers it just freed.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_>
__device__ __forceinline__ void mainloop3p(const K3mGemm& g, long long pa, long long pb, int m0, int n0, int kbeg,
                                           int kend, __bf16* img, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int NT = 64 * WM * WN, FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int STAGE = 3 * (TBM + TBN) * BK, PA = TBM * BK, PB = TBN * BK;
  using LA = PLoader<AK, TBM, NT>;
  using LB = PLoader<BK_, TBN, NT>;
  constexpr int VMC = LA::NI + LB::NI;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;
  if (nk == 0) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  const int h = lane >> 5, cl = lane & 31;
  auto rdA = [&](const __bf16* st, int pl, int i) {
    return AK ? *reinterpret_cast<const bf16x8*>(st + pl * PA + slot_off<BK>(wm + 32 * i + cl, h))
              : mn_frag<TBM>(st + pl * PA, wm + 32 * i, 0, lane);
  };
  auto rdB = [&](const __bf16* st, int pl, int j) {
    const __bf16* bs = st + 3 * PA;
    return BK_ ? *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, h))
               : mn_frag<TBN>(bs + pl * PB, wn + 32 * j, 0, lane);
  };
  LA la;
  LB lb;
  la.init(static_cast<const uint16_t*>(g.a), g.lda, pa, m0, kbeg, g.m);
  lb.init(static_cast<const uint16_t*>(g.b), g.ldb, pb, n0, kbeg, g.n);
  la.issue(img);
  lb.issue(img + 3 * PA);
  if (nk > 1) {
    la.issue(img + STAGE);
    lb.issue(img + STAGE + 3 * PA);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (nk > 2) {
    la.issue(img + 2 * STAGE);
    lb.issue(img + 2 * STAGE + 3 * PA);
  }
  bf16x8 a[3][FM], b[3][FN];
#pragma unroll
  for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
    for (int i = 0; i < FM; ++i) a[pl][i] = rdA(img, pl, i);
#pragma unroll
    for (int j = 0; j < FN; ++j) b[pl][j] = rdB(img, pl, j);
  }
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) {
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (kt + 3 < nk) {
      la.issue(img + cur * STAGE);
      lb.issue(img + cur * STAGE + 3 * PA);
    }
    const int nx = cur == 2 ? 0 : cur + 1;
    const __bf16* ns = img + nx * STAGE;   // stage of kt+1 (stale past the last tile: read, never used)
    bf16x8 na[3][FM], nb[3][FN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) na[pl][FM - 1] = rdA(ns, pl, FM - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < FM - 1; ++i) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0][j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) na[pl][i] = rdA(ns, pl, i);   // row i's A fragments are dead
      __builtin_amdgcn_sched_barrier(0);
    }
    constexpr int I = FM - 1;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][I], b[2][j], acc[I][j], 0, 0, 0);
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][I], b[1][j], acc[I][j], 0, 0, 0);
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][I], b[0][j], acc[I][j], 0, 0, 0);
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][I], b[1][j], acc[I][j], 0, 0, 0);
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][I], b[0][j], acc[I][j], 0, 0, 0);
      acc[I][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][I], b[0][j], acc[I][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) nb[pl][j] = rdB(ns, pl, j);   // column j's B fragments are dead
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int i = 0; i < FM; ++i) a[pl][i] = na[pl][i];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[pl][j] = nb[pl][j];
    }
    cur = nx;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}

// NST = 3: 256x256 / 8 waves / one workgroup per CU (mainloop3); NST = 2: 256x128 / 4 waves / two per CU
template <int TBM, int TBN, int WM, int WN, int NST>
struct Lds {
  static constexpr int STAGES = NST == 4 ? 3 : NST;
  static constexpr int STAGE_F = 3 * (TBM + TBN) * BK / 2;   // floats per stage
  static constexpr int EPI_F = WM * WN * 32 * (TBN / WN + 8);
  static constexpr int WORDS = STAGES * STAGE_F > EPI_F ? STAGES * STAGE_F : EPI_F;
};

template <int TBM, int TBN, int WM, int WN, int NST, bool AK, bool BK_, int EPI>
__global__ __launch_bounds__(64 * WM * WN, NST == 2 ? 2 : 1) void gemm_x6d_kernel(K3mGemm g, long long pa, long long pb) {
  constexpr int WORDS = Lds<TBM, TBN, WM, WN, NST>::WORDS;
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
  if constexpr (NST == 4)   // lab: three stages with the fragment reads of kt+1 under the MFMAs of kt
    mainloop3p<TBM, TBN, WM, WN, AK, BK_>(g, pa, pb, m0, n0, kbeg, kend, reinterpret_cast<__bf16*>(smem), acc);
  else if constexpr (NST == 3)
    mainloop3<TBM, TBN, WM, WN, AK, BK_>(g, pa, pb, m0, n0, kbeg, kend, reinterpret_cast<__bf16*>(smem), acc);
  else
    mainloop2<TBM, TBN, WM, WN, AK, BK_>(g, pa, pb, m0, n0, kbeg, kend, reinterpret_cast<__bf16*>(smem), acc);
  k3m_f32::epilogue<TBM, TBN, WM, WN, EPI, WORDS>(g, m0, n0, smem, acc, (int)blockIdx.y);
}

template <int TBM, int TBN, int WM, int WN, int NST, bool AK, bool BK_>
int launch(const K3mGemm& g, long long pa, long long pb, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  const dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_D_CASE(E)                                                                                         \
    case E:                                                                                                   \
      hipLaunchKernelGGL((gemm_x6d_kernel<TBM, TBN, WM, WN, NST, AK, BK_, E>), grid, dim3(64 * WM * WN), 0, st, g, pa, pb); \
      break;
    K3M_D_CASE(K3M_EPI_NONE)
    K3M_D_CASE(K3M_EPI_BIAS)
    K3M_D_CASE(K3M_EPI_BIAS_GELU)
    K3M_D_CASE(K3M_EPI_DGELU)
    K3M_D_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_D_CASE
    default: return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

// ------------------------------------------------------------------ exact three-way split
// planes[p][r][c] (p = 0, 1, 2 at planes + p*pstride, row stride ldp) = h, m, l of x[r][c]; 8 columns
// per thread (two 16-B loads, three 16-B stores).
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, long long ldx, int rows, int cols,
                                                     uint16_t* __restrict__ planes, long long ldp, long long pstride) {
  const int c8 = cols >> 3;
  const long long total = (long long)rows * c8;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(e / c8), c = (int)(e % c8) * 8;
    const floatx4 v0 = *reinterpret_cast<const floatx4*>(x + r * ldx + c);
    const floatx4 v1 = *reinterpret_cast<const floatx4*>(x + r * ldx + c + 4);
    k3m_x6::u32x2v h0, m0, l0, h1, m1, l1;
    k3m_x6::split4(v0, h0, m0, l0);
    k3m_x6::split4(v1, h1, m1, l1);
    uint16_t* p = planes + r * ldp + c;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    *reinterpret_cast<u32x4*>(p) = u32x4{h0[0], h0[1], h1[0], h1[1]};
    *reinterpret_cast<u32x4*>(p + pstride) = u32x4{m0[0], m0[1], m1[0], m1[1]};
    *reinterpret_cast<u32x4*>(p + 2 * pstride) = u32x4{l0[0], l0[1], l1[0], l1[1]};
  }
}

}  // namespace k3m_x6d

namespace {
bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
// lab knob: 0 = 256x256 three stages, 1 = 256x128 two workgroups per CU, 2 = variant 0 with pipelined fragment reads
const int kX6dVariant = k3m_env_int("K3M_X6D_VARIANT", 0);
}  // namespace

extern "C" int k3m_split3(const float* x, long long ldx, int rows, int cols, void* planes, long long ldp,
                          long long pstride, hipStream_t st) {
  K3M_ARG(rows >= 0 && cols >= 0);
  if (rows == 0 || cols == 0) return 0;
  K3M_ARG(x && planes && cols % 8 == 0 && ldx % 4 == 0 && ldp % 8 == 0 && pstride % 8 == 0 && ldx >= cols &&
          ldp >= cols && al16(x) && al16(planes));
  K3M_ARG(pstride >= (long long)(rows - 1) * ldp + cols);
  const long long total = (long long)rows * (cols / 8);
  const int blocks = (int)std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k3m_x6d::split3_kernel, dim3(blocks), dim3(256), 0, st, x, ldx, rows, cols,
                     static_cast<uint16_t*>(planes), ldp, pstride);
  K3M_CHECK_LAUNCH();
  return 0;
}

// Both operands pre-split (k3m_split3): g.a / g.b point at the h planes (bf16, leading dimensions
// g.lda / g.ldb in elements), the m and l planes follow at +pa / +2 pa (+pb / +2 pb) elements.
int k3m_gemm_x6d_impl(const K3mGemm& g, long long pa, long long pb, hipStream_t st) {
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  K3M_ARG(g.k % k3m_x6d::BK == 0 && al16(g.a) && al16(g.b) && g.lda % 8 == 0 && g.ldb % 8 == 0 && pa % 8 == 0 &&
          pb % 8 == 0);
  K3M_ARG((ak || g.m % 8 == 0) && (bk || g.n % 8 == 0));
  // 32-bit per-lane DMA offsets: the largest element offset of each plane must fit
  K3M_ARG((long long)(ak ? g.m : g.k) * (ak ? g.lda : g.lda) < (1LL << 32));
  K3M_ARG((long long)(bk ? g.n : g.k) * g.ldb < (1LL << 32));
  using namespace k3m_x6d;
  if (kX6dVariant == 2) {   // lab: 256x256, three stages, fragment reads of kt+1 under the MFMAs of kt
    if (ak && bk) return launch<256, 256, 4, 2, 4, true, true>(g, pa, pb, st);
    if (ak) return launch<256, 256, 2, 4, 4, true, false>(g, pa, pb, st);
    if (!bk) return launch<256, 256, 2, 4, 4, false, false>(g, pa, pb, st);
    return launch<256, 256, 2, 4, 4, false, true>(g, pa, pb, st);
  }
  if (kX6dVariant == 1) {   // 256x128, two workgroups per CU
    if (ak && bk) return launch<256, 128, 2, 2, 2, true, true>(g, pa, pb, st);
    if (ak) return launch<256, 128, 2, 2, 2, true, false>(g, pa, pb, st);
    if (!bk) return launch<256, 128, 2, 2, 2, false, false>(g, pa, pb, st);
    return launch<256, 128, 2, 2, 2, false, true>(g, pa, pb, st);
  }
  if (ak && bk) return launch<256, 256, 4, 2, 3, true, true>(g, pa, pb, st);
  if (ak) return launch<256, 256, 2, 4, 3, true, false>(g, pa, pb, st);
  if (!bk) return launch<256, 256, 2, 4, 3, false, false>(g, pa, pb, st);
  return launch<256, 256, 2, 4, 3, false, true>(g, pa, pb, st);
}
