// Persistent bf16x6 fp32 GEMM: one 512-thread workgroup per CU walks the output tiles (and split-K
// slices) of one GEMM or of a group of independent GEMMs, and overlaps each tile's epilogue with the
// next tile's first global loads.
//
// Why (profiles/r3_pmc_x6_ffn1.json): the non-persistent 256x256x16 kernel keeps the matrix pipes
// busy 51 % of the time at 1.95 GHz.  Per workgroup lifetime (~241 k cycles on the FFN1 forward) the
// MFMAs need ~147 k; the epilogue of a 256x256 fp32 tile writes 512 KB (C and the GELU pre-activation)
// at the CU's share of HBM write bandwidth (~12 B/cycle), ~43 k cycles with no matrix work on that CU,
// and every workgroup then pays its prologue load latency again.  Here the next tile's first two
// k-tiles are loaded into registers BEFORE the epilogue's stores are issued: the loads are older than
// the stores, so the next tile's first wait (vmcnt) covers the loads only and the 512 KB drain while
// the next tile's MFMAs run.  Same main loop, split, LDS images and epilogue as gemm_x6_tile.h.
#include "gemm_x6_tile.h"

namespace k3m_x6 {
namespace {

// Work unit u of the grid-stride walk -> (problem, split-K slice, tile origin, k range).  Units of one
// "wave" (u / gridDim.x) run concurrently: inside a wave the XCD remap gives each XCD a contiguous id
// range, then GROUP row-tiles walk N together (the A panel stays in the XCD's L2).
struct Unit {
  int p, slice, m0, n0, kbeg, kend;
};

template <int TBM, int TBN, int BK>
__device__ __forceinline__ Unit decode(const GemmGroup& grp, int u) {
  const int total = grp.start[grp.count];
  const int P = gridDim.x;
  const int base = (u / P) * P, cnt = min(P, total - base);
  const int id = base + K3M_F32_NS::xcd_remap(u - base, cnt);
  Unit r;
  r.p = 0;
  while (r.p + 1 < grp.count && id >= grp.start[r.p + 1]) ++r.p;
  const K3mGemm& g = grp.g[r.p];
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN, tiles = tm * tn;
  const int local = id - grp.start[r.p];
  r.slice = local / tiles;
  const int t = local - r.slice * tiles;
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tn, first_m = (t / group_sz) * GROUP, gm_sz = min(tm - first_m, GROUP);
  r.m0 = (first_m + (t % group_sz) % gm_sz) * TBM;
  r.n0 = ((t % group_sz) / gm_sz) * TBN;
  r.kbeg = 0;
  r.kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    r.kbeg = r.slice * per;
    r.kend = min(g.k, r.kbeg + per);
  }
  // workgroup-uniform: keep the unit in scalar registers (the main loop needs every VGPR)
  r.p = __builtin_amdgcn_readfirstlane(r.p);
  r.slice = __builtin_amdgcn_readfirstlane(r.slice);
  r.m0 = __builtin_amdgcn_readfirstlane(r.m0);
  r.n0 = __builtin_amdgcn_readfirstlane(r.n0);
  r.kbeg = __builtin_amdgcn_readfirstlane(r.kbeg);
  r.kend = __builtin_amdgcn_readfirstlane(r.kend);
  return r;
}

// The main loop of gemm_x6_tile.h cut in two: prefetch() issues the first global loads of a tile
// (register sets ra/rb, and ra1/rb1 for the two-set pipeline), run() consumes them.
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE>
struct Loop {
  static constexpr int NT = 64 * WM * WN;
  static constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  static constexpr int BUF = 3 * (TBM + TBN) * BK;
  static constexpr int PA = TBM * BK, PB = TBN * BK;
  Stage<AK, TBM, BK, NT> ra, ra1;
  Stage<BK_, TBN, BK, NT> rb, rb1;
  Src<AK, TBM, BK, NT> sa;
  Src<BK_, TBN, BK, NT> sb;
  long long lda, ldb;
  int nkf, krem;

  __device__ __forceinline__ void prefetch(const K3mGemm& g, const Unit& u) {
    lda = g.lda;
    ldb = g.ldb;
    sa.init(static_cast<const float*>(g.a), lda, u.m0, u.kbeg, g.m);
    sb.init(static_cast<const float*>(g.b), ldb, u.n0, u.kbeg, g.n);
    const int klen = u.kend - u.kbeg;
    nkf = klen > 0 ? klen / BK : 0;
    krem = klen > 0 ? klen - nkf * BK : 0;
    if (nkf > 0) {
      load_full<AK, TBM, BK, NT>(sa, lda, ra, nkf > 1);
      load_full<BK_, TBN, BK, NT>(sb, ldb, rb, nkf > 1);
    }
  }
  // the second register set of the two-set pipeline: issued after the epilogue, so that only one set
  // is live beside the accumulators while the epilogue runs
  __device__ __forceinline__ void prefetch2() {
    if constexpr (PIPE) {
      if (nkf > 0) {
        load_full<AK, TBM, BK, NT>(sa, lda, ra1, nkf > 2);
        load_full<BK_, TBN, BK, NT>(sb, ldb, rb1, nkf > 2);
      }
    }
  }

  __device__ __forceinline__ void compute(const __bf16* smem_stage, floatx16 (&acc)[FM][FN]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
    const int h = lane >> 5, cl = lane & 31;
    const __bf16* as = smem_stage;
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
  }

  // Precondition: prefetch() issued for this tile; the LDS is free (the previous epilogue ended on a
  // barrier).  Postcondition: acc holds the tile, the LDS is free again (last barrier).
  __device__ __forceinline__ void run(__bf16* smem, floatx16 (&acc)[FM][FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if (nkf > 0) {
      store_tile<AK, TBM, BK, NT>(smem, ra);
      store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
    }
    __syncthreads();
    if constexpr (!PIPE) {
      for (int kt = 0; kt < nkf; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nkf;
        if (more) {
          load_full<AK, TBM, BK, NT>(sa, lda, ra, kt + 2 < nkf);
          load_full<BK_, TBN, BK, NT>(sb, ldb, rb, kt + 2 < nkf);
        }
        compute(smem + cur * BUF, acc);
        if (more) {
          store_tile<AK, TBM, BK, NT>(smem + (cur ^ 1) * BUF, ra);
          store_tile<BK_, TBN, BK, NT>(smem + (cur ^ 1) * BUF + 3 * PA, rb);
        }
        __syncthreads();
      }
    } else {
      for (int kt = 0; kt < nkf; kt += 2) {
        load_full<AK, TBM, BK, NT>(sa, lda, ra, kt + 3 < nkf);
        load_full<BK_, TBN, BK, NT>(sb, ldb, rb, kt + 3 < nkf);
        compute(smem, acc);
        store_tile<AK, TBM, BK, NT>(smem + BUF, ra1);
        store_tile<BK_, TBN, BK, NT>(smem + BUF + 3 * PA, rb1);
        __syncthreads();
        if (kt + 1 >= nkf) break;
        load_full<AK, TBM, BK, NT>(sa, lda, ra1, kt + 4 < nkf);
        load_full<BK_, TBN, BK, NT>(sb, ldb, rb1, kt + 4 < nkf);
        compute(smem + BUF, acc);
        store_tile<AK, TBM, BK, NT>(smem, ra);
        store_tile<BK_, TBN, BK, NT>(smem + 3 * PA, rb);
        __syncthreads();
      }
    }
    if (krem > 0) {   // peeled partial k-tile (masked loads); the pointers rest on the last full tile
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
      compute(smem + cur * BUF, acc);
      __syncthreads();
    }
  }
};

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, int EPI, bool PIPE>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_x6_persist_kernel(GemmGroup grp) {
  constexpr int LDS_BF16 = 2 * 3 * (TBM + TBN) * BK;
  constexpr int EPI_F32 = WM * WN * 32 * (TBN / WN + 8);
  constexpr int WORDS = (LDS_BF16 / 2 > EPI_F32 ? LDS_BF16 / 2 : EPI_F32);
  __shared__ __attribute__((aligned(16))) float smem[WORDS];
  const int total = grp.start[grp.count];
  int u = blockIdx.x;
  if (u >= total) return;
  Loop<TBM, TBN, WM, WN, BK, AK, BK_, PIPE> lp;
  Unit cur = decode<TBM, TBN, BK>(grp, u);
  lp.prefetch(grp.g[cur.p], cur);
  lp.prefetch2();
  floatx16 acc[TBM / WM / 32][TBN / WN / 32];
  for (;;) {
    lp.run(reinterpret_cast<__bf16*>(smem), acc);
    const int nu = u + gridDim.x;
    const bool more = nu < total;
    const Unit nxt = more ? decode<TBM, TBN, BK>(grp, nu) : cur;
    // the next tile's first loads go out inside the epilogue, after the first accumulator slice has
    // moved to LDS (its registers are free) and before this tile's first global store
    auto hook = [&]() {
      if (more) lp.prefetch(grp.g[nxt.p], nxt);
    };
    K3M_F32_NS::epilogue<TBM, TBN, WM, WN, EPI, WORDS, decltype(hook), !(AK && !BK_)>(
        grp.g[cur.p], cur.m0, cur.n0, smem, acc, cur.slice, hook);
    if (!more) break;   // every wave leaves here: the exit condition is uniform over the workgroup
    lp.prefetch2();
    u = nu;
    cur = nxt;
  }
}

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE>
int launch(const GemmGroup& grp, int epi, int nblk, hipStream_t st) {
  const dim3 grid(nblk);
  switch (epi) {
#define K3M_P_CASE(E)                                                                                       \
    case E:                                                                                                 \
      hipLaunchKernelGGL((gemm_x6_persist_kernel<TBM, TBN, WM, WN, BK, AK, BK_, E, PIPE>), grid,            \
                         dim3(64 * WM * WN), 0, st, grp);                                                   \
      break;
    K3M_P_CASE(K3M_EPI_NONE)
    K3M_P_CASE(K3M_EPI_BIAS)
    K3M_P_CASE(K3M_EPI_BIAS_GELU)
    K3M_P_CASE(K3M_EPI_DGELU)
    K3M_P_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_P_CASE
    default: return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

}  // namespace
}  // namespace k3m_x6

// Persistent launch of a prepared group (start[] in 256 x TBN tiles, TBN = 256 or 128): one workgroup
// per CU (the x6 tiles use 96-144 KB of LDS), never more workgroups than units.
int k3m_x6_persistent_launch(const k3m_x6::GemmGroup& grp, bool t256, bool ak, bool bk, int cus, hipStream_t st) {
  const int total = grp.start[grp.count];
  if (total <= 0) return 0;
  const int nblk = total < cus ? total : cus;
  const int epi = grp.g[0].epilogue;
  using namespace k3m_x6;
  if (t256) {
    if (ak && bk) return launch<256, 256, 4, 2, 16, true, true, true>(grp, epi, nblk, st);
    if (ak) return launch<256, 256, 2, 4, 16, true, false, true>(grp, epi, nblk, st);
    if (!bk) return launch<256, 256, 2, 4, 16, false, false, false>(grp, epi, nblk, st);
    return K3M_EINVAL;
  }
  if (ak && bk) return launch<256, 128, 4, 2, 32, true, true, true>(grp, epi, nblk, st);
  if (ak) return launch<256, 128, 4, 2, 32, true, false, true>(grp, epi, nblk, st);
  if (bk) return launch<256, 128, 4, 2, 32, false, true, true>(grp, epi, nblk, st);
  return launch<256, 128, 4, 2, 32, false, false, false>(grp, epi, nblk, st);
}

// Two-workgroups-per-CU variant (A/B knob K3M_X6_VARIANT=1 in gemm.hip): 128x256x16 tiles of 4 waves (each
// 64x128, the accumulator footprint of the 256x256 kernel's waves), 72 KB of LDS, so that two workgroups
// share a CU and one's epilogue stores overlap the other's main loop (the vmcnt counter is in issue
// order for loads AND stores, so inside one workgroup a tile's stores stall the next tile's loads).
int k3m_x6_variant_launch(const K3mGemm& g, int variant, hipStream_t st) {
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  if (variant < 1 || variant > 4 || !(ak && bk) || (variant >= 3 && g.epilogue == K3M_EPI_DGELU)) return -1;
  if (variant >= 3 && g.epilogue != K3M_EPI_DGELU) {
    // one wave per SIMD: 256x256 tile over 2x2 waves of 128x128 (256 accumulators, up to 512 registers
    // per wave): twice the MFMAs per fragment read, no register aliasing between the staged global loads
    // and the fragments (variant 3: two register sets, 4: one)
    const int tm3 = (g.m + 255) / 256, tn3 = (g.n + 255) / 256;
    dim3 grid3(tm3 * tn3, g.splitk > 1 ? g.splitk : 1);
    switch (g.epilogue) {
#define K3M_V3_CASE(E)                                                                                     \
      case E:                                                                                              \
        if (variant == 3)                                                                                  \
          hipLaunchKernelGGL((k3m_x6::gemm_x6_kernel<256, 256, 2, 2, 16, true, true, true, E, 1, true>), grid3, \
                             dim3(256), 0, st, g);                                                         \
        else                                                                                               \
          hipLaunchKernelGGL((k3m_x6::gemm_x6_kernel<256, 256, 2, 2, 16, true, true, true, E, 1, false>), grid3, \
                             dim3(256), 0, st, g);                                                         \
        break;
      K3M_V3_CASE(K3M_EPI_NONE)
      K3M_V3_CASE(K3M_EPI_BIAS)
      K3M_V3_CASE(K3M_EPI_BIAS_GELU)
      K3M_V3_CASE(K3M_EPI_DGELU)
      K3M_V3_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_V3_CASE
      default: return K3M_EINVAL;
    }
    K3M_CHECK_LAUNCH();
    return 0;
  }
  const int tm = (g.m + 127) / 128, tn = (g.n + 255) / 256;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_V_CASE(E)                                                                                          \
    case E:                                                                                                    \
      if (variant == 1)                                                                                        \
        hipLaunchKernelGGL((k3m_x6::gemm_x6_kernel<128, 256, 2, 2, 16, true, true, true, E, 2, false>), grid, \
                           dim3(256), 0, st, g);                                                               \
      else                                                                                                     \
        hipLaunchKernelGGL((k3m_x6::gemm_x6_kernel<128, 256, 2, 2, 16, true, true, true, E, 2, true>), grid,  \
                           dim3(256), 0, st, g);                                                               \
      break;
    K3M_V_CASE(K3M_EPI_NONE)
    K3M_V_CASE(K3M_EPI_BIAS)
    K3M_V_CASE(K3M_EPI_BIAS_GELU)
    K3M_V_CASE(K3M_EPI_DGELU)
    K3M_V_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_V_CASE
    default: return K3M_EINVAL;
  }
  K3M_CHECK_LAUNCH();
  return 0;
}
