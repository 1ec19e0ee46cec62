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
#ifdef K3M_LAB_GROUP   // lab: row-tiles per N walk (scripts/lab/lab_build.sh -DK3M_LAB_GROUP=4)
  constexpr int GROUP = K3M_LAB_GROUP;
#else
  constexpr int GROUP = 8;
#endif
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

// ---------------------------------------------------------------------------------------------------
// Ping-pong main loop (K3M_X6_PP).  The two waves that share a SIMD (w and w + 4) run the same k-loop
// one phase apart, so that one wave's MFMAs run while its partner reads fragments, splits and writes the
// next k-tile and issues the global loads:
//
//   phase      0        1        2        3      ...
//   waves 0-3  M(0)     C(0)     M(1)     C(1)
//   waves 4-7  (wait)   M(0)     C(0)     M(1)
//
// M(t): read this wave's fragments of k-tile t (stage t&1) into registers; split this wave GROUP's half
//       of k-tile t+1 (loaded one iteration earlier) into stage (t+1)&1; load its half of k-tile t+2.
// C(t): the 6 (x BK/16) MFMAs per accumulator, registers only.
// One s_barrier ends every phase.  Stage (t+1)&1 is written in phases 2t (waves 0-3) and 2t+1 (waves
// 4-7) and first read in phase 2t+2; its previous k-tile t-1 was last read in phase 2t-1.  Each group
// stages half of every operand tile (rows [0, TILE/2) by waves 0-3, [TILE/2, TILE) by waves 4-7), one
// register set per thread (loads have two phases to land).  Waves 4-7 enter one barrier late and waves
// 0-3 leave one barrier late, so both execute 2 nt + 2 barriers per tile.
// In round 5's compiler-scheduled loop both waves of a SIMD reached the barrier, the fragment-read
// burst and the MFMAs together (MFMA busy 0.58 of the cycles, 55 % of wave cycles in WAIT_INST_ANY).
template <bool KC, int TILE, int BK>
struct PPHalf {
  static constexpr int NTG = 256;               // threads per wave group
  static constexpr int HT = TILE / 2;           // mn rows / columns staged by one group
  static constexpr int NV = HT * BK / 4;        // float4 per half tile
  static constexpr int NB = NV / NTG;
  static_assert(NV % NTG == 0, "half tile must be a whole number of float4 per thread");
  floatx4 r[NB];
  const float* p[NB];
  int kq[NB];

  __device__ __forceinline__ void init(const float* __restrict__ base, long long ld, int mn0, int kbeg, int MN, int t,
                                       int half) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int idx = t + NTG * b;
      if constexpr (KC) {
        const int row = half * HT + idx / (BK / 4), q = idx % (BK / 4);
        kq[b] = 4 * q;
        p[b] = base + (long long)min(mn0 + row, MN - 1) * ld + kbeg + 4 * q;
      } else {
        const int col = half * HT + 4 * (idx % (HT / 4)), kr = idx / (HT / 4);
        kq[b] = kr;
        p[b] = base + (long long)(kbeg + kr) * ld + max(0, min(mn0 + col, MN - 4));
      }
    }
  }
  // load the k-tile at the pointers and advance them.  krem < BK: a partial last tile; its lanes past
  // krem read the tile's first k (a valid address) and keep zeros, without exec-masked branches
  __device__ __forceinline__ void load(long long ld, int krem) {
    if (krem >= BK) {
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        r[b] = *reinterpret_cast<const floatx4*>(p[b]);
        p[b] += KC ? BK : BK * ld;
      }
    } else {
      const floatx4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const bool in = kq[b] < krem;
        const float* q = in ? p[b] : p[b] - (KC ? kq[b] : (long long)kq[b] * ld);
        const floatx4 v = *reinterpret_cast<const floatx4*>(q);
        r[b] = in ? v : z;
        p[b] += KC ? BK : BK * ld;
      }
    }
  }
  // split + write the half tile into the three planes of one operand image (plane stride TILE * BK)
  __device__ __forceinline__ void store(__bf16* __restrict__ lds, int t, int half) const { store_from(r, lds, t, half); }
  __device__ __forceinline__ void store_from(const floatx4 (&r)[NB], __bf16* __restrict__ lds, int t, int half) const {
    constexpr int PL = TILE * BK;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int idx = t + NTG * b;
      int off;
      if constexpr (KC) {
        const int row = half * HT + idx / (BK / 4), q = idx % (BK / 4);
        off = slot_off<BK>(row, q >> 1) + 4 * (q & 1);
      } else {
        const int c4 = half * (HT / 4) + idx % (HT / 4), kr = idx / (HT / 4);
        off = mn_off<TILE>(kr, c4 >> 1) + 4 * (c4 & 1);
      }
      u32x2v h, m, l;
      split4(r[b], h, m, l);
      *reinterpret_cast<u32x2v*>(lds + off) = h;
      *reinterpret_cast<u32x2v*>(lds + PL + off) = m;
      *reinterpret_cast<u32x2v*>(lds + 2 * PL + off) = l;
    }
  }
};

// s_waitcnt lgkmcnt(0) (vmcnt / expcnt left at their maxima) + s_barrier, pinned in program order
__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// lab-only issue priority variants of the ping-pong phases (scripts/lab/lab_build.sh -D...): the M-phase wave
// ahead of its MFMA partner for VALU / LDS issue (K3M_LAB_PP_PRIO), or waves 4-7 statically ahead
// (K3M_LAB_PP_PRIO_LATE, MI355X_MICROARCH.md "Two waves per SIMD" item 4)
__device__ __forceinline__ void pp_prio_m() {
#ifdef K3M_LAB_PP_PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
}
__device__ __forceinline__ void pp_prio_c() {
#ifdef K3M_LAB_PP_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_>
struct PPLoop {
  static_assert(WM * WN == 8, "ping-pong pairs waves w and w + 4 of an 8-wave workgroup");
  static constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32, KS = BK / 16;
  static constexpr int BUF = 3 * (TBM + TBN) * BK;
  static constexpr int PA = TBM * BK, PB = TBN * BK;
  PPHalf<AK, TBM, BK> ha;
  PPHalf<BK_, TBN, BK> hb;
  long long lda, ldb;
  int nt, krem;   // k-tiles (the last one partial when krem > 0), k values of the partial tile

  __device__ __forceinline__ int tile_k(int t) const { return (krem > 0 && t == nt - 1) ? krem : BK; }

  __device__ __forceinline__ void prefetch(const K3mGemm& g, const Unit& u) {
    const int t = threadIdx.x & 255, half = threadIdx.x >> 8;
    lda = g.lda;
    ldb = g.ldb;
    ha.init(static_cast<const float*>(g.a), lda, u.m0, u.kbeg, g.m, t, half);
    hb.init(static_cast<const float*>(g.b), ldb, u.n0, u.kbeg, g.n, t, half);
    const int klen = u.kend - u.kbeg;
    const int nkf = klen > 0 ? klen / BK : 0;
    krem = klen > 0 ? klen - nkf * BK : 0;
    nt = nkf + (krem > 0 ? 1 : 0);
    if (nt > 0) {
      const int kk = tile_k(0);
      ha.load(lda, kk);
      hb.load(ldb, kk);
    }
  }
  __device__ __forceinline__ void prefetch2() {}

  __device__ __forceinline__ void frags(const __bf16* stage, bf16x8 (&a)[KS][3][FM], bf16x8 (&b)[KS][3][FN]) const {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
    const int h = lane >> 5, cl = lane & 31;
    const __bf16* as = stage;
    const __bf16* bs = as + 3 * PA;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[ks][pl][i] = AK ? *reinterpret_cast<const bf16x8*>(as + pl * PA + slot_off<BK>(wm + 32 * i + cl, 2 * ks + h))
                            : mn_frag<TBM>(as + pl * PA, wm + 32 * i, ks, lane);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[ks][pl][j] = BK_ ? *reinterpret_cast<const bf16x8*>(bs + pl * PB + slot_off<BK>(wn + 32 * j + cl, 2 * ks + h))
                             : mn_frag<TBN>(bs + pl * PB, wn + 32 * j, ks, lane);
      }
  }

  __device__ __forceinline__ static void mfma(const bf16x8 (&a)[KS][3][FM], const bf16x8 (&b)[KS][3][FN],
                                              floatx16 (&acc)[FM][FN]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          // smallest terms first: (hl + mm + lh), (hm + mh), hh -- the order of Loop::compute
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0][i], b[ks][2][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1][i], b[ks][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][2][i], b[ks][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0][i], b[ks][1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][1][i], b[ks][0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][0][i], b[ks][0][j], acc[i][j], 0, 0, 0);
        }
  }

  __device__ __forceinline__ void stage_half(__bf16* stage) const {
    const int t = threadIdx.x & 255, half = threadIdx.x >> 8;
    ha.store(stage, t, half);
    hb.store(stage + 3 * PA, t, half);
  }

  // Same contract as Loop::run.
  __device__ __forceinline__ void run(__bf16* smem, floatx16 (&acc)[FM][FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const bool late = threadIdx.x >= 256;   // waves 4-7
    if (nt > 0) {
      stage_half(smem);
      if (nt > 1) {
        const int kk = tile_k(1);
        ha.load(lda, kk);
        hb.load(ldb, kk);
      }
    }
    pp_barrier();
    if (late) pp_barrier();
#ifdef K3M_LAB_PP_PRIO_LATE
    if (late) __builtin_amdgcn_s_setprio(1);
#endif
    for (int kt = 0; kt < nt; ++kt) {
      const int cur = kt & 1;
      bf16x8 a[KS][3][FM], b[KS][3][FN];
      pp_prio_m();
      frags(smem + cur * BUF, a, b);
      if (kt + 1 < nt) {
        stage_half(smem + (cur ^ 1) * BUF);
        if (kt + 2 < nt) {
          const int kk = tile_k(kt + 2);
          ha.load(lda, kk);
          hb.load(ldb, kk);
        }
      }
      pp_barrier();
      pp_prio_c();
      mfma(a, b, acc);
      pp_barrier();
    }
#if defined(K3M_LAB_PP_PRIO) || defined(K3M_LAB_PP_PRIO_LATE)
    __builtin_amdgcn_s_setprio(0);
#endif
    if (!late) pp_barrier();
  }
};

// Ping-pong loop with LDS-DMA staging of the raw fp32 k-tiles (PP = 2, the 256x256 weight-gradient walk).
// That walk streams both operands from HBM (K = 20,992 split 7-14 ways); PPLoop gives each register-staged
// load two phases to land and its waves then wait (profiles/r5d/pmc_wgrad_ffn1_pingpong.json: MFMA busy 0.40, 57 % of
// wave cycles parked in s_waitcnt).  Here every thread DMAs the float4s it will split (global_load_lds_dwordx4,
// lane-linear 1 KiB per wave instruction) into one of two raw fp32 buffers behind the x6 stages (2 x 32 KiB;
// 96 + 64 = 160 KiB of LDS), and reads them back itself: no barrier orders the raw buffers, only the issuing
// wave's counted vmcnt.  M(t) splits k-tile t+1 from its raw buffer, then DMAs k-tile t+3 into the same
// buffer: each DMA has two whole iterations to land, with no staging registers.  k-tile 0 still goes
// through registers (loaded inside the previous tile's epilogue, as PPLoop).
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_>
struct PPDLoop : PPLoop<TBM, TBN, WM, WN, BK, AK, BK_> {
  using Base = PPLoop<TBM, TBN, WM, WN, BK, AK, BK_>;
  using Base::ha;
  using Base::hb;
  using Base::lda;
  using Base::ldb;
  using Base::nt;
  using Base::krem;
  static constexpr int BUF = Base::BUF, PA = Base::PA, FM = Base::FM, FN = Base::FN, KS = Base::KS;
  static constexpr int NBA = PPHalf<AK, TBM, BK>::NB, NBB = PPHalf<BK_, TBN, BK>::NB, ND = NBA + NBB;
  static constexpr int RAW_FLOATS = 512 * 4 * ND;          // one raw k-tile: ND float4 per thread
  static constexpr int RAW_OFF_BF16 = 2 * BUF;             // raw buffers start after the two x6 stages

  // DMA this thread's float4s of the next k-tile into raw buffer rb and advance the pointers; lanes of a
  // partial tile past krem read the tile's first k (valid) and are zeroed when split
  // One LDS-DMA wave instruction as inline asm: issued through the builtin, the compiler's waitcnt pass
  // (which cannot tell the raw buffers from the x6 stages) puts a vmcnt(0) before every later LDS read,
  // i.e. waits for the DMAs still meant to be in flight.  Hidden from it, the DMAs are ordered only by
  // the counted vmcnt waits of run() (the compiler's own vmcnt counts for register loads stay
  // conservative: it sees fewer younger VMEM operations than there are).
  __device__ __forceinline__ static void dma16(const float* g, const float* lds) {
    // M0 = the wave-uniform LDS destination, written by the compiler through the "{m0}" operand (a clobbered
    // M0 would be a reserved-register clobber); s_nop 0: the M0 write -> LDS-DMA hazard
    const uint32_t m0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)lds;
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(__builtin_amdgcn_readfirstlane(m0))
                 : "memory");
  }
  template <bool KC, int TILE>
  __device__ __forceinline__ static void dma(PPHalf<KC, TILE, BK>& h, float* raw, int slot0, long long ld) {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int b = 0; b < PPHalf<KC, TILE, BK>::NB; ++b) {
      dma16(h.p[b], raw + ((slot0 + b) * 512 + w * 64) * 4);   // wave-uniform: lane l lands at + 4 l floats
      h.p[b] += KC ? BK : BK * ld;
    }
  }
  __device__ __forceinline__ void dma_tile(float* raw, int kk) {
    // the partial tile: clamp the lanes past kk to the tile's first k (the pointers are restored after)
    if (kk < BK) {
#pragma unroll
      for (int b = 0; b < NBA; ++b)
        if (ha.kq[b] >= kk) ha.p[b] -= AK ? ha.kq[b] : (long long)ha.kq[b] * lda;
#pragma unroll
      for (int b = 0; b < NBB; ++b)
        if (hb.kq[b] >= kk) hb.p[b] -= BK_ ? hb.kq[b] : (long long)hb.kq[b] * ldb;
    }
    dma<AK, TBM>(ha, raw, 0, lda);
    dma<BK_, TBN>(hb, raw, NBA, ldb);
  }
  // read back this thread's float4s of one raw k-tile, one operand's reads issued together (a serial
  // read -> split -> read chain costs one LDS round trip per float4; all four at once spill), zero a partial
  // tile's lanes past kk, split and write both operands' halves into the x6 stage
  __device__ __forceinline__ void split_raw(const float* raw, __bf16* stage, int kk) const {
    const int tid = threadIdx.x, t = tid & 255, half = tid >> 8;
    const floatx4 z = {0.f, 0.f, 0.f, 0.f};
    floatx4 ra[NBA];
#pragma unroll
    for (int b = 0; b < NBA; ++b) ra[b] = *reinterpret_cast<const floatx4*>(raw + (b * 512 + tid) * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NBA; ++b) ra[b] = ha.kq[b] < kk ? ra[b] : z;
    ha.store_from(ra, stage, t, half);
    floatx4 rb[NBB];
#pragma unroll
    for (int b = 0; b < NBB; ++b) rb[b] = *reinterpret_cast<const floatx4*>(raw + ((NBA + b) * 512 + tid) * 4);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int b = 0; b < NBB; ++b) rb[b] = hb.kq[b] < kk ? rb[b] : z;
    hb.store_from(rb, stage + 3 * PA, t, half);
  }

  __device__ __forceinline__ void run(__bf16* smem, floatx16 (&acc)[FM][FN]) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const bool late = threadIdx.x >= 256;
    float* raw0 = reinterpret_cast<float*>(smem + RAW_OFF_BF16);
    auto rawbuf = [&](int t) { return raw0 + (t & 1) * RAW_FLOATS; };
    if (nt > 0) this->stage_half(smem);                  // k-tile 0 from registers
    if (nt > 1) dma_tile(rawbuf(1), this->tile_k(1));
    if (nt > 2) dma_tile(rawbuf(2), this->tile_k(2));
    pp_barrier();
    if (late) pp_barrier();
#pragma nounroll
    for (int kt = 0; kt < nt; ++kt) {
      const int cur = kt & 1;
      bf16x8 a[KS][3][FM], b[KS][3][FN];
      this->frags(smem + cur * BUF, a, b);
      if (kt + 1 < nt) {
        __builtin_amdgcn_sched_barrier(0);
        // gfx9 s_waitcnt simm16: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt[5:4] << 14
        static_assert(ND < 16, "vmcnt immediate");
        if (kt + 2 < nt) __builtin_amdgcn_s_waitcnt(0x0F70 | ND);   // vmcnt(ND): k-tile t+2's DMAs may fly on
        else __builtin_amdgcn_s_waitcnt(0x0F70);                    // vmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
        const int kk = this->tile_k(kt + 1);
        __bf16* st = smem + (cur ^ 1) * BUF;
        split_raw(rawbuf(kt + 1), st, kk);
        if (kt + 3 < nt) {
          __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's reads of the raw buffer are back
          __builtin_amdgcn_sched_barrier(0);
          dma_tile(rawbuf(kt + 3), this->tile_k(kt + 3));
        }
      }
      pp_barrier();
      Base::mfma(a, b, acc);
      pp_barrier();
    }
    if (!late) pp_barrier();
  }
};

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE, int PP>
struct LoopSel {
  using T = Loop<TBM, TBN, WM, WN, BK, AK, BK_, PIPE>;
};
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE>
struct LoopSel<TBM, TBN, WM, WN, BK, AK, BK_, PIPE, 1> {
  using T = PPLoop<TBM, TBN, WM, WN, BK, AK, BK_>;
};
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE>
struct LoopSel<TBM, TBN, WM, WN, BK, AK, BK_, PIPE, 2> {
  using T = PPDLoop<TBM, TBN, WM, WN, BK, AK, BK_>;
};

// PP: 0 the compiler-scheduled loop (Loop), 1 the ping-pong loop (PPLoop), 2 with LDS-DMA staging (PPDLoop)
template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, int EPI, bool PIPE, int PP = 0>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_x6_persist_kernel(GemmGroup grp) {
  constexpr int LDS_BF16 = 2 * 3 * (TBM + TBN) * BK;
  constexpr int EPI_F32 = WM * WN * 32 * (TBN / WN + 8);
  constexpr int RAW = PP == 2 ? 2 * PPDLoop<TBM, TBN, WM, WN, BK, AK, BK_>::RAW_FLOATS : 0;
  constexpr int WORDS = (LDS_BF16 / 2 + RAW > EPI_F32 ? LDS_BF16 / 2 + RAW : EPI_F32);
  __shared__ __attribute__((aligned(16))) float smem[WORDS];
  const int total = grp.start[grp.count];
  int u = blockIdx.x;
  if (u >= total) return;
  typename LoopSel<TBM, TBN, WM, WN, BK, AK, BK_, PIPE, PP>::T lp;
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

template <int TBM, int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE, int PP = 0>
int launch(const GemmGroup& grp, int epi, int nblk, hipStream_t st) {
  const dim3 grid(nblk);
  switch (epi) {
#define K3M_P_CASE(E)                                                                                       \
    case E:                                                                                                 \
      hipLaunchKernelGGL((gemm_x6_persist_kernel<TBM, TBN, WM, WN, BK, AK, BK_, E, PIPE, PP>), grid,        \
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

// K3M_X6_PP: ping-pong main loops per operand-layout class, bitmask: 1 forward (both K-contiguous), 2 input
// gradient (B MN-contiguous), 4 weight gradient (both MN-contiguous), 8 A MN-contiguous / B K-contiguous;
// 16 = the 256x128 tiles too; 32 = the 256x256 weight-gradient walk too, on the LDS-DMA-staged PPDLoop;
// 64 = the 256x256 forward / input-gradient walks on PPDLoop as well (A/B only).  Default 63, each part
// measured same box, interleaved (profiles/r5d/README.txt): PPLoop on the K-contiguous 256x256 forwards / input
// gradients 4-7 % faster than the compiler-scheduled walk, on the 256x128 and image / co-attention shapes
// 5-15 %; the 256x256 weight gradients 22-27 % SLOWER on PPLoop (HBM-streamed operands, loads with two phases to
// land) and 1-3 % faster on PPDLoop; PPDLoop on the forwards 3-4 % slower than PPLoop.  Config 2: walk 527 ->
// PPLoop 541 -> + PPDLoop weight gradients 542 samples/s.
const int kPP = k3m_env_int("K3M_X6_PP", 63);

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
  const int cls = ak && bk ? 1 : ak ? 2 : !bk ? 4 : 8;
  const bool pp = (kPP & cls) != 0 && (t256 ? (cls != 4 || (kPP & 32) != 0) : (kPP & 16) != 0);
  if (t256) {
    if (ak && bk) return !pp ? launch<256, 256, 4, 2, 16, true, true, true>(grp, epi, nblk, st)
                      : (kPP & 64) ? launch<256, 256, 4, 2, 16, true, true, true, 2>(grp, epi, nblk, st)
                                   : launch<256, 256, 4, 2, 16, true, true, true, 1>(grp, epi, nblk, st);
    if (ak) return !pp ? launch<256, 256, 2, 4, 16, true, false, true>(grp, epi, nblk, st)
                : (kPP & 64) ? launch<256, 256, 2, 4, 16, true, false, true, 2>(grp, epi, nblk, st)
                             : launch<256, 256, 2, 4, 16, true, false, true, 1>(grp, epi, nblk, st);
    if (!bk) return pp ? launch<256, 256, 2, 4, 16, false, false, false, 2>(grp, epi, nblk, st)
                       : launch<256, 256, 2, 4, 16, false, false, false>(grp, epi, nblk, st);
    return K3M_EINVAL;
  }
  if (ak && bk) return pp ? launch<256, 128, 4, 2, 32, true, true, true, 1>(grp, epi, nblk, st)
                          : launch<256, 128, 4, 2, 32, true, true, true>(grp, epi, nblk, st);
  if (ak) return pp ? launch<256, 128, 4, 2, 32, true, false, true, 1>(grp, epi, nblk, st)
                    : launch<256, 128, 4, 2, 32, true, false, true>(grp, epi, nblk, st);
  if (bk) return pp ? launch<256, 128, 4, 2, 32, false, true, true, 1>(grp, epi, nblk, st)
                    : launch<256, 128, 4, 2, 32, false, true, true>(grp, epi, nblk, st);
  return pp ? launch<256, 128, 4, 2, 32, false, false, false, 1>(grp, epi, nblk, st)
            : launch<256, 128, 4, 2, 32, false, false, false>(grp, epi, nblk, st);
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
