// fp32 MFMA GEMM main body for gfx950 (v_mfma_f32_32x32x2_f32: exact f32, 157 TF/s peak).
//
// Block tile TBM x TBN x 32, WM x WN waves, each wave owning (TBM/WM) x (TBN/WN) = FM x FN MFMA
// tiles of 32x32.
//
// LDS image.  Both operands are staged into the SAME k-contiguous image [TILE][32] fp32 (128-B
// rows), with the 16-B chunk c of row r stored at slot c ^ ((r >> 1) & 7).  The K order inside a
// 32-deep tile is permuted so that lane l (row l&31, half h = l>>5) consumes k = 16h + 4j + q at
// MFMA step (j, q): one ds_read_b128 feeds four MFMAs (4 reads per 32x32 operand per k-tile instead
// of 16 ds_read_b32), and with the XOR swizzle each 16-lane read group covers all 64 banks once
// (conflict-free).  A and B use the same permutation, so the sum over k is unchanged (the fp32
// rounding order differs from a sequential chain, as it does for any blocked GEMM).
//
// Staging (register double buffer, one barrier per k-tile):
//   * K-contiguous operand (activations; torch Linear weights for x.W^T): 8 lanes per 128-B row,
//     one ds_write_b128 per float4;
//   * MN-contiguous operand (W for input gradients; dY^T and X for weight gradients): each thread
//     loads a 4(k) x 4(mn) block as four float4 row pieces and writes it transposed (four float4
//     k-runs) into the same image.
#pragma once
#include "common.h"

#include <type_traits>

#ifndef K3M_EPI_RING
#define K3M_EPI_RING 1
#endif

// The lab (scripts/lab) compiles these templates into its own executable under other namespace
// names: kernels with the same mangled name as libk3m_hip.so's would resolve to the library's code.
#ifndef K3M_F32_NS
#define K3M_F32_NS k3m_f32
#endif

namespace K3M_F32_NS {

constexpr int BK = 32;

__device__ __forceinline__ int swz(int r, int c) { return r * BK + ((c ^ ((r >> 1) & 7)) << 2); }

template <bool KC, int TILE, int NT>
struct Stage {
  // KC: TILE*8 float4 per tile; MN: 2*TILE blocks of 4x4 (4 float4 each)
  static constexpr int NB = KC ? (TILE * 8 + NT - 1) / NT : (2 * TILE + NT - 1) / NT;
  static constexpr int NR = KC ? NB : 4 * NB;
  floatx4 r[NR];
};

template <bool KC, bool VEC, int TILE, int NT>
__device__ __forceinline__ void load_tile(const float* __restrict__ p, long long ld, int mn0, int k0, int MN, int K,
                                          Stage<KC, TILE, NT>& s) {
  const int t = threadIdx.x;
  if constexpr (KC) {
#pragma unroll
    for (int it = 0; it < Stage<KC, TILE, NT>::NB; ++it) {
      const int idx = t + NT * it;
      if ((TILE * 8) % NT != 0 && idx >= TILE * 8) break;
      const int row = idx >> 3, c = idx & 7;
      const int gm = mn0 + row, gk = k0 + 4 * c;
      if constexpr (VEC) {
        s.r[it] = (gm < MN && gk < K) ? *reinterpret_cast<const floatx4*>(p + (long long)gm * ld + gk)
                                      : floatx4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) s.r[it][q] = (gm < MN && gk + q < K) ? p[(long long)gm * ld + gk + q] : 0.f;
      }
    }
  } else {
    constexpr int Q = TILE / 4;  // 4-wide mn groups per k row
#pragma unroll
    for (int b = 0; b < Stage<KC, TILE, NT>::NB; ++b) {
      const int idx = t + NT * b;
      if ((2 * TILE) % NT != 0 && idx >= 2 * TILE) break;
      const int q = idx % Q, g4 = idx / Q;
      const int gm = mn0 + 4 * q;
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

template <bool KC, int TILE, int NT>
__device__ __forceinline__ void store_tile(float* __restrict__ lds, const Stage<KC, TILE, NT>& s) {
  const int t = threadIdx.x;
  if constexpr (KC) {
#pragma unroll
    for (int it = 0; it < Stage<KC, TILE, NT>::NB; ++it) {
      const int idx = t + NT * it;
      if ((TILE * 8) % NT != 0 && idx >= TILE * 8) break;
      *reinterpret_cast<floatx4*>(lds + swz(idx >> 3, idx & 7)) = s.r[it];
    }
  } else {
    constexpr int Q = TILE / 4;
#pragma unroll
    for (int b = 0; b < Stage<KC, TILE, NT>::NB; ++b) {
      const int idx = t + NT * b;
      if ((2 * TILE) % NT != 0 && idx >= 2 * TILE) break;
      const int q = idx % Q, g4 = idx / Q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const floatx4 v = {s.r[4 * b][e], s.r[4 * b + 1][e], s.r[4 * b + 2][e], s.r[4 * b + 3][e]};
        *reinterpret_cast<floatx4*>(lds + swz(4 * q + e, g4)) = v;
      }
    }
  }
}

__device__ __forceinline__ int xcd_remap(int id, int nblk) {
  // bijective: blocks dispatched round-robin over 8 XCDs -> contiguous id ranges per XCD
  const int xcd = id & 7, q = nblk >> 3, rr = nblk & 7;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + (id >> 3);
}

// Block-tile coordinates: XCD remap, then GROUP rows of tiles walk N together (L2 reuse of the
// A panel inside one XCD).
template <int GROUP = 8>
__device__ __forceinline__ void tile_coords(int M, int N, int TBM, int TBN, int& m0, int& n0) {
  const int tm = (M + TBM - 1) / TBM, tn = (N + TBN - 1) / TBN;
  const int id = xcd_remap(blockIdx.x, tm * tn);
  const int group_sz = GROUP * tn;
  const int first_m = (id / group_sz) * GROUP;
  const int gm_sz = min(tm - first_m, GROUP);
  m0 = (first_m + (id % group_sz) % gm_sz) * TBM;
  n0 = ((id % group_sz) / gm_sz) * TBN;
}

// Main loop: acc[i][j] (+)= A[m0 + wm + 32i .., kbeg:kend] . B[n0 + wn + 32j .., kbeg:kend]^T.
// smem: 2 stages of (TBM + TBN) * BK floats.
template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, bool VEC>
__device__ __forceinline__ void mainloop(const float* __restrict__ A, long long lda, const float* __restrict__ B,
                                         long long ldb, int M, int N, int m0, int n0, int kbeg, int kend,
                                         float* smem, floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32]) {
  constexpr int NT = 64 * WM * WN;
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int BUF = (TBM + TBN) * BK;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  Stage<AK, TBM, NT> ra;
  Stage<BK_, TBN, NT> rb;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile<AK, VEC, TBM, NT>(A, lda, m0, kbeg, M, kend, ra);
    load_tile<BK_, VEC, TBN, NT>(B, ldb, n0, kbeg, N, kend, rb);
    store_tile<AK, TBM, NT>(smem, ra);
    store_tile<BK_, TBN, NT>(smem + TBM * BK, rb);
  }
  __syncthreads();
  const int h = lane >> 5, cl = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<AK, VEC, TBM, NT>(A, lda, m0, k0, M, kend, ra);
      load_tile<BK_, VEC, TBN, NT>(B, ldb, n0, k0, N, kend, rb);
    }
    const float* as = smem + cur * BUF;
    const float* bs = as + TBM * BK;
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4) {
      floatx4 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r = wm + 32 * i + cl;
        a[i] = *reinterpret_cast<const floatx4*>(as + swz(r, 4 * h + j4));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int r = wn + 32 * j + cl;
        b[j] = *reinterpret_cast<const floatx4*>(bs + swz(r, 4 * h + j4));
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<AK, TBM, NT>(smem + (cur ^ 1) * BUF, ra);
      store_tile<BK_, TBN, NT>(smem + (cur ^ 1) * BUF + TBM * BK, rb);
    }
    __syncthreads();
  }
}

}  // namespace K3M_F32_NS

namespace K3M_F32_NS {

// Epilogue, staged through LDS (free after the main loop's last barrier) so that global traffic is
// row-contiguous 16-B vectors: each wave writes one 32-row slice of its accumulators into a private
// [32][FN*32 + 8] region (the two half-waves' rows land 32 banks apart), reads it back 8
// consecutive columns per lane and applies the epilogue on the way out.
// acc[i][j][r] holds row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31 of MFMA tile (i, j).
// Split-K (splitk > 1): the block's slab ws[blockIdx.y] gets the raw sum (alpha/beta are applied
// by the reduction kernel).
struct NoHook {
  __device__ __forceinline__ void operator()() const {}
};

// hook(): called once, after the first accumulator slice is in LDS and before any global store (the
// persistent x6 kernel issues the next tile's loads there, when acc[0] is dead and the loads are
// older than every store of this tile).
// The epilogue reads the accumulators through a stager: stage(i, wl, ws, lane) writes the wave's
// 32-row group i into its [32][ws] fp32 LDS region (row-major, column 0 = the wave's first column).
template <int FM, int FN>
struct Acc32Ref {   // v_mfma_f32_32x32x*: acc[i][j][r] = row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31
  const floatx16 (&a)[FM][FN];
  __device__ __forceinline__ void stage(int i, float* wl, int ws, int lane) const {
    const int kl = lane >> 5, cl = lane & 31;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) wl[((r & 3) + 8 * (r >> 2) + 4 * kl) * ws + 32 * j + cl] = a[i][j][r];
  }
};

__device__ __forceinline__ void ld8(const float* p, float (&v)[8]) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p), b = *reinterpret_cast<const floatx4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}
__device__ __forceinline__ void st8(float* p, const float (&v)[8]) {
#ifdef K3M_LAB_NO_STORE   // lab only (scripts/lab/lab_build.sh): timing without the epilogue's stores, math kept
#pragma unroll
  for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(v[e]));
  return;
#endif
#ifdef K3M_LAB_NT_STORE   // lab (scripts/lab/lab_build.sh): streaming stores, no dirty L2 lines left at the kernel's end
  __builtin_nontemporal_store(floatx4{v[0], v[1], v[2], v[3]}, reinterpret_cast<floatx4*>(p));
  __builtin_nontemporal_store(floatx4{v[4], v[5], v[6], v[7]}, reinterpret_cast<floatx4*>(p + 4));
#else
  *reinterpret_cast<floatx4*>(p) = floatx4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<floatx4*>(p + 4) = floatx4{v[4], v[5], v[6], v[7]};
#endif
}

template <int EPI>
__device__ __forceinline__ void epi_math(const float (&v)[8], const float (&bb)[8], const float (&ax)[8],
                                         const float (&old)[8], float alpha, float beta, bool rd_old, float (&o)[8],
                                         float (&pa)[8]) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if constexpr (EPI == K3M_EPI_NONE) {
      o[e] = alpha * v[e];
    } else if constexpr (EPI == K3M_EPI_BIAS) {
      o[e] = alpha * (v[e] + bb[e]);
    } else if constexpr (EPI == K3M_EPI_BIAS_GELU) {
      pa[e] = v[e] + bb[e];
      o[e] = gelu_f(pa[e]);
    } else if constexpr (EPI == K3M_EPI_DGELU) {
      o[e] = alpha * v[e] * dgelu_f(ax[e]);
    } else {
      o[e] = sigmoid_f(v[e] + bb[e]);
    }
    if (rd_old) o[e] += beta * old[e];
  }
}

// K3M_GEMM_COLSUM_SLABS: column sums of one 32-row group of C.  Lanes sharing columns (lane % LPR) are
// reduced over the row lanes by XOR shuffles; lanes 0..LPR-1 write the group's slab row ws[slab][col..col+7].
template <int LPR>
__device__ __forceinline__ void colsum_flush(float (&cs)[8], float* ws, int slab, int N, int col, int lane,
                                             bool live) {
#pragma unroll
  for (int off = LPR; off < 64; off <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] += __shfl_xor(cs[e], off, 64);
  if (live && lane < LPR && col < N) {
    float* p = ws + (long long)slab * N + col;
    if (col + 8 <= N && (N & 3) == 0) {
      *reinterpret_cast<floatx4*>(p) = floatx4{cs[0], cs[1], cs[2], cs[3]};
      *reinterpret_cast<floatx4*>(p + 4) = floatx4{cs[4], cs[5], cs[6], cs[7]};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (col + e < N) p[e] = cs[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = 0.f;
}

// Global traffic of the epilogue is kept out of its own way.  vmcnt counts loads AND stores in issue
// order, so a load issued after a store cannot be waited for without waiting for that store: a
// per-pass bias load drained every store of the previous pass before the next pass could compute
// (one `s_waitcnt vmcnt(0)` per pass in the ISA, profiles/r3_epilogue_vmcnt.txt).  So (1) the lane's
// 8 bias values (its columns are the same in every pass) are loaded once and waited for before the
// first store; (2) interior tiles (inside C, 16-B aligned rows) run a branch-free pass sequence whose
// per-pass loads (dGELU pre-activation, old C for beta != 0) are issued RING passes ahead, so waiting
// for them retires only the stores of passes RING or more back.
template <int TBM, int TBN, int WM, int WN, int EPI, int CAP, class Hook, class AccR, bool FAST = true>
__device__ __forceinline__ void epilogue_r(const K3mGemm& g, int m0, int n0, float* smem, const AccR& acc, int slice,
                                           Hook hook) {
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int WCOLS = FN * 32, WS = WCOLS + 8, LPR = WCOLS / 8, RPP = 64 / LPR, NPS = 32 / RPP;
  static_assert(WM * WN * 32 * WS <= CAP, "epilogue staging exceeds the LDS tile");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  const int M = g.m, N = g.n;
  float* wl = smem + w * 32 * WS;
  const bool split = g.splitk > 1;
  float* C = split ? g.ws + (long long)(slice >= 0 ? slice : (int)blockIdx.y) * M * N : static_cast<float*>(g.c);
  const long long ldc = split ? N : g.ldc;
  const float alpha = split ? 1.f : g.alpha, beta = split ? 0.f : g.beta;
  float* aux = static_cast<float*>(g.aux);
  const float* bias = g.bias;
  constexpr bool HAS_AUX = EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_DGELU;
  constexpr bool HAS_BIAS = EPI == K3M_EPI_BIAS || EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_BIAS_SIGMOID;
  constexpr bool CAN_OLD = EPI == K3M_EPI_NONE || EPI == K3M_EPI_BIAS || EPI == K3M_EPI_DGELU;
  const bool cvec = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                    (!HAS_AUX || ((g.ldaux % 4 == 0) && ((reinterpret_cast<uintptr_t>(aux) & 15) == 0)));
  const bool rd_old = CAN_OLD && beta != 0.f;
  const bool bvec = HAS_BIAS && ((reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  const int lr = lane / LPR, lc = (lane % LPR) * 8;
  const int col = n0 + wn + lc;
  float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (HAS_BIAS) {
    if (bvec && col + 8 <= N) {
      ld8(bias + col, bb);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = col + e < N ? bias[col + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) asm volatile("" ::"v"(bb[e]));   // waited for here, before any store
  }
  auto row_of = [&](int i, int ps) { return m0 + wm + 32 * i + ps * RPP + lr; };
  // the dGELU input gradient can also leave the column sums of its output (the bias gradient of the Linear
  // it feeds, K3M_GEMM_COLSUM_SLABS: ws = [ceil(m/32)][n] slabs, one per 32-row group; k3m_gemm passes ws
  // only when the flag is set)
  constexpr bool CSUM = EPI == K3M_EPI_DGELU;
  float* const cws = (CSUM && !split) ? g.ws : nullptr;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // passes the per-pass loads run ahead (their registers: RING x 8 floats per load stream)
  constexpr int RING = K3M_EPI_RING;
  const bool interior = FAST && cvec && m0 + TBM <= M && n0 + TBN <= N;
  if constexpr (FAST) if (interior) {
    auto body = [&](auto old_tag) {
      constexpr bool OLD = decltype(old_tag)::value;
      constexpr bool LOADS = OLD || EPI == K3M_EPI_DGELU;
      constexpr int NQ = FM * NPS;
      float rax[RING][8], rold[RING][8];
      auto issue = [&](int q, int slot) {
        if constexpr (LOADS) {
          const long long r = row_of(q / NPS, q % NPS);
          if constexpr (EPI == K3M_EPI_DGELU) ld8(aux + r * g.ldaux + col, rax[slot]);
          if constexpr (OLD) ld8(C + r * ldc + col, rold[slot]);
        }
      };
#pragma unroll
      for (int q = 0; q < RING; ++q)
        if (q < NQ) issue(q, q);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc.stage(i, wl, WS, lane);
        __syncthreads();
        if (i == 0) hook();
#pragma unroll
        for (int ps = 0; ps < NPS; ++ps) {
          const int q = i * NPS + ps, slot = q % RING;
          const int rr = ps * RPP + lr;
          const long long row = row_of(i, ps);
          const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
          const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
          const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          float ax[8], old[8], o[8], pa[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            ax[e] = LOADS && EPI == K3M_EPI_DGELU ? rax[slot][e] : 0.f;
            old[e] = OLD ? rold[slot][e] : 0.f;
          }
          if (q + RING < NQ) issue(q + RING, slot);
          epi_math<EPI>(v, bb, ax, old, alpha, beta, OLD, o, pa);
          st8(C + row * ldc + col, o);
          if constexpr (EPI == K3M_EPI_BIAS_GELU) st8(aux + row * g.ldaux + col, pa);
          if constexpr (CSUM) {
            if (cws)
#pragma unroll
              for (int e = 0; e < 8; ++e) cs[e] += o[e];
          }
        }
        if constexpr (CSUM) {
          if (cws) colsum_flush<LPR>(cs, cws, (m0 + wm + 32 * i) >> 5, N, col, lane, true);
        }
        __syncthreads();
      }
    };
    if (rd_old) body(std::integral_constant<bool, true>());
    else body(std::integral_constant<bool, false>());
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    acc.stage(i, wl, WS, lane);
    __syncthreads();
    if (i == 0) hook();
    // edge tiles only: a rolled pass loop keeps this path's code (and its registers) small
#pragma unroll 1
    for (int ps = 0; ps < NPS; ++ps) {
      const int rr = ps * RPP + lr;
      const int row = row_of(i, ps);
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
      if (row >= M || col >= N) continue;
      const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const bool full = cvec && col + 8 <= N;
      float* cp = C + (long long)row * ldc + col;
      float* ap = HAS_AUX ? aux + (long long)row * g.ldaux + col : nullptr;
      float old[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, ax[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == K3M_EPI_DGELU) {
        if (full) ld8(ap, ax);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) ax[e] = col + e < N ? ap[e] : 0.f;
      }
      if (rd_old) {
        if (full) ld8(cp, old);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = col + e < N ? cp[e] : 0.f;
      }
      float o[8], pa[8];
      epi_math<EPI>(v, bb, ax, old, alpha, beta, rd_old, o, pa);
      if constexpr (CSUM) {
        if (cws)
#pragma unroll
          for (int e = 0; e < 8; ++e) cs[e] += col + e < N ? o[e] : 0.f;
      }
      if (full) {
        st8(cp, o);
        if constexpr (EPI == K3M_EPI_BIAS_GELU) st8(ap, pa);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < N) {
            cp[e] = o[e];
            if constexpr (EPI == K3M_EPI_BIAS_GELU) ap[e] = pa[e];
          }
      }
    }
    if constexpr (CSUM) {
      if (cws) colsum_flush<LPR>(cs, cws, (m0 + wm + 32 * i) >> 5, N, col, lane, m0 + wm + 32 * i < M);
    }
    __syncthreads();
  }
}

// FAST = false: no separate branch-free interior path (kernels already at their register limit, where the
// second copy of the pass sequence made the main loop spill: the 256x256 input-gradient walk)
template <int TBM, int TBN, int WM, int WN, int EPI, int CAP = 2 * (TBM + TBN) * BK, class Hook = NoHook,
          bool FAST = true>
__device__ __forceinline__ void epilogue(const K3mGemm& g, int m0, int n0, float* smem,
                                         const floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32], int slice = -1,
                                         Hook hook = Hook()) {
  const Acc32Ref<TBM / WM / 32, TBN / WN / 32> r{acc};
  epilogue_r<TBM, TBN, WM, WN, EPI, CAP, Hook, Acc32Ref<TBM / WM / 32, TBN / WN / 32>, FAST>(g, m0, n0, smem, r, slice,
                                                                                              hook);
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, bool VEC, int EPI, int OCC>
__global__ __launch_bounds__(64 * WM * WN, OCC) void gemm_f32_kernel(K3mGemm g) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (TBM + TBN) * BK];
  int m0, n0;
  tile_coords(g.m, g.n, TBM, TBN, m0, n0);
  int kbeg = 0, kend = g.k;
  if (g.splitk > 1) {
    const int per = ((g.k + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = blockIdx.y * per;
    kend = min(g.k, kbeg + per);
  }
  floatx16 acc[TBM / WM / 32][TBN / WN / 32];
  mainloop<TBM, TBN, WM, WN, AK, BK_, VEC>(static_cast<const float*>(g.a), g.lda, static_cast<const float*>(g.b),
                                           g.ldb, g.m, g.n, m0, n0, kbeg, kend, smem, acc);
  epilogue<TBM, TBN, WM, WN, EPI>(g, m0, n0, smem, acc);
}

}  // namespace K3M_F32_NS
