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
template <int TBM, int TBN, int WM, int WN, int EPI, int CAP = 2 * (TBM + TBN) * BK, class Hook = NoHook>
__device__ __forceinline__ void epilogue(const K3mGemm& g, int m0, int n0, float* smem,
                                         const floatx16 (&acc)[TBM / WM / 32][TBN / WN / 32], int slice = -1,
                                         Hook hook = Hook()) {
  constexpr int FM = TBM / WM / 32, FN = TBN / WN / 32;
  constexpr int WCOLS = FN * 32, WS = WCOLS + 8, LPR = WCOLS / 8, RPP = 64 / LPR;
  static_assert(WM * WN * 32 * WS <= CAP, "epilogue staging exceeds the LDS tile");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w / WN) * (TBM / WM), wn = (w % WN) * (TBN / WN);
  const int kl = lane >> 5, cl = lane & 31;
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
  const bool cvec = (ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                    (!HAS_AUX || ((g.ldaux % 4 == 0) && ((reinterpret_cast<uintptr_t>(aux) & 15) == 0)));
  const bool rd_old = (EPI == K3M_EPI_NONE || EPI == K3M_EPI_BIAS || EPI == K3M_EPI_DGELU) && beta != 0.f;
  const bool bvec = HAS_BIAS && ((reinterpret_cast<uintptr_t>(bias) & 15) == 0);
  const int lr = lane / LPR, lc = (lane % LPR) * 8;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) wl[((r & 3) + 8 * (r >> 2) + 4 * kl) * WS + 32 * j + cl] = acc[i][j][r];
    __syncthreads();
    if (i == 0) hook();
#pragma unroll
    for (int ps = 0; ps < 32 / RPP; ++ps) {
      const int rr = ps * RPP + lr;
      const int row = m0 + wm + 32 * i + rr;
      const int col = n0 + wn + lc;
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
      if (row >= M || col >= N) continue;
      const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const bool full = cvec && col + 8 <= N;
      float* cp = C + (long long)row * ldc + col;
      float* ap = HAS_AUX ? aux + (long long)row * g.ldaux + col : nullptr;
      float old[8], ax[8], bb[8];
      if constexpr (HAS_BIAS) {
        if (bvec && col + 8 <= N) {
          const floatx4 b0 = *reinterpret_cast<const floatx4*>(bias + col), b1 = *reinterpret_cast<const floatx4*>(bias + col + 4);
          bb[0] = b0[0]; bb[1] = b0[1]; bb[2] = b0[2]; bb[3] = b0[3]; bb[4] = b1[0]; bb[5] = b1[1]; bb[6] = b1[2]; bb[7] = b1[3];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) bb[e] = col + e < N ? bias[col + e] : 0.f;
        }
      }
      if constexpr (EPI == K3M_EPI_DGELU) {
        if (full) {
          const floatx4 x0 = *reinterpret_cast<const floatx4*>(ap), x1 = *reinterpret_cast<const floatx4*>(ap + 4);
          ax[0] = x0[0]; ax[1] = x0[1]; ax[2] = x0[2]; ax[3] = x0[3]; ax[4] = x1[0]; ax[5] = x1[1]; ax[6] = x1[2]; ax[7] = x1[3];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) ax[e] = col + e < N ? ap[e] : 0.f;
        }
      }
      if (rd_old) {
        if (full) {
          const floatx4 o0 = *reinterpret_cast<const floatx4*>(cp), o1 = *reinterpret_cast<const floatx4*>(cp + 4);
          old[0] = o0[0]; old[1] = o0[1]; old[2] = o0[2]; old[3] = o0[3]; old[4] = o1[0]; old[5] = o1[1]; old[6] = o1[2]; old[7] = o1[3];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = col + e < N ? cp[e] : 0.f;
        }
      }
      float o[8], pa[8];
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
      if (full) {
        *reinterpret_cast<floatx4*>(cp) = floatx4{o[0], o[1], o[2], o[3]};
        *reinterpret_cast<floatx4*>(cp + 4) = floatx4{o[4], o[5], o[6], o[7]};
        if constexpr (EPI == K3M_EPI_BIAS_GELU) {
          *reinterpret_cast<floatx4*>(ap) = floatx4{pa[0], pa[1], pa[2], pa[3]};
          *reinterpret_cast<floatx4*>(ap + 4) = floatx4{pa[4], pa[5], pa[6], pa[7]};
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < N) {
            cp[e] = o[e];
            if constexpr (EPI == K3M_EPI_BIAS_GELU) ap[e] = pa[e];
          }
      }
    }
    __syncthreads();
  }
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
