// bf16 MFMA GEMM for gfx950 (mixed precision: bf16 operands, fp32 accumulation, fp32 or bf16 C).
//
// v_mfma_f32_32x32x16_bf16 (2.5 PF/s dense peak): 128x128x64 block tile (64x128 / 64x64 for the
// small co-attention GEMMs), 4 waves in 2x2, each wave owning up to 2x2 MFMA tiles of 32x32.
//
// LDS image of an operand tile is [TILE][64] bf16 with K contiguous (128-B rows): one MFMA operand
// fragment is one ds_read_b128 (lane l reads row l&31, k-chunk 2*ks + (l>>5)).  The 16-B chunk c of
// row r is stored in slot c ^ ((r >> 1) & 7), which puts each 16-lane ds_read_b128 group
// ({0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) on 16 distinct (row parity, slot) bank quads:
// conflict-free reads (a plain [128][64] image is 8-way).
//
// Staging (register double buffer, one barrier per K-tile):
//   * K-contiguous operands (activations, torch Linear weights for x.W^T): 8 lanes per 128-B row,
//     written to LDS as-is (ds_write_b128);
//   * MN-contiguous operands (W for input gradients, dY^T and X for weight gradients): each thread
//     loads a 4(k) x 8(mn) block as four 16-B row pieces, transposes it in registers (16-bit
//     permutes) and writes eight 8-B k-runs (ds_write_b64) into the same K-contiguous image.
// Split-K writes fp32 slabs, reduced deterministically by a second kernel (weight gradients).
#include <cstdlib>

#include "common.h"
#include "gemm_b16_tile.h"
#include "gemm_b16_ws.h"

namespace {

constexpr int BK = 64, NT = 256;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short short8v __attribute__((ext_vector_type(8)));

// element offset (bf16 units) of k-chunk c (8 bf16) of row r in a swizzled [TILE][64] image
__device__ __forceinline__ int swz(int r, int c) { return r * BK + ((c ^ ((r >> 1) & 7)) << 3); }

__device__ __forceinline__ uint32_t lo_pair(uint32_t a, uint32_t b) { return (a & 0xffffu) | (b << 16); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t a, uint32_t b) { return (a >> 16) | (b & 0xffff0000u); }

// Operand staging modes.
//   KC  (0): K-contiguous operand -> swizzled [TILE][64] image, fragments by ds_read_b128.
//   MNR (1): MN-contiguous, TILE = 64 -> transposed in registers into the same [TILE][64] image.
//   MNT (2): MN-contiguous, TILE = 128 -> copied as-is into a [64 k][128 mn] image of 256-B rows
//            (16-B chunk ch of row k at slot ch ^ (((k&3)<<2) | ((k>>2)&3))) and read with the
//            gfx950 transposing ds_read_b64_tr_b16 (two per fragment): no register transpose and
//            4 ds_write_b128 per thread instead of 8 ds_write_b64.
enum { KC = 0, MNR = 1, MNT = 2 };

template <int MODE, int TILE>
struct Stage {
  static constexpr int NR = MODE == MNR ? 4 : TILE / 32;
  u32x4 r[NR];
};

__device__ __forceinline__ int mnt_off(int k, int ch) {  // element offset in the MNT image
  return k * 128 + ((ch ^ (((k & 3) << 2) | ((k >> 2) & 3))) << 3);
}

// Load the (TILE x BK) tile at (mn0, k0) into registers.
template <int MODE, bool VEC, int TILE>
__device__ __forceinline__ void load_tile(const uint16_t* __restrict__ p, long long ld, int mn0, int k0, int MN,
                                          int K, Stage<MODE, TILE>& s) {
  const int t = threadIdx.x;
  if constexpr (MODE == KC) {
#pragma unroll
    for (int it = 0; it < TILE / 32; ++it) {
      const int idx = t + NT * it;
      const int row = idx >> 3, ch = idx & 7;
      const int gm = mn0 + row, gk = k0 + ch * 8;
      if constexpr (VEC) {
        s.r[it] = (gm < MN && gk < K) ? *reinterpret_cast<const u32x4*>(p + (long long)gm * ld + gk)
                                      : u32x4{0u, 0u, 0u, 0u};
      } else {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t e0 = (gm < MN && gk + 2 * q < K) ? p[(long long)gm * ld + gk + 2 * q] : 0u;
          const uint32_t e1 = (gm < MN && gk + 2 * q + 1 < K) ? p[(long long)gm * ld + gk + 2 * q + 1] : 0u;
          w[q] = e0 | (e1 << 16);
        }
        s.r[it] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
  } else if constexpr (MODE == MNT) {
    static_assert(TILE == 128, "MNT images are 128 wide");
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = t + NT * it;
      const int kr = idx >> 4, ch = idx & 15;
      const int gk = k0 + kr, gm = mn0 + ch * 8;
      if constexpr (VEC) {
        s.r[it] = (gk < K && gm < MN) ? *reinterpret_cast<const u32x4*>(p + (long long)gk * ld + gm)
                                      : u32x4{0u, 0u, 0u, 0u};
      } else {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t e0 = (gk < K && gm + 2 * q < MN) ? p[(long long)gk * ld + gm + 2 * q] : 0u;
          const uint32_t e1 = (gk < K && gm + 2 * q + 1 < MN) ? p[(long long)gk * ld + gm + 2 * q + 1] : 0u;
          w[q] = e0 | (e1 << 16);
        }
        s.r[it] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
  } else {
    constexpr int G8 = TILE / 8;  // mn-groups of 8
    if (2 * TILE < NT && t >= 2 * TILE) return;
    const int g8 = t % G8, g4 = t / G8;
    const int gm = mn0 + g8 * 8;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int gk = k0 + g4 * 4 + kk;
      if constexpr (VEC) {
        s.r[kk] = (gk < K && gm < MN) ? *reinterpret_cast<const u32x4*>(p + (long long)gk * ld + gm)
                                      : u32x4{0u, 0u, 0u, 0u};
      } else {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t e0 = (gk < K && gm + 2 * q < MN) ? p[(long long)gk * ld + gm + 2 * q] : 0u;
          const uint32_t e1 = (gk < K && gm + 2 * q + 1 < MN) ? p[(long long)gk * ld + gm + 2 * q + 1] : 0u;
          w[q] = e0 | (e1 << 16);
        }
        s.r[kk] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
  }
}

template <int MODE, int TILE>
__device__ __forceinline__ void store_tile(uint16_t* __restrict__ lds, const Stage<MODE, TILE>& s) {
  const int t = threadIdx.x;
  if constexpr (MODE == KC) {
#pragma unroll
    for (int it = 0; it < TILE / 32; ++it) {
      const int idx = t + NT * it;
      *reinterpret_cast<u32x4*>(lds + swz(idx >> 3, idx & 7)) = s.r[it];
    }
  } else if constexpr (MODE == MNT) {
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int idx = t + NT * it;
      *reinterpret_cast<u32x4*>(lds + mnt_off(idx >> 4, idx & 15)) = s.r[it];
    }
  } else {
    constexpr int G8 = TILE / 8;
    if (2 * TILE < NT && t >= 2 * TILE) return;
    const int g8 = t % G8, g4 = t / G8;
    const int c = g4 >> 1, half = (g4 & 1) * 4;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int mn = g8 * 8 + 2 * w;
      const u32x2 e = {lo_pair(s.r[0][w], s.r[1][w]), lo_pair(s.r[2][w], s.r[3][w])};
      const u32x2 o = {hi_pair(s.r[0][w], s.r[1][w]), hi_pair(s.r[2][w], s.r[3][w])};
      *reinterpret_cast<u32x2*>(lds + swz(mn, c) + half) = e;
      *reinterpret_cast<u32x2*>(lds + swz(mn + 1, c) + half) = o;
    }
  }
}

typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4v;

// MFMA operand fragment of the 32-wide sub-tile at mn_base, k-step ks: lane l gets
// X[mn_base + (l&31)][16 ks + 8 (l>>5) + j], j = 0..7.
template <int MODE>
__device__ __forceinline__ bf16x8 frag(const uint16_t* img, int mn_base, int ks, int lane) {
  if constexpr (MODE == MNT) {
    // two 4(k) x 16(mn) transposed block reads per 16-lane group g: rows 16ks + 8h + 4t + q,
    // columns cb .. cb+15; lane 4q+p addresses row q, columns cb + 4p .. +3 (T10 in the guide)
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, h = lane >> 5;
    const int ch = ((mn_base + 16 * (g & 1)) >> 3) + (p >> 1);
    const int r0 = 16 * ks + 8 * h + q;
    const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_short4v*)(img + mnt_off(r0, ch) + 4 * (p & 1)));
    const short4v x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_short4v*)(img + mnt_off(r0 + 4, ch) + 4 * (p & 1)));
    const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    return __builtin_bit_cast(bf16x8, v);
  } else {
    return *reinterpret_cast<const bf16x8*>(img + swz(mn_base + (lane & 31), 2 * ks + (lane >> 5)));
  }
}

__device__ __forceinline__ int xcd_remap(int id, int nblk) {
  const int xcd = id & 7, q = nblk >> 3, rr = nblk & 7;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + (id >> 3);
}

// 8 consecutive elements <-> fp32 registers, as 16-B vectors (p 16-B aligned)
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

template <int TBM, int TBN, bool AK, bool BK_, bool VEC, int EPI, typename CT>
__global__ __launch_bounds__(NT, 2) void gemm_bf16_kernel(K3mGemm g) {
  constexpr int FM = TBM / 64, FN = TBN / 64;
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * (TBM + TBN) * BK];
  const int M = g.m, N = g.n, K = g.k;
  const int tm = (M + TBM - 1) / TBM, tn = (N + TBN - 1) / TBN;
  const int nblk = tm * tn;
  const int id = xcd_remap(blockIdx.x, nblk);
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tn;
  const int gidx = id / group_sz;
  const int first_m = gidx * GROUP;
  const int gm_sz = min(tm - first_m, GROUP);
  const int bm = first_m + (id % group_sz) % gm_sz;
  const int bn = (id % group_sz) / gm_sz;
  const int m0 = bm * TBM, n0 = bn * TBN;

  int kbeg = 0, kend = K;
  if (g.splitk > 1) {
    const int per = ((K + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = blockIdx.y * per;
    kend = min(K, kbeg + per);
  }
  const uint16_t* A = static_cast<const uint16_t*>(g.a);
  const uint16_t* B = static_cast<const uint16_t*>(g.b);
  constexpr int BUF = (TBM + TBN) * BK;  // one stage: A image [TBM][64] then B image [TBN][64]

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * (TBM / 2), wn = (w & 1) * (TBN / 2);
  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int AM = AK ? KC : (TBM == 128 ? MNT : MNR);
  constexpr int BM_ = BK_ ? KC : (TBN == 128 ? MNT : MNR);
  Stage<AM, TBM> ra;
  Stage<BM_, TBN> rb;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile<AM, VEC, TBM>(A, g.lda, m0, kbeg, M, kend, ra);
    load_tile<BM_, VEC, TBN>(B, g.ldb, n0, kbeg, N, kend, rb);
    store_tile<AM, TBM>(smem, ra);
    store_tile<BM_, TBN>(smem + TBM * BK, rb);
  }
  __syncthreads();
  const int kl = lane >> 5, cl = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<AM, VEC, TBM>(A, g.lda, m0, k0, M, kend, ra);
      load_tile<BM_, VEC, TBN>(B, g.ldb, n0, k0, N, kend, rb);
    }
    const uint16_t* as = smem + cur * BUF;
    const uint16_t* bs = as + TBM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = frag<AM>(as, wm + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = frag<BM_>(bs, wn + 32 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<AM, TBM>(smem + (cur ^ 1) * BUF, ra);
      store_tile<BM_, TBN>(smem + (cur ^ 1) * BUF + TBM * BK, rb);
    }
    // every fragment read of this stage has returned before any wave passes the barrier and
    // restages it (hipcc may sink the MFMAs, and with them the reads' waits, below the barrier)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue, staged through LDS (free after the last barrier) so that global traffic is row-
  // contiguous 16-B vectors: each wave writes one 32-row slice of its accumulators (fp32) into a
  // private [32][WN+8] region (stride = 8 mod 16 floats: the two half-waves' rows land 32 banks apart),
  // then reads it back 8 consecutive columns per lane and applies the epilogue on the way out.
  // acc[i][j][r] holds row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31 of MFMA tile (i, j).
  constexpr int WN = TBN / 2, WS = WN + 8, LPR = WN / 8, RPP = 64 / LPR;
  static_assert(4 * 32 * WS * 4 <= 2 * (TBM + TBN) * BK * 2, "epilogue staging exceeds the LDS tile");
  float* wl = reinterpret_cast<float*>(smem) + w * 32 * WS;
  const bool split = g.splitk > 1;
  CT* C = split ? reinterpret_cast<CT*>(g.ws + (long long)blockIdx.y * M * N) : static_cast<CT*>(g.c);
  const long long ldc = split ? N : g.ldc;
  const float alpha = split ? 1.f : g.alpha, beta = split ? 0.f : g.beta;
  CT* aux = static_cast<CT*>(g.aux);
  const float* bias = g.bias;
  constexpr bool HAS_AUX = EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_DGELU;
  constexpr bool HAS_BIAS = EPI == K3M_EPI_BIAS || EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_BIAS_SIGMOID;
  const bool cvec = (ldc % 8 == 0) && ((reinterpret_cast<uintptr_t>(C) & 15) == 0) &&
                    (!HAS_AUX || ((g.ldaux % 8 == 0) && ((reinterpret_cast<uintptr_t>(aux) & 15) == 0)));
  const int lr = lane / LPR, lc = (lane % LPR) * 8;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) wl[((r & 3) + 8 * (r >> 2) + 4 * kl) * WS + 32 * j + cl] = acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int ps = 0; ps < 32 / RPP; ++ps) {
      const int rr = ps * RPP + lr;
      const int row = m0 + wm + 32 * i + rr;
      const int col = n0 + wn + lc;
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc);
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(wl + rr * WS + lc + 4);
      if (row >= M || col >= N) continue;
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      const bool full = cvec && col + 8 <= N;
      CT* cp = C + (long long)row * ldc + col;
      CT* ap = HAS_AUX ? aux + (long long)row * g.ldaux + col : nullptr;
      float old[8], ax[8], bb[8];
      if constexpr (HAS_BIAS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) bb[e] = col + e < N ? bias[col + e] : 0.f;
      }
      if constexpr (EPI == K3M_EPI_DGELU) {
        if (full) load8(ap, ax);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) ax[e] = col + e < N ? to_f(ap[e]) : 0.f;
      }
      const bool rd_old = (EPI == K3M_EPI_NONE || EPI == K3M_EPI_BIAS || EPI == K3M_EPI_DGELU) && beta != 0.f;
      if (rd_old) {
        if (full) load8(cp, old);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) old[e] = col + e < N ? to_f(cp[e]) : 0.f;
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
          o[e] = gelu_fast(to_f(from_f<CT>(pa[e])));  // gelu of the stored pre-activation the backward sees
        } else if constexpr (EPI == K3M_EPI_DGELU) {
          o[e] = alpha * v[e] * dgelu_fast(ax[e]);
        } else {
          o[e] = sigmoid_f(v[e] + bb[e]);
        }
        if (rd_old) o[e] += beta * old[e];
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
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_bf16_kernel(const float* __restrict__ ws, int splits, int M,
                                                                 int N, float* __restrict__ C, long long ldc,
                                                                 float alpha, float beta) {
  const long long total = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ws[(long long)k * total + e];
    const int row = (int)(e / N), col = (int)(e % N);
    float* cp = C + (long long)row * ldc + col;
    float o = alpha * s;
    if (beta != 0.f) o += beta * *cp;
    *cp = o;
  }
}

template <int TBM, int TBN, bool AK, bool BK_, bool VEC, typename CT>
int launch_epi(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_GEMM_CASE(E) \
    case E: hipLaunchKernelGGL((gemm_bf16_kernel<TBM, TBN, AK, BK_, VEC, E, CT>), grid, dim3(NT), 0, st, g); break;
    K3M_GEMM_CASE(K3M_EPI_NONE)
    K3M_GEMM_CASE(K3M_EPI_BIAS)
    K3M_GEMM_CASE(K3M_EPI_BIAS_GELU)
    K3M_GEMM_CASE(K3M_EPI_DGELU)
    K3M_GEMM_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_GEMM_CASE
    default: return K3M_EINVAL;
  }
  return 0;
}

template <int TBM, int TBN, typename CT>
int launch_tile(const K3mGemm& g, bool ak, bool bk, bool vec, hipStream_t st) {
  if (ak && bk) return vec ? launch_epi<TBM, TBN, true, true, true, CT>(g, st) : launch_epi<TBM, TBN, true, true, false, CT>(g, st);
  if (ak) return vec ? launch_epi<TBM, TBN, true, false, true, CT>(g, st) : launch_epi<TBM, TBN, true, false, false, CT>(g, st);
  if (bk) return vec ? launch_epi<TBM, TBN, false, true, true, CT>(g, st) : launch_epi<TBM, TBN, false, true, false, CT>(g, st);
  return vec ? launch_epi<TBM, TBN, false, false, true, CT>(g, st) : launch_epi<TBM, TBN, false, false, false, CT>(g, st);
}

template <typename CT>
int launch_ct(const K3mGemm& g, bool ak, bool bk, bool vec, hipStream_t st) {
  auto nb = [&](int bm, int bn) {
    return (long long)((g.m + bm - 1) / bm) * ((g.n + bn - 1) / bn) * (g.splitk > 1 ? g.splitk : 1);
  };
  if (g.splitk > 1 || nb(128, 128) >= 384) return launch_tile<128, 128, CT>(g, ak, bk, vec, st);
  if (nb(64, 128) >= 384) return launch_tile<64, 128, CT>(g, ak, bk, vec, st);
  return launch_tile<64, 64, CT>(g, ak, bk, vec, st);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// ---------------------------------------------------------------- large-tile path (gemm_b16_tile.h)
// Eligible: 16-B aligned operands with ld % 8 == 0, K a multiple of 64, and either both operands
// K-contiguous (forward) or A K-contiguous / B MN-contiguous (input gradients) with any epilogue, or
// both MN-contiguous (weight gradients) with the plain fp32 epilogue.
bool big_ok(const K3mGemm& g, bool vec) {
  if (!vec || g.k % k3m_b16::BK != 0 || g.k == 0) return false;
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  if (!ak && bk) return false;
  if (!ak && !(g.epilogue == K3M_EPI_NONE && g.c_dtype == K3M_F32)) return false;   // weight gradients
  if (g.splitk > 1 && ((g.k + g.splitk - 1) / g.splitk) < k3m_b16::BK) return false;
  return true;
}

long long nb_of(const K3mGemm& g, int bm, int bn) {
  return (long long)((g.m + bm - 1) / bm) * ((g.n + bn - 1) / bn) * (g.splitk > 1 ? g.splitk : 1);
}

// MFMA shape per operand layout: 16x16x32 when B is K-contiguous (forward), 32x32x16 when it is
// MN-contiguous (input and weight gradients: their transposing fragment reads fit the LDS counter
// per 16-deep substep); K3M_B16_MF=16 / 32 forces one shape everywhere (A/B).
// (the round-3 K3M_B16_MF override is gone: one MFMA shape per operand layout halves the instantiations)
template <bool BK_> constexpr int mf_of() { return BK_ ? 16 : 32; }

// The large-tile GEMMs as a persistent walk of min(units, CUs) workgroups (gemm_persist_kernel): bit-identical,
// bf16 step +0.4 % in three interleaved pairs (profiles/r3_ab_b16_persist.txt); K3M_B16_PERSIST=0 launches one
// workgroup per tile (A/B knob)
const bool kB16Persist = k3m_env_flag("K3M_B16_PERSIST", true);
int b16_cus() {
  static int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return 256;
    return cus;
  }();
  return n;
}

// K3M_B16_PREFETCH=1: the walk issues each next tile's first k-tile inside the epilogue (A/B knob; bit-identical,
// +0.1 % on the bf16 step, within noise: off, profiles/r3_ab_b16_persist.txt)
const bool kB16Prefetch = k3m_env_flag("K3M_B16_PREFETCH", false);

// timing-only lab knobs of the persistent walk (never set in product runs): K3M_B16_LAB bit 0 = skip the C / aux
// stores, bit 1 = staggered start of K3M_B16_STAGGER ticks (10 ns) per workgroup group (b & 3), bit 2 = non-temporal
// C / aux stores in the interior-tile epilogue
const int kB16Lab = k3m_env_int("K3M_B16_LAB", 0);
const int kB16Stagger = k3m_env_int("K3M_B16_STAGGER", 500);

// K3M_B16_DUAL: the large-tile GEMMs on the two-workgroups-per-CU kernel (gemm_dual_kernel: 256 x 128 x 32
// tiles, 4 waves, three LDS stages) instead of the one-workgroup 256 x 256 / 256 x 128 walk.  0 = never,
// 1 = always, 2 (default) = the GELU / dGELU epilogues only: there one workgroup's epilogue VALU overlaps the
// other's MFMAs (FFN1 fwd -2 %, FFN2 dgrad+dGELU -4 %, co-attention PV FFN1 -14 %), while the plain main loop
// is 10-25 % slower at 256 x 128 x 32 (1.5x the operand bytes per MFMA of 256 x 256; profiles/r4b_ab_dual.txt)
const int kB16Dual = k3m_env_int("K3M_B16_DUAL", 2);
// K3M_B16_PP: the persistent walk with the ping-pong main loop (mainloop_pp, gemm_b16_tile.h), bit 0 for the
// v_mfma_f32_16x16x32 layouts (both operands K-contiguous), bit 1 for the 32x32x16 ones (MN-contiguous B); the
// 256 x 128 tiles only unless bit 2 is set (the 256 x 256 ping-pong loop spills its fragment addresses)
// measured slower on config 3 (profiles/r5d/README.txt): off
const int kB16PP = k3m_env_int("K3M_B16_PP", 0);
constexpr bool dual_epi(int epi) { return epi == K3M_EPI_BIAS_GELU || epi == K3M_EPI_DGELU; }
// K3M_B16_WS: the K-contiguous forwards with a bf16 C on the epilogue-wave kernel (gemm_b16_ws.h): bit 0 the bias+GELU
// epilogue, bit 1 bias / none.  Needs K % 32 == 0 and K >= 32 * ws::KMIN, beta = 0, no split-K, aligned C / aux / bias.
const int kB16WS = k3m_env_int("K3M_B16_WS", 0);
constexpr int ws_bit(int epi) { return epi == K3M_EPI_BIAS_GELU ? 1 : (epi == K3M_EPI_BIAS || epi == K3M_EPI_NONE) ? 2 : 0; }

long long nb_of(const K3mGemm& g, int bm, int bn);

template <bool AK, bool BK_, int EPI, typename CT, int MF>
void dual_launch(const k3m_b16::GemmGroup& grp_in, hipStream_t st) {
  k3m_b16::GemmGroup grp = grp_in;   // units re-counted for the 256 x 128 tiles
  int nb = 0;
  for (int i = 0; i < grp.count; ++i) {
    grp.start[i] = nb;
    nb += (int)nb_of(grp.g[i], 256, 128);
  }
  grp.start[grp.count] = nb;
  const int nblk = nb < 2 * b16_cus() ? nb : 2 * b16_cus();
  hipLaunchKernelGGL((k3m_b16::gemm_dual_kernel<256, 128, 2, 2, AK, BK_, EPI, CT, MF>), dim3(nblk), dim3(256), 0, st,
                     grp);
}

bool ws_ok(const k3m_b16::GemmGroup& grp) {
  for (int i = 0; i < grp.count; ++i) {
    const K3mGemm& g = grp.g[i];
    if (g.splitk > 1 || g.beta != 0.f || g.k % k3m_b16::ws::BKW != 0 || g.k < k3m_b16::ws::BKW * k3m_b16::ws::KMIN ||
        g.n < 8 || g.n % 8 != 0 || g.ldc % 8 != 0 || !aligned16(g.c))
      return false;
    if (g.epilogue != K3M_EPI_NONE && !aligned16(g.bias)) return false;
    if (g.epilogue == K3M_EPI_BIAS_GELU && (g.ldaux % 8 != 0 || !aligned16(g.aux))) return false;
    // byte offsets of the buffer stores are 32-bit
    if (((long long)(g.m - 1) * g.ldc + g.n) * 2 >= 0x7ffffff0LL) return false;
    if (g.epilogue == K3M_EPI_BIAS_GELU && ((long long)(g.m - 1) * g.ldaux + g.n) * 2 >= 0x7ffffff0LL) return false;
  }
  return true;
}

template <int EPI>
void ws_launch(const k3m_b16::GemmGroup& grp_in, hipStream_t st) {
  k3m_b16::GemmGroup grp = grp_in;   // units re-counted for the 256 x 128 tiles
  int nb = 0;
  for (int i = 0; i < grp.count; ++i) {
    grp.start[i] = nb;
    nb += (int)nb_of(grp.g[i], k3m_b16::ws::TBM, k3m_b16::ws::TBN);
  }
  grp.start[grp.count] = nb;
  const int nblk = nb < b16_cus() ? nb : b16_cus();
  hipLaunchKernelGGL((k3m_b16::ws::gemm_ws_kernel<EPI>), dim3(nblk), dim3(512), 0, st, grp);
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
void persist_launch(const k3m_b16::GemmGroup& grp_in, hipStream_t st) {
  if constexpr (AK && BK_ && std::is_same<CT, bf16_t>::value && ws_bit(EPI) != 0) {
    if ((kB16WS & ws_bit(EPI)) != 0 && ws_ok(grp_in)) {
      ws_launch<EPI>(grp_in, st);
      return;
    }
  }
  if (kB16Dual == 1 || (kB16Dual == 2 && dual_epi(EPI))) {
    dual_launch<AK, BK_, EPI, CT, MF>(grp_in, st);
    return;
  }
  k3m_b16::GemmGroup grp = grp_in;
  grp.lab = kB16Lab;
  grp.stagger = kB16Stagger;
  const int total = grp.start[grp.count];
  const int nblk = total < b16_cus() ? total : b16_cus();
  if ((kB16PP & (MF == 16 ? 1 : 2)) != 0 && (TBN == 128 || (kB16PP & 4) != 0))
    hipLaunchKernelGGL((k3m_b16::gemm_persist_kernel<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF, false, true>), dim3(nblk),
                       dim3(64 * WM * WN), 0, st, grp);
  else if (kB16Prefetch)
    hipLaunchKernelGGL((k3m_b16::gemm_persist_kernel<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF, true>), dim3(nblk),
                       dim3(64 * WM * WN), 0, st, grp);
  else
    hipLaunchKernelGGL((k3m_b16::gemm_persist_kernel<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF, false>), dim3(nblk),
                       dim3(64 * WM * WN), 0, st, grp);
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, int EPI, typename CT, int MF>
void one_launch(const K3mGemm& g, hipStream_t st) {
  if (kB16Persist) {
    k3m_b16::GemmGroup grp = {};
    grp.g[0] = g;
    grp.start[0] = 0;
    grp.start[1] = (int)nb_of(g, TBM, TBN);
    grp.count = 1;
    persist_launch<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF>(grp, st);
    return;
  }
  hipLaunchKernelGGL((k3m_b16::gemm_kernel<TBM, TBN, WM, WN, AK, BK_, EPI, CT, MF>), dim3((unsigned)nb_of(g, TBM, TBN)),
                     dim3(64 * WM * WN), 0, st, g);
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, typename CT, int MF>
int big_launch_epi_mf(const K3mGemm& g, hipStream_t st) {
  switch (g.epilogue) {
#define K3M_GEMM_CASE(E)                                                                                     \
    case E:                                                                                                  \
      one_launch<TBM, TBN, WM, WN, AK, BK_, E, CT, MF>(g, st);                                               \
      break;
    K3M_GEMM_CASE(K3M_EPI_NONE)
    K3M_GEMM_CASE(K3M_EPI_BIAS)
    K3M_GEMM_CASE(K3M_EPI_BIAS_GELU)
    K3M_GEMM_CASE(K3M_EPI_DGELU)
    K3M_GEMM_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_GEMM_CASE
    default: return K3M_EINVAL;
  }
  return 0;
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, typename CT>
int big_launch_epi(const K3mGemm& g, hipStream_t st) {
  return big_launch_epi_mf<TBM, TBN, WM, WN, AK, BK_, CT, mf_of<BK_>()>(g, st);
}

template <int TBM, int TBN, int WM, int WN>
int big_launch(const K3mGemm& g, hipStream_t st) {
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  if (!ak) {
    if (g.epilogue != K3M_EPI_NONE) return K3M_EINVAL;
    one_launch<TBM, TBN, WM, WN, false, false, K3M_EPI_NONE, float, 32>(g, st);
    return 0;
  }
  if (g.c_dtype == K3M_F32)
    return bk ? big_launch_epi<TBM, TBN, WM, WN, true, true, float>(g, st)
              : big_launch_epi<TBM, TBN, WM, WN, true, false, float>(g, st);
  return bk ? big_launch_epi<TBM, TBN, WM, WN, true, true, bf16_t>(g, st)
            : big_launch_epi<TBM, TBN, WM, WN, true, false, bf16_t>(g, st);
}

// tile policy: 256x256 when it still gives >= 1/2 of a wave of blocks, else 256x128 (A/B knob K3M_B16_256;
// 128 vs 192: bf16 step +0.35 %, 256: -4 %, profiles/r3_ab_b16_policy.txt)
const int kB16Min256 = k3m_env_int("K3M_B16_256", 128);
bool big_prefers_256(long long nb256) { return nb256 >= kB16Min256; }

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, typename CT, int MF>
int big_grouped_epi_mf(const k3m_b16::GemmGroup& grp, int epi, hipStream_t st) {
  const dim3 grid(grp.start[grp.count]);
  switch (epi) {
#define K3M_GROUP_CASE(E)                                                                                      \
    case E:                                                                                                    \
      if (kB16Persist)                                                                                         \
        persist_launch<TBM, TBN, WM, WN, AK, BK_, E, CT, MF>(grp, st);                                         \
      else                                                                                                     \
        hipLaunchKernelGGL((k3m_b16::gemm_grouped_kernel<TBM, TBN, WM, WN, AK, BK_, E, CT, MF>), grid,         \
                           dim3(64 * WM * WN), 0, st, grp);                                                    \
      break;
    K3M_GROUP_CASE(K3M_EPI_NONE)
    K3M_GROUP_CASE(K3M_EPI_BIAS)
    K3M_GROUP_CASE(K3M_EPI_BIAS_GELU)
    K3M_GROUP_CASE(K3M_EPI_DGELU)
    K3M_GROUP_CASE(K3M_EPI_BIAS_SIGMOID)
#undef K3M_GROUP_CASE
    default: return K3M_EINVAL;
  }
  return 0;
}

template <int TBM, int TBN, int WM, int WN, bool AK, bool BK_, typename CT>
int big_grouped_epi(const k3m_b16::GemmGroup& grp, int epi, hipStream_t st) {
  return big_grouped_epi_mf<TBM, TBN, WM, WN, AK, BK_, CT, mf_of<BK_>()>(grp, epi, st);
}

template <int TBM, int TBN, int WM, int WN>
int big_grouped(const k3m_b16::GemmGroup& grp, hipStream_t st) {
  const K3mGemm& g = grp.g[0];
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  if (!ak) {
    if (g.epilogue != K3M_EPI_NONE) return K3M_EINVAL;
    if (kB16Persist)
      persist_launch<TBM, TBN, WM, WN, false, false, K3M_EPI_NONE, float, 32>(grp, st);
    else
      hipLaunchKernelGGL((k3m_b16::gemm_grouped_kernel<TBM, TBN, WM, WN, false, false, K3M_EPI_NONE, float, 32>),
                         dim3(grp.start[grp.count]), dim3(64 * WM * WN), 0, st, grp);
    return 0;
  }
  if (g.c_dtype == K3M_F32)
    return bk ? big_grouped_epi<TBM, TBN, WM, WN, true, true, float>(grp, g.epilogue, st)
              : big_grouped_epi<TBM, TBN, WM, WN, true, false, float>(grp, g.epilogue, st);
  return bk ? big_grouped_epi<TBM, TBN, WM, WN, true, true, bf16_t>(grp, g.epilogue, st)
            : big_grouped_epi<TBM, TBN, WM, WN, true, false, bf16_t>(grp, g.epilogue, st);
}

int reduce_splits(const K3mGemm& g, hipStream_t st) {
  if (g.splitk > 1) {
    const long long total = (long long)g.m * g.n;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_bf16_kernel, dim3(blocks), dim3(256), 0, st, g.ws, g.splitk, g.m, g.n,
                       static_cast<float*>(g.c), g.ldc, g.alpha, g.beta);
    K3M_CHECK_LAUNCH();
  }
  return 0;
}

bool vec_of(const K3mGemm& g) {
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  const bool av = aligned16(g.a) && (g.lda % 8 == 0) && ((ak ? g.k : g.m) % 8 == 0);
  const bool bv = aligned16(g.b) && (g.ldb % 8 == 0) && ((bk ? g.k : g.n) % 8 == 0);
  return av && bv;
}

// K3M_BF16_BIG=0 keeps every bf16 GEMM on the 128x128 register-staged kernel (A/B switch)
const bool kBig = k3m_env_flag("K3M_BF16_BIG", true);
// fewest 256x128 tiles for the large-tile kernel; smaller grids take the 128x128 / 64x128 kernel (A/B knob;
// 80 vs 160: bf16 step +0.4-0.5 %, profiles/r3_ab_b16_policy.txt)
const int kB16Min = k3m_env_int("K3M_B16_MIN", 80);

}  // namespace

// K3M_GEMM_COLSUM_SLABS for the kernels whose epilogue does not fuse it: 32-row column sums of C
template <typename CT>
__global__ __launch_bounds__(256) void colsum32_kernel(const CT* __restrict__ c, long long ldc, int m, int n,
                                                       float* __restrict__ ws) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= n) return;
  const int r0 = blockIdx.y * 32, r1 = min(m, r0 + 32);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += to_f(c[(long long)r * ldc + col]);
  ws[(long long)blockIdx.y * n + col] = s;
}

// Called by k3m_gemm (gemm.hip) for dtype == K3M_BF16; arguments already validated there.
int k3m_gemm_bf16_impl(const K3mGemm& g, hipStream_t st, bool slabs_only, bool colsum) {
  K3M_ARG(g.splitk <= 1 || g.c_dtype == K3M_F32);
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  const bool vec = vec_of(g);
  int rc;
  const long long nb256 = nb_of(g, 256, 256), nb128 = nb_of(g, 256, 128);
  bool fused = false;   // the large-tile epilogue writes the COLSUM_SLABS itself
  if (kBig && big_ok(g, vec) && nb128 >= kB16Min) {
    rc = big_prefers_256(nb256) ? big_launch<256, 256, 2, 4>(g, st) : big_launch<256, 128, 4, 2>(g, st);
    fused = true;
  } else {
    rc = g.c_dtype == K3M_F32 ? launch_ct<float>(g, ak, bk, vec, st) : launch_ct<bf16_t>(g, ak, bk, vec, st);
  }
  if (rc) return rc;
  K3M_CHECK_LAUNCH();
  if (colsum && !fused) {
    const dim3 grid((g.n + 255) / 256, (g.m + 31) / 32);
    if (g.c_dtype == K3M_F32)
      hipLaunchKernelGGL(colsum32_kernel<float>, grid, dim3(256), 0, st, static_cast<const float*>(g.c), g.ldc, g.m,
                         g.n, g.ws);
    else
      hipLaunchKernelGGL(colsum32_kernel<bf16_t>, grid, dim3(256), 0, st, static_cast<const bf16_t*>(g.c), g.ldc, g.m,
                         g.n, g.ws);
    K3M_CHECK_LAUNCH();
  }
  return slabs_only ? 0 : reduce_splits(g, st);   // K3M_GEMM_SLABS_ONLY: the caller reduces the slabs
}

// Grouped bf16 problems (co-attention stages of the bf16 encoder): one large-tile grid when every
// problem is eligible and shares the template (*handled = true), else nothing is launched.
int k3m_gemm_bf16_grouped_impl(const K3mGemm* gs, int count, hipStream_t st, bool* handled,
                               const bool* slabs_only) {
  *handled = false;
  if (!kBig || count <= 0 || count > k3m_b16::GROUP_MAX) return 0;
  const K3mGemm& g0 = gs[0];
  k3m_b16::GemmGroup grp = {};
  bool live_slabs[k3m_b16::GROUP_MAX] = {};
  int live = 0;
  long long nb256 = 0, nb128 = 0;
  for (int i = 0; i < count; ++i) {
    const K3mGemm& g = gs[i];
    if (g.dtype != K3M_BF16 || g.a_trans != g0.a_trans || g.b_trans != g0.b_trans || g.epilogue != g0.epilogue ||
        g.c_dtype != g0.c_dtype || !big_ok(g, vec_of(g)) || (g.splitk > 1 && g.c_dtype != K3M_F32))
      return 0;
    if (g.m == 0 || g.n == 0) continue;
    live_slabs[live] = slabs_only[i];
    grp.g[live++] = g;
    nb256 += nb_of(g, 256, 256);
    nb128 += nb_of(g, 256, 128);
  }
  *handled = true;
  if (live == 0) return 0;
  k3m_lpt_order(grp.g, live_slabs, live);
  const bool t256 = big_prefers_256(nb256);
  int nb = 0;
  for (int i = 0; i < live; ++i) {
    grp.start[i] = nb;
    nb += (int)nb_of(grp.g[i], 256, t256 ? 256 : 128);
  }
  grp.start[live] = nb;
  grp.count = live;
  const int rc = t256 ? big_grouped<256, 256, 2, 4>(grp, st) : big_grouped<256, 128, 4, 2>(grp, st);
  if (rc) return rc;
  K3M_CHECK_LAUNCH();
  for (int i = 0; i < live; ++i) {
    if (live_slabs[i]) continue;
    const int r = reduce_splits(grp.g[i], st);
    if (r) return r;
  }
  return 0;
}
