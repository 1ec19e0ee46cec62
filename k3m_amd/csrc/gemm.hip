// MFMA GEMM for gfx950 with fused epilogues.
//
// fp32 path: v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 155 TF/s peak), 128x128x32 block tile
// (64x128 / 64x64 for the small co-attention GEMMs), 4 waves in 2x2, each wave owning up to 2x2
// MFMA tiles of 32x32 (64 accumulator VGPRs).  LDS holds both
// operands k-major ([BK][BM+pad]) so every MFMA operand read is a conflict-free ds_read_b32 over
// 32 consecutive floats.  Global->LDS staging is register double-buffered: the next K-tile's
// global loads are issued before the current tile's MFMAs and written to the other LDS buffer
// after them (one barrier per K-tile).
//
// Operand layouts (see include/k3m_hip.h): "K-contiguous" (x.W^T activations and torch Linear
// weights) and "MN-contiguous" (dY^T and X for weight gradients, W for input gradients) are both
// loaded with 16-byte vectors along their contiguous axis; the K-contiguous case is transposed
// while being written to LDS.  Split-K writes fp32 slabs reduced deterministically by a second
// kernel (weight gradients reduce over ~20k rows and have few output tiles).
#include "common.h"

namespace {

constexpr int BK = 32, NT = 256;

// Load one operand tile (BK x TILE) for k0.. into TILE/32 float4 registers per thread.
// KC = operand is K-contiguous in memory (element (mn, k) at p[mn*ld + k]); else MN-contiguous
// (element (mn, k) at p[k*ld + mn]).  Both map 8 consecutive lanes onto one contiguous 128-byte
// segment, so every wave instruction touches whole cache lines.
template <bool KC, bool VEC, int TILE>
__device__ __forceinline__ void load_tile(const float* __restrict__ p, long long ld, int mn0, int k0, int MN, int K,
                                          floatx4 (&r)[TILE / 32]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < TILE / 32; ++it) {
    const int idx = t + NT * it;
    if constexpr (KC) {
      const int mn = idx >> 3;          // row of the tile
      const int kq = idx & 7;           // float4 index along k
      const int gm = mn0 + mn, gk = k0 + kq * 4;
      if constexpr (VEC) {
        r[it] = (gm < MN && gk < K) ? *reinterpret_cast<const floatx4*>(p + (long long)gm * ld + gk)
                                    : floatx4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) r[it][q] = (gm < MN && gk + q < K) ? p[(long long)gm * ld + gk + q] : 0.f;
      }
    } else {
      constexpr int C4 = TILE / 4;      // float4 per k-row
      const int kr = idx / C4;
      const int c4 = (idx % C4) * 4;
      const int gk = k0 + kr, gm = mn0 + c4;
      if constexpr (VEC) {
        r[it] = (gk < K && gm < MN) ? *reinterpret_cast<const floatx4*>(p + (long long)gk * ld + gm)
                                    : floatx4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) r[it][q] = (gk < K && gm + q < MN) ? p[(long long)gk * ld + gm + q] : 0.f;
      }
    }
  }
}

// LDS row stride (floats) of the k-major image [BK][TILE + pad]: odd for the transposing scalar
// writes of K-contiguous operands (conflict-free), a multiple of 4 for float4 writes otherwise.
template <bool KC, int TILE>
constexpr int lds_stride() { return KC ? TILE + 1 : TILE + 4; }

template <bool KC, int TILE>
__device__ __forceinline__ void store_tile(float* __restrict__ s, const floatx4 (&r)[TILE / 32]) {
  constexpr int LDST = lds_stride<KC, TILE>();
  const int t = threadIdx.x;
#pragma unroll
  for (int it = 0; it < TILE / 32; ++it) {
    const int idx = t + NT * it;
    if constexpr (KC) {
      const int mn = idx >> 3, kq = idx & 7;
#pragma unroll
      for (int q = 0; q < 4; ++q) s[(kq * 4 + q) * LDST + mn] = r[it][q];
    } else {
      constexpr int C4 = TILE / 4;
      const int kr = idx / C4, c4 = (idx % C4) * 4;
      *reinterpret_cast<floatx4*>(s + kr * LDST + c4) = r[it];
    }
  }
}

__device__ __forceinline__ int xcd_remap(int id, int nblk) {
  // bijective: blocks dispatched round-robin over 8 XCDs -> contiguous id ranges per XCD
  const int xcd = id & 7, q = nblk >> 3, rr = nblk & 7;
  const int base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return base + (id >> 3);
}

// TBM x TBN block tile, 4 waves in 2x2, each wave (TBM/2) x (TBN/2) = FM x FN MFMA 32x32 tiles.
template <int TBM, int TBN, bool AK, bool BK_, bool VEC, int EPI>
__global__ __launch_bounds__(NT, 2) void gemm_f32_kernel(K3mGemm g) {
  constexpr int LDSA = lds_stride<AK, TBM>(), LDSB = lds_stride<BK_, TBN>();
  constexpr int FM = TBM / 64, FN = TBN / 64;
  __shared__ float As[2][BK * LDSA];
  __shared__ float Bs[2][BK * LDSB];
  const int M = g.m, N = g.n, K = g.k;
  const int tm = (M + TBM - 1) / TBM, tn = (N + TBN - 1) / TBN;
  const int nblk = tm * tn;
  const int id = xcd_remap(blockIdx.x, nblk);
  // grouped ordering: GROUP rows of tiles walk N together (L2 reuse of the A panel)
  constexpr int GROUP = 8;
  const int group_sz = GROUP * tn;
  const int gidx = id / group_sz;
  const int first_m = gidx * GROUP;
  const int gm_sz = min(tm - first_m, GROUP);
  const int bm = first_m + (id % group_sz) % gm_sz;
  const int bn = (id % group_sz) / gm_sz;
  const int m0 = bm * TBM, n0 = bn * TBN;

  // split-K range
  int kbeg = 0, kend = K;
  if (g.splitk > 1) {
    const int per = ((K + g.splitk - 1) / g.splitk + BK - 1) / BK * BK;
    kbeg = blockIdx.y * per;
    kend = min(K, kbeg + per);
  }
  const float* A = static_cast<const float*>(g.a);
  const float* B = static_cast<const float*>(g.b);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int wm = (w >> 1) * (TBM / 2), wn = (w & 1) * (TBN / 2);
  floatx16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  floatx4 ra[TBM / 32], rb[TBN / 32];
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    load_tile<AK, VEC, TBM>(A, g.lda, m0, kbeg, M, kend, ra);
    load_tile<BK_, VEC, TBN>(B, g.ldb, n0, kbeg, N, kend, rb);
    store_tile<AK, TBM>(As[0], ra);
    store_tile<BK_, TBN>(Bs[0], rb);
  }
  __syncthreads();
  const int kl = lane >> 5, cl = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BK;
      load_tile<AK, VEC, TBM>(A, g.lda, m0, k0, M, kend, ra);
      load_tile<BK_, VEC, TBN>(B, g.ldb, n0, k0, N, kend, rb);
    }
    const float* as = As[cur];
    const float* bs = Bs[cur];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      float a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = as[(kk + kl) * LDSA + wm + 32 * i + cl];
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = bs[(kk + kl) * LDSB + wn + 32 * j + cl];
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<AK, TBM>(As[cur ^ 1], ra);
      store_tile<BK_, TBN>(Bs[cur ^ 1], rb);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> row (r&3) + 8*(r>>2) + 4*(lane>>5), col lane&31
  float* C = static_cast<float*>(g.c);
  long long ldc = g.ldc;
  if (g.splitk > 1) {
    C = g.ws + (long long)blockIdx.y * M * N;
    ldc = N;
  }
  const float* bias = g.bias;
  float* aux = static_cast<float*>(g.aux);
  const float alpha = g.alpha, beta = g.beta;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn + j * 32 + cl;
      if (col >= N) continue;
      float bcol = 0.f;
      if constexpr (EPI == K3M_EPI_BIAS || EPI == K3M_EPI_BIAS_GELU || EPI == K3M_EPI_BIAS_SIGMOID) bcol = bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * kl;
        if (row >= M) continue;
        const float v = acc[i][j][r];
        float* cp = C + (long long)row * ldc + col;
        if constexpr (EPI == K3M_EPI_NONE) {
          float o = alpha * v;
          if (g.splitk <= 1 && beta != 0.f) o += beta * *cp;
          *cp = o;
        } else if constexpr (EPI == K3M_EPI_BIAS) {
          float o = alpha * (v + bcol);
          if (beta != 0.f) o += beta * *cp;
          *cp = o;
        } else if constexpr (EPI == K3M_EPI_BIAS_GELU) {
          const float pre = v + bcol;
          aux[(long long)row * g.ldaux + col] = pre;
          *cp = gelu_f(pre);
        } else if constexpr (EPI == K3M_EPI_DGELU) {
          float o = alpha * v * dgelu_f(aux[(long long)row * g.ldaux + col]);
          if (beta != 0.f) o += beta * *cp;
          *cp = o;
        } else {  // BIAS_SIGMOID
          *cp = sigmoid_f(v + bcol);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            float* __restrict__ C, long long ldc, float alpha,
                                                            float beta) {
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

template <int TBM, int TBN, bool AK, bool BK_, bool VEC>
int launch_epi(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_GEMM_CASE(E) \
    case E: hipLaunchKernelGGL((gemm_f32_kernel<TBM, TBN, AK, BK_, VEC, E>), grid, dim3(NT), 0, st, g); break;
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

template <int TBM, int TBN>
int launch_tile(const K3mGemm& g, bool ak, bool bk, bool vec, hipStream_t st) {
  if (ak && bk) return vec ? launch_epi<TBM, TBN, true, true, true>(g, st) : launch_epi<TBM, TBN, true, true, false>(g, st);
  if (ak) return vec ? launch_epi<TBM, TBN, true, false, true>(g, st) : launch_epi<TBM, TBN, true, false, false>(g, st);
  if (bk) return vec ? launch_epi<TBM, TBN, false, true, true>(g, st) : launch_epi<TBM, TBN, false, true, false>(g, st);
  return vec ? launch_epi<TBM, TBN, false, false, true>(g, st) : launch_epi<TBM, TBN, false, false, false>(g, st);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

long long nblocks(const K3mGemm& g, int bm, int bn) {
  return (long long)((g.m + bm - 1) / bm) * ((g.n + bn - 1) / bn) * (g.splitk > 1 ? g.splitk : 1);
}

}  // namespace

int k3m_gemm_bf16_impl(const K3mGemm& g, hipStream_t st);  // gemm_bf16.hip

extern "C" int k3m_gemm(const K3mGemm* gp, hipStream_t st) {
  if (!gp) return K3M_EINVAL;
  const K3mGemm& g = *gp;
  K3M_ARG(g.m >= 0 && g.n >= 0 && g.k >= 0);
  if (g.m == 0 || g.n == 0) return 0;
  K3M_ARG(g.dtype == K3M_F32 || g.dtype == K3M_BF16);
  K3M_ARG(g.c_dtype == K3M_F32 || (g.dtype == K3M_BF16 && g.c_dtype == K3M_BF16));
  K3M_ARG(g.a && g.b && g.c);
  K3M_ARG(g.splitk <= 1 || (g.epilogue == K3M_EPI_NONE && g.ws));
  K3M_ARG(g.epilogue == K3M_EPI_NONE || g.epilogue == K3M_EPI_DGELU || g.bias);
  K3M_ARG((g.epilogue != K3M_EPI_BIAS_GELU && g.epilogue != K3M_EPI_DGELU) || g.aux);
  if (g.dtype == K3M_BF16) return k3m_gemm_bf16_impl(g, st);
  // A: K-contiguous iff a_trans == 0; B: K-contiguous iff b_trans == 1
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  const bool av = aligned16(g.a) && (g.lda % 4 == 0) && ((ak ? g.k : g.m) % 4 == 0);
  const bool bv = aligned16(g.b) && (g.ldb % 4 == 0) && ((bk ? g.k : g.n) % 4 == 0);
  const bool vec = av && bv;
  // tile choice: the largest tile that still puts >= ~1.5 blocks on every CU (256 CUs, 2 blocks
  // per CU fit); small co-attention GEMMs (2,304-8,192 rows) otherwise leave CUs idle
  int rc;
  if (g.splitk > 1 || nblocks(g, 128, 128) >= 384) rc = launch_tile<128, 128>(g, ak, bk, vec, st);
  else if (nblocks(g, 64, 128) >= 384) rc = launch_tile<64, 128>(g, ak, bk, vec, st);
  else rc = launch_tile<64, 64>(g, ak, bk, vec, st);
  if (rc) return rc;
  K3M_CHECK_LAUNCH();
  if (g.splitk > 1) {
    const long long total = (long long)g.m * g.n;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, g.ws, g.splitk, g.m, g.n,
                       static_cast<float*>(g.c), g.ldc, g.alpha, g.beta);
    K3M_CHECK_LAUNCH();
  }
  return 0;
}
