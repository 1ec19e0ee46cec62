// MFMA GEMM entry point for gfx950 (k3m_gemm) and the fp32 tile policy.
//
// fp32 operands, default (K3M_F32_SPLIT_BF16X6): the bf16x6 split kernel of gemm_x6_tile.h on the
// bf16 matrix cores (fp32 accuracy, 2.67x the f32-MFMA roofline), tile chosen per shape:
//   * 256x256x16 (8 waves, 1 block/CU, 96 KB LDS) for the large GEMMs and the split-K weight
//     gradients when its half-as-many blocks do not cost an extra wave (prefer_256x256);
//   * 256x128x32 (8 waves, 1 block/CU, 144 KB LDS) otherwise (ops._splitk sizes the split to whole
//     waves of 256 of these blocks);
//   * 128x128x32 (4 waves) for mid-size grids;
//   * 64x64x16 for the small co-attention GEMMs.
// K3M_F32_MFMA_F32 (and unaligned operands): the v_mfma_f32_32x32x2_f32 kernel of gemm_f32_tile.h
// (exact f32 products and accumulation), tile chosen per shape:
//   * 256x256 (8 waves, 1 block/CU) when it still gives ~a block per CU: the fewest L2 bytes per FLOP;
//   * 128x128 (4 waves, 2 blocks/CU) for split-K weight gradients and mid-size grids;
//   * 64x128 / 64x64 for the small co-attention GEMMs (2,304-8,192 rows) that would otherwise leave
//     CUs idle.
// Split-K writes fp32 slabs (raw sums) reduced deterministically by splitk_reduce_kernel, which
// applies alpha/beta.  bf16 operands go to gemm_bf16.hip.
#include "gemm_x6_tile.h"

#include <cstdlib>

namespace {

using k3m_f32::gemm_f32_kernel;

// C = epilogue(sum of the split-K slabs in slice order): the element formulas of the tile epilogues
// (gemm_f32_tile.h epi_math), so a split problem ends exactly like the unsplit one would on its sums
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                            float* __restrict__ C, long long ldc, float alpha,
                                                            float beta, int epi, const float* __restrict__ bias,
                                                            float* __restrict__ aux, long long ldaux) {
  const long long total = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ws[(long long)k * total + e];
    const int row = (int)(e / N), col = (int)(e % N);
    float* cp = C + (long long)row * ldc + col;
    float o;
    bool can_old = true;
    switch (epi) {
      case K3M_EPI_BIAS: o = alpha * (s + bias[col]); break;
      case K3M_EPI_BIAS_GELU: {
        const float pa = s + bias[col];
        aux[(long long)row * ldaux + col] = pa;
        o = gelu_f(pa);
        can_old = false;
        break;
      }
      case K3M_EPI_DGELU: o = alpha * s * dgelu_f(aux[(long long)row * ldaux + col]); break;
      case K3M_EPI_BIAS_SIGMOID: o = sigmoid_f(s + bias[col]); can_old = false; break;
      default: o = alpha * s;
    }
    if (can_old && beta != 0.f) o += beta * *cp;
    *cp = o;
  }
}

template <int TBM, int TBN, int WM, int WN, int OCC, bool AK, bool BK_, bool VEC>
int launch_epi(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_GEMM_CASE(E)                                                                                     \
    case E:                                                                                                  \
      hipLaunchKernelGGL((gemm_f32_kernel<TBM, TBN, WM, WN, AK, BK_, VEC, E, OCC>), grid, dim3(64 * WM * WN), 0, st, g); \
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

template <int TBM, int TBN, int WM, int WN, int OCC>
int launch_tile(const K3mGemm& g, bool ak, bool bk, bool vec, hipStream_t st) {
  if (ak && bk) return vec ? launch_epi<TBM, TBN, WM, WN, OCC, true, true, true>(g, st) : launch_epi<TBM, TBN, WM, WN, OCC, true, true, false>(g, st);
  if (ak) return vec ? launch_epi<TBM, TBN, WM, WN, OCC, true, false, true>(g, st) : launch_epi<TBM, TBN, WM, WN, OCC, true, false, false>(g, st);
  if (bk) return vec ? launch_epi<TBM, TBN, WM, WN, OCC, false, true, true>(g, st) : launch_epi<TBM, TBN, WM, WN, OCC, false, true, false>(g, st);
  return vec ? launch_epi<TBM, TBN, WM, WN, OCC, false, false, true>(g, st) : launch_epi<TBM, TBN, WM, WN, OCC, false, false, false>(g, st);
}

// 256x256 tiles only for 16-B aligned operands with at least one K-contiguous side
template <int TBM, int TBN, int WM, int WN, int OCC>
int launch_tile_vec(const K3mGemm& g, bool ak, bool bk, hipStream_t st) {
  if (ak && bk) return launch_epi<TBM, TBN, WM, WN, OCC, true, true, true>(g, st);
  if (ak) return launch_epi<TBM, TBN, WM, WN, OCC, true, false, true>(g, st);
  return launch_epi<TBM, TBN, WM, WN, OCC, false, true, true>(g, st);
}

template <int TBM, int TBN, int WM, int WN, int BK, int OCC, bool AK, bool BK_, bool PIPE = true>
int launch_x6_epi(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  switch (g.epilogue) {
#define K3M_GEMM_CASE(E)                                                                                          \
    case E:                                                                                                       \
      hipLaunchKernelGGL((k3m_x6::gemm_x6_kernel<TBM, TBN, WM, WN, BK, AK, BK_, true, E, OCC, PIPE>), grid,           \
                         dim3(64 * WM * WN),                                                                      \
                         0, st, g);                                                                               \
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

template <int TBM, int TBN, int WM, int WN, int BK, int OCC>
int launch_x6(const K3mGemm& g, bool ak, bool bk, hipStream_t st) {
  if (ak && bk) return launch_x6_epi<TBM, TBN, WM, WN, BK, OCC, true, true>(g, st);
  if (ak) return launch_x6_epi<TBM, TBN, WM, WN, BK, OCC, true, false>(g, st);
  if (bk) return launch_x6_epi<TBM, TBN, WM, WN, BK, OCC, false, true>(g, st);
  // both operands MN-contiguous (the weight gradients dY^T.X): the single-register-set loop measured
  // 5-7% faster than the two-set pipeline on these shapes (scripts/lab, best of passes)
  if constexpr (TBM == 256) return launch_x6_epi<TBM, TBN, WM, WN, BK, OCC, false, false, false>(g, st);
  else return launch_x6_epi<TBM, TBN, WM, WN, BK, OCC, false, false>(g, st);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

long long nblocks(const K3mGemm& g, int bm, int bn) {
  return (long long)((g.m + bm - 1) / bm) * ((g.n + bn - 1) / bn) * (g.splitk > 1 ? g.splitk : 1);
}

// 256x256x16 vs 256x128x32 x6 tiles: the larger tile halves the split VALU and the LDS fragment
// reads per MFMA and ran 7-11 % faster per block-wave on the K3M shapes (scripts/lab,
// profiles/r1_gemm_lab_x6_v4.txt), but has half the blocks: take it unless it costs a whole extra wave
// of 256 blocks (the 8,192-row co-attention FFN: 384 blocks = 1.5 waves vs 768 = 3).
// K3M_X6_TILE256 (bitmask, default 15): 1 forward (both K-contiguous), 2 dgrad (B MN-contiguous),
// 4 weight gradients (both MN-contiguous), 8 the grouped launch; 0 keeps every GEMM on 256x128.
const int kTile256 = k3m_env_int("K3M_X6_TILE256", 15);

int tile256_class(bool ak, bool bk) { return ak && bk ? 1 : ak ? 2 : !bk ? 4 : 0; }

bool prefer_256x256(const K3mGemm& g) {
  if (!(kTile256 & tile256_class(g.a_trans == 0, g.b_trans == 1))) return false;
  const long long w128 = (nblocks(g, 256, 128) + 255) / 256, w256 = (nblocks(g, 256, 256) + 255) / 256;
  return 2.0 * (double)w256 / 1.08 < (double)w128;
}

// Persistent x6 walk (gemm_x6p.hip) for the 256-row tiles: K3M_X6_PERSIST=0 restores one workgroup per
// tile (A/B knob).
const int kPersist = k3m_env_int("K3M_X6_PERSIST", 1);
// fewest 256x128 tiles for the persistent 256-row walk (smaller grids take 128x128 / 64x64 tiles): 100 instead of
// 200 moves the 2,304-2,368-row co-attention GEMMs off one-workgroup-per-CU 128x128 tiles, fp32 step +0.4-1.1 %
// (profiles/r3_ab_x6_pmin.txt; A/B knob K3M_X6_P_MIN)
const int kPersistMin = k3m_env_int("K3M_X6_P_MIN", 100);
// fewest 128x128 tiles for the 128x128 x6 kernel; smaller grids take 64x64 tiles (A/B knob; 50 measured equal,
// profiles/r3_ab_knobs_recheck.txt)
const int kT128Min = k3m_env_int("K3M_X6_T128_MIN", 200);

int cu_count() {
  static int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return 256;
    return cus;
  }();
  return n;
}

}  // namespace

int k3m_x6_persistent_launch(const k3m_x6::GemmGroup& grp, bool t256, bool ak, bool bk, int cus, hipStream_t st);
int k3m_x6_variant_launch(const K3mGemm& g, int variant, hipStream_t st);   // lab tiles (gemm_x6p.hip)
namespace {
const int kVariant = k3m_env_int("K3M_X6_VARIANT", 0);
}  // namespace

namespace {
// one GEMM as a persistent group of one
int launch_x6_persistent_one(const K3mGemm& g, bool t256, bool ak, bool bk, hipStream_t st) {
  k3m_x6::GemmGroup grp = {};
  grp.g[0] = g;
  grp.start[0] = 0;
  grp.start[1] = (int)nblocks(g, 256, t256 ? 256 : 128);
  grp.count = 1;
  return k3m_x6_persistent_launch(grp, t256, ak, bk, cu_count(), st);
}
}  // namespace

int k3m_gemm_bf16_impl(const K3mGemm& g, hipStream_t st, bool slabs_only, bool colsum);  // gemm_bf16.hip
int k3m_gemm_bf16_grouped_impl(const K3mGemm* gs, int count, hipStream_t st, bool* handled, const bool* slabs_only);
// (the grouped problems carry their COLSUM_SLABS request as a non-null ws with splitk <= 1)

static int gemm_f32_dispatch(const K3mGemm& g, const K3mGemm& gr, int epi_out, bool slabs_only, hipStream_t st);

extern "C" int k3m_gemm(const K3mGemm* gp, hipStream_t st) {
  if (!gp) return K3M_EINVAL;
  const bool slabs_only = (gp->epilogue & K3M_GEMM_SLABS_ONLY) != 0;
  const bool colsum = (gp->epilogue & K3M_GEMM_COLSUM_SLABS) != 0;
  K3mGemm gl = *gp;
  gl.epilogue &= ~(K3M_GEMM_SLABS_ONLY | K3M_GEMM_COLSUM_SLABS);
  // kernels read a non-split ws as the COLSUM_SLABS request
  if (!colsum && gl.splitk <= 1) gl.ws = nullptr;
  const K3mGemm& g = gl;
  K3M_ARG(!slabs_only || (g.splitk > 1 && g.ldc == g.n));
  K3M_ARG(!colsum || (g.epilogue == K3M_EPI_DGELU && g.splitk <= 1 && g.beta == 0.f && g.ws));
  K3M_ARG(g.m >= 0 && g.n >= 0 && g.k >= 0);
  if (g.m == 0 || g.n == 0) return 0;
  K3M_ARG(g.dtype == K3M_F32 || g.dtype == K3M_BF16);
  K3M_ARG(g.c_dtype == K3M_F32 || (g.dtype == K3M_BF16 && g.c_dtype == K3M_BF16));
  K3M_ARG(g.a && g.b && g.c);
  K3M_ARG(g.splitk <= 1 || ((g.epilogue == K3M_EPI_NONE || !slabs_only) && g.ws));
  K3M_ARG(g.epilogue == K3M_EPI_NONE || g.epilogue == K3M_EPI_DGELU || g.bias);
  K3M_ARG((g.epilogue != K3M_EPI_BIAS_GELU && g.epilogue != K3M_EPI_DGELU) || g.aux);
  K3M_ARG(g.f32_algo == K3M_F32_SPLIT_BF16X6 || g.f32_algo == K3M_F32_MFMA_F32);
  K3M_ARG(g.a_planes == 0 && g.b_planes == 0);   // reserved (the round-3 pre-split lab path, scripts/lab/r3)
  if (g.dtype == K3M_BF16) {
    K3M_ARG(g.splitk <= 1 || g.epilogue == K3M_EPI_NONE);
    return k3m_gemm_bf16_impl(g, st, slabs_only, colsum);
  }
  // a split problem computes raw slabs (epilogue NONE); its epilogue runs in splitk_reduce_kernel
  const int epi_out = g.epilogue;
  K3mGemm gsplit = g;
  if (g.splitk > 1) gsplit.epilogue = K3M_EPI_NONE;
  return gemm_f32_dispatch(gsplit, g, epi_out, slabs_only, st);
}

namespace {
// fp32 C[m, n] (n <= 8) = alpha A B + beta C for the skinny products of the step (the 5-column image-location
// weight gradient, tn 1024 x 5 x 2,368): exact fp32 FMAs, 64 rows per workgroup.  Split over k (ops.small_splitk)
// each grid row y computes the k-slice y into its fp32 slab (ws + y m n, reduced in slab order with the epilogue by
// splitk_reduce_kernel), so the 16 row blocks of that product fill 256 workgroups; inside a workgroup the slice is
// dealt to the 4 waves in contiguous ranges and reduced through LDS in wave order (deterministic).  The 64 x 64
// tile kernels gave such a product 1-2 % of one CU's MFMA rate (64 us); unsplit, 16 workgroups were latency-bound.
constexpr int SKINNY_N = 8;
constexpr int SKINNY_U = 8;   // k values per thread in flight
constexpr int SKINNY_W = 4;   // waves per workgroup
__global__ __launch_bounds__(64 * SKINNY_W) void gemm_skinny_kernel(K3mGemm g) {
  __shared__ float red[SKINNY_W][64][SKINNY_N + 1];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = blockIdx.x * 64 + lane;
  const int mc = min(m, g.m - 1);   // clamped row: every lane loads, the store is masked
  const float* A = static_cast<const float*>(g.a);
  const float* B = static_cast<const float*>(g.b);
  const int splits = max(g.splitk, 1);
  const int kslice = (g.k + splits - 1) / splits;
  const int ks0 = blockIdx.y * kslice, ks1 = min(g.k, ks0 + kslice);
  float acc[SKINNY_N];
#pragma unroll
  for (int j = 0; j < SKINNY_N; ++j) acc[j] = 0.f;
  // wave w owns the contiguous k range [k0, k1) of the slice; SKINNY_U loads of A issued before their FMAs
  const int per = (ks1 - ks0 + SKINNY_W - 1) / SKINNY_W, k0 = ks0 + w * per, k1 = min(ks1, k0 + per);
  for (int kb = k0; kb < k1; kb += SKINNY_U) {
    float av[SKINNY_U];
#pragma unroll
    for (int u = 0; u < SKINNY_U; ++u) {
      const int k = min(kb + u, k1 - 1);
      const float x = g.a_trans ? A[(long long)k * g.lda + mc] : A[(long long)mc * g.lda + k];
      av[u] = kb + u < k1 ? x : 0.f;
    }
#pragma unroll
    for (int u = 0; u < SKINNY_U; ++u) {
      const int k = min(kb + u, k1 - 1);   // wave-uniform: B's row is a broadcast (scalar) load
#pragma unroll
      for (int j = 0; j < SKINNY_N; ++j)
        if (j < g.n) acc[j] = fmaf(av[u], g.b_trans ? B[(long long)j * g.ldb + k] : B[(long long)k * g.ldb + j], acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < SKINNY_N; ++j) red[w][lane][j] = acc[j];
  __syncthreads();
  if (w == 0 && m < g.m) {
    const bool slab = splits > 1;
    float* C = slab ? static_cast<float*>(g.ws) + (long long)blockIdx.y * g.m * g.n : static_cast<float*>(g.c);
    const long long ldc = slab ? g.n : g.ldc;
#pragma unroll
    for (int j = 0; j < SKINNY_N; ++j) {
      if (j >= g.n) break;
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < SKINNY_W; ++q) s += red[q][lane][j];
      float* cp = C + (long long)m * ldc + j;
      if (slab) {
        *cp = s;
      } else {
        float o = g.alpha * s;
        if (g.beta != 0.f) o += g.beta * *cp;
        *cp = o;
      }
    }
  }
}
}  // namespace

// the tile kernel for one fp32 problem (launch only; the split-K reduction is the caller's)
static int gemm_f32_tiles(const K3mGemm& g, hipStream_t st) {
  // A: K-contiguous iff a_trans == 0; B: K-contiguous iff b_trans == 1
  int rc;
  const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
  const bool av = aligned16(g.a) && (g.lda % 4 == 0) && ((ak ? g.k : g.m) % 4 == 0);
  const bool bv = aligned16(g.b) && (g.ldb % 4 == 0) && ((bk ? g.k : g.n) % 4 == 0);
  const bool vec = av && bv;
  // tile choice: the largest tile that still fills the 256 CUs; small co-attention GEMMs
  // (2,304-8,192 rows) otherwise leave CUs idle
  if (vec && g.f32_algo == K3M_F32_SPLIT_BF16X6) {
    const int vrc = kVariant ? k3m_x6_variant_launch(g, kVariant, st) : -1;
    if (vrc >= 0) {
      rc = vrc;
    } else if (g.splitk > 1 && g.k <= 256LL * g.splitk && nblocks(g, 256, 128) * g.splitk < 256) {
      // a small problem split over k (ops.small_splitk): the 64 x 64 tile, one k-slice per grid row
      rc = launch_x6<64, 64, 2, 2, 16, 2>(g, ak, bk, st);
    } else if (g.splitk > 1 || nblocks(g, 256, 128) >= kPersistMin) {
      if (kPersist) {
        rc = launch_x6_persistent_one(g, (ak || !bk) && prefer_256x256(g), ak, bk, st);
      } else if ((ak || !bk) && prefer_256x256(g)) {
        // wave layout per operand layout (scripts/lab, best of passes): 4x2 for the forward (both
        // K-contiguous), 2x4 when B is MN-contiguous (dgrad, and the single-register-set loop for
        // the weight gradients)
        if (ak && bk) rc = launch_x6_epi<256, 256, 4, 2, 16, 1, true, true>(g, st);
        else if (ak) rc = launch_x6_epi<256, 256, 2, 4, 16, 1, true, false>(g, st);
        else rc = launch_x6_epi<256, 256, 2, 4, 16, 1, false, false, false>(g, st);
      } else {
        rc = launch_x6<256, 128, 4, 2, 32, 1>(g, ak, bk, st);
      }
    }
    else if (nblocks(g, 128, 128) >= kT128Min) rc = launch_x6<128, 128, 2, 2, 32, 1>(g, ak, bk, st);
    // 64x64 runs at BK = 16: the BK = 32 build of this tile (ROCm 7.2 hipcc) returned C = alpha*AB
    // without the beta*C term for scattered 16-lane groups (scripts/lab/gemm_dbg.hip reproduces it;
    // tests/test_gpu_gemm_x6.py::test_x6_beta_all_tiles guards every tile path)
    else rc = launch_x6<64, 64, 2, 2, 16, 2>(g, ak, bk, st);
  } else if (vec && g.splitk <= 1 && (ak || bk) && nblocks(g, 256, 256) >= 200) rc = launch_tile_vec<256, 256, 2, 4, 1>(g, ak, bk, st);
  else if (g.splitk > 1 || nblocks(g, 128, 128) >= 384) rc = launch_tile<128, 128, 2, 2, 2>(g, ak, bk, vec, st);
  else if (nblocks(g, 64, 128) >= 384) rc = launch_tile<64, 128, 2, 2, 2>(g, ak, bk, vec, st);
  else rc = launch_tile<64, 64, 2, 2, 2>(g, ak, bk, vec, st);
  return rc;
}

static int gemm_f32_dispatch(const K3mGemm& g, const K3mGemm& gr, int epi_out, bool slabs_only, hipStream_t st) {
  // g: the problem as launched (epilogue NONE when split); gr: as requested (for the split-K reduction)
  int rc;
  if (g.n <= SKINNY_N && (g.splitk > 1 || epi_out == K3M_EPI_NONE) && g.k >= 256) {
    hipLaunchKernelGGL(gemm_skinny_kernel, dim3(k3m_cdiv(g.m, 64), std::max(g.splitk, 1)), dim3(64 * SKINNY_W), 0,
                       st, g);
    rc = 0;
  } else {
    rc = gemm_f32_tiles(g, st);
  }
  if (rc) return rc;
  K3M_CHECK_LAUNCH();
  if (g.splitk > 1 && !slabs_only) {
    const long long total = (long long)g.m * g.n;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, g.ws, g.splitk, g.m, g.n,
                       static_cast<float*>(g.c), g.ldc, g.alpha, g.beta, epi_out, gr.bias, static_cast<float*>(gr.aux),
                       gr.ldaux);
    K3M_CHECK_LAUNCH();
  }
  return 0;
}

// ------------------------------------------------------------------ grouped launch
namespace {

template <int TBN, int WM, int WN, int BK, bool AK, bool BK_, bool PIPE>
int launch_grouped_epi(const k3m_x6::GemmGroup& grp, int epi, hipStream_t st) {
  const dim3 grid(grp.start[grp.count]);
  switch (epi) {
#define K3M_GROUP_CASE(E)                                                                                          \
    case E:                                                                                                        \
      hipLaunchKernelGGL((k3m_x6::gemm_x6_grouped_kernel<256, TBN, WM, WN, BK, AK, BK_, true, E, 1, PIPE>), grid,     \
                         dim3(512), 0, st, grp);                                                                   \
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

}  // namespace

extern "C" int k3m_gemm_grouped(const K3mGemm* gs_in, int count, hipStream_t st) {
  K3M_ARG(gs_in && count >= 0 && count <= k3m_x6::GROUP_MAX);
  if (count == 0) return 0;
  // K3M_GEMM_SLABS_ONLY per problem: stripped here, remembered for the split-K reductions below
  K3mGemm gs[k3m_x6::GROUP_MAX];
  bool slabs_only[k3m_x6::GROUP_MAX], colsum[k3m_x6::GROUP_MAX];
  for (int i = 0; i < count; ++i) {
    gs[i] = gs_in[i];
    slabs_only[i] = (gs[i].epilogue & K3M_GEMM_SLABS_ONLY) != 0;
    colsum[i] = (gs[i].epilogue & K3M_GEMM_COLSUM_SLABS) != 0;
    gs[i].epilogue &= ~(K3M_GEMM_SLABS_ONLY | K3M_GEMM_COLSUM_SLABS);
    if (!colsum[i] && gs[i].splitk <= 1) gs[i].ws = nullptr;
    K3M_ARG(!slabs_only[i] || (gs[i].splitk > 1 && gs[i].ldc == gs[i].n));
    K3M_ARG(!colsum[i] || (gs[i].epilogue == K3M_EPI_DGELU && gs[i].splitk <= 1 && gs[i].beta == 0.f && gs[i].ws));
  }
  // one template for the whole group: same layout, epilogue, dtype, algorithm, 16-B aligned operands
  const K3mGemm& g0 = gs[0];
  if (g0.dtype == K3M_BF16) {   // bf16 encoder: the large-tile grouped kernel (gemm_bf16.hip) when eligible
    bool handled = false;
    const int r = k3m_gemm_bf16_grouped_impl(gs, count, st, &handled, slabs_only);
    if (handled || r) return r;
  }
  bool same = g0.dtype == K3M_F32 && g0.c_dtype == K3M_F32 && g0.f32_algo == K3M_F32_SPLIT_BF16X6;
  k3m_x6::GemmGroup grp = {};
  bool live_slabs[k3m_x6::GROUP_MAX] = {};
  int nb = 0, live = 0;
  long long nb128 = 0, nb256 = 0;
  for (int i = 0; i < count && same; ++i) {
    const K3mGemm& g = gs[i];
    same = g.a_trans == g0.a_trans && g.b_trans == g0.b_trans && g.epilogue == g0.epilogue && g.dtype == g0.dtype &&
           g.c_dtype == g0.c_dtype && g.f32_algo == g0.f32_algo && g.a_planes == 0 && g.b_planes == 0;
    const bool ak = g.a_trans == 0, bk = g.b_trans == 1;
    same = same && aligned16(g.a) && (g.lda % 4 == 0) && ((ak ? g.k : g.m) % 4 == 0) && aligned16(g.b) &&
           (g.ldb % 4 == 0) && ((bk ? g.k : g.n) % 4 == 0);
    if (g.m == 0 || g.n == 0) continue;
    live_slabs[live] = slabs_only[i];
    grp.g[live] = g;
    nb128 += nblocks(g, 256, 128);
    nb256 += nblocks(g, 256, 256);
    ++live;
  }
  if (!same) {   // not one template: launch each on its own
    for (int i = 0; i < count; ++i) {
      K3mGemm gi = gs[i];
      if (slabs_only[i]) gi.epilogue |= K3M_GEMM_SLABS_ONLY;
      if (colsum[i]) gi.epilogue |= K3M_GEMM_COLSUM_SLABS;
      const int rc = k3m_gemm(&gi, st);
      if (rc) return rc;
    }
    return 0;
  }
  for (int i = 0; i < live; ++i) {
    const K3mGemm& g = grp.g[i];
    K3M_ARG(g.a && g.b && g.c && g.k >= 0);
    K3M_ARG(g.splitk <= 1 || (g.epilogue == K3M_EPI_NONE && g.ws));
    K3M_ARG(g.epilogue == K3M_EPI_NONE || g.epilogue == K3M_EPI_DGELU || g.bias);   // (ws of a non-split
                                                                                    // problem: its colsum slabs)
    K3M_ARG((g.epilogue != K3M_EPI_BIAS_GELU && g.epilogue != K3M_EPI_DGELU) || g.aux);
  }
  if (live == 0) return 0;
  k3m_lpt_order(grp.g, live_slabs, live);
  const bool ak = g0.a_trans == 0, bk = g0.b_trans == 1;
  // same tile rule as k3m_gemm, over the whole grid (prefer_256x256)
  const long long w128 = (nb128 + 255) / 256, w256 = (nb256 + 255) / 256;
  const bool t256 = (kTile256 & 8) && (kTile256 & tile256_class(ak, bk)) && 2.0 * (double)w256 / 1.08 < (double)w128;
  for (int i = 0; i < live; ++i) {
    grp.start[i] = nb;
    nb += (int)nblocks(grp.g[i], 256, t256 ? 256 : 128);
  }
  grp.start[live] = nb;
  grp.count = live;
  int rc;
  if (kPersist) {
    rc = k3m_x6_persistent_launch(grp, t256, ak, bk, cu_count(), st);
  } else if (t256) {
    if (ak && bk) rc = launch_grouped_epi<256, 4, 2, 16, true, true, true>(grp, g0.epilogue, st);
    else if (ak) rc = launch_grouped_epi<256, 2, 4, 16, true, false, true>(grp, g0.epilogue, st);
    else rc = launch_grouped_epi<256, 2, 4, 16, false, false, false>(grp, g0.epilogue, st);
  } else if (ak && bk) rc = launch_grouped_epi<128, 4, 2, 32, true, true, true>(grp, g0.epilogue, st);
  else if (ak) rc = launch_grouped_epi<128, 4, 2, 32, true, false, true>(grp, g0.epilogue, st);
  else if (bk) rc = launch_grouped_epi<128, 4, 2, 32, false, true, true>(grp, g0.epilogue, st);
  else rc = launch_grouped_epi<128, 4, 2, 32, false, false, false>(grp, g0.epilogue, st);
  if (rc) return rc;
  K3M_CHECK_LAUNCH();
  for (int i = 0; i < live; ++i) {
    const K3mGemm& g = grp.g[i];
    if (g.splitk > 1 && !live_slabs[i]) {
      const long long total = (long long)g.m * g.n;
      const int blocks = (int)std::min<long long>((total + 255) / 256, 2048);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, g.ws, g.splitk, g.m, g.n,
                         static_cast<float*>(g.c), g.ldc, g.alpha, g.beta, (int)K3M_EPI_NONE, (const float*)nullptr,
                         (float*)nullptr, 0LL);
      K3M_CHECK_LAUNCH();
    }
  }
  return 0;
}
