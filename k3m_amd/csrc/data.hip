// GPU side of the K3M data path: the global-region collation of ConceptCapLoaderTrain_struc.__iter__
// (concept_cap_dataset_struc.py:381-397) fused with mask_region's feature zeroing (:913-915).
//
// For sample b:  feat'[r] = zero_feat[b][r] ? 0 : feat[b][r]                     (masked regions)
//                out[b][0] = (float)((double)(feat'[0] + feat'[1] + ... ) / cnt_b)  (global region)
//                out[b][1 + r] = feat'[r]
// cnt_b = #{r : masked_label[b][r] == 0} over all R slots (0 -> 1).  The fp32 row sum runs in row
// order and the division in double, as numpy's np.sum(float32, axis=1) / int64 count does, so the
// result is bit-identical to the reference's collation.  HBM-bound: one read and one write of the
// features (4 B·R·F read, 4 B·(R+1)·F written per sample), 16-B vectors along F.
#include "common.h"

namespace {

constexpr int COLL_THREADS = 64;   // one wave per block: F=2048 x B=64 gives 512 waves for 256 CUs
constexpr int COLL_BATCH = 36;     // row loads in flight per lane (all 36 regions of the driver)

__global__ __launch_bounds__(COLL_THREADS) void collate_regions_kernel(const float* __restrict__ feat, long long ldb,
                                                                       const uint8_t* __restrict__ zero_feat,
                                                                       const uint8_t* __restrict__ masked_label,
                                                                       const int32_t* __restrict__ divisor,
                                                                       int R, int F, float* __restrict__ out) {
  const int b = blockIdx.y;
  const uint8_t* zf = zero_feat ? zero_feat + (long long)b * R : nullptr;
  double cnt;
  if (divisor) {
    cnt = (double)divisor[b];   // num_boxes as given (0 -> inf / nan, as numpy)
  } else {
    const uint8_t* ml = masked_label + (long long)b * R;
    int c = 0;   // every lane counts (R is small; the flags are one cache line per sample)
    for (int r = 0; r < R; ++r) c += ml[r] == 0;
    cnt = (double)(c == 0 ? 1 : c);
  }
  const int f4 = blockIdx.x * COLL_THREADS + threadIdx.x;   // float4 column
  if (4 * f4 >= F) return;
  const float* src = feat + (long long)b * ldb + 4 * f4;
  float* dst = out + (long long)b * (R + 1) * F + 4 * f4;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  for (int r0 = 0; r0 < R; r0 += COLL_BATCH) {
    floatx4 v[COLL_BATCH];
#pragma unroll
    for (int j = 0; j < COLL_BATCH; ++j)
      if (r0 + j < R) v[j] = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(src + (long long)(r0 + j) * F));
#pragma unroll
    for (int j = 0; j < COLL_BATCH; ++j) {
      const int r = r0 + j;
      if (r < R) {
        if (zf && zf[r]) v[j] = floatx4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<floatx4*>(dst + (long long)(r + 1) * F) = v[j];
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] = r == 0 ? v[j][e] : __fadd_rn(s[e], v[j][e]);   // row order, fp32
      }
    }
  }
  floatx4 g;
#pragma unroll
  for (int e = 0; e < 4; ++e) g[e] = (float)((double)s[e] / cnt);
  *reinterpret_cast<floatx4*>(dst) = g;
}

}  // namespace

extern "C" int k3m_collate_regions(const float* feat, long long ldb, const uint8_t* zero_feat,
                                   const uint8_t* masked_label, const int32_t* divisor, int B, int R, int F, float* out,
                                   hipStream_t st) {
  K3M_ARG(feat && out && (masked_label || divisor) && B >= 0 && R > 0 && F > 0 && F % 4 == 0 && ldb >= (long long)R * F);
  K3M_ARG((reinterpret_cast<uintptr_t>(feat) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 && ldb % 4 == 0);
  if (B == 0) return 0;
  dim3 grid((F / 4 + COLL_THREADS - 1) / COLL_THREADS, B);
  hipLaunchKernelGGL(collate_regions_kernel, grid, dim3(COLL_THREADS), 0, st, feat, ldb, zero_feat, masked_label, divisor,
                     R, F, out);
  K3M_CHECK_LAUNCH();
  return 0;
}
