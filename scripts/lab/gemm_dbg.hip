// Debug harness: x6 kernels with beta != 0 (C read-modify-write) against an fp64 reference.
#include <cstdio>
#include <cstdlib>
#include <cmath>
#define K3M_F32_NS lab_f32
#define K3M_X6_NS lab_x6
#include "../../k3m_amd/csrc/gemm_x6_tile.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_kernel(float* p, long long n, uint64_t seed, float scale) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = scale * (2.f * k3m_uniform(seed, i) - 1.f);
}
// C64 = alpha * A.B + beta * C0   (A [m,k] row-major, B [k,n] row-major)
__global__ void ref64_kernel(const float* a, const float* b, const float* c0, int m, int n, int k, float alpha, float beta, double* c) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int l = 0; l < k; ++l) s += (double)a[(long long)i * k + l] * (double)b[(long long)l * n + j];
  c[(long long)i * n + j] = alpha * s + beta * (double)c0[(long long)i * n + j];
}
__global__ void count_bad(const float* c, const double* r, long long n, double tol, int* cnt, int* first) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    if (fabs((double)c[i] - r[i]) > tol) { if (atomicAdd(cnt, 1) == 0) *first = (int)i; }
}

template <int TBM, int TBN, int WM, int WN, int BK, int OCC, int EPI>
void launch(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  hipLaunchKernelGGL((lab_x6::gemm_x6_kernel<TBM, TBN, WM, WN, BK, true, false, true, EPI, OCC>), dim3(tm * tn), dim3(64 * WM * WN), 0, st, g);
}

__global__ void visit_kernel(int M, int N, int TBM, int TBN, int* visits) {
  int m0, n0;
  lab_f32::tile_coords<>(M, N, TBM, TBN, m0, n0);
  if (threadIdx.x == 0) atomicAdd(&visits[(m0 / TBM) * ((N + TBN - 1) / TBN) + n0 / TBN], 1);
}

template <int TBM, int TBN, int WM, int WN, int OCC, int EPI>
void launch_f32(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  hipLaunchKernelGGL((lab_f32::gemm_f32_kernel<TBM, TBN, WM, WN, true, false, true, EPI, OCC>), dim3(tm * tn), dim3(64 * WM * WN), 0, st, g);
}

int main() {
  const int m = 1000, n = 3072, k = 768;
  float *a, *b, *c0, *c; double* r; int* cnt;
  CK(hipMalloc(&a, (long long)m * k * 4)); CK(hipMalloc(&b, (long long)k * n * 4));
  CK(hipMalloc(&c0, (long long)m * n * 4)); CK(hipMalloc(&c, (long long)m * n * 4));
  CK(hipMalloc(&r, (long long)m * n * 8)); CK(hipMalloc(&cnt, 8));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, st, a, (long long)m * k, 1ull, 2.f);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, st, b, (long long)k * n, 2ull, 2.f);
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, st, c0, (long long)m * n, 3ull, 2.f);
  const float alpha = 0.5f, beta = 0.25f;
  hipLaunchKernelGGL(ref64_kernel, dim3(n / 256, m), dim3(256), 0, st, a, b, c0, m, n, k, alpha, beta, r);
  K3mGemm g = {};
  g.m = m; g.n = n; g.k = k; g.a_trans = 0; g.b_trans = 0; g.epilogue = 0; g.dtype = K3M_F32; g.c_dtype = K3M_F32;
  g.splitk = 1; g.lda = k; g.ldb = n; g.ldc = n; g.a = a; g.b = b; g.c = c; g.alpha = alpha; g.beta = beta;
  {
    int* visits; const int nt = 16 * 48;
    CK(hipMalloc(&visits, nt * 4)); CK(hipMemset(visits, 0, nt * 4));
    hipLaunchKernelGGL(visit_kernel, dim3(nt), dim3(64), 0, st, m, n, 64, 64, visits);
    int hv[16 * 48]; CK(hipMemcpy(hv, visits, nt * 4, hipMemcpyDeviceToHost));
    int bad = 0; for (int i = 0; i < nt; ++i) bad += hv[i] != 1;
    printf("tile_coords 64x64 grid: %d tiles visited != 1 time\n", bad);
  }
  struct V { const char* name; void (*f)(const K3mGemm&, hipStream_t); };
  V vs[] = {{"64x64 occ2 NONE", launch<64, 64, 2, 2, 32, 2, 0>}, {"64x64 occ1 NONE", launch<64, 64, 2, 2, 32, 1, 0>},
            {"128x128 occ1 NONE", launch<128, 128, 2, 2, 32, 1, 0>}, {"256x128 occ1 NONE", launch<256, 128, 4, 2, 32, 1, 0>},
            {"64x64 occ2 BIAS", launch<64, 64, 2, 2, 32, 2, 1>},
            {"64x64 bk16 occ2 NONE", launch<64, 64, 2, 2, 16, 2, 0>},
            {"f32 64x64 occ2 NONE", launch_f32<64, 64, 2, 2, 2, 0>},
            {"f32 128x128 occ2 NONE", launch_f32<128, 128, 2, 2, 2, 0>}};
  float* bias; CK(hipMalloc(&bias, n * 4)); CK(hipMemset(bias, 0, n * 4)); g.bias = bias;
  for (auto& v : vs) {
    int bad_total = 0;
    for (int rep = 0; rep < 20; ++rep) {
      CK(hipMemcpyAsync(c, c0, (long long)m * n * 4, hipMemcpyDeviceToDevice, st));
      v.f(g, st);
      CK(hipGetLastError());
      CK(hipMemsetAsync(cnt, 0, 8, st));
      hipLaunchKernelGGL(count_bad, dim3(1024), dim3(256), 0, st, c, r, (long long)m * n, 1e-3, cnt, cnt + 1);
      int h[2]; CK(hipMemcpy(h, cnt, 8, hipMemcpyDeviceToHost));
      if (h[0] && bad_total == 0) {
        printf("  %s rep %d: %d bad, first at row %d col %d\n", v.name, rep, h[0], h[1] / n, h[1] % n);
        float hc, hc0; double hr;
        CK(hipMemcpy(&hc, c + h[1], 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&hc0, c0 + h[1], 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&hr, r + h[1], 8, hipMemcpyDeviceToHost));
        const double ab = (hr - beta * (double)hc0) / alpha;
        printf("     c %.6f ref %.6f c0 %.6f AB %.6f | (c - beta*c0)/alpha %.6f  (c - alpha*AB)/beta %.6f\n", hc, hr, hc0, ab,
               (hc - beta * hc0) / alpha, (hc - alpha * ab) / beta);
      }
      bad_total += h[0];
    }
    printf("%-20s bad elements over 20 reps: %d\n", v.name, bad_total);
  }
  return 0;
}
