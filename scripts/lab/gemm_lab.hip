// GEMM lab: times fp32 GEMM variants against the shipped k3m_gemm on the K3M shapes and checks
// every variant's output against it.  Build: scripts/lab/build_lab.sh ; run: scripts/lab/gemm_lab
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <string>
#include <cstring>
#define K3M_F32_NS lab_f32
#define K3M_X6_NS lab_x6
#include "../../k3m_amd/csrc/gemm_x6_tile.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_kernel(float* p, long long n, uint64_t seed, float scale) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = scale * (2.f * k3m_uniform(seed, i) - 1.f);
}

__global__ void reduce_kernel(const float* ws, int s, long long total, float* c) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    float a = 0.f;
    for (int k = 0; k < s; ++k) a += ws[k * total + e];
    c[e] += a;
  }
}

__global__ void maxdiff_kernel(const float* a, const float* b, long long n, float* out) {
  float m = 0.f, r = 0.f;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    m = fmaxf(m, fabsf(a[i] - b[i]));
    r = fmaxf(r, fabsf(b[i]));
  }
  m = wave_max(m); r = wave_max(r);
  if ((threadIdx.x & 63) == 0) { atomicMax((int*)out, __float_as_int(m)); atomicMax((int*)out + 1, __float_as_int(r)); }
}

using namespace lab_f32;

typedef void (*Launcher)(const K3mGemm&, hipStream_t);

template <int TBM, int TBN, int WM, int WN, int OCC, int EPI, bool AK, bool BK_>
void launch(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  hipLaunchKernelGGL((gemm_f32_kernel<TBM, TBN, WM, WN, AK, BK_, true, EPI, OCC>), grid, dim3(64 * WM * WN), 0, st, g);
}

template <int TBM, int TBN, int WM, int WN, int BK, int OCC, int EPI, bool AK, bool BK_, bool PIPE = true, int VAR = 0>
void launch_x6(const K3mGemm& g, hipStream_t st) {
  const int tm = (g.m + TBM - 1) / TBM, tn = (g.n + TBN - 1) / TBN;
  dim3 grid(tm * tn, g.splitk > 1 ? g.splitk : 1);
  hipLaunchKernelGGL((lab_x6::gemm_x6_kernel<TBM, TBN, WM, WN, BK, AK, BK_, true, EPI, OCC, PIPE, VAR>), grid, dim3(64 * WM * WN), 0, st, g);
}

// fp64 reference C = A.B^T (nt) for the accuracy check
__global__ void ref64_kernel(const float* a, const float* b, int m, int n, int k, double* c) {
  const int i = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int l = 0; l < k; ++l) s += (double)a[(long long)i * k + l] * (double)b[(long long)j * k + l];
  c[(long long)i * n + j] = s;
}
__global__ void err_kernel(const float* c, const double* r, long long n, double* out) {
  double e2 = 0, emax = 0, rmax = 0;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const double d = (double)c[i] - r[i];
    e2 += d * d; emax = fmax(emax, fabs(d)); rmax = fmax(rmax, fabs(r[i]));
  }
  atomicAdd(out, e2);
  atomicMax((unsigned long long*)(out + 1), __double_as_longlong(emax));
  atomicMax((unsigned long long*)(out + 2), __double_as_longlong(rmax));
}

struct Shape { const char* name; int kind; int m, n, k, epi, splitk; };  // kind 0 nt, 1 nn, 2 tn

void launch_shipped(const K3mGemm& g, hipStream_t st) { k3m_gemm(&g, st); }

template <int EPI, bool AK, bool BK_>
std::vector<std::pair<std::string, Launcher>> variants() {
  return {
      {"shipped in loop", launch_shipped},
      {"x6 256x128 4x2 bk32", launch_x6<256, 128, 4, 2, 32, 1, EPI, AK, BK_>},
      {"x6 256x128 bk32 nopipe", launch_x6<256, 128, 4, 2, 32, 1, EPI, AK, BK_, false>},
      {"x6 256x256 2x4 bk16", launch_x6<256, 256, 2, 4, 16, 1, EPI, AK, BK_>},
      {"x6 256x256 2x4 bk16 nopipe", launch_x6<256, 256, 2, 4, 16, 1, EPI, AK, BK_, false>},
      {"x6 256x256 4x2 bk16", launch_x6<256, 256, 4, 2, 16, 1, EPI, AK, BK_>},
  };
}

template <bool AK, bool BK_>
std::vector<std::pair<std::string, Launcher>> variants_epi(int epi) {
  switch (epi) {
    case 0: return variants<0, AK, BK_>();
    case 1: return variants<1, AK, BK_>();
    case 2: return variants<2, AK, BK_>();
    default: return variants<3, AK, BK_>();
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const char* only_shape = argc > 2 ? argv[2] : nullptr;    // substring filters (profiling runs)
  const char* only_var = argc > 3 ? argv[3] : nullptr;
  const bool skip_acc = only_shape != nullptr;
  const int M = 20992;
  std::vector<Shape> shapes = {
      {"sq4096 nt", 0, 4096, 4096, 4096, 0, 1},
      {"fwd ffn1 gelu", 0, M, 3072, 768, 2, 1},
      {"fwd qkv", 0, M, 2304, 768, 1, 1},
      {"fwd ffn2", 0, M, 768, 3072, 1, 1},
      {"fwd out", 0, M, 768, 768, 1, 1},
      {"dgrad ffn2 dgelu", 1, M, 3072, 768, 3, 1},
      {"dgrad ffn1", 1, M, 768, 3072, 0, 1},
      {"dgrad qkv", 1, M, 768, 2304, 0, 1},
      {"wgrad ffn1 s5", 2, 3072, 768, M, 0, 5},
      {"wgrad ffn2 s5", 2, 768, 3072, M, 0, 5},
      {"wgrad qkv s2", 2, 2304, 768, M, 0, 2},
      {"wgrad ffn1 s7", 2, 3072, 768, M, 0, 7},
      {"wgrad qkv s9", 2, 2304, 768, M, 0, 9},
      {"wgrad out s28", 2, 768, 768, M, 0, 28},
      {"wgrad out s8", 2, 768, 768, M, 0, 8},
      {"co pv ffn1 gelu", 0, 8192, 3072, 768, 2, 1},
      {"co txt ffn2", 0, 2304, 768, 3072, 1, 1},
  };
  hipStream_t st;
  CK(hipStreamCreate(&st));
  float *a, *b, *c, *c0, *aux, *bias, *ws, *dm;
  const long long big = 20992LL * 3072;
  CK(hipMalloc(&a, big * 4)); CK(hipMalloc(&b, big * 4)); CK(hipMalloc(&c, big * 4)); CK(hipMalloc(&c0, big * 4));
  CK(hipMalloc(&aux, big * 4)); CK(hipMalloc(&bias, 4096 * 4)); CK(hipMalloc(&ws, 8 * 3072LL * 3072 * 4));
  CK(hipMalloc(&dm, 8));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, a, big, 1ull, 1.f);
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, b, big, 2ull, 0.05f);
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, st, aux, big, 3ull, 2.f);
  hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, st, bias, 4096, 4ull, 0.5f);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  if (!skip_acc) {
    // accuracy vs fp64: C = A.B^T, m = n = 1024, k = 4096, A ~ U(-1,1), B ~ 0.05 U(-1,1)
    const int m = 1024, n = 1024, k = 4096;
    double *r64, *er;
    CK(hipMalloc(&r64, (long long)m * n * 8)); CK(hipMalloc(&er, 24));
    hipLaunchKernelGGL(ref64_kernel, dim3(n / 256, m), dim3(256), 0, st, a, b, m, n, k, r64);
    K3mGemm g = {};
    g.m = m; g.n = n; g.k = k; g.a_trans = 0; g.b_trans = 1; g.epilogue = 0; g.dtype = K3M_F32; g.c_dtype = K3M_F32;
    g.splitk = 1; g.lda = k; g.ldb = k; g.ldc = n; g.a = a; g.b = b; g.c = c; g.alpha = 1.f; g.beta = 0.f;
    auto report = [&](const char* name) {
      CK(hipMemsetAsync(er, 0, 24, st));
      hipLaunchKernelGGL(err_kernel, dim3(256), dim3(256), 0, st, c, r64, (long long)m * n, er);
      double h[3];
      CK(hipMemcpy(h, er, 24, hipMemcpyDeviceToHost));
      printf("accuracy vs fp64 (1024x1024x4096 nt)  %-24s rms err %.3e  max err %.3e  max|ref| %.3e\n", name,
             sqrt(h[0] / ((double)m * n)), h[1], h[2]);
    };
    k3m_gemm(&g, st); report("shipped f32 MFMA");
    launch<256, 256, 2, 4, 1, 0, true, true>(g, st); report("v2 f32 MFMA 256x256");
    launch_x6<256, 128, 4, 2, 32, 1, 0, true, true>(g, st); report("x6 bf16x6 256x128");
    launch_x6<128, 128, 2, 2, 16, 2, 0, true, true>(g, st); report("x6 bf16x6 128x128");
    fflush(stdout);
  }
  for (const Shape& s : shapes) {
    if (only_shape && !strstr(s.name, only_shape)) continue;
    K3mGemm g = {};
    g.m = s.m; g.n = s.n; g.k = s.k;
    g.a_trans = s.kind == 2; g.b_trans = s.kind == 0;
    g.epilogue = s.epi; g.dtype = K3M_F32; g.c_dtype = K3M_F32; g.splitk = s.splitk;
    g.lda = s.kind == 2 ? s.m : s.k;
    g.ldb = s.kind == 0 ? s.k : s.n;
    g.ldc = s.n; g.ldaux = s.n;
    g.a = a; g.b = b; g.c = c0; g.bias = bias; g.aux = aux; g.ws = ws;
    g.alpha = 1.f; g.beta = s.kind == 2 ? 1.f : 0.f;
    const double flops = 2.0 * s.m * s.n * s.k;
    const long long cn = (long long)s.m * s.n;
    // reference: the shipped kernel, from C = 0
    auto run_ref = [&]() { CK(hipMemsetAsync(c0, 0, cn * 4, st)); if (k3m_gemm(&g, st)) { printf("k3m_gemm failed\n"); exit(1); } };
    run_ref();
    CK(hipStreamSynchronize(st));
    // time the reference (memset excluded: measure only the gemm calls)
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) k3m_gemm(&g, st);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-18s m=%5d n=%5d k=%5d  %-22s %8.3f ms %7.1f TF/s\n", s.name, s.m, s.n, s.k, "shipped k3m_gemm", ms,
           flops / (ms * 1e-3) / 1e12);
    run_ref();
    std::vector<std::pair<std::string, Launcher>> vs =
        s.kind == 0 ? variants_epi<true, true>(s.epi) : s.kind == 1 ? variants_epi<true, false>(s.epi) : variants_epi<false, false>(s.epi);
    const int passes = getenv("LAB_PASSES") ? atoi(getenv("LAB_PASSES")) : 1;
    for (int pass = 0; pass < passes; ++pass)
    for (auto& v : vs) {
      if (only_var && !strstr(v.first.c_str(), only_var)) continue;
      K3mGemm gv = g;
      gv.c = c;
      auto go = [&]() {
        v.second(gv, st);
        if (gv.splitk > 1) hipLaunchKernelGGL(reduce_kernel, dim3(2048), dim3(256), 0, st, ws, gv.splitk, cn, c);
      };
      CK(hipMemsetAsync(c, 0, cn * 4, st));
      go();
      CK(hipGetLastError());
      CK(hipMemsetAsync(dm, 0, 8, st));
      hipLaunchKernelGGL(maxdiff_kernel, dim3(1024), dim3(256), 0, st, c, c0, cn, dm);
      float hd[2];
      CK(hipMemcpy(hd, dm, 8, hipMemcpyDeviceToHost));
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) go();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= reps;
      printf("%-18s m=%5d n=%5d k=%5d  %-22s %8.3f ms %7.1f TF/s  maxdiff %.2e (max|ref| %.2e)%s\n", s.name, s.m, s.n, s.k,
             v.first.c_str(), ms, flops / (ms * 1e-3) / 1e12, hd[0], hd[1], hd[0] > 1e-4 * hd[1] + 1e-5 ? "  MISMATCH" : "");
      fflush(stdout);
    }
  }
  return 0;
}
