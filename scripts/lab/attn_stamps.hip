// Lab: per-phase timing of the short attention kernels (k3m_amd/csrc/attention.hip built with
// K3M_ATTN_STAMPS: wave 0 of every workgroup stamps the 100 MHz wall clock at each phase boundary).
// Prints, per shape, the kernel's span, the mean workgroup lifetime, the mean duration of each
// phase and how many workgroups were resident on average (sum of lifetimes / span).
//   ./attn_stamps [shape index]         (the wide engine's shapes, fp32, dropout 0.1)
#define K3M_ATTN_STAMPS 8192
#include "../../k3m_amd/csrc/attention.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

static float* dev_rand(size_t n, unsigned seed) {
  std::vector<float> h(n);
  unsigned x = seed * 2654435761u + 1u;
  for (size_t i = 0; i < n; ++i) {
    x = x * 1664525u + 1013904223u;
    h[i] = ((x >> 8) * (1.0f / 16777216.0f)) * 2.f - 1.f;
  }
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

static void report(const char* what, int nblk, int nst, const char* const* names) {
  std::vector<unsigned long long> st(8 * 8192);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(k3m_attn_stamps), st.size() * sizeof(unsigned long long)));
  nblk = std::min(nblk, 8192);
  unsigned long long t0 = ~0ull, t1 = 0;
  double life = 0, ph[8] = {0};
  for (int b = 0; b < nblk; ++b) {
    const unsigned long long* s = &st[b * 8];
    t0 = std::min(t0, s[0]);
    t1 = std::max(t1, s[nst - 1]);
    life += double(s[nst - 1] - s[0]);
    for (int k = 0; k + 1 < nst; ++k) ph[k] += double(s[k + 1] - s[k]);
  }
  const double tick_us = 0.01;  // 100 MHz
  std::printf("  %s: span %.1f us, workgroup lifetime %.2f us, resident %.1f;  phases (us):", what,
              (t1 - t0) * tick_us, life / nblk * tick_us, life / double(t1 - t0));
  for (int k = 0; k + 1 < nst; ++k) std::printf(" %s %.2f", names[k], ph[k] / nblk * tick_us);
  std::printf("\n");
}

int main(int argc, char** argv) {
  const int only = argc > 1 ? std::atoi(argv[1]) : -1;
  const int shapes[][5] = {{128, 128, 128, 12, 64}, {128, 36, 36, 12, 64}, {128, 37, 37, 8, 128},
                           {64, 128, 37, 8, 128},  {64, 37, 128, 8, 128}};
  const char* fn[] = {"stage_QK", "S", "V(w0)", "softmax", "PV"};
  const char* fr[] = {"stage", "S(w0)", "softmax(w0)", "PV+store(w0)"};
  const char* br[] = {"stage+D", "dPd(w0)", "dS,dV,dK", "dS image+dQ"};
  const char* bn[] = {"stage+D", "dS", "K+dQ", "Pd+dV", "Q+dK"};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  for (int si = 0; si < (int)(sizeof(shapes) / sizeof(shapes[0])); ++si) {
    if (only >= 0 && si != only) continue;
    const int* sh = shapes[si];
    const int nseq = sh[0], lq = sh[1], lk = sh[2], nh = sh[3], hd = sh[4], D = nh * hd;
    float* q = dev_rand((size_t)nseq * lq * D, 1);
    float* k = dev_rand((size_t)nseq * lk * D, 2);
    float* v = dev_rand((size_t)nseq * lk * D, 3);
    float* dctx = dev_rand((size_t)nseq * lq * D, 4);
    float *mask, *ctx, *probs, *dq, *dk, *dv;
    CK(hipMalloc(&mask, (size_t)nseq * lk * 4));
    CK(hipMemset(mask, 0, (size_t)nseq * lk * 4));
    CK(hipMalloc(&ctx, (size_t)nseq * lq * D * 4));
    CK(hipMalloc(&probs, (size_t)nseq * nh * lq * lk * 4));
    CK(hipMalloc(&dq, (size_t)nseq * lq * D * 4));
    CK(hipMalloc(&dk, (size_t)nseq * lk * D * 4));
    CK(hipMalloc(&dv, (size_t)nseq * lk * D * 4));
    const float sc = 1.f / std::sqrt((float)hd);
    std::printf("nseq=%d lq=%d lk=%d nh=%d d=%d (%d workgroups)\n", nseq, lq, lk, nh, hd, nseq * nh);
    for (int it = 0; it < 4; ++it)
      if (k3m_attn_fwd(q, D, k, D, v, D, mask, ctx, D, probs, nseq, lq, lk, nh, hd, sc, 0.1f, 1, 0, K3M_F32, st)) return 1;
    CK(hipStreamSynchronize(st));
    const char* env = std::getenv("K3M_ATTN_FWD_REG");
    const bool reg = !(env && env[0] == '0') && (hd == 64 || hd == 96 || hd == 128) && ((lk + 31) & ~31) * hd <= 8192;
    if (reg) report("fwd(reg)", nseq * nh, 5, fr);
    else report("fwd", nseq * nh, 6, fn);
    for (int it = 0; it < 4; ++it)
      if (k3m_attn_bwd(dctx, D, ctx, D, q, D, k, D, v, D, probs, dq, dk, dv, D, D, D, nseq, lq, lk, nh, hd, sc, 0.1f, 1,
                       0, K3M_F32, st))
        return 1;
    CK(hipStreamSynchronize(st));
    const char* envb = std::getenv("K3M_ATTN_BWD_REG");
    const bool regb = !(envb && envb[0] == '0') && (hd == 64 || hd == 96 || hd == 128) && ((lq + 31) & ~31) * hd <= 8192 && lk > 64;
    if (regb) report("bwd(reg)", nseq * nh, 5, br);
    else report("bwd", nseq * nh, 6, bn);
    for (float* p : {q, k, v, dctx, mask, ctx, probs, dq, dk, dv}) CK(hipFree(p));
  }
  return 0;
}
