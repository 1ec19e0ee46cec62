// Initial-interactive fusion (pre_sampling_sequence, vilbert_k3m.py:2331-2374) and the pooling
// of the fused sequences (get_sequence_pooled_output_final :2404-2409).
//
// Layout: the three streams' ReLU outputs are packed as c[row, k*D + ch] (k = individual, cross1,
// cross2) — exactly torch.cat(feature_list, 2) — so the three gate scorers run as ONE GEMM
// against the contiguous [3D, 3D] weight view and the gate kernel reads score k of channel ch at
// column k*D + ch.
#include "common.h"

namespace {

template <typename T>
__global__ void relu_cat3_kernel(const T* x0, const T* x1, const T* x2, T* c, int rows, int d) {
  const long long n = (long long)rows * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / d, ch = e % d;
    T* o = c + r * 3 * d + ch;
    o[0] = from_f<T>(fmaxf(to_f(x0[e]), 0.f));
    o[d] = from_f<T>(fmaxf(to_f(x1[e]), 0.f));
    o[2 * d] = from_f<T>(fmaxf(to_f(x2[e]), 0.f));
  }
}

template <typename T>
__global__ void gate_fwd_kernel(const float* a, const T* c, const float* noise, float* ys, uint8_t* idx, T* out,
                                int rows, int d, uint64_t seed, uint64_t off) {
  const long long n = (long long)rows * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / d, ch = e % d;
    const long long b3 = r * 3 * d + ch;
    float z[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float g;
      if (noise) {
        g = noise[(r * 3 + k) * d + ch];
      } else {
        // gumbel(0,1) = -log(Exp(1)) = -log(-log(U))
        const float u = k3m_uniform(seed, off + (unsigned long long)(r * 3 + k) * d + ch);
        g = -logf(-logf(u));
      }
      z[k] = a[b3 + k * d] + g;
    }
    const float m = fmaxf(z[0], fmaxf(z[1], z[2]));
    const float e0 = expf(z[0] - m), e1 = expf(z[1] - m), e2 = expf(z[2] - m);
    const float inv = 1.f / (e0 + e1 + e2);
    const float y0 = e0 * inv, y1 = e1 * inv, y2 = e2 * inv;
    int k = 0;
    float best = y0;
    if (y1 > best) { best = y1; k = 1; }
    if (y2 > best) { k = 2; }
    ys[b3] = y0;
    ys[b3 + d] = y1;
    ys[b3 + 2 * d] = y2;
    idx[e] = (uint8_t)k;
    out[e] = c[b3 + k * d];
  }
}

template <typename T>
__global__ void gate_bwd_kernel(const T* dout, const float* a, const T* c, const float* ys, const uint8_t* idx, T* dc,
                                T* dpre, int rows, int d) {
  const long long n = (long long)rows * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / d, ch = e % d;
    const long long b3 = r * 3 * d + ch;
    const float g = to_f(dout[e]);
    const int k = idx[e];
    float dy[3], y[3];
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      y[q] = ys[b3 + q * d];
      dy[q] = g * to_f(c[b3 + q * d]);
      s += y[q] * dy[q];
      dc[b3 + q * d] = from_f<T>(q == k ? g : 0.f);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float av = a[b3 + q * d];
      dpre[b3 + q * d] = from_f<T>(y[q] * (dy[q] - s) * av * (1.f - av));
    }
  }
}

template <typename T>
__global__ void relu_split3_bwd_kernel(const T* dc, const T* c, T* dx0, T* dx1, T* dx2, int rows, int d, int acc) {
  const long long n = (long long)rows * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long r = e / d, ch = e % d;
    const long long b3 = r * 3 * d + ch;
    T* dx[3] = {dx0, dx1, dx2};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!dx[k]) continue;
      const float g = to_f(c[b3 + k * d]) > 0.f ? to_f(dc[b3 + k * d]) : 0.f;
      dx[k][e] = from_f<T>(acc ? to_f(dx[k][e]) + g : g);
    }
  }
}

template <typename T>
__global__ void mean3_kernel(const T* x0, const T* x1, const T* x2, T* out, long long n) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    out[e] = from_f<T>((to_f(x0[e]) + to_f(x1[e]) + to_f(x2[e])) / 3.f);
}
template <typename T>
__global__ void mean3_bwd_kernel(const T* dout, T* dx0, T* dx1, T* dx2, long long n, int acc) {
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float g = to_f(dout[e]) / 3.f;
    T* dx[3] = {dx0, dx1, dx2};
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (dx[k]) dx[k][e] = from_f<T>(acc ? to_f(dx[k][e]) + g : g);
  }
}

// out[s, ch] (+)= scale * mean_{l >= start} x[s, l, ch]
template <typename T>
__global__ void seq_mean_kernel(const T* x, int nseq, int len, int start, int d, float scale, float* out, int acc) {
  const long long n = (long long)nseq * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long s = e / d, ch = e % d;
    float a = 0.f;
    for (int l = start; l < len; ++l) a += to_f(x[(s * len + l) * d + ch]);
    const float v = scale * (a / (float)(len - start));
    out[e] = acc ? out[e] + v : v;
  }
}
template <typename T>
__global__ void seq_mean_bwd_kernel(const float* dout, int nseq, int len, int start, int d, float scale, T* dx) {
  const long long n = (long long)nseq * len * d;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long ch = e % d, sl = e / d;
    const long long s = sl / len, l = sl % len;
    if (l < start) continue;
    dx[e] = from_f<T>(to_f(dx[e]) + scale * dout[s * d + ch] / (float)(len - start));
  }
}

int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 8192); }

}  // namespace

#define DISPATCH_T(dtype, ...)      \
  if ((dtype) == K3M_F32) {         \
    using T = float;                \
    __VA_ARGS__;                    \
  } else if ((dtype) == K3M_BF16) { \
    using T = bf16_t;               \
    __VA_ARGS__;                    \
  } else {                          \
    return K3M_EINVAL;              \
  }

extern "C" int k3m_relu_cat3(const void* x0, const void* x1, const void* x2, void* c, int rows, int d, int dtype,
                             hipStream_t st) {
  K3M_ARG(x0 && x1 && x2 && c);
  const long long n = (long long)rows * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(relu_cat3_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)x0,
                                       (const T*)x1, (const T*)x2, (T*)c, rows, d));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_gate_fwd(const float* a, const void* c, const float* noise, float* ys, uint8_t* idx, void* out,
                            int rows, int d, uint64_t seed, uint64_t off, int dtype, hipStream_t st) {
  K3M_ARG(a && c && ys && idx && out);
  const long long n = (long long)rows * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(gate_fwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, a, (const T*)c, noise,
                                       ys, idx, (T*)out, rows, d, seed, off));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_gate_bwd(const void* dout, const float* a, const void* c, const float* ys, const uint8_t* idx,
                            void* dc, void* dpre, int rows, int d, int dtype, hipStream_t st) {
  K3M_ARG(dout && a && c && ys && idx && dc && dpre);
  const long long n = (long long)rows * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(gate_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)dout, a,
                                       (const T*)c, ys, idx, (T*)dc, (T*)dpre, rows, d));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_relu_split3_bwd(const void* dc, const void* c, void* dx0, void* dx1, void* dx2, int rows, int d,
                                   int accumulate, int dtype, hipStream_t st) {
  K3M_ARG(dc && c);
  const long long n = (long long)rows * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(relu_split3_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)dc,
                                       (const T*)c, (T*)dx0, (T*)dx1, (T*)dx2, rows, d, accumulate));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_mean3(const void* x0, const void* x1, const void* x2, void* out, long long n, int dtype,
                         hipStream_t st) {
  K3M_ARG(x0 && x1 && x2 && out);
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(mean3_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)x0,
                                       (const T*)x1, (const T*)x2, (T*)out, n));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_mean3_bwd(const void* dout, void* dx0, void* dx1, void* dx2, long long n, int accumulate, int dtype,
                             hipStream_t st) {
  K3M_ARG(dout);
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(mean3_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)dout,
                                       (T*)dx0, (T*)dx1, (T*)dx2, n, accumulate));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_seq_mean(const void* x, int nseq, int len, int start, int d, float scale, float* out,
                            int accumulate, int dtype, hipStream_t st) {
  K3M_ARG(x && out && len > start);
  const long long n = (long long)nseq * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(seq_mean_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)x, nseq,
                                       len, start, d, scale, out, accumulate));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_seq_mean_bwd(const float* dout, int nseq, int len, int start, int d, float scale, void* dx,
                                int dtype, hipStream_t st) {
  K3M_ARG(dout && dx && len > start);
  const long long n = (long long)nseq * len * d;
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(seq_mean_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, dout, nseq, len,
                                       start, d, scale, (T*)dx));
  K3M_CHECK_LAUNCH();
  return 0;
}
