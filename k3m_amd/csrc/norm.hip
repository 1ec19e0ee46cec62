// Row kernels: LayerNorm (+dropout +residual) forward/backward, embeddings, column sums,
// elementwise helpers.  HBM-bound; one wave per row, 16-byte vectors along the row.
#include "common.h"

namespace {

constexpr int MAXV = 4;                // float4 chunks per lane: cols <= 64*4*4 = 1024
constexpr int K3M_COLSUM_SLABS = 256;  // row chunks of the column-sum first pass

template <typename T>
__device__ __forceinline__ floatx4 ld4(const T* p);
template <>
__device__ __forceinline__ floatx4 ld4<float>(const float* p) {
  return *reinterpret_cast<const floatx4*>(p);
}
template <>
__device__ __forceinline__ floatx4 ld4<bf16_t>(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return floatx4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                 __uint_as_float(u.y & 0xffff0000u)};
}
template <typename T>
__device__ __forceinline__ void st4(T* p, floatx4 v);
template <>
__device__ __forceinline__ void st4<float>(float* p, floatx4 v) {
  *reinterpret_cast<floatx4*>(p) = v;
}
template <>
__device__ __forceinline__ void st4<bf16_t>(bf16_t* p, floatx4 v) {
  uint2 u;
  u.x = (uint32_t)from_f<bf16_t>(v[0]).x | ((uint32_t)from_f<bf16_t>(v[1]).x << 16);
  u.y = (uint32_t)from_f<bf16_t>(v[2]).x | ((uint32_t)from_f<bf16_t>(v[3]).x << 16);
  *reinterpret_cast<uint2*>(p) = u;
}

// value as stored in T (identity for fp32, round-to-nearest bf16 otherwise)
template <typename T>
__device__ __forceinline__ floatx4 round4(floatx4 v) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = to_f(from_f<bf16_t>(v[q]));
  }
  return v;
}

// ------------------------------------------------------------------ LayerNorm forward
// NV = cols / 256 is a template parameter: with a runtime chunk count every load sat under a per-element
// condition, which hipcc compiles to a branch with a vmcnt(0) inside (each load its own round trip)
template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     T* __restrict__ y, T* __restrict__ xhat, float* __restrict__ rstd,
                                                     int rows, int cols, float eps, float p_in, float p_out,
                                                     uint64_t seed, uint64_t off_in, uint64_t off_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  constexpr int nv = NV;  // float4 chunks per lane
  const long long base = (long long)row * cols;
  floatx4 v[MAXV], r[MAXV];
  const T* rp = res ? res : x;   // every load unconditional and issued before the arithmetic
#pragma unroll
  for (int j = 0; j < nv; ++j) v[j] = ld4<T>(x + base + (lane + 64 * j) * 4);
#pragma unroll
  for (int j = 0; j < nv; ++j) r[j] = ld4<T>(rp + base + (lane + 64 * j) * 4);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    if (j < nv) {
      const int c = (lane + 64 * j) * 4;
      floatx4 a = v[j];
      if (p_in > 0.f) {
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] *= k3m_dropout_scale(seed, off_in + base + c + q, p_in);
      }
      if (res) a += r[j];
      v[j] = a;
      sum += a[0] + a[1] + a[2] + a[3];
    }
  }
  const float mean = wave_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (j < nv) {
      v[j] -= mean;
      sq += v[j][0] * v[j][0] + v[j][1] * v[j][1] + v[j][2] * v[j][2] + v[j][3] * v[j][3];
    }
  const float var = wave_sum(sq) / cols;
  const float rs = 1.0f / sqrtf(var + eps);
  if (lane == 0 && rstd) rstd[row] = rs;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (j < nv) {
      const int c = (lane + 64 * j) * 4;
      const floatx4 xh = v[j] * rs;
      if (xhat) st4<T>(xhat + base + c, xh);
      const floatx4 g = *reinterpret_cast<const floatx4*>(gamma + c);
      const floatx4 b = *reinterpret_cast<const floatx4*>(beta + c);
      floatx4 o = g * xh + b;
      if (p_out > 0.f) {
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] *= k3m_dropout_scale(seed, off_out + base + c + q, p_out);
      }
      st4<T>(y + base + c, o);
    }
}

// Column-slab reductions.  The LayerNorm backward and the column sums leave one fp32 slab of
// column partials per workgroup (ws[a][slab][c]); out_a[c] (+)= sum over slabs.  The slabs of MANY
// such reductions are summed by ONE batched launch (k3m_slab_reduce_batch, up to SLAB_JOBS jobs per
// launch): the engine's backward calls the _slabs forms and flushes the collected jobs once per
// encoder block, before the block is handed to the all-reduce (k3m_amd.ops.deferred_reductions);
// k3m_ln_bwd / k3m_colsum are the one-call forms (their own reduction right after the producer).  An in-kernel reduction (last
// arriving block sums, agent-scope hand-off) measured slower: its two acquire hops sit on the
// critical path of every call (scripts/lab/norm_fused_inkernel_slab_reduce.hip.txt).
// Each workgroup: 64 columns x 4 slab phases (phase p sums slabs p, p+4, ... with 8 loads in
// flight), phases combined in a fixed order: deterministic.
constexpr int SLAB_JOBS = 48;   // jobs per launch (kernel-argument block)
struct SlabJobs {
  const float* ws[SLAB_JOBS];
  float* out[SLAB_JOBS];
  int nslab[SLAB_JOBS];
  int cols[SLAB_JOBS];
  int accumulate[SLAB_JOBS];
  int vec[SLAB_JOBS];         // 1: few slabs, many columns (split-K slabs): 1,024 columns per workgroup
  int start[SLAB_JOBS + 1];   // first workgroup of each job: a 1-D grid with no idle workgroups when the
  int njobs;                  // jobs' widths differ (768 .. m*n of a split-K GEMM)
};
constexpr int SLAB_VEC_MAX = 64;   // vec mode: nslab <= this, cols % 4 == 0, 16-B aligned

__global__ __launch_bounds__(256) void slab_batch_kernel(SlabJobs jobs) {
  __shared__ float red[4][64];
  int j = 0;
  while (j + 1 < jobs.njobs && (int)blockIdx.x >= jobs.start[j + 1]) ++j;   // wave-uniform
  const int cols = jobs.cols[j], nslab = jobs.nslab[j];
  if (jobs.vec[j]) {
    // each thread: 4 consecutive columns (16-B loads), every slab in order 0..nslab-1
    const int c4 = (((int)blockIdx.x - jobs.start[j]) * 256 + (int)threadIdx.x) * 4;
    if (c4 >= cols) return;
    const float* src = jobs.ws[j] + c4;
    floatx4* o = reinterpret_cast<floatx4*>(jobs.out[j] + c4);
    const floatx4 old = *o;   // issued first, used last
    floatx4 acc = *reinterpret_cast<const floatx4*>(src);
    // slabs summed in order 0..nslab-1 (deterministic), loads issued up to 8 slabs ahead of the adds; the
    // last group is predicated (nslab is wave-uniform) rather than a one-load-at-a-time tail: split-K GEMMs
    // leave 2..9 slabs, and a serial tail kept one 16-B load per lane in flight (~4 TB/s)
    for (int k = 1; k < nslab; k += 8) {
      floatx4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < nslab) t[u] = *reinterpret_cast<const floatx4*>(src + (long long)(k + u) * cols);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (k + u < nslab) acc += t[u];
    }
    *o = jobs.accumulate[j] ? old + acc : acc;
    return;
  }
  const int cx = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = ((int)blockIdx.x - jobs.start[j]) * 64 + cx;
  const float* src = jobs.ws[j] + min(c, cols - 1);
  float s = 0.f;
  int k = ph;
  for (; k + 28 < nslab; k += 32) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(long long)(k + 4 * u) * cols];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; k < nslab; k += 4) s += src[(long long)k * cols];
  red[ph][cx] = s;
  __syncthreads();
  if (ph == 0 && c < cols) {
    const float t = (red[0][cx] + red[1][cx]) + (red[2][cx] + red[3][cx]);
    float* out = jobs.out[j];
    out[c] = jobs.accumulate[j] ? out[c] + t : t;
  }
}

// ------------------------------------------------------------------ LayerNorm backward
constexpr int LN_BWD_BLOCKS = K3M_LN_BWD_SLABS;

template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ xhat,
                                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                     T* __restrict__ dres, T* __restrict__ dx, float* __restrict__ ws,
                                                     int rows, int cols, float p_in, float p_out, uint64_t seed,
                                                     uint64_t off_in, uint64_t off_out, int acc_res, int want_sum) {
  // column partials of dgamma, dbeta and (want_sum) sum(dx): per wave in registers, then one
  // [3][cols] slab per block through LDS (summed by slab_batch_kernel)
  __shared__ float red[4][1024];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  constexpr int nv = NV;
  floatx4 gm[MAXV];
#pragma unroll
  for (int j = 0; j < nv; ++j) gm[j] = *reinterpret_cast<const floatx4*>(gamma + (lane + 64 * j) * 4);
  floatx4 pg[MAXV], pb[MAXV], px[MAXV];
#pragma unroll
  for (int j = 0; j < MAXV; ++j) {
    pg[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    pb[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    px[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  // two rows per wave and iteration: both rows' loads are in flight before either reduction
  // (one row at a time left this HBM-bound kernel at ~0.44 of the bandwidth roofline)
  const int S = gridDim.x * 4;
  for (int row0 = blockIdx.x * 4 + w; row0 < rows; row0 += 2 * S) {
    floatx4 dyl[2][MAXV], xh[2][MAXV], rr[2][MAXV];
    float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
    const T* rsrc = acc_res ? dres : dy;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // unconditional loads from a clamped row, zeroed after the load for a row past the end
      const int row = row0 + u * S;
      const bool ok = row < rows;
      const long long base = (long long)min(row, rows - 1) * cols;
#pragma unroll
      for (int j = 0; j < nv; ++j) {
        const int c = (lane + 64 * j) * 4;
        const floatx4 z = floatx4{0.f, 0.f, 0.f, 0.f};
        const floatx4 a = ld4<T>(dy + base + c), b = ld4<T>(xhat + base + c);
        rr[u][j] = ld4<T>(rsrc + base + c);
        dyl[u][j] = ok ? a : z;
        xh[u][j] = ok ? b : z;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long long base = (long long)(row0 + u * S) * cols;
#pragma unroll
      for (int j = 0; j < MAXV; ++j)
        if (j < nv) {
          const int c = (lane + 64 * j) * 4;
          floatx4 d = dyl[u][j];
          if (p_out > 0.f) {
#pragma unroll
            for (int q = 0; q < 4; ++q) d[q] *= k3m_dropout_scale(seed, off_out + base + c + q, p_out);
          }
          dyl[u][j] = d;
          const floatx4 xv = xh[u][j];
          pg[j] += d * xv;     // rows past the end hold zeros: they add nothing
          pb[j] += d;
          const floatx4 dxh = d * gm[j];
          s1[u] += dxh[0] + dxh[1] + dxh[2] + dxh[3];
          s2[u] += dxh[0] * xv[0] + dxh[1] * xv[1] + dxh[2] * xv[2] + dxh[3] * xv[3];
        }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int row = row0 + u * S;
      const float m1 = wave_sum(s1[u]) / cols, m2 = wave_sum(s2[u]) / cols;
      if (row >= rows) continue;
      const long long base = (long long)row * cols;
      const float rs = rstd[row];
#pragma unroll
      for (int j = 0; j < MAXV; ++j)
        if (j < nv) {
          const int c = (lane + 64 * j) * 4;
          floatx4 ds = (dyl[u][j] * gm[j] - m1 - xh[u][j] * m2) * rs;
          floatx4 dr = ds;
          if (acc_res) dr += rr[u][j];
          st4<T>(dres + base + c, dr);
          if (dx != dres) {
            if (p_in > 0.f) {
#pragma unroll
              for (int q = 0; q < 4; ++q) ds[q] *= k3m_dropout_scale(seed, off_in + base + c + q, p_in);
            }
            st4<T>(dx + base + c, ds);
          }
          if (want_sum) {   // the sum of dx as stored (bf16-rounded when T is bf16)
            px[j] += round4<T>(ds);
          }
        }
    }
  }
  // combine the 4 waves' column partials, write this block's slabs
  for (int k = 0; k < (want_sum ? 3 : 2); ++k) {
#pragma unroll
    for (int j = 0; j < MAXV; ++j)
      if (j < nv) {
        const int c = (lane + 64 * j) * 4;
        const floatx4 v = k == 0 ? pg[j] : (k == 1 ? pb[j] : px[j]);
        *reinterpret_cast<floatx4*>(&red[w][c]) = v;
      }
    __syncthreads();
    for (int c = threadIdx.x; c < cols; c += 256)
      ws[((long long)k * gridDim.x + blockIdx.x) * cols + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    __syncthreads();
  }
}

// ------------------------------------------------------------------ bf16 LayerNorm: half-wave rows, 16-B vectors
// The bf16 forms of the two kernels above.  With one wave per row and 8-B (4 x bf16) vectors, a bf16 row
// of 768 is three 512-B wave loads per operand and the kernels ran latency-bound at ~0.4 of the HBM
// roofline (config-3 step: 108 + 108 launches, 10 % of the step).  Here a row is a HALF wave and every
// access is a 16-B vector (8 bf16 per lane-chunk, cols/256 chunks per lane): twice the rows and the same
// bytes in flight per wave with half the load instructions.  Same arithmetic, dropout counters and slab
// layout as ln_fwd_kernel / ln_bwd_kernel (the row sums reduce in a different order).
constexpr int MAXV8 = 4;   // 16-B chunks per lane: cols <= 32 * 8 * 4 = 1024

__device__ __forceinline__ void unpack8bf(const uint4 u, float (&v)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __uint_as_float(w[q] << 16);
    v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}

__device__ __forceinline__ void ld8bf(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __uint_as_float(w[q] << 16);
    v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8bf(bf16_t* p, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = (uint32_t)from_f<bf16_t>(v[2 * q]).x | ((uint32_t)from_f<bf16_t>(v[2 * q + 1]).x << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
__device__ __forceinline__ void st8f(float* p, const float (&v)[8]) {
  *reinterpret_cast<floatx4*>(p) = floatx4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<floatx4*>(p + 4) = floatx4{v[4], v[5], v[6], v[7]};
}

__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p), b = *reinterpret_cast<const floatx4*>(p + 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = a[q];
    v[4 + q] = b[q];
  }
}
__device__ __forceinline__ float half_sum(float v) {   // over the 32 lanes of a half wave
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_bf16_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                          const float* __restrict__ gamma, const float* __restrict__ beta,
                                                          bf16_t* __restrict__ y, bf16_t* __restrict__ xhat,
                                                          float* __restrict__ rstd, int rows, int cols, float eps,
                                                          float p_in, float p_out, uint64_t seed, uint64_t off_in,
                                                          uint64_t off_out) {
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  const int l = threadIdx.x & 31;
  if (row >= rows) return;   // half-wave uniform; the shuffles below stay inside the half
  constexpr int nv = NV;
  const long long base = (long long)row * cols;
  const K3mDrop din = k3m_drop_init(seed, p_in), dout = k3m_drop_init(seed, p_out);
  float v[MAXV8][8];
  float rv[MAXV8][8];
  const bf16_t* rp = res ? res : x;   // unconditional loads, all issued before the arithmetic
#pragma unroll
  for (int j = 0; j < nv; ++j) ld8bf(x + base + (l + 32 * j) * 8, v[j]);
#pragma unroll
  for (int j = 0; j < nv; ++j) ld8bf(rp + base + (l + 32 * j) * 8, rv[j]);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV8; ++j)
    if (j < nv) {
      const int c = (l + 32 * j) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float a = v[j][e];
        if (p_in > 0.f) a *= k3m_drop(din, off_in + base + c + e);
        if (res) a += rv[j][e];
        v[j][e] = a;
        sum += a;
      }
    }
  const float mean = half_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV8; ++j)
    if (j < nv) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[j][e] -= mean;
        sq += v[j][e] * v[j][e];
      }
    }
  const float var = half_sum(sq) / cols;
  const float rs = 1.0f / sqrtf(var + eps);
  if (l == 0 && rstd) rstd[row] = rs;
#pragma unroll
  for (int j = 0; j < MAXV8; ++j)
    if (j < nv) {
      const int c = (l + 32 * j) * 8;
      float xh[8], g[8], b[8], o[8];
      ld8f(gamma + c, g);
      ld8f(beta + c, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[e] = v[j][e] * rs;
        o[e] = g[e] * xh[e] + b[e];
        if (p_out > 0.f) o[e] *= k3m_drop(dout, off_out + base + c + e);
      }
      if (xhat) st8bf(xhat + base + c, xh);
      st8bf(y + base + c, o);
    }
}

// LDS bytes of ln_bwd_bf16_kernel: gamma + the column partials (dgamma, dbeta, sum dx) of the 8 half waves
constexpr int ln_bwd_bf16_lds(int cols) { return (1 + 8 * 3) * cols * 4; }

template <int NV>
__global__ __launch_bounds__(256, NV <= 3 ? 2 : 1) void ln_bwd_bf16_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ xhat,
                                                          const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                          bf16_t* __restrict__ dres, bf16_t* __restrict__ dx,
                                                          float* __restrict__ ws, int rows, int cols, float p_in,
                                                          float p_out, uint64_t seed, uint64_t off_in, uint64_t off_out,
                                                          int acc_res, int want_sum) {
  // eight half-wave rows per block step (one row per half wave and step), software-pipelined: the next row's
  // dy / xhat loads (raw 16-B words) are issued before this row's arithmetic and stores (without it the loads
  // sat idle through each row's reduction and stores, ~3.7 TB/s at 20,992 x 768).  To fit that pipeline in
  // 2 waves per SIMD, the column partials of dgamma / dbeta / sum(dx) live in LDS (one private [3][cols]
  // slice per half wave, read-modify-written per row) instead of 3 x 8 x NV registers, gamma is read from LDS
  // (a global load in the row loop sat behind the prefetch in the in-order load counter), and xhat and the
  // residual stay packed until used.
  extern __shared__ float lnb_smem[];
  float* gam_s = lnb_smem;
  float* part = lnb_smem + cols;   // [8 half waves][3][cols]
  const int lane = threadIdx.x & 63, l = lane & 31, hw = threadIdx.x >> 5;
  constexpr int nv = NV;
  const K3mDrop din = k3m_drop_init(seed, p_in), dout = k3m_drop_init(seed, p_out);
  for (int c = threadIdx.x; c < cols; c += 256) gam_s[c] = gamma[c];
  for (int c = threadIdx.x; c < 24 * cols; c += 256) part[c] = 0.f;
  __syncthreads();
  float* pg = part + hw * 3 * cols;
  float* pb = pg + cols;
  float* px = pb + cols;
  const int S = gridDim.x * 8;
  const bf16_t* rsrc = acc_res ? dres : dy;
  uint4 nd[MAXV8], nx[MAXV8];
  int row = blockIdx.x * 8 + hw;
  if (row < rows) {
    const long long base = (long long)row * cols;
#pragma unroll
    for (int j = 0; j < nv; ++j) {
      nd[j] = *reinterpret_cast<const uint4*>(dy + base + (l + 32 * j) * 8);
      nx[j] = *reinterpret_cast<const uint4*>(xhat + base + (l + 32 * j) * 8);
    }
  }
  for (; row < rows; row += S) {
    const long long base = (long long)row * cols;
    float d[MAXV8][8];
    uint4 cx[MAXV8], co[MAXV8];
    const float rs = rstd[row];
#pragma unroll
    for (int j = 0; j < nv; ++j) {
      unpack8bf(nd[j], d[j]);
      cx[j] = nx[j];
      co[j] = *reinterpret_cast<const uint4*>(rsrc + base + (l + 32 * j) * 8);   // used last
    }
    __builtin_amdgcn_sched_barrier(0);   // rstd and the residual ahead of the prefetch in the load counter
    {
      // unconditional (the last step re-reads a valid row): under a branch, the wait counts after it were
      // those of the path without the prefetch, draining it
      const long long nbase = (long long)min(row + S, rows - 1) * cols;
#pragma unroll
      for (int j = 0; j < nv; ++j) {
        nd[j] = *reinterpret_cast<const uint4*>(dy + nbase + (l + 32 * j) * 8);
        nx[j] = *reinterpret_cast<const uint4*>(xhat + nbase + (l + 32 * j) * 8);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXV8; ++j)
      if (j < nv) {
        const int c = (l + 32 * j) * 8;
        float g[8], xv[8], ag[8], ab[8];
        ld8f(gam_s + c, g);
        ld8f(pg + c, ag);
        ld8f(pb + c, ab);
        unpack8bf(cx[j], xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float dd = d[j][e];
          if (p_out > 0.f) dd *= k3m_drop(dout, off_out + base + c + e);
          d[j][e] = dd;
          ag[e] += dd * xv[e];
          ab[e] += dd;
          const float dxh = dd * g[e];
          s1 += dxh;
          s2 += dxh * xv[e];
        }
        st8f(pg + c, ag);
        st8f(pb + c, ab);
      }
    const float m1 = half_sum(s1) / cols, m2 = half_sum(s2) / cols;
#pragma unroll
    for (int j = 0; j < MAXV8; ++j)
      if (j < nv) {
        const int c = (l + 32 * j) * 8;
        float g[8], ds[8], dr[8], xv[8];
        ld8f(gam_s + c, g);
        unpack8bf(cx[j], xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) ds[e] = (d[j][e] * g[e] - m1 - xv[e] * m2) * rs;
        if (acc_res) {
          float old[8];
          unpack8bf(co[j], old);
#pragma unroll
          for (int e = 0; e < 8; ++e) dr[e] = ds[e] + old[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) dr[e] = ds[e];
        }
        st8bf(dres + base + c, dr);
        if (dx != dres) {
          if (p_in > 0.f) {
#pragma unroll
            for (int e = 0; e < 8; ++e) ds[e] *= k3m_drop(din, off_in + base + c + e);
          }
          st8bf(dx + base + c, ds);
        }
        if (want_sum) {   // the sum of dx as stored (bf16-rounded)
          float ax[8];
          ld8f(px + c, ax);
#pragma unroll
          for (int e = 0; e < 8; ++e) ax[e] += to_f(from_f<bf16_t>(ds[e]));
          st8f(px + c, ax);
        }
      }
  }
  // the block's slab: per column, the two half waves of each wave first, then the 4 waves in order (the
  // order of the register version's shuffle + LDS fold)
  __syncthreads();
  for (int k = 0; k < (want_sum ? 3 : 2); ++k)
    for (int c = threadIdx.x; c < cols; c += 256) {
      float t[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] = part[(2 * q) * 3 * cols + k * cols + c] + part[(2 * q + 1) * 3 * cols + k * cols + c];
      ws[((long long)k * gridDim.x + blockIdx.x) * cols + c] = t[0] + t[1] + t[2] + t[3];
    }
}

// ------------------------------------------------------------------ embeddings
template <typename T>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                        const float* __restrict__ word, const float* __restrict__ pos,
                                                        const float* __restrict__ typ, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, T* y0, T* y1, T* y2, T* xhat,
                                                        float* rstd, int rows, int len, int cols, float eps,
                                                        float p_out, uint64_t seed, uint64_t off) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int nv = cols >> 8;
  const long long id = ids[row], t = tt[row];
  const int l = row % len;
  floatx4 v[MAXV];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (j < nv) {
      const int c = (lane + 64 * j) * 4;
      v[j] = *reinterpret_cast<const floatx4*>(word + id * cols + c) +
             *reinterpret_cast<const floatx4*>(pos + (long long)l * cols + c) +
             *reinterpret_cast<const floatx4*>(typ + t * cols + c);
      sum += v[j][0] + v[j][1] + v[j][2] + v[j][3];
    }
  const float mean = wave_sum(sum) / cols;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (j < nv) {
      v[j] -= mean;
      sq += v[j][0] * v[j][0] + v[j][1] * v[j][1] + v[j][2] * v[j][2] + v[j][3] * v[j][3];
    }
  const float rs = 1.0f / sqrtf(wave_sum(sq) / cols + eps);
  if (lane == 0) rstd[row] = rs;
  const long long base = (long long)row * cols;
#pragma unroll
  for (int j = 0; j < MAXV; ++j)
    if (j < nv) {
      const int c = (lane + 64 * j) * 4;
      const floatx4 xh = v[j] * rs;
      st4<T>(xhat + base + c, xh);
      floatx4 o = *reinterpret_cast<const floatx4*>(gamma + c) * xh + *reinterpret_cast<const floatx4*>(beta + c);
      if (p_out > 0.f) {
#pragma unroll
        for (int q = 0; q < 4; ++q) o[q] *= k3m_dropout_scale(seed, off + base + c + q, p_out);
      }
      st4<T>(y0 + base + c, o);
      if (y1) st4<T>(y1 + base + c, o);
      if (y2) st4<T>(y2 + base + c, o);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                        const T* __restrict__ ds, float* dword, float* dpos,
                                                        float* dtyp, int rows, int len, int cols) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  (void)tt;
  (void)dpos;
  (void)dtyp;
  (void)len;
  const long long id = ids[row];
  const long long base = (long long)row * cols;
  if (id == 0) return;   // padding_idx = 0 (vilbert_k3m.py:344): no gradient
  for (int c = lane; c < cols; c += 64) atomicAdd(dword + id * cols + c, to_f(ds[base + c]));
}

// Position and token-type gradients without contended atomics: the 36-128 position rows and the two
// type rows receive a term from EVERY token, so one atomic per (token, column) serialised thousands
// of adds on each address (embedding backward at 0.03 of its HBM roofline, profiles/r1_kernel_roofline_v2.txt).
// Here a block owns (position l, 256 columns) and sums the nseq tokens at that position in registers:
// dpos[l] gets a plain read-modify-write (one owner), the two type rows one atomic per block and column.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_pos_type_kernel(const int64_t* __restrict__ tt,
                                                                 const T* __restrict__ ds, float* dpos, float* dtyp,
                                                                 int nseq, int len, int cols) {
  const int l = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= cols) return;
  float sp = 0.f, s0 = 0.f, s1 = 0.f;
  for (int s = 0; s < nseq; ++s) {
    const long long row = (long long)s * len + l;
    const float g = to_f(ds[row * cols + c]);
    const long long t = tt[row];
    sp += g;
    if (t == 0) s0 += g;
    else if (t == 1) s1 += g;
    else atomicAdd(dtyp + t * cols + c, g);   // type_vocab_size > 2
  }
  dpos[(long long)l * cols + c] += sp;
  atomicAdd(dtyp + c, s0);
  atomicAdd(dtyp + cols + c, s1);
}

// Deterministic mode (k3m_embed_bwd_det, K3M_DETERMINISTIC): the same gradients with every sum in a fixed
// order.  Word rows: one wave per token row; the wave of the FIRST row holding an id owns it and sums the
// rows of every occurrence of that id in row order, then adds the total to dword[id] (one owner, plain
// read-modify-write).  A wave finds whether its row is a first occurrence with one 64-wide ballot per 64
// earlier ids.
template <typename T, int CPL>
__global__ __launch_bounds__(256) void embed_bwd_det_kernel(const int64_t* __restrict__ ids, const T* __restrict__ ds,
                                                            float* __restrict__ dword, int rows, int cols) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long long id = ids[row];
  if (id == 0) return;   // padding_idx = 0 (vilbert_k3m.py:344)
  for (int r0 = 0; r0 < row; r0 += 64) {
    const int r = r0 + lane;
    const bool same = r < row && ids[r] == id;
    if (__ballot(same) != 0ull) return;   // an earlier row owns this id
  }
  float acc[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc[q] = 0.f;
  for (int r0 = row; r0 < rows; r0 += 64) {
    const int r = r0 + lane;
    unsigned long long m = __ballot(r < rows && ids[r] == id);
    while (m) {   // matches in row order
      const int rr = r0 + __builtin_ctzll(m);
      m &= m - 1;
      const T* src = ds + (long long)rr * cols;
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const int c = lane + 64 * q;
        if (c < cols) acc[q] += to_f(src[c]);
      }
    }
  }
  float* dst = dword + id * cols;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = lane + 64 * q;
    if (c < cols) dst[c] += acc[q];
  }
}

// positions as embed_bwd_pos_type_kernel (one owner per (position, column)); the token-type sums of each
// position go to ws[l][t][c] and embed_type_reduce_kernel adds them up over the positions in order
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_pos_type_det_kernel(const int64_t* __restrict__ tt,
                                                                     const T* __restrict__ ds, float* dpos, float* ws,
                                                                     int nseq, int len, int cols) {
  const int l = blockIdx.x;
  const int c = blockIdx.y * 256 + threadIdx.x;
  if (c >= cols) return;
  float sp = 0.f, s0 = 0.f, s1 = 0.f;
  for (int s = 0; s < nseq; ++s) {
    const long long row = (long long)s * len + l;
    const float g = to_f(ds[row * cols + c]);
    sp += g;
    if (tt[row] == 0) s0 += g;
    else s1 += g;   // type_vocab_size 2 (checked on the host side of k3m_embed_bwd_det)
  }
  dpos[(long long)l * cols + c] += sp;
  ws[((long long)l * 2) * cols + c] = s0;
  ws[((long long)l * 2 + 1) * cols + c] = s1;
}
__global__ __launch_bounds__(256) void embed_type_reduce_kernel(const float* __restrict__ ws, float* dtyp, int len,
                                                                int cols) {
  const int i = blockIdx.x * 256 + threadIdx.x;   // (type, column)
  if (i >= 2 * cols) return;
  const int t = i / cols, c = i % cols;
  float a = 0.f;
  for (int l = 0; l < len; ++l) a += ws[((long long)l * 2 + t) * cols + c];
  dtyp[(long long)t * cols + c] += a;
}

// ------------------------------------------------------------------ column sums
template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(const T* __restrict__ x, long long ld, int rows, int cols,
                                                     float* __restrict__ ws) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float s = 0.f;
  for (int r = r0; r < r1; ++r) s += to_f(x[(long long)r * ld + c]);
  ws[(long long)blockIdx.y * cols + c] = s;
}

// 16-byte vector form: 64 column groups of 8 x 4 row phases per workgroup, 512 columns per block
template <typename T>
__device__ __forceinline__ void load8f(const T* p, float (&v)[8]);
template <>
__device__ __forceinline__ void load8f<float>(const float* p, float (&v)[8]) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p), b = *reinterpret_cast<const floatx4*>(p + 4);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = a[q];
    v[4 + q] = b[q];
  }
}
template <>
__device__ __forceinline__ void load8f<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[2 * q] = __uint_as_float(w[q] << 16);
    v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
  }
}
template <typename T>
__global__ __launch_bounds__(256) void colsum_vec_kernel(const T* __restrict__ x, long long ld, int rows, int cols,
                                                         float* __restrict__ ws) {
  __shared__ float red[4][512];
  const int cg = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 512 + cg * 8;
  const int chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cols) {
    int r = r0 + ph;
    for (; r + 4 < r1; r += 8) {   // two rows in flight per thread
      float a[8], b[8];
      load8f<T>(x + (long long)r * ld + c, a);
      load8f<T>(x + (long long)(r + 4) * ld + c, b);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += a[q] + b[q];
    }
    if (r < r1) {
      float a[8];
      load8f<T>(x + (long long)r * ld + c, a);
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += a[q];
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[ph][cg * 8 + q] = s[q];
  __syncthreads();
  for (int k = threadIdx.x; k < 512; k += 256) {
    const int cc = blockIdx.x * 512 + k;
    if (cc < cols) ws[(long long)blockIdx.y * cols + cc] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
  }
}

// ------------------------------------------------------------------ elementwise
template <typename T>
__global__ void dgelu_kernel(const T* g, const T* pre, T* out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = from_f<T>(to_f(g[i]) * dgelu_f(to_f(pre[i])));
}
template <typename T>
__global__ void add_kernel(T* y, const T* x, long long n, float alpha) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = from_f<T>(to_f(y[i]) + alpha * to_f(x[i]));
}
__global__ void cast_kernel(const float* x, uint16_t* y, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    y[i] = from_f<bf16_t>(x[i]).x;
}
template <typename X, typename Y>
__global__ void convert_kernel(const X* x, Y* y, long long n, int accumulate, float alpha) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float v = alpha * to_f(x[i]);
    y[i] = from_f<Y>(accumulate ? to_f(y[i]) + v : v);
  }
}
template <typename T>
__global__ void gather_rows_kernel(const T* src, long long lds, const int32_t* idx, int n, int cols, T* dst,
                                   long long ldd) {
  const int r = blockIdx.x;
  if (r >= n) return;
  const long long s = (long long)idx[r] * lds;
  for (int c = threadIdx.x; c < cols; c += blockDim.x) dst[(long long)r * ldd + c] = src[s + c];
}
template <typename T>
__global__ void scatter_add_rows_kernel(const T* src, long long lds, const int32_t* idx, int n, int cols, T* dst,
                                        long long ldd) {
  const int r = blockIdx.x;
  if (r >= n) return;
  const long long d = (long long)idx[r] * ldd;
  for (int c = threadIdx.x; c < cols; c += blockDim.x)
    dst[d + c] = from_f<T>(to_f(dst[d + c]) + to_f(src[(long long)r * lds + c]));
}

int grid_for(long long n) { return (int)std::min<long long>((n + 255) / 256, 4096); }

// The half-wave bf16 kernels win on long LayerNorms only (scripts/ln_bench.py, profiles/r3_ln_bf16.txt): forward
// 32.0 -> 27.5 us at 20,992 x 768 and 14.9 -> 12.7 at 8,192, backward 53.5 -> 47.7 at 20,992, while the short
// ones (2,304 rows) are 5-20 % slower.  A/B knob: K3M_LN_BF16_VEC=0 keeps every bf16 LayerNorm on the
// one-wave-per-row kernels.
const bool kLnBf16Vec = k3m_env_flag("K3M_LN_BF16_VEC", true);
constexpr int LN_VEC_FWD_ROWS = 4096;
// fewest rows for the half-wave bf16 backward (A/B knob K3M_LN_VEC_BWD_ROWS)
const int kLnVecBwdRows = k3m_env_int("K3M_LN_VEC_BWD_ROWS", 16384);

}  // namespace

#define DISPATCH_T(dtype, ...)            \
  if ((dtype) == K3M_F32) {               \
    using T = float;                      \
    __VA_ARGS__;                          \
  } else if ((dtype) == K3M_BF16) {       \
    using T = bf16_t;                     \
    __VA_ARGS__;                          \
  } else {                                \
    return K3M_EINVAL;                    \
  }

extern "C" int k3m_ln_fwd(const void* x, const void* res, const float* gamma, const float* beta, void* y, void* xhat,
                          float* rstd, int rows, int cols, float eps, float p_in, float p_out, uint64_t seed,
                          uint64_t off_in, uint64_t off_out, int dtype, hipStream_t st) {
  K3M_ARG(x && gamma && beta && y && rows >= 0 && cols % 256 == 0 && cols <= 1024 && cols > 0);
  if (rows == 0) return 0;
  const int nv = cols >> 8;
#define K3M_LN_NV(F)   \
  switch (nv) {        \
    case 1: F(1); break; \
    case 2: F(2); break; \
    case 3: F(3); break; \
    default: F(4);       \
  }
  if (dtype == K3M_BF16 && kLnBf16Vec && rows >= LN_VEC_FWD_ROWS) {
#define K3M_LNF16(NV_)                                                                                        \
  hipLaunchKernelGGL(ln_fwd_bf16_kernel<NV_>, dim3(k3m_cdiv(rows, 8)), dim3(256), 0, st, (const bf16_t*)x,   \
                      (const bf16_t*)res, gamma, beta, (bf16_t*)y, (bf16_t*)xhat, rstd, rows, cols, eps, p_in, \
                      p_out, seed, off_in, off_out)
    K3M_LN_NV(K3M_LNF16);
#undef K3M_LNF16
  } else {
#define K3M_LNF(NV_)                                                                                          \
  hipLaunchKernelGGL((ln_fwd_kernel<T, NV_>), dim3(k3m_cdiv(rows, 4)), dim3(256), 0, st, (const T*)x,       \
                      (const T*)res, gamma, beta, (T*)y, (T*)xhat, rstd, rows, cols, eps, p_in, p_out, seed,  \
                      off_in, off_out)
    DISPATCH_T(dtype, K3M_LN_NV(K3M_LNF));
#undef K3M_LNF
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

// at least kLnRowsPerSlab rows per slab (per workgroup): at 4, a short LayerNorm (2,304 rows) wrote 512 x 3
// slabs of cols fp32, more bytes than it reads; 8 measured 2,304 x 768 19.6 -> 17.1 us, 2,368 x 1,024 21.9 ->
// 20.3 (backward + its reduction, fp32 and bf16 alike), no change on the long ones (profiles/r3_ln_bf16.txt)
// ln_bwd_bf16_kernel's dynamic LDS exceeds the 64 KB default at cols = 1,024
template <int NV>
void ln_bwd_bf16_attr() {
  static const bool done = [] {
    (void)hipFuncSetAttribute((const void*)ln_bwd_bf16_kernel<NV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              ln_bwd_bf16_lds(NV * 256));
    return true;
  }();
  (void)done;
}

const int kLnRowsPerSlab = k3m_env_int("K3M_LN_ROWS_PER_SLAB", 8);
static int ln_bwd_slab_count(int rows) {
  return std::max(1, std::min(LN_BWD_BLOCKS, k3m_cdiv(rows, kLnRowsPerSlab)));
}

extern "C" int k3m_ln_bwd_nslab(int rows, int* nslab) {
  K3M_ARG(nslab && rows >= 0);
  *nslab = ln_bwd_slab_count(rows);
  return 0;
}

extern "C" int k3m_ln_bwd_slabs(const void* dy, const void* xhat, const float* rstd, const float* gamma, void* dres,
                                void* dx, int rows, int cols, float p_in, float p_out, uint64_t seed, uint64_t off_in,
                                uint64_t off_out, int acc_res, int want_sum, float* ws, int dtype, hipStream_t st) {
  K3M_ARG(dy && xhat && rstd && gamma && dres && dx && ws);
  K3M_ARG(cols % 256 == 0 && cols <= 1024 && rows >= 0);
  if (rows == 0) return 0;
  const int nb = ln_bwd_slab_count(rows);
  const int nv = cols >> 8;
  if (dtype == K3M_BF16 && kLnBf16Vec && rows >= kLnVecBwdRows) {
#define K3M_LNB16(NV_)                                                                                         \
  ln_bwd_bf16_attr<NV_>();                                                                                     \
  hipLaunchKernelGGL(ln_bwd_bf16_kernel<NV_>, dim3(nb), dim3(256), ln_bwd_bf16_lds(cols), st, (const bf16_t*)dy,                  \
                      (const bf16_t*)xhat, rstd, gamma, (bf16_t*)dres, (bf16_t*)dx, ws, rows, cols, p_in, p_out, \
                      seed, off_in, off_out, acc_res, want_sum)
    K3M_LN_NV(K3M_LNB16);
#undef K3M_LNB16
  } else {
#define K3M_LNB(NV_)                                                                                           \
  hipLaunchKernelGGL((ln_bwd_kernel<T, NV_>), dim3(nb), dim3(256), 0, st, (const T*)dy, (const T*)xhat, rstd, \
                      gamma, (T*)dres, (T*)dx, ws, rows, cols, p_in, p_out, seed, off_in, off_out, acc_res,    \
                      want_sum)
    DISPATCH_T(dtype, K3M_LN_NV(K3M_LNB));
#undef K3M_LNB
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_slab_reduce_batch(const float* const* ws, float* const* out, const int* nslab, const int* cols,
                                     const int* accumulate, int njobs, hipStream_t st) {
  K3M_ARG(njobs >= 0 && (njobs == 0 || (ws && out && nslab && cols && accumulate)));
  int j = 0;
  while (j < njobs) {
    // one launch: consecutive jobs with pairwise different outputs (a repeated output starts the
    // next launch, so accumulations into one array keep their order)
    SlabJobs jb;
    int n = 0, nblk = 0;
    for (; j < njobs && n < SLAB_JOBS; ++j) {
      K3M_ARG(ws[j] && out[j] && nslab[j] > 0 && cols[j] > 0);
      bool dup = false;
      for (int q = 0; q < n; ++q) dup |= jb.out[q] == out[j];
      if (dup) break;
      jb.ws[n] = ws[j];
      jb.out[n] = out[j];
      jb.nslab[n] = nslab[j];
      jb.cols[n] = cols[j];
      jb.accumulate[n] = accumulate[j];
      jb.vec[n] = nslab[j] <= SLAB_VEC_MAX && cols[j] % 4 == 0 && ((uintptr_t)ws[j] & 15) == 0 &&
                  ((uintptr_t)out[j] & 15) == 0;
      jb.start[n] = nblk;
      nblk += jb.vec[n] ? k3m_cdiv(cols[j], 1024) : k3m_cdiv(cols[j], 64);
      ++n;
    }
    jb.start[n] = nblk;
    jb.njobs = n;
    hipLaunchKernelGGL(slab_batch_kernel, dim3(nblk), dim3(256), 0, st, jb);
    K3M_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" int k3m_ln_bwd(const void* dy, const void* xhat, const float* rstd, const float* gamma, void* dres, void* dx,
                          float* dgamma, float* dbeta, float* dxsum, int rows, int cols, float p_in, float p_out,
                          uint64_t seed,
                          uint64_t off_in, uint64_t off_out, int acc_res, float* ws, int dtype, hipStream_t st) {
  K3M_ARG(dy && xhat && rstd && gamma && dres && dx && dgamma && dbeta && ws);
  K3M_ARG(cols % 256 == 0 && cols <= 1024 && rows >= 0);
  if (rows == 0) return 0;
  const int rc = k3m_ln_bwd_slabs(dy, xhat, rstd, gamma, dres, dx, rows, cols, p_in, p_out, seed, off_in, off_out,
                                  acc_res, dxsum != nullptr, ws, dtype, st);
  if (rc) return rc;
  const int nb = ln_bwd_slab_count(rows);
  const float* wsa[3] = {ws, ws + (long long)nb * cols, ws + 2LL * nb * cols};
  float* outs[3] = {dgamma, dbeta, dxsum};
  const int ns[3] = {nb, nb, nb}, cs[3] = {cols, cols, cols}, acc[3] = {1, 1, 1};
  return k3m_slab_reduce_batch(wsa, outs, ns, cs, acc, dxsum ? 3 : 2, st);
}

extern "C" int k3m_embed_fwd(const int64_t* ids, const int64_t* tt, const float* word, const float* pos,
                             const float* type, const float* gamma, const float* beta, void* y0, void* y1, void* y2,
                             void* xhat, float* rstd, int nseq, int len, int hidden, float eps, float p_out,
                             uint64_t seed, uint64_t off, int dtype, hipStream_t st) {
  K3M_ARG(ids && tt && word && pos && type && gamma && beta && y0 && xhat && rstd);
  K3M_ARG(hidden % 256 == 0 && hidden <= 1024);
  const int rows = nseq * len;
  if (rows == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_fwd_kernel<T>, dim3(k3m_cdiv(rows, 4)), dim3(256), 0, st, ids, tt, word,
                                       pos, type, gamma, beta, (T*)y0, (T*)y1, (T*)y2, (T*)xhat, rstd, rows, len,
                                       hidden, eps, p_out, seed, off));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_embed_bwd(const int64_t* ids, const int64_t* tt, const void* ds, float* dword, float* dpos,
                             float* dtype_, int nseq, int len, int hidden, int dtype, hipStream_t st) {
  K3M_ARG(ids && tt && ds && dword && dpos && dtype_);
  const int rows = nseq * len;
  if (rows == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_bwd_kernel<T>, dim3(k3m_cdiv(rows, 4)), dim3(256), 0, st, ids, tt,
                                       (const T*)ds, dword, dpos, dtype_, rows, len, hidden));
  K3M_CHECK_LAUNCH();
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_bwd_pos_type_kernel<T>, dim3(len, k3m_cdiv(hidden, 256)), dim3(256), 0, st,
                                       tt, (const T*)ds, dpos, dtype_, nseq, len, hidden));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_embed_bwd_det(const int64_t* ids, const int64_t* tt, const void* ds, float* dword, float* dpos,
                                 float* dtype_, int nseq, int len, int hidden, float* ws, int dtype, hipStream_t st) {
  K3M_ARG(ids && tt && ds && dword && dpos && dtype_ && ws && hidden <= 1024);
  const int rows = nseq * len;
  if (rows == 0) return 0;
  if (hidden <= 768) {
    DISPATCH_T(dtype, hipLaunchKernelGGL((embed_bwd_det_kernel<T, 12>), dim3(k3m_cdiv(rows, 4)), dim3(256), 0, st, ids,
                                         (const T*)ds, dword, rows, hidden));
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL((embed_bwd_det_kernel<T, 16>), dim3(k3m_cdiv(rows, 4)), dim3(256), 0, st, ids,
                                         (const T*)ds, dword, rows, hidden));
  }
  K3M_CHECK_LAUNCH();
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_bwd_pos_type_det_kernel<T>, dim3(len, k3m_cdiv(hidden, 256)), dim3(256), 0,
                                       st, tt, (const T*)ds, dpos, ws, nseq, len, hidden));
  hipLaunchKernelGGL(embed_type_reduce_kernel, dim3(k3m_cdiv(2 * hidden, 256)), dim3(256), 0, st, ws, dtype_, len,
                     hidden);
  K3M_CHECK_LAUNCH();
  return 0;
}

static int colsum_slab_count(int rows) { return std::max(1, std::min(K3M_COLSUM_SLABS, k3m_cdiv(rows, 64))); }

extern "C" int k3m_colsum_nslab(int rows, int* nslab) {
  K3M_ARG(nslab && rows >= 0);
  *nslab = colsum_slab_count(rows);
  return 0;
}

extern "C" int k3m_colsum_slabs(const void* x, long long ld, int rows, int cols, float* ws, int dtype, hipStream_t st) {
  K3M_ARG(x && ws && rows >= 0 && cols >= 0);
  if (cols == 0) return 0;
  const int chunks = colsum_slab_count(rows);
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && ld % 8 == 0 && cols % 8 == 0;
  if (vec) {
    DISPATCH_T(dtype, hipLaunchKernelGGL(colsum_vec_kernel<T>, dim3(k3m_cdiv(cols, 512), chunks), dim3(256), 0, st,
                                         (const T*)x, ld, rows, cols, ws));
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL(colsum_kernel<T>, dim3(k3m_cdiv(cols, 256), chunks), dim3(256), 0, st,
                                         (const T*)x, ld, rows, cols, ws));
  }
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_colsum(const void* x, long long ld, int rows, int cols, float* out, int accumulate, float* ws,
                          int dtype, hipStream_t st) {
  K3M_ARG(x && out && ws && rows >= 0 && cols >= 0);
  if (cols == 0) return 0;
  const int rc = k3m_colsum_slabs(x, ld, rows, cols, ws, dtype, st);
  if (rc) return rc;
  const float* wsa[1] = {ws};
  float* outs[1] = {out};
  const int ns[1] = {colsum_slab_count(rows)}, cs[1] = {cols}, acc[1] = {accumulate};
  return k3m_slab_reduce_batch(wsa, outs, ns, cs, acc, 1, st);
}

extern "C" int k3m_dgelu(const void* g, const void* pre, void* out, long long n, int dtype, hipStream_t st) {
  if (n == 0) return 0;
  K3M_ARG(g && pre && out);
  DISPATCH_T(dtype, hipLaunchKernelGGL(dgelu_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (const T*)g,
                                       (const T*)pre, (T*)out, n));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_add_inplace(void* y, const void* x, long long n, float alpha, int dtype, hipStream_t st) {
  K3M_ARG(y && x);
  if (n == 0) return 0;
  DISPATCH_T(dtype, hipLaunchKernelGGL(add_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, (T*)y, (const T*)x, n,
                                       alpha));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_cast_f32_bf16(const float* x, uint16_t* y, long long n, hipStream_t st) {
  K3M_ARG(x && y);
  if (n == 0) return 0;
  hipLaunchKernelGGL(cast_kernel, dim3(grid_for(n)), dim3(256), 0, st, x, y, n);
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_convert(const void* x, int xdtype, void* y, int ydtype, long long n, int accumulate, float alpha,
                           hipStream_t st) {
  K3M_ARG(x && y && n >= 0);
  if (n == 0) return 0;
  if (xdtype == K3M_F32 && ydtype == K3M_BF16)
    hipLaunchKernelGGL((convert_kernel<float, bf16_t>), dim3(grid_for(n)), dim3(256), 0, st, (const float*)x,
                       (bf16_t*)y, n, accumulate, alpha);
  else if (xdtype == K3M_BF16 && ydtype == K3M_F32)
    hipLaunchKernelGGL((convert_kernel<bf16_t, float>), dim3(grid_for(n)), dim3(256), 0, st, (const bf16_t*)x,
                       (float*)y, n, accumulate, alpha);
  else if (xdtype == K3M_F32 && ydtype == K3M_F32)
    hipLaunchKernelGGL((convert_kernel<float, float>), dim3(grid_for(n)), dim3(256), 0, st, (const float*)x,
                       (float*)y, n, accumulate, alpha);
  else if (xdtype == K3M_BF16 && ydtype == K3M_BF16)
    hipLaunchKernelGGL((convert_kernel<bf16_t, bf16_t>), dim3(grid_for(n)), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)y, n, accumulate, alpha);
  else
    return K3M_EINVAL;
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_gather_rows(const void* src, long long lds, const int32_t* idx, int n, int cols, void* dst,
                               long long ldd, int dtype, hipStream_t st) {
  if (n == 0) return 0;   // no labelled rows: nothing to move (buffers may be empty / NULL)
  K3M_ARG(src && idx && dst && n >= 0);
  DISPATCH_T(dtype, hipLaunchKernelGGL(gather_rows_kernel<T>, dim3(n), dim3(256), 0, st, (const T*)src, lds, idx, n,
                                       cols, (T*)dst, ldd));
  K3M_CHECK_LAUNCH();
  return 0;
}

extern "C" int k3m_scatter_add_rows(const void* src, long long lds, const int32_t* idx, int n, int cols, void* dst,
                                    long long ldd, int dtype, hipStream_t st) {
  if (n == 0) return 0;   // no labelled rows: nothing to move (buffers may be empty / NULL)
  K3M_ARG(src && idx && dst && n >= 0);
  DISPATCH_T(dtype, hipLaunchKernelGGL(scatter_add_rows_kernel<T>, dim3(n), dim3(256), 0, st, (const T*)src, lds, idx,
                                       n, cols, (T*)dst, ldd));
  K3M_CHECK_LAUNCH();
  return 0;
}
