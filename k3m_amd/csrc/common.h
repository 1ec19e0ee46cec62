// Shared device helpers for libk3m_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/k3m_hip.h"

#define K3M_CHECK_LAUNCH()                                   \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return -(int)_e;                   \
  } while (0)

#define K3M_ARG(cond)                                        \
  do {                                                       \
    if (!(cond)) return K3M_EINVAL;                          \
  } while (0)

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------- bf16 storage type
struct bf16_t {
  uint16_t x;
};

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16_t v) { return __uint_as_float(((uint32_t)v.x) << 16); }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f<bf16_t>(float v) {
  // round to nearest even; hipcc emits v_cvt_pk_bf16_f32, which keeps a NaN a NaN
  bf16_t r;
  r.x = __builtin_bit_cast(uint16_t, (__bf16)v);
  return r;
}

// ---------------------------------------------------------------- counter-based RNG
// Stateless: every dropout / gumbel site draws u(seed, offset + element) so the backward pass
// regenerates the forward mask instead of storing it.
//
// hipGraph replay (k3m_amd/graph.py): a captured launch keeps the by-value seed it was captured with,
// so a captured step passes seed = K3M_GRAPH_SEED | (device address of a 64-bit word) and every draw
// reads the step's seed from that word, which the host refills before each replay.  Host seeds are
// 63-bit, so eager launches (bit 63 clear) are unchanged.  Resolved inside k3m_seed_key, through
// which every draw goes.
__device__ __forceinline__ uint64_t k3m_seed_resolve(uint64_t seed) {
  if (seed & K3M_GRAPH_SEED) seed = *reinterpret_cast<const uint64_t*>(seed & ~K3M_GRAPH_SEED);
  return seed;
}
//
// Cost matters: the attention softmax and LayerNorm tails draw one value per element.  The 64-bit
// seed is expanded once per launch (splitmix64 of a kernel argument: wave-uniform, scalar ALU);
// per element the counter's high word is folded in with one multiply and the low word goes
// through Wellons' "lowbias32" finaliser (two multiplies, full avalanche).  That is 3 32-bit
// multiplies per element instead of the 12 of a per-element splitmix64.
__device__ __forceinline__ uint32_t k3m_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint64_t k3m_seed_key(uint64_t seed) {
  uint64_t z = k3m_seed_resolve(seed) + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t k3m_hash_key(uint64_t key, uint64_t ctr) {
  const uint32_t lo = (uint32_t)ctr, hi = (uint32_t)(ctr >> 32);
  return k3m_mix32(lo ^ (uint32_t)key ^ ((hi ^ (uint32_t)(key >> 32)) * 0x9E3779B1u));
}
__device__ __forceinline__ uint32_t k3m_hash(uint64_t seed, uint64_t ctr) {
  return k3m_hash_key(k3m_seed_key(seed), ctr);
}
// Dropout with keep probability (1-p): scale 1/(1-p) or 0.  An element is kept iff
// u = (h >> 8) * 2^-24 >= p, i.e. iff (h >> 8) >= thr = ceil(p * 2^24) (p * 2^24 is exact in fp32),
// so the test is one integer compare.  Set up once per launch (wave-uniform) with k3m_drop_init.
struct K3mDrop {
  uint64_t key;
  uint32_t thr;     // 0: p == 0, nothing dropped
  uint32_t thr16;   // ceil(p * 2^16): the attention draws' 16-bit threshold
  float scale;
};
__device__ __forceinline__ K3mDrop k3m_drop_init(uint64_t seed, float p) {
  K3mDrop d;
  d.key = k3m_seed_key(seed);
  d.thr = p > 0.f ? (uint32_t)ceilf(p * 16777216.0f) : 0u;
  d.thr16 = p > 0.f ? (uint32_t)ceilf(p * 65536.0f) : 0u;
  d.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  return d;
}
__device__ __forceinline__ float k3m_drop(const K3mDrop& d, uint64_t ctr) {
  if (d.thr == 0u) return 1.f;
  return (k3m_hash_key(d.key, ctr) >> 8) >= d.thr ? d.scale : 0.f;
}
__device__ __forceinline__ float k3m_dropout_scale(uint64_t seed, uint64_t ctr, float p) {
  return k3m_drop(k3m_drop_init(seed, p), ctr);
}
// Attention-probability dropout: one 32-bit draw per PAIR of keys.  Element (row, j) of a score block with lk keys
// per row (row = (sequence * heads + head) * lq + query) takes the (j & 1) half of
//   k3m_hash_key(key, off + row * ceil(lk / 2) + j / 2)
// and is kept iff that 16-bit value >= thr16 = ceil(p * 2^16).  The softmax of every attention kernel is VALU-bound
// and the hash was the largest part of it (three 32-bit multiplies per score): this halves the hashing, and a lane
// that holds both keys of a pair (the flash forwards) or swaps bits with the lane that does (the key-major
// backwards) draws once for two scores.  p resolves to 2^-16.
__device__ __forceinline__ uint64_t k3m_attn_ctr(uint64_t off, long long row, int lk, int j) {
  return off + (uint64_t)row * (uint64_t)((lk + 1) >> 1) + (uint64_t)(j >> 1);
}
__device__ __forceinline__ uint32_t k3m_attn_half(uint32_t h, int j) { return (j & 1) ? h >> 16 : h & 0xffffu; }
__device__ __forceinline__ float k3m_attn_drop(const K3mDrop& d, uint64_t off, long long row, int lk, int j) {
  if (d.thr == 0u) return 1.f;
  return k3m_attn_half(k3m_hash_key(d.key, k3m_attn_ctr(off, row, lk, j)), j) >= d.thr16 ? d.scale : 0.f;
}
__device__ __forceinline__ float k3m_attn_dropout_scale(uint64_t seed, float p, uint64_t off, long long row, int lk,
                                                       int j) {
  return k3m_attn_drop(k3m_drop_init(seed, p), off, row, lk, j);
}
// The high-word half of k3m_hash_key for counters that share ctr's high word: for a lane's run of pairs
// ctr + d whose low word does not carry (the caller checks),
//   k3m_hash_key(key, ctr + d) == k3m_mix32(((uint32_t)ctr + d) ^ k3m_pair_pre(key, ctr)).
__device__ __forceinline__ uint32_t k3m_pair_pre(uint64_t key, uint64_t ctr) {
  return (uint32_t)key ^ (((uint32_t)(ctr >> 32) ^ (uint32_t)(key >> 32)) * 0x9E3779B1u);
}
// dropout factor of bit r of a keep mask: scale (its bits sbits) or +0 -- a sign-extended bit field and an AND
__device__ __forceinline__ float k3m_keep_f(uint32_t keep, int r, uint32_t sbits) {
  return __uint_as_float((uint32_t)((int)(keep << (31 - r)) >> 31) & sbits);
}
// A row's pair draws from a lane's first pair (key jb, even): k3m_pair_draw(pr, d) is the draw of keys jb + 2 d and
// jb + 2 d + 1 (k3m_attn_drop), the high word mixed once per row and once more for a low word that carries.
struct K3mPairRow {
  uint32_t lo, pre0, pre1;
};
__device__ __forceinline__ K3mPairRow k3m_pair_row(const K3mDrop& d, uint64_t off, long long row, int lk, int jb) {
  const uint64_t pb = k3m_attn_ctr(off, row, lk, jb);
  return {(uint32_t)pb, k3m_pair_pre(d.key, pb), k3m_pair_pre(d.key, pb + (1ull << 32))};
}
__device__ __forceinline__ uint32_t k3m_pair_draw(const K3mPairRow& pr, uint32_t d) {
  const uint32_t x = pr.lo + d;
  return k3m_mix32(x ^ (x < pr.lo ? pr.pre1 : pr.pre0));
}
// Keep bits of a key-major lane (the backward kernels: this lane's key j, query rows rowu + rowl + 8 (r >> 2) +
// (r & 3) in bit r = 0 .. 15, the MFMA 32x32 accumulator order; rowu wave-uniform, rowl the lane's small part).
// Lanes 2m and 2m + 1 hold the keys of one pair for the same rows: the even lane draws the pair's values of rows
// r < 8, the odd lane those of r >= 8, and each passes the other key's 8 bits across with one DPP lane swap -- 8
// draws per lane instead of 16.  Needs j's parity == the lane's and both lanes of the pair active (key-major
// kernels index keys by lane from an even base, under wave-uniform branches).
__device__ __forceinline__ uint32_t k3m_attn_keep_km16(const K3mDrop& d, uint64_t off, long long rowu, int rowl, int lk,
                                                       int j) {
  const int odd = j & 1;
  const uint32_t lkp = (uint32_t)((lk + 1) >> 1);
  const uint64_t ub = off + (uint64_t)rowu * lkp;                           // wave-uniform
  uint32_t rel = (uint32_t)(rowl + 16 * odd) * lkp + (uint32_t)(j >> 1);   // < 2^32: rows and keys <= 512
  // opaque to loop-invariant code motion: the callers draw once per query chunk, and the eight per-row counters
  // hoisted out of that loop held 8 - 16 VGPRs across it (the d = 64 backward spilled)
  asm volatile("" : "+v"(rel));
  uint32_t mine = 0u, theirs = 0u;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const uint32_t h = k3m_hash_key(d.key, ub + (uint64_t)(rel + (uint32_t)(8 * (t >> 2) + (t & 3)) * lkp));
    mine |= (uint32_t)(k3m_attn_half(h, odd) >= d.thr16) << t;
    theirs |= (uint32_t)(k3m_attn_half(h, odd ^ 1) >= d.thr16) << t;
  }
  const uint32_t got = (uint32_t)__builtin_amdgcn_mov_dpp((int)theirs, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  return odd ? (got | (mine << 8)) : (mine | (got << 8));
}
// uniform in the OPEN interval (0, 1): both log(u) and log(-log(u)) stay finite (gumbel noise)
__device__ __forceinline__ float k3m_uniform(uint64_t seed, uint64_t ctr) {
  // 23 random bits: (k + 0.5) * 2^-23 is exact in fp32, so u lies in [2^-24, 1 - 2^-24] and never
  // rounds to 1 (a 24-bit (k + 0.5) * 2^-24 rounds to exactly 1.0 for k = 2^24 - 1).
  uint32_t h = k3m_hash(seed, ctr);
  return ((float)(h >> 9) + 0.5f) * (1.0f / 8388608.0f);
}

// ---------------------------------------------------------------- reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == 64*NW; red must hold NW floats; result broadcast to all.
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) s += red[i];
  return s;
}
template <int NW>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) s = fmaxf(s, red[i]);
  return s;
}

// fp32 erf-GELU (the reference's gelu, x * 0.5 * (1 + erf(x / sqrt 2)), vilbert_k3m.py) and its derivative in a
// branch-free form: Phi(x) from erfc(z) = t exp(-z^2 + P(t)), z = |x| / sqrt 2, t = 1 / (1 + z / 2) (the
// Chebyshev fit of Numerical Recipes' erfcc, fractional error < 1.2e-7 for every z).  In fp32 (numpy sweep of
// x in [-12, 12] against scipy, float64 reference): GELU max absolute error 1.6e-7 and max relative error 3.9e-6
// for |x| < 5, where the erff form's 1 + erf cancels (6.8e-7 absolute, 4.8 % relative in the left tail).  ocml's
// erff takes a divergent two-branch path (~35 VALU per element in the GEMM epilogues); this is ~18, no branch.
__device__ __forceinline__ float phi_cdf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
  float p = fmaf(0.17087277f, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  const float arg = fmaf(-z, z, fmaf(p, t, -1.26551223f));
  const float q = 0.5f * t * __builtin_amdgcn_exp2f(arg * 1.4426950408889634f);   // Phi(-|x|)
  return x >= 0.f ? 1.0f - q : q;
}
__device__ __forceinline__ float gelu_f(float x) { return x * phi_cdf(x); }
__device__ __forceinline__ float dgelu_f(float x) {
  const float pdf = 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);   // exp(-x^2/2)
  return fmaf(x, pdf, phi_cdf(x));
}
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + expf(-x)); }

// erf-GELU and its derivative with a short erfc (Abramowitz & Stegun 7.1.26: |erf error| <= 1.5e-7,
// i.e. Phi(x) to ~7.5e-8 absolute): one v_rcp, one v_exp, five FMAs shared by GELU and dGELU.
// Used by the bf16 GEMM epilogues, whose outputs round to 8 significant bits (the exact-erff forms
// above cost ~3x the VALU and serialised the epilogue of the output-heavy FFN GEMMs).
__device__ __forceinline__ void phi_fast(float x, float& Phi, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float poly = fmaf(1.061405429f, t, -1.453152027f);
  poly = fmaf(poly, t, 1.421413741f);
  poly = fmaf(poly, t, -0.284496736f);
  poly = fmaf(poly, t, 0.254829592f);
  poly *= t;
  const float e = __expf(-z * z);                 // exp(-x^2 / 2)
  const float half_erfc = 0.5f * poly * e;        // 0.5 * erfc(|x| / sqrt 2)
  Phi = x >= 0.f ? 1.0f - half_erfc : half_erfc;
  pdf = 0.3989422804014327f * e;
}
__device__ __forceinline__ float gelu_fast(float x) {
  float P, d;
  phi_fast(x, P, d);
  return x * P;
}
__device__ __forceinline__ float dgelu_fast(float x) {
  float P, d;
  phi_fast(x, P, d);
  return fmaf(x, d, P);
}

static inline int k3m_cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// Environment knobs (A/B switches), read once at library load.  Plain functions, not lambda
// initialisers: hipcc (ROCm 7.2) gives the closures of lambdas in REOPENED anonymous namespaces the
// same mangled name ($_0 ...), so one knob's initialiser silently ran another's getenv.
#include <cstdlib>
static inline int k3m_env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
static inline bool k3m_env_flag(const char* name, bool dflt) {   // "0" = off, anything else = on
  const char* e = std::getenv(name);
  return e ? !(e[0] == '0') : dflt;
}

// Longest-first order of a grouped launch's problems (stable; by the k length of one work unit, k / splitk).
// The persistent walks deal work units to the CUs round-robin in problem order, so a group mixing k = 1,024
// and k = 3,072 problems left some CUs three long units and others a short one; longest first, the last
// partial wave holds the short units (LPT scheduling).  Outputs are unchanged: every unit computes the same
// tile over the same k range in the same order.  K3M_GROUP_LPT=0 keeps the caller's order (A/B knob).
static inline long long k3m_unit_k(const K3mGemm& g) { return g.splitk > 1 ? (g.k + g.splitk - 1) / g.splitk : g.k; }
static inline void k3m_lpt_order(K3mGemm* g, bool* flag, int n) {
  static const bool on = k3m_env_flag("K3M_GROUP_LPT", true);
  if (!on) return;
  for (int i = 1; i < n; ++i) {
    const K3mGemm gi = g[i];
    const bool fi = flag[i];
    const long long wi = k3m_unit_k(gi);
    int j = i - 1;
    for (; j >= 0 && k3m_unit_k(g[j]) < wi; --j) {
      g[j + 1] = g[j];
      flag[j + 1] = flag[j];
    }
    g[j + 1] = gi;
    flag[j + 1] = fi;
  }
}
