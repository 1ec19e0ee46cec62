// bf16 MFMA operand helpers shared by the flash-attention kernels (attention_bf16.hip: L <= 128;
// attention_flash_long.hip: L <= 512).  Images are bf16 row-major [rows][NC chunks of 8], 16-B chunk c
// of row r stored at slot c ^ swz(r), so that ds_read_b128 row reads (32 rows x one chunk) and gfx950's
// transposing ds_read_b64_tr_b16 (4 rows x 16 columns per 16-lane group) are both bank-conflict-free.
#pragma once
#include "common.h"

namespace k3m_flash {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef short short8v __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) short4v lds_short4v;

// keep x where ok, zero elsewhere, per 32-bit word: a ?: select of a whole uint4 was lowered to a
// scratch-memory store + indexed reload of both candidates
__device__ __forceinline__ uint4 keep_if(bool ok, uint4 x) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_uint4(x.x & m, x.y & m, x.z & m, x.w & m);
}

// element offset of chunk c (8 bf16) of row r in an image whose rows hold NC chunks
template <int NC>
__device__ __forceinline__ int ioff(int r, int c) {
  if constexpr (NC == 16) return r * 128 + ((c ^ (((r & 3) << 2) | ((r >> 2) & 3))) << 3);
  else if constexpr (NC == 8) return r * 64 + ((c ^ ((((r >> 1) & 1) << 2) | ((r >> 2) & 3))) << 3);
  else return r * 32 + (c << 3);  // NC == 4: 64-B rows, the four rows of a transposed read never collide
}

__device__ __forceinline__ uint16_t bf_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }

// row fragment: X[rbase + (lane&31)][16 ks + 8 (lane>>5) .. +7]
template <int NC>
__device__ __forceinline__ bf16x8 rowfrag(const uint16_t* img, int rbase, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(img + ioff<NC>(rbase + (lane & 31), 2 * ks + (lane >> 5)));
}

// transposed fragment: element e of lane l = X[row(e)][cbase + (l&31)] with
//   PERM = false: row(e) = rbase + 8h + e                     (natural MFMA k order)
//   PERM = true:  row(e) = rbase + 8(e>>2) + 4h + (e&3)       (accumulator-as-operand k order)
template <int NC, bool PERM>
__device__ __forceinline__ bf16x8 trfrag(const uint16_t* img, int rbase, int cbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3, h = lane >> 5;
  const int ch = ((cbase + 16 * (g & 1)) >> 3) + (p >> 1);
  const int r0 = PERM ? rbase + 4 * h + q : rbase + 8 * h + q;
  const int r1 = PERM ? r0 + 8 : r0 + 4;
  const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + ioff<NC>(r0, ch) + 4 * (p & 1)));
  const short4v x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + ioff<NC>(r1, ch) + 4 * (p & 1)));
  const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// accumulator registers 8s..8s+7 as a bf16 operand fragment (k order: see trfrag PERM)
__device__ __forceinline__ bf16x8 accfrag(const floatx16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = (__bf16)a[8 * s + e];
  return f;
}

__device__ __forceinline__ floatx16 zero16() {
  floatx16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}


// transposed fragment for v_mfma_f32_16x16x32_bf16 operands: element e of lane l =
// X[rbase + 8 (l >> 4) + e][cbase + (l & 15)]  (lane -> row / column l & 15 of the 16-wide tile, its
// 16-lane group g = l >> 4 holds k = 8 g .. 8 g + 7 of the 32-deep step)
template <int NC>
__device__ __forceinline__ bf16x8 trfrag16(const uint16_t* img, int rbase, int cbase, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (cbase >> 3) + (p >> 1);
  const int r0 = rbase + 8 * g + q;
  const short4v x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + ioff<NC>(r0, ch) + 4 * (p & 1)));
  const short4v x1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4v*)(img + ioff<NC>(r0 + 4, ch) + 4 * (p & 1)));
  const short8v v = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

}  // namespace k3m_flash
