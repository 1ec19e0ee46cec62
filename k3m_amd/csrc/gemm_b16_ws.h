// bf16 GEMM with the epilogue on its own waves ("warp-specialised" walk, K3M_B16_WS) for the K-contiguous
// forwards of the bf16 encoder (x . W^T: QKV, attention output, FFN1 + GELU, FFN2, the co-attention stages).
//
// Why: a K = 768 forward with the GELU epilogue writes 4 bytes per output (C and
// the pre-activation) — per 256 x 128 tile as many bytes as the CU's share of HBM write bandwidth drains in about the
// time of the tile's MFMAs.  In the one-role kernels the waves that run the MFMAs also issue those stores, and
// vmcnt retires loads and stores in issue order, so the next tile's operand DMA waits for the store drain; the GELU
// VALU also runs on the MFMA waves between tiles.  Here the two are separated:
//
//  * 8 waves, one workgroup per CU, persistent walk over 256 x 128 tiles (same unit order as gemm_persist_kernel);
//  * waves 0-3 (one per SIMD) only read fragments from LDS and issue MFMAs: 128 x 64 each, v_mfma_f32_16x16x32_bf16
//    with the operands swapped (acc = B_j . A_i^T), so each lane holds 4 consecutive COLUMNS of one row of C;
//    at the end of a tile they add the bias, round to bf16 and write the tile into an LDS output image (8-byte
//    ds_writes, 64 KB), then go straight on with the next tile;
//  * waves 4-7 (one per SIMD) issue every operand LDS-DMA (4 stages of 32-deep k-tiles, 3 in flight, counted
//    vmcnt) and, spread over the next tile's k-steps, read the previous tile's image back 16 rows at a time, apply
//    the epilogue (GELU from the stored bf16 pre-activation, exactly as the one-role epilogue) and store C (and the
//    pre-activation) with 16-byte buffer stores.  Their stores queue only behind their own DMA issues; the MFMA
//    waves hold no vector-memory operation at all but one bias load per tile;
//  * one s_barrier per k-step for all 8 waves (the epilogue waves reach it after their DMA wait), two more at the
//    start and the end of the walk.
//
// Same products and the same accumulation order per element as the one-role kernels, one rounding to bf16 from the
// fp32 (accumulator + bias): bit-identical C and pre-activation (tests/test_gpu_gemm_b16_ws.py).
// Eligible: A row-major K-contiguous, B [N][K] (nt), bf16 C, epilogue none / bias / bias+GELU with beta = 0, no split-K,
// K % 32 == 0 and K >= 32 * KMIN for every problem (the epilogue waves need KMIN - 1 k-steps per tile).
#pragma once
#include "gemm_b16_tile.h"

namespace k3m_b16 {
namespace ws {

constexpr int TBM = 256, TBN = 128, BKW = 32, NSTG = 4;
constexpr int STAGE = (TBM + TBN) * BKW;   // bf16 elements per stage (24 KB)
constexpr int OUTE = TBM * TBN;            // bf16 elements of the output image (64 KB)
constexpr int LDS_E = NSTG * STAGE + OUTE; // 163,840 bytes: the whole LDS
constexpr int NCH = 16;                    // output chunks per tile: 16 rows x 128 columns, one per epilogue lane x 8
constexpr int KMIN = NCH + 1;              // k-steps per tile (chunks run at local steps 1 .. nk - 1)
constexpr uint32_t RSRC3 = 0x00020000u;    // raw buffer descriptor word 3 (gfx9 family)
constexpr int OOB = 0x7fffffff;            // buffer offset past every num_records: the store is dropped

// LDS-DMA of one K-contiguous operand tile ([TILE][32] bf16 image, chunk c of row r at slot c ^ swz4(r), as
// LoaderD), issued by the four epilogue waves e = 0..3: instruction i of wave e covers rows 16 (e + 4 i) ..+15
template <int TILE>
struct Ld {
  static constexpr int INSTS = TILE * BKW * 2 / 1024;
  static constexpr int NI = INSTS / 4;
  static_assert(INSTS % 4 == 0, "tile must split over the four epilogue waves");
  const uint16_t* base;
  uint32_t off[NI];
  __device__ __forceinline__ void init(const uint16_t* __restrict__ a, long long ld, int mn0, int MN, int e) {
    const int l = threadIdx.x & 63;
    base = a;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int row = (e + 4 * i) * 16 + (l >> 2), slot = l & 3;
      const int ch = slot ^ swz4(row);
      off[i] = (uint32_t)((long long)min(mn0 + row, MN - 1) * ld + ch * 8);
    }
  }
  __device__ __forceinline__ void issue(uint16_t* img, int e) {
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(base + off[i], img + (e + 4 * i) * 512);
    base += BKW;
  }
};
constexpr int NI_E = Ld<TBM>::NI + Ld<TBN>::NI;   // DMA instructions per k-step per epilogue wave (6)

// element offset of (row m, column n) in the output image: 256-B rows, 16-B chunk index XOR (m & 15) — the
// 16 rows of one ds_write_b64 lane group and the 8-lane groups of the ds_read_b128 read-back hit distinct banks
__device__ __forceinline__ int out_off(int m, int n) { return m * TBN + ((((n >> 3) ^ (m & 15)) << 3) | (n & 7)); }

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// vmcnt(n) for a wave-uniform n <= 2 (NI_E + 2): a scalar switch over immediate forms
__device__ __forceinline__ void vm_wait_n(int n) {
  switch (n) {
#define K3M_WS_W(N) case N: vm_wait<N>(); break;
    K3M_WS_W(0) K3M_WS_W(1) K3M_WS_W(2) K3M_WS_W(3) K3M_WS_W(4) K3M_WS_W(5) K3M_WS_W(6) K3M_WS_W(7) K3M_WS_W(8)
    K3M_WS_W(9) K3M_WS_W(10) K3M_WS_W(11) K3M_WS_W(12) K3M_WS_W(13) K3M_WS_W(14) K3M_WS_W(15) K3M_WS_W(16)
#undef K3M_WS_W
    default: vm_wait<0>(); break;
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, long long bytes) {
  const int n = bytes > 0x7ffffff0LL ? 0x7ffffff0 : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, n, (int)RSRC3);
}

// chunk c of a tile is handled at local step 1 + c (nk - 1) / NCH; -1 if none at step ls
__device__ __forceinline__ int chunk_at(int ls, int nk) {
  if (ls < 1) return -1;
  const int c = ((ls - 1) * NCH + nk - 2) / (nk - 1);
  return (c < NCH && 1 + c * (nk - 1) / NCH == ls) ? c : -1;
}

template <int EPI>
struct Cfg {
  static constexpr bool BIAS = EPI == K3M_EPI_BIAS || EPI == K3M_EPI_BIAS_GELU;
  static constexpr int SPC = EPI == K3M_EPI_BIAS_GELU ? 2 : 1;   // buffer stores per chunk per lane
};

// ---------------------------------------------------------------- MFMA waves (w = 0..3)
template <int EPI>
__device__ __forceinline__ void mfma_role(const GemmGroup& grp, uint16_t* smem, uint16_t* outb, int w, int lane) {
  using Cf = Cfg<EPI>;
  const int total = grp.start[grp.count], P = gridDim.x;
  const int wm = (w >> 1) * 128, wn = (w & 1) * 64;
  floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto frag_a = [&](const uint16_t* st, int i) {
    return *reinterpret_cast<const bf16x8*>(st + kc4_off(wm + 16 * i + (lane & 15), lane >> 4));
  };
  auto frag_b = [&](const uint16_t* st, int j) {
    return *reinterpret_cast<const bf16x8*>(st + TBM * BKW + kc4_off(wn + 16 * j + (lane & 15), lane >> 4));
  };
  __builtin_amdgcn_s_barrier();   // B0: k-steps 0 and 1 have landed
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 a[8], b[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = frag_a(smem, i);
#pragma unroll
  for (int j = 0; j < 4; ++j) b[j] = frag_b(smem, j);
  int gs = 0;   // global k-step
  for (int u = blockIdx.x; u < total; u += P) {
    PUnit<TBM, TBN, 2, 2> cur;
    cur.decode(grp, u);
    const K3mGemm& g = grp.g[cur.p];
    const int nk = g.k / BKW;
    floatx4 bv[4];
    for (int ls = 0; ls < nk; ++ls, ++gs) {
      // fragments of k-step gs + 1 (the next tile's first after the last; past the walk's end: a stale stage
      // nobody uses) under the MFMAs of k-step gs; A fragments reuse the registers their MFMAs just released
      const uint16_t* nst = smem + ((gs + 1) & 3) * STAGE;
      bf16x8 nb[4];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        a[i] = frag_a(nst, i);
        if (i < 4) nb[i] = frag_b(nst, i);
      }
      // one wave per SIMD issues the MFMAs: keep the fragment reads between them (4 MFMAs, then the 1-2 reads
      // whose registers those MFMAs released) instead of the compiler's all-reads-after-all-MFMAs order
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = nb[j];
      if constexpr (Cf::BIAS) {
        if (ls == nk - 1) {   // this tile's bias, landing during the barrier wait (the waves' only global loads)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int col = min(cur.n0 + wn + 16 * j + 4 * (lane >> 4), g.n - 4);
            bv[j] = *reinterpret_cast<const floatx4*>(g.bias + col);
          }
        }
      }
      // every fragment read of k-step gs + 1 done: its stage is rewritten right after the next barrier (DMA of
      // k-step gs + 5); this also retires the previous hand-off's image writes before the epilogue waves read them
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    // hand-off: fp32 (accumulator + bias) -> bf16 once, into the output image (the epilogue waves finished
    // reading the previous tile's image before the barrier just passed)
    const float alpha = g.alpha;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = acc[i][j][r];
          if constexpr (EPI == K3M_EPI_NONE) o[r] = alpha * v;
          else if constexpr (EPI == K3M_EPI_BIAS) o[r] = alpha * (v + bv[j][r]);
          else o[r] = v + bv[j][r];   // the pre-activation the backward reads
        }
        uint2 pk;
        pk.x = (uint32_t)from_f<bf16_t>(o[0]).x | ((uint32_t)from_f<bf16_t>(o[1]).x << 16);
        pk.y = (uint32_t)from_f<bf16_t>(o[2]).x | ((uint32_t)from_f<bf16_t>(o[3]).x << 16);
        const int m = wm + 16 * i + (lane & 15), n = wn + 16 * j + 4 * (lane >> 4);
        *reinterpret_cast<uint2*>(outb + out_off(m, n)) = pk;
        acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();   // B_tail: the last tile's image is complete
}

// ---------------------------------------------------------------- epilogue waves (e = 0..3)
// chunk c of the tile (m0, n0) of problem g: lane -> row 16 c + 4 e + (lane >> 4), columns 8 (lane & 15) .. + 7
template <int EPI>
__device__ __forceinline__ void epi_chunk(const K3mGemm& g, int m0, int n0, const uint16_t* outb, int c, int e,
                                          int lane) {
  const int r = 16 * c + 4 * e + (lane >> 4), q = lane & 15;
  const u32x4 x = *reinterpret_cast<const u32x4*>(outb + out_off(r, 8 * q));
  const int row = m0 + r, col = n0 + 8 * q;
  const bool ok = row < g.m && col < g.n;
  const long long cbytes = ((long long)(g.m - 1) * g.ldc + g.n) * 2;
  const __amdgpu_buffer_rsrc_t rc = rsrc_of(g.c, cbytes);
  const int coff = ok ? (int)(((long long)row * g.ldc + col) * 2) : OOB;
  if constexpr (EPI == K3M_EPI_BIAS_GELU) {
    u32x4 o;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float lo = gelu_fast(__uint_as_float(x[t] << 16)), hi = gelu_fast(__uint_as_float(x[t] & 0xffff0000u));
      o[t] = (uint32_t)from_f<bf16_t>(lo).x | ((uint32_t)from_f<bf16_t>(hi).x << 16);
    }
    __builtin_amdgcn_raw_buffer_store_b128(o, rc, coff, 0, 0);
    const long long abytes = ((long long)(g.m - 1) * g.ldaux + g.n) * 2;
    const __amdgpu_buffer_rsrc_t ra = rsrc_of(g.aux, abytes);
    const int aoff = ok ? (int)(((long long)row * g.ldaux + col) * 2) : OOB;
    __builtin_amdgcn_raw_buffer_store_b128(x, ra, aoff, 0, 0);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(x, rc, coff, 0, 0);
  }
}

template <int EPI>
__device__ __forceinline__ void epi_role(const GemmGroup& grp, uint16_t* smem, const uint16_t* outb, int e,
                                         int lane) {
  using Cf = Cfg<EPI>;
  constexpr int SPC = Cf::SPC;
  const int total = grp.start[grp.count], P = gridDim.x;
  // DMA cursor: unit du, k-step dk of it (dnk k-steps), global k-step dg
  Ld<TBM> la;
  Ld<TBN> lb;
  int du = blockIdx.x, dk = 0, dnk = 0, dg = 0;
  auto dinit = [&]() {
    PUnit<TBM, TBN, 2, 2> d;
    d.decode(grp, du);
    const K3mGemm& g = grp.g[d.p];
    dnk = g.k / BKW;
    la.init(static_cast<const uint16_t*>(g.a), g.lda, d.m0, g.m, e);
    lb.init(static_cast<const uint16_t*>(g.b), g.ldb, d.n0, g.n, e);
  };
  auto dma = [&]() -> bool {   // k-step dg into stage dg & 3; advances the cursor
    if (du >= total) return false;
    uint16_t* st = smem + (dg & 3) * STAGE;
    la.issue(st, e);
    lb.issue(st + TBM * BKW, e);
    ++dg;
    if (++dk == dnk) {
      du += P;
      dk = 0;
      if (du < total) dinit();
    }
    return true;
  };
  dinit();
  dma();
  dma();
  const int pro = (dma() ? 1 : 0) + (dma() ? 1 : 0);
  vm_wait_n(pro * NI_E);   // k-steps 0 and 1 landed, 2 and 3 in flight
  __builtin_amdgcn_s_barrier();   // B0
  __builtin_amdgcn_sched_barrier(0);
  int pu = -1;   // the previous tile (its image is in LDS)
  int prev_ops = pro == 2 ? NI_E : 0;   // vector-memory operations of the last step issued after its DMA wait point
  PUnit<TBM, TBN, 2, 2> prev;
  for (int u = blockIdx.x; u < total; u += P) {
    PUnit<TBM, TBN, 2, 2> cur;
    cur.decode(grp, u);
    const int nk = grp.g[cur.p].k / BKW;
    for (int ls = 0; ls < nk; ++ls) {
      // 1. a chunk of the previous tile: image read-back, epilogue, stores
      const int c = pu >= 0 ? chunk_at(ls, nk) : -1;
      if (c >= 0) epi_chunk<EPI>(grp.g[prev.p], prev.m0, prev.n0, outb, c, e, lane);
      // 2. k-step gs + 4 into the stage of k-step gs (its fragments were read, and waited for, before the last
      //    barrier): three k-steps in flight
      const bool d = dma();
      // 3. k-step gs + 2 must have landed before the barrier (it is read in the next k-step): the operations
      //    issued after it are the last step's and this step's stores and DMAs
      const int younger = prev_ops + (c >= 0 ? SPC : 0) + (d ? NI_E : 0);
      vm_wait_n(younger);
      prev_ops = (c >= 0 ? SPC : 0) + (d ? NI_E : 0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    pu = u;
    prev = cur;
  }
  __builtin_amdgcn_s_barrier();   // B_tail
  __builtin_amdgcn_sched_barrier(0);
  if (pu >= 0)
    for (int c = 0; c < NCH; ++c) epi_chunk<EPI>(grp.g[prev.p], prev.m0, prev.n0, outb, c, e, lane);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_ws_kernel(GemmGroup grp) {
  __shared__ __attribute__((aligned(16))) uint16_t smem[LDS_E];
  if ((int)blockIdx.x >= grp.start[grp.count]) return;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w < 4) mfma_role<EPI>(grp, smem, smem + NSTG * STAGE, w, lane);
  else epi_role<EPI>(grp, smem, smem + NSTG * STAGE, w - 4, lane);
}

}  // namespace ws
}  // namespace k3m_b16
