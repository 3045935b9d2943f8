// fp32-MFMA tile engine of the search kernels (ofr_knn.hip).
//
// One workgroup = 256 threads = 4 waves (one per SIMD) computes a TM x TN
// tile of  C[a][b] = sum_k A[a][k] * B[b][k]  with v_mfma_f32_32x32x2_f32
// (exact f32 products, f32 accumulation).  A = gallery rows, B = query rows;
// both are "rows with k contiguous", so a tile is two [rows][BK] LDS panels.
// Waves are arranged WM x WN; each owns (TM/WM) x (TN/WN) = RT x CT MFMA
// blocks of 32x32.
//
//   Big   (B >= 256):  TN = 256, 2x2 waves, 128x128 per wave, 2 stages  -> MFMA-bound
//   Small (B <= 32):   TN = 32,  4x1 waves,  64x32  per wave, 4 stages  -> HBM-bound
//                      streaming of the gallery (each row read once per batch)
//
// LDS image per operand and stage: [rows][32 fp32] = 128-B rows, 16-B chunks
// XOR-swizzled by ((row>>1)&7) so the ds_read_b128 fragment reads (16 rows x
// same chunk per lane group) hit 16 distinct 4-bank slots.  Both operands
// are staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows per
// wave-instruction) with the swizzle applied to the per-lane SOURCE address.
// NST stages: panel kt+NST-1 is issued after the barrier that retires panel
// kt-1's readers; a counted `s_waitcnt vmcnt` keeps the younger panels in
// flight across the raw s_barrier (no __syncthreads() in the loop: its fence
// would drain the DMA queue).
#pragma once
#include "ofr_common.h"

namespace ofr {
namespace tile {

constexpr int TM = 256;  // gallery rows per tile
constexpr int BK = 32;   // k per LDS panel
constexpr int NTHREADS = 256;

template <int TN_, int WM_, int WN_, int NST_>
struct Cfg {
  static constexpr int TN = TN_, WM = WM_, WN = WN_, NST = NST_;
  static constexpr int RT = TM / (WM * 32);   // 32-row gallery blocks per wave
  static constexpr int CT = TN / (WN * 32);   // 32-row query blocks per wave
  static constexpr int PANEL_A = TM * BK * 4;
  static constexpr int PANEL_B = TN * BK * 4;
  static constexpr int STAGE = PANEL_A + PANEL_B;
  static constexpr int LDS = NST * STAGE;
  static constexpr int INS_A = TM / 8 / 4;    // DMA wave-instructions per wave per panel
  static constexpr int INS_B = TN / 8 / 4 > 0 ? TN / 8 / 4 : 1;
  static constexpr int B_WAVES = TN / 8 < 4 ? TN / 8 : 4;   // waves that stage B (TN=16 -> 2)
  static_assert(WM * WN == 4, "4 waves");
  static_assert(RT >= 1 && CT >= 1, "tile too small for the wave grid");
  static_assert(TN >= 32, "every wave must issue the same DMA count (counted vmcnt)");
};
using CfgBig = Cfg<256, 2, 2, 2>;
using CfgSmall = Cfg<32, 4, 1, 4>;

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + swz_chunk(row, chunk) * 16; }

// rows [r0, r0 + ROWS) of M [rows][ld] (clamped to rows-1), k panel kt -> LDS panel (swizzled)
template <int ROWS>
__device__ __forceinline__ void dma_panel(const float* base, int64_t ld, int64_t rows, int64_t r0, char* panel, int kt) {
  constexpr int NINS = ROWS / 8;                 // 8 rows per wave-instruction
  constexpr int PER_WAVE = NINS >= 4 ? NINS / 4 : 1;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < PER_WAVE; ++t) {
    const int ins = wave * PER_WAVE + t;
    if (NINS < 4 && ins >= NINS) break;          // narrow panels: only the first waves stage them
    const int row = ins * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    int64_t grow = r0 + row;
    grow = grow < rows ? grow : rows - 1;
    const float* src = base + grow * ld + (int64_t)kt * BK + chunk * 4;
    __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)src, (OFR_LDS void*)(panel + ins * 1024), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (N == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if constexpr (N == 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if constexpr (N == 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // conservative
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// acc[rt][ct]: C/D map of v_mfma_f32_32x32x2_f32: col (query) = lane&31,
// row (gallery) = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
template <class C>
__device__ __forceinline__ void mainloop(char* smem, const float* A, int64_t lda, int64_t arows, int64_t a0,
                                         const float* Bm, int64_t ldb, int64_t brows, int64_t b0, int nk,
                                         f32x16 (&acc)[C::RT][C::CT]) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wr = wave / C::WN;
  const int wc = wave % C::WN;
  const int h = lane >> 5;
  const int r32 = lane & 31;
  // DMA instructions issued per wave per panel (for the counted waits)
  constexpr int IPW = C::INS_A + ((C::TN / 8) >= 4 ? C::INS_B : 1);

#pragma unroll
  for (int i = 0; i < C::RT; ++i)
#pragma unroll
    for (int j = 0; j < C::CT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // prologue: panels 0 .. NST-2
#pragma unroll
  for (int s = 0; s < C::NST - 1; ++s) {
    if (s < nk) {
      char* st = smem + s * C::STAGE;
      dma_panel<TM>(A, lda, arows, a0, st, s);
      dma_panel<C::TN>(Bm, ldb, brows, b0, st + C::PANEL_A, s);
    }
  }

  int arow[C::RT], brow[C::CT];
#pragma unroll
  for (int t = 0; t < C::RT; ++t) arow[t] = wr * (C::RT * 32) + t * 32 + r32;
#pragma unroll
  for (int t = 0; t < C::CT; ++t) brow[t] = wc * (C::CT * 32) + t * 32 + r32;

  for (int kt = 0; kt < nk; ++kt) {
    // panel kt must have landed; panels kt+1 .. kt+NST-2 may stay in flight
    const int younger = min(nk - 1 - kt, C::NST - 2);
    if (younger >= C::NST - 2) wait_vmcnt<(C::NST - 2) * IPW>();
    else wait_vmcnt<0>();
    barrier();   // every wave's panel-kt DMA landed; every wave finished reading panel kt-1
    {
      const int nxt = kt + C::NST - 1;
      if (nxt < nk) {
        char* st = smem + (nxt % C::NST) * C::STAGE;
        dma_panel<TM>(A, lda, arows, a0, st, nxt);
        dma_panel<C::TN>(Bm, ldb, brows, b0, st + C::PANEL_A, nxt);
      }
    }
    const char* cur = smem + (kt % C::NST) * C::STAGE;
#pragma unroll
    for (int kb = 0; kb < BK / 8; ++kb) {
      f32x4 a[C::RT], b[C::CT];
      const int chunk = 2 * kb + h;
#pragma unroll
      for (int t = 0; t < C::RT; ++t) a[t] = *reinterpret_cast<const f32x4*>(cur + lds_off(arow[t], chunk));
#pragma unroll
      for (int t = 0; t < C::CT; ++t)
        b[t] = *reinterpret_cast<const f32x4*>(cur + C::PANEL_A + lds_off(brow[t], chunk));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < C::RT; ++i)
#pragma unroll
          for (int j = 0; j < C::CT; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
    }
  }
  wait_vmcnt<0>();
  barrier();   // LDS free for the epilogue
}

// Bijective XCD-aware remap of a 1-D grid: blocks b and b+8 share an XCD under
// round-robin dispatch; give each XCD a contiguous run of the tile sequence.
// (Speed only — any placement is correct.)
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblocks) {
  const int64_t q = nblocks / 8, r = nblocks % 8;
  const int64_t x = bid % 8, s = bid / 8;
  const int64_t start = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return start + s;
}

}  // namespace tile
}  // namespace ofr
