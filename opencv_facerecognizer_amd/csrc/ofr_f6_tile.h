// fp6 (e2m3) MFMA tile engine of the certified search's first tier (ofr_knn_q8.hip).
//
// C[a][b] = sum_k A[a][k] * B[b][k] over e2m3 rows (values m/8 .. 7.5, exact products),
// v_mfma_scale_f32_32x32x64_f8f6f4 with both formats fp6 (cbsz = blgp = 2) and unit E8M0
// scales: the per-row scale is folded into the epilogue like the int8 tiers' scale.  The
// fp32 accumulation is the only inexact step: measured <= 3 * 2^-24 * sum|a b| over a
// 160-MFMA chain (tools/mx_probe.hip); the certificate budgets (nmfma + 64) * 2^-23.
// On gfx950 this instruction runs at twice the int8 MFMA rate per clock and moves 0.75 B
// per feature instead of 1.
//
// Global "f6 tiled" layout of a row set (gallery once, query batch per call), written by
// ofr_f6_quantize_rows: panels of 256 rows x stages of 128 features, one contiguous
// 24 KiB block per (panel, stage):
//     block(p, s) = base + (p * nst + s) * 24576
//     sub-block (j, h) at + (2j + h) * 6144       j = 64-feature MFMA step, h = 32-feature half
//         part0: 16 B per row at + row * 16       (4 KiB)
//         part1:  8 B per row at + 4096 + row * 8 (2 KiB)
// Features k = 128 s + 64 j + 32 h + e (e < 32) of a row form a 192-bit little-endian
// stream (part0 then part1), element e at bits 6e..6e+5 -- exactly the register image
// lane (h, r) of the MFMA takes for row r (tools/mx_probe.hip verified the map).  The
// LDS image of a stage is the same bytes: each DMA wave-instruction copies 1 KiB
// contiguous, and the fragment reads (ds_read_b128 of part0, ds_read_b64 of part1, 32
// consecutive rows per half-wave) are bank-conflict free without a swizzle.
#pragma once
#include "ofr_common.h"

namespace ofr {
namespace f6t {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TA = 256, TQ = 256;            // gallery x query rows per tile
constexpr int BK = 128;                      // features per stage
constexpr int PANEL = 24576;                 // bytes per (panel, stage) block = 256 rows x 96 B
constexpr int NW = 8, NT = NW * 64;          // 2 waves per SIMD
constexpr int WQ = 4, QW = TQ / WQ;          // wave grid 2 (gallery) x 4 (queries); 128 x 64 per wave
constexpr int CT = QW / 32;                  // 32-query blocks per wave (2)
constexpr int NST = 3;                       // LDS stages
constexpr int STAGE = 2 * PANEL;             // gallery block + query block
constexpr int LDS = NST * STAGE;             // 144 KiB
constexpr int IPW = STAGE / 1024 / NW;       // DMA wave-instructions per wave per stage (6)
constexpr int YOUNG = (NST - 2) * IPW;       // DMAs allowed in flight at the stage wait
constexpr int NFR = 2 * (4 + CT);            // ds_reads per MFMA step (b128 + b64 per fragment)
constexpr int MF = 4 * CT;                   // MFMAs per MFMA step

__host__ __device__ constexpr int64_t panels(int64_t rows) { return (rows + TA - 1) / TA; }
__host__ __device__ constexpr int64_t stages(int64_t d) { return (d + BK - 1) / BK; }
__host__ __device__ constexpr int64_t tiles_bytes(int64_t rows, int64_t d) {
  return panels(rows) * stages(d) * (int64_t)PANEL;
}

// Stage kt of gallery panel gp and query panel qp -> LDS stage buffer st:
// 48 wave-instructions of 1 KiB, waves 0-3 the gallery block, 4-7 the query block.
__device__ __forceinline__ void dma(const char* G, int64_t gp, const char* Q, int64_t qp, int64_t nst, int kt,
                                    char* st) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool gal = wave < 4;
  const char* blk = (gal ? G + (gp * nst + kt) * (int64_t)PANEL : Q + (qp * nst + kt) * (int64_t)PANEL);
  const int w4 = wave & 3;
  char* dst = st + (gal ? 0 : PANEL);
#pragma unroll
  for (int t = 0; t < IPW; ++t) {
    const int ins = w4 * IPW + t;
    __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)(blk + ins * 1024 + lane * 16),
                                     (OFR_LDS void*)(dst + ins * 1024), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else static_assert(N == 0 || N == 6, "vmcnt");
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ i32x8 frag(const char* blk, int j, int h, int row) {
  const char* sb = blk + (2 * j + h) * 6144;
  // opaque part1 address: keeps the compiler from pairing part1 reads of different
  // fragments into ds_read2_b64 (which lands them apart from part0 and costs v_movs)
  const OFR_LDS char* p1a = (const OFR_LDS char*)(sb + 4096 + row * 8);
  asm volatile("" : "+v"(p1a));
  const i32x4 p0 = *reinterpret_cast<const i32x4*>(sb + row * 16);
  const i32x2 p1 = *reinterpret_cast<const OFR_LDS i32x2*>(p1a);
  i32x8 f;
  f[0] = p0[0]; f[1] = p0[1]; f[2] = p0[2]; f[3] = p0[3];
  f[4] = p1[0]; f[5] = p1[1]; f[6] = 0; f[7] = 0;   // fp6: the MFMA reads v[0:5] only
  return f;
}

// Main loop.  Wave (wr, wc) owns gallery rows wr*128 + i*32 + (C/D row map) and query
// rows wc*64 + j*32 + lane&31 (C/D: column = lane & 31, row = (reg & 3) + 8 (reg >> 2) +
// 4 (lane >> 5)).  MODE 1/2: probe variants without k-loop DMA / without MFMA.
template <int MODE>
__device__ __forceinline__ void mainloop(char* smem, const char* G, int64_t gp, const char* Q, int64_t qp,
                                         int nst, f32x16 (&acc)[4][CT]) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / WQ, wc = wave % WQ, h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto issue = [&](int kt) { dma(G, gp, Q, qp, nst, kt, smem + (kt % NST) * STAGE); };
  // Branch-free k loop: the stage issued at kt is min(kt + NST - 1, last); past the end it
  // re-loads the last stage into the buffer nobody reads any more (constant vmcnt bookkeeping).
  const int last = nst - 1;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s < last ? s : last);

  i32x8 ga[2][4], qb[2][CT];
  auto frags = [&](const char* st, int j) {
#pragma unroll
    for (int c = 0; c < CT; ++c) qb[j][c] = frag(st + PANEL, j, h, wc * QW + c * 32 + r32);
#pragma unroll
    for (int i = 0; i < 4; ++i) ga[j][i] = frag(st, j, h, wr * 128 + i * 32 + r32);
  };
  auto mfmas = [&](int j) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < CT; ++c)
        acc[i][c] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(ga[j][i], qb[j][c], acc[i][c], 2, 2, 0,
                                                                    0x7f7f7f7f, 0, 0x7f7f7f7f);
  };

  for (int kt = 0; kt < nst; ++kt) {
    if constexpr (MODE == 1) wait_vm<0>();
    else wait_vm<YOUNG>();   // stage kt landed; the younger stage may stay in flight
    barrier();
    const char* st = smem + (kt % NST) * STAGE;
    frags(st, 0);
    if constexpr (MODE != 1) {
      const int nx = kt + NST - 1;
      issue(nx < last ? nx : last);
    }
    frags(st, 1);
    if constexpr (MODE != 2) {
      mfmas(0);
      mfmas(1);
    }
    // schedule: step-0 reads, the DMAs, step-0 MFMAs with step-1 reads threaded between
    // them (2 reads after each of the first 4, 1 after each of the last 4), step-1 MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, NFR, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, IPW, 0);
    static_assert(NFR == 12 && MF == 8, "schedule below");
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
  }
  wait_vm<0>();
  barrier();
}

}  // namespace f6t
}  // namespace ofr
