// int8 MFMA tile engine shared by the certified search (ofr_knn_q8.hip) and the
// exact projection (ofr_qproj.hip).
//
// C[a][b] = sum_k A[a][k] * B[b][k] over int8 rows, v_mfma_i32_32x32x32_i8,
// int32 accumulators.  A tile = TA = 256 rows of A (gallery slices / W slices)
// by TQ rows of B (query slices / images).  Both operands are staged by
// LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 full 128-B row lines per
// wave-instruction, XOR swizzle applied to the per-lane SOURCE address) into
// 128-B LDS rows; a counted/zero `s_waitcnt vmcnt` + raw s_barrier separates
// the stages (no __syncthreads() in the loop: its fence would drain the DMA
// queue).  The k loop is branch-free (one scheduling region) and its schedule
// is pinned with sched_group_barrier: k-half-0 fragment reads, the stage's
// DMAs, then each k-half's MFMAs with the next k-half's reads threaded between
// them.
#pragma once
#include "ofr_common.h"

namespace ofr {
namespace i8t {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int TA = 256;                            // A rows per tile
constexpr int ROWB = 128;                          // LDS/global bytes per row and k step (one 128-B line)

// Two tile shapes share the engine (SL = int8 slices per row):
//   SL = 1: 256 x 256 tile, k step 128 (x1 only), 2 LDS stages of 64 KiB, 8 waves (2 per
//           SIMD: one wave's LDS-DMA issue and barrier wait hide behind the other's MFMAs),
//           each 128 x 64 (acc 4x2 blocks, 128 registers)
//   SL = 2: 256 x 128 tile, k step 64 (x1 | x2 per 128-B line), 3 stages of 48 KiB, 4 waves,
//           each 128 x 64 with two accumulator sets (256 registers)
template <int SL>
struct Shape {
  static constexpr int TQ = SL == 1 ? 256 : 128;
  static constexpr int NW = SL == 1 ? 8 : 4;       // waves per workgroup
  static constexpr int NT = NW * 64;
  static constexpr int WQ = NW / 2;                // wave grid: 2 (gallery) x WQ (queries)
  static constexpr int QW = TQ / WQ;               // queries per wave (64)
  static constexpr int BK = ROWB / SL;             // features per k step
  static constexpr int NST = SL == 1 ? 2 : 3;
  static constexpr int CT = QW / 32;               // 32-query blocks per wave
  static constexpr int NKS = BK / 32;              // MFMA k-halves per step (each MFMA: k = 32)
  static constexpr int PG = TA * ROWB, PQ = TQ * ROWB;
  static constexpr int STAGE = PG + PQ;
  static constexpr int LDS = NST * STAGE;          // 128 / 144 KiB
  static constexpr int IPW = (TA + TQ) / 8 / NW;   // DMA wave-instructions per wave per stage (8 / 12)
  static constexpr int YOUNG = (NST - 2) * IPW;    // DMAs allowed in flight at the stage wait
  static constexpr int NFRAG = 4 + CT;             // fragment reads per k-half per slice
  static constexpr int MF_PER_KS = 4 * CT * (SL == 1 ? 1 : 3);
};

// 128-B LDS rows = 8 chunks of 16 B, XOR-swizzled by ((row >> 1) & 7) so that the 16
// rows of a ds_read_b128 lane group hit 16 distinct bank quads.  SL = 1: chunk c holds
// features 16c..16c+15 of the step; SL = 2: chunks 0-3 slice 1, 4-7 slice 2.
__device__ __forceinline__ int off(int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4); }

// rows [r0, r0 + ROWS) of a slice matrix, k step kt -> LDS panel.
// One wave-instruction moves 8 full rows (8 x 128 B = 1 KiB, one 128-B line per row).
template <int ROWS, int NW>
__device__ __forceinline__ void dma(const int8_t* base, int64_t ld, int64_t rows, int64_t r0, char* panel, int kt,
                                    int64_t cols) {
  constexpr int PER = ROWS / 8 / NW;
  static_assert(PER * 8 * NW == ROWS, "DMA split");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int ins = wave * PER + t;
    const int row = ins * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((row >> 1) & 7);
    int64_t gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    int64_t col = (int64_t)kt * ROWB + chunk * 16;
    col = col < cols ? col : cols - 16;          // stays inside the row; the A side is zero there
    const int8_t* src = base + gr * ld + col;
    __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)src, (OFR_LDS void*)(panel + ins * 1024), 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else static_assert(N == 0 || N == 12, "vmcnt");
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}


// Main loop.  Wave (wr, wc) of the 2 x WQ grid owns A rows wr*128 + i*32 + (C/D row map)
// and B rows wc*QW + j*32 + lane&31 (C/D of v_mfma_i32_32x32x32_i8: column = lane & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)).
//   SL = 1: acc0 += A1 . B1
//   SL = 2: acc0 += A1 . B1,  acc1 += A2 . B1 + A1 . B2   (slices interleaved per 128-B line)
// XB / XA: B / A hold uint8 (images); fragments are turned into x - 128 by an XOR with 0x80.
// bcols: readable bytes per B row (DMA columns past it are clamped into the row; the
// matching A columns are zero).
template <int SL, bool XB, bool XA = false>
__device__ __forceinline__ void mainloop(char* smem, const int8_t* A, int64_t lda, int64_t arows, int64_t a0,
                                         const int8_t* Bm, int64_t ldb, int64_t brows, int64_t b0, int64_t bcols,
                                         int nk, i32x16 (&acc0)[4][Shape<SL>::CT],
                                         i32x16 (&acc1)[4][SL == 2 ? Shape<SL>::CT : 1]) {
  using S = Shape<SL>;
  constexpr int CT = S::CT, NKS = S::NKS, QW = S::QW;
  constexpr int NACC1 = SL == 2 ? CT : 1;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / S::WQ, wc = wave % S::WQ, h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
#pragma unroll
      for (int j = 0; j < CT; ++j) acc0[i][j][r] = 0;
#pragma unroll
      for (int j = 0; j < NACC1; ++j) acc1[i][j][r] = 0;
    }

  auto issue = [&](int kt) {
    char* st = smem + (kt % S::NST) * S::STAGE;
    dma<TA, S::NW>(A, lda, arows, a0, st, kt, lda);
    dma<S::TQ, S::NW>(Bm, ldb, brows, b0, st + S::PG, kt, bcols);
  };
  // Branch-free k loop (one scheduling region): the step issued at kt is
  // min(kt + NST - 1, nk - 1); past the end it re-loads the last step into the
  // stage nobody reads any more, which keeps the vmcnt bookkeeping constant.
  const int last = nk - 1;
#pragma unroll
  for (int s = 0; s < S::NST - 1; ++s) issue(s < last ? s : last);

  // fragments of one k-half, double-buffered by k-half parity
  i32x4 g1[2][4], q1[2][CT], g2[2][4], q2[2][CT];
  auto frags = [&](const char* st, int ks) {
    const int b = ks & 1;
    const int c = 2 * ks + h;   // 16-B chunk; SL = 2: slice 2 at c + 4
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      q1[b][j] = *reinterpret_cast<const i32x4*>(st + S::PG + off(wc * QW + j * 32 + r32, c));
      if constexpr (XB) q1[b][j] ^= (int)0x80808080;   // uint8 x -> int8 x - 128
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 128 + i * 32 + r32;
      g1[b][i] = *reinterpret_cast<const i32x4*>(st + off(row, c));
      if constexpr (XA) g1[b][i] ^= (int)0x80808080;
      if constexpr (SL == 2) g2[b][i] = *reinterpret_cast<const i32x4*>(st + off(row, c + 4));
    }
    if constexpr (SL == 2) {
#pragma unroll
      for (int j = 0; j < CT; ++j)
        q2[b][j] = *reinterpret_cast<const i32x4*>(st + S::PG + off(wc * QW + j * 32 + r32, c + 4));
    }
  };
  // SL = 2: the two products into acc1 sit 8 instructions apart (no RAW stall)
  auto mfmas = [&](int ks) {
    const int b = ks & 1;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        acc0[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g1[b][i], q1[b][j], acc0[i][j], 0, 0, 0);
        if constexpr (SL == 2)
          acc1[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g2[b][i], q1[b][j], acc1[i][j], 0, 0, 0);
      }
    if constexpr (SL == 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j)
          acc1[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g1[b][i], q2[b][j], acc1[i][j], 0, 0, 0);
    }
  };

  constexpr int NFR = S::NFRAG * SL;          // ds_read_b128 per k-half
  constexpr int MF = S::MF_PER_KS;            // MFMAs per k-half
  static_assert(MF >= NFR, "MFMA : read interleave");
  for (int kt = 0; kt < nk; ++kt) {
    wait_vm<S::YOUNG>();   // step kt landed; younger steps may stay in flight
    barrier();
    const char* st = smem + (kt % S::NST) * S::STAGE;
    frags(st, 0);
    {
      const int nx = kt + S::NST - 1;
      issue(nx < last ? nx : last);
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks + 1 < NKS) frags(st, ks + 1);
      mfmas(ks);
    }
    // schedule: k-half-0 reads, the DMAs, then each k-half's MFMAs with the next
    // k-half's reads front-loaded between them (1 : 1, so they land before they are
    // needed), then the last k-half's MFMAs
    __builtin_amdgcn_sched_group_barrier(0x100, NFR, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, S::IPW, 0);
#pragma unroll
    for (int ks = 0; ks + 1 < NKS; ++ks) {
#pragma unroll
      for (int r = 0; r < NFR; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MF - NFR, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
  }
  wait_vm<0>();
  barrier();

}

// Bijective XCD-aware remap of a 1-D grid: blocks b and b+8 share an XCD under
// round-robin dispatch; give each XCD a contiguous run of the tile sequence.
__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblocks) {
  const int64_t q = nblocks / 8, r = nblocks % 8;
  const int64_t x = bid % 8, s = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

// Tile order.  Tiles come in groups of gg A tiles x all B tiles; inside a group the
// A tile varies fastest.  With the XCD-contiguous remap, the ~32 workgroups resident
// on one XCD then cover gg A panels x 32/gg B panels, so both operands are shared in
// that XCD's L2.
__device__ __forceinline__ void tile_coords(int64_t t, int64_t gg_, int64_t nta, int64_t ntb, int64_t& at,
                                            int64_t& bt) {
  const int64_t group = t / (gg_ * ntb), within = t % (gg_ * ntb);
  const int64_t abase = group * gg_;
  const int64_t gg = nta - abase < gg_ ? nta - abase : gg_;
  bt = within / gg;
  at = abase + within % gg;
}

}  // namespace i8t
}  // namespace ofr
