// fp6 (e2m3) MFMA tile engine of the certified search's first tier (ofr_knn_q8.hip).
//
// C[a][b] = sum_k A[a][k] * B[b][k] over e2m3 rows (values m/8 .. 7.5, exact products),
// v_mfma_scale_f32_32x32x64_f8f6f4 with both formats fp6 (cbsz = blgp = 2).  Per-row fp32 scales are
// folded into the epilogue like the int8 tiers' scale; the E8M0 block scales of the MFMA carry
// per-COLUMN-block scales (round 5, "bscale"): one byte per 32 features, the same for the gallery
// and the query rows, so an element decodes to s_row * 2^(bscale[k / 32] - 127) * v and the MFMA
// applies 2^(2 e_B) to each block's products (both operands take the block's byte).  A trained
// Fisherfaces W concentrates the feature variance in its leading columns (LDA eigenvalue order):
// one row scale would leave the other columns a few fp6 steps (residual 0.11 of the row norm against
// 0.029 on isotropic rows); column-block scales equalise the blocks first.  The
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
//         part1:  8 B per row at + 4096 + slot * 8 (2 KiB), slot = row ^ 16 h (p1_slot)
// Features k = 128 s + 64 j + 32 h + e (e < 32) of a row form a 192-bit little-endian
// stream (part0 then part1), element e at bits 6e..6e+5 -- exactly the register image
// lane (h, r) of the MFMA takes for row r (tools/mx_probe.hip verified the map).  The
// LDS image of a stage is the same bytes: each DMA wave-instruction copies 1 KiB
// contiguous.  Fragment reads are bank-conflict free for both MFMA shapes: 32x32x64 (a
// half-wave reads 32 consecutive rows of one sub-block: part0 ds_read_b128 and part1
// ds_read_b64, whose slot swizzle only permutes inside the 32 rows) and 16x16x128 (lanes
// 16q..16q+15 read 16 rows of sub-block q: the odd sub-blocks' part1 rows sit 16 slots away,
// in the other half of the 64 banks the b64 lane group {0-31} / {32-63} spans).
#pragma once
#include <type_traits>

#include "ofr_common.h"

namespace ofr {
namespace f6t {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x6 __attribute__((ext_vector_type(6)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int TA = 256, TQ = 256;            // gallery x query rows per tile
constexpr int BK = 128;                      // features per stage
constexpr int PANEL = 24576;                 // bytes per (panel, stage) block = 256 rows x 96 B
constexpr int NST = 3;                       // LDS stages
constexpr int STAGE = 2 * PANEL;             // gallery block + query block
constexpr int LDS = NST * STAGE;             // 144 KiB
constexpr int DMA_INS = STAGE / 1024;        // 1-KiB DMA wave-instructions per stage (48)

__host__ __device__ constexpr int p1_slot(int jh, int row) { return row ^ ((jh & 1) << 4); }
__host__ __device__ constexpr int64_t panels(int64_t rows) { return (rows + TA - 1) / TA; }
__host__ __device__ constexpr int64_t stages(int64_t d) { return (d + BK - 1) / BK; }
__host__ __device__ constexpr int64_t tiles_bytes(int64_t rows, int64_t d) {
  return panels(rows) * stages(d) * (int64_t)PANEL;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// ---- passes over several segments of stages (the two-slice tier f6x2) -----------------------
// NSEG = 1: stages [0, nst) of the gallery tiles G against the query tiles Q (tier f6).
// NSEG = 3: stages [0, 3 nst) = the segments [x1 | x1 | x2] . [y1 | y2 | y1] of the two-slice rows
// x~ = s (x1 + 2^-4 x2): segment 1 runs the MFMA with query block scale 2^-4, segment 2 with gallery
// block scale 2^-4 (E8M0 operands), so one accumulator holds x1.y1 + 2^-4 (x1.y2 + x2.y1) exactly
// up to the fp32 accumulation.  G2 / Q2: the second-slice tiles (same layout).
constexpr int SCALE_ONE = 0x7f7f7f7f;    // E8M0 2^0 in every byte
constexpr int SCALE_X2 = 0x7b7b7b7b;     // E8M0 2^-4
constexpr int X2_SHIFT = 4;              // second slice weight 2^-X2_SHIFT

// Column-block scales of stage ks: 4 E8M0 bytes, blocks 4 ks .. 4 ks + 3 (bs: never null -- the host
// passes a table of unit scales, q8s::unit_bscale, when the caller gives none).
//
// In the tile engines the dword comes in by an explicit scalar load (s_load_dword, inline asm) and is
// turned into the lane's operand by an asm VALU shift placed right behind one of the engine's own
// s_waitcnt lgkmcnt(0) (asm volatile statements keep their order).  A plain C++ load of it is not
// selected as a scalar load (the kernels write global memory, so it is not provably unclobbered): it
// becomes a vector load whose vmcnt the compiler then waits for among the stage copies, and its use
// gets hoisted to the top of the next stage (measured: an s_waitcnt vmcnt(13) at every stage top).
// The untracked scalar load only ever makes the compiler's own lgkmcnt waits stricter (LDS returns in
// order; an extra outstanding operation can only delay the count).
__device__ __forceinline__ uint32_t sload_bscale(const uint32_t* bs, int ks) {
  uint32_t raw;
  // uniform, but the compiler may hold it in a VGPR: the "s" constraint alone does not move it
  const uint32_t off = (uint32_t)__builtin_amdgcn_readfirstlane((int)(4u * (uint32_t)ks));
  asm volatile("s_load_dword %0, %1, %2" : "=s"(raw) : "s"(bs), "s"(off) : "memory");
  return raw;
}
// raw >> lsh (the lane's byte in the low byte), after the caller's lgkmcnt(0): asm, so that it stays
// behind that wait
__device__ __forceinline__ int lane_byte(uint32_t raw, uint32_t lsh) {
  int v;
  asm volatile("v_lshrrev_b32_e64 %0, %1, %2" : "=v"(v) : "v"(lsh), "s"(raw));
  return v;
}
// The MFMA scale operands of stage kt from the lane's block byte v (the operand reads the low byte
// only), minus the segment's 2^-4 on a second slice.  The block bytes are >= 0x40
// (ofr_f6_block_scales), so the subtraction stays inside the low byte.
template <int NSEG>
__device__ __forceinline__ void block_scales(int v, int kt, int nst, int& sa, int& sb) {
  if constexpr (NSEG == 1) {
    sa = v; sb = v;
  } else {
    sa = kt >= 2 * nst ? v - X2_SHIFT : v;
    sb = (kt >= nst && kt < 2 * nst) ? v - X2_SHIFT : v;
  }
}
// the stage of segment-relative index ks of stage kt (NSEG segments of nst stages)
template <int NSEG>
__device__ __forceinline__ int seg_stage(int kt, int nst) {
  if constexpr (NSEG == 1) return kt;
  else return kt - (kt >= 2 * nst ? 2 : (kt >= nst ? 1 : 0)) * nst;
}

template <int NSEG>
__device__ __forceinline__ void seg_src(int kt, int nst, const char* G, const char* G2, const char* Q, const char* Q2,
                                        const char*& g, const char*& q, int& ks) {
  if constexpr (NSEG == 1) {
    g = G; q = Q; ks = kt;
  } else {
    static_assert(NSEG == 3, "segments");
    const int sg = kt >= 2 * nst ? 2 : (kt >= nst ? 1 : 0);
    ks = kt - sg * nst;
    g = sg == 2 ? G2 : G;
    q = sg == 1 ? Q2 : Q;
  }
}

__device__ __forceinline__ i32x8 frag(const char* blk, int j, int h, int row) {
  const char* sb = blk + (2 * j + h) * 6144;
  // opaque part1 address: keeps the compiler from pairing part1 reads of different
  // fragments into ds_read2_b64 (which lands them apart from part0 and costs v_movs)
  const OFR_LDS char* p1a = (const OFR_LDS char*)(sb + 4096 + p1_slot(h, row) * 8);
  asm volatile("" : "+v"(p1a));
  const i32x4 p0 = *reinterpret_cast<const i32x4*>(sb + row * 16);
  const i32x2 p1 = *reinterpret_cast<const OFR_LDS i32x2*>(p1a);
  i32x8 f;
  f[0] = p0[0]; f[1] = p0[1]; f[2] = p0[2]; f[3] = p0[3];
  f[4] = p1[0]; f[5] = p1[1]; f[6] = 0; f[7] = 0;   // fp6: the MFMA reads v[0:5] only
  return f;
}

// The tile engine for NW waves: NW = 8 (2 per SIMD, 128 x 64 per wave, wave grid 2 x 4) or
// NW = 4 (1 per SIMD, 128 x 128 per wave, grid 2 x 2: a third fewer fragment bytes per MFMA,
// 256 accumulators per lane in AGPRs).  Wave (wr, wc) owns gallery rows wr*128 + i*32 + (C/D
// row map) and query rows wc*QW + c*32 + lane&31 (C/D: column = lane & 31, row = (reg & 3) +
// 8 (reg >> 2) + 4 (lane >> 5)).
template <int NW_>
struct Engine {
  static constexpr int NW = NW_, NT = NW * 64;
  static constexpr int WQ = NW / 2, QW = TQ / WQ;   // query columns per wave
  static constexpr int CT = QW / 32;                // 32-query blocks per wave
  static constexpr int IPW = DMA_INS / NW;          // DMA wave-instructions per wave per stage
  static constexpr int NFR = 2 * (4 + CT);          // ds_reads per MFMA step (b128 + b64 per fragment)
  static constexpr int MF = 4 * CT;                 // MFMAs per MFMA step
  static_assert(NW == 4 || NW == 8, "engine");

  // Stage kt of gallery panel gp and query panel qp -> LDS stage buffer st: DMA_INS
  // wave-instructions of 1 KiB, the first half the gallery block, the second the query block.
  static __device__ __forceinline__ void dma(const char* G, int64_t gp, const char* Q, int64_t qp, int64_t nst,
                                             int kt, char* st) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char* gb = G + (gp * nst + kt) * (int64_t)PANEL;
    const char* qb = Q + (qp * nst + kt) * (int64_t)PANEL;
#pragma unroll
    for (int t = 0; t < IPW; ++t) {
      const int ins = wave * IPW + t;   // gallery: ins < 24 (a wave's instructions never straddle)
      const bool gal = ins < DMA_INS / 2;
      const int off = (gal ? ins : ins - DMA_INS / 2) * 1024;
      __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)((gal ? gb : qb) + off + lane * 16),
                                       (OFR_LDS void*)(st + (gal ? 0 : PANEL) + off), 16, 0, 0);
    }
  }

  // The same copies by MUBUF buffer_load ... lds, issued by waves 0-3 alone (12 pieces each; waves
  // 4-7 issue none, so one wave of every SIMD keeps the matrix pipe fed while the other pays the
  // copies' issue cost: Engine16's loop).  A FLAT global_load_lds in flight makes the compiler's
  // waitcnt pass treat LDS reads as unordered (every first use of a fresh fragment then waits
  // lgkmcnt(0)); the buffer form keeps them counted.  One descriptor per operand panel (nst stages,
  // < 2^32 bytes), voffset = stage + instruction + lane; the wave index is scalar, so the
  // descriptor choice stays uniform (no waterfall loop).
  static __device__ __forceinline__ void dma_buf4(const char* G, int64_t gp, const char* Q, int64_t qp, int64_t nst,
                                                  int kt, char* st) {
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    if (wave >= 4) return;
    const int pb = (int)(nst * PANEL);
    __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(G + gp * nst * (int64_t)PANEL), 0, pb,
                                                                  0x00020000);
    __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)(Q + qp * nst * (int64_t)PANEL), 0, pb,
                                                                  0x00020000);
#pragma unroll
    for (int t = 0; t < 2 * IPW; ++t) {
      const int ins = wave * 2 * IPW + t;
      const bool gal = ins < DMA_INS / 2;
      const int off = (gal ? ins : ins - DMA_INS / 2) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(gal ? rg : rq, (OFR_LDS void*)(st + (gal ? 0 : PANEL) + off), 16,
                                               kt * PANEL + off + lane * 16, 0, 0, 0);
    }
  }

  // reads threaded through MFMAs: NFR reads over MF MFMAs, front-loaded (2 after each MFMA while
  // they last, then 1, then none)
  static __device__ __forceinline__ void interleave() {
    constexpr int two = NW == 8 ? 4 : 8;   // MFMAs followed by 2 reads
    constexpr int one = NW == 8 ? 4 : 0;   // then by 1
    static_assert(2 * two + one == NFR && two + one <= MF, "schedule");
#pragma unroll
    for (int r = 0; r < two; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
#pragma unroll
    for (int r = 0; r < one; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    if constexpr (MF - two - one > 0) __builtin_amdgcn_sched_group_barrier(0x008, MF - two - one, 0);
  }

  // Main loop, stage hand-off in the middle of a stage.  Per stage kt:
  //   A: fragments (kt, j=1) read between the MFMAs of (kt, j=0)
  //   wait for stage kt+1 to land, barrier (every wave has read all of stage kt)
  //   B: fragments (kt+1, j=0) read between the MFMAs of (kt, j=1); DMA of stage kt+3 into
  //      kt's buffer after the first MFMA
  // so every fragment read has a block of MFMAs to land behind and each barrier falls while
  // the matrix pipe still drains the previous block (2 % faster than a hand-off at the stage
  // boundary, which exposes the step-0 reads after every barrier: the round-1 engine probe).
  // Fragments double-buffered by j; 3 LDS stages (kt+1 read next, kt+2 and kt+3 in flight).
  // NSEG: segments of nst stages each (seg_src); G2 / Q2 only for NSEG = 3.  nst = the panels' stage
  // count (layout); nsp = the stages run per segment: nst, or with NSEG = 1 a prefix (the prefix tier)
  template <int NSEG = 1>
  static __device__ __forceinline__ void mainloop(char* smem, const char* G, int64_t gp, const char* Q, int64_t qp,
                                                  int nst, int nsp, f32x16 (&acc)[4][CT], const char* G2 = nullptr,
                                                  const char* Q2 = nullptr, const uint32_t* bs = nullptr) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave / WQ, wc = wave % WQ, h = lane >> 5, r32 = lane & 31;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto issue = [&](int kt) {
      const char *g, *q;
      int ks;
      seg_src<NSEG>(kt, nst, G, G2, Q, Q2, g, q, ks);
      dma(g, gp, q, qp, nst, ks, smem + (kt % NST) * STAGE);
    };
    // branch-free: a stage past the end re-loads the last one onto itself (same bytes)
    const int last = NSEG * nsp - 1;
    static_assert(NST == 3, "hand-off below assumes 3 stages");
#pragma unroll
    for (int s = 0; s < NST; ++s) issue(s < last ? s : last);

    // block scales: MFMA step j of a stage covers blocks 2 j + h of its four (the lane's half h)
    const uint32_t lsh0 = 8u * (uint32_t)h, lsh1 = 8u * (uint32_t)(2 + h);
    int sa[2], sb[2];
    auto scales = [&](uint32_t raw, int kt, int (&xa)[2], int (&xb)[2]) {   // behind an lgkmcnt(0)
      block_scales<NSEG>(lane_byte(raw, lsh0), kt, nst, xa[0], xb[0]);
      block_scales<NSEG>(lane_byte(raw, lsh1), kt, nst, xa[1], xb[1]);
    };
    {
      const uint32_t raw0 = sload_bscale(bs, seg_stage<NSEG>(0, nst));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      scales(raw0, 0, sa, sb);
    }

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
                                                                      sa[j], 0, sb[j]);
    };

    wait_vm<2 * IPW>();   // stage 0 landed; 1 and 2 may be in flight
    barrier();
    frags(smem, 0);
    for (int kt = 0; kt < last; ++kt) {
      // the next stage's block scales: a scalar load here, read after the barrier below (whose
      // lgkmcnt(0) it joins), so the wait for it never drains fresh fragment reads
      const uint32_t raw = sload_bscale(bs, seg_stage<NSEG>(kt + 1, nst));
      frags(smem + (kt % NST) * STAGE, 1);
      mfmas(0);
      interleave();
      wait_vm<IPW>();     // stage kt+1 landed; kt+2 may be in flight
      barrier();
      int na[2], nb[2];
      scales(raw, kt + 1, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      {
        const int nx = kt + NST;
        issue(nx < last ? nx : last);
      }
      frags(smem + ((kt + 1) % NST) * STAGE, 0);
      mfmas(1);
      interleave();
      __builtin_amdgcn_sched_group_barrier(0x020, IPW, 0);
      sa[0] = na[0]; sa[1] = na[1]; sb[0] = nb[0]; sb[1] = nb[1];
    }
    frags(smem + (last % NST) * STAGE, 1);
    mfmas(0);
    interleave();
    mfmas(1);
    wait_vm<0>();
    barrier();
  }
};

// ---- 16x16x128 engine (the sieve pass) -------------------------------------------------------
// Same stages, LDS image and DMA as Engine<8>; the MFMA is v_mfma_scale_f32_16x16x128_f8f6f4: on
// random fp6 operands the chip holds a higher clock for it than for the 32x32x64 form, +14 %
// sustained rate at equal work (tools/f6_shape_probe.hip).  One MFMA k-step = one 128-feature
// stage.  Lane l holds rows (l % 16) of a 16-row block and the 32 features of sub-block
// q = l / 16 (the f6 tiled sub-blocks are exactly these 32-feature groups).  C/D: query column
// l % 16 of the 16-query block, gallery rows 4 (l / 16) + reg.
// 8 waves (2 per SIMD), wave grid 2 x 4 as Engine<8>: wave (wr, wc) owns gallery rows
// wr*128 + 16 i + .. (i < 8) and queries wc*64 + 16 c + l % 16 (c < 4): 32 accumulators of 4.
struct Engine16 {
  static constexpr int NW = 8, NT = 512, WQ = 4, QW = 64, NA = 8, NB = 4;
  static constexpr int IPW = DMA_INS / NW;   // 6

  // fragments live as 6 registers (the fp6 MFMA reads v[0:5] of its 8-register operand slot)
  static __device__ __forceinline__ i32x6 frag16(const char* st, int row) {
    const int q = (threadIdx.x & 63) >> 4;
    const char* sb = st + q * 6144;
    i32x6 f;
    const OFR_LDS char* p1a = (const OFR_LDS char*)(sb + 4096 + p1_slot(q, row) * 8);
    asm volatile("" : "+v"(p1a));
    const i32x4 p0 = *reinterpret_cast<const i32x4*>(sb + row * 16);
    const i32x2 p1 = *reinterpret_cast<const OFR_LDS i32x2*>(p1a);
    f[0] = p0[0]; f[1] = p0[1]; f[2] = p0[2]; f[3] = p0[3]; f[4] = p1[0]; f[5] = p1[1];
    return f;
  }
  static __device__ __forceinline__ f32x4 mfma(const i32x6& a, const i32x6& b, const f32x4& c, int sa = SCALE_ONE,
                                               int sb = SCALE_ONE) {
    const i32x8 a8 = __builtin_shufflevector(a, a, 0, 1, 2, 3, 4, 5, -1, -1);
    const i32x8 b8 = __builtin_shufflevector(b, b, 0, 1, 2, 3, 4, 5, -1, -1);
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, c, 2, 2, 0, sa, 0, sb);
  }

  // Main loop (round 2-3 measurements in DESIGN.md §5: 23.3 -> 22.5 ms for the split barrier and the
  // MUBUF copies, 23.1 -> 22.6 ms for the copies issued by waves 0-3 alone).  The stage copies are
  // MUBUF buffer_load ... lds pieces issued by waves 0-3 (Engine<8>::dma_buf4), so no FLAT instruction
  // is ever in flight and the compiler counts the LDS reads.  Two barriers per stage kt:
  //   top: stage kt+1 landed (own copies: vmcnt) and visible (s_barrier) -- no LDS drain;
  //   after row 0 (whose refill a[0] is the only LDS read issued so far in the stage): lgkmcnt(2)
  //   (every read of stage kt's buffer, all issued in stage kt-1, is done) + s_barrier, then stage
  //   kt+3's copy into that buffer: 1.9 stages of copy lead out of three buffers.
  // Per stage the MFMAs of stage kt, each fragment replaced by stage kt+1's as soon as its last MFMA
  // is issued (A-major: a[i] after row i's 4 MFMAs, b[c] after row 7's MFMA c), so the fragments
  // need no second register set (acc 128 + fragments 72 registers).
  template <int NSEG = 1>
  static __device__ __forceinline__ void mainloop(char* smem, const char* G, int64_t gp, const char* Q, int64_t qp,
                                                  int nst, int nsp, f32x4 (&acc)[NA][NB], const char* G2 = nullptr,
                                                  const char* Q2 = nullptr, const uint32_t* bs = nullptr) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wr = wave / WQ, wc = wave % WQ, r16 = lane & 15;
    const uint32_t lsh = 8u * (uint32_t)(lane >> 4);   // the lane's 32-feature block of a stage
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int c = 0; c < NB; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int last = NSEG * nsp - 1;   // nsp: stages run per segment (Engine<8>::mainloop)
    auto issue = [&](int kt) {
      const char *g, *q;
      int ks;
      seg_src<NSEG>(kt, nst, G, G2, Q, Q2, g, q, ks);
      Engine<8>::dma_buf4(g, gp, q, qp, nst, ks, smem + (kt % NST) * STAGE);
    };
#pragma unroll
    for (int s = 0; s < NST; ++s) {   // buffer s takes stage min(s, last)
      const char *g, *q;
      int ks;
      seg_src<NSEG>(s < last ? s : last, nst, G, G2, Q, Q2, g, q, ks);
      Engine<8>::dma_buf4(g, gp, q, qp, nst, ks, smem + (s % NST) * STAGE);
    }
    i32x6 a[NA], b[NB];
    int sa, sb;
    {
      const uint32_t raw0 = sload_bscale(bs, seg_stage<NSEG>(0, nst));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      block_scales<NSEG>(lane_byte(raw0, lsh), 0, nst, sa, sb);
    }
    auto mm = [&](const i32x6& x, const i32x6& y, f32x4& c) { c = mfma(x, y, c, sa, sb); };
    auto readA = [&](const char* st, int i) { a[i] = frag16(st, wr * 128 + i * 16 + r16); };
    auto readB = [&](const char* st, int c) { b[c] = frag16(st + PANEL, wc * QW + c * 16 + r16); };
    wait_vm<4 * IPW>();
    barrier();
#pragma unroll
    for (int i = 0; i < NA; ++i) readA(smem, i);
#pragma unroll
    for (int c = 0; c < NB; ++c) readB(smem, c);
    for (int kt = 0; kt < last; ++kt) {
      const uint32_t raw = sload_bscale(bs, seg_stage<NSEG>(kt + 1, nst));   // the next stage's block scales
      __builtin_amdgcn_sched_barrier(0);
      wait_vm<2 * IPW>();   // stage kt+1 landed (kt+2 may be in flight)
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      const char* nxt = smem + ((kt + 1) % NST) * STAGE;
#pragma unroll
      for (int c = 0; c < NB; ++c) mm(a[0], b[c], acc[0][c]);
      readA(nxt, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_barrier(0);
      // Every read of the previous stage (all from the buffer re-filled below) must be done: with only
      // the refill's two LDS reads in flight lgkmcnt(2) would do (round 2), but the next stage's block
      // scales (a scalar load, out of order) share the counter, so this engine waits for all of them
      // (the non-default sieve engine, OFR_F6_SHAPE=16, and its two-slice pass).
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      int na, nb;
      block_scales<NSEG>(lane_byte(raw, lsh), kt + 1, nst, na, nb);
      __builtin_amdgcn_sched_barrier(0);
      {
        const int nx = kt + NST;
        issue(nx < last ? nx : last);
      }
#pragma unroll
      for (int i = 1; i < NA - 1; ++i) {
#pragma unroll
        for (int c = 0; c < NB; ++c) mm(a[i], b[c], acc[i][c]);
        readA(nxt, i);
      }
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        mm(a[NA - 1], b[c], acc[NA - 1][c]);
        readB(nxt, c);
      }
      readA(nxt, NA - 1);
      __builtin_amdgcn_sched_group_barrier(0x020, IPW, 0);
#pragma unroll
      for (int i = 1; i < NA - 1; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      sa = na;
      sb = nb;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int c = 0; c < NB; ++c) mm(a[i], b[c], acc[i][c]);
    wait_vm<0>();
    barrier();
  }
};

// ---- wide engine: 384 gallery x 256 query tiles, one wave per SIMD (round 3) -------------------
// The 256 x 256 engines move 48 KiB into the CU per 256x256x128 stage and read 144 KiB of fragments
// out of LDS for it; both streams cost SIMD issue time that does not overlap the MFMAs.
// A 384 x 256 tile moves 60 KiB per 384x256x128 stage (-17 % per MAC), and one wave per SIMD with a
// 192 x 128 wave tile (96 accumulators of 4 = 384 registers, the rest of the 512-entry file for
// fragments) reads 20 fragments per wave and stage (-44 % per MAC against 8 waves of 128 x 64).
// Wave w: gallery rows WR*192 + 16 i (i < 12), queries WC*128 + 16 c (c < 8), WR = w >> 1, WC = w & 1.
//
// LDS: gallery ring of 3 slots (36 KiB: the tile's three 128-row half panels of the stage), query
// ring of 2 slots (24 KiB: the query panel's stage block, its global image).  A half-panel image keeps
// the global sub-block structure at half size: sub-block q at q * 3 KiB, part0 (16 B per row) then
// part1 (8 B per row at slot r ^ 16 (q & 1), the global p1_slot), so every piece of a copy is 1 KiB
// contiguous on both sides and the fragment reads stay bank-conflict free.
// Per stage s and row i (12 rows of 8 MFMAs, the gallery fragments through a ring of 3 read two rows
// ahead, the 8 query fragments held and refilled for s + 1 after their last MFMA in row 11):
//   row 1 start : barrier A (every wave's reads of Q(s), issued in row 11 of s - 1, done)
//   rows 1 - 6  : one piece of Q(s + 2) per row into Q(s)'s slot (6 per wave, 24 per stage)
//   rows 0 - 6  : one piece of G(s + 2) per row (pieces 2..8 of the wave's 9) into G(s - 1)'s slot
//   row 10 start: own copies of G(s + 1), Q(s + 1) landed (vmcnt(15): only G(s + 2), Q(s + 2) may fly)
//                 + barrier B (every wave's reads of G(s), the last in row 9, done)
//   rows 10, 11 : pieces 0, 1 of G(s + 3) into G(s)'s slot; A[0], A[1] of s + 1 read
// so every copy has >= 1.3 stages of lead and the CU's copy path sees ~1 KiB per SIMD per 8 MFMAs
// instead of bursts.
struct EngineW {
  static constexpr int NW = 4, NT = 256;
  static constexpr int TGW = 384;                    // gallery rows per tile
  static constexpr int HPB = 12288;                  // a 128-row half panel of one stage
  static constexpr int GSLOT = 3 * HPB, QSLOT = PANEL;
  static constexpr int NGS = 3, NQS = 2;
  static constexpr int QBASE = NGS * GSLOT;          // the query ring after the gallery ring
  static constexpr int LDS_BYTES = NGS * GSLOT + NQS * QSLOT;   // 159,744
  static constexpr int NA = 12, NB = 8, RING = 3;
  static constexpr int NAA = 8;                      // row blocks whose accumulators live in AGPRs (8 x 8 x 4 = 256)
  static constexpr int GPW = 9, QPW = 6;             // copy pieces per wave and stage
  static_assert(NA % RING == 0, "the ring index must repeat across stages");

  // gallery tile gt: rows [384 gt, 384 gt + 384) = half panels 3 gt .. 3 gt + 2 of the 256-row panels,
  // which lie in panels p0 = 3 gt / 2 and p0 + 1.  gsrc[j]: the byte offset (stage 0) in the gallery
  // descriptor of the wave's gallery piece j.
  struct Feed {
    __amdgpu_buffer_rsrc_t rg, rq;
    __amdgpu_buffer_rsrc_t rg2, rq2;   // the second-slice tiles (NSEG = 3, the two-slice tier f6x2)
    uint32_t gsrc[GPW];
    const uint32_t* bs;                // column-block scales, one dword per stage (null: unit)
  };

  template <int W, int NSEG = 1>
  // gnst: stages per panel of the gallery tiles when they differ from the queries' (the prefix tier's
  // compact gallery tiles, round 6; < 0: nst)
  static __device__ __forceinline__ void feed_init(Feed& f, const char* G, int64_t N, const char* Q, int64_t qp,
                                                   int64_t nst, int64_t gt, const char* G2 = nullptr,
                                                   const char* Q2 = nullptr, const uint32_t* bs = nullptr,
                                                   int64_t gnst = -1) {
    f.bs = bs;
    const int64_t h0 = 3 * gt, p0 = h0 >> 1;
    const int64_t qb = nst * (int64_t)PANEL;                 // bytes per 256-row query panel
    const int64_t pb = (gnst < 0 ? nst : gnst) * (int64_t)PANEL;   // ... gallery panel
    const int64_t rem = panels(N) * pb - p0 * pb;
    const int64_t rec = rem < 2 * pb ? rem : 2 * pb;         // reads past the gallery return zeros
    f.rg = __builtin_amdgcn_make_buffer_rsrc((void*)(G + p0 * pb), 0, (int)rec, 0x00020000);
    f.rq = __builtin_amdgcn_make_buffer_rsrc((void*)(Q + qp * qb), 0, (int)qb, 0x00020000);
    if constexpr (NSEG == 3) {
      f.rg2 = __builtin_amdgcn_make_buffer_rsrc((void*)(G2 + p0 * pb), 0, (int)rec, 0x00020000);
      f.rq2 = __builtin_amdgcn_make_buffer_rsrc((void*)(Q2 + qp * qb), 0, (int)qb, 0x00020000);
    }
#pragma unroll
    for (int j = 0; j < GPW; ++j) {
      const int g = W * GPW + j, k = g / 12, q = (g % 12) / 3, part = g % 3;
      const int64_t h = h0 + k;
      const uint32_t rel = (uint32_t)(((h >> 1) - p0) * pb), hh = (uint32_t)(h & 1);
      f.gsrc[j] = rel + q * 6144 + (part < 2 ? hh * 2048 + part * 1024 : 4096 + hh * 1024);
    }
  }
  // piece J of wave W's share of stage ks (kso = ks * PANEL) of the gallery tile (9 of its 36) / query
  // panel (6 of 24) into the slot at LDS byte offset so
  // (rg / rq: the descriptor of the stage's segment, f.rg / f.rq or f.rg2 / f.rq2)
  template <int W, int J>
  static __device__ __forceinline__ void gcopy(const __amdgpu_buffer_rsrc_t rg, const Feed& f, uint32_t so,
                                               uint32_t kso) {
    constexpr int g = W * GPW + J, k = g / 12, q = (g % 12) / 3, part = g % 3;
    constexpr uint32_t cd = k * HPB + q * 3072 + (part < 2 ? part * 1024 : 2048);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (OFR_LDS void*)(uintptr_t)(so + cd), 16, (threadIdx.x & 63) * 16,
                                             f.gsrc[J] + kso, 0, 0);
  }
  template <int W, int J>
  static __device__ __forceinline__ void qcopy(const __amdgpu_buffer_rsrc_t rq, uint32_t so, uint32_t kso) {
    constexpr uint32_t o = (W * QPW + J) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rq, (OFR_LDS void*)(uintptr_t)(so + o), 16, (threadIdx.x & 63) * 16,
                                             o + kso, 0, 0);
  }

  // Fragment reads from per-lane base addresses of a slot plus compile-time offsets (one VALU add per
  // base and stage; the reads carry the rest in their offset field).  Part1 slots (the p1_slot swizzle)
  // of a 16-row block m are 16 m + l ^ 16 (q & 1) = 16 (m +- (q & 1)) + l: one base for even, one for
  // odd m.  Volatile: two part1 reads must not fuse into a ds_read2_b64 (its halves belong to different
  // fragments and would cost moves).
  struct Bases {
    uint32_t p0, p1e, p1o;
  };
  static __device__ __forceinline__ Bases abase(uint32_t slot) {   // gallery slot (half-panel images)
    const uint32_t lane = threadIdx.x & 63, q = lane >> 4, l = lane & 15, qo = (q & 1) << 4;
    return Bases{slot + q * 3072 + l * 16, slot + q * 3072 + 2048 + (l + qo) * 8, slot + q * 3072 + 2048 + (l - qo) * 8};
  }
  static __device__ __forceinline__ Bases bbase(uint32_t slot) {   // query slot (panel image)
    const uint32_t lane = threadIdx.x & 63, q = lane >> 4, l = lane & 15, qo = (q & 1) << 4;
    return Bases{slot + q * 6144 + l * 16, slot + q * 6144 + 4096 + (l + qo) * 8, slot + q * 6144 + 4096 + (l - qo) * 8};
  }
  static __device__ __forceinline__ i32x6 frag_at(uint32_t a0, uint32_t a1) {
    const i32x4 p0 = *reinterpret_cast<volatile const OFR_LDS i32x4*>((uintptr_t)a0);
    const i32x2 p1 = *reinterpret_cast<volatile const OFR_LDS i32x2*>((uintptr_t)a1);
    i32x6 f;
    f[0] = p0[0]; f[1] = p0[1]; f[2] = p0[2]; f[3] = p0[3]; f[4] = p1[0]; f[5] = p1[1];
    return f;
  }
  template <int R0>   // gallery rows R0 .. R0 + 15 of the tile (R0 a multiple of 16)
  static __device__ __forceinline__ i32x6 fragA(const Bases& b) {
    constexpr int k = R0 / 128, rl = R0 % 128;
    return frag_at(b.p0 + k * HPB + rl * 16, ((rl >> 4) & 1 ? b.p1o : b.p1e) + k * HPB + rl * 8);
  }
  template <int R0>   // query rows R0 .. R0 + 15 of the panel
  static __device__ __forceinline__ i32x6 fragB(const Bases& b) {
    return frag_at(b.p0 + R0 * 16, ((R0 >> 4) & 1 ? b.p1o : b.p1e) + R0 * 8);
  }

  // The accumulators are pinned by inline asm: 384 registers per lane exceed either register file,
  // and the compiler gives every MFMA of a function the same form (all AGPR or all VGPR), shuffling
  // the rest through v_accvgpr moves.  Row blocks i < NAA accumulate in AGPRs, the others in VGPRs.
  // Hazards: an accumulator is re-read (as srcC) 96 MFMAs after it was written; the epilogue reads
  // them after wait_drain().
  template <bool AG>
  static __device__ __forceinline__ void mfma(const i32x6& a, const i32x6& b, f32x4& c, int sc) {
    if constexpr (AG)
      asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:2 blgp:2"
                   : "+a"(c) : "v"(a), "v"(b), "v"(sc));
    else
      asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0] cbsz:2 blgp:2"
                   : "+v"(c) : "v"(a), "v"(b), "v"(sc));
  }
  template <bool AG>   // separate gallery (A) and query (B) block scales (NSEG = 3)
  static __device__ __forceinline__ void mfma2(const i32x6& a, const i32x6& b, f32x4& c, int sa, int sb) {
    if constexpr (AG)
      asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0] cbsz:2 blgp:2"
                   : "+a"(c) : "v"(a), "v"(b), "v"(sa), "v"(sb));
    else
      asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0] cbsz:2 blgp:2"
                   : "+v"(c) : "v"(a), "v"(b), "v"(sa), "v"(sb));
  }
  static __device__ __forceinline__ void wait_drain() {   // the last MFMAs' results readable
    asm volatile("s_nop 7\n s_nop 7\n s_nop 7\n s_nop 7" ::: "memory");
  }

  // NSEG: segments of nst stages (seg_src): 1 = the fp6 tier; 3 = the two-slice tier f6x2, whose
  // stages of segment 1 / 2 read the query / gallery second slices (f.rq2 / f.rg2) with block scale
  // 2^-4 on that operand (block_scales).  nst: the stages run per segment -- the panels' stage count
  // (feed_init's), or with NSEG = 1 a prefix of it (the prefix tier)
  template <int W, int NSEG = 1>
  static __device__ __forceinline__ void mainloop(const Feed& f, int nst, f32x4 (&acc)[NA][NB]) {
    constexpr int WR = W >> 1, WC = W & 1;
    // block scales of the current stage (sa: gallery operand, sb: query; NSEG = 1 uses sa for both)
    const uint32_t lsh = 8u * ((threadIdx.x & 63) >> 4);   // the lane's 32-feature block of a stage
    int sa, sb;
    {
      const uint32_t raw0 = sload_bscale(f.bs, seg_stage<NSEG>(0, nst));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      block_scales<NSEG>(lane_byte(raw0, lsh), 0, nst, sa, sb);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int c = 0; c < NB; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int last = NSEG * nst - 1;
    // byte offset of stage s (clamped to the last) inside its segment's tiles, and the segment's descriptors
    auto kso = [&](int s) {
      const int c = s < last ? s : last;
      if constexpr (NSEG == 1) return (uint32_t)c * (uint32_t)PANEL;
      else return (uint32_t)(c - (c >= 2 * nst ? 2 : (c >= nst ? 1 : 0)) * nst) * (uint32_t)PANEL;
    };
    auto rgs = [&](int s) {
      if constexpr (NSEG == 1) return f.rg;
      else return (s < last ? s : last) >= 2 * nst ? f.rg2 : f.rg;
    };
    auto rqs = [&](int s) {
      if constexpr (NSEG == 1) return f.rq;
      else {
        const int c = s < last ? s : last;
        return c >= nst && c < 2 * nst ? f.rq2 : f.rq;
      }
    };
    auto gall = [&](uint32_t so, int st) {
      const __amdgpu_buffer_rsrc_t r = rgs(st);
      const uint32_t ko = kso(st);
      gcopy<W, 0>(r, f, so, ko); gcopy<W, 1>(r, f, so, ko); gcopy<W, 2>(r, f, so, ko);
      gcopy<W, 3>(r, f, so, ko); gcopy<W, 4>(r, f, so, ko); gcopy<W, 5>(r, f, so, ko);
      gcopy<W, 6>(r, f, so, ko); gcopy<W, 7>(r, f, so, ko); gcopy<W, 8>(r, f, so, ko);
    };
    auto qall = [&](uint32_t so, int st) {
      const __amdgpu_buffer_rsrc_t r = rqs(st);
      const uint32_t ko = kso(st);
      qcopy<W, 0>(r, so, ko); qcopy<W, 1>(r, so, ko); qcopy<W, 2>(r, so, ko);
      qcopy<W, 3>(r, so, ko); qcopy<W, 4>(r, so, ko); qcopy<W, 5>(r, so, ko);
    };
    // ring slots (LDS byte offsets) of stages s, s + 1, s + 2 (gallery) and s, s + 1 (query)
    uint32_t g0 = 0, g1 = GSLOT, g2 = 2 * GSLOT, q0 = QBASE, q1 = QBASE + QSLOT;
    // prologue: G(0), Q(0), G(1), Q(1) and pieces 0, 1 of G(2)
    gall(g0, 0); qall(q0, 0); gall(g1, 1); qall(q1, 1);
    gcopy<W, 0>(rgs(2), f, g2, kso(2));
    gcopy<W, 1>(rgs(2), f, g2, kso(2));
    wait_vm<GPW + QPW + 2>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    i32x6 a[RING], b[NB];
    {
      const Bases ab = abase(g0), bb = bbase(q0);
      a[0] = fragA<WR * 192 + 0>(ab);
      a[1] = fragA<WR * 192 + 16>(ab);
      b[0] = fragB<WC * 128 + 0>(bb); b[1] = fragB<WC * 128 + 16>(bb); b[2] = fragB<WC * 128 + 32>(bb);
      b[3] = fragB<WC * 128 + 48>(bb); b[4] = fragB<WC * 128 + 64>(bb); b[5] = fragB<WC * 128 + 80>(bb);
      b[6] = fragB<WC * 128 + 96>(bb); b[7] = fragB<WC * 128 + 112>(bb);
    }
    for (int s = 0; s <= last; ++s) {
      const Bases ac = abase(g0), an = abase(g1), bn = bbase(q1);
      const uint32_t k2 = kso(s + 2), k3 = kso(s + 3);
      const __amdgpu_buffer_rsrc_t rg2s = rgs(s + 2), rq2s = rqs(s + 2), rg3s = rgs(s + 3);
      // the next stage's block scales: a scalar load in row 2 (behind barrier A), turned into the
      // lanes' operands right behind barrier B, whose lgkmcnt(0) the wait for it joins (no fresh
      // fragment read is in flight there); taken over at the end of the stage
      uint32_t raw = 0;
      int na = 0, nb = 0;
      auto row = [&](auto ii) {
        constexpr int i = decltype(ii)::value;
        constexpr bool AG = i < NAA;
        auto mm = [&](const i32x6& x, const i32x6& y, f32x4& c) {
          if constexpr (NSEG == 1) mfma<AG>(x, y, c, sa);
          else mfma2<AG>(x, y, c, sa, sb);
        };
        if constexpr (i == 2) raw = sload_bscale(f.bs, seg_stage<NSEG>(s < last ? s + 1 : last, nst));
        if constexpr (i == 1) {              // barrier A: Q(s) consumed by every wave
          // Q(s)'s reads (row 11 of s - 1) are older than row 0's gallery read, the only one allowed in flight
          asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (i == 10) {             // barrier B: G(s+1), Q(s+1) landed; G(s) consumed
          wait_vm<GPW + QPW>();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          block_scales<NSEG>(lane_byte(raw, lsh), s < last ? s + 1 : last, nst, na, nb);
          __builtin_amdgcn_sched_barrier(0);
        }
        // G(s+2) into G(s-1)'s slot (= g2's ring position), Q(s+2) into Q(s)'s (q0) -- rows 0-6, each copy
        // issued right behind an MFMA so that its issue overlaps the MFMA's execution -- G(s+3) into G(s)'s (g0)
        if constexpr (i == 10) gcopy<W, 0>(rg3s, f, g0, k3);   // piece 1: in the middle of rows 10 / 11
        if constexpr (i == NA - 1) {
          // rows 10 and 11 run together (below, i == 10)
        } else if constexpr (i == NA - 2) {
          // Rows 10 and 11 column by column, each query fragment refilled for s + 1 after its last use:
          // b[c] then has 15 - c MFMAs before its first use in row 0 of s + 1 (row-major: 7).  Gallery
          // ring: s + 1's A[0] into A[9]'s slot now, its A[1] into A[10]'s after the last pair.
          static_assert(NA % RING == 0 && (NA - 2) % RING == 1, "ring slots of rows 10 / 11");
          a[0] = fragA<WR * 192 + 0>(an);
          mm(a[1], b[0], acc[10][0]); mm(a[2], b[0], acc[11][0]); b[0] = fragB<WC * 128 + 0>(bn);
          mm(a[1], b[1], acc[10][1]); mm(a[2], b[1], acc[11][1]); b[1] = fragB<WC * 128 + 16>(bn);
          mm(a[1], b[2], acc[10][2]); mm(a[2], b[2], acc[11][2]); b[2] = fragB<WC * 128 + 32>(bn);
          mm(a[1], b[3], acc[10][3]); mm(a[2], b[3], acc[11][3]); b[3] = fragB<WC * 128 + 48>(bn);
          gcopy<W, 1>(rg3s, f, g0, k3);
          mm(a[1], b[4], acc[10][4]); mm(a[2], b[4], acc[11][4]); b[4] = fragB<WC * 128 + 64>(bn);
          mm(a[1], b[5], acc[10][5]); mm(a[2], b[5], acc[11][5]); b[5] = fragB<WC * 128 + 80>(bn);
          mm(a[1], b[6], acc[10][6]); mm(a[2], b[6], acc[11][6]); b[6] = fragB<WC * 128 + 96>(bn);
          mm(a[1], b[7], acc[10][7]); mm(a[2], b[7], acc[11][7]); b[7] = fragB<WC * 128 + 112>(bn);
          a[1] = fragA<WR * 192 + 16>(an);
        } else {
          mm(a[i % RING], b[0], acc[i][0]);
          a[(i + 2) % RING] = fragA<WR * 192 + (i + 2 < NA ? i + 2 : 0) * 16>(ac);
          if constexpr (i <= 6) gcopy<W, (i <= 6 ? i + 2 : 0)>(rg2s, f, g2, k2);
#pragma unroll
          for (int c = 1; c < 5; ++c) mm(a[i % RING], b[c], acc[i][c]);
          // Q(s+2) in rows 4-9, four MFMAs behind the row's G(s+2) piece
          if constexpr (i >= 4 && i <= 9) qcopy<W, (i >= 4 && i <= 9 ? i - 4 : 0)>(rq2s, q0, k2);
#pragma unroll
          for (int c = 5; c < NB; ++c) mm(a[i % RING], b[c], acc[i][c]);
        }
        __builtin_amdgcn_sched_barrier(0);
      };
      row(std::integral_constant<int, 0>{});
      row(std::integral_constant<int, 1>{});
      row(std::integral_constant<int, 2>{});
      row(std::integral_constant<int, 3>{});
      row(std::integral_constant<int, 4>{});
      row(std::integral_constant<int, 5>{});
      row(std::integral_constant<int, 6>{});
      row(std::integral_constant<int, 7>{});
      row(std::integral_constant<int, 8>{});
      row(std::integral_constant<int, 9>{});
      row(std::integral_constant<int, 10>{});
      row(std::integral_constant<int, 11>{});
      const uint32_t gt_ = g0;   // rotate: s+1 -> current, s+2 -> next, s (now re-filled with s+3) -> s+2's
      g0 = g1; g1 = g2; g2 = gt_;
      const uint32_t qt_ = q0;
      q0 = q1; q1 = qt_;
      sa = na;
      sb = nb;
      if (s == last) wait_drain();
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_vm<0>();
    barrier();
  }
};

}  // namespace f6t
}  // namespace ofr
