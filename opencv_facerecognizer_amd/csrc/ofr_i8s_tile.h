// Deep-staged int8 MFMA tile engine (gfx950) for the exact projection (ofr_qproj.hip).
//
// C[a][b] = sum_k A[a][k] * B[b][k] over int8 rows, v_mfma_i32_32x32x32_i8, int32 accumulators:
// 256 x 256 tile, 8 waves (2 per SIMD) of 128 x 64, the same fragment / accumulator map as
// ofr_i8_tile.h.  What differs is the feed.  ofr_i8_tile.h stages 128-feature steps (64 KiB) in two
// buffers, so a copy has one step of lead, and it copies with FLAT global_load_lds, which makes the
// compiler drain every LDS read before the first use of a fresh fragment.  At the projection's
// shape (W slices 40,192 x 10,112 streamed from HBM) the copies then stall the MFMAs (probe:
// 1.57 ms with copies, 1.29 ms without, 0.74 ms for the MFMAs alone).  Here:
//   * a stage is 64 features (32 KiB: 256 A rows + 256 B rows of 64 B), NST = 4 or 5 buffers, so a
//     stage's copy is issued NST - 2 stages before its first read;
//   * the copies are MUBUF buffer_load_dwordx4 ... lds, one buffer descriptor per operand panel
//     (rows past the panel's records read as zero: no clamping); the LDS image is 64-B rows whose
//     four 16-B chunks are XOR-swizzled by (row >> 2) & 3, applied to the per-lane source offset,
//     so that every ds_read_b128 lane group of a 32-row fragment hits 16 distinct bank quads;
//   * the stage hand-off sits in the middle of the stage: k-half 1's reads of stage kt run between
//     k-half 0's MFMAs, then the wait for stage kt+1 and one s_barrier, the copy of stage
//     kt + NST - 1 into the buffer stage kt - 1 vacated, and stage kt+1's k-half-0 reads between
//     k-half 1's MFMAs -- no barrier ever waits on a fresh LDS read.
#pragma once
#include "ofr_i8_tile.h"

namespace ofr {
namespace i8s {

using i8t::i32x16;
using i8t::i32x4;

constexpr int TA = 256, TB = 256;   // A rows x B rows per tile
constexpr int BK = 64;              // bytes (features) per stage and row
constexpr int NW = 8, NT = NW * 64;
constexpr int WQ = 4, QW = 64, CT = QW / 32;   // wave grid 2 (A) x 4 (B); 32-row B blocks per wave
constexpr int PANEL = TA * BK;      // 16 KiB
constexpr int STAGE = 2 * PANEL;    // A panel + B panel
constexpr int INS = STAGE / 1024;   // 1-KiB copy wave-instructions per stage (32)
constexpr int IPW = INS / NW;       // per wave (4): waves 0-3 copy the A panel, 4-7 the B panel
static_assert(IPW * NW == INS && (INS / 2) % IPW == 0, "a wave's copies stay in one panel");

template <int NST>
struct Lds {
  static constexpr int BYTES = NST * STAGE;   // 128 KiB (NST = 4) / 160 KiB (NST = 5)
};

__device__ __forceinline__ int off(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4); }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Stage kt of both panels into st.  ra / rb: buffer descriptors of the tile's A / B row panels
// (base = first row of the panel, num_records = its readable bytes); lda / ldb their row pitch.
// W4: the 32 pieces issued by waves 0-3 alone (8 each: 4 of A, 4 of B), waves 4-7 issue none.
template <bool W4 = false>
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t ra, int lda, __amdgpu_buffer_rsrc_t rb, int ldb, int kt,
                                    char* st) {
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  if constexpr (W4) {
    if (wave >= 4) return;
#pragma unroll
    for (int t = 0; t < 2 * IPW; ++t) {
      const bool a_side = t < IPW;
      const int ins = wave * IPW + (t % IPW);
      const int row = ins * 16 + (lane >> 2);
      const int chunk = (lane & 3) ^ ((row >> 2) & 3);
      const int voff = row * (a_side ? lda : ldb) + kt * BK + chunk * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_side ? ra : rb,
                                               (OFR_LDS void*)(st + (a_side ? 0 : PANEL) + ins * 1024), 16, voff, 0, 0, 0);
    }
    return;
  }
  const bool a_side = wave < NW / 2;   // uniform per wave
#pragma unroll
  for (int t = 0; t < IPW; ++t) {
    const int ins = (wave % (NW / 2)) * IPW + t;   // 1-KiB block of the panel: rows 16 ins .. 16 ins + 15
    const int row = ins * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const int ld = a_side ? lda : ldb;
    const int voff = row * ld + kt * BK + chunk * 16;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(a_side ? ra : rb, (OFR_LDS void*)(st + (a_side ? 0 : PANEL) + ins * 1024),
                                             16, voff, 0, 0, 0);
  }
}

// Main loop over nk stages.  XB: B holds uint8 (images), fragments become x - 128 by XOR 0x80.
// acc[i][j]: A block i (rows wr*128 + 32 i + C/D row map) x B block j (rows wc*64 + 32 j + lane&31).
template <int NST, bool XB, bool W4 = false>
__device__ __forceinline__ void mainloop(char* smem, __amdgpu_buffer_rsrc_t ra, int lda, __amdgpu_buffer_rsrc_t rb,
                                         int ldb, int nk, i32x16 (&acc)[4][CT]) {
  static_assert(NST == 4 || NST == 5, "stages");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / WQ, wc = wave % WQ, h = lane >> 5, r32 = lane & 31;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  // branch-free: a stage past the end re-loads the last stage into a buffer nobody reads any more
  const int last = nk - 1;
  auto issue = [&](int s) { dma<W4>(ra, lda, rb, ldb, s < last ? s : last, smem + (s % NST) * STAGE); };
  constexpr int PW = W4 ? 2 * IPW : IPW;   // pieces per issuing wave and stage
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) issue(s);

  i32x4 ga[2][4], qb[2][CT];
  auto frags = [&](const char* st, int ks) {   // ks = MFMA k-half (32 features) of the stage
    const int c = 2 * ks + h;
#pragma unroll
    for (int j = 0; j < CT; ++j) {
      qb[ks][j] = *reinterpret_cast<const i32x4*>(st + PANEL + off(wc * QW + j * 32 + r32, c));
      if constexpr (XB) qb[ks][j] ^= (int)0x80808080;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) ga[ks][i] = *reinterpret_cast<const i32x4*>(st + off(wr * 128 + i * 32 + r32, c));
  };
  auto mfmas = [&](int ks) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ga[ks][i], qb[ks][j], acc[i][j], 0, 0, 0);
  };
  // 6 reads over 8 MFMAs, one after each of the first six (the B fragments first); the B fragments'
  // XORs (x - 128) after the seventh MFMA, five MFMAs behind their reads: placed by the compiler,
  // each XOR would follow its read at once and wait out the LDS latency
  auto interleave = [&]() {
#pragma unroll
    for (int r = 0; r < 4 + CT; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if constexpr (XB) __builtin_amdgcn_sched_group_barrier(0x002, 4 * CT, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 4 * CT - (4 + CT) - 1, 0);
  };

  wait_vm<(NST - 2) * PW>();   // stage 0 landed (own copies); 1 .. NST-2 may be in flight
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  frags(smem, 0);
  for (int kt = 0; kt < nk; ++kt) {
    const char* st = smem + (kt % NST) * STAGE;
    frags(st, 1);
    mfmas(0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
    wait_vm<(NST - 3) * PW>();   // stage kt+1 landed; kt+2 .. kt+NST-2 may be in flight
    __builtin_amdgcn_s_barrier();   // ... for every wave; and every wave has consumed stage kt-1
    __builtin_amdgcn_sched_barrier(0);
    issue(kt + NST - 1);            // into stage kt-1's buffer
    frags(smem + ((kt + 1) % NST) * STAGE, 0);   // kt = last: unused reads of a stale buffer
    mfmas(1);
    if constexpr (!W4) __builtin_amdgcn_sched_group_barrier(0x020, IPW, 0);
    interleave();
    __builtin_amdgcn_sched_barrier(0);
  }
  wait_vm<0>();   // no copy may still target this workgroup's LDS when it retires
}

// Ping-pong main loop: the same tile, stages and copies, but the two waves of a SIMD never read
// fragments and issue MFMAs at the same time.  The wave groups g = wr (waves 0-3 and 4-7; the
// cyclic wave -> SIMD order puts one of each on every SIMD) run one s_barrier apart: per stage j a
// wave has a LOAD phase (its copies of stage j + NST - 2, the 12 fragment reads of stage j, the wait
// for its copies of stage j + 1, lgkmcnt(0) on its reads) and an MFMA phase (16 MFMAs at raised
// priority), each ending in an s_barrier.  Barrier H(n) is the n-th barrier every wave passes;
// group 0 ends LOAD(j) at H(2j+1) and MFMA(j) at H(2j+2), group 1 one barrier later, so while one
// wave of a SIMD issues its 16 MFMAs the other fetches the next stage's operands.
//   visibility: stage j+1's copies are waited for (own vmcnt) before LOAD(j)'s barrier, i.e. by
//     H(2j+2) for every wave; its first reader (group 0, LOAD(j+1)) starts after H(2j+2);
//   reuse: LOAD(j) copies into the buffer of stage j-2, whose last reads (group 1, LOAD(j-2),
//     drained by lgkmcnt(0) before its barrier H(2j-1)) precede the earliest copy (group 0 after
//     H(2j)).
template <int NST, bool XB>
__device__ __forceinline__ void mainloop_pp(char* smem, __amdgpu_buffer_rsrc_t ra, int lda, __amdgpu_buffer_rsrc_t rb,
                                            int ldb, int nk, i32x16 (&acc)[4][CT]) {
  static_assert(NST == 4 || NST == 5, "stages");
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / WQ, wc = wave % WQ, h = lane >> 5, r32 = lane & 31;
  const bool late = __builtin_amdgcn_readfirstlane(wr) != 0;   // group 1: one barrier behind
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  const int last = nk - 1;
  auto issue = [&](int s) { dma(ra, lda, rb, ldb, s < last ? s : last, smem + (s % NST) * STAGE); };
#pragma unroll
  for (int s = 0; s < NST - 2; ++s) issue(s);
  wait_vm<(NST - 3) * IPW>();   // own copies of stage 0 landed
  __builtin_amdgcn_s_barrier();   // H(0): stage 0 visible to every wave
  if (late) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  i32x4 ga[2][4], qb[2][CT];
  for (int kt = 0; kt < nk; ++kt) {
    // LOAD phase: the fragment reads first (their latency runs under the copies' issue)
    const char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 2 * ks + h;
#pragma unroll
      for (int j = 0; j < CT; ++j) qb[ks][j] = *reinterpret_cast<const i32x4*>(st + PANEL + off(wc * QW + j * 32 + r32, c));
#pragma unroll
      for (int i = 0; i < 4; ++i) ga[ks][i] = *reinterpret_cast<const i32x4*>(st + off(wr * 128 + i * 32 + r32, c));
    }
    issue(kt + NST - 2);
    wait_vm<(NST - 3) * IPW>();   // own copies of stage kt+1 landed (kt+2 .. kt+NST-2 may fly)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (XB) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < CT; ++j) qb[ks][j] ^= (int)0x80808080;
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    // MFMA phase
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < CT; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(ga[ks][i], qb[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (!late) __builtin_amdgcn_s_barrier();   // equal barrier counts for both groups
  wait_vm<0>();   // no copy may still target this workgroup's LDS when it retires
}

}  // namespace i8s
}  // namespace ofr
