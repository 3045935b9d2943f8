// Wide int8 MFMA tile engine of the exact projection (ofr_qproj.hip, round 3): the fp6 sieve's
// one-wave-per-SIMD design (f6t::EngineW, ofr_f6_tile.h) on v_mfma_i32_16x16x64_i8.
//
// C[a][b] = sum_k A[a][k] * B[b][k]: A = the W slices (int8 rows, [arows][lda]), B = the images
// (uint8 rows [B][ldb], turned into x - 128 by an XOR with 0x80 after the LDS read).  Tile = 384 A
// rows x 256 B rows; 4 waves, wave w owns ALL 384 A rows against B rows 64 w .. 64 w + 63, so the four
// slices of every feature (rows jb*128 + s*32 + j%32 of the projection layout) meet in one wave's
// accumulators: 24 x 4 blocks of 16 x 16 = 96 accumulators of 4 = 384 registers, pinned by inline-asm
// MFMAs (row blocks 0-15 in the 256 AGPRs, 16-23 in VGPRs; the compiler would give every MFMA the
// same register form and shuffle the surplus).  k stage = 64 bytes per row.
//
// LDS: an A ring of 3 slots (384 rows x 64 B = 24 KiB) and a B ring of 2 slots (256 x 64 B = 16 KiB),
// 104 KiB.  A row's 64 bytes are 4 chunks of 16 B stored at chunk ^ f(row), f(row) = 2 ((row >> 2) & 1):
// the fragment reads (lane l: row l % 16 of a 16-row block, chunk l / 16) are then bank-conflict free in
// every ds_read_b128 lane group.  A copy piece (buffer_load_dwordx4 ... lds, 1 KiB) is 16 rows x 64 B:
// lane l writes LDS l * 16 = row l / 4, position l % 4, so it loads chunk (l % 4) ^ f(l / 4) of its row
// (the swizzle lives in the per-lane source offset, a constant: f depends on bit 4 of l only).
// Per stage s, 24 rows of 4 MFMAs (the A fragments through a ring of 3 read two rows ahead, the 4 B
// fragments held and refilled for s + 1 after their last use in rows 22 / 23, run column by column):
//   row 0       : the B fragments XORed to x - 128 just before their first MFMA
//   row 2 start : barrier A (every wave's reads of B(s), issued in rows 22-23 of s - 1, done)
//   rows 0,4,8,12: pieces 2-5 of A(s + 2) into A(s - 1)'s slot;  rows 2,6,10,14: pieces of B(s + 2)
//   row 22 start: own copies of A(s + 1), B(s + 1) landed (vmcnt(10)) + barrier B (A(s) consumed)
//   rows 22, 23 : pieces 0, 1 of A(s + 3) into A(s)'s slot; A[0], A[1], B of s + 1 read
#pragma once
#include "ofr_common.h"

// OFR_PROJ_PROBE (probe builds only, tools/build_proj_probes.sh; results WRONG, timing only): bit 1 no barriers
// in the main loop, bit 2 no stage copies in the main loop, bit 4 no fragment reads in the main loop
#ifndef OFR_PROJ_PROBE
#define OFR_PROJ_PROBE 0
#endif
namespace ofr {
namespace i8w {

typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int TA = 384, TB = 256;          // A rows x B rows per tile
constexpr int BK = 64;                     // bytes (k) per stage
constexpr int NW = 4, NT = 256;
constexpr int ASLOT = TA * BK, BSLOT = TB * BK;   // 24 KiB, 16 KiB
constexpr int NAS = 3, NBS = 2;
constexpr int BBASE = NAS * ASLOT;
constexpr int LDS_BYTES = NAS * ASLOT + NBS * BSLOT;   // 106,496
constexpr int NA = 24, NB = 4, RING = 3;
constexpr int NAA = 16;                    // row blocks accumulating in AGPRs (16 x 4 x 4 = 256)
constexpr int APW = ASLOT / 1024 / NW;     // 6 A pieces per wave and stage
constexpr int BPW = BSLOT / 1024 / NW;     // 4 B pieces per wave and stage
static_assert(NA % RING == 0 && (NA - 2) % RING == 1, "ring slots of rows 22 / 23");

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct Feed {
  __amdgpu_buffer_rsrc_t ra, rb;
  uint32_t lda, ldb;
};
// A rows [a0, a0 + 384) of [arows][lda], B rows [b0, b0 + 256) of [brows][ldb]; reads past either
// panel's rows return zeros (the A rows past arows are zero slices, the B rows past the batch are not
// stored).  Offsets are 32-bit: 384 lda and 256 ldb must stay below 2^31 (the caller checks).
__device__ __forceinline__ void feed_init(Feed& f, const int8_t* A, int64_t lda, int64_t arows, int64_t a0,
                                          const uint8_t* Bm, int64_t ldb, int64_t brows, int64_t b0) {
  const int64_t ra = arows - a0 < TA ? arows - a0 : TA, rb = brows - b0 < TB ? brows - b0 : TB;
  f.ra = __builtin_amdgcn_make_buffer_rsrc((void*)(A + a0 * lda), 0, (int)(ra * lda), 0x00020000);
  f.rb = __builtin_amdgcn_make_buffer_rsrc((void*)(Bm + b0 * ldb), 0, (int)(rb * ldb), 0x00020000);
  f.lda = (uint32_t)lda;
  f.ldb = (uint32_t)ldb;
}
// REG staging (round 6, OFR_PROJ_STAGE=reg): a piece is loaded into four VGPRs by buffer_load_dwordx4 and
// stored by ds_write_b128 to the same LDS position the DMA would write (lane l: piece byte l * 16), the
// image pieces XORed to x - 128 on the way.  An LDS-DMA piece holds the wave's issue for ~60 cycles among
// MFMAs (MI355X_MICROARCH.md, latency table); the load + store pair costs a fraction of that, and the
// 40 VGPRs it needs are free at one wave per SIMD.
template <int W, int J>
__device__ __forceinline__ i32x4 aload(const Feed& f, uint32_t vo, uint32_t ko) {
  constexpr int p = W * APW + J;
  return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(f.ra, (int)vo, (int)((uint32_t)(16 * p) * f.lda + ko), 0));
}
template <int W, int J>
__device__ __forceinline__ i32x4 bload(const Feed& f, uint32_t vo, uint32_t ko) {
  constexpr int p = W * BPW + J;
  i32x4 v = __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(f.rb, (int)vo, (int)((uint32_t)(16 * p) * f.ldb + ko), 0));
  return v;
}
__device__ __forceinline__ i32x4 x80(i32x4 v) {
  v[0] ^= 0x80808080; v[1] ^= 0x80808080; v[2] ^= 0x80808080; v[3] ^= 0x80808080;
  return v;
}
// store piece P (global piece index) of a slot at LDS offset so
template <int P>
__device__ __forceinline__ void pstore(uint32_t so, const i32x4& v) {
  *reinterpret_cast<volatile OFR_LDS i32x4*>((uintptr_t)(so + P * 1024 + (threadIdx.x & 63) * 16)) = v;
}

// per-lane source offset of a piece (row l / 4 of the piece, swizzled chunk), times the row stride
__device__ __forceinline__ uint32_t lane_src(uint32_t ld) {
  const uint32_t l = threadIdx.x & 63, c = (l & 3) ^ (((l >> 4) & 1) << 1);
  return (l >> 2) * ld + c * 16;
}
// piece J of wave W's share of stage k (byte offset ko = 64 k) into the slot at LDS offset so
template <int W, int J>
__device__ __forceinline__ void acopy(const Feed& f, uint32_t vo, uint32_t so, uint32_t ko) {
  constexpr int p = W * APW + J;   // rows 16 p .. 16 p + 15
  __builtin_amdgcn_raw_ptr_buffer_load_lds(f.ra, (OFR_LDS void*)(uintptr_t)(so + p * 1024), 16, vo,
                                           (uint32_t)(16 * p) * f.lda + ko, 0, 0);
}
template <int W, int J>
__device__ __forceinline__ void bcopy(const Feed& f, uint32_t vo, uint32_t so, uint32_t ko) {
  constexpr int p = W * BPW + J;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(f.rb, (OFR_LDS void*)(uintptr_t)(so + p * 1024), 16, vo,
                                           (uint32_t)(16 * p) * f.ldb + ko, 0, 0);
}

// fragment of the 16-row block at row R0 of a slot: lane l reads row R0 + l % 16, chunk l / 16 (its
// stored position chunk ^ f(row); f depends on bit 2 of the row, i.e. bit 2 of l)
__device__ __forceinline__ uint32_t frag_base(uint32_t slot) {
  const uint32_t l = threadIdx.x & 63, r = l & 15, c = (l >> 4) ^ (((r >> 2) & 1) << 1);
  return slot + r * BK + c * 16;
}
template <int R0>
__device__ __forceinline__ i32x4 frag(uint32_t base) {
  return *reinterpret_cast<volatile const OFR_LDS i32x4*>((uintptr_t)(base + R0 * BK));
}
// uint8 x -> int8 x - 128, then wait states before an MFMA reads the result: the hazard recognizer
// does not see the inline-asm MFMAs, and without them the next MFMA read the bytes before the XOR
// (round 3: slice 0 of every other feature group wrong)
__device__ __forceinline__ i32x4 xor80(i32x4 v) {
  v[0] ^= 0x80808080; v[1] ^= 0x80808080; v[2] ^= 0x80808080; v[3] ^= 0x80808080;
  asm volatile("s_nop 4" : "+v"(v));
  return v;
}

template <bool AG>
__device__ __forceinline__ void mfma(const i32x4& a, const i32x4& b, i32x4& c) {
  if constexpr (AG)
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_i32_16x16x64_i8 %0, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b));
}

// nk stages (nk >= 1; copies past the last stage re-copy it into free slots, never read).
// acc[i][c]: A rows 16 i .. 16 i + 15 of the tile x B rows 64 W + 16 c .. + 15; C/D of lane l, reg r:
// A row 16 i + 4 (l / 16) + r, B row 64 W + 16 c + l % 16.
// REG (register staging): the same slots and barriers; per stage s the pieces of A(s + 2) 2-5 and B(s + 2),
// loaded at rows 22-23 of stage s - 1, are stored at rows REG_W0 + REG_WS j (A(s - 1)'s slot is free since
// barrier B of s - 1, B(s)'s since barrier A); A(s + 3) pieces 0, 1, loaded at row 6, are stored after
// barrier B (A(s) consumed).  The B slots hold x - 128 already.
#ifndef OFR_PROJ_REG_W0
#define OFR_PROJ_REG_W0 12
#endif
#ifndef OFR_PROJ_REG_WS
#define OFR_PROJ_REG_WS 1
#endif
constexpr int REG_W0 = OFR_PROJ_REG_W0, REG_WS = OFR_PROJ_REG_WS;   // REG: the row of the first store, rows between
static_assert(REG_W0 >= 3 && REG_W0 + 7 * REG_WS <= NA - 3, "REG stores between barrier A and barrier B");
template <int W, bool REG = false>
__device__ __forceinline__ void mainloop(const Feed& f, int nk, i32x4 (&acc)[NA][NB]) {
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int c = 0; c < NB; ++c) acc[i][c] = i32x4{0, 0, 0, 0};
  const int last = nk - 1;
  auto kso = [&](int s) { return (uint32_t)(s < last ? s : last) * (uint32_t)BK; };
  const uint32_t va = lane_src(f.lda), vb = lane_src(f.ldb);
  uint32_t g0 = 0, g1 = ASLOT, g2 = 2 * ASLOT, q0 = BBASE, q1 = BBASE + BSLOT;
  auto aall = [&](uint32_t so, uint32_t ko) {
    acopy<W, 0>(f, va, so, ko); acopy<W, 1>(f, va, so, ko); acopy<W, 2>(f, va, so, ko);
    acopy<W, 3>(f, va, so, ko); acopy<W, 4>(f, va, so, ko); acopy<W, 5>(f, va, so, ko);
  };
  auto ball = [&](uint32_t so, uint32_t ko) {
    bcopy<W, 0>(f, vb, so, ko); bcopy<W, 1>(f, vb, so, ko); bcopy<W, 2>(f, vb, so, ko); bcopy<W, 3>(f, vb, so, ko);
  };
  // REG staging registers: A(s + 2) pieces 2-5, B(s + 2) pieces 0-3; A(s + 3) pieces 0, 1
  i32x4 sa[4], sb[4], s01[2];
  auto areg = [&](uint32_t ko) {
    sa[0] = aload<W, 2>(f, va, ko); sa[1] = aload<W, 3>(f, va, ko);
    sa[2] = aload<W, 4>(f, va, ko); sa[3] = aload<W, 5>(f, va, ko);
  };
  auto breg = [&](uint32_t ko) {
    sb[0] = bload<W, 0>(f, vb, ko); sb[1] = bload<W, 1>(f, vb, ko);
    sb[2] = bload<W, 2>(f, vb, ko); sb[3] = bload<W, 3>(f, vb, ko);
  };
  auto a01reg = [&](uint32_t ko) { s01[0] = aload<W, 0>(f, va, ko); s01[1] = aload<W, 1>(f, va, ko); };
  auto a01st = [&](uint32_t so) { pstore<W * APW + 0>(so, s01[0]); pstore<W * APW + 1>(so, s01[1]); };
  auto allst = [&](uint32_t sA, uint32_t sB) {
    pstore<W * APW + 2>(sA, sa[0]); pstore<W * APW + 3>(sA, sa[1]);
    pstore<W * APW + 4>(sA, sa[2]); pstore<W * APW + 5>(sA, sa[3]);
    pstore<W * BPW + 0>(sB, x80(sb[0])); pstore<W * BPW + 1>(sB, x80(sb[1]));
    pstore<W * BPW + 2>(sB, x80(sb[2])); pstore<W * BPW + 3>(sB, x80(sb[3]));
  };
  if constexpr (REG) {
    // prologue: A(0), B(0), A(1), B(1), pieces 0, 1 of A(2) stored; A(2) 2-5 and B(2) held for stage 0
    for (int t = 0; t < 2; ++t) {
      const uint32_t sA = t ? g1 : g0, sB = t ? q1 : q0;
      a01reg(kso(t)); areg(kso(t)); breg(kso(t));
      a01st(sA); allst(sA, sB);
    }
    a01reg(kso(2));
    a01st(g2);
    areg(kso(2)); breg(kso(2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  } else {
    // prologue: A(0), B(0), A(1), B(1), pieces 0, 1 of A(2)
    aall(g0, kso(0)); ball(q0, kso(0)); aall(g1, kso(1)); ball(q1, kso(1));
    acopy<W, 0>(f, va, g2, kso(2));
    acopy<W, 1>(f, va, g2, kso(2));
    wait_vm<APW + BPW + 2>();
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  i32x4 a[RING], b[NB];
  {
    const uint32_t ab = frag_base(g0), bb = frag_base(q0);
    a[0] = frag<0>(ab);
    a[1] = frag<16>(ab);
    b[0] = frag<W * 64 + 0>(bb); b[1] = frag<W * 64 + 16>(bb);
    b[2] = frag<W * 64 + 32>(bb); b[3] = frag<W * 64 + 48>(bb);
  }
  for (int s = 0; s <= last; ++s) {
    const uint32_t ac = frag_base(g0), an = frag_base(g1), bn = frag_base(q1);
    const uint32_t k2 = kso(s + 2), k3 = kso(s + 3);
    auto row = [&](auto ii) {
      constexpr int i = decltype(ii)::value;
      constexpr bool AG = i < NAA;
      constexpr bool BAR = !(OFR_PROJ_PROBE & 1), CPY = !(OFR_PROJ_PROBE & 2);
      if constexpr (i == 2) {   // barrier A: B(s) consumed (its reads, rows 22-23 of s - 1, are older than row 0's)
        asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
        if constexpr (BAR) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (i == NA - 2) {   // barrier B: A(s+1), B(s+1) landed; A(s) consumed
        if constexpr (!REG) wait_vm<APW + BPW>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if constexpr (BAR) __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (REG) {
        if constexpr (CPY && i >= REG_W0 && i < REG_W0 + 8 * REG_WS && (i - REG_W0) % REG_WS == 0) {
          constexpr int w = (i - REG_W0) / REG_WS;
          if constexpr (w < 4) {
            pstore<W * APW + 2 + (w < 4 ? w : 0)>(g2, sa[w < 4 ? w : 0]);
          } else {
            pstore<W * BPW + (w >= 4 ? w - 4 : 0)>(q0, x80(sb[w >= 4 ? w - 4 : 0]));
          }
        }
        if constexpr (CPY && i == 6) a01reg(k3);
      } else {
        if constexpr (CPY && i % 4 == 0 && i <= 12) acopy<W, (i % 4 == 0 && i <= 12 ? 2 + i / 4 : 0)>(f, va, g2, k2);
        if constexpr (CPY && i % 4 == 2 && i <= 14) bcopy<W, (i % 4 == 2 && i <= 14 ? i / 4 : 0)>(f, vb, q0, k2);
        if constexpr (CPY && i == NA - 2) acopy<W, 0>(f, va, g0, k3);
      }
      if constexpr (i == NA - 1) {
        // rows 22 and 23 run together (below)
      } else if constexpr (i == NA - 2) {
        if constexpr (REG && CPY) {
          a01st(g0);   // A(s + 3) pieces 0, 1 into A(s)'s slot
          areg(k3);    // A(s + 3) pieces 2-5 and B(s + 3), stored in stage s + 1
        }
        a[0] = frag<0>(an);   // s + 1's A[0] into A[21]'s slot
        mfma<false>(a[1], b[0], acc[22][0]); mfma<false>(a[2], b[0], acc[23][0]); b[0] = frag<W * 64 + 0>(bn);
        mfma<false>(a[1], b[1], acc[22][1]); mfma<false>(a[2], b[1], acc[23][1]); b[1] = frag<W * 64 + 16>(bn);
        if constexpr (CPY && !REG) acopy<W, 1>(f, va, g0, k3);
        if constexpr (CPY && REG) breg(k3);
        mfma<false>(a[1], b[2], acc[22][2]); mfma<false>(a[2], b[2], acc[23][2]); b[2] = frag<W * 64 + 32>(bn);
        mfma<false>(a[1], b[3], acc[22][3]); mfma<false>(a[2], b[3], acc[23][3]); b[3] = frag<W * 64 + 48>(bn);
        a[1] = frag<16>(an);  // s + 1's A[1] into A[22]'s slot
      } else {
        // the B fragments arrive as raw image bytes: x - 128 (XOR 0x80) just before their first use
        if constexpr (i == 0 && !REG) b[0] = xor80(b[0]);
        mfma<AG>(a[i % RING], b[0], acc[i][0]);
        a[(i + 2) % RING] = frag<(i + 2 < NA ? i + 2 : 0) * 16>(ac);
        if constexpr (i == 0 && !REG) b[1] = xor80(b[1]);
        mfma<AG>(a[i % RING], b[1], acc[i][1]);
        if constexpr (i == 0 && !REG) b[2] = xor80(b[2]);
        mfma<AG>(a[i % RING], b[2], acc[i][2]);
        if constexpr (i == 0 && !REG) b[3] = xor80(b[3]);
        mfma<AG>(a[i % RING], b[3], acc[i][3]);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    [&]<int... I>(std::integer_sequence<int, I...>) { (row(std::integral_constant<int, I>{}), ...); }
    (std::make_integer_sequence<int, NA>{});
    // The last stage drains the MFMA pipe before leaving the loop: hipcc pads nothing after an asm MFMA
    // and places its loop-exit copies of the accumulators (register moves, spills) right after the last
    // one -- 8-pass XDL result -> any reader needs 12 wait states.
    if (s == last) asm volatile("s_nop 7\n s_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const uint32_t gt_ = g0;   // rotate: s+1 -> current, s+2 -> next, s (re-filled with s+3) -> s+2's
    g0 = g1; g1 = g2; g2 = gt_;
    const uint32_t qt_ = q0;
    q0 = q1; q1 = qt_;
  }
  wait_vm<0>();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

}  // namespace i8w
}  // namespace ofr
