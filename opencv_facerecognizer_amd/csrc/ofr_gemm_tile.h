// fp32-MFMA tile engine shared by the search (ofr_knn.hip) and projection
// (ofr_project.hip) kernels.
//
// One workgroup = 256 threads = 4 waves (one per SIMD) computes a 256x256
// tile of  C[a][b] = sum_k A[a][k] * B[b][k]  with v_mfma_f32_32x32x2_f32
// (exact f32 products, f32 accumulation).  A and B are both "rows with k
// contiguous" (gallery rows / W^T rows, query rows / image rows), so a tile
// is two [256][BK] LDS panels.  Waves are arranged 2x2; each owns a 128x128
// sub-tile = 4x4 MFMA blocks of 32x32 (256 accumulator registers).
//
// LDS image per operand and stage: [256 rows][32 fp32] = 128-B rows, 16-B
// chunks XOR-swizzled by ((row>>1)&7) so that the ds_read_b128 fragment
// reads (16 rows x same chunk per lane group) hit 16 distinct 4-bank slots.
// fp32 operands are staged by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8
// rows per wave-instruction) with the swizzle applied to the per-lane SOURCE
// address; uint8 operands are staged through registers (u8 -> f32 on the
// write).  Two stages: the next K-panel streams in while the current one
// feeds 256 MFMAs per wave (~16k cycles), one barrier per panel.
#pragma once
#include "ofr_common.h"

namespace ofr {
namespace tile {

constexpr int TM = 256;           // A rows per tile
constexpr int TN = 256;           // B rows per tile
constexpr int BK = 32;            // k per LDS panel
constexpr int NTHREADS = 256;
constexpr int PANEL_BYTES = 256 * BK * 4;          // 32 KiB per operand per stage
constexpr int STAGE_BYTES = 2 * PANEL_BYTES;       // A + B
constexpr int LDS_BYTES = 2 * STAGE_BYTES;         // 128 KiB

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * 128 + swz_chunk(row, chunk) * 16; }

// ---- fp32 operand by LDS-DMA ------------------------------------------------
struct LoaderF32 {
  const float* base;   // operand [rows][ld]
  int64_t ld;
  int64_t rows;        // valid rows; rows beyond are clamped (results masked later)
  int64_t r0;          // first row of this tile

  __device__ __forceinline__ void issue(char* lds_panel, int kt) const {
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int ins = wave * 8 + t;            // 32 wave-instructions x 8 rows
      const int row = ins * 8 + (lane >> 3);
      const int pchunk = lane & 7;
      const int chunk = pchunk ^ ((row >> 1) & 7);
      int64_t grow = r0 + row;
      grow = grow < rows ? grow : rows - 1;
      const float* src = base + grow * ld + (int64_t)kt * BK + chunk * 4;
      __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)src,
                                       (OFR_LDS void*)(lds_panel + ins * 1024), 16, 0, 0);
    }
  }
  __device__ __forceinline__ void commit(char*) const {}
  static constexpr bool kRegs = false;
};

// ---- uint8 operand through registers (u8 -> f32) ----------------------------
struct LoaderU8 {
  const uint8_t* base;  // [rows][ld] bytes, ld % 16 == 0
  int64_t ld;
  int64_t rows;
  int64_t r0;
  int64_t K;            // valid k (bytes beyond are zero-masked)
  uint4 v[2];

  __device__ __forceinline__ void issue(char*, int kt) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = threadIdx.x + 256 * s;     // 512 chunks of 16 B = 256 rows x 32 B
      const int row = q >> 1;
      const int half = q & 1;
      int64_t grow = r0 + row;
      grow = grow < rows ? grow : rows - 1;
      const int64_t k = (int64_t)kt * BK + half * 16;
      if (k < K) {
        v[s] = *reinterpret_cast<const uint4*>(base + grow * ld + k);
        if (k + 16 > K) {  // partial chunk: zero the bytes >= K
          const int keep = (int)(K - k);
          uint32_t w[4] = {v[s].x, v[s].y, v[s].z, v[s].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int lo = i * 4;
            uint32_t m = 0;
            if (keep >= lo + 4) m = 0xffffffffu;
            else if (keep > lo) m = (1u << (8 * (keep - lo))) - 1u;
            w[i] &= m;
          }
          v[s] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      } else {
        v[s] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void commit(char* lds_panel) const {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int q = threadIdx.x + 256 * s;
      const int row = q >> 1;
      const int half = q & 1;
      const uint32_t w[4] = {v[s].x, v[s].y, v[s].z, v[s].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        f32x4 f;
        f[0] = (float)(w[c] & 0xff);
        f[1] = (float)((w[c] >> 8) & 0xff);
        f[2] = (float)((w[c] >> 16) & 0xff);
        f[3] = (float)(w[c] >> 24);
        *reinterpret_cast<f32x4*>(lds_panel + lds_off(row, half * 4 + c)) = f;
      }
    }
  }
  static constexpr bool kRegs = true;
};

// ---- main loop ----------------------------------------------------------------
// acc[rt][ct] : rt = 32-row block of A inside the wave's 128 rows, ct = same for B.
// C/D map of v_mfma_f32_32x32x2_f32: col (B row) = lane&31,
// row (A row) = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
template <class LA, class LB>
__device__ __forceinline__ void mainloop(char* smem, LA& la, LB& lb, int nk, f32x16 (&acc)[4][4]) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wr = wave >> 1;  // A half
  const int wc = wave & 1;   // B half
  const int h = lane >> 5;
  const int r32 = lane & 31;

#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // prologue: panel 0 -> stage 0
  la.issue(smem, 0);
  lb.issue(smem + PANEL_BYTES, 0);
  la.commit(smem);
  lb.commit(smem + PANEL_BYTES);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // per-lane fragment byte offsets (row part), chunk added per k-block
  int arow[4], brow[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    arow[t] = wr * 128 + t * 32 + r32;
    brow[t] = wc * 128 + t * 32 + r32;
  }

  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      la.issue(nxt, kt + 1);
      lb.issue(nxt + PANEL_BYTES, kt + 1);
    }
#pragma unroll
    for (int kb = 0; kb < BK / 8; ++kb) {
      f32x4 a[4], b[4];
      const int chunk = 2 * kb + h;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = *reinterpret_cast<const f32x4*>(cur + lds_off(arow[t], chunk));
        b[t] = *reinterpret_cast<const f32x4*>(cur + PANEL_BYTES + lds_off(brow[t], chunk));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][e], b[j][e], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.commit(nxt);
      lb.commit(nxt + PANEL_BYTES);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
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
