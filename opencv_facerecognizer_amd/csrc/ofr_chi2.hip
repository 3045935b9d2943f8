// Chi-square nearest-neighbour search on gfx950 (VALU tile kernel).
//
// Replaces ChiSquareDistance (reference distance.py:112-116,
// sum((p-q)^2 / (p+q+eps))) inside NearestNeighbor.predict
// (classifier.py:104-119) for LBP spatial histograms (feature.py:286-302).
//
// chi^2 has no bilinear form, so it runs on the vector ALUs: one workgroup
// computes a 64-query x 64-gallery tile, 4x4 pairs per thread, histogram bins
// streamed through LDS in [bin][row] panels of 64 bins (uint8/16/32 counts or
// fp32 values widened once on the LDS write).  Coarse fp32 score per pair:
//     S = sum_b (a-c)^2 * rcp(a+c)   on values staged + 2^-100 (empty bins give exact 0)
// The best KC rows per query per tile go to cand[tile][query][KC]; the merge
// kernel then re-evaluates the reference formula EXACTLY in fp64 on the
// survivors, with p = value/denom (denom = cell pixel count for counts, the
// reference histogram being count/(py*px)) and eps = 2^-52.
#include <atomic>
#include <cmath>
#include <mutex>
#include <cstring>
#include <string>
#include <vector>

#include "ofr_f6_tile.h"
#include "ofr_i8_tile.h"
#include "ofr_keys.h"
#include "ofr_topk.h"

namespace ofr {

enum { DT_U8 = 0, DT_U16 = 1, DT_U32 = 2, DT_F32 = 3 };
constexpr int C2_TQ = 64, C2_TG = 64, C2_BB = 64;
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int DT>
__device__ __forceinline__ void load16(const void* base, int64_t ld, int64_t row, int64_t b0, float (&v)[16]) {
  if constexpr (DT == DT_U8) {
    const uint4 x = *reinterpret_cast<const uint4*>((const uint8_t*)base + row * ld + b0);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = (float)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
  } else if constexpr (DT == DT_U16) {
    const uint4* p = reinterpret_cast<const uint4*>((const uint16_t*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4 x = p[h];
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) v[8 * h + i] = (float)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
    }
  } else if constexpr (DT == DT_U32) {
    const uint4* p = reinterpret_cast<const uint4*>((const uint32_t*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint4 x = p[h];
      v[4 * h + 0] = (float)x.x;
      v[4 * h + 1] = (float)x.y;
      v[4 * h + 2] = (float)x.z;
      v[4 * h + 3] = (float)x.w;
    }
  } else {
    const f32x4* p = reinterpret_cast<const f32x4*>((const float*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const f32x4 x = p[h];
      v[4 * h + 0] = x[0];
      v[4 * h + 1] = x[1];
      v[4 * h + 2] = x[2];
      v[4 * h + 3] = x[3];
    }
  }
}

template <int DT>
__device__ __forceinline__ double load1(const void* base, int64_t idx) {
  if constexpr (DT == DT_U8) return (double)((const uint8_t*)base)[idx];
  else if constexpr (DT == DT_U16) return (double)((const uint16_t*)base)[idx];
  else if constexpr (DT == DT_U32) return (double)((const uint32_t*)base)[idx];
  else return (double)((const float*)base)[idx];
}

struct Chi2Args {
  const void* Q;
  int64_t B, ldq;
  const void* G;
  int64_t N, ldg;
  int64_t nbins;
  Cand* cand;  // [T][B][KC]
  int64_t ntq, ntg;
  double denom;   // exact pass: reference values are element / denom
};

// Exact pass (the certificate's fallback, few queries): the reference formula distance.py:115-116
// in fp64 per (pair, bin) -- p = value / denom, (p - q)^2 / (p + q + eps) -- on 16 x 16 pairs
// per workgroup, values staged once as fp64 p = v / denom in LDS.  The tile lists carry the sum
// rounded to fp32 (a 2^-24 relative key; the merge re-evaluates the survivors in fp64 again).
constexpr int C2X_T = 32;
template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_exact_tile_kernel(Chi2Args p) {
  __shared__ double Qs[C2_BB][C2X_T];
  __shared__ double Gs[C2_BB][C2X_T + 1];
  __shared__ float S[C2X_T][C2X_T + 1];
  const int64_t t = blockIdx.x;
  const int64_t gt = t / p.ntq, qt = t % p.ntq;
  const int64_t q0 = qt * C2X_T, g0 = gt * C2X_T;
  const int tid = threadIdx.x;
  const int tq = tid >> 4, tg = tid & 15;      // queries tq*2.., gallery tg*2..
  const double eps = 2.220446049250313e-16;    // np.finfo('float').eps, distance.py:115
  double acc[2][2] = {{0, 0}, {0, 0}};
  for (int64_t b0 = 0; b0 < p.nbins; b0 += C2_BB) {
    __syncthreads();
    for (int e = tid; e < C2_BB * C2X_T; e += 256) {
      const int r = e / C2_BB, b = e % C2_BB;
      const int64_t bb = b0 + b;
      const int64_t qr = min(q0 + r, p.B - 1), gr = min(g0 + r, p.N - 1);
      Qs[b][r] = bb < p.nbins ? load1<DT>(p.Q, qr * p.ldq + bb) / p.denom : 0.0;
      Gs[b][r] = bb < p.nbins ? load1<DT>(p.G, gr * p.ldg + bb) / p.denom : 0.0;
    }
    __syncthreads();
    const int nb = (int)min((int64_t)C2_BB, p.nbins - b0);
    for (int b = 0; b < nb; ++b) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const double x = Qs[b][tq * 2 + i], y = Gs[b][tg * 2 + j];
          const double df = x - y;
          acc[i][j] += (df * df) / (x + y + eps);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) S[tq * 2 + i][tg * 2 + j] = (float)acc[i][j];
  __syncthreads();
  if (tid < C2X_T) {
    const int64_t q = q0 + tid;
    TopList<KC> L;
    L.init();
    for (int j = 0; j < C2X_T; ++j) {
      const int64_t g = g0 + j;
      if (g < p.N) L.insert(S[tid][j], (int)g);
    }
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_tile_kernel(Chi2Args p) {
  __shared__ __attribute__((aligned(16))) float Qs[C2_BB][C2_TQ];
  __shared__ __attribute__((aligned(16))) float Gs[C2_BB][C2_TG];
  __shared__ float S[C2_TQ][C2_TG + 1];
  const int64_t t = blockIdx.x;
  const int64_t gt = t / p.ntq, qt = t % p.ntq;  // consecutive blocks share the gallery tile
  const int64_t q0 = qt * C2_TQ, g0 = gt * C2_TG;
  const int tid = threadIdx.x;
  const int tq = tid >> 4, tg = tid & 15;       // compute: queries tq*4.., gallery tg*4..
  const int lrow = tid >> 2, lseg = tid & 3;    // staging: row, 16-bin segment
  const int64_t qrow = min(q0 + lrow, p.B - 1);
  const int64_t grow = min(g0 + lrow, p.N - 1);

  f32x2 acc2[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc2[i][0] = acc2[i][1] = f32x2{0.f, 0.f};

  float vq[16], vg[16];
  const int nsteps = (int)(p.nbins / C2_BB);
  if (nsteps > 0) {
    load16<DT>(p.Q, p.ldq, qrow, lseg * 16, vq);
    load16<DT>(p.G, p.ldg, grow, lseg * 16, vg);
  }
  for (int s = 0; s < nsteps; ++s) {
    __syncthreads();
    // values are staged biased by 2^-100: a + c > 0 for every pair (no per-pair "+ tiny"), while
    // a - c and (a + c) for a, c >= 2^-76 round exactly as without the bias
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      Qs[lseg * 16 + i][lrow] = vq[i] + 0x1p-100f;
      Gs[lseg * 16 + i][lrow] = vg[i] + 0x1p-100f;
    }
    __syncthreads();
    if (s + 1 < nsteps) {
      load16<DT>(p.Q, p.ldq, qrow, (int64_t)(s + 1) * C2_BB + lseg * 16, vq);
      load16<DT>(p.G, p.ldg, grow, (int64_t)(s + 1) * C2_BB + lseg * 16, vg);
    }
    // packed fp32: per two (pair, bin) terms one v_pk_add for a - c, one for a + c, two v_rcp,
    // v_pk_mul, v_pk_fma
#pragma unroll 4
    for (int b = 0; b < C2_BB; ++b) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&Qs[b][tq * 4]);
      const f32x4 c = *reinterpret_cast<const f32x4*>(&Gs[b][tg * 4]);
      const f32x2 c01 = {c[0], c[1]}, c23 = {c[2], c[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 ai = {a[i], a[i]};
        const f32x2 d0 = ai - c01, s0 = ai + c01, d1 = ai - c23, s1 = ai + c23;
        const f32x2 r0 = {__builtin_amdgcn_rcpf(s0[0]), __builtin_amdgcn_rcpf(s0[1])};
        const f32x2 r1 = {__builtin_amdgcn_rcpf(s1[0]), __builtin_amdgcn_rcpf(s1[1])};
        acc2[i][0] = __builtin_elementwise_fma(d0 * d0, r0, acc2[i][0]);
        acc2[i][1] = __builtin_elementwise_fma(d1 * d1, r1, acc2[i][1]);
      }
    }
  }
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = acc2[i][j >> 1][j & 1];
  // tail bins (nbins % 64): plain loads
  for (int64_t b = (int64_t)nsteps * C2_BB; b < p.nbins; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = (float)load1<DT>(p.Q, min(q0 + tq * 4 + i, p.B - 1) * p.ldq + b);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = (float)load1<DT>(p.G, min(g0 + tg * 4 + j, p.N - 1) * p.ldg + b);
        const float df = a - c;
        acc[i][j] = __builtin_fmaf(df * df, __builtin_amdgcn_rcpf((a + c) + 1e-30f), acc[i][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) S[tq * 4 + i][tg * 4 + j] = acc[i][j];
  __syncthreads();
  if (tid < C2_TQ) {
    const int64_t q = q0 + tid;
    TopList<KC> L;
    L.init();
    for (int j = 0; j < C2_TG; ++j) {
      const int64_t g = g0 + j;
      if (g < p.N) L.insert(S[tid][j], (int)g);
    }
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

struct Chi2MergeArgs {
  const Cand* cand;
  int64_t T, B;
  const void* Q;
  int64_t ldq;
  const void* G;
  int64_t ldg, nbins;
  double denom;
  int k;
  int64_t index_base;
  double* out_d;
  int64_t* out_i;
  int* cert;      // nullable: 1 iff the result is provably the exact fp64 top-k
  double gamma;   // relative error bound of the coarse scores (and their keys)
  double scale;   // coarse score -> reference units (1 / denom for the fp32 pass, 1 for the exact pass)
  // MFMA pass (abs_c1 > 0): |S - S~| <= abs_c1 (Tq + Tg) in count units, Tq = the query's total
  // count, Tg <= *tg_max (the gallery's largest row total)
  double abs_c1;
  const float* tg_max;
};

template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_merge_rerank_kernel(Chi2MergeArgs p) {
  __shared__ Cand lists[256 * KC];
  __shared__ double exact[KC];
  __shared__ double red[4];
  const int64_t q = blockIdx.x;
  select_candidates<KC>(p.cand, p.T, p.B, q, lists);
  const double eps = 2.220446049250313e-16;  // np.finfo('float').eps, distance.py:115
  double tq = 0;
  if (p.abs_c1 > 0) {
    double a = 0;
    for (int64_t b = threadIdx.x; b < p.nbins; b += blockDim.x) a += load1<DT>(p.Q, q * p.ldq + b);
    tq = block_sum_f64(a, red);
  }
  for (int c = 0; c < KC; ++c) {
    const Cand cc = lists[c];
    double val = __builtin_inf();
    if (cc.i != CAND_EMPTY) {
      double a = 0;
      for (int64_t b = threadIdx.x; b < p.nbins; b += blockDim.x) {
        const double x = load1<DT>(p.Q, q * p.ldq + b) / p.denom;
        const double y = load1<DT>(p.G, (int64_t)cc.i * p.ldg + b) / p.denom;
        const double df = x - y;
        a += (df * df) / (x + y + eps);
      }
      val = block_sum_f64(a, red);
    }
    if (threadIdx.x == 0) exact[c] = val;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    double* od = p.out_d + q * p.k;
    const double dk = sort_and_write_wave<KC>(lists, exact, p.k, p.index_base, od, p.out_i + q * p.k);
    if (p.cert && threadIdx.x == 0) {
      // certificate: every row outside the KC candidates has coarse score >= tau (the KC-th
      // candidate; a tile's excluded rows are >= its own KC-th, which is >= tau), so its exact
      // distance is >= tau * scale / (1 + gamma).  The top-k is exact iff the k-th exact distance
      // lies strictly below that (a relative 1e-12 for the fp64 evaluation order).
      const Cand last = lists[KC - 1];
      double bnd = __builtin_inf();
      if (last.i != CAND_EMPTY && p.abs_c1 > 0)
        bnd = ((double)last.d - p.abs_c1 * (tq + (double)*p.tg_max)) * p.scale * (1.0 - 1e-12);
      else if (last.i != CAND_EMPTY)
        bnd = (double)last.d * p.scale / (1.0 + p.gamma) * (1.0 - 1e-12);
      p.cert[q] = (dk == dk) && (dk < bnd);
    }
  }
}

template <int DT, int KC>
static int launch_chi2(hipStream_t st, const Chi2Args& a, const Chi2MergeArgs& m, bool exact) {
  if (a.N > 0) {
    if (exact)
      hipLaunchKernelGGL((chi2_exact_tile_kernel<DT, KC>), dim3((unsigned)(a.ntq * a.ntg)), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((chi2_tile_kernel<DT, KC>), dim3((unsigned)(a.ntq * a.ntg)), dim3(256), 0, st, a);
    OFR_LAUNCH_CHECK("chi2_tile_kernel");
  }
  hipLaunchKernelGGL((chi2_merge_rerank_kernel<DT, KC>), dim3((unsigned)m.B), dim3(256), 0, st, m);
  OFR_LAUNCH_CHECK("chi2_merge_rerank_kernel");
  return OFR_OK;
}

template <int DT>
static int chi2_dispatch(hipStream_t st, int kc, const Chi2Args& a, const Chi2MergeArgs& m, bool exact) {
  return kc == 8 ? launch_chi2<DT, 8>(st, a, m, exact) : launch_chi2<DT, 16>(st, a, m, exact);
}

// ---- MFMA coarse pass for uint8 counts (the LBP spatial histograms) -------------------------
// chi^2 has no bilinear form, but for counts it has a short low-rank one.  Per bin
//     T(a, c) = (a - c)^2 / (a + c) = (a + c) - 4 F(a, c),   F(a, c) = a c / (a + c)  (0 at a = c = 0)
// so S(q, g) = sum_b T(a_b, c_b) = Tq + Tg - 4 sum_b F(a_b, c_b) with the row totals Tq, Tg exact.
// F is a positive semidefinite kernel on 0..255 whose spectrum falls off fast; its eight leading
// eigenpairs (of the (a+1)^-1/2-weighted matrix, so that the error scales with a + c) give
// F(a, c) ~= sum_r U[a][r] U[c][r], U an fp16 table [256][8] with U[0] = 0 (exact: F(0, c) = 0).
// One v_mfma_f32_16x16x32_f16 then sums 4 bins x 8 components for a 16 x 16 block: lane group q
// (lanes 16q..16q+15) supplies, for its row, the table row of its bin's count, gathered from LDS.
// Rigorous coarse-score bound (host-computed constants, chi2_table):
//   |S - S~| <= 4 (eta + gamma kappa)(Tq + Tg) + 2^-22 (Tq + Tg),
//   eta   = max_{a+c>0} |F(a,c) - sum_r U16[a][r] U16[c][r]| / (a + c)     (rank + fp16 rounding)
//   kappa = max_{a+c>0} sum_r |U16[a][r] U16[c][r]| / (a + c)              (sum |products| per bin)
//   gamma = (n_mfma + 64) 2^-23, n_mfma = nbins / 4 per accumulator       (fp32 accumulation, the
//           fp6 tier's budget: tools/mx_probe.hip measured <= 3 2^-24 per MFMA step)
// the last term covering the fp32 evaluation of Tq + Tg - 4 acc.  The merge re-ranks the best 16
// exactly (the reference formula, fp64) and certifies with this absolute bound.
namespace c2m {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int TG = 256, TQ = 256;          // gallery x query rows per tile
constexpr int NW = 8, NT = NW * 64;        // 8 waves (2 per SIMD), wave grid 2 (gallery) x 4 (queries)
constexpr int WQ = 4, QW = 64, NA = 8, NB = 4;   // wave: 128 gallery rows (8 blocks) x 64 queries (4)
constexpr int BB = 64;                     // bins per LDS stage = 16 MFMA k-steps of 4 bins
constexpr int PANEL = 256 * BB;            // 16 KiB: 256 rows x 64 count bytes
constexpr int STAGE = 2 * PANEL;
constexpr int NST = 3;
constexpr int TABLE = 256 * 16;            // fp16 [256][8]
constexpr int LDS = NST * STAGE + TABLE;   // 100 KiB
constexpr int DMA_INS = STAGE / 1024;      // 32 one-KiB copies per stage
constexpr int IPW = DMA_INS / NW;          // 4 per wave
constexpr int KC = keys::KC;               // candidates per (query, tile)

// LDS image of a stage panel: row r's 64 bytes = four 16-byte chunks, chunk g at position
// g ^ ((r >> 2) & 3), so that the 16 rows a lane group reads hit distinct banks
__device__ __forceinline__ int off(int row, int chunk) { return row * BB + ((chunk ^ ((row >> 2) & 3)) << 4); }

struct Args {
  const uint8_t* Q;
  int64_t B, ldq;
  const uint8_t* G;
  int64_t N, ldg, nbins;
  const uint16_t* table;   // fp16 bits [256][8]
  const float* tq;         // [B] query row totals
  const float* tg;         // [N] gallery row totals
  Cand* cand;              // [ntg][B][KC], tile-major
  int64_t ntq, ntg, gg;
};

// stage kt (bins [64 kt, 64 kt + 64)) of the tile's gallery rows [g0, g0 + 256) and query rows
// [q0, q0 + 256) -> LDS stage buffer st; rows past the end re-read the last row (never scored)
__device__ __forceinline__ void dma(const Args& p, int64_t g0, int64_t q0, int kt, char* st) {
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int ng = (int)(p.N - g0 < TG ? p.N - g0 : TG), nq = (int)(p.B - q0 < TQ ? p.B - q0 : TQ);
  __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(p.G + g0 * p.ldg), 0,
                                                                (int)((int64_t)ng * p.ldg), 0x00020000);
  __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)(p.Q + q0 * p.ldq), 0,
                                                                (int)((int64_t)nq * p.ldq), 0x00020000);
#pragma unroll
  for (int t = 0; t < IPW; ++t) {
    const int ins = wave * IPW + t;   // a wave's four copies are all gallery (waves 0-3) or all queries
    const bool gal = ins < DMA_INS / 2;
    const int row = (ins & 15) * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const int lim = gal ? ng : nq;
    const int r = row < lim ? row : lim - 1;
    const int voff = r * (int)(gal ? p.ldg : p.ldq) + kt * BB + chunk * 16;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(gal ? rg : rq, (OFR_LDS void*)(st + (gal ? 0 : PANEL) + (ins & 15) * 1024),
                                             16, voff, 0, 0, 0);
  }
}

__global__ void __launch_bounds__(NT, 1) chi2_mfma_kernel(Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  const int64_t g0 = gt * TG, q0 = qt * TQ;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / WQ, wc = wave % WQ, r16 = lane & 15, lq = lane >> 4;
  char* tab = smem + NST * STAGE;
  reinterpret_cast<uint2*>(tab)[threadIdx.x] = reinterpret_cast<const uint2*>(p.table)[threadIdx.x];   // 4 KiB
  const int nst = (int)(p.nbins / BB), last = nst - 1;
#pragma unroll
  for (int s = 0; s < NST - 1; ++s) dma(p, g0, q0, s < last ? s : last, smem + s * STAGE);

  f32x4 acc[NA][NB];
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int c = 0; c < NB; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int ra0 = wr * 128 + r16, rb0 = wc * QW + r16;   // + 16 i / + 16 c

  for (int kt = 0; kt < nst; ++kt) {
    f6t::wait_vm<IPW>();   // stage kt landed (kt + 1 may be in flight)
    f6t::barrier();        // ... for every wave; and every wave is done with stage kt - 1's buffer
    {
      const int nx = kt + NST - 1;
      dma(p, g0, q0, nx < last ? nx : last, smem + (nx % NST) * STAGE);
    }
    const char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int g = 0; g < BB / 16; ++g) {
      // counts of bins 16 g + 4 lq .. + 3 of every fragment row (one word per row; k-step s uses byte s)
      uint32_t wa[NA], wb[NB];
#pragma unroll
      for (int i = 0; i < NA; ++i) wa[i] = *reinterpret_cast<const uint32_t*>(st + off(ra0 + 16 * i, g) + 4 * lq);
#pragma unroll
      for (int c = 0; c < NB; ++c) wb[c] = *reinterpret_cast<const uint32_t*>(st + PANEL + off(rb0 + 16 * c, g) + 4 * lq);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        h8 fa[NA], fb[NB];
#pragma unroll
        for (int i = 0; i < NA; ++i) fa[i] = *reinterpret_cast<const h8*>(tab + (((wa[i] >> (8 * s)) & 0xffu) << 4));
#pragma unroll
        for (int c = 0; c < NB; ++c) fb[c] = *reinterpret_cast<const h8*>(tab + (((wb[c] >> (8 * s)) & 0xffu) << 4));
#pragma unroll
        for (int i = 0; i < NA; ++i)
#pragma unroll
          for (int c = 0; c < NB; ++c) acc[i][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i], fb[c], acc[i][c], 0, 0, 0);
      }
    }
  }
  f6t::wait_vm<0>();
  f6t::barrier();

  // epilogue: S~ = Tq + Tg - 4 acc -> keys; per lane the best KC of its 32 rows for each of its 4
  // queries, merged over the 4 lane groups (shuffles), then over the two row-waves (LDS)
  float* tq_l = reinterpret_cast<float*>(smem);                  // [256]
  float* tg_l = tq_l + TQ;                                       // [256]
  uint32_t* kbuf = reinterpret_cast<uint32_t*>(smem + 2048);     // [2][256][KC]
  if (threadIdx.x < TQ) {
    const int64_t q = q0 + threadIdx.x, g = g0 + threadIdx.x;
    tq_l[threadIdx.x] = q < p.B ? p.tq[q] : 0.f;
    tg_l[threadIdx.x] = g < p.N ? p.tg[g] : 0.f;
  }
  __syncthreads();
  const int nvalid = p.N - g0 < TG ? (int)(p.N - g0) : TG;
  auto epi = [&](auto ctc) {
    constexpr int c = decltype(ctc)::value;
    const int ql = wc * QW + 16 * c + r16;
    const float tqv = tq_l[ql];
    keys::KeyList L;
    L.init();
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gl = wr * 128 + 16 * i + 4 * lq + r;   // C/D of 16x16: row 4 (lane / 16) + reg, column lane % 16
        const float sc = (tqv + tg_l[gl]) - 4.0f * acc[i][c][r];
        L.insert(gl < nvalid ? keys::score_key(sc, gl) : keys::KEY_NONE);
      }
    uint32_t o[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) o[j] = (uint32_t)__shfl_xor((int)L.k[j], 16);
    L.merge(o);
#pragma unroll
    for (int j = 0; j < KC; ++j) o[j] = (uint32_t)__shfl_xor((int)L.k[j], 32);
    L.merge(o);
    if (lq == 0) {
      uint32_t* dst = kbuf + ((size_t)wr * TQ + ql) * KC;
#pragma unroll
      for (int j = 0; j < KC; j += 4) *reinterpret_cast<uint4*>(dst + j) = make_uint4(L.k[j], L.k[j + 1], L.k[j + 2], L.k[j + 3]);
    }
  };
  epi(std::integral_constant<int, 0>{});
  epi(std::integral_constant<int, 1>{});
  epi(std::integral_constant<int, 2>{});
  epi(std::integral_constant<int, 3>{});
  __syncthreads();
  if ((int)threadIdx.x < TQ) {
    const int ql = threadIdx.x;
    const int64_t q = q0 + ql;
    keys::KeyList L;
    uint32_t o[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      L.k[j] = kbuf[(size_t)ql * KC + j];
      o[j] = kbuf[((size_t)TQ + ql) * KC + j];
    }
    L.merge(o);
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const uint32_t kk = L.k[j];
        out[j] = kk == keys::KEY_NONE ? Cand{__builtin_inff(), CAND_EMPTY}
                                      : Cand{keys::key_score(kk), (int)(g0 + (kk & 0xffu))};
      }
    }
  }
}

// row totals (exact: < 2^24) and the gallery's largest (float bits are ordered like uints for >= 0)
__global__ void __launch_bounds__(256) row_total_kernel(const uint8_t* X, int64_t rows, int64_t ld, int64_t nbins,
                                                        float* tot, unsigned* maxbits) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const uint8_t* x = X + r * ld;
  uint32_t s = 0;
  for (int64_t b = (int64_t)lane * 16; b < nbins; b += 64 * 16) {
    const uint4 v = *reinterpret_cast<const uint4*>(x + b);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) s += (w[j] & 0xff) + ((w[j] >> 8) & 0xff) + ((w[j] >> 16) & 0xff) + (w[j] >> 24);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) {
    tot[r] = (float)s;
    if (maxbits) atomicMax(maxbits, __float_as_uint((float)s));
  }
}

}  // namespace c2m

// The fp16 table and its error constants, built once on the host (deterministic): subspace iteration
// for the 8 leading eigenpairs of Fw[a][c] = F(a, c) / sqrt((a+1)(c+1)), U = sqrt(a+1) V sqrt(L),
// rounded to fp16, row 0 zero; eta and kappa evaluated exactly (fp64) over all 256 x 256 pairs.
struct Chi2Table {
  uint16_t bits[256 * 8];
  double eta, kappa;
  uint16_t* dev = nullptr;   // device copy (per process; one device at a time is enough for the table)
  int dev_id = -1;
};

static void jacobi_eig(int n, std::vector<double>& A, std::vector<double>& V) {   // A symmetric n x n
  V.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i) V[(size_t)i * n + i] = 1.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) off += A[(size_t)i * n + j] * A[(size_t)i * n + j];
    if (off < 1e-30) break;
    for (int p = 0; p < n; ++p)
      for (int q = p + 1; q < n; ++q) {
        const double apq = A[(size_t)p * n + q];
        if (std::fabs(apq) < 1e-300) continue;
        const double theta = (A[(size_t)q * n + q] - A[(size_t)p * n + p]) / (2 * apq);
        const double tt = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1));
        const double cs = 1 / std::sqrt(tt * tt + 1), sn = tt * cs;
        for (int k = 0; k < n; ++k) {
          const double akp = A[(size_t)k * n + p], akq = A[(size_t)k * n + q];
          A[(size_t)k * n + p] = cs * akp - sn * akq;
          A[(size_t)k * n + q] = sn * akp + cs * akq;
        }
        for (int k = 0; k < n; ++k) {
          const double apk = A[(size_t)p * n + k], aqk = A[(size_t)q * n + k];
          A[(size_t)p * n + k] = cs * apk - sn * aqk;
          A[(size_t)q * n + k] = sn * apk + cs * aqk;
        }
        for (int k = 0; k < n; ++k) {
          const double vkp = V[(size_t)k * n + p], vkq = V[(size_t)k * n + q];
          V[(size_t)k * n + p] = cs * vkp - sn * vkq;
          V[(size_t)k * n + q] = sn * vkp + cs * vkq;
        }
      }
  }
}

static Chi2Table& chi2_table() {
  static Chi2Table T = [] {
    Chi2Table t{};
    constexpr int n = 256, R = 8, M = 16;   // M: subspace width
    std::vector<double> Fm((size_t)n * n);
    for (int a = 0; a < n; ++a)
      for (int c = 0; c < n; ++c) {
        const double s = (double)a + c;
        Fm[(size_t)a * n + c] = s > 0 ? (double)a * c / s / std::sqrt((a + 1.0) * (c + 1.0)) : 0.0;
      }
    auto Fw = [&](int a, int c) { return Fm[(size_t)a * n + c]; };
    std::vector<double> X((size_t)n * M), Y((size_t)n * M);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < M; ++j) X[(size_t)i * M + j] = std::cos(0.37 * (i + 1) * (j + 1)) + (i == j ? 1.0 : 0.0);
    std::vector<double> H, W;
    for (int it = 0; it < 40; ++it) {
      for (int i = 0; i < n; ++i)   // Y = Fw X
        for (int j = 0; j < M; ++j) {
          double acc = 0;
          for (int k = 0; k < n; ++k) acc += Fw(i, k) * X[(size_t)k * M + j];
          Y[(size_t)i * M + j] = acc;
        }
      for (int j = 0; j < M; ++j) {   // modified Gram-Schmidt on the columns of Y
        for (int l = 0; l < j; ++l) {
          double d = 0;
          for (int i = 0; i < n; ++i) d += Y[(size_t)i * M + j] * Y[(size_t)i * M + l];
          for (int i = 0; i < n; ++i) Y[(size_t)i * M + j] -= d * Y[(size_t)i * M + l];
        }
        double nn = 0;
        for (int i = 0; i < n; ++i) nn += Y[(size_t)i * M + j] * Y[(size_t)i * M + j];
        nn = std::sqrt(nn);
        for (int i = 0; i < n; ++i) Y[(size_t)i * M + j] /= nn;
      }
      X.swap(Y);
    }
    // Rayleigh-Ritz: H = X^T Fw X, X <- X W (descending eigenvalues)
    H.assign((size_t)M * M, 0.0);
    std::vector<double> FX((size_t)n * M);
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < M; ++j) {
        double acc = 0;
        for (int k = 0; k < n; ++k) acc += Fw(i, k) * X[(size_t)k * M + j];
        FX[(size_t)i * M + j] = acc;
      }
    for (int a = 0; a < M; ++a)
      for (int b = 0; b < M; ++b) {
        double acc = 0;
        for (int i = 0; i < n; ++i) acc += X[(size_t)i * M + a] * FX[(size_t)i * M + b];
        H[(size_t)a * M + b] = acc;
      }
    for (int a = 0; a < M; ++a)
      for (int b = a + 1; b < M; ++b) H[(size_t)a * M + b] = H[(size_t)b * M + a] = 0.5 * (H[(size_t)a * M + b] + H[(size_t)b * M + a]);
    jacobi_eig(M, H, W);
    std::vector<int> ord(M);
    for (int j = 0; j < M; ++j) ord[j] = j;
    std::sort(ord.begin(), ord.end(), [&](int x, int y) { return H[(size_t)x * M + x] > H[(size_t)y * M + y]; });
    double U[n][R];
    for (int r = 0; r < R; ++r) {
      const int j = ord[r];
      const double lam = std::max(H[(size_t)j * M + j], 0.0);
      for (int i = 0; i < n; ++i) {
        double v = 0;
        for (int k = 0; k < M; ++k) v += X[(size_t)i * M + k] * W[(size_t)k * M + j];
        U[i][r] = i == 0 ? 0.0 : std::sqrt(i + 1.0) * v * std::sqrt(lam);
      }
    }
    double U16[n][R];
    for (int i = 0; i < n; ++i)
      for (int r = 0; r < R; ++r) {
        const _Float16 h = (_Float16)U[i][r];
        U16[i][r] = (double)h;
        uint16_t b;
        std::memcpy(&b, &h, 2);
        t.bits[i * R + r] = b;
      }
    double eta = 0, kappa = 0;
    for (int a = 0; a < n; ++a)
      for (int c = 0; c < n; ++c) {
        if (a + c == 0) continue;
        double sum = 0, sabs = 0;
        for (int r = 0; r < R; ++r) {
          sum += U16[a][r] * U16[c][r];
          sabs += std::fabs(U16[a][r] * U16[c][r]);
        }
        const double F = (double)a * c / ((double)a + c);
        eta = std::max(eta, std::fabs(F - sum) / (a + c));
        kappa = std::max(kappa, sabs / (a + c));
      }
    t.eta = eta * (1 + 1e-9) + 1e-15;     // fp64 evaluation slack
    t.kappa = kappa * (1 + 1e-9);
    return t;
  }();
  return T;
}

static bool chi2_engine_valu() {   // OFR_CHI2_ENGINE=valu: the VALU tile kernel for every dtype (read per call)
  const char* e = getenv("OFR_CHI2_ENGINE");
  return e && std::string(e) == "valu";
}

}  // namespace ofr

using namespace ofr;

// MFMA pass workspace: tile lists [ceil(N/256)][B][16], query / gallery row totals, the largest total
struct Chi2MWs {
  size_t lists, tq, tg, tgmax, bytes;
};
static Chi2MWs chi2m_ws(int64_t B, int64_t N) {
  Chi2MWs w;
  const int64_t T = cdiv(N > 0 ? N : 1, c2m::TG);
  w.lists = 0;
  w.tq = round_up((int64_t)((size_t)T * B * c2m::KC * sizeof(Cand)), 256);
  w.tg = w.tq + round_up(B * 4, 256);
  w.tgmax = w.tg + round_up((N > 0 ? N : 1) * 4, 256);
  w.bytes = w.tgmax + 256;
  return w;
}

extern "C" size_t ofr_chi2_workspace_bytes(int64_t B, int64_t N, int k) {
  const int kc = pick_kc(k);
  const int64_t T = cdiv(N > 0 ? N : 1, C2X_T);   // the exact pass's 32-row tiles (>= the 64-row ones)
  return std::max((size_t)T * (size_t)B * kc * sizeof(Cand) + 256, chi2m_ws(B, N).bytes);
}

// the MFMA coarse pass (uint8 counts) + the exact re-rank with its absolute certificate
static int chi2_mfma_run(hipStream_t st, const uint8_t* Q, int64_t B, int64_t ldq, const uint8_t* G, int64_t N,
                         int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                         int64_t* out_i, void* workspace, int* cert) {
  Chi2Table& tb = chi2_table();
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e, "hipGetDevice");
  // per-device fp16 table (4 KiB): uploaded once under a lock and published only after the copy
  // completed, so a caller on another thread (one context per thread) never sees an unfilled table
  static std::atomic<uint16_t*> table_dev[64] = {};
  static std::mutex table_mu;
  static std::atomic<bool> attr_done{false};
  if (dev < 0 || dev >= 64) return fail(OFR_E_UNSUPPORTED, "ofr_chi2_knn: device index >= 64");
  uint16_t* table = table_dev[dev].load(std::memory_order_acquire);
  if (!table) {
    std::lock_guard<std::mutex> g(table_mu);
    table = table_dev[dev].load(std::memory_order_acquire);
    if (!table) {
      uint16_t* t = nullptr;
      e = hipMalloc((void**)&t, sizeof(tb.bits));
      if (e == hipSuccess) e = hipMemcpy(t, tb.bits, sizeof(tb.bits), hipMemcpyHostToDevice);
      if (e != hipSuccess) {
        if (t) (void)hipFree(t);
        return hip_status(e, "ofr_chi2_knn: table upload");
      }
      table_dev[dev].store(t, std::memory_order_release);
      table = t;
    }
  }
  if (!attr_done.load(std::memory_order_acquire)) {
    e = hipFuncSetAttribute((const void*)c2m::chi2_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, c2m::LDS);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(chi2_mfma)");
    attr_done.store(true, std::memory_order_release);
  }
  const Chi2MWs w = chi2m_ws(B, N);
  char* wsb = reinterpret_cast<char*>(workspace);
  float* tq = reinterpret_cast<float*>(wsb + w.tq);
  float* tg = reinterpret_cast<float*>(wsb + w.tg);
  unsigned* tgmax = reinterpret_cast<unsigned*>(wsb + w.tgmax);
  e = hipMemsetAsync(tgmax, 0, 4, st);
  if (e != hipSuccess) return hip_status(e, "hipMemsetAsync(tgmax)");
  hipLaunchKernelGGL(c2m::row_total_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, st, Q, B, ldq, nbins, tq,
                     (unsigned*)nullptr);
  OFR_LAUNCH_CHECK("row_total_kernel");
  hipLaunchKernelGGL(c2m::row_total_kernel, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, st, G, N, ldg, nbins, tg, tgmax);
  OFR_LAUNCH_CHECK("row_total_kernel");
  c2m::Args a;
  a.Q = Q; a.B = B; a.ldq = ldq; a.G = G; a.N = N; a.ldg = ldg; a.nbins = nbins;
  a.table = table; a.tq = tq; a.tg = tg;
  a.cand = reinterpret_cast<Cand*>(wsb + w.lists);
  a.ntq = cdiv(B, c2m::TQ);
  a.ntg = cdiv(N, c2m::TG);
  a.gg = a.ntg < 4 ? a.ntg : 4;
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_chi2_knn: grid too large");
  hipLaunchKernelGGL(c2m::chi2_mfma_kernel, dim3((unsigned)(a.ntq * a.ntg)), dim3(c2m::NT), c2m::LDS, st, a);
  OFR_LAUNCH_CHECK("chi2_mfma_kernel");
  const double n_mfma = (double)(nbins / 4);
  const double gamma = (n_mfma + 64.0) * 0x1p-23;
  Chi2MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, nbins, denom, k, index_base, out_d, out_i, cert, 0.0,
                  1.0 / denom};
  m.abs_c1 = 4.0 * (tb.eta + gamma * tb.kappa) + 0x1p-22;
  m.tg_max = reinterpret_cast<const float*>(tgmax);
  hipLaunchKernelGGL((chi2_merge_rerank_kernel<DT_U8, c2m::KC>), dim3((unsigned)B), dim3(256), 0, st, m);
  OFR_LAUNCH_CHECK("chi2_merge_rerank_kernel");
  return OFR_OK;
}

extern "C" void ofr_chi2_table(uint16_t* out) { std::memcpy(out, chi2_table().bits, sizeof(chi2_table().bits)); }

extern "C" double ofr_chi2_mfma_bound(int64_t nbins) {
  Chi2Table& tb = chi2_table();
  return 4.0 * (tb.eta + ((double)(nbins / 4) + 64.0) * 0x1p-23 * tb.kappa) + 0x1p-22;
}

static int chi2_run(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                    int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                    int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert, bool exact) {
  OFR_CHECK_ARG(dtype >= DT_U8 && dtype <= DT_F32, "ofr_chi2_knn: dtype must be 0 (u8), 1 (u16), 2 (u32) or 3 (f32)");
  OFR_CHECK_ARG(B >= 0 && N >= 0 && nbins >= 1 && denom > 0, "ofr_chi2_knn: bad sizes");
  if (k < 1 || k > OFR_MAX_K) return fail(OFR_E_UNSUPPORTED, "ofr_chi2_knn: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  const int esz = dtype == DT_U8 ? 1 : dtype == DT_U16 ? 2 : 4;
  OFR_CHECK_ARG(Q && out_d && out_i && workspace, "ofr_chi2_knn: null pointer");
  OFR_CHECK_ARG(ldq >= nbins && (ldq * esz) % 16 == 0 && ((uintptr_t)Q % 16) == 0,
                "ofr_chi2_knn: query rows must be 16-byte aligned (ldq*elem % 16 == 0)");
  if (N > 0) {
    OFR_CHECK_ARG(G, "ofr_chi2_knn: null gallery");
    OFR_CHECK_ARG(ldg >= nbins && (ldg * esz) % 16 == 0 && ((uintptr_t)G % 16) == 0,
                  "ofr_chi2_knn: gallery rows must be 16-byte aligned (ldg*elem % 16 == 0)");
    OFR_CHECK_ARG(N < 0x7fffffffLL - C2_TG, "ofr_chi2_knn: N too large for one shard");
  }
  const int kc = pick_kc(k);
  OFR_CHECK_ARG(workspace_bytes >= ofr_chi2_workspace_bytes(B, N, k), "ofr_chi2_knn: workspace too small");
  Chi2Args a;
  a.Q = Q; a.B = B; a.ldq = ldq; a.G = G; a.N = N; a.ldg = ldg; a.nbins = nbins; a.denom = denom;
  a.cand = reinterpret_cast<Cand*>(workspace);
  const int tq = exact ? C2X_T : C2_TQ, tg = exact ? C2X_T : C2_TG;
  a.ntq = cdiv(B, tq);
  a.ntg = N > 0 ? cdiv(N, tg) : 0;
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_chi2_knn: grid too large");
  // error bound of the coarse scores (relative): the fp32 pass sums ceil(nbins / 2) terms per
  // accumulator sequentially (two packed halves) and each term d^2 * rcp(s) carries <= 2 ulp
  // (d, s exact for integer counts < 2^24; <= 2 more ulp from their roundings for fp32 values);
  // the exact pass's key is its fp64 sum rounded to fp32 (1/2 ulp) plus the fp64 summation.
  const double gamma = exact ? 0x1p-23 + (double)nbins * 0x1p-52
                             : ((double)((nbins + 1) / 2) + 4.0) * 0x1p-24 + (dtype == DT_F32 ? 4.0 : 2.0) * 0x1p-23;
  hipStream_t st = (hipStream_t)stream;
  // uint8 counts (LBP spatial histograms): the low-rank MFMA coarse pass (OFR_CHI2_ENGINE=valu: the VALU kernel)
  if (!exact && dtype == DT_U8 && N > 0 && nbins % c2m::BB == 0 && ldq % 16 == 0 && ldg % 16 == 0 &&
      !chi2_engine_valu())
    return chi2_mfma_run(st, (const uint8_t*)Q, B, ldq, (const uint8_t*)G, N, ldg, nbins, denom, k, index_base,
                         out_d, out_i, workspace, cert);
  Chi2MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, nbins, denom, k, index_base, out_d, out_i, cert, gamma,
                  exact ? 1.0 : 1.0 / denom};
  switch (dtype) {
    case DT_U8: return chi2_dispatch<DT_U8>(st, kc, a, m, exact);
    case DT_U16: return chi2_dispatch<DT_U16>(st, kc, a, m, exact);
    case DT_U32: return chi2_dispatch<DT_U32>(st, kc, a, m, exact);
    default: return chi2_dispatch<DT_F32>(st, kc, a, m, exact);
  }
}

extern "C" int ofr_chi2_knn(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                            int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                            int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert) {
  return chi2_run(stream, dtype, Q, B, ldq, G, N, ldg, nbins, denom, k, index_base, out_d, out_i, workspace,
                  workspace_bytes, cert, false);
}

extern "C" int ofr_chi2_knn_exact(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G,
                                  int64_t N, int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base,
                                  double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert) {
  return chi2_run(stream, dtype, Q, B, ldq, G, N, ldg, nbins, denom, k, index_base, out_d, out_i, workspace,
                  workspace_bytes, cert, true);
}
