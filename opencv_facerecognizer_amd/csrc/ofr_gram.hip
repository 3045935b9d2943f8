// Exact Gram / scatter products of uint8 face data for Fisherfaces training (gfx950).
//
// Replaces the float64 products of the reference's training:
//   PCA.compute  feature.py:91-94   XC = X - mean; svd(XC): its Gram XC XC^T (n <= D) or the
//                                   covariance XC^T XC (n > D);
//   LDA.compute  feature.py:160-168 Sw = sum_i (X_i - m_i)(X_i - m_i)^T, Sb = sum_i n_i (m_i - m)(m_i - m)^T
//                                   (in pixel space when PCA keeps every dimension: a rotation).
// Pixels are integers, so every such product is an integer matrix plus rank-one / class-sum
// corrections:  with x' = x - 128 (int8, exact),
//     X'^T X'  (or X' X'^T)  on v_mfma_i32_32x32x32_i8  -- EXACT int32 per K chunk of < 2^17
//                            columns (|x' y'| <= 2^14), chunks summed in fp64 (exact: integers
//                            below 2^53),
// and the centring terms (column sums, class sums: exact integers) are applied in fp64 by the
// host pipeline (training.py).  The reference computes the same quantities from float64
// XC = X - mean, whose elements are already rounded; these are exact before the final fp64
// rounding.  The int8 engine (ofr_i8_tile.h, 256 x 256 tiles) runs at the int8 MFMA rate, 32x the
// fp32 MFMA and 64x the fp64 MFMA rate.  The Gram is symmetric: only tiles on or above the
// diagonal are computed, sym_lower_kernel mirrors them.
//
// Work per launch: 2 R^2 K / 2 int8 ops for the upper triangle (R = rows of the operand, K = its
// columns); bytes: R K (1 B per element) per 256-row tile pair re-read from L2.
#include "ofr_i8_tile.h"

namespace ofr {
namespace gram {

using i8t::i32x16;
using S = i8t::Shape<1>;

struct Args {
  const uint8_t* X;   // [R][ld] uint8, pad columns hold 128 (x' = 0)
  int64_t R, ld, k0;  // rows, row pitch, first column of this K chunk
  int nk;             // 128-column steps of this chunk
  int64_t nt;         // 256-row tiles
  double* C;
  int64_t ldc;
  int accumulate;     // C += chunk (else C = chunk)
};

// tile t of the upper triangle (row-major: (0,0), (0,1), ..., (0,nt-1), (1,1), ...)
__device__ __forceinline__ void tri_coords(int64_t t, int64_t nt, int64_t& at, int64_t& bt) {
  // rows a hold nt - a tiles; find the largest a with start(a) = a nt - a (a - 1) / 2 <= t
  int64_t a = (int64_t)((2.0 * nt + 1.0 - sqrt((2.0 * nt + 1.0) * (2.0 * nt + 1.0) - 8.0 * (double)t)) / 2.0);
  if (a < 0) a = 0;
  if (a > nt - 1) a = nt - 1;
  auto start = [&](int64_t r) { return r * nt - r * (r - 1) / 2; };
  while (a > 0 && start(a) > t) --a;
  while (a + 1 < nt && start(a + 1) <= t) ++a;
  at = a;
  bt = a + (t - start(a));
}

__global__ void __launch_bounds__(S::NT, 1) gram_u8_kernel(Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t at, bt;
  tri_coords(t, p.nt, at, bt);
  const int64_t a0 = at * i8t::TA, b0 = bt * S::TQ;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / S::WQ, wc = wave % S::WQ, h = lane >> 5, r32 = lane & 31;
  const int8_t* base = reinterpret_cast<const int8_t*>(p.X) + p.k0;
  const int64_t cols = (int64_t)p.nk * i8t::ROWB;
  i32x16 acc[4][S::CT], unused[4][1];
  i8t::mainloop<1, true, true>(smem, base, p.ld, p.R, a0, base, p.ld, p.R, b0, cols, p.nk, acc, unused);
  // C/D map of v_mfma_i32_32x32x32_i8: A row (reg & 3) + 8 (reg >> 2) + 4 h of the 32-block, B row lane & 31
#pragma unroll
  for (int ct = 0; ct < S::CT; ++ct) {
    const int64_t b = b0 + wc * S::QW + ct * 32 + r32;
    if (b >= p.R) continue;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t a = a0 + wr * 128 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (a >= p.R) continue;
        double* c = p.C + a * p.ldc + b;
        const double v = (double)acc[rt][ct][r];
        *c = p.accumulate ? *c + v : v;
      }
  }
}

// out[r][k] = in[k][r] (transpose) or in[r][k], k < K; 128 (x' = 0) in the pad columns [K, ldo).
// 64 x 64 tiles through LDS (coalesced both ways).
__global__ void __launch_bounds__(256) pad_u8_kernel(const uint8_t* in, int64_t rows_in, int64_t cols_in, int64_t ldi,
                                                     int transpose, uint8_t* out, int64_t rows_out, int64_t ldo) {
  __shared__ uint8_t tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;   // output tile
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t K = transpose ? rows_in : cols_in;   // valid output columns
  if (transpose) {
    for (int y = ty; y < 64; y += 4) {   // read in[c0 + y][r0 + tx]
      const int64_t ir = c0 + y, ic = r0 + tx;
      tile[y][tx] = (ir < rows_in && ic < cols_in) ? in[ir * ldi + ic] : (uint8_t)128;
    }
    __syncthreads();
    for (int y = ty; y < 64; y += 4) {
      const int64_t orow = r0 + y, ocol = c0 + tx;
      if (orow < rows_out && ocol < ldo) out[orow * ldo + ocol] = ocol < K ? tile[tx][y] : (uint8_t)128;
    }
  } else {
    for (int y = ty; y < 64; y += 4) {
      const int64_t orow = r0 + y, ocol = c0 + tx;
      if (orow < rows_out && ocol < ldo)
        out[orow * ldo + ocol] = (ocol < K && orow < rows_in) ? in[orow * ldi + ocol] : (uint8_t)128;
    }
  }
}

// C[b][a] = C[a][b] for a < b (lower triangle from the upper), 64 x 64 tile pairs through LDS
__global__ void __launch_bounds__(256) sym_lower_kernel(double* C, int64_t R, int64_t ldc) {
  __shared__ double tile[64][65];
  const int64_t ta = blockIdx.y, tb = blockIdx.x;   // source tile (ta, tb) with ta <= tb
  if (ta > tb) return;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int y = ty; y < 64; y += 4) {
    const int64_t a = ta * 64 + y, b = tb * 64 + tx;
    tile[y][tx] = (a < R && b < R) ? C[a * ldc + b] : 0.0;
  }
  __syncthreads();
  for (int y = ty; y < 64; y += 4) {
    const int64_t b = tb * 64 + y, a = ta * 64 + tx;   // destination row b, column a
    if (a < R && b < R && a < b) C[b * ldc + a] = tile[tx][y];
  }
}

// exact per-class column sums of x - shift (shift 0 or 128) over uint8 rows (classes given by
// perm / offsets), fp64 storage of the integers; means (nullable) = sums / n_class, rounded once
__global__ void __launch_bounds__(256) class_sums_u8_kernel(const uint8_t* X, int64_t D, int64_t ldx,
                                                            const int64_t* perm, const int64_t* offsets, int shift,
                                                            double* sums, double* means) {
  const int64_t c = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  const int64_t r0 = offsets[c], r1 = offsets[c + 1];
  int64_t s = 0;
  for (int64_t r = r0; r < r1; ++r) s += X[perm[r] * ldx + j];
  s -= (int64_t)shift * (r1 - r0);
  sums[c * D + j] = (double)s;
  if (means) means[c * D + j] = r1 > r0 ? (double)s / (double)(r1 - r0) : 0.0;
}

// r[n] = sum_j (X[n][j] - 128) s[j]: exact int64 (|s| <= 2^53 / (128 D) is the caller's bound)
__global__ void __launch_bounds__(256) row_dot_u8_kernel(const uint8_t* X, int64_t N, int64_t D, int64_t ldx,
                                                         const double* s, double* r) {
  __shared__ long long red[4];
  const int64_t n = blockIdx.x;
  long long acc = 0;
  for (int64_t j = threadIdx.x; j < D; j += blockDim.x) acc += (long long)((int)X[n * ldx + j] - 128) * (long long)s[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) r[n] = (double)(red[0] + red[1] + red[2] + red[3]);
}

// C[a][b] += alpha (u[a] + u[b]) + beta   (the rank-one centring of a Gram of rows)
__global__ void __launch_bounds__(256) center_gram_kernel(double* C, int64_t R, int64_t ldc, const double* u,
                                                          double alpha, double beta) {
  const int64_t a = blockIdx.y;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < R; b += (int64_t)gridDim.x * blockDim.x)
    C[a * ldc + b] += alpha * (u[a] + u[b]) + beta;
}

// Sw / Sb of pixel-space LDA from the exact pieces (all D x D, fp64):
//   Sw = G - T,  Sb = T - s s^T / N       (G = X'^T X', T = sum_i s_i s_i^T / n_i, s = column sums of X')
__global__ void __launch_bounds__(256) scatter_combine_kernel(const double* G, const double* T, const double* s,
                                                              double invN, int64_t D, int64_t ld, double* Sw,
                                                              double* Sb) {
  const int64_t a = blockIdx.y;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < D; b += (int64_t)gridDim.x * blockDim.x) {
    const double t = T[a * ld + b];
    if (Sw) Sw[a * ld + b] = G[a * ld + b] - t;
    Sb[a * ld + b] = t - s[a] * s[b] * invN;
  }
}

// C[a][b] += alpha u[a] v[b]
__global__ void __launch_bounds__(256) rank1_kernel(double* C, int64_t cols, int64_t ldc, const double* u,
                                                    const double* v, double alpha) {
  const int64_t a = blockIdx.y;
  const double ua = alpha * u[a];
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < cols; b += (int64_t)gridDim.x * blockDim.x)
    C[a * ldc + b] += ua * v[b];
}

// out[r][j] = A[r][j] / n[r]  (class means from class sums; n[r] = 0 -> 0)
__global__ void __launch_bounds__(256) row_div_kernel(const double* A, int64_t cols, int64_t lda, const double* n,
                                                      double* out, int64_t ldo) {
  const int64_t r = blockIdx.y;
  const double nr = n[r];
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < cols; j += (int64_t)gridDim.x * blockDim.x)
    out[r * ldo + j] = nr != 0.0 ? A[r * lda + j] / nr : 0.0;
}

}  // namespace gram
}  // namespace ofr

using namespace ofr;

extern "C" int ofr_pad_u8(void* stream, const uint8_t* X, int64_t rows, int64_t cols, int64_t ldx, int transpose,
                          uint8_t* out, int64_t ldo) {
  OFR_CHECK_ARG(rows >= 0 && cols >= 0 && ldx >= cols, "ofr_pad_u8: bad sizes");
  const int64_t orows = transpose ? cols : rows, K = transpose ? rows : cols;
  OFR_CHECK_ARG(ldo >= K, "ofr_pad_u8: ldo < output columns");
  if (orows == 0) return OFR_OK;
  OFR_CHECK_ARG(X && out, "ofr_pad_u8: null pointer");
  OFR_CHECK_ARG(cdiv(orows, 64) < 65536, "ofr_pad_u8: too many rows for one launch");
  hipLaunchKernelGGL(gram::pad_u8_kernel, dim3((unsigned)cdiv(ldo, 64), (unsigned)cdiv(orows, 64)), dim3(256), 0,
                     (hipStream_t)stream, X, rows, cols, ldx, transpose, out, orows, ldo);
  OFR_LAUNCH_CHECK("pad_u8_kernel");
  return OFR_OK;
}

extern "C" int ofr_gram_u8(void* stream, const uint8_t* X, int64_t R, int64_t K, int64_t ld, double* C, int64_t ldc) {
  OFR_CHECK_ARG(R >= 0 && K >= 0 && ld % 128 == 0 && ld >= round_up(K, 128) && ldc >= R,
                "ofr_gram_u8: bad sizes (ld % 128 == 0, >= round_up(K, 128), pad columns = 128)");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && C, "ofr_gram_u8: null pointer");
  OFR_CHECK_ARG(((uintptr_t)X & 15) == 0, "ofr_gram_u8: X must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)gram::gram_u8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       gram::S::LDS);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(gram_u8)");
    attr_done = true;
  }
  gram::Args a{};
  a.X = X; a.R = R; a.ld = ld; a.C = C; a.ldc = ldc;
  a.nt = cdiv(R, i8t::TA);
  const int64_t tiles = a.nt * (a.nt + 1) / 2;
  OFR_CHECK_ARG(tiles < 0x7fffffffLL, "ofr_gram_u8: too many tiles");
  const int64_t kpad = round_up(K > 0 ? K : 1, 128);
  // int32 stays exact: |x' y'| <= 2^14, so a chunk of < 2^17 columns sums to < 2^31
  constexpr int64_t KCHUNK = 131072;
  int64_t k0 = 0;
  do {
    const int64_t kc = std::min<int64_t>(KCHUNK - 128, kpad - k0);   // strictly below 2^31
    a.k0 = k0;
    a.nk = (int)(kc / 128);
    a.accumulate = k0 > 0;
    hipLaunchKernelGGL(gram::gram_u8_kernel, dim3((unsigned)tiles), dim3(gram::S::NT), gram::S::LDS, st, a);
    OFR_LAUNCH_CHECK("gram_u8_kernel");
    k0 += kc;
  } while (k0 < kpad);
  if (a.nt > 0) {
    const int64_t t64 = cdiv(R, 64);
    OFR_CHECK_ARG(t64 < 65536, "ofr_gram_u8: R too large to mirror");
    hipLaunchKernelGGL(gram::sym_lower_kernel, dim3((unsigned)t64, (unsigned)t64), dim3(256), 0, st, C, R, ldc);
    OFR_LAUNCH_CHECK("sym_lower_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_class_sums_u8(void* stream, const uint8_t* X, int64_t D, int64_t ldx, const int64_t* perm,
                                 const int64_t* offsets, int64_t c, int shift, double* sums, double* means) {
  OFR_CHECK_ARG(D >= 1 && ldx >= D && c >= 1 && c < 65536, "ofr_class_sums_u8: bad sizes");
  OFR_CHECK_ARG(shift == 0 || shift == 128, "ofr_class_sums_u8: shift must be 0 or 128");
  OFR_CHECK_ARG(X && perm && offsets && sums, "ofr_class_sums_u8: null pointer");
  hipLaunchKernelGGL(gram::class_sums_u8_kernel, dim3((unsigned)cdiv(D, 256), (unsigned)c), dim3(256), 0,
                     (hipStream_t)stream, X, D, ldx, perm, offsets, shift, sums, means);
  OFR_LAUNCH_CHECK("class_sums_u8_kernel");
  return OFR_OK;
}

extern "C" int ofr_row_dot_u8(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx, const double* s,
                              double* r) {
  OFR_CHECK_ARG(N >= 0 && D >= 1 && ldx >= D, "ofr_row_dot_u8: bad sizes");
  if (N == 0) return OFR_OK;
  OFR_CHECK_ARG(X && s && r && N < 0x7fffffffLL, "ofr_row_dot_u8: bad arguments");
  hipLaunchKernelGGL(gram::row_dot_u8_kernel, dim3((unsigned)N), dim3(256), 0, (hipStream_t)stream, X, N, D, ldx, s, r);
  OFR_LAUNCH_CHECK("row_dot_u8_kernel");
  return OFR_OK;
}

extern "C" int ofr_center_gram_f64(void* stream, double* C, int64_t R, int64_t ldc, const double* u, double alpha,
                                   double beta) {
  OFR_CHECK_ARG(R >= 0 && ldc >= R && R < 65536, "ofr_center_gram_f64: bad sizes");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(C && u, "ofr_center_gram_f64: null pointer");
  hipLaunchKernelGGL(gram::center_gram_kernel, dim3((unsigned)std::min<int64_t>(cdiv(R, 256), 64), (unsigned)R),
                     dim3(256), 0, (hipStream_t)stream, C, R, ldc, u, alpha, beta);
  OFR_LAUNCH_CHECK("center_gram_kernel");
  return OFR_OK;
}

extern "C" int ofr_scatter_combine_f64(void* stream, const double* G, const double* T, const double* s, double invN,
                                       int64_t D, int64_t ld, double* Sw, double* Sb) {
  OFR_CHECK_ARG(D >= 1 && ld >= D && D < 65536, "ofr_scatter_combine_f64: bad sizes");
  OFR_CHECK_ARG(G && T && s && Sb, "ofr_scatter_combine_f64: null pointer");
  hipLaunchKernelGGL(gram::scatter_combine_kernel, dim3((unsigned)std::min<int64_t>(cdiv(D, 256), 64), (unsigned)D),
                     dim3(256), 0, (hipStream_t)stream, G, T, s, invN, D, ld, Sw, Sb);
  OFR_LAUNCH_CHECK("scatter_combine_kernel");
  return OFR_OK;
}

extern "C" int ofr_rank1_f64(void* stream, double* C, int64_t rows, int64_t cols, int64_t ldc, const double* u,
                             const double* v, double alpha) {
  OFR_CHECK_ARG(rows >= 0 && cols >= 0 && ldc >= cols && rows < 65536 * 1024LL, "ofr_rank1_f64: bad sizes");
  if (rows == 0 || cols == 0) return OFR_OK;
  OFR_CHECK_ARG(C && u && v, "ofr_rank1_f64: null pointer");
  for (int64_t r0 = 0; r0 < rows; r0 += 65535) {
    const int64_t nr = std::min<int64_t>(65535, rows - r0);
    hipLaunchKernelGGL(gram::rank1_kernel, dim3((unsigned)std::min<int64_t>(cdiv(cols, 256), 64), (unsigned)nr),
                       dim3(256), 0, (hipStream_t)stream, C + r0 * ldc, cols, ldc, u + r0, v, alpha);
    OFR_LAUNCH_CHECK("rank1_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_row_div_f64(void* stream, const double* A, int64_t rows, int64_t cols, int64_t lda,
                               const double* n, double* out, int64_t ldo) {
  OFR_CHECK_ARG(rows >= 0 && cols >= 0 && lda >= cols && ldo >= cols, "ofr_row_div_f64: bad sizes");
  if (rows == 0 || cols == 0) return OFR_OK;
  OFR_CHECK_ARG(A && n && out, "ofr_row_div_f64: null pointer");
  for (int64_t r0 = 0; r0 < rows; r0 += 65535) {
    const int64_t nr = std::min<int64_t>(65535, rows - r0);
    hipLaunchKernelGGL(gram::row_div_kernel, dim3((unsigned)std::min<int64_t>(cdiv(cols, 256), 64), (unsigned)nr),
                       dim3(256), 0, (hipStream_t)stream, A + r0 * lda, cols, lda, n + r0, out + r0 * ldo, ldo);
    OFR_LAUNCH_CHECK("row_div_kernel");
  }
  return OFR_OK;
}
