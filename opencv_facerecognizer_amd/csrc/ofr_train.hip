// Training-side kernels (PCA Gram / LDA scatter / W = P.L) on gfx950.
//
// The reference trains Fisherfaces with numpy float64 (feature.py:83-108 PCA,
// :147-182 LDA, :211-235 Fisherfaces).  The dense products move to the fp64
// MFMA (v_mfma_f64_16x16x4_f64, 78.6 TF peak); the eigensolves stay on host
// LAPACK as the reference calls them.
//
// ofr_gemm_f64: 64x64 output tile per 256-thread workgroup (4 waves, 2x2,
// each 32x32 = 2x2 MFMA blocks of 16x16), K panels of 16 staged in LDS
// as [k][m] with an 80-double row pitch (conflict-free ds_read_b64 for the
// 16-lane x 4-k fragment reads).  f64 MFMA C/D map: col = lane&15,
// row = (lane>>4) + 4*reg;  A/B: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15].
#include "ofr_common.h"

namespace ofr {

constexpr int G64_T = 64, G64_BK = 16, G64_PITCH = 80;

struct Gemm64Args {
  int transA, transB;
  int64_t M, N, K;
  double alpha, beta;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  double* C;
  int64_t ldc;
};

// element (m, k) of op(A) where op(A) is M x K
__device__ __forceinline__ double opA(const Gemm64Args& p, int64_t m, int64_t k) {
  if (m >= p.M || k >= p.K) return 0.0;
  return p.transA ? p.A[k * p.lda + m] : p.A[m * p.lda + k];
}
// element (k, n) of op(B) where op(B) is K x N
__device__ __forceinline__ double opB(const Gemm64Args& p, int64_t k, int64_t n) {
  if (n >= p.N || k >= p.K) return 0.0;
  return p.transB ? p.B[n * p.ldb + k] : p.B[k * p.ldb + n];
}

__global__ void __launch_bounds__(256) gemm_f64_kernel(Gemm64Args p) {
  __shared__ double As[G64_BK][G64_PITCH];
  __shared__ double Bs[G64_BK][G64_PITCH];
  const int64_t m0 = (int64_t)blockIdx.y * G64_T, n0 = (int64_t)blockIdx.x * G64_T;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int wr = wave >> 1, wc = wave & 1;
  f64x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f64x4{0, 0, 0, 0};

  for (int64_t k0 = 0; k0 < p.K; k0 += G64_BK) {
    // stage 64 x 16 of op(A) and 16 x 64 of op(B); the index order follows the
    // contiguous dimension of the stored matrix for coalescing
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      int mm, kk;
      if (p.transA) { mm = e & 63; kk = e >> 6; } else { kk = e & 15; mm = e >> 4; }
      As[kk][mm] = opA(p, m0 + mm, k0 + kk);
      int nn, kb;
      if (p.transB) { kb = e & 15; nn = e >> 4; } else { nn = e & 63; kb = e >> 6; }
      Bs[kb][nn] = opB(p, k0 + kb, n0 + nn);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < G64_BK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk][wr * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk][wc * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 32 + i * 16 + (lane >> 4) + 4 * r;
        const int64_t n = n0 + wc * 32 + j * 16 + (lane & 15);
        if (m < p.M && n < p.N) {
          double* c = p.C + m * p.ldc + n;
          const double v = p.alpha * acc[i][j][r];
          *c = p.beta == 0.0 ? v : v + p.beta * *c;
        }
      }
}

// exact integer column sums of uint8 rows (row chunks, 64-bit atomics: exact and order-independent)
__global__ void col_sum_u8_kernel(const uint8_t* X, int64_t N, int64_t D, int64_t ldx, unsigned long long* sums) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  const int64_t rows = cdiv(N, (int64_t)gridDim.y);
  const int64_t r0 = (int64_t)blockIdx.y * rows, r1 = min(N, r0 + rows);
  unsigned long long s = 0;
  for (int64_t n = r0; n < r1; ++n) s += X[n * ldx + j];
  if (s) atomicAdd(&sums[j], s);
}
__global__ void div_u64_kernel(const unsigned long long* sums, int64_t D, int64_t N, double* mean) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < D) mean[j] = (double)sums[j] / (double)N;
}

constexpr int CM_CHUNKS = 128;
__global__ void col_mean_f64_partial(const double* X, int64_t N, int64_t D, int64_t ldx, double* part) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  const int64_t rows = cdiv(N, CM_CHUNKS);
  const int64_t r0 = (int64_t)blockIdx.y * rows, r1 = min(N, r0 + rows);
  double s = 0;
  for (int64_t n = r0; n < r1; ++n) s += X[n * ldx + j];
  part[(int64_t)blockIdx.y * D + j] = s;
}
__global__ void col_mean_f64_final(const double* part, int64_t N, int64_t D, double* mean) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  double s = 0;
  for (int c = 0; c < CM_CHUNKS; ++c) s += part[(int64_t)c * D + j];
  mean[j] = s / (double)N;
}

__global__ void center_u8_f64_kernel(const uint8_t* X, int64_t N, int64_t D, int64_t ldx, const double* mean,
                                     double* out, int64_t ldo) {
  const int64_t n = blockIdx.y;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < D; j += (int64_t)gridDim.x * blockDim.x)
    out[n * ldo + j] = (double)X[n * ldx + j] - mean[j];
}

__global__ void sub_mean_f64_kernel(const double* X, int64_t D, int64_t ldx, const double* mean, double* out,
                                    int64_t ldo) {
  const int64_t n = blockIdx.y;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < D; j += (int64_t)gridDim.x * blockDim.x)
    out[n * ldo + j] = X[n * ldx + j] - mean[j];
}

// unit 2-norm columns (one block per column, fixed-order reduction)
__global__ void normalize_cols_kernel(double* U, int64_t rows, int64_t ldu) {
  __shared__ double red[4];
  const int64_t c = blockIdx.x;
  double s = 0;
  for (int64_t r = threadIdx.x; r < rows; r += blockDim.x) {
    const double x = U[r * ldu + c];
    s += x * x;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const double nrm = sqrt(red[0] + red[1] + red[2] + red[3]);
  const double inv = nrm > 0 ? 1.0 / nrm : 0.0;
  for (int64_t r = threadIdx.x; r < rows; r += blockDim.x) U[r * ldu + c] *= inv;
}

// per (class, column): sum of the class's rows in perm order -> mean, then Mc rows
__global__ void class_mean_kernel(const double* F, int64_t D, int64_t ldf, const int64_t* perm, const int64_t* offsets,
                                  const double* total_mean, double* means, double* Mc, double* Mc_n) {
  const int64_t c = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  const int64_t s = offsets[c], e = offsets[c + 1];
  double acc = 0;
  for (int64_t r = s; r < e; ++r) acc += F[perm[r] * ldf + j];
  const double cnt = (double)(e - s);
  const double mu = e > s ? acc / cnt : 0.0;
  means[c * D + j] = mu;
  const double dm = mu - total_mean[j];
  Mc[c * D + j] = dm;
  Mc_n[c * D + j] = cnt * dm;
}

__global__ void class_center_kernel(const double* F, int64_t r_base, int64_t D, int64_t ldf, const int64_t* perm,
                                    const int64_t* offsets, int64_t c, const double* means, double* Fc) {
  // one block row per sample in perm order; class by binary search of the offsets
  const int64_t r = r_base + blockIdx.y;
  int64_t lo = 0, hi = c;  // find class k with offsets[k] <= r < offsets[k+1]
  while (hi - lo > 1) {
    const int64_t mid = (lo + hi) / 2;
    if (offsets[mid] <= r) lo = mid; else hi = mid;
  }
  const int64_t row = perm[r];
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < D; j += (int64_t)gridDim.x * blockDim.x)
    Fc[row * D + j] = F[row * ldf + j] - means[lo * D + j];
}

}  // namespace ofr

using namespace ofr;

extern "C" int ofr_gemm_f64(void* stream, int transA, int transB, int64_t M, int64_t N, int64_t K, double alpha,
                            const double* A, int64_t lda, const double* B, int64_t ldb, double beta, double* C,
                            int64_t ldc) {
  OFR_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "ofr_gemm_f64: bad sizes");
  if (M == 0 || N == 0) return OFR_OK;
  OFR_CHECK_ARG(C && ldc >= N, "ofr_gemm_f64: bad C");
  if (K > 0) {
    OFR_CHECK_ARG(A && B, "ofr_gemm_f64: null operand");
    OFR_CHECK_ARG(lda >= (transA ? M : K) && ldb >= (transB ? K : N), "ofr_gemm_f64: bad leading dimension");
  }
  OFR_CHECK_ARG(cdiv(M, G64_T) < 65536, "ofr_gemm_f64: M too large");
  Gemm64Args p{transA, transB, M, N, K, alpha, beta, A, lda, B, ldb, C, ldc};
  hipLaunchKernelGGL(gemm_f64_kernel, dim3((unsigned)cdiv(N, G64_T), (unsigned)cdiv(M, G64_T)), dim3(256), 0,
                     (hipStream_t)stream, p);
  OFR_LAUNCH_CHECK("gemm_f64_kernel");
  return OFR_OK;
}

extern "C" int ofr_col_mean_u8(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx, double* mean) {
  OFR_CHECK_ARG(N > 0 && D >= 1 && ldx >= D && X && mean, "ofr_col_mean_u8: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  unsigned long long* sums = nullptr;
  hipError_t e = hipMallocAsync((void**)&sums, sizeof(unsigned long long) * D, st);
  if (e != hipSuccess) return hip_status(e, "hipMallocAsync(col_mean_u8)");
  e = hipMemsetAsync(sums, 0, sizeof(unsigned long long) * D, st);
  if (e != hipSuccess) return hip_status(e, "hipMemsetAsync(col_mean_u8)");
  const unsigned chunks = (unsigned)std::min<int64_t>(256, std::max<int64_t>(1, N / 64));
  hipLaunchKernelGGL(col_sum_u8_kernel, dim3((unsigned)cdiv(D, 256), chunks), dim3(256), 0, st, X, N, D, ldx, sums);
  hipLaunchKernelGGL(div_u64_kernel, dim3((unsigned)cdiv(D, 256)), dim3(256), 0, st, sums, D, N, mean);
  hipError_t le = hipGetLastError();
  e = hipFreeAsync(sums, st);
  if (le != hipSuccess) return hip_status(le, "col_mean_u8 kernels");
  return e == hipSuccess ? OFR_OK : hip_status(e, "hipFreeAsync(col_mean_u8)");
}

extern "C" int ofr_col_mean_f64(void* stream, const double* X, int64_t N, int64_t D, int64_t ldx, double* mean) {
  OFR_CHECK_ARG(N > 0 && D >= 1 && ldx >= D && X && mean, "ofr_col_mean_f64: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * CM_CHUNKS * D, st);
  if (e != hipSuccess) return hip_status(e, "hipMallocAsync(col_mean_f64)");
  hipLaunchKernelGGL(col_mean_f64_partial, dim3((unsigned)cdiv(D, 256), CM_CHUNKS), dim3(256), 0, st, X, N, D, ldx,
                     part);
  hipLaunchKernelGGL(col_mean_f64_final, dim3((unsigned)cdiv(D, 256)), dim3(256), 0, st, part, N, D, mean);
  hipError_t le = hipGetLastError();
  e = hipFreeAsync(part, st);
  if (le != hipSuccess) return hip_status(le, "col_mean_f64 kernels");
  return e == hipSuccess ? OFR_OK : hip_status(e, "hipFreeAsync(col_mean_f64)");
}

extern "C" int ofr_center_u8_f64(void* stream, const uint8_t* X, int64_t N, int64_t D, int64_t ldx, const double* mean,
                                 double* out, int64_t ldo) {
  OFR_CHECK_ARG(N >= 0 && D >= 1 && ldx >= D && ldo >= D, "ofr_center_u8_f64: bad sizes");
  if (N == 0) return OFR_OK;
  OFR_CHECK_ARG(X && mean && out, "ofr_center_u8_f64: null pointer");
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(D, 256), 64);
  for (int64_t done = 0; done < N; done += 65535) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(center_u8_f64_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream,
                       X + done * ldx, chunk, D, ldx, mean, out + done * ldo, ldo);
    OFR_LAUNCH_CHECK("center_u8_f64_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_class_center_f64(void* stream, const double* F, int64_t N, int64_t D, int64_t ldf,
                                    const int64_t* perm, const int64_t* offsets, int64_t c, const double* total_mean,
                                    double* means, double* Fc, double* Mc, double* Mc_n) {
  OFR_CHECK_ARG(N >= 1 && D >= 1 && ldf >= D && c >= 1 && c < 65536, "ofr_class_center_f64: bad sizes");
  OFR_CHECK_ARG(F && perm && offsets && total_mean && means && Fc && Mc && Mc_n, "ofr_class_center_f64: null pointer");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(class_mean_kernel, dim3((unsigned)cdiv(D, 256), (unsigned)c), dim3(256), 0, st, F, D, ldf, perm,
                     offsets, total_mean, means, Mc, Mc_n);
  OFR_LAUNCH_CHECK("class_mean_kernel");
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(D, 256), 64);
  for (int64_t done = 0; done < N; done += 65535) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(class_center_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, st, F, done, D, ldf, perm,
                       offsets, c, means, Fc);
    OFR_LAUNCH_CHECK("class_center_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_sub_mean_f64(void* stream, const double* X, int64_t N, int64_t D, int64_t ldx, const double* mean,
                                double* out, int64_t ldo) {
  OFR_CHECK_ARG(N >= 0 && D >= 1 && ldx >= D && ldo >= D, "ofr_sub_mean_f64: bad sizes");
  if (N == 0) return OFR_OK;
  OFR_CHECK_ARG(X && mean && out, "ofr_sub_mean_f64: null pointer");
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(D, 256), 64);
  for (int64_t done = 0; done < N; done += 65535) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(sub_mean_f64_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream,
                       X + done * ldx, D, ldx, mean, out + done * ldo, ldo);
    OFR_LAUNCH_CHECK("sub_mean_f64_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_normalize_cols_f64(void* stream, double* U, int64_t rows, int64_t cols, int64_t ldu) {
  OFR_CHECK_ARG(rows >= 0 && cols >= 0 && ldu >= cols, "ofr_normalize_cols_f64: bad sizes");
  if (rows == 0 || cols == 0) return OFR_OK;
  OFR_CHECK_ARG(U && cols < 0x7fffffffLL, "ofr_normalize_cols_f64: bad arguments");
  hipLaunchKernelGGL(normalize_cols_kernel, dim3((unsigned)cols), dim3(256), 0, (hipStream_t)stream, U, rows, ldu);
  OFR_LAUNCH_CHECK("normalize_cols_kernel");
  return OFR_OK;
}
