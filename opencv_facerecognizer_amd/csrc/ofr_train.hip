// Training-side kernels (PCA Gram / LDA scatter / W = P.L) on gfx950.
//
// The reference trains Fisherfaces with numpy float64 (feature.py:83-108 PCA,
// :147-182 LDA, :211-235 Fisherfaces).  The dense products move to the fp64
// MFMA (v_mfma_f64_16x16x4_f64, 78.6 TF peak); the eigensolves stay on host
// LAPACK as the reference calls them.
//
// ofr_gemm_f64: 128 x 128 output tile per 256-thread workgroup (4 waves, 2 x 2, each 64 x 64 =
// 4 x 4 blocks of v_mfma_f64_16x16x4_f64, 128 accumulator VGPRs), K panels of 16 double-buffered
// in LDS as [k][m] / [k][n] with a 144-double pitch (rows k and k+1 in opposite bank halves: the
// 16-lane fragment reads are conflict free): the next panel's global loads (8 doubles per thread
// and operand, 16-B vector loads along the stored matrix's contiguous dimension) are in flight
// while the current panel's 4 k-steps run (64 MFMAs per wave, 64 cycles each).
// f64 MFMA maps (cdna_hip_programming.md): A/B lane l holds A[l&15][k=l>>4] / B[k=l>>4][l&15];
// C/D col = lane&15, row = (lane>>4) + 4*reg.  Two workgroups per CU (2 x 72 KiB LDS).
#include "ofr_common.h"

namespace ofr {

constexpr int G64_T = 128, G64_BK = 16, G64_PITCH = 144;

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

// 8 consecutive elements of op(X) (a 128 x 16 panel slab) -> registers, zero outside the matrix.
// trans = 0: X is stored [rows][K] (op(X) = X, K contiguous): thread t takes row t/2, k 8(t&1)..+7.
// trans = 1: X is stored [K][rows] (rows contiguous): thread t takes k t/16, rows 8(t&15)..+7.
__device__ __forceinline__ void load_slab(const double* X, int64_t ld, int64_t rows, int64_t K, int trans, int64_t r0,
                                          int64_t k0, double (&v)[8]) {
  const int t = threadIdx.x;
  if (!trans) {
    const int64_t r = r0 + (t >> 1), k = k0 + 8 * (t & 1);
    const bool rok = r < rows;
    const double* src = X + (rok ? r : 0) * ld + k;
    const bool vec = rok && k + 8 <= K && (((uintptr_t)src) & 15) == 0;
    if (vec) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const double2 x = *reinterpret_cast<const double2*>(src + e);
        v[e] = x.x;
        v[e + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (rok && k + e < K) ? src[e] : 0.0;
    }
  } else {
    const int64_t k = k0 + (t >> 4), r = r0 + 8 * (t & 15);
    const bool kok = k < K;
    const double* src = X + (kok ? k : 0) * ld + r;
    const bool vec = kok && r + 8 <= rows && (((uintptr_t)src) & 15) == 0;
    if (vec) {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const double2 x = *reinterpret_cast<const double2*>(src + e);
        v[e] = x.x;
        v[e + 1] = x.y;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (kok && r + e < rows) ? src[e] : 0.0;
    }
  }
}

// registers -> LDS panel [k][row] (the layout the fragments read)
__device__ __forceinline__ void store_slab(double (*P)[G64_PITCH], int trans, const double (&v)[8]) {
  const int t = threadIdx.x;
  if (!trans) {
    const int r = t >> 1, k = 8 * (t & 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) P[k + e][r] = v[e];
  } else {
    const int k = t >> 4, r = 8 * (t & 15);
#pragma unroll
    for (int e = 0; e < 8; ++e) P[k][r + e] = v[e];
  }
}

__global__ void __launch_bounds__(256, 2) gemm_f64_kernel(Gemm64Args p) {
  __shared__ double As[2][G64_BK][G64_PITCH];
  __shared__ double Bs[2][G64_BK][G64_PITCH];
  const int64_t m0 = (int64_t)blockIdx.y * G64_T, n0 = (int64_t)blockIdx.x * G64_T;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  f64x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f64x4{0, 0, 0, 0};
  // op(A) is M x K: stored [M][K] (transA = 0) or [K][M]; op(B) is K x N: stored [K][N] (transB = 0)
  // or [N][K] -- i.e. B's panel is a slab of B^T with the opposite storage flag
  double va[8], vb[8];
  const int npanel = (int)cdiv(p.K, G64_BK);
  load_slab(p.A, p.lda, p.M, p.K, p.transA, m0, 0, va);
  load_slab(p.B, p.ldb, p.N, p.K, !p.transB, n0, 0, vb);
  for (int kp = 0; kp < npanel; ++kp) {
    const int buf = kp & 1;
    store_slab(As[buf], p.transA, va);
    store_slab(Bs[buf], !p.transB, vb);
    __syncthreads();
    if (kp + 1 < npanel) {   // the next panel's loads fly under this panel's MFMAs
      load_slab(p.A, p.lda, p.M, p.K, p.transA, m0, (int64_t)(kp + 1) * G64_BK, va);
      load_slab(p.B, p.ldb, p.N, p.K, !p.transB, n0, (int64_t)(kp + 1) * G64_BK, vb);
    }
#pragma unroll
    for (int ks = 0; ks < G64_BK; ks += 4) {
      const int kk = ks + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[buf][kk][wr * 64 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[buf][kk][wc * 64 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + wr * 64 + i * 16 + (lane >> 4) + 4 * r;
        const int64_t n = n0 + wc * 64 + j * 16 + (lane & 15);
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

// per-class column sums of fp64 rows (sequential in perm order, as class_mean_kernel)
__global__ void class_sum_kernel(const double* F, int64_t D, int64_t ldf, const int64_t* perm, const int64_t* offsets,
                                 double* sums) {
  const int64_t c = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  double acc = 0;
  for (int64_t r = offsets[c]; r < offsets[c + 1]; ++r) acc += F[perm[r] * ldf + j];
  sums[c * D + j] = acc;
}

// means / Mc / Mc_n of class_mean_kernel from class sums and counts (a sharded set's all-reduced pieces)
__global__ void class_between_kernel(const double* sums, const double* counts, int64_t D, const double* total_mean,
                                     double* means, double* Mc, double* Mc_n) {
  const int64_t c = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  const double cnt = counts[c];
  const double mu = cnt > 0 ? sums[c * D + j] / cnt : 0.0;
  means[c * D + j] = mu;
  const double dm = mu - total_mean[j];
  Mc[c * D + j] = dm;
  Mc_n[c * D + j] = cnt * dm;
}

}  // namespace ofr

using namespace ofr;

extern "C" int ofr_class_sums_f64(void* stream, const double* F, int64_t D, int64_t ldf, const int64_t* perm,
                                  const int64_t* offsets, int64_t c, double* sums) {
  OFR_CHECK_ARG(D >= 1 && ldf >= D && c >= 1 && c < 65536, "ofr_class_sums_f64: bad sizes");
  OFR_CHECK_ARG(F && perm && offsets && sums, "ofr_class_sums_f64: null pointer");
  hipLaunchKernelGGL(class_sum_kernel, dim3((unsigned)cdiv(D, 256), (unsigned)c), dim3(256), 0, (hipStream_t)stream, F,
                     D, ldf, perm, offsets, sums);
  OFR_LAUNCH_CHECK("class_sum_kernel");
  return OFR_OK;
}

extern "C" int ofr_class_between_f64(void* stream, const double* sums, const double* counts, int64_t c, int64_t D,
                                     const double* total_mean, double* means, double* Mc, double* Mc_n) {
  OFR_CHECK_ARG(D >= 1 && c >= 1 && c < 65536, "ofr_class_between_f64: bad sizes");
  OFR_CHECK_ARG(sums && counts && total_mean && means && Mc && Mc_n, "ofr_class_between_f64: null pointer");
  hipLaunchKernelGGL(class_between_kernel, dim3((unsigned)cdiv(D, 256), (unsigned)c), dim3(256), 0,
                     (hipStream_t)stream, sums, counts, D, total_mean, means, Mc, Mc_n);
  OFR_LAUNCH_CHECK("class_between_kernel");
  return OFR_OK;
}

extern "C" int ofr_class_sub_f64(void* stream, const double* F, int64_t N, int64_t D, int64_t ldf, const int64_t* perm,
                                 const int64_t* offsets, int64_t c, const double* means, double* Fc) {
  OFR_CHECK_ARG(N >= 0 && D >= 1 && ldf >= D && c >= 1 && c < 65536, "ofr_class_sub_f64: bad sizes");
  if (N == 0) return OFR_OK;
  OFR_CHECK_ARG(F && perm && offsets && means && Fc, "ofr_class_sub_f64: null pointer");
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(D, 256), 64);
  for (int64_t done = 0; done < N; done += 65535) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(class_center_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream, F, done, D,
                       ldf, perm, offsets, c, means, Fc);
    OFR_LAUNCH_CHECK("class_center_kernel");
  }
  return OFR_OK;
}

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
