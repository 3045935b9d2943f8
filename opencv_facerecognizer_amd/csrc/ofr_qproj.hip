// Exact projection Y = X . W - shift on the int8 MFMA (gfx950).
//
// Replaces Fisherfaces.project (reference feature.py:241-242, np.dot(W.T, x)),
// PCA.project (:114-116) and LDA.project (:184-185) for uint8 faces.
//
// Why integers: a face has a large common component (Fisherfaces features of
// the bundled model are ~2300 in norm while neighbour distances are ~2), so
// an fp32-accumulated W^T x loses ~1e-3 of the DISTANCE.  Here every product
// and every sum is exact:
//   * W (fp32 or fp64) is split per output feature j into four int8 slices
//     with a power-of-two scale s_j:  W[i][j] = s_j (q1 + q2/2^7 + q3/2^14 + q4/2^21)
//     (exact for every fp32 element within 2^4 of the column maximum; the
//     rest is truncated at 2^-28 of the column maximum);
//   * x - 128 is an int8, so v_mfma_i32_32x32x32_i8 accumulates
//     sum_i (x_i - 128) q_s[i][j] exactly in int32 (|sum| < 2^29);
//   * the epilogue combines the four int32 sums and the exact offset
//     128 * sum_i W[i][j] in fp64 without rounding (<= 50 significant bits),
//     so  y_j = s_j (t_j + K_j)  is the exact value of  x . Wq[:, j];  the
//     optional shift is subtracted in fp64 and the result rounded ONCE to the
//     output type (fp32 for the device search, fp64 for the host API).
// The int8 path runs at 2x the bf16 MFMA rate, i.e. 4 slices cost half of one
// bf16 pass and 1/8 of the fp32 MFMA projection.
//
// Layouts: Aq [ceil(d/64)*256][ldk] int8, ldk = round_up(D, 64); the rows of
// feature block jb = j/32 are jb*128 + s*32 + j%32 (the four slices of 32
// features are the four 32-row MFMA blocks of one wave).  A 256x256 tile =
// 64 features x 4 slices by 256 images; 4 waves (2x2), each 128x128 =
// 4 slices x 4 image blocks, int32 accumulators.  LDS: [256][64 B] panels,
// 16-B chunks XOR-swizzled by ((row>>2)&3), A by LDS-DMA, images through
// registers (x ^ 0x80 = x - 128 as int8), two stages.
#include "ofr_common.h"

namespace ofr {
namespace q8 {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int TM = 256, TN = 256, BK = 64;
constexpr int PANEL = 256 * BK;          // 16 KiB
constexpr int STAGE = 2 * PANEL;         // A + B
constexpr int LDS_BYTES = 2 * STAGE;     // 64 KiB

__device__ __forceinline__ int off(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4); }

struct Args {
  const uint8_t* X;
  int64_t B, D, ldx;
  const int8_t* Aq;
  int64_t ldk;
  const double* scale;
  const double* K;
  const double* shift;
  int64_t d;
  void* Y;
  int64_t ldy;
  int y_f64;
  int nk;
  int64_t ntf, ntb;
};

__device__ __forceinline__ void issue_a(const Args& p, char* panel, int64_t arow0, int kt) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int ins = wave * 4 + t;        // 16 wave-instructions x 16 rows
    const int row = ins * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    const int8_t* src = p.Aq + (arow0 + row) * p.ldk + (int64_t)kt * BK + chunk * 16;
    __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)src, (OFR_LDS void*)(panel + ins * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ void load_b(const Args& p, int64_t b0, int kt, uint4 (&v)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int q = threadIdx.x + 256 * s;
    const int row = q >> 2, c = q & 3;
    int64_t b = b0 + row;
    b = b < p.B ? b : p.B - 1;
    const int64_t k = (int64_t)kt * BK + c * 16;
    if (k < p.D) {
      uint4 x = *reinterpret_cast<const uint4*>(p.X + b * p.ldx + k);
      x.x ^= 0x80808080u; x.y ^= 0x80808080u; x.z ^= 0x80808080u; x.w ^= 0x80808080u;
      v[s] = x;    // bytes >= D meet the zero pad of Aq
    } else {
      v[s] = make_uint4(0, 0, 0, 0);
    }
  }
}

__device__ __forceinline__ void store_b(char* panel, const uint4 (&v)[4]) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int q = threadIdx.x + 256 * s;
    *reinterpret_cast<uint4*>(panel + off(q >> 2, q & 3)) = v[s];
  }
}

__global__ void __launch_bounds__(256, 1) project_q8_kernel(Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // consecutive blocks share the weight tile: the 256-row W-slice panel is fetched from HBM once
  // (the image panels of a 4096-image batch, 41 MB, stay in the Infinity Cache)
  const int64_t t = blockIdx.x;
  const int64_t ft = t / p.ntb, bt = t % p.ntb;
  const int64_t f0 = ft * 64, b0 = bt * TN, arow0 = ft * TM;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;

  i32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;

  uint4 vb[4];
  issue_a(p, smem, arow0, 0);
  load_b(p, b0, 0, vb);
  store_b(smem + PANEL, vb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int kt = 0; kt < p.nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE;
    char* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    const bool more = kt + 1 < p.nk;
    if (more) {
      issue_a(p, nxt, arow0, kt + 1);
      load_b(p, b0, kt + 1, vb);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int chunk = 2 * ks + h;
      i32x4 a[4], b[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        a[s] = *reinterpret_cast<const i32x4*>(cur + off(wr * 128 + s * 32 + r32, chunk));
        b[s] = *reinterpret_cast<const i32x4*>(cur + PANEL + off(wc * 128 + s * 32 + r32, chunk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) store_b(nxt + PANEL, vb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // epilogue: rows (reg&3) + 8*(reg>>2) + 4*h of each 32-block are the same 32 features in all four slices
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int64_t b = b0 + wc * 128 + ct * 32 + r32;
    if (b >= p.B) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      double v[4];
      const int64_t j0 = f0 + wr * 32 + 8 * g + 4 * h;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * g + e;
        const int64_t j = j0 + e;
        double tv = (double)acc[0][ct][r];
        tv += (double)acc[1][ct][r] * 0x1p-7;
        tv += (double)acc[2][ct][r] * 0x1p-14;
        tv += (double)acc[3][ct][r] * 0x1p-21;
        if (j < p.d) {
          double y = p.scale[j] * (tv + p.K[j]);   // exact: x . Wq[:, j]
          if (p.shift) y -= p.shift[j];
          v[e] = y;
        } else {
          v[e] = 0.0;
        }
      }
      if (p.y_f64) {
        double* yr = (double*)p.Y + b * p.ldy;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (j0 + e < p.d) yr[j0 + e] = v[e];
      } else {
        float* yr = (float*)p.Y + b * p.ldy;
        if (j0 + 4 <= p.d && (((uintptr_t)(yr + j0)) & 15) == 0) {
          f32x4 f;
          f[0] = (float)v[0]; f[1] = (float)v[1]; f[2] = (float)v[2]; f[3] = (float)v[3];
          *reinterpret_cast<f32x4*>(yr + j0) = f;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (j0 + e < p.d) yr[j0 + e] = (float)v[e];
        }
      }
    }
  }
}

// ---- weight preparation: one block per output feature ----------------------------------
template <typename T>
__global__ void __launch_bounds__(256) prepare_kernel(const T* Wt, int64_t D, int64_t ldw, int8_t* Aq, int64_t ldk,
                                                      double* scale, double* Kout) {
  __shared__ double red[4];
  __shared__ long long isum[4][4];
  const int64_t j = blockIdx.x;
  const T* w = Wt + j * ldw;
  double mx = 0;
  for (int64_t i = threadIdx.x; i < D; i += blockDim.x) mx = fmax(mx, fabs((double)w[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  // power-of-two scale with max|w|/s in (63.5, 127]
  double s = 1.0;
  if (mx > 0) {
    int e;
    frexp(mx / 127.0, &e);          // mx/127 = m * 2^e, m in [0.5, 1)
    s = ldexp(1.0, e);
    if (mx / s > 127.0) s *= 2.0;
  }
  const int64_t jb = j >> 5, jr = j & 31;
  long long acc[4] = {0, 0, 0, 0};
  for (int64_t i = threadIdx.x; i < D; i += blockDim.x) {
    double r = (double)w[i] / s;    // exact (power of two)
    int q[4];
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      const double qi = rint(r);
      q[sl] = (int)qi;
      r = (r - qi) * 128.0;         // exact
    }
#pragma unroll
    for (int sl = 0; sl < 4; ++sl) {
      Aq[(jb * 128 + sl * 32 + jr) * ldk + i] = (int8_t)q[sl];
      acc[sl] += q[sl];
    }
  }
#pragma unroll
  for (int sl = 0; sl < 4; ++sl) {
    long long v = acc[sl];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) isum[wave][sl] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long S[4];
    for (int sl = 0; sl < 4; ++sl) S[sl] = isum[0][sl] + isum[1][sl] + isum[2][sl] + isum[3][sl];
    double tsum = (double)S[0];
    tsum += (double)S[1] * 0x1p-7;
    tsum += (double)S[2] * 0x1p-14;
    tsum += (double)S[3] * 0x1p-21;
    scale[j] = s;
    Kout[j] = 128.0 * tsum;           // sum_i 128 * Wq[i][j] / s  (x = (x-128) + 128)
  }
}

__global__ void center_round_kernel(const double* F, int64_t ldf, int64_t d, const double* shift, float* out,
                                    int64_t ldo) {
  const int64_t n = blockIdx.y;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
    out[n * ldo + j] = (float)(F[n * ldf + j] - (shift ? shift[j] : 0.0));
}

}  // namespace q8
}  // namespace ofr

using namespace ofr;

extern "C" size_t ofr_qproj_bytes(int64_t D, int64_t d) {
  return (size_t)(cdiv(d, 64) * 256) * (size_t)round_up(D, 64);
}

extern "C" int ofr_qproj_prepare(void* stream, int dtype, const void* Wt, int64_t d, int64_t D, int64_t ldw, int8_t* Aq,
                                 int64_t ldk, double* scale, double* K) {
  OFR_CHECK_ARG(dtype == OFR_DT_F32 || dtype == OFR_DT_F64, "ofr_qproj_prepare: dtype must be F32 or F64");
  OFR_CHECK_ARG(d >= 1 && D >= 1 && ldw >= D && ldk >= round_up(D, 64) && ldk % 64 == 0,
                "ofr_qproj_prepare: bad sizes (ldk must be a multiple of 64 >= round_up(D,64))");
  OFR_CHECK_ARG(Wt && Aq && scale && K && d < 0x7fffffffLL, "ofr_qproj_prepare: null pointer");
  hipStream_t st = (hipStream_t)stream;
  // the pad rows/columns of Aq must be zero: clear the whole operand first
  hipError_t e = hipMemsetAsync(Aq, 0, (size_t)(cdiv(d, 64) * 256) * ldk, st);
  if (e != hipSuccess) return hip_status(e, "hipMemsetAsync(Aq)");
  if (dtype == OFR_DT_F32)
    hipLaunchKernelGGL(q8::prepare_kernel<float>, dim3((unsigned)d), dim3(256), 0, st, (const float*)Wt, D, ldw, Aq, ldk,
                       scale, K);
  else
    hipLaunchKernelGGL(q8::prepare_kernel<double>, dim3((unsigned)d), dim3(256), 0, st, (const double*)Wt, D, ldw, Aq,
                       ldk, scale, K);
  OFR_LAUNCH_CHECK("qproj prepare_kernel");
  return OFR_OK;
}

extern "C" int ofr_project_u8_exact(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx, const int8_t* Aq,
                                    int64_t ldk, const double* scale, const double* K, int64_t d, const double* shift,
                                    void* Y, int64_t ldy, int y_dtype) {
  OFR_CHECK_ARG(B >= 0 && D >= 1 && d >= 1, "ofr_project_u8_exact: bad sizes");
  OFR_CHECK_ARG(y_dtype == OFR_DT_F32 || y_dtype == OFR_DT_F64, "ofr_project_u8_exact: y_dtype must be F32 or F64");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(X && Aq && scale && K && Y, "ofr_project_u8_exact: null pointer");
  OFR_CHECK_ARG(ldx >= D && ldx % 16 == 0 && ((uintptr_t)X % 16) == 0, "ofr_project_u8_exact: X rows must be 16-byte aligned, ldx >= D");
  OFR_CHECK_ARG(ldk >= round_up(D, 64) && ldk % 64 == 0 && ((uintptr_t)Aq % 16) == 0, "ofr_project_u8_exact: bad Aq layout");
  OFR_CHECK_ARG(ldy >= d, "ofr_project_u8_exact: ldy < d");
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)q8::project_q8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       q8::LDS_BYTES);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(project_q8)");
    attr_done = true;
  }
  q8::Args p;
  p.X = X; p.B = B; p.D = D; p.ldx = ldx; p.Aq = Aq; p.ldk = ldk; p.scale = scale; p.K = K; p.shift = shift;
  p.d = d; p.Y = Y; p.ldy = ldy; p.y_f64 = y_dtype == OFR_DT_F64;
  p.nk = (int)cdiv(D, q8::BK);
  p.ntf = cdiv(d, 64);
  p.ntb = cdiv(B, q8::TN);
  OFR_CHECK_ARG(p.ntf * p.ntb < 0x7fffffffLL, "ofr_project_u8_exact: grid too large");
  hipLaunchKernelGGL(q8::project_q8_kernel, dim3((unsigned)(p.ntf * p.ntb)), dim3(256), q8::LDS_BYTES,
                     (hipStream_t)stream, p);
  OFR_LAUNCH_CHECK("project_q8_kernel");
  return OFR_OK;
}

extern "C" int ofr_center_round_f64(void* stream, const double* F, int64_t N, int64_t d, int64_t ldf,
                                    const double* shift, float* out, int64_t ldo) {
  OFR_CHECK_ARG(N >= 0 && d >= 0 && ldf >= d && ldo >= d, "ofr_center_round_f64: bad sizes");
  if (N == 0 || d == 0) return OFR_OK;
  OFR_CHECK_ARG(F && out, "ofr_center_round_f64: null pointer");
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(d, 256), 64);
  for (int64_t done = 0; done < N; done += 65535) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(q8::center_round_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream,
                       F + done * ldf, ldf, d, shift, out + done * ldo, ldo);
    OFR_LAUNCH_CHECK("center_round_kernel");
  }
  return OFR_OK;
}
