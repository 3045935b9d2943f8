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
//   * x - 128 is an int8, so v_mfma_i32_16x16x64_i8 (the wide engine, ofr_i8w_tile.h) accumulates
//     sum_i (x_i - 128) q_s[i][j] exactly in int32 (|sum| < 2^29);
//   * the epilogue combines the four int32 sums and the exact offset
//     128 * sum_i W[i][j] in fp64 without rounding (<= 50 significant bits),
//     so  y_j = s_j (t_j + K_j)  is the exact value of  x . Wq[:, j];  the
//     optional shift is subtracted in fp64 and the result rounded ONCE to the
//     output type (fp32 for the device search, fp64 for the host API).
// The int8 path runs at 2x the bf16 MFMA rate, i.e. 4 slices cost half of one
// bf16 pass and 1/8 of the fp32 MFMA projection.
//
// Layouts: Aq [ceil(d/64)*256][ldk] int8, ldk % 128 == 0, ldk >= round_up(D, 128);
// the rows of feature block jb = j/32 are jb*128 + s*32 + j%32 (the four slices
// of 32 features are four 32-row blocks).  The product runs on the wide int8
// engine (ofr_i8w_tile.h): 384 slice rows (3 feature blocks x 4 slices) by 256
// images per tile, both operands by LDS-DMA (the images as raw uint8 rows; the
// fragments become x - 128 by an XOR with 0x80 after the LDS read); B <= 4 faces
// take a split-K GEMV over the slices instead (same integers, same epilogue).
#include <string.h>

#include <atomic>

#include "ofr_i8_tile.h"
#include "ofr_i8w_tile.h"

namespace ofr {
namespace q8 {

constexpr int GROUP_F = 4;   // feature tiles per tile group (i8t::tile_coords)
// the engine's rings, then the epilogue's 32 KiB per wave (project_w_body)
constexpr int PROJ_LDS = i8w::LDS_BYTES > 4 * 32768 ? i8w::LDS_BYTES : 4 * 32768;

struct Args {
  const uint8_t* X;
  int64_t B, D, ldx;
  const int8_t* Aq;
  int64_t ldk, arows;
  const double* scale;
  const double* K;
  const double* shift;
  int64_t d;
  void* Y;
  int64_t ldy;
  int y_f64;
  int nk;
  int64_t ntf, ntb, gg;
  int64_t t0;   // first tile of this launch (ofr_project_u8_exact_range)
};

// The wide engine (ofr_i8w_tile.h, round 3): 384 slice rows (96 features x 4 slices) x 256 images, 4
// waves, each all 384 rows x 64 images, so a feature's four slices meet in one wave.  Tile ft covers
// projection blocks jb = 3 ft .. 3 ft + 2 (rows jb*128 + s*32 + j%32); element reg of acc[i][c] of lane
// l: row 16 i + 4 (l / 16) + reg = block i / 8, slice (i % 8) / 2, feature (i % 2) * 16 + 4 (l / 16) + reg
// of the block; image 64 W + 16 c + l % 16.  The epilogue combines the four slices exactly as
// project_epilogue (the same fp64 operations in the same order: identical results).
template <int W, bool REG>
__device__ __forceinline__ void project_w_body(const Args& p, int64_t ft, int64_t b0) {
  i8w::i32x4 acc[i8w::NA][i8w::NB];
  i8w::Feed f;
  i8w::feed_init(f, p.Aq, p.ldk, p.arows, ft * i8w::TA, p.X, p.ldx, p.B, b0);
  i8w::mainloop<W, REG>(f, p.nk, acc);
  const int lane = threadIdx.x & 63, l16 = lane & 15, g = lane >> 4;
  // Epilogue through the wave's own 32 KiB of LDS (free after the main loop's last barrier): per
  // projection block, its 8 x 4 accumulators are stored as they are (ds_write takes AGPR data) and read
  // back one feature group at a time.  Converted straight from the registers, the compiler moved the
  // AGPR accumulators into VGPRs at the loop exit and spilled 95 of them to scratch right behind the
  // last asm MFMAs (whose results the hazard recognizer does not track); now no accumulator is spilled
  // (tests/test_spill_guard.py).  The "memory" clobber keeps the reads from being forwarded from the
  // stores.  Same fp64 operations in the same order as before: identical results.
  OFR_LDS i8w::i32x4* stash = (OFR_LDS i8w::i32x4*)(uintptr_t)(W * 32768);
  // features outer (their scale / K / shift loaded once), the wave's 4 image blocks inner
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int jbl = (jj + 2) % 3;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < i8w::NB; ++c) stash[(r * 4 + c) * 64 + lane] = acc[jbl * 8 + r][c];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t j0 = (ft * 3 + jbl) * 32 + h * 16 + 4 * g;
      double sj[4], kj[4], hj[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool ok = j0 + e < p.d;
        sj[e] = ok ? p.scale[j0 + e] : 0.0;
        kj[e] = ok ? p.K[j0 + e] : 0.0;
        hj[e] = ok && p.shift ? p.shift[j0 + e] : 0.0;
      }
#pragma unroll
      for (int c = 0; c < i8w::NB; ++c) {
        const int64_t b = b0 + W * 64 + c * 16 + l16;
        if (b >= p.B) continue;
        double v[4];
        const i8w::i32x4 s0 = stash[(h * 4 + c) * 64 + lane], s1 = stash[((h + 2) * 4 + c) * 64 + lane];
        const i8w::i32x4 s2 = stash[((h + 4) * 4 + c) * 64 + lane], s3 = stash[((h + 6) * 4 + c) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          double tv = (double)s0[e];
          tv += (double)s1[e] * 0x1p-7;
          tv += (double)s2[e] * 0x1p-14;
          tv += (double)s3[e] * 0x1p-21;
          double y = sj[e] * (tv + kj[e]);   // exact: x . Wq[:, j]
          if (p.shift) y -= hj[e];
          v[e] = j0 + e < p.d ? y : 0.0;
        }
        if (p.y_f64) {
          double* yr = (double*)p.Y + b * p.ldy;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (j0 + e < p.d) yr[j0 + e] = v[e];
        } else {
          float* yr = (float*)p.Y + b * p.ldy;
          if (j0 + 4 <= p.d && (((uintptr_t)(yr + j0)) & 15) == 0) {
            f32x4 o;
            o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
            *reinterpret_cast<f32x4*>(yr + j0) = o;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (j0 + e < p.d) yr[j0 + e] = (float)v[e];
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("" ::: "memory");
  }
}

// REG: the engine's register-staged stage copies (i8w::mainloop, OFR_PROJ_STAGE=reg) instead of LDS-DMA
template <bool REG>
__global__ void __launch_bounds__(i8w::NT, 1) project_q8w_kernel(Args p) {
  const int64_t t = p.t0 + i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t ft, bt;
  i8t::tile_coords(t, p.gg, p.ntf, p.ntb, ft, bt);
  const int64_t b0 = bt * i8w::TB;
  switch (__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))) {   // the wave's role, compile time below
    case 0: project_w_body<0, REG>(p, ft, b0); break;
    case 1: project_w_body<1, REG>(p, ft, b0); break;
    case 2: project_w_body<2, REG>(p, ft, b0); break;
    default: project_w_body<3, REG>(p, ft, b0); break;
  }
}

// ---- a few faces (B <= 4, the recognizers' one face per call): split-K GEMV ------------------
// The 256-row MFMA tile engine leaves most of the chip idle for one face (ceil(d/64) = 157
// workgroups at d = 9,999, each streaming 2.6 MB of slices).  Here workgroup (jb, ks) streams the
// 128 slice rows of 32-feature block jb over the ks-th of GEMV_KSPLIT K ranges: wave s = slice s,
// lane l the 16-byte column chunks l, l + 64, ...; per chunk the faces' bytes (x - 128 by XOR 0x80)
// are loaded once and dotted (v_dot4_i32_i8) with the chunk of each of the wave's 32 rows, so a
// wave-instruction loads 1 KiB of one row.  The int32 partial sums (exact) are reduced over the
// wave and added atomically into part [NB][arows]; gemv_finalize_kernel combines the four slices
// exactly as project_q8_kernel's epilogue (same operations, same order: identical results).
constexpr int GEMV_KSPLIT = 4;

template <int NB>
__global__ void __launch_bounds__(256) project_gemv_kernel(const uint8_t* X, int64_t ldx, int64_t D, const int8_t* Aq,
                                                           int64_t ldk, int64_t arows, int* part) {
  const int64_t jb = blockIdx.x / GEMV_KSPLIT;
  const int ks = (int)(blockIdx.x % GEMV_KSPLIT);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row0 = jb * 128 + wave * 32;
  const int64_t nch = (D + 15) / 16;
  const int64_t per = (nch + GEMV_KSPLIT - 1) / GEMV_KSPLIT;
  const int64_t c0 = ks * per, c1 = c0 + per < nch ? c0 + per : nch;
  int acc[32][NB];
#pragma unroll
  for (int r = 0; r < 32; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[r][b] = 0;
  for (int64_t c = c0 + lane; c < c1; c += 64) {
    uint4 xv[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const uint4 v = *reinterpret_cast<const uint4*>(X + b * ldx + c * 16);
      xv[b] = make_uint4(v.x ^ 0x80808080u, v.y ^ 0x80808080u, v.z ^ 0x80808080u, v.w ^ 0x80808080u);
    }
    // the group's row chunks are all loaded before any is used: RG loads in flight per lane
    constexpr int RG = NB == 1 ? 32 : 16;
#pragma unroll
    for (int r0 = 0; r0 < 32; r0 += RG) {
      uint4 a[RG];
#pragma unroll
      for (int r = 0; r < RG; ++r) a[r] = *reinterpret_cast<const uint4*>(Aq + (row0 + r0 + r) * ldk + c * 16);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < RG; ++r)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
          int t = acc[r0 + r][b];
          t = __builtin_amdgcn_sdot4((int)a[r].x, (int)xv[b].x, t, false);
          t = __builtin_amdgcn_sdot4((int)a[r].y, (int)xv[b].y, t, false);
          t = __builtin_amdgcn_sdot4((int)a[r].z, (int)xv[b].z, t, false);
          t = __builtin_amdgcn_sdot4((int)a[r].w, (int)xv[b].w, t, false);
          acc[r0 + r][b] = t;
        }
    }
  }
#pragma unroll
  for (int r = 0; r < 32; ++r)
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      int v = acc[r][b];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      if (lane == 0) atomicAdd(part + b * arows + row0 + r, v);
    }
}

__global__ void gemv_finalize_kernel(const int* part, int64_t arows, int64_t B, const double* scale, const double* K,
                                     const double* shift, int64_t d, void* Y, int64_t ldy, int y_f64) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * d) return;
  const int64_t b = t / d, j = t - b * d;
  const int* pr = part + b * arows + (j >> 5) * 128 + (j & 31);
  double tv = (double)pr[0];
  tv += (double)pr[32] * 0x1p-7;
  tv += (double)pr[64] * 0x1p-14;
  tv += (double)pr[96] * 0x1p-21;
  double y = scale[j] * (tv + K[j]);   // exact: x . Wq[:, j]
  if (shift) y -= shift[j];
  if (y_f64) ((double*)Y)[b * ldy + j] = y;
  else ((float*)Y)[b * ldy + j] = (float)y;
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
  return (size_t)(cdiv(d, 64) * 256) * (size_t)round_up(D, 128);
}

extern "C" int ofr_qproj_prepare(void* stream, int dtype, const void* Wt, int64_t d, int64_t D, int64_t ldw, int8_t* Aq,
                                 int64_t ldk, double* scale, double* K) {
  OFR_CHECK_ARG(dtype == OFR_DT_F32 || dtype == OFR_DT_F64, "ofr_qproj_prepare: dtype must be F32 or F64");
  OFR_CHECK_ARG(d >= 1 && D >= 1 && ldw >= D && ldk >= round_up(D, 128) && ldk % 128 == 0,
                "ofr_qproj_prepare: bad sizes (ldk must be a multiple of 128 >= round_up(D,128))");
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

// OFR_PROJ_GEMV=0 keeps B <= 4 on the tile engine (for comparisons)
static bool getenv_flag_gemv() {
  static const bool f = [] {
    const char* e = getenv("OFR_PROJ_GEMV");
    return !(e && atoi(e) == 0);
  }();
  return f;
}

// OFR_PROJ_STAGE: "reg" (register-staged stage copies) or "dma" (LDS-DMA); read once
static bool proj_stage_reg() {
  static const bool f = [] {
    const char* e = getenv("OFR_PROJ_STAGE");
    return e && strcmp(e, "reg") == 0;
  }();
  return f;
}

static int project_u8_exact(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx, const int8_t* Aq,
                            int64_t ldk, const double* scale, const double* K, int64_t d, const double* shift, void* Y,
                            int64_t ldy, int y_dtype, int64_t t0, int64_t t1) {
  OFR_CHECK_ARG(B >= 0 && D >= 1 && d >= 1, "ofr_project_u8_exact: bad sizes");
  OFR_CHECK_ARG(y_dtype == OFR_DT_F32 || y_dtype == OFR_DT_F64, "ofr_project_u8_exact: y_dtype must be F32 or F64");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(X && Aq && scale && K && Y, "ofr_project_u8_exact: null pointer");
  OFR_CHECK_ARG(ldx >= D && ldx % 16 == 0 && ((uintptr_t)X % 16) == 0, "ofr_project_u8_exact: X rows must be 16-byte aligned, ldx >= D");
  OFR_CHECK_ARG(ldk >= round_up(D, 128) && ldk % 128 == 0 && ((uintptr_t)Aq % 16) == 0,
                "ofr_project_u8_exact: bad Aq layout");
  OFR_CHECK_ARG(ldy >= d, "ofr_project_u8_exact: ldy < d");
  static std::atomic<bool> attr_done{false};
  if (!attr_done.load(std::memory_order_acquire)) {
    hipError_t e = hipFuncSetAttribute((const void*)q8::project_q8w_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, q8::PROJ_LDS);
    if (e == hipSuccess)
      e = hipFuncSetAttribute((const void*)q8::project_q8w_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              q8::PROJ_LDS);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(project_q8w)");
    attr_done.store(true, std::memory_order_release);
  }
  if (B <= 4 && getenv_flag_gemv()) {
    OFR_CHECK_ARG(t0 == 0 && t1 < 0, "ofr_project_u8_exact_range: B <= 4 takes the GEMV path (no tiles)");
    hipStream_t st = (hipStream_t)stream;
    const int64_t arows = cdiv(d, 64) * 256;
    int* part = nullptr;
    hipError_t e = hipMallocAsync((void**)&part, (size_t)B * arows * 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(part, 0, (size_t)B * arows * 4, st);
    if (e != hipSuccess) return hip_status(e, "ofr_project_u8_exact: partial sums");
    const unsigned grid = (unsigned)(cdiv(d, 32) * q8::GEMV_KSPLIT);
    switch (B) {
      case 1: hipLaunchKernelGGL(q8::project_gemv_kernel<1>, dim3(grid), dim3(256), 0, st, X, ldx, D, Aq, ldk, arows, part); break;
      case 2: hipLaunchKernelGGL(q8::project_gemv_kernel<2>, dim3(grid), dim3(256), 0, st, X, ldx, D, Aq, ldk, arows, part); break;
      case 3: hipLaunchKernelGGL(q8::project_gemv_kernel<3>, dim3(grid), dim3(256), 0, st, X, ldx, D, Aq, ldk, arows, part); break;
      default: hipLaunchKernelGGL(q8::project_gemv_kernel<4>, dim3(grid), dim3(256), 0, st, X, ldx, D, Aq, ldk, arows, part); break;
    }
    OFR_LAUNCH_CHECK("project_gemv_kernel");
    hipLaunchKernelGGL(q8::gemv_finalize_kernel, dim3((unsigned)cdiv(B * d, 256)), dim3(256), 0, st, part, arows, B,
                       scale, K, shift, d, Y, ldy, (int)(y_dtype == OFR_DT_F64));
    OFR_LAUNCH_CHECK("gemv_finalize_kernel");
    e = hipFreeAsync(part, st);
    return e == hipSuccess ? OFR_OK : hip_status(e, "ofr_project_u8_exact: hipFreeAsync");
  }
  q8::Args p;
  p.X = X; p.B = B; p.D = D; p.ldx = ldx; p.Aq = Aq; p.ldk = ldk; p.scale = scale; p.K = K; p.shift = shift;
  p.d = d; p.Y = Y; p.ldy = ldy; p.y_f64 = y_dtype == OFR_DT_F64;
  p.ntf = cdiv(d, 64);
  p.arows = p.ntf * 256;
  p.gg = p.ntf < q8::GROUP_F ? p.ntf : q8::GROUP_F;
  // the wide engine: tiles of 384 slice rows (3 projection blocks) x 256 images; its panels are
  // addressed with 32-bit buffer offsets
  OFR_CHECK_ARG((int64_t)i8w::TA * ldk < 0x7fffffffLL && (int64_t)i8w::TB * ldx < 0x7fffffffLL,
                "ofr_project_u8_exact: rows too long for the wide engine");
  p.ntf = cdiv(p.arows, i8w::TA);
  p.gg = p.ntf < q8::GROUP_F ? p.ntf : q8::GROUP_F;
  p.nk = (int)cdiv(D, i8w::BK);
  p.ntb = cdiv(B, i8w::TB);
  OFR_CHECK_ARG(p.ntf * p.ntb < 0x7fffffffLL, "ofr_project_u8_exact: grid too large");
  if (t1 < 0) t1 = p.ntf * p.ntb;
  OFR_CHECK_ARG(t0 >= 0 && t0 <= t1 && t1 <= p.ntf * p.ntb, "ofr_project_u8_exact_range: tiles out of range");
  if (t0 == t1) return OFR_OK;
  p.t0 = t0;
  if (proj_stage_reg())
    hipLaunchKernelGGL(q8::project_q8w_kernel<true>, dim3((unsigned)(t1 - t0)), dim3(i8w::NT), q8::PROJ_LDS,
                       (hipStream_t)stream, p);
  else
    hipLaunchKernelGGL(q8::project_q8w_kernel<false>, dim3((unsigned)(t1 - t0)), dim3(i8w::NT), q8::PROJ_LDS,
                       (hipStream_t)stream, p);
  OFR_LAUNCH_CHECK("project_q8w_kernel");
  return OFR_OK;
}

extern "C" int ofr_project_u8_exact(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx, const int8_t* Aq,
                                    int64_t ldk, const double* scale, const double* K, int64_t d, const double* shift,
                                    void* Y, int64_t ldy, int y_dtype) {
  return project_u8_exact(stream, X, B, D, ldx, Aq, ldk, scale, K, d, shift, Y, ldy, y_dtype, 0, -1);
}

// The launch in two tile ranges (round 6): the tiles are dealt to the CUs in rounds of one tile per CU, so a
// caller can run the full rounds and the last, partial round as two launches and put other work beside the
// second (the bench's merge_at "tail").  Same tiles, same integers: identical outputs.
extern "C" int64_t ofr_project_u8_exact_tiles(int64_t B, int64_t d) {
  if (B <= 0 || d <= 0) return 0;
  if (B <= 4 && getenv_flag_gemv()) return 0;
  return cdiv(cdiv(d, 64) * 256, i8w::TA) * cdiv(B, i8w::TB);
}

extern "C" int ofr_project_u8_exact_range(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx,
                                          const int8_t* Aq, int64_t ldk, const double* scale, const double* K,
                                          int64_t d, const double* shift, void* Y, int64_t ldy, int y_dtype,
                                          int64_t t0, int64_t t1) {
  OFR_CHECK_ARG(t1 >= 0, "ofr_project_u8_exact_range: t1 < 0");
  return project_u8_exact(stream, X, B, D, ldx, Aq, ldk, scale, K, d, shift, Y, ldy, y_dtype, t0, t1);
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
