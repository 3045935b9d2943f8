// Batched projection Y = X . W - shift on gfx950 (fp32 MFMA tile engine).
//
// Replaces Fisherfaces.project (reference feature.py:241-242, np.dot(W.T, x),
// no mean subtraction), PCA.project (feature.py:114-116, shift = P^T mu),
// LDA.project (feature.py:184-185) and the per-sample projection loops of
// PCA/LDA/Fisherfaces.compute (feature.py:104-108, 178-182, 231-235).
//
// Tile: 256 output features (rows of W^T, "A") x 256 images ("B").  A is
// fp32 W^T staged by LDS-DMA; B is the uint8 image batch staged through
// registers and widened to fp32 on the LDS write (or fp32 via LDS-DMA).
#include "ofr_gemm_tile.h"

namespace ofr {

struct ProjArgs {
  const float* Wt;
  int64_t d, ldw;
  const void* X;
  int64_t B, D, ldx;
  const float* shift;
  float* Y;
  int64_t ldy;
  int nk;
  int64_t ntf, ntb;  // feature tiles, image tiles
};

template <bool U8>
__global__ void __launch_bounds__(256, 1) project_kernel(ProjArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = tile::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t ft = t / p.ntb;
  const int64_t bt = t % p.ntb;
  const int64_t f0 = ft * tile::TM, b0 = bt * tile::TN;
  tile::LoaderF32 la{p.Wt, p.ldw, p.d, f0};
  f32x16 acc[4][4];
  if constexpr (U8) {
    tile::LoaderU8 lb{(const uint8_t*)p.X, p.ldx, p.B, b0, p.D, {}};
    tile::mainloop(smem, la, lb, p.nk, acc);
  } else {
    tile::LoaderF32 lb{(const float*)p.X, p.ldx, p.B, b0};
    tile::mainloop(smem, la, lb, p.nk, acc);
  }
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1;
  const int h = lane >> 5;
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    const int64_t b = b0 + wc * 128 + ct * 32 + (lane & 31);
    if (b >= p.B) continue;
    float* yrow = p.Y + b * p.ldy;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int64_t j = f0 + wr * 128 + rt * 32 + 8 * g + 4 * h;  // 4 consecutive features
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float s = (p.shift && j + e < p.d) ? p.shift[j + e] : 0.f;
          v[e] = acc[rt][ct][4 * g + e] - s;
        }
        if (j + 4 <= p.d && ((uintptr_t)(yrow + j) & 15) == 0) {
          *reinterpret_cast<f32x4*>(yrow + j) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (j + e < p.d) yrow[j + e] = v[e];
        }
      }
  }
}

template <bool U8>
static int launch_project(void* stream, const void* X, int64_t B, int64_t D, int64_t ldx, const float* Wt, int64_t d,
                          int64_t ldw, const float* shift, float* Y, int64_t ldy) {
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)project_kernel<U8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       tile::LDS_BYTES);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(project)");
    attr_done = true;
  }
  ProjArgs p;
  p.Wt = Wt; p.d = d; p.ldw = ldw; p.X = X; p.B = B; p.D = D; p.ldx = ldx;
  p.shift = shift; p.Y = Y; p.ldy = ldy;
  p.nk = (int)cdiv(D, tile::BK);
  p.ntf = cdiv(d, tile::TM);
  p.ntb = cdiv(B, tile::TN);
  OFR_CHECK_ARG(p.ntf * p.ntb < 0x7fffffffLL, "ofr_project: grid too large");
  hipLaunchKernelGGL((project_kernel<U8>), dim3((unsigned)(p.ntf * p.ntb)), dim3(256), tile::LDS_BYTES,
                     (hipStream_t)stream, p);
  OFR_LAUNCH_CHECK("project_kernel");
  return OFR_OK;
}

}  // namespace ofr

using namespace ofr;

extern "C" int ofr_project_u8(void* stream, const uint8_t* X, int64_t B, int64_t D, int64_t ldx, const float* Wt,
                              int64_t d, int64_t ldw, const float* shift, float* Y, int64_t ldy) {
  OFR_CHECK_ARG(B >= 0 && D >= 1 && d >= 1, "ofr_project_u8: bad sizes");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(X && Wt && Y, "ofr_project_u8: null pointer");
  OFR_CHECK_ARG(ldx >= D && ldx % 16 == 0, "ofr_project_u8: ldx must be a multiple of 16 >= D");
  OFR_CHECK_ARG(ldw % 32 == 0 && ldw >= round_up(D, 32), "ofr_project_u8: ldw must be a multiple of 32 >= round_up(D,32)");
  OFR_CHECK_ARG(ldy >= d, "ofr_project_u8: ldy < d");
  OFR_CHECK_ARG(((uintptr_t)X % 16) == 0 && ((uintptr_t)Wt % 16) == 0, "ofr_project_u8: X and Wt must be 16-byte aligned");
  return launch_project<true>(stream, X, B, D, ldx, Wt, d, ldw, shift, Y, ldy);
}

extern "C" int ofr_project_f32(void* stream, const float* X, int64_t B, int64_t D, int64_t ldx, const float* Wt,
                               int64_t d, int64_t ldw, const float* shift, float* Y, int64_t ldy) {
  OFR_CHECK_ARG(B >= 0 && D >= 1 && d >= 1, "ofr_project_f32: bad sizes");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(X && Wt && Y, "ofr_project_f32: null pointer");
  OFR_CHECK_ARG(ldx % 32 == 0 && ldx >= round_up(D, 32), "ofr_project_f32: ldx must be a multiple of 32 >= round_up(D,32)");
  OFR_CHECK_ARG(ldw % 32 == 0 && ldw >= round_up(D, 32), "ofr_project_f32: ldw must be a multiple of 32 >= round_up(D,32)");
  OFR_CHECK_ARG(ldy >= d, "ofr_project_f32: ldy < d");
  OFR_CHECK_ARG(((uintptr_t)X % 16) == 0 && ((uintptr_t)Wt % 16) == 0, "ofr_project_f32: X and Wt must be 16-byte aligned");
  return launch_project<false>(stream, X, B, D, ldx, Wt, d, ldw, shift, Y, ldy);
}
