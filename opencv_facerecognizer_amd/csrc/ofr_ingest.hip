// Face-tensor ingestion: (crop) + BGR->grey + resize of a ragged batch of images into the
// uint8 face rows the projection reads.
//
// Replaces, per image, cv2.imread(..., IMREAD_GRAYSCALE) + cv2.resize(im, size) (INTER_LINEAR)
// of TheTrainer.read_images (reference trainer/thetrainer.py:99-103) and the recognizers'
// face = img[y0:y1, x0:x1]; cv2.cvtColor(face, BGR2GRAY); cv2.resize(face, size, INTER_CUBIC)
// (bin/ocvf_recognizer.py:64-66, ocvf_recognizer_ros.py:113-115, ocvf_recognizer_rsb.py).
//
// Arithmetic = OpenCV's 8-bit fixed point (OpenCV 2.4.8, the python-opencv of README.md:44-48;
// absent here, restated in oracle/facerec_oracle.py cv_resize_u8 / cv_bgr2gray):
//   grey  = (1868 B + 9617 G + 4899 R + 2^13) >> 14
//   axis  : scale = 1 / (dst / src); f = (float)((i + 0.5) scale - 0.5); s = floor(f); f -= s;
//           weights w_k = rint(cbuf_k * 2048) (int16), cbuf = (1 - f, f) [linear] or
//           interpolateCubic(f), A = -0.75, in float [cubic]; taps clamped to the image;
//           linear COLUMNS past an edge use (2048, 0) at the edge pixel
//   pixel : H_r = sum_k S[row_r][tap_k] w_k (int32);  out = sat_u8((sum_r H_r beta_r + 2^21) >> 22)
//   same source and destination size: a copy (cv::resize's shortcut).
// One thread per output pixel computes its ksize rows of horizontal sums directly: the same
// integers as OpenCV's separable passes, so the result is bit-identical to the restatement.
// The float coefficient math must not be contracted into FMAs (Makefile: -ffp-contract=off).
//
// Work per output pixel: ksize^2 source bytes (x3 for BGR) read through L1/L2 and ksize^2 + ksize
// integer MACs -- a few MB per batch of 70 x 70 faces; HBM/launch-latency bound, no MFMA shape.
#include "ofr_common.h"

namespace ofr {
namespace ingest {

constexpr int COEF_BITS = 11;
constexpr int JOB_FIELDS = 7;   // offset, row bytes, x0, y0, w, h, channels

struct Axis {
  int s;       // first tap (before clamping)
  int w[4];    // weights
};

__device__ __forceinline__ int sat_s16(float v) {
  const float r = rintf(v);
  return r > 32767.f ? 32767 : (r < -32768.f ? -32768 : (int)r);
}

// one axis of resizeGeneric_ (LINEAR: 2 taps from s; CUBIC: 4 taps from s - 1)
template <int KS>
__device__ __forceinline__ Axis axis_coeffs(int i, int dsize, int ssize, bool is_x) {
  const double scale = 1.0 / ((double)dsize / (double)ssize);
  float f = (float)(((double)i + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  Axis a;
  if constexpr (KS == 2) {
    if (is_x && s < 0) {
      f = 0.f;
      s = 0;
    }
    if (is_x && s >= ssize - 1) {
      f = 0.f;
      s = ssize - 1;
    }
    a.s = s;
    a.w[0] = sat_s16((1.f - f) * 2048.f);
    a.w[1] = sat_s16(f * 2048.f);
    a.w[2] = a.w[3] = 0;
  } else {
    const float A = -0.75f, x = f;
    const float c0 = ((A * (x + 1.f) - 5.f * A) * (x + 1.f) + 8.f * A) * (x + 1.f) - 4.f * A;
    const float c1 = ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
    const float c2 = ((A + 2.f) * (1.f - x) - (A + 3.f)) * (1.f - x) * (1.f - x) + 1.f;
    const float c3 = 1.f - c0 - c1 - c2;
    a.s = s - 1;
    a.w[0] = sat_s16(c0 * 2048.f);
    a.w[1] = sat_s16(c1 * 2048.f);
    a.w[2] = sat_s16(c2 * 2048.f);
    a.w[3] = sat_s16(c3 * 2048.f);
  }
  return a;
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// grey value of pixel (x, y) of the crop (color.cpp RGB2Gray, BGR order, exact integers)
__device__ __forceinline__ int grey(const uint8_t* row0, int64_t ld, int ch, int x, int y) {
  const uint8_t* p = row0 + (int64_t)y * ld + (int64_t)x * ch;
  if (ch == 1) return p[0];
  return ((int)p[0] * 1868 + (int)p[1] * 9617 + (int)p[2] * 4899 + (1 << 13)) >> 14;
}

template <int KS>
__global__ void __launch_bounds__(256) resize_kernel(const uint8_t* src, const int64_t* jobs, int64_t bpj, int dh,
                                                     int dw, uint8_t* out) {
  const int64_t job = blockIdx.x / bpj;
  const int64_t pix = (blockIdx.x % bpj) * 256 + threadIdx.x;
  if (pix >= (int64_t)dh * dw) return;
  const int64_t* jb = jobs + job * JOB_FIELDS;
  const int64_t ld = jb[1];
  const int x0 = (int)jb[2], y0 = (int)jb[3], w = (int)jb[4], h = (int)jb[5], ch = (int)jb[6];
  const uint8_t* base = src + jb[0] + (int64_t)y0 * ld + (int64_t)x0 * ch;
  const int oy = (int)(pix / dw), ox = (int)(pix % dw);
  uint8_t v;
  if (w == dw && h == dh) {
    v = (uint8_t)grey(base, ld, ch, ox, oy);
  } else {
    const Axis ax = axis_coeffs<KS>(ox, dw, w, true);
    const Axis ay = axis_coeffs<KS>(oy, dh, h, false);
    int acc = 0;
#pragma unroll
    for (int r = 0; r < KS; ++r) {
      const int sy = clampi(ay.s + r, 0, h - 1);
      int hs = 0;
#pragma unroll
      for (int k = 0; k < KS; ++k) hs += grey(base, ld, ch, clampi(ax.s + k, 0, w - 1), sy) * ax.w[k];
      acc += hs * ay.w[r];
    }
    const int o = (acc + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS);
    v = (uint8_t)clampi(o, 0, 255);
  }
  out[job * (int64_t)dh * dw + pix] = v;
}

// One workgroup per face: the axis tables of the output grid are computed once (dw + dh entries,
// not per pixel), the crop is converted to grey once into LDS (when it fits GREY_CAP bytes), and
// every output pixel reads its KS x KS taps from LDS -- the same integers as resize_kernel (and
// OpenCV), a tenth of the work: no per-pixel fp64 coefficient math, no per-tap byte gathers and
// BGR conversions from global memory.  Crops larger than GREY_CAP read their taps as resize_kernel.
constexpr int GREY_CAP = 32 * 1024;
constexpr int MAX_SIDE = 1024;      // dh, dw <= MAX_SIDE for the per-face tables

template <int KS>
__global__ void __launch_bounds__(256) resize_face_kernel(const uint8_t* src, const int64_t* jobs, int dh, int dw,
                                                          uint8_t* out) {
  extern __shared__ __attribute__((aligned(16))) int tab[];   // [dw][1 + KS] x-table, [dh][1 + KS] y-table, grey
  int* xt = tab;
  int* yt = tab + dw * (1 + KS);
  uint8_t* gimg = reinterpret_cast<uint8_t*>(tab + (dw + dh) * (1 + KS));
  const int64_t job = blockIdx.x;
  const int64_t* jb = jobs + job * JOB_FIELDS;
  const int64_t ld = jb[1];
  const int x0 = (int)jb[2], y0 = (int)jb[3], w = (int)jb[4], h = (int)jb[5], ch = (int)jb[6];
  const uint8_t* base = src + jb[0] + (int64_t)y0 * ld + (int64_t)x0 * ch;
  uint8_t* o = out + job * (int64_t)dh * dw;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 columns x 4 rows, no divisions
  if (w == dw && h == dh) {   // cv::resize copies a same-size image
    for (int y = ty; y < dh; y += 4)
      for (int x = tx; x < dw; x += 64) o[y * dw + x] = (uint8_t)grey(base, ld, ch, x, y);
    return;
  }
  for (int i = threadIdx.x; i < dw + dh; i += blockDim.x) {
    const bool isx = i < dw;
    const Axis a = axis_coeffs<KS>(isx ? i : i - dw, isx ? dw : dh, isx ? w : h, isx);
    int* t = isx ? xt + i * (1 + KS) : yt + (i - dw) * (1 + KS);
    t[0] = a.s;
#pragma unroll
    for (int k = 0; k < KS; ++k) t[1 + k] = a.w[k];
  }
  const bool staged = (int64_t)w * h <= GREY_CAP;
  if (staged)
    for (int y = ty; y < h; y += 4)
      for (int x = tx; x < w; x += 64) gimg[y * w + x] = (uint8_t)grey(base, ld, ch, x, y);
  __syncthreads();
  for (int oy = ty; oy < dh; oy += 4) {
    const int* tyt = yt + oy * (1 + KS);
    int sy[KS];
#pragma unroll
    for (int r = 0; r < KS; ++r) sy[r] = clampi(tyt[0] + r, 0, h - 1);
    for (int ox = tx; ox < dw; ox += 64) {
      const int* txt = xt + ox * (1 + KS);
      int cx[KS];
#pragma unroll
      for (int k = 0; k < KS; ++k) cx[k] = clampi(txt[0] + k, 0, w - 1);
      int acc = 0;
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        int hs = 0;
        if (staged) {
          const uint8_t* row = gimg + sy[r] * w;
#pragma unroll
          for (int k = 0; k < KS; ++k) hs += (int)row[cx[k]] * txt[1 + k];
        } else {
#pragma unroll
          for (int k = 0; k < KS; ++k) hs += grey(base, ld, ch, cx[k], sy[r]) * txt[1 + k];
        }
        acc += hs * tyt[1 + r];
      }
      const int v = (acc + (1 << (2 * COEF_BITS - 1))) >> (2 * COEF_BITS);
      o[oy * dw + ox] = (uint8_t)clampi(v, 0, 255);
    }
  }
}

}  // namespace ingest
}  // namespace ofr

using namespace ofr;

extern "C" int ofr_ingest_faces(void* stream, const uint8_t* src, const int64_t* jobs, int64_t n, int dh, int dw,
                                int interp, uint8_t* out) {
  OFR_CHECK_ARG(n >= 0 && dh >= 1 && dw >= 1, "ofr_ingest_faces: bad sizes");
  OFR_CHECK_ARG(interp == 1 || interp == 2, "ofr_ingest_faces: interp must be 1 (INTER_LINEAR) or 2 (INTER_CUBIC)");
  if (n == 0) return OFR_OK;
  OFR_CHECK_ARG(src && jobs && out, "ofr_ingest_faces: null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (dh <= ingest::MAX_SIDE && dw <= ingest::MAX_SIDE && n < 0x7fffffffLL) {
    const int ks = interp == 1 ? 2 : 4;
    const size_t lds = (size_t)(dw + dh) * (1 + ks) * 4 + ingest::GREY_CAP;
    static bool attr[2] = {false, false};
    const void* fn = interp == 1 ? (const void*)ingest::resize_face_kernel<2> : (const void*)ingest::resize_face_kernel<4>;
    if (!attr[interp - 1]) {
      const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(
                                                   (size_t)2 * ingest::MAX_SIDE * 5 * 4 + ingest::GREY_CAP));
      if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(resize_face_kernel)");
      attr[interp - 1] = true;
    }
    if (interp == 1)
      hipLaunchKernelGGL(ingest::resize_face_kernel<2>, dim3((unsigned)n), dim3(256), lds, st, src, jobs, dh, dw, out);
    else
      hipLaunchKernelGGL(ingest::resize_face_kernel<4>, dim3((unsigned)n), dim3(256), lds, st, src, jobs, dh, dw, out);
    OFR_LAUNCH_CHECK("ingest resize_face_kernel");
    return OFR_OK;
  }
  const int64_t bpj = cdiv((int64_t)dh * dw, 256);
  OFR_CHECK_ARG(n * bpj < 0x7fffffffLL, "ofr_ingest_faces: batch too large for one launch");
  if (interp == 1)
    hipLaunchKernelGGL(ingest::resize_kernel<2>, dim3((unsigned)(n * bpj)), dim3(256), 0, st, src, jobs, bpj, dh, dw,
                       out);
  else
    hipLaunchKernelGGL(ingest::resize_kernel<4>, dim3((unsigned)(n * bpj)), dim3(256), 0, st, src, jobs, bpj, dh, dw,
                       out);
  OFR_LAUNCH_CHECK("ingest resize_kernel");
  return OFR_OK;
}
