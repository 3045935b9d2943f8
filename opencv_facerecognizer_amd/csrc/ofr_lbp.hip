// ExtendedLBP codes and per-cell histograms on gfx950 (bit-exact).
//
// Replaces ExtendedLBP.__call__ (reference lbp.py:80-130) and
// SpatialHistogram.spatially_enhanced_histogram (feature.py:286-302).
//
// Bit-exactness: the reference interpolates every neighbour in float64 with
// numpy array ops, i.e. per pixel and sample point i, in this order and
// without fused multiply-add:
//     N = w1*X[fy][fx];  N += w2*X[fy][cx];  N += w3*X[cy][fx];  N += w4*X[cy][cx]
// and sets bit i when N >= C (C = the uint8 centre pixel).  The weights come
// from np.sin/np.cos on the host (bits 4 and 6 of r=1,P=8 carry 2^-53 and
// 2^-52 round-off terms, so ties do NOT behave like integer LBP).  This file
// is compiled with -ffp-contract=off and the arithmetic below is written as
// separate fp64 multiplies and adds in the reference order.  A zero weight
// contributes an exact +0 (x >= 0), so zero terms are dropped on the host.
//
// Histograms: one workgroup per (image, band of cell rows); counters are u32
// LDS atomics, written out as 1/2/4-byte integers.  The reference's float
// histogram is count/(py*px) exactly (np.histogram(density=True)).
#include "ofr_common.h"

#pragma clang fp contract(off)

namespace ofr {

constexpr int MAXP = 32;

struct LbpGeom {
  int P;
  int H, W, dy, dx;   // image and code-image sizes
  int oy, ox;         // centre offset
  int nterm[MAXP];    // non-zero terms per point (1..4)
  int toff[MAXP][4];  // pixel offset (ty*W + tx) of each term, relative to the code pixel's block origin
  double tw[MAXP][4]; // weight of each term
};

__device__ __forceinline__ uint32_t lbp_code(const uint8_t* __restrict__ img, const LbpGeom& g, int y, int x) {
  const uint8_t* blk = img + (int64_t)y * g.W + x;  // block origin (top-left of the sampling block)
  const double C = (double)blk[g.oy * g.W + g.ox];
  uint32_t code = 0;
  for (int i = 0; i < g.P; ++i) {
    double N = g.tw[i][0] * (double)blk[g.toff[i][0]];
    for (int t = 1; t < g.nterm[i]; ++t) {
      const double prod = g.tw[i][t] * (double)blk[g.toff[i][t]];
      N = N + prod;
    }
    code |= (N >= C ? 1u : 0u) << i;
  }
  return code;
}

__global__ void elbp_codes_kernel(const uint8_t* __restrict__ imgs, int64_t n, LbpGeom g, uint32_t* __restrict__ codes) {
  const int64_t img = blockIdx.y;
  const uint8_t* im = imgs + img * (int64_t)g.H * g.W;
  uint32_t* out = codes + img * (int64_t)g.dy * g.dx;
  const int npx = g.dy * g.dx;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < npx; p += gridDim.x * blockDim.x) {
    const int y = p / g.dx, x = p - (p / g.dx) * g.dx;
    out[p] = lbp_code(im, g, y, x);
  }
}

struct HistArgs {
  int gr, gc, py, px, nbins_log2;
  int rows_per_wg;  // cell rows per workgroup
  int count_bytes;
};

__global__ void __launch_bounds__(256) elbp_hist_kernel(const uint8_t* __restrict__ imgs, LbpGeom g, HistArgs a,
                                                        void* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const int64_t img = blockIdx.y;
  const int cr0 = blockIdx.x * a.rows_per_wg;
  const int cr1 = min(a.gr, cr0 + a.rows_per_wg);
  const int nb = 1 << a.nbins_log2;
  const int ncell = (cr1 - cr0) * a.gc;
  for (int i = threadIdx.x; i < ncell * nb; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const uint8_t* im = imgs + img * (int64_t)g.H * g.W;
  const int wpx = a.gc * a.px;                 // covered code columns
  const int y0 = cr0 * a.py, y1 = cr1 * a.py;  // covered code rows
  const int npx = (y1 - y0) * wpx;
  for (int p = threadIdx.x; p < npx; p += blockDim.x) {
    const int yy = p / wpx, x = p - yy * wpx;
    const int y = y0 + yy;
    const uint32_t code = lbp_code(im, g, y, x);
    const int cell = (yy / a.py) * a.gc + x / a.px;
    atomicAdd(&hist[cell * nb + (int)code], 1u);
  }
  __syncthreads();
  const int64_t cell_base = img * (int64_t)a.gr * a.gc + (int64_t)cr0 * a.gc;
  const int total = ncell * nb;
  if (a.count_bytes == 1) {
    uint8_t* o = (uint8_t*)counts + cell_base * nb;
    for (int i = threadIdx.x; i < total; i += blockDim.x) o[i] = (uint8_t)hist[i];
  } else if (a.count_bytes == 2) {
    uint16_t* o = (uint16_t*)counts + cell_base * nb;
    for (int i = threadIdx.x; i < total; i += blockDim.x) o[i] = (uint16_t)hist[i];
  } else {
    uint32_t* o = (uint32_t*)counts + cell_base * nb;
    for (int i = threadIdx.x; i < total; i += blockDim.x) o[i] = hist[i];
  }
}

// Whole-image variant: one 1024-thread workgroup per image, the image staged in LDS (16-B loads)
// behind the u32 counters of all cells, codes computed from LDS (same fp64 arithmetic, same
// order) over a division-free 2-D walk, counts written four per 32-bit store.  Used when counters + image fit in 80 KiB, so two
// workgroups (32 waves) share a CU.
constexpr int LDS_IMG_BUDGET = 80 * 1024;

__global__ void __launch_bounds__(1024) elbp_hist_lds_kernel(const uint8_t* __restrict__ imgs, LbpGeom g, HistArgs a,
                                                             void* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const int64_t img = blockIdx.x;
  const int nb = 1 << a.nbins_log2;
  const int ncell = a.gr * a.gc;
  uint8_t* im = reinterpret_cast<uint8_t*>(hist + ncell * nb);
  const int npix = g.H * g.W;
  for (int i = threadIdx.x; i < ncell * nb; i += blockDim.x) hist[i] = 0;
  const uint8_t* src = imgs + img * (int64_t)npix;
  if ((npix & 15) == 0 && ((uintptr_t)src & 15) == 0) {
    for (int i = threadIdx.x; i < npix / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(im)[i] = reinterpret_cast<const uint4*>(src)[i];
  } else {
    for (int i = threadIdx.x; i < npix; i += blockDim.x) im[i] = src[i];
  }
  __syncthreads();
  const int wpx = a.gc * a.px;                 // covered code columns
  const int hpx = a.gr * a.py;                 // covered code rows
  // 2-D walk: thread (tx, ty) takes column x = tx (+128 ...) and RB rows ty, ty + 8, ... at a time.
  // Points outer, pixels inner: each (weight, offset) of the geometry is read once per RB pixels
  // (a runtime-indexed kernel-argument read is a scalar load whose lgkmcnt wait would also drain
  // the pending LDS atomics), and the atomics are issued after all codes of the group.
  constexpr int RB = 5;   // 8 x 5 = 40 rows per pass (120 code rows of a 128x128 face: 3 passes), <= 64 VGPRs
  const int tx = threadIdx.x & 127, ty = threadIdx.x >> 7;
  for (int x = tx; x < wpx; x += 128) {
    const int cx = x / a.px;
    for (int y0 = ty; y0 < hpx; y0 += 8 * RB) {
      uint32_t code[RB];
      double C[RB], N[RB];
      int base[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int y = min(y0 + 8 * r, hpx - 1);
        base[r] = y * g.W + x;
        C[r] = (double)im[base[r] + g.oy * g.W + g.ox];
        code[r] = 0;
      }
      for (int i = 0; i < g.P; ++i) {
        const int nt = g.nterm[i];
        {
          const int off = g.toff[i][0];
          const double w = g.tw[i][0];
#pragma unroll
          for (int r = 0; r < RB; ++r) N[r] = w * (double)im[base[r] + off];
        }
        for (int t = 1; t < nt; ++t) {   // lbp.py:123-126 order, no contraction
          const int off = g.toff[i][t];
          const double w = g.tw[i][t];
#pragma unroll
          for (int r = 0; r < RB; ++r) {
            const double prod = w * (double)im[base[r] + off];
            N[r] = N[r] + prod;
          }
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) code[r] |= (N[r] >= C[r] ? 1u : 0u) << i;
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const int y = y0 + 8 * r;
        if (y < hpx) atomicAdd(&hist[((y / a.py) * a.gc + cx) * nb + (int)code[r]], 1u);
      }
    }
  }
  __syncthreads();
  const int total = ncell * nb;
  const int64_t base = img * (int64_t)total;
  if (a.count_bytes == 1) {
    uint32_t* o = reinterpret_cast<uint32_t*>((uint8_t*)counts + base);
    for (int i = threadIdx.x; i < total / 4; i += blockDim.x)
      o[i] = hist[4 * i] | (hist[4 * i + 1] << 8) | (hist[4 * i + 2] << 16) | (hist[4 * i + 3] << 24);
  } else if (a.count_bytes == 2) {
    uint32_t* o = reinterpret_cast<uint32_t*>((uint16_t*)counts + base);
    for (int i = threadIdx.x; i < total / 2; i += blockDim.x) o[i] = hist[2 * i] | (hist[2 * i + 1] << 16);
  } else {
    uint32_t* o = (uint32_t*)counts + base;
    for (int i = threadIdx.x; i < total; i += blockDim.x) o[i] = hist[i];
  }
}

// ExtendedLBP(radius=1, neighbors=8) -- the reference's default operator and configs[3] -- with
// its 3x3 sampling block held in registers.  Thread (tx, ty) walks code column x = tx down a strip
// of rows; per code pixel it converts the 3 new pixels of the block's bottom row once and
// shifts the block, instead of re-reading and converting the 21 terms' pixels from LDS.  The
// arithmetic per point is lbp_code's (same products, same order, no contraction): the geometry
// is fixed at compile time -- which block cell each term reads and which weights are zero --
// and the host selects this kernel only when the caller's offsets and zero pattern are exactly
// these (R1P8_OFFS below; the weights themselves are the caller's, e.g. bits 4 and 6 carry
// the 2^-53 / 2^-52 terms of np.sin / np.cos).
struct R1P8 {
  double w[8][4];
};
constexpr int R1P8_OFFS[8][4] = {{1, 2, 1, 2}, {0, 1, 1, 2}, {0, 1, 0, 1}, {0, 0, 1, 1},
                                 {0, 0, 1, 0}, {1, 0, 2, 1}, {2, 0, 2, 1}, {1, 1, 2, 2}};
// non-zero terms per point: bit t set = weight t non-zero (points 0 and 2: weight 1.0 alone)
constexpr int R1P8_TERMS[8] = {0x1, 0xf, 0x1, 0xf, 0x5, 0xf, 0x3, 0xf};

__global__ void __launch_bounds__(1024) elbp_hist_r1p8_kernel(const uint8_t* __restrict__ imgs, LbpGeom g,
                                                              HistArgs a, R1P8 k, void* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const int64_t img = blockIdx.x;
  constexpr int nb = 256;
  const int ncell = a.gr * a.gc;
  uint8_t* im = reinterpret_cast<uint8_t*>(hist + ncell * nb);
  const int W = g.W, npix = g.H * W;
  for (int i = threadIdx.x; i < ncell * nb; i += blockDim.x) hist[i] = 0;
  const uint8_t* src = imgs + img * (int64_t)npix;
  if ((npix & 15) == 0 && ((uintptr_t)src & 15) == 0) {
    for (int i = threadIdx.x; i < npix / 16; i += blockDim.x)
      reinterpret_cast<uint4*>(im)[i] = reinterpret_cast<const uint4*>(src)[i];
  } else {
    for (int i = threadIdx.x; i < npix; i += blockDim.x) im[i] = src[i];
  }
  __syncthreads();
  const int wpx = a.gc * a.px, hpx = a.gr * a.py;
  const int tx = threadIdx.x & 127, ty = threadIdx.x >> 7;
  const int rows = (hpx + 7) >> 3;
  const int ya = ty * rows, yb = min(hpx, ya + rows);
  for (int x = tx; x < wpx && ya < yb; x += 128) {
    const uint8_t* col = im + x;
    double b00 = col[ya * W], b01 = col[ya * W + 1], b02 = col[ya * W + 2];
    double b10 = col[(ya + 1) * W], b11 = col[(ya + 1) * W + 1], b12 = col[(ya + 1) * W + 2];
    const int cxo = x / a.px;
    int cyc = ya / a.py, ry = ya - cyc * a.py;
    for (int y = ya; y < yb; ++y) {
      const uint8_t* r2 = col + (y + 2) * W;
      const double b20 = r2[0], b21 = r2[1], b22 = r2[2];
      const double C = b11;
      uint32_t code = 0;
      double N;
      N = k.w[0][0] * b12;
      code |= (N >= C ? 1u : 0u) << 0;
      N = k.w[1][0] * b01; N = N + k.w[1][1] * b02; N = N + k.w[1][2] * b11; N = N + k.w[1][3] * b12;
      code |= (N >= C ? 1u : 0u) << 1;
      N = k.w[2][0] * b01;
      code |= (N >= C ? 1u : 0u) << 2;
      N = k.w[3][0] * b00; N = N + k.w[3][1] * b01; N = N + k.w[3][2] * b10; N = N + k.w[3][3] * b11;
      code |= (N >= C ? 1u : 0u) << 3;
      N = k.w[4][0] * b00; N = N + k.w[4][2] * b10;
      code |= (N >= C ? 1u : 0u) << 4;
      N = k.w[5][0] * b10; N = N + k.w[5][1] * b11; N = N + k.w[5][2] * b20; N = N + k.w[5][3] * b21;
      code |= (N >= C ? 1u : 0u) << 5;
      N = k.w[6][0] * b20; N = N + k.w[6][1] * b21;
      code |= (N >= C ? 1u : 0u) << 6;
      N = k.w[7][0] * b11; N = N + k.w[7][1] * b12; N = N + k.w[7][2] * b21; N = N + k.w[7][3] * b22;
      code |= (N >= C ? 1u : 0u) << 7;
      atomicAdd(&hist[(cyc * a.gc + cxo) * nb + (int)code], 1u);
      if (++ry == a.py) {
        ry = 0;
        ++cyc;
      }
      b00 = b10; b01 = b11; b02 = b12;
      b10 = b20; b11 = b21; b12 = b22;
    }
  }
  __syncthreads();
  const int total = ncell * nb;
  const int64_t base = img * (int64_t)total;
  if (a.count_bytes == 1) {
    uint32_t* o = reinterpret_cast<uint32_t*>((uint8_t*)counts + base);
    for (int i = threadIdx.x; i < total / 4; i += blockDim.x)
      o[i] = hist[4 * i] | (hist[4 * i + 1] << 8) | (hist[4 * i + 2] << 16) | (hist[4 * i + 3] << 24);
  } else if (a.count_bytes == 2) {
    uint32_t* o = reinterpret_cast<uint32_t*>((uint16_t*)counts + base);
    for (int i = threadIdx.x; i < total / 2; i += blockDim.x) o[i] = hist[2 * i] | (hist[2 * i + 1] << 16);
  } else {
    uint32_t* o = (uint32_t*)counts + base;
    for (int i = threadIdx.x; i < total; i += blockDim.x) o[i] = hist[i];
  }
}

// the caller's geometry is the compiled r1p8 one: same offsets, same zero pattern, weight 1.0 alone
// for points 0 and 2
static bool r1p8_match(int P, const int32_t* offs, const double* w, int oy, int ox, int by, int bx, R1P8& k) {
  if (P != 8 || oy != 1 || ox != 1 || by != 3 || bx != 3) return false;
  for (int i = 0; i < 8; ++i)
    for (int t = 0; t < 4; ++t) {
      if (offs[4 * i + t] != R1P8_OFFS[i][t]) return false;
      const double wt = w[4 * i + t];
      if (((R1P8_TERMS[i] >> t) & 1) != (wt != 0.0 ? 1 : 0)) return false;
      k.w[i][t] = wt;
    }
  return w[0] == 1.0 && w[8] == 1.0;
}

static bool lbp_generic_forced() {
  static const bool f = [] {
    const char* e = getenv("OFR_LBP_GENERIC");
    return e && atoi(e) != 0;
  }();
  return f;
}

static int make_geom(LbpGeom& g, int H, int W, int P, const int32_t* offs, const double* w, int oy, int ox, int by,
                     int bx) {
  if (P < 1 || P > MAXP) return fail(OFR_E_UNSUPPORTED, "ofr_elbp: neighbors must be in [1, 32]");
  if (!offs || !w) return fail(OFR_E_INVALID, "ofr_elbp: null geometry");
  g.P = P;
  g.H = H;
  g.W = W;
  g.dy = H - by + 1;
  g.dx = W - bx + 1;
  g.oy = oy;
  g.ox = ox;
  for (int i = 0; i < P; ++i) {
    // (fy, fx), (fy, cx), (cy, fx), (cy, cx) with weights w1..w4 (lbp.py:123-126)
    const int fy = offs[4 * i + 0], fx = offs[4 * i + 1], cy = offs[4 * i + 2], cx = offs[4 * i + 3];
    if (fy < 0 || fx < 0 || cy >= by || cx >= bx || cy < fy || cx < fx)
      return fail(OFR_E_INVALID, "ofr_elbp: sample offsets outside the block");
    const int pos[4][2] = {{fy, fx}, {fy, cx}, {cy, fx}, {cy, cx}};
    int nt = 0;
    for (int t = 0; t < 4; ++t) {
      const double wt = w[4 * i + t];
      if (!(wt >= 0.0)) return fail(OFR_E_INVALID, "ofr_elbp: negative or NaN weight");
      if (wt == 0.0) continue;  // exact +0 contribution
      g.toff[i][nt] = pos[t][0] * W + pos[t][1];
      g.tw[i][nt] = wt;
      ++nt;
    }
    if (nt == 0) {  // all-zero weights: N = 0
      g.toff[i][0] = 0;
      g.tw[i][0] = 0.0;
      nt = 1;
    }
    g.nterm[i] = nt;
  }
  return OFR_OK;
}

}  // namespace ofr

using namespace ofr;

extern "C" int ofr_elbp_codes(void* stream, const uint8_t* imgs, int64_t n, int H, int W, int P,
                              const int32_t* offs_host, const double* w_host, int oy, int ox, int by, int bx,
                              uint32_t* codes) {
  OFR_CHECK_ARG(n >= 0 && H >= 1 && W >= 1, "ofr_elbp_codes: bad sizes");
  LbpGeom g;
  int rc = make_geom(g, H, W, P, offs_host, w_host, oy, ox, by, bx);
  if (rc) return rc;
  if (n == 0 || g.dy <= 0 || g.dx <= 0) return OFR_OK;
  OFR_CHECK_ARG(imgs && codes, "ofr_elbp_codes: null pointer");
  OFR_CHECK_ARG(n <= 65535 * 1024LL, "ofr_elbp_codes: too many images");
  const int npx = g.dy * g.dx;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(npx, 256), 64);
  int64_t done = 0;
  while (done < n) {
    const int64_t chunk = std::min<int64_t>(n - done, 65535);
    hipLaunchKernelGGL(elbp_codes_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream,
                       imgs + done * (int64_t)H * W, chunk, g, codes + done * (int64_t)npx);
    OFR_LAUNCH_CHECK("elbp_codes_kernel");
    done += chunk;
  }
  return OFR_OK;
}

extern "C" int ofr_elbp_hist_geom(void* stream, const uint8_t* imgs, int64_t n, int H, int W, int P,
                             const int32_t* offs_host, const double* w_host, int oy, int ox, int by, int bx, int gr,
                             int gc, void* counts, int count_bytes) {
  OFR_CHECK_ARG(n >= 0 && H >= 1 && W >= 1 && gr >= 1 && gc >= 1, "ofr_elbp_hist_geom: bad sizes");
  OFR_CHECK_ARG(count_bytes == 1 || count_bytes == 2 || count_bytes == 4, "ofr_elbp_hist_geom: count_bytes must be 1, 2 or 4");
  if (P > 15) return fail(OFR_E_UNSUPPORTED, "ofr_elbp_hist_geom: neighbors must be <= 15 for the LDS histogram");
  LbpGeom g;
  int rc = make_geom(g, H, W, P, offs_host, w_host, oy, ox, by, bx);
  if (rc) return rc;
  HistArgs a;
  a.gr = gr;
  a.gc = gc;
  a.py = g.dy > 0 ? g.dy / gr : 0;
  a.px = g.dx > 0 ? g.dx / gc : 0;
  a.nbins_log2 = P;
  a.count_bytes = count_bytes;
  const int64_t nb = 1LL << P;
  const int64_t cell_px = (int64_t)a.py * a.px;
  if (count_bytes == 1) OFR_CHECK_ARG(cell_px <= 255, "ofr_elbp_hist_geom: cell too large for 1-byte counts");
  if (count_bytes == 2) OFR_CHECK_ARG(cell_px <= 65535, "ofr_elbp_hist_geom: cell too large for 2-byte counts");
  if (n == 0) return OFR_OK;
  OFR_CHECK_ARG(imgs && counts, "ofr_elbp_hist_geom: null pointer");
  hipStream_t st = (hipStream_t)stream;
  if (cell_px == 0) {  // empty cells: all counts zero (the reference's histogram is then NaN)
    hipError_t e = hipMemsetAsync(counts, 0, (size_t)n * gr * gc * nb * count_bytes, st);
    return e == hipSuccess ? OFR_OK : hip_status(e, "hipMemsetAsync");
  }
  const int64_t nbins_total = (int64_t)gr * gc * nb;
  const size_t lds_whole = (size_t)nbins_total * 4 + round_up((int64_t)H * W, 16);
  // whole-image LDS variant: counters + image fit the budget, and the packed stores stay aligned
  R1P8 k8;
  if (lds_whole <= (size_t)LDS_IMG_BUDGET && nbins_total % 4 == 0 && n <= 0x7fffffffLL && !lbp_generic_forced() &&
      r1p8_match(P, offs_host, w_host, oy, ox, by, bx, k8)) {
    static bool attr8 = false;
    if (!attr8) {
      hipError_t e = hipFuncSetAttribute((const void*)elbp_hist_r1p8_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, LDS_IMG_BUDGET);
      if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(elbp_hist_r1p8)");
      attr8 = true;
    }
    hipLaunchKernelGGL(elbp_hist_r1p8_kernel, dim3((unsigned)n), dim3(1024), lds_whole, st, imgs, g, a, k8, counts);
    OFR_LAUNCH_CHECK("elbp_hist_r1p8_kernel");
    return OFR_OK;
  }
  if (lds_whole <= (size_t)LDS_IMG_BUDGET && nbins_total % 4 == 0 && n <= 0x7fffffffLL) {
    static bool attr_done = false;
    if (!attr_done) {
      hipError_t e = hipFuncSetAttribute((const void*)elbp_hist_lds_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, LDS_IMG_BUDGET);
      if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(elbp_hist_lds)");
      attr_done = true;
    }
    hipLaunchKernelGGL(elbp_hist_lds_kernel, dim3((unsigned)n), dim3(1024), lds_whole, st, imgs, g, a, counts);
    OFR_LAUNCH_CHECK("elbp_hist_lds_kernel");
    return OFR_OK;
  }
  const int64_t lds_cap = 64 * 1024;  // bytes of u32 counters per workgroup
  const int64_t row_bytes = (int64_t)gc * nb * 4;
  if (row_bytes > lds_cap) {
    return fail(OFR_E_UNSUPPORTED, "ofr_elbp_hist_geom: grid_cols * 2^P too large for one LDS band");
  }
  a.rows_per_wg = (int)std::max<int64_t>(1, std::min<int64_t>(gr, lds_cap / row_bytes));
  const unsigned gx = (unsigned)cdiv(gr, a.rows_per_wg);
  const size_t lds = (size_t)a.rows_per_wg * row_bytes;
  int64_t done = 0;
  while (done < n) {
    const int64_t chunk = std::min<int64_t>(n - done, 65535);
    hipLaunchKernelGGL(elbp_hist_kernel, dim3(gx, (unsigned)chunk), dim3(256), lds, st, imgs + done * (int64_t)H * W, g,
                       a, (void*)((char*)counts + done * gr * gc * nb * count_bytes));
    OFR_LAUNCH_CHECK("elbp_hist_kernel");
    done += chunk;
  }
  return OFR_OK;
}
