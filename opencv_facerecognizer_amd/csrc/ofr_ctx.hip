// The context-based C ABI of SURVEY §8b: ofr_ctx_create / ofr_project_u8 / ofr_gram / ofr_scatter
// / ofr_knn, for a caller binding the hot path through an FFI with plain row-major buffers (the
// layouts the reference's numpy code holds: X [B][D] uint8, W [D][d], F [N][d], Q [B][d],
// G [N][d]).  Each entry point lays its operands out for the library's kernels in a workspace the
// context owns (grown on demand, stream-ordered) and runs them:
//   ofr_project_u8 -> ofr_qproj_prepare + ofr_project_u8_exact (exact int8-slice engine)
//   ofr_gram       -> fp32 -> fp64 (exact) + ofr_gemm_f64 (fp64 MFMA, fp64 accumulation)
//   ofr_scatter    -> ofr_class_center_f64 + two ofr_gemm_f64 (feature.py:160-168)
//   ofr_knn        -> ofr_knn_f32 (Euclidean / Cosine, fp32 MFMA tiles + exact fp64 re-rank) or
//                     ofr_chi2_knn + ofr_chi2_knn_exact for the queries it leaves uncertified
//   ofr_elbp_hist  -> ofr_elbp_hist_geom (centre-relative sample offsets -> block geometry)
// A context belongs to one device and one thread at a time (the reference's calls are
// synchronous per caller); calls on it are ordered on the stream they are given.
#include <vector>

#include "ofr_common.h"

struct ofr_ctx {
  int device = 0;
  char* ws = nullptr;   // scratch, reused by every call
  size_t cap = 0;
  // the projection prepared last (kept for OFR_PROJ_REUSE_W)
  char* proj = nullptr;
  size_t proj_cap = 0;
  const float* proj_W = nullptr;
  int64_t proj_D = 0, proj_d = 0;
};

namespace ofr {
namespace ctxk {

static inline size_t up(size_t x) { return (x + 255) & ~(size_t)255; }

static int grow(char** buf, size_t* cap, size_t need, hipStream_t) {
  if (need <= *cap) return OFR_OK;
  // earlier calls may still use the old buffer, on this stream or another the caller used before
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_status(e, "ofr_ctx: device sync");
  if (*buf) {
    e = hipFree(*buf);
    if (e != hipSuccess) return hip_status(e, "ofr_ctx: hipFree");
    *buf = nullptr;
    *cap = 0;
  }
  e = hipMalloc((void**)buf, need);
  if (e != hipSuccess) return hip_status(e, "ofr_ctx: hipMalloc");
  *cap = need;
  return OFR_OK;
}

// out[j][i] = in[i][j]: [R][C] f32 -> [C][ldo] f32, 32 x 32 tiles through LDS
__global__ void __launch_bounds__(256) transpose_f32_kernel(const float* in, int64_t R, int64_t C, float* out,
                                                            int64_t ldo) {
  __shared__ float t[32][33];
  const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int r = ty; r < 32; r += 8)
    if (r0 + r < R && c0 + tx < C) t[r][tx] = in[(r0 + r) * C + c0 + tx];
  __syncthreads();
  for (int c = ty; c < 32; c += 8)
    if (c0 + c < C && r0 + tx < R) out[(c0 + c) * ldo + r0 + tx] = t[tx][c];
}

// [R][C] f32 -> [R][ldo] (f64 or zero-padded f32)
template <typename T>
__global__ void widen_rows_kernel(const float* in, int64_t R, int64_t C, T* out, int64_t ldo) {
  const int64_t n = R * ldo;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / ldo, c = i - r * ldo;
    out[i] = c < C ? (T)in[r * C + c] : (T)0;
  }
}

__global__ void narrow_f64_kernel(const double* in, int64_t n, float* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (float)in[i];
}

// shift[j] = sum_i W[i][j] mu[i] in fp64, i ascending (PCA.project's P^T mu, feature.py:114-116)
__global__ void shift_gemv_kernel(const float* W, int64_t D, int64_t d, const double* mu, double* shift) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d) return;
  double s = 0.0;
  for (int64_t i = 0; i < D; ++i) s += (double)W[i * d + j] * mu[i];
  shift[j] = s;
}

// rows [n] of src [.][ld] -> dst [n][ld]  (dir 0: gather dst[r] = src[rows[r]]; 1: scatter)
template <typename T>
__global__ void rows_kernel(const T* src, int64_t ld, const int64_t* rows, int64_t n, T* dst, int dir) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const int64_t s = dir == 0 ? rows[r] : r, t = dir == 0 ? r : rows[r];
  for (int64_t c = threadIdx.x; c < ld; c += blockDim.x) dst[t * ld + c] = src[s * ld + c];
}

static unsigned blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(n, 256), 8192)); }

}  // namespace ctxk
}  // namespace ofr

using namespace ofr;

extern "C" int ofr_ctx_create(int device, ofr_ctx** out) {
  OFR_CHECK_ARG(out, "ofr_ctx_create: null output");
  const int rc = ofr_device_check(device);
  if (rc) return rc;
  ofr_ctx* c = new ofr_ctx;
  c->device = device;
  *out = c;
  return OFR_OK;
}

extern "C" int ofr_ctx_destroy(ofr_ctx* c) {
  if (!c) return OFR_OK;
  int rc = OFR_OK;
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e == hipSuccess) e = hipSetDevice(c->device);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess && c->ws) e = hipFree(c->ws);
  if (e == hipSuccess && c->proj) e = hipFree(c->proj);
  if (e != hipSuccess) rc = hip_status(e, "ofr_ctx_destroy");
  (void)hipSetDevice(cur);
  delete c;
  return rc;
}

extern "C" int ofr_project_u8(ofr_ctx* c, void* stream, const uint8_t* X, int64_t B, int64_t D, const float* W,
                              int64_t d, const double* mu, float* Y, int flags) {
  OFR_CHECK_ARG(c, "ofr_project_u8: null context");
  OFR_CHECK_ARG(B >= 0 && D >= 1 && d >= 1, "ofr_project_u8: bad sizes");
  OFR_CHECK_ARG((flags & ~(OFR_FP64_ACC | OFR_PROJ_REUSE_W)) == 0, "ofr_project_u8: unknown flags");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(X && W && Y, "ofr_project_u8: null pointer");
  OFR_DEVICE_GUARD(c->device, "ofr_project_u8: set device");
  hipStream_t st = (hipStream_t)stream;
  const int64_t ldk = round_up(D, 128);
  const size_t aq = ofr_qproj_bytes(D, d);
  const size_t p_aq = 0, p_scale = ctxk::up(aq), p_k = p_scale + ctxk::up((size_t)d * 8), p_end = p_k + ctxk::up((size_t)d * 8);
  const bool reuse = (flags & OFR_PROJ_REUSE_W) && c->proj && c->proj_W == W && c->proj_D == D && c->proj_d == d;
  int rc;
  if (!reuse) {
    // the cache names W only once its slices are complete: a failed grow / prepare below must not
    // leave an older W's name on a half-overwritten projection
    c->proj_W = nullptr;
    // W [D][d] -> W^T [d][D] in the scratch, then the int8 slices into the context's projection
    rc = ctxk::grow(&c->ws, &c->cap, ctxk::up((size_t)d * D * 4), st);
    if (rc) return rc;
    float* Wt = (float*)c->ws;
    hipLaunchKernelGGL(ctxk::transpose_f32_kernel, dim3((unsigned)cdiv(d, 32), (unsigned)cdiv(D, 32)), dim3(256), 0,
                       st, W, D, d, Wt, D);
    OFR_LAUNCH_CHECK("transpose_f32_kernel");
    rc = ctxk::grow(&c->proj, &c->proj_cap, p_end, st);
    if (rc) return rc;
    rc = ofr_qproj_prepare(stream, OFR_DT_F32, Wt, d, D, D, (int8_t*)(c->proj + p_aq), ldk,
                           (double*)(c->proj + p_scale), (double*)(c->proj + p_k));
    if (rc) return rc;
    c->proj_W = W;
    c->proj_D = D;
    c->proj_d = d;
  }
  // scratch: shift [d] f64, then the padded faces when the rows are not 16-byte aligned
  const bool aligned = D % 16 == 0 && ((uintptr_t)X % 16) == 0;
  const size_t s_shift = 0, s_x = ctxk::up((size_t)d * 8);
  rc = ctxk::grow(&c->ws, &c->cap, s_x + (aligned ? 0 : ctxk::up((size_t)B * ldk)), st);
  if (rc) return rc;
  const double* shift = nullptr;
  if (mu) {
    hipLaunchKernelGGL(ctxk::shift_gemv_kernel, dim3((unsigned)cdiv(d, 256)), dim3(256), 0, st, W, D, d, mu,
                       (double*)(c->ws + s_shift));
    OFR_LAUNCH_CHECK("shift_gemv_kernel");
    shift = (const double*)(c->ws + s_shift);
  }
  const uint8_t* Xp = X;
  int64_t ldx = D;
  if (!aligned) {
    rc = ofr_pad_u8(stream, X, B, D, D, 0, (uint8_t*)(c->ws + s_x), ldk);
    if (rc) return rc;
    Xp = (const uint8_t*)(c->ws + s_x);
    ldx = ldk;
  }
  return ofr_project_u8_exact(stream, Xp, B, D, ldx, (const int8_t*)(c->proj + p_aq), ldk,
                              (const double*)(c->proj + p_scale), (const double*)(c->proj + p_k), d, shift, Y, d,
                              OFR_DT_F32);
}

extern "C" int ofr_gram(ofr_ctx* c, void* stream, const float* A, int64_t rows, int64_t cols, int side, int prec,
                        void* G) {
  OFR_CHECK_ARG(c, "ofr_gram: null context");
  OFR_CHECK_ARG(rows >= 1 && cols >= 1 && (side == OFR_GRAM_ATA || side == OFR_GRAM_AAT) &&
                    (prec == OFR_DT_F32 || prec == OFR_DT_F64),
                "ofr_gram: bad arguments");
  OFR_CHECK_ARG(A && G, "ofr_gram: null pointer");
  OFR_DEVICE_GUARD(c->device, "ofr_gram: set device");
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = side == OFR_GRAM_ATA ? cols : rows;
  const size_t s_a = 0, s_g = ctxk::up((size_t)rows * cols * 8);
  int rc = ctxk::grow(&c->ws, &c->cap, s_g + (prec == OFR_DT_F32 ? ctxk::up((size_t)n * n * 8) : 0), st);
  if (rc) return rc;
  double* A64 = (double*)(c->ws + s_a);
  hipLaunchKernelGGL(ctxk::widen_rows_kernel<double>, dim3(ctxk::blocks(rows * cols)), dim3(256), 0, st, A, rows, cols,
                     A64, cols);
  OFR_LAUNCH_CHECK("widen_rows_kernel");
  double* G64 = prec == OFR_DT_F64 ? (double*)G : (double*)(c->ws + s_g);
  // fp32 x fp32 products are exact in fp64; the sums accumulate in fp64 on the MFMA
  if (side == OFR_GRAM_ATA)
    rc = ofr_gemm_f64(stream, 1, 0, cols, cols, rows, 1.0, A64, cols, A64, cols, 0.0, G64, cols);
  else
    rc = ofr_gemm_f64(stream, 0, 1, rows, rows, cols, 1.0, A64, cols, A64, cols, 0.0, G64, rows);
  if (rc) return rc;
  if (prec == OFR_DT_F32) {
    hipLaunchKernelGGL(ctxk::narrow_f64_kernel, dim3(ctxk::blocks(n * n)), dim3(256), 0, st, G64, n * n, (float*)G);
    OFR_LAUNCH_CHECK("narrow_f64_kernel");
  }
  return OFR_OK;
}

extern "C" int ofr_scatter(ofr_ctx* c, void* stream, const float* F, const int32_t* y, int64_t N, int64_t d,
                           int32_t ncls, void* Sw, void* Sb, void* means) {
  OFR_CHECK_ARG(c, "ofr_scatter: null context");
  OFR_CHECK_ARG(N >= 1 && d >= 1 && ncls >= 1, "ofr_scatter: bad sizes");
  OFR_CHECK_ARG(F && y && Sw && Sb, "ofr_scatter: null pointer");
  OFR_DEVICE_GUARD(c->device, "ofr_scatter: set device");
  hipStream_t st = (hipStream_t)stream;
  // labels -> class-grouped row order (host: one read of y, as the reference iterates range(c))
  std::vector<int32_t> yh((size_t)N);
  hipError_t e = hipMemcpyAsync(yh.data(), y, (size_t)N * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_status(e, "ofr_scatter: labels readback");
  std::vector<int64_t> offsets((size_t)ncls + 1, 0), perm((size_t)N);
  for (int64_t n = 0; n < N; ++n) {
    if (yh[(size_t)n] < 0 || yh[(size_t)n] >= ncls)
      return fail(OFR_E_INVALID, "ofr_scatter: labels must be 0..c-1 (feature.py:164-165 iterates range(c))");
    ++offsets[(size_t)yh[(size_t)n] + 1];
  }
  for (int32_t i = 0; i < ncls; ++i) offsets[(size_t)i + 1] += offsets[(size_t)i];
  {
    std::vector<int64_t> fill(offsets.begin(), offsets.end() - 1);
    for (int64_t n = 0; n < N; ++n) perm[(size_t)fill[(size_t)yh[(size_t)n]]++] = n;   // stable
  }
  const size_t s_f = 0, s_fc = s_f + ctxk::up((size_t)N * d * 8), s_tot = s_fc + ctxk::up((size_t)N * d * 8),
               s_m = s_tot + ctxk::up((size_t)d * 8), s_mc = s_m + ctxk::up((size_t)ncls * d * 8),
               s_mn = s_mc + ctxk::up((size_t)ncls * d * 8), s_perm = s_mn + ctxk::up((size_t)ncls * d * 8),
               s_off = s_perm + ctxk::up((size_t)N * 8), s_end = s_off + ctxk::up((size_t)(ncls + 1) * 8);
  int rc = ctxk::grow(&c->ws, &c->cap, s_end, st);
  if (rc) return rc;
  char* w = c->ws;
  ::ofr::StreamSyncGuard uploads(st);   // perm / offsets are read asynchronously until the stream syncs
  e = hipMemcpyAsync(w + s_perm, perm.data(), (size_t)N * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = hipMemcpyAsync(w + s_off, offsets.data(), (size_t)(ncls + 1) * 8, hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return hip_status(e, "ofr_scatter: upload");
  double* F64 = (double*)(w + s_f);
  hipLaunchKernelGGL(ctxk::widen_rows_kernel<double>, dim3(ctxk::blocks(N * d)), dim3(256), 0, st, F, N, d, F64, d);
  OFR_LAUNCH_CHECK("widen_rows_kernel");
  rc = ofr_col_mean_f64(stream, F64, N, d, d, (double*)(w + s_tot));
  if (rc) return rc;
  double* M = means ? (double*)means : (double*)(w + s_m);
  rc = ofr_class_center_f64(stream, F64, N, d, d, (const int64_t*)(w + s_perm), (const int64_t*)(w + s_off), ncls,
                            (const double*)(w + s_tot), M, (double*)(w + s_fc), (double*)(w + s_mc),
                            (double*)(w + s_mn));
  if (rc) return rc;
  rc = ofr_gemm_f64(stream, 1, 0, d, d, N, 1.0, (const double*)(w + s_fc), d, (const double*)(w + s_fc), d, 0.0,
                    (double*)Sw, d);
  if (rc) return rc;
  rc = ofr_gemm_f64(stream, 1, 0, d, d, ncls, 1.0, (const double*)(w + s_mc), d, (const double*)(w + s_mn), d, 0.0,
                    (double*)Sb, d);
  if (rc) return rc;
  // the host vectors above were uploaded asynchronously: finish before they go out of scope
  e = hipStreamSynchronize(st);
  uploads.disarm();
  return e == hipSuccess ? OFR_OK : hip_status(e, "ofr_scatter: sync");
}

extern "C" int ofr_knn(ofr_ctx* c, void* stream, int metric, const float* Q, int64_t B, const float* G,
                       const float* g_norms, int64_t N, int64_t d, int k, int64_t index_base, float* out_d,
                       int64_t* out_i) {
  OFR_CHECK_ARG(c, "ofr_knn: null context");
  OFR_CHECK_ARG(metric == OFR_METRIC_EUCLIDEAN || metric == OFR_METRIC_COSINE || metric == OFR_METRIC_CHISQUARE,
                "ofr_knn: unknown metric");
  OFR_CHECK_ARG(B >= 0 && N >= 1 && d >= 1, "ofr_knn: bad sizes");
  if (k < 1 || k > OFR_MAX_K) return fail(OFR_E_UNSUPPORTED, "ofr_knn: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(Q && G && out_d && out_i, "ofr_knn: null pointer");
  OFR_DEVICE_GUARD(c->device, "ofr_knn: set device");
  hipStream_t st = (hipStream_t)stream;
  const bool chi = metric == OFR_METRIC_CHISQUARE;
  const int64_t ld = chi ? round_up(d, 4) : round_up(d, 32);
  const bool pad = ld != d || ((uintptr_t)Q % 16) != 0 || ((uintptr_t)G % 16) != 0;
  const size_t knn_ws = chi ? ofr_chi2_workspace_bytes(B, N, k) : ofr_knn_workspace_bytes(B, N, k);
  const size_t s_od = 0, s_aux = ctxk::up((size_t)B * k * 8), s_cert = s_aux + ctxk::up((size_t)N * 4),
               s_q = s_cert + ctxk::up((size_t)B * 4), s_g = s_q + (pad ? ctxk::up((size_t)B * ld * 4) : 0),
               s_knn = s_g + (pad ? ctxk::up((size_t)N * ld * 4) : 0), s_end = s_knn + ctxk::up(knn_ws);
  // ChiSquare: room for the exact pass over every query, so the region never moves mid-call
  const size_t x_rows = 0, x_q = ctxk::up((size_t)B * 8), x_d = x_q + ctxk::up((size_t)B * ld * 4),
               x_i = x_d + ctxk::up((size_t)B * k * 8), x_ws = x_i + ctxk::up((size_t)B * k * 8),
               x_end = x_ws + (chi ? ctxk::up(ofr_chi2_workspace_bytes(B, N, k)) : 0);
  int rc = ctxk::grow(&c->ws, &c->cap, s_end + (chi ? x_end : 0), st);
  if (rc) return rc;
  char* w = c->ws;
  const float* Qp = Q;
  const float* Gp = G;
  if (pad) {
    hipLaunchKernelGGL(ctxk::widen_rows_kernel<float>, dim3(ctxk::blocks(B * ld)), dim3(256), 0, st, Q, B, d,
                       (float*)(w + s_q), ld);
    OFR_LAUNCH_CHECK("widen_rows_kernel");
    hipLaunchKernelGGL(ctxk::widen_rows_kernel<float>, dim3(ctxk::blocks(N * ld)), dim3(256), 0, st, G, N, d,
                       (float*)(w + s_g), ld);
    OFR_LAUNCH_CHECK("widen_rows_kernel");
    Qp = (const float*)(w + s_q);
    Gp = (const float*)(w + s_g);
  }
  double* od = (double*)(w + s_od);
  if (!chi) {
    const float* aux = g_norms;
    if (!aux) {
      rc = ofr_row_aux(stream, metric, Gp, N, d, ld, (float*)(w + s_aux));
      if (rc) return rc;
      aux = (const float*)(w + s_aux);
    }
    rc = ofr_knn_f32(stream, metric, Qp, B, ld, Gp, N, ld, d, aux, k, index_base, od, out_i, w + s_knn, knn_ws);
    if (rc) return rc;
  } else {
    int* cert = (int*)(w + s_cert);
    rc = ofr_chi2_knn(stream, OFR_DT_F32, Qp, B, ld, Gp, N, ld, d, 1.0, k, index_base, od, out_i, w + s_knn, knn_ws,
                      cert);
    if (rc) return rc;
    // queries the fp32 pass could not certify: the exact fp64 pass on them alone
    std::vector<int> ch((size_t)B);
    hipError_t e = hipMemcpyAsync(ch.data(), cert, (size_t)B * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_status(e, "ofr_knn: certificate readback");
    std::vector<int64_t> open;
    for (int64_t b = 0; b < B; ++b)
      if (!ch[(size_t)b]) open.push_back(b);
    const int64_t n = (int64_t)open.size();
    if (n) {
      const size_t x_knn = ofr_chi2_workspace_bytes(n, N, k);
      char* x = c->ws + s_end;
      ::ofr::StreamSyncGuard upload(st);   // `open` is read asynchronously until the stream syncs
      e = hipMemcpyAsync(x + x_rows, open.data(), (size_t)n * 8, hipMemcpyHostToDevice, st);
      if (e != hipSuccess) return hip_status(e, "ofr_knn: rows upload");
      hipLaunchKernelGGL(ctxk::rows_kernel<float>, dim3((unsigned)n), dim3(256), 0, st, Qp, ld,
                         (const int64_t*)(x + x_rows), n, (float*)(x + x_q), 0);
      OFR_LAUNCH_CHECK("rows_kernel");
      rc = ofr_chi2_knn_exact(stream, OFR_DT_F32, x + x_q, n, ld, Gp, N, ld, d, 1.0, k, index_base, (double*)(x + x_d),
                              (int64_t*)(x + x_i), x + x_ws, x_knn, nullptr);
      if (rc) return rc;
      hipLaunchKernelGGL(ctxk::rows_kernel<double>, dim3((unsigned)n), dim3(256), 0, st, (const double*)(x + x_d),
                         (int64_t)k, (const int64_t*)(x + x_rows), n, od, 1);
      OFR_LAUNCH_CHECK("rows_kernel");
      hipLaunchKernelGGL(ctxk::rows_kernel<int64_t>, dim3((unsigned)n), dim3(256), 0, st, (const int64_t*)(x + x_i),
                         (int64_t)k, (const int64_t*)(x + x_rows), n, out_i, 1);
      OFR_LAUNCH_CHECK("rows_kernel");
      e = hipStreamSynchronize(st);   // `open` is read by the upload above
      upload.disarm();
      if (e != hipSuccess) return hip_status(e, "ofr_knn: sync");
    }
  }
  hipLaunchKernelGGL(ctxk::narrow_f64_kernel, dim3(ctxk::blocks(B * k)), dim3(256), 0, st, od, B * (int64_t)k, out_d);
  OFR_LAUNCH_CHECK("narrow_f64_kernel");
  return OFR_OK;
}

extern "C" int ofr_elbp_hist(ofr_ctx* c, void* stream, const uint8_t* imgs, int64_t n, int H, int W, const double* w,
                             const int32_t* off, int P, int gr, int gc, uint8_t* counts) {
  OFR_CHECK_ARG(c, "ofr_elbp_hist: null context");
  OFR_CHECK_ARG(w && off, "ofr_elbp_hist: null geometry");
  OFR_CHECK_ARG(P >= 1 && P <= 15, "ofr_elbp_hist: neighbors must be in [1, 15]");
  OFR_CHECK_ARG(H >= 1 && W >= 1 && gr >= 1 && gc >= 1 && n >= 0, "ofr_elbp_hist: bad sizes");
  // lbp.py:90-97 from the centre-relative floor / ceil offsets: the block spans
  // [min(0, min floor), max(0, max ceil)] on each axis and the centre sits at -min(0, min floor)
  int y0 = 0, x0 = 0, y1 = 0, x1 = 0;
  for (int i = 0; i < P; ++i) {
    y0 = std::min(y0, off[4 * i + 0]);
    x0 = std::min(x0, off[4 * i + 1]);
    y1 = std::max(y1, off[4 * i + 2]);
    x1 = std::max(x1, off[4 * i + 3]);
  }
  const int oy = -y0, ox = -x0, by = y1 - y0 + 1, bx = x1 - x0 + 1;
  std::vector<int32_t> boff((size_t)P * 4);
  for (int i = 0; i < P; ++i) {
    boff[(size_t)(4 * i + 0)] = off[4 * i + 0] + oy;
    boff[(size_t)(4 * i + 1)] = off[4 * i + 1] + ox;
    boff[(size_t)(4 * i + 2)] = off[4 * i + 2] + oy;
    boff[(size_t)(4 * i + 3)] = off[4 * i + 3] + ox;
  }
  const int dy = H - by + 1, dx = W - bx + 1;
  const int64_t cell = (int64_t)(dy > 0 ? dy / gr : 0) * (dx > 0 ? dx / gc : 0);
  if (cell > 255) return fail(OFR_E_UNSUPPORTED, "ofr_elbp_hist: cells of more than 255 pixels need ofr_elbp_hist_geom");
  OFR_DEVICE_GUARD(c->device, "ofr_elbp_hist: set device");
  return ofr_elbp_hist_geom(stream, imgs, n, H, W, P, boff.data(), w, oy, ox, by, bx, gr, gc, counts, 1);
}
