// Training eigensolves on the device.
//
// The reference solves its eigenproblems with host LAPACK: PCA's svd (feature.py:94) and LDA's
// eig(inv(Sw) Sb) (feature.py:170).  At configs[4] (D = 10,000) the symmetric-definite form of
// the LDA problem, Sb v = lambda Sw v, took 12-16 s of host LAPACK (dsygvd) against 2.1 s on the
// device (tools/bench_eigh.py, profiles/r02_eigh_probe.json), and the PCA covariance/Gram eigh
// 14.5 s against 1.1 s.  These entry points run rocSOLVER's divide-and-conquer drivers on the
// matrices where they already lie (the exact device Gram / scatter of ofr_gram.hip) and hand back
// the m LARGEST eigenpairs in descending order, row-major [n][m] like the reference's eigenvector
// matrices -- the LAPACK of the reference's own calls, moved next to the data, not a
// reimplementation: rocBLAS / rocSOLVER are bound at run time (dlopen), so the library loads
// without them and these calls return OFR_E_UNSUPPORTED.
//
// Symmetric input in row-major order is the same matrix in column-major order, so the solver
// reads it as is; its eigenvectors come back as the columns of a column-major matrix (= rows
// here) in ascending order and one tiled transpose kernel reverses, transposes and (for the
// generalized problem, as feature.lda_eigen) scales them to unit 2-norm.
#include <dlfcn.h>

#include <mutex>
#include <unordered_map>

#include "ofr_common.h"

namespace ofr {
namespace eig {

typedef void* rb_handle;
typedef int rb_status;   // rocblas_status_success = 0
enum { RB_FILL_LOWER = 122, RB_EVECT_ORIGINAL = 211, RB_EFORM_AX = 221 };

struct Solver {
  void* hb = nullptr;
  void* hs = nullptr;
  rb_status (*create)(rb_handle*) = nullptr;
  rb_status (*set_stream)(rb_handle, hipStream_t) = nullptr;
  rb_status (*syevd)(rb_handle, int, int, int, double*, int, double*, double*, int*) = nullptr;
  rb_status (*sygvd)(rb_handle, int, int, int, int, double*, int, double*, int, double*, double*, int*) = nullptr;
  std::mutex mu;
  std::unordered_map<int, rb_handle> handles;   // one per device, kept for the process
};

static Solver* solver() {
  static Solver s;
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] {
    for (const char* n : {"librocblas.so.5", "librocblas.so", "/opt/rocm/lib/librocblas.so.5"})
      if ((s.hb = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    for (const char* n : {"librocsolver.so.0", "librocsolver.so", "/opt/rocm/lib/librocsolver.so.0"})
      if ((s.hs = dlopen(n, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!s.hb || !s.hs) return;
    s.create = (decltype(s.create))dlsym(s.hb, "rocblas_create_handle");
    s.set_stream = (decltype(s.set_stream))dlsym(s.hb, "rocblas_set_stream");
    s.syevd = (decltype(s.syevd))dlsym(s.hs, "rocsolver_dsyevd");
    s.sygvd = (decltype(s.sygvd))dlsym(s.hs, "rocsolver_dsygvd");
    ok = s.create && s.set_stream && s.syevd && s.sygvd;
  });
  return ok ? &s : nullptr;
}

static int handle_for(Solver* s, hipStream_t stream, rb_handle* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_status(e, "hipGetDevice");
  std::lock_guard<std::mutex> g(s->mu);
  auto it = s->handles.find(dev);
  if (it == s->handles.end()) {
    rb_handle h = nullptr;
    if (s->create(&h) != 0) return fail(OFR_E_UNSUPPORTED, "rocblas_create_handle failed");
    it = s->handles.emplace(dev, h).first;
  }
  if (s->set_stream(it->second, stream) != 0) return fail(OFR_E_UNSUPPORTED, "rocblas_set_stream failed");
  *out = it->second;
  return OFR_OK;
}

// 1 / ||column j|| of the column-major n x n result (eigenvector j is contiguous), or 1
__global__ void __launch_bounds__(256) inv_norms_kernel(const double* V, int64_t ldv, int64_t n, int64_t j0,
                                                       double* inv) {
  const int64_t j = j0 + blockIdx.x;
  const double* v = V + j * ldv;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += v[i] * v[i];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) inv[blockIdx.x] = red[0] > 0.0 ? 1.0 / sqrt(red[0]) : 1.0;
}

// out[i][c] = V[(n-1-c) column][i] * scale[c] for c < m: the m largest, descending, row-major.
// 32 x 32 tiles through LDS: reads along the eigenvector, writes along the output row.
__global__ void __launch_bounds__(256) desc_transpose_kernel(const double* V, int64_t ldv, int64_t n, int64_t m,
                                                            const double* scale, double* out, int64_t ldo) {
  __shared__ double t[32][33];
  const int64_t c0 = (int64_t)blockIdx.y * 32, i0 = (int64_t)blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 8 rows of 32
  for (int r = ty; r < 32; r += 8) {
    const int64_t c = c0 + r, i = i0 + tx;
    if (c < m && i < n) t[r][tx] = V[(n - 1 - c) * ldv + i] * (scale ? scale[c] : 1.0);
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t i = i0 + r, c = c0 + tx;
    if (c < m && i < n) out[i * ldo + c] = t[tx][r];
  }
}

__global__ void desc_values_kernel(const double* w, int64_t n, int64_t m, double* out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < m) out[c] = w[n - 1 - c];
}

static inline size_t up(size_t x) { return (x + 255) & ~(size_t)255; }

struct Ws {
  double* w;
  double* e;
  double* inv;
  int* info;
};

static Ws carve(void* workspace, int64_t n, int64_t m) {
  char* p = (char*)workspace;
  Ws w;
  w.w = (double*)p;
  p += up((size_t)n * 8);
  w.e = (double*)p;
  p += up((size_t)n * 8);
  w.inv = (double*)p;
  p += up((size_t)std::max<int64_t>(m, 1) * 8);
  w.info = (int*)p;
  return w;
}

static int finish(hipStream_t st, const Ws& w, double* A, int64_t n, int64_t m, bool unit, double* evals,
                  double* evecs, int64_t ldv, const char* what) {
  int info = 0;
  hipError_t e = hipMemcpyAsync(&info, w.info, sizeof(int), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_status(e, what);
  if (info != 0)
    return fail(OFR_E_NUMERIC, std::string(what) + ": info = " + std::to_string(info) +
                                   (info > 0 ? " (not positive definite / no convergence)" : ""));
  if (m == 0) return OFR_OK;
  if (unit) {
    // inv[b] = 1 / ||eigenvector n-m+b|| (ascending); output column c holds eigenvector n-1-c,
    // i.e. scale[c] = inv[m-1-c]: reversed into the solver's E array (free after the solve)
    hipLaunchKernelGGL(inv_norms_kernel, dim3((unsigned)m), dim3(256), 0, st, A, n, n, n - m, w.inv);
    OFR_LAUNCH_CHECK("inv_norms_kernel");
    hipLaunchKernelGGL(desc_values_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, st, w.inv, m, m, w.e);
    OFR_LAUNCH_CHECK("desc_values_kernel");
  }
  hipLaunchKernelGGL(desc_transpose_kernel, dim3((unsigned)cdiv(n, 32), (unsigned)cdiv(m, 32)), dim3(256), 0, st, A, n,
                     n, m, unit ? (const double*)w.e : nullptr, evecs, ldv);
  OFR_LAUNCH_CHECK("desc_transpose_kernel");
  hipLaunchKernelGGL(desc_values_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, st, w.w, n, m, evals);
  OFR_LAUNCH_CHECK("desc_values_kernel");
  return OFR_OK;
}

}  // namespace eig
}  // namespace ofr

using namespace ofr;

extern "C" size_t ofr_eig_workspace_bytes(int64_t n, int64_t m) {
  return 2 * eig::up((size_t)std::max<int64_t>(n, 1) * 8) + eig::up((size_t)std::max<int64_t>(m, 1) * 8) + 256;
}

extern "C" int ofr_eigh_f64(void* stream, int64_t n, double* A, int64_t m, double* evals, double* evecs, int64_t ldv,
                            void* workspace, size_t workspace_bytes) {
  OFR_CHECK_ARG(n >= 1 && n < (1LL << 31) && m >= 0 && m <= n && ldv >= std::max<int64_t>(m, 1),
                "ofr_eigh_f64: bad sizes");
  OFR_CHECK_ARG(A && evals && (evecs || m == 0) && workspace, "ofr_eigh_f64: null pointer");
  OFR_CHECK_ARG(workspace_bytes >= ofr_eig_workspace_bytes(n, m), "ofr_eigh_f64: workspace too small");
  eig::Solver* s = eig::solver();
  if (!s) return fail(OFR_E_UNSUPPORTED, "ofr_eigh_f64: rocBLAS / rocSOLVER not found");
  hipStream_t st = (hipStream_t)stream;
  eig::rb_handle h;
  int rc = eig::handle_for(s, st, &h);
  if (rc) return rc;
  const eig::Ws w = eig::carve(workspace, n, m);
  if (s->syevd(h, eig::RB_EVECT_ORIGINAL, eig::RB_FILL_LOWER, (int)n, A, (int)n, w.w, w.e, w.info) != 0)
    return fail(OFR_E_UNSUPPORTED, "rocsolver_dsyevd rejected the call");
  return eig::finish(st, w, A, n, m, false, evals, evecs, ldv, "rocsolver_dsyevd");
}

extern "C" int ofr_sygv_f64(void* stream, int64_t n, double* Sb, double* Sw, int64_t m, double* evals, double* evecs,
                            int64_t ldv, void* workspace, size_t workspace_bytes) {
  OFR_CHECK_ARG(n >= 1 && n < (1LL << 31) && m >= 0 && m <= n && ldv >= std::max<int64_t>(m, 1),
                "ofr_sygv_f64: bad sizes");
  OFR_CHECK_ARG(Sb && Sw && evals && (evecs || m == 0) && workspace, "ofr_sygv_f64: null pointer");
  OFR_CHECK_ARG(workspace_bytes >= ofr_eig_workspace_bytes(n, m), "ofr_sygv_f64: workspace too small");
  eig::Solver* s = eig::solver();
  if (!s) return fail(OFR_E_UNSUPPORTED, "ofr_sygv_f64: rocBLAS / rocSOLVER not found");
  hipStream_t st = (hipStream_t)stream;
  eig::rb_handle h;
  int rc = eig::handle_for(s, st, &h);
  if (rc) return rc;
  const eig::Ws w = eig::carve(workspace, n, m);
  if (s->sygvd(h, eig::RB_EFORM_AX, eig::RB_EVECT_ORIGINAL, eig::RB_FILL_LOWER, (int)n, Sb, (int)n, Sw, (int)n, w.w,
               w.e, w.info) != 0)
    return fail(OFR_E_UNSUPPORTED, "rocsolver_dsygvd rejected the call");
  return eig::finish(st, w, Sb, n, m, true, evals, evecs, ldv, "rocsolver_dsygvd");
}
