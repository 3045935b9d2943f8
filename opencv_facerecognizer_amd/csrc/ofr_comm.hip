// Multi-GPU search inside the library: one process driving every GPU of the node, RCCL over xGMI.
//
// The reference has no parallelism; SURVEY §8b/§8e specify the sharded search: the
// gallery rows are sharded over the GPUs, every GPU computes the local top-k of the whole query
// batch, and ONE all-gather of the (distance, index) lists is followed by a merge.  The Python
// package does this with one process per GPU over torch.distributed (parallel.py); these entry
// points give a C / C++ caller the same path without Python: ofr_comm_init_all
// (ncclCommInitAll, one rank per device) and ofr_knn_sharded.
//
// ofr_knn_sharded, per device r (its own stream):
//   1. ofr_knn_f6 phase 1 on shard r (the certified fp6 tier's tile pass), then the split merge
//      (ofr_knn_f6_merge_pruned): stage 1 bounds each query's best-k squared distances from above,
//      one grouped all-gather of those bounds, kth_bound_kernel takes per query the k-th smallest
//      over the shards (an upper bound of the global k-th squared distance), stage 2 re-ranks only
//      the candidates that can fall below it -- local top-k with exact fp64 distances and global
//      row indices, and a lower bound of the squared distance of every local row outside the
//      candidates (-inf when the rank's sieve bucket overflowed);
//   2. pack [B][2k+1] doubles (distances, indices bit-copied, bound) and ncclAllGather them;
//   3. merge_certify_kernel: the global top-k of the ndev lists per query, certified iff the global
//      k-th squared distance is below every rank's bound (a -inf bound never certifies);
//   4. uncertified queries (host reads the certificate): their rows are gathered and go down the
//      single-GPU search's tier chain on every shard -- two-slice fp6 (f6x2), two-slice int8, then
//      the exact fp32 pass (ofr_knn_f32) -- each stage all-gathered, merged and certified again, so
//      the result is the exact fp64 top-k of the whole gallery (classifier.py:104-119) on every
//      device.
// RCCL is bound at run time (dlopen of librccl.so.1, the soname torch's own copy also carries), so
// the library loads and the single-GPU path works where RCCL is absent.
#include <dlfcn.h>

#include <vector>

#include "ofr_common.h"
#include "ofr_topk.h"

typedef struct ncclComm* ncclComm_t;
typedef int ncclResult_t;   // ncclSuccess = 0
enum { OFR_NCCL_UINT8 = 1 };   // ncclUint8 / ncclChar

struct ofr_comm {
  int ndev;
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
};

namespace ofr {
namespace comm {

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

static Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
      if (r.h) break;
    }
    if (r.h) {
      r.CommInitAll = (decltype(r.CommInitAll))dlsym(r.h, "ncclCommInitAll");
      r.CommDestroy = (decltype(r.CommDestroy))dlsym(r.h, "ncclCommDestroy");
      r.AllGather = (decltype(r.AllGather))dlsym(r.h, "ncclAllGather");
      r.GroupStart = (decltype(r.GroupStart))dlsym(r.h, "ncclGroupStart");
      r.GroupEnd = (decltype(r.GroupEnd))dlsym(r.h, "ncclGroupEnd");
      r.GetErrorString = (decltype(r.GetErrorString))dlsym(r.h, "ncclGetErrorString");
    }
  }
  const bool ok = r.h && r.CommInitAll && r.CommDestroy && r.AllGather && r.GroupStart && r.GroupEnd;
  return ok ? &r : nullptr;
}

static int nccl_status(ncclResult_t e, const char* where) {
  if (e == 0) return OFR_OK;
  Rccl* r = rccl();
  std::string msg = std::string(where) + ": " + (r && r->GetErrorString ? r->GetErrorString(e) : "RCCL error");
  set_error(msg);
  return 1000 + (int)e;   // positive: passthrough (hipError_t / ncclResult_t space)
}

// [B][2k+1] doubles: the k distances, the k indices (bit-copied), the bound (or +inf)
__global__ void pack_kernel(const double* d, const int64_t* i, const double* bound, int64_t B, int k, double* out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double* o = out + b * (2 * k + 1);
  for (int j = 0; j < k; ++j) {
    o[j] = d[b * k + j];
    o[k + j] = __longlong_as_double((long long)i[b * k + j]);
  }
  o[2 * k] = bound ? bound[b] : __builtin_inf();
}

// one thread per query: best k of the P gathered lists by (distance, index); cert = the global
// k-th squared distance below every list's bound (+inf = every row of that rank was a candidate)
__global__ void merge_certify_kernel(const double* in, int P, int64_t B, int k, double* out_d, int64_t* out_i,
                                     int* cert, const int64_t* rows) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double bd[OFR_MAX_K];
  int64_t bi[OFR_MAX_K];
  for (int j = 0; j < k; ++j) {
    bd[j] = __builtin_inf();
    bi[j] = -1;
  }
  double minb = __builtin_inf();
  for (int p = 0; p < P; ++p) {
    const double* l = in + ((int64_t)p * B + b) * (2 * k + 1);
    minb = fmin(minb, l[2 * k]) ;
    if (l[2 * k] != l[2 * k]) minb = -__builtin_inf();   // NaN bound: no bound
    for (int j = 0; j < k; ++j) {
      const double x = l[j];
      const int64_t xi = (int64_t)__double_as_longlong(l[k + j]);
      if (xi < 0) continue;
      if (!nan_last_before(x, xi, bd[k - 1], bi[k - 1] < 0 ? INT64_MAX : bi[k - 1])) continue;
      int s = k - 1;
      while (s > 0 && nan_last_before(x, xi, bd[s - 1], bi[s - 1] < 0 ? INT64_MAX : bi[s - 1])) {
        bd[s] = bd[s - 1];
        bi[s] = bi[s - 1];
        --s;
      }
      bd[s] = x;
      bi[s] = xi;
    }
  }
  const int64_t ob = rows ? rows[b] : b;
  for (int j = 0; j < k; ++j) {
    out_d[ob * k + j] = bd[j];
    out_i[ob * k + j] = bi[j];
  }
  if (cert) {
    const double kth = bd[k - 1];
    cert[ob] = (minb == __builtin_inf()) || (kth * kth < minb);
  }
}

// ub[q] = the k-th smallest of the P x k upper bounds all[p][q][0..k) (ascending per p)
__global__ void kth_bound_kernel(const double* all, int P, int64_t B, int k, double* ub) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  double best[OFR_MAX_K];
  for (int j = 0; j < k; ++j) best[j] = __builtin_inf();
  for (int p = 0; p < P; ++p)
    for (int j = 0; j < k; ++j) {
      const double v = all[((int64_t)p * B + q) * k + j];
      if (!(v < best[k - 1])) break;   // ascending: the rest of this shard's list is no better
      int t = k - 1;
      while (t > 0 && best[t - 1] > v) {
        best[t] = best[t - 1];
        --t;
      }
      best[t] = v;
    }
  ub[q] = best[k - 1];
}

// rows[0 .. count) = the b with cert[b] == 0, ascending (one workgroup: a block-wide prefix sum per
// 1024-query chunk); count[0] = their number
__global__ void __launch_bounds__(1024) open_rows_kernel(const int* cert, int64_t B, int64_t* rows, int* count) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) base = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < B; c0 += 1024) {
    const int64_t b = c0 + t;
    const int open = b < B && cert[b] == 0;
    const unsigned long long m = __ballot(open);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[w] = __popcll(m);
    __syncthreads();
    int off = base;
    for (int j = 0; j < w; ++j) off += wsum[j];
    if (open) rows[off + before] = b;
    __syncthreads();
    if (t == 0) {
      int tot = 0;
      for (int j = 0; j < 16; ++j) tot += wsum[j];
      base += tot;
    }
    __syncthreads();
  }
  if (t == 0) count[0] = base;
}

__global__ void gather_rows_kernel(const float* Q, int64_t ldq, const int64_t* rows, int64_t n, float* out) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const float* src = Q + rows[r] * ldq;
  for (int64_t j = threadIdx.x; j < ldq; j += blockDim.x) out[r * ldq + j] = src[j];
}

struct WsLayout {
  size_t knn, loc_d, loc_i, bound, send, recv, sub_q, rows, ubl, ubr, ub, qt1, qt2, qscale, qstats, q8, scert,
      tiles_bytes, total;
};

// per shard: the tier passes' workspace, the local lists, the packed exchange buffers, the open
// queries' rows and their quantized forms (sized for the whole batch; d <= ldq bounds the tiles)
static WsLayout layout(int64_t B, int64_t N, int64_t ldq, int k, int ndev) {
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  WsLayout w{};
  size_t off = 0;
  const size_t knn = std::max({ofr_knn_f6_workspace_bytes(B, N), ofr_knn_workspace_bytes(B, N, k),
                               ofr_knn_q8_workspace_bytes(B, N)});
  w.knn = off; off += up(knn);
  w.loc_d = off; off += up((size_t)B * k * 8);
  w.loc_i = off; off += up((size_t)B * k * 8);
  w.bound = off; off += up((size_t)B * 8);
  w.send = off; off += up((size_t)B * (2 * k + 1) * 8);
  w.recv = off; off += up((size_t)ndev * B * (2 * k + 1) * 8);
  w.sub_q = off; off += up((size_t)B * ldq * 4);
  w.rows = off; off += up((size_t)B * 8);
  w.ubl = off; off += up((size_t)B * k * 8);
  w.ubr = off; off += up((size_t)ndev * B * k * 8);
  w.ub = off; off += up((size_t)B * 8);
  w.tiles_bytes = ofr_f6_tiles_bytes(B, ldq);
  w.qt1 = off; off += up(w.tiles_bytes);
  w.qt2 = off; off += up(w.tiles_bytes);
  w.qscale = off; off += up((size_t)B * 4);
  w.qstats = off; off += up((size_t)B * 3 * 8);
  w.q8 = off; off += up((size_t)B * 2 * round_up(ldq, 64));
  w.scert = off; off += up((size_t)B * 4);
  w.total = off;
  return w;
}

// synchronises every shard's stream when the scope ends while armed (an early error return must
// not free host vectors that asynchronous uploads may still read)
struct SyncAll {
  const ofr_comm* c;
  const ofr_knn_shard* shards;
  bool armed = true;
  ~SyncAll() {
    if (!armed) return;
    for (int p = 0; p < c->ndev; ++p)
      if (hipSetDevice(c->devices[p]) == hipSuccess) (void)hipStreamSynchronize((hipStream_t)shards[p].stream);
  }
};

}  // namespace comm
}  // namespace ofr

using namespace ofr;

extern "C" int ofr_comm_init_all(int ndev, const int* devices, ofr_comm** out) {
  OFR_CHECK_ARG(ndev >= 1 && ndev <= 64 && out, "ofr_comm_init_all: bad arguments");
  comm::Rccl* r = comm::rccl();
  if (!r) return fail(OFR_E_UNSUPPORTED, "ofr_comm_init_all: RCCL (librccl.so.1) not found");
  ofr_comm* c = new ofr_comm;
  c->ndev = ndev;
  c->devices.assign(devices ? devices : nullptr, devices ? devices + ndev : nullptr);
  if (!devices)
    for (int i = 0; i < ndev; ++i) c->devices.push_back(i);
  c->comms.resize(ndev);
  const int rc = comm::nccl_status(r->CommInitAll(c->comms.data(), ndev, c->devices.data()), "ncclCommInitAll");
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return OFR_OK;
}

extern "C" int ofr_comm_destroy(ofr_comm* c) {
  if (!c) return OFR_OK;
  comm::Rccl* r = comm::rccl();
  int rc = OFR_OK;
  if (r)
    for (auto cm : c->comms)
      if (cm && !rc) rc = comm::nccl_status(r->CommDestroy(cm), "ncclCommDestroy");
  delete c;
  return rc;
}

extern "C" int ofr_comm_size(const ofr_comm* c) { return c ? c->ndev : 0; }

extern "C" size_t ofr_knn_sharded_workspace_bytes(int64_t B, int64_t N, int64_t ldq, int k, int ndev) {
  return comm::layout(B, N, ldq, k, ndev).total;
}

extern "C" int ofr_topk_pack(void* stream, const double* d, const int64_t* i, const double* bound, int64_t B, int k,
                             double* out) {
  OFR_CHECK_ARG(B >= 0 && k >= 1 && k <= OFR_MAX_K, "ofr_topk_pack: bad sizes");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(d && i && out, "ofr_topk_pack: null pointer");
  hipLaunchKernelGGL(comm::pack_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, d, i, bound, B,
                     k, out);
  OFR_LAUNCH_CHECK("pack_kernel");
  return OFR_OK;
}

extern "C" int ofr_kth_bound(void* stream, const double* all, int P, int64_t B, int k, double* ub) {
  OFR_CHECK_ARG(P >= 1 && B >= 0 && k >= 1 && k <= OFR_MAX_K, "ofr_kth_bound: bad sizes");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(all && ub, "ofr_kth_bound: null pointer");
  hipLaunchKernelGGL(comm::kth_bound_kernel, dim3((unsigned)cdiv(B, 128)), dim3(128), 0, (hipStream_t)stream, all, P, B,
                     k, ub);
  OFR_LAUNCH_CHECK("kth_bound_kernel");
  return OFR_OK;
}

extern "C" int ofr_open_rows(void* stream, const int* cert, int64_t B, int64_t* rows, int* count) {
  OFR_CHECK_ARG(B >= 0 && B < 0x7fffffffLL, "ofr_open_rows: bad size");
  OFR_CHECK_ARG(cert && rows && count, "ofr_open_rows: null pointer");
  hipLaunchKernelGGL(comm::open_rows_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, cert, B, rows, count);
  OFR_LAUNCH_CHECK("open_rows_kernel");
  return OFR_OK;
}

extern "C" int ofr_topk_merge_certify(void* stream, const double* lists, int P, int64_t B, int k, double* out_d,
                                      int64_t* out_i, int* cert) {
  OFR_CHECK_ARG(P >= 1 && B >= 0 && k >= 1 && k <= OFR_MAX_K, "ofr_topk_merge_certify: bad sizes");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(lists && out_d && out_i, "ofr_topk_merge_certify: null pointer");
  hipLaunchKernelGGL(comm::merge_certify_kernel, dim3((unsigned)cdiv(B, 128)), dim3(128), 0, (hipStream_t)stream,
                     lists, P, B, k, out_d, out_i, cert, (const int64_t*)nullptr);
  OFR_LAUNCH_CHECK("merge_certify_kernel");
  return OFR_OK;
}

extern "C" int ofr_knn_sharded(ofr_comm* c, const ofr_knn_shard* shards, int64_t B, int64_t d, int k) {
  OFR_CHECK_ARG(c && shards, "ofr_knn_sharded: null argument");
  OFR_CHECK_ARG(B >= 0 && d >= 1 && k >= 1 && k <= OFR_MAX_K, "ofr_knn_sharded: bad sizes");
  if (B == 0) return OFR_OK;
  comm::Rccl* r = comm::rccl();
  if (!r) return fail(OFR_E_UNSUPPORTED, "ofr_knn_sharded: RCCL not found");
  const int P = c->ndev;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) cur = c->devices[0];
  struct Restore {
    int dev;
    ~Restore() { (void)hipSetDevice(dev); }
  } restore{cur};
  std::vector<comm::WsLayout> L(P);
  const size_t row_bytes = (size_t)(2 * k + 1) * 8;
  // the prefix tier first (round 6): the same pstages on every shard, with its tiles and terms
  const int pst = shards[0].pstages;
  for (int p = 0; p < P; ++p) {
    const ofr_knn_shard& s = shards[p];
    OFR_CHECK_ARG(s.pstages == pst, "ofr_knn_sharded: pstages differs between shards (choose it from all-reduced sums)");
    OFR_CHECK_ARG(pst == 0 || (s.Qtp && s.qscalep && s.qstatsp && s.paux && s.spaux && s.St && s.Gtp && s.gscalep &&
                               s.gmaxp),
                  "ofr_knn_sharded: the prefix tier needs Qtp, qscalep, qstatsp, paux, spaux, its gallery tiles Gtp, "
                  "gscalep, gmaxp and the row sample St");
  }
  OFR_CHECK_ARG(pst >= 0 && pst <= cdiv(d, 128), "ofr_knn_sharded: pstages must be in [0, ceil(d / 128)]");
  const bool prefix = pst > 0 && pst < cdiv(d, 128);   // a prefix of every stage is the fp6 tier itself
  // 1: the first tier's tile pass (fp6, or the prefix tier) and the merge's selection + upper bounds on
  //    every shard
  for (int p = 0; p < P; ++p) {
    const ofr_knn_shard& s = shards[p];
    hipError_t e = hipSetDevice(c->devices[p]);
    if (e != hipSuccess) return hip_status(e, "hipSetDevice");
    L[p] = comm::layout(B, s.N, s.ldq, k, P);
    OFR_CHECK_ARG(s.workspace && s.workspace_bytes >= L[p].total, "ofr_knn_sharded: workspace too small");
    char* ws = (char*)s.workspace;
    int rc;
    if (prefix) {
      rc = ofr_knn_f6p_sampled(s.stream, 1, s.Q, B, s.ldq, s.Qtp, s.qscalep, s.qstatsp, s.G, s.N, s.ldg, d, s.Gtp,
                               s.gscalep, s.paux, s.gmaxp, k, s.index_base, nullptr, nullptr, nullptr, nullptr, s.St, s.Ns,
                               s.sscale, s.spaux, ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N), s.bscale, pst);
      if (rc) return rc;
      rc = ofr_knn_f6p_merge_pruned(s.stream, 1, s.Q, B, s.ldq, s.Qtp, s.qscalep, s.qstatsp, s.G, s.N, s.ldg, d, s.Gtp,
                                    s.gscalep, s.paux, s.gmaxp, k, s.index_base, nullptr, nullptr, nullptr, nullptr,
                                    (double*)(ws + L[p].ubl), ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N), pst);
      if (rc) return rc;
      continue;
    }
    rc = s.St ? ofr_knn_f6_sampled(s.stream, 1, s.Q, B, s.ldq, s.Qt, s.qscale, s.qstats, s.G, s.N, s.ldg, d, s.Gt,
                                   s.gscale, s.aux, s.gmax, k, s.index_base, nullptr, nullptr, nullptr, nullptr, s.St,
                                   s.Ns, s.sscale, s.saux, ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N), s.bscale)
              : ofr_knn_f6(s.stream, 1, s.Q, B, s.ldq, s.Qt, s.qscale, s.qstats, s.G, s.N, s.ldg, d, s.Gt, s.gscale,
                           s.aux, s.gmax, k, s.index_base, nullptr, nullptr, nullptr, nullptr, ws + L[p].knn,
                           ofr_knn_f6_workspace_bytes(B, s.N), s.bscale);
    if (rc) return rc;
    rc = ofr_knn_f6_merge_pruned(s.stream, 1, s.Q, B, s.ldq, s.Qt, s.qscale, s.qstats, s.G, s.N, s.ldg, d, s.Gt,
                                 s.gscale, s.aux, s.gmax, k, s.index_base, nullptr, nullptr, nullptr, nullptr,
                                 (double*)(ws + L[p].ubl), ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N));
    if (rc) return rc;
  }
  // 2: one grouped all-gather of the bounds; per query the k-th smallest = the global bound;
  //    the pruned exact re-rank on every shard, pack
  {
    int rc = comm::nccl_status(r->GroupStart(), "ncclGroupStart");
    if (rc) return rc;
    for (int p = 0; p < P; ++p) {
      char* ws = (char*)shards[p].workspace;
      rc = comm::nccl_status(r->AllGather(ws + L[p].ubl, ws + L[p].ubr, (size_t)B * k * 8, OFR_NCCL_UINT8,
                                          c->comms[p], (hipStream_t)shards[p].stream),
                             "ncclAllGather");
      if (rc) {
        r->GroupEnd();
        return rc;
      }
    }
    rc = comm::nccl_status(r->GroupEnd(), "ncclGroupEnd");
    if (rc) return rc;
  }
  for (int p = 0; p < P; ++p) {
    const ofr_knn_shard& s = shards[p];
    hipError_t e = hipSetDevice(c->devices[p]);
    if (e != hipSuccess) return hip_status(e, "hipSetDevice");
    char* ws = (char*)s.workspace;
    double* ld_ = (double*)(ws + L[p].loc_d);
    int64_t* li_ = (int64_t*)(ws + L[p].loc_i);
    double* lb_ = (double*)(ws + L[p].bound);
    int* lc_ = s.cert;   // local certificates land in the caller's cert, overwritten by the merge
    double* ub = (double*)(ws + L[p].ub);
    hipLaunchKernelGGL(comm::kth_bound_kernel, dim3((unsigned)cdiv(B, 128)), dim3(128), 0, (hipStream_t)s.stream,
                       (const double*)(ws + L[p].ubr), P, B, k, ub);
    OFR_LAUNCH_CHECK("kth_bound_kernel");
    int rc = prefix ? ofr_knn_f6p_merge_pruned(s.stream, 2, s.Q, B, s.ldq, s.Qtp, s.qscalep, s.qstatsp, s.G, s.N,
                                               s.ldg, d, s.Gtp, s.gscalep, s.paux, s.gmaxp, k, s.index_base, ld_, li_,
                                               lc_, lb_, ub, ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N), pst)
                    : ofr_knn_f6_merge_pruned(s.stream, 2, s.Q, B, s.ldq, s.Qt, s.qscale, s.qstats, s.G, s.N, s.ldg, d,
                                              s.Gt, s.gscale, s.aux, s.gmax, k, s.index_base, ld_, li_, lc_, lb_, ub,
                                              ws + L[p].knn, ofr_knn_f6_workspace_bytes(B, s.N));
    if (rc) return rc;
    hipLaunchKernelGGL(comm::pack_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, (hipStream_t)s.stream, ld_, li_,
                       lb_, B, k, (double*)(ws + L[p].send));
    OFR_LAUNCH_CHECK("pack_kernel");
  }
  // 3: one all-gather of the packed lists, then merge + global certificate on every device
  auto exchange = [&](int64_t n, const int64_t* const* rows_dev, bool certify) -> int {
    int rc = comm::nccl_status(r->GroupStart(), "ncclGroupStart");
    if (rc) return rc;
    for (int p = 0; p < P; ++p) {
      char* ws = (char*)shards[p].workspace;
      rc = comm::nccl_status(r->AllGather(ws + L[p].send, ws + L[p].recv, (size_t)n * row_bytes, OFR_NCCL_UINT8,
                                          c->comms[p], (hipStream_t)shards[p].stream),
                             "ncclAllGather");
      if (rc) {
        r->GroupEnd();
        return rc;
      }
    }
    rc = comm::nccl_status(r->GroupEnd(), "ncclGroupEnd");
    if (rc) return rc;
    for (int p = 0; p < P; ++p) {
      const ofr_knn_shard& s = shards[p];
      const hipError_t se = hipSetDevice(c->devices[p]);
      if (se != hipSuccess) return hip_status(se, "hipSetDevice");
      char* ws = (char*)s.workspace;
      hipLaunchKernelGGL(comm::merge_certify_kernel, dim3((unsigned)cdiv(n, 128)), dim3(128), 0, (hipStream_t)s.stream,
                         (const double*)(ws + L[p].recv), P, n, k, s.out_d, s.out_i, certify ? s.cert : nullptr,
                         rows_dev ? rows_dev[p] : (const int64_t*)nullptr);
      OFR_LAUNCH_CHECK("merge_certify_kernel");
    }
    return OFR_OK;
  };
  int rc = exchange(B, nullptr, true);
  if (rc) return rc;
  // 4: the queries the first tier left open go down the chain on every shard: (after the prefix tier:
  //    fp6,) f6x2, int8 x2, exact fp32; each stage searches their rows, exchanges the lists (with its
  //    bound) and certifies again
  enum Stage { F6 = 0, F6X2 = 1, Q8X2 = 2, F32 = 3 };
  bool have_f6x2 = true, have_q8x2 = true;
  for (int p = 0; p < P; ++p) {
    have_f6x2 = have_f6x2 && shards[p].Gt2 && shards[p].gscale2 && shards[p].gmax2;
    have_q8x2 = have_q8x2 && shards[p].G8 && shards[p].gscale8 && shards[p].gmax8 &&
                shards[p].ld8 >= 2 * round_up(d, 64) && shards[p].ld8 <= 2 * round_up(shards[p].ldq, 64);
  }
  int64_t* counts = shards[0].tier_counts;
  if (counts)
    for (int j = 0; j < 4; ++j) counts[j] = -1;
  comm::SyncAll guard{c, shards};
  std::vector<int> cert((size_t)B);
  std::vector<int64_t> rows((size_t)B);
  for (int64_t b = 0; b < B; ++b) rows[(size_t)b] = b;
  int64_t n = B;
  auto open_rows = [&]() -> int {   // rows whose certificate (device 0's copy) is 0, in place
    hipError_t e = hipSetDevice(c->devices[0]);
    if (e == hipSuccess)
      e = hipMemcpyAsync(cert.data(), shards[0].cert, (size_t)B * 4, hipMemcpyDeviceToHost, (hipStream_t)shards[0].stream);
    for (int p = 0; p < P && e == hipSuccess; ++p) {   // every stream done with the rows uploaded from `rows`
      e = hipSetDevice(c->devices[p]);
      if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)shards[p].stream);
    }
    if (e != hipSuccess) return hip_status(e, "ofr_knn_sharded: certificate readback");
    int64_t m = 0;
    for (int64_t j = 0; j < n; ++j)
      if (!cert[(size_t)rows[(size_t)j]]) rows[(size_t)m++] = rows[(size_t)j];
    n = m;
    return OFR_OK;
  };
  rc = open_rows();
  if (rc) return rc;
  if (prefix) {
    if (shards[0].prefix_open) shards[0].prefix_open[0] = n;
  } else if (counts) {
    counts[0] = n;
  }
  for (int stage : {(int)F6, (int)F6X2, (int)Q8X2, (int)F32}) {
    if (stage == F6 && !prefix) continue;
    if (stage == F6 && n == 0 && counts) counts[0] = 0;
    if (n == 0) break;
    if (stage == F6X2 && !have_f6x2) continue;
    if (stage == Q8X2 && !have_q8x2) continue;
    if (stage != F32 && n <= 32) continue;   // a handful of queries: the exact streaming pass is as cheap
    std::vector<const int64_t*> rows_dev(P);
    for (int p = 0; p < P; ++p) {
      const ofr_knn_shard& s = shards[p];
      hipError_t e = hipSetDevice(c->devices[p]);
      if (e != hipSuccess) return hip_status(e, "hipSetDevice");
      const hipStream_t st = (hipStream_t)s.stream;
      char* ws = (char*)s.workspace;
      int64_t* rd = (int64_t*)(ws + L[p].rows);
      e = hipMemcpyAsync(rd, rows.data(), (size_t)n * 8, hipMemcpyHostToDevice, st);
      if (e != hipSuccess) return hip_status(e, "ofr_knn_sharded: rows upload");
      rows_dev[p] = rd;
      float* sq = (float*)(ws + L[p].sub_q);
      hipLaunchKernelGGL(comm::gather_rows_kernel, dim3((unsigned)n), dim3(256), 0, st, s.Q, s.ldq, rd, n, sq);
      OFR_LAUNCH_CHECK("gather_rows_kernel");
      double* ld_ = (double*)(ws + L[p].loc_d);
      int64_t* li_ = (int64_t*)(ws + L[p].loc_i);
      double* lb_ = (double*)(ws + L[p].bound);
      int* lc_ = (int*)(ws + L[p].scert);
      float* qs = (float*)(ws + L[p].qscale);
      double* qst = (double*)(ws + L[p].qstats);
      if (stage == F6) {   // the prefix tier's open queries: the fp6 tier on their rows
        rc = ofr_f6_quantize_rows(s.stream, sq, n, d, s.ldq, ws + L[p].qt1, L[p].tiles_bytes, qs, qst, nullptr,
                                  nullptr, s.bscale);
        if (rc) return rc;
        rc = s.St ? ofr_knn_f6_sampled(s.stream, 3, sq, n, s.ldq, ws + L[p].qt1, qs, qst, s.G, s.N, s.ldg, d, s.Gt,
                                       s.gscale, s.aux, s.gmax, k, s.index_base, ld_, li_, lc_, lb_, s.St, s.Ns,
                                       s.sscale, s.saux, ws + L[p].knn, ofr_knn_f6_workspace_bytes(n, s.N), s.bscale)
                  : ofr_knn_f6(s.stream, 3, sq, n, s.ldq, ws + L[p].qt1, qs, qst, s.G, s.N, s.ldg, d, s.Gt, s.gscale,
                               s.aux, s.gmax, k, s.index_base, ld_, li_, lc_, lb_, ws + L[p].knn,
                               ofr_knn_f6_workspace_bytes(n, s.N), s.bscale);
      } else if (stage == F6X2) {
        rc = ofr_f6x2_quantize_rows(s.stream, sq, n, d, s.ldq, ws + L[p].qt1, ws + L[p].qt2, L[p].tiles_bytes, qs, qst,
                                    nullptr, nullptr, s.bscale);
        if (rc) return rc;
        rc = s.St && s.St2
                 ? ofr_knn_f6x2_sampled(s.stream, 3, sq, n, s.ldq, ws + L[p].qt1, ws + L[p].qt2, qs, qst, s.G, s.N,
                                        s.ldg, d, s.Gt, s.Gt2, s.gscale2, s.aux, s.gmax2, k, s.index_base, ld_, li_,
                                        lc_, lb_, s.St, s.St2, s.Ns, s.sscale, s.saux, ws + L[p].knn,
                                        ofr_knn_f6_workspace_bytes(n, s.N), s.bscale)
                 : ofr_knn_f6x2(s.stream, 3, sq, n, s.ldq, ws + L[p].qt1, ws + L[p].qt2, qs, qst, s.G, s.N, s.ldg, d,
                                s.Gt, s.Gt2, s.gscale2, s.aux, s.gmax2, k, s.index_base, ld_, li_, lc_, lb_,
                                ws + L[p].knn, ofr_knn_f6_workspace_bytes(n, s.N), s.bscale);
      } else if (stage == Q8X2) {
        // the query slices share the gallery's row layout (ofr_knn_q8 takes one ld for both)
        rc = ofr_q8_quantize_rows(s.stream, 2, sq, n, d, s.ldq, (int8_t*)(ws + L[p].q8), s.ld8, qs, qst, nullptr,
                                  nullptr);
        if (rc) return rc;
        rc = ofr_knn_q8(s.stream, 3, 2, sq, n, s.ldq, (const int8_t*)(ws + L[p].q8), qs, qst, s.G, s.N, s.ldg, d, s.G8,
                        s.ld8, s.gscale8, s.aux, s.gmax8, k, s.index_base, ld_, li_, lc_, lb_, ws + L[p].knn,
                        ofr_knn_q8_workspace_bytes(n, s.N));
      } else {
        rc = ofr_knn_f32(s.stream, OFR_METRIC_EUCLIDEAN, sq, n, s.ldq, s.G, s.N, s.ldg, d, s.aux, k, s.index_base, ld_,
                         li_, ws + L[p].knn, ofr_knn_workspace_bytes(n, s.N, k));
      }
      if (rc) return rc;
      hipLaunchKernelGGL(comm::pack_kernel, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, st, ld_, li_,
                         stage == F32 ? (const double*)nullptr : (const double*)lb_, n, k, (double*)(ws + L[p].send));
      OFR_LAUNCH_CHECK("pack_kernel");
    }
    // the exact pass leaves cert 0 on its rows (0 = resolved by the exact tier); a quantized tier
    // writes its global certificate there
    std::vector<const int64_t*> rptr(rows_dev.begin(), rows_dev.end());
    rc = exchange(n, rptr.data(), stage != F32);
    if (rc) return rc;
    if (stage == F32) {
      if (counts) counts[3] = n;
      break;
    }
    rc = open_rows();
    if (rc) return rc;
    if (counts) counts[stage] = n;
  }
  // every device's stream must finish its reads of `rows` (host vector) before it goes out of scope
  for (int p = 0; p < P; ++p) {
    hipError_t e = hipSetDevice(c->devices[p]);
    if (e == hipSuccess) e = hipStreamSynchronize((hipStream_t)shards[p].stream);
    if (e != hipSuccess) return hip_status(e, "ofr_knn_sharded: stream sync");
  }
  guard.armed = false;
  return OFR_OK;
}
