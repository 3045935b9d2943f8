// Any k: the k nearest gallery rows of every query, evaluated exactly in fp64 (round 5).
//
// Replaces NearestNeighbor.predict (reference classifier.py:104-119) for the k the certified tiers
// and the fp32 tile pass do not serve (their candidate lists hold 16 rows per tile): the reference
// returns the k nearest for any k (`np.argsort(distances)[:k]`, :113-119), and all of them when
// k > N.  Two kernels per block of queries:
//   deep_dist_kernel   the reference's distance of every (query, row) pair in fp64 -- Euclidean
//                      sqrt(sum (p - q)^2) (distance.py:57-60), Cosine -p.q / sqrt(p.p q.q)
//                      (:74-77, NaN for a zero row as numpy's 0/0), ChiSquare
//                      sum (p - q)^2 / (p + q + eps) (:112-116) -- on 64 x 64 tiles with the
//                      features staged through LDS (fp32 rows, or count rows / denom: the
//                      reference's float64 histogram values bit for bit);
//   deep_select_kernel per query the k smallest (distance, row) pairs: an 8-pass radix select of
//                      the k-th order key (order-preserving u64 of the distance, NaN last as
//                      argsort puts it), an ordered gather (keys below it, then the lowest rows of
//                      its ties) and a bitonic sort of the <= 4096 survivors in LDS;
//   min(k, N) > 4096   (round 6) a stable segmented radix sort of every query's (key, row) pairs
//                      (rocPRIM), its first k taken: the same order, ties by row.
// Rows past N come back as (+inf, -1), the convention of every search entry point.
// Roofline: fp64 VALU (2 flops per pair and feature for Euclidean / Cosine, ~12 for ChiSquare's
// division) -- a rare path (k > 16), no certificate needed.  Each distance is the reference formula
// in fp64, its terms summed in feature order with fma: within ~1 ulp of numpy's pairwise float64 sum
// (distance.py:60, :115-116), so rows whose reference distances are within an ulp may order
// differently from np.argsort (tests/test_gpu_deep_k.py compares up to such near-ties).
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "ofr_common.h"

namespace ofr {
namespace deep {

constexpr int TQ = 64, TG = 64, KB = 32;   // query x gallery rows per tile, features per LDS step
constexpr int MAXK = 4096;                 // survivors sorted in LDS

template <class T>
__device__ __forceinline__ double load_val(const void* p, int64_t i, double inv_denom, double denom) {
  const double v = (double)reinterpret_cast<const T*>(p)[i];
  return denom == 1.0 ? v : v / denom;   // count / denom, rounded once (numpy's histogram value)
}

__device__ __forceinline__ double val(const void* p, int dt, int64_t i, double denom) {
  switch (dt) {
    case OFR_DT_U8: return load_val<uint8_t>(p, i, 0, denom);
    case OFR_DT_U16: return load_val<uint16_t>(p, i, 0, denom);
    case OFR_DT_U32: return load_val<uint32_t>(p, i, 0, denom);
    case OFR_DT_F64: return load_val<double>(p, i, 0, denom);
    default: return load_val<float>(p, i, 0, denom);
  }
}

struct DistArgs {
  const void* Q;
  int64_t ldq;
  int qdt;
  const void* G;
  int64_t ldg;
  int gdt;
  int64_t d, B, N;
  double denom;
  int metric;
  double* D;   // [B][N]
};

// 256 threads: thread (ty, tx) = (t / 16, t % 16) owns queries ty + 16 i, rows tx + 16 j (i, j < 4).
template <int METRIC>
__global__ void __launch_bounds__(256) deep_dist_kernel(DistArgs a) {
  __shared__ double qs[KB][TQ + 1], gs[KB][TG + 1];
  const int t = threadIdx.x, ty = t >> 4, tx = t & 15;
  const int64_t q0 = (int64_t)blockIdx.y * TQ, g0 = (int64_t)blockIdx.x * TG;
  double acc[4][4], qq[4], gg[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    qq[i] = gg[i] = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
  }
  for (int64_t k0 = 0; k0 < a.d; k0 += KB) {
    // stage KB features of the tile's 64 queries and 64 rows (zeros past d / B / N)
    for (int e = t; e < KB * TQ; e += 256) {
      const int r = e / KB, c = e % KB;
      const int64_t k = k0 + c, q = q0 + r, g = g0 + r;
      qs[c][r] = (k < a.d && q < a.B) ? val(a.Q, a.qdt, q * a.ldq + k, a.denom) : 0.0;
      gs[c][r] = (k < a.d && g < a.N) ? val(a.G, a.gdt, g * a.ldg + k, a.denom) : 0.0;
    }
    __syncthreads();
    const int kn = a.d - k0 < KB ? (int)(a.d - k0) : KB;
    for (int c = 0; c < kn; ++c) {
      double qv[4], gv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        qv[i] = qs[c][ty + 16 * i];
        gv[i] = gs[c][tx + 16 * i];
      }
      if constexpr (METRIC == OFR_METRIC_COSINE) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          qq[i] = fma(qv[i], qv[i], qq[i]);
          gg[i] = fma(gv[i], gv[i], gg[i]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if constexpr (METRIC == OFR_METRIC_EUCLIDEAN) {
            const double df = qv[i] - gv[j];
            acc[i][j] = fma(df, df, acc[i][j]);
          } else if constexpr (METRIC == OFR_METRIC_COSINE) {
            acc[i][j] = fma(qv[i], gv[j], acc[i][j]);
          } else {
            const double df = qv[i] - gv[j];
            acc[i][j] += (df * df) / ((qv[i] + gv[j]) + 2.220446049250313e-16);   // distance.py:115-116
          }
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t q = q0 + ty + 16 * i;
    if (q >= a.B) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t g = g0 + tx + 16 * j;
      if (g >= a.N) continue;
      double v = acc[i][j];
      if constexpr (METRIC == OFR_METRIC_EUCLIDEAN) v = sqrt(v);
      if constexpr (METRIC == OFR_METRIC_COSINE) v = -v / sqrt(qq[i] * gg[j]);   // 0 / 0 = NaN, as numpy
      a.D[q * a.N + g] = v;
    }
  }
}

// order-preserving key of a distance: -0 as +0, NaN above everything (argsort puts it last)
__device__ __forceinline__ uint64_t dkey(double v) {
  if (v != v) return ~0ull;
  if (v == 0.0) v = 0.0;
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double kdist(uint64_t k) {
  if (k == ~0ull) return __longlong_as_double(0x7ff8000000000000ll);
  const uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double((long long)b);
}

// One workgroup per query of the block: out rows [q][k] for the block's queries.
__global__ void __launch_bounds__(256) deep_select_kernel(const double* D, int64_t N, int64_t B, int k,
                                                          int64_t index_base, double* out_d, int64_t* out_i) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t skey[MAXK];
  __shared__ int32_t srow[MAXK];
  __shared__ uint32_t s_sel[2];   // [0] bucket, [1] count below it
  __shared__ int n_lt, n_eq;
  __shared__ uint32_t wsum[4];
  const int64_t q = blockIdx.x;
  if (q >= B) return;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const double* row = D + q * N;
  const int keff = (int64_t)k < N ? k : (int)N;
  uint64_t prefix = 0, mask = 0;
  uint32_t remaining = (uint32_t)keff;   // rank (1-based) of the threshold key among the candidates
  for (int pass = 0; pass < 8 && keff > 0; ++pass) {
    const int shift = 56 - 8 * pass;
    hist[t] = 0;
    __syncthreads();
    for (int64_t j = t; j < N; j += 256) {
      const uint64_t key = dkey(row[j]);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (t == 0) {
      uint32_t cum = 0;
      int b = 0;
      for (; b < 255; ++b) {
        if (cum + hist[b] >= remaining) break;
        cum += hist[b];
      }
      s_sel[0] = (uint32_t)b;
      s_sel[1] = cum;
    }
    __syncthreads();
    prefix |= (uint64_t)s_sel[0] << shift;
    mask |= 0xffull << shift;
    remaining -= s_sel[1];
    __syncthreads();
  }
  // prefix = T, the keff-th smallest key; take every key < T and the `remaining` lowest rows of T
  if (t == 0) {
    n_lt = 0;
    n_eq = 0;
  }
  __syncthreads();
  const int n_below = keff - (int)remaining;
  for (int64_t j0 = 0; j0 < N && keff > 0; j0 += 256) {
    const int64_t j = j0 + t;
    const uint64_t key = j < N ? dkey(row[j]) : ~0ull;
    const bool lt = j < N && key < prefix, eq = j < N && key == prefix;
    if (lt) {
      const int s = atomicAdd(&n_lt, 1);
      skey[s] = key;
      srow[s] = (int32_t)j;
    }
    // ties at T in row order: a block-wide exclusive prefix count of eq
    const uint64_t bal = __ballot(eq);
    const int before_w = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    int base = n_eq;
    for (int w = 0; w < wave; ++w) base += (int)wsum[w];
    const int tot = (int)(wsum[0] + wsum[1] + wsum[2] + wsum[3]);
    if (eq) {
      const int r = base + before_w;
      if (r < (int)remaining) {
        skey[n_below + r] = key;
        srow[n_below + r] = (int32_t)j;
      }
    }
    __syncthreads();
    if (t == 0) n_eq += tot;
    __syncthreads();
    if (n_eq >= (int)remaining && n_lt >= n_below) break;   // uniform: both in LDS after the barrier
  }
  // bitonic sort of keff entries by (key, row), padded to a power of two with (max, max)
  int P2 = 1;
  while (P2 < keff) P2 <<= 1;
  for (int e = keff + t; e < P2; e += 256) {
    skey[e] = ~0ull;
    srow[e] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= P2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int e = t; e < P2; e += 256) {
        const int o = e ^ stride;
        if (o > e) {
          const bool up = (e & size) == 0;
          const uint64_t ka = skey[e], kb = skey[o];
          const int32_t ra = srow[e], rb = srow[o];
          const bool gt = ka > kb || (ka == kb && ra > rb);
          if (gt == up) {
            skey[e] = kb; skey[o] = ka;
            srow[e] = rb; srow[o] = ra;
          }
        }
      }
      __syncthreads();
    }
  for (int e = t; e < k; e += 256) {
    const bool ok = e < keff;
    out_d[q * k + e] = ok ? kdist(skey[e]) : __builtin_inf();
    out_i[q * k + e] = ok ? index_base + srow[e] : -1;
  }
}

// min(k, N) > MAXK: the order keys and rows of a block of queries (in place over the distances)
__global__ void deep_keys_kernel(double* D, int32_t* rows, int64_t n, int64_t N) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t key = dkey(D[i]);
    reinterpret_cast<uint64_t*>(D)[i] = key;
    rows[i] = (int32_t)(i % N);
  }
}
__global__ void deep_take_kernel(const uint64_t* keys, const int32_t* rows, int64_t N, int64_t nb, int k, int keff,
                                 int64_t index_base, double* out_d, int64_t* out_i) {
  const int64_t q = blockIdx.y;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < k; e += gridDim.x * blockDim.x) {
    const bool ok = e < keff;
    out_d[q * k + e] = ok ? kdist(keys[q * N + e]) : __builtin_inf();
    out_i[q * k + e] = ok ? index_base + rows[q * N + e] : -1;
  }
}
__global__ void deep_offsets_kernel(int* off, int64_t nb, int64_t N) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i <= nb) off[i] = (int)(i * N);
}

}  // namespace deep
}  // namespace ofr

using namespace ofr;

// rows of queries per block of the distance matrix: [Bc][N] fp64 in at most 2 GiB (at least one tile)
static int64_t deep_block(int64_t B, int64_t N) {
  int64_t bc = ((int64_t)1 << 31) / (8 * std::max<int64_t>(N, 1));
  bc = bc / deep::TQ * deep::TQ;
  bc = std::max<int64_t>(bc, deep::TQ);
  return std::min<int64_t>(bc, std::max<int64_t>(B, 1));
}

extern "C" size_t ofr_knn_deep_workspace_bytes(int64_t B, int64_t N) {
  return (size_t)deep_block(B, N) * (size_t)std::max<int64_t>(N, 1) * 8 + 256;
}

extern "C" int ofr_knn_deep(void* stream, int metric, const void* Q, int64_t B, int64_t ldq, int qdtype,
                            const void* G, int64_t N, int64_t ldg, int gdtype, int64_t d, double denom, int k,
                            int64_t index_base, double* out_d, int64_t* out_i, void* workspace,
                            size_t workspace_bytes) {
  OFR_CHECK_ARG(metric == OFR_METRIC_EUCLIDEAN || metric == OFR_METRIC_COSINE || metric == OFR_METRIC_CHISQUARE,
                "ofr_knn_deep: unknown metric");
  OFR_CHECK_ARG(B >= 0 && N >= 0 && d >= 1 && ldq >= d && ldg >= d && k >= 1, "ofr_knn_deep: bad sizes");
  OFR_CHECK_ARG(qdtype >= OFR_DT_U8 && qdtype <= OFR_DT_F64 && gdtype >= OFR_DT_U8 && gdtype <= OFR_DT_F64,
                "ofr_knn_deep: bad dtype");
  OFR_CHECK_ARG(denom > 0.0, "ofr_knn_deep: denom must be positive");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(Q && out_d && out_i && (N == 0 || (G && workspace)), "ofr_knn_deep: null pointer");
  OFR_CHECK_ARG(N < 0x7fffffffLL, "ofr_knn_deep: N too large");
  OFR_CHECK_ARG(N == 0 || workspace_bytes >= ofr_knn_deep_workspace_bytes(B, N), "ofr_knn_deep: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const bool sorted = std::min<int64_t>(k, N) > deep::MAXK;
  // the sort path's blocks: a quarter of the distance block (the keys, rows and their sorted copies
  // take 3x its bytes more, allocated per call: this path is rare)
  const int64_t bc = sorted ? std::max<int64_t>(1, std::min(deep_block(B, N) / 4, ((int64_t)1 << 30) / std::max<int64_t>(N, 1)))
                            : deep_block(B, N);
  char* sbuf = nullptr;
  if (sorted) {
    size_t tmp = 0;
    const int64_t n = bc * N;
    hipError_t e = rocprim::segmented_radix_sort_pairs(nullptr, tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                       (const int32_t*)nullptr, (int32_t*)nullptr, (unsigned int)n,
                                                       (unsigned int)bc, (const int*)nullptr, (const int*)nullptr, 0, 64,
                                                       st);
    if (e != hipSuccess) return hip_status(e, "ofr_knn_deep: segmented sort size");
    e = hipMallocAsync((void**)&sbuf, (size_t)n * 16 + (size_t)(bc + 1) * 4 + tmp + 256, st);
    if (e != hipSuccess) return hip_status(e, "ofr_knn_deep: sort buffers");
  }
  struct Free {
    char* p;
    hipStream_t s;
    ~Free() {
      if (p) (void)hipFreeAsync(p, s);
    }
  } free_sbuf{sbuf, st};
  for (int64_t b0 = 0; b0 < B; b0 += bc) {
    const int64_t nb = std::min(bc, B - b0);
    const int esz = qdtype == OFR_DT_U8 ? 1 : qdtype == OFR_DT_U16 ? 2 : qdtype == OFR_DT_F64 ? 8 : 4;
    if (N > 0) {
      deep::DistArgs a{(const char*)Q + b0 * ldq * esz, ldq, qdtype, G, ldg, gdtype, d, nb, N, denom, metric,
                       (double*)workspace};
      const dim3 grid((unsigned)cdiv(N, deep::TG), (unsigned)cdiv(nb, deep::TQ));
      OFR_CHECK_ARG(grid.y < 65536, "ofr_knn_deep: query block too large");
      if (metric == OFR_METRIC_EUCLIDEAN)
        hipLaunchKernelGGL(deep::deep_dist_kernel<OFR_METRIC_EUCLIDEAN>, grid, dim3(256), 0, st, a);
      else if (metric == OFR_METRIC_COSINE)
        hipLaunchKernelGGL(deep::deep_dist_kernel<OFR_METRIC_COSINE>, grid, dim3(256), 0, st, a);
      else
        hipLaunchKernelGGL(deep::deep_dist_kernel<OFR_METRIC_CHISQUARE>, grid, dim3(256), 0, st, a);
      OFR_LAUNCH_CHECK("deep_dist_kernel");
    }
    if (sorted) {
      const int64_t n = nb * N;
      uint64_t* kout = reinterpret_cast<uint64_t*>(sbuf);
      int32_t* rin = reinterpret_cast<int32_t*>(sbuf + (size_t)bc * N * 8);
      int32_t* rout = rin + bc * N;
      int* off = reinterpret_cast<int*>(rout + bc * N);
      void* tmp = reinterpret_cast<char*>(off) + round_up((bc + 1) * 4, 256);
      size_t tmpb = 0;
      hipError_t e = rocprim::segmented_radix_sort_pairs(nullptr, tmpb, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                         (const int32_t*)nullptr, (int32_t*)nullptr, (unsigned int)n,
                                                         (unsigned int)nb, off, off + 1, 0, 64, st);
      if (e != hipSuccess) return hip_status(e, "ofr_knn_deep: segmented sort size");
      hipLaunchKernelGGL(deep::deep_keys_kernel, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 65536)), dim3(256), 0,
                         st, (double*)workspace, rin, n, N);
      OFR_LAUNCH_CHECK("deep_keys_kernel");
      hipLaunchKernelGGL(deep::deep_offsets_kernel, dim3((unsigned)cdiv(nb + 1, 256)), dim3(256), 0, st, off, nb, N);
      OFR_LAUNCH_CHECK("deep_offsets_kernel");
      // stable: equal keys keep their row order (rows ascending in), the ties of np.argsort's order here
      e = rocprim::segmented_radix_sort_pairs(tmp, tmpb, (const uint64_t*)workspace, kout, rin, rout, (unsigned int)n,
                                              (unsigned int)nb, off, off + 1, 0, 64, st);
      if (e != hipSuccess) return hip_status(e, "ofr_knn_deep: segmented sort");
      const int keff = (int)std::min<int64_t>(k, N);
      hipLaunchKernelGGL(deep::deep_take_kernel, dim3((unsigned)cdiv(k, 256), (unsigned)nb), dim3(256), 0, st, kout,
                         rout, N, nb, k, keff, index_base, out_d + b0 * k, out_i + b0 * k);
      OFR_LAUNCH_CHECK("deep_take_kernel");
    } else {
      hipLaunchKernelGGL(deep::deep_select_kernel, dim3((unsigned)nb), dim3(256), 0, st, (const double*)workspace, N,
                         nb, k, index_base, out_d + b0 * k, out_i + b0 * k);
      OFR_LAUNCH_CHECK("deep_select_kernel");
    }
  }
  return OFR_OK;
}
