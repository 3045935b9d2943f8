// Batched k-nearest-neighbour search (Euclidean / Cosine) on gfx950.
//
// Replaces NearestNeighbor.predict (reference classifier.py:76-129): the
// per-gallery-item distance loop :104-108 (EuclideanDistance distance.py:57-60,
// CosineDistance :74-77), argsort :113 and the top-k slice :118-119.
//
// pass 1  knn_tile_kernel   256 gallery rows x 256 queries per workgroup on
//         the fp32 MFMA tile engine; epilogue turns dot products into coarse
//         scores (Euclidean on centred features: ||g||^2 - 2 q.g; Cosine:
//         -(q.g)/||g||) and keeps the best KC (score, row) per query per
//         tile: per-lane insertion over the lane's 64 rows, a bitonic merge
//         with the partner half-wave (shfl_xor 32), and an LDS merge of the
//         two row-halves of the tile.  Candidates: cand[tile][query][KC].
// pass 2  knn_merge_rerank_kernel   one workgroup per query: best R=KC of
//         all tile candidates (per-thread insertion + LDS bitonic tree), then
//         the REFERENCE distance recomputed exactly in fp64 for those R rows
//         (direct (q-g)^2 sum / -q.g/sqrt(q.q g.g)), sorted by (distance,
//         index), best k written as fp64 + int64.
#include <type_traits>
#include "ofr_gemm_tile.h"
#include "ofr_topk.h"

namespace ofr {

struct KnnTileArgs {
  const float* Q;
  int64_t B, ldq;
  const float* G;
  int64_t N, ldg;
  int nk;
  const float* aux;
  Cand* cand;      // [T][B][KC]
  int64_t ntb;     // query tiles
  int64_t ntg;     // gallery tiles
};

template <class C, int METRIC, int KC>
__global__ void __launch_bounds__(256, 1) knn_tile_kernel(KnnTileArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = tile::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t gt = t / p.ntb;  // gallery tile (consecutive t share it)
  const int64_t qt = t % p.ntb;
  const int64_t g0 = gt * tile::TM, q0 = qt * C::TN;

  f32x16 acc[C::RT][C::CT];
  tile::mainloop<C>(smem, p.G, p.ldg, p.N, g0, p.Q, p.ldq, p.B, q0, p.nk, acc);

  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wr = wave / C::WN, wc = wave % C::WN;
  const int h = lane >> 5;
  Cand* buf = reinterpret_cast<Cand*>(smem);  // [WM][TN][KC]

  // gallery aux of the tile staged once in LDS (past the candidate buffer): keeps
  // the epilogue free of per-element global loads and of a 16*RT register table
  float* gtab = reinterpret_cast<float*>(smem + C::LDS - tile::TM * 4);
  static_assert((size_t)C::WM * C::TN * KC * sizeof(Cand) + tile::TM * 4 <= (size_t)C::LDS, "epilogue LDS");
  {
    const int64_t g = g0 + threadIdx.x;
    gtab[threadIdx.x] = g < p.N ? p.aux[g] : __builtin_nanf("");
  }
  __syncthreads();

  // one instantiation per query block: a constant ct keeps acc[][ct] in registers
  auto epi = [&](auto ctc) {
    constexpr int ct = decltype(ctc)::value;
    TopList<KC> L;
    L.init();
#pragma unroll
    for (int rt = 0; rt < C::RT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gl = wr * (C::RT * 32) + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float dot = acc[rt][ct][r];
        const float ga = gtab[gl];
        float s;
        if (METRIC == OFR_METRIC_EUCLIDEAN) s = __builtin_fmaf(-2.f, dot, ga);
        else s = -dot * ga;
        L.insert(s, (int)(g0 + gl));   // NaN (masked rows) never inserts
      }
    float od[KC];
    int oi[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      od[j] = __shfl_xor(L.d[j], 32);
      oi[j] = __shfl_xor(L.i[j], 32);
    }
    L.merge(od, oi);
    if (h == 0) {
      const int ql = wc * (C::CT * 32) + ct * 32 + (lane & 31);
      Cand* dst = buf + ((size_t)wr * C::TN + ql) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) dst[j] = Cand{L.d[j], L.i[j]};
    }
  };
  static_assert(C::CT <= 4, "epilogue unroll");
  epi(std::integral_constant<int, 0>{});
  if constexpr (C::CT > 1) epi(std::integral_constant<int, 1>{});
  if constexpr (C::CT > 2) epi(std::integral_constant<int, 2>{});
  if constexpr (C::CT > 3) epi(std::integral_constant<int, 3>{});
  __syncthreads();
  if ((int)threadIdx.x < C::TN) {
    const int ql = threadIdx.x;
    const int64_t q = q0 + ql;
    TopList<KC> L;
    const Cand* s0 = buf + (size_t)ql * KC;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      L.d[j] = s0[j].d;
      L.i[j] = s0[j].i;
    }
#pragma unroll
    for (int w = 1; w < C::WM; ++w) {
      float od[KC];
      int oi[KC];
      const Cand* sw = buf + ((size_t)w * C::TN + ql) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        od[j] = sw[j].d;
        oi[j] = sw[j].i;
      }
      L.merge(od, oi);
    }
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

// ---- pass 2 ---------------------------------------------------------------------
struct MergeArgs {
  const Cand* cand;  // [T][B][KC]
  int64_t T, B;
  const float* Q;
  int64_t ldq;
  const float* G;
  int64_t ldg, d;
  int metric, k;
  int64_t index_base;
  double* out_d;
  int64_t* out_i;
};

template <int KC>
__global__ void __launch_bounds__(256) knn_merge_rerank_kernel(MergeArgs p) {
  __shared__ Cand lists[256 * KC];
  __shared__ double exact[KC];
  __shared__ double red[4];
  const int64_t q = blockIdx.x;
  select_candidates<KC>(p.cand, p.T, p.B, q, lists);
  // exact fp64 re-evaluation of the reference distance for the KC survivors
  const float* qr = p.Q + q * p.ldq;
  double qq = 0;
  if (p.metric == OFR_METRIC_COSINE) {
    double a = 0;
    for (int64_t j = threadIdx.x; j < p.d; j += blockDim.x) {
      const double x = qr[j];
      a += x * x;
    }
    qq = block_sum_f64(a, red);
  }
  for (int c = 0; c < KC; ++c) {
    const Cand cc = lists[c];  // block-uniform
    double val = __builtin_inf();
    if (cc.i != CAND_EMPTY) {
      const float* gr = p.G + (int64_t)cc.i * p.ldg;
      double a = 0, gg = 0;
      if (p.metric == OFR_METRIC_EUCLIDEAN) {
        for (int64_t j = threadIdx.x; j < p.d; j += blockDim.x) {   // distance.py:60
          const double df = (double)qr[j] - (double)gr[j];
          a += df * df;
        }
        val = sqrt(block_sum_f64(a, red));
      } else {
        for (int64_t j = threadIdx.x; j < p.d; j += blockDim.x) {   // distance.py:77
          const double x = qr[j], y = gr[j];
          a += x * y;
          gg += y * y;
        }
        const double dot = block_sum_f64(a, red);
        const double g2 = block_sum_f64(gg, red);
        val = -dot / sqrt(g2 * qq);
      }
    }
    if (threadIdx.x == 0) exact[c] = val;
  }
  __syncthreads();
  if (threadIdx.x < 64) sort_and_write_wave<KC>(lists, exact, p.k, p.index_base, p.out_d + q * p.k, p.out_i + q * p.k);
}

// ---- helpers ----------------------------------------------------------------------
__global__ void row_aux_kernel(int metric, const float* G, int64_t N, int64_t d, int64_t ldg, float* aux) {
  // one wave per row
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* g = G + row * ldg;
  double s = 0;
  for (int64_t j = lane; j < d; j += 64) {
    const double x = g[j];
    s += x * x;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) aux[row] = metric == OFR_METRIC_COSINE ? (float)(1.0 / sqrt(s)) : (float)s;
}

// unit rows for the certified Cosine search: out = fp32(g / ||g|| - shift), in fp64 and rounded once
// (shift nullable), zero rows stay zero; one wave per row
__global__ void normalize_rows_kernel(const float* G, int64_t N, int64_t d, int64_t ldg, const double* shift,
                                      float* out, int64_t ldo) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* g = G + row * ldg;
  double s = 0;
  for (int64_t j = lane; j < d; j += 64) {
    const double x = g[j];
    s += x * x;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const double inv = s > 0 ? 1.0 / sqrt(s) : 0.0;
  float* o = out + row * ldo;
  for (int64_t j = lane; j < ldo; j += 64)
    o[j] = j < d ? (float)((double)g[j] * inv - (shift ? shift[j] : 0.0)) : 0.f;
}

// CosineDistance (distance.py:74-77) of given (query, row) pairs in fp64 on the stored fp32 rows,
// then each query's k sorted by (distance, row); one wave per query, k <= 16
__global__ void cosine_pairs_kernel(const float* Q, int64_t ldq, const float* G, int64_t ldg, int64_t d,
                                    int64_t B, int k, double* out_d, int64_t* out_i) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= B) return;
  const float* qr = Q + q * ldq;
  double qq = 0;
  for (int64_t j = lane; j < d; j += 64) qq += (double)qr[j] * (double)qr[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) qq += __shfl_xor(qq, o);
  double dist[16];
  int64_t idx[16];
  for (int c = 0; c < k; ++c) {
    const int64_t i = out_i[q * k + c];
    double val = __builtin_inf();
    if (i >= 0) {
      const float* gr = G + i * ldg;
      double a = 0, gg = 0;
      for (int64_t j = lane; j < d; j += 64) {
        const double x = qr[j], y = gr[j];
        a += x * y;
        gg += y * y;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        gg += __shfl_xor(gg, o);
      }
      val = -a / sqrt(gg * qq);
    }
    dist[c] = val;
    idx[c] = i;
  }
  if (lane == 0) {
    for (int c = 1; c < k; ++c)   // insertion sort by (distance, row), empty (-1) rows last
      for (int u = c; u > 0; --u) {
        // empty (-1) rows last, then NaN distances (as the reference's argsort), then (distance, row)
        const bool sw = idx[u - 1] < 0 ? idx[u] >= 0
                                       : (idx[u] >= 0 && nan_last_before(dist[u], idx[u], dist[u - 1], idx[u - 1]));
        if (!sw) break;
        const double td = dist[u]; dist[u] = dist[u - 1]; dist[u - 1] = td;
        const int64_t ti = idx[u]; idx[u] = idx[u - 1]; idx[u - 1] = ti;
      }
    for (int c = 0; c < k; ++c) {
      out_d[q * k + c] = dist[c];
      out_i[q * k + c] = idx[c];
    }
  }
}

// column means in two deterministic passes: fixed row chunks, then an ordered sum of the chunks
constexpr int COLMEAN_CHUNKS = 256;
__global__ void col_mean_partial_kernel(const float* G, int64_t N, int64_t d, int64_t ldg, double* part) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (j >= d) return;
  const int64_t rows = cdiv(N, COLMEAN_CHUNKS);
  const int64_t r0 = c * rows, r1 = min(N, r0 + rows);
  double s = 0;
  for (int64_t n = r0; n < r1; ++n) s += G[n * ldg + j];
  part[c * d + j] = s;
}
__global__ void col_mean_final_kernel(const double* part, int64_t N, int64_t d, double* mean) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= d) return;
  double s = 0;
  for (int c = 0; c < COLMEAN_CHUNKS; ++c) s += part[(int64_t)c * d + j];
  mean[j] = s / (double)N;
}

__global__ void sub_rows_kernel(float* G, int64_t N, int64_t d, int64_t ldg, const float* shift) {
  const int64_t n = blockIdx.y;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
    G[n * ldg + j] -= shift[j];
}

__global__ void topk_merge_kernel(const double* in_d, const int64_t* in_i, int64_t B, int P, int kin, int k,
                                  double* out_d, int64_t* out_i) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  const double* dd = in_d + q * (int64_t)P * kin;
  const int64_t* ii = in_i + q * (int64_t)P * kin;
  int pos[64];
  for (int p = 0; p < P; ++p) pos[p] = 0;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    for (int p = 0; p < P; ++p) {
      if (pos[p] >= kin) continue;
      const int64_t c = (int64_t)p * kin + pos[p];
      if (ii[c] < 0) continue;
      if (best < 0) { best = p; continue; }
      const int64_t b = (int64_t)best * kin + pos[best];
      const double x = dd[c], y = dd[b];
      const bool xn = x != x, yn = y != y;
      const bool before = (!xn && yn) || (!xn && !yn && better_d(x, ii[c], y, ii[b])) || (xn && yn && ii[c] < ii[b]);
      if (before) best = p;
    }
    if (best < 0) {
      out_d[q * k + j] = __builtin_inf();
      out_i[q * k + j] = -1;
    } else {
      const int64_t b = (int64_t)best * kin + pos[best];
      out_d[q * k + j] = dd[b];
      out_i[q * k + j] = ii[b];
      ++pos[best];
    }
  }
}


}  // namespace ofr

using namespace ofr;

extern "C" size_t ofr_knn_workspace_bytes(int64_t B, int64_t N, int k) {
  const int kc = pick_kc(k);
  const int64_t T = cdiv(N > 0 ? N : 1, tile::TM);
  return (size_t)T * (size_t)B * kc * sizeof(Cand) + 256;
}

template <class C, int METRIC, int KC>
static int launch_tiles(hipStream_t st, KnnTileArgs a) {
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)knn_tile_kernel<C, METRIC, KC>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, C::LDS);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(knn_tile)");
    attr_done = true;
  }
  a.ntb = cdiv(a.B, C::TN);
  const int64_t nblocks = a.ntb * a.ntg;
  if (nblocks >= 0x7fffffffLL) return fail(OFR_E_INVALID, "ofr_knn_f32: grid too large");
  hipLaunchKernelGGL((knn_tile_kernel<C, METRIC, KC>), dim3((unsigned)nblocks), dim3(256), C::LDS, st, a);
  OFR_LAUNCH_CHECK("knn_tile_kernel");
  return OFR_OK;
}

template <int METRIC, int KC>
static int launch_knn(hipStream_t st, const KnnTileArgs& a, const MergeArgs& m, int phases) {
  if (phases & 1) {
    // narrow query tiles stream the gallery once per batch (HBM-bound regime); wide tiles are MFMA-bound
    const int rc = a.B <= tile::CfgSmall::TN ? launch_tiles<tile::CfgSmall, METRIC, KC>(st, a)
                                             : launch_tiles<tile::CfgBig, METRIC, KC>(st, a);
    if (rc) return rc;
  }
  if (phases & 2) {
    hipLaunchKernelGGL((knn_merge_rerank_kernel<KC>), dim3((unsigned)m.B), dim3(256), 0, st, m);
    OFR_LAUNCH_CHECK("knn_merge_rerank_kernel");
  }
  return OFR_OK;
}

static int knn_impl(void* stream, int metric, const float* Q, int64_t B, int64_t ldq, const float* G, int64_t N,
                    int64_t ldg, int64_t d, const float* aux, int k, int64_t index_base, double* out_d,
                    int64_t* out_i, void* workspace, size_t workspace_bytes, int phases) {
  OFR_CHECK_ARG(metric == OFR_METRIC_EUCLIDEAN || metric == OFR_METRIC_COSINE, "ofr_knn_f32: metric must be EUCLIDEAN or COSINE");
  OFR_CHECK_ARG(B >= 0 && N >= 0 && d >= 1, "ofr_knn_f32: bad sizes");
  if (k < 1 || k > OFR_MAX_K) return fail(OFR_E_UNSUPPORTED, "ofr_knn_f32: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(Q && ((phases & 2) == 0 || (out_d && out_i)), "ofr_knn_f32: null pointer");
  OFR_CHECK_ARG(ldq % 32 == 0 && ldq >= round_up(d, 32), "ofr_knn_f32: ldq must be a multiple of 32 >= round_up(d,32)");
  hipStream_t st = (hipStream_t)stream;
  if (N == 0) {
    // nothing to search: every slot is (+inf, -1)
    if (!(phases & 2)) return OFR_OK;
    MergeArgs m{nullptr, 0, B, Q, ldq, G, ldg, d, metric, k, index_base, out_d, out_i};
    hipLaunchKernelGGL((knn_merge_rerank_kernel<8>), dim3((unsigned)B), dim3(256), 0, st, m);
    OFR_LAUNCH_CHECK("knn_merge_rerank_kernel");
    return OFR_OK;
  }
  OFR_CHECK_ARG(G && aux, "ofr_knn_f32: null gallery");
  OFR_CHECK_ARG(ldg % 32 == 0 && ldg >= round_up(d, 32), "ofr_knn_f32: ldg must be a multiple of 32 >= round_up(d,32)");
  OFR_CHECK_ARG(N < 0x7fffffffLL - tile::TM, "ofr_knn_f32: N too large for one shard");
  OFR_CHECK_ARG(((uintptr_t)Q % 16) == 0 && ((uintptr_t)G % 16) == 0, "ofr_knn_f32: Q and G must be 16-byte aligned");
  const int kc = pick_kc(k);
  OFR_CHECK_ARG(workspace && workspace_bytes >= ofr_knn_workspace_bytes(B, N, k), "ofr_knn_f32: workspace too small");
  KnnTileArgs a;
  a.Q = Q; a.B = B; a.ldq = ldq; a.G = G; a.N = N; a.ldg = ldg;
  a.nk = (int)cdiv(d, tile::BK);
  a.aux = aux;
  a.cand = reinterpret_cast<Cand*>(workspace);
  a.ntb = 0;  // set per tile configuration
  a.ntg = cdiv(N, tile::TM);
  MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, d, metric, k, index_base, out_d, out_i};
  if (metric == OFR_METRIC_EUCLIDEAN)
    return kc == 8 ? launch_knn<OFR_METRIC_EUCLIDEAN, 8>(st, a, m, phases)
                   : launch_knn<OFR_METRIC_EUCLIDEAN, 16>(st, a, m, phases);
  return kc == 8 ? launch_knn<OFR_METRIC_COSINE, 8>(st, a, m, phases) : launch_knn<OFR_METRIC_COSINE, 16>(st, a, m, phases);
}

#define OFR_KNN_PARAMS                                                                                              \
  void *stream, int metric, const float *Q, int64_t B, int64_t ldq, const float *G, int64_t N, int64_t ldg, int64_t d, \
      const float *aux, int k, int64_t index_base, double *out_d, int64_t *out_i, void *workspace,                   \
      size_t workspace_bytes
#define OFR_KNN_ARGS stream, metric, Q, B, ldq, G, N, ldg, d, aux, k, index_base, out_d, out_i, workspace, workspace_bytes

extern "C" int ofr_knn_f32(OFR_KNN_PARAMS) { return knn_impl(OFR_KNN_ARGS, 3); }
extern "C" int ofr_knn_tiles_f32(OFR_KNN_PARAMS) { return knn_impl(OFR_KNN_ARGS, 1); }
extern "C" int ofr_knn_merge_f32(OFR_KNN_PARAMS) { return knn_impl(OFR_KNN_ARGS, 2); }

extern "C" int ofr_row_aux(void* stream, int metric, const float* G, int64_t N, int64_t d, int64_t ldg, float* aux) {
  OFR_CHECK_ARG(metric == OFR_METRIC_EUCLIDEAN || metric == OFR_METRIC_COSINE, "ofr_row_aux: bad metric");
  OFR_CHECK_ARG(N >= 0 && d >= 0 && ldg >= d, "ofr_row_aux: bad sizes");
  if (N == 0) return OFR_OK;
  hipLaunchKernelGGL(row_aux_kernel, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, (hipStream_t)stream, metric, G, N, d, ldg, aux);
  OFR_LAUNCH_CHECK("row_aux_kernel");
  return OFR_OK;
}

extern "C" int ofr_normalize_rows_f32(void* stream, const float* G, int64_t N, int64_t d, int64_t ldg,
                                      const double* shift, float* out, int64_t ldo) {
  OFR_CHECK_ARG(N >= 0 && d >= 1 && ldg >= d && ldo >= d, "ofr_normalize_rows_f32: bad sizes");
  if (N == 0) return OFR_OK;
  OFR_CHECK_ARG(G && out, "ofr_normalize_rows_f32: null pointer");
  hipLaunchKernelGGL(normalize_rows_kernel, dim3((unsigned)cdiv(N, 4)), dim3(256), 0, (hipStream_t)stream, G, N, d,
                     ldg, shift, out, ldo);
  OFR_LAUNCH_CHECK("normalize_rows_kernel");
  return OFR_OK;
}

extern "C" int ofr_cosine_pairs(void* stream, const float* Q, int64_t B, int64_t ldq, const float* G, int64_t N,
                                int64_t ldg, int64_t d, int k, double* out_d, int64_t* out_i) {
  OFR_CHECK_ARG(B >= 0 && N >= 0 && d >= 1 && ldq >= d && ldg >= d && k >= 1 && k <= 16,
                "ofr_cosine_pairs: bad sizes (k <= 16)");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(Q && G && out_d && out_i, "ofr_cosine_pairs: null pointer");
  hipLaunchKernelGGL(cosine_pairs_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, (hipStream_t)stream, Q, ldq, G,
                     ldg, d, B, k, out_d, out_i);
  OFR_LAUNCH_CHECK("cosine_pairs_kernel");
  return OFR_OK;
}

extern "C" int ofr_col_mean(void* stream, const float* G, int64_t N, int64_t d, int64_t ldg, double* mean) {
  OFR_CHECK_ARG(N > 0 && d >= 0 && ldg >= d, "ofr_col_mean: bad sizes");
  if (d == 0) return OFR_OK;
  hipStream_t st = (hipStream_t)stream;
  double* part = nullptr;
  hipError_t e = hipMallocAsync((void**)&part, sizeof(double) * COLMEAN_CHUNKS * d, st);
  if (e != hipSuccess) return hip_status(e, "hipMallocAsync(col_mean)");
  hipLaunchKernelGGL(col_mean_partial_kernel, dim3((unsigned)cdiv(d, 256), COLMEAN_CHUNKS), dim3(256), 0, st, G, N, d,
                     ldg, part);
  hipLaunchKernelGGL(col_mean_final_kernel, dim3((unsigned)cdiv(d, 256)), dim3(256), 0, st, part, N, d, mean);
  hipError_t le = hipGetLastError();
  e = hipFreeAsync(part, st);
  if (le != hipSuccess) return hip_status(le, "col_mean kernels");
  if (e != hipSuccess) return hip_status(e, "hipFreeAsync(col_mean)");
  return OFR_OK;
}

extern "C" int ofr_sub_rows(void* stream, float* G, int64_t N, int64_t d, int64_t ldg, const float* shift) {
  OFR_CHECK_ARG(N >= 0 && d >= 0 && ldg >= d && N < 65536LL * 1024, "ofr_sub_rows: bad sizes");
  if (N == 0 || d == 0) return OFR_OK;
  const unsigned gx = (unsigned)std::min<int64_t>(cdiv(d, 256), 64);
  int64_t done = 0;
  while (done < N) {
    const int64_t chunk = std::min<int64_t>(N - done, 65535);
    hipLaunchKernelGGL(sub_rows_kernel, dim3(gx, (unsigned)chunk), dim3(256), 0, (hipStream_t)stream,
                       G + done * ldg, chunk, d, ldg, shift);
    OFR_LAUNCH_CHECK("sub_rows_kernel");
    done += chunk;
  }
  return OFR_OK;
}

extern "C" int ofr_topk_merge(void* stream, const double* in_d, const int64_t* in_i, int64_t B, int P, int kin, int k,
                              double* out_d, int64_t* out_i) {
  OFR_CHECK_ARG(B >= 0 && P >= 1 && P <= 64 && kin >= 1 && k >= 1, "ofr_topk_merge: bad sizes (P <= 64)");
  if (B == 0) return OFR_OK;
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)cdiv(B, 128)), dim3(128), 0, (hipStream_t)stream, in_d, in_i, B,
                     P, kin, k, out_d, out_i);
  OFR_LAUNCH_CHECK("topk_merge_kernel");
  return OFR_OK;
}
