// Top-k building blocks shared by the search kernels (Euclidean/Cosine on the
// MFMA tile engine, ChiSquare on the VALU tile kernel).
//
// Ordering everywhere: ascending distance, ties to the LOWER gallery index
// (deterministic; the reference's np.argsort quicksort leaves exact-tie
// order unspecified, classifier.py:113).  NaN scores never enter a list.
#pragma once
#include "ofr_common.h"

namespace ofr {

struct Cand {
  float d;
  int i;
};

constexpr int CAND_EMPTY = 0x7fffffff;

template <int KC>
struct TopList {
  float d[KC];
  int i[KC];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      d[j] = __builtin_inff();
      i[j] = CAND_EMPTY;
    }
  }
  // insert keeping ascending (d, i) order; static register indexing only
  __device__ __forceinline__ void insert(float v, int id) {
    if (better_f(v, id, d[KC - 1], i[KC - 1])) {
      d[KC - 1] = v;
      i[KC - 1] = id;
#pragma unroll
      for (int j = KC - 1; j > 0; --j) {
        const bool sw = better_f(d[j], i[j], d[j - 1], i[j - 1]);
        const float td = d[j], tp = d[j - 1];
        const int ti = i[j], tq = i[j - 1];
        d[j - 1] = sw ? td : tp;
        i[j - 1] = sw ? ti : tq;
        d[j] = sw ? tp : td;
        i[j] = sw ? tq : ti;
      }
    }
  }
  // merge with another ascending list, keep the best KC ascending (bitonic merge)
  __device__ __forceinline__ void merge(const float (&od)[KC], const int (&oi)[KC]) {
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const float bd = od[KC - 1 - j];
      const int bi = oi[KC - 1 - j];
      if (better_f(bd, bi, d[j], i[j])) {
        d[j] = bd;
        i[j] = bi;
      }
    }
#pragma unroll
    for (int s = KC / 2; s > 0; s >>= 1) {
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        if ((j & s) == 0) {
          const bool sw = better_f(d[j + s], i[j + s], d[j], i[j]);
          const float x = d[j], y = d[j + s];
          const int xi = i[j], yi = i[j + s];
          d[j] = sw ? y : x;
          i[j] = sw ? yi : xi;
          d[j + s] = sw ? x : y;
          i[j + s] = sw ? xi : yi;
        }
      }
    }
  }
};

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// Best KC of cand[t][q][KC] over t < T (each tile list ascending) for query q,
// reduced over the 256-thread block; result in lists[0..KC) (shared memory).
template <int KC>
__device__ __forceinline__ void select_candidates(const Cand* __restrict__ cand, int64_t T, int64_t B, int64_t q,
                                                  Cand* lists) {
  TopList<KC> L;
  L.init();
  for (int64_t t = threadIdx.x; t < T; t += blockDim.x) {
    const Cand* c = cand + ((size_t)t * B + q) * KC;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const Cand x = c[j];
      if (!better_f(x.d, x.i, L.d[KC - 1], L.i[KC - 1])) break;
      L.insert(x.d, x.i);
    }
  }
  for (int j = 0; j < KC; ++j) lists[threadIdx.x * KC + j] = Cand{L.d[j], L.i[j]};
  __syncthreads();
  for (int active = (int)blockDim.x / 2; active > 0; active >>= 1) {
    if ((int)threadIdx.x < active) {
      float od[KC];
      int oi[KC];
      const Cand* o = lists + (threadIdx.x + active) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        od[j] = o[j].d;
        oi[j] = o[j].i;
      }
      L.merge(od, oi);
#pragma unroll
      for (int j = 0; j < KC; ++j) lists[threadIdx.x * KC + j] = Cand{L.d[j], L.i[j]};
    }
    __syncthreads();
  }
}

__device__ __forceinline__ bool nan_last_before(double x, int64_t xi, double y, int64_t yi) {
  const bool xn = x != x, yn = y != y;
  return (!xn && yn) || (!xn && !yn && better_d(x, xi, y, yi)) || (xn && yn && xi < yi);
}

// Thread 0: sort the KC exact distances by (distance, index), NaN last, and write the best k.
template <int KC>
__device__ __forceinline__ void sort_and_write(const Cand* lists, const double* exact, int k, int64_t index_base,
                                               double* out_d, int64_t* out_i) {
  double dd[KC];
  int64_t ii[KC];
  for (int c = 0; c < KC; ++c) {
    const Cand cc = lists[c];
    const bool ok = cc.i != CAND_EMPTY;
    dd[c] = ok ? exact[c] : __builtin_inf();
    ii[c] = ok ? (int64_t)cc.i : INT64_MAX;
  }
  for (int a = 1; a < KC; ++a) {
    const double x = dd[a];
    const int64_t xi = ii[a];
    int b = a - 1;
    while (b >= 0 && nan_last_before(x, xi, dd[b], ii[b])) {
      dd[b + 1] = dd[b];
      ii[b + 1] = ii[b];
      --b;
    }
    dd[b + 1] = x;
    ii[b + 1] = xi;
  }
  for (int j = 0; j < k; ++j) {
    const bool ok = j < KC && ii[j] != INT64_MAX;
    out_d[j] = ok ? dd[j] : __builtin_inf();
    out_i[j] = ok ? ii[j] + index_base : -1;
  }
}

// The same on one whole wave (every lane of it calls this; round 6): lane c ranks candidate c against
// the other KC -- ties, i.e. equal (distance, index) keys, occur only between empty entries and go by c,
// as the insertion sort above keeps them -- and writes it at its rank if that is below k.  Returns the
// k-th distance (min(k, KC)-th) in every lane.  The thread-0 form sorts a dynamically indexed array in
// scratch memory (~120 dependent scratch moves per query); this one reads the KC entries from LDS.
template <int KC>
__device__ __forceinline__ double sort_and_write_wave(const Cand* lists, const double* exact, int k, int64_t index_base,
                                                      double* out_d, int64_t* out_i) {
  const int lane = threadIdx.x & 63;
  double x = __builtin_inf();
  int64_t xi = INT64_MAX;
  if (lane < KC) {
    const Cand cc = lists[lane];
    if (cc.i != CAND_EMPTY) {
      x = exact[lane];
      xi = (int64_t)cc.i;
    }
  }
  int rank = 0;
#pragma unroll
  for (int u = 0; u < KC; ++u) {
    const Cand cu = lists[u];
    const bool ok = cu.i != CAND_EMPTY;
    const double y = ok ? exact[u] : __builtin_inf();
    const int64_t yi = ok ? (int64_t)cu.i : INT64_MAX;
    rank += nan_last_before(y, yi, x, xi) || (u < lane && !nan_last_before(x, xi, y, yi));
  }
  if (lane < KC && rank < k) {
    const bool ok = xi != INT64_MAX;
    out_d[rank] = ok ? x : __builtin_inf();
    out_i[rank] = ok ? xi + index_base : -1;
  }
  for (int j = KC + lane; j < k; j += 64) {   // k > KC: nothing more to place
    out_d[j] = __builtin_inf();
    out_i[j] = -1;
  }
  const int kk = k < KC ? k : KC;
  const uint64_t m = __ballot(lane < KC && rank == kk - 1);
  const int src = m ? __ffsll((long long)m) - 1 : 0;
  const double dk = __shfl(xi != INT64_MAX ? x : __builtin_inf(), src);
  return m ? dk : __builtin_inf();
}

static inline int pick_kc(int k) { return k <= 8 ? 8 : 16; }

}  // namespace ofr
