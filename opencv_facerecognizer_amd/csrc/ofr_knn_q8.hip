// Certified int8 coarse pass of the Euclidean k-NN search (gfx950).
//
// Replaces, like ofr_knn.hip, NearestNeighbor.predict (reference
// classifier.py:104-119) with EuclideanDistance (distance.py:57-60), for
// batches B > 32 where the search is compute-bound.
//
// Representation.  Every centred fp32 row x (gallery once, queries per batch)
// is split with a power-of-two scale s_x (max|x|/s_x in (63.5,127]) into two
// int8 slices:  x~ = s_x (x1 + 2^-7 x2),  x1 in [-127,127], x2 in [-64,64].
// Per row we keep a_x = ||x~||, e_x = ||x - x~||, t_x = s_x 2^-7 ||x2|| (fp64).
//
// Coarse score.  v_mfma_i32_32x32x32_i8 accumulates EXACTLY
//     P0 = x1.y1,   P1 = x1.y2 + x2.y1        (int32, |P| < 2^29)
// and the epilogue forms  S~ = ||g||^2 - 2 s_q s_g (P0 + 2^-7 P1)  in fp32.
// For the true score S = ||g||^2 - 2 q.g = d^2 - ||q||^2 (fp32 rows):
//     |S - S~| <= 2 (a_q e_g + e_q a_g + e_q e_g + t_q t_g) + roundoff
// (Cauchy-Schwarz on q.g = q~.g~ + q~.r_g + r_q.g~ + r_q.r_g, and the dropped
// term s_q s_g 2^-14 q2.g2).  With gallery-wide maxima (A, E, T, auxmax) this
// gives a per-query bound dS(q).
//
// Certificate.  Each 256-row gallery tile keeps its best KC=16 coarse scores
// per query; the merge keeps the best R=16 overall (tau = the 16th).  Every
// row outside the final list has S~ >= tau (a tile contributing < 16 rows
// below tau cannot hide one).  After the EXACT fp64 re-rank of the 16
// candidates, the top-k is proven equal to the exact top-k when
//     S_k(exact) < tau - dS(q)
// (strictly: no excluded row can reach or tie the k-th).  cert[q] = 1 then;
// otherwise 0 and the caller re-runs that query on the fp32 path.
#include <type_traits>

#include "ofr_topk.h"

namespace ofr {
namespace q8s {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 16;
constexpr int TG = 256, TQ = 128, BK = 64, NST = 3;
constexpr int PG = TG * BK, PQ = TQ * BK;          // 16 KiB, 8 KiB per slice panel
constexpr int STAGE = 2 * PG + 2 * PQ;             // 48 KiB
constexpr int LDS = NST * STAGE;                   // 144 KiB
constexpr int IPW = 4 + 4 + 2 + 2;                 // DMA wave-instructions per wave per panel

__device__ __forceinline__ int off(int row, int chunk) { return row * BK + ((chunk ^ ((row >> 2) & 3)) << 4); }

template <int ROWS>
__device__ __forceinline__ void dma(const int8_t* base, int64_t ldk, int64_t rows, int64_t r0, char* panel, int kt) {
  constexpr int NINS = ROWS / 16;        // 16 rows x 64 B per wave-instruction
  constexpr int PER = NINS / 4;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < PER; ++t) {
    const int ins = wave * PER + t;
    const int row = ins * 16 + (lane >> 2);
    const int chunk = (lane & 3) ^ ((row >> 2) & 3);
    int64_t gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    const int8_t* src = base + gr * ldk + (int64_t)kt * BK + chunk * 16;
    __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)src, (OFR_LDS void*)(panel + ins * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct TileArgs {
  const int8_t *G1, *G2;
  int64_t N, ldk;
  const float* gscale;
  const float* aux;
  const int8_t *Q1, *Q2;
  int64_t B;
  const float* qscale;
  int nk;
  Cand* cand;   // [T][B][KC]
  int64_t ntq, ntg;
};

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblocks) {
  const int64_t q = nblocks / 8, r = nblocks % 8;
  const int64_t x = bid % 8, s = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

__global__ void __launch_bounds__(256, 1) tile_kernel(TileArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t gt = t / p.ntq, qt = t % p.ntq;     // consecutive tiles share the gallery tile
  const int64_t g0 = gt * TG, q0 = qt * TQ;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave >> 1, wc = wave & 1, h = lane >> 5, r32 = lane & 31;

  i32x16 acc0[4][2], acc1[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc0[i][j][r] = 0;
        acc1[i][j][r] = 0;
      }

  auto issue = [&](int kt) {
    char* st = smem + (kt % NST) * STAGE;
    dma<TG>(p.G1, p.ldk, p.N, g0, st, kt);
    dma<TG>(p.G2, p.ldk, p.N, g0, st + PG, kt);
    dma<TQ>(p.Q1, p.ldk, p.B, q0, st + 2 * PG, kt);
    dma<TQ>(p.Q2, p.ldk, p.B, q0, st + 2 * PG + PQ, kt);
  };
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < p.nk) issue(s);

  for (int kt = 0; kt < p.nk; ++kt) {
    if (kt + 1 < p.nk) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");   // (NST-2) panels x IPW in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    if (kt + NST - 1 < p.nk) issue(kt + NST - 1);
    const char* st = smem + (kt % NST) * STAGE;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      const int chunk = 2 * ks + h;
      i32x4 g1[4], g2[4], q1[2], q2[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wr * 128 + i * 32 + r32;
        g1[i] = *reinterpret_cast<const i32x4*>(st + off(row, chunk));
        g2[i] = *reinterpret_cast<const i32x4*>(st + PG + off(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = wc * 64 + j * 32 + r32;
        q1[j] = *reinterpret_cast<const i32x4*>(st + 2 * PG + off(row, chunk));
        q2[j] = *reinterpret_cast<const i32x4*>(st + 2 * PG + PQ + off(row, chunk));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc0[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g1[i], q1[j], acc0[i][j], 0, 0, 0);
          acc1[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g2[i], q1[j], acc1[i][j], 0, 0, 0);
          acc1[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(g1[i], q2[j], acc1[i][j], 0, 0, 0);
        }
    }
  }
  barrier();

  // epilogue: coarse scores, per-lane top-16 over the lane's 64 gallery rows, merges.
  // The tile's gallery aux / scale go through LDS (one coalesced load, no per-element global waits).
  Cand* buf = reinterpret_cast<Cand*>(smem);                       // [2][TQ][KC]  (32 KiB)
  float* gtab = reinterpret_cast<float*>(smem + 2 * TQ * KC * sizeof(Cand));   // [TG][2]
  {
    const int64_t g = g0 + threadIdx.x;
    const bool ok = g < p.N;
    gtab[2 * threadIdx.x + 0] = ok ? p.aux[g] : 0.f;
    gtab[2 * threadIdx.x + 1] = ok ? p.gscale[g] : 0.f;
  }
  __syncthreads();
  // one body per query block (ct is a template constant: a runtime index would send acc to scratch)
  auto epi = [&](auto ctc) {
    constexpr int ct = decltype(ctc)::value;
    int64_t q = q0 + wc * 64 + ct * 32 + r32;
    const float sq2 = 2.0f * p.qscale[q < p.B ? q : p.B - 1];
    TopList<KC> L;
    L.init();
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gl = wr * 128 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float c = (float)acc0[rt][ct][r] + (float)acc1[rt][ct][r] * 0x1p-7f;
        const float sc = gtab[2 * gl] - sq2 * gtab[2 * gl + 1] * c;
        // rows past N get NaN: never inserted
        L.insert(g0 + gl < p.N ? sc : __builtin_nanf(""), (int)(g0 + gl));
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
      Cand* dst = buf + ((size_t)wr * TQ + wc * 64 + ct * 32 + r32) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) dst[j] = Cand{L.d[j], L.i[j]};
    }
  };
  epi(std::integral_constant<int, 0>{});
  epi(std::integral_constant<int, 1>{});
  __syncthreads();
  if ((int)threadIdx.x < TQ) {
    const int ql = threadIdx.x;
    const int64_t q = q0 + ql;
    TopList<KC> L;
    float od[KC];
    int oi[KC];
    const Cand* s0 = buf + (size_t)ql * KC;
    const Cand* s1 = buf + ((size_t)TQ + ql) * KC;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      L.d[j] = s0[j].d;
      L.i[j] = s0[j].i;
      od[j] = s1[j].d;
      oi[j] = s1[j].i;
    }
    L.merge(od, oi);
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

struct MergeArgs {
  const Cand* cand;
  int64_t T, B;
  const float* Q;
  int64_t ldq;
  const float* G;
  int64_t ldg, d;
  const double* qstats;   // [B][3]: a, e, t
  const double* gmax;     // [4]: A, E, T, auxmax
  int k;
  int64_t index_base;
  double* out_d;
  int64_t* out_i;
  int* cert;
};

__global__ void __launch_bounds__(256) merge_kernel(MergeArgs p) {
  __shared__ Cand lists[256 * KC];
  __shared__ double exact[KC];
  __shared__ double red[4];
  const int64_t q = blockIdx.x;
  select_candidates<KC>(p.cand, p.T, p.B, q, lists);
  const float* qr = p.Q + q * p.ldq;
  double qq = 0;
  for (int64_t j = threadIdx.x; j < p.d; j += blockDim.x) {
    const double x = qr[j];
    qq += x * x;
  }
  qq = block_sum_f64(qq, red);
  for (int c = 0; c < KC; ++c) {
    const Cand cc = lists[c];
    double val = __builtin_inf();
    if (cc.i != CAND_EMPTY) {
      const float* gr = p.G + (int64_t)cc.i * p.ldg;
      double a = 0;
      for (int64_t j = threadIdx.x; j < p.d; j += blockDim.x) {   // distance.py:60
        const double df = (double)qr[j] - (double)gr[j];
        a += df * df;
      }
      val = sqrt(block_sum_f64(a, red));
    }
    if (threadIdx.x == 0) exact[c] = val;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* od = p.out_d + q * p.k;
    int64_t* oi = p.out_i + q * p.k;
    sort_and_write<KC>(lists, exact, p.k, p.index_base, od, oi);
    // certificate
    int nvalid = 0;
    for (int c = 0; c < KC; ++c) nvalid += lists[c].i != CAND_EMPTY;
    int ok;
    if (nvalid < KC) {
      ok = 1;   // every gallery row was a candidate
    } else {
      const double tau = (double)lists[KC - 1].d;
      const double a = p.qstats[q * 3 + 0], e = p.qstats[q * 3 + 1], tq = p.qstats[q * 3 + 2];
      const double A = p.gmax[0], E = p.gmax[1], T = p.gmax[2], auxmax = p.gmax[3];
      double dS = 2.0 * (a * E + e * A + e * E + tq * T) + 0x1p-20 * (auxmax + 2.0 * a * A);
      dS = dS * (1.0 + 1e-6) + 1e-300;
      const int kk = p.k < KC ? p.k : KC;
      const double dk = od[kk - 1];
      const double Sk = dk * dk - qq;
      ok = (dk == dk) && (Sk + 1e-12 * (dk * dk + qq) < tau - dS);
    }
    p.cert[q] = ok;
  }
}

// ---- quantization of fp32 rows ----------------------------------------------------------
__global__ void __launch_bounds__(256) quantize_kernel(const float* X, int64_t ldx, int64_t d, int8_t* X1, int8_t* X2,
                                                       int64_t ldk, float* scale, double* stats) {
  __shared__ double red[4][3];
  const int64_t row = blockIdx.x;
  const float* x = X + row * ldx;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float mx = 0.f;
  for (int64_t i = threadIdx.x; i < d; i += blockDim.x) mx = fmaxf(mx, fabsf(x[i]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) red[wave][0] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf((float)red[0][0], (float)red[1][0]), fmaxf((float)red[2][0], (float)red[3][0]));
  __syncthreads();
  double s = 1.0;
  if (mx > 0.f) {
    int e;
    frexp((double)mx / 127.0, &e);
    s = ldexp(1.0, e);
    if ((double)mx / s > 127.0) s *= 2.0;
  }
  double sa = 0, se = 0, st = 0;
  int8_t* o1 = X1 + row * ldk;
  int8_t* o2 = X2 + row * ldk;
  for (int64_t i = threadIdx.x; i < ldk; i += blockDim.x) {
    int v1 = 0, v2 = 0;
    if (i < d) {
      const double xv = (double)x[i];
      const double r = xv / s;                // exact (power of two)
      const double f1 = rint(r);
      const double f2 = rint((r - f1) * 128.0);
      v1 = (int)f1;
      v2 = (int)f2;
      const double xt = s * (f1 + f2 * 0x1p-7);  // exact
      sa += xt * xt;
      se += (xv - xt) * (xv - xt);
      st += f2 * f2;
    }
    o1[i] = (int8_t)v1;
    o2[i] = (int8_t)v2;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o);
    se += __shfl_xor(se, o);
    st += __shfl_xor(st, o);
  }
  if (lane == 0) {
    red[wave][0] = sa;
    red[wave][1] = se;
    red[wave][2] = st;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double A = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    const double E = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    const double T = red[0][2] + red[1][2] + red[2][2] + red[3][2];
    scale[row] = (float)s;
    // norms rounded up a hair so that fp64 summation error never shrinks the bound
    stats[row * 3 + 0] = sqrt(A) * (1.0 + 1e-12);
    stats[row * 3 + 1] = sqrt(E) * (1.0 + 1e-12);
    stats[row * 3 + 2] = s * 0x1p-7 * sqrt(T) * (1.0 + 1e-12);
  }
}

__global__ void __launch_bounds__(256) maxima_kernel(const double* stats, const float* aux, int64_t R, double* gmax) {
  __shared__ double red[4][4];
  double m[4] = {0, 0, 0, 0};
  for (int64_t r = threadIdx.x; r < R; r += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 3; ++c) m[c] = fmax(m[c], stats[r * 3 + c]);
    if (aux) m[3] = fmax(m[3], (double)aux[r]);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m[c] = fmax(m[c], __shfl_xor(m[c], o));
    if (lane == 0) red[wave][c] = m[c];
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int c = 0; c < 4; ++c) gmax[c] = fmax(fmax(red[0][c], red[1][c]), fmax(red[2][c], red[3][c]));
}

}  // namespace q8s
}  // namespace ofr

using namespace ofr;

extern "C" int ofr_q8_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int8_t* X1,
                                    int8_t* X2, int64_t ldk, float* scale, double* stats, const float* aux,
                                    double* maxima) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d && ldk >= round_up(d, 64) && ldk % 64 == 0,
                "ofr_q8_quantize_rows: bad sizes (ldk must be a multiple of 64 >= round_up(d,64))");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && X1 && X2 && scale && stats, "ofr_q8_quantize_rows: null pointer");
  OFR_CHECK_ARG(R < 0x7fffffffLL, "ofr_q8_quantize_rows: too many rows");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(q8s::quantize_kernel, dim3((unsigned)R), dim3(256), 0, st, X, ldx, d, X1, X2, ldk, scale, stats);
  OFR_LAUNCH_CHECK("q8 quantize_kernel");
  if (maxima) {
    hipLaunchKernelGGL(q8s::maxima_kernel, dim3(1), dim3(256), 0, st, stats, aux, R, maxima);
    OFR_LAUNCH_CHECK("q8 maxima_kernel");
  }
  return OFR_OK;
}

extern "C" size_t ofr_knn_q8_workspace_bytes(int64_t B, int64_t N) {
  return (size_t)cdiv(N > 0 ? N : 1, q8s::TG) * (size_t)B * q8s::KC * sizeof(Cand) + 256;
}

extern "C" int ofr_knn_q8(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const int8_t* Q1,
                          const int8_t* Q2, const float* qscale, const double* qstats, const float* G, int64_t N,
                          int64_t ldg, int64_t d, const int8_t* G1, const int8_t* G2, int64_t ldk,
                          const float* gscale, const float* aux, const double* gmax, int k, int64_t index_base,
                          double* out_d, int64_t* out_i, int* cert, void* workspace, size_t workspace_bytes) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 3, "ofr_knn_q8: phases must be 1 (tiles), 2 (merge) or 3");
  OFR_CHECK_ARG(B >= 0 && N >= 1 && d >= 1, "ofr_knn_q8: bad sizes (empty galleries use ofr_knn_f32)");
  if (k < 1 || k > q8s::KC) return fail(OFR_E_UNSUPPORTED, "ofr_knn_q8: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(ldk % 64 == 0 && ldk >= round_up(d, 64), "ofr_knn_q8: bad ldk");
  OFR_CHECK_ARG(ldq >= d && ldg >= d, "ofr_knn_q8: bad leading dimensions");
  OFR_CHECK_ARG(Q && Q1 && Q2 && qscale && qstats && G && G1 && G2 && gscale && aux && gmax && workspace,
                "ofr_knn_q8: null pointer");
  OFR_CHECK_ARG(((uintptr_t)Q1 | (uintptr_t)Q2 | (uintptr_t)G1 | (uintptr_t)G2) % 16 == 0, "ofr_knn_q8: slices must be 16-byte aligned");
  OFR_CHECK_ARG(N < 0x7fffffffLL - q8s::TG, "ofr_knn_q8: N too large for one shard");
  OFR_CHECK_ARG(workspace_bytes >= ofr_knn_q8_workspace_bytes(B, N), "ofr_knn_q8: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  q8s::TileArgs a;
  a.G1 = G1; a.G2 = G2; a.N = N; a.ldk = ldk; a.gscale = gscale; a.aux = aux;
  a.Q1 = Q1; a.Q2 = Q2; a.B = B; a.qscale = qscale;
  a.nk = (int)cdiv(d, q8s::BK);
  a.cand = reinterpret_cast<Cand*>(workspace);
  a.ntq = cdiv(B, q8s::TQ);
  a.ntg = cdiv(N, q8s::TG);
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_knn_q8: grid too large");
  if (phases & 1) {
    static bool attr_done = false;
    if (!attr_done) {
      hipError_t e = hipFuncSetAttribute((const void*)q8s::tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         q8s::LDS);
      if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(q8 tile)");
      attr_done = true;
    }
    hipLaunchKernelGGL(q8s::tile_kernel, dim3((unsigned)(a.ntq * a.ntg)), dim3(256), q8s::LDS, st, a);
    OFR_LAUNCH_CHECK("q8 tile_kernel");
  }
  if (phases & 2) {
    OFR_CHECK_ARG(out_d && out_i && cert, "ofr_knn_q8: null output");
    q8s::MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, d, qstats, gmax, k, index_base, out_d, out_i, cert};
    hipLaunchKernelGGL(q8s::merge_kernel, dim3((unsigned)B), dim3(256), 0, st, m);
    OFR_LAUNCH_CHECK("q8 merge_kernel");
  }
  return OFR_OK;
}
