// Chi-square nearest-neighbour search on gfx950 (VALU tile kernel).
//
// Replaces ChiSquareDistance (reference distance.py:112-116,
// sum((p-q)^2 / (p+q+eps))) inside NearestNeighbor.predict
// (classifier.py:104-119) for LBP spatial histograms (feature.py:286-302).
//
// chi^2 has no bilinear form, so it runs on the vector ALUs: one workgroup
// computes a 64-query x 64-gallery tile, 4x4 pairs per thread, histogram bins
// streamed through LDS in [bin][row] panels of 64 bins (uint8/16/32 counts or
// fp32 values widened once on the LDS write).  Coarse fp32 score per pair:
//     S = sum_b (a-c)^2 * rcp(a+c)   on values staged + 2^-100 (empty bins give exact 0)
// The best KC rows per query per tile go to cand[tile][query][KC]; the merge
// kernel then re-evaluates the reference formula EXACTLY in fp64 on the
// survivors, with p = value/denom (denom = cell pixel count for counts, the
// reference histogram being count/(py*px)) and eps = 2^-52.
#include "ofr_topk.h"

namespace ofr {

enum { DT_U8 = 0, DT_U16 = 1, DT_U32 = 2, DT_F32 = 3 };
constexpr int C2_TQ = 64, C2_TG = 64, C2_BB = 64;
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int DT>
__device__ __forceinline__ void load16(const void* base, int64_t ld, int64_t row, int64_t b0, float (&v)[16]) {
  if constexpr (DT == DT_U8) {
    const uint4 x = *reinterpret_cast<const uint4*>((const uint8_t*)base + row * ld + b0);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = (float)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
  } else if constexpr (DT == DT_U16) {
    const uint4* p = reinterpret_cast<const uint4*>((const uint16_t*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4 x = p[h];
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) v[8 * h + i] = (float)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
    }
  } else if constexpr (DT == DT_U32) {
    const uint4* p = reinterpret_cast<const uint4*>((const uint32_t*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint4 x = p[h];
      v[4 * h + 0] = (float)x.x;
      v[4 * h + 1] = (float)x.y;
      v[4 * h + 2] = (float)x.z;
      v[4 * h + 3] = (float)x.w;
    }
  } else {
    const f32x4* p = reinterpret_cast<const f32x4*>((const float*)base + row * ld + b0);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const f32x4 x = p[h];
      v[4 * h + 0] = x[0];
      v[4 * h + 1] = x[1];
      v[4 * h + 2] = x[2];
      v[4 * h + 3] = x[3];
    }
  }
}

template <int DT>
__device__ __forceinline__ double load1(const void* base, int64_t idx) {
  if constexpr (DT == DT_U8) return (double)((const uint8_t*)base)[idx];
  else if constexpr (DT == DT_U16) return (double)((const uint16_t*)base)[idx];
  else if constexpr (DT == DT_U32) return (double)((const uint32_t*)base)[idx];
  else return (double)((const float*)base)[idx];
}

struct Chi2Args {
  const void* Q;
  int64_t B, ldq;
  const void* G;
  int64_t N, ldg;
  int64_t nbins;
  Cand* cand;  // [T][B][KC]
  int64_t ntq, ntg;
  double denom;   // exact pass: reference values are element / denom
};

// Exact pass (the certificate's fallback, few queries): the reference formula distance.py:115-116
// in fp64 per (pair, bin) -- p = value / denom, (p - q)^2 / (p + q + eps) -- on 16 x 16 pairs
// per workgroup, values staged once as fp64 p = v / denom in LDS.  The tile lists carry the sum
// rounded to fp32 (a 2^-24 relative key; the merge re-evaluates the survivors in fp64 again).
constexpr int C2X_T = 32;
template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_exact_tile_kernel(Chi2Args p) {
  __shared__ double Qs[C2_BB][C2X_T];
  __shared__ double Gs[C2_BB][C2X_T + 1];
  __shared__ float S[C2X_T][C2X_T + 1];
  const int64_t t = blockIdx.x;
  const int64_t gt = t / p.ntq, qt = t % p.ntq;
  const int64_t q0 = qt * C2X_T, g0 = gt * C2X_T;
  const int tid = threadIdx.x;
  const int tq = tid >> 4, tg = tid & 15;      // queries tq*2.., gallery tg*2..
  const double eps = 2.220446049250313e-16;    // np.finfo('float').eps, distance.py:115
  double acc[2][2] = {{0, 0}, {0, 0}};
  for (int64_t b0 = 0; b0 < p.nbins; b0 += C2_BB) {
    __syncthreads();
    for (int e = tid; e < C2_BB * C2X_T; e += 256) {
      const int r = e / C2_BB, b = e % C2_BB;
      const int64_t bb = b0 + b;
      const int64_t qr = min(q0 + r, p.B - 1), gr = min(g0 + r, p.N - 1);
      Qs[b][r] = bb < p.nbins ? load1<DT>(p.Q, qr * p.ldq + bb) / p.denom : 0.0;
      Gs[b][r] = bb < p.nbins ? load1<DT>(p.G, gr * p.ldg + bb) / p.denom : 0.0;
    }
    __syncthreads();
    const int nb = (int)min((int64_t)C2_BB, p.nbins - b0);
    for (int b = 0; b < nb; ++b) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const double x = Qs[b][tq * 2 + i], y = Gs[b][tg * 2 + j];
          const double df = x - y;
          acc[i][j] += (df * df) / (x + y + eps);
        }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) S[tq * 2 + i][tg * 2 + j] = (float)acc[i][j];
  __syncthreads();
  if (tid < C2X_T) {
    const int64_t q = q0 + tid;
    TopList<KC> L;
    L.init();
    for (int j = 0; j < C2X_T; ++j) {
      const int64_t g = g0 + j;
      if (g < p.N) L.insert(S[tid][j], (int)g);
    }
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_tile_kernel(Chi2Args p) {
  __shared__ __attribute__((aligned(16))) float Qs[C2_BB][C2_TQ];
  __shared__ __attribute__((aligned(16))) float Gs[C2_BB][C2_TG];
  __shared__ float S[C2_TQ][C2_TG + 1];
  const int64_t t = blockIdx.x;
  const int64_t gt = t / p.ntq, qt = t % p.ntq;  // consecutive blocks share the gallery tile
  const int64_t q0 = qt * C2_TQ, g0 = gt * C2_TG;
  const int tid = threadIdx.x;
  const int tq = tid >> 4, tg = tid & 15;       // compute: queries tq*4.., gallery tg*4..
  const int lrow = tid >> 2, lseg = tid & 3;    // staging: row, 16-bin segment
  const int64_t qrow = min(q0 + lrow, p.B - 1);
  const int64_t grow = min(g0 + lrow, p.N - 1);

  f32x2 acc2[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc2[i][0] = acc2[i][1] = f32x2{0.f, 0.f};

  float vq[16], vg[16];
  const int nsteps = (int)(p.nbins / C2_BB);
  if (nsteps > 0) {
    load16<DT>(p.Q, p.ldq, qrow, lseg * 16, vq);
    load16<DT>(p.G, p.ldg, grow, lseg * 16, vg);
  }
  for (int s = 0; s < nsteps; ++s) {
    __syncthreads();
    // values are staged biased by 2^-100: a + c > 0 for every pair (no per-pair "+ tiny"), while
    // a - c and (a + c) for a, c >= 2^-76 round exactly as without the bias
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      Qs[lseg * 16 + i][lrow] = vq[i] + 0x1p-100f;
      Gs[lseg * 16 + i][lrow] = vg[i] + 0x1p-100f;
    }
    __syncthreads();
    if (s + 1 < nsteps) {
      load16<DT>(p.Q, p.ldq, qrow, (int64_t)(s + 1) * C2_BB + lseg * 16, vq);
      load16<DT>(p.G, p.ldg, grow, (int64_t)(s + 1) * C2_BB + lseg * 16, vg);
    }
    // packed fp32: per two (pair, bin) terms one v_pk_add for a - c, one for a + c, two v_rcp,
    // v_pk_mul, v_pk_fma
#pragma unroll 4
    for (int b = 0; b < C2_BB; ++b) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(&Qs[b][tq * 4]);
      const f32x4 c = *reinterpret_cast<const f32x4*>(&Gs[b][tg * 4]);
      const f32x2 c01 = {c[0], c[1]}, c23 = {c[2], c[3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 ai = {a[i], a[i]};
        const f32x2 d0 = ai - c01, s0 = ai + c01, d1 = ai - c23, s1 = ai + c23;
        const f32x2 r0 = {__builtin_amdgcn_rcpf(s0[0]), __builtin_amdgcn_rcpf(s0[1])};
        const f32x2 r1 = {__builtin_amdgcn_rcpf(s1[0]), __builtin_amdgcn_rcpf(s1[1])};
        acc2[i][0] = __builtin_elementwise_fma(d0 * d0, r0, acc2[i][0]);
        acc2[i][1] = __builtin_elementwise_fma(d1 * d1, r1, acc2[i][1]);
      }
    }
  }
  float acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = acc2[i][j >> 1][j & 1];
  // tail bins (nbins % 64): plain loads
  for (int64_t b = (int64_t)nsteps * C2_BB; b < p.nbins; ++b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = (float)load1<DT>(p.Q, min(q0 + tq * 4 + i, p.B - 1) * p.ldq + b);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float c = (float)load1<DT>(p.G, min(g0 + tg * 4 + j, p.N - 1) * p.ldg + b);
        const float df = a - c;
        acc[i][j] = __builtin_fmaf(df * df, __builtin_amdgcn_rcpf((a + c) + 1e-30f), acc[i][j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) S[tq * 4 + i][tg * 4 + j] = acc[i][j];
  __syncthreads();
  if (tid < C2_TQ) {
    const int64_t q = q0 + tid;
    TopList<KC> L;
    L.init();
    for (int j = 0; j < C2_TG; ++j) {
      const int64_t g = g0 + j;
      if (g < p.N) L.insert(S[tid][j], (int)g);
    }
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)gt * p.B + q) * KC;
#pragma unroll
      for (int j = 0; j < KC; ++j) out[j] = Cand{L.d[j], L.i[j]};
    }
  }
}

struct Chi2MergeArgs {
  const Cand* cand;
  int64_t T, B;
  const void* Q;
  int64_t ldq;
  const void* G;
  int64_t ldg, nbins;
  double denom;
  int k;
  int64_t index_base;
  double* out_d;
  int64_t* out_i;
  int* cert;      // nullable: 1 iff the result is provably the exact fp64 top-k
  double gamma;   // relative error bound of the coarse scores (and their keys)
  double scale;   // coarse score -> reference units (1 / denom for the fp32 pass, 1 for the exact pass)
};

template <int DT, int KC>
__global__ void __launch_bounds__(256) chi2_merge_rerank_kernel(Chi2MergeArgs p) {
  __shared__ Cand lists[256 * KC];
  __shared__ double exact[KC];
  __shared__ double red[4];
  const int64_t q = blockIdx.x;
  select_candidates<KC>(p.cand, p.T, p.B, q, lists);
  const double eps = 2.220446049250313e-16;  // np.finfo('float').eps, distance.py:115
  for (int c = 0; c < KC; ++c) {
    const Cand cc = lists[c];
    double val = __builtin_inf();
    if (cc.i != CAND_EMPTY) {
      double a = 0;
      for (int64_t b = threadIdx.x; b < p.nbins; b += blockDim.x) {
        const double x = load1<DT>(p.Q, q * p.ldq + b) / p.denom;
        const double y = load1<DT>(p.G, (int64_t)cc.i * p.ldg + b) / p.denom;
        const double df = x - y;
        a += (df * df) / (x + y + eps);
      }
      val = block_sum_f64(a, red);
    }
    if (threadIdx.x == 0) exact[c] = val;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double* od = p.out_d + q * p.k;
    sort_and_write<KC>(lists, exact, p.k, p.index_base, od, p.out_i + q * p.k);
    if (p.cert) {
      // certificate: every row outside the KC candidates has coarse score >= tau (the KC-th
      // candidate; a tile's excluded rows are >= its own KC-th, which is >= tau), so its exact
      // distance is >= tau * scale / (1 + gamma).  The top-k is exact iff the k-th exact distance
      // lies strictly below that (a relative 1e-12 for the fp64 evaluation order).
      const int kk = p.k < KC ? p.k : KC;
      const Cand last = lists[KC - 1];
      const double dk = od[kk - 1];
      double bnd = __builtin_inf();
      if (last.i != CAND_EMPTY) bnd = (double)last.d * p.scale / (1.0 + p.gamma) * (1.0 - 1e-12);
      p.cert[q] = (dk == dk) && (dk < bnd);
    }
  }
}

template <int DT, int KC>
static int launch_chi2(hipStream_t st, const Chi2Args& a, const Chi2MergeArgs& m, bool exact) {
  if (a.N > 0) {
    if (exact)
      hipLaunchKernelGGL((chi2_exact_tile_kernel<DT, KC>), dim3((unsigned)(a.ntq * a.ntg)), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((chi2_tile_kernel<DT, KC>), dim3((unsigned)(a.ntq * a.ntg)), dim3(256), 0, st, a);
    OFR_LAUNCH_CHECK("chi2_tile_kernel");
  }
  hipLaunchKernelGGL((chi2_merge_rerank_kernel<DT, KC>), dim3((unsigned)m.B), dim3(256), 0, st, m);
  OFR_LAUNCH_CHECK("chi2_merge_rerank_kernel");
  return OFR_OK;
}

template <int DT>
static int chi2_dispatch(hipStream_t st, int kc, const Chi2Args& a, const Chi2MergeArgs& m, bool exact) {
  return kc == 8 ? launch_chi2<DT, 8>(st, a, m, exact) : launch_chi2<DT, 16>(st, a, m, exact);
}

}  // namespace ofr

using namespace ofr;

extern "C" size_t ofr_chi2_workspace_bytes(int64_t B, int64_t N, int k) {
  const int kc = pick_kc(k);
  const int64_t T = cdiv(N > 0 ? N : 1, C2X_T);   // the exact pass's 32-row tiles (>= the 64-row ones)
  return (size_t)T * (size_t)B * kc * sizeof(Cand) + 256;
}

static int chi2_run(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                    int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                    int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert, bool exact) {
  OFR_CHECK_ARG(dtype >= DT_U8 && dtype <= DT_F32, "ofr_chi2_knn: dtype must be 0 (u8), 1 (u16), 2 (u32) or 3 (f32)");
  OFR_CHECK_ARG(B >= 0 && N >= 0 && nbins >= 1 && denom > 0, "ofr_chi2_knn: bad sizes");
  if (k < 1 || k > OFR_MAX_K) return fail(OFR_E_UNSUPPORTED, "ofr_chi2_knn: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  const int esz = dtype == DT_U8 ? 1 : dtype == DT_U16 ? 2 : 4;
  OFR_CHECK_ARG(Q && out_d && out_i && workspace, "ofr_chi2_knn: null pointer");
  OFR_CHECK_ARG(ldq >= nbins && (ldq * esz) % 16 == 0 && ((uintptr_t)Q % 16) == 0,
                "ofr_chi2_knn: query rows must be 16-byte aligned (ldq*elem % 16 == 0)");
  if (N > 0) {
    OFR_CHECK_ARG(G, "ofr_chi2_knn: null gallery");
    OFR_CHECK_ARG(ldg >= nbins && (ldg * esz) % 16 == 0 && ((uintptr_t)G % 16) == 0,
                  "ofr_chi2_knn: gallery rows must be 16-byte aligned (ldg*elem % 16 == 0)");
    OFR_CHECK_ARG(N < 0x7fffffffLL - C2_TG, "ofr_chi2_knn: N too large for one shard");
  }
  const int kc = pick_kc(k);
  OFR_CHECK_ARG(workspace_bytes >= ofr_chi2_workspace_bytes(B, N, k), "ofr_chi2_knn: workspace too small");
  Chi2Args a;
  a.Q = Q; a.B = B; a.ldq = ldq; a.G = G; a.N = N; a.ldg = ldg; a.nbins = nbins; a.denom = denom;
  a.cand = reinterpret_cast<Cand*>(workspace);
  const int tq = exact ? C2X_T : C2_TQ, tg = exact ? C2X_T : C2_TG;
  a.ntq = cdiv(B, tq);
  a.ntg = N > 0 ? cdiv(N, tg) : 0;
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_chi2_knn: grid too large");
  // error bound of the coarse scores (relative): the fp32 pass sums ceil(nbins / 2) terms per
  // accumulator sequentially (two packed halves) and each term d^2 * rcp(s) carries <= 2 ulp
  // (d, s exact for integer counts < 2^24; <= 2 more ulp from their roundings for fp32 values);
  // the exact pass's key is its fp64 sum rounded to fp32 (1/2 ulp) plus the fp64 summation.
  const double gamma = exact ? 0x1p-23 + (double)nbins * 0x1p-52
                             : ((double)((nbins + 1) / 2) + 4.0) * 0x1p-24 + (dtype == DT_F32 ? 4.0 : 2.0) * 0x1p-23;
  Chi2MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, nbins, denom, k, index_base, out_d, out_i, cert, gamma,
                  exact ? 1.0 : 1.0 / denom};
  hipStream_t st = (hipStream_t)stream;
  switch (dtype) {
    case DT_U8: return chi2_dispatch<DT_U8>(st, kc, a, m, exact);
    case DT_U16: return chi2_dispatch<DT_U16>(st, kc, a, m, exact);
    case DT_U32: return chi2_dispatch<DT_U32>(st, kc, a, m, exact);
    default: return chi2_dispatch<DT_F32>(st, kc, a, m, exact);
  }
}

extern "C" int ofr_chi2_knn(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G, int64_t N,
                            int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base, double* out_d,
                            int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert) {
  return chi2_run(stream, dtype, Q, B, ldq, G, N, ldg, nbins, denom, k, index_base, out_d, out_i, workspace,
                  workspace_bytes, cert, false);
}

extern "C" int ofr_chi2_knn_exact(void* stream, int dtype, const void* Q, int64_t B, int64_t ldq, const void* G,
                                  int64_t N, int64_t ldg, int64_t nbins, double denom, int k, int64_t index_base,
                                  double* out_d, int64_t* out_i, void* workspace, size_t workspace_bytes, int* cert) {
  return chi2_run(stream, dtype, Q, B, ldq, G, N, ldg, nbins, denom, k, index_base, out_d, out_i, workspace,
                  workspace_bytes, cert, true);
}
