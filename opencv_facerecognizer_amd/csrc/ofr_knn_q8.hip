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
// per query (as keys: the score truncated toward -inf by < 256 ulp, ties by
// row); the merge keeps the best R=16 overall (tau = the 16th, truncated).
// Every row outside the final list has S~ >= tau (a tile contributing < 16
// rows below tau cannot hide one; truncation only lowers tau).  After the EXACT fp64 re-rank of the 16
// candidates, the top-k is proven equal to the exact top-k when
//     S_k(exact) < tau - dS(q)
// (strictly: no excluded row can reach or tie the k-th).  cert[q] = 1 then;
// otherwise 0 and the caller re-runs that query on the fp32 path.
#include <cstdlib>
#include <type_traits>

#include "ofr_f6_tile.h"
#include "ofr_i8_tile.h"
#include "ofr_keys.h"
#include "ofr_topk.h"

namespace ofr {
namespace q8s {

using i8t::i32x4;
using i8t::i32x16;
using i8t::Shape;

constexpr int KC = 16;
constexpr int TG = i8t::TA;                        // gallery rows per tile
constexpr int GROUP_G = 4;                         // gallery tiles per tile group (i8t::tile_coords)

struct TileArgs {
  const int8_t* G;     // gallery slices [N][ld]
  int64_t N, ld;
  const float* gscale;
  const float* aux;
  const int8_t* Q;     // query slices [B][ld]
  int64_t B;
  const float* qscale;
  int nk;
  Cand* cand;   // [B][T][KC] (query-major)
  int64_t ntq, ntg;
  int64_t gg;   // gallery tiles per tile group (see tile_coords)
  // fp6 sieve (tile_kernel_f6 MODE 8, see below); gstride: tile t reads gallery panel t * gstride
  int64_t gstride;
  const uint32_t* theta;   // [B] keep threshold (a key with the low byte 0; KEY_NONE keeps every row)
  int* count;              // [B] rows kept so far
  Cand* bucket;            // [B][cap] the kept rows (truncated coarse score, row)
  int64_t cap;
  // two-slice fp6 tier (NSEG = 3 kernels): the second-slice tiles; nk = 3 x the stages of one slice
  const int8_t* G2;
  const int8_t* Q2;
  int serp;   // wide sieve pass: odd tile groups walk the query tiles backwards (tile_kernel_f6w)
  // fp6 tiers: column-block scales, one dword of 4 E8M0 bytes per 128-feature stage (null: unit;
  // ofr_f6_block_scales), the same for the gallery and the query tiles
  const uint32_t* bs;
  // stages run per segment: nk / NSEG, or fewer -- the prefix tier f6p scores only the first nkp
  // stages of the tiles (nk stays their layout)
  int nkp;
  // stages per 256-row panel of the GALLERY tiles the prefix passes read (round 6: the prefix tier's own
  // compact tiles, ofr_f6p_quantize_rows, hold only its nkp stages; every other pass: nk)
  int gnk;
};

// ---- keys of the tile epilogue (ofr_keys.h: order-preserving u32 keys, med3 key lists) ----
static_assert(keys::KC == KC, "key lists hold KC candidates");
using keys::KEY_NONE;
using keys::KeyList;
using keys::key_float;
using keys::key_score;
using keys::med3;
using keys::score_key;
using keys::umax;
using keys::umin;

// Tile epilogue shared by the int8 and fp6 engines: coarse scores -> keys, per-lane best
// 16 of the lane's 64 gallery rows, merge with the partner half-wave, then across the two
// row-waves through LDS; writes the tile's best KC per query to p.cand.
// cval(rt, ctc, r): coarse product q~.g~ / (s_q s_g) of accumulator register r of row block
// rt and query block ctc (an integral_constant: a runtime index would send acc to scratch).
template <int CT, int TQ, int QW, int WQ, class CV>
__device__ __forceinline__ void tile_epilogue(char* smem, const TileArgs& p, int64_t gt, int64_t g0, int64_t q0,
                                              CV&& cval) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / WQ, wc = wave % WQ, h = lane >> 5, r32 = lane & 31;
  uint32_t* kbuf = reinterpret_cast<uint32_t*>(smem);                      // [2][TQ][KC]
  float* gtab = reinterpret_cast<float*>(smem + 2 * TQ * KC * 4);          // [TG][2]
  if (threadIdx.x < TG) {
    const int64_t g = g0 + threadIdx.x;
    const bool ok = g < p.N;
    gtab[2 * threadIdx.x + 0] = ok ? p.aux[g] : 0.f;
    gtab[2 * threadIdx.x + 1] = ok ? p.gscale[g] : 0.f;
  }
  __syncthreads();
  const int nvalid = p.N - g0 < TG ? (int)(p.N - g0) : TG;
  auto epi = [&](auto ctc) {
    constexpr int ct = decltype(ctc)::value;
    if constexpr (ct < CT) {
      const int ql = wc * QW + ct * 32 + r32;
      const int64_t q = q0 + ql;
      const float sq2 = 2.0f * p.qscale[q < p.B ? q : p.B - 1];
      KeyList L;
      L.init();
#pragma unroll
      for (int rt = 0; rt < 4; ++rt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int gl = wr * 128 + rt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float c = cval(rt, ctc, r);
          const float sc = gtab[2 * gl] - sq2 * gtab[2 * gl + 1] * c;
          L.insert(gl < nvalid ? score_key(sc, gl) : KEY_NONE);
        }
      uint32_t o[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) o[j] = (uint32_t)__shfl_xor((int)L.k[j], 32);
      L.merge(o);
      if (h == 0) {
        uint32_t* dst = kbuf + ((size_t)wr * TQ + ql) * KC;
#pragma unroll
        for (int j = 0; j < KC; j += 4)
          *reinterpret_cast<uint4*>(dst + j) = make_uint4(L.k[j], L.k[j + 1], L.k[j + 2], L.k[j + 3]);
      }
    }
  };
  static_assert(CT <= 4, "epilogue unroll");
  epi(std::integral_constant<int, 0>{});
  epi(std::integral_constant<int, 1>{});
  epi(std::integral_constant<int, 2>{});
  epi(std::integral_constant<int, 3>{});
  __syncthreads();
  if ((int)threadIdx.x < TQ) {
    const int ql = threadIdx.x;
    const int64_t q = q0 + ql;
    KeyList L;
    uint32_t o[KC];
    const uint32_t* s0 = kbuf + (size_t)ql * KC;
    const uint32_t* s1 = kbuf + ((size_t)TQ + ql) * KC;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      L.k[j] = s0[j];
      o[j] = s1[j];
    }
    L.merge(o);
    if (q < p.B) {
      Cand* out = p.cand + ((size_t)q * p.ntg + gt) * KC;   // query-major: the merge streams one query's lists
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        const uint32_t kk = L.k[j];
        out[j] = kk == KEY_NONE ? Cand{__builtin_inff(), CAND_EMPTY}
                                : Cand{key_score(kk), (int)(g0 + (kk & 0xffu))};
      }
    }
  }
}

// ---- fp6 sieve ------------------------------------------------------------------------
// The list epilogue above costs ~10 us per tile (64 sorted inserts per lane and query block)
// and writes 16 candidates per (query, tile): 2 GB per pass at B = 4096, N = 1M.  The sieve
// replaces it for the fp6 tier at B > 32.  A sample pass (the list kernel over every
// SIEVE_STRIDE-th gallery tile) gives per query theta = the 16th best truncated key of the
// sample, an upper bound of the 16th best over the whole gallery.  The full pass then keeps
// only rows whose truncated key is <= theta (one compare per (query, row); hits are staged in
// LDS and appended to a per-query bucket), ~16 * SIEVE_STRIDE rows per query on gallery-like
// data.  Certificate (merge_kernel): a row outside the final 16 either failed the test
// (truncated key > theta) or was kept and lost to the 16th, so tau = min(theta, 16th kept)
// bounds every excluded row exactly as before.  theta only steers the volume: a bucket that
// overflows its cap makes the query uncertified (bound -inf), never wrong.
constexpr int64_t SIEVE_STRIDE = 64;   // panel sample (ofr_knn_f6): gallery tiles 0, 64, 128, ...
constexpr int64_t SIEVE_CAP = 32768;   // kept rows per query (256 KiB; ~16 * SIEVE_STRIDE expected, heavy tail)
constexpr int SIEVE_HCAP = 8192;       // LDS hit slots per tile (64 KiB)
constexpr int SIEVE_RANK = 16;         // theta = this-th best key of the sample (ofr_knn_f6's sieve_rank)
// ofr_knn_f6_sampled: the sample is a row sample (gallery rows 0, 64, 128, ...: ofr_f6_sample_rows)
// instead of whole panels, theta its SIEVE_RANK_ROWS-th best key (~4 x 64 rows kept per query)
constexpr int64_t SAMPLE_STEP = 64;
constexpr int SIEVE_RANK_ROWS = 4;

// Hits of one 256 x 256 tile: (a, s) = (aux, gscale) of gallery row threadIdx.x (padding rows:
// (+inf, 0); they are also excluded explicitly, since a NaN th passes everything), sq2 / th per
// query block of this lane (th = key_float(theta | 0xff): truncated key <= theta  <=>
// !(score > th); NaN for KEY_NONE keeps every row).  More than SIEVE_HCAP hits in one tile push
// every query of the tile past its bucket cap (uncertified, no candidates read by the merge).
template <int TQ, int GB = 8, int TGR = TG, int HCAP = SIEVE_HCAP>
__device__ __forceinline__ void sieve_flush(char* smem, const TileArgs& p, int64_t g0, int64_t q0);

// The tile's staged hits -> per-query buckets (after the compares and a barrier).  A hit packs
// (tile query << GB) | tile gallery row; TGR gallery rows per tile (the staging area follows their
// [TGR][2] operand table), HCAP staging slots.
template <int TQ, int GB, int TGR, int HCAP>
__device__ __forceinline__ void sieve_flush(char* smem, const TileArgs& p, int64_t g0, int64_t q0) {
  const uint32_t* nhit = reinterpret_cast<const uint32_t*>(smem + TGR * 8);
  const uint2* hits = reinterpret_cast<const uint2*>(smem + TGR * 8 + 16);
  const uint32_t nh = *nhit;
  if (nh > (uint32_t)HCAP) {   // hits lost: push every query of the tile past its cap (uncertified)
    // saturating (max, not add): any number of overflowing tiles leaves the count at cap + 1 plus
    // at most one increment per gallery row, which the host bounds below 2^31 (ofr_knn_f6)
    if ((int)threadIdx.x < TQ && q0 + threadIdx.x < p.B) atomicMax(p.count + q0 + threadIdx.x, (int)p.cap + 1);
    return;
  }
  for (uint32_t e = threadIdx.x; e < nh; e += blockDim.x) {
    const uint2 hv = hits[e];
    const int64_t q = q0 + (int)(hv.y >> GB);
    const int gl = (int)(hv.y & ((1u << GB) - 1u));
    if (q < p.B) {
      const int slot = atomicAdd(p.count + q, 1);
      if (slot < p.cap) p.bucket[q * p.cap + slot] = Cand{__uint_as_float(hv.x), (int)(g0 + gl)};
    }
  }
}

// The int8 tiers' tile pass (SL int8 slices per row): per (query, tile) the best KC keys.
template <int SL>
__global__ void __launch_bounds__(Shape<SL>::NT, 1) tile_kernel(TileArgs p) {
  using S = Shape<SL>;
  constexpr int CT = S::CT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  const int64_t g0 = gt * TG, q0 = qt * S::TQ;

  i32x16 acc0[4][CT], acc1[4][SL == 2 ? CT : 1];
  i8t::mainloop<SL, false>(smem, p.G, p.ld, p.N, g0, p.Q, p.ld, p.B, q0, p.ld, p.nk, acc0, acc1);
  tile_epilogue<CT, S::TQ, S::QW, S::WQ>(smem, p, gt, g0, q0, [&](int rt, auto ctc, int r) {
    constexpr int ct = decltype(ctc)::value;
    float c = (float)acc0[rt][ct][r];
    if constexpr (SL == 2) c += (float)acc1[rt][ct][r] * 0x1p-7f;
    return c;
  });
}

// fp6 tier, the sieve's sample pass: p.G / p.Q are f6 tiled buffers (ofr_f6_tile.h), p.nk = stages,
// NW waves (f6t::Engine, 32x32x64 MFMA); tile lists of the best KC keys per (query, tile), tile t =
// gallery panel t * gstride.
template <int NW, int NSEG = 1>
__global__ void __launch_bounds__(NW * 64, 1) tile_kernel_f6(TileArgs p) {
  using E = f6t::Engine<NW>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int CT = E::CT;
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  const int64_t gp = gt * p.gstride;
  const int64_t g0 = gp * TG, q0 = qt * f6t::TQ;
  f6t::f32x16 acc[4][CT];
  E::template mainloop<NSEG>(smem, reinterpret_cast<const char*>(p.G), gp, reinterpret_cast<const char*>(p.Q), qt,
                             p.nk / NSEG, p.nkp, acc, reinterpret_cast<const char*>(p.G2),
                             reinterpret_cast<const char*>(p.Q2), p.bs);
  auto cval = [&](int rt, auto ctc, int r) {
    constexpr int ct = decltype(ctc)::value;
    return acc[rt][ct][r];
  };
  tile_epilogue<CT, f6t::TQ, E::QW, E::WQ>(smem, p, gt, g0, q0, cval);
}

// Sieve epilogue of the 16x16x128 engine (f6t::Engine16): element reg r of accumulator (i, c) of
// lane l is gallery row wr*128 + 16 i + 4 (l / 16) + r, query wc*64 + 16 c + l % 16.
__device__ __forceinline__ void sieve_epilogue16(char* smem, const TileArgs& p, int64_t g0, int64_t q0, float ga,
                                                 float gs, const float (&sq2)[4], const float (&th)[4],
                                                 const f6t::f32x4 (&acc)[8][4]) {
  using E = f6t::Engine16;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = wave / E::WQ, wc = wave % E::WQ, g4 = (lane >> 4) * 4, r16 = lane & 15;
  float* gtab = reinterpret_cast<float*>(smem);                                  // [TG][2]
  uint32_t* nhit = reinterpret_cast<uint32_t*>(smem + TG * 8);
  uint2* hits = reinterpret_cast<uint2*>(smem + TG * 8 + 16);                    // [SIEVE_HCAP]
  const int nvalid = p.N - g0 < TG ? (int)(p.N - g0) : TG;
  if (threadIdx.x < TG) {
    gtab[2 * threadIdx.x + 0] = ga;
    gtab[2 * threadIdx.x + 1] = gs;
  }
  if (threadIdx.x == 0) *nhit = 0;
  __syncthreads();
  // per row block the lane's 16 compares first (branch-free), then one wave-wide test: a block holds
  // ~1 kept pair per wave on gallery data, so most blocks skip the staging (f6w_body, round 3)
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int gl0 = wr * 128 + i * 16 + g4;        // this lane's 4 consecutive gallery rows
    const float4 t0 = reinterpret_cast<const float4*>(gtab)[gl0 / 2];
    const float4 t1 = reinterpret_cast<const float4*>(gtab)[gl0 / 2 + 1];
    const float av[4] = {t0.x, t0.z, t1.x, t1.z}, sv[4] = {t0.y, t0.w, t1.y, t1.w};
    float sc[4][4];
    uint32_t m = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[r][c] = av[r] - sq2[c] * sv[r] * acc[i][c][r];
        m |= (!(sc[r][c] > th[c]) && gl0 + r < nvalid) ? 1u << (r * 4 + c) : 0u;
      }
    if (__builtin_amdgcn_ballot_w64(m != 0) == 0) continue;   // uniform
    while (m) {   // rare: ~16 * SIEVE_STRIDE of the N rows per query
      const int b = __builtin_ctz(m);
      m &= m - 1;
      const int r = b >> 2, c = b & 3;
      float v = sc[0][0];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) v = (rr * 4 + cc == b) ? sc[rr][cc] : v;
      const int ql = wc * E::QW + c * 16 + r16;
      const uint32_t kb = __float_as_uint(key_score(score_key(v, 0)));
      const uint32_t slot = atomicAdd(nhit, 1u);
      if (slot < (uint32_t)SIEVE_HCAP) hits[slot] = make_uint2(kb, ((uint32_t)ql << 8) | (uint32_t)(gl0 + r));
    }
  }
  __syncthreads();
  sieve_flush<f6t::TQ>(smem, p, g0, q0);
}

// fp6 sieve pass on the 16x16x128 engine (f6t::Engine16, 256 x 256 tiles, 8 waves): the two-slice
// tier's engine (NSEG = 3) and the sieve pass under OFR_F6_SHAPE=16.
template <int NSEG = 1>
__global__ void __launch_bounds__(512, 1) tile_kernel_f6s(TileArgs p) {
  using E = f6t::Engine16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  const int64_t gp = gt * p.gstride;
  const int64_t g0 = gp * TG, q0 = qt * f6t::TQ;
  f6t::f32x4 acc[8][4];
  E::mainloop<NSEG>(smem, reinterpret_cast<const char*>(p.G), gp, reinterpret_cast<const char*>(p.Q), qt, p.nk / NSEG,
                    p.nkp, acc, reinterpret_cast<const char*>(p.G2), reinterpret_cast<const char*>(p.Q2), p.bs);
  // sieve operands after the main loop (the 16x16 engine needs every register in it)
  float ga = __builtin_inff(), gs = 0.f, sq2[4], th[4];
  if (threadIdx.x < TG && g0 + threadIdx.x < p.N) {
    ga = p.aux[g0 + threadIdx.x];
    gs = p.gscale[g0 + threadIdx.x];
  }
  const int wc = (threadIdx.x >> 6) % E::WQ, r16 = threadIdx.x & 15;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int64_t q = q0 + wc * E::QW + c * 16 + r16;
    const bool ok = q < p.B;
    sq2[c] = 2.0f * p.qscale[ok ? q : p.B - 1];
    th[c] = ok ? key_float(p.theta[q] | 0xffu) : -__builtin_inff();
  }
  sieve_epilogue16(smem, p, g0, q0, ga, gs, sq2, th, acc);
}

// fp6 sieve pass on the wide engine (f6t::EngineW): 384 gallery x 256 query tiles, 4 waves (one per
// SIMD), p.ntg = ceil(N / 384) gallery tiles; NSEG = 3: the two-slice tier's three segments of p.nk / 3
// stages (p.G2 / p.Q2 the second slices).  The epilogue is sieve_epilogue16's for the 192 x 128
// wave tile: element r of acc[i][c] of lane l is gallery row WR*192 + 16 i + 4 (l / 16) + r, query
// WC*128 + 16 c + l % 16.
// The wave's main loop (its copy-piece offsets compile-time: one body per wave index W) ...
template <int W, int NSEG>
__device__ __forceinline__ void f6w_main(const TileArgs& p, int64_t g0, int64_t q0,
                                         f6t::f32x4 (&acc)[f6t::EngineW::NA][f6t::EngineW::NB]) {
  using E = f6t::EngineW;
  E::Feed f;
  E::feed_init<W, NSEG>(f, reinterpret_cast<const char*>(p.G), p.N, reinterpret_cast<const char*>(p.Q), q0 / f6t::TQ,
                        p.nk / NSEG, g0 / E::TGW, reinterpret_cast<const char*>(p.G2),
                        reinterpret_cast<const char*>(p.Q2), p.bs, p.gnk / NSEG);
  E::mainloop<W, NSEG>(f, p.nkp, acc);
}

// ... and the sieve epilogue, ONE copy for the four waves (the wave's row / column offsets at run time):
// four specialised copies of its ~4,000 instructions (the 384 unrolled hit sites) overflowed the
// instruction cache every tile.
__device__ __forceinline__ void f6w_epilogue(char* smem, const TileArgs& p, int64_t g0, int64_t q0, int wave,
                                             f6t::f32x4 (&acc)[f6t::EngineW::NA][f6t::EngineW::NB]) {
  using E = f6t::EngineW;
  const int WR = wave >> 1;
  float* gtab = reinterpret_cast<float*>(smem);                                   // [384][2]
  uint32_t* nhit = reinterpret_cast<uint32_t*>(smem + E::TGW * 8);
  uint2* hits = reinterpret_cast<uint2*>(smem + E::TGW * 8 + 16);                 // [HCAPW]
  // 2x SIEVE_HCAP: a 384-row tile collects 1.5x the hits of a 256-row one (loose thresholds, small d)
  constexpr int HCAPW = 2 * SIEVE_HCAP;
  static_assert(E::TGW * 8 + 16 + HCAPW * 8 <= E::LDS_BYTES, "hit staging fits the ring's LDS");
  const int nvalid = p.N - g0 < E::TGW ? (int)(p.N - g0) : E::TGW;
  for (int r = threadIdx.x; r < E::TGW; r += E::NT) {
    const bool ok = r < nvalid;
    gtab[2 * r + 0] = ok ? p.aux[g0 + r] : __builtin_inff();
    gtab[2 * r + 1] = ok ? p.gscale[g0 + r] : 0.f;
  }
  if (threadIdx.x == 0) *nhit = 0;
  const int lane = threadIdx.x & 63, wc = wave & 1, g4 = (lane >> 4) * 4, r16 = lane & 15;
  float sq2[E::NB], th[E::NB];
#pragma unroll
  for (int c = 0; c < E::NB; ++c) {
    const int64_t q = q0 + wc * 128 + c * 16 + r16;
    const bool ok = q < p.B;
    sq2[c] = 2.0f * p.qscale[ok ? q : p.B - 1];
    th[c] = ok ? key_float(p.theta[q] | 0xffu) : -__builtin_inff();
  }
  __syncthreads();
  // Per row block: the lane's 32 coarse scores sc = fma(-(sq2 sv), acc, a) in packed pairs (two rows
  // of one query per v_pk_fma_f32), per query column the min over the 4 rows, one v_cmp_ngt per column
  // (NaN th, "keep every row", passes) and a wave-wide OR: a block holds ~1 kept pair per wave on
  // gallery data, so most blocks skip the staging.  A block that passes re-tests its 32 scores exactly
  // (the padding rows, a = +inf, pass only a NaN th and are excluded there).
  typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int i = 0; i < E::NA; ++i) {
    const int gl0 = WR * 192 + i * 16 + g4;        // this lane's 4 consecutive gallery rows
    const float4 t0 = reinterpret_cast<const float4*>(gtab)[gl0 / 2];
    const float4 t1 = reinterpret_cast<const float4*>(gtab)[gl0 / 2 + 1];
    const f32x2 avp[2] = {f32x2{t0.x, t0.z}, f32x2{t1.x, t1.z}}, svp[2] = {f32x2{t0.y, t0.w}, f32x2{t1.y, t1.w}};
    float sc[4][E::NB];
    uint64_t col[E::NB];   // per query column: the lanes with a candidate hit (wave-uniform)
    uint64_t any = 0;
#pragma unroll
    for (int c = 0; c < E::NB; ++c) {
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const f32x2 t = svp[rp] * sq2[c];
        const f32x2 x = __builtin_elementwise_fma(-t, f32x2{acc[i][c][2 * rp], acc[i][c][2 * rp + 1]}, avp[rp]);
        sc[2 * rp][c] = x.x;
        sc[2 * rp + 1][c] = x.y;
      }
      const float mn = fminf(fminf(sc[0][c], sc[1][c]), fminf(sc[2][c], sc[3][c]));
      col[c] = __builtin_amdgcn_ballot_w64(!(mn > th[c]));
      any |= col[c];
    }
    if (any == 0) continue;   // uniform
    // ~2 kept pairs per block on gallery data, in one or two query columns: only those are examined
#pragma unroll
    for (int c = 0; c < E::NB; ++c) {
      if (col[c] == 0) continue;   // uniform
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!(sc[r][c] > th[c]) && gl0 + r < nvalid) {   // rare: ~16 * SIEVE_STRIDE of the N rows per query
          const int ql = wc * 128 + c * 16 + r16;
          const uint32_t kb = __float_as_uint(key_score(score_key(sc[r][c], 0)));
          const uint32_t slot = atomicAdd(nhit, 1u);
          if (slot < (uint32_t)HCAPW) hits[slot] = make_uint2(kb, ((uint32_t)ql << 9) | (uint32_t)(gl0 + r));
        }
    }
  }
  __syncthreads();
  sieve_flush<f6t::TQ, 9, E::TGW, HCAPW>(smem, p, g0, q0);
}

template <int NSEG>
__global__ void __launch_bounds__(256, 1) tile_kernel_f6w(TileArgs p) {
  using E = f6t::EngineW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  // serpentine: the last query panels of a group are the first of the next, while still in L2
  if (p.serp && ((t / (p.gg * p.ntq)) & 1)) qt = p.ntq - 1 - qt;
  const int64_t g0 = gt * E::TGW, q0 = qt * f6t::TQ;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  f6t::f32x4 acc[E::NA][E::NB];
  if constexpr (NSEG == 1) {
    switch (wave) {   // the wave's role, compile time in the main loop
      case 0: f6w_main<0, NSEG>(p, g0, q0, acc); break;
      case 1: f6w_main<1, NSEG>(p, g0, q0, acc); break;
      case 2: f6w_main<2, NSEG>(p, g0, q0, acc); break;
      default: f6w_main<3, NSEG>(p, g0, q0, acc); break;
    }
    f6w_epilogue(smem, p, g0, q0, wave, acc);
  } else {
    // the two-slice pass keeps one epilogue per wave: compiled shared, its extra segment registers
    // spill and the epilogue read one accumulator (row block 7, query block 7) wrongly
    // (tools/diag_f6x2_engines.py, profiles/r05_diag_f6x2.txt)
    switch (wave) {
      case 0: f6w_main<0, NSEG>(p, g0, q0, acc); f6w_epilogue(smem, p, g0, q0, 0, acc); break;
      case 1: f6w_main<1, NSEG>(p, g0, q0, acc); f6w_epilogue(smem, p, g0, q0, 1, acc); break;
      case 2: f6w_main<2, NSEG>(p, g0, q0, acc); f6w_epilogue(smem, p, g0, q0, 2, acc); break;
      default: f6w_main<3, NSEG>(p, g0, q0, acc); f6w_epilogue(smem, p, g0, q0, 3, acc); break;
    }
  }
}

// ---- prefix tier's sieve pass: persistent, one workgroup per CU ------------------------------------
// With 1 or 2 stages per tile (the prefix tier f6p) the wide engine's tile spends ~6x its MFMA time
// on fixed costs -- the first copies' latency, the operand-table and threshold loads, the epilogue and
// the hit flush -- none of it overlapped (tile_kernel_f6w runs one workgroup per CU: its 384
// accumulators fill the register file).  tile_kernel_f6p keeps one workgroup per CU resident and
// walks work items = (384-row gallery tile, group of query panels).  Per panel:
//   top      the panel's query stages landed (copied during the previous panel's compares); the
//            previous panel's hits get their bucket slots (global atomics, answered under the MFMAs)
//   MFMAs    the nsp stages from LDS (the gallery tile resident for the whole item), the first MFMA
//            from a zero accumulator
//   then     the previous panel's hits written to the buckets; the next panel's (or item's) copies
//            issued and its operand tables loaded; the compares: every (row block, query column) in
//            one branch-free pass (a wave mask per row block), then only the row blocks with a hit
//            again, row by row, into the LDS hit list of this panel.
// Same wave tiling, fragments, MFMAs and score arithmetic as f6t::EngineW / f6w_epilogue: the kept rows
// and keys equal tile_kernel_f6w's (tests/test_gpu_prefix.py).  Phase clocks: tools/prefix_sweep.py
// --trace on a -DOFR_F6P_TRACE build.
#ifdef OFR_F6P_TRACE
// probe builds only: shader-clock stamps of workgroup 0's phases for its first 64 panels, into the
// sample lists region of the workspace (p.cand: dead once the thresholds are set)
__device__ int f6p_trace_panel;
__device__ __forceinline__ void f6p_trace_mark(const TileArgs& p, int k) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && f6p_trace_panel < 64)
    reinterpret_cast<unsigned long long*>(p.cand)[f6p_trace_panel * 8 + k] = __builtin_amdgcn_s_memtime();
}
#define F6P_MARK(k) f6p_trace_mark(p, k)
#else
#define F6P_MARK(k)
#endif
namespace f6p {
using E = f6t::EngineW;
constexpr int NSPMAX = 2;                                   // prefix stages held in LDS
constexpr int GS = 0;                                       // gallery slots [NSPMAX][E::GSLOT]
constexpr int QS = NSPMAX * E::GSLOT;                       // query slots [NSPMAX][E::QSLOT]
// operand tables, raw copies of the global arrays (buffer_load ... lds: no registers, no waits until the
// next panel's top): per panel slot (2) the queries' scale [256] and threshold key [256]; per item slot
// (2) the tile rows' aux [384] and scale [384]
constexpr int QSC = QS + NSPMAX * E::QSLOT;                 // [2][256] f32 query scale (a power of two)
constexpr int QTH = QSC + 2 * 1024;                         // [2][256] u32 theta
constexpr int GAUX = QTH + 2 * 1024;                        // [2][384] f32 row aux (|g_m|^2)
constexpr int GSCL = GAUX + 2 * 1536;                       // [2][384] f32 row scale
constexpr int NHIT = GSCL + 2 * 1536;                       // [4] hits of the panel per wave
constexpr int HITS = NHIT + 16;                             // [4][HCAPW] (key, query << 9 | row)
constexpr int HCAPW = 959;                                  // hit slots per wave and (tile, panel)
constexpr int HCAP = 4 * HCAPW;                             // the rest of the LDS
constexpr int LDS_BYTES = HITS + HCAP * 8;
static_assert(LDS_BYTES <= 163840, "prefix pass LDS");

// c = a.b into an AGPR accumulator (first stage: no accumulator read).  AGPR row blocks only: with a
// VGPR destination ("=v", even early-clobber) the compiler gave the result the registers of a fragment
// that a previous, still executing MFMA was reading (the last row's query fragments die there); the
// hazard recognizer does not see into asm, so that MFMA read them overwritten -- one-stage passes lost
// query column block 5 (tests/test_gpu_prefix.py, round 5).  VGPR row blocks start from accumulators
// zeroed before the stage's first MFMA (as f6t::EngineW), with the accumulating form.
__device__ __forceinline__ void mfma0a(const f6t::i32x6& a, const f6t::i32x6& b, f6t::f32x4& c, int sa, int sb) {
  asm volatile("v_mfma_scale_f32_16x16x128_f8f6f4 %0, %1, %2, 0, %3, %4 op_sel_hi:[0,0,0] cbsz:2 blgp:2"
               : "=&a"(c) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

// wave W's copy pieces of the gallery tile gt (all NSP stages) / of query panel qp
template <int W, int NSP>
__device__ __forceinline__ void copy_gallery(const TileArgs& p, int64_t gt) {
  E::Feed f;
  E::feed_init<W, 1>(f, reinterpret_cast<const char*>(p.G), p.N, reinterpret_cast<const char*>(p.Q), 0, p.gnk, gt);
#pragma unroll
  for (int s = 0; s < NSP; ++s) {
    const uint32_t so = GS + s * E::GSLOT, ko = (uint32_t)s * f6t::PANEL;
    E::gcopy<W, 0>(f.rg, f, so, ko); E::gcopy<W, 1>(f.rg, f, so, ko); E::gcopy<W, 2>(f.rg, f, so, ko);
    E::gcopy<W, 3>(f.rg, f, so, ko); E::gcopy<W, 4>(f.rg, f, so, ko); E::gcopy<W, 5>(f.rg, f, so, ko);
    E::gcopy<W, 6>(f.rg, f, so, ko); E::gcopy<W, 7>(f.rg, f, so, ko); E::gcopy<W, 8>(f.rg, f, so, ko);
  }
}
template <int W, int NSP>
__device__ __forceinline__ void copy_queries(const TileArgs& p, int64_t qp) {
  const int64_t pb = (int64_t)p.nk * f6t::PANEL;
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(p.Q) + qp * pb), 0, (int)pb, 0x00020000);
#pragma unroll
  for (int s = 0; s < NSP; ++s) {
    const uint32_t so = QS + s * E::QSLOT, ko = (uint32_t)s * f6t::PANEL;
    E::qcopy<W, 0>(rq, so, ko); E::qcopy<W, 1>(rq, so, ko); E::qcopy<W, 2>(rq, so, ko);
    E::qcopy<W, 3>(rq, so, ko); E::qcopy<W, 4>(rq, so, ko); E::qcopy<W, 5>(rq, so, ko);
  }
}
template <int NSP>
__device__ __forceinline__ void copies(int wave, const TileArgs& p, bool gallery, int64_t gt, int64_t qp) {
  switch (wave) {
    case 0: if (gallery) copy_gallery<0, NSP>(p, gt); copy_queries<0, NSP>(p, qp); break;
    case 1: if (gallery) copy_gallery<1, NSP>(p, gt); copy_queries<1, NSP>(p, qp); break;
    case 2: if (gallery) copy_gallery<2, NSP>(p, gt); copy_queries<2, NSP>(p, qp); break;
    default: if (gallery) copy_gallery<3, NSP>(p, gt); copy_queries<3, NSP>(p, qp); break;
  }
}

// Lane-derived values come from tid, the thread index laundered through an empty asm at every panel:
// computed from threadIdx.x they are loop invariants, and the compiler hoisted every fragment address
// and hit payload of the four waves out of the persistent loops -- ~2,000 registers, spilled.
__device__ __forceinline__ E::Bases lane_bases(uint32_t slot, uint32_t tid, uint32_t qstride, uint32_t p1off) {
  const uint32_t lane = tid & 63, q = lane >> 4, l = lane & 15, qo = (q & 1) << 4;
  return E::Bases{slot + q * qstride + l * 16, slot + q * qstride + p1off + (l + qo) * 8,
                  slot + q * qstride + p1off + (l - qo) * 8};
}
// The MFMAs of one (tile, panel): stages [0, NSP) from the LDS slots into acc (stage 0 starts from
// zero).  As in f6t::EngineW, the next stage's fragments are read in the last rows of the current one
// (gallery rows 0 and 1 into the ring slots rows 10 and 11 free, each query fragment right after its
// last MFMA in row 11), so only the panel's first stage waits for its reads.
//
// Query scales: the prefix queries' row scales are powers of two 2^e_q (ofr_f6_quantize_rows_prefix), and
// e_q joins the query operand's E8M0 block scale (per lane: the lane's column), so acc = s_q (q~ . g~)
// exactly -- a power-of-two rescaling commutes with every rounding of the MFMA -- and the compares need
// no per-query product (the same scores, bit for bit, as the unfolded f6w pass: tests/test_gpu_prefix.py).
template <int W, int NSP>
__device__ __forceinline__ void panel_mfmas(const int (&sc)[NSPMAX], const uint32_t* qex, uint32_t tid,
                                            f6t::f32x4 (&acc)[E::NA][E::NB]) {
  constexpr int WR = W >> 1, WC = W & 1;
  int eq[E::NB];   // the lane's query exponent per column block; past B the table reads 0: e_q = 0
#pragma unroll
  for (int c = 0; c < E::NB; ++c) {
    const uint32_t sb = qex[WC * 128 + c * 16 + (tid & 15)];
    eq[c] = sb != 0u ? (int)((sb >> 23) & 0xffu) - 127 : 0;
  }
#pragma unroll
  for (int i = E::NAA; i < E::NA; ++i)   // the VGPR accumulators zeroed before any MFMA: their registers
#pragma unroll                           // are theirs alone
    for (int c = 0; c < E::NB; ++c) acc[i][c] = f6t::f32x4{0.f, 0.f, 0.f, 0.f};
  f6t::i32x6 a[E::RING], b[E::NB];
  {
    const E::Bases ab = lane_bases(GS, tid, 3072, 2048), bb = lane_bases(QS, tid, 6144, 4096);   // E::abase / bbase
    b[0] = E::fragB<WC * 128 + 0>(bb); b[1] = E::fragB<WC * 128 + 16>(bb); b[2] = E::fragB<WC * 128 + 32>(bb);
    b[3] = E::fragB<WC * 128 + 48>(bb); b[4] = E::fragB<WC * 128 + 64>(bb); b[5] = E::fragB<WC * 128 + 80>(bb);
    b[6] = E::fragB<WC * 128 + 96>(bb); b[7] = E::fragB<WC * 128 + 112>(bb);
    a[0] = E::fragA<WR * 192 + 0>(ab);
    a[1] = E::fragA<WR * 192 + 16>(ab);
  }
  auto stage = [&](auto sv) {
    constexpr int S = decltype(sv)::value;
    constexpr bool NEXT = S + 1 < NSP;
    const int scs = sc[S];
    int sbq[E::NB];   // query operand scales: the block's byte + e_q (bytes in [0, 191]: no carry out)
#pragma unroll
    for (int c = 0; c < E::NB; ++c) sbq[c] = scs + eq[c];
    const E::Bases ab = lane_bases(GS + S * E::GSLOT, tid, 3072, 2048);
    const E::Bases an = lane_bases(GS + (NEXT ? S + 1 : S) * E::GSLOT, tid, 3072, 2048);
    const E::Bases bn = lane_bases(QS + (NEXT ? S + 1 : S) * E::QSLOT, tid, 6144, 4096);
    auto row = [&](auto ii) {
      constexpr int i = decltype(ii)::value;
      constexpr bool AG = i < E::NAA;
      if constexpr (i + 2 < E::NA) a[(i + 2) % E::RING] = E::fragA<WR * 192 + (i + 2 < E::NA ? i + 2 : 0) * 16>(ab);
      else if constexpr (NEXT) a[(i + 2) % E::RING] = E::fragA<WR * 192 + (i + 2 - E::NA) * 16>(an);
      auto mm = [&](int c) {
        if constexpr (S == 0 && AG) mfma0a(a[i % E::RING], b[c], acc[i][c], scs, sbq[c]);
        else E::mfma2<AG>(a[i % E::RING], b[c], acc[i][c], scs, sbq[c]);
      };
      if constexpr (i == E::NA - 1 && NEXT) {
        mm(0); b[0] = E::fragB<WC * 128 + 0>(bn);
        mm(1); b[1] = E::fragB<WC * 128 + 16>(bn);
        mm(2); b[2] = E::fragB<WC * 128 + 32>(bn);
        mm(3); b[3] = E::fragB<WC * 128 + 48>(bn);
        mm(4); b[4] = E::fragB<WC * 128 + 64>(bn);
        mm(5); b[5] = E::fragB<WC * 128 + 80>(bn);
        mm(6); b[6] = E::fragB<WC * 128 + 96>(bn);
        mm(7); b[7] = E::fragB<WC * 128 + 112>(bn);
      } else {
#pragma unroll
        for (int c = 0; c < E::NB; ++c) mm(c);
      }
      __builtin_amdgcn_sched_barrier(0);   // rows in order: fragments read two rows ahead, not all at once
    };
    row(std::integral_constant<int, 0>{}); row(std::integral_constant<int, 1>{});
    row(std::integral_constant<int, 2>{}); row(std::integral_constant<int, 3>{});
    row(std::integral_constant<int, 4>{}); row(std::integral_constant<int, 5>{});
    row(std::integral_constant<int, 6>{}); row(std::integral_constant<int, 7>{});
    row(std::integral_constant<int, 8>{}); row(std::integral_constant<int, 9>{});
    row(std::integral_constant<int, 10>{}); row(std::integral_constant<int, 11>{});
  };
  stage(std::integral_constant<int, 0>{});
  if constexpr (NSP > 1) stage(std::integral_constant<int, 1>{});
}
template <int NSP>
__device__ __forceinline__ void mfmas(int wave, const int (&sc)[NSPMAX], const char* smem, int qb, uint32_t tid,
                                      f6t::f32x4 (&acc)[E::NA][E::NB]) {
  const uint32_t* qex = reinterpret_cast<const uint32_t*>(smem + QSC) + qb * 256;
  switch (wave) {
    case 0: panel_mfmas<0, NSP>(sc, qex, tid, acc); break;
    case 1: panel_mfmas<1, NSP>(sc, qex, tid, acc); break;
    case 2: panel_mfmas<2, NSP>(sc, qex, tid, acc); break;
    default: panel_mfmas<3, NSP>(sc, qex, tid, acc); break;
  }
  E::wait_drain();
}

// The sieve compares of one (tile, panel): f6w_epilogue's, with the operand tables in LDS and the hits
// into the wave's own LDS list.  (Rolling the hit path into one copy per column block or per row block,
// 21k -> 12k / 6.8k instructions, measured no faster: profiles/r05_rolled_hits_ab.txt.  Round 5 tried a branch-free first pass over all row blocks with a second pass for
// the blocks with a hit: it kept every accumulator live through both, spilled, and was slower.)
// The VGPR accumulators (row blocks NAA..NA-1) go first: their registers are free for the rest.
__device__ __forceinline__ void compares(char* smem, const TileArgs& p, int64_t g0, int64_t q0, int wave,
                                         uint32_t tid, int qb, int gb, f6t::f32x4 (&acc)[E::NA][E::NB]) {
  const int WR = wave >> 1;
  const uint32_t* qth = reinterpret_cast<const uint32_t*>(smem + QTH) + qb * 256;
  const float* gaux = reinterpret_cast<const float*>(smem + GAUX) + gb * E::TGW;
  const float* gscl = reinterpret_cast<const float*>(smem + GSCL) + gb * E::TGW;
  uint2* hits = reinterpret_cast<uint2*>(smem + HITS) + wave * HCAPW;   // the wave's own list: no atomics,
  uint32_t cnt = 0;                                                      // its fill count uniform (SGPR)
  const int nvalid = p.N - g0 < E::TGW ? (int)(p.N - g0) : E::TGW;
  const int lane = tid & 63, wc = wave & 1, g4 = (lane >> 4) * 4, r16 = lane & 15;
  float th[E::NB];   // theta as a float: fix_query_tables made it at the panel's top
#pragma unroll
  for (int c = 0; c < E::NB; ++c) th[c] = __uint_as_float(qth[wc * 128 + c * 16 + r16]);
  typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int ii = 0; ii < E::NA; ++ii) {
    const int i = (ii + E::NAA) % E::NA;
    const int gl0 = WR * 192 + i * 16 + g4;
    // rows past N read zeros (aux 0, scale 0: a score of 0), which the hit test below excludes
    const float4 ta = *reinterpret_cast<const float4*>(gaux + gl0);
    const float4 ts = *reinterpret_cast<const float4*>(gscl + gl0);
    // 2 s_g: the query scale is in acc already (panel_mfmas); sc = fma(-2 s_g, acc, a) in packed pairs
    const f32x2 avp[2] = {f32x2{ta.x, ta.y}, f32x2{ta.z, ta.w}};
    const f32x2 tp[2] = {f32x2{ts.x, ts.y} + f32x2{ts.x, ts.y}, f32x2{ts.z, ts.w} + f32x2{ts.z, ts.w}};
    float sc[4][E::NB];
    uint64_t col[E::NB];
    uint64_t any = 0;
#pragma unroll
    for (int c = 0; c < E::NB; ++c) {
#pragma unroll
      for (int rp = 0; rp < 2; ++rp) {
        const f32x2 x = __builtin_elementwise_fma(-tp[rp], f32x2{acc[i][c][2 * rp], acc[i][c][2 * rp + 1]}, avp[rp]);
        sc[2 * rp][c] = x.x;
        sc[2 * rp + 1][c] = x.y;
      }
      const float mn = fminf(fminf(sc[0][c], sc[1][c]), fminf(sc[2][c], sc[3][c]));
      col[c] = __builtin_amdgcn_ballot_w64(!(mn > th[c]));   // NaN th ("keep every row") passes
      any |= col[c];
    }
    if (any == 0) continue;   // uniform; ~2 kept pairs per panel and wave on gallery data
#pragma unroll
    for (int c = 0; c < E::NB; ++c) {
      if (col[c] == 0) continue;   // uniform
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool h = !(sc[r][c] > th[c]) && gl0 + r < nvalid;   // padding rows (aux +inf): only a NaN th
        const uint64_t m = __builtin_amdgcn_ballot_w64(h);
        if (m == 0) continue;   // uniform
        if (h) {
          const int ql = wc * 128 + c * 16 + r16;
          const uint32_t kb = __float_as_uint(key_score(score_key(sc[r][c], 0)));
          const uint32_t slot = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (slot < (uint32_t)HCAPW) {
            hits[slot] = make_uint2(kb, ((uint32_t)ql << 9) | (uint32_t)(gl0 + r));
          } else {   // the list is full (small galleries: ~3 % of the pairs kept): straight to the bucket
            const int bs = atomicAdd(p.count + q0 + ql, 1);
            if (bs < p.cap) p.bucket[(q0 + ql) * p.cap + bs] = Cand{__uint_as_float(kb), (int)(g0 + gl0 + r)};
          }
        }
        cnt += (uint32_t)__builtin_popcountll(m);
      }
    }
  }
  if (lane == 0) reinterpret_cast<uint32_t*>(smem + NHIT)[wave] = cnt < (uint32_t)HCAPW ? cnt : (uint32_t)HCAPW;
}

// Flush of the hit lists (tile rows from g0, queries from q0) into the per-query buckets, split so that
// the global atomics' round trip runs under the next panel's MFMAs: begin takes each thread's hit into
// registers -- the list is free for the next compares -- and reserves its slot (a longer list, rare on
// large galleries, is flushed here whole; hits past the list's capacity went to the buckets directly),
// end writes the entries.
struct Pending {
  int64_t q;
  int slot;   // the atomic's answer: read only in flush_end (no wait for it before)
  uint2 hv;
};
__device__ __forceinline__ Pending flush_begin(char* smem, const TileArgs& p, int64_t g0, int64_t q0,
                                               uint32_t tid) {
  Pending pd{-1, 0, make_uint2(0u, 0u)};
  const uint32_t* nw = reinterpret_cast<const uint32_t*>(smem + NHIT);   // the four waves' lists (the rest
  const uint32_t n0 = nw[0], n1 = nw[1], n2 = nw[2], n3 = nw[3];          // went to the buckets)
  const uint32_t nh = n0 + n1 + n2 + n3;
  const uint2* hits = reinterpret_cast<const uint2*>(smem + HITS);
  auto entry = [&](uint32_t e) {   // entry e of the concatenated lists
    uint32_t w = 0;
    if (e >= n0) { e -= n0; w = 1; if (e >= n1) { e -= n1; w = 2; if (e >= n2) { e -= n2; w = 3; } } }
    return hits[w * HCAPW + e];
  };
  if (nh > (uint32_t)E::NT) {
    for (uint32_t e = tid; e < nh; e += E::NT) {
      const uint2 hv = entry(e);
      const int64_t q = q0 + (int)(hv.y >> 9);
      if (q < p.B) {
        const int slot = atomicAdd(p.count + q, 1);
        if (slot < p.cap) p.bucket[q * p.cap + slot] = Cand{__uint_as_float(hv.x), (int)(g0 + (hv.y & 511u))};
      }
    }
  } else if (tid < nh) {
    pd.hv = entry(tid);
    pd.q = q0 + (int)(pd.hv.y >> 9);
    if (pd.q < p.B) pd.slot = atomicAdd(p.count + pd.q, 1);
    else pd.q = -1;
  }
  return pd;
}
__device__ __forceinline__ void flush_end(const TileArgs& p, int64_t g0, const Pending& pd) {
  int slot = pd.slot;
  // first use of the atomic's answer: the compiler otherwise sign-extended it right behind the atomic,
  // waiting for the round trip there
  asm volatile("" : "+v"(slot));
  if (pd.q >= 0 && slot < p.cap)
    p.bucket[pd.q * p.cap + slot] = Cand{__uint_as_float(pd.hv.x), (int)(g0 + (pd.hv.y & 511u))};
}

// raw operand tables by LDS-DMA (4 B per lane, one 256-B piece per wave-instruction): query scales and
// thetas of the 256 queries from q0 into panel slot qb; aux and scales of the 384 rows from g0 into item
// slot gb (reads past the arrays' ends return zeros)
__device__ __forceinline__ void table_piece(const void* base, int64_t n_left, uint32_t lds, int piece, uint32_t lane) {
  const int bytes = n_left <= 0 ? 0 : (n_left >= (1 << 20) ? (1 << 22) : (int)(n_left * 4));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, bytes, 0x00020000);
  // the piece offset in voffset: the range check covers voffset + offset, not soffset
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (OFR_LDS void*)(uintptr_t)(lds + piece * 256), 4, piece * 256 + lane * 4,
                                           0, 0, 0);
}
__device__ __forceinline__ void load_query_tables(const TileArgs& p, int wave, uint32_t lane, int64_t q0, int qb) {
  table_piece(p.qscale + q0, p.B - q0, QSC + qb * 1024, wave, lane);
  table_piece(p.theta + q0, p.B - q0, QTH + qb * 1024, wave, lane);
}
// the raw theta table of slot qb -> key_float(theta | 0xff), in place; past B: no row kept (the copies
// read zeros there).  The scales stay raw (panel_mfmas reads them before the next barrier).
__device__ __forceinline__ void fix_query_tables(char* smem, const TileArgs& p, int64_t q0, int qb, uint32_t tid) {
  uint32_t* qth = reinterpret_cast<uint32_t*>(smem + QTH) + qb * 256;
  const uint32_t t = qth[tid];
  qth[tid] = __float_as_uint(q0 + tid < p.B ? key_float(t | 0xffu) : -__builtin_inff());
}
__device__ __forceinline__ void load_tile_tables(const TileArgs& p, int wave, uint32_t lane, int64_t g0, int gb) {
  table_piece(p.aux + g0, p.N - g0, GAUX + gb * 1536, wave, lane);
  table_piece(p.gscale + g0, p.N - g0, GSCL + gb * 1536, wave, lane);
  if (wave < 2) {   // pieces 4 and 5 of the 384 rows
    table_piece(p.aux + g0, p.N - g0, GAUX + gb * 1536, wave + 4, lane);
    table_piece(p.gscale + g0, p.N - g0, GSCL + gb * 1536, wave + 4, lane);
  }
}
}  // namespace f6p

// p.ntg gallery tiles of 384 rows x p.ntq query panels; work item w = (gallery tile w / ngrp, query
// panels [qg * (w % ngrp), ...) of the group size qg); NSP = p.nkp <= f6p::NSPMAX stages.
template <int NSP>
__global__ void __launch_bounds__(256, 1) tile_kernel_f6p(TileArgs p, int64_t qg) {
  using E = f6t::EngineW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t ngrp = (p.ntq + qg - 1) / qg, items = p.ntg * ngrp;
  // the stages' block scales (the same for every tile)
  const uint32_t lsh = 8u * ((threadIdx.x & 63) >> 4);
  int sc[f6p::NSPMAX];
  {
    const uint32_t r0 = f6t::sload_bscale(p.bs, 0), r1 = f6t::sload_bscale(p.bs, NSP > 1 ? 1 : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sc[0] = f6t::lane_byte(r0, lsh);
    sc[1] = f6t::lane_byte(r1, lsh);
  }
  int64_t w = blockIdx.x;
  if (w >= items) return;
  // 32-bit index arithmetic (the host bounds items below 2^31)
  const uint32_t ng32 = (uint32_t)ngrp, qg32 = (uint32_t)qg;
  auto item_gt = [&](int64_t it) { return (int64_t)((uint32_t)it / ng32); };
  auto item_q0 = [&](int64_t it) { return (int64_t)(((uint32_t)it % ng32) * qg32); };
  auto item_q1 = [&](int64_t it) { const int64_t e = item_q0(it) + qg; return e < p.ntq ? e : p.ntq; };
  // prologue: the first item's gallery stages and first panel, its operand tables, empty hit lists
  f6p::load_tile_tables(p, wave, threadIdx.x & 63, item_gt(w) * E::TGW, 0);
  f6p::load_query_tables(p, wave, threadIdx.x & 63, item_q0(w) * f6t::TQ, 0);
  f6p::copies<NSP>(wave, p, true, item_gt(w), item_q0(w));
  int buf = 0, gb = 0;                // table slots of the current panel / item
  int64_t pg0 = 0, pq0 = 0;           // the previous panel's tile row / query base (its hits: the list)
  bool prev = false;
  for (;;) {
    const int64_t gt = item_gt(w), qp1 = item_q1(w);
    for (int64_t qp = item_q0(w); qp < qp1; ++qp) {
#ifdef OFR_F6P_TRACE
      if (blockIdx.x == 0 && threadIdx.x == 0) f6p_trace_panel = (int)(qp - item_q0(w)) + 16 * (int)(w / gridDim.x);
#endif
      F6P_MARK(0);
      f6t::wait_vm<0>();   // this panel's copies (and the previous panel's bucket stores)
      f6t::barrier();
      F6P_MARK(1);
      uint32_t tid = threadIdx.x;      // f6p::lane_bases
      asm volatile("" : "+v"(tid));
      f6p::fix_query_tables(smem, p, qp * f6t::TQ, buf, tid);   // read after the MFMAs' barrier
      const f6p::Pending pd = prev ? f6p::flush_begin(smem, p, pg0, pq0, tid) : f6p::Pending{-1, 0, {0u, 0u}};
      F6P_MARK(6);
      f6t::f32x4 acc[E::NA][E::NB];   // per panel: stage 0 writes every accumulator
      f6p::mfmas<NSP>(wave, sc, smem, buf, tid, acc);
      F6P_MARK(7);
      f6t::barrier();   // every wave's fragment reads of the slots done: refill them
      F6P_MARK(2);
      f6p::flush_end(p, pg0, pd);
      // what comes next: the next panel of this item, or the next item's gallery tile and first panel
      const bool more = qp + 1 < qp1;
      const int64_t wn = more ? w : w + gridDim.x;
      const bool next = more || wn < items;
      if (next) {   // the next panel's (and item's) tables and stages, landed by the next panel's top
        const int64_t qn = more ? qp + 1 : item_q0(wn);
        f6p::load_query_tables(p, wave, tid & 63, qn * f6t::TQ, buf ^ 1);
        if (!more) f6p::load_tile_tables(p, wave, tid & 63, item_gt(wn) * E::TGW, gb ^ 1);
        f6p::copies<NSP>(wave, p, !more, item_gt(wn), qn);
      }
      __syncthreads();   // flush_begin's reads of the hit lists done before the compares refill them
      F6P_MARK(3);
      f6p::compares(smem, p, gt * E::TGW, qp * f6t::TQ, wave, tid, buf, gb, acc);
      F6P_MARK(4);
      __syncthreads();   // every wave's compares done: the tables may change (next panel's top)
      F6P_MARK(5);
      pg0 = gt * E::TGW;
      pq0 = qp * f6t::TQ;
      prev = true;
      buf ^= 1;
      if (!more) gb ^= 1;
    }
    w += gridDim.x;
    if (w >= items) break;
  }
  // the last panel's hits
  f6t::wait_vm<0>();
  f6t::barrier();
  const f6p::Pending pd = f6p::flush_begin(smem, p, pg0, pq0, threadIdx.x);
  f6p::flush_end(p, pg0, pd);
}

// ---- prefix tier's sieve pass, one stage: two workgroups per CU (round 6) ---------------------------
// tile_kernel_f6p runs ONE wave per SIMD (its 192 x 128 wave tiles hold 384 accumulators), so the score
// compares after each panel's MFMAs -- 384 per lane, dependent VALU chains -- run alone: ~8,300 of a
// panel's ~17,500 cycles, the MFMAs ~1,500 (profiles/r05_f6p_phase_trace.txt).  With one
// prefix stage an MFMA block is a single instruction and its fragments are read once, so a much smaller
// wave tile costs little LDS traffic: here each wave owns 64 gallery rows x 128 queries (32 blocks of
// 16 x 16, 128 accumulator VGPRs, no AGPR reads), a workgroup 256 rows x 128 queries, and TWO workgroups
// share every CU -- two waves per SIMD, so one wave's compares issue while the other's MFMAs run, and
// the VALU issues at the two-wave rate.  The MFMAs are compiler builtins (the compiler sees their
// hazards; no accumulator is pinned by asm: tests/test_spill_guard.py holds this kernel to zero spills).
// Work item = (256-row gallery tile = one panel of the tiled layout, group of 128-query steps = half
// panels of the query tiles).  The gallery rows' fragments are read into registers once per item (the
// tile's 24 KiB image is then free for the next item's copy); per step, behind ONE barrier:
//   top      own copies landed + barrier; the next step's half panel (12 KiB) and its tables copied
//            into the other buffer; on an item's 2nd step the next item's gallery tile and tables
//   flush    the previous step's hits (this wave's LDS list) get their bucket slots: global atomics,
//            answered under this step's MFMAs
//   MFMAs    8 query fragments x 4 row blocks
//   compares per query column the 16 rows' scores fma(-2 s_g, acc, a) (the same arithmetic and query
//            scale folding as tile_kernel_f6p: bit-identical keys), their min against theta; only a
//            column with a hit is scored again row by row into the wave's LDS hit list
//   end      the flushed entries written to the buckets
namespace pp {
using E = f6t::EngineW;
constexpr int NT = 256;
constexpr int TGR = 256;                       // gallery rows per item (one panel of the tiled layout)
constexpr int TQH = 128;                       // queries per step (half a query panel)
constexpr int GT = 0;                          // the gallery tile's stage-0 image (24 KiB, panel layout)
constexpr int QB = GT + f6t::PANEL;            // [2] half-panel images (E::HPB = 12 KiB each)
constexpr int QT = QB + 2 * E::HPB;            // [2][128] (theta as a float, the query's scale exponent)
constexpr int GTB = QT + 2 * 1024;             // [2] {f32 aux [256], f32 scale [256]}
constexpr int HITS = GTB + 2 * 2048;           // [4][HCAPW] (key bits, ql << 9 | row)
constexpr int HCAPW = 256;                     // a wave's hits per step (~1 on gallery data; past it: atomics)
constexpr int SCR = HITS + 4 * HCAPW * 8;      // [4][4 KiB] per wave: a flagged column's 16 scores per lane
constexpr int LDS_BYTES = SCR + 4 * 4096;
static_assert(LDS_BYTES <= 81920, "two workgroups per CU");
typedef int i32x8 __attribute__((ext_vector_type(8)));

// wave's pieces of the stage-0 image of gallery panel gt (24 pieces of 1 KiB) into GT
__device__ __forceinline__ void copy_gtile(const TileArgs& p, int64_t gt, int wave, uint32_t lane) {
  const int64_t pb = (int64_t)p.gnk * f6t::PANEL;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(p.G) + gt * pb), 0, f6t::PANEL, 0x00020000);
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const int piece = wave * 6 + j;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (OFR_LDS void*)(uintptr_t)(GT + piece * 1024), 16, lane * 16,
                                             piece * 1024, 0, 0);
  }
}
// half h = step & 1 of query panel step >> 1 (stage 0) into QB slot buf: sub-block q = wave, its part0 rows
// [128 h, 128 h + 128) (2 pieces) and part1 slots of those rows (1 piece) -- the HPB image E::abase reads
__device__ __forceinline__ void copy_qhalf(const TileArgs& p, int64_t step, int buf, int wave, uint32_t lane) {
  const int64_t pb = (int64_t)p.nk * f6t::PANEL, pnl = step >> 1;
  const int h = (int)(step & 1);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(reinterpret_cast<const char*>(p.Q) + pnl * pb), 0, f6t::PANEL, 0x00020000);
#pragma unroll
  for (int part = 0; part < 3; ++part) {
    const int src = wave * 6144 + (part < 2 ? h * 2048 + part * 1024 : 4096 + h * 1024);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        r, (OFR_LDS void*)(uintptr_t)(QB + buf * E::HPB + wave * 3072 + part * 1024), 16, lane * 16, src, 0, 0);
  }
}
__device__ __forceinline__ void copy_qtables(const uint2* qtab, int64_t nq, int64_t step, int buf, int wave,
                                             uint32_t lane) {
  f6p::table_piece(qtab + step * TQH, 2 * (nq - step * TQH), QT + buf * 1024, wave, lane);
}
__device__ __forceinline__ void copy_gtables(const TileArgs& p, int64_t g0, int buf, int wave, uint32_t lane) {
  f6p::table_piece(p.aux + g0, p.N - g0, GTB + buf * 2048, wave, lane);
  f6p::table_piece(p.gscale + g0, p.N - g0, GTB + buf * 2048 + 1024, wave, lane);
}
__device__ __forceinline__ i32x8 frag8(uint32_t a0, uint32_t a1) {
  const f6t::i32x6 f = E::frag_at(a0, a1);
  i32x8 v;
  v[0] = f[0]; v[1] = f[1]; v[2] = f[2]; v[3] = f[3]; v[4] = f[4]; v[5] = f[5]; v[6] = 0; v[7] = 0;
  return v;
}

// LDS reads through integer addresses, volatile (as E::frag_at): hipcc makes a read through smem wait for
// every LDS-DMA copy in flight (s_waitcnt vmcnt(0): the next step's copies, issued at the step's top), not
// these; none of them reads a region a copy in flight writes
__device__ __forceinline__ uint2 lds_u2(uint32_t a) {
  const f6t::i32x2 v = *reinterpret_cast<volatile const OFR_LDS f6t::i32x2*>((uintptr_t)a);
  return make_uint2((uint32_t)v[0], (uint32_t)v[1]);
}
__device__ __forceinline__ uint32_t lds_u32(uint32_t a) {
  return *reinterpret_cast<volatile const OFR_LDS uint32_t*>((uintptr_t)a);
}
__device__ __forceinline__ float4 lds_f4(uint32_t a) {
  const f6t::i32x4 v = *reinterpret_cast<volatile const OFR_LDS f6t::i32x4*>((uintptr_t)a);
  return make_float4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
}

struct Pend {
  int64_t q;   // < 0: none
  int slot;
  uint2 hv;
};
// the wave's list of the previous step (n entries, uniform) -> bucket slots; more than one entry per lane
// (rare on large galleries) is flushed here whole
__device__ __forceinline__ Pend flush_begin(const TileArgs& p, uint32_t hits, uint32_t n, int64_t g0, int64_t q0,
                                            uint32_t lane) {
  // slot is left unset where no atomic writes it (read only where q >= 0): a constant there made the
  // compiler wait for every memory operation in flight (vmcnt(0)) before overwriting the atomic's
  // destination register on the no-flush path
  Pend pd;
  pd.q = -1;
  pd.hv = make_uint2(0u, 0u);
  if (n > 64u) {
    for (uint32_t e = lane; e < n; e += 64u) {
      const uint2 hv = lds_u2(hits + e * 8u);
      const int64_t q = q0 + (int)(hv.y >> 9);
      if (q < p.B) {
        const int slot = atomicAdd(p.count + q, 1);
        if (slot < p.cap) p.bucket[q * p.cap + slot] = Cand{__uint_as_float(hv.x), (int)(g0 + (hv.y & 511u))};
      }
    }
  } else if (lane < n) {
    pd.hv = lds_u2(hits + lane * 8u);
    pd.q = q0 + (int)(pd.hv.y >> 9);
    if (pd.q < p.B) pd.slot = atomicAdd(p.count + pd.q, 1);
    else pd.q = -1;
  }
  return pd;
}
__device__ __forceinline__ void flush_end(const TileArgs& p, int64_t g0, const Pend& pd) {
  int slot = pd.slot;
  asm volatile("" : "+v"(slot));   // first use of the atomic's answer here, not right behind the atomic
  if (pd.q >= 0 && slot < p.cap)
    p.bucket[pd.q * p.cap + slot] = Cand{__uint_as_float(pd.hv.x), (int)(g0 + (pd.hv.y & 511u))};
}
}  // namespace pp

// theta keys -> the pass's per-query table (thetas as floats, -inf past B; the power-of-two query scales'
// exponents), nq = round_up(B, 128) entries
__global__ void prefix_tables_kernel(const uint32_t* theta, const float* qscale, int64_t B, int64_t nq, uint2* out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq) return;
  float th = -__builtin_inff();
  int eq = 0;
  if (q < B) {
    th = key_float(theta[q] | 0xffu);   // KEY_NONE -> NaN: every row kept
    const uint32_t sb = __float_as_uint(qscale[q]);
    eq = sb != 0u ? (int)((sb >> 23) & 0xffu) - 127 : 0;
  }
  out[q] = make_uint2(__float_as_uint(th), (uint32_t)eq);
}

// OFR_PP_PROBE (probe builds only, tools/probe_prefix_pass.py): bit 1 no bucket flush, bit 2 no compares
// (the accumulators kept alive), bit 4 no MFMAs (zero accumulators), bit 8 no hit path (the compares' hit
// masks computed and dropped)
#ifndef OFR_PP_PROBE
#define OFR_PP_PROBE 0
#endif
// p.ntg = ceil(N / 256) gallery tiles; steps of 128 queries, ceil(B / 128); item w = (tile w / ngrp, steps
// [qg (w % ngrp), ...)).  qtab: prefix_tables_kernel's table.
//
// FOLD (round 6, the default engine 3): the gallery rows' power-of-two scales (the prefix tier's own tiles,
// ofr_f6p_quantize_rows) join the gallery operand's E8M0 scale with the factor 2 (per lane: its A row), and
// -|g_m|^2 is the MFMA's accumulator input (per lane: its 4 output rows, one register set per row block for
// every query column), so the MFMA writes D = 2 s_g s_q (q~.g~) - |g_m|^2 = -(the coarse score) itself:
// the compares are one max per score (v_max3) and one compare per query column, against -theta, instead of
// an fma and a min per score (tools/probe_prefix_pass.py: the compares and their hit path were 0.55 of the
// pass's 0.84 ms).  The hit path tests the 16 rows of a flagged column block row by row with one ballot
// each (no per-lane select chains).  The scores differ from FOLD = false's fma(-2 s_g, acc, aux) by the
// accumulation order of one fp32 rounding: the merge's bound for the prefix tier carries 2^-14 aux for it.
template <bool FOLD>
__global__ void __launch_bounds__(256, 2) prefix_pass_kernel(TileArgs p, const uint2* qtab, int64_t qg) {
  using E = f6t::EngineW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63;
  const int64_t nsteps = (p.B + pp::TQH - 1) / pp::TQH, nq = nsteps * pp::TQH;
  const int64_t ngrp = (nsteps + qg - 1) / qg, items = p.ntg * ngrp;
  int64_t w = blockIdx.x;
  if (w >= items) return;
  int scs;   // the lane's stage-0 block scale byte (its 32-feature block lane >> 4)
  {
    const uint32_t r0 = f6t::sload_bscale(p.bs, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    scs = f6t::lane_byte(r0, 8u * (lane >> 4));
  }
  const uint32_t ng32 = (uint32_t)ngrp, qg32 = (uint32_t)qg;
  auto item_gt = [&](int64_t it) { return (int64_t)((uint32_t)it / ng32); };
  auto item_s0 = [&](int64_t it) { return (int64_t)(((uint32_t)it % ng32) * qg32); };
  auto item_s1 = [&](int64_t it) { const int64_t e = item_s0(it) + qg; return e < nsteps ? e : nsteps; };
  // fragment bases: gallery tile (panel image, rows wave * 64 + 16 i) and the two half-panel slots
  const E::Bases gbas = E::bbase(pp::GT), qbas0 = E::abase(pp::QB);
  const uint32_t hits_a = pp::HITS + (uint32_t)wave * pp::HCAPW * 8u;   // the wave's hit list (LDS address)
  const int g4 = (int)(lane >> 4) * 4, r16 = (int)(lane & 15);
  // prologue
  pp::copy_gtile(p, item_gt(w), wave, lane);
  pp::copy_gtables(p, item_gt(w) * pp::TGR, 0, wave, lane);
  pp::copy_qhalf(p, item_s0(w), 0, wave, lane);
  pp::copy_qtables(qtab, nq, item_s0(w), 0, wave, lane);
  int qb = 0, gb = 0;
  bool gpend = false;                  // the next item's gallery tile: copied once every wave has read this one's
  uint32_t cnt = 0;                    // this wave's hits of the previous step (uniform)
  int64_t pg0 = 0, pq0 = 0;            // the previous step's tile row / query base (the list's entries)
  pp::Pend pdb{-1, 0, make_uint2(0u, 0u)};   // entries whose atomics the previous step issued
  int64_t pg1 = 0;                     // their tile row base
  bool flushed = false;                // memory operations issued after the copies (vmcnt(1) at the top)
  pp::i32x8 A[4];
  const f6t::f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  // FOLD, per item: the accumulator inputs (-|g_m|^2 of the lane's output rows of each row block; -inf past
  // N), the gallery operand scales (block byte + e_g + 1 of the lane's A row) and the lane's valid rows
  f6t::f32x4 Cin[4];
  int sa[4];
  uint32_t vmask = 0;
  for (;;) {
    const int64_t gt = item_gt(w), s0 = item_s0(w), s1 = item_s1(w), wn = w + gridDim.x;
    const bool more_items = wn < items;
    const int64_t g0 = gt * pp::TGR;
    const int nvalid = p.N - g0 < pp::TGR ? (int)(p.N - g0) : pp::TGR;
    for (int64_t s = s0; s < s1; ++s) {
      // this step's copies landed: they were issued before the previous step's bucket atomics, so with
      // an atomic (or any later memory operation) issued since, vmcnt(1) proves them in order
      if (flushed) f6t::wait_vm<1>();
      else f6t::wait_vm<0>();
      f6t::barrier();
      // the entries whose slots the previous step's atomics reserved: written now, a step later, and
      // before this step's copies are issued (so no store follows the copies)
      if constexpr (!(OFR_PP_PROBE & 1)) pp::flush_end(p, pg1, pdb);
      if (s == s0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t r0 = (uint32_t)(wave * 64 + 16 * i);
          A[i] = pp::frag8(gbas.p0 + r0 * 16, ((i & 1) ? gbas.p1o : gbas.p1e) + r0 * 8);
        }
        if constexpr (FOLD) {
          const uint32_t gtb = pp::GTB + (uint32_t)gb * 2048u;
          vmask = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float4 a4 = pp::lds_f4(gtb + (uint32_t)(wave * 64 + 16 * i + g4) * 4u);
            const int rb = wave * 64 + 16 * i + g4;
            Cin[i][0] = rb + 0 < nvalid ? -a4.x : -__builtin_inff();
            Cin[i][1] = rb + 1 < nvalid ? -a4.y : -__builtin_inff();
            Cin[i][2] = rb + 2 < nvalid ? -a4.z : -__builtin_inff();
            Cin[i][3] = rb + 3 < nvalid ? -a4.w : -__builtin_inff();
#pragma unroll
            for (int r = 0; r < 4; ++r) vmask |= rb + r < nvalid ? 1u << (4 * i + r) : 0u;
            // the lane's A row wave * 64 + 16 i + r16: its scale 2^e (0 past N: e = 0)
            const uint32_t sb = pp::lds_u32(gtb + 1024u + (uint32_t)(wave * 64 + 16 * i + r16) * 4u);
            const int eg = sb != 0u ? (int)((sb >> 23) & 0xffu) - 127 : 0;
            sa[i] = scs + eg + 1;   // block byte (64..127) + e_g (-64..64) + 1: in [1, 192]
          }
        }
        if (more_items) gpend = true;
      } else if (gpend) {   // every wave read its fragments of this item's tile before this step's barrier
        pp::copy_gtile(p, item_gt(wn), wave, lane);
        pp::copy_gtables(p, item_gt(wn) * pp::TGR, gb ^ 1, wave, lane);
        gpend = false;
      }
      const int64_t sn = s + 1 < s1 ? s + 1 : (more_items ? item_s0(wn) : -1);
      if (sn >= 0) {
        pp::copy_qhalf(p, sn, qb ^ 1, wave, lane);
        pp::copy_qtables(qtab, nq, sn, qb ^ 1, wave, lane);
      }
      const pp::Pend pd = (OFR_PP_PROBE & 1) ? pp::Pend{-1, 0, make_uint2(0u, 0u)}
                                             : pp::flush_begin(p, hits_a, cnt, pg0, pq0, lane);
      flushed = (OFR_PP_PROBE & 1) ? false : cnt > 0u;
      // MFMAs: acc[i][c] = rows wave * 64 + 16 i, queries 16 c of the step
      const uint32_t qta = pp::QT + (uint32_t)qb * 1024u + (uint32_t)r16 * 8u;   // the lane's column c at + 128 c
      f6t::f32x4 acc[4][8];
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t qo = (uint32_t)qb * E::HPB;   // the step's half-panel slot
        const pp::i32x8 b = pp::frag8(qbas0.p0 + qo + c * 256, ((c & 1) ? qbas0.p1o : qbas0.p1e) + qo + c * 128);
        const int sbq = scs + (int)pp::lds_u32(qta + c * 128u + 4u);   // block byte + e_q (in [0, 191]: no carry)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if constexpr (OFR_PP_PROBE & 4) {
            acc[i][c] = zero;
            asm volatile("" :: "v"(b), "v"(A[i]), "v"(sbq));
          } else if constexpr (FOLD) {
            acc[i][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[i], b, Cin[i], 2, 2, 0, sa[i], 0, sbq);
          } else {
            acc[i][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[i], b, zero, 2, 2, 0, scs, 0, sbq);
          }
        }
      }
      uint32_t ncnt = 0;
      if constexpr (FOLD) {
        // compares: per query column the max of its 16 rows' D = -score against -theta (NaN theta: "keep
        // every row", passes); v_max3 trees
        uint32_t hitc = 0;
        if constexpr (OFR_PP_PROBE & 2) {
#pragma unroll
          for (int c = 0; c < 8; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(acc[i][c]));
        } else
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float th = __uint_as_float(pp::lds_u32(qta + c * 128u));
          // IEEE maximum (NaN-propagating; no NaN here): v_maximum3_f32 straight on the MFMA results -- fmaxf
          // (maxnum) would first quiet each of them (a v_max_f32 x, x per score)
          auto mx3 = [](float a, float b, float d) {
            return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), d);
          };
          const f6t::f32x4 &a0 = acc[0][c], &a1 = acc[1][c], &a2 = acc[2][c], &a3 = acc[3][c];
          const float t0 = mx3(a0[0], a0[1], a0[2]), t1 = mx3(a0[3], a1[0], a1[1]), t2 = mx3(a1[2], a1[3], a2[0]);
          const float t3 = mx3(a2[1], a2[2], a2[3]), t4 = mx3(a3[0], a3[1], a3[2]);
          const float mx = __builtin_elementwise_maximum(mx3(t0, t1, t2), mx3(t3, t4, a3[3]));
          hitc |= !(mx < -th) ? (1u << c) : 0u;
        }
        if constexpr (OFR_PP_PROBE & 8) {
          asm volatile("" ::"v"(hitc));
          hitc = 0;
        }
        if (__builtin_amdgcn_ballot_w64(hitc != 0u)) {   // uniform; ~1 kept pair per step and wave on gallery data
          // Hit path: per flagged column block, the lane's 16-row pass mask by VALU compares alone (no ballot or
          // branch per row: testing the rows one ballot at a time cost half the pass, tools/probe_prefix_pass.py
          // probe bit 8), then a wave-uniform loop over the lanes' set bits, one kept row per lane and round (on
          // gallery data one round); the kept score is read back from the wave's LDS scratch by its row index.
          // lane-derived payloads from a laundered lane index: computed from threadIdx.x they are loop
          // invariants, and the compiler hoisted the (column, row) payloads out of the loops and spilled them
          uint32_t lid = lane;
          asm volatile("" : "+v"(lid));
          const uint32_t scr = pp::SCR + (uint32_t)wave * 4096u + (lid & 63u) * 16u;
          const int rg4 = (int)(lid >> 4) * 4;
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            if (!__builtin_amdgcn_ballot_w64((hitc >> c) & 1u)) continue;   // uniform
            const float nth = -__uint_as_float(pp::lds_u32(qta + c * 128u));
            const int ql = c * 16 + (int)(lid & 15u);
            uint32_t hm = 0;   // rows j = 4 i + r of this lane that pass
#pragma unroll
            for (int j = 0; j < 16; ++j) hm |= !(acc[j >> 2][c][j & 3] < nth) ? (1u << j) : 0u;
            hm &= (int64_t)s * pp::TQH + ql < p.B ? vmask : 0u;
            if (hm) {   // the lane's scores of this column into its scratch (read back by row index below)
#pragma unroll
              for (int i = 0; i < 4; ++i)
                *reinterpret_cast<volatile OFR_LDS f6t::f32x4*>((uintptr_t)(scr + 1024u * i)) = acc[i][c];
            }
            for (;;) {   // wave-uniform: one kept row per lane and round
              const bool act = hm != 0u;
              const uint64_t mk = __builtin_amdgcn_ballot_w64(act);
              if (mk == 0) break;
              if (act) {
                const int j = __builtin_ctz(hm);
                hm &= hm - 1u;
                const float v = __uint_as_float(pp::lds_u32(scr + 1024u * (uint32_t)(j >> 2) + 4u * (uint32_t)(j & 3)));
                const uint32_t kb = __float_as_uint(key_score(score_key(-v, 0)));
                const int row = wave * 64 + 16 * (j >> 2) + rg4 + (j & 3);
                const uint32_t slot = ncnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                if (slot < (uint32_t)pp::HCAPW) {   // volatile integer address: no wait for the copies in flight
                  f6t::i32x2 e;
                  e[0] = (int)kb;
                  e[1] = (int)(((uint32_t)ql << 9) | (uint32_t)row);
                  *reinterpret_cast<volatile OFR_LDS f6t::i32x2*>((uintptr_t)(hits_a + slot * 8u)) = e;
                } else {   // the list is full (small galleries keep a large share): straight to the bucket
                  const int64_t q = (int64_t)s * pp::TQH + ql;
                  const int bs = atomicAdd(p.count + q, 1);
                  if (bs < p.cap) p.bucket[q * p.cap + bs] = Cand{__uint_as_float(kb), (int)(g0 + row)};
                }
              }
              ncnt += (uint32_t)__builtin_popcountll(mk);
            }
          }
        }
      } else {
        // compares: per query column the min of its 16 rows' scores against theta
        const uint32_t gta = pp::GTB + (uint32_t)gb * 2048u + (uint32_t)(wave * 64 + g4) * 4u;   // aux; scale at + 1024
        float av[4][4], tp[4][4];
  #pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 a4 = pp::lds_f4(gta + 64u * i);
          const float4 s4 = pp::lds_f4(gta + 1024u + 64u * i);
          av[i][0] = a4.x; av[i][1] = a4.y; av[i][2] = a4.z; av[i][3] = a4.w;
          tp[i][0] = s4.x + s4.x; tp[i][1] = s4.y + s4.y; tp[i][2] = s4.z + s4.z; tp[i][3] = s4.w + s4.w;
        }
        uint32_t hitc = 0;
        if constexpr (OFR_PP_PROBE & 2) {
  #pragma unroll
          for (int c = 0; c < 8; ++c)
  #pragma unroll
            for (int i = 0; i < 4; ++i) asm volatile("" :: "v"(acc[i][c]));
        } else
  #pragma unroll
        for (int c = 0; c < 8; ++c) {
          const float th = __uint_as_float(pp::lds_u32(qta + c * 128u));
          float m[4];
  #pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float x0 = __builtin_fmaf(-tp[i][0], acc[i][c][0], av[i][0]);
            const float x1 = __builtin_fmaf(-tp[i][1], acc[i][c][1], av[i][1]);
            const float x2 = __builtin_fmaf(-tp[i][2], acc[i][c][2], av[i][2]);
            const float x3 = __builtin_fmaf(-tp[i][3], acc[i][c][3], av[i][3]);
            m[i] = fminf(fminf(x0, x1), fminf(x2, x3));
          }
          const float mn = fminf(fminf(m[0], m[1]), fminf(m[2], m[3]));
          hitc |= !(mn > th) ? (1u << c) : 0u;   // NaN theta ("keep every row") passes
        }
          if constexpr (OFR_PP_PROBE & 8) {
          asm volatile("" ::"v"(hitc));
          hitc = 0;
        }
        if (__builtin_amdgcn_ballot_w64(hitc != 0u)) {   // uniform; ~2 kept pairs per step and wave on gallery data
          // the scores again, from laundered row terms: the compiler would otherwise keep all 128 scores of the
          // pass above alive for this rare path (common subexpressions)
  #pragma unroll
          for (int i = 0; i < 4; ++i)
  #pragma unroll
            for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(tp[i][r]), "+v"(av[i][r]));
  #pragma unroll
          for (int c = 0; c < 8; ++c) {
            if (!__builtin_amdgcn_ballot_w64((hitc >> c) & 1u)) continue;   // uniform
            const float th = __uint_as_float(pp::lds_u32(qta + c * 128u));
            const int ql = c * 16 + r16;
            const bool qok = (int64_t)s * pp::TQH + ql < p.B;
            float sc[16];
            uint32_t hm = 0;   // the lane's rows j = 4 i + r that pass
  #pragma unroll
            for (int i = 0; i < 4; ++i)
  #pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int j = 4 * i + r;
                sc[j] = __builtin_fmaf(-tp[i][r], acc[i][c][r], av[i][r]);
                const int row = wave * 64 + 16 * i + g4 + r;
                hm |= (!(sc[j] > th) && row < nvalid && qok) ? (1u << j) : 0u;
              }
            // one kept row per lane and round, in row order: a wave-uniform loop of (on gallery data) one round
            for (;;) {
              const bool act = hm != 0u;
              const uint64_t mk = __builtin_amdgcn_ballot_w64(act);
              if (mk == 0) break;   // uniform
              const int j = act ? __builtin_ctz(hm) : 0;
              hm &= hm - 1u;
              float v = sc[0];
  #pragma unroll
              for (int jj = 1; jj < 16; ++jj) v = j == jj ? sc[jj] : v;
              const int row = wave * 64 + 16 * (j >> 2) + g4 + (j & 3);
              if (act) {
                const uint32_t kb = __float_as_uint(key_score(score_key(v, 0)));
                const uint32_t slot =
                    ncnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
                if (slot < (uint32_t)pp::HCAPW) {   // volatile integer address: no wait for the copies in flight
                  f6t::i32x2 e;
                  e[0] = (int)kb;
                  e[1] = (int)(((uint32_t)ql << 9) | (uint32_t)row);
                  *reinterpret_cast<volatile OFR_LDS f6t::i32x2*>((uintptr_t)(hits_a + slot * 8u)) = e;
                } else {   // the list is full (small galleries keep a large share): straight to the bucket
                  const int64_t q = (int64_t)s * pp::TQH + ql;
                  const int bs = atomicAdd(p.count + q, 1);
                  if (bs < p.cap) p.bucket[q * p.cap + bs] = Cand{__uint_as_float(kb), (int)(g0 + row)};
                }
              }
              ncnt += (uint32_t)__builtin_popcountll(mk);
            }
          }
        }
      }
      flushed = flushed || ncnt > (uint32_t)pp::HCAPW;   // direct bucket writes of an overflowing list
      pdb = pd;
      pg1 = pg0;
      cnt = ncnt < (uint32_t)pp::HCAPW ? ncnt : (uint32_t)pp::HCAPW;
      pg0 = g0;
      pq0 = s * pp::TQH;
      qb ^= 1;
    }
    if (gpend) {   // a one-step item: its fragment reads are behind every wave only after a barrier
      __syncthreads();
      pp::copy_gtile(p, item_gt(wn), wave, lane);
      pp::copy_gtables(p, item_gt(wn) * pp::TGR, gb ^ 1, wave, lane);
      gpend = false;
      flushed = false;   // these copies follow the atomics: the next top waits for everything
    }
    if (!more_items) break;
    w = wn;
    gb ^= 1;
  }
  // the last two steps' hits
  f6t::wait_vm<0>();
  pp::flush_end(p, pg1, pdb);
  const pp::Pend pd = pp::flush_begin(p, hits_a, cnt, pg0, pq0, lane);
  pp::flush_end(p, pg0, pd);
}

// ---- prefix tier's sieve pass, wave-decoupled (round 6, engine 4) ------------------------------------
// prefix_pass_kernel<true> shares each 128-query half panel between its 4 waves through LDS, so every step
// ends in a workgroup barrier, and a wave that finds hits (~1 kept pair per wave-step on gallery data) makes
// the other three wait: rocprofv3 counted the waves parked 0.52 of their cycles, 0.29 without the hit path
// (profiles/r06_prefix_pass_pmc.txt).  Here every wave runs alone: it owns 64 gallery rows of the work
// item's 256-row tile (its A fragments, row scales and prefix terms in registers for the item) and walks
// the item's 64-query steps loading each step's 4 query fragments and its thresholds straight from L2
// into VGPRs (the 4 waves of a workgroup read the same steps about together: L1 hits), no LDS staging
// and no barrier; the next step's fragments are loaded right behind this step's MFMAs, under its compares.
// Per step: 16 MFMAs 16x16x128 (row scales 2 s_g in the gallery operand's E8M0 scale, -|g_m|^2 as the
// accumulator input: D = -score), per query column one v_maximum3 tree and one compare, the hit path of
// prefix_pass_kernel<true> into a wave-private LDS list, flushed to the buckets once per work item.
namespace pw {
constexpr int NT = 256;
constexpr int HCAPW = 256;            // a wave's kept pairs per work item (~32 on gallery data; past it: atomics)
constexpr int HITS = 0;               // [4][HCAPW] (key bits, query << 6 | row of the wave's 64)
constexpr int SCR = HITS + 4 * HCAPW * 8;   // [4][RB KiB] a flagged column's 4 RB scores per lane
constexpr int lds_bytes(int rb) { return SCR + 4 * 1024 * rb; }
typedef int i32x8 __attribute__((ext_vector_type(8)));

// the fragment of rows [row, row + 16) (lane l: row + l % 16, 32-feature block l / 16) of the 256-row panel at
// byte pbase of an f6 tiled buffer, stage 0: part0 16 B and part1 8 B (p1_slot) of sub-block l / 16
__device__ __forceinline__ i32x8 gfrag(__amdgpu_buffer_rsrc_t r, uint32_t pbase, uint32_t row, uint32_t lane) {
  const uint32_t q = lane >> 4, rr = row + (lane & 15u);
  const uint32_t o0 = pbase + q * 6144u + rr * 16u;
  const uint32_t o1 = pbase + q * 6144u + 4096u + (rr ^ ((q & 1u) << 4)) * 8u;
  const f6t::i32x4 a = __builtin_bit_cast(f6t::i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)o0, 0, 0));
  const f6t::i32x2 b = __builtin_bit_cast(f6t::i32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)o1, 0, 0));
  i32x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = 0; v[7] = 0;
  return v;
}
}  // namespace pw

// RB row blocks of 16 gallery rows per wave, QB query blocks of 16 per step (RB x QB = 16 MFMAs per step):
// <8, 2> = 128 rows x 32 queries (the default: half the query-fragment loads per MFMA of <4, 4>), <4, 4> =
// 64 rows x 64 queries (OFR_F6P_WAVE=4).  An item is 4 RB 16 gallery rows (256 or 512: one or two panels of the compact
// tiles) and a group of qg steps, ceil(N / (64 RB)) x ceil(nsteps / qg) items dealt to the workgroups by
// stride; each wave walks the same items on its own.  qtab: prefix_tables_kernel's table over
// round_up(B, 16 QB) queries (theta as a float, -inf past B; e_q).
// PF: query steps in flight (1, the default: the next step's loads under this step's compares; 2: probe)
template <int RB, int QB, int PF>
__global__ void __launch_bounds__(256, 2) prefix_wave_kernel(TileArgs p, const uint2* qtab, int64_t qg) {
  static_assert((RB == 4 && QB == 4) || (RB == 8 && QB == 2), "wave tile shapes");
  constexpr int WR = 16 * RB, TGI = 4 * WR, TQ = 16 * QB;   // rows per wave, rows per item, queries per step
  constexpr int RSH = RB == 4 ? 6 : 7;                        // hit payload: (query << RSH) | row of the wave's
  constexpr uint32_t WSCR = 1024u * RB;                       // the wave's LDS scratch (a column's scores)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63;
  const int64_t nsteps = (p.B + TQ - 1) / TQ, ntg = (p.N + TGI - 1) / TGI;
  // items in tile octets (ntg rounded up to 8): see the item map below
  const int64_t ngrp = (nsteps + qg - 1) / qg, items = ((ntg + 7) & ~(int64_t)7) * ngrp;
  if ((int64_t)blockIdx.x >= items) return;
  int scs;   // the lane's stage-0 block scale byte (its 32-feature block lane >> 4)
  {
    const uint32_t r0 = f6t::sload_bscale(p.bs, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    scs = f6t::lane_byte(r0, 8u * (lane >> 4));
  }
  // buffer descriptors: the compact gallery tiles, the query tiles (stage stride nk), the row terms, the table
  const int64_t gpb = (int64_t)p.gnk * f6t::PANEL, qpb = (int64_t)p.nk * f6t::PANEL;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.G, 0, (int)(f6t::panels(p.N) * gpb), 0x00020000);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(
      (void*)p.Q, 0, (int)(f6t::panels(p.B) * qpb), 0x00020000);
  const __amdgpu_buffer_rsrc_t raux = __builtin_amdgcn_make_buffer_rsrc((void*)p.aux, 0, (int)(p.N * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc((void*)p.gscale, 0, (int)(p.N * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rtab = __builtin_amdgcn_make_buffer_rsrc((void*)qtab, 0, (int)(nsteps * TQ * 8),
                                                                         0x00020000);
  const uint32_t hits_a = pw::HITS + (uint32_t)wave * pw::HCAPW * 8u;   // the wave's kept pairs (LDS address)
  const int g4 = (int)(lane >> 4) * 4, r16 = (int)(lane & 15);
  const uint32_t ng32 = (uint32_t)ngrp, qg32 = (uint32_t)qg;
  for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
    // item w: gallery tile (w / (8 ngrp)) 8 + w % 8, query group (w / 8) % ngrp -- the ngrp items of one tile
    // are w, w + 8, ...: on workgroups of one XCD (workgroup b runs on XCD b % 8, the grid is a multiple of 8)
    // at about one time, so the tile's fragments come from that XCD's L2 after the first (round 6)
    const uint32_t wu = (uint32_t)w;
    const int64_t gt = (int64_t)((wu / (8u * ng32)) * 8u + (wu & 7u)), s0 = (int64_t)(((wu >> 3) % ng32) * qg32);
    if (gt >= ntg) continue;   // uniform: the last octet's missing tiles
    const int64_t s1 = s0 + qg < nsteps ? s0 + qg : nsteps;
    const int64_t g0 = gt * TGI + wave * WR;   // the wave's first row
    const int nvalid = p.N - g0 < WR ? (int)(p.N - g0) : WR;
    if (nvalid <= 0) continue;   // uniform: the last item's empty quarters
    // the item's gallery operands: A fragments of row blocks i, accumulator inputs -|g_m|^2 (-inf past N) of the
    // lane's output rows, operand scales block byte + e_g + 1 of the lane's A rows, the valid-row mask
    pw::i32x8 A[RB];
    f6t::f32x4 Cin[RB];
    int sa[RB];
    uint32_t vmask = 0;
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const uint32_t wr = (uint32_t)(wave * WR + 16 * i);   // row of the item: panel wr >> 8, row wr & 255
      A[i] = pw::gfrag(rg, (uint32_t)((gt * (TGI / 256) + (wr >> 8)) * gpb), wr & 255u, lane);
      const int rb = 16 * i + g4;
      const f6t::i32x4 a4 = __builtin_bit_cast(
          f6t::i32x4, __builtin_amdgcn_raw_buffer_load_b128(raux, (int)((g0 + rb) * 4), 0, 0));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Cin[i][r] = rb + r < nvalid ? -__int_as_float(a4[r]) : -__builtin_inff();
        vmask |= rb + r < nvalid ? 1u << (4 * i + r) : 0u;
      }
      const uint32_t sb = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsc, (int)((g0 + 16 * i + r16) * 4), 0, 0);
      const int eg = sb != 0u ? (int)((sb >> 23) & 0xffu) - 127 : 0;
      sa[i] = scs + eg + 1;   // block byte (64..127) + e_g (-64..64) + 1: in [1, 192]
    }
    // a step's query fragments and table entries (lane: query TQ s + 16 c + l % 16)
    auto qload = [&](int64_t st, pw::i32x8 (&b)[QB], uint2 (&t)[QB]) {
#pragma unroll
      for (int c = 0; c < QB; ++c) {
        const int64_t qr = st * TQ + 16 * c;   // panel qr >> 8, row qr & 255
        b[c] = pw::gfrag(rq, (uint32_t)((qr >> 8) * qpb), (uint32_t)(qr & 255), lane);
        const f6t::i32x2 e = __builtin_bit_cast(
            f6t::i32x2, __builtin_amdgcn_raw_buffer_load_b64(rtab, (int)((qr + r16) * 8), 0, 0));
        t[c] = make_uint2((uint32_t)e[0], (uint32_t)e[1]);
      }
    };
    uint32_t ncnt = 0;   // kept pairs of this item in the wave's list (uniform)
    // one step: its MFMAs on the fragments in B / tb, then the load of step st + PF into them (PF buffers in
    // flight: the L2 latency of a step's loads spans PF - 1 other steps' work), then the compares and hits
    auto step = [&](int64_t st, pw::i32x8 (&B)[QB], uint2 (&tb)[QB]) {
      float th[QB];
      f6t::f32x4 acc[RB][QB];
#pragma unroll
      for (int c = 0; c < QB; ++c) {
        th[c] = __uint_as_float(tb[c].x);
        const int sbq = scs + (int)tb[c].y;   // block byte + e_q (in [0, 191]: no carry)
#pragma unroll
        for (int i = 0; i < RB; ++i)
          acc[i][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[i], B[c], Cin[i], 2, 2, 0, sa[i], 0, sbq);
      }
      if (st + PF < s1) qload(st + PF, B, tb);   // the operands PF steps on, under this step's compares
      if constexpr (OFR_PP_PROBE & 2) {   // probe: no compares (the MFMA results consumed by an empty asm)
#pragma unroll
        for (int c = 0; c < QB; ++c)
#pragma unroll
          for (int i = 0; i < RB; ++i) asm volatile("" ::"v"(acc[i][c]));
        return;
      }
      uint32_t hitc = 0;
      auto mx3 = [](float a, float b, float d) {
        return __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), d);
      };
#pragma unroll
      for (int c = 0; c < QB; ++c) {
        float mx;
        if constexpr (RB == 4) {
          const f6t::f32x4 &a0 = acc[0][c], &a1 = acc[1][c], &a2 = acc[2][c], &a3 = acc[3][c];
          const float t0 = mx3(a0[0], a0[1], a0[2]), t1 = mx3(a0[3], a1[0], a1[1]), t2 = mx3(a1[2], a1[3], a2[0]);
          const float t3 = mx3(a2[1], a2[2], a2[3]), t4 = mx3(a3[0], a3[1], a3[2]);
          mx = __builtin_elementwise_maximum(mx3(t0, t1, t2), mx3(t3, t4, a3[3]));
        } else {
          float t[RB];
#pragma unroll
          for (int i = 0; i < RB; ++i)
            t[i] = mx3(acc[i][c][0], acc[i][c][1], __builtin_elementwise_maximum(acc[i][c][2], acc[i][c][3]));
          mx = mx3(mx3(t[0], t[1], t[2]), mx3(t[3], t[4], t[5]), __builtin_elementwise_maximum(t[6], t[7]));
        }
        hitc |= !(mx < -th[c]) ? (1u << c) : 0u;   // NaN theta ("keep every row") passes
      }
      if constexpr (OFR_PP_PROBE & 8) {   // probe: compares kept (their mask consumed by an empty asm), hits dropped
        asm volatile("" ::"v"(hitc));
        return;
      }
      if (__builtin_amdgcn_ballot_w64(hitc != 0u)) {   // uniform
        uint32_t lid = lane;   // laundered: the payloads are not hoisted out of the loops (spills)
        asm volatile("" : "+v"(lid));
        const uint32_t scr = pw::SCR + (uint32_t)wave * WSCR + (lid & 63u) * 16u;
        const int rg4 = (int)(lid >> 4) * 4;
#pragma unroll
        for (int c = 0; c < QB; ++c) {
          if (!__builtin_amdgcn_ballot_w64((hitc >> c) & 1u)) continue;   // uniform
          const float nth = -th[c];
          const int64_t q = st * TQ + 16 * c + (int)(lid & 15u);
          uint32_t hm = 0;   // rows j = 4 i + r of this lane that pass
#pragma unroll
          for (int j = 0; j < 4 * RB; ++j) hm |= !(acc[j >> 2][c][j & 3] < nth) ? (1u << j) : 0u;
          hm &= q < p.B ? vmask : 0u;
          if (hm) {
#pragma unroll
            for (int i = 0; i < RB; ++i)
              *reinterpret_cast<volatile OFR_LDS f6t::f32x4*>((uintptr_t)(scr + 1024u * i)) = acc[i][c];
          }
          for (;;) {   // wave-uniform: one kept row per lane and round
            const bool act = hm != 0u;
            const uint64_t mk = __builtin_amdgcn_ballot_w64(act);
            if (mk == 0) break;
            if (act) {
              const int j = __builtin_ctz(hm);
              hm &= hm - 1u;
              const float v = __uint_as_float(pp::lds_u32(scr + 1024u * (uint32_t)(j >> 2) + 4u * (uint32_t)(j & 3)));
              const uint32_t kb = __float_as_uint(key_score(score_key(-v, 0)));
              const int row = 16 * (j >> 2) + rg4 + (j & 3);   // of the wave's WR
              const uint32_t slot = ncnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32),
                                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u));
              if (slot < (uint32_t)pw::HCAPW) {
                f6t::i32x2 e;
                e[0] = (int)kb;
                e[1] = (int)(((uint32_t)q << RSH) | (uint32_t)row);
                *reinterpret_cast<volatile OFR_LDS f6t::i32x2*>((uintptr_t)(hits_a + slot * 8u)) = e;
              } else {   // the list is full (small galleries keep a large share): straight to the bucket
                const int bs = atomicAdd(p.count + q, 1);
                if (bs < p.cap) p.bucket[q * p.cap + bs] = Cand{__uint_as_float(kb), (int)(g0 + row)};
              }
            }
            ncnt += (uint32_t)__builtin_popcountll(mk);
          }
        }
      }
    };
    pw::i32x8 B0[QB], B1[QB];
    uint2 t0[QB], t1[QB];
    qload(s0, B0, t0);
    if constexpr (PF == 1) {
      for (int64_t st = s0; st < s1; ++st) step(st, B0, t0);
    } else {
      if (s0 + 1 < s1) qload(s0 + 1, B1, t1);
      for (int64_t st = s0; st < s1; st += 2) {
        step(st, B0, t0);
        if (st + 1 < s1) step(st + 1, B1, t1);
      }
    }
    // the item's kept pairs -> bucket slots and entries
    const uint32_t n = ncnt < (uint32_t)pw::HCAPW ? ncnt : (uint32_t)pw::HCAPW;
    for (uint32_t e = lane; e < n; e += 64u) {
      const uint2 hv = pp::lds_u2(hits_a + e * 8u);
      const int64_t q = (int64_t)(hv.y >> RSH);
      const int slot = atomicAdd(p.count + q, 1);
      if (slot < p.cap) p.bucket[q * p.cap + slot] = Cand{__uint_as_float(hv.x), (int)(g0 + (hv.y & (uint32_t)(WR - 1)))};
    }
  }
}

// ---- the prefix tier's sample pass as a wave pass (round 6) -------------------------------------------
// The sieve threshold of the prefix tier is the rank-th best prefix score (rank <= 2 here) over the row
// sample (every 64th gallery row, the f6 tier's sample tiles and row scales, the prefix terms spaux).  The
// 32x32x64 tile kernel with its top-16 epilogue took 0.09 ms for a 15.6k-row sample at B = 4,096 (992
// workgroups, fixed costs per tile); here the prefix_wave_kernel<8, 2> layout -- each wave 128 sample rows
// resident, 32-query steps from L2 -- with no hit path: per query column each lane keeps the two best of its
// 32 scores, two shuffles combine the column's 4 lane groups, and the wave writes the (best, second) keys of
// its 128 rows per query to keys[q][T] (T = ceil(Ns / 128)); sieve_threshold2_kernel takes the rank-th of
// each query's 2 T keys.  The gallery scales are the f6 tier's (not powers of two): score = fma(-2 s_g, acc,
// aux) after an MFMA with the block scales only, as prefix_pass_kernel<false>.
namespace sw {
constexpr int RB = 8, QB = 2, WR = 128, TGI = 512, TQ = 32;
}
__global__ void __launch_bounds__(256, 2) sample_wave_kernel(TileArgs p, uint2* keys, int64_t T, int64_t qg) {
  using namespace sw;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63;
  const int64_t nsteps = (p.B + TQ - 1) / TQ, ntg = (p.N + TGI - 1) / TGI;
  const int64_t ngrp = (nsteps + qg - 1) / qg, items = ntg * ngrp;
  if ((int64_t)blockIdx.x >= items) return;
  int scs;   // the lane's stage-0 block scale byte (its 32-feature block lane >> 4)
  {
    const uint32_t r0 = f6t::sload_bscale(p.bs, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    scs = f6t::lane_byte(r0, 8u * (lane >> 4));
  }
  // the sample's and the queries' tiles: full-depth f6 tiled buffers (stage stride nk), stage 0 read
  const int64_t pb = (int64_t)p.nk * f6t::PANEL;
  const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)p.G, 0, (int)(f6t::panels(p.N) * pb),
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)p.Q, 0, (int)(f6t::panels(p.B) * pb),
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t raux = __builtin_amdgcn_make_buffer_rsrc((void*)p.aux, 0, (int)(p.N * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc((void*)p.gscale, 0, (int)(p.N * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rqs = __builtin_amdgcn_make_buffer_rsrc((void*)p.qscale, 0, (int)(p.B * 4), 0x00020000);
  const int g4 = (int)(lane >> 4) * 4, r16 = (int)(lane & 15);
  const uint32_t ng32 = (uint32_t)ngrp, qg32 = (uint32_t)qg;
  for (int64_t w = blockIdx.x; w < items; w += gridDim.x) {
    const int64_t gt = (int64_t)((uint32_t)w / ng32), s0 = (int64_t)(((uint32_t)w % ng32) * qg32);
    const int64_t s1 = s0 + qg < nsteps ? s0 + qg : nsteps;
    const int64_t g0 = gt * TGI + wave * WR;   // the wave's first sample row
    const int nvalid = p.N - g0 < WR ? (int)(p.N - g0) : WR;
    if (nvalid <= 0) continue;   // uniform
    const int64_t tw = gt * 4 + wave;   // the wave's 128-row list index
    pw::i32x8 A[RB];
    float av[RB][4], tp[RB][4];   // the lane's output rows: prefix term (+inf past Ns), 2 s_g
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const uint32_t wr = (uint32_t)(wave * WR + 16 * i);
      A[i] = pw::gfrag(rg, (uint32_t)((gt * (TGI / 256) + (wr >> 8)) * pb), wr & 255u, lane);
      const int rb = 16 * i + g4;
      const f6t::i32x4 a4 = __builtin_bit_cast(
          f6t::i32x4, __builtin_amdgcn_raw_buffer_load_b128(raux, (int)((g0 + rb) * 4), 0, 0));
      const f6t::i32x4 s4 = __builtin_bit_cast(
          f6t::i32x4, __builtin_amdgcn_raw_buffer_load_b128(rsc, (int)((g0 + rb) * 4), 0, 0));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool ok = rb + r < nvalid;
        av[i][r] = ok ? __int_as_float(a4[r]) : __builtin_inff();
        tp[i][r] = ok ? 2.0f * __int_as_float(s4[r]) : 0.0f;
      }
    }
    auto qload = [&](int64_t st, pw::i32x8 (&b)[QB], int (&sq)[QB]) {
#pragma unroll
      for (int c = 0; c < QB; ++c) {
        const int64_t qr = st * TQ + 16 * c;
        b[c] = pw::gfrag(rq, (uint32_t)((qr >> 8) * pb), (uint32_t)(qr & 255), lane);
        const uint32_t sb = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rqs, (int)((qr + r16) * 4), 0, 0);
        sq[c] = scs + (sb != 0u ? (int)((sb >> 23) & 0xffu) - 127 : 0);   // block byte + e_q
      }
    };
    pw::i32x8 B[QB];
    int sq[QB];
    qload(s0, B, sq);
    const f6t::f32x4 zero = {0.f, 0.f, 0.f, 0.f};
    for (int64_t st = s0; st < s1; ++st) {
      f6t::f32x4 acc[RB][QB];
#pragma unroll
      for (int c = 0; c < QB; ++c)
#pragma unroll
        for (int i = 0; i < RB; ++i)
          acc[i][c] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[i], B[c], zero, 2, 2, 0, scs, 0, sq[c]);
      if (st + 1 < s1) qload(st + 1, B, sq);
#pragma unroll
      for (int c = 0; c < QB; ++c) {
        float m1 = __builtin_inff(), m2 = __builtin_inff();   // the lane's two best scores
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = __builtin_fmaf(-tp[i][r], acc[i][c][r], av[i][r]);
            m2 = fminf(m2, fmaxf(m1, x));
            m1 = fminf(m1, x);
          }
#pragma unroll
        for (int o = 16; o < 64; o <<= 1) {   // the column's 4 lane groups (rows 4 (l / 16) + ...)
          const float b1 = __shfl_xor(m1, o), b2 = __shfl_xor(m2, o);
          m2 = fminf(fmaxf(m1, b1), fminf(m2, b2));
          m1 = fminf(m1, b1);
        }
        const int64_t q = st * TQ + 16 * c + r16;
        if (lane < 16 && q < p.B) keys[q * T + tw] = make_uint2(score_key(m1, 0), score_key(m2, 0));
      }
    }
  }
}

__device__ __forceinline__ uint32_t arm_token(int64_t B);   // below (the sieve's arm token)
// Thresholds from sample_wave_kernel's key pairs: theta[q] = the rank-th (1 or 2) smallest of the query's 2 T
// keys; resets the bucket counts and arms the sieve (as sieve_threshold_kernel).  One wave per query.
__global__ void __launch_bounds__(256) sieve_threshold2_kernel(const uint2* keys, int64_t T, uint32_t* theta, int* count,
                                                               int64_t B, int rank, uint32_t* armed) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *armed = arm_token(B);
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= B) return;
  uint32_t k1 = KEY_NONE, k2 = KEY_NONE;
  for (int64_t e = lane; e < T; e += 64) {
    const uint2 v = keys[q * T + e];   // v.x <= v.y
    k2 = umin(umax(k1, v.x), umin(k2, v.y));
    k1 = umin(k1, v.x);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t b1 = (uint32_t)__shfl_xor((int)k1, o), b2 = (uint32_t)__shfl_xor((int)k2, o);
    k2 = umin(umax(k1, b1), umin(k2, b2));
    k1 = umin(k1, b1);
  }
  if (lane == 0) {
    theta[q] = rank <= 1 ? k1 : k2;
    count[q] = 0;
  }
}

// ---- small batches (B <= 32): HBM-streaming fp6 pass --------------------------------------
// One workgroup per 256-row gallery panel, wave w owns rows 32w..32w+31 against the (single)
// 32-row query block, loading its fragments straight to VGPRs from the f6 tiled layout (each
// gallery byte is used once: no LDS staging; the 243 KB of query fragments stay in L2).
// SU steps of loads (96 B per lane each) are in flight per wave: enough to stream HBM even at
// one 8-wave workgroup per CU.
// Epilogue: the 32 x 32 scores of each wave -> per-query best 16 (keys, as tile_epilogue),
// merged over the 8 waves through LDS -> the panel's best 16 rows per query.
constexpr int SU = 8;   // loads in flight per wave (round-1 probe: 8 + non-temporal = 74 % of HBM peak, 4 = 68 %)

template <bool NT = false>
__device__ __forceinline__ f6t::i32x8 stream_frag(const char* stage, int j, int h, int row) {
  const char* sb = stage + (2 * j + h) * 6144;
  f6t::i32x4 p0;
  f6t::i32x2 p1;
  if constexpr (NT) {   // streamed once: non-temporal, keeps L2 for the query fragments
    p0 = __builtin_nontemporal_load(reinterpret_cast<const f6t::i32x4*>(sb + row * 16));
    p1 = __builtin_nontemporal_load(reinterpret_cast<const f6t::i32x2*>(sb + 4096 + f6t::p1_slot(h, row) * 8));
  } else {
    p0 = *reinterpret_cast<const f6t::i32x4*>(sb + row * 16);
    p1 = *reinterpret_cast<const f6t::i32x2*>(sb + 4096 + f6t::p1_slot(h, row) * 8);
  }
  f6t::i32x8 f;
  f[0] = p0[0]; f[1] = p0[1]; f[2] = p0[2]; f[3] = p0[3];
  f[4] = p1[0]; f[5] = p1[1]; f[6] = 0; f[7] = 0;
  return f;
}

// U loads in flight per wave, NT non-temporal gallery loads (the library uses <SU, true>; other
// values are probe variants)
template <int U = SU, bool NT = false>
__global__ void __launch_bounds__(512) stream_kernel_f6(TileArgs p) {
  __shared__ uint32_t kbuf[8][32][KC];
  __shared__ float gtab[TG][2];
  const int64_t gt = blockIdx.x, g0 = gt * TG;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, h = lane >> 5, r32 = lane & 31;
  if (threadIdx.x < TG) {
    const int64_t g = g0 + threadIdx.x;
    const bool ok = g < p.N;
    gtab[threadIdx.x][0] = ok ? p.aux[g] : 0.f;
    gtab[threadIdx.x][1] = ok ? p.gscale[g] : 0.f;
  }
  const char* gpan = reinterpret_cast<const char*>(p.G) + gt * (int64_t)p.gnk * f6t::PANEL;
  const char* qpan = reinterpret_cast<const char*>(p.Q);
  const int nsteps = 2 * p.nkp, grow = wave * 32 + r32;   // nkp <= nk: the prefix tier's first stages
  f6t::f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = 0; k0 < nsteps; k0 += U) {
    f6t::i32x8 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u < nsteps ? k0 + u : nsteps - 1;
      a[u] = stream_frag<NT>(gpan + (k >> 1) * (int64_t)f6t::PANEL, k & 1, h, grow);
      b[u] = stream_frag<false>(qpan + (k >> 1) * (int64_t)f6t::PANEL, k & 1, h, r32);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u < nsteps) {
        // 64-feature step k = 2 stage + j: the lane's block is 2 j + h of the stage's four
        const int k = k0 + u;
        const int sc = (int)(p.bs[k >> 1] >> (8u * (uint32_t)(2 * (k & 1) + h)));
        acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[u], b[u], acc, 2, 2, 0, sc, 0, sc);
      }
  }
  __syncthreads();
  const int nvalid = p.N - g0 < TG ? (int)(p.N - g0) : TG;
  const float sq2 = 2.0f * p.qscale[r32 < p.B ? r32 : p.B - 1];
  KeyList L;
  L.init();
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int gl = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
    const float sc = gtab[gl][0] - sq2 * gtab[gl][1] * acc[r];
    L.insert(gl < nvalid ? score_key(sc, gl) : KEY_NONE);
  }
  uint32_t o[KC];
#pragma unroll
  for (int j = 0; j < KC; ++j) o[j] = (uint32_t)__shfl_xor((int)L.k[j], 32);
  L.merge(o);
  if (h == 0) {
#pragma unroll
    for (int j = 0; j < KC; ++j) kbuf[wave][r32][j] = L.k[j];
  }
  __syncthreads();
  if (threadIdx.x < 32 && (int64_t)threadIdx.x < p.B) {
    const int q = threadIdx.x;
#pragma unroll
    for (int j = 0; j < KC; ++j) L.k[j] = kbuf[0][q][j];
    for (int w = 1; w < 8; ++w) {
#pragma unroll
      for (int j = 0; j < KC; ++j) o[j] = kbuf[w][q][j];
      L.merge(o);
    }
    Cand* out = p.cand + ((size_t)q * p.ntg + gt) * KC;
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      const uint32_t kk = L.k[j];
      out[j] = kk == KEY_NONE ? Cand{__builtin_inff(), CAND_EMPTY} : Cand{key_score(kk), (int)(g0 + (kk & 0xffu))};
    }
  }
}

// ---- pass 2 ----------------------------------------------------------------------------

struct MergeArgs {
  const Cand* cand;       // tile lists [B][T][KC], or the sieve's buckets [B][cap]
  int64_t T, B;
  const float* Q;
  int64_t ldq;
  const float* G;
  int64_t ldg, d;
  const double* qstats;   // [B][3]: a, e, t
  const double* gmax;     // [4]: A, E, T, auxmax
  double gamma;           // fp32 accumulation bound of the coarse products / (a_q A): 0 for int8
  int k;
  int64_t index_base;
  double* out_d;
  int64_t* out_i;
  int* cert;
  double* bound;   // optional: squared-distance lower bound of every row outside the candidates
  const int* count;        // sieve: rows kept per query (null for tile lists)
  const uint32_t* theta;   // sieve: the keep thresholds
  int64_t cap;
  // split merge of a sharded gallery (ofr_knn_f6_merge_pruned): mode 1 selects the candidates and
  // writes them (sel [B][KC]), |q|^2, dS and the overflow flag (qd [B][3]) and the squared-distance
  // upper bounds of the best k (ub_local [B][k]); mode 2 re-ranks the selection, pruned by the
  // global bound ub [B] (the k-th smallest upper bound over every shard).  Mode 0: both at once.
  int mode;
  Cand* sel;
  double* qd;
  double* ub_local;
  const double* ub;
  // prefix tier f6p: the coarse scores cover features [0, dpre) only (0: all d).  A row's squared
  // distance is at least that of its first dpre features, S_m + |q_m|^2 with S_m = |g_m|^2 - 2 q_m.g_m
  // (the prefix scores, within dS of the keys), so the bounds below use |q_m|^2 for |q|^2 and a key
  // bounds nothing from above (no ub_local).
  int64_t dpre;
  int* evals;   // optional [B]: candidates re-ranked exactly per query (the merge's bytes: evals x d x 4)
  // deep continuation (round 6; sieve buckets, mode 0, the block-cooperative re-rank): a query the best 16
  // candidates do not certify re-ranks the bucket's next 16 by key, and so on (at most `deep` rounds), until
  // its k-th exact distance clears the bound of the rows it has not re-ranked or the bucket runs out; 0: off
  int deep;
};
constexpr int DEEP_ROUNDS = 32;   // the default round cap

// Best KC (distance, index) of the n candidates at src (16-byte aligned) into lists[0..KC),
// ascending; one 256-thread block.  16 B per lane and load (two candidates), fully coalesced,
// a per-thread sorted list, then a tree merge through lists[256 * KC].
__device__ __forceinline__ void block_best(const Cand* src, int64_t n, Cand* lists) {
  TopList<KC> L;
  L.init();
  const uint4* s4 = reinterpret_cast<const uint4*>(src);
  const int64_t n4 = n / 2;
  // BU loads in flight per thread: with few queries (B <= 32, one block each) the stream of
  // T * 16 candidates is latency-bound otherwise (285 us for one query at N = 1M)
  constexpr int BU = 8;
  for (int64_t e0 = threadIdx.x; e0 < n4; e0 += (int64_t)BU * blockDim.x) {
    uint4 v[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
      const int64_t e = e0 + (int64_t)u * blockDim.x;
      v[u] = e < n4 ? s4[e] : make_uint4(__float_as_uint(__builtin_inff()), CAND_EMPTY,
                                         __float_as_uint(__builtin_inff()), CAND_EMPTY);
    }
#pragma unroll
    for (int u = 0; u < BU; ++u) {
      const float d0 = __uint_as_float(v[u].x), d1 = __uint_as_float(v[u].z);
      if (better_f(d0, (int)v[u].y, L.d[KC - 1], L.i[KC - 1])) L.insert(d0, (int)v[u].y);
      if (better_f(d1, (int)v[u].w, L.d[KC - 1], L.i[KC - 1])) L.insert(d1, (int)v[u].w);
    }
  }
  if ((n & 1) && threadIdx.x == 0) L.insert(src[n - 1].d, src[n - 1].i);
#pragma unroll
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

// Best KC of a short candidate list (a sieve bucket) into lists[0..KC) (4 KC entries of LDS): per-thread
// lists, a shuffle merge inside each wave, then the four wave lists by thread 0.  The same KC best
// (distance, index) pairs as block_best (a unique set), in ascending order.
__device__ __forceinline__ void block_best_small(const Cand* src, int64_t n, Cand* lists) {
  TopList<KC> L;
  L.init();
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    const Cand c = src[e];
    if (better_f(c.d, c.i, L.d[KC - 1], L.i[KC - 1])) L.insert(c.d, c.i);
  }
  for (int off = 1; off < 64; off <<= 1) {
    float od[KC];
    int oi[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      od[j] = __shfl_xor(L.d[j], off);
      oi[j] = __shfl_xor(L.i[j], off);
    }
    L.merge(od, oi);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0 && wave > 0) {
#pragma unroll
    for (int j = 0; j < KC; ++j) lists[wave * KC + j] = Cand{L.d[j], L.i[j]};
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      float od[KC];
      int oi[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        od[j] = lists[w * KC + j].d;
        oi[j] = lists[w * KC + j].i;
      }
      L.merge(od, oi);
    }
#pragma unroll
    for (int j = 0; j < KC; ++j) lists[j] = Cand{L.d[j], L.i[j]};
  }
  __syncthreads();
}

// block_best_small over the entries strictly after `after` in (distance, index) order: the next KC (the deep
// continuation of the merge walks a bucket 16 candidates at a time)
__device__ __forceinline__ void block_best_small_after(const Cand* src, int64_t n, Cand* lists, Cand after) {
  TopList<KC> L;
  L.init();
  for (int64_t e = threadIdx.x; e < n; e += blockDim.x) {
    const Cand c = src[e];
    if (better_f(after.d, after.i, c.d, c.i) && better_f(c.d, c.i, L.d[KC - 1], L.i[KC - 1])) L.insert(c.d, c.i);
  }
  for (int off = 1; off < 64; off <<= 1) {
    float od[KC];
    int oi[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) {
      od[j] = __shfl_xor(L.d[j], off);
      oi[j] = __shfl_xor(L.i[j], off);
    }
    L.merge(od, oi);
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0 && wave > 0) {
#pragma unroll
    for (int j = 0; j < KC; ++j) lists[wave * KC + j] = Cand{L.d[j], L.i[j]};
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) {
      float od[KC];
      int oi[KC];
#pragma unroll
      for (int j = 0; j < KC; ++j) {
        od[j] = lists[w * KC + j].d;
        oi[j] = lists[w * KC + j].i;
      }
      L.merge(od, oi);
    }
#pragma unroll
    for (int j = 0; j < KC; ++j) lists[j] = Cand{L.d[j], L.i[j]};
  }
  __syncthreads();
}

// Small batches: the streaming pass leaves T * KC candidates per query (62.5k at N = 1M), and one
// merge block per query inserting them into per-thread sorted lists is divergent and serial
// (240 us per query).  PM blocks per query first reduce contiguous chunks to their best KC.
constexpr int PM = 64;
__global__ void __launch_bounds__(256) premerge_kernel(const Cand* cand, int64_t T, Cand* out) {
  __shared__ Cand lists[256 * KC];
  const int64_t q = blockIdx.y;
  const int64_t n = T * KC;
  const int64_t chunk = ((n + PM - 1) / PM + 1) & ~(int64_t)1;   // even: chunks start 16-B aligned
  const int64_t b = (int64_t)blockIdx.x * chunk;
  const int64_t e = b + chunk < n ? b + chunk : n;
  block_best(cand + q * n + (b < n ? b : 0), e > b ? e - b : 0, lists);
  if ((int)threadIdx.x < KC) out[(q * PM + blockIdx.x) * KC + threadIdx.x] = lists[threadIdx.x];
}

// the sieve's arm token for a B-query batch: a magic word and B (a stale or uninitialised workspace
// word, or one armed for another batch size, does not match)
__device__ __forceinline__ uint32_t arm_token(int64_t B) {
  const uint32_t t = 0x5EE7A11Du ^ (uint32_t)(B * 2654435761u);
  return t ? t : 1u;   // never 0: the disarmed value
}

// Sieve thresholds from the sample pass's tile lists: theta[q] = the rank-th best key (KEY_NONE
// when the sample holds fewer than rank rows; rank <= KC); resets the bucket counts.  One wave per query (four
// per block): each lane keeps the best 16 keys of its strided share (KeyList, one v_med3 per slot),
// then six shuffle rounds merge the lanes' lists (the same value as sorting the whole list by
// (score, index): only the 16th score is used, and score_key is monotone).
__global__ void __launch_bounds__(256) sieve_threshold_kernel(const Cand* lists, int64_t T, uint32_t* theta,
                                                              int* count, int64_t B, int rank, uint32_t* armed) {
  // the buckets are reset: one sieve pass may follow (sieve_arm_kernel checks this exact value)
  if (blockIdx.x == 0 && threadIdx.x == 0) *armed = arm_token(B);
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= B) return;
  const Cand* src = lists + (size_t)q * T * KC;
  const int64_t n = T * KC;
  KeyList L;
  L.init();
  constexpr int U = 4;   // loads in flight per lane
  for (int64_t e0 = lane; e0 < n; e0 += 64 * U) {
    Cand c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t e = e0 + 64 * u;
      c[u] = e < n ? src[e] : Cand{__builtin_inff(), CAND_EMPTY};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) L.insert(c[u].i != CAND_EMPTY ? score_key(c[u].d, 0) : KEY_NONE);
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t o[KC];
#pragma unroll
    for (int j = 0; j < KC; ++j) o[j] = (uint32_t)__shfl_xor((int)L.k[j], off);
    L.merge(o);
  }
  if (lane == 0) {
    uint32_t t = L.k[KC - 1];
#pragma unroll
    for (int j = 0; j < KC; ++j) t = j == rank - 1 ? L.k[j] : t;   // register array: constant indices
    theta[q] = t;
    count[q] = 0;
  }
}

// Before a sieve pass: it appends to the buckets, so it is valid once per sample pass (which resets them
// and arms the flag).  A second sieve pass on the same thresholds (phases 8 called twice) would append
// every kept row again, and duplicated candidates could certify a top-k that repeats one row: it is
// made to overflow every bucket instead (uncertified, bound -inf).  One workgroup; disarms.
// Given keep thresholds (round 6, ofr_knn_f6_set_thresholds): theta[q] = the smallest order key whose bucket's
// lower end key_score(theta) is >= smax[q] (the sieve keeps every row whose coarse score is <= the upper end of
// that bucket, and the certificate's bound from theta then covers smax); NaN or +inf: KEY_NONE (keep every row).
// Resets the counts and arms one sieve pass of a B-query batch, as sieve_threshold_kernel does.
__global__ void __launch_bounds__(256) set_thresholds_kernel(const double* smax, int64_t B, uint32_t* theta, int* count,
                                                             uint32_t* armed) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *armed = arm_token(B);
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  const double v = smax[q];
  uint32_t t = KEY_NONE;
  if (v == v && v < 3.0e38) {
    float f = (float)(v > -3.0e38 ? v : -3.0e38);
    if ((double)f < v)   // the next float up
      f = f == 0.0f ? __uint_as_float(1u) : __uint_as_float(__float_as_uint(f) + (f > 0.0f ? 1u : 0xffffffffu));
    t = score_key(f, 0);
    for (int it = 0; it < 2 && (double)key_score(t) < v && t < KEY_NONE - 0x1ffu; ++it) t += 0x100u;
    if ((double)key_score(t) < v) t = KEY_NONE;
  }
  theta[q] = t;
  count[q] = 0;
}

__global__ void __launch_bounds__(256) sieve_arm_kernel(uint32_t* armed, int* count, int64_t B, int cap) {
  // (a workspace never armed for this B holds anything: only the threshold kernel's token for B arms it;
  // uninitialised memory equals it with probability 2^-32)
  __shared__ uint32_t a;
  if (threadIdx.x == 0) a = __atomic_load_n(armed, __ATOMIC_RELAXED);
  __syncthreads();
  if (threadIdx.x == 0) *armed = 0u;
  if (a != arm_token(B))
    for (int64_t q = threadIdx.x; q < B; q += blockDim.x) count[q] = cap + 1;
}

// One block per query.  (1) best KC of the tile lists (query-major: cand[q][t][KC], one
// contiguous stream) or of the query's sieve bucket; (2) the exact fp64 distance
// (distance.py:60) of the survivors in coarse order, one wave per candidate (float4 loads, lane
// partial sums, shuffle reduction), until the coarse bound proves the rest cannot reach the
// k-th; (3) sort by (distance, index) and the certificate.
// SMALL: the sieve's buckets (~120-260 rows per query): block_best_small and 4 KC list entries of LDS
// instead of block_best's 256 KC (32 KiB), so 4x as many merge blocks fit a CU.
// COOP (round 6, the default): each candidate's exact distance is summed by the whole block -- every
// thread holds its 10 float4 of the query row in registers for the block's life (d <= 10,240) and issues
// its 10 float4 of the candidate row at once, one block reduction per candidate -- and the stop test runs
// after every candidate, not every fourth: one HBM round trip per re-rank, no query re-reads from L2.
// The per-candidate sum order differs from the wave form (!COOP), so the two give distances within one
// fp64 rounding of each other; one library uses one form for every tier.
// DEEP (sieve buckets, COOP): a second launch behind the plain one (launch_merge) for the queries it left
// uncertified -- every other block returns at once -- which redoes the query's merge and then continues it
// (MergeArgs::deep); kept out of the first launch, whose registers it would crowd (0.338 -> 0.364 ms).
template <bool SMALL, bool COOP, bool DEEP = false>
__global__ void __launch_bounds__(256, COOP ? 4 : 1) merge_kernel(MergeArgs p) {
  __shared__ Cand lists[(SMALL ? 4 : 256) * KC];
  __shared__ double exact[KC];
  __shared__ double red[4];
  __shared__ double red2[2][4];
  __shared__ int stop_flag;
  const int64_t q = blockIdx.x;
  if constexpr (DEEP) {   // certified, or a bucket that dropped rows: nothing to continue
    if (p.cert[q] != 0 || !p.count || !p.theta || p.count[q] > p.cap || p.count[q] < 0) return;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  bool overflow = false;
  const float* qr = p.Q + q * p.ldq;
  double qq, dS;
  const int kk = p.k < KC ? p.k : KC;
  const int64_t d4 = p.d >> 2;
  const bool vec = ((p.ldq | p.ldg) & 3) == 0 && (((uintptr_t)p.Q | (uintptr_t)p.G) & 15) == 0;
  // exact squared distance (distance.py:60, in fp64) of candidate cc, one wave (the sum in every lane)
  auto exact_d2 = [&](const Cand& cc) -> double {
    double a = 0;
    const float* gr = p.G + (int64_t)cc.i * p.ldg;
    int64_t j0 = 0;
    if (vec) {
      const float4* q4 = reinterpret_cast<const float4*>(qr);
      const float4* g4 = reinterpret_cast<const float4*>(gr);
      // DU float4 pairs in flight per lane (a lone query's merge is one block: its loop is bound by
      // the memory latency); the sum runs in the same order as one float4 per iteration
      constexpr int DU = 4;
      for (int64_t j = lane; j < d4; j += 64 * DU) {
        float4 x[DU], y[DU];
#pragma unroll
        for (int u = 0; u < DU; ++u) {
          const int64_t jj = j + 64 * u;
          x[u] = jj < d4 ? q4[jj] : make_float4(0.f, 0.f, 0.f, 0.f);
          y[u] = jj < d4 ? g4[jj] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < DU; ++u) {
          if (j + 64 * u < d4) {
            const double e0 = (double)x[u].x - (double)y[u].x, e1 = (double)x[u].y - (double)y[u].y;
            const double e2 = (double)x[u].z - (double)y[u].z, e3 = (double)x[u].w - (double)y[u].w;
            a += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
          }
        }
      }
      j0 = d4 * 4;
    }
    for (int64_t j = j0 + lane; j < p.d; j += 64) {
      const double df = (double)qr[j] - (double)gr[j];
      a += df * df;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    return a;
  };
  // COOP: the block's query row, float4 j = threadIdx.x + 256 u, held when d fits (MQ float4 per thread)
  constexpr int MQ = 10;
  const bool qres = vec && d4 <= 256 * MQ && (p.mode != 1 || p.dpre > 0);   // (mode 1 of f6: no re-rank)
  float4 qv[MQ];
  // buffer loads of float4 j = threadIdx.x + 256 u of a row's first d4 float4: one 32-bit offset per load
  // (no 64-bit addresses), and the range check returns zeros past d4 (the offset in voffset: the check
  // covers voffset + offset, not soffset)
  auto row_load = [&](const float* row, int64_t n4, float4* v, auto nu) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row), 0, (int)(n4 * 16), 0x00020000);
#pragma unroll
    for (int u = 0; u < decltype(nu)::value; ++u)
      v[u] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)((threadIdx.x + 256 * u) * 16), 0, 0));
  };
  using NQ = std::integral_constant<int, MQ>;
  using NC = std::integral_constant<int, 4>;   // float4 per thread and chunk past MQ
  auto load_query = [&]() { row_load(qr, d4, qv, NQ{}); };   // right before the re-rank (not live during the selection)
  int rb = 0;   // red2 buffer of the next block reduction (two: one barrier per reduction)
  // COOP: exact squared distance of gallery row `row`, the whole block (block-uniform call; the sum in
  // every thread): per thread its float4 in u order, the scalar tail, then lanes by xor shuffles and the
  // four waves in a fixed order
  auto exact_block = [&](int row) -> double {
    row = __builtin_amdgcn_readfirstlane(row);   // block-uniform: a scalar buffer descriptor
    const float* gr = p.G + (int64_t)row * p.ldg;
    double a = 0;
    if (qres) {
      float4 y[MQ];
      row_load(gr, d4, y, NQ{});   // every load issued at once: one HBM round trip per candidate
#pragma unroll
      for (int u = 0; u < MQ; ++u) {   // padding lanes add (0 - 0)^2 = 0 exactly
        // laundered: else the compiler hoists the 40 fp64 conversions of the query out of the candidate
        // loop (80 VGPRs, 218 in all)
        float4 x = qv[u];
        asm volatile("" : "+v"(x.x), "+v"(x.y), "+v"(x.z), "+v"(x.w));
        const double e0 = (double)x.x - (double)y[u].x, e1 = (double)x.y - (double)y[u].y;
        const double e2 = (double)x.z - (double)y[u].z, e3 = (double)x.w - (double)y[u].w;
        a += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
      }
      for (int64_t j = d4 * 4 + threadIdx.x; j < p.d; j += 256) {
        const double df = (double)qr[j] - (double)gr[j];
        a += df * df;
      }
    } else {
      int64_t j0 = 0;
      if (vec) {   // d > 10,240: the query re-read per chunk of 1,024 float4
        for (int64_t c0 = 0; c0 < d4; c0 += 256 * NC::value) {
          float4 x[NC::value], y[NC::value];
          const int64_t n4 = d4 - c0 < 256 * NC::value ? d4 - c0 : 256 * NC::value;
          row_load(qr + 4 * c0, n4, x, NC{});
          row_load(gr + 4 * c0, n4, y, NC{});
#pragma unroll
          for (int u = 0; u < NC::value; ++u) {
            const double e0 = (double)x[u].x - (double)y[u].x, e1 = (double)x[u].y - (double)y[u].y;
            const double e2 = (double)x[u].z - (double)y[u].z, e3 = (double)x[u].w - (double)y[u].w;
            a += e0 * e0 + e1 * e1 + e2 * e2 + e3 * e3;
          }
        }
        j0 = d4 * 4;
      }
      for (int64_t j = j0 + threadIdx.x; j < p.d; j += 256) {
        const double df = (double)qr[j] - (double)gr[j];
        a += df * df;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    double* rr = red2[rb];
    rb ^= 1;
    if (lane == 0) rr[wave] = a;
    __syncthreads();
    return (rr[0] + rr[1]) + (rr[2] + rr[3]);
  };
  if (p.mode == 2) {   // the selection of a mode-1 launch
    if (threadIdx.x < KC) lists[threadIdx.x] = p.sel[q * KC + threadIdx.x];
    qq = p.qd[q * 3 + 0];
    dS = p.qd[q * 3 + 1];
    overflow = p.qd[q * 3 + 2] != 0.0;
    __syncthreads();
  } else {
    if (p.count) {
      const int64_t c = p.count[q];
      overflow = c > p.cap || c < 0;   // rows were dropped (and a tile-level overflow writes none): no candidates
      if constexpr (SMALL) block_best_small(p.cand + (size_t)q * p.cap, overflow ? 0 : c, lists);
      else block_best(p.cand + (size_t)q * p.cap, overflow ? 0 : c, lists);
    } else if constexpr (!SMALL) {
      block_best(p.cand + (size_t)q * p.T * KC, p.T * KC, lists);
    }
    // loads batched 8 deep: with few queries (one block each) a loop with one load per iteration is
    // bound by the memory latency, not the bytes
    constexpr int RU = 8;
    const int64_t dm = p.dpre > 0 && p.dpre < p.d ? p.dpre : p.d;   // the features the keys cover
    qq = 0;
    for (int64_t j0 = threadIdx.x; j0 < dm; j0 += (int64_t)RU * blockDim.x) {
      float x[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int64_t j = j0 + (int64_t)u * blockDim.x;
        x[u] = j < dm ? qr[j] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) qq += (double)x[u] * (double)x[u];
    }
    // qq = |q_m|^2 over the keys' features (all d but for the prefix tier), the base of every bound
    qq = block_sum_f64(qq, red);
    // dS(q): |S - S~| <= dS for every row, S = d^2 - |q|^2
    const double qa = p.qstats[q * 3 + 0], qe = p.qstats[q * 3 + 1], qt = p.qstats[q * 3 + 2];
    const double A = p.gmax[0], E = p.gmax[1], T = p.gmax[2], auxmax = p.gmax[3];
    // the prefix tier's pass adds -aux inside the MFMA's fp32 accumulation (prefix_pass_kernel<true>: at most
    // 129 roundings of partial sums <= aux + sum|products|, <= 129 2^-24 aux < 2^-17 aux) -- 2^-14 there
    const double auxe = p.dpre > 0 ? 0x1p-14 : 0x1p-20;
    dS = 2.0 * (qa * E + qe * A + qe * E + qt * T) + auxe * auxmax + 0x1p-20 * (2.0 * qa * A) + 2.0 * p.gamma * qa * A;
    dS = dS * (1.0 + 1e-6) + 1e-300;
    if (p.mode == 1) {
      if (threadIdx.x < KC) p.sel[q * KC + threadIdx.x] = lists[threadIdx.x];
      if (p.dpre > 0) {
        // a prefix key bounds nothing from above: the exact squared distances of the first kk
        // candidates do (round 6) -- k real rows of this shard lie that close, so the k-th smallest
        // of these over the shards bounds the global k-th; the other shards' candidates whose prefix
        // lower bound exceeds it are then never re-ranked (mode 2)
        if constexpr (COOP) {
          if (qres) load_query();
          for (int c = 0; c < kk; ++c) {   // block-uniform: lists (after a barrier) and overflow
            const Cand cc = lists[c];
            const double a = cc.i != CAND_EMPTY && !overflow ? exact_block(cc.i) : __builtin_inf();
            if (threadIdx.x == 0) exact[c] = a;
          }
        } else {
          for (int c = wave; c < kk; c += 4) {
            const Cand cc = lists[c];
            const double a = cc.i != CAND_EMPTY && !overflow ? exact_d2(cc) : __builtin_inf();
            if (lane == 0) exact[c] = a;
          }
        }
        __syncthreads();
      }
      if (threadIdx.x == 0) {
        p.qd[q * 3 + 0] = qq;
        p.qd[q * 3 + 1] = dS;
        p.qd[q * 3 + 2] = overflow ? 1.0 : 0.0;
        // upper bound of d^2 of the j-th candidate: its truncated key t is within 256 ulp below
        // the fp32 coarse score (|sc - t| <= |t| 2^-15, 2^-14 taken), S <= sc + dS, d^2 = S + |q|^2;
        // the lists are in ascending key order, so the bounds ascend too
        if (p.dpre > 0) {   // the exact values, ascending (insertion sort of <= 16), a relative 1e-12 up
          for (int j = 1; j < kk; ++j) {
            const double v = exact[j];
            int t = j - 1;
            for (; t >= 0 && exact[t] > v; --t) exact[t + 1] = exact[t];
            exact[t + 1] = v;
          }
          for (int j = 0; j < kk; ++j) p.ub_local[q * kk + j] = exact[j] * (1.0 + 1e-12) + 1e-300;
        } else {
          for (int j = 0; j < kk; ++j) {
            const Cand c = lists[j];
            const double t = (double)c.d;
            p.ub_local[q * kk + j] = c.i == CAND_EMPTY || overflow
                                         ? __builtin_inf()
                                         : (t + fabs(t) * 0x1p-14 + dS + qq) * (1.0 + 1e-12) + 1e-300;
          }
        }
      }
      return;
    }
  }
  // lower bound of d^2 of any row whose (truncated) coarse score is >= s, less a relative 1e-12
  // for the fp64 evaluation
  auto d2_lower = [&](double s) { return (s - dS + qq) - 1e-12 * (fabs(s) + dS + 2.0 * qq); };
  // sharded (mode 2): no row whose lower bound exceeds ub -- an upper bound of the GLOBAL k-th
  // squared distance -- can be among the global k nearest, so it need not be re-ranked
  const double ubq = p.ub ? p.ub[q] : __builtin_inf();
  int skip_all = 0;
  if (p.ub) {
    if (threadIdx.x == 0)
      stop_flag = lists[0].i == CAND_EMPTY || d2_lower((double)lists[0].d) > ubq;
    __syncthreads();
    skip_all = stop_flag;
    if (skip_all && (int)threadIdx.x < KC) exact[threadIdx.x] = __builtin_inf();
  }
  // exact fp64 distance (distance.py:60) of the candidates in coarse order, 4 per round (one per
  // wave); stop once the next candidate's lower bound exceeds the k-th exact distance so far:
  // it and every later one (and every row outside the list) are strictly farther
  int nevals = 0;   // candidates re-ranked exactly (wave 0's count; MergeArgs::evals)
  bool deep_need = false;   // the first 16 candidates, all re-ranked, do not certify (block-uniform)
  if constexpr (COOP) {
    // one candidate at a time; lane c of every wave keeps exact[c] (mine), so the stop test needs no
    // LDS round trip: the same test as the wave form's, after every candidate
    double mine = __builtin_inf(), best = __builtin_inf();
    if (qres && !skip_all) load_query();
    int c = 0;
    for (; c < KC && !skip_all; ++c) {
      const Cand cc = lists[c];   // block-uniform
      if (cc.i == CAND_EMPTY) break;   // every later one is empty too
      if (c > 0) {
        double lim = ubq;
        if (c >= kk) {
          double kth = best;
          if (kk > 1) {   // the kk-th smallest of exact[0..c): lane t ranks its value among them
            const double v = lane < c ? mine : __builtin_inf();
            int lt = 0, le = 0;
            for (int u = 0; u < c; ++u) {
              const double e = __shfl(mine, u);
              lt += e < v;
              le += e <= v;
            }
            const uint64_t m = __ballot(lane < c && lt < kk && kk <= le);
            kth = m ? __shfl(v, __ffsll((long long)m) - 1) : __builtin_inf();
          }
          lim = fmin(kth * kth, ubq);
        }
        if (d2_lower((double)cc.d) > lim) break;
      }
      const double e = sqrt(exact_block(cc.i));
      if (lane == c) mine = e;
      best = fmin(best, e);
      ++nevals;
    }
    if (wave == 0 && lane < KC) exact[lane] = lane < c ? mine : __builtin_inf();
    if constexpr (SMALL && DEEP) {
      // every thread decides alike from its registers (no barrier on the common, certified path): a stop
      // before the 16th candidate certifies, an exhausted bucket cannot continue
      if (p.deep && p.count && p.theta && p.mode == 0 && !overflow && !skip_all && c == KC) {
        double kth = best;
        if (kk > 1) {
          const double v = mine;
          int lt = 0, le = 0;
          for (int u = 0; u < KC; ++u) {
            const double e = __shfl(mine, u);
            lt += e < v;
            le += e <= v;
          }
          const uint64_t m = __ballot(lane < KC && lt < kk && kk <= le);
          kth = m ? __shfl(v, __ffsll((long long)m) - 1) : __builtin_inf();
        }
        uint32_t tk = lists[KC - 1].i != CAND_EMPTY ? score_key(lists[KC - 1].d, 0) : KEY_NONE;
        tk = umin(tk, p.theta[q]);
        const double bnd = tk != KEY_NONE ? d2_lower((double)key_score(tk)) : __builtin_inf();
        deep_need = !(kth == kth && kth * kth < bnd) && lists[KC - 1].i != CAND_EMPTY;
      }
    }
  }
  for (int r = 0; r < (COOP ? 0 : KC / 4) && !skip_all; ++r) {
    const int c = 4 * r + wave;
    const Cand cc = lists[c];
    const double a = cc.i != CAND_EMPTY ? exact_d2(cc) : 0.0;
    if (lane == 0) exact[c] = cc.i != CAND_EMPTY ? sqrt(a) : __builtin_inf();
    __syncthreads();
    const int done = 4 * r + 4;
    if (wave == 0) {   // the stop test, on one wave: lane t ranks exact[t] among exact[0..done)
      nevals += (lists[done - 4].i != CAND_EMPTY) + (lists[done - 3].i != CAND_EMPTY) +
                (lists[done - 2].i != CAND_EMPTY) + (lists[done - 1].i != CAND_EMPTY);
      int st = 0;
      if (done < KC && done >= kk) {
        if (lists[done].i == CAND_EMPTY) {
          st = 1;
        } else {
          const double v = lane < done ? exact[lane] : __builtin_inf();   // kk-th smallest of exact[0..done)
          int lt = 0, le = 0;
          for (int u = 0; u < done; ++u) {
            const double e = exact[u];
            lt += e < v;
            le += e <= v;
          }
          const uint64_t m = __ballot(lane < done && lt < kk && kk <= le);   // lanes holding the kk-th value
          const double kth = m ? __shfl(v, __ffsll((long long)m) - 1) : __builtin_inf();
          st = d2_lower((double)lists[done].d) > fmin(kth * kth, ubq);
        }
      } else if (done < KC && p.ub) {
        st = lists[done].i == CAND_EMPTY || d2_lower((double)lists[done].d) > ubq;
      }
      if (lane == 0) stop_flag = st;
    }
    __syncthreads();
    if (stop_flag) {
      if ((int)threadIdx.x >= done && (int)threadIdx.x < KC) exact[threadIdx.x] = __builtin_inf();
      break;
    }
  }
  uint32_t tk_deep = 0;   // the deep continuation's bound key (min(16th key of its last round, theta))
  bool deep_ran = false;
  if constexpr (SMALL && COOP && DEEP) {
    if (deep_need) {
      __shared__ Cand run_l[KC];          // the best KC re-ranked so far, ascending by (distance, row)
      __shared__ double run_e[KC];
      __shared__ int dstate;
      __shared__ uint32_t dtk;
      // wave 0: run <- the best KC of run (unless fresh) and (lists, exact), by (distance, row)
      auto merge_run = [&](bool fresh) {
        double x = __builtin_inf();
        int64_t xi = INT64_MAX;
        if (lane < KC) {
          if (!fresh && run_l[lane].i != CAND_EMPTY) {
            x = run_e[lane];
            xi = run_l[lane].i;
          }
        } else if (lane < 2 * KC) {
          const Cand cc = lists[lane - KC];
          if (cc.i != CAND_EMPTY && exact[lane - KC] == exact[lane - KC] && exact[lane - KC] < __builtin_inf()) {
            x = exact[lane - KC];
            xi = cc.i;
          }
        }
        int rank = 0;
        for (int u = 0; u < 2 * KC; ++u) {
          const double y = __shfl(x, u);
          const int64_t yi = __shfl(xi, u);
          rank += better_d(y, yi, x, xi) || (y == x && yi == xi && u < lane);
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < 2 * KC && rank < KC) {
          run_l[rank] = Cand{0.f, xi != INT64_MAX ? (int)xi : CAND_EMPTY};
          run_e[rank] = x;
        }
      };
      __syncthreads();   // exact[] of the first 16 written (wave 0)
      if (wave == 0) merge_run(true);
      __syncthreads();
      for (int round = 0; round <= p.deep; ++round) {
        if (threadIdx.x == 0) {   // certified by the rows re-ranked so far?  (as the final certificate)
          uint32_t tk = lists[KC - 1].i != CAND_EMPTY ? score_key(lists[KC - 1].d, 0) : KEY_NONE;
          tk = umin(tk, p.theta[q]);
          const double kth = run_l[kk - 1].i != CAND_EMPTY ? run_e[kk - 1] : __builtin_inf();
          const double bnd = tk != KEY_NONE ? d2_lower((double)key_score(tk)) : __builtin_inf();
          dtk = tk;
          dstate = (kth == kth && kth * kth < bnd) ? 1 : (lists[KC - 1].i == CAND_EMPTY || round == p.deep ? 2 : 0);
        }
        __syncthreads();
        if (dstate != 0) break;   // block-uniform
        deep_ran = true;
        const Cand after = lists[KC - 1];
        const double kth = run_l[kk - 1].i != CAND_EMPTY ? run_e[kk - 1] : __builtin_inf();
        __syncthreads();   // every thread has `after` before the lists are replaced
        block_best_small_after(p.cand + (size_t)q * p.cap, p.count[q], lists, after);
        if (qres) load_query();   // re-read: the query registers are not live across the selection (spills)
        double mine2 = __builtin_inf();
        int c = 0;
        for (; c < KC; ++c) {   // in key order, while a candidate's lower bound can still reach the k-th
          const Cand cc = lists[c];
          if (cc.i == CAND_EMPTY || d2_lower((double)cc.d) > kth * kth) break;
          const double e = sqrt(exact_block(cc.i));
          if (lane == c) mine2 = e;
          ++nevals;
        }
        if (wave == 0 && lane < KC) exact[lane] = lane < c ? mine2 : __builtin_inf();
        __syncthreads();
        if (wave == 0) merge_run(false);
        __syncthreads();
      }
      if (deep_ran) {   // the final sort takes the best KC re-ranked, the certificate the last round's bound
        if (wave == 0 && lane < KC) {
          lists[lane] = run_l[lane];
          exact[lane] = run_e[lane];
        }
        tk_deep = dtk;
      }
    }
  }
  __syncthreads();
  if (wave == 0) {
    double* od = p.out_d + q * p.k;
    int64_t* oi = p.out_i + q * p.k;
    const double dk = sort_and_write_wave<KC>(lists, exact, p.k, p.index_base, od, oi);
    if (p.evals && lane == 0) p.evals[q] = nevals;
    if (lane != 0) return;
    // certificate.  Every row outside the KC candidates has coarse score >= tau, hence exact
    // score S = d^2 - |q|^2 >= tau - dS, i.e. d^2 >= bound = tau - dS + |q|^2 (less a relative
    // 1e-12 for the fp64 evaluation); the local top-k is exact iff d_k^2 < bound.  tau = the
    // 16th key (none when every gallery row is a candidate), with the sieve min(theta, 16th).
    // A sharded search compares the GLOBAL k-th with every rank's bound instead (parallel.py).
    uint32_t tk = lists[KC - 1].i != CAND_EMPTY ? score_key(lists[KC - 1].d, 0) : KEY_NONE;
    if (p.theta) tk = umin(tk, p.theta[q]);
    if (deep_ran) tk = tk_deep;
    double bnd = __builtin_inf();
    if (overflow) bnd = -__builtin_inf();   // the bucket dropped kept rows: no bound
    else if (tk != KEY_NONE) bnd = d2_lower((double)key_score(tk));
    p.cert[q] = (dk == dk) && (dk * dk < bnd);
    if (p.bound) p.bound[q] = bnd;
  }
}

// ---- quantization of fp32 rows ----------------------------------------------------------
// SL = 1: x~ = s x1, row layout plain [ld];  SL = 2: x~ = s (x1 + 2^-7 x2), per 64
// features 64 bytes of x1 then 64 bytes of x2 (one 128-B line).
template <int SL>
__global__ void __launch_bounds__(256) quantize_kernel(const float* X, int64_t ldx, int64_t d, int8_t* Xs,
                                                       int64_t ld, float* scale, double* stats) {
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
  int8_t* o = Xs + row * ld;
  const int64_t dk = ld / SL;
  for (int64_t i = threadIdx.x; i < dk; i += blockDim.x) {
    int v1 = 0, v2 = 0;
    if (i < d) {
      const double xv = (double)x[i];
      const double r = xv / s;                // exact (power of two)
      const double f1 = rint(r);
      const double f2 = SL == 2 ? rint((r - f1) * 128.0) : 0.0;
      v1 = (int)f1;
      v2 = (int)f2;
      const double xt = s * (f1 + f2 * 0x1p-7);  // exact
      sa += xt * xt;
      se += (xv - xt) * (xv - xt);
      st += f2 * f2;
    }
    if constexpr (SL == 1) {
      o[i] = (int8_t)v1;
    } else {
      const int64_t at = (i >> 6) * 128 + (i & 63);
      o[at] = (int8_t)v1;
      o[at + 64] = (int8_t)v2;
    }
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

// fp6 tier: x~ = s v, v in e2m3 (|v| <= 7.5: m/8 below 2, steps 1/4 in [2,4), 1/2 in [4,7.5]),
// s = max|x| / 7.5 as an fp32 number (any real scale is allowed: it is applied in the
// epilogue, not by the MFMA), rounded up so that every |x|/s <= 7.5.  One block per row;
// thread t writes the 24 bytes of the 32-feature groups g = t, t + 256, ... into the f6
// tiled layout (ofr_f6_tile.h).  stats as quantize_kernel (third = 0).
__device__ __forceinline__ uint32_t e2m3_code(double r, double& q) {
  const double a = fabs(r);
  double v;
  if (a < 2.0) v = rint(a * 8.0) * 0.125;
  else if (a < 4.0) v = rint(a * 4.0) * 0.25;
  else v = rint(a * 2.0) * 0.5;
  uint32_t code;
  if (v < 1.0) code = (uint32_t)(v * 8.0);
  else {
    const int e = v < 2.0 ? 1 : (v < 4.0 ? 2 : 3);
    const double inv = e == 1 ? 1.0 : (e == 2 ? 0.5 : 0.25);   // 2^-(e-1), exact
    code = ((uint32_t)e << 3) | (uint32_t)((v * inv - 1.0) * 8.0);
  }
  q = r < 0 ? -v : v;
  return (r < 0 && v != 0.0) ? (code | 32u) : code;
}

// X2: also the second slice of the two-slice tier f6x2, x~ = s (v1 + 2^-4 v2) with v2 = e2m3 of
// 2^4 (x/s - v1) (|x/s - v1| <= 1/4, so |2^4 (x/s - v1)| <= 4 < 7.5), written to tiles2 in the same
// layout; tiles (the first slice) may then be null -- a gallery's f6 tier already holds it, the same
// bytes and scale.  Stats of f6x2: a = s (|v1| + 2^-4 |v2|) >= |x~| (it also bounds the sum of
// |products| the fp32 accumulation error is proportional to), e = |x - x~|, t = s 2^-4 |v2| (the
// dropped 2^-8 x2.y2 term is at most t_q t_g).
//
// Column-block scales (bscale, null: unit; ofr_f6_block_scales): feature k of every row is quantized
// as x / 2^e with e = bscale[k / 32] - 127, so the row scale s = max_k |x_k| / 2^e_k / 7.5 and
// x~_k = s 2^e_k v_k (the MFMA applies 2^e_k to both operands of block k / 32).  The stats are of x~
// in the original coordinates: a = ||x~||, e = ||x - x~|| (f6x2: a = s (||v1||' + 2^-4 ||v2||') with
// ||v||' = (sum_k 2^2e_k v_k^2)^1/2 -- it bounds ||x~|| and the sum of |products| alike, t likewise).
template <bool X2>
__global__ void __launch_bounds__(256) quantize_f6_kernel(const float* X, int64_t ldx, int64_t d, int64_t nst,
                                                          int64_t row0, char* tiles, float* scale, double* stats,
                                                          char* tiles2, const uint8_t* bscale, int64_t nsw,
                                                          int pow2) {
  __shared__ float redf[4];
  __shared__ double red[4][3];
  const int64_t row = row0 + blockIdx.x;   // destination row (X row blockIdx.x)
  const float* x = X + (int64_t)blockIdx.x * ldx;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // 2^-e_B, exact (e_B in [-63, 0]: a normal power of two)
  auto binv = [&](int64_t g) { return bscale ? __builtin_ldexpf(1.0f, 127 - (int)bscale[g]) : 1.0f; };
  float mx = 0.f;
  for (int64_t i = threadIdx.x; i < d; i += blockDim.x) mx = fmaxf(mx, fabsf(x[i]) * binv(i >> 5));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) redf[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(redf[0], redf[1]), fmaxf(redf[2], redf[3]));
  float s = 1.0f;
  if (pow2) {   // s = 2^e, the least with mx / s <= 7.5, e in [-64, 64] (the prefix pass folds e into the MFMA)
    int e = 0;
    if (mx > 0.f) {
      const double m = __builtin_frexp((double)mx / 7.5, &e);   // mx / 7.5 = m 2^e, m in [0.5, 1)
      if (m == 0.5) --e;
      e = e < -64 ? -64 : (e > 64 ? 64 : e);
    }
    s = __builtin_ldexpf(1.0f, e);
  } else if (mx > 0.f) {
    s = (float)((double)mx / 7.5);
    while ((double)mx / (double)s > 7.5) s = __uint_as_float(__float_as_uint(s) + 1u);
  }
  const double sd = (double)s;
  const double inv_sd = 1.0 / sd;   // x * (1/s) instead of x / s: any rounding of x/s is fine (the
                                    // stats below are of the values actually stored)
  const bool vec4 = ((ldx & 3) == 0) && (((uintptr_t)X & 15) == 0);
  double sa = 0, se = 0, s2 = 0;
  const int64_t ngroups = nsw * 4;   // the stages written: all nst, or a prefix (ofr_f6_quantize_rows_prefix)
  const int64_t poff = (row >> 8) * nst * (int64_t)f6t::PANEL;
  const int rl = (int)(row & 255);
  for (int64_t g = threadIdx.x; g < ngroups; g += blockDim.x) {
    uint32_t w[6] = {0, 0, 0, 0, 0, 0}, w2[6] = {0, 0, 0, 0, 0, 0};
    // this 32-feature group is column block g: x / (s 2^e) and s 2^e v, both exact power-of-two rescalings
    const double bi = (double)binv(g), bs = 1.0 / bi;
    const double inv_b = inv_sd * bi, sd_b = sd * bs;
    float xg[32];
    if (vec4 && g * 32 + 32 <= d) {
#pragma unroll
      for (int e = 0; e < 32; e += 4) {
        const float4 v4 = *reinterpret_cast<const float4*>(x + g * 32 + e);
        xg[e] = v4.x; xg[e + 1] = v4.y; xg[e + 2] = v4.z; xg[e + 3] = v4.w;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 32; ++e) xg[e] = g * 32 + e < d ? x[g * 32 + e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      const int64_t k = g * 32 + e;
      if (k < d) {
        const double xv = (double)xg[e];
        double qv;
        const uint32_t c = e2m3_code(xv * inv_b, qv);
        double xt = sd_b * qv;   // exact: 24-bit s times a 4-bit significand and a power of two
        const int bit = 6 * e;
        if constexpr (X2) {
          double qv2;
          const uint32_t c2 = e2m3_code((xv - xt) * inv_b * 16.0, qv2);
          sa += bs * bs * qv * qv;
          s2 += bs * bs * qv2 * qv2;
          xt += sd_b * qv2 * 0.0625;   // exact (a 28-bit significand at most)
          w2[bit >> 5] |= c2 << (bit & 31);
          if ((bit & 31) > 26) w2[(bit >> 5) + 1] |= c2 >> (32 - (bit & 31));
        } else {
          sa += xt * xt;
        }
        se += (xv - xt) * (xv - xt);
        w[bit >> 5] |= c << (bit & 31);
        if ((bit & 31) > 26) w[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
      }
    }
    const int64_t st = g >> 2;
    const int jh = (int)(g & 3);   // 2 j + h
    const int64_t off = poff + st * f6t::PANEL + jh * 6144;
    if (tiles) {
      *reinterpret_cast<uint4*>(tiles + off + rl * 16) = make_uint4(w[0], w[1], w[2], w[3]);
      *reinterpret_cast<uint2*>(tiles + off + 4096 + f6t::p1_slot(jh, rl) * 8) = make_uint2(w[4], w[5]);
    }
    if constexpr (X2) {
      *reinterpret_cast<uint4*>(tiles2 + off + rl * 16) = make_uint4(w2[0], w2[1], w2[2], w2[3]);
      *reinterpret_cast<uint2*>(tiles2 + off + 4096 + f6t::p1_slot(jh, rl) * 8) = make_uint2(w2[4], w2[5]);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sa += __shfl_xor(sa, o);
    se += __shfl_xor(se, o);
    s2 += __shfl_xor(s2, o);
  }
  if (lane == 0) {
    red[wave][0] = sa;
    red[wave][1] = se;
    red[wave][2] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double A = red[0][0] + red[1][0] + red[2][0] + red[3][0];
    const double E = red[0][1] + red[1][1] + red[2][1] + red[3][1];
    const double S2 = red[0][2] + red[1][2] + red[2][2] + red[3][2];
    scale[row] = s;
    // norms rounded up a hair so that fp64 summation error never shrinks the bound
    if constexpr (X2) {
      stats[row * 3 + 0] = sd * (sqrt(A) + 0.0625 * sqrt(S2)) * (1.0 + 1e-12);
      stats[row * 3 + 1] = sqrt(E) * (1.0 + 1e-12);
      stats[row * 3 + 2] = sd * 0.0625 * sqrt(S2) * (1.0 + 1e-12);
    } else {
      stats[row * 3 + 0] = sqrt(A) * (1.0 + 1e-12);
      stats[row * 3 + 1] = sqrt(E) * (1.0 + 1e-12);
      stats[row * 3 + 2] = 0.0;
    }
  }
}

// saux[j] = aux[j * step] for j in [j0, j1) (the row sample's aux terms)
__global__ void sample_aux_kernel(const float* aux, int64_t j0, int64_t j1, int64_t step, float* saux) {
  const int64_t j = j0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j < j1) saux[j] = aux[j * step];
}

// zero rows of the last panel past R (they are never selected: the epilogue masks rows >= N)
__global__ void f6_zero_tail(char* tiles, int64_t R, int64_t nst) {
  const int64_t p = R >> 8;
  const int r0 = (int)(R & 255);
  char* pbase = tiles + p * nst * (int64_t)f6t::PANEL;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nst * 4 * (256 - r0);
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t sjh = i / (256 - r0);
    const int rl = r0 + (int)(i % (256 - r0));
    char* sb = pbase + (sjh >> 2) * f6t::PANEL + (sjh & 3) * 6144;
    *reinterpret_cast<uint4*>(sb + rl * 16) = make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint2*>(sb + 4096 + f6t::p1_slot((int)(sjh & 3), rl) * 8) = make_uint2(0, 0);
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

// Column-block statistics of the fp6 tiers (ofr_f6_block_sumsq): sums[b] += sum over the rows of
// x_k^2 for the 32 features k of block b (fp64 atomics, one per block and workgroup).
__global__ void __launch_bounds__(256) block_sumsq_kernel(const float* X, int64_t R, int64_t d, int64_t ldx,
                                                          int64_t rows_per_wg, double* sums) {
  const int64_t nb = (d + 31) / 32;
  const int64_t r0 = blockIdx.y * rows_per_wg, r1 = r0 + rows_per_wg < R ? r0 + rows_per_wg : R;
  for (int64_t b = blockIdx.x * 8 + (threadIdx.x >> 5); b < nb && b < (int64_t)(blockIdx.x + 1) * 8; b += 8) {
    const int64_t k = b * 32 + (threadIdx.x & 31);
    double acc = 0.0;
    if (k < d)
      for (int64_t r = r0; r < r1; ++r) {
        const double v = (double)X[r * ldx + k];
        acc += v * v;
      }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 32);
    if ((threadIdx.x & 31) == 0) atomicAdd(sums + b, acc);
  }
}

// sums[nb] -> E8M0 bytes [4 nst]: e_b = rint(log2(rms_b / rms_max)) clamped to [-63, 0] (block 0 of the
// largest mean square gets 2^0), 127 (2^0) for empty blocks and the padding blocks past d.
__global__ void __launch_bounds__(256) block_scales_kernel(const double* sums, int64_t nb, int64_t npad,
                                                           uint8_t* bscale) {
  __shared__ double red[4];
  double m = 0.0;
  for (int64_t b = threadIdx.x; b < nb; b += blockDim.x) m = fmax(m, sums[b]);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
  if (lane == 0) red[wave] = m;
  __syncthreads();
  m = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  for (int64_t b = threadIdx.x; b < npad; b += blockDim.x) {
    int e = 0;
    if (b < nb && sums[b] > 0.0 && m > 0.0) {
      const double l = 0.5 * log2(sums[b] / m);
      e = (int)rint(l);
      e = e < -63 ? -63 : (e > 0 ? 0 : e);
    }
    bscale[b] = (uint8_t)(127 + e);
  }
}

// Unit column-block scales (E8M0 2^0 in every byte) for callers that pass none: the engines always
// load a stage's dword (one code path), from this table when bscale is null.
constexpr int UNIT_BS_STAGES = 4096;   // d <= 524,288 without a caller table
struct UnitScales {
  uint32_t v[UNIT_BS_STAGES];
  constexpr UnitScales() : v() {
    for (int i = 0; i < UNIT_BS_STAGES; ++i) v[i] = 0x7f7f7f7fu;
  }
};
__device__ UnitScales unit_bs_table = UnitScales();

}  // namespace q8s
}  // namespace ofr

using namespace ofr;

// the unit table's address on the current device (a __device__ variable exists once per device)
static const uint32_t* unit_bscale() {
  static const uint32_t* addr[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!addr[dev]) {
    void* a = nullptr;
    if (hipGetSymbolAddress(&a, HIP_SYMBOL(q8s::unit_bs_table)) != hipSuccess) return nullptr;
    addr[dev] = (const uint32_t*)a;
  }
  return addr[dev];
}

// compute units of the current device (the persistent prefix pass runs one workgroup on each)
static int device_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 0;
  return cus[dev];
}

// query panels per work item of tile_kernel_f6p: the largest group (fewest gallery-tile loads) whose
// last round of items over the CUs wastes little -- the makespan in panels, ceil(items / cus) x qg,
// plus half a panel per item for its gallery copies and tables, is minimal
static int64_t f6p_group(int64_t ntg, int64_t ntq, int cus) {
  if (const char* e = getenv("OFR_F6P_GROUP")) {   // probe override
    const int64_t v = atoll(e);
    if (v >= 1) return v < ntq ? v : ntq;
  }
  int64_t best = ntq, cost = INT64_MAX;
  for (int64_t div = 1; div <= ntq; div *= 2) {
    const int64_t qg = (ntq + div - 1) / div, items = ntg * ((ntq + qg - 1) / qg);
    const int64_t rounds = (items + cus - 1) / cus, c = rounds * (2 * qg + 1);
    if (c < cost) {
      cost = c;
      best = qg;
    }
  }
  return best;
}

// query steps per work item of the wave-decoupled prefix pass: the largest ceil(ntq / 2^j) that deals
// every workgroup about 24 items or more, but 8 steps at least.  Swept at B = 4,096 on galleries of one
// rank's share at G = 1/2/4/8 (profiles/r06_prefix_group_ab.txt): the best step counts were 16 / 8-16 / 8 /
// 4-8; one item per workgroup (64 steps at N = 125k) measured 3x slower (0.45 vs 0.15 ms).
static int64_t f6p_group_wave(int64_t ntg, int64_t ntq, int slots, int per_wg) {
  if (const char* e = getenv("OFR_F6P_GROUP")) {   // probe override
    const int64_t v = atoll(e);
    if (v >= 1) return v < ntq ? v : ntq;
  }
  int64_t qg = ntq;
  for (int64_t div = 1; div <= ntq; div *= 2) {
    qg = (ntq + div - 1) / div;
    if (ntg * ((ntq + qg - 1) / qg) >= per_wg * (int64_t)slots || qg <= 8) break;
  }
  return qg;
}

static int64_t q8_min_ld(int slices, int64_t d) { return slices == 1 ? round_up(d, 128) : 2 * round_up(d, 64); }

extern "C" int ofr_q8_quantize_rows(void* stream, int slices, const float* X, int64_t R, int64_t d, int64_t ldx,
                                    int8_t* Xs, int64_t ld, float* scale, double* stats, const float* aux,
                                    double* maxima) {
  OFR_CHECK_ARG(slices == 1 || slices == 2, "ofr_q8_quantize_rows: slices must be 1 or 2");
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d && ld >= q8_min_ld(slices, d) && ld % 128 == 0,
                "ofr_q8_quantize_rows: bad sizes (ld: multiple of 128, >= round_up(d,128) for 1 slice, "
                ">= 2 round_up(d,64) for 2)");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && Xs && scale && stats, "ofr_q8_quantize_rows: null pointer");
  OFR_CHECK_ARG(R < 0x7fffffffLL, "ofr_q8_quantize_rows: too many rows");
  hipStream_t st = (hipStream_t)stream;
  if (slices == 1)
    hipLaunchKernelGGL(q8s::quantize_kernel<1>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, d, Xs, ld, scale, stats);
  else
    hipLaunchKernelGGL(q8s::quantize_kernel<2>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, d, Xs, ld, scale, stats);
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

template <int SL>
static int q8_tiles(hipStream_t st, q8s::TileArgs a) {
  using S = q8s::Shape<SL>;
  static bool attr_done = false;
  if (!attr_done) {
    hipError_t e = hipFuncSetAttribute((const void*)q8s::tile_kernel<SL>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS);
    if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(q8 tile)");
    attr_done = true;
  }
  hipLaunchKernelGGL((q8s::tile_kernel<SL>), dim3((unsigned)(a.ntq * a.ntg)), dim3(S::NT), S::LDS, st, a);
  OFR_LAUNCH_CHECK("q8 tile_kernel");
  return OFR_OK;
}

// the merge's re-rank form (OFR_MERGE_ENGINE: 1 = one wave per candidate, four per round, probe;
// default the block-cooperative form)
template <bool SMALL>
static void launch_merge(hipStream_t st, const q8s::MergeArgs& m) {
  const char* e = getenv("OFR_MERGE_ENGINE");
  if (e && e[0] == '1') {
    hipLaunchKernelGGL((q8s::merge_kernel<SMALL, false>), dim3((unsigned)m.B), dim3(256), 0, st, m);
    return;
  }
  hipLaunchKernelGGL((q8s::merge_kernel<SMALL, true>), dim3((unsigned)m.B), dim3(256), 0, st, m);
  if constexpr (SMALL) {   // the deep continuation of what the plain merge left open (sieve buckets)
    if (m.deep > 0 && m.mode == 0 && m.count && m.theta)
      hipLaunchKernelGGL((q8s::merge_kernel<true, true, true>), dim3((unsigned)m.B), dim3(256), 0, st, m);
  }
}

extern "C" int ofr_knn_q8(void* stream, int phases, int slices, const float* Q, int64_t B, int64_t ldq,
                          const int8_t* Qs, const float* qscale, const double* qstats, const float* G, int64_t N,
                          int64_t ldg, int64_t d, const int8_t* Gs, int64_t ld, const float* gscale,
                          const float* aux, const double* gmax, int k, int64_t index_base, double* out_d,
                          int64_t* out_i, int* cert, double* bound, void* workspace, size_t workspace_bytes) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 3, "ofr_knn_q8: phases must be 1 (tiles), 2 (merge) or 3");
  OFR_CHECK_ARG(slices == 1 || slices == 2, "ofr_knn_q8: slices must be 1 or 2");
  OFR_CHECK_ARG(B >= 0 && N >= 1 && d >= 1, "ofr_knn_q8: bad sizes (empty galleries use ofr_knn_f32)");
  if (k < 1 || k > q8s::KC) return fail(OFR_E_UNSUPPORTED, "ofr_knn_q8: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(ld % 128 == 0 && ld >= q8_min_ld(slices, d), "ofr_knn_q8: bad slice leading dimension");
  OFR_CHECK_ARG(ldq >= d && ldg >= d, "ofr_knn_q8: bad leading dimensions");
  OFR_CHECK_ARG(Q && Qs && qscale && qstats && G && Gs && gscale && aux && gmax && workspace,
                "ofr_knn_q8: null pointer");
  OFR_CHECK_ARG(((uintptr_t)Qs | (uintptr_t)Gs) % 16 == 0, "ofr_knn_q8: slices must be 16-byte aligned");
  OFR_CHECK_ARG(N < 0x7fffffffLL - q8s::TG, "ofr_knn_q8: N too large for one shard");
  OFR_CHECK_ARG(workspace_bytes >= ofr_knn_q8_workspace_bytes(B, N), "ofr_knn_q8: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  q8s::TileArgs a{};
  a.G = Gs; a.N = N; a.ld = ld; a.gscale = gscale; a.aux = aux;
  a.Q = Qs; a.B = B; a.qscale = qscale;
  a.nk = (int)cdiv(d, slices == 1 ? q8s::Shape<1>::BK : q8s::Shape<2>::BK);
  a.cand = reinterpret_cast<Cand*>(workspace);
  a.ntq = cdiv(B, slices == 1 ? q8s::Shape<1>::TQ : q8s::Shape<2>::TQ);
  a.ntg = cdiv(N, q8s::TG);
  a.gg = a.ntg < q8s::GROUP_G ? a.ntg : q8s::GROUP_G;
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_knn_q8: grid too large");
  if (phases & 1) {
    const int rc = slices == 1 ? q8_tiles<1>(st, a) : q8_tiles<2>(st, a);
    if (rc) return rc;
  }
  if (phases & 2) {
    OFR_CHECK_ARG(out_d && out_i && cert, "ofr_knn_q8: null output");
    q8s::MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, d, qstats, gmax, 0.0, k, index_base, out_d, out_i, cert, bound};
    launch_merge<false>(st, m);
    OFR_LAUNCH_CHECK("q8 merge_kernel");
  }
  return OFR_OK;
}

/* ---- fp6 tier ------------------------------------------------------------------------- */

extern "C" size_t ofr_f6_tiles_bytes(int64_t R, int64_t d) {
  return R <= 0 || d <= 0 ? 0 : (size_t)f6t::tiles_bytes(R, d);
}

// bscale (null: unit) must be 4-byte aligned and hold 4 * ceil(d / 128) bytes (ofr_f6_block_scales)
static bool bscale_ok(const uint8_t* bscale) { return ((uintptr_t)bscale & 3) == 0; }

extern "C" int ofr_f6_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx,
                                       int64_t row0, void* tiles, size_t tiles_bytes, float* scale, double* stats,
                                       const uint8_t* bscale) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d && row0 >= 0, "ofr_f6_quantize_rows_at: bad sizes");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && tiles && scale && stats, "ofr_f6_quantize_rows_at: null pointer");
  OFR_CHECK_ARG(row0 + R < 0x7fffffffLL, "ofr_f6_quantize_rows_at: too many rows");
  OFR_CHECK_ARG(tiles_bytes >= ofr_f6_tiles_bytes(row0 + R, d), "ofr_f6_quantize_rows_at: tile buffer too small");
  OFR_CHECK_ARG((uintptr_t)tiles % 16 == 0, "ofr_f6_quantize_rows_at: tiles must be 16-byte aligned");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_f6_quantize_rows_at: bscale must be 4-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nst = f6t::stages(d);
  hipLaunchKernelGGL(q8s::quantize_f6_kernel<false>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, d, nst, row0,
                     (char*)tiles, scale, stats, nullptr, bscale, nst, 0);
  OFR_LAUNCH_CHECK("f6 quantize_kernel");
  const int64_t end = row0 + R;
  if (end % 256) {
    hipLaunchKernelGGL(q8s::f6_zero_tail, dim3(256), dim3(256), 0, st, (char*)tiles, end, nst);
    OFR_LAUNCH_CHECK("f6 zero_tail");
  }
  return OFR_OK;
}

extern "C" int ofr_f6x2_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx,
                                         int64_t row0, void* tiles1, void* tiles2, size_t tiles_bytes, float* scale,
                                         double* stats, const uint8_t* bscale) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d && row0 >= 0, "ofr_f6x2_quantize_rows_at: bad sizes");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && tiles2 && scale && stats, "ofr_f6x2_quantize_rows_at: null pointer");
  OFR_CHECK_ARG(row0 + R < 0x7fffffffLL, "ofr_f6x2_quantize_rows_at: too many rows");
  OFR_CHECK_ARG(tiles_bytes >= ofr_f6_tiles_bytes(row0 + R, d), "ofr_f6x2_quantize_rows_at: tile buffer too small");
  OFR_CHECK_ARG(((uintptr_t)tiles1 | (uintptr_t)tiles2) % 16 == 0,
                "ofr_f6x2_quantize_rows_at: tiles must be 16-byte aligned");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_f6x2_quantize_rows_at: bscale must be 4-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nst = f6t::stages(d);
  hipLaunchKernelGGL(q8s::quantize_f6_kernel<true>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, d, nst, row0,
                     (char*)tiles1, scale, stats, (char*)tiles2, bscale, nst, 0);
  OFR_LAUNCH_CHECK("f6x2 quantize_kernel");
  const int64_t end = row0 + R;
  if (end % 256) {
    for (void* t : {tiles1, tiles2}) {
      if (!t) continue;
      hipLaunchKernelGGL(q8s::f6_zero_tail, dim3(256), dim3(256), 0, st, (char*)t, end, nst);
      OFR_LAUNCH_CHECK("f6x2 zero_tail");
    }
  }
  return OFR_OK;
}

// The prefix tier's query rows: only the first pstages stages of each row's tiles are written (the
// prefix pass reads no others), from the first min(d, 128 pstages) features -- their own row scale and
// stats (a, e of the prefix: the prefix scores' error bound needs no more; the full tier re-quantizes).
extern "C" int ofr_f6_quantize_rows_prefix(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx,
                                           int pstages, void* tiles, size_t tiles_bytes, float* scale,
                                           double* stats, const uint8_t* bscale) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d, "ofr_f6_quantize_rows_prefix: bad sizes");
  OFR_CHECK_ARG(pstages >= 1 && pstages <= f6t::stages(d), "ofr_f6_quantize_rows_prefix: pstages in [1, ceil(d / 128)]");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && tiles && scale && stats, "ofr_f6_quantize_rows_prefix: null pointer");
  OFR_CHECK_ARG(R < 0x7fffffffLL, "ofr_f6_quantize_rows_prefix: too many rows");
  OFR_CHECK_ARG(tiles_bytes >= ofr_f6_tiles_bytes(R, d), "ofr_f6_quantize_rows_prefix: tile buffer too small");
  OFR_CHECK_ARG((uintptr_t)tiles % 16 == 0, "ofr_f6_quantize_rows_prefix: tiles must be 16-byte aligned");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_f6_quantize_rows_prefix: bscale must be 4-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t nst = f6t::stages(d), dm = std::min<int64_t>(d, (int64_t)pstages * f6t::BK);
  hipLaunchKernelGGL(q8s::quantize_f6_kernel<false>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, dm, nst, (int64_t)0,
                     (char*)tiles, scale, stats, nullptr, bscale, (int64_t)pstages, 1);
  OFR_LAUNCH_CHECK("f6 quantize_kernel (prefix)");
  if (R % 256) {
    hipLaunchKernelGGL(q8s::f6_zero_tail, dim3(256), dim3(256), 0, st, (char*)tiles, R, nst);
    OFR_LAUNCH_CHECK("f6 zero_tail");
  }
  return OFR_OK;
}

// The prefix tier's own gallery tiles (round 6): the first pstages 128-feature stages of each row in the
// f6 tiled layout of pstages stages per panel (ofr_f6p_tiles_bytes), quantized from the first
// dm = min(d, 128 pstages) features with a POWER-OF-TWO row scale s = 2^e (the least with max|x_k / 2^e_k|
// <= 7.5 s) and their prefix stats (a = ||x~_m||, e = ||x_m - x~_m||).  A power-of-two s is exact in the
// MFMA's E8M0 operand scale, so the prefix pass folds 2 s_g into the gallery operand and -|g_m|^2 into the
// accumulator input: its output IS the negated coarse score (prefix_pass_kernel<true>).  The f6 tiers keep
// their fp32 row scales (a finer cut of the full rows).
extern "C" size_t ofr_f6p_tiles_bytes(int64_t R, int pstages) {
  return pstages >= 1 ? (size_t)f6t::panels(R > 0 ? R : 1) * (size_t)pstages * (size_t)f6t::PANEL : 0;
}

extern "C" int ofr_f6p_quantize_rows_at(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int64_t row0,
                                        int pstages, void* tiles, size_t tiles_bytes, float* scale, double* stats,
                                        const uint8_t* bscale) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d && row0 >= 0, "ofr_f6p_quantize_rows_at: bad sizes");
  OFR_CHECK_ARG(pstages >= 1 && pstages <= f6t::stages(d), "ofr_f6p_quantize_rows_at: pstages in [1, ceil(d / 128)]");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && tiles && scale && stats, "ofr_f6p_quantize_rows_at: null pointer");
  OFR_CHECK_ARG(row0 + R < 0x7fffffffLL, "ofr_f6p_quantize_rows_at: too many rows");
  OFR_CHECK_ARG(tiles_bytes >= ofr_f6p_tiles_bytes(row0 + R, pstages), "ofr_f6p_quantize_rows_at: tile buffer too small");
  OFR_CHECK_ARG((uintptr_t)tiles % 16 == 0, "ofr_f6p_quantize_rows_at: tiles must be 16-byte aligned");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_f6p_quantize_rows_at: bscale must be 4-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  const int64_t dm = std::min<int64_t>(d, (int64_t)pstages * f6t::BK);
  hipLaunchKernelGGL(q8s::quantize_f6_kernel<false>, dim3((unsigned)R), dim3(256), 0, st, X, ldx, dm, (int64_t)pstages,
                     row0, (char*)tiles, scale, stats, nullptr, bscale, (int64_t)pstages, 1);
  OFR_LAUNCH_CHECK("f6p quantize_kernel (gallery)");
  const int64_t end = row0 + R;
  if (end % 256) {
    hipLaunchKernelGGL(q8s::f6_zero_tail, dim3(256), dim3(256), 0, st, (char*)tiles, end, (int64_t)pstages);
    OFR_LAUNCH_CHECK("f6 zero_tail");
  }
  return OFR_OK;
}

extern "C" int ofr_q8_maxima(void* stream, const double* stats, const float* aux, int64_t R, double* maxima) {
  OFR_CHECK_ARG(R >= 0 && stats && maxima, "ofr_q8_maxima: bad arguments");
  hipLaunchKernelGGL(q8s::maxima_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, stats, aux, R, maxima);
  OFR_LAUNCH_CHECK("q8 maxima_kernel");
  return OFR_OK;
}

extern "C" int ofr_f6_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, void* tiles,
                                    size_t tiles_bytes, float* scale, double* stats, const float* aux,
                                    double* maxima, const uint8_t* bscale) {
  const int rc = ofr_f6_quantize_rows_at(stream, X, R, d, ldx, 0, tiles, tiles_bytes, scale, stats, bscale);
  if (rc || R == 0 || !maxima) return rc;
  return ofr_q8_maxima(stream, stats, aux, R, maxima);
}

// ofr_f6p_quantize_rows_at from row 0, then the maxima of the prefix stats and of the prefix terms
// paux (|g_m|^2, ofr_row_aux over the first min(d, 128 pstages) features): the f6p tier's gmax
extern "C" int ofr_f6p_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, int pstages,
                                     void* tiles, size_t tiles_bytes, float* scale, double* stats, const float* paux,
                                     double* maxima, const uint8_t* bscale) {
  const int rc = ofr_f6p_quantize_rows_at(stream, X, R, d, ldx, 0, pstages, tiles, tiles_bytes, scale, stats, bscale);
  if (rc || R == 0 || !maxima) return rc;
  return ofr_q8_maxima(stream, stats, paux, R, maxima);
}

extern "C" int ofr_f6x2_quantize_rows(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, void* tiles1,
                                      void* tiles2, size_t tiles_bytes, float* scale, double* stats, const float* aux,
                                      double* maxima, const uint8_t* bscale) {
  const int rc = ofr_f6x2_quantize_rows_at(stream, X, R, d, ldx, 0, tiles1, tiles2, tiles_bytes, scale, stats,
                                           bscale);
  if (rc || R == 0 || !maxima) return rc;
  return ofr_q8_maxima(stream, stats, aux, R, maxima);
}

extern "C" int64_t ofr_f6_sample_step(void) { return q8s::SAMPLE_STEP; }

extern "C" int ofr_f6_block_sumsq(void* stream, const float* X, int64_t R, int64_t d, int64_t ldx, double* sums) {
  OFR_CHECK_ARG(R >= 0 && d >= 1 && ldx >= d, "ofr_f6_block_sumsq: bad sizes");
  if (R == 0) return OFR_OK;
  OFR_CHECK_ARG(X && sums, "ofr_f6_block_sumsq: null pointer");
  const int64_t nb = cdiv(d, 32), rows = 4096;
  OFR_CHECK_ARG(cdiv(R, rows) < 65536, "ofr_f6_block_sumsq: too many rows for one call");
  hipLaunchKernelGGL(q8s::block_sumsq_kernel, dim3((unsigned)cdiv(nb, 8), (unsigned)cdiv(R, rows)), dim3(256), 0,
                     (hipStream_t)stream, X, R, d, ldx, rows, sums);
  OFR_LAUNCH_CHECK("f6 block_sumsq_kernel");
  return OFR_OK;
}

extern "C" int ofr_f6_block_scales(void* stream, const double* sums, int64_t d, uint8_t* bscale) {
  OFR_CHECK_ARG(d >= 1 && sums && bscale, "ofr_f6_block_scales: bad arguments");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_f6_block_scales: bscale must be 4-byte aligned");
  hipLaunchKernelGGL(q8s::block_scales_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, sums, cdiv(d, 32),
                     4 * f6t::stages(d), bscale);
  OFR_LAUNCH_CHECK("f6 block_scales_kernel");
  return OFR_OK;
}

extern "C" int ofr_f6x2_sample_rows(void* stream, const float* X, int64_t N, int64_t ldx, int64_t d, int64_t j0,
                                    int64_t j1, void* tiles2, size_t tiles_bytes, float* scale, double* stats,
                                    const uint8_t* bscale) {
  OFR_CHECK_ARG(j0 >= 0 && j1 >= j0 && d >= 1 && ldx >= d && N >= 0, "ofr_f6x2_sample_rows: bad sizes");
  OFR_CHECK_ARG(j1 <= cdiv(N, q8s::SAMPLE_STEP), "ofr_f6x2_sample_rows: j1 past the gallery's sample (ceil(N / 64))");
  if (j1 == j0) return OFR_OK;
  OFR_CHECK_ARG(X, "ofr_f6x2_sample_rows: null pointer");
  OFR_CHECK_ARG(ldx < INT64_MAX / q8s::SAMPLE_STEP, "ofr_f6x2_sample_rows: leading dimension too large");
  return ofr_f6x2_quantize_rows_at(stream, X + j0 * q8s::SAMPLE_STEP * ldx, j1 - j0, d, ldx * q8s::SAMPLE_STEP, j0,
                                   nullptr, tiles2, tiles_bytes, scale, stats, bscale);
}

extern "C" int ofr_f6_sample_rows(void* stream, const float* X, int64_t N, int64_t ldx, int64_t d, int64_t j0,
                                  int64_t j1, const float* aux, void* tiles, size_t tiles_bytes, float* scale,
                                  double* stats, float* saux, const uint8_t* bscale) {
  OFR_CHECK_ARG(j0 >= 0 && j1 >= j0 && d >= 1 && ldx >= d && N >= 0, "ofr_f6_sample_rows: bad sizes");
  OFR_CHECK_ARG(j1 <= cdiv(N, q8s::SAMPLE_STEP), "ofr_f6_sample_rows: j1 past the gallery's sample (ceil(N / 64))");
  if (j1 == j0) return OFR_OK;
  OFR_CHECK_ARG(X && aux && saux, "ofr_f6_sample_rows: null pointer");
  OFR_CHECK_ARG(ldx < INT64_MAX / q8s::SAMPLE_STEP, "ofr_f6_sample_rows: leading dimension too large");
  const int rc = ofr_f6_quantize_rows_at(stream, X + j0 * q8s::SAMPLE_STEP * ldx, j1 - j0, d,
                                         ldx * q8s::SAMPLE_STEP, j0, tiles, tiles_bytes, scale, stats, bscale);
  if (rc) return rc;
  hipLaunchKernelGGL(q8s::sample_aux_kernel, dim3((unsigned)cdiv(j1 - j0, 256)), dim3(256), 0, (hipStream_t)stream,
                     aux, j0, j1, q8s::SAMPLE_STEP, saux);
  OFR_LAUNCH_CHECK("f6 sample_aux_kernel");
  return OFR_OK;
}

// waves of the sample pass's fp6 engine (f6t::Engine<8>, 32x32x64 MFMA)
constexpr int F6_NW = 8;

// name of the fp6 sieve kernel ofr_knn_f6 launches for B > 32, as rocprofv3 reports it (bench.py
// labels its roofline entry with it, so the record names the variant that actually ran)
static int f6_shape();
extern "C" const char* ofr_f6_sieve_kernel(void) {
  static const std::string names[2] = {
      "q8s::tile_kernel_f6s<1> (16x16x128 fp6 engine, 256x256 tiles, 8 waves)",
      "q8s::tile_kernel_f6w<1> (16x16x128 fp6 engine, 384x256 tiles, 1 wave per SIMD)"};
  return names[f6_shape() == 16 ? 0 : 1].c_str();
}

// name of the kernel the prefix tier's sieve pass (ofr_knn_f6p_sampled, B > 32) launches for pstages
static bool f6p_persistent();
static int f6p_engine();
extern "C" const char* ofr_f6p_sieve_kernel(int pstages) {
  static const std::string names[4] = {
      "q8s::tile_kernel_f6p (persistent prefix pass: one workgroup per CU, 384-row gallery tile resident in LDS, "
      "16x16x128 fp6 MFMA)",
      "q8s::prefix_pass_kernel<false> (persistent one-stage prefix pass: two workgroups per CU, 64 x 128 wave tiles, "
      "16x16x128 fp6 MFMA)",
      "q8s::prefix_pass_kernel<true> (persistent one-stage prefix pass: two workgroups per CU, 64 x 128 wave tiles, "
      "16x16x128 fp6 MFMA with the row scales and -|g_m|^2 folded in: D = -score)",
      "q8s::prefix_wave_kernel (persistent one-stage prefix pass, waves decoupled: 128 x 32 wave steps, query "
      "fragments straight from L2, no barriers; 16x16x128 fp6 MFMA with the row scales and -|g_m|^2 folded in)"};
  if (pstages == 1 && f6_shape() == 384 && f6p_persistent() && f6p_engine() >= 2)
    return names[f6p_engine() - 1].c_str();
  if (pstages >= 1 && pstages <= q8s::f6p::NSPMAX && f6_shape() == 384 && f6p_persistent())
    return names[0].c_str();
  return ofr_f6_sieve_kernel();
}

// Engine of the sieve pass: 384 = v_mfma_scale_f32_16x16x128 on 384 x 256 tiles, one wave per SIMD
// (f6t::EngineW, default since round 3: 22.2 -> 20.1 ms); 16 = the same MFMA on 256 x 256 tiles, 8
// waves (f6t::Engine16, OFR_F6_SHAPE=16: the comparison engine of tests/test_gpu_sieve.py).  Read at
// every call (the workspace does not depend on it), so a test can run both sieve engines in one
// process; any other value is an error (-1), not a silent default.
static int f6_shape() {
  const char* e = getenv("OFR_F6_SHAPE");
  if (!e || !*e) return 384;
  const int v = atoi(e);
  return v == 16 || v == 384 ? v : -1;
}

// gallery tiles per tile group of the wide sieve pass (i8t::tile_coords): 2, so the ~32 workgroups
// resident on one XCD cover 2 gallery x 16 query tiles (every query panel of a 4096 batch) -- same-box
// A/B (profiles/r03_f6w_group_ab.log): 20.57-20.76 ms per pass at 2, 20.70 at 4, 21.2-21.4 at 3,
// 21.6-21.7 at 8, 23.1-23.2 at 16.
constexpr int F6W_GROUP = 2;

// serpentine query order across the wide sieve pass's tile groups: the query panels a group ends on
// are the ones the next group starts on, while their stages are still in the XCD's L2 -- same-box
// A/B (profiles/r04_f6w_order_ab.txt): 60.0 -> 51.9 GB of L2<->fabric traffic per launch (FETCH_SIZE
// x 2), 21.56 -> 21.45 ms.
constexpr int F6W_SERP = 1;

// The prefix tier's sieve pass on tile_kernel_f6p (persistent; default) or, OFR_F6P_PERSIST=0, on
// tile_kernel_f6w (one workgroup per tile: the A/B reference).  Read at every call.
static bool f6p_persistent() {
  const char* e = getenv("OFR_F6P_PERSIST");
  return !(e && e[0] == '0');
}
// Engine of the one-stage prefix pass: 4 = prefix_wave_kernel (waves decoupled, no barriers; default: 0.49 vs
// 0.63-0.66 ms alone, profiles/r06_prefix_engines_ab.txt), 3 = prefix_pass_kernel<true> (two workgroups per CU
// sharing query panels through LDS, row scales and prefix terms folded into the MFMA), 2 =
// prefix_pass_kernel<false> (the same pass with the fma epilogue), 1 = tile_kernel_f6p<1> (one wave per SIMD).
// 1-3: A/B references.  OFR_F6P_ENGINE, read at every call.
static int f6p_engine() {
  const char* e = getenv("OFR_F6P_ENGINE");
  return e && e[0] >= '1' && e[0] <= '3' ? e[0] - '0' : 4;
}
// CUs the persistent prefix pass leaves free (OFR_F6P_RESERVE, probe): work queued on other streams --
// the previous batch's merge -- otherwise waits for the whole pass
static int f6p_reserve() {
  const char* e = getenv("OFR_F6P_RESERVE");
  const int v = e && *e ? atoi(e) : 0;
  return v < 0 ? 0 : v;
}

// f6 workspace: B <= 32 the stream kernel's tile lists; otherwise the sieve's sample lists,
// thresholds, counts and buckets (each 256-byte aligned)
struct SieveWs {
  size_t lists, theta, count, bucket, armed, bytes;
};
// the panel sample's stride (ofr_knn_f6: every 64th 256-row panel)
static int64_t sieve_stride() { return q8s::SIEVE_STRIDE; }

// Rank of the sample's key that becomes the sieve threshold theta (at least k).  theta only steers
// the volume: the certificate's tau = min(theta, 16th kept key) bounds every row left out whatever
// theta is, and with >= 16 rows kept tau is the 16th kept key either way.  The 16th best of a 1/64
// sample keeps ~16 x 64 rows per query on gallery data; a lower rank keeps proportionally fewer (fewer
// sieve hits and a shorter bucket for the merge), but a panel sample of a gallery stored identity by
// identity holds whole clusters of one face (profiles/r04_sieve_stride_rank_ab.txt: ranks 4 and 8
// leave queries uncertified).  A row sample (ofr_knn_f6_sampled) holds at most a row or two of any
// cluster, and its 4th best key keeps ~4 x 64 rows.
static int sieve_rank(bool rows) { return rows ? q8s::SIEVE_RANK_ROWS : q8s::SIEVE_RANK; }

// The prefix tier's rank: its keys separate the own identity from the rest by a wide gap, and a row
// sample holds at most one row of an identity, so the sample's 2nd best key is another identity's and
// keeps ~2 x 64 rows per query (hits and bucket halved against rank 4: +4 % queries/s, same-box A/B
// profiles/r05_rank_ab.txt; certificates unchanged).  OFR_F6P_RANK: probe override.
constexpr int SIEVE_RANK_PREFIX = 2;
static int f6p_rank() {
  const char* e = getenv("OFR_F6P_RANK");
  const int v = e && *e ? atoi(e) : SIEVE_RANK_PREFIX;
  return v < 1 ? 1 : (v > q8s::KC ? q8s::KC : v);
}

// sample rows of an N-row gallery (ofr_knn_f6_sampled: at most this many)
static int64_t sample_rows(int64_t N) { return cdiv(N > 0 ? N : 1, q8s::SAMPLE_STEP); }

static SieveWs sieve_ws(int64_t B, int64_t N) {
  // sample lists: panel sample (ofr_knn_f6) or row sample (ofr_knn_f6_sampled), whichever has more tiles
  const int64_t ts = std::max(cdiv(cdiv(N > 0 ? N : 1, q8s::TG), sieve_stride()), cdiv(sample_rows(N), q8s::TG));
  SieveWs w;
  w.lists = 0;
  w.theta = round_up((int64_t)(B * ts * q8s::KC * sizeof(Cand)), 256);
  w.count = w.theta + round_up(B * 4, 256);
  w.bucket = w.count + round_up(B * 4, 256);
  w.armed = w.bucket + (size_t)B * q8s::SIEVE_CAP * sizeof(Cand);   // sieve_arm_kernel's flag
  w.bytes = w.armed + 256;
  return w;
}

// B <= 32: tile lists [B][T][KC], then the premerge lists [B][PM][KC]
static size_t stream_ws_lists(int64_t B, int64_t N) {
  return (size_t)round_up((int64_t)cdiv(N > 0 ? N : 1, q8s::TG) * B * q8s::KC * (int64_t)sizeof(Cand), 256);
}

// the regime's regions, then the split merge's selection sel [B][KC] and qd [B][3]
static size_t f6_ws_core(int64_t B, int64_t N) {
  return B <= 32 ? stream_ws_lists(B, N) + (size_t)round_up((int64_t)(B * q8s::PM * q8s::KC * sizeof(Cand)), 256)
                 : (size_t)round_up((int64_t)sieve_ws(B, N).bytes, 256);
}
static size_t f6_ws_qd(int64_t B) { return (size_t)round_up((int64_t)(B * q8s::KC * sizeof(Cand)), 256); }

// the merge's per-query count of exact re-ranks, after the split merge's qd [B][3]
static size_t f6_ws_evals(int64_t B, int64_t N) {
  return f6_ws_core(B, N) + f6_ws_qd(B) + (size_t)round_up(B * 3 * (int64_t)sizeof(double), 256);
}
extern "C" size_t ofr_knn_f6_workspace_bytes(int64_t B, int64_t N) {
  return f6_ws_evals(B, N) + (size_t)round_up(B * 4, 256);
}
extern "C" size_t ofr_knn_f6_merge_evals_offset(int64_t B, int64_t N) { return f6_ws_evals(B, N); }

extern "C" size_t ofr_knn_f6_sieve_counts_offset(int64_t B, int64_t N) {
  return B <= 32 ? (size_t)-1 : sieve_ws(B, N).count;
}

extern "C" int ofr_knn_f6_set_thresholds(void* stream, const double* smax, int64_t B, int64_t N, void* workspace,
                                         size_t workspace_bytes) {
  OFR_CHECK_ARG(B > 32 && N >= 1, "ofr_knn_f6_set_thresholds: the sieve runs for B > 32 (pad the batch)");
  OFR_CHECK_ARG(smax && workspace, "ofr_knn_f6_set_thresholds: null pointer");
  OFR_CHECK_ARG(workspace_bytes >= ofr_knn_f6_workspace_bytes(B, N), "ofr_knn_f6_set_thresholds: workspace too small");
  const SieveWs w = sieve_ws(B, N);
  char* wsb = reinterpret_cast<char*>(workspace);
  hipLaunchKernelGGL(q8s::set_thresholds_kernel, dim3((unsigned)cdiv(B, 256)), dim3(256), 0, (hipStream_t)stream, smax,
                     B, reinterpret_cast<uint32_t*>(wsb + w.theta), reinterpret_cast<int*>(wsb + w.count),
                     reinterpret_cast<uint32_t*>(wsb + w.armed));
  OFR_LAUNCH_CHECK("set_thresholds_kernel");
  return OFR_OK;
}

// the row sample of ofr_knn_f6_sampled
struct F6Sample {
  const void* tiles;
  int64_t n;
  const float* scale;
  const float* aux;
  const void* tiles2;   // second-slice tiles of the same rows (ofr_knn_f6x2_sampled)
};

static int knn_f6_impl(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                       const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
                       const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
                       int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound, void* workspace,
                       size_t workspace_bytes, int merge_mode, double* ub, const void* Qt2 = nullptr,
                       const void* Gt2 = nullptr, const F6Sample* smp = nullptr, const uint8_t* bscale = nullptr,
                       int pstages = 0);

extern "C" int ofr_knn_f6(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                          const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg,
                          int64_t d, const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
                          int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
                          void* workspace, size_t workspace_bytes, const uint8_t* bscale) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 15,
                "ofr_knn_f6: phases: bits 1 (tiles) = 4 (sample + thresholds) + 8 (sieve), 2 (merge)");
  return knn_f6_impl(stream, phases, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, 0, nullptr, nullptr, nullptr, nullptr,
                     bscale);
}

extern "C" int ofr_knn_f6_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                                  const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg,
                                  int64_t d, const void* Gt, const float* gscale, const float* aux,
                                  const double* gmax, int k, int64_t index_base, double* out_d, int64_t* out_i,
                                  int* cert, double* bound, const void* St, int64_t Ns, const float* sscale,
                                  const float* saux, void* workspace, size_t workspace_bytes,
                                  const uint8_t* bscale) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 15,
                "ofr_knn_f6_sampled: phases: bits 1 (tiles) = 4 (sample + thresholds) + 8 (sieve), 2 (merge)");
  OFR_CHECK_ARG(St && sscale && saux, "ofr_knn_f6_sampled: null sample pointer");
  OFR_CHECK_ARG(Ns >= 1 && Ns <= sample_rows(N), "ofr_knn_f6_sampled: sample rows must be in [1, ceil(N / 64)]");
  OFR_CHECK_ARG((uintptr_t)St % 16 == 0, "ofr_knn_f6_sampled: sample tiles must be 16-byte aligned");
  const F6Sample smp{St, Ns, sscale, saux, nullptr};
  return knn_f6_impl(stream, phases, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, 0, nullptr, nullptr, nullptr, &smp, bscale);
}

// Prefix tier f6p: ofr_knn_f6_sampled with the sample and sieve passes scoring only the
// first pstages 128-feature stages.  Gt / gscale / gmax: the prefix tier's own compact gallery tiles
// (ofr_f6p_quantize_rows: pstages stages per panel, power-of-two row scales, prefix stats and maxima);
// St / sscale: the f6 tier's row sample (its first stages).  aux / saux are the PREFIX terms |g_m|^2 of
// the rows and of the row sample (ofr_row_aux over the first min(d, 128 pstages) features).  Every row's squared distance is at least its
// prefix distance, so the certificate holds as for f6; the B x N coarse work shrinks by pstages / nst.
extern "C" int ofr_knn_f6p_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                                   const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg,
                                   int64_t d, const void* Gt, const float* gscale, const float* aux,
                                   const double* gmax, int k, int64_t index_base, double* out_d, int64_t* out_i,
                                   int* cert, double* bound, const void* St, int64_t Ns, const float* sscale,
                                   const float* saux, void* workspace, size_t workspace_bytes,
                                   const uint8_t* bscale, int pstages) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 15,
                "ofr_knn_f6p_sampled: phases: bits 1 (tiles) = 4 (sample + thresholds) + 8 (sieve), 2 (merge)");
  OFR_CHECK_ARG(d >= 1 && pstages >= 1 && pstages <= f6t::stages(d),
                "ofr_knn_f6p_sampled: pstages must be in [1, ceil(d / 128)]");
  OFR_CHECK_ARG(St && sscale && saux, "ofr_knn_f6p_sampled: null sample pointer");
  OFR_CHECK_ARG(Ns >= 1 && Ns <= sample_rows(N), "ofr_knn_f6p_sampled: sample rows must be in [1, ceil(N / 64)]");
  OFR_CHECK_ARG((uintptr_t)St % 16 == 0, "ofr_knn_f6p_sampled: sample tiles must be 16-byte aligned");
  const F6Sample smp{St, Ns, sscale, saux, nullptr};
  return knn_f6_impl(stream, phases, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, 0, nullptr, nullptr, nullptr, &smp, bscale,
                     pstages);
}

extern "C" int ofr_knn_f6x2_sampled(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                                    const void* Qt2, const float* qscale, const double* qstats, const float* G,
                                    int64_t N, int64_t ldg, int64_t d, const void* Gt, const void* Gt2,
                                    const float* gscale, const float* aux, const double* gmax, int k,
                                    int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound,
                                    const void* St, const void* St2, int64_t Ns, const float* sscale,
                                    const float* saux, void* workspace, size_t workspace_bytes,
                                    const uint8_t* bscale) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 15,
                "ofr_knn_f6x2_sampled: phases: bits 1 (tiles) = 4 (sample + thresholds) + 8 (sieve), 2 (merge)");
  OFR_CHECK_ARG(Qt2 && Gt2, "ofr_knn_f6x2_sampled: null second-slice tiles");
  if (B >= 1 && B <= 32)
    return fail(OFR_E_UNSUPPORTED, "ofr_knn_f6x2_sampled: needs more than 32 queries (the sieve pass)");
  OFR_CHECK_ARG(St && St2 && sscale && saux, "ofr_knn_f6x2_sampled: null sample pointer");
  OFR_CHECK_ARG(Ns >= 1 && Ns <= sample_rows(N), "ofr_knn_f6x2_sampled: sample rows must be in [1, ceil(N / 64)]");
  OFR_CHECK_ARG(((uintptr_t)St | (uintptr_t)St2) % 16 == 0, "ofr_knn_f6x2_sampled: sample tiles must be 16-byte aligned");
  const F6Sample smp{St, Ns, sscale, saux, St2};
  return knn_f6_impl(stream, phases, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, 0, nullptr, Qt2, Gt2, &smp, bscale);
}

extern "C" int ofr_knn_f6x2(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                            const void* Qt2, const float* qscale, const double* qstats, const float* G, int64_t N,
                            int64_t ldg, int64_t d, const void* Gt, const void* Gt2, const float* gscale,
                            const float* aux, const double* gmax, int k, int64_t index_base, double* out_d,
                            int64_t* out_i, int* cert, double* bound, void* workspace, size_t workspace_bytes,
                            const uint8_t* bscale) {
  OFR_CHECK_ARG(phases >= 1 && phases <= 15,
                "ofr_knn_f6x2: phases: bits 1 (tiles) = 4 (sample + thresholds) + 8 (sieve), 2 (merge)");
  OFR_CHECK_ARG(Qt2 && Gt2, "ofr_knn_f6x2: null second-slice tiles");
  if (B >= 1 && B <= 32) return fail(OFR_E_UNSUPPORTED, "ofr_knn_f6x2: needs more than 32 queries (the sieve pass)");
  return knn_f6_impl(stream, phases, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, 0, nullptr, Qt2, Gt2, nullptr, bscale);
}

extern "C" int ofr_knn_f6_merge_pruned(void* stream, int stage, const float* Q, int64_t B, int64_t ldq,
                                       const void* Qt, const float* qscale, const double* qstats, const float* G,
                                       int64_t N, int64_t ldg, int64_t d, const void* Gt, const float* gscale,
                                       const float* aux, const double* gmax, int k, int64_t index_base,
                                       double* out_d, int64_t* out_i, int* cert, double* bound, double* ub,
                                       void* workspace, size_t workspace_bytes) {
  OFR_CHECK_ARG(stage == 1 || stage == 2, "ofr_knn_f6_merge_pruned: stage must be 1 (select) or 2 (re-rank)");
  OFR_CHECK_ARG(ub != nullptr, "ofr_knn_f6_merge_pruned: null ub");
  return knn_f6_impl(stream, 2, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, stage, ub);
}

extern "C" int ofr_knn_f6p_merge_pruned(void* stream, int stage, const float* Q, int64_t B, int64_t ldq,
                                        const void* Qt, const float* qscale, const double* qstats, const float* G,
                                        int64_t N, int64_t ldg, int64_t d, const void* Gt, const float* gscale,
                                        const float* aux, const double* gmax, int k, int64_t index_base,
                                        double* out_d, int64_t* out_i, int* cert, double* bound, double* ub,
                                        void* workspace, size_t workspace_bytes, int pstages) {
  OFR_CHECK_ARG(stage == 1 || stage == 2, "ofr_knn_f6p_merge_pruned: stage must be 1 (select) or 2 (re-rank)");
  OFR_CHECK_ARG(ub != nullptr, "ofr_knn_f6p_merge_pruned: null ub");
  OFR_CHECK_ARG(d >= 1 && pstages >= 1 && pstages <= f6t::stages(d),
                "ofr_knn_f6p_merge_pruned: pstages must be in [1, ceil(d / 128)]");
  return knn_f6_impl(stream, 2, Q, B, ldq, Qt, qscale, qstats, G, N, ldg, d, Gt, gscale, aux, gmax, k, index_base,
                     out_d, out_i, cert, bound, workspace, workspace_bytes, stage, ub, nullptr, nullptr, nullptr,
                     nullptr, pstages);
}

static int knn_f6_impl(void* stream, int phases, const float* Q, int64_t B, int64_t ldq, const void* Qt,
                       const float* qscale, const double* qstats, const float* G, int64_t N, int64_t ldg, int64_t d,
                       const void* Gt, const float* gscale, const float* aux, const double* gmax, int k,
                       int64_t index_base, double* out_d, int64_t* out_i, int* cert, double* bound, void* workspace,
                       size_t workspace_bytes, int merge_mode, double* ub, const void* Qt2, const void* Gt2,
                       const F6Sample* smp, const uint8_t* bscale, int pstages) {
  const bool two = Gt2 != nullptr;   // the two-slice tier f6x2: three segments of stages (f6t::seg_src)
  OFR_CHECK_ARG(B >= 0 && N >= 1 && d >= 1, "ofr_knn_f6: bad sizes (empty galleries use ofr_knn_f32)");
  if (k < 1 || k > q8s::KC) return fail(OFR_E_UNSUPPORTED, "ofr_knn_f6: k must be in [1, 16]");
  if (B == 0) return OFR_OK;
  OFR_CHECK_ARG(ldq >= d && ldg >= d, "ofr_knn_f6: bad leading dimensions");
  OFR_CHECK_ARG(Q && Qt && qscale && qstats && G && Gt && gscale && aux && gmax && workspace,
                "ofr_knn_f6: null pointer");
  OFR_CHECK_ARG(((uintptr_t)Qt | (uintptr_t)Gt | (uintptr_t)Qt2 | (uintptr_t)Gt2 | (uintptr_t)workspace) % 16 == 0,
                "ofr_knn_f6: tiles and workspace must be 16-byte aligned");
  OFR_CHECK_ARG(!two || B > 32, "ofr_knn_f6x2: needs more than 32 queries");
  OFR_CHECK_ARG(bscale_ok(bscale), "ofr_knn_f6: bscale must be 4-byte aligned");
  // the sieve's per-query count reaches at most cap + 1 + N (saturating overflow + one per row)
  OFR_CHECK_ARG(N < 0x7fffffffLL - 2 * q8s::SIEVE_CAP, "ofr_knn_f6: N too large for one shard");
  OFR_CHECK_ARG(workspace_bytes >= ofr_knn_f6_workspace_bytes(B, N), "ofr_knn_f6: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  const bool sieve = B > 32;
  q8s::TileArgs a{};
  a.G = (const int8_t*)Gt; a.N = N; a.ld = 0; a.gscale = gscale; a.aux = aux;
  a.Q = (const int8_t*)Qt; a.B = B; a.qscale = qscale;
  a.nk = (int)f6t::stages(d) * (two ? 3 : 1);
  // prefix tier: the first pstages stages (one slice only); otherwise every stage of each segment
  a.nkp = pstages > 0 && !two && pstages < f6t::stages(d) ? pstages : (int)f6t::stages(d);
  // the prefix tier's gallery tiles are its own compact ones (pstages stages per panel, round 6)
  a.gnk = a.nkp < (int)f6t::stages(d) ? a.nkp : a.nk;
  a.G2 = (const int8_t*)Gt2; a.Q2 = (const int8_t*)Qt2;
  a.bs = reinterpret_cast<const uint32_t*>(bscale);
  if (!a.bs) {
    if (f6t::stages(d) > q8s::UNIT_BS_STAGES)
      return fail(OFR_E_UNSUPPORTED, "ofr_knn_f6: d > 524288 needs a column-block scale table (bscale)");
    a.bs = unit_bscale();
    if (!a.bs) return fail(OFR_E_DEVICE, "ofr_knn_f6: unit block-scale table not found on the device");
  }
  a.cand = reinterpret_cast<Cand*>(workspace);
  a.ntq = f6t::panels(B);
  a.ntg = f6t::panels(N);
  a.gg = a.ntg < q8s::GROUP_G ? a.ntg : q8s::GROUP_G;
  a.gstride = 1;
  const SieveWs w = sieve_ws(B, N);
  char* wsb = reinterpret_cast<char*>(workspace);
  uint32_t* theta = reinterpret_cast<uint32_t*>(wsb + w.theta);
  int* count = reinterpret_cast<int*>(wsb + w.count);
  Cand* bucket = reinterpret_cast<Cand*>(wsb + w.bucket);
  uint32_t* armed = reinterpret_cast<uint32_t*>(wsb + w.armed);
  OFR_CHECK_ARG(a.ntq * a.ntg < 0x7fffffffLL, "ofr_knn_f6: grid too large");
  OFR_CHECK_ARG(f6_shape() > 0, "ofr_knn_f6: OFR_F6_SHAPE must be 384 (default) or 16");
  if (a.gnk != a.nk && sieve && f6_shape() != 384)
    return fail(OFR_E_UNSUPPORTED, "ofr_knn_f6p: the prefix tier's compact gallery tiles need OFR_F6_SHAPE=384");
  if (phases & 1) phases |= 12;   // phase 1 = sample + thresholds (4), then the sieve (8)
  if (phases & 12) {
    if (!sieve) {   // HBM regime: one 32-query block, gallery streamed straight to VGPRs
      if (phases & 4) {
        hipLaunchKernelGGL((q8s::stream_kernel_f6<q8s::SU, true>), dim3((unsigned)a.ntg), dim3(512), 0, st, a);
        OFR_LAUNCH_CHECK("f6 stream_kernel");
      }
    } else {
      static bool attr_done = false;
      if (!attr_done) {
        for (const void* f : {(const void*)q8s::tile_kernel_f6<F6_NW>, (const void*)q8s::tile_kernel_f6<F6_NW, 3>,
                              (const void*)q8s::tile_kernel_f6s<1>, (const void*)q8s::tile_kernel_f6s<3>}) {
          hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, f6t::LDS);
          if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(f6 tile)");
        }
        for (const void* f : {(const void*)q8s::tile_kernel_f6w<1>, (const void*)q8s::tile_kernel_f6w<3>}) {
          hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, f6t::EngineW::LDS_BYTES);
          if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(f6 wide tile)");
        }
        for (const void* f : {(const void*)q8s::tile_kernel_f6p<1>, (const void*)q8s::tile_kernel_f6p<2>}) {
          hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, q8s::f6p::LDS_BYTES);
          if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(f6 prefix pass)");
        }
        {
          hipError_t e = hipFuncSetAttribute((const void*)q8s::prefix_pass_kernel<false>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, q8s::pp::LDS_BYTES);
          if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)q8s::prefix_pass_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    q8s::pp::LDS_BYTES);
          if (e != hipSuccess) return hip_status(e, "hipFuncSetAttribute(prefix_pass_kernel)");
        }
        attr_done = true;
      }
      // sample pass: tile lists of every SIEVE_STRIDE-th gallery panel, or of the row sample -> thresholds
      q8s::TileArgs s = a;
      const bool rows = smp && (!two || smp->tiles2);
      if (rows) {
        s.G = (const int8_t*)smp->tiles;
        if (two) s.G2 = (const int8_t*)smp->tiles2;
        s.N = smp->n;
        s.gscale = smp->scale;
        s.aux = smp->aux;
        s.ntg = f6t::panels(smp->n);
      } else {
        s.gstride = sieve_stride();
        s.ntg = cdiv(a.ntg, s.gstride);
      }
      s.gg = s.ntg < q8s::GROUP_G ? s.ntg : q8s::GROUP_G;
      s.cand = reinterpret_cast<Cand*>(wsb + w.lists);
      const bool prefix = a.nkp < f6t::stages(d);
      const int rank = std::max(k, prefix && rows ? f6p_rank() : sieve_rank(rows));
      // the prefix tier's one-stage sample as a wave pass (sample_wave_kernel; OFR_F6P_SAMPLE=tiles: the tile pass)
      const char* spe = getenv("OFR_F6P_SAMPLE");
      const bool swave = (phases & 4) && prefix && rows && a.nkp == 1 && !two && rank <= 2 && f6_shape() == 384 &&
                         device_cus() > 0 && !(spe && spe[0] == 't');
      if (!(phases & 4)) {
        // sieve only: the thresholds of a preceding phases-4 call are in the workspace
      } else if (swave) {
        const int64_t T = cdiv(s.N, (int64_t)q8s::sw::WR);
        OFR_CHECK_ARG((size_t)B * T * sizeof(uint2) <= w.theta - w.lists, "ofr_knn_f6: workspace too small (sample keys)");
        uint2* skeys = reinterpret_cast<uint2*>(wsb + w.lists);
        const int slots = 2 * std::max(1, device_cus());
        const int64_t nst = cdiv(B, (int64_t)q8s::sw::TQ), ntgs = cdiv(s.N, (int64_t)q8s::sw::TGI);
        const int64_t qgs = f6p_group_wave(ntgs, nst, slots, 12);
        const int64_t itm = ntgs * cdiv(nst, qgs);
        OFR_CHECK_ARG(itm < 0x7fffffffLL, "ofr_knn_f6: grid too large (sample)");
        hipLaunchKernelGGL(q8s::sample_wave_kernel, dim3((unsigned)std::min<int64_t>(itm, slots)), dim3(256), 0, st, s,
                           skeys, T, qgs);
        OFR_LAUNCH_CHECK("f6p sample_wave_kernel");
        hipLaunchKernelGGL(q8s::sieve_threshold2_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, st, skeys, T, theta,
                           count, B, rank, armed);
        OFR_LAUNCH_CHECK("f6p sieve_threshold2_kernel");
      } else if (two)
        hipLaunchKernelGGL((q8s::tile_kernel_f6<F6_NW, 3>), dim3((unsigned)(s.ntq * s.ntg)), dim3(F6_NW * 64),
                           f6t::LDS, st, s);
      else
        hipLaunchKernelGGL((q8s::tile_kernel_f6<F6_NW>), dim3((unsigned)(s.ntq * s.ntg)), dim3(F6_NW * 64),
                           f6t::LDS, st, s);
      if ((phases & 4) && !swave) {
        OFR_LAUNCH_CHECK("f6 tile_kernel (sieve sample)");
        hipLaunchKernelGGL(q8s::sieve_threshold_kernel, dim3((unsigned)cdiv(B, 4)), dim3(256), 0, st, s.cand, s.ntg,
                           theta, count, B, rank, armed);
        OFR_LAUNCH_CHECK("f6 sieve_threshold_kernel");
      }
      a.theta = theta;
      a.count = count;
      a.bucket = bucket;
      a.cap = q8s::SIEVE_CAP;
      if (phases & 8) {
        hipLaunchKernelGGL(q8s::sieve_arm_kernel, dim3(1), dim3(256), 0, st, armed, count, B, (int)q8s::SIEVE_CAP);
        OFR_LAUNCH_CHECK("f6 sieve_arm_kernel");
      }
      if (!(phases & 8)) {
        // sample + thresholds only
      } else if (f6_shape() == 384 && a.nkp == 1 && a.nkp < f6t::stages(d) && !two && f6p_persistent() &&
                 f6p_engine() >= 2 && device_cus() > 0) {
        // the one-stage prefix pass: two workgroups per CU (prefix_pass_kernel)
        q8s::TileArgs wa = a;
        wa.ntg = cdiv(N, q8s::pp::TGR);
        const int64_t nsteps = cdiv(B, q8s::pp::TQH), nq = nsteps * q8s::pp::TQH;
        // the per-query table lives in the sample lists' region, dead once the thresholds are set
        OFR_CHECK_ARG((size_t)nq * sizeof(uint2) <= w.theta - w.lists, "ofr_knn_f6: workspace too small (prefix tables)");
        uint2* qtab = reinterpret_cast<uint2*>(wsb + w.lists);
        if (f6p_engine() != 4) {
          hipLaunchKernelGGL(q8s::prefix_tables_kernel, dim3((unsigned)cdiv(nq, 256)), dim3(256), 0, st, theta, a.qscale,
                             B, nq, qtab);
          OFR_LAUNCH_CHECK("f6 prefix_tables_kernel");
        }
        const int slots = 2 * std::max(1, device_cus() - f6p_reserve());
        const int64_t qg = f6p_group(wa.ntg, nsteps, slots);
        const int64_t items = wa.ntg * cdiv(nsteps, qg);
        OFR_CHECK_ARG(items < 0x7fffffffLL, "ofr_knn_f6: grid too large");
        const unsigned grid = (unsigned)std::min<int64_t>(items, slots);
        if (f6p_engine() == 4) {   // wave-decoupled: its own step length, table length and grouping
          // 128 gallery rows x 32 queries per wave step (default: half the query-fragment loads per MFMA,
          // 0.51 -> 0.40 ms at 1M, profiles/r06_prefix_wave_shape_ab.txt); OFR_F6P_WAVE=4: 64 x 64
          const char* wv = getenv("OFR_F6P_WAVE");
          const bool w8 = !(wv && wv[0] == '4');
          const int64_t tq = w8 ? 32 : 64, tgi = w8 ? 512 : 256;
          const int64_t ns4 = cdiv(B, tq), nq4 = ns4 * tq, ntg4 = cdiv(N, tgi);
          OFR_CHECK_ARG((size_t)nq4 * sizeof(uint2) <= w.theta - w.lists, "ofr_knn_f6: workspace too small (prefix tables)");
          hipLaunchKernelGGL(q8s::prefix_tables_kernel, dim3((unsigned)cdiv(nq4, 256)), dim3(256), 0, st, theta,
                             a.qscale, B, nq4, qtab);
          OFR_LAUNCH_CHECK("f6 prefix_tables_kernel");
          const int64_t qg4 = f6p_group_wave(ntg4, ns4, slots, w8 ? 12 : 24);
          const int64_t items4 = round_up(ntg4, 8) * cdiv(ns4, qg4);   // the kernel's tile octets
          OFR_CHECK_ARG(items4 < 0x7fffffffLL, "ofr_knn_f6: grid too large");
          const dim3 g4((unsigned)std::min<int64_t>(items4, slots));
          // probe OFR_F6P_PREFETCH=2: two steps in flight (242 VGPRs) measured equal (profiles/r06_prefix_wave_parts.txt)
          const char* pf = getenv("OFR_F6P_PREFETCH");
          if (w8)
            hipLaunchKernelGGL((q8s::prefix_wave_kernel<8, 2, 1>), g4, dim3(q8s::pw::NT), q8s::pw::lds_bytes(8), st, wa,
                               qtab, qg4);
          else if (pf && pf[0] == '2')
            hipLaunchKernelGGL((q8s::prefix_wave_kernel<4, 4, 2>), g4, dim3(q8s::pw::NT), q8s::pw::lds_bytes(4), st, wa,
                               qtab, qg4);
          else
            hipLaunchKernelGGL((q8s::prefix_wave_kernel<4, 4, 1>), g4, dim3(q8s::pw::NT), q8s::pw::lds_bytes(4), st, wa,
                               qtab, qg4);
        } else if (f6p_engine() == 3)
          hipLaunchKernelGGL(q8s::prefix_pass_kernel<true>, dim3(grid), dim3(q8s::pp::NT), q8s::pp::LDS_BYTES, st, wa,
                             qtab, qg);
        else
          hipLaunchKernelGGL(q8s::prefix_pass_kernel<false>, dim3(grid), dim3(q8s::pp::NT), q8s::pp::LDS_BYTES, st, wa,
                             qtab, qg);
      } else if (f6_shape() == 384 && a.nkp <= q8s::f6p::NSPMAX && a.nkp < f6t::stages(d) && !two &&
                 f6p_persistent() && device_cus() > 0) {
        // the prefix tier's short pass: persistent workgroups, the gallery tile resident (tile_kernel_f6p)
        q8s::TileArgs wa = a;
        wa.ntg = cdiv(N, f6t::EngineW::TGW);
        const int cus = std::max(1, device_cus() - f6p_reserve());
        const int64_t qg = f6p_group(wa.ntg, wa.ntq, cus);
        const int64_t items = wa.ntg * cdiv(wa.ntq, qg);
        OFR_CHECK_ARG(items < 0x7fffffffLL, "ofr_knn_f6: grid too large");
        const unsigned grid = (unsigned)std::min<int64_t>(items, cus);
        if (a.nkp == 1)
          hipLaunchKernelGGL(q8s::tile_kernel_f6p<1>, dim3(grid), dim3(f6t::EngineW::NT), q8s::f6p::LDS_BYTES, st, wa,
                             qg);
        else
          hipLaunchKernelGGL(q8s::tile_kernel_f6p<2>, dim3(grid), dim3(f6t::EngineW::NT), q8s::f6p::LDS_BYTES, st, wa,
                             qg);
      } else if (f6_shape() == 384) {
        q8s::TileArgs wa = a;   // 384-row gallery tiles over the same 256-row panel layout
        wa.ntg = cdiv(N, f6t::EngineW::TGW);
        wa.gg = wa.ntg < F6W_GROUP ? wa.ntg : F6W_GROUP;
        wa.serp = F6W_SERP;
        OFR_CHECK_ARG(wa.ntq * wa.ntg < 0x7fffffffLL, "ofr_knn_f6: grid too large");
        if (two)
          hipLaunchKernelGGL(q8s::tile_kernel_f6w<3>, dim3((unsigned)(wa.ntq * wa.ntg)), dim3(f6t::EngineW::NT),
                             f6t::EngineW::LDS_BYTES, st, wa);
        else
          hipLaunchKernelGGL(q8s::tile_kernel_f6w<1>, dim3((unsigned)(wa.ntq * wa.ntg)), dim3(f6t::EngineW::NT),
                             f6t::EngineW::LDS_BYTES, st, wa);
      } else if (two)
        hipLaunchKernelGGL((q8s::tile_kernel_f6s<3>), dim3((unsigned)(a.ntq * a.ntg)), dim3(f6t::Engine16::NT),
                           f6t::LDS, st, a);
      else
        hipLaunchKernelGGL((q8s::tile_kernel_f6s<1>), dim3((unsigned)(a.ntq * a.ntg)), dim3(f6t::Engine16::NT),
                           f6t::LDS, st, a);
      OFR_LAUNCH_CHECK("f6 tile_kernel (sieve)");
    }
  }
  if (phases & 2) {
    OFR_CHECK_ARG(merge_mode == 1 || (out_d && out_i && cert), "ofr_knn_f6: null output");
    // fp32 accumulation over nst * 2 MFMAs: |err| <= (n + 64) 2^-23 sum|q~ g~| / (s_q s_g),
    // sum|q~ g~| <= a_q a_g <= a_q A (tools/mx_probe.hip measures <= 3 * 2^-24 at n = 160)
    const double gamma = (double)(2 * a.nk + 64) * 0x1p-23;
    q8s::MergeArgs m{a.cand, a.ntg, B, Q, ldq, G, ldg, d, qstats, gmax, gamma, k, index_base, out_d, out_i, cert, bound};
    m.mode = merge_mode;
    m.dpre = a.nkp < f6t::stages(d) ? (int64_t)a.nkp * f6t::BK : 0;
    m.sel = reinterpret_cast<Cand*>(wsb + f6_ws_core(B, N));
    m.qd = reinterpret_cast<double*>(wsb + f6_ws_core(B, N) + f6_ws_qd(B));
    m.evals = reinterpret_cast<int*>(wsb + f6_ws_evals(B, N));
    // the deep continuation (sieve buckets, the one-stage merge; OFR_MERGE_DEEP=0: off, =N: N rounds at most)
    {
      const char* e = getenv("OFR_MERGE_DEEP");
      const int rounds = e && e[0] ? atoi(e) : q8s::DEEP_ROUNDS;
      m.deep = sieve && merge_mode == 0 && rounds > 0 ? std::min(rounds, 4096) : 0;
    }
    if (merge_mode == 1) m.ub_local = ub;
    if (merge_mode == 2) m.ub = ub;
    if (sieve) {
      m.cand = bucket;
      m.count = count;
      m.theta = theta;
      m.cap = q8s::SIEVE_CAP;
    } else if (merge_mode == 2) {
      // the selection is read back from sel: no premerge
    } else if (a.ntg > q8s::PM) {
      Cand* pm = reinterpret_cast<Cand*>(wsb + stream_ws_lists(B, N));
      hipLaunchKernelGGL(q8s::premerge_kernel, dim3(q8s::PM, (unsigned)B), dim3(256), 0, st, a.cand, a.ntg, pm);
      OFR_LAUNCH_CHECK("f6 premerge_kernel");
      m.cand = pm;
      m.T = q8s::PM;
    }
    if (sieve)
      launch_merge<true>(st, m);
    else
      launch_merge<false>(st, m);
    OFR_LAUNCH_CHECK("f6 merge_kernel");
  }
  return OFR_OK;
}
