// Feed / compute probe for the fp6 tile kernel (diagnostic tool, not part of the library).
// Times q8s::tile_kernel_f6<NW, MODE> on random e2m3 tiles (MODE bits: see main).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/f6_probe.hip \
//         opencv_facerecognizer_amd/csrc/ofr_api.hip -o tools/f6_probe
//   ./tools/f6_probe [N] [B] [d] [reps]
#define OFR_F6_STAMPS 1
#include "../opencv_facerecognizer_amd/csrc/ofr_knn_q8.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ofr;

namespace ofr {
namespace f6t {
// ---- 16x16x128 engine, query operand straight to registers (experimental sieve pass) ----------
// The LDS carries only the gallery block (24 KiB per stage, NSQ stages, one 1-KiB LDS-DMA
// wave-instruction per 3 of the stage's 24 per wave); each wave owns 32 queries (2 fragments,
// loaded from the query tiles in global memory -- L2-resident across the tile group -- D = NSQ - 2
// stages ahead into NSQ - 1 register sets) against all 256 gallery rows, whose 16 fragments per
// stage stream through a ring of R registers sets read R - 1 steps ahead (2 MFMAs per step).
// Half the LDS-DMA bytes and LDS writes of Engine16 and no query fragment reads from LDS, for
// a third more gallery fragment reads.  C/D of acc[i][c]: gallery rows 16 i + 4 (l / 16) + reg,
// query 32 wave + 16 c + l % 16.
template <int NSQ, int R, int D = NSQ - 2>
struct EngineQ {
  static constexpr int NW = 8, NT = 512, NA = 16, NB = 2;
  static constexpr int NQS = D + 1;                      // query register sets
  static constexpr int GINS = PANEL / 1024 / NW;         // 3 DMA wave-instructions per wave per stage
  static constexpr int VM_PER_IT = GINS + 2 * NB;        // VMEM instructions per wave per stage (7)
  static constexpr int LDS_BYTES = NSQ * PANEL;
  static_assert(NSQ >= 4 && NSQ <= 6 && R >= 2 && R <= 8 && D >= 1 && D <= NSQ - 2, "EngineQ");
  // per stage the query loads are issued first, then the DMA: at the start of stage kt the wave
  // needs Q(kt) (issued D stages before) and DMA(kt+1) (NSQ-2 stages before) complete
  static constexpr int VM_WAIT = D < NSQ - 2 ? GINS + (D - 1) * VM_PER_IT : (D - 1) * VM_PER_IT;
  static constexpr int VM_WAIT_NODMA = (D - 1) * 2 * NB;

  static __device__ __forceinline__ void dma(const char* G, int64_t gp, int64_t nst, int kt, char* st) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const char* gb = G + (gp * nst + kt) * (int64_t)PANEL;
#pragma unroll
    for (int t = 0; t < GINS; ++t) {
      const int off = (wave * GINS + t) * 1024;
      __builtin_amdgcn_global_load_lds((const OFR_GLOBAL void*)(gb + off + lane * 16), (OFR_LDS void*)(st + off), 16,
                                       0, 0);
    }
  }
  // the lane's query fragment c of stage kt straight from the tiled layout; zero past the last stage
  static __device__ __forceinline__ i32x6 qfrag(const char* Q, int64_t qp, int64_t nst, int kt, int c) {
    const int lane = threadIdx.x & 63, q = lane >> 4, row = (threadIdx.x >> 6) * 32 + c * 16 + (lane & 15);
    const bool past = kt >= nst;   // uniform
    const char* sb = Q + (qp * nst + (past ? nst - 1 : kt)) * (int64_t)PANEL + q * 6144;
    const i32x4 p0 = *(const OFR_GLOBAL i32x4*)(sb + row * 16);
    const i32x2 p1 = *(const OFR_GLOBAL i32x2*)(sb + 4096 + p1_slot(q, row) * 8);
    const int z = past ? 0 : -1;
    i32x6 f;
    f[0] = p0[0] & z; f[1] = p0[1] & z; f[2] = p0[2] & z; f[3] = p0[3] & z; f[4] = p1[0] & z; f[5] = p1[1] & z;
    return f;
  }

  template <int MODE>
  static __device__ __forceinline__ void mainloop(char* smem, const char* G, int64_t gp, const char* Q, int64_t qp,
                                                  int nst, f32x4 (&acc)[NA][NB]) {
    const int r16 = threadIdx.x & 15;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int c = 0; c < NB; ++c) acc[i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int last = nst - 1;
    auto clampk = [&](int k) { return k < last ? k : last; };
    auto buf = [&](int k) { return smem + (k % NSQ) * PANEL; };
    i32x6 qs[NQS][NB];
    i32x6 g[R];
    // prologue: DMA of stages 0 .. NSQ-2 and the query fragments of stages 0 .. D-1, in the
    // per-iteration order (stage s's DMA then the queries of stage s - (NSQ-1) + D = s - 1)
#pragma unroll
    for (int s = 0; s < NSQ - 1; ++s) {
      if constexpr ((MODE & 1) == 0) dma(G, gp, nst, clampk(s), buf(s));
      if (s >= 1 && s - 1 < D) {
#pragma unroll
        for (int c = 0; c < NB; ++c) qs[s - 1][c] = qfrag(Q, qp, nst, s - 1, c);
      }
    }
    wait_vm<0>();
    barrier();
#pragma unroll
    for (int j = 0; j < R - 1; ++j) g[j] = Engine16::frag16(smem, j * 16 + r16);

    auto iter = [&](int kt, auto setc) {
      constexpr int S = decltype(setc)::value;               // register set of stage kt
      if constexpr ((MODE & 1) == 0) wait_vm<VM_WAIT>();
      else wait_vm<VM_WAIT_NODMA>();
      barrier();   // stage kt+1 landed everywhere; the buffer of stage kt-1 is free
#pragma unroll
      for (int c = 0; c < NB; ++c) qs[(S + D) % NQS][c] = qfrag(Q, qp, nst, kt + D, c);
      if constexpr ((MODE & 1) == 0) dma(G, gp, nst, clampk(kt + NSQ - 1), buf(kt + NSQ - 1));
      const char* cur = buf(kt);
      const char* nxt = buf(kt + 1);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int j = i + R - 1;
        g[j % R] = Engine16::frag16(j < NA ? cur : nxt, (j % NA) * 16 + r16);
#pragma unroll
        for (int c = 0; c < NB; ++c) acc[i][c] = Engine16::mfma(g[i % R], qs[S][c], acc[i][c]);
      }
      __builtin_amdgcn_sched_group_barrier(0x020, VM_PER_IT, 0);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, NB, 0);
      }
    };
    // stages past the end (kt >= nst, up to the next multiple of NQS) keep the schedule with
    // zero query fragments (0 x finite = +0 exactly): one instance of each register-set
    // iteration, no tail copy
    for (int kt = 0; kt < nst; kt += NQS) {
      iter(kt, std::integral_constant<int, 0>{});
      if constexpr (NQS > 1) iter(kt + 1, std::integral_constant<int, 1>{});
      if constexpr (NQS > 2) iter(kt + 2, std::integral_constant<int, 2>{});
      if constexpr (NQS > 3) iter(kt + 3, std::integral_constant<int, 3>{});
      if constexpr (NQS > 4) iter(kt + 4, std::integral_constant<int, 4>{});
    }
    wait_vm<0>();
    barrier();
  }
};

}  // namespace f6t
namespace q8s {
// fp6 sieve pass on the query-direct 16x16x128 engine (f6t::EngineQ, experimental: selected by
// OFR_F6_SHAPE=17).  MODE probe bits: 1 = no k-loop DMA, 4 = no epilogue.
template <int MODE, int NSQ, int R, int D = NSQ - 2>
__global__ void __launch_bounds__(512, 1) tile_kernel_f6q(TileArgs p) {
  using E = f6t::EngineQ<NSQ, R, D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int64_t t = i8t::xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  int64_t gt, qt;
  i8t::tile_coords(t, p.gg, p.ntg, p.ntq, gt, qt);
  const int64_t gp = gt * p.gstride;
  const int64_t g0 = gp * TG, q0 = qt * f6t::TQ;
  f6t::f32x4 acc[E::NA][E::NB];
  E::template mainloop<MODE & 1>(smem, reinterpret_cast<const char*>(p.G), gp, reinterpret_cast<const char*>(p.Q), qt,
                                 p.nk, acc);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r16 = lane & 15, g4 = (lane >> 4) * 4;
  float sq2[E::NB], th[E::NB];
#pragma unroll
  for (int c = 0; c < E::NB; ++c) {
    const int64_t q = q0 + wave * 32 + c * 16 + r16;
    const bool ok = q < p.B;
    sq2[c] = 2.0f * p.qscale[ok ? q : p.B - 1];
    th[c] = ok ? key_float(p.theta[q] | 0xffu) : -__builtin_inff();
  }
  if constexpr ((MODE & 4) != 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < E::NA; ++i)
#pragma unroll
      for (int c = 0; c < E::NB; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += acc[i][c][r];
    if (s == 1.2345f) p.cand[0].d = s;
    return;
  }
  float* gtab = reinterpret_cast<float*>(smem);                                  // [TG][2]
  uint32_t* nhit = reinterpret_cast<uint32_t*>(smem + TG * 8);
  uint2* hits = reinterpret_cast<uint2*>(smem + TG * 8 + 16);                    // [SIEVE_HCAP]
  const int nvalid = p.N - g0 < TG ? (int)(p.N - g0) : TG;
  if (threadIdx.x < TG) {
    const bool ok = g0 + threadIdx.x < p.N;
    gtab[2 * threadIdx.x + 0] = ok ? p.aux[g0 + threadIdx.x] : __builtin_inff();
    gtab[2 * threadIdx.x + 1] = ok ? p.gscale[g0 + threadIdx.x] : 0.f;
  }
  if (threadIdx.x == 0) *nhit = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < E::NA; ++i) {
    const int gl0 = i * 16 + g4;                   // this lane's 4 consecutive gallery rows
    const float4 t0 = reinterpret_cast<const float4*>(gtab)[gl0 / 2];
    const float4 t1 = reinterpret_cast<const float4*>(gtab)[gl0 / 2 + 1];
    const float av[4] = {t0.x, t0.z, t1.x, t1.z}, sv[4] = {t0.y, t0.w, t1.y, t1.w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gl = gl0 + r;
#pragma unroll
      for (int c = 0; c < E::NB; ++c) {
        const float sc = av[r] - sq2[c] * sv[r] * acc[i][c][r];
        if (!(sc > th[c]) && gl < nvalid) {
          const int ql = wave * 32 + c * 16 + r16;
          const uint32_t kb = __float_as_uint(key_score(score_key(sc, 0)));
          const uint32_t slot = atomicAdd(nhit, 1u);
          if (slot < (uint32_t)SIEVE_HCAP) hits[slot] = make_uint2(kb, ((uint32_t)ql << 8) | (uint32_t)gl);
        }
      }
    }
  }
  __syncthreads();
  sieve_flush<f6t::TQ>(smem, p, g0, q0);
}

}  // namespace q8s
}  // namespace ofr

__global__ void fill_u8(uint8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (uint8_t)x;
  }
}
__global__ void fill_f(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int NW, int MODE>
static int run(q8s::TileArgs a, int reps, const char* tag) {
  const double ops = 2.0 * (double)a.ntg * f6t::TA * a.ntq * f6t::TQ * a.nk * f6t::BK;
  CK(hipFuncSetAttribute((const void*)q8s::tile_kernel_f6<NW, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, f6t::LDS));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(a.ntq * a.ntg);
  hipLaunchKernelGGL((q8s::tile_kernel_f6<NW, MODE>), dim3(grid), dim3(NW * 64), f6t::LDS, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::tile_kernel_f6<NW, MODE>), dim3(grid), dim3(NW * 64), f6t::LDS, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)grid * a.nk * f6t::STAGE;
  printf("f6 nw=%d %-12s mode=%-2d gg=%-3ld ms=%8.2f  executed=%7.1f TOPS (%.1f%% of 10000)  LDS-fill=%6.2f TB/s\n", NW, tag, MODE,
         (long)a.gg, ms, ops / ms / 1e9, ops / ms / 1e9 / 100.0, bytes / ms / 1e9);
  fflush(stdout);
  return 0;
}

template <int MODE>
static int run16(q8s::TileArgs a, int reps, const char* tag) {
  const double ops = 2.0 * (double)a.ntg * f6t::TA * a.ntq * f6t::TQ * a.nk * f6t::BK;
  CK(hipFuncSetAttribute((const void*)q8s::tile_kernel_f6s<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, f6t::LDS));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(a.ntq * a.ntg);
  hipLaunchKernelGGL((q8s::tile_kernel_f6s<MODE>), dim3(grid), dim3(512), f6t::LDS, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::tile_kernel_f6s<MODE>), dim3(grid), dim3(512), f6t::LDS, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("f6 16x16 %-12s mode=%-2d gg=%-3ld ms=%8.2f  executed=%7.1f TOPS (%.1f%% of 10000)\n", tag, MODE, (long)a.gg, ms,
         ops / ms / 1e9, ops / ms / 1e9 / 100.0);
  fflush(stdout);
  return 0;
}

template <int MODE>
static int runw(q8s::TileArgs a, int reps, const char* tag) {
  using E = f6t::EngineW;
  a.ntg = (a.N + E::TGW - 1) / E::TGW;
  if (a.gg > a.ntg) a.gg = a.ntg;
  const double ops = 2.0 * (double)a.N * a.ntq * f6t::TQ * a.nk * f6t::BK;
  CK(hipFuncSetAttribute((const void*)q8s::tile_kernel_f6w<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, E::LDS_BYTES));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(a.ntq * a.ntg);
  hipLaunchKernelGGL((q8s::tile_kernel_f6w<MODE>), dim3(grid), dim3(E::NT), E::LDS_BYTES, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::tile_kernel_f6w<MODE>), dim3(grid), dim3(E::NT), E::LDS_BYTES, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("f6 wide384 %-12s mode=%-2d gg=%-3ld ms=%8.2f  executed=%7.1f TOPS (%.1f%% of 10000)\n", tag, MODE, (long)a.gg, ms,
         ops / ms / 1e9, ops / ms / 1e9 / 100.0);
  fflush(stdout);
  return 0;
}

template <int MODE, int NSQ, int R, int D>
static int runq(q8s::TileArgs a, int reps, const char* tag) {
  const double ops = 2.0 * (double)a.ntg * f6t::TA * a.ntq * f6t::TQ * a.nk * f6t::BK;
  const int lds = f6t::EngineQ<NSQ, R, D>::LDS_BYTES;
  CK(hipFuncSetAttribute((const void*)q8s::tile_kernel_f6q<MODE, NSQ, R, D>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(a.ntq * a.ntg);
  hipLaunchKernelGGL((q8s::tile_kernel_f6q<MODE, NSQ, R, D>), dim3(grid), dim3(512), lds, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::tile_kernel_f6q<MODE, NSQ, R, D>), dim3(grid), dim3(512), lds, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("f6 qdirect nsq=%d r=%d d=%d %-12s mode=%-2d gg=%-3ld ms=%8.2f  executed=%7.1f TOPS (%.1f%% of 10000)\n", NSQ, R,
         D, tag, MODE, (long)a.gg, ms, ops / ms / 1e9, ops / ms / 1e9 / 100.0);
  fflush(stdout);
  return 0;
}

template <int U, bool NT>
static int run_stream(q8s::TileArgs a, int reps, const char* tag) {
  a.ntq = 1;
  a.B = 32;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((q8s::stream_kernel_f6<U, NT>), dim3((unsigned)a.ntg), dim3(512), 0, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::stream_kernel_f6<U, NT>), dim3((unsigned)a.ntg), dim3(512), 0, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)a.ntg * f6t::TA * a.nk * 96.0;
  printf("stream %-10s U=%d nt=%d ms=%7.3f  %6.0f GB/s (%.1f%% of 8000)\n", tag, U, (int)NT, ms, bytes / ms / 1e6,
         bytes / ms / 1e6 / 80.0);
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t B = argc > 2 ? atoll(argv[2]) : 4096;
  const int64_t d = argc > 3 ? atoll(argv[3]) : 9999;
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  uint8_t *G, *Q;
  float *gs, *aux, *qs;
  Cand* cand;
  const size_t gb = f6t::tiles_bytes(N, d), qb = f6t::tiles_bytes(B, d);
  CK(hipMalloc(&G, gb));
  CK(hipMalloc(&Q, qb));
  CK(hipMalloc(&gs, N * 4)); CK(hipMalloc(&aux, N * 4)); CK(hipMalloc(&qs, B * 4));
  const int64_t ntg = f6t::panels(N);
  CK(hipMalloc(&cand, ntg * B * q8s::KC * sizeof(Cand)));
  fill_u8<<<4096, 256>>>(G, gb, 1);
  fill_u8<<<4096, 256>>>(Q, qb, 3);
  fill_f<<<1024, 256>>>(gs, N, 1.f); fill_f<<<1024, 256>>>(aux, N, 1.f); fill_f<<<64, 256>>>(qs, B, 1.f);
  CK(hipDeviceSynchronize());
  q8s::TileArgs a{};
  a.G = (const int8_t*)G; a.N = N; a.ld = 0; a.gscale = gs; a.aux = aux;
  a.Q = (const int8_t*)Q; a.B = B; a.qscale = qs; a.cand = cand; a.ntg = ntg;
  a.ntq = f6t::panels(B);
  a.nk = (int)f6t::stages(d);
  a.gstride = 1;
  // sieve operands: a threshold below every score (-FLT_MAX): the pure cost of the test
  uint32_t* theta;
  int* count;
  CK(hipMalloc(&theta, B * 4));
  CK(hipMalloc(&count, B * 4));
  std::vector<uint32_t> th(B, 0x00800000u);
  CK(hipMemcpy(theta, th.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemset(count, 0, B * 4));
  a.theta = theta; a.count = count; a.bucket = cand; a.cap = 16;
  printf("N=%ld B=%ld d=%ld\n", (long)N, (long)B, (long)d);
  if (getenv("STREAM_ONLY")) {
    for (int rep = 0; rep < 2; ++rep)
      if (run_stream<4, false>(a, 20, "base") || run_stream<8, false>(a, 20, "u8") || run_stream<2, false>(a, 20, "u2") ||
          run_stream<4, true>(a, 20, "nt") || run_stream<8, true>(a, 20, "u8+nt"))
        return 1;
    return 0;
  }
  if (getenv("SHAPE16")) {   // the 16x16x128 sieve engine next to the 32x32x64 one
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<0>(a, reps, "sieve16") || run16<1024>(a, reps, "mubuf2b16") || run16<1024 + 4096>(a, reps, "mubuf2b-rs2") ||
          run16<1024 + 4096 + 8192>(a, reps, "mubuf2b-rs1"))
        return 1;
    return 0;
  }
  if (getenv("WIDE_DEPTH")) {   // per-tile fixed cost: the wide pass at this d (time = rounds x (fixed + nst x stage))
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (runw<0>(a, reps, "wide") || runw<4>(a, reps, "wide-noepi")) return 1;
    return 0;
  }
  if (getenv("WIDE")) {   // the 384 x 256 one-wave-per-SIMD engine (f6t::EngineW) vs the library pass
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<275456>(a, reps, "lib4w") || run16<275456 + 4>(a, reps, "lib4w-noepi") || runw<0>(a, reps, "wide") ||
          runw<4>(a, reps, "wide-noepi") || runw<5>(a, reps, "wide-nocopy"))
        return 1;
    for (int g : {2, 4, 8}) {
      a.gg = g;
      if (runw<0>(a, reps, "wide-gg")) return 1;
    }
    return 0;
  }
  if (getenv("GGDMA")) {   // the DMA-only variant and the 4-issuing-wave pass against the tile-group width
    for (int g : {1, 2, 4, 8, 16}) {
      a.gg = g < ntg ? g : ntg;
      if (run16<13312 + 4 + 16384 + 65536>(a, reps, "dma-only-gg") || run16<13312 + 4 + 262144>(a, reps, "noepi-4w-gg"))
        return 1;
    }
    return 0;
  }
  if (getenv("ASYM")) {   // the asymmetric loop against the library pass
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<275456>(a, reps, "lib4w") || run16<16777216>(a, reps, "asym") || run16<16777216 + 4>(a, reps, "asym-noepi"))
        return 1;
    return 0;
  }
  if (getenv("STAMPS")) {   // phases of a stage of the library pass (s_memtime, waves 0-3 vs 4-7)
    a.gg = 4 < ntg ? 4 : ntg;
    if (run16<275456>(a, reps, "lib4w") || run16<275456 + 8388608>(a, reps, "lib4w-stamped")) return 1;
    std::vector<unsigned long long> h(f6t::STAMP_WG * 8 * f6t::STAMP_N);
    CK(hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(f6t::g_f6_stamps), h.size() * 8));
    const char* names[5] = {"rows before re-fill barrier", "re-fill wait+barrier", "copy issue", "remaining rows",
                            "top wait (copies landed)+barrier"};
    for (int role = 0; role < 2; ++role) {
      double sum[5] = {0, 0, 0, 0, 0}, n = 0;
      for (int b = 0; b < f6t::STAMP_WG; ++b)
        for (int w = role * 4; w < role * 4 + 4; ++w) {
          const unsigned long long* o = h.data() + ((size_t)b * 8 + w) * f6t::STAMP_N;
          for (int j = 0; j < 5; ++j) sum[j] += (double)o[j];
          n += (double)o[5];
        }
      printf("waves %d-%d (%s), cycles per stage:", role * 4, role * 4 + 3, role ? "no copies" : "issue the copies");
      double tot = 0;
      for (int j = 0; j < 5; ++j) tot += sum[j] / n;
      for (int j = 0; j < 5; ++j) printf("  %s %.0f", names[j], sum[j] / n);
      printf("  | total %.0f\n", tot);
    }
    return 0;
  }
  if (getenv("DEEP32")) {   // the 32x32x64 engine with 64-feature half-stages in 6 buffers vs the library pass
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<275456>(a, reps, "lib4w") || run<8, 8>(a, reps, "sieve32") || run<8, 40>(a, reps, "sieve32-deep") ||
          run<8, 44>(a, reps, "deep-noepi") || run<8, 13>(a, reps, "nodma-noepi32"))
        return 1;
    return 0;
  }
  if (getenv("NOP1")) {   // the library pass with / without the part1 reads (b64) of every fragment
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<275456>(a, reps, "lib4w") || run16<275456 + 1048576>(a, reps, "lib4w-nop1") ||
          run16<275456 + 4>(a, reps, "noepi4w") || run16<275456 + 4 + 1048576>(a, reps, "noepi4w-nop1") ||
          run16<275456 + 2097152>(a, reps, "lib4w-spread") || run16<275456 + 4 + 2097152>(a, reps, "noepi4w-spread"))
        return 1;
    return 0;
  }
  if (getenv("FEED4W")) {   // copies issued by waves 0-3 only: with / without refills, epilogue; ping-pong
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<13312>(a, reps, "lib") || run16<13312 + 262144>(a, reps, "lib-4w") || run16<524288>(a, reps, "pingpong") ||
          run16<524288 + 4>(a, reps, "pingpong-noepi") || run16<13312 + 4>(a, reps, "noepi") ||
          run16<13312 + 4 + 262144>(a, reps, "noepi-4w") || run16<13312 + 4 + 16384>(a, reps, "noepi-norefill") ||
          run16<13312 + 4 + 16384 + 262144>(a, reps, "noepi-norefill-4w"))
        return 1;
    return 0;
  }
  if (getenv("FEEDTEST")) {   // the library sieve pass without its epilogue, without its fragment refills
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<13312>(a, reps, "lib") || run16<13312 + 4>(a, reps, "noepi") ||
          run16<13312 + 4 + 16384>(a, reps, "noepi-norefill") || run16<13312 + 4 + 16384 + 65536>(a, reps, "dma-only") ||
          run16<13312 + 4 + 16384 + 65536 + 131072>(a, reps, "dma-only-L2") || run16<13312 + 4 + 131072>(a, reps, "noepi-L2") ||
          run16<13312 + 4 + 16384 + 65536 + 262144>(a, reps, "dma-only-4w") || run16<13312 + 4 + 262144>(a, reps, "noepi-4w") ||
          run16<5>(a, reps, "nodma-noepi"))
        return 1;
    return 0;
  }
  if (getenv("QDIRECT")) {   // query operand straight to registers (f6t::EngineQ) vs Engine16
    a.gg = 4 < ntg ? 4 : ntg;
    for (int rep = 0; rep < 2; ++rep)
      if (run16<0>(a, reps, "sieve16") || run16<5>(a, reps, "nodma-noepi16") || runq<0, 4, 2, 1>(a, reps, "sieve") ||
          runq<4, 4, 2, 1>(a, reps, "noepi") || runq<5, 4, 2, 1>(a, reps, "nodma-noepi") ||
          runq<0, 5, 2, 1>(a, reps, "sieve") || runq<0, 6, 2, 1>(a, reps, "sieve") || runq<0, 4, 3, 1>(a, reps, "sieve") ||
          runq<0, 5, 2, 2>(a, reps, "sieve"))
        return 1;
    return 0;
  }
  if (getenv("GG_SWEEP")) {   // tile-group width (gallery panels per group) vs the sieve pass time
    for (int g : {1, 2, 4, 8, 16, 32}) {
      a.gg = g < ntg ? g : ntg;
      if (run<8, 8>(a, reps, "sieve-gg")) return 1;
    }
    return 0;
  }
  a.gg = 4 < ntg ? 4 : ntg;
  // MODE bits: 8 = sieve epilogue (else tile lists); 4 = no epilogue; 1 = no k-loop DMA;
  // 2 / 16 = no gallery / query block in the DMA
  for (int rep = 0; rep < 2; ++rep) {
    if (run<8, 8>(a, reps, "sieve") || run<8, 4>(a, reps, "noepi") || run<8, 5>(a, reps, "nodma") ||
        run<8, 6>(a, reps, "no-gal-dma") || run<8, 20>(a, reps, "no-q-dma"))
      return 1;
  }
  return 0;
}
