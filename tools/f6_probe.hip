// Feed / compute probe for the fp6 tile kernel (diagnostic tool, not part of the library).
// Times q8s::tile_kernel_f6<NW, MODE> on random e2m3 tiles (MODE bits: see main).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/f6_probe.hip \
//         opencv_facerecognizer_amd/csrc/ofr_api.hip -o tools/f6_probe
//   ./tools/f6_probe [N] [B] [d] [reps]
#include "../opencv_facerecognizer_amd/csrc/ofr_knn_q8.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace ofr;

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
      if (run<8, 8>(a, reps, "sieve32") || run16<0>(a, reps, "sieve16") || run16<4>(a, reps, "noepi16") ||
          run16<5>(a, reps, "nodma-noepi16") || run<8, 5>(a, reps, "nodma-noepi32"))
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
