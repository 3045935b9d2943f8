// Feed / compute probe for the int8 tile kernels (diagnostic tool, not part of the library).
// Times q8s::tile_kernel<SL, MODE> on random slices: MODE 0 = search, 1 = no k-loop DMA
// (MFMA + LDS only), 2 = no MFMA (DMA feed only); SL = 1 or 2 int8 slices per row.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/q8_probe.hip \
//         opencv_facerecognizer_amd/csrc/ofr_api.hip -o tools/q8_probe
//   ./tools/q8_probe [N] [B] [d] [reps]
#include "../opencv_facerecognizer_amd/csrc/ofr_knn_q8.hip"
#include <cstdio>
#include <cstdlib>

using namespace ofr;

__global__ void fill_i8(int8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (int8_t)((int)(x % 255u) - 127);
  }
}
__global__ void fill_f(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}

// ceiling: back-to-back v_mfma_i32_32x32x32_i8 on register operands, 16 accumulators per wave,
// one wave per SIMD on every CU (what the matrix cores sustain at the clock they hold)
__global__ void __launch_bounds__(256, 1) mfma_ceiling(const int* seed, int iters, int* out) {
  typedef int v4 __attribute__((ext_vector_type(4)));
  typedef int v16 __attribute__((ext_vector_type(16)));
  v4 a[4], b[4];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 4; ++e) {
      a[i][e] = seed[(threadIdx.x + 7 * i + e) & 255] * 0x01010101;
      b[i][e] = seed[(threadIdx.x + 13 * i + 3 * e) & 255] * 0x01030507;
    }
  v16 acc[4][4];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  int s = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <int SL, int MODE>
static int run(q8s::TileArgs a, int64_t d, int reps, const char* tag) {
  using S = q8s::Shape<SL>;
  a.nk = (int)cdiv(d, S::BK);
  a.ntq = cdiv(a.B, S::TQ);
  const double ops = (SL == 1 ? 1.0 : 3.0) * 2.0 * (double)a.ntg * q8s::TG * a.ntq * S::TQ * a.nk * S::BK;
  CK(hipFuncSetAttribute((const void*)q8s::tile_kernel<SL, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const unsigned grid = (unsigned)(a.ntq * a.ntg);
  hipLaunchKernelGGL((q8s::tile_kernel<SL, MODE>), dim3(grid), dim3(S::NT), S::LDS, 0, a);
  CK(hipGetLastError());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((q8s::tile_kernel<SL, MODE>), dim3(grid), dim3(S::NT), S::LDS, 0, a);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)grid * a.nk * S::STAGE;
  printf("SL=%d %-8s mode=%d gg=%-3ld ms=%8.2f  executed=%7.1f TOPS (%.1f%% of 5000)  LDS-fill=%6.2f TB/s\n", SL, tag,
         MODE, (long)a.gg, ms, ops / ms / 1e9, ops / ms / 1e9 / 50.0, bytes / ms / 1e9);
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t B = argc > 2 ? atoll(argv[2]) : 4096;
  const int64_t d = argc > 3 ? atoll(argv[3]) : 9999;
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  const int64_t ld = 2 * round_up(d, 128);   // fits both layouts
  int8_t *G, *Q;
  float *gs, *aux, *qs;
  Cand* cand;
  CK(hipMalloc(&G, N * ld));
  CK(hipMalloc(&Q, B * ld));
  CK(hipMalloc(&gs, N * 4)); CK(hipMalloc(&aux, N * 4)); CK(hipMalloc(&qs, B * 4));
  const int64_t ntg = cdiv(N, q8s::TG);
  CK(hipMalloc(&cand, ntg * B * q8s::KC * sizeof(Cand)));
  fill_i8<<<4096, 256>>>(G, N * ld, 1);
  fill_i8<<<4096, 256>>>(Q, B * ld, 3);
  fill_f<<<1024, 256>>>(gs, N, 1.f); fill_f<<<1024, 256>>>(aux, N, 1.f); fill_f<<<64, 256>>>(qs, B, 1.f);
  CK(hipDeviceSynchronize());
  q8s::TileArgs a;
  a.G = G; a.N = N; a.ld = ld; a.gscale = gs; a.aux = aux;
  a.Q = Q; a.B = B; a.qscale = qs; a.cand = cand; a.ntg = ntg;
  printf("N=%ld B=%ld d=%ld\n", (long)N, (long)B, (long)d);
  {
    int *seed, *outv;
    CK(hipMalloc(&seed, 256 * 4)); CK(hipMalloc(&outv, 1024 * 256 * 4));
    fill_f<<<1, 256>>>((float*)seed, 256, 1.2345f);
    const int iters = 20000, grid = 1024;
    hipLaunchKernelGGL(mfma_ceiling, dim3(grid), dim3(256), 0, 0, seed, 100, outv);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(mfma_ceiling, dim3(grid), dim3(256), 0, 0, seed, iters, outv);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = 2.0 * 32 * 32 * 32 * 16.0 * iters * 4.0 * grid;
    printf("mfma ceiling (registers only): %.1f TOPS (%.1f%% of 5000)\n", ops / ms / 1e9, ops / ms / 1e9 / 50.0);
  }
  const int ggs[] = {1, 2, 4, 8};
  for (int g : ggs) {
    a.gg = g < ntg ? g : ntg;
    if (run<1, 0>(a, d, reps, "search")) return 1;
  }
  a.gg = 4 < ntg ? 4 : ntg;
  if (run<1, 1>(a, d, reps, "no-dma")) return 1;
  if (run<1, 2>(a, d, reps, "no-mfma")) return 1;
  if (run<2, 0>(a, d, reps, "search")) return 1;
  if (run<2, 1>(a, d, reps, "no-dma")) return 1;
  if (run<2, 2>(a, d, reps, "no-mfma")) return 1;
  return 0;
}
