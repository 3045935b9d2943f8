// Feed probe (diagnostic tool, not part of the library): how fast can a workgroup per CU copy the
// fp6 sieve pass's operand blocks into LDS, as a function of the stage size and of how many
// stages are in flight?  Pure LDS-DMA (MUBUF buffer_load_dwordx4 ... lds, 1 KiB per wave-instruction,
// 8 waves) over the bench shape's tiles: per tile (gallery panel gp, query panel qp) and stage kt
// the gallery block and the query block of the f6 tiled layout (ofr_f6_tile.h), in the library's
// XCD-aware grouped tile order.  Per stage: wait for the own copies of stage kt (counted vmcnt),
// s_barrier, issue stage kt + LEAD into buffer (kt + LEAD) % NBUF -- the library's protocol without
// MFMAs or fragment reads.  Prints ms and the copy rate per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/feed_probe.hip -o tools/feed_probe
//   ./tools/feed_probe [N] [B] [d] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
      return 1;                                                                          \
    }                                                                                    \
  } while (0)

constexpr int PANEL = 24576;   // bytes per (256-row panel, 128-feature stage) block of the f6 tiled layout

__device__ __forceinline__ int64_t xcd_remap(int64_t bid, int64_t nblocks) {
  const int64_t q = nblocks / 8, r = nblocks % 8;
  const int64_t x = bid % 8, s = bid / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + s;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// HALF = 1: a stage is 64 features (12 KiB of each panel block, 24 KiB per stage), else 128 (48 KiB)
template <int HALF, int NBUF, int LEAD>
__global__ void __launch_bounds__(512, 1) feed_kernel(const char* G, const char* Q, int64_t ntg, int64_t ntq, int nst,
                                                      int64_t gg_, int* sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int SB = HALF ? PANEL / 2 : PANEL;   // bytes of one operand per stage
  constexpr int STAGE = 2 * SB, INS = STAGE / 1024, IPW = INS / 8;
  static_assert(NBUF * STAGE <= 160 * 1024 && LEAD < NBUF && IPW * 8 == INS, "shape");
  const int64_t t = xcd_remap(blockIdx.x, (int64_t)gridDim.x);
  const int64_t group = t / (gg_ * ntq), within = t % (gg_ * ntq);
  const int64_t abase = group * gg_;
  const int64_t gg = ntg - abase < gg_ ? ntg - abase : gg_;
  const int64_t qp = within / gg, gp = abase + within % gg;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int pb = nst * PANEL;
  __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(G + gp * (int64_t)pb), 0, pb, 0x00020000);
  __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)(Q + qp * (int64_t)pb), 0, pb, 0x00020000);
  const int steps = HALF ? 2 * nst : nst, last = steps - 1;
  auto issue = [&](int s) {
    const int ks = s < last ? s : last;
    const int src = HALF ? (ks >> 1) * PANEL + (ks & 1) * SB : ks * PANEL;
    char* st = smem + (s % NBUF) * STAGE;
#pragma unroll
    for (int u = 0; u < IPW; ++u) {
      const int ins = wave * IPW + u;
      const bool gal = ins < INS / 2;
      const int off = (gal ? ins : ins - INS / 2) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(gal ? rg : rq, (__attribute__((address_space(3))) void*)(st + (gal ? 0 : SB) + off),
                                               16, src + off + lane * 16, 0, 0, 0);
    }
  };
#pragma unroll
  for (int s = 0; s < LEAD; ++s) issue(s);
  for (int kt = 0; kt < steps; ++kt) {
    wait_vm<(LEAD - 1) * IPW>();   // own copies of stage kt landed; kt+1 .. kt+LEAD-1 may fly
    __builtin_amdgcn_s_barrier();
    issue(kt + LEAD);
  }
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  if (threadIdx.x == 0 && smem[0] == 123 && smem[1] == 45) sink[0] = 1;   // keep the copies observable
}

template <int HALF, int NBUF, int LEAD>
static int run(const char* G, const char* Q, int64_t ntg, int64_t ntq, int nst, int reps, int* sink) {
  constexpr int STAGE = 2 * (HALF ? PANEL / 2 : PANEL);
  const int lds = NBUF * STAGE;
  CK(hipFuncSetAttribute((const void*)feed_kernel<HALF, NBUF, LEAD>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const unsigned grid = (unsigned)(ntg * ntq);
  const int64_t gg = 4;
  hipLaunchKernelGGL((feed_kernel<HALF, NBUF, LEAD>), dim3(grid), dim3(512), lds, 0, G, Q, ntg, ntq, nst, gg, sink);
  CK(hipGetLastError());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((feed_kernel<HALF, NBUF, LEAD>), dim3(grid), dim3(512), lds, 0, G, Q, ntg, ntq, nst, gg, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double bytes = (double)ntg * ntq * nst * 2.0 * PANEL;
  printf("stage %2d KiB  buffers %d  in flight %d (%3d KiB)  ms=%7.2f  %6.2f TB/s  %5.1f GB/s per CU\n",
         STAGE / 1024, NBUF, LEAD, LEAD * STAGE / 1024, ms, bytes / ms / 1e9, bytes / ms / 1e6 / 256.0);
  fflush(stdout);
  return 0;
}

__global__ void fill(char* p, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (char)(i * 2654435761u >> 13);
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t B = argc > 2 ? atoll(argv[2]) : 4096;
  const int64_t d = argc > 3 ? atoll(argv[3]) : 9999;
  const int reps = argc > 4 ? atoi(argv[4]) : 3;
  const int64_t ntg = (N + 255) / 256, ntq = (B + 255) / 256;
  const int nst = (int)((d + 127) / 128);
  char *G, *Q;
  int* sink;
  CK(hipMalloc(&G, (size_t)ntg * nst * PANEL));
  CK(hipMalloc(&Q, (size_t)ntq * nst * PANEL));
  CK(hipMalloc(&sink, 4));
  fill<<<4096, 256>>>(G, (size_t)ntg * nst * PANEL);
  fill<<<1024, 256>>>(Q, (size_t)ntq * nst * PANEL);
  CK(hipDeviceSynchronize());
  printf("N=%ld B=%ld d=%ld: %ld tiles x %d stages of 48 KiB\n", (long)N, (long)B, (long)d, (long)(ntg * ntq), nst);
  for (int rep = 0; rep < 2; ++rep) {
    if (run<0, 3, 1>(G, Q, ntg, ntq, nst, reps, sink) || run<0, 3, 2>(G, Q, ntg, ntq, nst, reps, sink) ||
        run<1, 6, 2>(G, Q, ntg, ntq, nst, reps, sink) || run<1, 6, 3>(G, Q, ntg, ntq, nst, reps, sink) ||
        run<1, 6, 4>(G, Q, ntg, ntq, nst, reps, sink) || run<1, 6, 5>(G, Q, ntg, ntq, nst, reps, sink))
      return 1;
  }
  return 0;
}
