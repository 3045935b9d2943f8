// Compile-time probe: can the fp6 sieve pass take a dedicated producer wave?
// The sieve kernel's 8 MFMA waves each hold 128 fp32 accumulators + 72 fragment registers (~233
// VGPRs, 2 waves per SIMD).  A 9th wave that only issues the stage copies must live on one of the
// four SIMDs beside two MFMA waves -- but a kernel's VGPR allocation is ONE number for all of its
// waves, so a 576-thread workgroup must fit three waves of that allocation on a SIMD: at most
// floor(512 / 3) = 170 -> 168 registers per wave.  Built here with __launch_bounds__(576, 1) around
// the same Engine16 main loop, the compiler's resource report shows the cap and the spills:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -c tools/producer_wave_probe.hip \
//         -Rpass-analysis=kernel-resource-usage -o /tmp/pw.o
#include "../opencv_facerecognizer_amd/csrc/ofr_f6_tile.h"

using namespace ofr;

template <int NT>
__global__ void __launch_bounds__(NT, 1) sieve_body(const char* G, const char* Q, int nst, float* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f6t::f32x4 acc[8][4];
  if (threadIdx.x < 512) {       // the 8 MFMA waves (a producer wave 8 would only copy)
    f6t::Engine16::mainloop<1024 + 4096 + 8192>(smem, G, blockIdx.x, Q, blockIdx.y, nst, acc);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) s += acc[i][c][0] + acc[i][c][1] + acc[i][c][2] + acc[i][c][3];
    out[blockIdx.x * NT + threadIdx.x] = s;
  }
}

template __global__ void sieve_body<512>(const char*, const char*, int, float*);   // today's kernel
template __global__ void sieve_body<576>(const char*, const char*, int, float*);   // + one producer wave
