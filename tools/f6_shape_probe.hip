// Shape probe for the fp6 search engine (diagnostic tool, not part of the library):
// v_mfma_scale_f32_16x16x128_f8f6f4 against v_mfma_scale_f32_32x32x64_f8f6f4, both operands fp6 e2m3.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/f6_shape_probe.hip -o tools/f6_shape_probe
// 1. layout of the 16x16x128 form: lane l holds A[row l%16][k = 32 (l/16) + j] (and B[k][col l%16]),
//    j = 0..31 as the same 192-bit stream as the 32x32x64 form; C/D: col = lane % 16,
//    row = 4 (lane / 16) + reg.  Checked against the exact host product.
// 2. sustained rate on random operands, every CU, 2 waves per SIMD, a 128 x 64 output tile per wave
//    (8 accumulators of 32x32 or 32 of 16x16), operands (a) in registers, (b) re-read from LDS
//    every MFMA step (the search engine's fragment traffic, no DMA).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static double e2m3(int c) {
  const int s = (c >> 5) & 1, e = (c >> 3) & 3, m = c & 7;
  const double v = e == 0 ? m / 8.0 : std::ldexp(1.0 + m / 8.0, e - 1);
  return s ? -v : v;
}

__global__ void one16(const i32x8* a, const i32x8* b, float* out) {
  const int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], acc, 2, 2, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

template <int SHAPE, bool LDS>
__global__ void __launch_bounds__(512, 1) rate(const int* seed, int iters, float* out) {
  __shared__ __attribute__((aligned(16))) char lds[65536];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 65536 / 4; i += 512) reinterpret_cast<int*>(lds)[i] = seed[i & 255] ^ (i * 0x9e3779b9);
  __syncthreads();
  constexpr int NA = SHAPE == 32 ? 4 : 8, NB = SHAPE == 32 ? 2 : 4;   // fragments per step (128 x 64 tile)
  constexpr int NACC = NA * NB;
  i32x8 a[NA], b[NB];
  for (int i = 0; i < NA; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = e < 6 ? seed[(threadIdx.x + 7 * i + e) & 255] : 0;
  for (int i = 0; i < NB; ++i)
    for (int e = 0; e < 8; ++e) b[i][e] = e < 6 ? seed[(threadIdx.x + 13 * i + 3 * e) & 255] : 0;
  const int s = 0x7f7f7f7f;
  using Acc = typename std::conditional<SHAPE == 32, f32x16, f32x4>::type;
  Acc acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < (SHAPE == 32 ? 16 : 4); ++r) acc[i][r] = 0.f;
  // per step: SHAPE 32 does two k-halves of 64 (16 MFMAs), SHAPE 16 one k of 128 (32 MFMAs)
  for (int it = 0; it < iters; ++it) {
    if constexpr (LDS) {
      const int base = ((it & 3) * 12288 + wave * 1536) & 0xffff;
      for (int i = 0; i < NA; ++i) {
        const char* p = lds + ((base + i * 1536 + lane * 16) & 0xfff0);
        const i32x4 p0 = *reinterpret_cast<const i32x4*>(p);
        const i32x2 p1 = *reinterpret_cast<const i32x2*>(lds + ((base + 8192 + i * 512 + lane * 8) & 0xfff8));
        a[i][0] = p0[0]; a[i][1] = p0[1]; a[i][2] = p0[2]; a[i][3] = p0[3]; a[i][4] = p1[0]; a[i][5] = p1[1];
      }
      for (int i = 0; i < NB; ++i) {
        const char* p = lds + ((base + 20000 + i * 1536 + lane * 16) & 0xfff0);
        const i32x4 p0 = *reinterpret_cast<const i32x4*>(p);
        const i32x2 p1 = *reinterpret_cast<const i32x2*>(lds + ((base + 40000 + i * 512 + lane * 8) & 0xfff8));
        b[i][0] = p0[0]; b[i][1] = p0[1]; b[i][2] = p0[2]; b[i][3] = p0[3]; b[i][4] = p1[0]; b[i][5] = p1[1];
      }
    }
    if constexpr (SHAPE == 32) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < NA; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j)
            acc[i * NB + j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[i], b[j], acc[i * NB + j], 2, 2, 0, s, 0, s);
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i * NB + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i * NB + j], 2, 2, 0, s, 0, s);
    }
  }
  float t = 0.f;
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < (SHAPE == 32 ? 16 : 4); ++r) t += acc[i][r];
  if (t == 1.2345f) out[0] = t;
}

template <int SHAPE, bool LDS>
static void time_rate(const int* seed, float* out, const char* tag) {
  const int cus = 256, iters = 4000;
  const int grid = cus * 1;   // one 512-thread workgroup per CU = 2 waves per SIMD
  hipLaunchKernelGGL((rate<SHAPE, LDS>), dim3(grid), dim3(512), 0, 0, seed, 100, out);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // ~2 s of back-to-back launches: the clock the chip holds under this load
  float ms = 0.f;
  int reps = 0;
  CK(hipEventRecord(e0));
  for (reps = 0; reps < 40; ++reps) hipLaunchKernelGGL((rate<SHAPE, LDS>), dim3(grid), dim3(512), 0, 0, seed, iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double ops = 2.0 * 128 * 64 * 128 * (double)iters * 8 /* waves */ * grid * reps;
  printf("%-28s %8.1f ms  %7.1f TOPS (%.1f%% of 10000)\n", tag, ms, ops / ms / 1e9, ops / ms / 1e9 / 100.0);
  fflush(stdout);
}

int main() {
  // 1. layout of the 16x16x128 form
  std::vector<int> codeA(16 * 128), codeB(128 * 16);
  uint32_t st = 777;
  auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (int)(st >> 26); };
  for (auto& c : codeA) c = rnd();
  for (auto& c : codeB) c = rnd();
  std::vector<i32x8> fa(64), fb(64);
  for (int l = 0; l < 64; ++l) {
    uint32_t wa[8] = {0}, wb[8] = {0};
    for (int j = 0; j < 32; ++j) {
      const int k = 32 * (l / 16) + j, bit = 6 * j;
      const uint32_t ca = codeA[(l % 16) * 128 + k], cb = codeB[k * 16 + (l % 16)];
      wa[bit >> 5] |= ca << (bit & 31);
      wb[bit >> 5] |= cb << (bit & 31);
      if ((bit & 31) > 26) { wa[(bit >> 5) + 1] |= ca >> (32 - (bit & 31)); wb[(bit >> 5) + 1] |= cb >> (32 - (bit & 31)); }
    }
    for (int e = 0; e < 8; ++e) { fa[l][e] = (int)wa[e]; fb[l][e] = (int)wb[e]; }
  }
  i32x8 *da, *db;
  float* dout;
  CK(hipMalloc(&da, 64 * sizeof(i32x8))); CK(hipMalloc(&db, 64 * sizeof(i32x8))); CK(hipMalloc(&dout, 4096 * 4));
  CK(hipMemcpy(da, fa.data(), 64 * sizeof(i32x8), hipMemcpyHostToDevice));
  CK(hipMemcpy(db, fb.data(), 64 * sizeof(i32x8), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(one16, dim3(1), dim3(64), 0, 0, da, db, dout);
  std::vector<float> got(256);
  CK(hipMemcpy(got.data(), dout, 256 * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * (l / 16) + r, col = l % 16;
      double ref = 0;
      for (int k = 0; k < 128; ++k) ref += e2m3(codeA[row * 128 + k]) * e2m3(codeB[k * 16 + col]);
      if (std::fabs(ref - got[l * 4 + r]) > 1e-3 * (1 + std::fabs(ref))) ++bad;
    }
  printf("16x16x128 fp6 layout: %s (%d mismatches of 256)\n", bad ? "FAIL" : "OK", bad);
  // 2. rates
  int* seed;
  CK(hipMalloc(&seed, 256 * 4));
  std::vector<int> sv(256);
  for (auto& v : sv) v = (int)(rnd() * 0x01041041u) ^ (int)(st);
  CK(hipMemcpy(seed, sv.data(), 256 * 4, hipMemcpyHostToDevice));
  for (int rep = 0; rep < 2; ++rep) {
    time_rate<32, false>(seed, dout, "32x32x64 regs");
    time_rate<16, false>(seed, dout, "16x16x128 regs");
    time_rate<32, true>(seed, dout, "32x32x64 lds-frags");
    time_rate<16, true>(seed, dout, "16x16x128 lds-frags");
  }
  return 0;
}
