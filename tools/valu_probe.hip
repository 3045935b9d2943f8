// VALU throughput probe for the chi-square tile kernel's arithmetic (gfx950): cycles per
// wave-instruction of the candidate instructions, every CU busy, 8 waves per SIMD, independent
// chains (8 accumulators per lane).  Prints one line per instruction:
//   name  ns/launch  wave-instructions/launch  cycles per wave-instruction per SIMD (at 2.4 GHz nominal)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/valu_probe.hip -o tools/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

constexpr int ITER = 4096, CH = 8;

#define BODY(NAME, T, INIT, ...)                                                        \
  __global__ void __launch_bounds__(256) NAME(float* out, float seed) {                \
    T v[CH];                                                                           \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) v[c] = INIT;                        \
    for (int i = 0; i < ITER; ++i) {                                                   \
      _Pragma("unroll") for (int c = 0; c < CH; ++c) { __VA_ARGS__; }                   \
    }                                                                                  \
    float s = 0;                                                                       \
    _Pragma("unroll") for (int c = 0; c < CH; ++c) s += (float)v[c][0];                 \
    if (s == 12345.f) out[threadIdx.x] = s;                                            \
  }

typedef float f1 __attribute__((ext_vector_type(1)));
typedef _Float16 hh1 __attribute__((ext_vector_type(1)));

BODY(k_fma_f32, f1, ((f1){seed + c}), v[c] = (f1){__builtin_fmaf(v[c][0], 1.0001f, 0.5f)})
BODY(k_add_f32, f1, ((f1){seed + c}), v[c] = (f1){v[c][0] + 0.5f})
BODY(k_pk_fma_f32, f2, ((f2){seed + c, seed - c}), v[c] = __builtin_elementwise_fma(v[c], (f2){1.0001f, 1.0001f}, (f2){0.5f, 0.5f}))
BODY(k_pk_add_f32, f2, ((f2){seed + c, seed - c}), v[c] = v[c] + (f2){0.5f, 0.25f})
BODY(k_rcp_f32, f1, ((f1){seed + c}), v[c] = (f1){__builtin_amdgcn_rcpf(v[c][0]) + 1.0f})
BODY(k_pk_add_f16, h2, ((h2){(_Float16)(seed + c), (_Float16)(seed - c)}), v[c] = v[c] + (h2){(_Float16)0.5f, (_Float16)0.25f})
BODY(k_pk_fma_f16, h2, ((h2){(_Float16)(seed + c), (_Float16)(seed - c)}),
     v[c] = __builtin_elementwise_fma(v[c], (h2){(_Float16)1.0f, (_Float16)1.0f}, (h2){(_Float16)0.5f, (_Float16)0.25f}))
BODY(k_rcp_f16, hh1, ((hh1){(_Float16)(seed + c)}), v[c] = (hh1){(_Float16)(__builtin_amdgcn_rcph(v[c][0]) + (_Float16)1.0f)})
BODY(k_dot2_f32_f16, f1, ((f1){seed + c}),
     v[c] = (f1){__builtin_amdgcn_fdot2((h2){(_Float16)1.0f, (_Float16)0.5f}, (h2){(_Float16)seed, (_Float16)c}, v[c][0], false)})

int main() {
  int n_cu = 256;
  const int blocks = n_cu * 8;   // 8 x 256-thread blocks per CU = 8 waves per SIMD
  float* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K {
    const char* name;
    void (*f)(float*, float);
    int ops_per;   // instructions per OP (as written)
  } ks[] = {{"v_fma_f32", k_fma_f32, 1},       {"v_add_f32", k_add_f32, 1},       {"v_pk_fma_f32", k_pk_fma_f32, 1},
            {"v_pk_add_f32", k_pk_add_f32, 1}, {"v_rcp_f32(+add)", k_rcp_f32, 2}, {"v_pk_add_f16", k_pk_add_f16, 1},
            {"v_pk_fma_f16", k_pk_fma_f16, 1}, {"v_rcp_f16(+add)", k_rcp_f16, 2}, {"v_dot2_f32_f16", k_dot2_f32_f16, 1}};
  for (auto& k : ks) {
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.5f);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 1.5f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double waves_per_simd = (double)blocks * 4 / (n_cu * 4);   // 4 waves per block
        const double instr = waves_per_simd * ITER * CH;                 // OPs per SIMD per launch
        const double cyc = (ms / 10 * 1e-3) * 2.4e9 / instr;
        printf("%-18s %9.3f ms/launch  %.2f cycles per OP per SIMD (at 2.4 GHz)\n", k.name, ms / 10, cyc);
      }
    }
  }
  return 0;
}
