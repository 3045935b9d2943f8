// Probe of the block-scaled fp6 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, e2m3 operands) on gfx950
// (diagnostic tool, not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mx_probe.hip -o tools/mx_probe && ./tools/mx_probe
// 1. operand layout: lane l = (h = l >> 5, r = l & 31) holds A[row r][k = 32h + j] and
//    B[k = 32h + j][col r], j = 0..31, as a 192-bit little-endian bit stream (element j at
//    bits 6j..6j+5 of v[0:5]); its E8M0 scale byte (opsel 0) scales that 32-element block.
//    Checked against an exact host product on random codes and scales.
// 2. accumulation numerics: a chain of 160 MFMAs (K = 10240) against the exact sum, error
//    relative to sum |a b|, on random data and on a cancelling sum.
// 2b. the same for v_mfma_scale_f32_16x16x128_f8f6f4 (the sieve engines' MFMA): lane l = (q = l >> 4,
//    r = l & 15) holds A[row r][k = 32q + j] / B[k = 32q + j][col r] and the E8M0 scale of that block;
//    C/D register g of lane l = row 4 (l >> 4) + g, col l & 15.  Per-(row, block) scales 2^-7..2^7 and
//    column-block scales (one byte per 32 features, the same for all rows: the fp6 tier's layout).
// 3. rate: back-to-back scaled fp6 MFMAs on register operands, 1 and 2 waves per SIMD, all
//    CUs, next to v_mfma_i32_32x32x32_i8.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

static double e2m3(int c) {
  const int s = (c >> 5) & 1, e = (c >> 3) & 3, m = c & 7;
  const double v = e == 0 ? m / 8.0 : std::ldexp(1.0 + m / 8.0, e - 1);
  return s ? -v : v;
}

// [nmf][64 lanes][8 dwords] A and B fragments, [nmf][64] scale dwords
__global__ void chain(const i32x8* a, const i32x8* b, const int* sa, const int* sb, int nmf, float* out) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  for (int m = 0; m < nmf; ++m)
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[m * 64 + l], b[m * 64 + l], acc, 2, 2, 0, sa[m * 64 + l], 0,
                                                         sb[m * 64 + l]);
  for (int r = 0; r < 16; ++r) out[l * 16 + r] = acc[r];
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void chain16(const i32x8* a, const i32x8* b, const int* sa, const int* sb, int nmf, float* out) {
  const int l = threadIdx.x;
  f32x4 acc = {};
  for (int m = 0; m < nmf; ++m)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[m * 64 + l], b[m * 64 + l], acc, 2, 2, 0, sa[m * 64 + l], 0,
                                                          sb[m * 64 + l]);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

__global__ void __launch_bounds__(512, 1) rate_fp6(const int* seed, int iters, float* out, long long* stamps) {
  i32x8 a[4], b[2];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = seed[(threadIdx.x + 7 * i + e) & 255];
  for (int i = 0; i < 2; ++i)
    for (int e = 0; e < 8; ++e) b[i][e] = seed[(threadIdx.x + 13 * i + 3 * e) & 255];
  const int s = 0x7f7f7f7f;
  f32x16 acc[4][2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a[i], b[j], acc[i][j], 2, 2, 0, s, 0, s);
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
  float t = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) t += acc[i][j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

__global__ void __launch_bounds__(512, 1) rate_i8(const int* seed, int iters, float* out, long long* stamps) {
  i32x4 a[4], b[2];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 4; ++e) a[i][e] = seed[(threadIdx.x + 7 * i + e) & 255];
  for (int i = 0; i < 2; ++i)
    for (int e = 0; e < 4; ++e) b[i][e] = seed[(threadIdx.x + 13 * i + 3 * e) & 255];
  i32x16 acc[4][2];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    stamps[2 * w] = t1 - t0;
    stamps[2 * w + 1] = r1 - r0;
  }
  int t = 0;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) t += acc[i][j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (float)t;
}

struct Frag {
  std::vector<int> code;   // [nmf][32 rows][64 k] 6-bit codes
  std::vector<int> scale;  // [nmf][32 rows][2 blocks] E8M0
};

static void pack(const Frag& f, int nmf, std::vector<int>& dw, std::vector<int>& sc) {
  dw.assign((size_t)nmf * 64 * 8, 0);
  sc.assign((size_t)nmf * 64, 0);
  for (int m = 0; m < nmf; ++m)
    for (int l = 0; l < 64; ++l) {
      const int h = l >> 5, r = l & 31;
      uint32_t* w = (uint32_t*)&dw[((size_t)m * 64 + l) * 8];
      for (int j = 0; j < 32; ++j) {
        const uint32_t c = (uint32_t)f.code[((size_t)m * 32 + r) * 64 + 32 * h + j] & 63u;
        const int bit = 6 * j;
        w[bit >> 5] |= c << (bit & 31);
        if ((bit & 31) > 26) w[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
      }
      sc[(size_t)m * 64 + l] = f.scale[((size_t)m * 32 + r) * 2 + h];
    }
}

static double run_chain(const Frag& A, const Frag& B, int nmf, double* maxrel, double* maxabs_over_sum, bool print) {
  std::vector<int> ad, as, bd, bs;
  pack(A, nmf, ad, as);
  pack(B, nmf, bd, bs);
  int *da, *dsa, *db, *dsb;
  float* dout;
  CK(hipMalloc(&da, ad.size() * 4)); CK(hipMalloc(&db, bd.size() * 4));
  CK(hipMalloc(&dsa, as.size() * 4)); CK(hipMalloc(&dsb, bs.size() * 4));
  CK(hipMalloc(&dout, 64 * 16 * 4));
  CK(hipMemcpy(da, ad.data(), ad.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bd.data(), bd.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, as.data(), as.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, bs.data(), bs.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, dsa, dsb, nmf, dout);
  CK(hipDeviceSynchronize());
  std::vector<float> out(64 * 16);
  CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
  double worst = 0, worst_abs = 0;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int reg = 0; reg < 16; ++reg) {
      const int col = l & 31, row = (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5);
      double ex = 0, sabs = 0;
      for (int m = 0; m < nmf; ++m)
        for (int k = 0; k < 64; ++k) {
          const double av = e2m3(A.code[((size_t)m * 32 + row) * 64 + k]) *
                            std::ldexp(1.0, A.scale[((size_t)m * 32 + row) * 2 + k / 32] - 127);
          const double bv = e2m3(B.code[((size_t)m * 32 + col) * 64 + k]) *
                            std::ldexp(1.0, B.scale[((size_t)m * 32 + col) * 2 + k / 32] - 127);
          ex += av * bv;
          sabs += std::fabs(av * bv);
        }
      const double got = out[l * 16 + reg];
      const double err = std::fabs(got - ex);
      if (err > 1e-3 * sabs + 1e-30) ++bad;
      if (sabs > 0) worst_abs = std::fmax(worst_abs, err / sabs);
      if (ex != 0) worst = std::fmax(worst, err / std::fabs(ex));
      if (print && l < 2 && reg < 2) printf("   lane %d reg %d: got %.9g exact %.9g\n", l, reg, got, ex);
    }
  *maxrel = worst;
  *maxabs_over_sum = worst_abs;
  CK(hipFree(da)); CK(hipFree(db)); CK(hipFree(dsa)); CK(hipFree(dsb)); CK(hipFree(dout));
  return bad;
}

// 16x16x128: codes [nmf][16 rows][128 k], scales [nmf][16 rows][4 blocks]
static double run_chain16(const Frag& A, const Frag& B, int nmf, double* maxabs_over_sum) {
  std::vector<int> ad((size_t)nmf * 64 * 8, 0), as((size_t)nmf * 64), bd((size_t)nmf * 64 * 8, 0), bs((size_t)nmf * 64);
  auto pk = [&](const Frag& f, std::vector<int>& dw, std::vector<int>& sc) {
    for (int m = 0; m < nmf; ++m)
      for (int l = 0; l < 64; ++l) {
        const int q = l >> 4, r = l & 15;
        uint32_t* w = (uint32_t*)&dw[((size_t)m * 64 + l) * 8];
        for (int j = 0; j < 32; ++j) {
          const uint32_t c = (uint32_t)f.code[((size_t)m * 16 + r) * 128 + 32 * q + j] & 63u;
          const int bit = 6 * j;
          w[bit >> 5] |= c << (bit & 31);
          if ((bit & 31) > 26) w[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
        }
        sc[(size_t)m * 64 + l] = f.scale[((size_t)m * 16 + r) * 4 + q];
      }
  };
  pk(A, ad, as);
  pk(B, bd, bs);
  int *da, *dsa, *db, *dsb;
  float* dout;
  CK(hipMalloc(&da, ad.size() * 4)); CK(hipMalloc(&db, bd.size() * 4));
  CK(hipMalloc(&dsa, as.size() * 4)); CK(hipMalloc(&dsb, bs.size() * 4));
  CK(hipMalloc(&dout, 64 * 4 * 4));
  CK(hipMemcpy(da, ad.data(), ad.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, bd.data(), bd.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, as.data(), as.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, bs.data(), bs.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(chain16, dim3(1), dim3(64), 0, 0, (const i32x8*)da, (const i32x8*)db, dsa, dsb, nmf, dout);
  CK(hipDeviceSynchronize());
  std::vector<float> out(64 * 4);
  CK(hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost));
  double worst_abs = 0;
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int g = 0; g < 4; ++g) {
      const int col = l & 15, row = 4 * (l >> 4) + g;
      double ex = 0, sabs = 0;
      for (int m = 0; m < nmf; ++m)
        for (int k = 0; k < 128; ++k) {
          const double av = e2m3(A.code[((size_t)m * 16 + row) * 128 + k]) *
                            std::ldexp(1.0, A.scale[((size_t)m * 16 + row) * 4 + k / 32] - 127);
          const double bv = e2m3(B.code[((size_t)m * 16 + col) * 128 + k]) *
                            std::ldexp(1.0, B.scale[((size_t)m * 16 + col) * 4 + k / 32] - 127);
          ex += av * bv;
          sabs += std::fabs(av * bv);
        }
      const double err = std::fabs((double)out[l * 4 + g] - ex);
      if (err > 1e-3 * sabs + 1e-30) ++bad;
      if (sabs > 0) worst_abs = std::fmax(worst_abs, err / sabs);
    }
  *maxabs_over_sum = worst_abs;
  CK(hipFree(da)); CK(hipFree(db)); CK(hipFree(dsa)); CK(hipFree(dsb)); CK(hipFree(dout));
  return bad;
}

static Frag rand_frag16(int nmf, uint32_t& s, int smin, int smax, bool colblock) {
  Frag f;
  f.code.resize((size_t)nmf * 16 * 128);
  f.scale.resize((size_t)nmf * 16 * 4);
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; };
  for (auto& c : f.code) c = rnd() & 63;
  for (int m = 0; m < nmf; ++m)
    for (int b = 0; b < 4; ++b) {
      const int cb = smin + (int)(rnd() % (uint32_t)(smax - smin + 1));
      for (int r = 0; r < 16; ++r)
        f.scale[((size_t)m * 16 + r) * 4 + b] = colblock ? cb : smin + (int)(rnd() % (uint32_t)(smax - smin + 1));
    }
  return f;
}

static Frag rand_frag(int nmf, uint32_t& s, int smin, int smax, bool cancel_sign) {
  Frag f;
  f.code.resize((size_t)nmf * 32 * 64);
  f.scale.resize((size_t)nmf * 32 * 2);
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; };
  for (auto& c : f.code) c = rnd() & 63;
  for (auto& c : f.scale) c = smin + (int)(rnd() % (uint32_t)(smax - smin + 1));
  if (cancel_sign)  // alternate signs per mfma so that the running sum cancels
    for (int m = 0; m < nmf; ++m)
      for (int i = 0; i < 32 * 64; ++i) {
        int& c = f.code[(size_t)m * 32 * 64 + i];
        c = (c & 31) | ((m & 1) << 5);
      }
  return f;
}

int main(int argc, char** argv) {
  uint32_t s = 12345;
  double rel, abs_sum;
  // 1. layout: one MFMA, random codes, scales 2^-3..2^3
  {
    Frag A = rand_frag(1, s, 124, 130, false), B = rand_frag(1, s, 124, 130, false);
    const double bad = run_chain(A, B, 1, &rel, &abs_sum, true);
    printf("layout (1 mfma): %s, %d mismatches, max err / sum|ab| = %.3e\n", bad == 0 ? "OK" : "FAIL", (int)bad, abs_sum);
  }
  // subnormal-only codes (exponent 0)
  {
    Frag A = rand_frag(1, s, 127, 127, false), B = rand_frag(1, s, 127, 127, false);
    for (auto& c : A.code) c &= 0x27;
    for (auto& c : B.code) c &= 0x27;
    const double bad = run_chain(A, B, 1, &rel, &abs_sum, false);
    printf("subnormals: %s, %d mismatches, max err / sum|ab| = %.3e\n", bad == 0 ? "OK" : "FAIL", (int)bad, abs_sum);
  }
  // 2. numerics over a K = 10240 chain
  for (int trial = 0; trial < 3; ++trial) {
    Frag A = rand_frag(160, s, 120, 134, false), B = rand_frag(160, s, 120, 134, false);
    const double bad = run_chain(A, B, 160, &rel, &abs_sum, false);
    printf("chain 160 random (scales 2^-7..2^7): %d mismatches, max err / sum|ab| = %.3e (%.2f x 2^-24)\n", (int)bad,
           abs_sum, abs_sum * 16777216.0);
  }
  for (int trial = 0; trial < 3; ++trial) {
    Frag A = rand_frag(160, s, 127, 127, true), B = rand_frag(160, s, 127, 127, false);
    for (auto& c : B.code) c &= 31;
    const double bad = run_chain(A, B, 160, &rel, &abs_sum, false);
    printf("chain 160 cancelling: %d mismatches, max err / sum|ab| = %.3e (%.2f x 2^-24)\n", (int)bad, abs_sum,
           abs_sum * 16777216.0);
  }
  // 2b. the 16x16x128 form
  {
    Frag A = rand_frag16(1, s, 124, 130, false), B = rand_frag16(1, s, 124, 130, false);
    const double bad = run_chain16(A, B, 1, &abs_sum);
    printf("16x16x128 layout (1 mfma, per-lane scales): %s, %d mismatches, max err / sum|ab| = %.3e\n",
           bad == 0 ? "OK" : "FAIL", (int)bad, abs_sum);
  }
  for (int trial = 0; trial < 3; ++trial) {
    Frag A = rand_frag16(80, s, 107, 127, true), B = A;
    Frag Bq = rand_frag16(80, s, 107, 127, true);
    for (size_t i = 0; i < B.scale.size(); ++i) B.code = Bq.code;   // same column-block scales, other codes
    const double bad = run_chain16(A, B, 80, &abs_sum);
    printf("16x16x128 chain 80, column-block scales 2^-20..2^0: %d mismatches, max err / sum|ab| = %.3e (%.2f x 2^-24)\n",
           (int)bad, abs_sum, abs_sum * 16777216.0);
  }
  for (int trial = 0; trial < 3; ++trial) {
    Frag A = rand_frag16(80, s, 120, 134, false), B = rand_frag16(80, s, 120, 134, false);
    const double bad = run_chain16(A, B, 80, &abs_sum);
    printf("16x16x128 chain 80, per-lane scales 2^-7..2^7: %d mismatches, max err / sum|ab| = %.3e (%.2f x 2^-24)\n",
           (int)bad, abs_sum, abs_sum * 16777216.0);
  }
  if (argc > 1) return 0;   // numerics only
  // 3. rate
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int* seed;
  float* out;
  CK(hipMalloc(&seed, 256 * 4));
  std::vector<int> hs(256);
  for (auto& v : hs) { s ^= s << 13; s ^= s >> 17; s ^= s << 5; v = (int)s; }
  CK(hipMemcpy(seed, hs.data(), 256 * 4, hipMemcpyHostToDevice));
  CK(hipMalloc(&out, (size_t)ncu * 512 * 4));
  long long* stamps;
  CK(hipMalloc(&stamps, (size_t)ncu * 8 * 2 * 8));
  std::vector<long long> hst((size_t)ncu * 16);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int iters = 20000;
  for (int rep = 0; rep < 2; ++rep)
    for (int threads : {256, 512}) {
      for (int kind = 0; kind < 2; ++kind) {
        auto launch = [&]() {
          if (kind == 0) hipLaunchKernelGGL(rate_fp6, dim3(ncu), dim3(threads), 0, 0, seed, iters, out, stamps);
          else hipLaunchKernelGGL(rate_i8, dim3(ncu), dim3(threads), 0, 0, seed, iters, out, stamps);
        };
        launch();
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double k = kind == 0 ? 64 : 32;
        const double ops = 2.0 * 32 * 32 * k * 8.0 * iters * (threads / 64) * ncu;
        const int nw = ncu * threads / 64;
        CK(hipMemcpy(hst.data(), stamps, (size_t)nw * 16, hipMemcpyDeviceToHost));
        std::vector<double> cyc, clk;
        for (int w = 0; w < nw; ++w) {
          cyc.push_back((double)hst[2 * w] / (8.0 * iters));
          clk.push_back((double)hst[2 * w] / (double)hst[2 * w + 1] * 0.1);
        }
        std::sort(cyc.begin(), cyc.end());
        std::sort(clk.begin(), clk.end());
        printf("rate %s, %d waves/CU: %.1f ms, %.0f TOPS; per wave %.1f cycles per MFMA (median), clock %.2f GHz\n",
               kind == 0 ? "fp6 scaled 32x32x64" : "i8 32x32x32", threads / 64, ms, ops / ms * 1e-9, cyc[nw / 2],
               clk[nw / 2]);
      }
    }
  return 0;
}
