// Order-preserving u32 keys of coarse scores and the sorted key lists the tile epilogues keep
// (shared by the int8 / fp6 search tiers, ofr_knn_q8.hip, and the chi-square MFMA pass, ofr_chi2.hip).
// A coarse score becomes an order-preserving u32 whose low 8 bits are replaced by the row's index
// inside a 256-row tile: u32 order = (score, index) order with the score truncated by < 256 ulp
// toward -inf.  A sorted list of keys takes a new key with one v_med3_u32 per slot, no compares on
// indices, no branches.  The truncated value is a LOWER bound of the fp32 coarse score, the side
// the certificates need.
#pragma once
#include "ofr_common.h"

namespace ofr {
namespace keys {

constexpr int KC = 16;   // keys per list
constexpr uint32_t KEY_NONE = 0xffffffffu;

__device__ __forceinline__ uint32_t score_key(float sc, int local) {
  const uint32_t b = __float_as_uint(sc);
  const uint32_t m = (uint32_t)((int32_t)b >> 31) | 0x80000000u;
  return ((b ^ m) & ~0xffu) | (uint32_t)local;
}
__device__ __forceinline__ float key_score(uint32_t k) {
  const uint32_t t = k & ~0xffu;
  return __uint_as_float((t & 0x80000000u) ? (t ^ 0x80000000u) : ~t);
}
// the float whose order key is u (inverse of the map in score_key; 0xffffffff -> NaN)
__device__ __forceinline__ float key_float(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u ^ 0x80000000u) : ~u);
}
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return a < b ? b : a; }
// median of three = clamp(v, lo, hi) for lo <= hi (the compiler cannot prove lo <= hi itself)
__device__ __forceinline__ uint32_t med3(uint32_t v, uint32_t lo, uint32_t hi) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(v), "v"(lo), "v"(hi));
  return r;
}

struct KeyList {  // KC keys, ascending
  uint32_t k[KC];
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int j = 0; j < KC; ++j) k[j] = KEY_NONE;
  }
  __device__ __forceinline__ void insert(uint32_t v) {
#pragma unroll
    for (int j = KC - 1; j > 0; --j) k[j] = med3(v, k[j - 1], k[j]);
    k[0] = umin(v, k[0]);
  }
  // best KC of this ascending list and another ascending list (bitonic merge)
  __device__ __forceinline__ void merge(const uint32_t (&o)[KC]) {
#pragma unroll
    for (int j = 0; j < KC; ++j) k[j] = umin(k[j], o[KC - 1 - j]);
#pragma unroll
    for (int s = KC / 2; s > 0; s >>= 1)
#pragma unroll
      for (int j = 0; j < KC; ++j)
        if ((j & s) == 0) {
          const uint32_t x = k[j], y = k[j + s];
          k[j] = umin(x, y);
          k[j + s] = umax(x, y);
        }
  }
};

}  // namespace keys
}  // namespace ofr
