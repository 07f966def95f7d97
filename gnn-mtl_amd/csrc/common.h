// Shared helpers for the gnnea HIP kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this library:
//  * wave64: a "wave" is 64 lanes; lane = threadIdx.x & 63.
//  * all launches are 256-thread workgroups (4 waves) unless a kernel says otherwise.
//  * the C-ABI never throws: every entry point returns 0, a negative gnnea code
//    (see include/gnnea.h) or a positive hipError_t.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "../../include/gnnea.h"

#define GNNEA_LAUNCH_CHECK()                          \
  do {                                                \
    hipError_t _e = hipGetLastError();                \
    if (_e != hipSuccess) return (int)_e;             \
  } while (0)

#define GNNEA_HIP(expr)                               \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return (int)_e;             \
  } while (0)

namespace gnnea {

constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Wave-uniform wave index inside the workgroup (provably uniform for the compiler).
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float readlane_f(float v, int k) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}
__device__ __forceinline__ int readlane_i(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

__device__ __forceinline__ double readlane_d(double v, int k) {
  long long b = __builtin_bit_cast(long long, v);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  long long r = ((long long)(unsigned)lo) | ((long long)hi << 32);
  return __builtin_bit_cast(double, r);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    T w = __shfl_xor(v, o, 64);
    v = w > v ? w : v;
  }
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5, "XCD swizzle must be
// bijective"): consecutive logical blocks land on the same XCD so that rows that share
// neighbours (ring edges, self loops) share one L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// Activations fused into epilogues.  Codes match include/gnnea.h GNNEA_ACT_*.
template <int ACT>
__device__ __forceinline__ float act_fwd(float x) {
  if constexpr (ACT == GNNEA_ACT_IDENTITY) return x;
  else if constexpr (ACT == GNNEA_ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == GNNEA_ACT_ELU) return x > 0.f ? x : expm1f(x);
  else if constexpr (ACT == GNNEA_ACT_LEAKY_RELU) return x > 0.f ? x : 0.01f * x;
  else if constexpr (ACT == GNNEA_ACT_SIGMOID) return 1.f / (1.f + expf(-x));
  else return tanhf(x);
}

// Derivative expressed through the activation's OUTPUT y (so backward needs only y).
template <int ACT>
__device__ __forceinline__ float act_grad_from_out(float y) {
  if constexpr (ACT == GNNEA_ACT_IDENTITY) return 1.f;
  else if constexpr (ACT == GNNEA_ACT_RELU) return y > 0.f ? 1.f : 0.f;
  else if constexpr (ACT == GNNEA_ACT_ELU) return y > 0.f ? 1.f : y + 1.f;
  else if constexpr (ACT == GNNEA_ACT_LEAKY_RELU) return y > 0.f ? 1.f : 0.01f;
  else if constexpr (ACT == GNNEA_ACT_SIGMOID) return y * (1.f - y);
  else return 1.f - y * y;
}

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  acc.z = fmaf(a, x.z, acc.z);
  acc.w = fmaf(a, x.w, acc.w);
  return acc;
}

inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace gnnea
