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
__device__ __forceinline__ T wave_sum_shfl(T v) {
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

// Sums over the 64 lanes without the LDS path: DPP quad / half-row / row mirrors leave every lane
// of a 16-lane row with that row's sum, then the four row sums are read as scalars and added in
// row order.  Every lane ends with the same value.
template <int CTRL>
__device__ __forceinline__ double mov_dpp_f64(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((long long)(unsigned)lo) | ((long long)hi << 32));
}
template <int CTRL>
__device__ __forceinline__ float mov_dpp_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL,
                                                            0xf, 0xf, false));
}
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += mov_dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += mov_dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += mov_dpp_f64<0x141>(v);  // row_half_mirror
  v += mov_dpp_f64<0x140>(v);  // row_mirror
  return ((readlane_d(v, 0) + readlane_d(v, 16)) + readlane_d(v, 32)) + readlane_d(v, 48);
}
__device__ __forceinline__ float wave_sum_f32(float v) {
  v += mov_dpp_f32<0xB1>(v);
  v += mov_dpp_f32<0x4E>(v);
  v += mov_dpp_f32<0x141>(v);
  v += mov_dpp_f32<0x140>(v);
  return ((readlane_f(v, 0) + readlane_f(v, 16)) + readlane_f(v, 32)) + readlane_f(v, 48);
}

// sum over the wave, every lane gets the result: VALU-only (DPP / permlane) for f32 and f64
template <typename T>
__device__ __forceinline__ T wave_sum(T v) { return wave_sum_shfl(v); }
template <>
__device__ __forceinline__ float wave_sum<float>(float v) { return wave_sum_f32(v); }
template <>
__device__ __forceinline__ double wave_sum<double>(double v) { return wave_sum_f64(v); }

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

// act_fwd<GNNEA_ACT_RELU> on four values (x > 0 ? x : 0, the library's relu everywhere)
__device__ __forceinline__ float4 f4_relu(float4 v) {
  return make_float4(v.x > 0.f ? v.x : 0.f, v.y > 0.f ? v.y : 0.f, v.z > 0.f ? v.z : 0.f,
                     v.w > 0.f ? v.w : 0.f);
}

__device__ __forceinline__ float4 f4_fma(float a, float4 x, float4 acc) {
  acc.x = fmaf(a, x.x, acc.x);
  acc.y = fmaf(a, x.y, acc.y);
  acc.z = fmaf(a, x.z, acc.z);
  acc.w = fmaf(a, x.w, acc.w);
  return acc;
}

// The HighWay gate g = sigmoid(gate_pre + b) (layers/layers.py:71): the hardware exponential and
// reciprocal (v_exp_f32 of x log2 e, v_rcp_f32; a few ulp, ~1e-6 relative at |x| ~ 10) instead of
// the library expf and an IEEE division (about 25 instructions per element, which made the
// backward that recomputes g slower than reading a stored one).  Every kernel that forms the
// gate calls this one function, so a forward's and a backward's g are the same bits.
__device__ __forceinline__ float gate_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}

// bf16 storage (cfg-5): 16-bit brain floats carried as uint16_t, arithmetic in fp32.
// f32 -> bf16 rounds to nearest even with NaN -> 0x7fc0, bit-identical to c10::BFloat16.
typedef uint16_t bf16_t;
__device__ __forceinline__ float bf16_to_f32(bf16_t b) {
  return __builtin_bit_cast(float, (uint32_t)b << 16);
}
__device__ __forceinline__ bf16_t f32_to_bf16(float f) {
  const uint32_t u = __builtin_bit_cast(uint32_t, f);
  if (f != f) return (bf16_t)0x7fc0;
  return (bf16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// Four consecutive elements of a feature row: one 16-B (fp32) or 8-B (bf16) load per lane.
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  typedef float4 raw;
  static __device__ __forceinline__ float4 get(const raw& r) { return r; }
  static __device__ __forceinline__ raw put(float4 v) { return v; }
  static __device__ __forceinline__ raw zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }
};
template <> struct Vec4<bf16_t> {
  typedef uint2 raw;
  static __device__ __forceinline__ raw zero() { return make_uint2(0u, 0u); }
  static __device__ __forceinline__ float4 get(const raw& r) {
    return make_float4(__builtin_bit_cast(float, r.x << 16),
                       __builtin_bit_cast(float, r.x & 0xffff0000u),
                       __builtin_bit_cast(float, r.y << 16),
                       __builtin_bit_cast(float, r.y & 0xffff0000u));
  }
  static __device__ __forceinline__ raw put(float4 v) {
    raw r;
    r.x = (uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
    r.y = (uint32_t)f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16);
    return r;
  }
};
// 16 bytes of a feature row: 4 fp32 or 8 bf16 values
__device__ __forceinline__ void unpack16(const uint4& u, float (&f)[4]) {
  f[0] = __builtin_bit_cast(float, u.x);
  f[1] = __builtin_bit_cast(float, u.y);
  f[2] = __builtin_bit_cast(float, u.z);
  f[3] = __builtin_bit_cast(float, u.w);
}
__device__ __forceinline__ void unpack16(const uint4& u, float (&f)[8]) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = __builtin_bit_cast(float, w[k] << 16);
    f[2 * k + 1] = __builtin_bit_cast(float, w[k] & 0xffff0000u);
  }
}

template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16_t>(bf16_t v) { return bf16_to_f32(v); }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t from_f32<bf16_t>(float v) { return f32_to_bf16(v); }

// ---- the x3 split (fp32 GEMMs on the bf16 matrix cores): x = h + m + l, each bf16, round to
// nearest even: h = bf16(x), m = bf16(x - h), l = bf16(x - h - m).  Two elements at a time into
// packed bf16 pairs (dword q of an 8-element MFMA operand holds elements 2q, 2q + 1): one
// v_cvt_pk_bf16_f32 per level, the residuals as packed fp32 subtractions -- the same values as
// element-wise casts with about half the vector instructions.
typedef float x3_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 x3_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t x3_cvt2(x3_f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, x3_bf16x2));
}
__device__ __forceinline__ x3_f32x2 x3_unpk(uint32_t p) {  // a packed bf16 pair -> two fp32
  return x3_f32x2{__builtin_bit_cast(float, p << 16), __builtin_bit_cast(float, p & 0xffff0000u)};
}
__device__ __forceinline__ void x3_split_pair(float x0, float x1, uint32_t& h, uint32_t& m,
                                              uint32_t& l) {
  const x3_f32x2 xv = {x0, x1};
  h = x3_cvt2(xv);
  const x3_f32x2 r = xv - x3_unpk(h);
  m = x3_cvt2(r);
  l = x3_cvt2(r - x3_unpk(m));
}

inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }

// fp64 exp for the log-sum-exp inner loops (arguments are shifted logits, x <= ~0):
// n = rint(x / ln2), r = x - n ln2 (two-step Cody-Waite, |r| <= 0.347), degree-12 Taylor in
// Horner form (truncation 4e-17 relative), scaled by 2^n with ldexp (gradual underflow to 0).
// Relative error <= ~4e-16 against exp() on [-745, 709]; returns 0 below -745.2 (and for
// -inf), like exp().  About half the instructions of the libm path, whose range checks and
// per-call fp64 literal materialisation dominate the Sinkhorn row / column passes.
__device__ __forceinline__ double exp_f64(double x) {
  constexpr double kLog2e = 1.4426950408889634074;
  constexpr double kLn2Hi = 6.93147180369123816490e-01;
  constexpr double kLn2Lo = 1.90821492927058770002e-10;
  const double n = __builtin_rint(x * kLog2e);
  double r = __builtin_fma(-n, kLn2Hi, x);
  r = __builtin_fma(-n, kLn2Lo, r);
  double p = 2.08767569878680989792e-09;                 // 1/12!
  p = __builtin_fma(p, r, 2.50521083854417187751e-08);   // 1/11!
  p = __builtin_fma(p, r, 2.75573192239858906526e-07);   // 1/10!
  p = __builtin_fma(p, r, 2.75573192239858906526e-06);   // 1/9!
  p = __builtin_fma(p, r, 2.48015873015873015873e-05);   // 1/8!
  p = __builtin_fma(p, r, 1.98412698412698412698e-04);   // 1/7!
  p = __builtin_fma(p, r, 1.38888888888888888889e-03);   // 1/6!
  p = __builtin_fma(p, r, 8.33333333333333333333e-03);   // 1/5!
  p = __builtin_fma(p, r, 4.16666666666666666667e-02);   // 1/4!
  p = __builtin_fma(p, r, 1.66666666666666666667e-01);   // 1/3!
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p = __builtin_fma(p, r, 1.0);
  const double y = __builtin_ldexp(p, (int)n);
  return x < -745.2 ? 0.0 : y;
}

// ---- GAT helpers shared by gat.hip and gat_sliced.hip ----
template <int H>
__device__ __forceinline__ float hsel(const float (&w)[H], int h) {
  float r = w[0];
#pragma unroll
  for (int k = 1; k < H; ++k) r = (h == k) ? w[k] : r;
  return r;
}

__device__ __forceinline__ float lrelu(float z, float alpha) { return z > 0.f ? z : alpha * z; }

// Sums of NV values over each head's LPH lanes at once, by reduce-scatter: DPP steps on lane bits
// 3 (row_mirror, only when a head spans whole rows), 2 (row_half_mirror), 1 (quad reverse), 0
// (quad swap) each pair a lane with a partner that agrees on the bits split before, halving the
// live values; heads wider than a row add xor-16 / xor-32 steps on the one remaining value.
// Afterwards lane h*LPH + grp_lane<NV, LPH>(v) holds head h's full sum of value v.
template <int CTRL, int CNT, int NV>
__device__ __forceinline__ void rs_step(float (&p)[NV], bool up) {
  if constexpr (CNT > 1) {
    constexpr int half = CNT / 2;
#pragma unroll
    for (int t = 0; t < half; ++t) {
      const float keep = up ? p[t + half] : p[t];
      const float send = up ? p[t] : p[t + half];
      p[t] = keep + mov_dpp_f32<CTRL>(send);
    }
  } else {
    p[0] += mov_dpp_f32<CTRL>(p[0]);
  }
}
template <int NV, int LPH>
__device__ __forceinline__ float grp_sum(float (&p)[NV], int lane) {
  static_assert(LPH >= 8 && (NV & (NV - 1)) == 0 && NV <= (LPH >= 16 ? 16 : 8), "grp_sum shape");
  if constexpr (LPH >= 16) {
    rs_step<0x140, NV, NV>(p, lane & 8);      // row_mirror: lane ^ 15
    rs_step<0x141, NV / 2, NV>(p, lane & 4);  // row_half_mirror: lane ^ 7
    rs_step<0x1B, NV / 4, NV>(p, lane & 2);   // quad_perm [3,2,1,0]: lane ^ 3
    rs_step<0xB1, NV / 8, NV>(p, lane & 1);   // quad_perm [1,0,3,2]: lane ^ 1
  } else {
    rs_step<0x141, NV, NV>(p, lane & 4);
    rs_step<0x1B, NV / 2, NV>(p, lane & 2);
    rs_step<0xB1, NV / 4, NV>(p, lane & 1);
  }
  float v = p[0];
  if constexpr (LPH >= 32) v += __shfl_xor(v, 16, 64);
  if constexpr (LPH >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
template <int NV, int LPH>
__device__ __forceinline__ constexpr int grp_lane(int v) { return v * ((LPH >= 16 ? 16 : 8) / NV); }

// The same reduce-scatter over the whole wave with max (order-free, so exact), and the all-reduce
// forms: every lane ends with all NV values (reduce-scatter, then one scalar read per value) --
// NV values for the price of about one wave_sum instead of NV of them.
template <int CTRL, int CNT, int NV>
__device__ __forceinline__ void rs_step_max(float (&p)[NV], bool up) {
  if constexpr (CNT > 1) {
    constexpr int half = CNT / 2;
#pragma unroll
    for (int t = 0; t < half; ++t) {
      const float keep = up ? p[t + half] : p[t];
      const float o = mov_dpp_f32<CTRL>(up ? p[t] : p[t + half]);
      p[t] = o > keep ? o : keep;
    }
  } else {
    const float o = mov_dpp_f32<CTRL>(p[0]);
    p[0] = o > p[0] ? o : p[0];
  }
}
template <int NV>
__device__ __forceinline__ float grp_max64(float (&p)[NV], int lane) {
  static_assert((NV & (NV - 1)) == 0 && NV <= 16, "grp_max64 shape");
  rs_step_max<0x140, NV, NV>(p, lane & 8);
  rs_step_max<0x141, NV / 2, NV>(p, lane & 4);
  rs_step_max<0x1B, NV / 4, NV>(p, lane & 2);
  rs_step_max<0xB1, NV / 8, NV>(p, lane & 1);
  float v = p[0], w = __shfl_xor(v, 16, 64);
  v = w > v ? w : v;
  w = __shfl_xor(v, 32, 64);
  return w > v ? w : v;
}
template <int NV>
__device__ __forceinline__ void wave_allsum(float (&p)[NV], int lane) {
  const float r = grp_sum<NV, 64>(p, lane);
#pragma unroll
  for (int v = 0; v < NV; ++v) p[v] = readlane_f(r, grp_lane<NV, 64>(v));
}
template <int NV>
__device__ __forceinline__ void wave_allmax(float (&p)[NV], int lane) {
  const float r = grp_max64<NV>(p, lane);
#pragma unroll
  for (int v = 0; v < NV; ++v) p[v] = readlane_f(r, grp_lane<NV, 64>(v));
}

}  // namespace gnnea
