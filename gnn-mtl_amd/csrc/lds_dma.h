// LDS-DMA and raw LDS access helpers shared by the persistent MFMA GEMMs (gemm.hip k_gemm_x3p,
// gemm_bf16.hip k_gemm_bf16p): global_load_lds staging (no registers), inline-asm LDS reads and
// writes (hipcc waits vmcnt(0) for an in-flight LDS-DMA before plain LDS accesses, since it
// cannot tell the ring's buffers apart), compile-time loops.
#pragma once
#include "common.h"

namespace gnnea {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__device__ __forceinline__ void glds16(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 16, 0, 0);
}
// 4 B per lane: for sources only 4-B aligned (bf16 rows of 300 elements are 600 B, and a 16-B
// piece of the last row would run past K into the next row / past the allocation)
__device__ __forceinline__ void glds4(const void* g, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)g, (lds_void_t*)lds_wave_base, 4, 0, 0);
}
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const lds_void_t*)p;
}
__device__ __forceinline__ u32x4 ds_read128(uint32_t addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int OFF>  // immediate byte offset (ds_* offsets are 16-bit)
__device__ __forceinline__ u32x4 ds_read128_o(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}
// (a float result type, not a per-element __builtin_bit_cast of a u32x4 lane: hipcc 7.2
// miscompiles bit_cast of an ext-vector element lvalue to element 0)
__device__ __forceinline__ f32x4_t ds_read128f(uint32_t addr) {
  f32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}

template <int I>
struct IntC {
  static constexpr int value = I;
};
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(IntC<I>{});
    static_for<N, I + 1>(f);
  }
}

__device__ __forceinline__ void ds_write32(uint32_t addr, float v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(addr), "v"(v));
}

}  // namespace gnnea
