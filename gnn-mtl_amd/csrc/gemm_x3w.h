// Weight-resident fp32 projection GEMM through the three-way bf16 split (gemm_x3w.hip): C = A·op(B)
// (+ bias + beta·C, then relu when act = GNNEA_ACT_RELU) for tall A with K in (288, 320].  Internal to libgnnea (gemm.hip's gemm_x3 dispatches
// to it; no C-ABI entry of its own).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gnnea {
bool gemm_x3w_applies(int trans_a, int64_t M, int64_t N, int64_t K, int64_t lda, const void* A,
                      float beta, int64_t ldc, int64_t cs, const void* C, const void* C2,
                      int64_t cs2, int act = 0);
int64_t gemm_x3w_ws_bytes(int64_t N);
int gemm_x3w_launch(int trans_b, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                    const float* B, int64_t ldb, const float* bias, float* C, int64_t ldc,
                    int64_t cs, float* C2, int64_t cs2, void* ws, int64_t ws_bytes,
                    hipStream_t s, float beta = 0.f, int act = 0);
// the relu Linear's sign bits (k_gemm_f16x2_ring's epilogue modes 3 / 2): 16 bytes per row and
// 112-column tile; only K in (288, 320] at N <= 336 on the default f16x2 form
int64_t f16x2_mask_ld(int64_t N);
bool f16x2_mask_applies(int64_t M, int64_t N, int64_t K, int64_t lda, const void* A, int64_t ldc,
                        const void* C);
int f16x2_mask_launch(int ep, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                      int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                      int64_t ldc, const uint8_t* Mi, uint8_t* Mo, int64_t ldm, void* ws,
                      int64_t ws_bytes, hipStream_t s);
}  // namespace gnnea
