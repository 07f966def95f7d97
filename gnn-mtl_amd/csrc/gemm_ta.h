// Full-width weight-gradient GEMM (gemm_ta.hip): dW partials = Aᵀ·B for A [K][M], B [K][N] with
// M <= 320, N <= 320, written as split-K fp32 slabs that the caller reduces (k_gemm_reduce /
// k_gemm_bf16_reduce).  Internal to libgnnea (no C-ABI entry of its own).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gnnea {
bool gemm_ta_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                     const void* B, int es);
int64_t gemm_ta_ws_bytes(int64_t M, int64_t N, int64_t K);
// dbslab_out != null (gemm_ta_db_applies): also the column sums of A as splits x M partials
// (B's padding column N read as ones), workspace gemm_ta_db_ws_bytes; ta_db_reduce sums them
bool gemm_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                        const void* B, int es);
int ta_db_reduce(int64_t M, int splits, const float* part, float* db, hipStream_t s);
int64_t gemm_ta_db_ws_bytes(int64_t M, int64_t N, int64_t K);
template <typename T>
int gemm_ta_launch(int64_t M, int64_t N, int64_t K, const T* A, int64_t lda, const T* B,
                   int64_t ldb, void* ws, int64_t ws_bytes, hipStream_t s, float** slab_out,
                   int* splits_out, float** dbslab_out = nullptr);
}  // namespace gnnea
