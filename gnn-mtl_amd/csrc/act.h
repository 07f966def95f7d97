// Row-major activation passes shared by the GEMM entry points (act.hip): the act applied in place
// to a GEMM output whose kernel has no fused epilogue for it.  Internal to libgnnea.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace gnnea {
int act_rows_f32(float* C, int64_t ldc, int64_t M, int64_t N, int act, hipStream_t s);
int act_rows_bf16(bf16_t* C, int64_t ldc, int64_t M, int64_t N, int act, hipStream_t s);
}  // namespace gnnea
