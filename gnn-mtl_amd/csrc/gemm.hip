// Dense projection on MFMA: C = op(A)·op(B) (+ bias) (+ beta*C), f32 in / f32 accumulate.
// Replaces nn.Linear (layers/layers.py:32,61,93), torch.mm(input, W) (att_layers.py:33) and
// torch.spmm(x, kernel_gate) (layers/layers.py:69), forward and backward.
//
// v_mfma_f32_32x32x2_f32 (gfx950: exact f32, bit-for-bit a k-ordered fmaf chain; 64 FLOP per
// clock per SIMD).  Geometry: 256-thread workgroup = 4 waves in 2x2, block tile 128x128,
// BK = 32, each wave 64x64 = 2x2 MFMA tiles of 32x32 (64 accumulator VGPRs).  Operand tiles
// are staged k-major in LDS ([BK][128+1] floats: column reads by 32 consecutive lanes are
// conflict-free, the +1 pad breaks the transposing writes' bank collisions); the next K-tile
// is prefetched into registers while the current one feeds the MFMAs (async-stage split).
// Large-K / small-output products (weight gradients, K = N_nodes) split K over workgroups into
// fp32 slabs reduced in fixed order by a second kernel: deterministic, no atomics.
#include "common.h"

namespace gnnea {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32, LDT = 129;

template <int TA, int TB>
__global__ __launch_bounds__(256, 2) void k_gemm_f32(int M, int N, int K, const float* __restrict__ A,
                                                     int64_t lda, const float* __restrict__ B,
                                                     int64_t ldb, const float* __restrict__ bias,
                                                     float beta, float* __restrict__ C, int64_t ldc,
                                                     int k_per_split, float* __restrict__ slab,
                                                     int tiles_n) {
  __shared__ float As[BK * LDT];
  __shared__ float Bs[BK * LDT];
  const int tiles = gridDim.x;
  const int t_id = xcd_remap(blockIdx.x, tiles);
  const int bn = t_id % tiles_n, bm = t_id / tiles_n;
  const int m0 = bm * BM, n0 = bn * BN;
  const int split = blockIdx.y;
  const int kb = split * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;

  float ra[16], rb[16];
  // load op(A)[m0:m0+128, k0:k0+32] and op(B)[k0:k0+32, n0:n0+128] into registers
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int m, k;
      if (TA == 0) { k = tid & 31; m = (tid >> 5) + 8 * q; }
      else { m = tid & 127; k = (tid >> 7) + 2 * q; }
      const int gm = m0 + m, gk = k0 + k;
      float v = 0.f;
      if (gm < M && gk < ke) v = TA == 0 ? A[(int64_t)gm * lda + gk] : A[(int64_t)gk * lda + gm];
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int n, k;
      if (TB == 0) { n = tid & 127; k = (tid >> 7) + 2 * q; }
      else { k = tid & 31; n = (tid >> 5) + 8 * q; }
      const int gn = n0 + n, gk = k0 + k;
      float v = 0.f;
      if (gn < N && gk < ke) v = TB == 0 ? B[(int64_t)gk * ldb + gn] : B[(int64_t)gn * ldb + gk];
      rb[q] = v;
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int m, k;
      if (TA == 0) { k = tid & 31; m = (tid >> 5) + 8 * q; }
      else { m = tid & 127; k = (tid >> 7) + 2 * q; }
      As[k * LDT + m] = ra[q];
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      int n, k;
      if (TB == 0) { n = tid & 127; k = (tid >> 7) + 2 * q; }
      else { k = tid & 31; n = (tid >> 5) + 8 * q; }
      Bs[k * LDT + n] = rb[q];
    }
  };

  const int kh = lane >> 5, li = lane & 31;
  if (kb < ke) {
    load_tile(kb);
    for (int k0 = kb; k0 < ke; k0 += BK) {
      __syncthreads();  // previous tile fully consumed
      store_tile();
      __syncthreads();
      if (k0 + BK < ke) load_tile(k0 + BK);  // in flight under the MFMAs
#pragma unroll
      for (int kk = 0; kk < BK; kk += 2) {
        const float a0 = As[(kk + kh) * LDT + wm * 64 + li];
        const float a1 = As[(kk + kh) * LDT + wm * 64 + 32 + li];
        const float b0 = Bs[(kk + kh) * LDT + wn * 64 + li];
        const float b1 = Bs[(kk + kh) * LDT + wn * 64 + 32 + li];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
    }
  }

  // epilogue: 32x32 C/D map  col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int col = n0 + wn * 64 + u * 32 + li;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
        if (row >= M) continue;
        const float v = acc[t][u][r];
        if (slab) {
          slab[((int64_t)split * M + row) * N + col] = v;
        } else {
          float o = v;
          if (bias) o += bias[col];
          if (beta != 0.f) o += beta * C[(int64_t)row * ldc + col];
          C[(int64_t)row * ldc + col] = o;
        }
      }
    }
}

__global__ void k_gemm_reduce(int M, int N, int splits, const float* __restrict__ slab,
                              const float* __restrict__ bias, float beta, float* __restrict__ C,
                              int64_t ldc) {
  const int64_t n = (int64_t)M * N;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < splits; ++q) s += slab[(int64_t)q * n + t];
    const int64_t row = t / N, col = t - row * N;
    if (bias) s += bias[col];
    float* c = C + row * ldc + col;
    if (beta != 0.f) s += beta * *c;
    *c = s;
  }
}

// split-K only when the output grid cannot fill the chip and K is long
static int pick_splits(int64_t M, int64_t N, int64_t K, int64_t ws_bytes) {
  const int64_t tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (tiles >= 512 || K < 4 * BK) return 1;
  int64_t s = (1024 + tiles - 1) / tiles;
  const int64_t by_k = K / (4 * BK);
  if (s > by_k) s = by_k;
  if (s > 256) s = 256;
  while (s > 1 && s * M * N * 4 > ws_bytes) --s;
  return (int)(s < 1 ? 1 : s);
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_gemm_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  return pick_splits(M, N, K, INT64_MAX / 2) * M * N * 4;
}

extern "C" int gnnea_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                              const float* A, int64_t lda, const float* B, int64_t ldb,
                              const float* bias, float beta, float* C, int64_t ldc, void* ws,
                              int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!C || ldc < N || (K > 0 && (!A || !B))) return GNNEA_EINVAL;
  if (K > 0) {
    if ((trans_a ? lda < M : lda < K) || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int tiles_n = (int)((N + BN - 1) / BN);
  const int tiles = (int)(((M + BM - 1) / BM) * tiles_n);
  const int splits = ws ? pick_splits(M, N, K, ws_bytes) : 1;
  const int kps = (int)(((K + splits - 1) / splits + BK - 1) / BK * BK);
  float* slab = splits > 1 ? (float*)ws : nullptr;
  const dim3 grid(tiles, splits);
#define GNNEA_GEMM(TA, TB)                                                                      \
  hipLaunchKernelGGL((k_gemm_f32<TA, TB>), grid, dim3(256), 0, s, (int)M, (int)N, (int)K, A, lda, \
                     B, ldb, bias, beta, C, ldc, kps > 0 ? kps : BK, slab, tiles_n)
  if (!trans_a && !trans_b) GNNEA_GEMM(0, 0);
  else if (!trans_a && trans_b) GNNEA_GEMM(0, 1);
  else if (trans_a && !trans_b) GNNEA_GEMM(1, 0);
  else GNNEA_GEMM(1, 1);
#undef GNNEA_GEMM
  GNNEA_LAUNCH_CHECK();
  if (splits > 1) {
    const int64_t n = M * N;
    const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, splits, slab,
                       bias, beta, C, ldc);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}
