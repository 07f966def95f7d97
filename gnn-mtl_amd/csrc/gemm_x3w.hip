// fp32 projection GEMMs with the WEIGHT RESIDENT in LDS: C[M][N] = A[M][K] · op(B) (+ bias)
// (+ beta C) (relu) for the EA layers' tall projections (x·Wᵀ + b, dX = dY·W, x·[Wᵀ|K_g] and the
// HighWay input gradient [dh | dg]·[W ; K_gᵀ]: layers/layers.py:32,61, att_layers.py:33 and their
// autograd), K in (288, 320] (and (576, 608] for the f16x2 form).
//
// k_gemm_x3p (gemm.hip) streams both operands through an LDS-DMA ring: the B tile is re-read from
// L2 for every row tile and each k-step costs a barrier and DMA issue slots.  Here (as
// gemm_bf16.hip's k_gemm_bf16w for bf16) a column tile of the weight, split into planes, stays in
// LDS for the whole launch (one 8-wave workgroup per CU) and the activations go straight from
// HBM into registers: no barrier and no LDS traffic for A.  The product is computed transposed,
// Dᵀ = W_tile · Aᵀ on the 16x16x32 MFMA: the weight tile is the MFMA's A operand (ds_read_b128 of
// 8 k per lane, conflict-free), 16 activation rows per wave its B operand, split in registers; a
// lane's accumulators come out as 4 consecutive output columns of one row (16-B stores straight
// from registers, the bias added from LDS).  The k dimension is permuted alike for both
// operands: at step s the lanes of k-quarter kq hold k = 32 s + 4 kq + {0..3} and
// 32 s + 16 + 4 kq + {0..3}, so a wave-instruction's 64 lanes read 16 rows x 64 contiguous bytes.
// Workgroup b owns column tile (b / 8) % ntn and the row stream (b / (8 ntn)) * 8 + b % 8: the
// column tiles of the same rows are on one XCD (b mod 8), so A is read from HBM once and from L2
// by the other tiles.  Two forms:
//   k_gemm_x3w_ring    three bf16 pieces per operand, six products (gemm.hip's x3), 80-column
//                      tiles (GNNEA_X3W=2: the higher-fidelity fallback)
//   k_gemm_f16x2_ring  two fp16 pieces per operand with power-of-two row / column scaling, three
//                      products, 112-column tiles (64 for K = 600) -- the default
#include "common.h"
#include "gemm_x3w.h"

namespace gnnea {

typedef __bf16 w3_bf16x8 __attribute__((ext_vector_type(8)));
typedef float w3_f32x4 __attribute__((ext_vector_type(4)));

constexpr int W3_NC = 80;   // columns per tile
constexpr int W3_KC = 10;   // k-steps of 32 (K <= 320)
constexpr int W3_PLANE = W3_KC * 4 * W3_NC;  // 16-B units per plane of a tile
constexpr int64_t W3_TILE_BYTES = 3ll * W3_PLANE * 16;

// P[nt][p][s][kq][n][8]: element e = plane p of W_op[nt*80 + n][32 s + 16 (e / 4) + 4 kq + e % 4]
// (0 outside): lane kq's eight k of step s, the activation side's permutation
__global__ __launch_bounds__(256) void k_pack_x3w(const float* __restrict__ B, int64_t ldb,
                                                  int b_nk, int N, int K, int ntn,
                                                  bf16_t* __restrict__ P) {
  const int64_t per_plane = (int64_t)W3_PLANE * 8;
  const int64_t total = (int64_t)ntn * per_plane;  // elements of one plane, all tiles
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(t & 7);
    int64_t r = t >> 3;
    const int n = (int)(r % W3_NC);
    r /= W3_NC;
    const int kq = (int)(r & 3);
    r >>= 2;
    const int s = (int)(r % W3_KC);
    const int nt = (int)(r / W3_KC);
    const int col = nt * W3_NC + n, k = 32 * s + 16 * (e >> 2) + 4 * kq + (e & 3);
    float x = 0.f;
    if (col < N && k < K) x = b_nk ? B[(int64_t)col * ldb + k] : B[(int64_t)k * ldb + col];
    const __bf16 h = (__bf16)x;
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    const __bf16 l = (__bf16)(r1 - (float)m);
    bf16_t* dst = P + (int64_t)nt * 3 * per_plane + (t - (int64_t)nt * per_plane);
    dst[0] = __builtin_bit_cast(bf16_t, h);
    dst[per_plane] = __builtin_bit_cast(bf16_t, m);
    dst[2 * per_plane] = __builtin_bit_cast(bf16_t, l);
  }
}

// The activation split of the ring kernel, two elements at a time into packed bf16 pairs
// (dword q of a fragment = elements 2q, 2q + 1): round-to-nearest-even, h = bf16(x),
// m = bf16(x - h), l = bf16(x - h - m) (gemm.hip's split, pairwise instructions).
struct W3SplitP {
  uint32_t h[4], m[4], l[4];
  __device__ __forceinline__ w3_bf16x8 vh() const { return __builtin_bit_cast(w3_bf16x8, *(const uint4*)h); }
  __device__ __forceinline__ w3_bf16x8 vm() const { return __builtin_bit_cast(w3_bf16x8, *(const uint4*)m); }
  __device__ __forceinline__ w3_bf16x8 vl() const { return __builtin_bit_cast(w3_bf16x8, *(const uint4*)l); }
};

__device__ __forceinline__ uint32_t w3_pk(__bf16 a, __bf16 b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
}

__device__ __forceinline__ void w3_split_pair(float x0, float x1, uint32_t& h, uint32_t& m,
                                              uint32_t& l) {
  x3_split_pair(x0, x1, h, m, l);  // the same values as per-element casts
}

// The same product with 8 waves (two per SIMD: each one's LDS-read latency and split under the
// other's MFMAs) and a register ring instead of a whole-tile double buffer: a wave keeps ONE tile's
// 20 activation quads, and the quads of step s are replaced by the next tile's step s as soon as
// they have been read (a prefetch distance of one tile, 80 registers instead of 160).
__global__ __launch_bounds__(512) void k_gemm_x3w_ring(int M, int N, int K, int ntn,
                                                       const float* __restrict__ A, int64_t lda,
                                                       const bf16_t* __restrict__ P,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ C, int64_t ldc,
                                                       int64_t cs, float* __restrict__ C2,
                                                       int64_t cs2, float beta, int relu) {
  constexpr int NW = 8, BM = 16 * NW;
  __shared__ __attribute__((aligned(16))) uint4 wl[3 * W3_PLANE];
  __shared__ __attribute__((aligned(16))) float bsh[W3_NC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const int nt = (b / 8) % ntn;
  const int rs = (b / (8 * ntn)) * 8 + b % 8, nrs = (int)gridDim.x / ntn;
  const int n0 = nt * W3_NC;
  {  // the resident weight tile
    const uint4* src = (const uint4*)(P + (int64_t)nt * 3 * W3_PLANE * 8);
    for (int i = tid; i < 3 * W3_PLANE; i += 64 * NW) wl[i] = src[i];
    if (tid < W3_NC) bsh[tid] = bias && n0 + tid < N ? bias[n0 + tid] : 0.f;
  }
  __syncthreads();
  const int tm = (M + BM - 1) / BM;
  const int kq = lane >> 4, ml = lane & 15;
  const uint4* wlane = wl + kq * W3_NC + ml;
  uint4 f[2 * W3_KC];
  auto row_ptr = [&](int rt) {
    return A + (int64_t)min(rt * BM + w * 16 + ml, M - 1) * lda;
  };
  // K in (288, 320]: steps 0..8 are inside every row (immediate offsets from the lane's base);
  // only the last step's quads can reach K (clamped to the row's first quad, zeroed at use)
  auto load_step = [&](const float* p, int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (s < W3_KC - 1) {
        f[2 * s + j] = *(const uint4*)(p + 4 * kq + 32 * s + 16 * j);
      } else {
        const int k = 32 * s + 16 * j + 4 * kq;
        f[2 * s + j] = *(const uint4*)(p + (k < K ? k : 0));
      }
    }
  };
  auto raw_step = [&](int s, float (&x)[8]) {
    uint4 q0 = f[2 * s], q1 = f[2 * s + 1];
    if (s == W3_KC - 1) {
      const int k = 32 * s + 4 * kq;
      if (k >= K) q0 = make_uint4(0u, 0u, 0u, 0u);
      if (k + 16 >= K) q1 = make_uint4(0u, 0u, 0u, 0u);
    }
    x[0] = __builtin_bit_cast(float, q0.x); x[1] = __builtin_bit_cast(float, q0.y);
    x[2] = __builtin_bit_cast(float, q0.z); x[3] = __builtin_bit_cast(float, q0.w);
    x[4] = __builtin_bit_cast(float, q1.x); x[5] = __builtin_bit_cast(float, q1.y);
    x[6] = __builtin_bit_cast(float, q1.z); x[7] = __builtin_bit_cast(float, q1.w);
  };
  auto split_pair = [&](const float (&x)[8], int q, W3SplitP& t) {
    w3_split_pair(x[2 * q], x[2 * q + 1], t.h[q], t.m[q], t.l[q]);
  };
  if (rs < tm) {
    const float* p = row_ptr(rs);
#pragma unroll
    for (int s = 0; s < W3_KC; ++s) load_step(p, s);
  }
  for (int rt = rs; rt < tm; rt += nrs) {
    // the next tile's rows (past the end: a valid row, loaded and never used)
    const float* pn = row_ptr(rt + nrs < tm ? rt + nrs : rt);
    w3_f32x4 acc[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[j] = w3_f32x4{0.f, 0.f, 0.f, 0.f};
    W3SplitP acur;
    {
      float x[8];
      raw_step(0, x);
      load_step(pn, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) split_pair(x, q, acur);
    }
#pragma unroll
    for (int s = 0; s < W3_KC; ++s) {
      __builtin_amdgcn_sched_barrier(0);
      // the next step's quads are split straight from the ring, then replaced by the next
      // tile's (after the block loop); the weight fragments are read per block (the partner
      // wave on the SIMD covers their latency)
      float xn[8];
      if (s + 1 < W3_KC) raw_step(s + 1, xn);
      W3SplitP anx;
      const uint4* wp = wlane + s * 4 * W3_NC;
      const w3_bf16x8 ah = acur.vh(), am = acur.vm(), al = acur.vl();
#pragma unroll
      for (int jn = 0; jn < 5; ++jn) {
        __builtin_amdgcn_sched_barrier(0);
        const w3_bf16x8 wh = __builtin_bit_cast(w3_bf16x8, wp[16 * jn]);
        const w3_bf16x8 wm = __builtin_bit_cast(w3_bf16x8, wp[W3_PLANE + 16 * jn]);
        const w3_bf16x8 wlo = __builtin_bit_cast(w3_bf16x8, wp[2 * W3_PLANE + 16 * jn]);
        w3_f32x4& c = acc[jn];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, al, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, am, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wlo, ah, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, am, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wm, ah, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, ah, c, 0, 0, 0);
        if (s + 1 < W3_KC && jn < 4) split_pair(xn, jn, anx);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (s + 1 < W3_KC) {
        acur = anx;
        load_step(pn, s + 1);
      }
    }
    const int m = rt * BM + w * 16 + ml;
    if (m < M) {
#pragma unroll
      for (int jn = 0; jn < 5; ++jn) {
        const int c = 16 * jn + 4 * kq;
        int n = n0 + c;
        // (opaque to loop-invariant code motion: hoisted out of the tile loop, the 64-bit column
        // offsets are spilled, and a scratch reload waits vmcnt(0), draining the ring's loads)
        asm volatile("" : "+v"(n));
        if (n < N) {  // N % 4 == 0: a group is wholly in or out
          const float4 bv = *(const float4*)(bsh + c);
          const w3_f32x4 a4 = acc[jn];
          float4 o = make_float4(a4[0] + bv.x, a4[1] + bv.y, a4[2] + bv.z, a4[3] + bv.w);
          float4* cp = (float4*)(C + ((int64_t)(n >> 6) * cs + (int64_t)m * ldc + (n & 63)));
          if (beta != 0.f) {  // C = A·B + bias + beta C (uniform branch)
            const float4 cv = *cp;
            o.x += beta * cv.x; o.y += beta * cv.y; o.z += beta * cv.z; o.w += beta * cv.w;
          }
          if (relu) o = f4_relu(o);  // the Linear's act (layers/layers.py:121-122), uniform
          *cp = o;
          if (C2) *(float4*)(C2 + ((int64_t)(n >> 6) * cs2 + (int64_t)m * 64 + (n & 63))) = o;
        }
      }
    }
  }
}


// ---- k_gemm_f16x2_ring: the same projection through a TWO-way fp16 split, three products ----
// The x3 forms above spend six bf16 MFMAs per fp32 product (h·l, m·m, l·h, h·m, m·h, h·h).  fp16
// carries 11 significant bits to bf16's 8, so two fp16 pieces hold 22 bits of an fp32 operand:
//   x = hi + lo,  hi = f16(x·s),  lo = f16(x·s - hi)            (|lo| <= 2^-11 |hi|)
// and a·w = (hi_a hi_w + hi_a lo_w + lo_a hi_w) / (s_a t_w) up to lo_a·lo_w and lo's rounding, each
// <= 2^-22 |a||w| (x3 mode 2's dropped products are at 2^-21; fp32 accumulation's K·2^-24 bound
// dominates both at K ~ 300).  fp16's exponent range is what needs care: every activation ROW
// and every weight COLUMN is scaled by a power of two s = 2^(14 - floor(log2 max|x|)) so that its
// largest element lands in [2^14, 2^15) (the scaling and its inverse are exact); elements more
// than 2^24 below their row's maximum become fp16 subnormals (absolute error <= 2^-25 of the
// row's maximum there, nothing relative to the dot product's magnitude).  Non-finite inputs
// propagate (an inf row maximum gives inf / NaN outputs, as the fp32 product would).  Half the
// MFMAs of the x3 ring, same fp16 rate as bf16 (v_mfma_f32_16x16x32_f16).
// Structure: the ring kernel's (80-column weight tile resident in LDS, now two fp16 planes =
// 100 KB; 8 waves, 16 rows each; column tiles of a row stream on one XCD), except that a tile's
// activations are split WHOLE at its start (the row maximum needs all of them): the 20 raw
// quads -> 10 hi + 10 lo fragments, then the next tile's 20 quads are issued into the freed
// registers, a full tile of MFMAs ahead of their use.
typedef _Float16 f2_f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f2_f16x2 __attribute__((ext_vector_type(2)));

// exponent of the scale: e = floor(log2 m) clamped to [-112, 127] (m = 0 / fp32-subnormal:
// -112, so the scale stays a normal fp32 2^(14 - e) <= 2^126; inf / NaN: 127)
__device__ __forceinline__ int f2_exp(float m) {
  const int e = (int)((__builtin_bit_cast(uint32_t, m) >> 23) & 255u) - 127;
  return e < -112 ? -112 : (e > 127 ? 127 : e);
}
__device__ __forceinline__ float f2_pow2(int e) {  // 2^e for e in [-126, 127]
  return __builtin_bit_cast(float, (uint32_t)(e + 127) << 23);
}
// (x0, x1) -> packed fp16 pairs hi = f16(x s), lo = f16(x s - hi): four v_fma_mix (the scaling
// inside the fused multiply-add, the residual read back from hi's fp16 halves); the compiler's own
// form recomputes hi for the residual (seven instructions per pair)
__device__ __forceinline__ uint32_t f2_split_pair(float x0, float x1, float s, uint32_t& lo) {
  uint32_t h, l;
  asm("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(h) : "v"(x0), "v"(s));
  asm("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(h) : "v"(x1), "v"(s));
  asm("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(x0), "v"(s), "v"(h));
  asm("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "+v"(l) : "v"(x1), "v"(s), "v"(h));
  lo = l;
  return h;
}
// mx = max(mx, |a|, |b|) in one instruction (fmaxf's NaN canonicalisation of loaded values would
// add one v_max per element)
__device__ __forceinline__ float f2_max3abs(float mx, float a, float b) {
  asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(mx) : "v"(a), "v"(b));
  return mx;
}

// column scales of the weight operand: tsc[n] = 2^(14 - e_n), tinv[n] = 2^(e_n - 14) over
// W_op[n][0..K) (n < ntn * nc; past N: 1).  One wave per column, the k range strided over its
// lanes (a serial loop per column took 69 us per call)
__global__ __launch_bounds__(64) void k_colscale_f16x2(const float* __restrict__ B, int64_t ldb,
                                                       int b_nk, int N, int K, int nn,
                                                       float* __restrict__ tsc,
                                                       float* __restrict__ tinv) {
  const int n = blockIdx.x, lane = threadIdx.x;
  if (n >= nn) return;
  float m = 0.f;
  if (n < N)
    for (int k = lane; k < K; k += 64)
      m = fmaxf(m, fabsf(b_nk ? B[(int64_t)n * ldb + k] : B[(int64_t)k * ldb + n]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if (lane == 0) {
    const int e = f2_exp(m);
    tsc[n] = f2_pow2(14 - e);
    tinv[n] = f2_pow2(e - 14);
  }
}

// P[nt][p][s][kq][n][8], p = 0 hi / 1 lo: the x3 pack's layout (kc k-steps, nc-column tiles)
// with two fp16 planes of the column-scaled weight
__global__ __launch_bounds__(256) void k_pack_f16x2(const float* __restrict__ B, int64_t ldb,
                                                    int b_nk, int N, int K, int ntn, int kc,
                                                    int nc, const float* __restrict__ tsc,
                                                    uint16_t* __restrict__ P) {
  const int64_t per_plane = (int64_t)kc * 4 * nc * 8;
  const int64_t total = (int64_t)ntn * per_plane;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(t & 7);
    int64_t r = t >> 3;
    const int n = (int)(r % nc);
    r /= nc;
    const int kq = (int)(r & 3);
    r >>= 2;
    const int s = (int)(r % kc);
    const int nt = (int)(r / kc);
    const int col = nt * nc + n, k = 32 * s + 16 * (e >> 2) + 4 * kq + (e & 3);
    float x = 0.f;
    if (col < N && k < K) x = (b_nk ? B[(int64_t)col * ldb + k] : B[(int64_t)k * ldb + col]) * tsc[col];
    const _Float16 h = (_Float16)x;
    const _Float16 l = (_Float16)(x - (float)h);
    uint16_t* dst = P + (int64_t)nt * 2 * per_plane + (t - (int64_t)nt * per_plane);
    dst[0] = __builtin_bit_cast(uint16_t, h);
    dst[per_plane] = __builtin_bit_cast(uint16_t, l);
  }
}


// KC k-steps of 32 (K in (32 (KC - 1), 32 KC]), NC-column weight tiles.  The k dimension runs in
// CHUNKS of up to 10 steps, each with its own row scale and accumulators (K = 600: two): a
// chunk's 20 raw quads are split whole once they have landed, and the next chunk's (this tile's
// or the next tile's first) are issued into the freed registers, one chunk of MFMAs ahead.
// Epilogue modes EP (the relu Linear's masked backward, as gemm_bf16.hip's k_gemm_bf16w):
//  3 relu as mode 0, and the sign bits of the stored output -> Mo: per row and column tile 16 bytes,
//    byte 2 jn + h holding columns 16 jn + 8 h + 0..7 of the tile (bit e: column + e > 0);
//  2 the stored value is acc * relu'(y) with relu'(y) from those bits (Mi), read with the tile's
//    last chunk, before the next tile's activations are issued.
template <int KC, int NC, int CH, int NW, int EP = 0>
__global__ __launch_bounds__(64 * NW) void k_gemm_f16x2_ring(int M, int N, int K, int ntn,
                                                         const float* __restrict__ A, int64_t lda,
                                                         const uint16_t* __restrict__ P,
                                                         const float* __restrict__ tinv_g,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ C, int64_t ldc,
                                                         int64_t cs, float* __restrict__ C2,
                                                         int64_t cs2, float beta, int relu,
                                                         const uint8_t* __restrict__ Mi = nullptr,
                                                         uint8_t* __restrict__ Mo = nullptr,
                                                         int64_t ldm = 0) {
  constexpr int BM = 16 * NW, NJ = NC / 16;
  static_assert(EP == 0 || NJ <= 8, "sign bits: 16 bytes per row and tile");
  constexpr int PL = KC * 4 * NC;           // 16-B units per plane of a tile
  constexpr int NCH = (KC + CH - 1) / CH;   // k-chunks of CH steps
  static_assert(NC % 16 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) uint4 wl[2 * PL];
  __shared__ __attribute__((aligned(16))) float bsh[NC];
  __shared__ __attribute__((aligned(16))) float tsh[NC];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x;
  const int nt = (b / 8) % ntn;
  const int rs = (b / (8 * ntn)) * 8 + b % 8, nrs = (int)gridDim.x / ntn;
  const int n0 = nt * NC;
  {  // the resident weight tile, its column scales' inverses and the bias
    const uint4* src = (const uint4*)(P + (int64_t)nt * 2 * PL * 8);
    for (int i = tid; i < 2 * PL; i += 64 * NW) wl[i] = src[i];
    if (tid < NC) {
      bsh[tid] = bias && n0 + tid < N ? bias[n0 + tid] : 0.f;
      tsh[tid] = tinv_g[n0 + tid];
    }
  }
  __syncthreads();
  const int tm = (M + BM - 1) / BM;
  const int kq = lane >> 4, ml = lane & 15;
  const uint4* wlane = wl + kq * NC + ml;
  uint4 f[2 * CH];
  auto row_ptr = [&](int rt) {
    return A + (int64_t)min(rt * BM + w * 16 + ml, M - 1) * lda;
  };
  // chunk c's quads: steps 10 c .. ; steps before the last are inside every row, the last one's
  // quads past K read the row's first quad (valid) and are zeroed at use
  auto load_chunk = [&](const float* p, const int c) {
#pragma unroll
    for (int i = 0; i < 2 * CH; ++i) {
      const int st = CH * c + i / 2, j = i & 1;
      if (st < KC - 1) {
        f[i] = *(const uint4*)(p + 4 * kq + 32 * st + 16 * j);
      } else if (st == KC - 1) {
        const int k = 32 * st + 16 * j + 4 * kq;
        f[i] = *(const uint4*)(p + (k < K ? k : 0));
      }
    }
  };
  if (rs < tm) load_chunk(row_ptr(rs), 0);
  for (int rt = rs; rt < tm; rt += nrs) {
    w3_f32x4 acc[NJ];
    int er = 0;     // the row's scale exponent so far (the largest chunk maximum's)
    // beta != 0 on the wide (K = 600) form: the tile's C, loaded ahead of the next tile's
    // activations (the 80 / 112-column forms have no registers to spare: C read in the epilogue)
    constexpr bool CAHEAD = KC > 10;
    float4 cv[CAHEAD ? NJ : 1];
    uint4 mk;  // EP 2: the row's sign bytes of this column tile
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int s0 = CH * c, ns = KC - s0 < CH ? KC - s0 : CH;
      __builtin_amdgcn_sched_barrier(0);
      if (s0 + ns == KC) {
        const int k = 32 * (KC - 1) + 4 * kq, i = 2 * (KC - 1 - s0);
        if (k >= K) f[i] = make_uint4(0u, 0u, 0u, 0u);
        if (k + 16 >= K) f[i + 1] = make_uint4(0u, 0u, 0u, 0u);
      }
      // the row's maximum over the chunk: this lane's elements, then the row's k-quarter lanes
      float mx = 0.f;
#pragma unroll
      for (int q = 0; q < 2 * ns; ++q) {
        mx = f2_max3abs(mx, __builtin_bit_cast(float, f[q].x), __builtin_bit_cast(float, f[q].y));
        mx = f2_max3abs(mx, __builtin_bit_cast(float, f[q].z), __builtin_bit_cast(float, f[q].w));
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16));
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      // one scale per row: a chunk with a larger maximum than the earlier ones rescales their
      // accumulated sums down by the exact power of two (what falls below fp32's range there is
      // < 2^-100 of the row's largest term); a smaller one is split at the row's scale
      const int ec = f2_exp(mx);
      if (c == 0) {
        er = ec;
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] = w3_f32x4{0.f, 0.f, 0.f, 0.f};
      } else if (ec > er) {
        const float d = er - ec < -126 ? 0.f : f2_pow2(er - ec);  // (beyond: fp32 underflow)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] *= d;
        er = ec;
      }
      const float sr = f2_pow2(14 - er);
      uint32_t ah[2 * CH][2], al[2 * CH][2];
#pragma unroll
      for (int q = 0; q < 2 * ns; ++q) {
        ah[q][0] = f2_split_pair(__builtin_bit_cast(float, f[q].x),
                                 __builtin_bit_cast(float, f[q].y), sr, al[q][0]);
        ah[q][1] = f2_split_pair(__builtin_bit_cast(float, f[q].z),
                                 __builtin_bit_cast(float, f[q].w), sr, al[q][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
      // beta != 0 (uniform): C's tile is read before the next tile's activations are issued, so
      // the epilogue waits for these loads only, not for the activations in flight behind them
      if (CAHEAD && c == NCH - 1 && beta != 0.f) {
        const int mm = min(rt * BM + w * 16 + ml, M - 1);
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn) {
          const int nn = min(n0 + 16 * jn + 4 * kq, N - 4);
          cv[jn] = *(const float4*)(C + ((int64_t)(nn >> 6) * cs + (int64_t)mm * ldc + (nn & 63)));
        }
      }
      if constexpr (EP == 2) {
        if (c == NCH - 1)
          mk = *(const uint4*)(Mi + (int64_t)min(rt * BM + w * 16 + ml, M - 1) * ldm + nt * 16);
      }
      // the next chunk's activations, a chunk of MFMAs ahead (past the last tile: none)
      // (unconditional, past the last tile the last tile again: the same outstanding-load
      // count on every path, so the compiler's waits never cover the loads in flight)
      if (c + 1 < NCH)
        load_chunk(row_ptr(rt), c + 1);
      else
        load_chunk(row_ptr(rt + nrs < tm ? rt + nrs : rt), 0);
      // the chunk's (step, column block) blocks in order; with registers to spare (CH <= 5 at
      // 8 waves) each block's two weight fragments are read two blocks ahead, under the MFMAs of
      // the blocks before it (read per block, each block waited ~100 cycles for its reads)
      constexpr bool WPF = CH <= 5 && NW <= 8;
      uint4 bw[3][2];
      auto rd = [&](int q, uint4 (&d)[2]) {
        const uint4* wp = wlane + (s0 + q / NJ) * 4 * NC + 16 * (q % NJ);
        d[0] = wp[0];
        d[1] = wp[PL];
      };
      if constexpr (WPF) {
        rd(0, bw[0]);
        if (ns * NJ > 1) rd(1, bw[1]);
      }
#pragma unroll
      for (int q = 0; q < CH * NJ; ++q) {
        const int s = q / NJ, jn = q % NJ;
        if (s >= ns) break;
        const f2_f16x8 xh = __builtin_bit_cast(
            f2_f16x8, make_uint4(ah[2 * s][0], ah[2 * s][1], ah[2 * s + 1][0], ah[2 * s + 1][1]));
        const f2_f16x8 xl = __builtin_bit_cast(
            f2_f16x8, make_uint4(al[2 * s][0], al[2 * s][1], al[2 * s + 1][0], al[2 * s + 1][1]));
        uint4 cur[2];
        if constexpr (WPF) {
          if (q + 2 < ns * NJ) rd(q + 2, bw[(q + 2) % 3]);
          cur[0] = bw[q % 3][0];
          cur[1] = bw[q % 3][1];
        } else {
          rd(q, cur);
        }
        __builtin_amdgcn_sched_barrier(0);
        const f2_f16x8 wh = __builtin_bit_cast(f2_f16x8, cur[0]);
        const f2_f16x8 wlo = __builtin_bit_cast(f2_f16x8, cur[1]);
        w3_f32x4& cc = acc[jn];
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wlo, xh, cc, 0, 0, 0);
        cc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xh, cc, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const float rinv = f2_pow2(er - 14);
    const int m = rt * BM + w * 16 + ml;
    if (m < M) {
      uint32_t nb = 0;  // EP 3: the sign nibbles, column block jn at bits 4 jn
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) {
        const int c = 16 * jn + 4 * kq;
        int n = n0 + c;
        asm volatile("" : "+v"(n));  // (see k_gemm_x3w_ring)
        if (n < N) {
          const float4 bv = *(const float4*)(bsh + c);
          const float4 tv = *(const float4*)(tsh + c);
          // unscaled exactly (powers of two, the column's first), then one rounding with the bias
          const w3_f32x4 a4 = acc[jn];
          float4 o = make_float4(a4[0] * tv.x * rinv + bv.x, a4[1] * tv.y * rinv + bv.y,
                                 a4[2] * tv.z * rinv + bv.z, a4[3] * tv.w * rinv + bv.w);
          float4* cp = (float4*)(C + ((int64_t)(n >> 6) * cs + (int64_t)m * ldc + (n & 63)));
          if (beta != 0.f) {
            const float4 c4 = CAHEAD ? cv[CAHEAD ? jn : 0] : *cp;
            o.x += beta * c4.x; o.y += beta * c4.y; o.z += beta * c4.z; o.w += beta * c4.w;
          }
          if constexpr (EP == 2) {  // o * relu'(y): act_bwd's G on the stored product
            const uint32_t wd = jn >> 1 == 0 ? mk.x : (jn >> 1 == 1 ? mk.y : (jn >> 1 == 2 ? mk.z : mk.w));
            const uint32_t bits = wd >> (8 * (2 * (jn & 1) + (kq >> 1)) + 4 * (kq & 1));
            o.x *= (bits & 1u) ? 1.f : 0.f;
            o.y *= (bits & 2u) ? 1.f : 0.f;
            o.z *= (bits & 4u) ? 1.f : 0.f;
            o.w *= (bits & 8u) ? 1.f : 0.f;
          }
          if (relu) o = f4_relu(o);
          *cp = o;
          if (C2) *(float4*)(C2 + ((int64_t)(n >> 6) * cs2 + (int64_t)m * 64 + (n & 63))) = o;
          if constexpr (EP == 3)
            nb |= ((o.x > 0.f ? 1u : 0u) | (o.y > 0.f ? 2u : 0u) | (o.z > 0.f ? 4u : 0u) |
                   (o.w > 0.f ? 8u : 0u)) << (4 * jn);
        }
      }
      if constexpr (EP == 3) {
        // byte 2 jn + h = the nibbles of kq = 2 h (low) and 2 h + 1 (high): partners lane ^ 16,
        // then the two h halves (lane ^ 32) meet in the kq = 0 lane, which stores the 16 bytes
        const uint32_t p1 = __shfl_xor(nb, 16);
        const uint32_t lo = (kq & 1) ? p1 : nb, hi = (kq & 1) ? nb : p1;
        uint32_t bl = 0, bh = 0;  // this h's bytes, jn 0..3 and 4..7
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn) {
          const uint32_t by = ((lo >> (4 * jn)) & 15u) | (((hi >> (4 * jn)) & 15u) << 4);
          if (jn < 4) bl |= by << (8 * jn);
          else bh |= by << (8 * (jn - 4));
        }
        const uint32_t ql = __shfl_xor(bl, 32), qh = __shfl_xor(bh, 32);
        if (kq == 0) {  // (h = 0: own bytes B0, the partner's B1)
          uint32_t d[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t s0 = q < 2 ? bl : bh, s1 = q < 2 ? ql : qh;
            const int sh = 16 * (q & 1);
            d[q] = ((s0 >> sh) & 255u) | (((s1 >> sh) & 255u) << 8) |
                   (((s0 >> (sh + 8)) & 255u) << 16) | (((s1 >> (sh + 8)) & 255u) << 24);
          }
          *(uint4*)(Mo + (int64_t)m * ldm + nt * 16) = make_uint4(d[0], d[1], d[2], d[3]);
        }
      }
    }
  }
}

// ---- host side ----

// The tall K <= 320 (and K = 600) fp32 projections: k_gemm_f16x2_ring (two fp16 pieces, three
// products) by default; GNNEA_X3W=2 selects the x3 ring (three bf16 pieces, six products: ~24
// significant bits against ~22, the higher-fidelity fallback; tests/test_gpu_gemm_range.py pins
// both).  Measured on one box: 2M x 300 x 300 1.89 vs 2.18 ms, x·[Wᵀ|K_g] 3.92 vs 4.25, the
// K = 600 input gradient with +C 5.34 vs 6.16 (profiles/r04_gemm_ab_f16x2_v2.json).  The other
// round-3/4 forms (the 4-wave x3w, the two-fragment ring) measured slower and were removed.
static int x3w_mode() {
  static const int mode = [] {
    const char* e = getenv("GNNEA_X3W");
    return e && atoi(e) == 2 ? 2 : 4;
  }();
  return mode;
}

// the f16x2 forms: K in (288, 320] on 80-column tiles, K in (576, 608] (the HighWay input
// gradient [dh | dg]·[W ; K_gᵀ], K = 600) on 64-column tiles (2 planes x 19 steps x 64 columns =
// 152 KB of LDS)
constexpr int F2_NC_WIDE = 64, F2_KC_WIDE = 19;
// K <= 320 tile width: 112 columns (143 KB of weight; the activations re-read by 3 column
// tiles at N = 300 instead of 4, 6 at N = 600 instead of 8; 12 % of the MFMAs on padding at
// N = 300): 2M x 300 x 300 1.79 vs 1.87 ms on 80-column tiles, x·[Wᵀ|K_g] 3.45 vs 3.81, HGCN-EA
// step 88.0 vs 89.3 (profiles/r04_gemm_ab_f16x2_nc112.json)
constexpr int F2_NC = 112;
static bool f16x2_k(int64_t K, int* kc, int* nc) {
  if (K > 32 * (W3_KC - 1) && K <= 32 * W3_KC) {
    *kc = W3_KC, *nc = F2_NC;
    return true;
  }
  if (K > 32 * (F2_KC_WIDE - 1) && K <= 32 * F2_KC_WIDE) {
    *kc = F2_KC_WIDE, *nc = F2_NC_WIDE;
    return true;
  }
  return false;
}
static int64_t f16x2_ws_bytes(int64_t N, int kc, int nc) {
  const int64_t ntn = (N + nc - 1) / nc;
  return ntn * (2ll * kc * 4 * nc * 16 + 2ll * nc * 4);
}

int64_t gemm_x3w_ws_bytes(int64_t N) {  // the largest of the forms
  const int64_t x3 = (N + W3_NC - 1) / W3_NC * W3_TILE_BYTES;
  const int64_t f2 = f16x2_ws_bytes(N, F2_KC_WIDE, F2_NC_WIDE);
  const int64_t f3 = f16x2_ws_bytes(N, W3_KC, F2_NC);
  const int64_t m = x3 > f2 ? x3 : f2;
  return m > f3 ? m : f3;
}

bool gemm_x3w_applies(int trans_a, int64_t M, int64_t N, int64_t K, int64_t lda, const void* A,
                      float beta, int64_t ldc, int64_t cs, const void* C, const void* C2,
                      int64_t cs2, int act) {
  // beta != 0 and a fused act only on the ring forms (modes 2 - 4)
  int kc, nc;
  const bool kok = x3w_mode() == 4 ? f16x2_k(K, &kc, &nc)
                                   : (K > 32 * (W3_KC - 1) && K <= 32 * W3_KC);
  return !trans_a &&
         (act == GNNEA_ACT_IDENTITY || act == GNNEA_ACT_RELU) && A && C && M >= 65536 &&
         M < (1ll << 31) && N >= 64 && N <= 4096 && N % 4 == 0 && kok && K % 4 == 0 &&
         lda >= K && lda % 4 == 0 && (((uintptr_t)A) & 15) == 0 &&
         ldc % 4 == 0 && cs % 4 == 0 && (((uintptr_t)C) & 15) == 0 &&
         (!C2 || (cs2 % 4 == 0 && (((uintptr_t)C2) & 15) == 0));
}

static int cu_count() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return ncu;
}

// persistent grid: a multiple of 8 * ntn workgroups (column tiles of a row stream 8 apart)
static int ring_grid(int ntn, int64_t M, int bm) {
  const int unit = 8 * ntn;
  const int64_t tm = (M + bm - 1) / bm;
  int grid = cu_count() / unit * unit;
  if (grid < unit) grid = unit;
  if ((int64_t)grid / ntn > tm) grid = (int)((tm + 7) / 8 * 8 * ntn);
  return grid;
}

static int f16x2_launch(int trans_b, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                        const float* B, int64_t ldb, const float* bias, float* C, int64_t ldc,
                        int64_t cs, float* C2, int64_t cs2, void* ws, int64_t ws_bytes,
                        hipStream_t s, float beta, int relu, int ep = 0,
                        const uint8_t* Mi = nullptr, uint8_t* Mo = nullptr, int64_t ldm = 0) {
  int kc, nc;
  if (!f16x2_k(K, &kc, &nc)) return GNNEA_EINVAL;
  if (ws_bytes < f16x2_ws_bytes(N, kc, nc)) return GNNEA_EWORKSPACE;
  const int ntn = (int)((N + nc - 1) / nc);
  float* tsc = (float*)((char*)ws + (int64_t)ntn * 2 * kc * 4 * nc * 16);  // after the planes
  float* tinv = tsc + (int64_t)ntn * nc;
  const int nn = ntn * nc;
  hipLaunchKernelGGL(k_colscale_f16x2, dim3(nn), dim3(64), 0, s, B, ldb, trans_b ? 1 : 0, (int)N,
                     (int)K, nn, tsc, tinv);
  GNNEA_LAUNCH_CHECK();
  const int64_t tot = (int64_t)ntn * kc * 4 * nc * 8;
  const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
  hipLaunchKernelGGL(k_pack_f16x2, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 1 : 0, (int)N,
                     (int)K, ntn, kc, nc, (const float*)tsc, (uint16_t*)ws);
  GNNEA_LAUNCH_CHECK();
  // k-chunk of CH steps and NW waves per workgroup (the register budget: 10 x 8 at 256
  // registers, 5 x 8 with the weight fragments two blocks ahead, 3 x 16 at 128 = four waves per
  // SIMD).  Measured on one box (profiles/r05_gemm_ring_occupancy_ab.json): x·[Wᵀ|K_g]
  // (ntn = 6) 3.43 -> 3.26 ms with 3 x 16 (5 x 8: 3.45-3.49), the K = 600 input gradient
  // 4.94 -> 4.52 with 5 x 8, 2M x 300 x 300 (ntn = 3) 1.74 -> 1.70 with 5 x 8 (3 x 16: 1.78)
#define GNNEA_F2R(KC_, NC_, CH_, NW_)                                                          \
  hipLaunchKernelGGL((k_gemm_f16x2_ring<KC_, NC_, CH_, NW_>), dim3(ring_grid(ntn, M, 16 * NW_)), \
                     dim3(64 * NW_), 0, s, (int)M, (int)N, (int)K, ntn, A, lda,                \
                     (const uint16_t*)ws, (const float*)tinv, bias, C, ldc, cs, C2, cs2, beta, relu)
  if (ep != 0) {  // (f16x2_mask_applies: kc == W3_KC, ntn < 4)
    const dim3 g(ring_grid(ntn, M, 16 * 8)), bl(64 * 8);
    if (ep == 2)
      hipLaunchKernelGGL((k_gemm_f16x2_ring<W3_KC, F2_NC, 5, 8, 2>), g, bl, 0, s, (int)M, (int)N,
                         (int)K, ntn, A, lda, (const uint16_t*)ws, (const float*)tinv, bias, C, ldc,
                         cs, C2, cs2, beta, relu, Mi, nullptr, ldm);
    else
      hipLaunchKernelGGL((k_gemm_f16x2_ring<W3_KC, F2_NC, 5, 8, 3>), g, bl, 0, s, (int)M, (int)N,
                         (int)K, ntn, A, lda, (const uint16_t*)ws, (const float*)tinv, bias, C, ldc,
                         cs, C2, cs2, beta, relu, nullptr, Mo, ldm);
  } else if (kc == W3_KC) {
    if (ntn >= 4) GNNEA_F2R(W3_KC, F2_NC, 3, 16);
    else GNNEA_F2R(W3_KC, F2_NC, 5, 8);
  } else {
    GNNEA_F2R(F2_KC_WIDE, F2_NC_WIDE, 5, 8);
  }
#undef GNNEA_F2R
  GNNEA_LAUNCH_CHECK();
  return 0;
}

int64_t f16x2_mask_ld(int64_t N) { return 16 * ((N + F2_NC - 1) / F2_NC); }

bool f16x2_mask_applies(int64_t M, int64_t N, int64_t K, int64_t lda, const void* A, int64_t ldc,
                        const void* C) {
  int kc, nc;
  return x3w_mode() == 4 && f16x2_k(K, &kc, &nc) && kc == W3_KC && (N + F2_NC - 1) / F2_NC < 4 &&
         gemm_x3w_applies(0, M, N, K, lda, A, 0.f, ldc, 64, C, nullptr, 0, GNNEA_ACT_RELU);
}

int f16x2_mask_launch(int ep, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                      int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                      int64_t ldc, const uint8_t* Mi, uint8_t* Mo, int64_t ldm, void* ws,
                      int64_t ws_bytes, hipStream_t s) {
  if ((ep != 2 && ep != 3) || !f16x2_mask_applies(M, N, K, lda, A, ldc, C) ||
      ldm < f16x2_mask_ld(N) || ldm % 16 || ((uintptr_t)(ep == 2 ? (const void*)Mi : Mo) & 15))
    return GNNEA_EINVAL;
  if (!ws || ws_bytes < gemm_x3w_ws_bytes(N)) return GNNEA_EWORKSPACE;
  return f16x2_launch(trans_b, M, N, K, A, lda, B, ldb, bias, C, ldc, 64, nullptr, 0, ws, ws_bytes,
                      s, 0.f, ep == 3 ? 1 : 0, ep, Mi, Mo, ldm);
}

int gemm_x3w_launch(int trans_b, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                    const float* B, int64_t ldb, const float* bias, float* C, int64_t ldc,
                    int64_t cs, float* C2, int64_t cs2, void* ws, int64_t ws_bytes,
                    hipStream_t s, float beta, int act) {
  const int relu = act == GNNEA_ACT_RELU ? 1 : 0;
  if (!ws || ws_bytes < gemm_x3w_ws_bytes(N)) return GNNEA_EWORKSPACE;
  if (x3w_mode() == 4)
    return f16x2_launch(trans_b, M, N, K, A, lda, B, ldb, bias, C, ldc, cs, C2, cs2, ws, ws_bytes,
                        s, beta, relu);
  const int ntn = (int)((N + W3_NC - 1) / W3_NC);
  bf16_t* P = (bf16_t*)ws;
  {
    const int64_t tot = (int64_t)ntn * W3_PLANE * 8;
    const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
    // B op-form [N][K]: trans_b = 1 means B is stored [N][K]
    hipLaunchKernelGGL(k_pack_x3w, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 1 : 0, (int)N,
                       (int)K, ntn, P);
    GNNEA_LAUNCH_CHECK();
  }
  const int grid = ring_grid(ntn, M, 128);
  hipLaunchKernelGGL(k_gemm_x3w_ring, dim3(grid), dim3(512), 0, s, (int)M, (int)N, (int)K, ntn, A,
                     lda, P, bias, C, ldc, cs, C2, cs2, beta, relu);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

// ---- C-ABI: the fp32 relu Linear's sign bits (gnnea.h) ----
using namespace gnnea;

extern "C" int gnnea_gemm_f32_mask_applies(int64_t M, int64_t N, int64_t K, int64_t lda,
                                           int64_t ldc) {
  const void* dummy = (const void*)(uintptr_t)256;  // (alignment is checked on the real call)
  return M > 0 && f16x2_mask_applies(M, N, K, lda, dummy, ldc, dummy) ? 1 : 0;
}

extern "C" int64_t gnnea_gemm_f32_mask_ld(int64_t N) {
  if (N < 0) return GNNEA_EINVAL;
  return f16x2_mask_ld(N);
}

extern "C" int64_t gnnea_gemm_f32_mask_ws_bytes(int64_t N) {
  if (N < 0) return GNNEA_EINVAL;
  return gemm_x3w_ws_bytes(N);
}

// C = relu(A·op(B) + bias) (bit-identical to gnnea_gemm_x3_act_f32's relu on this kernel) and the
// sign bits of C (16 bytes per row and 112-column tile: byte 16 t + 2 j + h holds columns
// 112 t + 16 j + 8 h + 0..7, bit e set where that column's value > 0)
extern "C" int gnnea_gemm_f32_relu_mask(int trans_b, int64_t M, int64_t N, int64_t K,
                                        const float* A, int64_t lda, const float* B, int64_t ldb,
                                        const float* bias, float* C, int64_t ldc, void* Mo,
                                        int64_t ldm, void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (!A || !B || !C || !Mo || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  return f16x2_mask_launch(3, trans_b, M, N, K, A, lda, B, ldb, bias, C, ldc, nullptr,
                           (uint8_t*)Mo, ldm, ws, ws_bytes, (hipStream_t)stream);
}

// G = (A·op(B)) * relu'(y), relu'(y) from gnnea_gemm_f32_relu_mask's bits of y: bit-identical to
// gnnea_gemm_x3_f32 followed by gnnea_act_bwd_colsum_f32's G
extern "C" int gnnea_gemm_f32_dmask_bits(int trans_b, int64_t M, int64_t N, int64_t K,
                                         const float* A, int64_t lda, const float* B, int64_t ldb,
                                         const void* Mi, int64_t ldm, float* G, int64_t ldg,
                                         void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (!A || !B || !G || !Mi || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  return f16x2_mask_launch(2, trans_b, M, N, K, A, lda, B, ldb, nullptr, G, ldg,
                           (const uint8_t*)Mi, nullptr, ldm, ws, ws_bytes, (hipStream_t)stream);
}
