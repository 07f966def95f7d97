// a7. GAT attention-vector gradient (autograd of att_layers.py:38, a·[h_i || h_j]):
//   da1[h] = Σ_i ds1[i,h] · H[i, h-block],   da2[h] = Σ_j ds2[j,h] · H[j, h-block]
// i.e. out[c] = Σ_r ds[r, c / d_head] · H[r, c] for every column c of the head-concatenated H,
// and the bias gradients (column sums, ds ≡ 1: autograd of nn.Linear's bias, layers.py:32).
// One streaming pass over H (N·D·s bytes, HBM bound) instead of an [N, heads]ᵀ·[N, D] GEMM whose
// off-diagonal head blocks are thrown away; da1 and da2 of one layer share the pass when they
// weight the same rows (K = 2 weight sets, gnnea_gat_da2_*).
//
// Stage 1 (k_da_stream): a workgroup of 4 waves owns a contiguous row range, the waves take its
// rows round robin, U = 4 rows per wave (2 with two weight sets) loaded before their FMAs.  Lane l owns the 16-B granules
// l, l + 64, ... of a row (bf16: 8 elements, fp32: 4); lanes past the row's last granule re-read
// it (their sums are discarded), so every load is unconditional and the compiler's waits sit at
// the FMAs.  A row's head weights are one scalar load (the row index is wave-uniform); with four
// heads a granule spans at most two of them (d_head >= its elements), picked once per granule.  The
// waves' sums meet in LDS, one partial row per workgroup and weight set.  Stage 2
// (k_gat_da_final) adds the partials in workgroup order: deterministic, no atomics.
// A granule read may pass the row's last column (D·s not a multiple of 16): rows whose granules
// would pass the END of the table take the element path (gnnea reads nothing outside H).
#include "common.h"

namespace gnnea {

constexpr int kDaWaves = 4, kDaU = 4;

template <typename T> struct Gran;
template <> struct Gran<float> {
  static constexpr int E = 4;
  static __device__ __forceinline__ void get(const uint4& u, float (&f)[4]) { unpack16(u, f); }
};
template <> struct Gran<bf16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ void get(const uint4& u, float (&f)[8]) { unpack16(u, f); }
};

// K weight sets (ds1, ds2), HH: 4 = four heads (one 16-B scalar load per row and set), 1 = one
// head (ds[r]), 0 = any (per-element loads), -1 = all-ones weights (column sums)
template <typename T, int NG, int K, int HH>
__global__ __launch_bounds__(64 * kDaWaves) void k_da_stream(const T* __restrict__ H, int64_t ldh,
                                                             int64_t n_rows, int64_t n_fast,
                                                             int64_t rpb, int D, int heads,
                                                             int d_head,
                                                             const float* __restrict__ ds1,
                                                             const float* __restrict__ ds2,
                                                             float* __restrict__ part) {
  constexpr int E = Gran<T>::E;
  constexpr int NE = NG * E;  // elements per lane
  const int G = (D + E - 1) / E;  // granules per row
  const int w = wave_id(), lane = lane_id();
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(n_rows, r0 + rpb);
  const int64_t rf = min(r1, n_fast);  // rows [r0, rf) by granules
  int gq[NG];
  int hd[NE];  // head of each owned element (clamped; columns >= D are never written)
  int ha[NG], hb[NG], sp[NG];  // HH = 4 (d_head >= E): a granule's heads ha, hb = ha + 1 (split at sp)
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    gq[q] = min(lane + 64 * q, G - 1);
#pragma unroll
    for (int t = 0; t < E; ++t) {
      const int c = gq[q] * E + t;
      hd[q * E + t] = HH == 1 || HH < 0 ? 0 : min(c / d_head, heads - 1);
    }
    ha[q] = hd[q * E];
    hb[q] = min(ha[q] + 1, 3);
    sp[q] = min(E, (ha[q] + 1) * d_head - gq[q] * E);
  }
  float acc[K][NE];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int t = 0; t < NE; ++t) acc[k][t] = 0.f;

  auto weights = [&](int64_t r, int k, float (&wv)[NE]) {
    const float* ds = k == 0 ? ds1 : ds2;
    if constexpr (HH < 0) {
#pragma unroll
      for (int t = 0; t < NE; ++t) wv[t] = 1.f;
    } else if constexpr (HH == 1) {
      const float v = ds[r];
#pragma unroll
      for (int t = 0; t < NE; ++t) wv[t] = v;
    } else if constexpr (HH == 4) {
      const float4 d4 = *(const float4*)(ds + r * 4);  // r wave-uniform: a scalar load
      auto sel = [&](int h) { return h == 0 ? d4.x : (h == 1 ? d4.y : (h == 2 ? d4.z : d4.w)); };
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        const float wa = sel(ha[q]), wb = sel(hb[q]);
#pragma unroll
        for (int t = 0; t < E; ++t) wv[q * E + t] = t < sp[q] ? wa : wb;
      }
    } else {
#pragma unroll
      for (int t = 0; t < NE; ++t) wv[t] = ds[r * heads + hd[t]];
    }
  };
  auto fma_row = [&](int64_t r, const float (&x)[NE]) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float wv[NE];
      weights(r, k, wv);
#pragma unroll
      for (int t = 0; t < NE; ++t) acc[k][t] = fmaf(wv[t], x[t], acc[k][t]);
    }
  };
  auto load_row = [&](int64_t r, uint4 (&u)[NG]) {
    const T* row = H + r * ldh;
#pragma unroll
    for (int q = 0; q < NG; ++q) u[q] = *(const uint4*)(row + gq[q] * E);
  };
  auto unpack = [&](const uint4 (&u)[NG], float (&x)[NE]) {
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      float f[E];
      Gran<T>::get(u[q], f);
#pragma unroll
      for (int t = 0; t < E; ++t) x[q * E + t] = f[t];
    }
  };
  constexpr int WS = kDaWaves;
  constexpr int U = K == 2 || HH == 0 || NG > 2 ? 2 : kDaU;  // rows in flight per wave
  int64_t r = r0 + w;
  for (; r + (U - 1) * WS < rf; r += U * WS) {
    uint4 u[U][NG];
#pragma unroll
    for (int i = 0; i < U; ++i) load_row(r + WS * i, u[i]);
#pragma unroll
    for (int i = 0; i < U; ++i) {
      float x[NE];
      unpack(u[i], x);
      fma_row(r + WS * i, x);
    }
  }
  for (; r < rf; r += WS) {
    uint4 u[NG];
    load_row(r, u);
    float x[NE];
    unpack(u, x);
    fma_row(r, x);
  }
  for (; r < r1; r += WS) {  // the table's last rows: element loads inside the row
    float x[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) {
      const int c = gq[t / E] * E + t % E;
      x[t] = c < D ? to_f32<T>(H[r * ldh + c]) : 0.f;
    }
    fma_row(r, x);
  }

  // the waves' sums in LDS, one partial row per weight set: part[blk][k][Dp]
  __shared__ float red[kDaWaves][K][64 * NE];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int t = 0; t < NE; ++t) red[w][k][t * 64 + lane] = acc[k][t];
  __syncthreads();
  const int Dp = (D + 3) & ~3;
  for (int i = threadIdx.x; i < K * D; i += 64 * kDaWaves) {
    const int k = i / D, c = i - k * D;
    const int g = c / E, t = c % E;
    const int q = g / 64, l = g % 64;
    const int slot = (q * E + t) * 64 + l;
    float s = red[0][k][slot];
#pragma unroll
    for (int v = 1; v < kDaWaves; ++v) s += red[v][k][slot];
    part[((int64_t)blockIdx.x * K + k) * Dp + c] = s;
  }
}

// 64 columns per workgroup, the 8 waves stride the partial rows (4 independent sums per lane),
// combined in wave order through LDS: deterministic, latency hidden across the waves.
// part rows are ld = roundup4(D) floats apart; partial b of set k is row b * K + k.
__global__ __launch_bounds__(512) void k_gat_da_final(const float* __restrict__ part, int nb,
                                                      int K, int D, float* __restrict__ out1,
                                                      float* __restrict__ out2) {
  __shared__ float red[8][64];
  const int w = wave_id(), lane = lane_id();
  const int k = blockIdx.y;
  const int c = blockIdx.x * 64 + lane;
  const int64_t ld = (D + 3) & ~3;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int b = w;
    for (; b + 24 < nb; b += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += part[((int64_t)(b + 8 * u) * K + k) * ld + c];
    }
    for (int u = 0; b < nb; b += 8, ++u) s[u & 3] += part[((int64_t)b * K + k) * ld + c];
  }
  red[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (w == 0 && c < D) {
    float t = 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v) t += red[v][lane];
    (k == 0 ? out1 : out2)[c] = t;
  }
}

// 8 workgroups per CU of 256 rows or more each
static int da_blocks(int64_t n_rows) {
  const int64_t b = (n_rows + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

template <typename T>
static int da_t(const T* H, int64_t ldh, int64_t n_rows, int heads, int d_head, const float* ds1,
                const float* ds2, int hh, float* out1, float* out2, void* ws, int64_t ws_bytes,
                hipStream_t s) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  const int D = heads * d_head;
  const int K = out2 ? 2 : 1;
  if (!out1) return GNNEA_EINVAL;
  if (n_rows == 0) {
    GNNEA_HIP(hipMemsetAsync(out1, 0, sizeof(float) * D, s));
    if (out2) GNNEA_HIP(hipMemsetAsync(out2, 0, sizeof(float) * D, s));
    return 0;
  }
  if (!H || ldh < D || (hh >= 0 && !ds1) || (K == 2 && !ds2)) return GNNEA_EINVAL;
  // granule loads need 4-B aligned rows; four heads: 16-B aligned weight rows
  if ((((uintptr_t)H) & 3) || (ldh * (int64_t)sizeof(T)) % 4) return GNNEA_EALIGN;
  constexpr int E = Gran<T>::E;
  // four heads: 16-B weight rows, a granule spans at most two heads
  if (hh == 4 && ((((uintptr_t)ds1) & 15) || (((uintptr_t)ds2) & 15) || d_head < E)) hh = 0;
  const int G = (D + E - 1) / E, NG = (G + 63) / 64;
  if (NG > 4) return GNNEA_EINVAL;  // D <= 1024 fp32 / 2048 bf16
  const int nb = da_blocks(n_rows);
  const int Dp = (D + 3) & ~3;
  if (!ws || ws_bytes < (int64_t)nb * K * Dp * 4) return GNNEA_EWORKSPACE;
  // rows whose last granule stays inside the table (the final row may end inside a granule)
  // (a column block of a wider buffer may end at the buffer end: only D bounds the row)
  const int64_t n_fast = (int64_t)G * E <= D ? n_rows : n_rows - 1;
  const int64_t rpb = (n_rows + nb - 1) / nb;
  float* part = (float*)ws;
#define GNNEA_DA_L(NGV, KV, HV)                                                                \
  hipLaunchKernelGGL((k_da_stream<T, NGV, KV, HV>), dim3(nb), dim3(64 * kDaWaves), 0, s, H,   \
                     ldh, n_rows, n_fast, rpb, D, heads, d_head, ds1, ds2, part)
#define GNNEA_DA_K(NGV)                                                                        \
  case NGV:                                                                                    \
    if (hh < 0) GNNEA_DA_L(NGV, 1, -1);                                                        \
    else if (K == 2) {                                                                         \
      if (hh == 4) GNNEA_DA_L(NGV, 2, 4); else GNNEA_DA_L(NGV, 2, 0);                          \
    } else if (hh == 4) GNNEA_DA_L(NGV, 1, 4);                                                 \
    else if (hh == 1) GNNEA_DA_L(NGV, 1, 1);                                                   \
    else GNNEA_DA_L(NGV, 1, 0);                                                                \
    break;
  switch (NG) {
    GNNEA_DA_K(1)
    GNNEA_DA_K(2)
    GNNEA_DA_K(3)
    GNNEA_DA_K(4)
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_DA_K
#undef GNNEA_DA_L
  GNNEA_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_gat_da_final, dim3((D + 63) / 64, K), dim3(512), 0, s, part, nb, K, D,
                     out1, out2);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

static int hh_of(int heads) { return heads == 4 ? 4 : heads == 1 ? 1 : 0; }

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_gat_da_ws_bytes(int64_t n_rows, int32_t D) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  return (int64_t)da_blocks(n_rows) * 2 * ((D + 3) & ~3) * 4;  // room for two weight sets
}

extern "C" int gnnea_gat_da_f32(const float* H, int64_t ldh, int64_t n_rows, int heads,
                                int d_head, const float* ds, float* out, void* ws,
                                int64_t ws_bytes, void* stream) {
  return da_t<float>(H, ldh, n_rows, heads, d_head, ds, nullptr, hh_of(heads), out, nullptr, ws,
                     ws_bytes, (hipStream_t)stream);
}

extern "C" int gnnea_gat_da_bf16(const void* H, int64_t ldh, int64_t n_rows, int heads,
                                 int d_head, const float* ds, float* out, void* ws,
                                 int64_t ws_bytes, void* stream) {
  return da_t<bf16_t>((const bf16_t*)H, ldh, n_rows, heads, d_head, ds, nullptr, hh_of(heads),
                      out, nullptr, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int gnnea_gat_da2_f32(const float* H, int64_t ldh, int64_t n_rows, int heads,
                                 int d_head, const float* ds1, const float* ds2, float* out1,
                                 float* out2, void* ws, int64_t ws_bytes, void* stream) {
  if (!out2) return GNNEA_EINVAL;
  return da_t<float>(H, ldh, n_rows, heads, d_head, ds1, ds2, hh_of(heads), out1, out2, ws,
                     ws_bytes, (hipStream_t)stream);
}

extern "C" int gnnea_gat_da2_bf16(const void* H, int64_t ldh, int64_t n_rows, int heads,
                                  int d_head, const float* ds1, const float* ds2, float* out1,
                                  float* out2, void* ws, int64_t ws_bytes, void* stream) {
  if (!out2) return GNNEA_EINVAL;
  return da_t<bf16_t>((const bf16_t*)H, ldh, n_rows, heads, d_head, ds1, ds2, hh_of(heads), out1,
                      out2, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int gnnea_colsum_f32(const float* X, int64_t ldx, int64_t n_rows, int32_t D,
                                float* out, void* ws, int64_t ws_bytes, void* stream) {
  if (D < 1) return D == 0 ? 0 : GNNEA_EINVAL;
  return da_t<float>(X, ldx, n_rows, 1, D, nullptr, nullptr, -1, out, nullptr, ws, ws_bytes,
                     (hipStream_t)stream);
}

extern "C" int gnnea_colsum_bf16(const void* X, int64_t ldx, int64_t n_rows, int32_t D,
                                 float* out, void* ws, int64_t ws_bytes, void* stream) {
  if (D < 1) return D == 0 ? 0 : GNNEA_EINVAL;
  return da_t<bf16_t>((const bf16_t*)X, ldx, n_rows, 1, D, nullptr, nullptr, -1, out, nullptr,
                      ws, ws_bytes, (hipStream_t)stream);
}
