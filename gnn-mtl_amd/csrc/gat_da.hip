// a7. GAT attention-vector gradient (autograd of att_layers.py:38, a·[h_i || h_j]):
//   da1[h] = Σ_i ds1[i,h] · H[i, h-block],   da2[h] = Σ_j ds2[j,h] · H[j, h-block]
// i.e. out[c] = Σ_r ds[r, c / d_head] · H[r, c] for every column c of the head-concatenated H.
// One streaming pass over H (N·D·s bytes, HBM bound) instead of an [N, heads]ᵀ·[N, D] GEMM whose
// off-diagonal head blocks are thrown away: stage 1, up to 256 workgroups each sums a
// contiguous row range into registers (16 waves on interleaved rows, 4 rows in flight per wave,
// lane = float4 column chunk), combined across the waves in LDS into one partial row per workgroup; stage 2 adds the
// workgroup partials in workgroup order (deterministic, no atomics).
#include "common.h"

namespace gnnea {

constexpr int kDaBlocks = 256, kDaWaves = 16;

// HH: the head count when it is 4 (one 16-B load of a row's ds, broadcast to the wave, and a
// per-element select of its lane's head), 0 = any (one ds load per element)
template <int NCH, typename T, int HH>
__global__ __launch_bounds__(64 * kDaWaves) void k_gat_da_part(const typename Vec4<T>::raw* __restrict__ H,
                                                     int64_t ldh4, int64_t n_rows, int heads,
                                                     int d_head, int D4,
                                                     const float* __restrict__ ds,
                                                     float* __restrict__ part) {
  __shared__ float4 red[kDaWaves][64 * NCH];
  const int w = wave_id(), lane = lane_id();
  const int64_t rpb = (n_rows + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = (int64_t)blockIdx.x * rpb, r1 = min(n_rows, r0 + rpb);
  float4 acc[NCH];
  int hd[NCH][4];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * (lane + 64 * q) + t;
      hd[q][t] = min(c / d_head, heads - 1);
    }
  }
  auto fma_row = [&](int64_t r, const float4 (&h)[NCH]) {
    const float* dr = ds + r * heads;
    if constexpr (HH == 4) {  // r is wave-uniform: one 16-B load, selects per element
      const float4 d4 = *(const float4*)dr;
      auto sel = [&](int k) { return k == 0 ? d4.x : (k == 1 ? d4.y : (k == 2 ? d4.z : d4.w)); };
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        acc[q].x = fmaf(sel(hd[q][0]), h[q].x, acc[q].x);
        acc[q].y = fmaf(sel(hd[q][1]), h[q].y, acc[q].y);
        acc[q].z = fmaf(sel(hd[q][2]), h[q].z, acc[q].z);
        acc[q].w = fmaf(sel(hd[q][3]), h[q].w, acc[q].w);
      }
    } else {
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        acc[q].x = fmaf(dr[hd[q][0]], h[q].x, acc[q].x);
        acc[q].y = fmaf(dr[hd[q][1]], h[q].y, acc[q].y);
        acc[q].z = fmaf(dr[hd[q][2]], h[q].z, acc[q].z);
        acc[q].w = fmaf(dr[hd[q][3]], h[q].w, acc[q].w);
      }
    }
  };
  auto load_row = [&](int64_t r, float4 (&h)[NCH]) {
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int c4 = lane + 64 * q;
      h[q] = c4 < D4 ? Vec4<T>::get(H[r * ldh4 + c4]) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // the wave's rows r0+w, r0+w+W, ... in order; four of them loaded before their FMAs
  constexpr int W = kDaWaves;
  int64_t r = r0 + w;
  for (; r + 3 * W < r1; r += 4 * W) {
    float4 h[4][NCH];
#pragma unroll
    for (int u = 0; u < 4; ++u) load_row(r + W * u, h[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) fma_row(r + W * u, h[u]);
  }
  for (; r < r1; r += W) {
    float4 h[NCH];
    load_row(r, h);
    fma_row(r, h);
  }
#pragma unroll
  for (int q = 0; q < NCH; ++q) red[w][lane + 64 * q] = acc[q];
  __syncthreads();
  for (int c4 = threadIdx.x; c4 < D4; c4 += 64 * W) {
    float4 s = red[0][c4];
#pragma unroll
    for (int k = 1; k < W; ++k) {
      const float4 o = red[k][c4];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
    }
    ((float4*)part)[(int64_t)blockIdx.x * D4 + c4] = s;
  }
}

// 64 columns per workgroup, the 8 waves stride the partials (4 independent sums per lane),
// combined in wave order through LDS: deterministic, latency hidden across the waves.
__global__ __launch_bounds__(512) void k_gat_da_final(const float* __restrict__ part, int nb,
                                                      int D, float* __restrict__ out) {
  __shared__ float red[8][64];
  const int w = wave_id(), lane = lane_id();
  const int c = blockIdx.x * 64 + lane;
  const int64_t ld = (D + 3) & ~3;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    int b = w;
    for (; b + 24 < nb; b += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += part[(int64_t)(b + 8 * u) * ld + c];
    }
    for (int u = 0; b < nb; b += 8, ++u) s[u & 3] += part[(int64_t)b * ld + c];
  }
  red[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (w == 0 && c < D) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][lane];
    out[c] = t;
  }
}

static int da_blocks(int64_t n_rows) {
  const int64_t b = (n_rows + 63) / 64;  // >= 64 rows per workgroup (4 per wave), <= 256 of them
  return (int)(b < 1 ? 1 : (b > kDaBlocks ? kDaBlocks : b));
}

template <typename T>
static int gat_da_t(const T* H, int64_t ldh, int64_t n_rows, int heads, int d_head,
                    const float* ds, float* out, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  const int D = heads * d_head;
  if (!out) return GNNEA_EINVAL;
  if (n_rows == 0) return (int)hipMemsetAsync(out, 0, sizeof(float) * D, s);
  // rows are read as whole 4-element vectors up to Dp = roundup4(D) (the GAT layer pads H so);
  // the columns past D are summed into the partials but never written out
  const int Dp = (D + 3) & ~3;
  if (!H || !ds || ldh % 4 || ldh < Dp ||
      (((uintptr_t)H) & (sizeof(typename Vec4<T>::raw) - 1)))
    return GNNEA_EINVAL;
  const int D4 = Dp / 4, nch = (D4 + 63) / 64;
  const int nb = da_blocks(n_rows);
  if (!ws || ws_bytes < (int64_t)nb * Dp * 4) return GNNEA_EWORKSPACE;
  float* part = (float*)ws;
  typedef typename Vec4<T>::raw R;
  const bool h4 = heads == 4 && (((uintptr_t)ds) & 15) == 0;
#define GNNEA_DA(N)                                                                            \
  case N:                                                                                      \
    if (h4)                                                                                    \
      hipLaunchKernelGGL((k_gat_da_part<N, T, 4>), dim3(nb), dim3(64 * kDaWaves), 0, s,        \
                         (const R*)H, ldh / 4, n_rows, heads, d_head, D4, ds, part);           \
    else                                                                                       \
      hipLaunchKernelGGL((k_gat_da_part<N, T, 0>), dim3(nb), dim3(64 * kDaWaves), 0, s,        \
                         (const R*)H, ldh / 4, n_rows, heads, d_head, D4, ds, part);           \
    break;
  switch (nch) {
    GNNEA_DA(1)
    GNNEA_DA(2)
    GNNEA_DA(3)
    GNNEA_DA(4)
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_DA
  GNNEA_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_gat_da_final, dim3((D + 63) / 64), dim3(512), 0, s, part, nb, D, out);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_gat_da_ws_bytes(int64_t n_rows, int32_t D) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  return (int64_t)da_blocks(n_rows) * ((D + 3) & ~3) * 4;
}

extern "C" int gnnea_gat_da_f32(const float* H, int64_t ldh, int64_t n_rows, int heads,
                                int d_head, const float* ds, float* out, void* ws,
                                int64_t ws_bytes, void* stream) {
  return gat_da_t<float>(H, ldh, n_rows, heads, d_head, ds, out, ws, ws_bytes,
                         (hipStream_t)stream);
}

extern "C" int gnnea_gat_da_bf16(const void* H, int64_t ldh, int64_t n_rows, int heads,
                                 int d_head, const float* ds, float* out, void* ws,
                                 int64_t ws_bytes, void* stream) {
  return gat_da_t<bf16_t>((const bf16_t*)H, ldh, n_rows, heads, d_head, ds, out, ws, ws_bytes,
                          (hipStream_t)stream);
}
