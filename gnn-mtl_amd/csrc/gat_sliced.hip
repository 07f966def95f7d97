// a5-a6. GAT forward over a slice-major source table (the k_spmm_sliced layout of
// spmm_sliced.hip, applied to att_layers.py:29-61 x heads, concatenated at :86).
//
// k_gat_fwd (gat.hip) gathers every neighbour's whole head-concatenated row (1,200 B at
// d = 4 x 75: two load instructions per edge, the second with 11 of 64 lanes) from a 1.2-GB KG
// table.  Here the table is cut into 64-column fp32 slices (256 MB per KG slice, the Infinity
// Cache's size; one 256-B line pair per gathered piece) and the launch walks the slices one
// after another, as the sliced SpMM does.  Two kernels:
//   k_gat_rowstats  (wave per destination row, lanes over its edges): per head the row max
//                   m = max_j score_ij and the denominator den = sum_j exp(score_ij - m) — the
//                   records the backward needs — and every edge's numerator weights
//                   exp(score - m) * dropout mask ([nnz][heads] fp32, written once, read as
//                   coalesced rows by each slice pass instead of re-gathering s2 per slice);
//   k_gat_fwd_sliced (wave per (slice, row), 4 groups of 16 lanes as k_spmm_sliced): per chunk
//                   of 64 edges lane k loads edge k's weights for the (at most two) heads the
//                   slice's 64 columns belong to (d_head >= 32), broadcast by shuffle; each group
//                   accumulates w * Hs[j] for its edges,
//                   the group partials are summed in fixed order and group 0 writes
//                   act(acc / den) into the row-major output (the concat layout).
// fp32 arithmetic; the weights are those of k_gat_fwd (same exp, same max), the sum order is the
// sliced SpMM's, so outputs agree with k_gat_fwd to fp32 rounding.
#include "common.h"

namespace gnnea {

__device__ __forceinline__ float lrelu_s(float z, float alpha) { return z > 0.f ? z : alpha * z; }

template <int H>
__global__ __launch_bounds__(256) void k_gat_rowstats(const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col, int n_rows,
                                                      const float* __restrict__ s1,
                                                      const float* __restrict__ s2, float alpha,
                                                      const float* __restrict__ emask,
                                                      float* __restrict__ wgt,
                                                      float* __restrict__ m_out,
                                                      float* __restrict__ den_out) {
  const int row = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptr[row], end = rowptr[row + 1];
  float si[H], mx[H], den[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    si[h] = s1[(int64_t)row * H + h];
    mx[h] = -INFINITY;
    den[h] = 0.f;
  }
  for (int e = beg + lane; e < end; e += 64) {
    const int j = col[e];
#pragma unroll
    for (int h = 0; h < H; ++h) mx[h] = fmaxf(mx[h], -lrelu_s(si[h] + s2[(int64_t)j * H + h], alpha));
  }
#pragma unroll
  for (int h = 0; h < H; ++h) mx[h] = wave_max(mx[h]);
  for (int e = beg + lane; e < end; e += 64) {
    const int j = col[e];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float w = __expf(-lrelu_s(si[h] + s2[(int64_t)j * H + h], alpha) - mx[h]);
      den[h] += w;  // the row sum uses the un-dropped weights (att_layers.py:45-51)
      wgt[(int64_t)e * H + h] = emask ? w * emask[(int64_t)e * H + h] : w;
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) den[h] = wave_sum(den[h]);
  if (lane == 0) {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      m_out[(int64_t)row * H + h] = mx[h];
      den_out[(int64_t)row * H + h] = den[h];
    }
  }
}

template <int ACT, int U, typename TY>
__global__ __launch_bounds__(256) void k_gat_fwd_sliced(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, int n_rows, int nbs,
    int H, int D, int dh, const uint4* __restrict__ Hs, int64_t sstride16,
    const float* __restrict__ wgt, const float* __restrict__ den_in, TY* __restrict__ Y,
    int64_t ldy) {
  const int b = blockIdx.x;
  const int s = b / nbs;
  const int row = xcd_remap(b - s * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane >> 4, c = lane & 15;
  const int c0 = s * 64 + 4 * c;
  const bool own = c0 < D;
  // the slice's heads (d_head >= 32: at most two per 64 columns) and this lane's columns' heads
  const int h0 = min((s * 64) / dh, H - 1);
  const int h1 = min((s * 64 + 63) / dh, H - 1);
  bool second[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) second[t] = (c0 + t) / dh != h0;
  const uint4* X = Hs + (int64_t)s * sstride16 + c;
  const int beg = rowptr[row], end = rowptr[row + 1];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mj = 0;
    float w0 = 0.f, w1 = 0.f;
    if (lane < cnt) {  // edge base + lane: its (masked) weights for the slice's two heads
      mj = col[base + lane];
      w0 = wgt[(int64_t)(base + lane) * H + h0];
      w1 = wgt[(int64_t)(base + lane) * H + h1];
    }
    for (int k = 0; k < cnt; k += 4 * U) {
      uint4 r[U];
      float v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + 4 * u + g;  // <= 63: k is a multiple of 4U that divides 64
        const int j = __shfl(mj, e & 63, 64);
        v0[u] = __shfl(w0, e & 63, 64);
        v1[u] = __shfl(w1, e & 63, 64);
        if (e < cnt && own) {
          r[u] = X[(int64_t)j * 16];
        } else {
          r[u] = make_uint4(0u, 0u, 0u, 0u);
          v0[u] = v1[u] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float f[4] = {__builtin_bit_cast(float, r[u].x), __builtin_bit_cast(float, r[u].y),
                            __builtin_bit_cast(float, r[u].z), __builtin_bit_cast(float, r[u].w)};
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = fmaf(second[t] ? v1[u] : v0[u], f[t], acc[t]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] += __shfl_xor(acc[t], 16, 64);
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] += __shfl_xor(acc[t], 32, 64);
  if (g != 0 || !own) return;
  const float d0 = den_in[(int64_t)row * H + h0], d1 = den_in[(int64_t)row * H + h1];
  const float r0 = d0 > 0.f ? 1.f / d0 : 0.f, r1 = d1 > 0.f ? 1.f / d1 : 0.f;
  float o[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = c0 + t < D ? act_fwd<ACT>(acc[t] * (second[t] ? r1 : r0)) : 0.f;
  typedef typename Vec4<TY>::raw RY;
  *(RY*)(Y + (int64_t)row * ldy + c0) = Vec4<TY>::put(make_float4(o[0], o[1], o[2], o[3]));
}

}  // namespace gnnea

using namespace gnnea;

// the sliced forward: rowstats (m_out, den_out, per-edge weights in wgt: nnz x heads fp32,
// indexed by the absolute CSR position) + the aggregation; Hs slice-major fp32
// [ceil(D/64)][n_src][64] (sstride floats per slice), D % 4 == 0, d_head >= 32, ldy % 4 == 0
extern "C" int gnnea_gat_fwd_sliced_f32(const int32_t* rowptr, const int32_t* col,
                                        int32_t n_rows, const float* Hs, int64_t sstride,
                                        int heads, int d_head, const float* s1, const float* s2,
                                        float alpha, const float* edge_mask, int act, float* Y,
                                        int64_t ldy, float* m_out, float* den_out, float* wgt,
                                        void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int D = heads * d_head;
  if (n_rows < 0 || heads < 1 || heads > 8 || d_head < 32 || D % 4 || sstride % 64 ||
      ldy % 4 || ldy < D)
    return GNNEA_EINVAL;
  if (act != GNNEA_ACT_IDENTITY && act != GNNEA_ACT_RELU) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!rowptr || !col || !Hs || !s1 || !s2 || !Y || !m_out || !den_out || !wgt)
    return GNNEA_EINVAL;
  if (((uintptr_t)Hs & 15) || ((uintptr_t)Y & 15)) return GNNEA_EALIGN;
  const int nbs = div_up(n_rows, 4);
  switch (heads) {
#define GNNEA_RS(HH)                                                                             \
  case HH:                                                                                       \
    hipLaunchKernelGGL(k_gat_rowstats<HH>, dim3(nbs), dim3(256), 0, st, rowptr, col, n_rows, s1, \
                       s2, alpha, edge_mask, wgt, m_out, den_out);                               \
    break;
    GNNEA_RS(1) GNNEA_RS(2) GNNEA_RS(3) GNNEA_RS(4) GNNEA_RS(5) GNNEA_RS(6) GNNEA_RS(7)
    GNNEA_RS(8)
#undef GNNEA_RS
  }
  GNNEA_LAUNCH_CHECK();
  const int S = div_up(D, 64);
  const dim3 grid((unsigned)((int64_t)S * nbs));
  if (act == GNNEA_ACT_RELU)
    hipLaunchKernelGGL((k_gat_fwd_sliced<GNNEA_ACT_RELU, 4, float>), grid, dim3(256), 0, st,
                       rowptr, col, n_rows, nbs, heads, D, d_head, (const uint4*)Hs, sstride / 4,
                       wgt, den_out, Y, ldy);
  else
    hipLaunchKernelGGL((k_gat_fwd_sliced<GNNEA_ACT_IDENTITY, 4, float>), grid, dim3(256), 0, st,
                       rowptr, col, n_rows, nbs, heads, D, d_head, (const uint4*)Hs, sstride / 4,
                       wgt, den_out, Y, ldy);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
