// a2-a3. CSR neighbour aggregation over a slice-major feature table
// (replaces torch.spmm(adj, hidden) at layers/layers.py:35 when hidden exceeds the Infinity Cache).
//
// Table layout: the D feature columns are cut into S = ⌈D/64⌉ slices of 64 columns; element
// (r, c) lives at Xs[(c / 64)·sstride + r·64 + c % 64] (slice stride sstride ≥ n·64 floats).  One
// slice of a 1M-row KG is 256 MB, the size of the Infinity Cache, and every gathered piece is one
// 256-B pair of whole 128-B lines.  The launch walks the slices one after another (slice-major
// workgroup order), so while slice s is being aggregated its 256 MB table is what the gathers
// touch; measured on one cfg-4 KG (1M rows, 21M edges, D = 300): 3.40 ms against 4.26 ms for
// the row-major kernel over 1,200-B rows (tools/ubench/probe_slice.hip).
//
// Per wave: one destination row.  The 64 lanes are 4 groups of 16; lane c of a group owns the
// float4 at columns 4c..4c+3 of the slice, group g takes the row's neighbours g, g+4, ...,
// U per group in flight (16·U·256 B per wave).  The four group partials are summed at the end
// (fixed order: xor 16, then xor 32) and group 0 writes the row-major output row piece with the
// activation fused.  Deterministic; the summation order differs from the row-major kernel's
// CSR-order chain, so the two agree to fp32 rounding, not bit for bit.
#include "common.h"

namespace gnnea {

constexpr int kSliceW = 64;

// HighWay epilogue operands (layers/layers.py:64-76): gate_pre is read from a slice-major table
// at column offset goff (the fused HighWay layer's projection Z = x·[Wᵀ | K_g] is ONE sliced
// table: hidden in columns [0, D), gate_pre in [D, 2D)); resid, S, g are row-major.
struct SlicedHighway {
  const float4* gate;  // slice-major table holding gate_pre (nullptr: plain act epilogue)
  int64_t gsstride4;
  int goff;
  const float* bias;   // bias_gate (nullable)
  const float* resid;
  int64_t ldr;
  float* save_s;
  float* save_g;
  int64_t lds;
};

__device__ __forceinline__ float sigm_f(float x) { return 1.f / (1.f + expf(-x)); }

template <int ACT, int U, bool HW>
__global__ __launch_bounds__(256) void k_spmm_sliced(const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int n_rows,
                                                     int nbs, int D,
                                                     const float4* __restrict__ Xs,
                                                     int64_t sstride4, float* __restrict__ Y,
                                                     int64_t ldy, SlicedHighway hw) {
  const int b = blockIdx.x;
  const int s = b / nbs;
  const int row = xcd_remap(b - s * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane >> 4, c = lane & 15;
  const int c0 = s * kSliceW + 4 * c;
  const bool own = c0 < D;
  const float4* X = Xs + (int64_t)s * sstride4 + c;
  const int beg = rowptr[row], end = rowptr[row + 1];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int mc = lane < cnt ? col[base + lane] : 0;
    const float mv = lane < cnt ? val[base + lane] : 0.f;
    for (int k = 0; k < cnt; k += 4 * U) {
      float4 r[U];
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + 4 * u + g;  // <= 63: k is a multiple of 4U that divides 64
        const int j = __shfl(mc, e & 63, 64);
        v[u] = __shfl(mv, e & 63, 64);
        if (e < cnt && own) {
          r[u] = X[(int64_t)j * (kSliceW / 4)];
        } else {
          r[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          v[u] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc = f4_fma(v[u], r[u], acc);
    }
  }
  acc.x += __shfl_xor(acc.x, 16, 64);
  acc.y += __shfl_xor(acc.y, 16, 64);
  acc.z += __shfl_xor(acc.z, 16, 64);
  acc.w += __shfl_xor(acc.w, 16, 64);
  acc.x += __shfl_xor(acc.x, 32, 64);
  acc.y += __shfl_xor(acc.y, 32, 64);
  acc.z += __shfl_xor(acc.z, 32, 64);
  acc.w += __shfl_xor(acc.w, 32, 64);
  if (g == 0 && own) {
    const float4 sv = make_float4(act_fwd<ACT>(acc.x), act_fwd<ACT>(acc.y), act_fwd<ACT>(acc.z),
                                  act_fwd<ACT>(acc.w));
    if constexpr (!HW) {
      *(float4*)(Y + (int64_t)row * ldy + c0) = sv;
    } else {
      const int gc = hw.goff + c0;  // gate_pre column in its table (multiple of 4)
      float4 gp = hw.gate[(int64_t)(gc >> 6) * hw.gsstride4 + (int64_t)row * (kSliceW / 4) +
                          ((gc & 63) >> 2)];
      if (hw.bias) {
        const float4 b = *(const float4*)(hw.bias + c0);
        gp.x += b.x; gp.y += b.y; gp.z += b.z; gp.w += b.w;
      }
      const float4 gt = make_float4(sigm_f(gp.x), sigm_f(gp.y), sigm_f(gp.z), sigm_f(gp.w));
      const float4 r = *(const float4*)(hw.resid + (int64_t)row * hw.ldr + c0);
      // reference order: transform_gate * support + carry_gate * residual, carry = 1 - g
      float4 o;
      o.x = gt.x * sv.x + (1.f - gt.x) * r.x;
      o.y = gt.y * sv.y + (1.f - gt.y) * r.y;
      o.z = gt.z * sv.z + (1.f - gt.z) * r.z;
      o.w = gt.w * sv.w + (1.f - gt.w) * r.w;
      *(float4*)(Y + (int64_t)row * ldy + c0) = o;
      if (hw.save_s) *(float4*)(hw.save_s + (int64_t)row * hw.lds + c0) = sv;
      if (hw.save_g) *(float4*)(hw.save_g + (int64_t)row * hw.lds + c0) = gt;
    }
  }
}

// Row-major [n, D] -> slice-major table.  BWD: the table holds G = dY ⊙ act'(Y) (the backward
// aggregation's input, fused with its activation derivative); otherwise a copy of X = dY.
// One wave per row (no integer division per element), lane q moves float4 q, q+64, ...
template <int ACT, bool BWD>
__global__ __launch_bounds__(256) void k_slice_fill(const float4* __restrict__ dY, int64_t ld4,
                                                    const float4* __restrict__ Yo,
                                                    int64_t ldo4, int64_t n, int D4,
                                                    float4* __restrict__ Gs, int64_t sstride4) {
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();
  if (r >= n) return;
  for (int q = lane_id(); q < D4; q += 64) {
    float4 v = dY[r * ld4 + q];
    if constexpr (BWD) {
      const float4 y = Yo[r * ldo4 + q];
      v.x *= act_grad_from_out<ACT>(y.x);
      v.y *= act_grad_from_out<ACT>(y.y);
      v.z *= act_grad_from_out<ACT>(y.z);
      v.w *= act_grad_from_out<ACT>(y.w);
    }
    Gs[(int64_t)(q >> 4) * sstride4 + r * (kSliceW / 4) + (q & 15)] = v;
  }
}

static bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }  // nullptr passes

template <bool BWD>
static int slice_fill(const float* dY, int64_t ld, const float* Y, int64_t ldo, int64_t n, int D,
                      float* Gs, int64_t sstride, int act, hipStream_t s) {
  if (n < 0 || D < 0) return GNNEA_EINVAL;
  if (n == 0 || D == 0) return 0;
  if (!dY || !Gs || (BWD && !Y)) return GNNEA_EINVAL;
  if (D % 4 || ld % 4 || (BWD && ldo % 4) || sstride % 4 || ld < D || (BWD && ldo < D) ||
      sstride < n * kSliceW || !al16(dY) || !al16(Gs) || (BWD && !al16(Y)))
    return GNNEA_EINVAL;
  if ((n + 3) / 4 >= (1ll << 31)) return GNNEA_EINVAL;
  const int nb = (int)((n + 3) / 4);
#define GNNEA_SF(A)                                                                            \
  hipLaunchKernelGGL((k_slice_fill<A, BWD>), dim3(nb), dim3(256), 0, s, (const float4*)dY,     \
                     ld / 4, (const float4*)Y, ldo / 4, n, D / 4, (float4*)Gs, sstride / 4)
  switch (BWD ? act : GNNEA_ACT_IDENTITY) {
    case GNNEA_ACT_IDENTITY: GNNEA_SF(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_SF(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_SF(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_SF(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_SF(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_SF(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_SF
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

namespace gnnea {

template <bool HW>
static int spmm_sliced(const int32_t* rowptr, const int32_t* col, const float* val,
                       int32_t n_rows, int32_t D, const float* Xs, int64_t sstride, float* Y,
                       int64_t ldy, int act, const SlicedHighway& hw, hipStream_t s) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !Xs || !Y) return GNNEA_EINVAL;
  if (D % 4 || ldy % 4 || ldy < D || sstride % 4 || sstride < kSliceW || !al16(Xs) || !al16(Y))
    return GNNEA_EINVAL;
  if (HW && (!hw.gate || !hw.resid || hw.goff < 0 || hw.goff % 4 || hw.gsstride4 < kSliceW / 4 ||
             hw.ldr % 4 || hw.ldr < D || !al16(hw.gate) || !al16(hw.resid) || !al16(hw.bias) ||
             ((hw.save_s || hw.save_g) && (hw.lds % 4 || hw.lds < D)) || !al16(hw.save_s) ||
             !al16(hw.save_g)))
    return GNNEA_EINVAL;
  const int nbs = (n_rows + 3) / 4;
  const int S = (D + kSliceW - 1) / kSliceW;
  if ((int64_t)nbs * S >= (1ll << 31)) return GNNEA_EINVAL;
#define GNNEA_SS(A)                                                                            \
  hipLaunchKernelGGL((k_spmm_sliced<A, 4, HW>), dim3(nbs * S), dim3(256), 0, s, rowptr, col,   \
                     val, n_rows, nbs, D, (const float4*)Xs, sstride / 4, Y, ldy, hw)
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_SS(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_SS(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_SS(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_SS(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_SS(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_SS(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_SS
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

extern "C" int gnnea_spmm_sliced_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                                     int32_t n_rows, int32_t D, const float* Xs, int64_t sstride,
                                     float* Y, int64_t ldy, int act, void* stream) {
  const SlicedHighway none{nullptr, 0, 0, nullptr, nullptr, 0, nullptr, nullptr, 0};
  return spmm_sliced<false>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy, act, none,
                            (hipStream_t)stream);
}

extern "C" int gnnea_spmm_highway_sliced_f32(const int32_t* rowptr, const int32_t* col,
                                             const float* val, int32_t n_rows, int32_t D,
                                             const float* Xs, int64_t sstride,
                                             const float* gate_s, int64_t gsstride,
                                             int32_t goff, const float* bias_gate,
                                             const float* resid, int64_t ldr, float* Y,
                                             int64_t ldy, float* save_s, float* save_g,
                                             int64_t lds, int act, void* stream) {
  if (gsstride % 4) return GNNEA_EINVAL;
  const SlicedHighway hw{(const float4*)gate_s, gsstride / 4, goff, bias_gate, resid, ldr,
                         save_s, save_g, lds};
  return spmm_sliced<true>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy, act, hw,
                           (hipStream_t)stream);
}

extern "C" int gnnea_slice_pack_f32(const float* X, int64_t ldx, int64_t n, int32_t D,
                                    float* Xs, int64_t sstride, void* stream) {
  return slice_fill<false>(X, ldx, nullptr, 0, n, D, Xs, sstride, GNNEA_ACT_IDENTITY,
                           (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_sliced_f32(const float* dY, int64_t lddy, const float* Y,
                                        int64_t ldy, int64_t n, int32_t D, int act, float* Gs,
                                        int64_t sstride, void* stream) {
  return slice_fill<true>(dY, lddy, Y, ldy, n, D, Gs, sstride, act, (hipStream_t)stream);
}
