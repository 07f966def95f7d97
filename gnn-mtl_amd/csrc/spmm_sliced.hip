// a2-a4. CSR neighbour aggregation over a slice-major feature table
// (replaces torch.spmm(adj, hidden) at layers/layers.py:35 when hidden exceeds the Infinity Cache).
//
// Table layout: the D feature columns are cut into S = ⌈D/W⌉ slices of W columns, W·sizeof(T) =
// 256 B (W = 64 fp32, 128 bf16); element (r, c) lives at Xs[(c / W)·sstride + r·W + c % W]
// (slice stride sstride ≥ n·W elements).  One fp32 slice of a 1M-row KG is 256 MB, the size of
// the Infinity Cache, and every gathered piece is one 256-B pair of whole 128-B lines.  The launch
// walks the slices one after another (slice-major workgroup order), so while slice s is being
// aggregated its table is what the gathers touch; measured on one cfg-4 KG (1M rows, 21M edges,
// D = 300 fp32): 3.40 ms against 4.26 ms for the row-major kernel over 1,200-B rows
// (tools/ubench/probe_slice.hip).
//
// Per wave: one destination row.  The 64 lanes are 4 groups of 16; lane c of a group owns the
// 16 B (E = 4 fp32 / 8 bf16 elements) at columns E·c.. of the slice, group g takes the row's
// neighbours g, g+4, ..., U per group in flight (16·U·256 B per wave).  The four group partials
// are summed at the end (fixed order: xor 16, then xor 32) and group 0 writes the row-major output
// row piece with the activation (or the HighWay blend) fused.  fp32 arithmetic for both storage
// types.  Deterministic; the summation order differs from the row-major kernel's CSR-order chain,
// so the two agree to fp32 rounding, not bit for bit.
#include "common.h"

#include <stdlib.h>

namespace gnnea {

template <typename T>
struct SliceOf {
  static constexpr int W = 256 / (int)sizeof(T);  // columns per slice
  static constexpr int E = 16 / (int)sizeof(T);   // elements per lane (16 B)
};
constexpr int kSliceW = SliceOf<float>::W;

// HighWay epilogue operands (layers/layers.py:64-76), fp32 tables only: gate_pre is read from a
// slice-major table at column offset goff (the fused HighWay layer's projection
// Z = x·[Wᵀ | K_g] is ONE sliced table: hidden in columns [0, D), gate_pre in [D, 2D)); resid,
// S, g are row-major.
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
  // (relu only) instead of S, its sign: byte [row][16 slice + lane] holds bit q = S > 0 for the
  // lane's column 4 lane + q of the slice; the backward takes act' from it and S - x from the
  // output (out - x = g (S - x)), so S itself is never stored
  uint8_t* save_m = nullptr;
  int64_t ldm = 0;
};

__device__ __forceinline__ float sigm_f(float x) { return gate_sigmoid(x); }

// The gathers of a row are issued unconditionally (edges past the chunk re-read its last edge's
// piece with weight 0; lanes past D read their group's first 16 B and discard the sum), in
// batches of 4U edges with the next batch in flight while one is summed (register double buffer),
// so no gathered piece is waited on inside a branch (behind per-lane conditions, one batch at a
// time, the same kernel measured slower: round 3).  Per-lane sum order: edge k + 4u + g, u
// ascending.
template <int ACT, int U, bool HW, typename TX, typename TY>
__global__ __launch_bounds__(256) void k_spmm_sliced(const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int n_rows,
                                                     int nbs, int D,
                                                     const uint4* __restrict__ Xs,
                                                     int64_t sstride16, TY* __restrict__ Y,
                                                     int64_t ldy, SlicedHighway hw) {
  constexpr int E = SliceOf<TX>::E, W = SliceOf<TX>::W;
  const int b = blockIdx.x;
  const int s = b / nbs;
  const int row = xcd_remap(b - s * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane >> 4, c = lane & 15;
  const int c0 = s * W + E * c;
  const bool own = c0 < D;
  const int beg = rowptr[row], end = rowptr[row + 1];
  // HighWay epilogue operands (gate_pre, bias_gate, resid of this row piece) loaded by every
  // lane from a clamped column BEFORE the gathers: the groups share group 0's addresses (no extra
  // lines), and their latency hides under the row's gathers instead of following them (read in
  // the epilogue they cost one serial round trip per row after the reduction)
  float4 hgp[E / 4], hrr[E / 4];
  if constexpr (HW) {
#pragma unroll
    for (int k = 0; k < E / 4; ++k) {
      const int cc = min(c0 + 4 * k, D - 4);
      const int gc = hw.goff + cc;
      hgp[k] = hw.gate[(int64_t)(gc >> 6) * hw.gsstride4 + (int64_t)row * (kSliceW / 4) +
                       ((gc & 63) >> 2)];
      hrr[k] = *(const float4*)(hw.resid + (int64_t)row * hw.ldr + cc);
      if (hw.bias) {
        const float4 bv = *(const float4*)(hw.bias + cc);
        hgp[k].x += bv.x; hgp[k].y += bv.y; hgp[k].z += bv.z; hgp[k].w += bv.w;
      }
    }
  }
  float acc[E];
#pragma unroll
  for (int k = 0; k < E; ++k) acc[k] = 0.f;
  const uint4* Xp = Xs + (int64_t)s * sstride16 + (own ? c : 0);
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int el = base + min(lane, cnt - 1);
    const int mc = col[el];
    const float mv = val[el] * (lane < cnt ? 1.f : 0.f);  // (a select would sink the load)
    uint4 ra[U], rb[U];
    auto issue = [&](uint4 (&r)[U], int k) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = __shfl(mc, min(k + 4 * u + g, cnt - 1), 64);
        r[u] = Xp[(int64_t)j * 16];
      }
    };
    auto consume = [&](const uint4 (&r)[U], int k) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + 4 * u + g;
        // (the shuffle runs in every lane: a bpermute from a lane masked off by the
        // condition would return its inactive value)
        const float vs = __shfl(mv, e & 63, 64);
        const float v = e < cnt ? vs : 0.f;
        float f[E];
        unpack16(r[u], f);
#pragma unroll
        for (int q = 0; q < E; ++q) acc[q] = fmaf(v, f[q], acc[q]);
      }
    };
    issue(ra, 0);
    for (int k = 0; k < cnt; k += 8 * U) {
      issue(rb, k + 4 * U);
      __builtin_amdgcn_sched_barrier(0);  // the next batch's gathers ahead of this batch's FMAs
      consume(ra, k);
      issue(ra, k + 8 * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(rb, k + 4 * U);
    }
  }
#pragma unroll
  for (int q = 0; q < E; ++q) acc[q] += __shfl_xor(acc[q], 16, 64);
#pragma unroll
  for (int q = 0; q < E; ++q) acc[q] += __shfl_xor(acc[q], 32, 64);
  if (g != 0 || !own) return;
#pragma unroll
  for (int k = 0; k < E / 4; ++k) {
    const int cc = c0 + 4 * k;  // chunks of 4 columns (D % 4 == 0)
    if (cc >= D) break;
    const float4 sv = make_float4(act_fwd<ACT>(acc[4 * k]), act_fwd<ACT>(acc[4 * k + 1]),
                                  act_fwd<ACT>(acc[4 * k + 2]), act_fwd<ACT>(acc[4 * k + 3]));
    typedef typename Vec4<TY>::raw RY;
    if constexpr (!HW) {
      *(RY*)(Y + (int64_t)row * ldy + cc) = Vec4<TY>::put(sv);
      if constexpr (E == 4) {  // (the GCN layer's relu: its sign bits for the backward, as HW)
        if (hw.save_m)
          hw.save_m[(int64_t)row * hw.ldm + 16 * s + c] = (uint8_t)(
              (sv.x > 0.f) | ((sv.y > 0.f) << 1) | ((sv.z > 0.f) << 2) | ((sv.w > 0.f) << 3));
      }
    } else {
      const float4 gp = hgp[k];  // gate_pre + bias_gate (loaded before the gathers)
      const float4 gt = make_float4(sigm_f(gp.x), sigm_f(gp.y), sigm_f(gp.z), sigm_f(gp.w));
      const float4 rr = hrr[k];
      // reference order: transform_gate * support + carry_gate * residual, carry = 1 - g
      float4 o;
      o.x = gt.x * sv.x + (1.f - gt.x) * rr.x;
      o.y = gt.y * sv.y + (1.f - gt.y) * rr.y;
      o.z = gt.z * sv.z + (1.f - gt.z) * rr.z;
      o.w = gt.w * sv.w + (1.f - gt.w) * rr.w;
      *(float4*)(Y + (int64_t)row * ldy + cc) = o;
      if (hw.save_s) *(float4*)(hw.save_s + (int64_t)row * hw.lds + cc) = sv;
      if (hw.save_m)
        hw.save_m[(int64_t)row * hw.ldm + 16 * s + c] =
            (uint8_t)((sv.x > 0.f) | ((sv.y > 0.f) << 1) | ((sv.z > 0.f) << 2) | ((sv.w > 0.f) << 3));
      if (hw.save_g) *(float4*)(hw.save_g + (int64_t)row * hw.lds + cc) = gt;
    }
  }
}

// Row-major [n, D] -> slice-major table, 4 elements per lane step.  BWD: the table holds
// G = dY ⊙ act'(Y) (the backward aggregation's input, fused with its activation derivative);
// otherwise a copy of X = dY.  One wave per row (no integer division per element).
template <int ACT, bool BWD, typename T>
__global__ __launch_bounds__(256) void k_slice_fill(const typename Vec4<T>::raw* __restrict__ dY,
                                                    int64_t ld4,
                                                    const typename Vec4<T>::raw* __restrict__ Yo,
                                                    int64_t ldo4, int64_t n, int D4,
                                                    typename Vec4<T>::raw* __restrict__ Gs,
                                                    int64_t sstride4) {
  constexpr int W4 = SliceOf<T>::W / 4;  // 4-element chunks per slice row
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();
  if (r >= n) return;
  for (int q = lane_id(); q < D4; q += 64) {
    typename Vec4<T>::raw v = dY[r * ld4 + q];
    if constexpr (BWD) {
      float4 d = Vec4<T>::get(v);
      const float4 y = Vec4<T>::get(Yo[r * ldo4 + q]);
      d.x *= act_grad_from_out<ACT>(y.x);
      d.y *= act_grad_from_out<ACT>(y.y);
      d.z *= act_grad_from_out<ACT>(y.z);
      d.w *= act_grad_from_out<ACT>(y.w);
      v = Vec4<T>::put(d);
    }
    Gs[(int64_t)(q / W4) * sstride4 + r * W4 + (q % W4)] = v;
  }
}

template <typename T>
static bool aln(const void* p) {  // aligned for one Vec4<T> (nullptr passes)
  return (((uintptr_t)p) & (sizeof(typename Vec4<T>::raw) - 1)) == 0;
}
static bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }  // nullptr passes

template <bool BWD, typename T>
static int slice_fill(const T* dY, int64_t ld, const T* Y, int64_t ldo, int64_t n, int D, T* Gs,
                      int64_t sstride, int act, hipStream_t s) {
  constexpr int W = SliceOf<T>::W;
  if (n < 0 || D < 0) return GNNEA_EINVAL;
  if (n == 0 || D == 0) return 0;
  if (!dY || !Gs || (BWD && !Y)) return GNNEA_EINVAL;
  if (D % 4 || ld % 4 || (BWD && ldo % 4) || sstride % 4 || ld < D || (BWD && ldo < D) ||
      sstride < n * W || !aln<T>(dY) || !al16(Gs) || (BWD && !aln<T>(Y)))
    return GNNEA_EINVAL;
  if ((n + 3) / 4 >= (1ll << 31)) return GNNEA_EINVAL;
  const int nb = (int)((n + 3) / 4);
  typedef typename Vec4<T>::raw R;
#define GNNEA_SF(A)                                                                            \
  hipLaunchKernelGGL((k_slice_fill<A, BWD, T>), dim3(nb), dim3(256), 0, s, (const R*)dY,       \
                     ld / 4, (const R*)Y, ldo / 4, n, D / 4, (R*)Gs, sstride / 4)
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

// G = dY * relu'(Y) written slice-major with relu' from the forward's sign bits (mask byte q of a
// row = its 4-element chunk q, bit e = element 4 q + e > 0): fp32 (16 chunks per slice row)
__global__ __launch_bounds__(256) void k_slice_fill_bits(const float4* __restrict__ dY,
                                                         int64_t ld4,
                                                         const uint8_t* __restrict__ M,
                                                         int64_t ldm, int64_t n, int D4,
                                                         float4* __restrict__ Gs,
                                                         int64_t sstride4) {
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();
  if (r >= n) return;
  for (int q = lane_id(); q < D4; q += 64) {
    float4 d = dY[r * ld4 + q];
    const uint32_t b = M[r * ldm + q];
    d.x *= (b & 1u) ? 1.f : 0.f;  // (act_grad_from_out<relu>: y > 0 ? 1 : 0, multiplied)
    d.y *= (b & 2u) ? 1.f : 0.f;
    d.z *= (b & 4u) ? 1.f : 0.f;
    d.w *= (b & 8u) ? 1.f : 0.f;
    Gs[(int64_t)(q >> 4) * sstride4 + r * 16 + (q & 15)] = d;
  }
}

template <bool HW, typename TX, typename TY>
static int spmm_sliced(const int32_t* rowptr, const int32_t* col, const float* val,
                       int32_t n_rows, int32_t D, const TX* Xs, int64_t sstride, TY* Y,
                       int64_t ldy, int act, const SlicedHighway& hw, hipStream_t s) {
  constexpr int W = SliceOf<TX>::W;
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !Xs || !Y) return GNNEA_EINVAL;
  if (D % 4 || ldy % 4 || ldy < D || sstride % W || sstride < W || !al16(Xs) || !aln<TY>(Y))
    return GNNEA_EINVAL;
  if (HW && (!hw.gate || !hw.resid || hw.goff < 0 || hw.goff % 4 || hw.gsstride4 < kSliceW / 4 ||
             hw.ldr % 4 || hw.ldr < D || !al16(hw.gate) || !al16(hw.resid) || !al16(hw.bias) ||
             ((hw.save_s || hw.save_g) && (hw.lds % 4 || hw.lds < D)) || !al16(hw.save_s) ||
             !al16(hw.save_g)))
    return GNNEA_EINVAL;
  const int nbs = (n_rows + 3) / 4;
  const int S = (D + W - 1) / W;
  if ((int64_t)nbs * S >= (1ll << 31)) return GNNEA_EINVAL;
  const int64_t ss16 = sstride * (int64_t)sizeof(TX) / 16;
#define GNNEA_SS(A)                                                                            \
  hipLaunchKernelGGL((k_spmm_sliced<A, 2, HW, TX, TY>), dim3(nbs * S), dim3(256), 0, s, rowptr, \
                     col, val, n_rows, nbs, D, (const uint4*)Xs, ss16, Y, ldy, hw)
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

constexpr SlicedHighway kNoHighway{nullptr, 0, 0, nullptr, nullptr, 0, nullptr, nullptr, 0};

// bf16 over 64-column slices (the GAT tables' layout, gnnea_slice_pack64_bf16): a slice row piece
// is 128 B = one line and one cfg-5 KG slice (2M rows) is 256 MB, the Infinity Cache's size (the
// 128-column form above is 512 MB per KG slice).  Lane c of an 8-lane group owns 8 columns (16 B:
// 8-B lane accesses run at 0.54-0.70 of the 16-B rate, MI355X_MICROARCH.md), the 8 groups take
// neighbours g, g + 8, ...: one wave instruction gathers 8 whole row pieces.  Gathers issued
// unconditionally in double-buffered batches of 8U edges (the PIPE scheme of k_spmm_sliced),
// fp32 sums, the group partials summed in fixed order (xor 8, 16, 32), group 0 writes the row
// piece with the activation fused (a last slice ending 4 columns into a lane's 8 stores 4).
constexpr int kS64U = 2;  // edges per group and batch
template <int ACT, int U, typename TY>
__global__ __launch_bounds__(256) void k_spmm_sliced64_bf16(const int32_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ col,
                                                            const float* __restrict__ val,
                                                            int n_rows, int nbs, int D,
                                                            const uint4* __restrict__ Xs,
                                                            int64_t sstride16, TY* __restrict__ Y,
                                                            int64_t ldy) {
  const int b = blockIdx.x;
  const int s = b / nbs;
  const int row = xcd_remap(b - s * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane >> 3, c = lane & 7;
  const int c0 = s * 64 + 8 * c;
  const bool own = c0 < D;
  const uint4* Xp = Xs + (int64_t)s * sstride16 + (own ? c : 0);
  const int beg = rowptr[row], end = rowptr[row + 1];
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int el = base + min(lane, cnt - 1);
    const int mc = col[el];
    const float mv = val[el] * (lane < cnt ? 1.f : 0.f);
    uint4 ra[U], rb[U];
    auto issue = [&](uint4 (&r)[U], int k) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = __shfl(mc, min(k + 8 * u + g, cnt - 1), 64);
        r[u] = Xp[(int64_t)j * 8];
      }
    };
    auto consume = [&](const uint4 (&r)[U], int k) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + 8 * u + g;
        const float vs = __shfl(mv, e & 63, 64);
        const float v = e < cnt ? vs : 0.f;
        const float4 lo = Vec4<bf16_t>::get(make_uint2(r[u].x, r[u].y));
        const float4 hi = Vec4<bf16_t>::get(make_uint2(r[u].z, r[u].w));
        acc[0] = fmaf(v, lo.x, acc[0]);
        acc[1] = fmaf(v, lo.y, acc[1]);
        acc[2] = fmaf(v, lo.z, acc[2]);
        acc[3] = fmaf(v, lo.w, acc[3]);
        acc[4] = fmaf(v, hi.x, acc[4]);
        acc[5] = fmaf(v, hi.y, acc[5]);
        acc[6] = fmaf(v, hi.z, acc[6]);
        acc[7] = fmaf(v, hi.w, acc[7]);
      }
    };
    issue(ra, 0);
    for (int k = 0; k < cnt; k += 16 * U) {
      issue(rb, k + 8 * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(ra, k);
      issue(ra, k + 16 * U);
      __builtin_amdgcn_sched_barrier(0);
      consume(rb, k + 8 * U);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] += __shfl_xor(acc[q], 8, 64);
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] += __shfl_xor(acc[q], 16, 64);
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] += __shfl_xor(acc[q], 32, 64);
  if (g != 0 || !own) return;
  typedef typename Vec4<TY>::raw RY;
  const float4 s0 = make_float4(act_fwd<ACT>(acc[0]), act_fwd<ACT>(acc[1]), act_fwd<ACT>(acc[2]),
                                act_fwd<ACT>(acc[3]));
  *(RY*)(Y + (int64_t)row * ldy + c0) = Vec4<TY>::put(s0);
  if (c0 + 4 < D) {  // D % 4 == 0: the lane's second 4 columns are wholly in or out
    const float4 s1 = make_float4(act_fwd<ACT>(acc[4]), act_fwd<ACT>(acc[5]),
                                  act_fwd<ACT>(acc[6]), act_fwd<ACT>(acc[7]));
    *(RY*)(Y + (int64_t)row * ldy + c0 + 4) = Vec4<TY>::put(s1);
  }
}

template <typename TY>
static int spmm_sliced64_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                              int32_t n_rows, int32_t D, const bf16_t* Xs, int64_t sstride, TY* Y,
                              int64_t ldy, int act, hipStream_t s) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !Xs || !Y) return GNNEA_EINVAL;
  if (D % 4 || ldy % 4 || ldy < D || sstride % 64 || sstride < 64) return GNNEA_EINVAL;
  if ((((uintptr_t)Xs) & 15) || !aln<TY>(Y)) return GNNEA_EALIGN;
  const int nbs = (n_rows + 3) / 4;
  const int S = (D + 63) / 64;
  if ((int64_t)nbs * S >= (1ll << 31)) return GNNEA_EINVAL;
  const int64_t ss16 = sstride / 8;  // 16-B units
#define GNNEA_S64(A)                                                                           \
  hipLaunchKernelGGL((k_spmm_sliced64_bf16<A, kS64U, TY>), dim3(nbs * S), dim3(256), 0, s, rowptr, \
                     col, val, n_rows, nbs, D, (const uint4*)Xs, ss16, Y, ldy)
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_S64(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_S64(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_S64(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_S64(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_S64(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_S64(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_S64
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_spmm_sliced_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                                     int32_t n_rows, int32_t D, const float* Xs, int64_t sstride,
                                     float* Y, int64_t ldy, int act, void* stream) {
  return spmm_sliced<false, float, float>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy, act,
                                          kNoHighway, (hipStream_t)stream);
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
  return spmm_sliced<true, float, float>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy, act,
                                         hw, (hipStream_t)stream);
}

// the fused HighWay layer's forward with the relu sign mask in place of S (SlicedHighway::save_m:
// [n_rows][ldm] bytes, ldm >= 16 * ceil(D / 64)); act must be relu
extern "C" int gnnea_spmm_highway_sliced_m_f32(const int32_t* rowptr, const int32_t* col,
                                               const float* val, int32_t n_rows, int32_t D,
                                               const float* Xs, int64_t sstride,
                                               const float* gate_s, int64_t gsstride,
                                               int32_t goff, const float* bias_gate,
                                               const float* resid, int64_t ldr, float* Y,
                                               int64_t ldy, uint8_t* save_m, int64_t ldm, int act,
                                               void* stream) {
  if (gsstride % 4 || act != GNNEA_ACT_RELU || !save_m || ldm < 16 * ((D + 63) / 64))
    return GNNEA_EINVAL;
  SlicedHighway hw{(const float4*)gate_s, gsstride / 4, goff, bias_gate, resid, ldr,
                   nullptr, nullptr, 0};
  hw.save_m = save_m;
  hw.ldm = ldm;
  return spmm_sliced<true, float, float>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy, act,
                                         hw, (hipStream_t)stream);
}

// gnnea_spmm_sliced_f32 with relu, also writing the output's sign bits (save_m [n_rows][ldm]
// bytes, ldm >= D / 4: byte q = the 4-element chunk q, bit e = element 4 q + e > 0)
extern "C" int gnnea_spmm_sliced_m_f32(const int32_t* rowptr, const int32_t* col,
                                       const float* val, int32_t n_rows, int32_t D,
                                       const float* Xs, int64_t sstride, float* Y, int64_t ldy,
                                       uint8_t* save_m, int64_t ldm, void* stream) {
  if (!save_m || ldm < (D + 3) / 4) return GNNEA_EINVAL;
  SlicedHighway hw = kNoHighway;
  hw.save_m = save_m;
  hw.ldm = ldm;
  return spmm_sliced<false, float, float>(rowptr, col, val, n_rows, D, Xs, sstride, Y, ldy,
                                          GNNEA_ACT_RELU, hw, (hipStream_t)stream);
}

// gnnea_act_bwd_sliced_f32 (relu) with relu'(Y) from gnnea_spmm_sliced_m_f32's sign bits
extern "C" int gnnea_act_bwd_sliced_bits_f32(const float* dY, int64_t lddy, const uint8_t* M,
                                             int64_t ldm, int64_t n, int32_t D, float* Gs,
                                             int64_t sstride, void* stream) {
  if (n < 0 || D < 0) return GNNEA_EINVAL;
  if (n == 0 || D == 0) return 0;
  if (!dY || !M || !Gs || D % 4 || lddy % 4 || lddy < D || ldm < D / 4 || sstride % 4 ||
      sstride < n * kSliceW || !al16(dY) || !al16(Gs) || (n + 3) / 4 >= (1ll << 31))
    return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_slice_fill_bits, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, (const float4*)dY, lddy / 4, M, ldm, n, D / 4,
                     (float4*)Gs, sstride / 4);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_slice_pack_f32(const float* X, int64_t ldx, int64_t n, int32_t D,
                                    float* Xs, int64_t sstride, void* stream) {
  return slice_fill<false, float>(X, ldx, nullptr, 0, n, D, Xs, sstride, GNNEA_ACT_IDENTITY,
                                  (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_sliced_f32(const float* dY, int64_t lddy, const float* Y,
                                        int64_t ldy, int64_t n, int32_t D, int act, float* Gs,
                                        int64_t sstride, void* stream) {
  return slice_fill<true, float>(dY, lddy, Y, ldy, n, D, Gs, sstride, act, (hipStream_t)stream);
}

// ---- bf16 storage (cfg-5): 128-column slices, fp32 arithmetic, outputs rounded once ----------

extern "C" int gnnea_spmm_sliced_bf16(const int32_t* rowptr, const int32_t* col,
                                      const float* val, int32_t n_rows, int32_t D,
                                      const void* Xs, int64_t sstride, void* Y, int64_t ldy,
                                      int y_dtype, int act, void* stream) {
  if (y_dtype == GNNEA_BF16)
    return spmm_sliced<false, bf16_t, bf16_t>(rowptr, col, val, n_rows, D, (const bf16_t*)Xs,
                                              sstride, (bf16_t*)Y, ldy, act, kNoHighway,
                                              (hipStream_t)stream);
  if (y_dtype == GNNEA_F32)
    return spmm_sliced<false, bf16_t, float>(rowptr, col, val, n_rows, D, (const bf16_t*)Xs,
                                             sstride, (float*)Y, ldy, act, kNoHighway,
                                             (hipStream_t)stream);
  return GNNEA_EINVAL;
}

extern "C" int gnnea_slice_pack_bf16(const void* X, int64_t ldx, int64_t n, int32_t D, void* Xs,
                                     int64_t sstride, void* stream) {
  return slice_fill<false, bf16_t>((const bf16_t*)X, ldx, nullptr, 0, n, D, (bf16_t*)Xs,
                                   sstride, GNNEA_ACT_IDENTITY, (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_sliced_bf16(const void* dY, int64_t lddy, const void* Y,
                                         int64_t ldy, int64_t n, int32_t D, int act, void* Gs,
                                         int64_t sstride, void* stream) {
  return slice_fill<true, bf16_t>((const bf16_t*)dY, lddy, (const bf16_t*)Y, ldy, n, D,
                                  (bf16_t*)Gs, sstride, act, (hipStream_t)stream);
}

// bf16 over 64-column slices (128 B per row piece; the layout of gnnea_slice_pack64_bf16):
// element (r, c) at Xs[(c/64)*sstride + r*64 + c%64], sstride % 64 == 0, 8-B aligned Xs
extern "C" int gnnea_spmm_sliced64_bf16(const int32_t* rowptr, const int32_t* col,
                                        const float* val, int32_t n_rows, int32_t D,
                                        const void* Xs, int64_t sstride, void* Y, int64_t ldy,
                                        int y_dtype, int act, void* stream) {
  if (y_dtype == GNNEA_BF16)
    return spmm_sliced64_bf16<bf16_t>(rowptr, col, val, n_rows, D, (const bf16_t*)Xs, sstride,
                                      (bf16_t*)Y, ldy, act, (hipStream_t)stream);
  if (y_dtype == GNNEA_F32)
    return spmm_sliced64_bf16<float>(rowptr, col, val, n_rows, D, (const bf16_t*)Xs, sstride,
                                     (float*)Y, ldy, act, (hipStream_t)stream);
  return GNNEA_EINVAL;
}
