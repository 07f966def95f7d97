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

#include <stdlib.h>

namespace gnnea {

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
    for (int h = 0; h < H; ++h) mx[h] = fmaxf(mx[h], -lrelu(si[h] + s2[(int64_t)j * H + h], alpha));
  }
#pragma unroll
  for (int h = 0; h < H; ++h) mx[h] = wave_max(mx[h]);
  for (int e = beg + lane; e < end; e += 64) {
    const int j = col[e];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float w = __expf(-lrelu(si[h] + s2[(int64_t)j * H + h], alpha) - mx[h]);
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

// every 64-column slice must hold at most two heads (the kernels keep h0 / h1 per slice and two
// product partials per edge): d_head >= 64, or d_head in [32, 63] with no slice straddling three
// heads (d_head 40: slice 1 = columns 64..127 = heads 1, 2, 3 -> refused)
static bool gat_two_heads_per_slice(int heads, int d_head) {
  if (heads < 1 || d_head < 32) return false;
  const int D = heads * d_head;
  for (int s = 0; 64 * s < D; ++s) {
    const int h0 = (64 * s) / d_head, h1 = min((64 * s + 63) / d_head, heads - 1);
    if (h1 - h0 > 1) return false;
  }
  return true;
}

// Lane map of the gather passes over a 64-column slice: every lane owns E = 4 columns of the
// row piece (one 16-B fp32 / 8-B bf16 load per neighbour), LPG = 16 lanes per piece, NG = 4
// groups per wave each on its own neighbour.  (bf16 with 16-B lanes -- 8 columns, 8 groups of 8
// -- measured slower at cfg-5: 11.6 vs 8.7 ms for the source pass per KG, 6.5 vs 6.4 forward.)
template <typename T>
struct GatLanes {
  static constexpr int E = 4;
  static constexpr int LPG = 64 / E;
  static constexpr int NG = 64 / LPG;
  typedef typename Vec4<T>::raw R;  // one lane's load
};

// E consecutive columns from c0 of a row-major row (4-column chunks; columns >= D read as 0)
template <typename T, int E>
__device__ __forceinline__ void load_cols(const T* row, int c0, int D, float (&v)[E]) {
  typedef typename Vec4<T>::raw R;
#pragma unroll
  for (int k = 0; k < E / 4; ++k) {
    float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c0 + 4 * k < D) f = Vec4<T>::get(*(const R*)(row + c0 + 4 * k));
    v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
  }
}
template <typename T, int E>
__device__ __forceinline__ void store_cols(T* row, int c0, int D, const float (&v)[E]) {
  typedef typename Vec4<T>::raw R;
#pragma unroll
  for (int k = 0; k < E / 4; ++k)
    if (c0 + 4 * k < D)
      *(R*)(row + c0 + 4 * k) =
          Vec4<T>::put(make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]));
}

// one lane's piece of a gathered slice row through a buffer resource on the slice base (wave-
// uniform, scalar): the 32-bit offset row * (64 sizeof(T)) + lane piece is one vector multiply-
// add, where a 64-bit per-lane address took three; host-checked: a slice spans < 4 GB
template <typename R>
__device__ __forceinline__ R load_piece(const __amdgpu_buffer_rsrc_t& rs, uint32_t off) {
  if constexpr (sizeof(R) == 16) {
    return __builtin_bit_cast(R, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  } else {
    static_assert(sizeof(R) == 8, "piece size");
    return __builtin_bit_cast(R, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
  }
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t slice_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0xffffffffu, 0x00020000);
}

template <int ACT, int U, typename TX, typename TY>
__global__ __launch_bounds__(256) void k_gat_fwd_sliced(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, int n_rows, int nbs,
    int H, int D, int dh, const typename GatLanes<TX>::R* __restrict__ Hs, int64_t sstrideR,
    const float* __restrict__ wgt, const float* __restrict__ den_in, TY* __restrict__ Y,
    int64_t ldy, int s0) {
  constexpr int E = GatLanes<TX>::E, LPG = GatLanes<TX>::LPG, NG = GatLanes<TX>::NG;
  typedef typename GatLanes<TX>::R RX;
  const int b = blockIdx.x;
  const int sb = b / nbs;
  const int s = s0 + sb;  // slices [s0, s0 + gridDim.x / nbs) of this launch
  const int row = xcd_remap(b - sb * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane / LPG, c = lane % LPG;
  const int c0 = s * 64 + E * c;
  const bool own = c0 < D;
  // the slice's heads (at most two per 64 columns, gat_two_heads_per_slice) and this lane's
  // columns' heads
  const int h0 = min((s * 64) / dh, H - 1);
  const int h1 = min((s * 64 + 63) / dh, H - 1);
  bool second[E];
#pragma unroll
  for (int t = 0; t < E; ++t) second[t] = (c0 + t) / dh != h0;
  // every lane loads unconditionally: edges past the chunk take row 0 with weight 0, lanes past D
  // re-read the row's first piece (finite; never stored)
  const __amdgpu_buffer_rsrc_t xs = slice_rsrc(Hs + (int64_t)s * sstrideR);
  const uint32_t loff = (uint32_t)(own ? c : 0) * (uint32_t)sizeof(RX);
  const int beg = rowptr[row], end = rowptr[row + 1];
  float acc[E];
#pragma unroll
  for (int t = 0; t < E; ++t) acc[t] = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mj = 0;
    float w0 = 0.f, w1 = 0.f;
    if (lane < cnt) {  // edge base + lane: its (masked) weights for the slice's two heads
      mj = col[base + lane];
      w0 = wgt[(int64_t)(base + lane) * H + h0];
      w1 = wgt[(int64_t)(base + lane) * H + h1];
    }
    for (int k = 0; k < cnt; k += NG * U) {
      RX r[U];
      float v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + NG * u + g;  // <= 63: k is a multiple of NG*U that divides 64
        const int j = __shfl(mj, e & 63, 64);
        v0[u] = __shfl(w0, e & 63, 64);
        v1[u] = __shfl(w1, e & 63, 64);
        r[u] = load_piece<RX>(xs, (uint32_t)j * (uint32_t)(LPG * sizeof(RX)) + loff);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float4 fv = Vec4<TX>::get(r[u]);
        float f[E] = {fv.x, fv.y, fv.z, fv.w};
#pragma unroll
        for (int t = 0; t < E; ++t) acc[t] = fmaf(second[t] ? v1[u] : v0[u], f[t], acc[t]);
      }
    }
  }
  // the group partials in fixed order (xor LPG, 2 LPG, ...)
#pragma unroll
  for (int o = LPG; o < 64; o <<= 1) {
#pragma unroll
    for (int t = 0; t < E; ++t) acc[t] += __shfl_xor(acc[t], o, 64);
  }
  if (g != 0 || !own) return;
  const float d0 = den_in[(int64_t)row * H + h0], d1 = den_in[(int64_t)row * H + h1];
  const float r0 = d0 > 0.f ? 1.f / d0 : 0.f, r1 = d1 > 0.f ? 1.f / d1 : 0.f;
  float o[E];
#pragma unroll
  for (int t = 0; t < E; ++t) o[t] = act_fwd<ACT>(acc[t] * (second[t] ? r1 : r0));
  store_cols<TY, E>(Y + (int64_t)row * ldy, c0, D, o);
}

// Row-major [n, D] -> 64-column slice-major table [ceil(D/64)][n][64] (the GAT layout for both
// storage types: 256 B per fp32 slice row, 128 B = one line per bf16 slice row, so one bf16 KG
// slice of a 2M-row cfg-5 KG is 256 MB), one wave per row.
template <typename T>
__global__ __launch_bounds__(256) void k_pack64(const typename Vec4<T>::raw* __restrict__ X,
                                                int64_t ld4, int64_t n, int D4,
                                                typename Vec4<T>::raw* __restrict__ Xs,
                                                int64_t sstride4) {
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();
  if (r >= n) return;
  for (int q = lane_id(); q < D4; q += 64)
    Xs[(int64_t)(q >> 4) * sstride4 + r * 16 + (q & 15)] = X[r * ld4 + q];
}

// ---------------------------------------------------------------------------------------- //
// Backward over the slice-major G (the k_gat_bwd_prep / _src / _dst scheme of gat.hip, with the
// source-side gather cut into 64-column slices as the forward above).  k_gat_bwd_src gathers
// each in-neighbour's whole 1,200-B G row from a 1.2-GB KG table; here:
//   k_gat_bwd_prep_s (dest rows i): G = dY * act'(Y) written slice-major, records {s1, m, 1/den,
//                     c = G_i . h'_i} as gat.hip;
//   k_gat_bwd_w      (source rows j, 32 lanes per row): wT[e][h] = alpha_ij * mask_ij in A^T
//                     order (one record gather per edge, once);
//   k_gat_bwd_src_sl (slice, source row j) as k_gat_fwd_sliced: dH_j[slice] = sum_i w_ij G_i,
//                     and per edge the slice's share of the per-head products G_i,h . H_j,h for
//                     the (at most two) heads the slice holds — reduced over each 16-lane group
//                     by reduce-scatter (grp_sum) and stored as pd[s][e][2];
//   k_gat_bwd_edge   (source rows j, 32 lanes per row): da_ij,h = the head's slice partials
//                     summed in slice order, dz_ij = -LeakyReLU'(z) alpha (mask da - c_i) in A^T
//                     order (coalesced; storing it at A positions instead measured 1.69 -> 3.65
//                     ms per cfg-4 launch against 2.77 -> 2.28 for the destination pass),
//                     ds2_j = sum_i dz; optionally dH_j += ds2_j (x) a2;
//   k_gat_bwd_dst_s  (dest rows i, 32 lanes per row): its dH row loaded first (in flight under
//                     the dz gathers),
//                     ds1_i through the transpose position map, dH_i += ds1_i (x) a1
//                     (+ ds2_i (x) a2 when the edge pass left it, square unsharded case).
// fp32 arithmetic; G, H and dH in the storage type T (fp32, or bf16 for cfg-5: 64-column slices of
// 128 B, every stored value rounded once per pass); sums in a different order from gat.hip's
// single pass (fp32 rounding level).
// ---------------------------------------------------------------------------------------- //

template <int ACT, int H, int NCH, typename T>
__global__ __launch_bounds__(256) void k_gat_bwd_prep_s(int n_rows, int D, int dh,
                                                        const typename Vec4<T>::raw* __restrict__ dY,
                                                        const typename Vec4<T>::raw* __restrict__ Y,
                                                        int64_t ld4, const float* __restrict__ s1,
                                                        const float* __restrict__ mrow,
                                                        const float* __restrict__ den,
                                                        typename Vec4<T>::raw* __restrict__ Gs,
                                                        int64_t sstride4,
                                                        float4* __restrict__ rec) {
  const int row = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  // the per-head sums reduce-scattered over the wave (grp_sum, as k_gat_bwd_prep4): the lane that
  // ends with head hw's sum writes its record; the record's row statistics, read up front (read in
  // the epilogue they were one more serial round trip per row after the sums)
  constexpr int HP = H <= 1 ? 1 : H <= 2 ? 2 : H <= 4 ? 4 : 8;
  const int hw = lane % (16 / HP) == 0 && lane < 16 ? lane / (16 / HP) : 0;
  const int64_t ro = (int64_t)row * H + (hw < H ? hw : 0);
  const float rs1 = s1[ro], rmx = mrow[ro], rdv = den[ro];
  float cp[HP];
#pragma unroll
  for (int h = 0; h < HP; ++h) cp[h] = 0.f;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    if (4 * c4 >= D) continue;
    const float4 dy = Vec4<T>::get(dY[(int64_t)row * ld4 + c4]);
    const float4 y = Vec4<T>::get(Y[(int64_t)row * ld4 + c4]);
    const float ys[4] = {y.x, y.y, y.z, y.w};
    float gs[4] = {dy.x, dy.y, dy.z, dy.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      gs[t] = c < D ? gs[t] * act_grad_from_out<ACT>(ys[t]) : 0.f;
    }
    // the record's G.h' uses the G the source pass gathers (rounded to T once)
    const typename Vec4<T>::raw gr = Vec4<T>::put(make_float4(gs[0], gs[1], gs[2], gs[3]));
    const float4 gq = Vec4<T>::get(gr);
    const float gv[4] = {gq.x, gq.y, gq.z, gq.w};
    if (dh >= 4) {  // (uniform) four elements span at most two heads: hq and the next
      const int hq = (4 * c4) / dh, es = (hq + 1) * dh - 4 * c4;
      float pa = 0.f, pb = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float v = 4 * c4 + t < D ? gv[t] * ys[t] : 0.f;
        pa += t < es ? v : 0.f;
        pb += t < es ? 0.f : v;
      }
#pragma unroll
      for (int h = 0; h < HP; ++h) cp[h] += (h == hq ? pa : 0.f) + (h == hq + 1 ? pb : 0.f);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = 4 * c4 + t;
        const int hh = c < D ? c / dh : HP;
#pragma unroll
        for (int h = 0; h < HP; ++h) cp[h] += (hh == h) ? gv[t] * ys[t] : 0.f;
      }
    }
    // column 4*c4 -> slice c4 / 16, offset 4 * (c4 % 16)
    Gs[(int64_t)(c4 >> 4) * sstride4 + (int64_t)row * 16 + (c4 & 15)] = gr;
  }
  const float cs = grp_sum<HP, 64>(cp, lane);
  if (lane % (16 / HP) == 0 && lane < 16 && hw < H)
    rec[(int64_t)row * H + hw] = make_float4(rs1, rmx, rdv > 0.f ? 1.f / rdv : 0.f, cs);
}

template <int H, int LPR>  // LPR lanes per source row
__global__ __launch_bounds__(256) void k_gat_bwd_w(const int32_t* __restrict__ rowptrT,
                                                   const int32_t* __restrict__ colT,
                                                   const int64_t* __restrict__ permT, int n_rows,
                                                   const float* __restrict__ s2, float alpha,
                                                   const float* __restrict__ emask,
                                                   const float4* __restrict__ rec,
                                                   float* __restrict__ wT) {
  const int row = xcd_remap(blockIdx.x, gridDim.x) * (256 / LPR) + threadIdx.x / LPR;
  if (row >= n_rows) return;
  const int l = threadIdx.x % LPR;
  float sj[H];
#pragma unroll
  for (int h = 0; h < H; ++h) sj[h] = s2[(int64_t)row * H + h];
  const int end = rowptrT[row + 1];
  for (int e = rowptrT[row] + l; e < end; e += LPR) {
    const int i = colT[e];
    const int64_t pe = emask ? permT[e] : 0;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float4 r = rec[(int64_t)i * H + h];  // {s1_i, m_i, 1/den_i, c_i}
      const float al = __expf(-lrelu(r.x + sj[h], alpha) - r.y) * r.z;
      wT[(int64_t)e * H + h] = emask ? al * emask[pe * H + h] : al;
    }
  }
}

template <int U, typename T>
__global__ __launch_bounds__(256) void k_gat_bwd_src_sl(
    const int32_t* __restrict__ rowptrT, const int32_t* __restrict__ colT, int n_rows, int nbs,
    int H, int D, int dh, const typename GatLanes<T>::R* __restrict__ Gs, int64_t sstrideR,
    const T* __restrict__ Hm, int64_t ldh, int64_t hss, const float* __restrict__ wT,
    T* __restrict__ dH, int64_t lddh, int64_t dhss, float* __restrict__ pd, int64_t pstride,
    int s0) {
  constexpr int E = GatLanes<T>::E, LPG = GatLanes<T>::LPG, NG = GatLanes<T>::NG;
  typedef typename GatLanes<T>::R RX;
  const int b = blockIdx.x;
  const int sb = b / nbs;
  const int s = s0 + sb;  // slices [s0, s0 + gridDim.x / nbs) of this launch
  const int row = xcd_remap(b - sb * nbs, nbs) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id(), g = lane / LPG, c = lane % LPG;
  const int c0 = s * 64 + E * c;
  const bool own = c0 < D;
  const int h0 = min((s * 64) / dh, H - 1);
  const int h1 = min((s * 64 + 63) / dh, H - 1);
  const bool two = h1 != h0;  // uniform per slice
  bool second[E];
  float hj0[E], hj1[E];  // H_j split by head; zero past D (the table's padding is never read)
  {
    float v[E];
    // H_j's columns of slice s: Hm + s * hss + row * ldh + (c - 64 s) (row-major: hss = 64;
    // a slice-major table: ldh = 64, hss = its slice stride)
    load_cols<T, E>(Hm + (int64_t)s * (hss - 64) + (int64_t)row * ldh, c0, D, v);
#pragma unroll
    for (int t = 0; t < E; ++t) {
      second[t] = (c0 + t) / dh != h0;
      const float vt = c0 + t < D ? v[t] : 0.f;
      hj0[t] = second[t] ? 0.f : vt;
      hj1[t] = second[t] ? vt : 0.f;
    }
  }
  // unconditional loads as k_gat_fwd_sliced: edges past the chunk take row 0 with weight 0 (their
  // products are never stored), lanes past D re-read the row's first piece (finite; hj = 0 there,
  // acc never stored); columns in [D, 4 ceil(D/4)) hold zeros (k_gat_bwd_prep_s writes them)
  const __amdgpu_buffer_rsrc_t xs = slice_rsrc(Gs + (int64_t)s * sstrideR);
  const uint32_t loff = (uint32_t)(own ? c : 0) * (uint32_t)sizeof(RX);
  float* pds = pd + (int64_t)s * pstride;
  const int beg = rowptrT[row], end = rowptrT[row + 1];
  float acc[E];
#pragma unroll
  for (int t = 0; t < E; ++t) acc[t] = 0.f;
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mj = 0;
    float w0 = 0.f, w1 = 0.f;
    if (lane < cnt) {
      mj = colT[base + lane];
      w0 = wT[(int64_t)(base + lane) * H + h0];
      w1 = wT[(int64_t)(base + lane) * H + h1];
    }
    for (int k = 0; k < cnt; k += NG * U) {
      RX r[U];
      float v0[U], v1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + NG * u + g;
        const int j = __shfl(mj, e & 63, 64);
        v0[u] = __shfl(w0, e & 63, 64);
        v1[u] = __shfl(w1, e & 63, 64);
        r[u] = load_piece<RX>(xs, (uint32_t)j * (uint32_t)(LPG * sizeof(RX)) + loff);
      }
      float q[2 * U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float4 fv = Vec4<T>::get(r[u]);
        const float f[E] = {fv.x, fv.y, fv.z, fv.w};
        float qa = 0.f, qb = 0.f;
#pragma unroll
        for (int t = 0; t < E; ++t) {
          acc[t] = fmaf(second[t] ? v1[u] : v0[u], f[t], acc[t]);
          qa = fmaf(f[t], hj0[t], qa);
          qb = fmaf(f[t], hj1[t], qb);
        }
        q[u] = qa;
        q[U + u] = qb;
      }
      // per-group sums of the LPG lanes: value v (edge u = v % U, head slot v / U) lands on
      // lane grp_lane(v) of the group; that lane stores it
      if (two) {
        const float sum = grp_sum<2 * U, LPG>(q, lane);
        constexpr int SP = (LPG >= 16 ? 16 : 8) / (2 * U);
        const int v = c / SP, e = k + NG * (v % U) + g;
        if (c % SP == 0 && e < cnt) pds[(int64_t)(base + e) * 2 + v / U] = sum;
      } else {
        float qq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) qq[u] = q[u];
        const float sum = grp_sum<U, LPG>(qq, lane);
        constexpr int SP = (LPG >= 16 ? 16 : 8) / U;
        const int e = k + NG * (c / SP) + g;
        if (c % SP == 0 && e < cnt) pds[(int64_t)(base + e) * 2] = sum;
      }
    }
  }
#pragma unroll
  for (int o = LPG; o < 64; o <<= 1) {
#pragma unroll
    for (int t = 0; t < E; ++t) acc[t] += __shfl_xor(acc[t], o, 64);
  }
  if (g != 0 || !own) return;
  store_cols<T, E>(dH + (int64_t)s * (dhss - 64) + (int64_t)row * lddh, c0, D, acc);
}

template <int H, int LPR, typename T>  // LPR lanes per source row
__global__ __launch_bounds__(256) void k_gat_bwd_edge(
    const int32_t* __restrict__ rowptrT, const int32_t* __restrict__ colT,
    const int64_t* __restrict__ permT, int n_rows, int S, int D, int dh,
    const float* __restrict__ s2, float alpha, const float* __restrict__ emask,
    const float4* __restrict__ rec, const float2* __restrict__ pd, int64_t pstride2,
    const float* __restrict__ a, T* __restrict__ dH, int64_t lddh, float* __restrict__ dzT,
    float* __restrict__ ds2) {
  const int row = xcd_remap(blockIdx.x, gridDim.x) * (256 / LPR) + threadIdx.x / LPR;
  if (row >= n_rows) return;  // whole LPR-lane groups leave together
  const int l = threadIdx.x % LPR;
  float sj[H], d2[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    sj[h] = s2[(int64_t)row * H + h];
    d2[h] = 0.f;
  }
  const int end = rowptrT[row + 1];
  for (int e = rowptrT[row] + l; e < end; e += LPR) {
    const int i = colT[e];
    const int64_t pe = emask ? permT[e] : 0;
    float da[H];
#pragma unroll
    for (int h = 0; h < H; ++h) da[h] = 0.f;
    for (int s = 0; s < S; ++s) {  // the head's slice partials in slice order
      const float2 p = pd[(int64_t)s * pstride2 + e];
      const int h0 = min((s * 64) / dh, H - 1), h1 = min((s * 64 + 63) / dh, H - 1);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        if (h == h0) da[h] += p.x;
        else if (h == h1) da[h] += p.y;
      }
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float4 r = rec[(int64_t)i * H + h];
      const float z = r.x + sj[h];
      const float al = __expf(-lrelu(z, alpha) - r.y) * r.z;
      const float ml = emask ? emask[pe * H + h] : 1.f;
      const float dz = -(al * (ml * da[h] - r.w)) * (z > 0.f ? 1.f : alpha);
      dzT[(int64_t)e * H + h] = dz;
      d2[h] += dz;
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) d2[h] += __shfl_xor(d2[h], o, LPR);
  }
  if (l < H) ds2[(int64_t)row * H + l] = hsel<H>(d2, l);
  if (!dH) return;
  typedef typename Vec4<T>::raw RX;
  T* out = dH + (int64_t)row * lddh;
  for (int c4 = l; 4 * c4 < D; c4 += LPR) {
    const float4 v = Vec4<T>::get(*(RX*)(out + 4 * c4));
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cc = 4 * c4 + t, h = cc / dh;
      o[t] += hsel<H>(d2, h) * a[h * 2 * dh + dh + (cc - h * dh)];
    }
    *(RX*)(out + 4 * c4) = Vec4<T>::put(make_float4(o[0], o[1], o[2], o[3]));
  }
}

template <int H, int NCH, int L, typename T>  // L lanes per destination row (NCH: 4-element slots at 64 lanes)
__global__ __launch_bounds__(256) void k_gat_bwd_dst_s(const int32_t* __restrict__ rowptr,
                                                       const int64_t* __restrict__ tpos,
                                                       int n_rows, int D, int dh,
                                                       const float* __restrict__ dzT,
                                                       const float* __restrict__ a,
                                                       const float* __restrict__ ds2,
                                                       typename Vec4<T>::raw* __restrict__ dH,
                                                       int64_t lddh4, float* __restrict__ ds1) {
  constexpr int NC = NCH * 64 / L;
  const int row = xcd_remap(blockIdx.x, gridDim.x) * (256 / L) + threadIdx.x / L;
  if (row >= n_rows) return;  // whole L-lane groups leave together
  const int l = threadIdx.x % L;
  const int beg = rowptr[row], end = rowptr[row + 1];
  float4 v[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {  // independent of dz: issued before the gather chain
    const int c4 = l + L * k;
    v[k] = 4 * c4 < D ? Vec4<T>::get(dH[(int64_t)row * lddh4 + c4]) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // the lane's columns' heads and a1 / a2 values, likewise before the chain (read after it they
  // were one more dependent round trip per row, with an integer division per element)
  int hc[NC][4];
  float a1v[NC][4], a2v[NC][4];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = min(4 * (l + L * k) + t, D - 1), h = c / dh, d = c - h * dh;
      hc[k][t] = h;
      a1v[k][t] = a[h * 2 * dh + d];
      a2v[k][t] = ds2 ? a[h * 2 * dh + dh + d] : 0.f;
    }
  }
  float p[H], q[H];
#pragma unroll
  for (int h = 0; h < H; ++h) p[h] = 0.f;
  for (int e = beg + l; e < end; e += L) {
    const int64_t t = tpos[e];
#pragma unroll
    for (int h = 0; h < H; ++h) p[h] += dzT[t * H + h];
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) p[h] += __shfl_xor(p[h], o, L);
    q[h] = ds2 ? ds2[(int64_t)row * H + h] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c4 = l + L * k;
    if (4 * c4 >= D) continue;
    float o[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int h = hc[k][t];
      o[t] += hsel<H>(p, h) * a1v[k][t];
      if (ds2) o[t] += hsel<H>(q, h) * a2v[k][t];
    }
    dH[(int64_t)row * lddh4 + c4] = Vec4<T>::put(make_float4(o[0], o[1], o[2], o[3]));
  }
  if (l < H) ds1[(int64_t)row * H + l] = hsel<H>(p, l);
}

}  // namespace gnnea


using namespace gnnea;

namespace {

template <typename T>
bool alv(const void* p) {  // aligned for one Vec4<T> (nullptr passes)
  return (((uintptr_t)p) & (sizeof(typename Vec4<T>::raw) - 1)) == 0;
}

// neighbours in flight per 16-lane group: 4 x 16 B (fp32) / 8 x 8 B (bf16) per lane
template <typename T>
constexpr int kGatU = sizeof(T) == 4 ? 4 : 8;

template <typename T>
int gat_fwd_sliced(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const T* Hs,
                   int64_t sstride, int heads, int d_head, const float* s1, const float* s2,
                   float alpha, const float* edge_mask, int act, T* Y, int64_t ldy, float* m_out,
                   float* den_out, float* wgt, hipStream_t st, int s_begin = 0, int s_end = -1,
                   bool stats = true) {
  const int D = heads * d_head;
  if (n_rows < 0 || heads < 1 || heads > 8 || !gat_two_heads_per_slice(heads, d_head) ||
      D % 4 || sstride % 64 || ldy % 4 || ldy < D)
    return GNNEA_EINVAL;
  if (act != GNNEA_ACT_IDENTITY && act != GNNEA_ACT_RELU) return GNNEA_EINVAL;
  const int S = div_up(D, 64);
  if (s_end < 0) s_end = S;
  if (s_begin < 0 || s_begin > s_end || s_end > S) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!rowptr || !col || !s1 || !s2 || !m_out || !den_out || !wgt) return GNNEA_EINVAL;
  if (s_end > s_begin && (!Hs || !Y)) return GNNEA_EINVAL;
  if (!alv<T>(Hs) || !alv<T>(Y)) return GNNEA_EALIGN;
  if ((uint64_t)sstride * sizeof(T) > 0xffffffffull) return GNNEA_EINVAL;  // (load_piece)
  const int nbs = div_up(n_rows, 4);
  if (stats) switch (heads) {
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
  if (s_end == s_begin) return 0;
  const dim3 grid((unsigned)((int64_t)(s_end - s_begin) * nbs));
  typedef typename GatLanes<T>::R R;
  if (act == GNNEA_ACT_RELU)
    hipLaunchKernelGGL((k_gat_fwd_sliced<GNNEA_ACT_RELU, kGatU<T>, T, T>), grid, dim3(256), 0, st,
                       rowptr, col, n_rows, nbs, heads, D, d_head, (const R*)Hs, sstride / 4,
                       wgt, den_out, Y, ldy, s_begin);
  else
    hipLaunchKernelGGL((k_gat_fwd_sliced<GNNEA_ACT_IDENTITY, kGatU<T>, T, T>), grid, dim3(256), 0,
                       st, rowptr, col, n_rows, nbs, heads, D, d_head, (const R*)Hs, sstride / 4,
                       wgt, den_out, Y, ldy, s_begin);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int pack64(const T* X, int64_t ldx, int64_t n, int32_t D, T* Xs, int64_t sstride,
           hipStream_t st) {
  if (n < 0 || D < 0) return GNNEA_EINVAL;
  if (n == 0 || D == 0) return 0;
  if (!X || !Xs || D % 4 || ldx % 4 || ldx < D || sstride % 64 || sstride < n * 64)
    return GNNEA_EINVAL;
  if (!alv<T>(X) || !alv<T>(Xs)) return GNNEA_EALIGN;
  if ((n + 3) / 4 >= (1ll << 31)) return GNNEA_EINVAL;
  typedef typename Vec4<T>::raw R;
  hipLaunchKernelGGL((k_pack64<T>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st,
                     (const R*)X, ldx / 4, n, D / 4, (R*)Xs, sstride / 4);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// the sliced forward: rowstats (m_out, den_out, per-edge weights in wgt: nnz x heads fp32,
// indexed by the absolute CSR position) + the aggregation; Hs slice-major 64-column table
// [ceil(D/64)][n_src][64] (sstride elements per slice), D % 4 == 0, every slice at most two heads
// (gat_two_heads_per_slice), ldy % 4 == 0
extern "C" int gnnea_gat_fwd_sliced_f32(const int32_t* rowptr, const int32_t* col,
                                        int32_t n_rows, const float* Hs, int64_t sstride,
                                        int heads, int d_head, const float* s1, const float* s2,
                                        float alpha, const float* edge_mask, int act, float* Y,
                                        int64_t ldy, float* m_out, float* den_out, float* wgt,
                                        void* stream) {
  return gat_fwd_sliced<float>(rowptr, col, n_rows, Hs, sstride, heads, d_head, s1, s2, alpha,
                               edge_mask, act, Y, ldy, m_out, den_out, wgt, (hipStream_t)stream);
}

extern "C" int gnnea_gat_fwd_sliced_bf16(const int32_t* rowptr, const int32_t* col,
                                         int32_t n_rows, const void* Hs, int64_t sstride,
                                         int heads, int d_head, const float* s1, const float* s2,
                                         float alpha, const float* edge_mask, int act, void* Y,
                                         int64_t ldy, float* m_out, float* den_out, float* wgt,
                                         void* stream) {
  return gat_fwd_sliced<bf16_t>(rowptr, col, n_rows, (const bf16_t*)Hs, sstride, heads, d_head,
                                s1, s2, alpha, edge_mask, act, (bf16_t*)Y, ldy, m_out, den_out,
                                wgt, (hipStream_t)stream);
}

// row-major [n, D] -> the 64-column slice-major GAT table (sstride elements per slice)
extern "C" int gnnea_slice_pack64_f32(const float* X, int64_t ldx, int64_t n, int32_t D,
                                      float* Xs, int64_t sstride, void* stream) {
  return pack64<float>(X, ldx, n, D, Xs, sstride, (hipStream_t)stream);
}

extern "C" int gnnea_slice_pack64_bf16(const void* X, int64_t ldx, int64_t n, int32_t D,
                                       void* Xs, int64_t sstride, void* stream) {
  return pack64<bf16_t>((const bf16_t*)X, ldx, n, D, (bf16_t*)Xs, sstride, (hipStream_t)stream);
}

// ---- sliced backward entry points -------------------------------------------------------- //
#define GNNEA_HEADS_SWITCH(CASE) \
  switch (heads) { CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8) }

// lanes per source row of the weight and edge passes: 32 (cfg-4, mean in-degree 21: edge pass
// 1.70 / 1.45 / 2.02 ms and weights 0.68 / 0.60 / 0.84 ms at 16 / 32 / 8 lanes); lanes per row
// of the destination pass: 32 (two rows per wave; 2.37 vs 3.13 ms per cfg-4 layer at 64)

static bool gat_sl_shape(int heads, int d_head, int64_t sstride) {
  const int D = heads * d_head;
  return heads >= 1 && heads <= 8 && gat_two_heads_per_slice(heads, d_head) && D % 4 == 0 &&
         D <= 1024 && sstride % 64 == 0;
}

namespace {

template <typename T>
int gat_bwd_prep_sliced(int32_t n_rows, int heads, int d_head, const T* dY, const T* Y,
                        int64_t ldy, const float* s1, const float* m, const float* den, int act,
                        T* Gs, int64_t sstride, float* rec, hipStream_t st) {
  const int D = heads * d_head;
  if (n_rows < 0 || !gat_sl_shape(heads, d_head, sstride) || ldy % 4 || ldy < D)
    return GNNEA_EINVAL;
  if (act != GNNEA_ACT_IDENTITY && act != GNNEA_ACT_RELU) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!dY || !Y || !s1 || !m || !den || !Gs || !rec) return GNNEA_EINVAL;
  if (!alv<T>(dY) || !alv<T>(Y) || !alv<T>(Gs) || ((uintptr_t)rec & 15)) return GNNEA_EALIGN;
  const int nch = (D / 4 + 63) / 64;
  const dim3 grid(div_up(n_rows, 4));
  typedef typename Vec4<T>::raw R;
#define GNNEA_PREP(ACT, HH, NC)                                                              \
  hipLaunchKernelGGL((k_gat_bwd_prep_s<ACT, HH, NC, T>), grid, dim3(256), 0, st, n_rows, D,  \
                     d_head, (const R*)dY, (const R*)Y, ldy / 4, s1, m, den, (R*)Gs,         \
                     sstride / 4, (float4*)rec)
#define GNNEA_PREP_NC(ACT, HH)            \
  switch (nch) {                          \
    case 1: GNNEA_PREP(ACT, HH, 1); break; \
    case 2: GNNEA_PREP(ACT, HH, 2); break; \
    case 3: GNNEA_PREP(ACT, HH, 3); break; \
    default: GNNEA_PREP(ACT, HH, 4); break; \
  }
#define GNNEA_PREP_H(HH)                                                    \
  case HH:                                                                  \
    if (act == GNNEA_ACT_RELU) { GNNEA_PREP_NC(GNNEA_ACT_RELU, HH) }        \
    else { GNNEA_PREP_NC(GNNEA_ACT_IDENTITY, HH) }                         \
    break;
  GNNEA_HEADS_SWITCH(GNNEA_PREP_H)
#undef GNNEA_PREP_H
#undef GNNEA_PREP_NC
#undef GNNEA_PREP
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// a table operand of the source pass: row-major (ss = 64: row stride ld >= D) or slice-major
// (ld = 64, ss = the slice stride, at least n rows of 64)
static bool gat_tab_ok(int64_t ld, int64_t ss, int D, int64_t n) {
  if (ss == 64) return ld % 4 == 0 && ld >= D;
  return ld == 64 && ss % 64 == 0 && ss >= n * 64;
}

template <typename T>
int gat_bwd_src_sliced(const int32_t* rowptrT, const int32_t* colT, const int64_t* permT,
                       int32_t n_rows, int heads, int d_head, const T* Hm, int64_t ldh,
                       const float* s2, float alpha, const float* emask, const float* rec,
                       const T* Gs, int64_t sstride, float* wT, float* pd, int64_t nnzT, T* dH,
                       int64_t lddh, hipStream_t st, int64_t hss = 64, int64_t dhss = 64,
                       int s_begin = 0, int s_end = -1, bool weights = true) {
  const int D = heads * d_head;
  if (n_rows < 0 || !gat_sl_shape(heads, d_head, sstride) || !gat_tab_ok(ldh, hss, D, n_rows) ||
      !gat_tab_ok(lddh, dhss, D, n_rows) || nnzT < 0)
    return GNNEA_EINVAL;
  const int S = div_up(D, 64);
  if (s_end < 0) s_end = S;
  if (s_begin < 0 || s_begin > s_end || s_end > S) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!rowptrT || !colT || !s2 || !rec || !wT || !pd || (emask && !permT)) return GNNEA_EINVAL;
  if (s_end > s_begin && (!Hm || !Gs || !dH)) return GNNEA_EINVAL;
  if (!alv<T>(Hm) || !alv<T>(Gs) || !alv<T>(dH)) return GNNEA_EALIGN;
  if ((uint64_t)sstride * sizeof(T) > 0xffffffffull) return GNNEA_EINVAL;  // (load_piece)
  if (weights) {
#define GNNEA_W1(HH, LP)                                                                        \
  hipLaunchKernelGGL((k_gat_bwd_w<HH, LP>), dim3(div_up(n_rows, 256 / LP)), dim3(256), 0, st,   \
                     rowptrT, colT, permT, n_rows, s2, alpha, emask, (const float4*)rec, wT)
#define GNNEA_W(HH)                                              \
  case HH:                                                       \
    GNNEA_W1(HH, 32);                                            \
    break;
  GNNEA_HEADS_SWITCH(GNNEA_W)
#undef GNNEA_W
#undef GNNEA_W1
  GNNEA_LAUNCH_CHECK();
  }
  if (s_end == s_begin) return 0;
  const int nbs = div_up(n_rows, 4);
  hipLaunchKernelGGL((k_gat_bwd_src_sl<kGatU<T>, T>),
                     dim3((unsigned)((int64_t)(s_end - s_begin) * nbs)), dim3(256), 0, st, rowptrT,
                     colT, n_rows, nbs, heads, D, d_head, (const typename GatLanes<T>::R*)Gs,
                     sstride / 4, Hm, ldh, hss, wT, dH, lddh, dhss, pd, 2 * nnzT, s_begin);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int gat_bwd_edge_sliced(const int32_t* rowptrT, const int32_t* colT, const int64_t* permT,
                        int32_t n_rows, int heads, int d_head, const float* s2, float alpha,
                        const float* emask, const float* rec, const float* pd, int64_t nnzT,
                        const float* a, T* dH, int64_t lddh, float* dzT, float* ds2,
                        hipStream_t st) {
  const int D = heads * d_head;
  if (n_rows < 0 || !gat_sl_shape(heads, d_head, 64) || nnzT < 0 ||
      (dH && (lddh % 4 || lddh < D)))
    return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!rowptrT || !colT || !s2 || !rec || !pd || !a || !dzT || !ds2 || (emask && !permT))
    return GNNEA_EINVAL;
  if (!alv<T>(dH)) return GNNEA_EALIGN;
  const int S = div_up(D, 64);
#define GNNEA_E1(HH, LP)                                                                        \
  hipLaunchKernelGGL((k_gat_bwd_edge<HH, LP, T>), dim3(div_up(n_rows, 256 / LP)), dim3(256), 0, \
                     st, rowptrT, colT, permT, n_rows, S, D, d_head, s2, alpha, emask,          \
                     (const float4*)rec, (const float2*)pd, nnzT, a, dH, lddh, dzT, ds2)
#define GNNEA_E(HH)                                              \
  case HH:                                                       \
    GNNEA_E1(HH, 32);                                            \
    break;
  GNNEA_HEADS_SWITCH(GNNEA_E)
#undef GNNEA_E
#undef GNNEA_E1
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
int gat_bwd_dst_sliced(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows, int heads,
                       int d_head, const float* dzT, const float* a, const float* ds2, T* dH,
                       int64_t lddh, float* ds1, hipStream_t st) {
  const int D = heads * d_head;
  if (n_rows < 0 || !gat_sl_shape(heads, d_head, 64) || lddh % 4 || lddh < D)
    return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  if (!rowptr || !tpos || !dzT || !a || !dH || !ds1) return GNNEA_EINVAL;
  if (!alv<T>(dH)) return GNNEA_EALIGN;
  const int nch = (D / 4 + 63) / 64;
  typedef typename Vec4<T>::raw R;
#define GNNEA_D(HH, NC)                                                                            \
  hipLaunchKernelGGL((k_gat_bwd_dst_s<HH, NC, 32, T>), dim3(div_up(n_rows, 8)), dim3(256), 0, st,  \
                     rowptr, tpos, n_rows, D, d_head, dzT, a, ds2, (R*)dH, lddh / 4, ds1)
#define GNNEA_D_H(HH)                        \
  case HH:                                   \
    switch (nch) {                           \
      case 1: GNNEA_D(HH, 1); break;         \
      case 2: GNNEA_D(HH, 2); break;         \
      case 3: GNNEA_D(HH, 3); break;         \
      default: GNNEA_D(HH, 4); break;        \
    }                                        \
    break;
  GNNEA_HEADS_SWITCH(GNNEA_D_H)
#undef GNNEA_D_H
#undef GNNEA_D
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace

// G (slice-major [ceil(D/64)][n_rows][64], sstride elements per slice) and the records
extern "C" int gnnea_gat_bwd_prep_sliced_f32(int32_t n_rows, int heads, int d_head,
                                             const float* dY, const float* Y, int64_t ldy,
                                             const float* s1, const float* m, const float* den,
                                             int act, float* Gs, int64_t sstride, float* rec,
                                             void* stream) {
  return gat_bwd_prep_sliced<float>(n_rows, heads, d_head, dY, Y, ldy, s1, m, den, act, Gs,
                                    sstride, rec, (hipStream_t)stream);
}
extern "C" int gnnea_gat_bwd_prep_sliced_bf16(int32_t n_rows, int heads, int d_head,
                                              const void* dY, const void* Y, int64_t ldy,
                                              const float* s1, const float* m, const float* den,
                                              int act, void* Gs, int64_t sstride, float* rec,
                                              void* stream) {
  return gat_bwd_prep_sliced<bf16_t>(n_rows, heads, d_head, (const bf16_t*)dY, (const bf16_t*)Y,
                                     ldy, s1, m, den, act, (bf16_t*)Gs, sstride, rec,
                                     (hipStream_t)stream);
}

// source rows j of A^T (one KG block): per-edge weights wT, then the slice passes writing
// dH_j = sum_i w_ij G_i (row-major, ldh) and the per-slice product partials pd [S][nnzT][2];
// wT / pd are indexed by the absolute A^T position (rowptrT values), nnzT = A^T's entry count
extern "C" int gnnea_gat_bwd_src_sliced_f32(const int32_t* rowptrT, const int32_t* colT,
                                            const int64_t* permT, int32_t n_rows, int heads,
                                            int d_head, const float* Hm, int64_t ldh,
                                            const float* s2, float alpha, const float* emask,
                                            const float* rec, const float* Gs, int64_t sstride,
                                            float* wT, float* pd, int64_t nnzT, float* dH,
                                            int64_t lddh, void* stream) {
  return gat_bwd_src_sliced<float>(rowptrT, colT, permT, n_rows, heads, d_head, Hm, ldh, s2,
                                   alpha, emask, rec, Gs, sstride, wT, pd, nnzT, dH, lddh,
                                   (hipStream_t)stream);
}
extern "C" int gnnea_gat_bwd_src_sliced_bf16(const int32_t* rowptrT, const int32_t* colT,
                                             const int64_t* permT, int32_t n_rows, int heads,
                                             int d_head, const void* Hm, int64_t ldh,
                                             const float* s2, float alpha, const float* emask,
                                             const float* rec, const void* Gs, int64_t sstride,
                                             float* wT, float* pd, int64_t nnzT, void* dH,
                                             int64_t lddh, void* stream) {
  return gat_bwd_src_sliced<bf16_t>(rowptrT, colT, permT, n_rows, heads, d_head,
                                    (const bf16_t*)Hm, ldh, s2, alpha, emask, rec,
                                    (const bf16_t*)Gs, sstride, wT, pd, nnzT, (bf16_t*)dH, lddh,
                                    (hipStream_t)stream);
}

// dz (A^T order), ds2 and, when dH is non-NULL, dH_j += ds2_j (x) a2 for the source rows
extern "C" int gnnea_gat_bwd_edge_sliced_f32(const int32_t* rowptrT, const int32_t* colT,
                                             const int64_t* permT, int32_t n_rows, int heads,
                                             int d_head, const float* s2, float alpha,
                                             const float* emask, const float* rec,
                                             const float* pd, int64_t nnzT, const float* a,
                                             float* dH, int64_t lddh, float* dzT, float* ds2,
                                             void* stream) {
  return gat_bwd_edge_sliced<float>(rowptrT, colT, permT, n_rows, heads, d_head, s2, alpha,
                                    emask, rec, pd, nnzT, a, dH, lddh, dzT, ds2,
                                    (hipStream_t)stream);
}
extern "C" int gnnea_gat_bwd_edge_sliced_bf16(const int32_t* rowptrT, const int32_t* colT,
                                              const int64_t* permT, int32_t n_rows, int heads,
                                              int d_head, const float* s2, float alpha,
                                              const float* emask, const float* rec,
                                              const float* pd, int64_t nnzT, const float* a,
                                              void* dH, int64_t lddh, float* dzT, float* ds2,
                                              void* stream) {
  return gat_bwd_edge_sliced<bf16_t>(rowptrT, colT, permT, n_rows, heads, d_head, s2, alpha,
                                     emask, rec, pd, nnzT, a, (bf16_t*)dH, lddh, dzT, ds2,
                                     (hipStream_t)stream);
}

// ds1 and dH_i += ds1_i (x) a1 (+ ds2_i (x) a2 when ds2 is non-NULL) for the destination rows
extern "C" int gnnea_gat_bwd_dst_sliced_f32(const int32_t* rowptr, const int64_t* tpos,
                                            int32_t n_rows, int heads, int d_head,
                                            const float* dzT, const float* a, const float* ds2,
                                            float* dH, int64_t lddh, float* ds1, void* stream) {
  return gat_bwd_dst_sliced<float>(rowptr, tpos, n_rows, heads, d_head, dzT, a, ds2, dH, lddh,
                                   ds1, (hipStream_t)stream);
}
extern "C" int gnnea_gat_bwd_dst_sliced_bf16(const int32_t* rowptr, const int64_t* tpos,
                                             int32_t n_rows, int heads, int d_head,
                                             const float* dzT, const float* a, const float* ds2,
                                             void* dH, int64_t lddh, float* ds1, void* stream) {
  return gat_bwd_dst_sliced<bf16_t>(rowptr, tpos, n_rows, heads, d_head, dzT, a, ds2,
                                    (bf16_t*)dH, lddh, ds1, (hipStream_t)stream);
}

// ---- slice ranges (the staged halo of a row-sharded GAT layer, gnnea/dist_graph.py) ---------- //
// the forward over slices [s_begin, s_end) of Hs only; stats != 0 runs the row statistics /
// edge weights first (m_out, den_out, wgt) — with s_begin == s_end that is all it does
extern "C" int gnnea_gat_fwd_sliced_range_f32(const int32_t* rowptr, const int32_t* col,
                                              int32_t n_rows, const float* Hs, int64_t sstride,
                                              int heads, int d_head, const float* s1,
                                              const float* s2, float alpha,
                                              const float* edge_mask, int act, float* Y,
                                              int64_t ldy, float* m_out, float* den_out,
                                              float* wgt, int s_begin, int s_end, int stats,
                                              void* stream) {
  return gat_fwd_sliced<float>(rowptr, col, n_rows, Hs, sstride, heads, d_head, s1, s2, alpha,
                               edge_mask, act, Y, ldy, m_out, den_out, wgt, (hipStream_t)stream,
                               s_begin, s_end, stats != 0);
}
extern "C" int gnnea_gat_fwd_sliced_range_bf16(const int32_t* rowptr, const int32_t* col,
                                               int32_t n_rows, const void* Hs, int64_t sstride,
                                               int heads, int d_head, const float* s1,
                                               const float* s2, float alpha,
                                               const float* edge_mask, int act, void* Y,
                                               int64_t ldy, float* m_out, float* den_out,
                                               float* wgt, int s_begin, int s_end, int stats,
                                               void* stream) {
  return gat_fwd_sliced<bf16_t>(rowptr, col, n_rows, (const bf16_t*)Hs, sstride, heads, d_head,
                                s1, s2, alpha, edge_mask, act, (bf16_t*)Y, ldy, m_out, den_out,
                                wgt, (hipStream_t)stream, s_begin, s_end, stats != 0);
}

// the source pass over slices [s_begin, s_end) (weights != 0: the per-edge weights wT first);
// H and dH each row-major (hss / dhss = 64, ldh / lddh >= D) or slice-major 64-column tables
// (ldh / lddh = 64, hss / dhss = their slice strides) — the halo's slice tables of a row shard
extern "C" int gnnea_gat_bwd_src_sliced_range_f32(
    const int32_t* rowptrT, const int32_t* colT, const int64_t* permT, int32_t n_rows, int heads,
    int d_head, const float* Hm, int64_t ldh, int64_t hss, const float* s2, float alpha,
    const float* emask, const float* rec, const float* Gs, int64_t sstride, float* wT, float* pd,
    int64_t nnzT, float* dH, int64_t lddh, int64_t dhss, int s_begin, int s_end, int weights,
    void* stream) {
  return gat_bwd_src_sliced<float>(rowptrT, colT, permT, n_rows, heads, d_head, Hm, ldh, s2,
                                   alpha, emask, rec, Gs, sstride, wT, pd, nnzT, dH, lddh,
                                   (hipStream_t)stream, hss, dhss, s_begin, s_end, weights != 0);
}
extern "C" int gnnea_gat_bwd_src_sliced_range_bf16(
    const int32_t* rowptrT, const int32_t* colT, const int64_t* permT, int32_t n_rows, int heads,
    int d_head, const void* Hm, int64_t ldh, int64_t hss, const float* s2, float alpha,
    const float* emask, const float* rec, const void* Gs, int64_t sstride, float* wT, float* pd,
    int64_t nnzT, void* dH, int64_t lddh, int64_t dhss, int s_begin, int s_end, int weights,
    void* stream) {
  return gat_bwd_src_sliced<bf16_t>(rowptrT, colT, permT, n_rows, heads, d_head,
                                    (const bf16_t*)Hm, ldh, s2, alpha, emask, rec,
                                    (const bf16_t*)Gs, sstride, wT, pd, nnzT, (bf16_t*)dH, lddh,
                                    (hipStream_t)stream, hss, dhss, s_begin, s_end, weights != 0);
}
