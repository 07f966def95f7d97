// a5-a7. Sparse GAT, every head in one edge pass (layers/att_layers.py:29-61, 82-91).
//
// The reference materialises cat(h[row], h[col]) (E x 2*d_head per head, att_layers.py:38),
// exponentiates, and runs two torch.spmm per head (:45, :54).  Here the attention logit is
// factorised per node (s1 = H·a[:d], s2 = H·a[d:], computed once per layer), and one wave per
// destination row walks the row's edges once for ALL heads:
//   pass 1 (lane-parallel over edges, 4-16 B per edge): row max of the logit per head;
//   pass 2: lane k computes edge k's weights exp(score - max) for every head, then the wave
//           gathers neighbour rows H_j (16 B per lane, the whole head-concatenated 1200-B row)
//           and applies the per-element head weight broadcast by readlane.
// The head-concatenated layout of H is exactly the concat=True output layout of
// GraphAttentionLayer (att_layers.py:86), so Y is written in place of torch.cat.
#include "common.h"

namespace gnnea {

// ---------------------------------------------------------------------------------------- //
// Head-grouped lane layout (scores and backward src pass).  With HP = H rounded up to a power of
// two, each head owns LPH = 64 / HP consecutive lanes and lane s of a head owns the EPL
// consecutive elements d = s*EPL + t of that head (d < d_head).  Every lane then works for ONE
// head: per-head dot products are sums over a lane group (DPP steps inside 16-lane rows, one
// bpermute per extra row), and no per-element head selection is needed.
// ---------------------------------------------------------------------------------------- //
template <int H> struct Pow2 { static constexpr int v = H <= 1 ? 1 : H <= 2 ? 2 : H <= 4 ? 4 : 8; };

template <int H, int EPL>
struct HeadLanes {
  static constexpr int HP = Pow2<H>::v, LPH = 64 / HP;
  int h, d0;           // the lane's head and first element within the head
  bool ok[EPL];        // element exists
  int c[EPL];          // column in the head-concatenated row (clamped in range when !ok)
  __device__ __forceinline__ HeadLanes(int lane, int dh) {
    h = lane / LPH;
    d0 = (lane % LPH) * EPL;
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      ok[t] = h < H && d0 + t < dh;
      c[t] = ok[t] ? h * dh + d0 + t : 0;
    }
  }
};

struct __attribute__((aligned(4))) U3 { uint32_t x, y, z; };

template <int W>
__device__ __forceinline__ void load_dw(const char* p, uint32_t* d) {
  if constexpr (W >= 4) {
    const uint4 v = *(const uint4*)p;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    if constexpr (W > 4) load_dw<W - 4>(p + 16, d + 4);
  } else if constexpr (W == 3) {
    const U3 v = *(const U3*)p;
    d[0] = v.x; d[1] = v.y; d[2] = v.z;
  } else if constexpr (W == 2) {
    const uint2 v = *(const uint2*)p;
    d[0] = v.x; d[1] = v.y;
  } else {
    d[0] = *(const uint32_t*)p;
  }
}

// the same window through a buffer resource on the (wave-uniform) row base: the row address is
// scalar arithmetic, the lane's window offset the 32-bit voffset -- no 64-bit vector address
// per edge (a global pointer formed as base + row * ld + lane offset is re-associated by the
// compiler into a per-lane 64-bit multiply-add)
template <int W>
__device__ __forceinline__ void load_dw_row(const char* row, uint32_t off, uint32_t* d) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, 0x7fffffff, 0x00020000);
  typedef unsigned int u2 __attribute__((ext_vector_type(2)));
  typedef unsigned int u3 __attribute__((ext_vector_type(3)));
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  int q = 0;
#pragma unroll
  for (; q + 4 <= W; q += 4) {
    const u4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 4 * q, 0, 0);
    d[q] = v.x; d[q + 1] = v.y; d[q + 2] = v.z; d[q + 3] = v.w;
  }
  if constexpr (W % 4 == 3) {
    const u3 v = __builtin_amdgcn_raw_buffer_load_b96(rs, off + 4 * q, 0, 0);
    d[q] = v.x; d[q + 1] = v.y; d[q + 2] = v.z;
  } else if constexpr (W % 4 == 2) {
    const u2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 4 * q, 0, 0);
    d[q] = v.x; d[q + 1] = v.y;
  } else if constexpr (W % 4 == 1) {
    d[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4 * q, 0, 0);
  }
}

template <typename T, int EPL> struct RowWin;
template <int EPL> struct RowWin<float, EPL> {
  static constexpr int W = EPL;
  static __host__ __device__ int64_t byte_off(int c) { return 4 * (int64_t)c; }
  static __device__ __forceinline__ void unpack(const uint32_t (&d)[W], uint32_t, float (&f)[EPL]) {
#pragma unroll
    for (int t = 0; t < EPL; ++t) f[t] = __builtin_bit_cast(float, d[t]);
  }
};
template <int EPL> struct RowWin<bf16_t, EPL> {
  static constexpr int W = (EPL + 2) / 2;  // EPL halfwords + a possible leading one
  static __host__ __device__ int64_t byte_off(int c) { return (2 * (int64_t)c) & ~(int64_t)3; }
  // shb: the window's byte shift (2 when the first element is odd): one v_alignbyte per element
  // pair brings halfwords (2p, 2p + 1) into a dword, then a shift / a mask widens each to f32
  static __device__ __forceinline__ void unpack(const uint32_t (&d)[W], uint32_t shb,
                                                float (&f)[EPL]) {
#pragma unroll
    for (int p = 0; 2 * p < EPL; ++p) {
      const uint32_t v = __builtin_amdgcn_alignbyte(d[p + 1 < W ? p + 1 : W - 1], d[p], shb);
      f[2 * p] = __builtin_bit_cast(float, v << 16);
      if (2 * p + 1 < EPL) f[2 * p + 1] = __builtin_bit_cast(float, v & 0xffff0000u);
    }
  }
};


// s1[i,h] = sum_d H[i, h*dh+d] * a[h, d];  s2[i,h] = sum_d H[i, h*dh+d] * a[h, dh+d]
// A wave walks rows (grid-stride) with the lane's slice of a preloaded.
// A lane's EPL consecutive elements are read as whole 16-B windows: bf16 (EPL <= 6) ONE load of
// the 4-B aligned window holding them (as k_gat_bwd_src's WIN), fp32 (EPL <= 8) the 16 or 32 B
// from its first element -- one or two load instructions per row instead of EPL element loads,
// which left the pass at 2.5 (bf16) / 3.6 (fp32) TB/s; a window may run into the next row, so the
// last row takes the element loads, in a pass of its own (every main-loop load unconditional).
template <int H, int EPL, typename T>
__global__ __launch_bounds__(256) void k_gat_scores(const T* __restrict__ Hm, int64_t ldh,
                                                    int n_rows, int dh,
                                                    const float* __restrict__ a,
                                                    float* __restrict__ s1,
                                                    float* __restrict__ s2) {
  using L = HeadLanes<H, EPL>;
  constexpr bool WIN = sizeof(T) == 2 ? EPL <= 6 : EPL <= 8;
  const int lane = lane_id();
  const L hl(lane, dh);
  float a1[EPL], a2[EPL];
#pragma unroll
  for (int t = 0; t < EPL; ++t) {
    const int d = hl.ok[t] ? hl.d0 + t : 0;
    const int hh = hl.ok[t] ? hl.h : 0;
    a1[t] = hl.ok[t] ? a[hh * 2 * dh + d] : 0.f;
    a2[t] = hl.ok[t] ? a[hh * 2 * dh + dh + d] : 0.f;
  }
  const bool wsh = (hl.c[0] & 1) != 0;  // WIN (bf16): the window's halfword shift
  auto score = [&](const float (&xv)[EPL], int row) {
    float p[2] = {0.f, 0.f};
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      const float v = hl.ok[t] ? xv[t] : 0.f;
      p[0] = fmaf(v, a1[t], p[0]);
      p[1] = fmaf(v, a2[t], p[1]);
    }
    const float r = grp_sum<2, L::LPH>(p, lane);
    const int o = lane % L::LPH;
    if (hl.h < H) {
      if (o == grp_lane<2, L::LPH>(0)) s1[(int64_t)row * H + hl.h] = r;
      if (o == grp_lane<2, L::LPH>(1)) s2[(int64_t)row * H + hl.h] = r;
    }
  };
  // RR rows per round, every load of the round issued before any is used (one row's loads in
  // flight per wave left the pass latency-bound); the per-row arithmetic is unchanged
  constexpr int RR = WIN ? 8 : 4;
  const int nmain = WIN ? n_rows - 1 : n_rows;  // (WIN: rows whose window stays in the table)
  const int nw = gridDim.x * 4;
  for (int base = blockIdx.x * 4 + wave_id(); base < nmain; base += RR * nw) {
    float xv[RR][EPL];
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      const T* x = Hm + (int64_t)min(base + k * nw, nmain - 1) * ldh;
      if constexpr (WIN) {  // the exact window (RowWin: EPL dwords / the 4-B aligned halfwords)
        uint32_t dw[RowWin<T, EPL>::W];
        load_dw<RowWin<T, EPL>::W>((const char*)x + RowWin<T, EPL>::byte_off(hl.c[0]), dw);
        RowWin<T, EPL>::unpack(dw, wsh ? 2u : 0u, xv[k]);
      } else {
#pragma unroll
        for (int t = 0; t < EPL; ++t) xv[k][t] = to_f32<T>(x[hl.c[t]]);
      }
    }
#pragma unroll
    for (int k = 0; k < RR; ++k) {
      const int row = base + k * nw;
      if (row >= nmain) break;  // uniform
      score(xv[k], row);
    }
  }
  if (WIN && blockIdx.x == 0 && wave_id() == 0) {  // the last row, element loads
    const T* x = Hm + (int64_t)(n_rows - 1) * ldh;
    float xv[EPL];
#pragma unroll
    for (int t = 0; t < EPL; ++t) xv[t] = to_f32<T>(x[hl.c[t]]);
    score(xv, n_rows - 1);
  }
}

template <int ACT, int H, int NCH, typename T>
__global__ __launch_bounds__(256) void k_gat_fwd(const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col, int n_rows,
                                                 const typename Vec4<T>::raw* __restrict__ Hm,
                                                 int64_t ldh4,
                                                 int D, int dh, const float* __restrict__ s1,
                                                 const float* __restrict__ s2, float alpha,
                                                 const float* __restrict__ emask,
                                                 typename Vec4<T>::raw* __restrict__ Y,
                                                 int64_t ldy4,
                                                 float* __restrict__ m_out,
                                                 float* __restrict__ den_out) {
  constexpr int kFE = 2;  // edges per chunk (measured: 2 beats 1 and 4)
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptr[row], end = rowptr[row + 1];

  float si[H];
#pragma unroll
  for (int h = 0; h < H; ++h) si[h] = s1[(int64_t)row * H + h];

  // head index of each owned element (H = "no head": padding column)
  int hd[NCH][4];
  bool own[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    own[q] = 4 * c4 < D;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      hd[q][t] = c < D ? c / dh : H;
    }
  }

  // pass 1: per-head row max of score = -LeakyReLU(s1_i + s2_j)
  float mx[H];
#pragma unroll
  for (int h = 0; h < H; ++h) mx[h] = -INFINITY;
  for (int e = beg + lane; e < end; e += 64) {
    const int j = col[e];
#pragma unroll
    for (int h = 0; h < H; ++h) mx[h] = fmaxf(mx[h], -lrelu(si[h] + s2[(int64_t)j * H + h], alpha));
  }
#pragma unroll
  for (int h = 0; h < H; ++h) mx[h] = wave_max(mx[h]);

  float den[H];
#pragma unroll
  for (int h = 0; h < H; ++h) den[h] = 0.f;
  float4 acc[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mj = 0;
    float wl[H];
#pragma unroll
    for (int h = 0; h < H; ++h) wl[h] = 0.f;
    if (lane < cnt) {
      mj = col[base + lane];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float w = __expf(-lrelu(si[h] + s2[(int64_t)mj * H + h], alpha) - mx[h]);
        den[h] += w;  // the row sum uses the un-dropped weights (att_layers.py:45-51)
        wl[h] = emask ? w * emask[(int64_t)(base + lane) * H + h] : w;
      }
    }
    // kFE edges at a time: their neighbour rows are gathered together (kFE * NCH loads in
    // flight), then accumulated in edge order
    for (int k = 0; k < cnt; k += kFE) {
      typename Vec4<T>::raw r[kFE][NCH];
      float w[kFE][H];
#pragma unroll
      for (int e = 0; e < kFE; ++e) {
        const int ke = min(k + e, cnt - 1);  // past the chunk: a valid row, not accumulated
        const typename Vec4<T>::raw* x = Hm + (int64_t)readlane_i(mj, ke) * ldh4 + lane;
#pragma unroll
        for (int h = 0; h < H; ++h) w[e][h] = readlane_f(wl[h], ke);
#pragma unroll
        for (int q = 0; q < NCH; ++q)
          if (own[q]) r[e][q] = x[64 * q];
      }
#pragma unroll
      for (int e = 0; e < kFE; ++e) {
        if (k + e >= cnt) break;  // uniform
#pragma unroll
        for (int q = 0; q < NCH; ++q)
          if (own[q]) {
            const float4 xv = Vec4<T>::get(r[e][q]);
            acc[q].x = fmaf(hsel<H>(w[e], hd[q][0]), xv.x, acc[q].x);
            acc[q].y = fmaf(hsel<H>(w[e], hd[q][1]), xv.y, acc[q].y);
            acc[q].z = fmaf(hsel<H>(w[e], hd[q][2]), xv.z, acc[q].z);
            acc[q].w = fmaf(hsel<H>(w[e], hd[q][3]), xv.w, acc[q].w);
          }
      }
    }
  }
  float rinv[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    den[h] = wave_sum(den[h]);
    rinv[h] = den[h] > 0.f ? 1.f / den[h] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    if (!own[q]) continue;
    float4 o;
    o.x = hd[q][0] < H ? act_fwd<ACT>(acc[q].x * hsel<H>(rinv, hd[q][0])) : 0.f;
    o.y = hd[q][1] < H ? act_fwd<ACT>(acc[q].y * hsel<H>(rinv, hd[q][1])) : 0.f;
    o.z = hd[q][2] < H ? act_fwd<ACT>(acc[q].z * hsel<H>(rinv, hd[q][2])) : 0.f;
    o.w = hd[q][3] < H ? act_fwd<ACT>(acc[q].w * hsel<H>(rinv, hd[q][3])) : 0.f;
    Y[(int64_t)row * ldy4 + lane + 64 * q] = Vec4<T>::put(o);
  }
  if (lane < H) {
    m_out[(int64_t)row * H + lane] = hsel<H>(mx, lane);
    den_out[(int64_t)row * H + lane] = hsel<H>(den, lane);
  }
}

// ---------------------------------------------------------------------------------------- //
// Backward: one gather sweep over A^T instead of two over A.                                //
//   prep (rows i): G_i = dY_i * act'(Y_i); record R_i,h = {s1, row max m, 1/den, c = G_i.h'_i}
//   src  (rows j of A^T, in-neighbours i): alpha_ij from R_i, gather G_i:
//        dH_j = sum_i alpha*mask*G_i  (+ ds2_j (x) a2),   da_ij,h = G_i,h . H_j,h (own row),
//        dz_ij = -LeakyReLU'(z) * alpha * (mask*da - c_i),  ds2_j = sum_i dz   -> dz in A^T order
//   dst  (rows i of A): ds1_i = sum_j dz_ij (read through the inverse permutation),
//        dH_i += ds1_i (x) a1
// ---------------------------------------------------------------------------------------- //

// prep over FOUR rows per wave: every dY / Y load of the four rows issued before any is used (a
// row per wave kept one row's loads in flight and measured slower, round 4; removed); per row the
// element arithmetic and the wave sums in a fixed order.
template <int ACT, int H, int NCH, typename T>
__global__ __launch_bounds__(256) void k_gat_bwd_prep4(int n_rows, int D, int dh,
                                                       const typename Vec4<T>::raw* __restrict__ dY,
                                                       const typename Vec4<T>::raw* __restrict__ Y,
                                                       int64_t ld4,
                                                       const float* __restrict__ s1,
                                                       const float* __restrict__ mrow,
                                                       const float* __restrict__ den,
                                                       typename Vec4<T>::raw* __restrict__ G,
                                                       float4* __restrict__ rec) {
  typedef typename Vec4<T>::raw R;
  constexpr int HP = Pow2<H>::v;  // the per-head sums reduce-scattered over the wave (grp_sum)
  const int r0 = (blockIdx.x * 4 + wave_id()) * 4;
  if (r0 >= n_rows) return;
  const int lane = lane_id();
  // the lane that ends with head h's sum: grp_lane<HP, 64>(h) = h * (16 / HP); its record loads
  const int hw = lane % (16 / HP) == 0 && lane < 16 ? lane / (16 / HP) : 0;
  // per chunk: the head of the lane's first element and how many of its four are in that head
  // (a chunk of four spans at most two heads: dh >= 4), the rest in the next
  int hq[NCH], es[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c = 4 * (lane + 64 * q);
    hq[q] = c < D ? c / dh : HP;
    es[q] = c < D ? (hq[q] + 1) * dh - c : 4;
  }
  R vd[4][NCH], vy[4][NCH];
  float rs1[4], rmx[4], rdv[4];  // the records' row statistics, read with the rows
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int64_t rw = min(r0 + rr, n_rows - 1);
    const int64_t ro = rw * H + (hw < H ? hw : 0);
    rs1[rr] = s1[ro];
    rmx[rr] = mrow[ro];
    rdv[rr] = den[ro];
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int c4 = min(lane + 64 * q, (D + 3) / 4 - 1);
      vd[rr][q] = dY[rw * ld4 + c4];
      vy[rr][q] = Y[rw * ld4 + c4];
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int row = r0 + rr;
    if (row >= n_rows) break;  // uniform
    float cp[HP];
#pragma unroll
    for (int h = 0; h < HP; ++h) cp[h] = 0.f;
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int c4 = lane + 64 * q;
      if (4 * c4 >= D) continue;
      const float4 dy = Vec4<T>::get(vd[rr][q]);
      const float4 y = Vec4<T>::get(vy[rr][q]);
      const float ys[4] = {y.x, y.y, y.z, y.w};
      float gs[4] = {dy.x, dy.y, dy.z, dy.w};
      float pa = 0.f, pb = 0.f;  // G.Y over the elements in head hq and in the next
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        gs[t] = 4 * c4 + t < D ? gs[t] * act_grad_from_out<ACT>(ys[t]) : 0.f;
        const float v = gs[t] * ys[t];
        if (dh >= 4) {  // (uniform) at most two heads per chunk
          pa += t < es[q] ? v : 0.f;
          pb += t < es[q] ? 0.f : v;
        } else {
          const int hh = (4 * c4 + t) / dh;
#pragma unroll
          for (int h = 0; h < HP; ++h) cp[h] += hh == h ? v : 0.f;
        }
      }
#pragma unroll
      for (int h = 0; h < HP; ++h) cp[h] += (h == hq[q] ? pa : 0.f) + (h == hq[q] + 1 ? pb : 0.f);
      G[(int64_t)row * ld4 + c4] = Vec4<T>::put(make_float4(gs[0], gs[1], gs[2], gs[3]));
    }
    const float cs = grp_sum<HP, 64>(cp, lane);
    if (lane % (16 / HP) == 0 && lane < 16 && hw < H)
      rec[(int64_t)row * H + hw] = make_float4(rs1[rr], rmx[rr],
                                               rdv[rr] > 0.f ? 1.f / rdv[rr] : 0.f, cs);
  }
}

// Head-grouped layout: per in-edge (i, j) the lane accumulates alpha*mask*G_i into its own
// elements and the product G_i . H_j over them; kEB edges' G rows are gathered together (the next
// chunk's in flight meanwhile) and their per-head dot products reduced by one grp_sum (lane h*LPH + grp_lane(e) gets edge e, head h).
// WIN (bf16, EPL <= 6, g_rows known): a lane's EPL consecutive elements of G_i are read as ONE
// 16-B load of the 4-B aligned window holding them (one load instruction per edge instead of EPL
// 2-B loads; the window may run into the next row, so G's last row takes the element loads --
// the gathered row is wave-uniform per edge, so the choice is a uniform branch).
template <int H, int EPL, typename T, bool WIN = false>
__global__ __launch_bounds__(256) void k_gat_bwd_src(
    const int32_t* __restrict__ rowptrT, const int32_t* __restrict__ colT,
    const int64_t* __restrict__ permT, int n_rows, int dh, const T* __restrict__ Hm,
    int64_t ldh, const float* __restrict__ s2, float alpha, const float* __restrict__ emask,
    const float4* __restrict__ rec, const T* __restrict__ G, int64_t ldg,
    const float* __restrict__ a, T* __restrict__ dH, int64_t lddh, float* __restrict__ dzT,
    float* __restrict__ ds2, int64_t g_rows) {
  using L = HeadLanes<H, EPL>;
  constexpr int LPH = L::LPH;
  constexpr int kEB = 2;  // edges per chunk (measured: 2 beats 4 and 8 once double-buffered)
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();  // source node j
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptrT[row], end = rowptrT[row + 1];
  const L hl(lane, dh);
  const int hme = hl.h < H ? hl.h : 0;

  float hj[EPL], acc[EPL], a2l[EPL];
  {
    const T* x = Hm + (int64_t)row * ldh;
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      const float v = to_f32<T>(x[hl.c[t]]);
      hj[t] = hl.ok[t] ? v : 0.f;
      acc[t] = 0.f;
      // the epilogue's a_2 terms, read now: read there, each was a serial L2 round trip between
      // the row's last edge and its stores
      a2l[t] = hl.ok[t] ? a[hme * 2 * dh + dh + hl.d0 + t] : 0.f;
    }
  }
  float sj[H], ds2p[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    sj[h] = s2[(int64_t)row * H + h];
    ds2p[h] = 0.f;
  }

  // chunk loads depend only on the in-neighbour ids: chunk c + 1 is in flight while chunk c is
  // reduced (register double buffer), and chunk 0 goes out before the attention records arrive
  float gA[kEB][EPL], gB[kEB][EPL];
  const int wbyte = (2 * hl.c[0]) & ~3;  // WIN: the lane's window, halfword shift
  const bool wsh = (hl.c[0] & 1) != 0;
  auto load = [&](float (&g)[kEB][EPL], int mi, int k, int cnt) {
#pragma unroll
    for (int e = 0; e < kEB; ++e) {
      const int r = readlane_i(mi, min(k + e, cnt - 1));
      const T* gr = G + (int64_t)r * ldg;
      if (WIN && r + 1 < g_rows) {
        const uint4 v = *(const uint4*)((const char*)gr + wbyte);
        const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < EPL; ++t) {  // halfword t + wsh of the window, widened to f32
          const uint32_t lo = (t & 1) ? (dw[t >> 1] & 0xffff0000u) : (dw[t >> 1] << 16);
          const uint32_t hi = (t & 1) ? (dw[(t + 1) >> 1] << 16) : (dw[t >> 1] & 0xffff0000u);
          g[e][t] = __uint_as_float(wsh ? hi : lo);
        }
      } else {
#pragma unroll
        for (int t = 0; t < EPL; ++t) g[e][t] = to_f32<T>(gr[hl.c[t]]);
      }
    }
  };
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mi = 0;
    int64_t pe = 0;
    if (lane < cnt) {
      mi = colT[base + lane];  // destination row i of the forward edge (i, j)
      pe = permT[base + lane];
    }
    float4 rr[H];
#pragma unroll
    for (int h = 0; h < H; ++h) rr[h] = rec[(int64_t)mi * H + h];  // {s1_i, m_i, 1/den_i, c_i}
    load(gA, mi, 0, cnt);
    float al[H], zl[H], ml[H], cl[H], wl[H], dzl[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float z = rr[h].x + sj[h];
      zl[h] = z;
      al[h] = lane < cnt ? __expf(-lrelu(z, alpha) - rr[h].y) * rr[h].z : 0.f;
      cl[h] = rr[h].w;
      ml[h] = (emask && lane < cnt) ? emask[pe * H + h] : 1.f;
      wl[h] = al[h] * ml[h];
      dzl[h] = 0.f;
    }
    auto process = [&](const float (&g)[kEB][EPL], int k) {
      float w[kEB];
#pragma unroll
      for (int e = 0; e < kEB; ++e) {
        const int ke = min(k + e, cnt - 1);
        float we = 0.f;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const float v = readlane_f(wl[h], ke);
          we = hme == h ? v : we;
        }
        w[e] = we;
      }
      float pd[kEB];
#pragma unroll
      for (int e = 0; e < kEB; ++e) {
        float q = 0.f;
#pragma unroll
        for (int t = 0; t < EPL; ++t) {
          const float gv = hl.ok[t] ? g[e][t] : 0.f;
          if (k + e < cnt) acc[t] = fmaf(w[e], gv, acc[t]);  // uniform branch
          q = fmaf(gv, hj[t], q);
        }
        pd[e] = q;
      }
      const float v = grp_sum<kEB, LPH>(pd, lane);
#pragma unroll
      for (int e = 0; e < kEB; ++e) {
        if (k + e >= cnt) break;  // uniform
        float da[H];
#pragma unroll
        for (int h = 0; h < H; ++h) da[h] = readlane_f(v, h * LPH + grp_lane<kEB, LPH>(e));
        if (lane == k + e) {
#pragma unroll
          for (int h = 0; h < H; ++h)
            dzl[h] = -(al[h] * (ml[h] * da[h] - cl[h])) * (zl[h] > 0.f ? 1.f : alpha);
        }
      }
    };
    for (int k = 0; k < cnt; k += 2 * kEB) {
      if (k + kEB < cnt) load(gB, mi, k + kEB, cnt);
      process(gA, k);
      if (k + kEB >= cnt) break;
      if (k + 2 * kEB < cnt) load(gA, mi, k + 2 * kEB, cnt);
      process(gB, k + kEB);
    }
    if (lane < cnt) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        dzT[(int64_t)(base + lane) * H + h] = dzl[h];
        ds2p[h] += dzl[h];
      }
    }
  }
  float d2me = 0.f;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float d2 = wave_sum(ds2p[h]);
    d2me = hme == h ? d2 : d2me;
    if (lane == 0) ds2[(int64_t)row * H + h] = d2;
  }
  T* out = dH + (int64_t)row * lddh;
#pragma unroll
  for (int t = 0; t < EPL; ++t)
    if (hl.ok[t]) out[hl.c[t]] = from_f32<T>(acc[t] + d2me * a2l[t]);
}

// dst with FOUR destination rows per wave: per row a chain of dependent loads (rowptr -> tpos ->
// dzT -> the dH row's read-modify-write), so one row per wave kept one chain in flight (measured
// slower, round 4; removed).  Here lane group g (16 lanes) walks row r0 + g's edges (ds1 partials summed
// over the group in fixed order: lane-strided edges, then xor 1, 2, 4, 8), and the wave then
// updates the four dH rows with all of their loads issued before any is used.
template <int H, int NCH, typename T>
__global__ __launch_bounds__(256) void k_gat_bwd_dst4(const int32_t* __restrict__ rowptr,
                                                      const int64_t* __restrict__ tpos,
                                                      int n_rows, int D, int dh,
                                                      const float* __restrict__ dzT,
                                                      const float* __restrict__ a,
                                                      typename Vec4<T>::raw* __restrict__ dH,
                                                      int64_t lddh4,
                                                      float* __restrict__ ds1) {
  const int r0 = (blockIdx.x * 4 + wave_id()) * 4;
  if (r0 >= n_rows) return;
  const int lane = lane_id(), g = lane >> 4, l16 = lane & 15;
  const bool live = r0 + g < n_rows;
  const int row = live ? r0 + g : n_rows - 1;
  const int beg = rowptr[row], end = live ? rowptr[row + 1] : beg;
  float p[H];
#pragma unroll
  for (int h = 0; h < H; ++h) p[h] = 0.f;
  for (int e = beg + l16; e < end; e += 16) {
    const int64_t t = tpos[e];
    if constexpr (H == 4) {
      const float4 v = *(const float4*)(dzT + t * 4);
      p[0] += v.x; p[1] += v.y; p[2] += v.z; p[3] += v.w;
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) p[h] += dzT[t * H + h];
    }
  }
  // the group's head sums reduce-scattered inside its 16-lane row (DPP, no LDS): lane
  // grp_lane<HP, 16>(h) of the group ends with head h's sum
  constexpr int HP = Pow2<H>::v;
  float pp[HP];
#pragma unroll
  for (int h = 0; h < HP; ++h) pp[h] = h < H ? p[h] : 0.f;
  const float gsum = grp_sum<HP, 16>(pp, lane);
  const int hw = l16 % (16 / HP) == 0 ? l16 / (16 / HP) : H;
  if (live && hw < H) ds1[(int64_t)row * H + hw] = gsum;
  // the four rows' dH pieces: every load first
  typedef typename Vec4<T>::raw R;
  R v[4][NCH];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int rw = min(r0 + rr, n_rows - 1);
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int c4 = min(lane + 64 * q, (D + 3) / 4 - 1);
      v[rr][q] = dH[(int64_t)rw * lddh4 + c4];
    }
  }
  // a1 of the lane's columns and their heads: the same for the four rows, read once
  float av[NCH][4];
  int hc[NCH][4];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = min(4 * (lane + 64 * q) + t, D - 1), h = c / dh;
      hc[q][t] = h;
      av[q][t] = a[h * 2 * dh + (c - h * dh)];
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    if (r0 + rr >= n_rows) break;  // uniform
    float ph[H];  // row r0 + rr's head sums: scalar reads from its group's lanes
#pragma unroll
    for (int h = 0; h < H; ++h) ph[h] = readlane_f(gsum, 16 * rr + grp_lane<HP, 16>(h));
#pragma unroll
    for (int q = 0; q < NCH; ++q) {
      const int c4 = lane + 64 * q;
      if (4 * c4 >= D) continue;
      const float4 x = Vec4<T>::get(v[rr][q]);
      float o[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int c = 4 * c4 + t;
        if (c < D) o[t] += hsel<H>(ph, hc[q][t]) * av[q][t];
      }
      dH[(int64_t)(r0 + rr) * lddh4 + c4] = Vec4<T>::put(make_float4(o[0], o[1], o[2], o[3]));
    }
  }
}

static bool ok_ld(int64_t ld, int D) { return ld % 4 == 0 && ld >= ((D + 3) / 4) * 4; }

// ---------------------------------------------------------------------------------------- //
// Head-grouped, pipelined row-major passes (the default where they apply).                   //
// The passes above are latency-chain bound, not bandwidth bound: a gathered row read inside a //
// uniform branch (the bf16 window / element choice, the edge mask) is waited on right where   //
// it is issued, so one neighbour row per wave is in flight, and the forward's per-edge logit  //
// and mask loads are serialised behind the same kind of branch.  Here every lane reads its    //
// head's EPL consecutive elements of a gathered row as ONE window of W dwords (bf16: the 4-B  //
// aligned dwords holding them, a halfword shift when the first element is odd; fp32: the      //
// EPL dwords), issued unconditionally (indices clamped to the chunk, the surplus tail loads   //
// re-read the last edge's row) in groups of F edges, two groups in flight (register double    //
// buffer), the edge mask a template flag.  Rows are still one wave each, in CSR order, and     //
// every per-element sum runs in edge order: the forward's outputs equal k_gat_fwd's.           //
// Host-checked: every lane's window ends inside the row's ld (no read past the table).        //
// ---------------------------------------------------------------------------------------- //
template <int H>
__device__ __forceinline__ void load_heads(const float* p, float (&v)[H]) {
  if constexpr (H == 4) {  // 16-B aligned rows (host-checked)
    const float4 q = *(const float4*)p;
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int h = 0; h < H; ++h) v[h] = p[h];
  }
}

template <int H, int EPL, typename T, bool EM, int F>
__global__ __launch_bounds__(256) void k_gat_fwd_hg(const int32_t* __restrict__ rowptr,
                                                    const int32_t* __restrict__ col, int n_rows,
                                                    const T* __restrict__ Hm, int64_t ldh, int D,
                                                    int dh, const float* __restrict__ s1,
                                                    const float* __restrict__ s2, float alpha,
                                                    const float* __restrict__ emask, int act,
                                                    T* __restrict__ Y, int64_t ldy,
                                                    float* __restrict__ m_out,
                                                    float* __restrict__ den_out) {
  constexpr int HPW = Pow2<H>::v;  // heads padded to a power of two (the all-reduces)
  using L = HeadLanes<H, EPL>;
  using WN = RowWin<T, EPL>;
  constexpr int W = WN::W;
  // per wave: the chunk's edge weights [edge][head]; each lane reads its head's weight of an edge
  // as one broadcast ds_read (H readlanes + selects per edge before)
  __shared__ float sh_w[4][64 * H];
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  float* shw = sh_w[wave_id()];
  const int beg = rowptr[row], end = rowptr[row + 1];
  const L hl(lane, dh);
  const int hme = hl.h < H ? hl.h : 0;
  // the gathered row's address: a wave-uniform (scalar) row base plus the lane's 32-bit window
  // offset (load_dw_row)
  const uint32_t woff = (uint32_t)WN::byte_off(hl.c[0]);
  const uint32_t wsh = (hl.c[0] & 1) ? 2u : 0u;
  const char* Hb = (const char*)Hm;
  const int64_t ldb = ldh * (int64_t)sizeof(T);

  float si[H];
#pragma unroll
  for (int h = 0; h < H; ++h) si[h] = s1[(int64_t)row * H + h];

  // lane k of a chunk: edge base + k's neighbour and logits (-LeakyReLU(s1_i + s2_j))
  int mj = 0;
  float sc[H];
  auto chunk = [&](int base, int cnt) {
    mj = col[base + min(lane, cnt - 1)];
    float v[H];
    load_heads<H>(s2 + (int64_t)mj * H, v);
    // (a select on the loaded value would let the compiler sink the load into a branch)
    const float pen = lane < cnt ? 0.f : -INFINITY;
#pragma unroll
    for (int h = 0; h < H; ++h) sc[h] = pen - lrelu(si[h] + v[h], alpha);
  };
  float mx[H], den[H], acc[EPL];
#pragma unroll
  for (int h = 0; h < H; ++h) den[h] = 0.f;
#pragma unroll
  for (int t = 0; t < EPL; ++t) acc[t] = 0.f;
  if (end > beg) {
    chunk(beg, min(64, end - beg));
    if (end - beg > 64) {  // long rows: the row maximum over every chunk first
      float m2[H];
#pragma unroll
      for (int h = 0; h < H; ++h) m2[h] = sc[h];
      for (int base = beg + 64; base < end; base += 64) {
        chunk(base, min(64, end - base));
#pragma unroll
        for (int h = 0; h < H; ++h) m2[h] = fmaxf(m2[h], sc[h]);
      }
      float mp[HPW];  // (all heads in one all-reduce, exact)
#pragma unroll
      for (int h = 0; h < HPW; ++h) mp[h] = h < H ? m2[h] : 0.f;
      wave_allmax<HPW>(mp, lane);
#pragma unroll
      for (int h = 0; h < H; ++h) mx[h] = mp[h];
      chunk(beg, min(64, end - beg));
    } else {
      float mp[HPW];
#pragma unroll
      for (int h = 0; h < HPW; ++h) mp[h] = h < H ? sc[h] : 0.f;
      wave_allmax<HPW>(mp, lane);
#pragma unroll
      for (int h = 0; h < H; ++h) mx[h] = mp[h];
    }
    for (int base = beg; base < end; base += 64) {
      const int cnt = min(64, end - base);
      if (base != beg) chunk(base, cnt);
      uint32_t ga[F][W], gb[F][W];
      auto issue = [&](uint32_t (&g)[F][W], int k) {
#pragma unroll
        for (int e = 0; e < F; ++e) {
          const int j = readlane_i(mj, min(k + e, cnt - 1));
          load_dw_row<W>(Hb + (int64_t)j * ldb, woff, g[e]);
        }
      };
      issue(ga, 0);  // depends on the neighbour ids only: out before the weights are known
      float em[H];
      if constexpr (EM) load_heads<H>(emask + (int64_t)(base + min(lane, cnt - 1)) * H, em);
      float wl[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float w = __expf(sc[h] - mx[h]);  // 0 past the chunk (sc = -inf there)
        den[h] += w;  // the row sum uses the un-dropped weights (att_layers.py:45-51)
        wl[h] = EM ? w * em[h] : w;
        shw[lane * H + h] = wl[h];  // lanes past the chunk: 0
      }
      // no early exits between a group's issue and its use: every edge of a group is consumed,
      // so the compiler's wait counts stay exact across the loop's back edge.  Edges past the
      // chunk have weight 0 (sc = -inf there) and re-read a live edge's finite row: their fma
      // adds +-0, no select needed
      auto consume = [&](const uint32_t (&g)[F][W], int k) {
        float we[F];
#pragma unroll
        for (int e = 0; e < F; ++e) we[e] = shw[min(k + e, 63) * H + hme];
#pragma unroll
        for (int e = 0; e < F; ++e) {
          float x[EPL];
          WN::unpack(g[e], wsh, x);
#pragma unroll
          for (int t = 0; t < EPL; ++t) acc[t] = fmaf(we[e], x[t], acc[t]);
        }
      };
      // (sched_barrier: keep each group's loads ahead of the previous group's arithmetic)
      for (int k = 0; k < cnt; k += 2 * F) {
        issue(gb, k + F);
        __builtin_amdgcn_sched_barrier(0);
        consume(ga, k);
        issue(ga, k + 2 * F);
        __builtin_amdgcn_sched_barrier(0);
        consume(gb, k + F);
      }
    }
  } else {
#pragma unroll
    for (int h = 0; h < H; ++h) mx[h] = -INFINITY;
  }
  float rinv[H];
  {
    float dp[HPW];  // every head's row sum in one all-reduce
#pragma unroll
    for (int h = 0; h < HPW; ++h) dp[h] = h < H ? den[h] : 0.f;
    wave_allsum<HPW>(dp, lane);
#pragma unroll
    for (int h = 0; h < H; ++h) {
      den[h] = dp[h];
      rinv[h] = den[h] > 0.f ? 1.f / den[h] : 0.f;
    }
  }
  const float ri = hsel<H>(rinv, hme);
  T* y = Y + (int64_t)row * ldy;
#pragma unroll
  for (int t = 0; t < EPL; ++t) {
    if (!hl.ok[t]) continue;
    const float v = acc[t] * ri;
    y[hl.c[t]] = from_f32<T>(act == GNNEA_ACT_RELU ? act_fwd<GNNEA_ACT_RELU>(v)
                             : act == GNNEA_ACT_ELU ? act_fwd<GNNEA_ACT_ELU>(v) : v);
  }
  const int Dp = (D + 3) & ~3;  // the row's padding columns hold zeros (k_gat_fwd's layout)
  if (lane < Dp - D) y[D + lane] = from_f32<T>(0.f);
  if (lane < H) {
    m_out[(int64_t)row * H + lane] = hsel<H>(mx, lane);
    den_out[(int64_t)row * H + lane] = hsel<H>(den, lane);
  }
}

// The source pass of the backward (k_gat_bwd_src's math) with G gathered as pipelined windows:
// F edges per group, two groups in flight; per group one grp_sum gives every edge's per-head
// G_i . H_j; dz = -(alpha (mask da - c_i)) LeakyReLU'(z) lands in the edge's lane.
template <int H, int EPL, typename T, bool EM, int F>
__global__ __launch_bounds__(256) void k_gat_bwd_src_hg(
    const int32_t* __restrict__ rowptrT, const int32_t* __restrict__ colT,
    const int64_t* __restrict__ permT, int n_rows, int dh, const T* __restrict__ Hm,
    int64_t ldh, const float* __restrict__ s2, float alpha, const float* __restrict__ emask,
    const float4* __restrict__ rec, const T* __restrict__ G, int64_t ldg,
    const float* __restrict__ a, T* __restrict__ dH, int64_t lddh, float* __restrict__ dzT,
    float* __restrict__ ds2) {
  constexpr int HPW = Pow2<H>::v;  // heads padded to a power of two (the all-reduces)
  using L = HeadLanes<H, EPL>;
  using WN = RowWin<T, EPL>;
  constexpr int W = WN::W;
  constexpr int LPH = L::LPH;
  // per wave: the chunk's edge weights [edge][head] (each lane then loads its head's weight of an
  // edge: one broadcast ds_read instead of H readlanes + selects) and the per-edge per-head
  // G_i . H_j sums, written by the lanes grp_sum leaves them in and read back by the edge's lane
  // once per chunk (instead of H readlanes + selects per edge)
  __shared__ float sh_w[4][64 * H];
  __shared__ float sh_d[4][64 * H];
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();  // source node j
  if (row >= n_rows) return;
  const int lane = lane_id();
  float* shw = sh_w[wave_id()];
  float* shd = sh_d[wave_id()];
  // the lane holding (edge e, head h) of a group's grp_sum: h * LPH + S e, S = 16 / F (8 / F)
  constexpr int GS = (LPH >= 16 ? 16 : 8) / F;
  const int gp = lane % LPH;
  const bool g_hold = gp < GS * F && gp % GS == 0 && lane / LPH < H;
  const int g_slot = (gp / GS) * H + lane / LPH;  // + k * H
  const int beg = rowptrT[row], end = rowptrT[row + 1];
  const L hl(lane, dh);
  const int hme = hl.h < H ? hl.h : 0;
  const uint32_t woff = (uint32_t)WN::byte_off(hl.c[0]);  // (load_dw_row's lane offset)
  const uint32_t wsh = (hl.c[0] & 1) ? 2u : 0u;
  const char* Gb = (const char*)G;
  const int64_t ldb = ldg * (int64_t)sizeof(T);

  float hj[EPL], acc[EPL], a2l[EPL];
  {
    const T* x = Hm + (int64_t)row * ldh;
#pragma unroll
    for (int t = 0; t < EPL; ++t) {
      const float v = to_f32<T>(x[hl.c[t]]);
      hj[t] = hl.ok[t] ? v : 0.f;
      acc[t] = 0.f;
      // the epilogue's a_2 terms, read now: read there, each was a serial L2 round trip between
      // the row's last edge and its stores
      a2l[t] = hl.ok[t] ? a[hme * 2 * dh + dh + hl.d0 + t] : 0.f;
    }
  }
  float ds2p[H];
#pragma unroll
  for (int h = 0; h < H; ++h) ds2p[h] = 0.f;

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int el = base + min(lane, cnt - 1);
    const int mi = colT[el];  // destination row i of the forward edge (i, j)
    uint32_t ga[F][W], gb[F][W];
    auto issue = [&](uint32_t (&g)[F][W], int k) {
#pragma unroll
      for (int e = 0; e < F; ++e) {
        const int r = readlane_i(mi, min(k + e, cnt - 1));
        load_dw_row<W>(Gb + (int64_t)r * ldb, woff, g[e]);
      }
    };
    issue(ga, 0);  // depends on the neighbour ids only
    float4 rr[H];
#pragma unroll
    for (int h = 0; h < H; ++h) rr[h] = rec[(int64_t)mi * H + h];  // {s1_i, m_i, 1/den_i, c_i}
    float ml[H];
    if constexpr (EM) load_heads<H>(emask + permT[el] * H, ml);
    float al[H], cl[H], sl[H], wl[H], dzl[H];
    const float msk = lane < cnt ? 1.f : 0.f;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float z = rr[h].x + s2[(int64_t)row * H + h];
      // lanes past the chunk hold a valid edge's record: scaled to 0 (a select on the loaded
      // values would let the compiler sink their loads into a branch)
      al[h] = __expf(-lrelu(z, alpha) - rr[h].y) * rr[h].z * msk;
      cl[h] = rr[h].w;
      sl[h] = z > 0.f ? 1.f : alpha;
      if constexpr (!EM) ml[h] = 1.f;
      wl[h] = EM ? al[h] * ml[h] : al[h];
      shw[lane * H + h] = wl[h];  // lanes past the chunk: 0
    }
    auto consume = [&](const uint32_t (&g)[F][W], int k) {
      float pd[F], we[F];
#pragma unroll
      for (int e = 0; e < F; ++e) we[e] = shw[min(k + e, 63) * H + hme];
      // edges past the chunk: weight 0 (shw), a live edge's finite row re-read, so their fma
      // adds +-0; elements past the head (hl.ok false) meet hj = 0 in the dot product and are
      // never stored from acc -- no selects
#pragma unroll
      for (int e = 0; e < F; ++e) {
        float x[EPL];
        WN::unpack(g[e], wsh, x);
        float q = 0.f;
#pragma unroll
        for (int t = 0; t < EPL; ++t) {
          acc[t] = fmaf(we[e], x[t], acc[t]);
          q = fmaf(x[t], hj[t], q);
        }
        pd[e] = q;
      }
      const float v = grp_sum<F, LPH>(pd, lane);
      // slots past the chunk (k + e >= cnt, still < 64) take sums that are never read
      if (g_hold) shd[k * H + g_slot] = v;
    };
    for (int k = 0; k < cnt; k += 2 * F) {
      issue(gb, k + F);
      __builtin_amdgcn_sched_barrier(0);
      consume(ga, k);
      issue(ga, k + 2 * F);
      __builtin_amdgcn_sched_barrier(0);
      consume(gb, k + F);
    }
#pragma unroll
    for (int h = 0; h < H; ++h) {  // the edge's lane: dz = -(alpha (mask da - c_i)) LReLU'(z)
      const float da = shd[lane * H + h];
      dzl[h] = -(al[h] * (ml[h] * da - cl[h])) * sl[h];
    }
    if (lane < cnt) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        dzT[(int64_t)(base + lane) * H + h] = dzl[h];
        ds2p[h] += dzl[h];
      }
    }
  }
  float d2me = 0.f;
  float dp[HPW];  // every head's sum in one all-reduce
#pragma unroll
  for (int h = 0; h < HPW; ++h) dp[h] = h < H ? ds2p[h] : 0.f;
  wave_allsum<HPW>(dp, lane);
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float d2 = dp[h];
    d2me = hme == h ? d2 : d2me;
    if (lane == 0) ds2[(int64_t)row * H + h] = d2;
  }
  T* out = dH + (int64_t)row * lddh;
#pragma unroll
  for (int t = 0; t < EPL; ++t)
    if (hl.ok[t]) out[hl.c[t]] = from_f32<T>(acc[t] + d2me * a2l[t]);
}


// every lane's window ends inside the row's ld (elements, T-sized) for this head layout
template <typename T, int EPL>
static bool hg_window_fits(int heads, int dh, int64_t ld) {
  const int hp = heads <= 1 ? 1 : heads <= 2 ? 2 : heads <= 4 ? 4 : 8, lph = 64 / hp;
  for (int h = 0; h < heads; ++h)
    for (int s = 0; s < lph; ++s) {
      const int d0 = s * EPL;
      if (d0 >= dh) continue;  // an idle lane reads the row's start
      const int c = h * dh + d0;
      if (RowWin<T, EPL>::byte_off(c) + 4 * RowWin<T, EPL>::W > ld * (int64_t)sizeof(T))
        return false;
    }
  return true;
}

}  // namespace gnnea

using namespace gnnea;

// heads x NCH dispatch: heads in {1,2,4,8} (+3,6 for completeness), NCH in 1..4 (D <= 1024)
#define GNNEA_GAT_DISPATCH(CALL)                                   \
  do {                                                             \
    const int nch = (D4 + 63) / 64;                                \
    if (nch < 1 || nch > 4) return GNNEA_EINVAL;                   \
    switch (heads * 8 + nch) {                                     \
      CALL(1, 1) CALL(1, 2) CALL(1, 3) CALL(1, 4)                  \
      CALL(2, 1) CALL(2, 2) CALL(2, 3) CALL(2, 4)                  \
      CALL(3, 1) CALL(3, 2) CALL(3, 3) CALL(3, 4)                  \
      CALL(4, 1) CALL(4, 2) CALL(4, 3) CALL(4, 4)                  \
      CALL(6, 1) CALL(6, 2) CALL(6, 3) CALL(6, 4)                  \
      CALL(8, 1) CALL(8, 2) CALL(8, 3) CALL(8, 4)                  \
      default: return GNNEA_EINVAL;                                \
    }                                                              \
  } while (0)

// heads x EPL dispatch of the head-grouped kernels: EPL = ceil(d_head / LPH) rounded up to one of
// {1,2,3,4,5,6,8,12,16} (d_head <= 16 * 64 / heads_pow2)
static int epl_of(int heads, int dh) {
  const int hp = heads <= 1 ? 1 : heads <= 2 ? 2 : heads <= 4 ? 4 : 8;
  const int e = (dh + 64 / hp - 1) / (64 / hp);
  static const int opts[] = {1, 2, 3, 4, 5, 6, 8, 12, 16};
  for (int o : opts)
    if (e <= o) return o;
  return -1;
}
#define GNNEA_GAT_HL_DISPATCH(CALL)                                        \
  do {                                                                     \
    const int epl = epl_of(heads, d_head);                                 \
    if (epl < 0 || heads > 8 || heads == 5 || heads == 7) return GNNEA_EINVAL; \
    switch (heads * 32 + epl) {                                            \
      CALL(1, 1) CALL(1, 2) CALL(1, 3) CALL(1, 4) CALL(1, 5) CALL(1, 6) CALL(1, 8) CALL(1, 12) CALL(1, 16) \
      CALL(2, 1) CALL(2, 2) CALL(2, 3) CALL(2, 4) CALL(2, 5) CALL(2, 6) CALL(2, 8) CALL(2, 12) CALL(2, 16) \
      CALL(3, 1) CALL(3, 2) CALL(3, 3) CALL(3, 4) CALL(3, 5) CALL(3, 6) CALL(3, 8) CALL(3, 12) CALL(3, 16) \
      CALL(4, 1) CALL(4, 2) CALL(4, 3) CALL(4, 4) CALL(4, 5) CALL(4, 6) CALL(4, 8) CALL(4, 12) CALL(4, 16) \
      CALL(6, 1) CALL(6, 2) CALL(6, 3) CALL(6, 4) CALL(6, 5) CALL(6, 6) CALL(6, 8) CALL(6, 12) CALL(6, 16) \
      CALL(8, 1) CALL(8, 2) CALL(8, 3) CALL(8, 4) CALL(8, 5) CALL(8, 6) CALL(8, 8) CALL(8, 12) CALL(8, 16) \
      default: return GNNEA_EINVAL;                                        \
    }                                                                      \
  } while (0)

template <typename T>
static bool alv(const void* p) {  // aligned for one Vec4<T> access (16 B fp32, 8 B bf16)
  return p == nullptr || (((uintptr_t)p) & (sizeof(typename Vec4<T>::raw) - 1)) == 0;
}

// ---- head-grouped pipelined passes: heads in {1,2,4,8}, EPL in {2,3,4,5,6,8} ----
static int hg_epl(int heads, int dh) {
  if (heads != 1 && heads != 2 && heads != 4 && heads != 8) return -1;
  const int e = (dh + 64 / heads - 1) / (64 / heads);
  static const int opts[] = {2, 3, 4, 5, 6, 8};
  for (int o : opts)
    if (e <= o) return o;
  return -1;
}
template <typename T>
static bool hg_applies(int heads, int dh, int64_t ld, const float* s2, const float* emask) {
  const int epl = hg_epl(heads, dh);
  bool fits = false;
  switch (epl) {
    case 2: fits = hg_window_fits<T, 2>(heads, dh, ld); break;
    case 3: fits = hg_window_fits<T, 3>(heads, dh, ld); break;
    case 4: fits = hg_window_fits<T, 4>(heads, dh, ld); break;
    case 5: fits = hg_window_fits<T, 5>(heads, dh, ld); break;
    case 6: fits = hg_window_fits<T, 6>(heads, dh, ld); break;
    case 8: fits = hg_window_fits<T, 8>(heads, dh, ld); break;
    default: return false;
  }
  // four heads: the per-edge logits / mask rows are read as one 16-B load
  return fits && (heads != 4 || ((((uintptr_t)s2) & 15) == 0 && (((uintptr_t)emask) & 15) == 0));
}
#define GNNEA_GAT_HG_DISPATCH(CALL)                                                          \
  switch (heads * 32 + hg_epl(heads, d_head)) {                                              \
    CALL(1, 2) CALL(1, 3) CALL(1, 4) CALL(1, 5) CALL(1, 6) CALL(1, 8)                        \
    CALL(2, 2) CALL(2, 3) CALL(2, 4) CALL(2, 5) CALL(2, 6) CALL(2, 8)                        \
    CALL(4, 2) CALL(4, 3) CALL(4, 4) CALL(4, 5) CALL(4, 6) CALL(4, 8)                        \
    CALL(8, 2) CALL(8, 3) CALL(8, 4) CALL(8, 5) CALL(8, 6) CALL(8, 8)                        \
    default: return GNNEA_EINVAL;                                                            \
  }

template <typename T>
static int gat_scores_t(const T* Hm, int64_t ldh, int32_t n_rows, int heads, int d_head,
                        const float* a, float* s1, float* s2, hipStream_t s) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head;
  if (!Hm || !a || !s1 || !s2) return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !alv<T>(Hm)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4) < 2048 ? div_up(n_rows, 4) : 2048;  // waves walk rows
#define CALL(HH, EE)                                                                          \
  case HH * 32 + EE:                                                                          \
    hipLaunchKernelGGL((k_gat_scores<HH, EE, T>), dim3(nb), dim3(256), 0, s, Hm, ldh, n_rows, \
                       d_head, a, s1, s2);                                                    \
    break;
  GNNEA_GAT_HL_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int gat_fwd_t(const int32_t* rowptr, const int32_t* col, int32_t n_rows, const T* Hm,
                     int64_t ldh, int heads, int d_head, const float* s1, const float* s2,
                     float alpha, const float* edge_mask, int act, T* Y, int64_t ldy,
                     float* m_out, float* den_out, hipStream_t s) {
  typedef typename Vec4<T>::raw R;
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!rowptr || !col || !Hm || !s1 || !s2 || !Y || !m_out || !den_out) return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !ok_ld(ldy, D) || !alv<T>(Hm) || !alv<T>(Y)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  if (hg_applies<T>(heads, d_head, ldh, s2, edge_mask) &&
      (act == GNNEA_ACT_IDENTITY || act == GNNEA_ACT_RELU || act == GNNEA_ACT_ELU)) {
#define GNNEA_HG_L(HH, EE, EMV, FF)                                                           \
  hipLaunchKernelGGL((k_gat_fwd_hg<HH, EE, T, EMV, FF>), dim3(nb), dim3(256), 0, s, rowptr,   \
                     col, n_rows, Hm, ldh, D, d_head, s1, s2, alpha, edge_mask, act, Y, ldy,  \
                     m_out, den_out)
#define CALL(HH, EE)                                                                          \
  case HH * 32 + EE:                                                                          \
    if (edge_mask) GNNEA_HG_L(HH, EE, true, 4);                                               \
    else GNNEA_HG_L(HH, EE, false, 4);                                                        \
    break;
    GNNEA_GAT_HG_DISPATCH(CALL);
#undef CALL
#undef GNNEA_HG_L
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
#define CALL_A(A, HH, NN)                                                                       \
  hipLaunchKernelGGL((k_gat_fwd<A, HH, NN, T>), dim3(nb), dim3(256), 0, s, rowptr, col, n_rows, \
                     (const R*)Hm, ldh / 4, D, d_head, s1, s2, alpha, edge_mask, (R*)Y,         \
                     ldy / 4, m_out, den_out)
#define CALL(HH, NN)                                                   \
  case HH * 8 + NN:                                                    \
    switch (act) {                                                     \
      case GNNEA_ACT_IDENTITY: CALL_A(GNNEA_ACT_IDENTITY, HH, NN); break; \
      case GNNEA_ACT_RELU: CALL_A(GNNEA_ACT_RELU, HH, NN); break;         \
      case GNNEA_ACT_ELU: CALL_A(GNNEA_ACT_ELU, HH, NN); break;           \
      default: return GNNEA_EINVAL;                                    \
    }                                                                  \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
#undef CALL_A
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int gat_bwd_prep_t(int32_t n_rows, int heads, int d_head, const T* dY, const T* Y,
                          int64_t ld, const float* s1, const float* m, const float* den, int act,
                          T* G, float* rec, hipStream_t s) {
  typedef typename Vec4<T>::raw R;
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!dY || !Y || !s1 || !m || !den || !G || !rec) return GNNEA_EINVAL;
  if (!ok_ld(ld, D) || !alv<T>(dY) || !alv<T>(Y) || !alv<T>(G) || !alv<float>(rec))
    return GNNEA_EALIGN;
  if (act != GNNEA_ACT_IDENTITY && act != GNNEA_ACT_RELU) return GNNEA_EINVAL;
  const int nb = div_up(n_rows, 16);
#define CALL_A(A, HH, NN)                                                                      \
  hipLaunchKernelGGL((k_gat_bwd_prep4<A, HH, NN, T>), dim3(nb), dim3(256), 0, s, n_rows, D,   \
                     d_head, (const R*)dY, (const R*)Y, ld / 4, s1, m, den, (R*)G, (float4*)rec)
#define CALL(HH, NN)                                                        \
  case HH * 8 + NN:                                                         \
    if (act == GNNEA_ACT_RELU) CALL_A(GNNEA_ACT_RELU, HH, NN);              \
    else CALL_A(GNNEA_ACT_IDENTITY, HH, NN);                                \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
#undef CALL_A
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int gat_bwd_src_t(const int32_t* rowptrT, const int32_t* colT, const int64_t* permT,
                         int32_t n_rows, int heads, int d_head, const T* H, int64_t ldh,
                         const float* s2, float alpha, const float* edge_mask, const float* rec,
                         const T* G, int64_t ldg, const float* a, T* dH, int64_t lddh,
                         float* dzT, float* ds2, hipStream_t s, int64_t g_rows = 0) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head;
  if (!rowptrT || !colT || !permT || !H || !s2 || !rec || !G || !a || !dH || !dzT || !ds2)
    return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !ok_ld(ldg, D) || !ok_ld(lddh, D) || !alv<T>(H) || !alv<T>(G) ||
      !alv<T>(dH) || !alv<float>(rec))
    return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  if (hg_applies<T>(heads, d_head, ldg, s2, edge_mask) && (((uintptr_t)rec) & 15) == 0) {
#define GNNEA_HG_L(HH, EE, EMV, FF)                                                           \
  hipLaunchKernelGGL((k_gat_bwd_src_hg<HH, EE, T, EMV, FF>), dim3(nb), dim3(256), 0, s,       \
                     rowptrT, colT, permT, n_rows, d_head, H, ldh, s2, alpha, edge_mask,      \
                     (const float4*)rec, G, ldg, a, dH, lddh, dzT, ds2)
#define CALL(HH, EE)                                                                          \
  case HH * 32 + EE:                                                                          \
    if (edge_mask) GNNEA_HG_L(HH, EE, true, 1);                                               \
    else GNNEA_HG_L(HH, EE, false, 1);                                                        \
    break;
    // (one edge per gather group, F = 1: the source pass's per-group reduce-scatter then runs
    // per edge; cfg-5 6.32 -> 6.11 ms per launch against F = 4, F = 2 6.18)
    GNNEA_GAT_HG_DISPATCH(CALL);
#undef CALL
#undef GNNEA_HG_L
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
  // the window path: bf16 rows with 4-B aligned starts (the runs of EPL <= 6 elements fit 16 B)
  const bool win = std::is_same<T, bf16_t>::value && g_rows > 1 && ldg % 2 == 0 &&
                   (((uintptr_t)G) & 3) == 0;
#define CALL(HH, EE)                                                                          \
  case HH * 32 + EE:                                                                          \
    if (EE <= 6 && win)                                                                       \
      hipLaunchKernelGGL((k_gat_bwd_src<HH, EE, T, (EE <= 6 && std::is_same<T, bf16_t>::value)>), \
                         dim3(nb), dim3(256), 0, s,                                           \
                         rowptrT, colT, permT, n_rows, d_head, H, ldh, s2, alpha, edge_mask,  \
                         (const float4*)rec, G, ldg, a, dH, lddh, dzT, ds2, g_rows);          \
    else                                                                                      \
      hipLaunchKernelGGL((k_gat_bwd_src<HH, EE, T>), dim3(nb), dim3(256), 0, s, rowptrT,      \
                         colT, permT, n_rows, d_head, H, ldh, s2, alpha, edge_mask,           \
                         (const float4*)rec, G, ldg, a, dH, lddh, dzT, ds2, (int64_t)0);      \
    break;
  GNNEA_GAT_HL_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int gat_bwd_dst_t(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows, int heads,
                         int d_head, const float* dzT, const float* a, T* dH, int64_t lddh,
                         float* ds1, hipStream_t s) {
  typedef typename Vec4<T>::raw R;
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!rowptr || !tpos || !dzT || !a || !dH || !ds1) return GNNEA_EINVAL;
  if (!ok_ld(lddh, D) || !alv<T>(dH)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 16);
#define CALL(HH, NN)                                                                          \
  case HH * 8 + NN:                                                                           \
    hipLaunchKernelGGL((k_gat_bwd_dst4<HH, NN, T>), dim3(nb), dim3(256), 0, s, rowptr, tpos,  \
                       n_rows, D, d_head, dzT, a, (R*)dH, lddh / 4, ds1);                     \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// ---- C-ABI: fp32 and bf16 feature storage (H, Y, dY, G, dH); logits, records, dz stay fp32 --

extern "C" int gnnea_gat_scores_f32(const float* Hm, int64_t ldh, int32_t n_rows, int heads,
                                    int d_head, const float* a, float* s1, float* s2,
                                    void* stream) {
  return gat_scores_t<float>(Hm, ldh, n_rows, heads, d_head, a, s1, s2, (hipStream_t)stream);
}

extern "C" int gnnea_gat_fwd_f32(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                                 const float* Hm, int64_t ldh, int heads, int d_head,
                                 const float* s1, const float* s2, float alpha,
                                 const float* edge_mask, int act, float* Y, int64_t ldy,
                                 float* m_out, float* den_out, void* stream) {
  return gat_fwd_t<float>(rowptr, col, n_rows, Hm, ldh, heads, d_head, s1, s2, alpha, edge_mask,
                          act, Y, ldy, m_out, den_out, (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_prep_f32(int32_t n_rows, int heads, int d_head, const float* dY,
                                      const float* Y, int64_t ld, const float* s1,
                                      const float* m, const float* den, int act, float* G,
                                      float* rec, void* stream) {
  return gat_bwd_prep_t<float>(n_rows, heads, d_head, dY, Y, ld, s1, m, den, act, G, rec,
                               (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_src_f32(const int32_t* rowptrT, const int32_t* colT,
                                     const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                     const float* H, int64_t ldh, const float* s2, float alpha,
                                     const float* edge_mask, const float* rec, const float* G,
                                     int64_t ldg, const float* a, float* dH, int64_t lddh,
                                     float* dzT, float* ds2, void* stream) {
  return gat_bwd_src_t<float>(rowptrT, colT, permT, n_rows, heads, d_head, H, ldh, s2, alpha,
                              edge_mask, rec, G, ldg, a, dH, lddh, dzT, ds2,
                              (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_dst_f32(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows,
                                     int heads, int d_head, const float* dzT, const float* a,
                                     float* dH, int64_t lddh, float* ds1, void* stream) {
  return gat_bwd_dst_t<float>(rowptr, tpos, n_rows, heads, d_head, dzT, a, dH, lddh, ds1,
                              (hipStream_t)stream);
}

extern "C" int gnnea_gat_scores_bf16(const void* Hm, int64_t ldh, int32_t n_rows, int heads,
                                     int d_head, const float* a, float* s1, float* s2,
                                     void* stream) {
  return gat_scores_t<bf16_t>((const bf16_t*)Hm, ldh, n_rows, heads, d_head, a, s1, s2,
                              (hipStream_t)stream);
}

extern "C" int gnnea_gat_fwd_bf16(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                                  const void* Hm, int64_t ldh, int heads, int d_head,
                                  const float* s1, const float* s2, float alpha,
                                  const float* edge_mask, int act, void* Y, int64_t ldy,
                                  float* m_out, float* den_out, void* stream) {
  return gat_fwd_t<bf16_t>(rowptr, col, n_rows, (const bf16_t*)Hm, ldh, heads, d_head, s1, s2,
                           alpha, edge_mask, act, (bf16_t*)Y, ldy, m_out, den_out,
                           (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_prep_bf16(int32_t n_rows, int heads, int d_head, const void* dY,
                                       const void* Y, int64_t ld, const float* s1,
                                       const float* m, const float* den, int act, void* G,
                                       float* rec, void* stream) {
  return gat_bwd_prep_t<bf16_t>(n_rows, heads, d_head, (const bf16_t*)dY, (const bf16_t*)Y, ld,
                                s1, m, den, act, (bf16_t*)G, rec, (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_src_bf16(const int32_t* rowptrT, const int32_t* colT,
                                      const int64_t* permT, int32_t n_rows, int heads,
                                      int d_head, const void* H, int64_t ldh, const float* s2,
                                      float alpha, const float* edge_mask, const float* rec,
                                      const void* G, int64_t ldg, const float* a, void* dH,
                                      int64_t lddh, float* dzT, float* ds2, void* stream) {
  return gat_bwd_src_t<bf16_t>(rowptrT, colT, permT, n_rows, heads, d_head, (const bf16_t*)H,
                               ldh, s2, alpha, edge_mask, rec, (const bf16_t*)G, ldg, a,
                               (bf16_t*)dH, lddh, dzT, ds2, (hipStream_t)stream);
}

extern "C" int gnnea_gat_bwd_src_rows_bf16(const int32_t* rowptrT, const int32_t* colT,
                                           const int64_t* permT, int32_t n_rows, int heads,
                                           int d_head, const void* H, int64_t ldh,
                                           const float* s2, float alpha, const float* edge_mask,
                                           const float* rec, const void* G, int64_t ldg,
                                           int64_t g_rows, const float* a, void* dH,
                                           int64_t lddh, float* dzT, float* ds2, void* stream) {
  if (g_rows < 0) return GNNEA_EINVAL;
  return gat_bwd_src_t<bf16_t>(rowptrT, colT, permT, n_rows, heads, d_head, (const bf16_t*)H,
                               ldh, s2, alpha, edge_mask, rec, (const bf16_t*)G, ldg, a,
                               (bf16_t*)dH, lddh, dzT, ds2, (hipStream_t)stream, g_rows);
}

extern "C" int gnnea_gat_bwd_dst_bf16(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows,
                                      int heads, int d_head, const float* dzT, const float* a,
                                      void* dH, int64_t lddh, float* ds1, void* stream) {
  return gat_bwd_dst_t<bf16_t>(rowptr, tpos, n_rows, heads, d_head, dzT, a, (bf16_t*)dH, lddh,
                               ds1, (hipStream_t)stream);
}
