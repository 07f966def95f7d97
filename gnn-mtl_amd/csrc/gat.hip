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

template <int H>
__device__ __forceinline__ float hsel(const float (&w)[H], int h) {
  float r = w[0];
#pragma unroll
  for (int k = 1; k < H; ++k) r = (h == k) ? w[k] : r;
  return r;
}

__device__ __forceinline__ float lrelu(float z, float alpha) { return z > 0.f ? z : alpha * z; }

// s1[i,h] = sum_d H[i, h*dh+d] * a[h, d];  s2[i,h] = sum_d H[i, h*dh+d] * a[h, dh+d]
template <int H, int NCH>
__global__ __launch_bounds__(256) void k_gat_scores(const float4* __restrict__ Hm, int64_t ldh4,
                                                    int n_rows, int D, int dh,
                                                    const float* __restrict__ a,
                                                    float* __restrict__ s1,
                                                    float* __restrict__ s2) {
  const int row = blockIdx.x * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  float p1[H], p2[H];
#pragma unroll
  for (int h = 0; h < H; ++h) p1[h] = p2[h] = 0.f;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    if (4 * c4 >= D) continue;
    const float4 x = Hm[(int64_t)row * ldh4 + c4];
    const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      if (c >= D) continue;
      const int h = c / dh, d = c - h * dh;
      const float v1 = xs[t] * a[h * 2 * dh + d];
      const float v2 = xs[t] * a[h * 2 * dh + dh + d];
#pragma unroll
      for (int k = 0; k < H; ++k) {
        p1[k] += (h == k) ? v1 : 0.f;
        p2[k] += (h == k) ? v2 : 0.f;
      }
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float r1 = wave_sum(p1[h]), r2 = wave_sum(p2[h]);
    if (lane == 0) {
      s1[(int64_t)row * H + h] = r1;
      s2[(int64_t)row * H + h] = r2;
    }
  }
}

template <int ACT, int H, int NCH>
__global__ __launch_bounds__(256) void k_gat_fwd(const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col, int n_rows,
                                                 const float4* __restrict__ Hm, int64_t ldh4,
                                                 int D, int dh, const float* __restrict__ s1,
                                                 const float* __restrict__ s2, float alpha,
                                                 const float* __restrict__ emask,
                                                 float4* __restrict__ Y, int64_t ldy4,
                                                 float* __restrict__ m_out,
                                                 float* __restrict__ den_out) {
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
    int k = 0;
    for (; k + 2 <= cnt; k += 2) {
      const int j0 = readlane_i(mj, k), j1 = readlane_i(mj, k + 1);
      float w0[H], w1[H];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        w0[h] = readlane_f(wl[h], k);
        w1[h] = readlane_f(wl[h], k + 1);
      }
      const float4* x0 = Hm + (int64_t)j0 * ldh4 + lane;
      const float4* x1 = Hm + (int64_t)j1 * ldh4 + lane;
      float4 r0[NCH], r1[NCH];
#pragma unroll
      for (int q = 0; q < NCH; ++q)
        if (own[q]) {
          r0[q] = x0[64 * q];
          r1[q] = x1[64 * q];
        }
#pragma unroll
      for (int q = 0; q < NCH; ++q)
        if (own[q]) {
          acc[q].x = fmaf(hsel<H>(w0, hd[q][0]), r0[q].x, acc[q].x);
          acc[q].y = fmaf(hsel<H>(w0, hd[q][1]), r0[q].y, acc[q].y);
          acc[q].z = fmaf(hsel<H>(w0, hd[q][2]), r0[q].z, acc[q].z);
          acc[q].w = fmaf(hsel<H>(w0, hd[q][3]), r0[q].w, acc[q].w);
          acc[q].x = fmaf(hsel<H>(w1, hd[q][0]), r1[q].x, acc[q].x);
          acc[q].y = fmaf(hsel<H>(w1, hd[q][1]), r1[q].y, acc[q].y);
          acc[q].z = fmaf(hsel<H>(w1, hd[q][2]), r1[q].z, acc[q].z);
          acc[q].w = fmaf(hsel<H>(w1, hd[q][3]), r1[q].w, acc[q].w);
        }
    }
    for (; k < cnt; ++k) {
      const int j0 = readlane_i(mj, k);
      float w0[H];
#pragma unroll
      for (int h = 0; h < H; ++h) w0[h] = readlane_f(wl[h], k);
      const float4* x0 = Hm + (int64_t)j0 * ldh4 + lane;
#pragma unroll
      for (int q = 0; q < NCH; ++q)
        if (own[q]) {
          const float4 r = x0[64 * q];
          acc[q].x = fmaf(hsel<H>(w0, hd[q][0]), r.x, acc[q].x);
          acc[q].y = fmaf(hsel<H>(w0, hd[q][1]), r.y, acc[q].y);
          acc[q].z = fmaf(hsel<H>(w0, hd[q][2]), r.z, acc[q].z);
          acc[q].w = fmaf(hsel<H>(w0, hd[q][3]), r.w, acc[q].w);
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
    Y[(int64_t)row * ldy4 + lane + 64 * q] = o;
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

// Sum of p[h] over the 64 lanes for every head at once, by reduce-scatter: stage s halves the
// number of live values per lane by exchanging across lane bit (5 - s); afterwards each lane
// holds the full sum for one head, hp_of_lane(lane).  HP (power of two) shuffles+log2 instead
// of 6*HP.  Returns the value; head_lane(h) gives a lane holding head h.
template <int HP>
__device__ __forceinline__ float rs_sum(float (&p)[HP], int lane) {
  int cnt = HP, bit = 32;
#pragma unroll
  for (int st = 0; st < 6; ++st) {
    if (cnt > 1) {
      const bool up = lane & bit;
      const int half = cnt / 2;
#pragma unroll
      for (int t = 0; t < HP / 2; ++t) {
        if (t < half) {
          const float keep = up ? p[t + half] : p[t];
          const float send = up ? p[t] : p[t + half];
          p[t] = keep + __shfl_xor(send, bit, 64);
        }
      }
      cnt = half;
    } else {
      p[0] += __shfl_xor(p[0], bit, 64);
    }
    bit >>= 1;
  }
  return p[0];
}
template <int HP>
__device__ __forceinline__ int head_lane(int h) {
  // stage s keeps the upper half on lanes with bit (5 - s) set
  int lane = 0, cnt = HP, bit = 32;
  while (cnt > 1) {
    const int half = cnt / 2;
    if (h >= half) { lane |= bit; h -= half; }
    cnt = half;
    bit >>= 1;
  }
  return lane;
}
template <int H> struct Pow2 { static constexpr int v = H <= 1 ? 1 : H <= 2 ? 2 : H <= 4 ? 4 : 8; };

template <int ACT, int H, int NCH>
__global__ __launch_bounds__(256) void k_gat_bwd_prep(int n_rows, int D, int dh,
                                                      const float4* __restrict__ dY,
                                                      const float4* __restrict__ Y, int64_t ld4,
                                                      const float* __restrict__ s1,
                                                      const float* __restrict__ mrow,
                                                      const float* __restrict__ den,
                                                      float4* __restrict__ G,
                                                      float4* __restrict__ rec) {
  const int row = blockIdx.x * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  float cp[H];
#pragma unroll
  for (int h = 0; h < H; ++h) cp[h] = 0.f;
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    if (4 * c4 >= D) continue;
    const float4 dy = dY[(int64_t)row * ld4 + c4], y = Y[(int64_t)row * ld4 + c4];
    const float ys[4] = {y.x, y.y, y.z, y.w};
    float gs[4] = {dy.x, dy.y, dy.z, dy.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      gs[t] = c < D ? gs[t] * act_grad_from_out<ACT>(ys[t]) : 0.f;
      const int hh = c < D ? c / dh : H;
      // P = h' (pre-activation); for relu / identity G * Y == G * h' element-wise
#pragma unroll
      for (int h = 0; h < H; ++h) cp[h] += (hh == h) ? gs[t] * ys[t] : 0.f;
    }
    G[(int64_t)row * ld4 + c4] = make_float4(gs[0], gs[1], gs[2], gs[3]);
  }
#pragma unroll
  for (int h = 0; h < H; ++h) cp[h] = wave_sum(cp[h]);
  if (lane < H) {
    const int64_t o = (int64_t)row * H + lane;
    const float dv = den[o];
    rec[o] = make_float4(s1[o], mrow[o], dv > 0.f ? 1.f / dv : 0.f, hsel<H>(cp, lane));
  }
}

template <int H, int NCH>
__global__ __launch_bounds__(256) void k_gat_bwd_src(
    const int32_t* __restrict__ rowptrT, const int32_t* __restrict__ colT,
    const int64_t* __restrict__ permT, int n_rows, int D, int dh, const float4* __restrict__ Hm,
    int64_t ldh4, const float* __restrict__ s2, float alpha, const float* __restrict__ emask,
    const float4* __restrict__ rec, const float4* __restrict__ G, int64_t ldg4,
    const float* __restrict__ a, float4* __restrict__ dH, int64_t lddh4, float* __restrict__ dzT,
    float* __restrict__ ds2) {
  constexpr int HP = Pow2<H>::v;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();  // source node j
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptrT[row], end = rowptrT[row + 1];

  int hd[NCH][4];
  bool own[NCH];
  float4 hj[NCH], acc[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    own[q] = 4 * c4 < D;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      hd[q][t] = c < D ? c / dh : H;
    }
    hj[q] = own[q] ? Hm[(int64_t)row * ldh4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float sj[H], ds2p[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    sj[h] = s2[(int64_t)row * H + h];
    ds2p[h] = 0.f;
  }

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int mi = 0;
    float al[H], zl[H], ml[H], cl[H], wl[H], dzl[H];
#pragma unroll
    for (int h = 0; h < H; ++h) al[h] = zl[h] = cl[h] = wl[h] = dzl[h] = 0.f, ml[h] = 1.f;
    if (lane < cnt) {
      mi = colT[base + lane];  // destination row i of the forward edge (i, j)
      const int64_t e = permT[base + lane];
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const float4 r = rec[(int64_t)mi * H + h];  // {s1_i, m_i, 1/den_i, c_i}
        const float z = r.x + sj[h];
        zl[h] = z;
        al[h] = __expf(-lrelu(z, alpha) - r.y) * r.z;
        cl[h] = r.w;
        ml[h] = emask ? emask[e * H + h] : 1.f;
        wl[h] = al[h] * ml[h];
      }
    }
    for (int k = 0; k < cnt; ++k) {
      const int i = readlane_i(mi, k);
      float w[H];
#pragma unroll
      for (int h = 0; h < H; ++h) w[h] = readlane_f(wl[h], k);
      const float4* gr = G + (int64_t)i * ldg4 + lane;
      float pd[HP];
#pragma unroll
      for (int h = 0; h < HP; ++h) pd[h] = 0.f;
#pragma unroll
      for (int q = 0; q < NCH; ++q)
        if (own[q]) {
          const float4 g = gr[64 * q];
          const float gs[4] = {g.x, g.y, g.z, g.w};
          const float hs[4] = {hj[q].x, hj[q].y, hj[q].z, hj[q].w};
          float o[4] = {acc[q].x, acc[q].y, acc[q].z, acc[q].w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            o[t] = fmaf(hsel<H>(w, hd[q][t]), gs[t], o[t]);
            const float gh = gs[t] * hs[t];
#pragma unroll
            for (int h = 0; h < H; ++h) pd[h] += (hd[q][t] == h) ? gh : 0.f;
          }
          acc[q] = make_float4(o[0], o[1], o[2], o[3]);
        }
      const float v = rs_sum<HP>(pd, lane);
      float da[H];
#pragma unroll
      for (int h = 0; h < H; ++h) da[h] = readlane_f(v, head_lane<HP>(h));
      if (lane == k) {
#pragma unroll
        for (int h = 0; h < H; ++h)
          dzl[h] = -(al[h] * (ml[h] * da[h] - cl[h])) * (zl[h] > 0.f ? 1.f : alpha);
      }
    }
    if (lane < cnt) {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        dzT[(int64_t)(base + lane) * H + h] = dzl[h];
        ds2p[h] += dzl[h];
      }
    }
  }
  float d2[H];
#pragma unroll
  for (int h = 0; h < H; ++h) d2[h] = wave_sum(ds2p[h]);
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    if (!own[q]) continue;
    float o[4] = {acc[q].x, acc[q].y, acc[q].z, acc[q].w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * (lane + 64 * q) + t;
      const int h = hd[q][t];
      o[t] = h < H ? o[t] + hsel<H>(d2, h) * a[h * 2 * dh + dh + (c - h * dh)] : 0.f;
    }
    dH[(int64_t)row * lddh4 + lane + 64 * q] = make_float4(o[0], o[1], o[2], o[3]);
  }
  if (lane < H) ds2[(int64_t)row * H + lane] = hsel<H>(d2, lane);
}

template <int H, int NCH>
__global__ __launch_bounds__(256) void k_gat_bwd_dst(const int32_t* __restrict__ rowptr,
                                                     const int64_t* __restrict__ tpos, int n_rows,
                                                     int D, int dh, const float* __restrict__ dzT,
                                                     const float* __restrict__ a,
                                                     float4* __restrict__ dH, int64_t lddh4,
                                                     float* __restrict__ ds1) {
  const int row = blockIdx.x * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptr[row], end = rowptr[row + 1];
  float p[H];
#pragma unroll
  for (int h = 0; h < H; ++h) p[h] = 0.f;
  for (int e = beg + lane; e < end; e += 64) {
    const int64_t t = tpos[e];
#pragma unroll
    for (int h = 0; h < H; ++h) p[h] += dzT[t * H + h];
  }
#pragma unroll
  for (int h = 0; h < H; ++h) p[h] = wave_sum(p[h]);
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    const int c4 = lane + 64 * q;
    if (4 * c4 >= D) continue;
    float4 v = dH[(int64_t)row * lddh4 + c4];
    float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = 4 * c4 + t;
      if (c < D) {
        const int h = c / dh;
        o[t] += hsel<H>(p, h) * a[h * 2 * dh + (c - h * dh)];
      }
    }
    dH[(int64_t)row * lddh4 + c4] = make_float4(o[0], o[1], o[2], o[3]);
  }
  if (lane < H) ds1[(int64_t)row * H + lane] = hsel<H>(p, lane);
}

static bool ok_ld(int64_t ld, int D) { return ld % 4 == 0 && ld >= ((D + 3) / 4) * 4; }
static bool al16(const void* p) { return p == nullptr || (((uintptr_t)p) & 15) == 0; }

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

extern "C" int gnnea_gat_scores_f32(const float* Hm, int64_t ldh, int32_t n_rows, int heads,
                                    int d_head, const float* a, float* s1, float* s2,
                                    void* stream) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!Hm || !a || !s1 || !s2) return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !al16(Hm)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  hipStream_t s = (hipStream_t)stream;
#define CALL(HH, NN)                                                                         \
  case HH * 8 + NN:                                                                          \
    hipLaunchKernelGGL((k_gat_scores<HH, NN>), dim3(nb), dim3(256), 0, s, (const float4*)Hm, \
                       ldh / 4, n_rows, D, d_head, a, s1, s2);                               \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_gat_fwd_f32(const int32_t* rowptr, const int32_t* col, int32_t n_rows,
                                 const float* Hm, int64_t ldh, int heads, int d_head,
                                 const float* s1, const float* s2, float alpha,
                                 const float* edge_mask, int act, float* Y, int64_t ldy,
                                 float* m_out, float* den_out, void* stream) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!rowptr || !col || !Hm || !s1 || !s2 || !Y || !m_out || !den_out) return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !ok_ld(ldy, D) || !al16(Hm) || !al16(Y)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  hipStream_t s = (hipStream_t)stream;
#define CALL_A(A, HH, NN)                                                                     \
  hipLaunchKernelGGL((k_gat_fwd<A, HH, NN>), dim3(nb), dim3(256), 0, s, rowptr, col, n_rows,  \
                     (const float4*)Hm, ldh / 4, D, d_head, s1, s2, alpha, edge_mask,         \
                     (float4*)Y, ldy / 4, m_out, den_out)
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

extern "C" int gnnea_gat_bwd_prep_f32(int32_t n_rows, int heads, int d_head, const float* dY,
                                      const float* Y, int64_t ld, const float* s1,
                                      const float* m, const float* den, int act, float* G,
                                      float* rec, void* stream) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!dY || !Y || !s1 || !m || !den || !G || !rec) return GNNEA_EINVAL;
  if (!ok_ld(ld, D) || !al16(dY) || !al16(Y) || !al16(G) || !al16(rec)) return GNNEA_EALIGN;
  if (act != GNNEA_ACT_IDENTITY && act != GNNEA_ACT_RELU) return GNNEA_EINVAL;
  const int nb = div_up(n_rows, 4);
  hipStream_t s = (hipStream_t)stream;
#define CALL_A(A, HH, NN)                                                                      \
  hipLaunchKernelGGL((k_gat_bwd_prep<A, HH, NN>), dim3(nb), dim3(256), 0, s, n_rows, D, d_head, \
                     (const float4*)dY, (const float4*)Y, ld / 4, s1, m, den, (float4*)G,      \
                     (float4*)rec)
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

extern "C" int gnnea_gat_bwd_src_f32(const int32_t* rowptrT, const int32_t* colT,
                                     const int64_t* permT, int32_t n_rows, int heads, int d_head,
                                     const float* H, int64_t ldh, const float* s2, float alpha,
                                     const float* edge_mask, const float* rec, const float* G,
                                     int64_t ldg, const float* a, float* dH, int64_t lddh,
                                     float* dzT, float* ds2, void* stream) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!rowptrT || !colT || !permT || !H || !s2 || !rec || !G || !a || !dH || !dzT || !ds2)
    return GNNEA_EINVAL;
  if (!ok_ld(ldh, D) || !ok_ld(ldg, D) || !ok_ld(lddh, D) || !al16(H) || !al16(G) || !al16(dH) ||
      !al16(rec))
    return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  hipStream_t s = (hipStream_t)stream;
#define CALL(HH, NN)                                                                          \
  case HH * 8 + NN:                                                                           \
    hipLaunchKernelGGL((k_gat_bwd_src<HH, NN>), dim3(nb), dim3(256), 0, s, rowptrT, colT,     \
                       permT, n_rows, D, d_head, (const float4*)H, ldh / 4, s2, alpha,        \
                       edge_mask, (const float4*)rec, (const float4*)G, ldg / 4, a,           \
                       (float4*)dH, lddh / 4, dzT, ds2);                                      \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_gat_bwd_dst_f32(const int32_t* rowptr, const int64_t* tpos, int32_t n_rows,
                                     int heads, int d_head, const float* dzT, const float* a,
                                     float* dH, int64_t lddh, float* ds1, void* stream) {
  if (n_rows < 0 || heads < 1 || d_head < 1) return GNNEA_EINVAL;
  if (n_rows == 0) return 0;
  const int D = heads * d_head, D4 = (D + 3) / 4;
  if (!rowptr || !tpos || !dzT || !a || !dH || !ds1) return GNNEA_EINVAL;
  if (!ok_ld(lddh, D) || !al16(dH)) return GNNEA_EALIGN;
  const int nb = div_up(n_rows, 4);
  hipStream_t s = (hipStream_t)stream;
#define CALL(HH, NN)                                                                          \
  case HH * 8 + NN:                                                                           \
    hipLaunchKernelGGL((k_gat_bwd_dst<HH, NN>), dim3(nb), dim3(256), 0, s, rowptr, tpos,      \
                       n_rows, D, d_head, dzT, a, (float4*)dH, lddh / 4, ds1);                \
    break;
  GNNEA_GAT_DISPATCH(CALL);
#undef CALL
  GNNEA_LAUNCH_CHECK();
  return 0;
}
