// §8f #2: the entity-alignment margin loss, fused gather + L1 + hinge (forward) and its
// sign-scatter backward.  Replaces EAModel.get_loss / UEAModel.get_loss (models/models_ea.py:
// 103-123, 169-183), which materialises four (t*k) x D row gathers, their differences and
// abs values, and backpropagates through index_put.
//
//   A_i   = sum_d |out[left_i] - out[right_i]|
//   h_sij = relu((A_i + 1) - sum_d |out[nl_s[i*k+j]] - out[nr_s[i*k+j]]|)     s = 1, 2
//   loss  = sum h / (2 t k)        (the sum is taken by the caller over h, deterministically)
//
// Terms j in [0, M), M = 2tk + t: side-1 negatives (nl1, nr1), side-2 negatives (nl2, nr2), then
// the t pairs (left, right).  d loss/d out = c * sum_j m_j * (e_{a_j} - e_{b_j}) (x) sgn(x_a - x_b)
// with c = grad/(2tk), m_j = -[h_j > 0] for a negative and m_j = n_i (active terms of pair i) for a
// pair; the forward writes m.  Every coefficient is an integer, so the backward sums them exactly:
//   grad[r] = c * sum_{(j, other) incident to r} m_j * sgn(x_r - x_other)
// over the incidence CSR of the term rows (built once per negative set with gnnea_coo_to_csr),
// one wave per output row: no atomics, deterministic, bit-identical run to run.
// Forward: one workgroup (4 waves) per pair i, a term per wave, lanes over the feature columns.
#include "common.h"

namespace gnnea {

template <int VEC, int NC>
struct RowFrag {
  float v[NC][VEC];
};

// (T = bf16_t: the rows' bf16 values widened exactly, so every sum below is the one the fp32
// kernels compute on the fp32 copy of the same rows)
template <int VEC, int NC, typename T = float>
__device__ __forceinline__ void load_row(const T* __restrict__ p, int D, RowFrag<VEC, NC>& r) {
  const int lane = lane_id();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int d = (c * 64 + lane) * VEC;
    if constexpr (VEC == 4) {
      const float4 x = d < D ? Vec4<T>::get(*(const typename Vec4<T>::raw*)(p + d))
                             : make_float4(0.f, 0.f, 0.f, 0.f);
      r.v[c][0] = x.x;
      r.v[c][1] = x.y;
      r.v[c][2] = x.z;
      r.v[c][3] = x.w;
    } else {
      r.v[c][0] = d < D ? to_f32<T>(p[d]) : 0.f;
    }
  }
}

template <int VEC, int NC>
__device__ __forceinline__ float l1_rows(const float* __restrict__ a, const float* __restrict__ b,
                                         int D) {
  RowFrag<VEC, NC> x, y;
  load_row<VEC, NC>(a, D, x);
  load_row<VEC, NC>(b, D, y);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) s += fabsf(x.v[c][e] - y.v[c][e]);
  return wave_sum(s);
}

__device__ __forceinline__ float sgn(float x) { return (float)((x > 0.f) - (x < 0.f)); }

// Sign codes of a term (float4 lane map only): byte q = c*64 + lane holds, for its 4 columns,
// 2 bits each, the 2-bit two's complement of sgn(x_a - x_b): 01 = +1, 11 = -1, 00 = equal.  The backward reads them instead of
// re-gathering both rows: sgn(x_r - x_other) is +code at the a-end, -code at the b-end, the exact
// values the row gather would give (same fp32 operands).
template <int NC, typename T>
__device__ __forceinline__ float l1_rows_code(const T* __restrict__ a, const T* __restrict__ b,
                                              int D, uint8_t* __restrict__ code) {
  RowFrag<4, NC> x, y;
  load_row<4, NC, T>(a, D, x);
  load_row<4, NC, T>(b, D, y);
  const int lane = lane_id();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    uint32_t byte = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = x.v[c][e] - y.v[c][e];
      s += fabsf(d);
      byte |= ((d > 0.f) ? 1u : (d < 0.f) ? 3u : 0u) << (2 * e);
    }
    const int q = c * 64 + lane;
    if (4 * q < D) code[q] = (uint8_t)byte;
  }
  return wave_sum(s);
}

// L1 distance of two loaded row fragments (wave-reduced); CODE also stores the term's sign codes
// (float4 map, see l1_rows_code).  Same per-lane order and reduction as l1_rows.
template <int VEC, int NC, bool CODE>
__device__ __forceinline__ float l1_frag(const RowFrag<VEC, NC>& x, const RowFrag<VEC, NC>& y,
                                         int D, uint8_t* __restrict__ code) {
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    uint32_t byte = 0;
#pragma unroll
    for (int e = 0; e < VEC; ++e) {
      const float d = x.v[c][e] - y.v[c][e];
      s += fabsf(d);
      if constexpr (CODE) byte |= ((d > 0.f) ? 1u : (d < 0.f) ? 3u : 0u) << (2 * e);
    }
    if constexpr (CODE) {
      static_assert(VEC == 4, "sign codes use the float4 lane map");
      const int q = c * 64 + lane_id();
      if (4 * q < D) code[q] = (uint8_t)byte;
    }
  }
  return wave_sum(s);
}

template <int VEC, int NC, bool CODE = false, typename T = float>
__global__ __launch_bounds__(256) void k_margin_fwd(const T* __restrict__ out, int64_t ld,
                                                    int D, int t, int k,
                                                    const int64_t* __restrict__ left,
                                                    const int64_t* __restrict__ right,
                                                    const int64_t* __restrict__ nl1,
                                                    const int64_t* __restrict__ nr1,
                                                    const int64_t* __restrict__ nl2,
                                                    const int64_t* __restrict__ nr2,
                                                    float* __restrict__ A, float* __restrict__ h,
                                                    float* __restrict__ m,
                                                    uint8_t* __restrict__ codes = nullptr,
                                                    int64_t sb = 0) {
  __shared__ float As;
  __shared__ int nact;
  const int i = blockIdx.x, w = wave_id(), lane = lane_id();
  if (threadIdx.x == 0) nact = 0;
  const int64_t tk = (int64_t)t * k;
  auto l1 = [&](int64_t ra, int64_t rb, int64_t term) {
    if constexpr (CODE)
      return l1_rows_code<NC, T>(out + ra * ld, out + rb * ld, D, codes + term * sb);
    else
      return l1_rows<VEC, NC>(out + ra * ld, out + rb * ld, D);
  };
  if (w == 0) {
    const float a = l1(left[i], right[i], 2 * tk + i);
    if (lane == 0) {
      As = a;
      A[i] = a;
    }
  }
  __syncthreads();
  const float d1 = As + 1.0f;
  // U negative terms per wave per round: all 2U row loads are issued before the first reduction
  constexpr int U = 4;
  for (int q0 = w * U; q0 < 2 * k; q0 += 4 * U) {
    RowFrag<VEC, NC> xa[U], xb[U];
    int64_t term[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = q0 + u < 2 * k ? q0 + u : q0;
      const int s = q >= k, j = q - s * k;
      const int64_t e = (int64_t)i * k + j;
      term[u] = s * tk + e;
      load_row<VEC, NC, T>(out + (s ? nl2[e] : nl1[e]) * ld, D, xa[u]);
      load_row<VEC, NC, T>(out + (s ? nr2[e] : nr1[e]) * ld, D, xb[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (q0 + u >= 2 * k) break;  // wave-uniform
      const float B = l1_frag<VEC, NC, CODE>(xa[u], xb[u], D, codes + term[u] * sb);
      const float hv = fmaxf(d1 - B, 0.f);
      if (lane == 0) {
        h[term[u]] = hv;
        m[term[u]] = hv > 0.f ? -1.f : 0.f;
        if (hv > 0.f) atomicAdd(&nact, 1);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) m[2 * tk + i] = (float)nact;
}

// Backward work item = one chunk of <= kMarginChunk incidence entries of one output row:
// {row, beg, end, slot}.  slot < 0: the row has a single chunk and the wave writes grad[row];
// otherwise the chunk's partial (integer-valued, exact in fp32) goes to scratch[slot] and
// k_margin_combine adds a long row's chunks in slot order.  Long rows (hub entities that are the
// hard negative of many pairs) are thus spread over many waves; the result stays deterministic.
// Active entries are compacted per 64-entry batch and gathered four at a time.
template <int VEC, int NC>
__global__ __launch_bounds__(256) void k_margin_bwd(const float* __restrict__ out, int64_t ld,
                                                    int D, int t, int k,
                                                    const int64_t* __restrict__ left,
                                                    const int64_t* __restrict__ right,
                                                    const int64_t* __restrict__ nl1,
                                                    const int64_t* __restrict__ nr1,
                                                    const int64_t* __restrict__ nl2,
                                                    const int64_t* __restrict__ nr2,
                                                    const float* __restrict__ m,
                                                    const int32_t* __restrict__ inc_ent,
                                                    const int4* __restrict__ items, int n_items,
                                                    const float* __restrict__ gout, float inv,
                                                    float* __restrict__ grad, int64_t ldg,
                                                    float* __restrict__ scratch) {
  const int it = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (it >= n_items) return;
  const int4 item = items[it];
  const int row = item.x, beg = item.y, end = item.z, slot = item.w;
  const int lane = lane_id();
  const int64_t tk = (int64_t)t * k, M = 2 * tk + t;
  RowFrag<VEC, NC> self, acc;
  load_row<VEC, NC>(out + (int64_t)row * ld, D, self);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc.v[c][e] = 0.f;
  auto add = [&](float mq, int64_t o) {
    RowFrag<VEC, NC> x;
    load_row<VEC, NC>(out + o * ld, D, x);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc.v[c][e] += mq * sgn(self.v[c][e] - x.v[c][e]);
  };
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    // lane-parallel decode of up to 64 incident entries: multiplier and the other row
    float mj = 0.f;
    int64_t other = 0;
    if (lane < cnt) {
      const int64_t p = inc_ent[base + lane];
      const bool role_b = p >= M;
      const int64_t j = role_b ? p - M : p;
      mj = m[j];
      if (mj != 0.f) {
        if (j < tk) other = role_b ? nl1[j] : nr1[j];
        else if (j < 2 * tk) other = role_b ? nl2[j - tk] : nr2[j - tk];
        else other = role_b ? left[j - 2 * tk] : right[j - 2 * tk];
      }
    }
    // active entries in lane order, four gathers in flight
    unsigned long long act = __ballot(mj != 0.f);
    auto pop = [&](float& mq, int64_t& o) {
      const int q = __builtin_ctzll(act);
      act &= act - 1;
      mq = readlane_f(mj, q);
      o = ((int64_t)readlane_i((int)(other >> 32), q) << 32) |
          (uint32_t)readlane_i((int)(other & 0xffffffff), q);
    };
    while (__popcll(act) >= 4) {
      float m0, m1, m2, m3;
      int64_t o0, o1, o2, o3;
      pop(m0, o0);
      pop(m1, o1);
      pop(m2, o2);
      pop(m3, o3);
      RowFrag<VEC, NC> x0, x1, x2, x3;
      load_row<VEC, NC>(out + o0 * ld, D, x0);
      load_row<VEC, NC>(out + o1 * ld, D, x1);
      load_row<VEC, NC>(out + o2 * ld, D, x2);
      load_row<VEC, NC>(out + o3 * ld, D, x3);
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < VEC; ++e) {
          const float sv = self.v[c][e];
          acc.v[c][e] += m0 * sgn(sv - x0.v[c][e]);
          acc.v[c][e] += m1 * sgn(sv - x1.v[c][e]);
          acc.v[c][e] += m2 * sgn(sv - x2.v[c][e]);
          acc.v[c][e] += m3 * sgn(sv - x3.v[c][e]);
        }
    }
    while (act) {
      float mq;
      int64_t o;
      pop(mq, o);
      add(mq, o);
    }
  }
  const float c0 = slot < 0 ? gout[0] * inv : 1.0f;
  float* dst = slot < 0 ? grad + (int64_t)row * ldg : scratch + (int64_t)slot * D;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int d = (c * 64 + lane) * VEC;
    if (d >= D) continue;
#pragma unroll
    for (int e = 0; e < VEC; ++e) dst[d + e] = c0 * acc.v[c][e];
  }
}

// Backward from the forward's sign codes: per work item (one row's chunk of incidence entries)
// the wave reads, for every active incident term, its NC code bytes per lane (coalesced, 64 B per
// chunk) instead of gathering the other row: no feature-row traffic at all.  Entries are added
// in incidence order with the same integer multipliers as k_margin_bwd, so the gradient is
// bit-identical to it.
typedef short short2v __attribute__((ext_vector_type(2)));

// PK (|multiplier| <= 2k <= 510, so 64 entries sum below 2^15): each code byte is looked up in a
// 256-entry LDS table of its four signs as two packed int16 pairs and accumulated with packed
// 16-bit multiply-adds (2 instructions per 4 columns instead of 8), flushed into the int32
// accumulators after every 64-entry batch.  Exact like the int32 path.
template <int NC, bool PK = false, typename TG = float>
__global__ __launch_bounds__(256) void k_margin_bwd_code(int D, int64_t M,
                                                         const float* __restrict__ m,
                                                         const uint8_t* __restrict__ codes,
                                                         int64_t sb,
                                                         const int32_t* __restrict__ inc_ent,
                                                         const int4* __restrict__ items,
                                                         int n_items,
                                                         const float* __restrict__ gout,
                                                         float inv, TG* __restrict__ grad,
                                                         int64_t ldg,
                                                         float* __restrict__ scratch) {
  __shared__ uint2 lut[PK ? 256 : 1];
  if constexpr (PK) {
    const uint32_t b = threadIdx.x;  // 256 threads: one table entry each
    auto sx = [&](int e) { return (uint32_t)(uint16_t)(int16_t)(((int)(b << (30 - 2 * e))) >> 30); };
    lut[b] = make_uint2(sx(0) | (sx(1) << 16), sx(2) | (sx(3) << 16));
    __syncthreads();
  }
  const int it = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (it >= n_items) return;
  const int4 item = items[it];
  const int row = item.x, beg = item.y, end = item.z, slot = item.w;
  const int lane = lane_id();
  bool own[NC];
  int acc[NC][4];  // integer multipliers x signs: exact, so order-free
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    own[c] = 4 * (c * 64 + lane) < D;
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[c][e] = 0;
  }
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    int f = 0;  // signed multiplier: +m_j at the a-end, -m_j at the b-end (|m_j| <= 2k)
    int64_t j = 0;
    if (lane < cnt) {
      const int64_t p = inc_ent[base + lane];
      const bool role_b = p >= M;
      j = role_b ? p - M : p;
      const int mj = (int)m[j];
      f = role_b ? -mj : mj;
    }
    unsigned long long act = __ballot(f != 0);
    short2v pacc[NC][2];
#pragma unroll
    for (int c = 0; c < NC; ++c) pacc[c][0] = pacc[c][1] = (short2v){0, 0};
    while (act) {
      // up to U active entries per round, branch-free (an exhausted slot re-reads lane 0's
      // valid term with multiplier 0) so all U code loads are in flight together
      constexpr int U = 16;
      int fq[U];
      uint32_t cb[U][NC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool v = act != 0ull;
        const int q = v ? __builtin_ctzll(act) : 0;
        act &= act - 1;
        fq[u] = v ? readlane_i(f, q) : 0;
        const int64_t jq = ((int64_t)readlane_i((int)(j >> 32), q) << 32) |
                           (uint32_t)readlane_i((int)(j & 0xffffffff), q);
        const uint8_t* cp = codes + jq * sb;
#pragma unroll
        for (int c = 0; c < NC; ++c) cb[u][c] = own[c] ? cp[c * 64 + lane] : 0u;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if constexpr (PK) {
            const uint2 w = lut[cb[u][c]];
            const short2v fv = {(short)fq[u], (short)fq[u]};
            pacc[c][0] += __builtin_bit_cast(short2v, w.x) * fv;
            pacc[c][1] += __builtin_bit_cast(short2v, w.y) * fv;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              // v_bfe_i32 of the 2-bit field, then v_mad_i32_i24
              const int sg = ((int)(cb[u][c] << (30 - 2 * e))) >> 30;
              acc[c][e] = __mul24(sg, fq[u]) + acc[c][e];
            }
          }
        }
      }
    }
    if constexpr (PK) {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        acc[c][0] += pacc[c][0].x;
        acc[c][1] += pacc[c][0].y;
        acc[c][2] += pacc[c][1].x;
        acc[c][3] += pacc[c][1].y;
      }
    }
  }
  const float c0 = slot < 0 ? gout[0] * inv : 1.0f;
  if (slot < 0) {  // the row's gradient (bf16: rounded once, as torch's cast of the fp32 value)
    TG* dst = grad + (int64_t)row * ldg;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!own[c]) continue;
      const int d = (c * 64 + lane) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[d + e] = from_f32<TG>(c0 * (float)acc[c][e]);
    }
  } else {  // a long row's chunk partial (fp32, integer-valued)
    float* dst = scratch + (int64_t)slot * D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!own[c]) continue;
      const int d = (c * 64 + lane) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[d + e] = c0 * (float)acc[c][e];
    }
  }
}

// long rows: grad[row] = c * sum of the row's chunk partials, in slot order (one wave per row)
template <typename TG = float>
__global__ __launch_bounds__(256) void k_margin_combine(const int32_t* __restrict__ long_rows,
                                                        const int32_t* __restrict__ long_ptr,
                                                        int n_long, int D,
                                                        const float* __restrict__ scratch,
                                                        const float* __restrict__ gout, float inv,
                                                        TG* __restrict__ grad, int64_t ldg) {
  const int w = blockIdx.x * 4 + wave_id();
  if (w >= n_long) return;
  const int row = long_rows[w], s0 = long_ptr[w], s1 = long_ptr[w + 1];
  const float c0 = gout[0] * inv;
  for (int d = lane_id(); d < D; d += 64) {
    float sum = 0.f;
    for (int sl = s0; sl < s1; ++sl) sum += scratch[(int64_t)sl * D + d];
    grad[(int64_t)row * ldg + d] = from_f32<TG>(c0 * sum);
  }
}

struct MarginArgs {
  const float* out;
  int64_t ld;
  int D, t, k;
  const int64_t *left, *right, *nl1, *nr1, *nl2, *nr2;
};

template <int VEC, int NC>
static void launch_fwd(const MarginArgs& a, float* A, float* h, float* m, hipStream_t s) {
  hipLaunchKernelGGL((k_margin_fwd<VEC, NC>), dim3(a.t), dim3(256), 0, s, a.out, a.ld, a.D, a.t,
                     a.k, a.left, a.right, a.nl1, a.nr1, a.nl2, a.nr2, A, h, m);
}
template <int VEC, int NC>
static void launch_bwd(const MarginArgs& a, const float* m, const int32_t* inc_ent,
                       const int4* items, int n_items, const float* gout, float inv, float* grad,
                       int64_t ldg, float* scratch, hipStream_t s) {
  hipLaunchKernelGGL((k_margin_bwd<VEC, NC>), dim3(div_up(n_items, 4)), dim3(256), 0, s, a.out,
                     a.ld, a.D, a.t, a.k, a.left, a.right, a.nl1, a.nr1, a.nl2, a.nr2, m, inc_ent,
                     items, n_items, gout, inv, grad, ldg, scratch);
}

// NC = columns per lane chunk count; float4 path when rows are 16-B aligned
#define GNNEA_MARGIN_DISPATCH(LAUNCH, ...)                                                    \
  do {                                                                                        \
    const bool v4 = (a.D % 4 == 0) && (a.ld % 4 == 0) && (((uintptr_t)a.out & 15) == 0) && \
                    aligned_out;      \
    const int nc = v4 ? div_up(a.D, 256) : div_up(a.D, 64);                                   \
    if (v4) {                                                                                 \
      switch (nc) {                                                                           \
        case 1: LAUNCH<4, 1>(__VA_ARGS__); break;                                             \
        case 2: LAUNCH<4, 2>(__VA_ARGS__); break;                                             \
        case 3: LAUNCH<4, 3>(__VA_ARGS__); break;                                             \
        case 4: LAUNCH<4, 4>(__VA_ARGS__); break;                                             \
        default: return GNNEA_EINVAL;                                                         \
      }                                                                                       \
    } else {                                                                                  \
      switch (nc) {                                                                           \
        case 1: LAUNCH<1, 1>(__VA_ARGS__); break;                                             \
        case 2: LAUNCH<1, 2>(__VA_ARGS__); break;                                             \
        case 3: LAUNCH<1, 3>(__VA_ARGS__); break;                                             \
        case 4: LAUNCH<1, 4>(__VA_ARGS__); break;                                             \
        case 5: LAUNCH<1, 5>(__VA_ARGS__); break;                                             \
        case 6: LAUNCH<1, 6>(__VA_ARGS__); break;                                             \
        case 7: LAUNCH<1, 7>(__VA_ARGS__); break;                                             \
        case 8: LAUNCH<1, 8>(__VA_ARGS__); break;                                             \
        default: return GNNEA_EINVAL;                                                         \
      }                                                                                       \
    }                                                                                         \
  } while (0)

static int margin_check(const MarginArgs& a) {
  if (a.t < 0 || a.k < 0 || a.D < 0 || a.D > 1024 || a.ld < a.D || !a.out) return GNNEA_EINVAL;
  if (a.t > 0 && (!a.left || !a.right)) return GNNEA_EINVAL;
  if (a.t > 0 && a.k > 0 && (!a.nl1 || !a.nr1 || !a.nl2 || !a.nr2)) return GNNEA_EINVAL;
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_margin_fwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                                    const int64_t* left, const int64_t* right,
                                    const int64_t* neg_left, const int64_t* neg_right,
                                    const int64_t* neg2_left, const int64_t* neg2_right,
                                    float* A, float* h, float* m, void* stream) {
  const MarginArgs a{out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left, neg2_right};
  if (const int rc = margin_check(a)) return rc;
  if (a.t == 0) return 0;
  if (!A || !m || (a.k > 0 && !h)) return GNNEA_EINVAL;
  const bool aligned_out = true;
  GNNEA_MARGIN_DISPATCH(launch_fwd, a, A, h, m, (hipStream_t)stream);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_margin_bwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                                    const int64_t* left, const int64_t* right,
                                    const int64_t* neg_left, const int64_t* neg_right,
                                    const int64_t* neg2_left, const int64_t* neg2_right,
                                    const float* m, const int32_t* inc_ent,
                                    const int32_t* items, int32_t n_items,
                                    const int32_t* long_rows, const int32_t* long_ptr,
                                    int32_t n_long, float* scratch, const float* grad_loss,
                                    float scale, float* grad, int64_t ldg, void* stream) {
  const MarginArgs a{out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left, neg2_right};
  if (n_items < 0 || n_long < 0) return GNNEA_EINVAL;
  if (const int rc = margin_check(a)) return rc;
  if (n_items == 0) return 0;
  if (!m || !inc_ent || !items || !grad_loss || !grad || ldg < D) return GNNEA_EINVAL;
  if (n_long > 0 && (!long_rows || !long_ptr || !scratch)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const bool aligned_out = true;
  GNNEA_MARGIN_DISPATCH(launch_bwd, a, m, inc_ent, (const int4*)items, n_items, grad_loss, scale,
                        grad, ldg, scratch, s);
  if (n_long > 0)
    hipLaunchKernelGGL(k_margin_combine<float>, dim3(div_up(n_long, 4)), dim3(256), 0, s, long_rows,
                       long_ptr, n_long, D, scratch, grad_loss, scale, grad, ldg);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// ---- sign-code forward / backward (float4 rows: D % 4 == 0, ld % 4 == 0, 16-B aligned out) ----
// T = bf16_t (cfg-5 storage): the rows read as bf16 and widened exactly, the gradient rounded to
// bf16 once -- bit-identical to the fp32 kernels on the fp32 copy of the rows followed by a cast
// of the gradient, without the copy, the cast and the fp32 gradient buffer.
template <typename T>
static int margin_fwd_code(const T* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                           const int64_t* left, const int64_t* right, const int64_t* neg_left,
                           const int64_t* neg_right, const int64_t* neg2_left,
                           const int64_t* neg2_right, float* A, float* h, float* m, void* codes,
                           int64_t sb, void* stream) {
  if (t < 0 || k < 0 || D < 0 || D > 1024 || ld < D || !out) return GNNEA_EINVAL;
  if (t > 0 && (!left || !right)) return GNNEA_EINVAL;
  if (t > 0 && k > 0 && (!neg_left || !neg_right || !neg2_left || !neg2_right)) return GNNEA_EINVAL;
  if (t == 0) return 0;
  if (!A || !m || (k > 0 && !h) || !codes) return GNNEA_EINVAL;
  if (D % 4 || ld % 4 || (((uintptr_t)out) & (4 * sizeof(T) - 1)) || sb < (D + 3) / 4)
    return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
#define GNNEA_FC(N)                                                                               \
  case N:                                                                                         \
    hipLaunchKernelGGL((k_margin_fwd<4, N, true, T>), dim3(t), dim3(256), 0, s, out, ld, D, t, k, \
                       left, right, neg_left, neg_right, neg2_left, neg2_right, A, h, m,          \
                       (uint8_t*)codes, sb);                                                      \
    break;
  switch (div_up(D, 256)) {
    GNNEA_FC(1)
    GNNEA_FC(2)
    GNNEA_FC(3)
    GNNEA_FC(4)
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_FC
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename TG>
static int margin_bwd_code(int32_t D, int32_t t, int32_t k, const float* m, const void* codes,
                           int64_t sb, const int32_t* inc_ent, const int32_t* items,
                           int32_t n_items, const int32_t* long_rows, const int32_t* long_ptr,
                           int32_t n_long, float* scratch, const float* grad_loss, float scale,
                           TG* grad, int64_t ldg, void* stream) {
  if (n_items < 0 || n_long < 0 || D < 0 || D > 1024 || D % 4 || t < 0 || k < 0)
    return GNNEA_EINVAL;
  if (n_items == 0) return 0;
  if (!m || !codes || !inc_ent || !items || !grad_loss || !grad || ldg < D || sb < (D + 3) / 4)
    return GNNEA_EINVAL;
  if (n_long > 0 && (!long_rows || !long_ptr || !scratch)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int64_t M = 2ll * t * k + t;
  // packed 16-bit accumulation needs 64 * max|m_j| = 64 * 2k < 2^15
  const bool pk = k <= 255;
#define GNNEA_BC(N)                                                                               \
  case N:                                                                                         \
    if (pk)                                                                                       \
      hipLaunchKernelGGL((k_margin_bwd_code<N, true, TG>), dim3(div_up(n_items, 4)), dim3(256),   \
                         0, s, D, M, m, (const uint8_t*)codes, sb, inc_ent, (const int4*)items,   \
                         n_items, grad_loss, scale, grad, ldg, scratch);                          \
    else                                                                                          \
      hipLaunchKernelGGL((k_margin_bwd_code<N, false, TG>), dim3(div_up(n_items, 4)), dim3(256),  \
                         0, s, D, M, m, (const uint8_t*)codes, sb, inc_ent, (const int4*)items,   \
                         n_items, grad_loss, scale, grad, ldg, scratch);                          \
    break;
  switch (div_up(D, 256)) {
    GNNEA_BC(1)
    GNNEA_BC(2)
    GNNEA_BC(3)
    GNNEA_BC(4)
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_BC
  if (n_long > 0)
    hipLaunchKernelGGL(k_margin_combine<TG>, dim3(div_up(n_long, 4)), dim3(256), 0, s, long_rows,
                       long_ptr, n_long, D, scratch, grad_loss, scale, grad, ldg);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_margin_fwd_code_f32(const float* out, int64_t ld, int32_t D, int32_t t,
                                         int32_t k, const int64_t* left, const int64_t* right,
                                         const int64_t* neg_left, const int64_t* neg_right,
                                         const int64_t* neg2_left, const int64_t* neg2_right,
                                         float* A, float* h, float* m, void* codes, int64_t sb,
                                         void* stream) {
  return margin_fwd_code<float>(out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left,
                                neg2_right, A, h, m, codes, sb, stream);
}

extern "C" int gnnea_margin_fwd_code_bf16(const void* out, int64_t ld, int32_t D, int32_t t,
                                          int32_t k, const int64_t* left, const int64_t* right,
                                          const int64_t* neg_left, const int64_t* neg_right,
                                          const int64_t* neg2_left, const int64_t* neg2_right,
                                          float* A, float* h, float* m, void* codes, int64_t sb,
                                          void* stream) {
  return margin_fwd_code<bf16_t>((const bf16_t*)out, ld, D, t, k, left, right, neg_left,
                                 neg_right, neg2_left, neg2_right, A, h, m, codes, sb, stream);
}

extern "C" int gnnea_margin_bwd_code_f32(int32_t D, int32_t t, int32_t k, const float* m,
                                         const void* codes, int64_t sb, const int32_t* inc_ent,
                                         const int32_t* items, int32_t n_items,
                                         const int32_t* long_rows, const int32_t* long_ptr,
                                         int32_t n_long, float* scratch, const float* grad_loss,
                                         float scale, float* grad, int64_t ldg, void* stream) {
  return margin_bwd_code<float>(D, t, k, m, codes, sb, inc_ent, items, n_items, long_rows,
                                long_ptr, n_long, scratch, grad_loss, scale, grad, ldg, stream);
}

extern "C" int gnnea_margin_bwd_code_bf16(int32_t D, int32_t t, int32_t k, const float* m,
                                          const void* codes, int64_t sb, const int32_t* inc_ent,
                                          const int32_t* items, int32_t n_items,
                                          const int32_t* long_rows, const int32_t* long_ptr,
                                          int32_t n_long, float* scratch, const float* grad_loss,
                                          float scale, void* grad, int64_t ldg, void* stream) {
  return margin_bwd_code<bf16_t>(D, t, k, m, codes, sb, inc_ent, items, n_items, long_rows,
                                 long_ptr, n_long, scratch, grad_loss, scale, (bf16_t*)grad, ldg,
                                 stream);
}
