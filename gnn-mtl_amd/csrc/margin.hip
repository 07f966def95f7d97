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

template <int VEC, int NC>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int D, RowFrag<VEC, NC>& r) {
  const int lane = lane_id();
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int d = (c * 64 + lane) * VEC;
    if constexpr (VEC == 4) {
      const float4 x = d < D ? *(const float4*)(p + d) : make_float4(0.f, 0.f, 0.f, 0.f);
      r.v[c][0] = x.x;
      r.v[c][1] = x.y;
      r.v[c][2] = x.z;
      r.v[c][3] = x.w;
    } else {
      r.v[c][0] = d < D ? p[d] : 0.f;
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

template <int VEC, int NC>
__global__ __launch_bounds__(256) void k_margin_fwd(const float* __restrict__ out, int64_t ld,
                                                    int D, int t, int k,
                                                    const int64_t* __restrict__ left,
                                                    const int64_t* __restrict__ right,
                                                    const int64_t* __restrict__ nl1,
                                                    const int64_t* __restrict__ nr1,
                                                    const int64_t* __restrict__ nl2,
                                                    const int64_t* __restrict__ nr2,
                                                    float* __restrict__ A, float* __restrict__ h,
                                                    float* __restrict__ m) {
  __shared__ float As;
  __shared__ int nact;
  const int i = blockIdx.x, w = wave_id(), lane = lane_id();
  if (threadIdx.x == 0) nact = 0;
  if (w == 0) {
    const float a = l1_rows<VEC, NC>(out + left[i] * ld, out + right[i] * ld, D);
    if (lane == 0) {
      As = a;
      A[i] = a;
    }
  }
  __syncthreads();
  const float d1 = As + 1.0f;
  const int64_t tk = (int64_t)t * k;
  for (int q = w; q < 2 * k; q += 4) {
    const int s = q >= k, j = q - s * k;
    const int64_t e = (int64_t)i * k + j;
    const int64_t ra = s ? nl2[e] : nl1[e], rb = s ? nr2[e] : nr1[e];
    const float B = l1_rows<VEC, NC>(out + ra * ld, out + rb * ld, D);
    const float hv = fmaxf(d1 - B, 0.f);
    if (lane == 0) {
      h[s * tk + e] = hv;
      m[s * tk + e] = hv > 0.f ? -1.f : 0.f;
      if (hv > 0.f) atomicAdd(&nact, 1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) m[2 * tk + i] = (float)nact;
}

// one wave per output row; lanes over columns (float4 when VEC == 4)
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
                                                    const int32_t* __restrict__ inc_rowptr,
                                                    const int32_t* __restrict__ inc_ent, int n_rows,
                                                    const float* __restrict__ gout, float inv,
                                                    float* __restrict__ grad, int64_t ldg) {
  const int row = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int64_t tk = (int64_t)t * k, M = 2 * tk + t;
  RowFrag<VEC, NC> self, acc;
  load_row<VEC, NC>(out + row * ld, D, self);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc.v[c][e] = 0.f;
  const int beg = inc_rowptr[row], end = inc_rowptr[row + 1];
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
    for (int q = 0; q < cnt; ++q) {
      const float mq = readlane_f(mj, q);
      if (mq == 0.f) continue;  // inactive hinge term (wave-uniform)
      const int64_t o = ((int64_t)readlane_i((int)(other >> 32), q) << 32) |
                        (uint32_t)readlane_i((int)(other & 0xffffffff), q);
      RowFrag<VEC, NC> x;
      load_row<VEC, NC>(out + o * ld, D, x);
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc.v[c][e] += mq * sgn(self.v[c][e] - x.v[c][e]);
    }
  }
  const float c0 = gout[0] * inv;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int d = (c * 64 + lane) * VEC;
    if (d >= D) continue;
    float* g = grad + row * ldg + d;
    if constexpr (VEC == 4) {
      *(float4*)g = make_float4(c0 * acc.v[c][0], c0 * acc.v[c][1], c0 * acc.v[c][2],
                                c0 * acc.v[c][3]);
    } else {
      g[0] = c0 * acc.v[c][0];
    }
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
static void launch_bwd(const MarginArgs& a, const float* m, const int32_t* inc_rowptr,
                       const int32_t* inc_ent, int n_rows, const float* gout, float inv,
                       float* grad, int64_t ldg, hipStream_t s) {
  hipLaunchKernelGGL((k_margin_bwd<VEC, NC>), dim3(div_up(n_rows, 4)), dim3(256), 0, s, a.out,
                     a.ld, a.D, a.t, a.k, a.left, a.right, a.nl1, a.nr1, a.nl2, a.nr2, m,
                     inc_rowptr, inc_ent, n_rows, gout, inv, grad, ldg);
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
                                    const float* m, const int32_t* inc_rowptr,
                                    const int32_t* inc_ent, int32_t n_rows,
                                    const float* grad_loss, float scale, float* grad, int64_t ldg,
                                    void* stream) {
  const MarginArgs a{out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left, neg2_right};
  if (n_rows < 0) return GNNEA_EINVAL;
  if (const int rc = margin_check(a)) return rc;
  if (n_rows == 0) return 0;
  if (!inc_rowptr || !grad_loss || !grad || ldg < D || (a.t > 0 && (!m || !inc_ent)))
    return GNNEA_EINVAL;
  const bool aligned_out = (ldg % 4 == 0) && (((uintptr_t)grad & 15) == 0);
  GNNEA_MARGIN_DISPATCH(launch_bwd, a, m, inc_rowptr, inc_ent, n_rows, grad_loss, scale, grad, ldg,
                        (hipStream_t)stream);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
