// §8f #2: the entity-alignment margin loss, fused gather + L1 + hinge (forward) and its
// sign-scatter backward.  Replaces EAModel.get_loss / UEAModel.get_loss (models/models_ea.py:
// 103-123, 169-183), which materialises four (t*k) x D row gathers, their differences and
// abs values, and backpropagates through index_put.
//
//   A_i   = sum_d |out[left_i] - out[right_i]|
//   h_sij = relu((A_i + 1) - sum_d |out[nl_s[i*k+j]] - out[nr_s[i*k+j]]|)     s = 1, 2
//   loss  = sum h / (2 t k)        (the sum is taken by the caller over h, deterministically)
//
// One workgroup (4 waves) per pair i; a term is one wave, lanes over the feature columns.
// Backward: every active term adds -c*sign(a-b) to row a and +c*sign(a-b) to row b, and the pair
// rows get +-n_i*c*sign(l-r) (n_i = active terms of pair i).  Rows equal to the pair's "anchor"
// (the first term's fixed side: nl_1 = left_i and nr_2 = right_i in the reference's construction)
// accumulate in registers and are flushed once per wave; all other rows use fp32 atomics.
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
                                                    float* __restrict__ A, float* __restrict__ h) {
  __shared__ float As;
  const int i = blockIdx.x, w = wave_id(), lane = lane_id();
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
    if (lane == 0) h[s * tk + e] = fmaxf(d1 - B, 0.f);
  }
}

template <int VEC, int NC>
__device__ __forceinline__ void atomic_row(float* __restrict__ g, int D, const RowFrag<VEC, NC>& r,
                                           float c) {
  const int lane = lane_id();
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) {
    const int d = (cc * 64 + lane) * VEC;
    if (d < D)
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (r.v[cc][e] != 0.f) atomicAdd(g + d + e, c * r.v[cc][e]);
  }
}

template <int VEC, int NC>
__global__ __launch_bounds__(256) void k_margin_bwd(const float* __restrict__ out, int64_t ld,
                                                    int D, int t, int k,
                                                    const int64_t* __restrict__ left,
                                                    const int64_t* __restrict__ right,
                                                    const int64_t* __restrict__ nl1,
                                                    const int64_t* __restrict__ nr1,
                                                    const int64_t* __restrict__ nl2,
                                                    const int64_t* __restrict__ nr2,
                                                    const float* __restrict__ h,
                                                    const float* __restrict__ gout, float inv,
                                                    float* __restrict__ grad, int64_t ldg) {
  __shared__ int nact;
  const int i = blockIdx.x, w = wave_id(), lane = lane_id();
  const float c = gout[0] * inv;
  const int64_t tk = (int64_t)t * k;
  if (threadIdx.x == 0) nact = 0;
  __syncthreads();
  const int64_t anc1 = nl1[(int64_t)i * k], anc2 = nr2[(int64_t)i * k];
  RowFrag<VEC, NC> acc1, acc2;
#pragma unroll
  for (int cc = 0; cc < NC; ++cc)
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc1.v[cc][e] = acc2.v[cc][e] = 0.f;
  int cnt = 0;
  for (int q = w; q < 2 * k; q += 4) {
    const int s = q >= k, j = q - s * k;
    const int64_t e = (int64_t)i * k + j;
    if (!(h[s * tk + e] > 0.f)) continue;  // wave-uniform
    ++cnt;
    const int64_t ra = s ? nl2[e] : nl1[e], rb = s ? nr2[e] : nr1[e];
    RowFrag<VEC, NC> x, y;
    load_row<VEC, NC>(out + ra * ld, D, x);
    load_row<VEC, NC>(out + rb * ld, D, y);
#pragma unroll
    for (int cc = 0; cc < NC; ++cc)
#pragma unroll
      for (int e2 = 0; e2 < VEC; ++e2) x.v[cc][e2] = sgn(x.v[cc][e2] - y.v[cc][e2]);
    // row a gets -c*sgn, row b gets +c*sgn
    const bool a_anchor = s == 0 && ra == anc1, b_anchor = s == 1 && rb == anc2;
    if (a_anchor) {
#pragma unroll
      for (int cc = 0; cc < NC; ++cc)
#pragma unroll
        for (int e2 = 0; e2 < VEC; ++e2) acc1.v[cc][e2] -= x.v[cc][e2];
    } else {
      atomic_row<VEC, NC>(grad + ra * ldg, D, x, -c);
    }
    if (b_anchor) {
#pragma unroll
      for (int cc = 0; cc < NC; ++cc)
#pragma unroll
        for (int e2 = 0; e2 < VEC; ++e2) acc2.v[cc][e2] += x.v[cc][e2];
    } else {
      atomic_row<VEC, NC>(grad + rb * ldg, D, x, c);
    }
  }
  if (lane == 0 && cnt) atomicAdd(&nact, cnt);
  atomic_row<VEC, NC>(grad + anc1 * ldg, D, acc1, c);
  atomic_row<VEC, NC>(grad + anc2 * ldg, D, acc2, c);
  __syncthreads();
  if (w == 0 && nact) {
    const int64_t rl = left[i], rr = right[i];
    RowFrag<VEC, NC> x, y;
    load_row<VEC, NC>(out + rl * ld, D, x);
    load_row<VEC, NC>(out + rr * ld, D, y);
#pragma unroll
    for (int cc = 0; cc < NC; ++cc)
#pragma unroll
      for (int e2 = 0; e2 < VEC; ++e2) x.v[cc][e2] = sgn(x.v[cc][e2] - y.v[cc][e2]);
    const float cn = c * (float)nact;
    atomic_row<VEC, NC>(grad + rl * ldg, D, x, cn);
    atomic_row<VEC, NC>(grad + rr * ldg, D, x, -cn);
  }
}

struct MarginArgs {
  const float* out;
  int64_t ld;
  int D, t, k;
  const int64_t *left, *right, *nl1, *nr1, *nl2, *nr2;
};

template <int VEC, int NC>
static void launch_fwd(const MarginArgs& a, float* A, float* h, hipStream_t s) {
  hipLaunchKernelGGL((k_margin_fwd<VEC, NC>), dim3(a.t), dim3(256), 0, s, a.out, a.ld, a.D, a.t,
                     a.k, a.left, a.right, a.nl1, a.nr1, a.nl2, a.nr2, A, h);
}
template <int VEC, int NC>
static void launch_bwd(const MarginArgs& a, const float* h, const float* gout, float inv,
                       float* grad, int64_t ldg, hipStream_t s) {
  hipLaunchKernelGGL((k_margin_bwd<VEC, NC>), dim3(a.t), dim3(256), 0, s, a.out, a.ld, a.D, a.t,
                     a.k, a.left, a.right, a.nl1, a.nr1, a.nl2, a.nr2, h, gout, inv, grad, ldg);
}

// NC = columns per lane chunk count; float4 path when rows are 16-B aligned
#define GNNEA_MARGIN_DISPATCH(LAUNCH, ...)                                                    \
  do {                                                                                        \
    const bool v4 = (a.D % 4 == 0) && (a.ld % 4 == 0) && (((uintptr_t)a.out & 15) == 0);      \
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
  if (a.t < 0 || a.k < 0 || a.D < 0) return GNNEA_EINVAL;
  if (a.t == 0 || a.k == 0) return 1;
  if (!a.out || !a.left || !a.right || !a.nl1 || !a.nr1 || !a.nl2 || !a.nr2 || a.ld < a.D)
    return GNNEA_EINVAL;
  if (a.D > 1024) return GNNEA_EINVAL;
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_margin_fwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                                    const int64_t* left, const int64_t* right,
                                    const int64_t* neg_left, const int64_t* neg_right,
                                    const int64_t* neg2_left, const int64_t* neg2_right,
                                    float* A, float* h, void* stream) {
  const MarginArgs a{out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left, neg2_right};
  const int rc = margin_check(a);
  if (rc) return rc < 0 ? rc : 0;
  if (!A || !h) return GNNEA_EINVAL;
  GNNEA_MARGIN_DISPATCH(launch_fwd, a, A, h, (hipStream_t)stream);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_margin_bwd_f32(const float* out, int64_t ld, int32_t D, int32_t t, int32_t k,
                                    const int64_t* left, const int64_t* right,
                                    const int64_t* neg_left, const int64_t* neg_right,
                                    const int64_t* neg2_left, const int64_t* neg2_right,
                                    const float* h, const float* grad_loss, float scale,
                                    float* grad, int64_t ldg, void* stream) {
  const MarginArgs a{out, ld, D, t, k, left, right, neg_left, neg_right, neg2_left, neg2_right};
  const int rc = margin_check(a);
  if (rc) return rc < 0 ? rc : 0;
  if (!h || !grad_loss || !grad || ldg < D) return GNNEA_EINVAL;
  GNNEA_MARGIN_DISPATCH(launch_bwd, a, h, grad_loss, scale, grad, ldg, (hipStream_t)stream);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
