// Activation passes over row-major feature matrices (the MLP decoder's Linear layers,
// layers/layers.py:111-122: act(dropout(x·Wᵀ + b))).
//
//   act_rows_*                 the act in place on a GEMM output whose kernel has no fused epilogue
//                              for it (the fp32 ring and the bf16 weight-resident projections apply
//                              relu in their epilogues; every other GEMM kernel runs this after);
//   gnnea_act_fwd_*            Y = act(X) over a contiguous buffer (the non-fused Linear path);
//   gnnea_act_bwd_colsum_*     the act's backward and the bias gradient in ONE pass:
//                                G = dY * act'(Y)  (act' from the output, as k_act_bwd),
//                                db = column sums of G (the stored, rounded G values),
//                              instead of the act backward, then a second read of G by colsum.
//                              Per step and relu layer at cfg-4 (2M x 300 fp32) that is 2.4 GB
//                              less HBM traffic: 7.2 GB (dY, Y in, G out) instead of 9.6.
//
// Bytes per element: act_rows 2 sizeof(T) (read + write in place); act_bwd_colsum 3 sizeof(T).
// Both are HBM-bound streaming passes: 16-B (fp32) / 8-B (bf16) accesses, four rows in flight
// per lane.
//
// The column sums are deterministic: every workgroup owns a fixed row range (a function of the
// row count only), sums it per lane in a fixed order, folds its row lanes in LDS in a fixed
// order and writes one fp32 partial row to the workspace; a second launch adds the partials of
// each column in workgroup order in fp64.
#include "act.h"

namespace gnnea {

template <typename T, int V> struct ActVec;
template <typename T> struct ActVec<T, 4> {
  typedef typename Vec4<T>::raw raw;
  static __device__ __forceinline__ void get(const raw& r, float (&f)[4]) {
    const float4 v = Vec4<T>::get(r);
    f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
  }
  static __device__ __forceinline__ raw put(const float (&f)[4]) {
    return Vec4<T>::put(make_float4(f[0], f[1], f[2], f[3]));
  }
};
template <typename T> struct ActVec<T, 1> {
  typedef T raw;
  static __device__ __forceinline__ void get(const raw& r, float (&f)[1]) { f[0] = to_f32<T>(r); }
  static __device__ __forceinline__ raw put(const float (&f)[1]) { return from_f32<T>(f[0]); }
};

template <int ACT, typename T, int V>
__global__ __launch_bounds__(256) void k_act_rows(T* __restrict__ C, int64_t ldc, int64_t M,
                                                  int ng) {
  typedef ActVec<T, V> IO;
  const int64_t n = M * ng, stride = (int64_t)gridDim.x * 256;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n; t += stride) {
    const int64_t r = t / ng;
    const int g = (int)(t - r * ng);
    typename IO::raw* p = (typename IO::raw*)(C + r * ldc) + g;
    float f[V];
    IO::get(*p, f);
#pragma unroll
    for (int v = 0; v < V; ++v) f[v] = act_fwd<ACT>(f[v]);
    *p = IO::put(f);
  }
}

// One workgroup per fixed row range [r0, r1); column groups (V elements) in chunks of 256: the
// chunk's CG groups x RL = 256 / CG row lanes, each lane stepping RL rows, four rows in flight.
template <int ACT, typename T, int V>
__global__ __launch_bounds__(256) void k_act_bwd_colsum(const T* __restrict__ dY, int64_t lddy,
                                                        const T* __restrict__ Y, int64_t ldy,
                                                        int64_t n_rows, int D, int64_t rpb,
                                                        T* __restrict__ G, int64_t ldg,
                                                        float* __restrict__ part) {
  typedef ActVec<T, V> IO;
  typedef typename IO::raw raw;
  __shared__ float sh[256 * V];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  const int64_t r1 = r0 + rpb < n_rows ? r0 + rpb : n_rows;
  const int ng = D / V;
  for (int c0 = 0; c0 < ng; c0 += 256) {
    const int cgn = ng - c0 < 256 ? ng - c0 : 256;
    const int rl_n = 256 / cgn, rl = tid / cgn, cg = c0 + tid % cgn;
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    if (rl < rl_n) {
      auto one = [&](const raw& dr, const raw& yr, int64_t r) {
        float d[V], y[V], g[V];
        IO::get(dr, d);
        IO::get(yr, y);
#pragma unroll
        for (int v = 0; v < V; ++v) g[v] = d[v] * act_grad_from_out<ACT>(y[v]);
        const raw gr = IO::put(g);
        ((raw*)(G + r * ldg))[cg] = gr;
        IO::get(gr, g);  // the stored (rounded) values are what the bias gradient sums
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += g[v];
      };
      int64_t r = r0 + rl;
      for (; r + 3 * rl_n < r1; r += 4 * rl_n) {
        raw dr[4], yr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          dr[u] = ((const raw*)(dY + (r + u * rl_n) * lddy))[cg];
          yr[u] = ((const raw*)(Y + (r + u * rl_n) * ldy))[cg];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) one(dr[u], yr[u], r + u * rl_n);
      }
      for (; r < r1; r += rl_n)
        one(((const raw*)(dY + r * lddy))[cg], ((const raw*)(Y + r * ldy))[cg], r);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) sh[tid * V + v] = acc[v];
    __syncthreads();
    if (tid < cgn) {
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float s = 0.f;
        for (int q = 0; q < rl_n; ++q) s += sh[(q * cgn + tid) * V + v];
        part[(int64_t)blockIdx.x * D + (int64_t)(c0 + tid) * V + v] = s;
      }
    }
    __syncthreads();
  }
}

// 64 columns per workgroup; the 8 waves stride the partial rows (wave w: rows w, w + 8, ...,
// four independent fp64 sums per lane), combined in wave order through LDS: a fixed order
// (deterministic), with the loads of many rows in flight.  (One thread per column summing the
// 2048 rows in sequence took 0.79 ms: every row a dependent round trip.)
__global__ __launch_bounds__(512) void k_colsum_parts(const float* __restrict__ part, int nb,
                                                      int D, float* __restrict__ db) {
  __shared__ double red[8][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + lane;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  if (c < D) {
    int b = w;
    for (; b + 24 < nb; b += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s[u] += (double)part[(int64_t)(b + 8 * u) * D + c];
    }
    for (int u = 0; b < nb; b += 8, ++u) s[u & 3] += (double)part[(int64_t)b * D + c];
  }
  red[w][lane] = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  if (w == 0 && c < D) {
    double t = 0.0;
#pragma unroll
    for (int v = 0; v < 8; ++v) t += red[v][lane];
    db[c] = (float)t;
  }
}

// The non-concatenated GAT layer's head mean (layers/att_layers.py:89-91, torch.mean over the
// stacked heads): Y[i][d] = (sum_h X[i][h dh + d]) / heads, the sum in fp32 in head order, one
// rounding; backward dX[i][h dh + d] = dY[i][d] / heads.  (torch's mean on bf16 ran as an
// upcast copy, the reduction and a downcast copy per layer and direction.)
template <typename T>
__global__ __launch_bounds__(256) void k_head_mean(const T* __restrict__ X, int64_t ldx, int64_t n,
                                                   int heads, int dh, T* __restrict__ Y,
                                                   int64_t ldy) {
  const int64_t total = n * dh;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / dh;
    const int d = (int)(e - i * dh);
    const T* x = X + i * ldx + d;
    float s = 0.f;
    for (int h = 0; h < heads; ++h) s += to_f32<T>(x[(int64_t)h * dh]);
    Y[i * ldy + d] = from_f32<T>(s / (float)heads);
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_head_mean_bwd(const T* __restrict__ dY, int64_t ldy,
                                                       int64_t n, int heads, int dh,
                                                       T* __restrict__ dX, int64_t ldx) {
  const int64_t total = n * dh;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / dh;
    const int d = (int)(e - i * dh);
    const T v = from_f32<T>(to_f32<T>(dY[i * ldy + d]) / (float)heads);
    T* x = dX + i * ldx + d;
    for (int h = 0; h < heads; ++h) x[(int64_t)h * dh] = v;
  }
}

// ---- host side ----

static int act_grid(int64_t n) { return (int)(n / 256 + 1 < 8192 ? n / 256 + 1 : 8192); }

template <typename T>
static bool vec_ok(const void* p, int64_t ld, int64_t N) {
  constexpr uintptr_t al = 4 * sizeof(T) - 1;
  return N % 4 == 0 && ld % 4 == 0 && !(((uintptr_t)p) & al);
}

template <typename T>
static int act_rows_t(T* C, int64_t ldc, int64_t M, int64_t N, int act, hipStream_t s) {
  if (M < 0 || N < 0 || (M > 0 && ldc < N)) return GNNEA_EINVAL;
  if (M == 0 || N == 0 || act == GNNEA_ACT_IDENTITY) return 0;
  if (!C || N >= (1ll << 31)) return GNNEA_EINVAL;
  const bool v4 = vec_ok<T>(C, ldc, N);
  const int ng = (int)(v4 ? N / 4 : N);
  const int nb = act_grid(M * ng);
#define GNNEA_AR(A)                                                                              \
  if (v4) hipLaunchKernelGGL((k_act_rows<A, T, 4>), dim3(nb), dim3(256), 0, s, C, ldc, M, ng);   \
  else hipLaunchKernelGGL((k_act_rows<A, T, 1>), dim3(nb), dim3(256), 0, s, C, ldc, M, ng);
  switch (act) {
    case GNNEA_ACT_RELU: GNNEA_AR(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_AR(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_AR(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_AR(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_AR(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_AR
  GNNEA_LAUNCH_CHECK();
  return 0;
}

int act_rows_f32(float* C, int64_t ldc, int64_t M, int64_t N, int act, hipStream_t s) {
  return act_rows_t<float>(C, ldc, M, N, act, s);
}
int act_rows_bf16(bf16_t* C, int64_t ldc, int64_t M, int64_t N, int act, hipStream_t s) {
  return act_rows_t<bf16_t>(C, ldc, M, N, act, s);
}

// the row ranges: a function of the row count only (so the sums do not depend on the device)
static int64_t colsum_blocks(int64_t n_rows) {
  const int64_t nb = (n_rows + 63) / 64;
  return nb < 2048 ? (nb > 0 ? nb : 1) : 2048;
}

template <typename T>
static int act_bwd_colsum_t(const T* dY, int64_t lddy, const T* Y, int64_t ldy, int64_t n_rows,
                            int32_t D, int act, T* G, int64_t ldg, float* db, void* ws,
                            int64_t ws_bytes, hipStream_t s) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (D == 0) return 0;
  if (!db) return GNNEA_EINVAL;
  if (n_rows == 0) return hipMemsetAsync(db, 0, (size_t)D * 4, s) == hipSuccess ? 0 : GNNEA_EINVAL;
  if (!dY || !Y || !G || lddy < D || ldy < D || ldg < D) return GNNEA_EINVAL;
  const int64_t nb = colsum_blocks(n_rows);
  if (!ws || ws_bytes < nb * D * 4) return GNNEA_EWORKSPACE;
  const int64_t rpb = (n_rows + nb - 1) / nb;
  const bool v4 = vec_ok<T>(dY, lddy, D) && vec_ok<T>(Y, ldy, D) && vec_ok<T>(G, ldg, D);
  float* part = (float*)ws;
#define GNNEA_ABC(A)                                                                              \
  if (v4) hipLaunchKernelGGL((k_act_bwd_colsum<A, T, 4>), dim3((unsigned)nb), dim3(256), 0, s,   \
                             dY, lddy, Y, ldy, n_rows, (int)D, rpb, G, ldg, part);               \
  else hipLaunchKernelGGL((k_act_bwd_colsum<A, T, 1>), dim3((unsigned)nb), dim3(256), 0, s, dY,  \
                          lddy, Y, ldy, n_rows, (int)D, rpb, G, ldg, part);
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_ABC(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_ABC(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_ABC(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_ABC(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_ABC(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_ABC(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_ABC
  GNNEA_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_colsum_parts, dim3((D + 63) / 64), dim3(512), 0, s, part, (int)nb,
                     (int)D, db);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int act_fwd_t(const T* X, T* Y, int64_t n, int act, hipStream_t s) {
  if (n < 0) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!X || !Y) return GNNEA_EINVAL;
  if (X != Y && hipMemcpyAsync(Y, X, (size_t)n * sizeof(T), hipMemcpyDeviceToDevice, s) !=
                    hipSuccess)
    return GNNEA_EINVAL;
  if (act == GNNEA_ACT_IDENTITY) return 0;
  // as n / 4 rows of four when it vectorises, else n rows of one
  if (vec_ok<T>(Y, 4, n)) return act_rows_t<T>(Y, 4, n / 4, 4, act, s);
  return act_rows_t<T>(Y, 1, n, 1, act, s);
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_act_fwd_f32(const float* X, float* Y, int64_t n, int act, void* stream) {
  return act_fwd_t<float>(X, Y, n, act, (hipStream_t)stream);
}

extern "C" int gnnea_act_fwd_bf16(const void* X, void* Y, int64_t n, int act, void* stream) {
  return act_fwd_t<bf16_t>((const bf16_t*)X, (bf16_t*)Y, n, act, (hipStream_t)stream);
}

extern "C" int64_t gnnea_act_bwd_colsum_ws_bytes(int64_t n_rows, int32_t D) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  return colsum_blocks(n_rows) * D * 4;
}

extern "C" int gnnea_act_bwd_colsum_f32(const float* dY, int64_t lddy, const float* Y,
                                        int64_t ldy, int64_t n_rows, int32_t D, int act, float* G,
                                        int64_t ldg, float* db, void* ws, int64_t ws_bytes,
                                        void* stream) {
  return act_bwd_colsum_t<float>(dY, lddy, Y, ldy, n_rows, D, act, G, ldg, db, ws, ws_bytes,
                                 (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_colsum_bf16(const void* dY, int64_t lddy, const void* Y,
                                         int64_t ldy, int64_t n_rows, int32_t D, int act, void* G,
                                         int64_t ldg, float* db, void* ws, int64_t ws_bytes,
                                         void* stream) {
  return act_bwd_colsum_t<bf16_t>((const bf16_t*)dY, lddy, (const bf16_t*)Y, ldy, n_rows, D, act,
                                  (bf16_t*)G, ldg, db, ws, ws_bytes, (hipStream_t)stream);
}

template <typename T>
static int head_mean_t(const T* X, int64_t ldx, int64_t n, int heads, int dh, T* Y, int64_t ldy,
                       int bwd, hipStream_t s) {
  if (n < 0 || heads < 1 || dh < 1) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!X || !Y) return GNNEA_EINVAL;
  // forward: X [n][heads dh] (ld ldx), Y [n][dh] (ld ldy); backward: X = dY [n][dh], Y = dX
  if (bwd ? (ldx < dh || ldy < (int64_t)heads * dh) : (ldx < (int64_t)heads * dh || ldy < dh))
    return GNNEA_EINVAL;
  const int nb = act_grid(n * dh);
  if (bwd)
    hipLaunchKernelGGL(k_head_mean_bwd<T>, dim3(nb), dim3(256), 0, s, X, ldx, n, heads, dh, Y, ldy);
  else
    hipLaunchKernelGGL(k_head_mean<T>, dim3(nb), dim3(256), 0, s, X, ldx, n, heads, dh, Y, ldy);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_head_mean_f32(const float* X, int64_t ldx, int64_t n, int32_t heads,
                                   int32_t dh, float* Y, int64_t ldy, int bwd, void* stream) {
  return head_mean_t<float>(X, ldx, n, heads, dh, Y, ldy, bwd, (hipStream_t)stream);
}
extern "C" int gnnea_head_mean_bf16(const void* X, int64_t ldx, int64_t n, int32_t heads,
                                    int32_t dh, void* Y, int64_t ldy, int bwd, void* stream) {
  return head_mean_t<bf16_t>((const bf16_t*)X, ldx, n, heads, dh, (bf16_t*)Y, ldy, bwd,
                             (hipStream_t)stream);
}
