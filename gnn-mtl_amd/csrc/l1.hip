// §8f #1: L1 (cityblock) distances, hard-negative top-k and Hits@k ranks on the device.
// Replaces BaseModel.get_neg (models/models_ea.py:19-30: scipy cdist 'cityblock' + argsort
// [1:k+1]), get_hits (utils/eval_utils.py:71-98: cdist + argsort rank of the true match, both
// directions) and the cdist of UEAModel.generate_pairs (models/models_ea.py:143-167).
//
// Exactness: scipy casts fp32 inputs to fp64 and sums |u_d - v_d| over d in order.  Every term
// is exact in fp64 and the kernels accumulate the same terms in the same order, so distances are
// bit-identical to scipy's; ranks / selections then match exactly, ties excepted (numpy's argsort
// order among equal distances is unspecified; here ties go to the lower index).
//
// Distance tiles: 256 threads, 64 queries x 64 candidates per workgroup, each thread 4 x 4 fp64
// accumulators, 32-dim slabs of both operands staged through LDS as fp32 (k-major, 16-B reads).
// L1 has no matrix-core form (it is not a dot product); this is VALU fp64 work.
#include "common.h"

namespace gnnea {

constexpr int LT = 64, LK = 32, LLD = LT + 4;

struct L1Tile {
  double acc[4][4];
};

// Accumulate the 64x64 tile (q0.., x0..) of sum_d |Q[q][d] - X[x][d]| over all D dims.
__device__ __forceinline__ void l1_tile(const float* __restrict__ Q, int64_t ldq, int nq, int q0,
                                        const float* __restrict__ X, int64_t ldx, int nx, int x0,
                                        int D, float* Qs, float* Xs, L1Tile& t) {
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) t.acc[a][b] = 0.0;
  for (int d0 = 0; d0 < D; d0 += LK) {
    // stage: 64 rows x 32 dims of each operand; thread -> (row = tid / 4, 8 dims)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = tid >> 2, dd = (tid & 3) * 8;
      const float* src = h == 0 ? Q : X;
      const int64_t ld = h == 0 ? ldq : ldx;
      const int base = h == 0 ? q0 : x0, lim = h == 0 ? nq : nx;
      float* dst = h == 0 ? Qs : Xs;
      const int gr = base + row;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int gd = d0 + dd + e;
        dst[(dd + e) * LLD + row] = (gr < lim && gd < D) ? src[(int64_t)gr * ld + gd] : 0.f;
      }
    }
    __syncthreads();
    const int kmax = min(LK, D - d0);
    for (int k = 0; k < kmax; ++k) {
      const float4 qv = *(const float4*)(Qs + k * LLD + 4 * ty);
      const float4 xv = *(const float4*)(Xs + k * LLD + 4 * tx);
      const double q[4] = {(double)qv.x, (double)qv.y, (double)qv.z, (double)qv.w};
      const double x[4] = {(double)xv.x, (double)xv.y, (double)xv.z, (double)xv.w};
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) t.acc[a][b] += fabs(q[a] - x[b]);
    }
    __syncthreads();
  }
}

// keys[q][x] = (float)dist (round-to-nearest is monotone: selection on keys keeps the exact set)
__global__ __launch_bounds__(256) void k_l1_keys(const float* __restrict__ Q, int64_t ldq, int nq,
                                                 const float* __restrict__ X, int64_t ldx, int nx,
                                                 int D, float* __restrict__ keys, int64_t ldk) {
  __shared__ __attribute__((aligned(16))) float Qs[LK * LLD];
  __shared__ __attribute__((aligned(16))) float Xs[LK * LLD];
  const int x0 = blockIdx.x * LT, q0 = blockIdx.y * LT;
  L1Tile t;
  l1_tile(Q, ldq, nq, q0, X, ldx, nx, x0, D, Qs, Xs, t);
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q = q0 + 4 * ty + a;
    if (q >= nq) continue;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int x = x0 + 4 * tx + b;
      if (x < nx) keys[(int64_t)q * ldk + x] = (float)t.acc[a][b];
    }
  }
}

// exact fp64 distance of one (query, candidate) pair, sequential over d (scipy's order)
__device__ __forceinline__ double l1_exact(const float* __restrict__ q, const float* __restrict__ x,
                                           int D) {
  double s = 0.0;
  for (int d = 0; d < D; ++d) s += fabs((double)q[d] - (double)x[d]);
  return s;
}

__global__ void k_l1_pairs(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                           int64_t ldb, int n, int D, double* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = l1_exact(A + (int64_t)i * lda, B + (int64_t)i * ldb, D);
}

// rank[q] += #{x : d(q,x) < diag[q]  or (d == diag[q] and x_off + x < q)}   (stable-sort
// position; X a block of the candidates starting at candidate x_off)
__global__ __launch_bounds__(256) void k_l1_rank(const float* __restrict__ Q, int64_t ldq, int nq,
                                                 const float* __restrict__ X, int64_t ldx, int nx,
                                                 int D, const double* __restrict__ diag, int x_off,
                                                 int* __restrict__ rank) {
  __shared__ __attribute__((aligned(16))) float Qs[LK * LLD];
  __shared__ __attribute__((aligned(16))) float Xs[LK * LLD];
  __shared__ int cnt[LT];
  const int x0 = blockIdx.x * LT, q0 = blockIdx.y * LT;
  if (threadIdx.x < LT) cnt[threadIdx.x] = 0;
  L1Tile t;
  l1_tile(Q, ldq, nq, q0, X, ldx, nx, x0, D, Qs, Xs, t);
  const int ty = threadIdx.x >> 4, tx = threadIdx.x & 15;
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q = q0 + 4 * ty + a;
    if (q >= nq) continue;
    const double dq = diag[q];
    int c = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int x = x0 + 4 * tx + b;
      const double v = t.acc[a][b];
      c += (x < nx && (v < dq || (v == dq && x_off + x < q))) ? 1 : 0;
    }
    if (c) atomicAdd(&cnt[4 * ty + a], c);
  }
  __syncthreads();
  if (threadIdx.x < LT && q0 + threadIdx.x < nq && cnt[threadIdx.x])
    atomicAdd(&rank[q0 + threadIdx.x], cnt[threadIdx.x]);
}

// ---- per-row top-K by radix select on the fp32 keys, then exact (fp64, index) order ------- //
// Rounding to fp32 is monotone, so the K smallest exact distances are among the keys <= the K-th
// smallest key `thr`.  Those < thr (fewer than K) are collected unordered; those == thr in index
// order until kSelCap is full (exact duplicates therefore keep the lowest indices).  Only more than
// kSelCap - K distinct distances inside one fp32 ulp can truncate the set; such rows are counted
// in *overflow.
constexpr int kSelCap = 1024;

__global__ __launch_bounds__(256) void k_topk_rows(const float* __restrict__ keys, int64_t ldk,
                                                   int nx, int K, const float* __restrict__ Q,
                                                   int64_t ldq, const float* __restrict__ X,
                                                   int64_t ldx, int D, int skip,
                                                   int64_t* __restrict__ out_idx,
                                                   double* __restrict__ out_dist, int ldo,
                                                   int* __restrict__ overflow) {
  __shared__ int hist[256];
  __shared__ unsigned prefix_s, kth_s;
  __shared__ int nsel, wcnt[4];
  __shared__ double sd[kSelCap];
  __shared__ int si[kSelCap];
  const int qi = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const unsigned* kr = (const unsigned*)(keys + (int64_t)qi * ldk);
  // radix select of the K-th smallest key (non-negative floats: uint order == float order)
  unsigned prefix = 0, mask = 0;
  int k = K;
  for (int shift = 24; shift >= 0; shift -= 8) {
    hist[tid] = 0;
    __syncthreads();
    for (int x = tid; x < nx; x += 256) {
      const unsigned u = kr[x];
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1);
    }
    __syncthreads();
    if (tid == 0) {
      int acc = 0, b = 0;
      for (; b < 255; ++b) {
        if (acc + hist[b] >= k) break;
        acc += hist[b];
      }
      prefix_s = prefix | ((unsigned)b << shift);
      kth_s = (unsigned)(k - acc);
    }
    __syncthreads();
    prefix = prefix_s;
    k = (int)kth_s;
    mask |= 255u << shift;
  }
  const unsigned thr = prefix;
  if (tid == 0) nsel = 0;
  __syncthreads();
  const float* qrow = Q + (int64_t)qi * ldq;
  for (int x = tid; x < nx; x += 256)
    if (kr[x] < thr) {
      const int s = atomicAdd(&nsel, 1);
      si[s] = x;
    }
  __syncthreads();
  int n = nsel;  // < K
  bool full = false;
  for (int x0 = 0; x0 < nx && !full; x0 += 256) {  // ties at thr, in index order
    const int x = x0 + tid;
    const bool f = x < nx && kr[x] == thr;
    const unsigned long long bal = __ballot(f);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wcnt[w] = __popcll(bal);
    __syncthreads();
    int off = n;
    for (int v = 0; v < w; ++v) off += wcnt[v];
    const int tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    if (f && off + before < kSelCap) si[off + before] = x;
    full = n + tot > kSelCap;
    n = min(n + tot, kSelCap);
    __syncthreads();
  }
  if (full && tid == 0 && overflow) atomicAdd(overflow, 1);
  for (int s = tid; s < n; s += 256) sd[s] = l1_exact(qrow, X + (int64_t)si[s] * ldx, D);
  // bitonic sort of (dist, index) over the padded power of two
  int np = 1;
  while (np < n) np <<= 1;
  for (int s = n + tid; s < np; s += 256) {
    sd[s] = INFINITY;
    si[s] = 0x7fffffff;
  }
  __syncthreads();
  for (int size = 2; size <= np; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int s = tid; s < np; s += 256) {
        const int p = s ^ stride;
        if (p > s) {
          const bool up = (s & size) == 0;
          const bool gt = sd[s] > sd[p] || (sd[s] == sd[p] && si[s] > si[p]);
          if (gt == up) {
            const double td = sd[s];
            sd[s] = sd[p];
            sd[p] = td;
            const int ti = si[s];
            si[s] = si[p];
            si[p] = ti;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int s = tid; s + skip < K; s += 256) {
    out_idx[(int64_t)qi * ldo + s] = si[s + skip];
    if (out_dist) out_dist[(int64_t)qi * ldo + s] = sd[s + skip];
  }
}

// Per-term L1 distances over a column block (the column-sharded EA loss, gnnea/dist_loss.py):
// out[j] = sum_d |X[a_j][d] - X[b_j][d]| in fp64 (every term exact, summed in a fixed lane order),
// LPT lanes per term (LPT | 64, so a term's lanes leave together), 4-B loads, consecutive lanes on
// consecutive columns of the two gathered rows.
template <int LPT>
__global__ __launch_bounds__(256) void k_l1_terms(const float* __restrict__ X, int64_t ldx, int D,
                                                  int64_t n, const int64_t* __restrict__ a,
                                                  const int64_t* __restrict__ b,
                                                  double* __restrict__ out) {
  const int64_t term = ((int64_t)blockIdx.x * 256 + threadIdx.x) / LPT;
  if (term >= n) return;
  const int l = threadIdx.x % LPT;
  const float* xa = X + a[term] * ldx;
  const float* xb = X + b[term] * ldx;
  double s = 0.0;
  for (int d = l; d < D; d += LPT) s += fabs((double)xa[d] - (double)xb[d]);
#pragma unroll
  for (int o = LPT / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, LPT);
  if (l == 0) out[term] = s;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_l1_terms_f32(const float* X, int64_t ldx, int32_t D, int64_t n,
                                  const int64_t* a, const int64_t* b, double* out, void* stream) {
  if (n < 0 || D < 0 || ldx < D) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!X || !a || !b || !out) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const int lpt = D <= 16 ? 16 : D <= 64 ? 32 : 64;  // lanes per term
  const int64_t nb = (n * lpt + 255) / 256;
  if (nb >= (1ll << 31)) return GNNEA_EINVAL;
  if (lpt == 16)
    hipLaunchKernelGGL(k_l1_terms<16>, dim3((unsigned)nb), dim3(256), 0, s, X, ldx, D, n, a, b, out);
  else if (lpt == 32)
    hipLaunchKernelGGL(k_l1_terms<32>, dim3((unsigned)nb), dim3(256), 0, s, X, ldx, D, n, a, b, out);
  else
    hipLaunchKernelGGL(k_l1_terms<64>, dim3((unsigned)nb), dim3(256), 0, s, X, ldx, D, n, a, b, out);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_l1_keys_f32(const float* Q, int64_t ldq, int32_t nq, const float* X,
                                 int64_t ldx, int32_t nx, int32_t D, float* keys, int64_t ldk,
                                 void* stream) {
  if (nq < 0 || nx < 0 || D < 0) return GNNEA_EINVAL;
  if (nq == 0 || nx == 0) return 0;
  if (!Q || !X || !keys || ldq < D || ldx < D || ldk < nx) return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_l1_keys, dim3(div_up(nx, LT), div_up(nq, LT)), dim3(256), 0,
                     (hipStream_t)stream, Q, ldq, nq, X, ldx, nx, D, keys, ldk);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_l1_pairs_f32(const float* A, int64_t lda, const float* B, int64_t ldb,
                                  int32_t n, int32_t D, double* out, void* stream) {
  if (n < 0 || D < 0) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!A || !B || !out || lda < D || ldb < D) return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_l1_pairs, dim3(div_up(n, 256)), dim3(256), 0, (hipStream_t)stream, A, lda,
                     B, ldb, n, D, out);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_l1_rank_f32(const float* Q, int64_t ldq, int32_t nq, const float* X,
                                 int64_t ldx, int32_t nx, int32_t D, const double* diag,
                                 int32_t* rank, void* stream) {
  if (nq < 0 || nx < 0 || D < 0) return GNNEA_EINVAL;
  if (nq == 0) return 0;
  if (!Q || !X || !diag || !rank || ldq < D || ldx < D) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  GNNEA_HIP(hipMemsetAsync(rank, 0, sizeof(int32_t) * nq, s));
  if (nx == 0) return 0;
  hipLaunchKernelGGL(k_l1_rank, dim3(div_up(nx, LT), div_up(nq, LT)), dim3(256), 0, s, Q, ldq, nq,
                     X, ldx, nx, D, diag, 0, rank);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// The count over one block of the candidates, [x_off, x_off + nx) (the rank's share of get_hits
// across GPUs, gnnea/dist_search.py): the per-block counts sum to gnnea_l1_rank_f32's.
extern "C" int gnnea_l1_rank_range_f32(const float* Q, int64_t ldq, int32_t nq, const float* X,
                                       int64_t ldx, int32_t nx, int32_t D, const double* diag,
                                       int32_t x_off, int32_t* rank, void* stream) {
  if (nq < 0 || nx < 0 || D < 0 || x_off < 0) return GNNEA_EINVAL;
  if (nq == 0) return 0;
  if (!Q || !diag || !rank || ldq < D || (nx > 0 && (!X || ldx < D))) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  GNNEA_HIP(hipMemsetAsync(rank, 0, sizeof(int32_t) * nq, s));
  if (nx == 0) return 0;
  hipLaunchKernelGGL(k_l1_rank, dim3(div_up(nx, LT), div_up(nq, LT)), dim3(256), 0, s, Q, ldq, nq,
                     X, ldx, nx, D, diag, x_off, rank);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_topk_rows_f32(const float* keys, int64_t ldk, int32_t nq, int32_t nx,
                                   int32_t K, const float* Q, int64_t ldq, const float* X,
                                   int64_t ldx, int32_t D, int32_t skip, int64_t* out_idx,
                                   double* out_dist, int32_t ldo, int32_t* overflow,
                                   void* stream) {
  if (nq < 0 || nx < 0 || K < 0 || D < 0 || skip < 0 || skip > K) return GNNEA_EINVAL;
  if (nq == 0 || K == skip) return 0;
  if (K > nx || K > kSelCap / 2) return GNNEA_EINVAL;
  if (!keys || !Q || !X || !out_idx || ldk < nx || ldq < D || ldx < D || ldo < K - skip)
    return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_topk_rows, dim3(nq), dim3(256), 0, (hipStream_t)stream, keys, ldk, nx, K,
                     Q, ldq, X, ldx, D, skip, out_idx, out_dist, ldo, overflow);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
