// Dense projection on MFMA with bf16 operands (cfg-5 storage): C = op(A)·op(B) (+ bias)
// (+ beta*C), bf16 in, fp32 accumulate, C written bf16 (rounded once) or fp32.
// Same call sites as gemm.hip (nn.Linear, torch.mm(input, W), torch.spmm(x, kernel_gate)).
//
// v_mfma_f32_32x32x16_bf16: lane l (r = l & 31, h = l >> 5) supplies A[row r][k = 8h + j] and
// B[k = 8h + j][col r], j = 0..7, as one 16-B fragment; C/D as the f32 form.  Block tile
// BM = 64 rows x BN = 64*WT columns (the whole 300-wide output at WT = 5), BK = 32 (two MFMA
// k-steps); 4 waves in 2 x 2, each 32 x 32*WT.  Both operands are staged in double-buffered LDS
// as [row][k] with K contiguous (row stride 40 elements = 80 B: 16-B aligned fragments, rows
// spread over the banks), so every fragment is ONE ds_read_b128.  An operand whose rows are
// contiguous in memory (op(X) = X^T) is transposed while it is written to LDS (8 2-B stores per
// 16-B chunk, k fastest across the lanes so each store instruction covers 32 consecutive k of
// two 8-row groups: conflict-free; row-group-fastest lanes hit 2 banks, 32-way).  Next tile's global loads are in flight under the current tile's MFMAs.
// Split-K for the weight gradients as in gemm.hip: fp32 slabs, fixed-order reduction.
#include "common.h"

#include <stdlib.h>

#include <type_traits>

namespace gnnea {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16_b __attribute__((ext_vector_type(16)));

constexpr int HBM = 64, HBK = 32, HLD = HBK + 8;
#ifndef GNNEA_BF16_TRANS_QUADS
#define GNNEA_BF16_TRANS_QUADS 1
#endif
constexpr bool TRANS_QUADS = GNNEA_BF16_TRANS_QUADS;  // 0: HLoader's 2-B transposing stores

__device__ __forceinline__ bf16_t u4_elem(const uint4& v, int e) {
  const uint32_t w = e < 2 ? v.x : e < 4 ? v.y : e < 6 ? v.z : v.w;
  return (bf16_t)((e & 1) ? (w >> 16) : (w & 0xffffu));
}

// ROWS x HBK tile of op(X) (bf16) in registers, 8-element chunks; rows >= nrows or k >= kend
// read as 0.  op(X)[row][k] = X[row][k] (K_CONTIG) or X[k][row].  VEC: each chunk is two 8-B
// loads of 4 elements (ld and the contiguous extent % 4 == 0, 8-B aligned base: every half is
// entirely inside or outside the operand -- K = 300 rows of 600 B qualify, 16-B loads would not).
template <bool K_CONTIG, int ROWS, bool VEC>
struct HLoader {
  static constexpr int NC = ROWS * HBK / 8 / 256;
  uint4 r[NC];
  __device__ void load(const bf16_t* __restrict__ X, int64_t ld, int row0, int nrows, int k0,
                       int kend, int tid) {
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int idx = tid + 256 * q;
      int row, k;
      if (K_CONTIG) { row = idx / (HBK / 8); k = (idx % (HBK / 8)) * 8; }
      else { k = idx % HBK; row = (idx / HBK) * 8; }
      const int gr = row0 + row, gk = k0 + k;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (VEC) {
        uint2 lo = make_uint2(0u, 0u), hi = make_uint2(0u, 0u);
        if (K_CONTIG) {
          if (gr < nrows) {
            const bf16_t* p = X + (int64_t)gr * ld + gk;
            if (gk < kend) lo = *(const uint2*)p;
            if (gk + 4 < kend) hi = *(const uint2*)(p + 4);
          }
        } else {
          if (gk < kend) {
            const bf16_t* p = X + (int64_t)gk * ld + gr;
            if (gr < nrows) lo = *(const uint2*)p;
            if (gr + 4 < nrows) hi = *(const uint2*)(p + 4);
          }
        }
        v = make_uint4(lo.x, lo.y, hi.x, hi.y);
      } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int rr = K_CONTIG ? gr : gr + e, kk = K_CONTIG ? gk + e : gk;
          const uint32_t x = (rr < nrows && kk < kend)
                                 ? (K_CONTIG ? X[(int64_t)rr * ld + kk] : X[(int64_t)kk * ld + rr])
                                 : 0u;
          w[e >> 1] |= x << (16 * (e & 1));
        }
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      r[q] = v;
    }
  }
  __device__ void store(bf16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NC; ++q) {
      const int idx = tid + 256 * q;
      if (K_CONTIG) {
        const int row = idx / (HBK / 8), k = (idx % (HBK / 8)) * 8;
        *(uint4*)(S + row * HLD + k) = r[q];
      } else {
        const int k = idx % HBK, row = (idx / HBK) * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) S[(row + e) * HLD + k] = u4_elem(r[q], e);
      }
    }
  }
};

// ROWS x HBK tile of op(X) = X^T (rows contiguous in memory, VEC layout) in registers as quads
// of 4 k x 8 rows (four 16-B row-runs, each two 8-B loads), written to LDS as 8 ds_write_b64 of
// 4 consecutive k per row: a quarter of the store instructions of HLoader's 2-B transposing
// stores.  Taken for the wide operand only (ROWS >= 256: the B tile): on the 64-row A tile the
// 64 quads fall to one wave, whose longer load/store chain every k-step then waits on (dW =
// dY^T X with both tall operands quad-loaded measured 3.7x slower), and only without split-K
// (QT: the split-K weight gradients, 800 k-steps per workgroup at 2M rows, measured 2.4x slower
// with the quad B tile as well; dX = dY W, K = 300, 1.91 -> 1.37 ms at 2M rows with it).
template <int ROWS>
struct HLoaderT {
  static constexpr int NQ = ROWS * HBK / 32;     // quads per tile
  static constexpr int NQT = (NQ + 255) / 256;   // per thread (the last pass partly idle)
  uint4 r[NQT][4];
  __device__ void load(const bf16_t* __restrict__ X, int64_t ld, int row0, int nrows, int k0,
                       int kend, int tid) {
#pragma unroll
    for (int q = 0; q < NQT; ++q) {
      const int idx = tid + 256 * q;
      const int k = (idx % (HBK / 4)) * 4, gr = row0 + (idx / (HBK / 4)) * 8;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        uint2 lo = make_uint2(0u, 0u), hi = make_uint2(0u, 0u);
        const int gk = k0 + k + kk;
        if ((NQ % 256 == 0 || idx < NQ) && gk < kend) {
          const bf16_t* p = X + (int64_t)gk * ld + gr;
          if (gr < nrows) lo = *(const uint2*)p;
          if (gr + 4 < nrows) hi = *(const uint2*)(p + 4);
        }
        r[q][kk] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    }
  }
  __device__ void store(bf16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NQT; ++q) {
      const int idx = tid + 256 * q;
      if (NQ % 256 != 0 && idx >= NQ) continue;
      const int k = (idx % (HBK / 4)) * 4, row = (idx / (HBK / 4)) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t lo = (uint32_t)u4_elem(r[q][0], e) | ((uint32_t)u4_elem(r[q][1], e) << 16);
        const uint32_t hi = (uint32_t)u4_elem(r[q][2], e) | ((uint32_t)u4_elem(r[q][3], e) << 16);
        *(uint2*)(S + (row + e) * HLD + k) = make_uint2(lo, hi);
      }
    }
  }
};

template <bool K_CONTIG, int ROWS, bool VEC, bool QT>
using HLoad = typename std::conditional<!K_CONTIG && VEC && QT && TRANS_QUADS && ROWS >= 256,
                                        HLoaderT<ROWS>,
                                        HLoader<K_CONTIG, ROWS, VEC>>::type;

// Output addressing: element (row, col) at (col / 128)·cs + row·ldc + col % 128.  cs = 128 is the
// plain row-major matrix; ldc = 128, cs = n·128 the bf16 slice-major table (256-B slices) that
// gnnea_spmm_sliced_bf16 gathers from.
__device__ __forceinline__ int64_t c_index_bf(int64_t row, int64_t col, int64_t ldc, int64_t cs) {
  return (col >> 7) * cs + row * ldc + (col & 127);
}

template <int TA, int TB, int WT, bool VEC, typename TC, int EPI = 0, bool QT = false>
__global__ __launch_bounds__(256) void k_gemm_bf16(int M, int N, int K,
                                                   const bf16_t* __restrict__ A, int64_t lda,
                                                   const bf16_t* __restrict__ B, int64_t ldb,
                                                   const float* __restrict__ bias, float beta,
                                                   TC* __restrict__ C, int64_t ldc, int64_t cs,
                                                   int k_per_split, float* __restrict__ slab,
                                                   int tiles_n) {
  constexpr int BN = 64 * WT;
  constexpr bool AK = TA == 0, BKc = TB == 1;  // operand contiguous along K?
  constexpr int SA = HBM * HLD, SB = BN * HLD;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (SA + SB)];
  auto As = [&](int b) { return smem + b * SA; };
  auto Bs = [&](int b) { return smem + 2 * SA + b * SB; };

  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = t_id % tiles_n, bm = t_id / tiles_n;
  const int m0 = bm * HBM, n0 = bn * BN;
  const int split = blockIdx.y;
  const int kb = split * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int kh = lane >> 5, li = lane & 31;

  f32x16_b acc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  HLoad<AK, HBM, VEC, QT> la;
  HLoad<BKc, BN, VEC, QT> lb;
  const int nsteps = ke > kb ? (ke - kb + HBK - 1) / HBK : 0;
  if (nsteps > 0) {
    la.load(A, lda, m0, M, kb, ke, tid);
    lb.load(B, ldb, n0, N, kb, ke, tid);
    la.store(As(0), tid);
    lb.store(Bs(0), tid);
    __syncthreads();
  }
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {  // in flight under the MFMAs below
      la.load(A, lda, m0, M, kb + (s + 1) * HBK, ke, tid);
      lb.load(B, ldb, n0, N, kb + (s + 1) * HBK, ke, tid);
    }
    const bf16_t* a_s = As(cur);
    const bf16_t* b_s = Bs(cur);
#pragma unroll
    for (int ks = 0; ks < HBK; ks += 16) {
      const bf16x8 a = *(const bf16x8*)(a_s + (wm * 32 + li) * HLD + ks + 8 * kh);
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        const bf16x8 b = *(const bf16x8*)(b_s + (wn * 32 * WT + t * 32 + li) * HLD + ks + 8 * kh);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[t], 0, 0, 0);
      }
    }
    if (more) {
      la.store(As(cur ^ 1), tid);
      lb.store(Bs(cur ^ 1), tid);
    }
    __syncthreads();
  }

  // epilogue: 32x32 C/D map  col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  if constexpr (EPI == 1) {
    // bf16 C, no split, beta = 0, 8-B aligned rows (host-checked): the tile is rounded into LDS
    // (free after the loop's last barrier; [64][BN + 8] bf16 <= the operand buffers) and leaves
    // as 8-B row chunks, consecutive lanes on consecutive chunks of a row, instead of one 2-B
    // store per element per lane
    constexpr int TLD = BN + 8;
    bf16_t* T = smem;
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      const int cl = wn * 32 * WT + t * 32 + li;
      const float bv = (bias && n0 + cl < N) ? bias[n0 + cl] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        T[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh) * TLD + cl] = from_f32<bf16_t>(acc[t][r] + bv);
    }
    __syncthreads();
    for (int idx = tid; idx < HBM * (BN / 4); idx += 256) {
      const int rl = idx / (BN / 4), c4 = idx - rl * (BN / 4);
      const int row = m0 + rl, col = n0 + 4 * c4;
      if (row >= M || col >= N) continue;
      const bf16_t* src = T + rl * TLD + 4 * c4;
      bf16_t* dst = (bf16_t*)C + c_index_bf(row, col, ldc, cs);
      if (col + 4 <= N) {
        *(uint2*)dst = *(const uint2*)src;
      } else {
        for (int e = 0; col + e < N; ++e) dst[e] = src[e];
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < WT; ++t) {
    const int col = n0 + wn * 32 * WT + t * 32 + li;
    if (col >= N) continue;
    const float bv = (bias && !slab) ? bias[col] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * kh;
      if (row >= M) continue;
      const float v = acc[t][r];
      if (slab) {
        slab[((int64_t)split * M + row) * N + col] = v;
      } else {
        float o = v + bv;
        TC* cp = C + c_index_bf(row, col, ldc, cs);
        if (beta != 0.f) o += beta * to_f32<TC>(*cp);
        *cp = from_f32<TC>(o);
      }
    }
  }
}

// fixed-order reduction of the split-K slabs into C (bf16 or fp32)
template <typename TC>
__global__ void k_gemm_bf16_reduce(int M, int N, int splits, const float* __restrict__ slab,
                                   const float* __restrict__ bias, float beta,
                                   TC* __restrict__ C, int64_t ldc, int64_t cs) {
  const int64_t n = (int64_t)M * N;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    float a = 0.f, b = 0.f;
    int q = 0;
    for (; q + 2 <= splits; q += 2) {  // two slabs in flight
      a += slab[(int64_t)q * n + t];
      b += slab[(int64_t)(q + 1) * n + t];
    }
    if (q < splits) a += slab[(int64_t)q * n + t];
    float s = a + b;
    const int64_t row = t / N, col = t - row * N;
    if (bias) s += bias[col];
    TC* c = C + c_index_bf(row, col, ldc, cs);
    if (beta != 0.f) s += beta * to_f32<TC>(*c);
    *c = from_f32<TC>(s);
  }
}

static int bf16_wt(int64_t N) {
  const int64_t wt = (N + 63) / 64;
  return (int)(wt < 1 ? 1 : (wt > 5 ? 5 : wt));
}

static int bf16_splits(int64_t M, int64_t N, int64_t K, int64_t ws_bytes) {
  const int64_t bn = 64 * bf16_wt(N);
  const int64_t tiles = ((M + HBM - 1) / HBM) * ((N + bn - 1) / bn);
  if (tiles >= 512 || K < 8 * HBK) return 1;
  int64_t s = (384 + tiles - 1) / tiles;
  const int64_t by_k = K / (8 * HBK);
  if (s > by_k) s = by_k;
  if (s > 256) s = 256;
  while (s > 1 && s * M * N * 4 > ws_bytes) --s;
  return (int)(s < 1 ? 1 : s);
}

static bool bf16_lds_epilogue() {
  static const bool on = [] {  // A/B comparison only (GNNEA_BF16_EPI=0: per-element stores)
    const char* e = getenv("GNNEA_BF16_EPI");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int TA, int TB, int WT, typename TC>
static void launch_bf16_wt(dim3 grid, hipStream_t s, bool vec, int M, int N, int K,
                           const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                           const float* bias, float beta, TC* C, int64_t ldc, int64_t cs,
                           int kps, float* slab, int tiles_n) {
  if constexpr (std::is_same<TC, bf16_t>::value) {
    if (vec && !slab && beta == 0.f && (((uintptr_t)C) & 7) == 0 && ldc % 4 == 0 &&
        cs % 4 == 0 && bf16_lds_epilogue()) {
      hipLaunchKernelGGL((k_gemm_bf16<TA, TB, WT, true, TC, 1, true>), grid, dim3(256), 0, s, M,
                         N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
      return;
    }
  }
  if (vec && !slab && TB == 0) {
    hipLaunchKernelGGL((k_gemm_bf16<TA, TB, WT, true, TC, 0, true>), grid, dim3(256), 0, s, M, N,
                       K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
    return;
  }
  if (vec)
    hipLaunchKernelGGL((k_gemm_bf16<TA, TB, WT, true, TC>), grid, dim3(256), 0, s, M, N, K, A,
                       lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
  else
    hipLaunchKernelGGL((k_gemm_bf16<TA, TB, WT, false, TC>), grid, dim3(256), 0, s, M, N, K, A,
                       lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
}

template <int TA, int TB, typename TC>
static void launch_bf16_t(int wt, dim3 grid, hipStream_t s, bool vec, int M, int N, int K,
                          const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                          const float* bias, float beta, TC* C, int64_t ldc, int64_t cs,
                          int kps, float* slab, int tiles_n) {
#define GNNEA_WT(W)                                                                          \
  launch_bf16_wt<TA, TB, W, TC>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc,   \
                                cs, kps, slab, tiles_n)
  switch (wt) {
    case 1: GNNEA_WT(1); break;
    case 2: GNNEA_WT(2); break;
    case 3: GNNEA_WT(3); break;
    case 4: GNNEA_WT(4); break;
    default: GNNEA_WT(5); break;
  }
#undef GNNEA_WT
}

template <typename TC>
static int gemm_bf16_t(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                       const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                       const float* bias, float beta, TC* C, int64_t ldc, void* ws,
                       int64_t ws_bytes, hipStream_t s, int64_t cs = 128) {
  const int wt = bf16_wt(N);
  const int64_t bn = 64 * wt;
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = (int)(((M + HBM - 1) / HBM) * tiles_n);
  const int splits = ws ? bf16_splits(M, N, K, ws_bytes) : 1;
  const int kps = (int)(((K + splits - 1) / splits + HBK - 1) / HBK * HBK);
  float* slab = splits > 1 ? (float*)ws : nullptr;
  const int64_t a_contig = trans_a ? M : K, b_contig = trans_b ? K : N;
  const bool vec = K > 0 && lda % 4 == 0 && ldb % 4 == 0 && a_contig % 4 == 0 &&
                   b_contig % 4 == 0 && (((uintptr_t)A) & 7) == 0 && (((uintptr_t)B) & 7) == 0;
  const dim3 grid(tiles, splits);
  const int kk = kps > 0 ? kps : HBK;
  const int m = (int)M, n = (int)N, k = (int)K;
  if (!trans_a && !trans_b) launch_bf16_t<0, 0, TC>(wt, grid, s, vec, m, n, k, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else if (!trans_a && trans_b) launch_bf16_t<0, 1, TC>(wt, grid, s, vec, m, n, k, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else if (trans_a && !trans_b) launch_bf16_t<1, 0, TC>(wt, grid, s, vec, m, n, k, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else launch_bf16_t<1, 1, TC>(wt, grid, s, vec, m, n, k, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  GNNEA_LAUNCH_CHECK();
  if (splits > 1) {
    const int64_t nn = M * N;
    const int nb = (int)((nn + 255) / 256 < 4096 ? (nn + 255) / 256 : 4096);
    hipLaunchKernelGGL((k_gemm_bf16_reduce<TC>), dim3(nb), dim3(256), 0, s, m, n, splits, slab,
                       bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_gemm_bf16_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  return bf16_splits(M, N, K, INT64_MAX / 2) * M * N * 4;
}

extern "C" int gnnea_gemm_bf16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                               const void* A, int64_t lda, const void* B, int64_t ldb,
                               const float* bias, float beta, void* C, int64_t ldc, int c_dtype,
                               void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!C || ldc < N || (K > 0 && (!A || !B))) return GNNEA_EINVAL;
  if (K > 0) {
    if ((trans_a ? lda < M : lda < K) || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  if (c_dtype == GNNEA_BF16)
    return gemm_bf16_t<bf16_t>(trans_a, trans_b, M, N, K, (const bf16_t*)A, lda,
                               (const bf16_t*)B, ldb, bias, beta, (bf16_t*)C, ldc, ws, ws_bytes,
                               s);
  if (c_dtype == GNNEA_F32)
    return gemm_bf16_t<float>(trans_a, trans_b, M, N, K, (const bf16_t*)A, lda,
                              (const bf16_t*)B, ldb, bias, beta, (float*)C, ldc, ws, ws_bytes,
                              s);
  return GNNEA_EINVAL;
}

extern "C" int gnnea_gemm_sliced_bf16(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                      const void* A, int64_t lda, const void* B, int64_t ldb,
                                      const float* bias, float beta, void* Cs, int64_t sstride,
                                      void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!Cs || sstride % 128 || sstride < M * 128 || (K > 0 && (!A || !B))) return GNNEA_EINVAL;
  if (K > 0) {
    if ((trans_a ? lda < M : lda < K) || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  }
  return gemm_bf16_t<bf16_t>(trans_a, trans_b, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B,
                             ldb, bias, beta, (bf16_t*)Cs, 128, ws, ws_bytes,
                             (hipStream_t)stream, sstride);
}
