// Dense projection on MFMA: C = op(A)·op(B) (+ bias) (+ beta*C), f32 in / f32 accumulate.
// Replaces nn.Linear (layers/layers.py:32,61,93), torch.mm(input, W) (att_layers.py:33) and
// torch.spmm(x, kernel_gate) (layers/layers.py:69), forward and backward.
//
// v_mfma_f32_32x32x2_f32 (gfx950: exact f32, bit-for-bit a k-ordered fmaf chain; 64 FLOP per
// clock per SIMD).  The feature projections here are tall and thin (M = 2M nodes, N = K = 300),
// so the block tile spans the whole output width: BM = 64 rows x BN = 64*WT columns (WT = 5 ->
// 320 >= 300, one column tile, X streamed from HBM exactly once), BK = 16.  4 waves in 2x2, each
// wave 32 x 32*WT = WT accumulator tiles.  Operand tiles are staged in double-buffered LDS in the
// layout their global rows already have (no transposes): an operand that is contiguous along K
// is kept [row][BK+1] (the +1 makes the 32 lanes' column reads hit 32 banks), one contiguous along
// M/N is kept [k][64*WT+4] and written with 16-B stores.  Next tile's global loads are issued into
// registers before the MFMAs of the current one (one barrier per K step).
// Large-K / small-output products (weight gradients, K = N_nodes) split K over workgroups into
// fp32 slabs reduced in fixed order by a second kernel: deterministic, no atomics.
#include <cstdlib>
#include <type_traits>
#include "common.h"
#include "gemm_ta.h"
#include "gemm_x3w.h"
#include "act.h"
#include "lds_dma.h"

namespace gnnea {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 64, GBK = 16;

// LDS geometry of one operand tile: ROWS x GBK with K contiguous ("rk") or K-major ("kr").
template <bool K_CONTIG, int ROWS>
struct Tile {
  static constexpr int LD = K_CONTIG ? GBK + 1 : ROWS + 4;
  static constexpr int SIZE = K_CONTIG ? ROWS * LD : GBK * LD;
  __device__ static int at(int row, int k) { return K_CONTIG ? row * LD + k : k * LD + row; }
};

// Load a ROWS x GBK tile of op(X) into registers. op(X)[row][k] = X[row][k] (K_CONTIG) or
// X[k][row]; rows >= nrows or k >= kend read as 0.  VEC: 16-B loads (ld % 4 == 0, aligned).
template <bool K_CONTIG, int ROWS, bool VEC, int NT = 256>
struct Loader {
  static constexpr int NTOT = ROWS * GBK / 4;  // float4 of the tile
  static constexpr int NV = (NTOT + NT - 1) / NT;  // float4 per thread
  float4 r[NV];
  __device__ void load(const float* __restrict__ X, int64_t ld, int row0, int nrows, int k0,
                       int kend, int tid) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int idx = tid + NT * q;
      if (NTOT % NT != 0 && idx >= NTOT) { r[q] = make_float4(0.f, 0.f, 0.f, 0.f); continue; }
      int row, k;
      if (K_CONTIG) { row = idx / (GBK / 4); k = (idx % (GBK / 4)) * 4; }
      else { k = idx / (ROWS / 4); row = (idx % (ROWS / 4)) * 4; }
      const int gr = row0 + row, gk = k0 + k;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (VEC) {
        if (K_CONTIG) {
          if (gr < nrows && gk < kend) v = *(const float4*)(X + (int64_t)gr * ld + gk);
        } else {
          if (gk < kend && gr < nrows) v = *(const float4*)(X + (int64_t)gk * ld + gr);
        }
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = K_CONTIG ? gr : gr + e, kk = K_CONTIG ? gk + e : gk;
          t[e] = (rr < nrows && kk < kend)
                     ? (K_CONTIG ? X[(int64_t)rr * ld + kk] : X[(int64_t)kk * ld + rr])
                     : 0.f;
        }
        v = make_float4(t[0], t[1], t[2], t[3]);
      }
      r[q] = v;
    }
  }
  __device__ void store(float* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int idx = tid + NT * q;
      if (NTOT % NT != 0 && idx >= NTOT) continue;
      if (K_CONTIG) {
        const int row = idx / (GBK / 4), k = (idx % (GBK / 4)) * 4;
        float* p = S + Tile<true, ROWS>::at(row, k);
        p[0] = r[q].x; p[1] = r[q].y; p[2] = r[q].z; p[3] = r[q].w;
      } else {
        const int k = idx / (ROWS / 4), row = (idx % (ROWS / 4)) * 4;
        *(float4*)(S + Tile<false, ROWS>::at(row, k)) = r[q];
      }
    }
  }
};

// Output addressing: element (row, col) of C at (col / 64)·cs + row·ldc + col % 64.  cs = 64 is
// the plain row-major matrix; ldc = 64, cs = n·64 is the slice-major table [⌈N/64⌉][n][64] that
// the sliced SpMM gathers from (gnnea_spmm_sliced_f32).
__device__ __forceinline__ int64_t c_index(int64_t row, int64_t col, int64_t ldc, int64_t cs) {
  return (col >> 6) * cs + row * ldc + (col & 63);
}

// Epilogue of the MFMA GEMM kernels: WT accumulator tiles in the 32x32 C/D map (col = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5)) at rows m_w.., columns n_w..; addresses from one row base
// per r and one column offset per t (no 64-bit multiply per element).  slab: split-K partials.
template <int WT>
__device__ __forceinline__ void store_tiles(const f32x16 (&acc)[WT], int M, int N, int m_w, int n_w,
                                            int kh, int li, const float* __restrict__ bias,
                                            float beta, float* __restrict__ C, int64_t ldc,
                                            int64_t cs, float* __restrict__ slab, int split) {
  int64_t coff[WT];
  float bv[WT];
  bool cok[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t) {
    const int col = n_w + t * 32 + li;
    cok[t] = col < N;
    coff[t] = slab ? col : c_index(0, col, ldc, cs);
    bv[t] = (bias && !slab && cok[t]) ? bias[col] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m_w + (r & 3) + 8 * (r >> 2) + 4 * kh;
    if (row >= M) continue;
    float* base = slab ? slab + ((int64_t)split * M + row) * N : C + (int64_t)row * ldc;
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      if (!cok[t]) continue;
      float* c = base + coff[t];
      if (slab) {
        *c = acc[t][r];
      } else {
        float o = acc[t][r] + bv[t];
        if (beta != 0.f) o += beta * *c;
        *c = o;
      }
    }
  }
}

template <int TA, int TB, int WT, bool VEC, int BMX = GBM>
__global__ __launch_bounds__(4 * BMX) void k_gemm_wide(int M, int N, int K, const float* __restrict__ A,
                                                   int64_t lda, const float* __restrict__ B,
                                                   int64_t ldb, const float* __restrict__ bias,
                                                   float beta, float* __restrict__ C,
                                                   int64_t ldc, int64_t cs, int k_per_split,
                                                   float* __restrict__ slab, int tiles_n) {
  constexpr int BN = 64 * WT;
  constexpr bool AK = TA == 0, BK_ = TB == 1;  // operand contiguous along K?
  constexpr int NT = 4 * BMX;  // 4 waves per 32-row pair: 2 x 2 (64 rows) or 4 x 2 (128)
  using TA_ = Tile<AK, BMX>;
  using TB_ = Tile<BK_, BN>;
  __shared__ float smem[2 * (TA_::SIZE + TB_::SIZE)];
  // buffer b of A at smem + b*SIZE_A, of B at smem + 2*SIZE_A + b*SIZE_B
  auto As = [&](int b) { return smem + b * TA_::SIZE; };
  auto Bs = [&](int b) { return smem + 2 * TA_::SIZE + b * TB_::SIZE; };

  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = t_id % tiles_n, bm = t_id / tiles_n;
  const int m0 = bm * BMX, n0 = bn * BN;
  const int split = blockIdx.y;
  const int kb = split * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int kh = lane >> 5, li = lane & 31;

  f32x16 acc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  Loader<AK, BMX, VEC, NT> la;
  Loader<BK_, BN, VEC, NT> lb;
  const int nsteps = ke > kb ? (ke - kb + GBK - 1) / GBK : 0;
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
      la.load(A, lda, m0, M, kb + (s + 1) * GBK, ke, tid);
      lb.load(B, ldb, n0, N, kb + (s + 1) * GBK, ke, tid);
    }
    const float* a_s = As(cur);
    const float* b_s = Bs(cur);
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const float a = a_s[TA_::at(wm * 32 + li, kk + kh)];
#pragma unroll
      for (int t = 0; t < WT; ++t) {
        const float b = b_s[TB_::at(wn * 32 * WT + t * 32 + li, kk + kh)];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[t], 0, 0, 0);
      }
    }
    if (more) {
      la.store(As(cur ^ 1), tid);
      lb.store(Bs(cur ^ 1), tid);
    }
    __syncthreads();
  }

  store_tiles<WT>(acc, M, N, m0 + wm * 32, n0 + wn * 32 * WT, kh, li, bias, beta, C, ldc, cs,
                  slab, split);
}

// ---- fp32 GEMM on the bf16 MFMA: three-way split operands, six products ------------------------
// Every fp32 operand element x is split exactly into x = h + m + l + r with h = bf16(x),
// m = bf16(x - h), l = bf16(x - h - m) (|r| <= 2^-24 |x|: the two subtractions are exact), staged
// in LDS as three bf16 planes.  C = Σ over the six products whose order is <= 2 (l·h, m·m, h·l,
// m·h, h·m, h·h, small ones first) on v_mfma_f32_32x32x16_bf16 with fp32 accumulation: the
// dropped terms (m·l, l·m, l·l) are below 2^-24 relative, so the result carries fp32 rounding
// (emulated on the CPU: 3.6e-7 norm-relative vs fp64 at K = 300, plain fp32 6.7e-7).  Six bf16
// MFMAs cost 6/16 of one f32 MFMA (bf16 dense 2.5 PF vs f32 157 TF): the 360-GFLOP projections
// of the training step move from the f32 MFMA bound (2.3 ms) toward their HBM bound (0.76 ms).
// Tile as k_gemm_wide: BM = 64 x BN = 64*WT, 4 waves 2 x 2, BK = 16 (one MFMA k-step); planes
// [row][k] K-contiguous with a 48-B row stride (16-B fragments, conflict-free b128 reads); an
// operand contiguous along M/N is transposed while its planes are written.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int XLD = GBK + 8;  // bf16 elements per LDS plane row

// the hardware conversion (v_cvt_pk_bf16_f32, round to nearest even) on plain casts
__device__ __forceinline__ bf16_t to_bf16_hw(float x) {
  return __builtin_bit_cast(bf16_t, (__bf16)x);
}
__device__ __forceinline__ void split3(float x, bf16_t& h, bf16_t& m, bf16_t& l) {
  h = to_bf16_hw(x);
  const float r1 = x - bf16_to_f32(h);
  m = to_bf16_hw(r1);
  l = to_bf16_hw(r1 - bf16_to_f32(m));
}

template <bool K_CONTIG, int ROWS, bool VEC, int NT = 256>
struct X3Loader : Loader<K_CONTIG, ROWS, VEC, NT> {
  using Loader<K_CONTIG, ROWS, VEC, NT>::r;
  static constexpr int NV = Loader<K_CONTIG, ROWS, VEC, NT>::NV;
  static constexpr int PLANE = ROWS * XLD;
  // planes at S, S + PLANE, S + 2*PLANE (h, m, l)
  __device__ void store3(bf16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int idx = tid + NT * q;
      if (Loader<K_CONTIG, ROWS, VEC, NT>::NTOT % NT != 0 &&
          idx >= Loader<K_CONTIG, ROWS, VEC, NT>::NTOT)
        continue;
      const float v[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
      bf16_t h[4], m[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split3(v[e], h[e], m[e], l[e]);
      if (K_CONTIG) {  // 4 consecutive k of one row: one 8-B store per plane
        const int row = idx / (GBK / 4), k = (idx % (GBK / 4)) * 4;
        bf16_t* p = S + row * XLD + k;
        *(uint2*)p = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
        *(uint2*)(p + PLANE) =
            make_uint2(m[0] | ((uint32_t)m[1] << 16), m[2] | ((uint32_t)m[3] << 16));
        *(uint2*)(p + 2 * PLANE) =
            make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
      } else {  // 4 consecutive rows at one k
        const int k = idx / (ROWS / 4), row = (idx % (ROWS / 4)) * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bf16_t* p = S + (row + e) * XLD + k;
          p[0] = h[e];
          p[PLANE] = m[e];
          p[2 * PLANE] = l[e];
        }
      }
    }
  }
};

// Tile loader for a [K][rows] (rows-contiguous) fp32 source that stages K-contiguous bf16
// planes: a thread loads 4 consecutive rows at one k (one float4) and writes them element-wise,
// with k fastest across the lanes: each 2-B store instruction covers 16 consecutive k of four
// 4-row groups (48-dword offsets: conflict-free).  Row-group-fastest lanes (X3Loader<false>)
// hit the same few banks, 8-16-way conflicted.
template <int ROWS, int NT, bool VEC>
struct X3LoaderT {
  static constexpr int NTOT = ROWS * GBK / 4;
  static constexpr int NV = (NTOT + NT - 1) / NT;
  static constexpr int PLANE = ROWS * XLD;
  float4 r[NV];
  __device__ void load(const float* __restrict__ X, int64_t ld, int row0, int nrows, int k0,
                       int kend, int tid) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int idx = tid + NT * q;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (NTOT % NT == 0 || idx < NTOT) {
        const int k = idx % GBK, row = (idx / GBK) * 4;
        const int gr = row0 + row, gk = k0 + k;
        if (gk < kend) {
          const float* p = X + (int64_t)gk * ld + gr;
          if (VEC) {
            if (gr < nrows) v = *(const float4*)p;
          } else {
            v.x = gr < nrows ? p[0] : 0.f;
            v.y = gr + 1 < nrows ? p[1] : 0.f;
            v.z = gr + 2 < nrows ? p[2] : 0.f;
            v.w = gr + 3 < nrows ? p[3] : 0.f;
          }
        }
      }
      r[q] = v;
    }
  }
  __device__ void store3(bf16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int idx = tid + NT * q;
      if (NTOT % NT != 0 && idx >= NTOT) continue;
      const int k = idx % GBK, row = (idx / GBK) * 4;
      const float v[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bf16_t h, m, l;
        split3(v[e], h, m, l);
        bf16_t* p = S + (row + e) * XLD + k;
        p[0] = h;
        p[PLANE] = m;
        p[2 * PLANE] = l;
      }
    }
  }
};

// B (the small weight operand) arrives pre-split: three bf16 planes [3][n][ldp] K-contiguous,
// zero-padded to ldp = roundup16(K) columns (k_split3_planes, once per call), so the kernel splits
// only A and every B fragment load is a 16-B copy.
constexpr int kPlaneAlign = 16;

__global__ __launch_bounds__(256) void k_split3_planes(const float* __restrict__ W, int64_t ldw,
                                                       int trans, int n, int K, int ldp,
                                                       bf16_t* __restrict__ P, int64_t pstride) {
  // plane element (r, k), r < n, k < ldp:  W[r][k] (trans = 0: W is [n][K]) or W[k][r]
  const int64_t total = (int64_t)n * ldp;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(t / ldp), k = (int)(t - (int64_t)r * ldp);
    const float x = k < K ? (trans ? W[(int64_t)k * ldw + r] : W[(int64_t)r * ldw + k]) : 0.f;
    bf16_t h, m, l;
    split3(x, h, m, l);
    P[t] = h;
    P[pstride + t] = m;
    P[2 * pstride + t] = l;
  }
}

// the same planes k-block-major for k_gemm_x3p: P[p][kb][r][16] (r < NP = N rounded up to the
// column tile, zero rows past N; kb < KP/16), so one k-step's B tile of a plane is one contiguous
// run of 32-B rows (its DMA reads whole cache lines).  With a bias, plane row k = K holds the
// bias split three ways (the kernel multiplies it by an A column of ones: exact, the bias joins
// the fp32 accumulation instead of being added in the epilogue); KP >= K + 1 then.
__global__ __launch_bounds__(256) void k_split3_planes_kb(const float* __restrict__ W, int64_t ldw,
                                                          int trans, int n, int K, int NP, int KP,
                                                          const float* __restrict__ bias,
                                                          bf16_t* __restrict__ P) {
  const int64_t total = (int64_t)NP * KP;  // per plane
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int kb = (int)(t / ((int64_t)NP * GBK));
    const int rem = (int)(t - (int64_t)kb * NP * GBK);
    const int r = rem / GBK, k = kb * GBK + rem % GBK;
    float x = 0.f;
    if (r < n) {
      if (k < K) x = trans ? W[(int64_t)k * ldw + r] : W[(int64_t)r * ldw + k];
      else if (k == K && bias) x = bias[r];
    }
    bf16_t h, m, l;
    split3(x, h, m, l);
    P[t] = h;
    P[total + t] = m;
    P[2 * total + t] = l;
  }
}

template <int ROWS, int NT = 256>
struct PLoader {  // ROWS x GBK of each of the three planes, 16-B chunks of 8 k
  static constexpr int NCH = 3 * ROWS * (GBK / 8);
  static constexpr int NQ = (NCH + NT - 1) / NT;
  uint4 r[NQ];
  __device__ void load(const bf16_t* __restrict__ P, int64_t ldp, int64_t pstride, int row0,
                       int nrows, int k0, int tid) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = tid + NT * q;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (idx < NCH) {
        const int p = idx / (ROWS * 2), rem = idx - p * ROWS * 2;
        const int row = rem >> 1, k8 = (rem & 1) * 8;
        if (row0 + row < nrows)
          v = *(const uint4*)(P + p * pstride + (int64_t)(row0 + row) * ldp + k0 + k8);
      }
      r[q] = v;
    }
  }
  __device__ void store(bf16_t* __restrict__ S, int tid) const {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int idx = tid + NT * q;
      if (idx < NCH) {
        const int p = idx / (ROWS * 2), rem = idx - p * ROWS * 2;
        const int row = rem >> 1, k8 = (rem & 1) * 8;
        *(uint4*)(S + p * ROWS * XLD + row * XLD + k8) = r[q];
      }
    }
  }
};

constexpr int XBM = 128, XNT = 512;  // 8 waves in 4 x 2, each 32 x 32*WT

// TA: the weight-gradient form dW = Aᵀ·B with A stored [K][M] and B stored [K][N] (both tall,
// M-/N-contiguous): both operands are split on the fly (X3LoaderT), no pre-split planes;
// split-K fills the chip (the output is only M x N).
template <int WT, bool VEC, bool TA = false>
__global__ __launch_bounds__(XNT) void k_gemm_x3(int M, int N, int K, const float* __restrict__ A,
                                                 int64_t lda, const bf16_t* __restrict__ Bp,
                                                 int64_t ldp, int64_t pstride,
                                                 const float* __restrict__ Braw, int64_t ldb,
                                                 const float* __restrict__ bias, float beta,
                                                 float* __restrict__ C, int64_t ldc, int64_t cs,
                                                 int k_per_split, float* __restrict__ slab,
                                                 int tiles_n) {
  constexpr int BN = 64 * WT;
  constexpr int SA = 3 * XBM * XLD, SB = 3 * BN * XLD;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (SA + SB)];
  auto As = [&](int b) { return smem + b * SA; };
  auto Bs = [&](int b) { return smem + 2 * SA + b * SB; };

  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int bn = t_id % tiles_n, bm = t_id / tiles_n;
  const int m0 = bm * XBM, n0 = bn * BN;
  const int split = blockIdx.y;
  const int kb = split * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int kh = lane >> 5, li = lane & 31;

  f32x16 acc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  typename std::conditional<TA, X3LoaderT<XBM, XNT, VEC>, X3Loader<true, XBM, VEC, XNT>>::type la;
  typename std::conditional<TA, X3LoaderT<BN, XNT, VEC>, PLoader<BN, XNT>>::type lb;
  auto load_b = [&](int k0) {
    if constexpr (TA) lb.load(Braw, ldb, n0, N, k0, ke, tid);
    else lb.load(Bp, ldp, pstride, n0, N, k0, tid);
  };
  auto store_b = [&](bf16_t* S) {
    if constexpr (TA) lb.store3(S, tid);
    else lb.store(S, tid);
  };
  const int nsteps = ke > kb ? (ke - kb + GBK - 1) / GBK : 0;
  constexpr int PA = XBM * XLD, PB = BN * XLD;
  // the six products of one 16-deep k-step from LDS buffer cur
  auto compute = [&](int cur) {
    const bf16_t* a_s = As(cur) + (wm * 32 + li) * XLD + 8 * kh;
    const bf16x8_t ah = *(const bf16x8_t*)a_s;
    const bf16x8_t am = *(const bf16x8_t*)(a_s + PA);
    const bf16x8_t al = *(const bf16x8_t*)(a_s + 2 * PA);
    bf16x8_t bh[WT], bm_[WT], bl[WT];
#pragma unroll
    for (int t = 0; t < WT; ++t) {
      const bf16_t* b_s = Bs(cur) + (wn * 32 * WT + t * 32 + li) * XLD + 8 * kh;
      bh[t] = *(const bf16x8_t*)b_s;
      bm_[t] = *(const bf16x8_t*)(b_s + PB);
      bl[t] = *(const bf16x8_t*)(b_s + 2 * PB);
    }
    // small products first; each product over the WT independent accumulators
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[t], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm_[t], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[t], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[t], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm_[t], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < WT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[t], acc[t], 0, 0, 0);
  };
  // (a second register stage for the TA form, loads two k-steps ahead, spilled at WT = 5)
  if (nsteps > 0) {
    la.load(A, lda, m0, M, kb, ke, tid);
    load_b(kb);
    la.store3(As(0), tid);
    store_b(Bs(0));
    __syncthreads();
  }
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {  // in flight under the MFMAs below
      la.load(A, lda, m0, M, kb + (s + 1) * GBK, ke, tid);
      load_b(kb + (s + 1) * GBK);
    }
    compute(cur);
    if (more) {
      la.store3(As(cur ^ 1), tid);
      store_b(Bs(cur ^ 1));
    }
    __syncthreads();
  }

  store_tiles<WT>(acc, M, N, m0 + wm * 32, n0 + wn * 32 * WT, kh, li, bias, beta, C, ldc, cs,
                  slab, split);
}

// ---- k_gemm_x3p: the projection form (A [M][K] K-contiguous fp32, B pre-split planes) with an
// LDS-DMA pipeline, two workgroups per CU.
// k_gemm_x3 above (one 512-thread workgroup per CU, register-staged, A split once per k-step into
// LDS planes) measured MFMA busy ≈ 27 %: it is latency-bound — one 16-deep k-step of MFMA work
// (≈0.8 µs per SIMD) is all that covers the next step's loads, the split + LDS-write phase runs
// with the matrix cores idle, and the 160-KB epilogue of every 128 x 320 tile is not overlapped.
// Here a 256-thread workgroup owns a 128 x 32*WT tile (4 waves stacked along M, each 32 rows x
// all 32*WT columns: the same per-wave work as k_gemm_x3's 32 x 32*WT), 3-stage LDS ring of
// ≈23 KB stages (WT = 5: the raw fp32 A tile, 128 rows x 64 B, and the three bf16 planes of the B
// tile, 160 rows x 32 B each), ≈70 KB in all, so two workgroups share a CU (two waves per SIMD,
// up to 256 registers each) and each one's barriers and epilogue hide under the other's MFMAs,
// with two k-steps of DMA in flight behind the one being multiplied.  Staging is
// global_load_lds (16 B per lane, no registers).  Each wave reads its A rows as fp32 and splits
// them in registers (no LDS plane writes).  Counted vmcnt + raw s_barrier (no vmcnt(0) in the
// loop); the fragment reads are inline asm, because hipcc waits vmcnt(0) before any LDS read
// while an LDS-DMA is in flight (it cannot tell the ring's buffers apart).  LDS images are
// lane-linear (DMA destination = base + lane * 16), so the bank swizzles go on the SOURCE
// addresses and the same XOR on the reads: A row r's 16-B slot s at s ^ ((r >> 2) & 3), B row
// r's 16-B half h at h ^ ((r >> 3) & 1) (16 consecutive lanes of a b128 read then hit 16
// distinct slots).  The six products and their order are k_gemm_x3's.  A is read once per column
// tile (2 at N = 300); the two tiles of an M block are adjacent ids, i.e. on one XCD at once.
// Requirements (host-checked): K % 4 == 0, lda % 4 == 0, A 16-B aligned; rows >= M / N read a
// clamped valid row (their outputs are not stored), A quads with k >= K read a valid address and
// are zeroed in registers, the B planes are zero-padded to ldp.
// NW waves stacked along M (4: two workgroups per CU, 3-stage ring; 8: one per CU, 4 stages,
// half the B-tile traffic per row of A)
template <int WT, int NW>
struct X3P {
  static constexpr int BM = 32 * NW, NT = 64 * NW;
  static constexpr int BN = 32 * WT;
  static constexpr int A_CHUNKS = BM * GBK * 4 / 1024;          // 16 rows x 64 B each: 2 per wave
  static constexpr int A_BYTES = A_CHUNKS * 1024;
  static constexpr int PLANE_BYTES = BN * GBK * 2;              // BN rows x 32 B
  static constexpr int B_CHUNKS = 3 * PLANE_BYTES / 1024;       // 3*WT
  static constexpr int B_CHUNKS_PAD = (B_CHUNKS + NW - 1) / NW * NW;  // same count on every wave
  static constexpr int DMA_BYTES = A_BYTES + B_CHUNKS_PAD * 1024;
  static constexpr int EPI_LD = NW == 8 ? 32 : 36;               // epilogue row stride (floats)
  static constexpr int EPI_BYTES = NW * 32 * EPI_LD * 4;         // the waves' epilogue regions
  static constexpr int STAGE = DMA_BYTES > EPI_BYTES ? DMA_BYTES : (EPI_BYTES + 1023) / 1024 * 1024;
  static constexpr int LOADS = A_CHUNKS / NW + B_CHUNKS_PAD / NW;  // DMA instr. / wave / stage
  // ring stages: 4 when they fit one workgroup per CU (NW = 8), 3 for two per CU (NW = 4)
  // (a 5-stage ring, which fits 160 KB at WT = 5, measured no faster: 2.52 vs 2.50 ms)
  static constexpr int NS = NW == 8 ? (4 * STAGE <= 160 * 1024 ? 4 : 3) : 3;
  static_assert(A_CHUNKS == 2 * NW, "A: two 1-KB chunks per wave");
};

// One 32 x 32 accumulator tile of a wave, written to C with 16-B stores through a private LDS
// region (32 rows of LD floats; LD = 36 keeps the two half-waves' rows on different banks):
// lanes write their column, then read 4 consecutive columns of a row (8 lanes per 128-B row
// piece).  The LDS accesses are inline asm (hipcc would wait vmcnt(0) for the ring's DMA before
// plain ones).  vec4 (N % 4 == 0, ldc % 4 == 0, cs % 4 == 0, C 16-B aligned): EXACTLY four
// 16-B stores per lane per tile, out-of-range lanes storing to `dummy` (the k-loop counts them in
// its vmcnt waits); otherwise scalar stores.
template <int LD>  // epilogue row stride in floats
__device__ __forceinline__ void store_tile_v4(const f32x16& acc, uint32_t region, int M, int N,
                                              int m_w, int n_t, int kh, int li, int lane,
                                              float beta, float* __restrict__ C, int64_t ldc,
                                              int64_t cs, bool vec4, float* __restrict__ dummy,
                                              float* __restrict__ C2, int64_t cs2) {
  const uint32_t wb = region + (4 * kh) * LD * 4 + li * 4;
#pragma unroll
  for (int r = 0; r < 16; ++r) ds_write32(wb + ((r & 3) + 8 * (r >> 2)) * LD * 4, acc[r]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint32_t rbase = region + (lane >> 3) * LD * 4 + (lane & 7) * 16;
  f32x4_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = ds_read128f(rbase + i * 8 * LD * 4);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = (lane >> 3) + 8 * i, c4 = (lane & 7) * 4;
    const int grow = m_w + row, gcol = n_t + c4;
    float o[4] = {v[i][0], v[i][1], v[i][2], v[i][3]};
    if (vec4) {
      const bool ok = grow < M && gcol < N;
      float* c = ok ? C + c_index(grow, gcol, ldc, cs) : dummy + 4 * lane;
      if (beta != 0.f && ok) {
        const float4 cc = *(const float4*)c;
        o[0] += beta * cc.x; o[1] += beta * cc.y; o[2] += beta * cc.z; o[3] += beta * cc.w;
      }
      *(float4*)c = make_float4(o[0], o[1], o[2], o[3]);
      if (C2) {  // the slice-major copy [ceil(N/64)][M][64] (exactly one more store per i)
        float* c2 = ok ? C2 + c_index(grow, gcol, 64, cs2) : dummy + 4 * lane;
        *(float4*)c2 = make_float4(o[0], o[1], o[2], o[3]);
      }
    } else if (grow < M) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (gcol + e >= N) continue;
        float* c = C + c_index(grow, gcol + e, ldc, cs);
        float x = o[e];
        if (beta != 0.f) x += beta * *c;
        *c = x;
        if (C2) C2[c_index(grow, gcol + e, 64, cs2)] = x;
      }
    }
  }
}

// Persistent: 2 workgroups per CU, each walks tiles blockIdx.x, + gridDim.x, ... (XCD-remapped)
// as ONE stream of k-steps, so the DMA ring runs across tile boundaries (the next tile's first
// stages are in flight while the last ones of the current tile are multiplied) and a tile's
// epilogue (16-B stores through LDS) is written while the next tile's stages land.
template <int WT, int NW>
__global__ __launch_bounds__(64 * NW) void k_gemm_x3p(int M, int N, int K, const float* __restrict__ A,
                                                  int64_t lda, const bf16_t* __restrict__ Bp,
                                                  int64_t ldp, int64_t pstride,
                                                  const float* __restrict__ bias, float beta,
                                                  float* __restrict__ C, int64_t ldc, int64_t cs,
                                                  int tiles_n, int ntiles, int vec4,
                                                  float* __restrict__ dummy,
                                                  float* __restrict__ C2, int64_t cs2) {
  using G = X3P<WT, NW>;
  constexpr int NS = G::NS;
  constexpr int TH = WT > 5 ? WT / 2 : WT, NH = WT / TH;  // column tiles per half, halves
  static_assert(TH * NH == WT && NH <= 2, "WT > 5 must be 2 x TH");
  static_assert(32 * WT * GBK * 2 % 1024 == 0, "B plane must be whole 1-KB DMA chunks");
  static_assert(G::EPI_BYTES <= G::STAGE, "epilogue regions must fit one stage");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * G::STAGE];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kh = lane >> 5, li = lane & 31;
  // with a bias, A gets a column of ones at k = K (the planes hold the bias there)
  const bool hb = bias != nullptr;
  const int nsteps = (K + (hb ? 1 : 0) + GBK - 1) / GBK;
  const int gsz = gridDim.x;
  const int nq = (int)blockIdx.x < ntiles ? (ntiles - (int)blockIdx.x + gsz - 1) / gsz : 0;
  const int total = nq * nsteps;
  auto tile_of = [&](int q, int& m0, int& n0) {
    const int t_id = xcd_remap((int)blockIdx.x + q * gsz, ntiles);
    m0 = (t_id / tiles_n) * G::BM;
    n0 = (t_id % tiles_n) * G::BN;
  };

  // ---- issue side: the next stage of the stream (tile iq, k-step is) ----
  int iq = 0, is = 0;
  const float* a_src[2];
  int a_slot[2];
  const bf16_t* b_src[G::B_CHUNKS_PAD / NW];
  auto set_issue_tile = [&](int q) {
    int m0, n0;
    tile_of(q, m0, n0);
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const int ar = 16 * (w + NW * qq) + (lane >> 2);  // A row in the tile
      a_slot[qq] = (lane & 3) ^ ((ar >> 2) & 3);       // logical 16-B slot
      a_src[qq] = A + (int64_t)min(m0 + ar, M - 1) * lda + 4 * a_slot[qq];
    }
    // k-block-major planes: plane p, k-block kb, row n at ((p * KB + kb) * NP + n) * 16
#pragma unroll
    for (int qq = 0; qq < G::B_CHUNKS_PAD / NW; ++qq) {
      int c = w + NW * qq;
      if (c >= G::B_CHUNKS) c = G::B_CHUNKS - 1;  // padding chunk: any valid source
      const int p = c / WT, r = (c % WT) * 32 + (lane >> 1);
      const int h = (lane & 1) ^ ((r >> 3) & 1);
      b_src[qq] = Bp + p * pstride + (int64_t)(n0 + r) * GBK + 8 * h;
    }
  };
  auto issue_next = [&](int buf) {
    if (is == 0) set_issue_tile(iq);
    unsigned char* st = smem + buf * G::STAGE;
    const int k0 = is * GBK;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      // a quad past K reads a valid address (k = 0 of the row) and is zeroed at use
      const float* ap = (k0 + 4 * a_slot[qq] < K) ? a_src[qq] + k0 : a_src[qq] - 4 * a_slot[qq];
      glds16(ap, st + (w + NW * qq) * 1024);
    }
#pragma unroll
    for (int qq = 0; qq < G::B_CHUNKS_PAD / NW; ++qq)
      glds16(b_src[qq] + (int64_t)is * ldp, st + G::A_BYTES + (w + NW * qq) * 1024);
    if (++is == nsteps) { is = 0; ++iq; }
  };

  f32x16 acc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // per-lane LDS read offsets (bytes within a stage)
  const int ra = w * 32 + li;
  const int a_off0 = ra * 64 + 16 * ((2 * kh) ^ ((ra >> 2) & 3));
  const int a_off1 = ra * 64 + 16 * ((2 * kh + 1) ^ ((ra >> 2) & 3));
  // B row t*32 + li: bit 3 of the row is li's, so every column tile's offset is b_off0 + t KB
  const int b_off0 = G::A_BYTES + li * 32 + 16 * (kh ^ ((li >> 3) & 1));

  const uint32_t smem_lds = lds_addr(smem);
  auto epilogue = [&](int q, int buf) {
    int m0, n0;
    tile_of(q, m0, n0);
    const uint32_t region = smem_lds + buf * G::STAGE + w * 32 * G::EPI_LD * 4;
#pragma unroll
    for (int t = 0; t < WT; ++t)
      store_tile_v4<G::EPI_LD>(acc[t], region, M, N, m0 + w * 32, n0 + 32 * t, kh, li, lane, beta, C, ldc,
                    cs, vec4 != 0, dummy, C2, cs2);
  };
  // vmcnt allowance for the first step after an epilogue: its 16-B stores (exactly 4 per tile
  // of 32 columns when vec4 and no beta loads) were issued after the DMA that step waits for
  const bool count_stores = vec4 != 0 && beta == 0.f &&
                            G::LOADS * (NS - 2) + (C2 ? 8 : 4) * WT <= 63;

#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < total) issue_next(i);
  int cur = 0, s = 0, q = 0;
  for (int g = 0; g < total; ++g) {
    const bool epi = s == 0 && q > 0;
    // wait for this wave's DMA of stage g; stage g + 1 stays in flight, and at the step after
    // an epilogue also that epilogue's stores (issued between the two DMAs).  Then one barrier:
    // every wave's stage g has landed AND every wave has finished reading buffer (g - 1) % 3
    // (its reads were waited for before its MFMAs), which stage g + 2 then refills
    {
      const int later = total - 1 - g < NS - 2 ? total - 1 - g : NS - 2;  // stages issued after g
      if (later == NS - 2 && count_stores && q > 0 && s >= 1 && s <= NS - 2) {
        if (C2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LOADS * (NS - 2) + 8 * WT > 63 ? 63 : G::LOADS * (NS - 2) + 8 * WT) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LOADS * (NS - 2) + 4 * WT) : "memory");
      } else if (later == NS - 2) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LOADS * (NS - 2)) : "memory");
      } else if (later == 1) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::LOADS) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int prev = cur == 0 ? NS - 1 : cur - 1;
    if (epi) {  // the previous tile's outputs, through buffer prev, then a clean accumulator
      epilogue(q - 1, prev);
      __builtin_amdgcn_s_barrier();  // every wave's epilogue reads of prev are done
      asm volatile("" ::: "memory");
#pragma unroll
      for (int t = 0; t < WT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    }
    if (g + NS - 1 < total) issue_next(prev);
    const uint32_t st = smem_lds + cur * G::STAGE;
    const f32x4_t x0 = ds_read128f(st + a_off0);
    const f32x4_t x1 = ds_read128f(st + a_off1);
    u32x4 braw[3 * TH];
    const uint32_t bst = st + b_off0;
    static_for<TH>([&](auto tt) {
      constexpr int t = decltype(tt)::value;
      braw[3 * t] = ds_read128_o<t * 1024>(bst);
      braw[3 * t + 1] = ds_read128_o<t * 1024 + G::PLANE_BYTES>(bst);
      braw[3 * t + 2] = ds_read128_o<t * 1024 + 2 * G::PLANE_BYTES>(bst);
    });
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(3 * TH) : "memory");  // the two A reads
    __builtin_amdgcn_sched_barrier(0);
    float xa[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      xa[j] = x0[j];
      xa[4 + j] = x1[j];
    }
    const int kval = K - (s * GBK + 8 * kh);  // valid k of this lane's 8
    if (kval < 8) {  // past K: zeros, and the column of ones at k = K under a bias
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j >= kval) xa[j] = (hb && j == kval) ? 1.f : 0.f;
    }
    // pairwise (common.h x3_split_pair: split3's values, half the instructions)
    uint4 h4, m4, l4;
    x3_split_pair(xa[0], xa[1], h4.x, m4.x, l4.x);
    x3_split_pair(xa[2], xa[3], h4.y, m4.y, l4.y);
    x3_split_pair(xa[4], xa[5], h4.z, m4.z, l4.z);
    x3_split_pair(xa[6], xa[7], h4.w, m4.w, l4.w);
    const bf16x8_t ah = __builtin_bit_cast(bf16x8_t, h4);
    const bf16x8_t am = __builtin_bit_cast(bf16x8_t, m4);
    const bf16x8_t al = __builtin_bit_cast(bf16x8_t, l4);
    // the wave's column tiles in NH halves of TH (a 320-wide wave tile keeps 160 accumulator
    // registers; its B fragments are read half by half, the second half's reads in flight
    // under the first half's MFMAs)
#pragma unroll
    for (int hf = 0; hf < NH; ++hf) {
      if (hf > 0) {  // (NH <= 2: the second half)
        static_for<TH>([&](auto tt) {
          constexpr int t = decltype(tt)::value + TH;
          braw[3 * (t - TH)] = ds_read128_o<t * 1024>(bst);
          braw[3 * (t - TH) + 1] = ds_read128_o<t * 1024 + G::PLANE_BYTES>(bst);
          braw[3 * (t - TH) + 2] = ds_read128_o<t * 1024 + 2 * G::PLANE_BYTES>(bst);
        });
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bf16x8_t bh[TH], bm_[TH], bl[TH];
#pragma unroll
      for (int t = 0; t < TH; ++t) {
        bh[t] = __builtin_bit_cast(bf16x8_t, braw[3 * t]);
        bm_[t] = __builtin_bit_cast(bf16x8_t, braw[3 * t + 1]);
        bl[t] = __builtin_bit_cast(bf16x8_t, braw[3 * t + 2]);
      }
      f32x16* ac = acc + hf * TH;
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm_[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm_[t], ac[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TH; ++t) ac[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[t], ac[t], 0, 0, 0);
    }
    cur = cur == NS - 1 ? 0 : cur + 1;
    if (++s == nsteps) { s = 0; ++q; }
  }
  if (total > 0) {  // the last tile: every DMA has landed (vmcnt(0) at the last step)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    epilogue(q - 1, 0);
  }
}

// slab reduction in fixed split order (deterministic); 4 outputs per thread when the rows allow
__global__ void k_gemm_reduce(int M, int N, int splits, const float* __restrict__ slab,
                              const float* __restrict__ bias, float beta, float* __restrict__ C,
                              int64_t ldc, int64_t cs) {
  const int64_t n = (int64_t)M * N;
  const bool v4 =
      (N % 4 == 0) && (ldc % 4 == 0) && (cs % 4 == 0) && ((((uintptr_t)C) & 15) == 0);
  if (v4) {
    const int64_t n4 = n / 4;
    const float4* sl = (const float4*)slab;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n4;
         t += (int64_t)gridDim.x * blockDim.x) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
      int q = 0;
      for (; q + 2 <= splits; q += 2) {  // two slabs in flight
        const float4 x = sl[(int64_t)q * n4 + t], y = sl[(int64_t)(q + 1) * n4 + t];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
      }
      if (q < splits) {
        const float4 x = sl[(int64_t)q * n4 + t];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      }
      float o[4] = {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w};
      const int64_t e = 4 * t, row = e / N, col = e - row * N;
      float* c = C + c_index(row, col, ldc, cs);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (bias) o[k] += bias[col + k];
        if (beta != 0.f) o[k] += beta * c[k];
      }
      *(float4*)c = make_float4(o[0], o[1], o[2], o[3]);
    }
    return;
  }
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < splits; ++q) s += slab[(int64_t)q * n + t];
    const int64_t row = t / N, col = t - row * N;
    if (bias) s += bias[col];
    float* c = C + c_index(row, col, ldc, cs);
    if (beta != 0.f) s += beta * *c;
    *c = s;
  }
}

static int pick_wt(int64_t N) {
  const int64_t wt = (N + 63) / 64;
  return (int)(wt < 1 ? 1 : (wt > 5 ? 5 : wt));
}

// split-K only when the output grid cannot fill the chip and K is long
static int pick_splits(int64_t M, int64_t N, int64_t K, int64_t ws_bytes, int bm = GBM) {
  const int64_t bn = 64 * pick_wt(N);
  const int64_t tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  if (tiles >= 512 || K < 8 * GBK) return 1;
  // ~384 workgroups of 4 waves (~512 of 8 waves: two per CU), the slabs stay small
  const int64_t target = bm == GBM ? 384 : 512;
  int64_t s = (target + tiles - 1) / tiles;
  const int64_t by_k = K / (8 * GBK);
  if (s > by_k) s = by_k;
  if (s > 256) s = 256;
  while (s > 1 && s * M * N * 4 > ws_bytes) --s;
  return (int)(s < 1 ? 1 : s);
}

static bool al16(const void* p) { return (((uintptr_t)p) & 15) == 0; }

template <int TA, int TB, int WT>
static void launch_wt(dim3 grid, hipStream_t s, bool vec, int M, int N, int K, const float* A,
                      int64_t lda, const float* B, int64_t ldb, const float* bias, float beta,
                      float* C, int64_t ldc, int64_t cs, int kps, float* slab, int tiles_n) {
  // 64-row tiles: 128-row / 8-wave tiles measured slower for dW = dYᵀ·x (6.0 vs 4.9 ms at cfg-4)
  constexpr int BMX = GBM;
  if (vec)
    hipLaunchKernelGGL((k_gemm_wide<TA, TB, WT, true, BMX>), grid, dim3(4 * BMX), 0, s, M, N, K,
                       A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
  else
    hipLaunchKernelGGL((k_gemm_wide<TA, TB, WT, false, BMX>), grid, dim3(4 * BMX), 0, s, M, N, K,
                       A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n);
}

template <int TA, int TB>
static void launch_t(int wt, dim3 grid, hipStream_t s, bool vec, int M, int N, int K,
                     const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias,
                     float beta, float* C, int64_t ldc, int64_t cs, int kps, float* slab, int tiles_n) {
  switch (wt) {
    case 1: launch_wt<TA, TB, 1>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n); break;
    case 2: launch_wt<TA, TB, 2>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n); break;
    case 3: launch_wt<TA, TB, 3>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n); break;
    case 4: launch_wt<TA, TB, 4>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n); break;
    default: launch_wt<TA, TB, 5>(grid, s, vec, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, kps, slab, tiles_n); break;
  }
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_gemm_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  const int64_t a = pick_splits(M, N, K, INT64_MAX / 2), b = pick_splits(M, N, K, INT64_MAX / 2, 128);
  return (a > b ? a : b) * M * N * 4;
}

static int gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                    int64_t lda, const float* B, int64_t ldb, const float* bias, float beta,
                    float* C, int64_t ldc, int64_t cs, void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!C || (K > 0 && (!A || !B))) return GNNEA_EINVAL;
  if (cs == 64 ? ldc < N : (ldc < (N < 64 ? N : 64) || cs < M * ldc)) return GNNEA_EINVAL;
  if (K > 0) {
    if ((trans_a ? lda < M : lda < K) || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  }
  hipStream_t s = (hipStream_t)stream;
  const int wt = pick_wt(N);
  const int64_t bn = 64 * wt;
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int bmx = GBM;  // launch_wt's tile height
  const int tiles = (int)(((M + bmx - 1) / bmx) * tiles_n);
  const int splits = ws ? pick_splits(M, N, K, ws_bytes, bmx) : 1;
  const int kps = (int)(((K + splits - 1) / splits + GBK - 1) / GBK * GBK);
  float* slab = splits > 1 ? (float*)ws : nullptr;
  // 16-B loads need every float4 fully inside or fully outside the operand along its
  // contiguous dimension and 16-B aligned rows
  const int64_t a_contig = trans_a ? M : K, b_contig = trans_b ? K : N;
  const bool vec = K > 0 && lda % 4 == 0 && ldb % 4 == 0 && a_contig % 4 == 0 &&
                   b_contig % 4 == 0 && al16(A) && al16(B);
  const dim3 grid(tiles, splits);
  const int kk = kps > 0 ? kps : GBK;
  if (!trans_a && !trans_b) launch_t<0, 0>(wt, grid, s, vec, (int)M, (int)N, (int)K, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else if (!trans_a && trans_b) launch_t<0, 1>(wt, grid, s, vec, (int)M, (int)N, (int)K, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else if (trans_a && !trans_b) launch_t<1, 0>(wt, grid, s, vec, (int)M, (int)N, (int)K, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  else launch_t<1, 1>(wt, grid, s, vec, (int)M, (int)N, (int)K, A, lda, B, ldb, bias, beta, C, ldc, cs, kk, slab, tiles_n);
  GNNEA_LAUNCH_CHECK();
  if (splits > 1) {
    const int64_t n = M * N;
    const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, splits, slab,
                       bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int gnnea_gemm_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                              const float* A, int64_t lda, const float* B, int64_t ldb,
                              const float* bias, float beta, float* C, int64_t ldc, void* ws,
                              int64_t ws_bytes, void* stream) {
  return gemm_f32(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, 64, ws,
                  ws_bytes, stream);
}

extern "C" int gnnea_gemm_sliced_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                     const float* A, int64_t lda, const float* B, int64_t ldb,
                                     const float* bias, float beta, float* Cs, int64_t sstride,
                                     void* ws, int64_t ws_bytes, void* stream) {
  if (sstride % 4 != 0) return GNNEA_EINVAL;
  return gemm_f32(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, Cs, 64, sstride, ws,
                  ws_bytes, stream);
}

// ---- fp32 GEMM through three-way bf16 splits (k_gemm_x3) -----------------------------------
// op(A) must be K-contiguous (trans_a = 0: the tall operand of the projections); a transposed A
// (the weight gradients dW = dYᵀ·x, both operands tall) runs on the f32 MFMA kernel instead.
// planes for either kernel (k_gemm_x3p: rows padded to its column tile, one more k for the
// bias row) + a 1-KB dummy store target for k_gemm_x3p's out-of-range lanes
static int64_t x3_planes_bytes(int64_t N, int64_t K) {
  const int64_t kp = (K + 1 + kPlaneAlign - 1) / kPlaneAlign * kPlaneAlign;
  const int64_t np = (N + 319) / 320 * 320;  // k_gemm_x3p's padded rows (>= N, any tile width)
  const int64_t p = (3 * np * kp * 2 + 255) & ~(int64_t)255;
  const int64_t w = gemm_x3w_ws_bytes(N);  // or gemm_x3w.hip's weight tiles
  return (p > w ? p : w) + 1024;
}

static int gemm_x3_ta(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                      const float* B, int64_t ldb, const float* bias, float beta, float* C,
                      int64_t ldc, int64_t cs, void* ws, int64_t ws_bytes, hipStream_t s);


static int gemm_x3(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K, const float* A,
                   int64_t lda, const float* B, int64_t ldb, const float* bias, float beta,
                   float* C, int64_t ldc, int64_t cs, void* ws, int64_t ws_bytes, void* stream,
                   float* C2 = nullptr, int64_t cs2 = 0, int act = GNNEA_ACT_IDENTITY) {
  if (C2 && (cs2 % 4 != 0 || cs2 < M * 64 || cs != 64)) return GNNEA_EINVAL;
  // the weight-resident form (gemm_x3w.hip) for the tall K <= 320 projections; it writes C2 too
  // and applies a relu in its epilogue
  if (B && (cs == 64 ? ldc >= N : (ldc >= 64 && cs >= M * ldc)) &&
      (trans_b ? ldb >= K : ldb >= N) &&
      gemm_x3w_applies(trans_a, M, N, K, lda, A, beta, ldc, cs, C, C2, cs2, act) && ws &&
      ws_bytes >= gemm_x3w_ws_bytes(N))
    return gemm_x3w_launch(trans_b, M, N, K, A, lda, B, ldb, bias, C, ldc, cs, C2, cs2, ws,
                           ws_bytes, (hipStream_t)stream, beta, act);
  if (act != GNNEA_ACT_IDENTITY) {  // any other kernel: the product, then the act in place
    if (C2 || cs != 64) return GNNEA_EINVAL;
    const int rc = gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, ws,
                           ws_bytes, stream);
    if (rc) return rc;
    return act_rows_f32(C, ldc, M, N, act, (hipStream_t)stream);
  }
  if (C2) {  // a slice-major copy as well: fused into k_gemm_x3p's epilogue, else packed after
    const bool lda_ok = !trans_a && lda % 4 == 0 && K % 4 == 0 && (((uintptr_t)A) & 15) == 0;
    const int64_t pb = x3_planes_bytes(N, K);
    // the same condition as k_gemm_x3p's launch below (pipe on, float4 A, no split-K): any other
    // kernel leaves C2 unwritten, so it is packed after
    const bool fused = lda_ok && ws && ws_bytes >= pb &&
                       pick_splits(M, N, K, ws_bytes - pb) == 1;
    if (!fused) {
      const int rc = gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs,
                             ws, ws_bytes, stream);
      if (rc) return rc;
      return gnnea_slice_pack_f32(C, ldc, (int32_t)M, (int32_t)N, C2, cs2, stream);
    }
  }
  if (trans_a && !trans_b && K > 0)
    return gemm_x3_ta(M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, ws, ws_bytes,
                      (hipStream_t)stream);
  if (trans_a || K == 0)
    return gemm_f32(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, ws,
                    ws_bytes, stream);
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!C || !A || !B) return GNNEA_EINVAL;
  if (cs == 64 ? ldc < N : (ldc < (N < 64 ? N : 64) || cs < M * ldc)) return GNNEA_EINVAL;
  if (lda < K || (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  const int64_t pbytes = x3_planes_bytes(N, K);
  if (!ws || ws_bytes < pbytes) return GNNEA_EWORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  const int ldp = (int)((K + kPlaneAlign - 1) / kPlaneAlign * kPlaneAlign);
  const int64_t pstride = N * ldp;
  bf16_t* planes = (bf16_t*)ws;
  const bool vec = lda % 4 == 0 && K % 4 == 0 && al16(A);
  const int splits = pick_splits(M, N, K, ws_bytes - pbytes);
  if (!(vec && splits == 1)) {
    const int64_t tot = N * ldp;
    const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
    // B op-form [N][K]: trans_b = 1 means B is stored [N][K] (no transpose needed)
    hipLaunchKernelGGL(k_split3_planes, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 0 : 1,
                       (int)N, (int)K, ldp, planes, pstride);
    GNNEA_LAUNCH_CHECK();
  }
  if (vec && splits == 1) {  // k_gemm_x3p: LDS-DMA pipeline, two workgroups per CU
    // 32*WT-column tiles, WT <= 5 (N = 300: two 160-column tiles)
    int wtp = (int)((N + 31) / 32 < 5 ? (N + 31) / 32 : 5);
    const int tn = (int)((N + 32 * wtp - 1) / (32 * wtp));
    const int np = tn * 32 * wtp;  // <= the 320-row rounding x3_planes_bytes reserves
    const int kp = (int)((K + (bias ? 1 : 0) + kPlaneAlign - 1) / kPlaneAlign * kPlaneAlign);
    float* dummy = (float*)((char*)ws + pbytes - 1024);
    {
      const int64_t tot = (int64_t)np * kp;
      const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
      hipLaunchKernelGGL(k_split3_planes_kb, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 0 : 1,
                         (int)N, (int)K, np, kp, bias, planes);
      GNNEA_LAUNCH_CHECK();
    }
    // 8 waves (256-row tiles, one workgroup per CU) for tall operands, else 4 (128 rows, two)
    const int nw = M >= 65536 ? 8 : 4;
    const int64_t tm = (M + 32 * nw - 1) / (32 * nw);
    if (tm * tn >= (1ll << 31)) return GNNEA_EINVAL;
    const int ntiles = (int)(tm * tn);
    static const int ncu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    const int per_cu = nw == 8 ? 1 : 2;  // persistent: as many workgroups as fit at once
    const dim3 grid((unsigned)(ntiles < per_cu * ncu ? ntiles : per_cu * ncu));
    const int vec4 = N % 4 == 0 && ldc % 4 == 0 && cs % 4 == 0 && al16(C);
#define GNNEA_X3P_L(W, NWV)                                                                      \
  hipLaunchKernelGGL((k_gemm_x3p<W, NWV>), grid, dim3(64 * NWV), 0, s, (int)M, (int)N, (int)K, A, \
                     lda, planes, (int64_t)np * GBK, (int64_t)np * kp, bias, beta, C, ldc, cs, tn, \
                     ntiles, vec4, dummy, C2, cs2)
#define GNNEA_X3P(W)                                                                             \
  case W:                                                                                        \
    if (nw == 8) GNNEA_X3P_L(W, 8);                                                              \
    else GNNEA_X3P_L(W, 4);                                                                      \
    break;
    switch (wtp) {
      GNNEA_X3P(1)
      GNNEA_X3P(2)
      GNNEA_X3P(3)
      GNNEA_X3P(4)
      default:
      GNNEA_X3P(5)
    }
#undef GNNEA_X3P
#undef GNNEA_X3P_L
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
  // wider than one 320-column tile: 128-column tiles (WT = 2, the finer work split) measured
  // faster than 2 x 320 (2M x 600 x 300: 5.76 vs 6.05 ms; 30k rows: 0.109 vs 0.118 ms)
  const int wt = N > 320 ? 2 : pick_wt(N);
  const int64_t bn = 64 * wt;
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = (int)(((M + XBM - 1) / XBM) * tiles_n);
  const int kps = (int)(((K + splits - 1) / splits + GBK - 1) / GBK * GBK);
  float* slab = splits > 1 ? (float*)((char*)ws + pbytes) : nullptr;
  const dim3 grid(tiles, splits);
#define GNNEA_X3(W)                                                                              \
  case W:                                                                                        \
    if (vec)                                                                                     \
      hipLaunchKernelGGL((k_gemm_x3<W, true>), grid, dim3(XNT), 0, s, (int)M, (int)N, (int)K, A, \
                         lda, planes, (int64_t)ldp, pstride, nullptr, (int64_t)0, bias, beta, C, \
                         ldc, cs, kps, slab, tiles_n);                                           \
    else                                                                                         \
      hipLaunchKernelGGL((k_gemm_x3<W, false>), grid, dim3(XNT), 0, s, (int)M, (int)N, (int)K,   \
                         A, lda, planes, (int64_t)ldp, pstride, nullptr, (int64_t)0, bias, beta, \
                         C, ldc, cs, kps, slab, tiles_n);                                        \
    break;
  switch (wt) {
    GNNEA_X3(1)
    GNNEA_X3(2)
    GNNEA_X3(3)
    GNNEA_X3(4)
    default:
    GNNEA_X3(5)
  }
#undef GNNEA_X3
  GNNEA_LAUNCH_CHECK();
  if (splits > 1) {
    const int64_t n = M * N;
    const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, splits, slab,
                       bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

// dW = Aᵀ·B on the split-on-the-fly kernel: only split-K slabs in the workspace
static int64_t x3_ta_splits(int64_t M, int64_t N, int64_t K, int64_t ws_bytes) {
  // one 129-KB workgroup per CU: whole waves of 256 (2 per CU), each split >= 8 k-steps
  const int64_t bn = 64 * pick_wt(N);
  const int64_t tiles = ((M + XBM - 1) / XBM) * ((N + bn - 1) / bn);
  if (tiles >= 256 || K < 16 * GBK) return 1;
  constexpr int64_t target = 512;  // workgroups to aim for
  int64_t s = target / tiles;
  const int64_t by_k = K / (8 * GBK);
  if (s > by_k) s = by_k;
  while (s > 1 && s * M * N * 4 > ws_bytes) --s;
  return s < 1 ? 1 : s;
}

static int gemm_x3_ta(int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                      const float* B, int64_t ldb, const float* bias, float beta, float* C,
                      int64_t ldc, int64_t cs, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!C || !A || !B) return GNNEA_EINVAL;
  if (cs == 64 ? ldc < N : (ldc < (N < 64 ? N : 64) || cs < M * ldc)) return GNNEA_EINVAL;
  if (lda < M || ldb < N) return GNNEA_EINVAL;
  if (gemm_ta_applies(M, N, K, lda, ldb, A, B, 4)) {  // whole-width tiles (gemm_ta.hip)
    float* slab = nullptr;
    int used = 0;
    const int rc = gemm_ta_launch<float>(M, N, K, A, lda, B, ldb, ws, ws ? ws_bytes : 0, s,
                                         &slab, &used);
    if (rc) return rc;
    const int64_t n = M * N;
    const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, used, slab,
                       bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
  int wt = pick_wt(N);
  const int64_t bn = 64 * wt;
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = (int)(((M + XBM - 1) / XBM) * tiles_n);
  const int splits = (int)x3_ta_splits(M, N, K, ws ? ws_bytes : 0);
  if (splits > 1 && (!ws || ws_bytes < (int64_t)splits * M * N * 4)) return GNNEA_EWORKSPACE;
  const int kps = (int)(((K + splits - 1) / splits + GBK - 1) / GBK * GBK);
  float* slab = splits > 1 ? (float*)ws : nullptr;
  // float4 loads run along M (A) and N (B): both must be 4-aligned
  const bool vec = lda % 4 == 0 && M % 4 == 0 && al16(A) && ldb % 4 == 0 && N % 4 == 0 && al16(B);
  const dim3 grid(tiles, splits);
#define GNNEA_X3T(W)                                                                             \
  case W:                                                                                        \
    if (vec)                                                                                     \
      hipLaunchKernelGGL((k_gemm_x3<W, true, true>), grid, dim3(XNT), 0, s, (int)M, (int)N,      \
                         (int)K, A, lda, nullptr, (int64_t)0, (int64_t)0, B, ldb, bias, beta, C, \
                         ldc, cs, kps, slab, tiles_n);                                           \
    else                                                                                         \
      hipLaunchKernelGGL((k_gemm_x3<W, false, true>), grid, dim3(XNT), 0, s, (int)M, (int)N,     \
                         (int)K, A, lda, nullptr, (int64_t)0, (int64_t)0, B, ldb, bias, beta, C, \
                         ldc, cs, kps, slab, tiles_n);                                           \
    break;
  switch (wt) {
    GNNEA_X3T(1)
    GNNEA_X3T(2)
    GNNEA_X3T(3)
    GNNEA_X3T(4)
    default:
    GNNEA_X3T(5)
  }
#undef GNNEA_X3T
  GNNEA_LAUNCH_CHECK();
  if (splits > 1) {
    const int64_t n = M * N;
    const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
    hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, splits, slab,
                       bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

extern "C" int64_t gnnea_gemm_x3t_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  const int64_t a = x3_ta_splits(M, N, K, INT64_MAX / 2) * M * N * 4;
  const int64_t b = gemm_ta_ws_bytes(M, N, K);  // whole-width form (gemm_ta.hip)
  return a > b ? a : b;
}

extern "C" int64_t gnnea_gemm_x3_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  return x3_planes_bytes(N, K) + pick_splits(M, N, K, INT64_MAX / 2) * M * N * 4;
}

extern "C" int gnnea_gemm_x3_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda,
                                           int64_t ldb) {
  const void* dummy = (const void*)(uintptr_t)256;  // (alignment is checked on the real call)
  return gemm_ta_db_applies(M, N, K, lda, ldb, dummy, dummy, 4) ? 1 : 0;
}

extern "C" int64_t gnnea_gemm_x3_ta_db_ws_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  return gemm_ta_db_ws_bytes(M, N, K);
}

// The weight and bias gradients of one Linear-like layer in one pass over its output gradient:
// C = Aᵀ·B (A [K][M] = dh, B [K][N] = x; gnnea_gemm_x3_f32's trans_a product, the same kernel and
// values) and db = column sums of A (fp32 [M]), from the kernel's ones column in B's tile padding
// (N % 160 != 0; gnnea_gemm_x3_ta_db_applies).  Replaces gnnea_colsum_f32's separate pass over A.
extern "C" int gnnea_gemm_x3_ta_db_f32(int64_t M, int64_t N, int64_t K, const float* A,
                                       int64_t lda, const float* B, int64_t ldb, float* C,
                                       int64_t ldc, float* db, void* ws, int64_t ws_bytes,
                                       void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C || !db || ldc < N) return GNNEA_EINVAL;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!gemm_ta_db_applies(M, N, K, lda, ldb, A, B, 4)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float* slab = nullptr;
  float* dbslab = nullptr;
  int used = 0;
  const int rc = gemm_ta_launch<float>(M, N, K, A, lda, B, ldb, ws, ws ? ws_bytes : 0, s, &slab,
                                       &used, &dbslab);
  if (rc) return rc;
  const int64_t n = M * N;
  const int nb = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(k_gemm_reduce, dim3(nb), dim3(256), 0, s, (int)M, (int)N, used, slab,
                     nullptr, 0.f, C, ldc, (int64_t)64);
  GNNEA_LAUNCH_CHECK();
  return ta_db_reduce(M, used, dbslab, db, s);
}

// fp32 GEMM through three-way bf16 splits on the bf16 MFMA (k_gemm_x3); workspace from
// gnnea_gemm_x3_ws_bytes (the split planes of op(B) + split-K slabs)
extern "C" int gnnea_gemm_x3_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                 const float* A, int64_t lda, const float* B, int64_t ldb,
                                 const float* bias, float beta, float* C, int64_t ldc, void* ws,
                                 int64_t ws_bytes, void* stream) {
  return gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, 64, ws, ws_bytes,
                 stream);
}

// C = act(A·op(B) + bias): the Linear layer with its act (layers/layers.py:121-122); relu rides
// the weight-resident ring's epilogue, any other (kernel, act) pair runs the act in place after
extern "C" int gnnea_gemm_x3_act_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                     const float* A, int64_t lda, const float* B, int64_t ldb,
                                     const float* bias, int act, float* C, int64_t ldc, void* ws,
                                     int64_t ws_bytes, void* stream) {
  if (act < GNNEA_ACT_IDENTITY || act > GNNEA_ACT_TANH) return GNNEA_EINVAL;
  return gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, 0.f, C, ldc, 64, ws, ws_bytes,
                 stream, nullptr, 0, act);
}

// C row-major AND its slice-major copy C2s [ceil(N/64)][M][64] (slice stride sstride2) from one
// GEMM: the second store rides the epilogue of k_gemm_x3p (the GAT projection feeds the
// row-major backward and the sliced forward aggregation)
extern "C" int gnnea_gemm_x3_dual_f32(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                      const float* A, int64_t lda, const float* B, int64_t ldb,
                                      const float* bias, float beta, float* C, int64_t ldc,
                                      float* C2s, int64_t sstride2, void* ws, int64_t ws_bytes,
                                      void* stream) {
  if (!C2s) return GNNEA_EINVAL;
  return gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, 64, ws, ws_bytes,
                 stream, C2s, sstride2);
}

extern "C" int gnnea_gemm_x3_sliced_f32(int trans_a, int trans_b, int64_t M, int64_t N,
                                        int64_t K, const float* A, int64_t lda, const float* B,
                                        int64_t ldb, const float* bias, float beta, float* Cs,
                                        int64_t sstride, void* ws, int64_t ws_bytes,
                                        void* stream) {
  if (sstride % 4 != 0) return GNNEA_EINVAL;
  return gemm_x3(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, Cs, 64, sstride, ws,
                 ws_bytes, stream);
}
