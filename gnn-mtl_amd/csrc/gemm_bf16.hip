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
#include "gemm_ta.h"
#include "lds_dma.h"
#include "act.h"

#include <stdlib.h>

#include <type_traits>

namespace gnnea {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16_b __attribute__((ext_vector_type(16)));

constexpr int HBM = 64, HBK = 32, HLD = HBK + 8;
constexpr bool TRANS_QUADS = true;  // (false: HLoader's 2-B transposing stores, slower)

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

// ---- k_gemm_bf16p: the projection form (A [M][K] K-contiguous bf16, B the small weight) on the
// persistent LDS-DMA pipeline of gemm.hip's k_gemm_x3p, one product instead of six.
// k_gemm_bf16 above re-stages the whole 300 x 300 weight through registers for every 64-row tile,
// keeps one k-step of loads in flight and runs a 10-step k-loop per tile (cfg-5, 4M x 300 x 300:
// 2.8 ms = 1.7 TB/s of the 4.8 GB of compulsory I/O).  Here one 512-thread workgroup per CU walks
// its 256-row x 32*WT-column tiles as ONE stream of 32-deep k-stages through a 4-stage LDS ring
// filled by global_load_lds (no registers): the next tile's stages land while the current tile's
// last ones are multiplied, and a tile's epilogue (through LDS, whole 8-B / 16-B row chunks) runs
// while the next tile's stages land.  A stage = the A tile (256 rows x 64 B) and the B tile
// (32*WT rows x 64 B) of the weight, pre-packed once per call k-block-major ([kb][NP][32] bf16,
// zero-padded; with a bias, rows k = K, K+1, K+2 hold it split three ways into bf16 and A gets
// ones there: the bias joins the fp32 accumulation exactly).  A rows of K = 300 bf16 are 600 B:
// 16-B LDS-DMA granules from 4-B aligned addresses are exact on gfx950
// (tools/ubench/probe_glds.hip); the granule at k = 296 runs 4 elements into the next row, which
// the k-mask zeroes, so the last row (no next row) is left to the register-staged kernel
// (gemm_bf16p).  AW = 4 (4-B granules, no overrun) is kept as an alternative: 2.27 vs 2.02 ms
// at 4M x 300 x 300 measured for the 16-B form.  LDS images are lane-linear; the bank swizzle (16-B slot s of row r at
// s ^ ((r >> 2) & 3), as k_gemm_x3p's A) goes on the source addresses and the reads.
template <int WT, int AW, int NW_>
struct BFP {
  static constexpr int NW = NW_, BM = 32 * NW, NT = 64 * NW, BN = 32 * WT;
  static constexpr int KS = 32;                                  // k per stage (2 MFMA k-steps)
  static constexpr int A_BYTES = BM * KS * 2;                    // 16 KB
  static constexpr int A_LOADS = A_BYTES / (64 * AW) / NW;       // per wave: 2 (AW 16), 8 (AW 4)
  static constexpr int B_CHUNKS = BN * KS * 2 / 1024;            // 1-KB chunks of 16 rows
  // every wave DMAs B_FULL chunks, waves w < B_EXTRA one more (no padding chunks)
  static constexpr int B_FULL = B_CHUNKS / NW, B_EXTRA = B_CHUNKS % NW;
  static constexpr int EPI_BYTES = NW * 32 * 32 * 4;            // the waves' epilogue regions
  static constexpr int STAGE = A_BYTES + B_CHUNKS * 1024 > EPI_BYTES ? A_BYTES + B_CHUNKS * 1024
                                                                     : EPI_BYTES;
  static constexpr int LOADS_LO = A_LOADS + B_FULL;              // DMA instr. / wave / stage
  static constexpr int LOADS_HI = LOADS_LO + (B_EXTRA ? 1 : 0);
  static constexpr int NS = 4;
  static constexpr int EPI_LD = 32;                              // epilogue row stride (floats)
  static_assert(NW * 32 * EPI_LD * 4 <= STAGE, "epilogue regions must fit one stage");
  static_assert(NS * STAGE <= 160 * 1024, "LDS");
};

// 32 x 32 accumulator tile -> C (TC = bf16 / fp32) through the wave's private LDS region: lanes
// write their column, read a row's consecutive columns back and store them as one 16-B chunk:
// 8 bf16 columns (two stores per lane per tile) or 4 fp32 columns (four).  vec: EXACTLY that many
// stores per lane (out-of-range lanes to `dummy`), which the k-loop's vmcnt waits count.
// Element (row, col) at c_index_bf(row, col, ldc, cs).
template <typename TC>
struct BfpEpi {
  static constexpr int CPL = 16 / sizeof(TC);  // columns per lane-store
  static constexpr int STORES = 32 * 32 / 64 / CPL;
};
template <typename TC>
__device__ __forceinline__ void bfp_store_tile(const f32x16_b& acc, uint32_t region, int M, int N,
                                               int m_w, int n_t, int kh, int li, int lane,
                                               float beta, TC* __restrict__ C, int64_t ldc,
                                               int64_t cs, bool vec, TC* __restrict__ dummy) {
  constexpr int LD = 32, CPL = BfpEpi<TC>::CPL, RPI = 64 / (32 / CPL);  // rows per instruction
  const uint32_t wb = region + (4 * kh) * LD * 4 + li * 4;
#pragma unroll
  for (int r = 0; r < 16; ++r) ds_write32(wb + ((r & 3) + 8 * (r >> 2)) * LD * 4, acc[r]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const int lr = lane / (32 / CPL), lc = (lane % (32 / CPL)) * CPL;  // row in the group, column
  const uint32_t rbase = region + lr * LD * 4 + lc * 4;
  f32x4_t v[2 * BfpEpi<TC>::STORES];
#pragma unroll
  for (int i = 0; i < BfpEpi<TC>::STORES; ++i) {
    v[2 * i] = ds_read128f(rbase + i * RPI * LD * 4);
    if (CPL == 8) v[2 * i + 1] = ds_read128f(rbase + i * RPI * LD * 4 + 16);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < BfpEpi<TC>::STORES; ++i) {
    const int grow = m_w + lr + RPI * i, gcol = n_t + lc;
    float o[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      o[e] = v[2 * i][e];
      o[4 + e] = CPL == 8 ? v[2 * i + 1][e] : 0.f;
    }
    if (vec) {
      const bool ok = grow < M && gcol < N;
      TC* c = ok ? C + c_index_bf(grow, gcol, ldc, cs) : dummy + CPL * lane;
      if (beta != 0.f && ok) {
#pragma unroll
        for (int e = 0; e < CPL; ++e) o[e] += beta * to_f32<TC>(c[e]);
      }
      if constexpr (CPL == 8) {
        uint4 u;
        u.x = (uint32_t)f32_to_bf16(o[0]) | ((uint32_t)f32_to_bf16(o[1]) << 16);
        u.y = (uint32_t)f32_to_bf16(o[2]) | ((uint32_t)f32_to_bf16(o[3]) << 16);
        u.z = (uint32_t)f32_to_bf16(o[4]) | ((uint32_t)f32_to_bf16(o[5]) << 16);
        u.w = (uint32_t)f32_to_bf16(o[6]) | ((uint32_t)f32_to_bf16(o[7]) << 16);
        // the row's last chunk may hold 4 columns (N % 8 == 4): one 8-B store (still ONE store)
        if (!ok || gcol + 8 <= N) *(uint4*)c = u;
        else *(uint2*)c = make_uint2(u.x, u.y);
      } else {
        *(float4*)c = make_float4(o[0], o[1], o[2], o[3]);
      }
    } else if (grow < M) {
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        if (gcol + e >= N) continue;
        TC* c = C + c_index_bf(grow, gcol + e, ldc, cs);
        float x = o[e];
        if (beta != 0.f) x += beta * to_f32<TC>(*c);
        *c = from_f32<TC>(x);
      }
    }
  }
}

// Two adjacent 32 x 32 tiles -> bf16 C as 64-column (128-B) row pieces: the tile pair is rounded
// to bf16 into the wave's [32][64] LDS region (4 KB; 16-B chunk c of row r at c ^ (r & 7)), read
// back as 8 rows x 8 chunks per instruction and stored as 16-B chunks, 128 B of every row per
// instruction (a single tile leaves 64-B row pieces, which measured 0.8 ms of stores at
// 4M x 300: 2.4 GB).  EXACTLY four stores per lane when vec (dummy for out-of-range lanes; a row's
// last chunk with 4 valid columns is one 8-B store).
__device__ __forceinline__ void ds_write16(uint32_t addr, uint32_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(addr), "v"(v));
}
__device__ __forceinline__ void bfp_store_pair_bf16(const f32x16_b& a0, const f32x16_b& a1,
                                                    uint32_t region, int M, int N, int m_w,
                                                    int n_t, int kh, int li, int lane,
                                                    bf16_t* __restrict__ C, int64_t ldc,
                                                    int64_t cs, bf16_t* __restrict__ dummy) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int col = 32 * ct + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * kh;
      const uint32_t a = region + row * 128 + 16 * ((col >> 3) ^ (row & 7)) + 2 * (col & 7);
      ds_write16(a, (uint32_t)f32_to_bf16(ct == 0 ? a0[r] : a1[r]));
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  u32x4 v[4];
  const int lr = lane >> 3, ch = lane & 7;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = lr + 8 * i;
    v[i] = ds_read128(region + row * 128 + 16 * (ch ^ (row & 7)));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int grow = m_w + lr + 8 * i, gcol = n_t + 8 * ch;
    const bool ok = grow < M && gcol < N;
    bf16_t* c = ok ? C + c_index_bf(grow, gcol, ldc, cs) : dummy + 8 * lane;
    const uint4 u = make_uint4(v[i].x, v[i].y, v[i].z, v[i].w);
    if (!ok || gcol + 8 <= N) *(uint4*)c = u;
    else *(uint2*)c = make_uint2(u.x, u.y);
  }
}

// wait for this wave's DMA of the stage about to be read, with `later` stages issued after it
// still in flight (and, right after an epilogue, that epilogue's ST stores, issued between)
template <int L, int NS, int ST>  // ST: the epilogue's stores per lane
__device__ __forceinline__ void bfp_wait(int later, bool stores_after) {
  if (later == NS - 2 && stores_after)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NS - 2) + ST) : "memory");
  else if (later == NS - 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L * (NS - 2)) : "memory");
  else if (later == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int WT, int AW, int NW_, typename TC>
__global__ __launch_bounds__(64 * NW_) void k_gemm_bf16p(int M, int N, int K,
                                                   const bf16_t* __restrict__ A, int64_t lda,
                                                   const bf16_t* __restrict__ Bp, int NP, int hb,
                                                   float beta, TC* __restrict__ C, int64_t ldc,
                                                   int64_t cs, int tiles_n, int ntiles, int vec,
                                                   TC* __restrict__ dummy) {
  using G = BFP<WT, AW, NW_>;
  constexpr int NW = G::NW, NS = G::NS;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NS * G::STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kh = lane >> 5, li = lane & 31;
  const int nsteps = (K + (hb ? 3 : 0) + G::KS - 1) / G::KS;
  const int gsz = gridDim.x;
  const int nq = (int)blockIdx.x < ntiles ? (ntiles - (int)blockIdx.x + gsz - 1) / gsz : 0;
  const int total = nq * nsteps;
  auto tile_of = [&](int q, int& m0, int& n0) {
    const int t_id = xcd_remap((int)blockIdx.x + q * gsz, ntiles);
    m0 = (t_id / tiles_n) * G::BM;
    n0 = (t_id % tiles_n) * G::BN;
  };

  // ---- issue side: the next stage of the stream (tile iq, k-stage is) ----
  int iq = 0, is = 0;
  const bf16_t* a_src[G::A_LOADS];  // row base + the lane's (swizzled) k offset in the stage
  int a_koff[G::A_LOADS];
  const bf16_t* b_src[G::B_FULL + 1];
  const bool b_extra = G::B_EXTRA > 0 && w < G::B_EXTRA;  // wave-uniform
  auto set_issue_tile = [&](int q) {
    int m0, n0;
    tile_of(q, m0, n0);
#pragma unroll
    for (int i = 0; i < G::A_LOADS; ++i) {
      const int ci = w + NW * i;  // the workgroup's i-th A instruction of this wave
      int row, koff;
      if (AW == 16) {  // 16 rows x 4 slots of 16 B
        row = 16 * ci + (lane >> 2);
        koff = 8 * ((lane & 3) ^ ((row >> 2) & 3));
      } else {  // 4 rows x 16 dwords
        row = 4 * ci + (lane >> 4);
        koff = 8 * (((lane >> 2) & 3) ^ ((row >> 2) & 3)) + 2 * (lane & 3);
      }
      a_koff[i] = koff;
      a_src[i] = A + (int64_t)min(m0 + row, M - 1) * lda;
    }
#pragma unroll
    for (int i = 0; i <= G::B_FULL; ++i) {
      const int cb = i < G::B_FULL ? w + NW * i : NW * G::B_FULL + (b_extra ? w : 0);
      const int row = 16 * cb + (lane >> 2);
      b_src[i] = Bp + (int64_t)(n0 + row) * G::KS + 8 * ((lane & 3) ^ ((row >> 2) & 3));
    }
  };
  auto issue_next = [&](int buf) {
    if (is == 0) set_issue_tile(iq);
    unsigned char* st = smem + buf * G::STAGE;
    const int k0 = is * G::KS;
#pragma unroll
    for (int i = 0; i < G::A_LOADS; ++i) {
      // a granule past K reads the row's k = 0 (valid) and is zeroed at use
      const int k = k0 + a_koff[i];
      const bf16_t* ap = a_src[i] + (k < K ? k : 0);
      if (AW == 16) glds16(ap, st + (w + NW * i) * 1024);
      else glds4(ap, st + (w + NW * i) * 256);
    }
#pragma unroll
    for (int i = 0; i < G::B_FULL; ++i)
      glds16(b_src[i] + (int64_t)is * NP * G::KS, st + G::A_BYTES + (w + NW * i) * 1024);
    if (b_extra)
      glds16(b_src[G::B_FULL] + (int64_t)is * NP * G::KS,
             st + G::A_BYTES + (NW * G::B_FULL + w) * 1024);
    if (++is == nsteps) { is = 0; ++iq; }
  };

  f32x16_b acc[WT];
#pragma unroll
  for (int t = 0; t < WT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // per-lane LDS read offsets (bytes within a stage); rows of 64 B, slot 2*ks + kh swizzled
  const int ra = w * 32 + li;
  const int a_off[2] = {ra * 64 + 16 * ((0 + kh) ^ ((ra >> 2) & 3)),
                        ra * 64 + 16 * ((2 + kh) ^ ((ra >> 2) & 3))};
  // B row t*32 + li: (row >> 2) & 3 is li's, so tile t's offset is b_off + t * 2 KB
  const int b_off[2] = {G::A_BYTES + li * 64 + 16 * ((0 + kh) ^ ((li >> 2) & 3)),
                        G::A_BYTES + li * 64 + 16 * ((2 + kh) ^ ((li >> 2) & 3))};
  const uint32_t smem_lds = lds_addr(smem);
  auto epilogue = [&](int q, int buf) {
    int m0, n0;
    tile_of(q, m0, n0);
    const uint32_t region = smem_lds + buf * G::STAGE + w * 32 * G::EPI_LD * 4;
    if constexpr (std::is_same<TC, bf16_t>::value) {
      if (vec != 0 && beta == 0.f) {  // tile pairs as 128-B row pieces
#pragma unroll
        for (int t = 0; t + 1 < WT; t += 2)
          bfp_store_pair_bf16(acc[t], acc[t + 1], region, M, N, m0 + w * 32, n0 + 32 * t, kh, li,
                              lane, C, ldc, cs, dummy);
        if (WT % 2)
          bfp_store_tile<TC>(acc[WT - 1], region, M, N, m0 + w * 32, n0 + 32 * (WT - 1), kh, li,
                             lane, beta, C, ldc, cs, true, dummy);
        return;
      }
    }
#pragma unroll
    for (int t = 0; t < WT; ++t)
      bfp_store_tile<TC>(acc[t], region, M, N, m0 + w * 32, n0 + 32 * t, kh, li, lane, beta, C,
                         ldc, cs, vec != 0, dummy);
  };
  // vmcnt allowance for the first steps after an epilogue: its stores (exactly 4 per tile when
  // vec and no beta loads) were issued after the DMA those steps wait for
  // epilogue stores per lane: bf16 tile pairs 4 + a single tile 2 (= 2 per tile), fp32 4 per tile
  constexpr int ST = BfpEpi<TC>::STORES * WT;
  const bool count_stores = vec != 0 && beta == 0.f && G::LOADS_HI * (NS - 2) + ST <= 63;

#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < total) issue_next(i);
  int cur = 0, s = 0, q = 0;
  for (int g = 0; g < total; ++g) {
    const bool epi = s == 0 && q > 0;
    {
      const int later = total - 1 - g < NS - 2 ? total - 1 - g : NS - 2;  // stages issued after g
      const bool st_after = count_stores && q > 0 && s >= 1 && s <= NS - 2;
      if (b_extra) bfp_wait<G::LOADS_HI, NS, ST>(later, st_after);
      else bfp_wait<G::LOADS_LO, NS, ST>(later, st_after);
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
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 araw = ds_read128(st + a_off[ks]);
      u32x4 braw[WT];
      static_for<WT>([&](auto tt) {
        constexpr int t = decltype(tt)::value;
        braw[t] = ds_read128_o<t * 2048>(st + b_off[ks]);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int kb0 = s * G::KS + ks * 16 + 8 * kh;  // this lane's first k
      if (kb0 + 8 > K) {  // past K: zeros; ones at k = K, K+1, K+2 under a bias
        uint32_t d[4] = {araw.x, araw.y, araw.z, araw.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = kb0 + j;
          const uint32_t val = k < K ? ((d[j >> 1] >> (16 * (j & 1))) & 0xffffu)
                                     : ((hb && k < K + 3) ? 0x3f80u : 0u);
          d[j >> 1] = (d[j >> 1] & ~(0xffffu << (16 * (j & 1)))) | (val << (16 * (j & 1)));
        }
        araw = u32x4{d[0], d[1], d[2], d[3]};
      }
      const bf16x8 a = __builtin_bit_cast(bf16x8, araw);
#pragma unroll
      for (int t = 0; t < WT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, __builtin_bit_cast(bf16x8, braw[t]),
                                                         acc[t], 0, 0, 0);
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

// the weight op(B) [N][K] packed k-block-major for k_gemm_bf16p: P[kb][r][32] bf16, r < NP (the
// column tiles' rows, zero past N), kb < KP / 32; with a bias, rows k = K, K+1, K+2 hold it split
// into three bf16 terms (h + m + l = bias to fp32 rounding; A's ones there add it exactly in fp32)
__global__ __launch_bounds__(256) void k_pack_bf16_planes(const bf16_t* __restrict__ B,
                                                          int64_t ldb, int b_nk, int N, int K,
                                                          int NP, int KP,
                                                          const float* __restrict__ bias,
                                                          bf16_t* __restrict__ P) {
  const int64_t total = (int64_t)NP * KP;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int kb = (int)(t / ((int64_t)NP * 32));
    const int rem = (int)(t - (int64_t)kb * NP * 32);
    const int r = rem / 32, k = kb * 32 + rem % 32;
    bf16_t v = 0;
    if (r < N) {
      if (k < K) {
        v = b_nk ? B[(int64_t)r * ldb + k] : B[(int64_t)k * ldb + r];
      } else if (bias && k < K + 3) {
        const float x = bias[r];
        const bf16_t h = f32_to_bf16(x);
        const float r1 = x - bf16_to_f32(h);
        const bf16_t m = f32_to_bf16(r1);
        v = k == K ? h : (k == K + 1 ? m : f32_to_bf16(r1 - bf16_to_f32(m)));
      }
    }
    P[t] = v;
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

template <int TA, int TB, int WT, typename TC>
static void launch_bf16_wt(dim3 grid, hipStream_t s, bool vec, int M, int N, int K,
                           const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                           const float* bias, float beta, TC* C, int64_t ldc, int64_t cs,
                           int kps, float* slab, int tiles_n) {
  if constexpr (std::is_same<TC, bf16_t>::value) {
    if (vec && !slab && beta == 0.f && (((uintptr_t)C) & 7) == 0 && ldc % 4 == 0 &&
        cs % 4 == 0) {  // the LDS-staged epilogue: 128-B row pieces
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

// k_gemm_bf16p applies to the tall projection form: A [M][K] K-contiguous (rows 4-B aligned, K
// even), M >= 64K rows, the whole output 2 column tiles of 160 at most per 320 (N > 128)
static bool bf16p_applies(int trans_a, int64_t M, int64_t N, int64_t K, int64_t lda,
                          const void* A) {
  return !trans_a && M >= 65536 && N > 128 && N <= 4096 && K > 0 && K % 2 == 0 &&
         lda % 2 == 0 && (((uintptr_t)A) & 3) == 0;
}
// column tile of k_gemm_bf16p: 32 * 5 = 160 columns (a 320-wide tile that reads A once at
// N = 300 needs 160 accumulator registers per lane: at two waves per SIMD it spilled to scratch,
// 36 ms at 4M x 300 x 300 against 2.2 ms)
constexpr int kBf16pWT = 5;
static int64_t bf16p_planes_bytes(int64_t N, int64_t K) {  // + a 2-KB dummy store target
  const int64_t np = (N + 319) / 320 * 320, kp = (K + 3 + 31) / 32 * 32;
  return ((np * kp * 2 + 255) & ~(int64_t)255) + 2048;
}

template <int WT, int AW, int NW, typename TC>
static void launch_bf16p(hipStream_t s, int grid, int M, int N, int K, const bf16_t* A,
                         int64_t lda, const bf16_t* P, int NP, int hb, float beta, TC* C,
                         int64_t ldc, int64_t cs, int tiles_n, int ntiles, int vec, TC* dummy) {
  hipLaunchKernelGGL((k_gemm_bf16p<WT, AW, NW, TC>), dim3(grid), dim3(64 * NW), 0, s, M, N, K,
                     A, lda, P, NP, hb, beta, C, ldc, cs, tiles_n, ntiles, vec, dummy);
}

// waves per workgroup: 8 (256-row tiles, one workgroup per CU) or 4 (128-row tiles, two per CU:
// one's barriers and epilogue under the other's MFMAs); 8 measured faster at the cfg-5 shapes
static int bf16p_nw() { return 8; }

template <typename TC>
static int gemm_bf16_t(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                       const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                       const float* bias, float beta, TC* C, int64_t ldc, void* ws,
                       int64_t ws_bytes, hipStream_t s, int64_t cs = 128,
                       int act = GNNEA_ACT_IDENTITY);

template <typename TC>
static int gemm_bf16p(int trans_b, int64_t M, int64_t N, int64_t K, const bf16_t* A,
                      int64_t lda, const bf16_t* B, int64_t ldb, const float* bias, float beta,
                      TC* C, int64_t ldc, int64_t cs, void* ws, hipStream_t s) {
  constexpr int BN = 32 * kBf16pWT;
  const int NP = (int)((N + BN - 1) / BN * BN), KP = (int)((K + 3 + 31) / 32 * 32);
  bf16_t* P = (bf16_t*)ws;
  TC* dummy = (TC*)((char*)ws + bf16p_planes_bytes(N, K) - 2048);
  {
    const int64_t tot = (int64_t)NP * KP;
    const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
    hipLaunchKernelGGL(k_pack_bf16_planes, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 1 : 0,
                       (int)N, (int)K, NP, KP, bias, P);
    GNNEA_LAUNCH_CHECK();
  }
  // A in 16-B granules: a row's last granule may run (8 - K % 8) % 8 elements past K, into the
  // row's padding or the next row (zeroed at use); the last row has no next row, so without
  // enough padding it is computed by the register-staged kernel instead
  const int over = (8 - (int)(K % 8)) % 8;
  const int64_t Mp = lda - K >= over ? M : M - 1;
  const int nw = bf16p_nw();
  const int tiles_n = NP / BN;
  const int64_t tm = (Mp + 32 * nw - 1) / (32 * nw);
  if (tm * tiles_n >= (1ll << 31)) return GNNEA_EINVAL;
  const int ntiles = (int)(tm * tiles_n);
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int per_cu = nw == 8 ? 1 : 2;  // persistent: as many workgroups as fit at once
  const int grid = ntiles < per_cu * ncu ? ntiles : per_cu * ncu;
  const int vec = N % 4 == 0 && ldc % 4 == 0 && cs % 4 == 0 &&
                  (((uintptr_t)C) & (4 * sizeof(TC) - 1)) == 0;
  if (nw == 8)
    launch_bf16p<5, 16, 8, TC>(s, grid, (int)Mp, (int)N, (int)K, A, lda, P, NP, bias != nullptr,
                               beta, C, ldc, cs, tiles_n, ntiles, vec, dummy);
  else
    launch_bf16p<5, 16, 4, TC>(s, grid, (int)Mp, (int)N, (int)K, A, lda, P, NP, bias != nullptr,
                               beta, C, ldc, cs, tiles_n, ntiles, vec, dummy);
  GNNEA_LAUNCH_CHECK();
  if (Mp < M)  // the last row (its own launch; no workspace: no split-K)
    return gemm_bf16_t<TC>(0, trans_b, 1, N, K, A + Mp * lda, lda, B, ldb, bias, beta,
                           C + Mp * ldc, ldc, nullptr, 0, s, cs);
  return 0;
}

// ---- k_gemm_bf16w: the projection form with the weight RESIDENT in LDS and the activations
// streamed straight into registers (no LDS staging, no barrier in the k-loop).  For the cfg-5
// shapes (K <= 320, a 160-column weight tile = 97 KB bf16 fits the LDS) the product is computed
// transposed, D^T = W_tile . A^T on v_mfma_f32_32x32x16_bf16: the weight tile is the MFMA's A
// operand (ds_read_b128 from the resident image), 32 activation rows per wave are its B operand
// (one 16-B global load per lane per k-step), and a lane's accumulators come out as runs of 4
// consecutive output COLUMNS of one row -- stored as 8-B (bf16) / 16-B (fp32) pieces straight
// from registers.  The k dimension is permuted (A and W alike): lanes of k-half kh hold k in
// [kh Kh + 8 s, +8) at step s, Kh = 8 kc, so each lane streams one contiguous run of its row.
// One wave per SIMD (512 registers): the next tile's activations (kc fragments) are in flight
// while the current tile is multiplied.  Workgroup b owns column tile (b / 8) % ntn and the row
// stream of the blocks b and b + 8 * (ntn - 1)... (so the column tiles of the same rows run on
// one XCD, sharing its L2 for the activations).
// (Staging a wave's bf16 output tile in LDS to store 16-B row pieces measured 6-8 % slower,
// profiles/r04_gemm_bf16_epilogue_ab.json; two register sets of activations in flight measured
// the same as three, and a k permutation reading 32 contiguous bytes per row the same as
// 16 B from each of 64 rows: none kept.)
constexpr int kBwCols = 160, kBwKC = 20;  // column tile, max k-steps (K <= 320)

__global__ __launch_bounds__(256) void k_pack_bf16w(const bf16_t* __restrict__ B, int64_t ldb,
                                                    int b_nk, int N, int K, int kc, int ntn,
                                                    bf16_t* __restrict__ P) {
  // P[nt][s][kh][n][8]: element e = W_op[nt*160 + n][kh*8kc + 8s + e] (zero outside)
  const int64_t total = (int64_t)ntn * kc * 2 * kBwCols * 8;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int e = (int)(t & 7);
    int64_t r = t >> 3;
    const int n = (int)(r % kBwCols);
    r /= kBwCols;
    const int kh = (int)(r & 1);
    r >>= 1;
    const int s = (int)(r % kc);
    const int nt = (int)(r / kc);
    const int col = nt * kBwCols + n, k = kh * 8 * kc + 8 * s + e;
    bf16_t v = 0;
    if (col < N && k < K) v = b_nk ? B[(int64_t)col * ldb + k] : B[(int64_t)k * ldb + col];
    P[t] = v;
  }
}

// Epilogue modes EP (bf16 out):
//  1 (the backward of a relu Linear whose output y fed this product): the stored value is
//    g = bf16(acc) * relu'(y) at the same position (act_bwd_colsum's g on the product it would
//    read, bit for bit), y read for the tile before the next tile's activations are issued;
//  2 the same with relu'(y) from the sign bits mode 3 wrote (Ym: 1 bit per element instead of
//    16: 20 bytes per row and column tile, byte 4 t + g of a tile holds columns 32 t + 8 g + 0..7);
//  3 (the forward of that relu Linear) relu as mode 0, and the sign bits of the stored y -> Mo.
// (Column sums of g kept per lane across the tiles as well -- 80 more registers -- spilled: the
// bias gradient is a separate streaming pass over g.)
template <typename TC, int KC, int EP = 0>
__global__ __launch_bounds__(256, 1) void k_gemm_bf16w(int M, int N, int K, int ntn,
                                                      const bf16_t* __restrict__ A, int64_t lda,
                                                      const bf16_t* __restrict__ P,
                                                      const float* __restrict__ bias,
                                                      TC* __restrict__ C, int64_t ldc,
                                                      int64_t cs, int relu,
                                                      const void* __restrict__ Ym = nullptr,
                                                      int64_t ldym = 0,
                                                      uint8_t* __restrict__ Mo = nullptr,
                                                      int64_t ldmo = 0) {
  static_assert(EP == 0 || std::is_same<TC, bf16_t>::value, "the masked forms store bf16");
  constexpr bool DM = EP == 1 || EP == 2;
  __shared__ __attribute__((aligned(16))) uint4 wl[KC * 2 * kBwCols];  // [s][kh][n] x 16 B
  // the tile's bias in LDS: a global load in the epilogue would wait (vmcnt counts in order)
  // for the next tile's activation loads issued before it
  __shared__ __attribute__((aligned(16))) float bsh[kBwCols];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kh = lane >> 5, li = lane & 31;
  const int b = blockIdx.x;
  const int nt = (b / 8) % ntn;
  const int rs = (b / (8 * ntn)) * 8 + b % 8, nrs = (int)gridDim.x / ntn;
  const int n0 = nt * kBwCols;
  constexpr int Kh = 8 * KC;
  {  // the resident weight tile
    const uint4* src = (const uint4*)(P + (int64_t)nt * KC * 2 * kBwCols * 8);
    for (int i = tid; i < KC * 2 * kBwCols; i += 256) wl[i] = src[i];
    if (tid < kBwCols) bsh[tid] = bias && n0 + tid < N ? bias[n0 + tid] : 0.f;
  }
  __syncthreads();
  const int tm = (M + 127) / 128;  // 128-row tiles: 4 waves x 32 rows
  // one k-step fragment of the lane's row: 8 bf16 at k = kh Kh + 8 s.  Only the last steps can reach K (K > 16 (KC - 1)); there a chunk holding K is read
  // as the 16 B ending at K (in bounds, K even) and a chunk past K reads the same 16 B; both
  // are fixed up when they are USED (tail_fix: shifted down by words / zeroed).  Fixing them
  // up here, as loads are issued, made the compiler wait vmcnt(0) right after the next tile's
  // loads — the whole tile's load latency exposed every tile (0.89 ms -> see DESIGN §9).
  constexpr int s_tail = KC - 2;
  auto k0_of = [&](int s) { return kh * Kh + 8 * s; };
  auto issue = [&](uint4 (&f)[KC], int rt) {
    const bf16_t* row = A + (int64_t)min(rt * 128 + w * 32 + li, M - 1) * lda;
#pragma unroll
    for (int s = 0; s < s_tail; ++s) f[s] = *(const uint4*)(row + k0_of(s));
#pragma unroll
    for (int s = s_tail; s < KC; ++s) {
      const int k0 = k0_of(s);
      f[s] = *(const uint4*)(row + (k0 + 8 <= K ? k0 : K - 8));
    }
  };
  auto tail_fix = [&](int s, uint4 v) {
    if (s < s_tail) return v;
    const int k0 = k0_of(s);
    if (k0 + 8 <= K) return v;
    if (k0 >= K) return make_uint4(0, 0, 0, 0);
    const int sh = (k0 + 8 - K) >> 1;  // 1..3 words
    return make_uint4(sh == 1 ? v.y : (sh == 2 ? v.z : v.w), sh == 1 ? v.z : (sh == 2 ? v.w : 0u),
                      sh == 1 ? v.w : 0u, 0u);
  };
  const uint4* wlane = wl + kh * kBwCols + li;  // + (2 s) * 160 + 32 t
  // EP 1: the tile's y pieces (the output positions, clamped in bounds: unconditional loads);
  // EP 2: the row's 20 sign bytes of this column tile
  uint2 ym[EP == 1 ? 20 : 1];
  uint32_t mb[EP == 2 ? 5 : 1];
  auto load_y = [&](int rt) {
    const int64_t m = min(rt * 128 + w * 32 + li, M - 1);
    if constexpr (EP == 1) {
#pragma unroll
      for (int q = 0; q < 20; ++q) {
        const int n = min(n0 + 32 * (q >> 2) + 8 * (q & 3) + 4 * kh, N - 4);
        ym[q] = *(const uint2*)((const bf16_t*)Ym + m * ldym + n);
      }
    } else if constexpr (EP == 2) {
      const uint32_t* mp = (const uint32_t*)((const uint8_t*)Ym + m * ldym + nt * 20);
#pragma unroll
      for (int t = 0; t < 5; ++t) mb[t] = mp[t];
    }
  };
  auto compute_store = [&](const uint4 (&f)[KC], int rt) {
    f32x16_b acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    uint4 wc[5], wn[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) wc[t] = wlane[32 * t];
#pragma unroll
    for (int s = 0; s < KC; ++s) {
      if (s + 1 < KC) {  // the next step's weight fragments in flight under this step's MFMAs
#pragma unroll
        for (int t = 0; t < 5; ++t) wn[t] = wlane[(2 * (s + 1)) * kBwCols + 32 * t];
      }
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 x = __builtin_bit_cast(bf16x8, tail_fix(s, f[s]));
#pragma unroll
      for (int t = 0; t < 5; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, wc[t]), x,
                                                         acc[t], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 5; ++t) wc[t] = wn[t];
    }
    // lane: output row m, columns n0 + 32 t + 8 g + 4 kh + (0..3) = acc[t][4 g .. 4 g + 3]
    const int m = rt * 128 + w * 32 + li;
    if (m >= M) return;
    uint32_t nb[3] = {0u, 0u, 0u};  // EP 3: the sign nibbles, (t, g) = q at bits 4 (q % 8)
#pragma unroll
    for (int t = 0; t < 5; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + 32 * t + 8 * g + 4 * kh;
        if (n < N) {  // N % 4 == 0: a group is wholly in or out
          float4 o = make_float4(acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2],
                                 acc[t][4 * g + 3]);
          const float4 bv = *(const float4*)(bsh + (n - n0));
          o.x += bv.x; o.y += bv.y; o.z += bv.z; o.w += bv.w;
          if (relu) o = f4_relu(o);  // the Linear's act (layers/layers.py:121-122), uniform
          TC* c = C + c_index_bf(m, n, ldc, cs);
          if constexpr (DM) {
            // g = bf16(bf16(o) * relu'(y)): the product rounded as stored, then the derivative
            float d4[4];
            if constexpr (EP == 1) {
              const uint2 yv = ym[4 * t + g];
              d4[0] = act_grad_from_out<GNNEA_ACT_RELU>(bf16_to_f32((bf16_t)(yv.x & 0xffffu)));
              d4[1] = act_grad_from_out<GNNEA_ACT_RELU>(bf16_to_f32((bf16_t)(yv.x >> 16)));
              d4[2] = act_grad_from_out<GNNEA_ACT_RELU>(bf16_to_f32((bf16_t)(yv.y & 0xffffu)));
              d4[3] = act_grad_from_out<GNNEA_ACT_RELU>(bf16_to_f32((bf16_t)(yv.y >> 16)));
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e) d4[e] = (mb[t] >> (8 * g + 4 * kh + e)) & 1u ? 1.f : 0.f;
            }
            const float o4[4] = {o.x, o.y, o.z, o.w};
            bf16_t gb[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) gb[e] = f32_to_bf16(bf16_to_f32(f32_to_bf16(o4[e])) * d4[e]);
            *(uint2*)c = make_uint2((uint32_t)gb[0] | ((uint32_t)gb[1] << 16),
                                    (uint32_t)gb[2] | ((uint32_t)gb[3] << 16));
          } else if constexpr (EP == 3) {
            const bf16_t y0 = f32_to_bf16(o.x), y1 = f32_to_bf16(o.y), y2 = f32_to_bf16(o.z),
                         y3 = f32_to_bf16(o.w);
            *(uint2*)c = make_uint2((uint32_t)y0 | ((uint32_t)y1 << 16),
                                    (uint32_t)y2 | ((uint32_t)y3 << 16));
            // relu'(y) = y > 0 on the stored value (y >= 0: its bits nonzero)
            const uint32_t nib = (y0 != 0 ? 1u : 0u) | (y1 != 0 ? 2u : 0u) | (y2 != 0 ? 4u : 0u) |
                                 (y3 != 0 ? 8u : 0u);
            const int q = 4 * t + g;
            nb[q >> 3] |= nib << (4 * (q & 7));
          } else if constexpr (std::is_same<TC, bf16_t>::value) {
            *(uint2*)c = make_uint2((uint32_t)f32_to_bf16(o.x) | ((uint32_t)f32_to_bf16(o.y) << 16),
                                    (uint32_t)f32_to_bf16(o.z) | ((uint32_t)f32_to_bf16(o.w) << 16));
          } else {
            *(float4*)c = o;
          }
        }
      }
    }
    if constexpr (EP == 3) {
      // the row's bytes: columns 8 g .. 8 g + 3 from the kh = 0 lane, + 4 .. + 7 from its kh = 1
      // partner (the same row); kh = 0 lanes store dwords t = 0..2, kh = 1 lanes t = 3, 4
      uint32_t ot[3];
#pragma unroll
      for (int i = 0; i < 3; ++i) ot[i] = __shfl_xor(nb[i], 32);
      uint32_t* mp = (uint32_t*)(Mo + (int64_t)m * ldmo + nt * 20);
#pragma unroll
      for (int t = 0; t < 5; ++t) {
        uint32_t d = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q = 4 * t + g;
          const uint32_t a0 = (nb[q >> 3] >> (4 * (q & 7))) & 15u;
          const uint32_t a1 = (ot[q >> 3] >> (4 * (q & 7))) & 15u;
          d |= (kh ? (a1 | (a0 << 4)) : (a0 | (a1 << 4))) << (8 * g);
        }
        if (kh ? t >= 3 : t < 3) mp[t] = d;
      }
    }
  };
  // every iteration issues the next tile's loads unconditionally (past the last tile: the last
  // tile again, never used), so that the outstanding-load count at each use is the same on
  // every path through the loop and the compiler's waits cover only the tile being used
  // (DM: the tile's y is loaded before the next tile's activations, so the epilogue's wait for it
  // does not cover them)
  if (rs >= tm) return;
  uint4 fa[KC], fb[KC];
  int rt = rs;
  issue(fa, rt);
  while (true) {
    const int r1 = rt + nrs;
    load_y(rt);
    issue(fb, min(r1, tm - 1));
    compute_store(fa, rt);
    if (r1 >= tm) break;
    const int r2 = r1 + nrs;
    load_y(r1);
    issue(fa, min(r2, tm - 1));
    compute_store(fb, r1);
    if (r2 >= tm) break;
    rt = r2;
  }
}

static bool bf16w_applies(int trans_a, int64_t M, int64_t N, int64_t K, int64_t lda,
                          const void* A) {
  const char* e = getenv("GNNEA_BF16_WRES");  // A/B comparison only (=0: k_gemm_bf16p)
  const bool on = !(e && e[0] == '0');
  // instantiated for 19 and 20 k-steps of 16 (K in (288, 320]: the 300-wide cfg-5 products)
  return on && !trans_a && M >= 65536 && N > 128 && N <= 4096 && N % 4 == 0 && K > 288 &&
         K <= 16 * kBwKC && K % 2 == 0 && lda % 2 == 0 && (((uintptr_t)A) & 3) == 0;
}
static int bf16w_kc(int64_t K) { return (int)(((K + 7) / 8 + 1) / 2); }
static int64_t bf16w_planes_bytes(int64_t N, int64_t K) {
  const int64_t ntn = (N + kBwCols - 1) / kBwCols;
  return ntn * bf16w_kc(K) * 2 * kBwCols * 16;
}

template <typename TC>
static int gemm_bf16w(int trans_b, int64_t M, int64_t N, int64_t K, const bf16_t* A,
                      int64_t lda, const bf16_t* B, int64_t ldb, const float* bias, TC* C,
                      int64_t ldc, int64_t cs, void* ws, hipStream_t s, int relu) {
  const int kc = bf16w_kc(K), ntn = (int)((N + kBwCols - 1) / kBwCols);
  bf16_t* P = (bf16_t*)ws;
  {
    const int64_t tot = (int64_t)ntn * kc * 2 * kBwCols * 8;
    const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
    hipLaunchKernelGGL(k_pack_bf16w, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 1 : 0, (int)N,
                       (int)K, kc, ntn, P);
    GNNEA_LAUNCH_CHECK();
  }
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  // persistent grid: a multiple of 8 * ntn workgroups (column tiles of a row stream 8 apart)
  const int unit = 8 * ntn;
  const int64_t tm = (M + 127) / 128;
  int grid = ncu / unit * unit;
  if (grid < unit) grid = unit;
  if ((int64_t)grid / ntn > tm) grid = (int)((tm + 7) / 8 * 8 * ntn);
  if (kc == 19)
    hipLaunchKernelGGL((k_gemm_bf16w<TC, 19>), dim3(grid), dim3(256), 0, s, (int)M, (int)N,
                       (int)K, ntn, A, lda, P, bias, C, ldc, cs, relu);
  else
    hipLaunchKernelGGL((k_gemm_bf16w<TC, 20>), dim3(grid), dim3(256), 0, s, (int)M, (int)N,
                       (int)K, ntn, A, lda, P, bias, C, ldc, cs, relu);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// the masked backward product (k_gemm_bf16w<bf16, KC, true>): G = bf16(A·op(B)) * relu'(Y);
// workspace = the weight planes
static int bf16w_grid(int64_t M, int ntn) {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  const int unit = 8 * ntn;
  const int64_t tm = (M + 127) / 128;
  int grid = ncu / unit * unit;
  if (grid < unit) grid = unit;
  if ((int64_t)grid / ntn > tm) grid = (int)((tm + 7) / 8 * 8 * ntn);
  return grid;
}
static bool dmask_applies(int64_t M, int64_t N, int64_t K, int64_t lda, const void* A,
                          int64_t ldy, const void* Y, int64_t ldg, const void* G) {
  return bf16w_applies(0, M, N, K, lda, A) && ldy >= N && ldy % 4 == 0 && ldg >= N &&
         ldg % 4 == 0 && (((uintptr_t)Y | (uintptr_t)G) & 7) == 0;
}
static int64_t dmask_ws_bytes(int64_t N, int64_t K) { return bf16w_planes_bytes(N, K); }
static int64_t mask_ld(int64_t N) { return 20 * ((N + kBwCols - 1) / kBwCols); }

// the weight-resident kernel with epilogue mode EP (bf16 out, row-major, no split)
template <int EP>
static int bf16w_ep_launch(int trans_b, int64_t M, int64_t N, int64_t K, const bf16_t* A,
                           int64_t lda, const bf16_t* B, int64_t ldb, const float* bias,
                           bf16_t* C, int64_t ldc, int relu, const void* Ym, int64_t ldym,
                           uint8_t* Mo, int64_t ldmo, void* ws, hipStream_t s) {
  const int kc = bf16w_kc(K), ntn = (int)((N + kBwCols - 1) / kBwCols);
  bf16_t* P = (bf16_t*)ws;
  {
    const int64_t tot = (int64_t)ntn * kc * 2 * kBwCols * 8;
    const int nb = (int)((tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048);
    hipLaunchKernelGGL(k_pack_bf16w, dim3(nb), dim3(256), 0, s, B, ldb, trans_b ? 1 : 0, (int)N,
                       (int)K, kc, ntn, P);
    GNNEA_LAUNCH_CHECK();
  }
  const int grid = bf16w_grid(M, ntn);
  if (kc == 19)
    hipLaunchKernelGGL((k_gemm_bf16w<bf16_t, 19, EP>), dim3(grid), dim3(256), 0, s, (int)M,
                       (int)N, (int)K, ntn, A, lda, P, bias, C, ldc, (int64_t)128, relu, Ym, ldym,
                       Mo, ldmo);
  else
    hipLaunchKernelGGL((k_gemm_bf16w<bf16_t, 20, EP>), dim3(grid), dim3(256), 0, s, (int)M,
                       (int)N, (int)K, ntn, A, lda, P, bias, C, ldc, (int64_t)128, relu, Ym, ldym,
                       Mo, ldmo);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename TC>
static int gemm_bf16_t(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                       const bf16_t* A, int64_t lda, const bf16_t* B, int64_t ldb,
                       const float* bias, float beta, TC* C, int64_t ldc, void* ws,
                       int64_t ws_bytes, hipStream_t s, int64_t cs, int act) {
  // (beta != 0: the old C would be loaded behind the next tile's activations: k_gemm_bf16p)
  if (beta == 0.f && bf16w_applies(trans_a, M, N, K, lda, A) && ws &&
      ws_bytes >= bf16w_planes_bytes(N, K) && ldc % 4 == 0 && cs % 4 == 0 &&
      (((uintptr_t)C) & (4 * sizeof(TC) - 1)) == 0 &&
      (act == GNNEA_ACT_IDENTITY || act == GNNEA_ACT_RELU))
    return gemm_bf16w<TC>(trans_b, M, N, K, A, lda, B, ldb, bias, C, ldc, cs, ws, s,
                          act == GNNEA_ACT_RELU ? 1 : 0);
  if (act != GNNEA_ACT_IDENTITY) {  // any other kernel: the product, then the act in place
    if (cs != 128) return GNNEA_EINVAL;
    const int rc = gemm_bf16_t<TC>(trans_a, trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc,
                                   ws, ws_bytes, s, cs);
    if (rc) return rc;
    if constexpr (std::is_same<TC, bf16_t>::value) return act_rows_bf16(C, ldc, M, N, act, s);
    else return act_rows_f32(C, ldc, M, N, act, s);
  }
  if (bf16p_applies(trans_a, M, N, K, lda, A) && ws && ws_bytes >= bf16p_planes_bytes(N, K))
    return gemm_bf16p<TC>(trans_b, M, N, K, A, lda, B, ldb, bias, beta, C, ldc, cs, ws, s);
  const int wt = bf16_wt(N);
  const int64_t bn = 64 * wt;
  const int tiles_n = (int)((N + bn - 1) / bn);
  const int tiles = (int)(((M + HBM - 1) / HBM) * tiles_n);
  if (trans_a && !trans_b && cs == 128 && gemm_ta_applies(M, N, K, lda, ldb, A, B, 2)) {
    float* slab = nullptr;  // whole-width weight-gradient tiles (gemm_ta.hip)
    int used = 0;
    const int rc = gemm_ta_launch<bf16_t>(M, N, K, A, lda, B, ldb, ws, ws ? ws_bytes : 0, s,
                                          &slab, &used);
    if (rc) return rc;
    const int64_t nn = M * N;
    const int nb = (int)((nn + 255) / 256 < 4096 ? (nn + 255) / 256 : 4096);
    hipLaunchKernelGGL((k_gemm_bf16_reduce<TC>), dim3(nb), dim3(256), 0, s, (int)M, (int)N, used,
                       slab, bias, beta, C, ldc, cs);
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
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
  int64_t split = bf16_splits(M, N, K, INT64_MAX / 2) * M * N * 4;
  if (gemm_ta_ws_bytes(M, N, K) > split) split = gemm_ta_ws_bytes(M, N, K);  // gemm_ta.hip
  int64_t planes = bf16p_planes_bytes(N, K);  // k_gemm_bf16p / k_gemm_bf16w (shape-dependent)
  if (bf16w_planes_bytes(N, K) > planes) planes = bf16w_planes_bytes(N, K);
  return split > planes ? split : planes;
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
                               s, 128);
  if (c_dtype == GNNEA_F32)
    return gemm_bf16_t<float>(trans_a, trans_b, M, N, K, (const bf16_t*)A, lda,
                              (const bf16_t*)B, ldb, bias, beta, (float*)C, ldc, ws, ws_bytes,
                              s, 128);
  return GNNEA_EINVAL;
}

// C = act(A·op(B) + bias) (the Linear layer with its act, layers/layers.py:121-122): relu rides
// the weight-resident kernel's epilogue, any other (kernel, act) pair runs the act in place after
extern "C" int gnnea_gemm_bf16_act(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                                   const void* A, int64_t lda, const void* B, int64_t ldb,
                                   const float* bias, int act, void* C, int64_t ldc, int c_dtype,
                                   void* ws, int64_t ws_bytes, void* stream) {
  if (act < GNNEA_ACT_IDENTITY || act > GNNEA_ACT_TANH) return GNNEA_EINVAL;
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
                               (const bf16_t*)B, ldb, bias, 0.f, (bf16_t*)C, ldc, ws, ws_bytes,
                               s, 128, act);
  if (c_dtype == GNNEA_F32)
    return gemm_bf16_t<float>(trans_a, trans_b, M, N, K, (const bf16_t*)A, lda,
                              (const bf16_t*)B, ldb, bias, 0.f, (float*)C, ldc, ws, ws_bytes, s,
                              128, act);
  return GNNEA_EINVAL;
}

extern "C" int gnnea_gemm_bf16_dmask_applies(int64_t M, int64_t N, int64_t K, int64_t lda,
                                             int64_t ldy, int64_t ldg) {
  return M > 0 && M < (1ll << 31) && N < (1ll << 31) && dmask_applies(M, N, K, lda, nullptr, ldy,
                                                                      nullptr, ldg, nullptr)
             ? 1 : 0;
}

extern "C" int64_t gnnea_gemm_bf16_dmask_ws_bytes(int64_t N, int64_t K) {
  if (N < 0 || K < 0) return GNNEA_EINVAL;
  return dmask_ws_bytes(N, K);
}

// The backward of y = relu(x Wᵀ + b) through the product that consumed y (MLPDecoder's relu
// Linear layers, models/decoders.py; layers/layers.py:121-122): G = bf16(A·op(B)) * relu'(Y),
// bit-identical to gnnea_gemm_bf16 followed by gnnea_act_bwd_colsum_bf16's G.  Only where the
// weight-resident kernel applies (gnnea_gemm_bf16_dmask_applies), else GNNEA_EINVAL.
extern "C" int gnnea_gemm_bf16_dmask(int trans_b, int64_t M, int64_t N, int64_t K, const void* A,
                                     int64_t lda, const void* B, int64_t ldb, const void* Y,
                                     int64_t ldy, void* G, int64_t ldg, void* ws,
                                     int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || !A || !B || !Y || !G || !ws) return GNNEA_EINVAL;
  if (trans_b ? ldb < K : ldb < N) return GNNEA_EINVAL;
  if (!dmask_applies(M, N, K, lda, A, ldy, Y, ldg, G)) return GNNEA_EINVAL;
  if (ws_bytes < dmask_ws_bytes(N, K)) return GNNEA_EWORKSPACE;
  return bf16w_ep_launch<1>(trans_b, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb,
                            nullptr, (bf16_t*)G, ldg, 0, Y, ldy, nullptr, 0, ws,
                            (hipStream_t)stream);
}

extern "C" int64_t gnnea_gemm_bf16_mask_ld(int64_t N) {
  if (N < 0) return GNNEA_EINVAL;
  return mask_ld(N);
}

// C = relu(A·op(B) + bias) (bf16, as gnnea_gemm_bf16_act with relu on the weight-resident kernel,
// bit for bit) and its sign bits M[row][...] (gnnea_gemm_bf16_mask_ld(N) bytes per row at least:
// byte 20 t + 4 u + g of a row holds columns 160 t + 32 u + 8 g + 0..7, bit e = column + e > 0)
// for gnnea_gemm_bf16_dmask_bits.  Where gnnea_gemm_bf16_dmask_applies (with ldy = ldc).
extern "C" int gnnea_gemm_bf16_relu_mask(int trans_b, int64_t M, int64_t N, int64_t K,
                                         const void* A, int64_t lda, const void* B, int64_t ldb,
                                         const float* bias, void* C, int64_t ldc, void* Mo,
                                         int64_t ldm, void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || !A || !B || !C || !Mo || !ws) return GNNEA_EINVAL;
  if (trans_b ? ldb < K : ldb < N) return GNNEA_EINVAL;
  if (!dmask_applies(M, N, K, lda, A, ldc, C, ldc, C) || ldm < mask_ld(N) || ldm % 4 ||
      ((uintptr_t)Mo & 3))
    return GNNEA_EINVAL;
  if (ws_bytes < dmask_ws_bytes(N, K)) return GNNEA_EWORKSPACE;
  return bf16w_ep_launch<3>(trans_b, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, bias,
                            (bf16_t*)C, ldc, 1, nullptr, 0, (uint8_t*)Mo, ldm, ws,
                            (hipStream_t)stream);
}

// gnnea_gemm_bf16_dmask with relu'(y) from the sign bits gnnea_gemm_bf16_relu_mask wrote
extern "C" int gnnea_gemm_bf16_dmask_bits(int trans_b, int64_t M, int64_t N, int64_t K,
                                          const void* A, int64_t lda, const void* B, int64_t ldb,
                                          const void* Mi, int64_t ldm, void* G, int64_t ldg,
                                          void* ws, int64_t ws_bytes, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || !A || !B || !Mi || !G || !ws) return GNNEA_EINVAL;
  if (trans_b ? ldb < K : ldb < N) return GNNEA_EINVAL;
  if (!dmask_applies(M, N, K, lda, A, ldg, G, ldg, G) || ldm < mask_ld(N) || ldm % 4 ||
      ((uintptr_t)Mi & 3))
    return GNNEA_EINVAL;
  if (ws_bytes < dmask_ws_bytes(N, K)) return GNNEA_EWORKSPACE;
  return bf16w_ep_launch<2>(trans_b, M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb,
                            nullptr, (bf16_t*)G, ldg, 0, Mi, ldm, nullptr, 0, ws,
                            (hipStream_t)stream);
}

extern "C" int gnnea_gemm_bf16_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda,
                                             int64_t ldb) {
  const void* dummy = (const void*)(uintptr_t)256;  // (alignment is checked on the real call)
  return gemm_ta_db_applies(M, N, K, lda, ldb, dummy, dummy, 2) ? 1 : 0;
}

// gnnea_gemm_x3_ta_db_f32 for bf16 operands: C = Aᵀ·B (gnnea_gemm_bf16's trans_a product, the
// same kernel and values; C bf16 or fp32 by c_dtype) and db = column sums of A (fp32 [M]) from
// the ones column in B's tile padding.  Workspace: gnnea_gemm_x3_ta_db_ws_bytes.
extern "C" int gnnea_gemm_bf16_ta_db(int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                                     const void* B, int64_t ldb, void* C, int64_t ldc, int c_dtype,
                                     float* db, void* ws, int64_t ws_bytes, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || !A || !B || !C || !db || ldc < N) return GNNEA_EINVAL;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (c_dtype != GNNEA_BF16 && c_dtype != GNNEA_F32) return GNNEA_EINVAL;
  if (!gemm_ta_db_applies(M, N, K, lda, ldb, A, B, 2)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  float* slab = nullptr;
  float* dbslab = nullptr;
  int used = 0;
  const int rc = gemm_ta_launch<bf16_t>(M, N, K, (const bf16_t*)A, lda, (const bf16_t*)B, ldb, ws,
                                        ws ? ws_bytes : 0, s, &slab, &used, &dbslab);
  if (rc) return rc;
  const int64_t nn = M * N;
  const int nb = (int)((nn + 255) / 256 < 4096 ? (nn + 255) / 256 : 4096);
  if (c_dtype == GNNEA_BF16)
    hipLaunchKernelGGL((k_gemm_bf16_reduce<bf16_t>), dim3(nb), dim3(256), 0, s, (int)M, (int)N,
                       used, slab, nullptr, 0.f, (bf16_t*)C, ldc, (int64_t)128);
  else
    hipLaunchKernelGGL((k_gemm_bf16_reduce<float>), dim3(nb), dim3(256), 0, s, (int)M, (int)N,
                       used, slab, nullptr, 0.f, (float*)C, ldc, (int64_t)128);
  GNNEA_LAUNCH_CHECK();
  return ta_db_reduce(M, used, dbslab, db, s);
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
