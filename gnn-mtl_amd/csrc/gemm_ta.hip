// Weight gradients dW = Aᵀ·B (autograd of nn.Linear / torch.mm, layers/layers.py:32,61,
// att_layers.py:33): A [K][M], B [K][N] both tall (K = the graph's rows, M, N <= 320), the
// output tiny.  The general kernels (gemm.hip k_gemm_x3 TA form, gemm_bf16.hip k_gemm_bf16) tile
// the OUTPUT in 64- / 128-row blocks, so every row block re-reads all of B from HBM (5x / 3x the
// compulsory bytes at M = 300).  Here a workgroup owns ALL M rows (<= 320) x one 160-column half
// of N over a K range (split-K over the whole chip, one 8-wave workgroup per CU), so B is read
// once and A twice — and the two halves of one K range are adjacent workgroup ids, i.e. on one XCD
// at the same time, so A's second read is an L2 hit.  Partials go to fp32 slabs reduced in fixed
// split order (deterministic, no atomics).
//
// k-step of 32 rows: A [32][320] and B [32][160] are staged through registers (16-B chunks, a row
// run per wave: coalesced) into LDS images [k][m] / [k][n] laid out as they are in memory; the
// MFMA operands (v_mfma_f32_16x16x32_bf16: lane l supplies rows/cols l%16 at k = 8(l/16) + 0..7)
// are read TRANSPOSED by ds_read_b64_tr_b16 (two per operand), so no element-wise transposing
// stores.  Image rows are 704 B (A) / 320 B (B) apart and the 32-B blocks of rows 8..15 mod 16 are
// swapped (byte offset ^ 32): the four rows a 16-lane group reads and the partner group's four
// rows 8 further down then hit 8 disjoint 8-dword bank groups.  8 waves in 4 (m) x 2 (n), each
// 80 x 80 = 5 x 5 accumulator tiles (100 registers).
// fp32 operands (x3): every element is split into bf16 h + m + l when it is written to LDS (three
// planes per operand) and the six products of gemm.hip's x3 scheme (small ones first) run per
// tile, so the result carries fp32 rounding like the other fp32 GEMMs.
// Loads are unconditional (chunks past M / N re-read the row's first chunk: only output rows /
// columns that are never stored see them; k-steps past a split's end re-read its last step, and
// rows past the split end are zeroed when written to LDS), so the compiler's waits sit at the LDS
// writes, one or two k-steps behind the loads (bf16: two register sets in flight).  The table's
// last row never reads past the table: a 16-B chunk that would (bf16, M·2 % 16 == 8) is read 8 B
// earlier and shifted down.
#include <type_traits>

#include "common.h"
#include "gemm_ta.h"
#include "lds_dma.h"

namespace gnnea {

typedef short ta_v4s __attribute__((ext_vector_type(4)));
typedef short ta_v8s __attribute__((ext_vector_type(8)));
typedef __bf16 ta_bf16x8 __attribute__((ext_vector_type(8)));
typedef float ta_f32x4 __attribute__((ext_vector_type(4)));

constexpr int TA_NT = 512, TA_BK = 32, TA_MP = 320, TA_NP = 160;
constexpr int TA_RSA = 704, TA_RSB = 320;  // LDS image row strides (bytes)
constexpr int TA_IMG_A = TA_BK * TA_RSA, TA_IMG_B = TA_BK * TA_RSB;

template <typename T> struct TaTraits;
template <> struct TaTraits<bf16_t> {
  static constexpr int PL = 1, CE = 8, NS = 2;  // planes, elements per 16-B chunk, register sets
};
template <> struct TaTraits<float> {
  static constexpr int PL = 3, CE = 4, NS = 1;
};

typedef __attribute__((address_space(3))) ta_v4s lds_v4s;

__device__ __forceinline__ ta_bf16x8 ta_frag(const char* base, uint32_t off, int rs) {
  const ta_v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off));
  const ta_v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(base + off + 4 * rs));
  const ta_v8s v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(ta_bf16x8, v);
}

template <typename T>
struct TaTile {
  static constexpr int CE = TaTraits<T>::CE;
  static constexpr int CA = TA_MP / CE, CB = TA_NP / CE;  // 16-B chunks per image row
  static constexpr int TOT = TA_BK * (CA + CB);
  static constexpr int NCH = (TOT + TA_NT - 1) / TA_NT;  // chunks per thread
};

template <typename T>
struct TaRegs {
  uint4 v[TaTile<T>::NCH];
};

// chunk q of this thread: A or B, image row, chunk column
template <typename T>
__device__ __forceinline__ void ta_chunk(int idx, bool& isa, int& row, int& c) {
  using Ti = TaTile<T>;
  isa = idx < TA_BK * Ti::CA;
  const int i2 = isa ? idx : idx - TA_BK * Ti::CA;
  const int cpr = isa ? Ti::CA : Ti::CB;
  row = i2 / cpr;
  c = i2 - row * cpr;
}

template <typename T>
__device__ __forceinline__ void ta_load(TaRegs<T>& R, const T* __restrict__ A, int64_t lda,
                                        const T* __restrict__ B, int64_t ldb, int M, int N, int n0,
                                        int K, int k0, int ke, int tid) {
  using Ti = TaTile<T>;
#pragma unroll
  for (int q = 0; q < Ti::NCH; ++q) {
    // threads past the tile's last chunk repeat a real one (same data, same LDS slot): every
    // load and write is unconditional, so no load is sunk to its write
    const int idx = tid + TA_NT * q < Ti::TOT ? tid + TA_NT * q : tid + TA_NT * q - Ti::TOT;
    bool isa;
    int row, c;
    ta_chunk<T>(idx, isa, row, c);
    const int gk = min(k0 + row, ke - 1);
    const T* X = isa ? A : B;
    const int64_t ld = isa ? lda : ldb;
    const int lim = isa ? M : N;                 // valid elements of the row
    const int col = (isa ? 0 : n0) + c * Ti::CE;  // first element of the chunk
    const char* rb = (const char*)(X + (int64_t)gk * ld);
    int64_t off = col < lim ? (int64_t)col * sizeof(T) : 0;  // past the row: its first chunk
    // the table's last row: a chunk running past the row end is read 8 B earlier
    if (gk == K - 1 && col < lim && (col + Ti::CE) * (int)sizeof(T) > lim * (int)sizeof(T)) off -= 8;
    R.v[q] = *(const uint4*)(rb + off);
  }
}

// dbn >= 0 (bf16, the bias column): B's element dbn (in the tile's padding) is written as 1.0
template <typename T>
__device__ __forceinline__ void ta_write(const TaRegs<T>& R, char* lds, int M, int N, int n0,
                                         int K, int k0, int ke, int tid, int dbn = -1) {
  using Ti = TaTile<T>;
#pragma unroll
  for (int q = 0; q < Ti::NCH; ++q) {
    const int idx = tid + TA_NT * q < Ti::TOT ? tid + TA_NT * q : tid + TA_NT * q - Ti::TOT;
    bool isa;
    int row, c;
    ta_chunk<T>(idx, isa, row, c);
    uint4 u = R.v[q];
    const int gk = k0 + row;
    const int lim = isa ? M : N;
    const int col = (isa ? 0 : n0) + c * Ti::CE;
    if (gk == K - 1 && col < lim && (col + Ti::CE) * (int)sizeof(T) > lim * (int)sizeof(T))
      u = make_uint4(u.z, u.w, 0u, 0u);  // read 8 B early: shift down
    if (gk >= ke) u = make_uint4(0u, 0u, 0u, 0u);  // past the split's K range
    if constexpr (sizeof(T) == 2) {
      if (!isa && dbn >= col && dbn < col + Ti::CE && gk < ke) {
        const int e = dbn - col;
        const uint32_t mk = 0xffffu << (16 * (e & 1)), one = 0x3F80u << (16 * (e & 1));
        u.x = (e >> 1) == 0 ? (u.x & ~mk) | one : u.x;
        u.y = (e >> 1) == 1 ? (u.y & ~mk) | one : u.y;
        u.z = (e >> 1) == 2 ? (u.z & ~mk) | one : u.z;
        u.w = (e >> 1) == 3 ? (u.w & ~mk) | one : u.w;
      }
    }
    const uint32_t swz = ((row >> 3) & 1) << 5;
    char* img = lds + (isa ? 0 : TaTraits<T>::PL * TA_IMG_A);
    const int rs = isa ? TA_RSA : TA_RSB;
    if constexpr (sizeof(T) == 2) {
      *(uint4*)(img + row * rs + ((c * 16) ^ swz)) = u;
    } else {  // four fp32 -> h / m / l planes, 8 B each
      const float f[4] = {__builtin_bit_cast(float, u.x), __builtin_bit_cast(float, u.y),
                          __builtin_bit_cast(float, u.z), __builtin_bit_cast(float, u.w)};
      uint32_t h[2] = {0u, 0u}, m[2] = {0u, 0u}, l[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16_t hb = __builtin_bit_cast(bf16_t, (__bf16)f[e]);
        const float r1 = f[e] - bf16_to_f32(hb);
        const bf16_t mb = __builtin_bit_cast(bf16_t, (__bf16)r1);
        const bf16_t lb = __builtin_bit_cast(bf16_t, (__bf16)(r1 - bf16_to_f32(mb)));
        h[e >> 1] |= (uint32_t)hb << (16 * (e & 1));
        m[e >> 1] |= (uint32_t)mb << (16 * (e & 1));
        l[e >> 1] |= (uint32_t)lb << (16 * (e & 1));
      }
      const int plane = isa ? TA_IMG_A : TA_IMG_B;
      char* p = img + row * rs + ((c * 8) ^ swz);
      *(uint2*)p = make_uint2(h[0], h[1]);
      *(uint2*)(p + plane) = make_uint2(m[0], m[1]);
      *(uint2*)(p + 2 * plane) = make_uint2(l[0], l[1]);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(TA_NT, 1) void k_gemm_ta(int M, int N, int K,
                                                      const T* __restrict__ A, int64_t lda,
                                                      const T* __restrict__ B, int64_t ldb,
                                                      int kps, int tiles_n,
                                                      float* __restrict__ slab,
                                                      float* __restrict__ dbslab) {
  constexpr int PL = TaTraits<T>::PL;
  __shared__ __attribute__((aligned(16))) char lds[PL * (TA_IMG_A + TA_IMG_B)];
  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = t_id % tiles_n, split = t_id / tiles_n;
  const int n0 = tn * TA_NP;
  const int kb = split * kps;
  const int ke = min(K, kb + kps);
  if (kb >= ke) return;  // (the host sizes the grid so that every split has rows)
  const int nsteps = (ke - kb + TA_BK - 1) / TA_BK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;  // 80-row x 80-column wave tile
  const int dbn = dbslab ? N : -1;  // the ones column (bias gradient), see k_gemm_ta_x3d
  const int nrel = N - n0 - wn * 80;
  const int jdb = dbslab && nrel >= 0 && nrel < 80 ? nrel / 16 : -1;
  const bool ones_lane = jdb >= 0 && (lane & 15) == nrel % 16;

  ta_f32x4 acc[5][5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = ta_f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addresses: lane 16g + 4q + p reads image row 8g + q (+4), columns 4p..4p+3
  // of a 16-column block
  const int g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const uint32_t swz = (g & 1) << 5;
  const uint32_t a_off = (8 * g + q4) * TA_RSA, b_off = (8 * g + q4) * TA_RSB;
  auto a_at = [&](int i) { return a_off + ((2 * (wm * 80 + 16 * i + 4 * p4)) ^ swz); };
  auto b_at = [&](int j) { return b_off + ((2 * (wn * 80 + 16 * j + 4 * p4)) ^ swz); };
  const char* imgA = lds;
  const char* imgB = lds + PL * TA_IMG_A;

  auto compute = [&]() {
    if constexpr (PL == 1) {
      ta_bf16x8 bf[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) bf[j] = ta_frag(imgB, b_at(j), TA_RSB);
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const ta_bf16x8 af = ta_frag(imgA, a_at(i), TA_RSA);
#pragma unroll
        for (int j = 0; j < 5; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf[j], acc[i][j], 0, 0, 0);
      }
    } else {  // three planes: one B triple at a time (registers), the A triples re-read
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const ta_bf16x8 bh = ta_frag(imgB, b_at(j), TA_RSB);
        const ta_bf16x8 bm = ta_frag(imgB + TA_IMG_B, b_at(j), TA_RSB);
        const ta_bf16x8 bl = ta_frag(imgB + 2 * TA_IMG_B, b_at(j), TA_RSB);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const ta_bf16x8 ah = ta_frag(imgA, a_at(i), TA_RSA);
          const ta_bf16x8 am = ta_frag(imgA + TA_IMG_A, a_at(i), TA_RSA);
          const ta_bf16x8 al = ta_frag(imgA + 2 * TA_IMG_A, a_at(i), TA_RSA);
          // gemm.hip's x3 order: small products first
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);  // one B triple live at a time (register budget)
      }
    }
  };
  const int last = nsteps - 1;
  auto kstep = [&](int s) { return kb + min(s, last) * TA_BK; };

  // no early exit between a load and the LDS write that consumes it (the compiler would sink
  // the loads past the exit test, behind the MFMAs): steps past the end re-stage the last one
  if constexpr (TaTraits<T>::NS == 2) {
    TaRegs<T> R0, R1;
    ta_load<T>(R0, A, lda, B, ldb, M, N, n0, K, kstep(0), ke, tid);
    ta_load<T>(R1, A, lda, B, ldb, M, N, n0, K, kstep(1), ke, tid);
    ta_write<T>(R0, lds, M, N, n0, K, kstep(0), ke, tid, dbn);
    __syncthreads();
    for (int s = 0; s < nsteps; s += 2) {
      ta_load<T>(R0, A, lda, B, ldb, M, N, n0, K, kstep(s + 2), ke, tid);
      __builtin_amdgcn_sched_barrier(0);  // the loads stay ahead of the MFMAs
      compute();  // step s
      __syncthreads();
      ta_write<T>(R1, lds, M, N, n0, K, kstep(s + 1), ke, tid, dbn);
      __syncthreads();
      ta_load<T>(R1, A, lda, B, ldb, M, N, n0, K, kstep(s + 3), ke, tid);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < nsteps) compute();  // step s + 1
      __syncthreads();
      ta_write<T>(R0, lds, M, N, n0, K, kstep(s + 2), ke, tid, dbn);
      __syncthreads();
    }
  } else {
    TaRegs<T> R;
    ta_load<T>(R, A, lda, B, ldb, M, N, n0, K, kstep(0), ke, tid);
    ta_write<T>(R, lds, M, N, n0, K, kstep(0), ke, tid, dbn);
    __syncthreads();
    for (int s = 0; s < nsteps; ++s) {
      ta_load<T>(R, A, lda, B, ldb, M, N, n0, K, kstep(s + 1), ke, tid);
      __builtin_amdgcn_sched_barrier(0);
      compute();
      __syncthreads();
      ta_write<T>(R, lds, M, N, n0, K, kstep(s + 1), ke, tid, dbn);
      __syncthreads();
    }
  }

  // 16x16 accumulator map: column = lane % 16, row = 4 (lane / 16) + r
  float* out = slab + (int64_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int n = n0 + wn * 80 + 16 * j + (lane & 15);
      if (n >= N) {
        if (j == jdb && ones_lane) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = wm * 80 + 16 * i + 4 * (lane >> 4) + r;
            if (m < M) dbslab[(int64_t)split * M + m] = acc[i][j][r];
          }
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * 80 + 16 * i + 4 * (lane >> 4) + r;
        if (m < M) out[(int64_t)m * N + n] = acc[i][j][r];
      }
    }
  }
}

// ---- k_gemm_ta_x3d: the fp32 form fed by LDS-DMA, split at the fragment read ----
// k_gemm_ta<float> splits every element into h / m / l planes when it writes LDS: a 97.5-KB image
// per 32-row k-step, so there is one stage, one register set of loads in flight, and the split +
// write phase of every step runs with the matrix cores idle (2.61 ms at 2M x 300 x 300, ~5.2k
// cycles per k-step above the MFMA time).  Here the RAW fp32 tiles go to LDS by global_load_lds
// (A [32][320] + B [32][160] = 60 KB per stage, two stages: the next step's DMA in flight under
// this step's MFMAs, one barrier per step, no load registers) and each wave splits the fragments
// it reads: lane l of a 16x16x32 operand needs rows k = 8 (l / 16) + 0..7 of its column, eight
// ds_read_b32 (image rows 1280 / 640 B apart; the 16-B chunks of rows 8..15 mod 16 XOR 4, so the
// two 16-lane row groups of a half-wave hit disjoint banks), then three v_cvt_pk_bf16_f32 rounds
// per pair give the h / m / l operands already packed.  A's five fragments are split once per step
// and stay in registers (60); B's are split one column tile at a time, the next one's reads in
// flight under the current tile's 30 MFMAs.  Same six products in the same order as k_gemm_ta.
// LDS reads are inline asm (hipcc would wait vmcnt(0) for the in-flight DMA before plain ones)
// with explicit lgkmcnt waits.  Rows past a split's end are DMA'd from its last row and zeroed in
// registers (one uniform branch, last step only).
// dbslab != null (the bias gradient of the same layer, db = column sums of A): B's padding column
// N (N < the tile width) is read as ones, so output column N is sum_k A[k][m] (the x3 split of 1
// is exact: h = 1, m = l = 0) -> dbslab[split][m]; one wave's one column block, a uniform branch.
constexpr int TD_RSA = 1280, TD_RSB = 640;                   // image row strides (bytes)
constexpr int TD_IMG_A = TA_BK * TD_RSA, TD_IMG_B = TA_BK * TD_RSB;
constexpr int TD_STAGE = TD_IMG_A + TD_IMG_B;                // 61,440 B
constexpr int TD_DMA = TD_STAGE / 1024;                      // 1-KB DMA blocks per stage (60)
constexpr int TD_PER_WAVE = (TD_DMA + 7) / 8;                // 8

__device__ __forceinline__ float td_ld(uint32_t addr) {
  float v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
template <int OFF>
__device__ __forceinline__ float td_ld_o(uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}

struct TdTriple {
  ta_bf16x8 h, m, l;
};

// x = h + m + l exactly (the x3 split of gemm.hip / k_gemm_ta, round to nearest even), pairwise
// (common.h x3_split_pair: the same values, about half the vector instructions)
__device__ __forceinline__ TdTriple td_split(const float (&x)[8]) {
  uint4 h, m, l;
  x3_split_pair(x[0], x[1], h.x, m.x, l.x);
  x3_split_pair(x[2], x[3], h.y, m.y, l.y);
  x3_split_pair(x[4], x[5], h.z, m.z, l.z);
  x3_split_pair(x[6], x[7], h.w, m.w, l.w);
  TdTriple t;
  t.h = __builtin_bit_cast(ta_bf16x8, h);
  t.m = __builtin_bit_cast(ta_bf16x8, m);
  t.l = __builtin_bit_cast(ta_bf16x8, l);
  return t;
}

template <int RS>
__device__ __forceinline__ void td_read8(uint32_t addr, float (&x)[8]) {
  static_for<8>([&](auto ee) {
    constexpr int e = decltype(ee)::value;
    x[e] = td_ld_o<e * RS>(addr);
  });
}

__global__ __launch_bounds__(TA_NT, 1) void k_gemm_ta_x3d(int M, int N, int K,
                                                          const float* __restrict__ A,
                                                          int64_t lda,
                                                          const float* __restrict__ B,
                                                          int64_t ldb, int kps, int tiles_n,
                                                          float* __restrict__ slab,
                                                          float* __restrict__ dbslab) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * TD_STAGE];
  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = t_id % tiles_n, split = t_id / tiles_n;
  const int n0 = tn * TA_NP;
  const int kb = split * kps;
  const int ke = min(K, kb + kps);
  if (kb >= ke) return;  // (the host sizes the grid so that every split has rows)
  const int nsteps = (ke - kb + TA_BK - 1) / TA_BK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w & 3, wn = w >> 2;

  // DMA block i = w + 8 t of a stage: image bytes [i KB, i KB + 1 KB), lane-linear; the lane's
  // source row / column follow from its image position (chunk positions XOR-swizzled)
  int d_row[TD_PER_WAVE], d_off[TD_PER_WAVE];
  bool d_isa[TD_PER_WAVE];
#pragma unroll
  for (int t = 0; t < TD_PER_WAVE; ++t) {
    int i = w + 8 * t;
    if (i >= TD_DMA) i = TD_DMA - 1;  // waves 4..7 repeat the last block (same bytes, same slot)
    const int off = i * 1024 + lane * 16;
    const bool isa = off < TD_IMG_A;
    const int o2 = isa ? off : off - TD_IMG_A;
    const int rs = isa ? TD_RSA : TD_RSB;
    const int row = o2 / rs;
    const int pos = (o2 - row * rs) / 16;
    const int c = pos ^ (((row >> 3) & 1) << 2);   // logical 16-B chunk of the row
    int col = (isa ? 0 : n0) + 4 * c;
    if (col >= (isa ? M : N)) col = isa ? 0 : n0;  // past the row: a valid chunk (never stored)
    d_row[t] = row;
    d_off[t] = col;
    d_isa[t] = isa;
  }
  auto issue = [&](int s, int buf) {
    const int k0 = kb + s * TA_BK;
    const bool tail = k0 + TA_BK > ke;  // uniform
    unsigned char* st = smem + buf * TD_STAGE;
#pragma unroll
    for (int t = 0; t < TD_PER_WAVE; ++t) {
      int i = w + 8 * t;
      if (i >= TD_DMA) i = TD_DMA - 1;
      const int r = tail ? min(k0 + d_row[t], ke - 1) : k0 + d_row[t];
      const float* src = d_isa[t] ? A + (int64_t)r * lda + d_off[t] : B + (int64_t)r * ldb + d_off[t];
      glds16(src, st + i * 1024);
    }
  };

  ta_f32x4 acc[5][5];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = ta_f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read addresses (stage 0): lane l -> column l % 16 of a 16-wide tile, rows
  // 8 (l / 16) + e; chunk (col / 4) ^ (4 * ((l / 16) & 1)), dword col % 4
  const int g = lane >> 4, cl = lane & 15;
  // the ones column: this wave's column block jdb (uniform, -1: none) and its lane
  const int nrel = N - n0 - wn * 80;
  const int jdb = dbslab && nrel >= 0 && nrel < 80 ? nrel / 16 : -1;
  const bool ones_lane = jdb >= 0 && cl == nrel % 16;
  const uint32_t base = lds_addr(smem);
  uint32_t a_ad[5], b_ad[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int m = wm * 80 + 16 * i + cl;
    a_ad[i] = base + 8 * g * TD_RSA + (((m >> 2) ^ ((g & 1) << 2)) << 4) + (m & 3) * 4;
    const int n = wn * 80 + 16 * i + cl;
    b_ad[i] = base + TD_IMG_A + 8 * g * TD_RSB + (((n >> 2) ^ ((g & 1) << 2)) << 4) + (n & 3) * 4;
  }

  issue(0, 0);
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of step s
    __builtin_amdgcn_s_barrier();  // everyone's landed; everyone is done with buffer buf ^ 1
    asm volatile("" ::: "memory");
    if (s + 1 < nsteps) issue(s + 1, buf ^ 1);
    const uint32_t so = buf * TD_STAGE;
    const int k0 = kb + s * TA_BK;
    const int kval = ke - k0 - 8 * g;  // valid rows of this lane's eight (>= 8 but at the tail)
    const bool tail = k0 + TA_BK > ke;  // uniform

    // A fragment i + 1 (the last time: B's first) in flight while fragment i is split
    TdTriple at[5];
    float xa[2][8], xb[8];
    td_read8<TD_RSA>(a_ad[0] + so, xa[0]);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      if (i + 1 < 5)
        td_read8<TD_RSA>(a_ad[i + 1] + so, xa[(i + 1) & 1]);
      else
        td_read8<TD_RSB>(b_ad[0] + so, xb);
      asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      float (&x)[8] = xa[i & 1];
      if (tail) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = e < kval ? x[e] : 0.f;
      }
      at[i] = td_split(x);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (tail) {
#pragma unroll
        for (int e = 0; e < 8; ++e) xb[e] = e < kval ? xb[e] : 0.f;
      }
      if (j == jdb) {  // (uniform)
#pragma unroll
        for (int e = 0; e < 8; ++e) xb[e] = ones_lane ? (tail && e >= kval ? 0.f : 1.f) : xb[e];
      }
      const TdTriple bt = td_split(xb);
      if (j + 1 < 5) td_read8<TD_RSB>(b_ad[j + 1] + so, xb);  // in flight under the MFMAs
      // product-major: five independent accumulators between two dependent MFMAs (each
      // accumulator still sums its six products in k_gemm_ta's order)
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].l, bt.h, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].m, bt.m, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].h, bt.l, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].m, bt.h, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].h, bt.m, acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 5; ++i)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(at[i].h, bt.h, acc[i][j], 0, 0, 0);
    }
  }

  float* out = slab + (int64_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int n = n0 + wn * 80 + 16 * j + (lane & 15);
      if (n >= N) {
        if (j == jdb && ones_lane) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = wm * 80 + 16 * i + 4 * (lane >> 4) + r;
            if (m < M) dbslab[(int64_t)split * M + m] = acc[i][j][r];
          }
        }
        continue;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = wm * 80 + 16 * i + 4 * (lane >> 4) + r;
        if (m < M) out[(int64_t)m * N + n] = acc[i][j][r];
      }
    }
  }
}

// ---- host side ----

static int ta_splits(int64_t M, int64_t N, int64_t K, int64_t ws_bytes) {
  const int tiles_n = (int)((N + TA_NP - 1) / TA_NP);
  int64_t s = 256 / tiles_n;                 // one workgroup per CU
  const int64_t by_k = K / (2 * TA_BK);      // >= two k-steps per split
  if (s > by_k) s = by_k;
  while (s > 1 && s * M * N * 4 > ws_bytes) --s;
  return (int)(s < 1 ? 1 : s);
}

bool gemm_ta_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                     const void* B, int es) {
  // 4-element rows and row strides (8-B bf16 / 16-B fp32 granules), >= one chunk per row
  return M >= 8 && N >= 8 && M <= TA_MP && N <= 2 * TA_NP && K >= 4 * TA_BK &&
         K < (1ll << 31) && M % 4 == 0 && N % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 &&
         lda >= M && ldb >= N && (((uintptr_t)A) % (4 * es)) == 0 &&
         (((uintptr_t)B) % (4 * es)) == 0;
}

int64_t gemm_ta_ws_bytes(int64_t M, int64_t N, int64_t K) {
  return (int64_t)ta_splits(M, N, K, INT64_MAX / 4) * M * N * 4;
}

bool gemm_ta_db_applies(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, const void* A,
                        const void* B, int es) {
  return gemm_ta_applies(M, N, K, lda, ldb, A, B, es) && N % TA_NP != 0;
}

// db[m] = sum over the splits' partial column sums, in split order
__global__ void k_db_reduce(int M, int splits, const float* __restrict__ part,
                            float* __restrict__ db) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float a = 0.f;
  for (int q = 0; q < splits; ++q) a += part[(int64_t)q * M + m];
  db[m] = a;
}

int ta_db_reduce(int64_t M, int splits, const float* part, float* db, hipStream_t s) {
  hipLaunchKernelGGL(k_db_reduce, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, (int)M,
                     splits, part, db);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

int64_t gemm_ta_db_ws_bytes(int64_t M, int64_t N, int64_t K) {
  return (int64_t)ta_splits(M, N + 1, K, INT64_MAX / 4) * M * (N + 1) * 4;
}

template <typename T>
int gemm_ta_launch(int64_t M, int64_t N, int64_t K, const T* A, int64_t lda, const T* B,
                   int64_t ldb, void* ws, int64_t ws_bytes, hipStream_t s, float** slab_out,
                   int* splits_out, float** dbslab_out) {
  // (with the bias column: the slabs, then splits x M partial column sums)
  const int splits = ta_splits(M, dbslab_out ? N + 1 : N, K, ws ? ws_bytes : 0);
  if (!ws || ws_bytes < (int64_t)splits * M * (dbslab_out ? N + 1 : N) * 4)
    return GNNEA_EWORKSPACE;
  const int tiles_n = (int)((N + TA_NP - 1) / TA_NP);
  const int kps = (int)(((K + splits - 1) / splits + TA_BK - 1) / TA_BK * TA_BK);
  // every split must own rows (kps rounding can leave the last ones empty): trim the grid
  const int used = (int)((K + kps - 1) / kps);
  float* slab = (float*)ws;
  float* dbslab = dbslab_out ? slab + (int64_t)splits * M * N : nullptr;
  if constexpr (std::is_same<T, float>::value) {  // fp32: split at the fragment read
    hipLaunchKernelGGL(k_gemm_ta_x3d, dim3(used * tiles_n), dim3(TA_NT), 0, s, (int)M, (int)N,
                       (int)K, (const float*)A, lda, (const float*)B, ldb, kps, tiles_n, slab,
                       dbslab);
  } else {
    hipLaunchKernelGGL((k_gemm_ta<T>), dim3(used * tiles_n), dim3(TA_NT), 0, s, (int)M, (int)N,
                       (int)K, A, lda, B, ldb, kps, tiles_n, slab, dbslab);
  }
  if (dbslab_out) *dbslab_out = dbslab;
  GNNEA_LAUNCH_CHECK();
  *slab_out = slab;
  *splits_out = used;
  return 0;
}

template int gemm_ta_launch<bf16_t>(int64_t, int64_t, int64_t, const bf16_t*, int64_t,
                                    const bf16_t*, int64_t, void*, int64_t, hipStream_t, float**,
                                    int*, float**);
template int gemm_ta_launch<float>(int64_t, int64_t, int64_t, const float*, int64_t, const float*,
                                   int64_t, void*, int64_t, hipStream_t, float**, int*, float**);

}  // namespace gnnea
