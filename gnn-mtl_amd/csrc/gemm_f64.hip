// fp64 GEMM on the f64 matrix cores for the GW / FGW outer loops (SinkhornOT/cderivation.py:
// get_init_matrices :146-157, get_LT :160-162, GW_cost_matrix :179-182, FGW_cost_matrix
// :185-188): every outer iteration of iterative_1 (SinkhornOT/iterative_projection.py:6-58)
// forms C1 · T · C2ᵀ (2·I·J·(I+J) flops) in the problem's dtype, fp64 on the reference path.
//
//   D[M,N] = alpha · op(A)[M,K] · op(B)[K,N] + beta · E[M,N]      (E may alias D, or be NULL)
//
// so L = constC − C1·X is one launch (alpha = −1, beta = 1, E = constC) and the products never
// round-trip through a separate elementwise pass.  v_mfma_f64_16x16x4_f64 (exact fp64 products
// and sums, k order inside a 4-deep step as the hardware adds them).  Tile 64 x 64 x 16 per
// 256-thread workgroup, 4 waves in 2 x 2, each 32 x 32 = 2 x 2 MFMA tiles (16 doubles of
// accumulator per lane); operand tiles staged through double-buffered LDS from registers (the
// next k-step's loads are in flight under the current MFMAs); any transpose of A or B is
// absorbed by the loader (LDS is always [k][row] for A and [k][col] for B, read one double per
// lane as the 16x16x4 operand maps want: A[l&15][k = l>>4], B[k = l>>4][l&15]).
// C/D map of the f64 form: col = lane & 15, row = (lane >> 4) + 4 * reg.
#include "common.h"

namespace gnnea {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int DBM = 64, DBN = 64, DBK = 16, DNT = 256;
constexpr int DLD = DBM + 1;  // LDS row (one k) of a 64-wide tile, +1 double against conflicts

// one 64 x 16 operand tile into registers: element (row r, k) of op(X), 4 per thread
struct DLoader {
  double v[4];
  __device__ void load(const double* __restrict__ X, int64_t ld, bool trans, int row0, int nrows,
                       int k0, int K, int tid) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + DNT * q;  // 0..1023
      int r, k;
      if (trans) {  // op(X)[r][k] = X[k][r]: rows contiguous in memory -> r fastest
        r = idx % DBM;
        k = idx / DBM;
      } else {  // X[r][k]: k contiguous -> k fastest
        k = idx % DBK;
        r = idx / DBK;
      }
      const int gr = row0 + r, gk = k0 + k;
      v[q] = (gr < nrows && gk < K) ? (trans ? X[(int64_t)gk * ld + gr] : X[(int64_t)gr * ld + gk])
                                    : 0.0;
    }
  }
  __device__ void store(double* __restrict__ S, bool trans, int tid) const {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + DNT * q;
      int r, k;
      if (trans) {
        r = idx % DBM;
        k = idx / DBM;
      } else {
        k = idx % DBK;
        r = idx / DBK;
      }
      S[k * DLD + r] = v[q];
    }
  }
};

// tb: op(B) = Bᵀ, i.e. B stored [N][K]; op(B)[k][n] is loaded as the "rows" n of a [n][k] tile
__global__ __launch_bounds__(DNT) void k_gemm_f64(int M, int N, int K, int ta, int tb,
                                                  const double* __restrict__ A, int64_t lda,
                                                  const double* __restrict__ B, int64_t ldb,
                                                  double alpha, const double* E, int64_t lde,
                                                  double beta, double* D, int64_t ldd,
                                                  int tiles_n) {
  __shared__ double sa[2][DBK * DLD];
  __shared__ double sb[2][DBK * DLD];
  const int t_id = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t_id / tiles_n) * DBM, n0 = (t_id % tiles_n) * DBN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int lr = lane & 15, lk = lane >> 4;

  f64x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f64x4){0.0, 0.0, 0.0, 0.0};

  // B as a [n][k] operand: stored [K][N] (tb = 0) means op(B)[k][n] = B[k][n] -> "trans" load
  DLoader la, lb;
  const int nsteps = (K + DBK - 1) / DBK;
  if (nsteps > 0) {
    la.load(A, lda, ta != 0, m0, M, 0, K, tid);
    lb.load(B, ldb, tb == 0, n0, N, 0, K, tid);
    la.store(sa[0], ta != 0, tid);
    lb.store(sb[0], tb == 0, tid);
    __syncthreads();
  }
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {
      la.load(A, lda, ta != 0, m0, M, (s + 1) * DBK, K, tid);
      lb.load(B, ldb, tb == 0, n0, N, (s + 1) * DBK, K, tid);
    }
#pragma unroll
    for (int kk = 0; kk < DBK; kk += 4) {
      double a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = sa[cur][(kk + lk) * DLD + wm * 32 + i * 16 + lr];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = sb[cur][(kk + lk) * DLD + wn * 32 + j * 16 + lr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      la.store(sa[cur ^ 1], ta != 0, tid);
      lb.store(sb[cur ^ 1], tb == 0, tid);
    }
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + lr;
      if (col >= N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + lk + 4 * r;
        if (row >= M) continue;
        double o = alpha * acc[i][j][r];
        if (E && beta != 0.0) o += beta * E[(int64_t)row * lde + col];
        D[(int64_t)row * ldd + col] = o;
      }
    }
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_gemm_f64(int trans_a, int trans_b, int64_t M, int64_t N, int64_t K,
                              const double* A, int64_t lda, const double* B, int64_t ldb,
                              double alpha, const double* E, int64_t lde, double beta, double* D,
                              int64_t ldd, void* stream) {
  if (M < 0 || N < 0 || K < 0) return GNNEA_EINVAL;
  if (M == 0 || N == 0) return 0;
  if (M >= (1ll << 31) || N >= (1ll << 31) || K >= (1ll << 31)) return GNNEA_EINVAL;
  if (!D || (K > 0 && (!A || !B))) return GNNEA_EINVAL;
  if (ldd < N || (E && lde < N)) return GNNEA_EINVAL;
  if (K > 0 && (trans_a ? lda < M : lda < K)) return GNNEA_EINVAL;
  if (K > 0 && (trans_b ? ldb < K : ldb < N)) return GNNEA_EINVAL;
  const int64_t tn = (N + DBN - 1) / DBN, tm = (M + DBM - 1) / DBM;
  if (tm * tn >= (1ll << 31)) return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_gemm_f64, dim3((unsigned)(tm * tn)), dim3(DNT), 0, (hipStream_t)stream,
                     (int)M, (int)N, (int)K, trans_a, trans_b, A, lda, B, ldb, alpha, E, lde,
                     beta, D, ldd, (int)tn);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
