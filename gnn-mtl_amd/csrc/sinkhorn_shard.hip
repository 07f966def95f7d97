// a9 across GPUs: utils/ot_loss.py:5-76 (Sinkhorn-Knopp, fp64) with the cost rows sharded over the
// ranks ("row-shard C; each iteration needs one collective of the J-length column
// LSE partials as (max, sum-exp) pairs").
//
// Log domain, f = log u (this rank's I_loc rows), g = log v (all J columns, replicated):
//   iteration it:  g_it,j = log b_j - LSE_i(f_{it-1},i - M_ij/reg)    column pass, over ALL rows
//                  f_it,i = log a_i - LSE_j(g_it,j  - M_ij/reg)       row pass, local rows
// (the reference's v = b / K^T u then u = 1 / (K/a) v, K_ij = exp(-M_ij/reg); a term is dropped
// where K underflows to 0 in fp64, as in sinkhorn_log.hip).  The column LSE is the only
// cross-rank quantity: each rank reduces its rows to one (max, sum-exp) pair per column, plus its
// previous row pass's failure flag (gnnea_sinkhorn_shard_colpart), the caller all-gathers the
// [W][2J + 2] pair rows, and every rank merges them in rank order (gnnea_sinkhorn_shard_step), so
// g and every stop decision are bit-identical on all ranks with no further collective:
//   - u inf / NaN in iteration it-1 (any rank's flag): break of it-1 (:57-62), iterate it-2 kept;
//   - err = ||v (K^T u) - b|| of iterate it-1 when (it-1) % 10 == 0 (:64-66) — K^T u_{it-1} is
//     exactly this iteration's column LSE, so the test costs nothing extra;
//   - K^T u == 0 or v inf / NaN in iteration it: break, iterate it-1 kept.
// A u failure of the very last iteration is settled by gnnea_sinkhorn_shard_close.  Plan rows,
// the local part of sum P.M and the local column sums follow (gnnea_sinkhorn_shard_finish); the
// caller all-reduces the two partial sums.  This file is the log-domain form (variant 1, or J
// above the scaling form's sweep limit); variant 0 with J <= 16384 dispatches to the scaling form
// with K resident per rank (sinkhorn.hip, skscale::shard_*): same protocol, J + 2 doubles a row.
#include "common.h"

namespace gnnea {
namespace skshard {

constexpr double kExpUnderflow = -745.1332191019412;  // exp_f64(x) == 0 below
constexpr double kLnTrueMin = -744.4400719213812;     // log(DBL_TRUE_MIN)
constexpr double kExpOverflow = 709.782712893384;     // exp_f64(x) == inf above
constexpr int kCH = 8;                                // loads in flight per lane
constexpr int kMaxSplits = 16;                        // row splits of the local column pass

// status words shared with sinkhorn.hip (include/gnnea.h GNNEA_SK_ST_*) + this path's flags
enum { ST_DONE = 0, ST_ITERS = 1, ST_REASON = 2, ST_SLOT = 3, ST_UFAIL = 6, ST_VFAIL = 7 };

struct Lse {
  double m, s;
  __device__ __forceinline__ void init() { m = -INFINITY; s = 0.0; }
  __device__ __forceinline__ void merge(double m2, double s2) {
    if (m2 == -INFINITY) return;
    if (m == -INFINITY) { m = m2; s = s2; return; }
    if (m2 > m) { s = s * exp_f64(m - m2) + s2; m = m2; }
    else s += s2 * exp_f64(m2 - m);
  }
  __device__ __forceinline__ double value() const { return m == -INFINITY ? -INFINITY : m + log(s); }
};

// chunked online LSE: one rescale exp per chunk + one exp per value (sinkhorn_log.hip lse_chunk)
__device__ __forceinline__ void lse_chunk(Lse& l, const double (&x)[kCH]) {
  double cm = x[0];
#pragma unroll
  for (int k = 1; k < kCH; ++k) cm = fmax(cm, x[k]);
  if (cm == -INFINITY) return;
  const double nm = fmax(l.m, cm);
  double acc = l.m == -INFINITY ? 0.0 : l.s * exp_f64(l.m - nm);
#pragma unroll
  for (int k = 0; k < kCH; ++k) acc += exp_f64(x[k] - nm);
  l.m = nm;
  l.s = acc;
}

__device__ __forceinline__ double term(double pot, double c, double inv_reg) {
  const double k = -c * inv_reg;
  return k < kExpUnderflow ? -INFINITY : k + pot;
}

__device__ __forceinline__ void mark_done(int64_t* st, int64_t iters, int64_t reason,
                                          int64_t slot) {
  if (atomicCAS((unsigned long long*)&st[ST_DONE], 0ull, 1ull) == 0ull) {
    st[ST_ITERS] = iters;
    st[ST_REASON] = reason;
    st[ST_SLOT] = slot;
  }
}

struct Dev {
  int64_t* st;
  double* sd;
  double *f, *g, *la, *lb, *bw, *errpart, *pm, *ps;
  int nerr;
};

// local column pass, split: workgroup = 16 waves x 64 consecutive columns over one row split
template <typename T>
__global__ __launch_bounds__(1024) void k_sh_colpart(const T* __restrict__ C, int64_t ldc, int I,
                                                     int J, double inv_reg, Dev d, int slot_f,
                                                     int rows_per_split) {
  if (d.st[ST_DONE]) return;
  __shared__ double sm[16][64], ss[16][64];
  const int lane = lane_id(), w = wave_id();
  const int j = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rows_per_split, r1 = min(I, r0 + rows_per_split);
  const double* __restrict__ f = d.f + (int64_t)slot_f * I;
  Lse l;
  l.init();
  if (j < J) {
    for (int i0 = r0 + w; i0 < r1; i0 += 16 * kCH) {
      double x[kCH];
#pragma unroll
      for (int k = 0; k < kCH; ++k) {
        const int i = i0 + 16 * k;
        x[k] = i < r1 ? term(f[i], (double)C[(int64_t)i * ldc + j], inv_reg) : -INFINITY;
      }
      lse_chunk(l, x);
    }
  }
  sm[w][lane] = l.m;
  ss[w][lane] = l.s;
  __syncthreads();
  if (w != 0 || j >= J) return;
  for (int q = 1; q < 16; ++q) l.merge(sm[q][lane], ss[q][lane]);
  d.pm[(int64_t)blockIdx.y * J + j] = l.m;
  d.ps[(int64_t)blockIdx.y * J + j] = l.s;
}

// the splits merged in order -> this rank's pair row: pair[2j] = m, pair[2j+1] = s,
// pair[2J] = its previous row pass's u-failure flag
__global__ __launch_bounds__(256) void k_sh_pairs(Dev d, int J, int ns, double* __restrict__ pair) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const bool done = d.st[ST_DONE] != 0;
  if (j < J) {
    Lse l;
    l.init();
    if (!done)
      for (int q = 0; q < ns; ++q) l.merge(d.pm[(int64_t)q * J + j], d.ps[(int64_t)q * J + j]);
    pair[2 * j] = l.m;
    pair[2 * j + 1] = l.s;
  }
  if (j == 0) {
    pair[2 * J] = d.st[ST_UFAIL] ? 1.0 : 0.0;
    pair[2 * J + 1] = 0.0;
  }
}

__device__ __forceinline__ bool any_ufail(const double* __restrict__ pairs, int W, int J) {
  bool u = false;
  for (int r = 0; r < W; ++r) u |= pairs[(int64_t)r * (2 * J + 2) + 2 * J] != 0.0;
  return u;
}

// merge the W gathered pair rows (rank order) -> g_it (slot it & 1), v / K^T u failure flag, the
// err^2 partials of iterate it-1.  Nothing is written when a rank's u failed (the loop ends on
// iterate it-2, whose g lives in the slot this iteration would overwrite).
__global__ __launch_bounds__(256) void k_sh_colfin(const double* __restrict__ pairs, int W, int J,
                                                   Dev d, int it) {
  if (d.st[ST_DONE] || any_ufail(pairs, W, J)) return;
  const int j = blockIdx.x * 256 + threadIdx.x;
  double e2 = 0.0;
  bool fail = false;
  if (j < J) {
    Lse t;
    t.init();
    for (int r = 0; r < W; ++r) {
      const double* pr = pairs + (int64_t)r * (2 * J + 2);
      t.merge(pr[2 * j], pr[2 * j + 1]);
    }
    const double lse = t.value();  // log (K^T u_{it-1})_j
    const int cur = it & 1, prev = cur ^ 1;
    const double x = exp_f64(d.g[(int64_t)prev * J + j] + lse) - d.bw[j];  // (:65-66)
    e2 = x * x;
    const double gj = d.lb[j] - lse;                       // v = b / K^T u  (:54)
    fail = !(lse >= kLnTrueMin) || !(gj <= kExpOverflow);  // K^T u == 0, v inf / NaN  (:57-59)
    d.g[(int64_t)cur * J + j] = gj;
  }
  e2 = wave_sum(e2);
  __shared__ double red[4];
  if (lane_id() == 0) red[wave_id()] = e2;
  if (__any(fail) && lane_id() == 0) atomicOr((unsigned long long*)&d.st[ST_VFAIL], 1ull);
  __syncthreads();
  if (threadIdx.x == 0) d.errpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// the loop decisions of iteration it in the reference's order (one thread, identical on every
// rank: it reads only gathered / replicated data)
__global__ void k_sh_decide(const double* __restrict__ pairs, int W, int J, Dev d, int it) {
  if (d.st[ST_DONE]) return;
  if (any_ufail(pairs, W, J)) {  // iteration it-1 broke on u: keep iterate it-2
    mark_done(d.st, it - 1, 2, it & 1);
    return;
  }
  const int prev = it - 1;
  if (prev >= 0 && prev % 10 == 0) {
    double e = 0.0;
    for (int b = 0; b < d.nerr; ++b) e += d.errpart[b];
    const double err = sqrt(e);
    d.sd[GNNEA_SK_SD_ERR] = err;
    if (!(err > d.sd[GNNEA_SK_SD_TOL])) {  // the while condition fails before iteration it
      mark_done(d.st, prev + 1, 1, prev & 1);
      return;
    }
  }
  if (d.st[ST_VFAIL]) mark_done(d.st, it, 2, (it + 1) & 1);
  d.st[ST_UFAIL] = 0;  // consumed (this rank's flag travelled in the gathered pairs)
}

// f_it for the local rows: one wave per row, LSE over all J with kCH loads in flight per lane
template <typename T>
__global__ __launch_bounds__(256) void k_sh_row(const T* __restrict__ C, int64_t ldc, int I, int J,
                                                double inv_reg, Dev d, int it) {
  if (d.st[ST_DONE]) return;
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (i >= I) return;
  const int lane = lane_id();
  const int cur = it & 1;
  const double* __restrict__ gc = d.g + (int64_t)cur * J;
  const T* __restrict__ Ci = C + (int64_t)i * ldc;
  Lse l;
  l.init();
  for (int j0 = 0; j0 < J; j0 += 64 * kCH) {
    double x[kCH];
#pragma unroll
    for (int k = 0; k < kCH; ++k) {
      const int j = j0 + 64 * k + lane;
      x[k] = j < J ? term(gc[j], (double)Ci[j], inv_reg) : -INFINITY;
    }
    lse_chunk(l, x);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) l.merge(__shfl_xor(l.m, o, 64), __shfl_xor(l.s, o, 64));
  if (lane == 0) {
    const double fi = d.la[i] - l.value();  // u = 1 / ((K/a) v)  (:55)
    d.f[(int64_t)cur * I + i] = fi;
    if (!(fi <= kExpOverflow)) atomicOr((unsigned long long*)&d.st[ST_UFAIL], 1ull);
  }
}

__global__ void k_sh_init(int I, int J, int I_global, double tol, const double* __restrict__ a,
                          const double* __restrict__ b, Dev d) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 32) {
    if (t < 8) d.st[t] = 0;
    else d.sd[t] = t == GNNEA_SK_SD_TOL ? tol : 0.0;
  }
  // slot 1 = the "previous" iterate of iteration 0: u0 = 1/I, v0 = 1/J (:38-39)
  for (int i = t; i < I; i += gridDim.x * blockDim.x) {
    d.f[I + i] = -log((double)I_global);
    d.la[i] = log(a[i]);
  }
  for (int j = t; j < J; j += gridDim.x * blockDim.x) {
    d.g[J + j] = -log((double)J);
    d.lb[j] = log(b[j]);
    d.bw[j] = b[j];
  }
}

// after the loop: a u failure of the last iteration (any rank) ends it on iterate iters-2, else
// the loop ran out of iterations on iterate iters-1 (slot 1 = the initial scalings at iters 0)
__global__ void k_sh_close(const double* __restrict__ flags, int W, Dev d, int iters_run) {
  if (d.st[ST_DONE]) return;
  bool u = false;
  for (int r = 0; r < W; ++r) u |= flags[r] != 0.0;
  if (u && iters_run > 0) mark_done(d.st, iters_run - 1, 2, iters_run & 1);
  else mark_done(d.st, iters_run, 0, iters_run > 0 ? (iters_run - 1) & 1 : 1);
}

__global__ void k_sh_flag(Dev d, double* __restrict__ out) {
  if (threadIdx.x == 0) out[0] = (!d.st[ST_DONE] && d.st[ST_UFAIL]) ? 1.0 : 0.0;
}

// plan rows, row sums, per-row sum P.M (P_ij = exp(f_i + g_j - M_ij/reg), zero where K == 0)
template <typename T, typename PT>
__global__ __launch_bounds__(256) void k_sh_plan(const T* __restrict__ C, int64_t ldc, int I,
                                                 int J, double inv_reg, Dev d,
                                                 PT* __restrict__ plan, int64_t ldp,
                                                 double* __restrict__ row_sum,
                                                 double* __restrict__ loss_rows) {
  const int slot = (int)(d.st[ST_SLOT] & 1);
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (i >= I) return;
  const int lane = lane_id();
  const double fi = d.f[(int64_t)slot * I + i];
  const double* __restrict__ gs = d.g + (int64_t)slot * J;
  const T* __restrict__ Ci = C + (int64_t)i * ldc;
  double rs = 0.0, ls = 0.0;
  for (int j = lane; j < J; j += 64) {
    const double c = (double)Ci[j];
    const double x = term(fi + gs[j], c, inv_reg);
    const double p = x == -INFINITY ? 0.0 : exp_f64(x);
    if (plan) plan[(int64_t)i * ldp + j] = (PT)p;
    rs += p;
    ls += p * c;
  }
  rs = wave_sum(rs);
  ls = wave_sum(ls);
  if (lane == 0) {
    if (row_sum) row_sum[i] = rs;
    loss_rows[i] = ls;
  }
}

// sum of the per-row losses in row order -> loss[0]
__global__ __launch_bounds__(1024) void k_sh_loss(const double* __restrict__ rows, int I,
                                                  double* __restrict__ loss) {
  __shared__ double red[1024];
  double s = 0.0;
  for (int i = threadIdx.x; i < I; i += 1024) s += rows[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0];
}

// this rank's column sums of P (one thread per column, local rows in order)
template <typename T>
__global__ __launch_bounds__(256) void k_sh_colsum(const T* __restrict__ C, int64_t ldc, int I,
                                                   int J, double inv_reg, Dev d,
                                                   double* __restrict__ col_sum) {
  const int slot = (int)(d.st[ST_SLOT] & 1);
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= J) return;
  const double gj = d.g[(int64_t)slot * J + j];
  const double* __restrict__ f = d.f + (int64_t)slot * I;
  double s = 0.0;
  for (int i = 0; i < I; ++i) {
    const double x = term(f[i] + gj, (double)C[(int64_t)i * ldc + j], inv_reg);
    s += x == -INFINITY ? 0.0 : exp_f64(x);
  }
  col_sum[j] = s;
}

}  // namespace skshard
}  // namespace gnnea

// the scaling-form variant (sinkhorn.hip): taken for variant 0 and J <= its sweep's limit
namespace gnnea {
namespace skscale {
bool shard_ok(const gnnea_sinkhorn* p);
int64_t shard_ws_bytes(int I, int J);
int shard_pair_len(const gnnea_sinkhorn* p);
int shard_init(const gnnea_sinkhorn* p, int I_global, void* stream);
int shard_colpart(const gnnea_sinkhorn* p, double* pair, void* stream);
int shard_step(const gnnea_sinkhorn* p, int it, const double* pairs, int W, void* stream);
int shard_finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype, int64_t ldp,
                 double* row_sum, double* loss_part, double* col_part, void* stream);
}  // namespace skscale
}  // namespace gnnea

using namespace gnnea;
using namespace gnnea::skshard;

// workspace: status block | f[2][I] | g[2][J] | log a[I] | log b[J] | b[J] | errpart | split
// partials [ns][J] x 2 | per-row losses [I]
static int64_t sh_al(int64_t x) { return (x + 255) & ~(int64_t)255; }
struct ShWs {
  int64_t f, g, la, lb, bw, err, pm, ps, loss, total;
  int nerr;
};
static ShWs sh_plan(int I, int J) {
  ShWs w;
  int64_t o = GNNEA_SK_STATUS_BYTES;
  w.f = o; o = sh_al(o + 16ll * I);
  w.g = o; o = sh_al(o + 16ll * J);
  w.la = o; o = sh_al(o + 8ll * I);
  w.lb = o; o = sh_al(o + 8ll * J);
  w.bw = o; o = sh_al(o + 8ll * J);
  w.nerr = (J + 255) / 256;
  w.err = o; o = sh_al(o + 8ll * w.nerr);
  w.pm = o; o = sh_al(o + 8ll * kMaxSplits * J);
  w.ps = o; o = sh_al(o + 8ll * kMaxSplits * J);
  w.loss = o; o = sh_al(o + 8ll * I);
  w.total = o;
  return w;
}

static Dev sh_dev(const gnnea_sinkhorn* p) {
  const ShWs w = sh_plan(p->I, p->J);
  char* b = (char*)p->ws;
  Dev d;
  d.st = (int64_t*)b;
  d.sd = (double*)b;
  d.f = (double*)(b + w.f);
  d.g = (double*)(b + w.g);
  d.la = (double*)(b + w.la);
  d.lb = (double*)(b + w.lb);
  d.bw = (double*)(b + w.bw);
  d.errpart = (double*)(b + w.err);
  d.pm = (double*)(b + w.pm);
  d.ps = (double*)(b + w.ps);
  d.nerr = w.nerr;
  return d;
}

static int sh_splits(int I, int J) {  // fill ~512 workgroups of the local column pass
  const int strips = (J + 63) / 64;
  int ns = (512 + strips - 1) / strips;
  const int by_rows = (I + 127) / 128;
  ns = ns > by_rows ? by_rows : ns;
  ns = ns > kMaxSplits ? kMaxSplits : ns;
  return ns < 1 ? 1 : ns;
}

static bool sh_ok(const gnnea_sinkhorn* p) {
  return p && p->ws && p->C && p->a && p->b && p->I >= 1 && p->J >= 1 && p->ldc >= p->J &&
         p->mode == GNNEA_SK_KNOPP && (p->c_dtype == GNNEA_F32 || p->c_dtype == GNNEA_F64) &&
         p->eps > 0.0;
}

extern "C" int64_t gnnea_sinkhorn_shard_ws_bytes(int I_local, int J) {
  if (I_local < 1 || J < 1) return GNNEA_EINVAL;
  const int64_t lg = sh_plan(I_local, J).total, sc = skscale::shard_ws_bytes(I_local, J);
  return sc > lg ? sc : lg;
}

// doubles per rank of the gathered row: J + 2 (scaling form: column sums, flag) or 2J + 2
// (log domain: (max, sum-exp) pairs, flag)
extern "C" int gnnea_sinkhorn_shard_pair_len(const gnnea_sinkhorn* p) {
  if (!sh_ok(p)) return GNNEA_EINVAL;
  return skscale::shard_ok(p) ? skscale::shard_pair_len(p) : 2 * p->J + 2;
}

extern "C" int gnnea_sinkhorn_shard_init(const gnnea_sinkhorn* p, int I_global, void* stream) {
  if (!sh_ok(p) || I_global < p->I) return GNNEA_EINVAL;
  if (skscale::shard_ok(p)) return skscale::shard_init(p, I_global, stream);
  const int n = p->I > p->J ? p->I : p->J;
  hipLaunchKernelGGL(k_sh_init, dim3(div_up(n > 32 ? n : 32, 256)), dim3(256), 0,
                     (hipStream_t)stream, p->I, p->J, I_global, p->tol, p->a, p->b, sh_dev(p));
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_shard_colpart(const gnnea_sinkhorn* p, int it, double* pair,
                                            void* stream) {
  if (!sh_ok(p) || it < 0 || !pair) return GNNEA_EINVAL;
  if (skscale::shard_ok(p)) return skscale::shard_colpart(p, pair, stream);
  hipStream_t s = (hipStream_t)stream;
  const Dev d = sh_dev(p);
  const int ns = sh_splits(p->I, p->J);
  const int rps = (p->I + ns - 1) / ns;
  const int slot_f = (it + 1) & 1;  // f_{it-1}
  const double inv_reg = 1.0 / p->eps;
  const dim3 grid(div_up(p->J, 64), ns);
  if (p->c_dtype == GNNEA_F32)
    hipLaunchKernelGGL(k_sh_colpart<float>, grid, dim3(1024), 0, s, (const float*)p->C, p->ldc,
                       p->I, p->J, inv_reg, d, slot_f, rps);
  else
    hipLaunchKernelGGL(k_sh_colpart<double>, grid, dim3(1024), 0, s, (const double*)p->C, p->ldc,
                       p->I, p->J, inv_reg, d, slot_f, rps);
  hipLaunchKernelGGL(k_sh_pairs, dim3(div_up(p->J, 256)), dim3(256), 0, s, d, p->J, ns, pair);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_shard_step(const gnnea_sinkhorn* p, int it, const double* pairs,
                                         int W, void* stream) {
  if (!sh_ok(p) || it < 0 || !pairs || W < 1) return GNNEA_EINVAL;
  if (skscale::shard_ok(p)) return skscale::shard_step(p, it, pairs, W, stream);
  hipStream_t s = (hipStream_t)stream;
  const Dev d = sh_dev(p);
  const double inv_reg = 1.0 / p->eps;
  hipLaunchKernelGGL(k_sh_colfin, dim3(d.nerr), dim3(256), 0, s, pairs, W, p->J, d, it);
  hipLaunchKernelGGL(k_sh_decide, dim3(1), dim3(1), 0, s, pairs, W, p->J, d, it);
  if (p->c_dtype == GNNEA_F32)
    hipLaunchKernelGGL(k_sh_row<float>, dim3(div_up(p->I, 4)), dim3(256), 0, s,
                       (const float*)p->C, p->ldc, p->I, p->J, inv_reg, d, it);
  else
    hipLaunchKernelGGL(k_sh_row<double>, dim3(div_up(p->I, 4)), dim3(256), 0, s,
                       (const double*)p->C, p->ldc, p->I, p->J, inv_reg, d, it);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_shard_flag(const gnnea_sinkhorn* p, double* flag, void* stream) {
  if (!sh_ok(p) || !flag) return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_sh_flag, dim3(1), dim3(64), 0, (hipStream_t)stream, sh_dev(p), flag);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_shard_close(const gnnea_sinkhorn* p, const double* flags, int W,
                                          void* stream) {
  if (!sh_ok(p) || !flags || W < 1 || p->iters_run < 0) return GNNEA_EINVAL;
  hipLaunchKernelGGL(k_sh_close, dim3(1), dim3(1), 0, (hipStream_t)stream, flags, W, sh_dev(p),
                     p->iters_run);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_shard_finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype,
                                           int64_t ldp, double* row_sum, double* loss_part,
                                           double* col_part, void* stream) {
  if (!sh_ok(p) || !loss_part) return GNNEA_EINVAL;
  if (plan && ((plan_dtype != GNNEA_F32 && plan_dtype != GNNEA_F64) || ldp < p->J))
    return GNNEA_EINVAL;
  if (skscale::shard_ok(p))
    return skscale::shard_finish(p, plan, plan_dtype, ldp, row_sum, loss_part, col_part, stream);
  hipStream_t s = (hipStream_t)stream;
  const Dev d = sh_dev(p);
  double* loss_rows = (double*)((char*)p->ws + sh_plan(p->I, p->J).loss);
  const double inv_reg = 1.0 / p->eps;
  const dim3 grow(div_up(p->I, 4));
#define GNNEA_SHP(T, PT)                                                                       \
  hipLaunchKernelGGL((k_sh_plan<T, PT>), grow, dim3(256), 0, s, (const T*)p->C, p->ldc, p->I,  \
                     p->J, inv_reg, d, (PT*)plan, ldp, row_sum, loss_rows)
  if (p->c_dtype == GNNEA_F32) {
    if (plan_dtype == GNNEA_F32) GNNEA_SHP(float, float);
    else GNNEA_SHP(float, double);
  } else {
    if (plan_dtype == GNNEA_F32) GNNEA_SHP(double, float);
    else GNNEA_SHP(double, double);
  }
#undef GNNEA_SHP
  hipLaunchKernelGGL(k_sh_loss, dim3(1), dim3(1024), 0, s, loss_rows, p->I, loss_part);
  if (col_part) {
    if (p->c_dtype == GNNEA_F32)
      hipLaunchKernelGGL(k_sh_colsum<float>, dim3(div_up(p->J, 256)), dim3(256), 0, s,
                         (const float*)p->C, p->ldc, p->I, p->J, inv_reg, d, col_part);
    else
      hipLaunchKernelGGL(k_sh_colsum<double>, dim3(div_up(p->J, 256)), dim3(256), 0, s,
                         (const double*)p->C, p->ldc, p->I, p->J, inv_reg, d, col_part);
  }
  GNNEA_LAUNCH_CHECK();
  return 0;
}
