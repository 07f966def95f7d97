// a9-a12. Sinkhorn solvers in the reference's own scaling form (fp64 arithmetic, fp32 or fp64
// cost storage, the kernel matrix K kept resident in HBM as fp64).
//
//   KNOPP (utils/ot_loss.py:5-76): K = exp(M / -reg) once; per iteration
//       v = b / (K^T u)       (:53-54)      u = 1 / (Kp v),  Kp = (1/a) K   (:45, :55)
//     break with the previous (u, v) on K^T u == 0 or NaN / inf in u, v (:57-62);
//     err = ||v (K^T u) - b||_2 for iterates with cpt % 10 == 0 (:64-66), tested by the loop
//     condition before the next iteration (:50).  Plan P = u K v, loss = sum P M (:74-75).
//   STAB / GEN / RELAX (SinkhornOT/sinkhorn_loss.py:159-356): K = clamp(exp((u + v - C)/eps), 0,
//   1e30); per iteration a = clamp((mu / K b)^p_row), b = clamp((nu / K^T a)^p_col); absorption
//   (ii % 10 == 0, max(a|b) > 1e20, last iteration): u += eps log a, v += eps log b, K recomputed,
//   b = 1, transport = sum K C, relative-tolerance break.
//
// One sweep over K per iteration (k_sk_sweep): a workgroup of 8 waves owns R consecutive rows;
// per group of 8 rows each wave reduces one row against the column scaling (K x, the row update:
// u or a), then the 8 waves re-read the group's rows (L2-hot) column-sliced and accumulate that
// row update into the workgroup's partial of the NEXT column pass (K^T u or K^T a) in registers.
// k_sk_colfin sums the ~256 workgroup partials of each column in fixed order and applies the
// column update.  K is streamed once per iteration (I*J*8 bytes: Infinity-Cache / HBM bandwidth
// bound); exp work is one pass at initialisation (KNOPP) or per absorption (every 10th iteration).
// A device status block gates every kernel, so iterations enqueued past the stop are no-ops.
#include "common.h"

#include <stdlib.h>

namespace gnnea {

constexpr double kBig = 1e20;   // sinkhorn_loss.py:11
constexpr double kHuge = 1e30;  // sinkhorn_loss.py:12
constexpr int kSweepWaves = 8;  // waves (rows per group) of a sweep workgroup
// widest J the fused sweep serves: its column slices live in registers (NCM <= 32 per lane; above
// 16 the column scaling moves to LDS so the K double buffer still fits); beyond it the log-domain
// passes take over
constexpr int kMaxJ = 64 * kSweepWaves * 32;
constexpr int kMaxSweepWg = 64 * 8;  // column partials the update kernel sums in one round
// the on-chip KNOPP kernel (k_sk_res): thread tile rows / columns, tile rows kept in VGPRs
constexpr int kResRA = 9, kResCA = 16, kResRR = 5, kResLR = kResRA - kResRR;
constexpr int kResRows = 16 * kResRA, kResCols = 16 * kResCA;  // 144 x 256 per workgroup
constexpr int kResMaxWg = 256;

enum { ST_DONE = 0, ST_ITERS = 1, ST_REASON = 2, ST_SLOT = 3, ST_BIG = 4, ST_FAIL = 5, ST_UFAIL = 6 };
enum { SD_ERR = GNNEA_SK_SD_ERR, SD_TPREV = GNNEA_SK_SD_TPREV, SD_LOSS = GNNEA_SK_SD_LOSS,
       SD_TOL = GNNEA_SK_SD_TOL, SD_TNEW = GNNEA_SK_SD_TNEW };

static inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// rows per sweep workgroup: about 256 workgroups (one per CU) whatever I is
static int sk_rows_per_wg(int I) { return (I + 255) / 256; }

struct SkWs {
  int64_t K, u, v, pu, pv, rowbuf, part, errpart, total;
  int64_t flags, rowpart, colpart, rowaux, colaux;  // the on-chip KNOPP path (k_sk_res)
  int ns, nfin, rpw;
};

constexpr int kFinCols = 16;  // columns per update workgroup (64 slots split the partials)
constexpr int64_t kResFlagBytes = 4 * (2 * kResMaxWg + 64);  // rflag[256], cflag[256], entry counter

static SkWs sk_plan(int I, int J) {
  SkWs w;
  w.rpw = sk_rows_per_wg(I);
  if ((I + w.rpw - 1) / w.rpw > kMaxSweepWg) w.rpw = (I + kMaxSweepWg - 1) / kMaxSweepWg;
  w.ns = (I + w.rpw - 1) / w.rpw;  // sweep workgroups = column partials per column
  w.nfin = (J + kFinCols - 1) / kFinCols;
  int64_t o = GNNEA_SK_STATUS_BYTES;
  w.u = o; o = al256(o + 2 * 8ll * I);
  w.v = o; o = al256(o + 2 * 8ll * J);
  w.pu = o; o = al256(o + 8ll * I);
  w.pv = o; o = al256(o + 8ll * J);
  w.rowbuf = o; o = al256(o + 8ll * I);
  w.part = o; o = al256(o + 8ll * w.ns * J);
  w.errpart = o; o = al256(o + 8ll * w.nfin);
  // + 64 KB: the wide sweep's unclamped loads run up to ~2,600 elements past the last row's end
  w.K = o; o = al256(o + 8ll * I * J + 65536);
  // k_sk_res: flags (row / column phase epochs per workgroup, the entry counter) and the
  // double-buffered row / column partials (sized for the largest grid, kResMaxWg workgroups)
  const int P = div_up(I, kResRows), Q = div_up(J, kResCols);  // res_geom's grid
  w.flags = o; o = al256(o + kResFlagBytes);
  w.rowpart = o; o = al256(o + 8ll * 2 * Q * I);
  w.colpart = o; o = al256(o + 8ll * 2 * P * J);
  w.rowaux = o; o = al256(o + 8ll * 2 * 2 * kResMaxWg);
  w.colaux = o; o = al256(o + 8ll * 2 * kResMaxWg);
  w.total = o;
  return w;
}

struct SkArgs {
  int mode, I, J, ns, nfin, rpw;
  int ig;     // rows of the whole problem (u0 = 1/ig); I unless the rows are sharded
  int shard;  // row-sharded (gnnea_sinkhorn_shard_*): a bad u is flagged, not decided locally
  int64_t ldc;
  double eps, p_row, p_col;
  const double *a, *b;  // source / target weights (a, b or mu, nu)
};

struct SkDev {
  int64_t* st;   // status ints
  double* sd;    // status doubles
  double *K, *u, *v, *pu, *pv, *rowbuf, *part, *errpart;
  double *rowpart, *colpart, *rowaux, *colaux;
  unsigned *rflag, *cflag, *ecnt;
};

static SkDev sk_dev(const gnnea_sinkhorn* p) {
  const SkWs w = sk_plan(p->I, p->J);
  char* b = (char*)p->ws;
  SkDev d;
  d.st = (int64_t*)b;
  d.sd = (double*)b;
  d.K = (double*)(b + w.K);
  d.u = (double*)(b + w.u);
  d.v = (double*)(b + w.v);
  d.pu = (double*)(b + w.pu);
  d.pv = (double*)(b + w.pv);
  d.rowbuf = (double*)(b + w.rowbuf);
  d.part = (double*)(b + w.part);
  d.errpart = (double*)(b + w.errpart);
  d.rowpart = (double*)(b + w.rowpart);
  d.colpart = (double*)(b + w.colpart);
  d.rowaux = (double*)(b + w.rowaux);
  d.colaux = (double*)(b + w.colaux);
  d.rflag = (unsigned*)(b + w.flags);
  d.cflag = d.rflag + kResMaxWg;
  d.ecnt = d.rflag + 2 * kResMaxWg;
  return d;
}

static SkArgs sk_args(const gnnea_sinkhorn* p) {
  const SkWs w = sk_plan(p->I, p->J);
  SkArgs a;
  a.mode = p->mode;
  a.I = p->I;
  a.J = p->J;
  a.ns = w.ns;
  a.nfin = w.nfin;
  a.rpw = w.rpw;
  a.ldc = p->ldc;
  a.eps = p->eps;
  const bool gen = p->mode == GNNEA_SK_GEN, relax = p->mode == GNNEA_SK_RELAX;
  a.p_row = gen ? p->p : 1.0;
  a.p_col = (gen || relax) ? p->p : 1.0;
  a.a = p->a;
  a.b = p->b;
  a.ig = p->I;
  a.shard = 0;
  return a;
}

__device__ __forceinline__ void mark_done(int64_t* st, int64_t iters, int64_t reason,
                                          int64_t slot) {
  if (atomicCAS((unsigned long long*)&st[ST_DONE], 0ull, 1ull) == 0ull) {
    st[ST_ITERS] = iters;
    st[ST_REASON] = reason;
    st[ST_SLOT] = slot;
  }
}

__device__ __forceinline__ double myclamp(double x) {  // torch.clamp(x, 0, 1e30)
  return x != x ? x : fmin(fmax(x, 0.0), kHuge);
}

// (mu / s) ** p  as torch: p == 1 leaves the quotient untouched.  Out of line: the sweep calls it
// from one lane per row and must not pay pow's registers in its streaming loop.
__device__ __noinline__ double pow_slow(double q, double p) { return pow(q, p); }
__device__ __forceinline__ double powp(double q, double p) { return p == 1.0 ? q : pow_slow(q, p); }

// ---------------------------------------------------------------------------------------- //
// K construction
// ---------------------------------------------------------------------------------------- //
// KNOPP: K = exp(M / -reg)      (torch.div(M, -reg, out=K); torch.exp(K, out=K))
// STAB : K = clamp(exp(((pu_i + pv_j) - C_ij) / eps)), and the row sums of K * C for transport
template <typename T, bool KNOPP>
__global__ __launch_bounds__(256) void k_sk_kbuild(const T* __restrict__ C, SkArgs a, SkDev d,
                                                   int it, int max_iter, int init) {
  if (!KNOPP) {
    if (d.st[ST_DONE]) return;
    const bool absorb = init || (it % 10 == 0) || d.st[ST_BIG] || it == max_iter - 1;
    if (!absorb) return;
  }
  const int i = xcd_remap(blockIdx.x, gridDim.x) * 4 + wave_id();
  if (i >= a.I) return;
  const int lane = lane_id();
  const T* Ci = C + (int64_t)i * a.ldc;
  double* Ki = d.K + (int64_t)i * a.J;
  const double pui = KNOPP ? 0.0 : d.pu[i];
  const double neg_reg = -a.eps;
  double acc = 0.0;
  for (int j = lane; j < a.J; j += 64) {
    const double c = (double)Ci[j];
    double k;
    if (KNOPP) {
      k = exp_f64(c / neg_reg);
    } else {
      k = myclamp(exp_f64(((pui + d.pv[j]) - c) / a.eps));
      acc += k * c;
    }
    Ki[j] = k;
  }
  if (!KNOPP) {
    acc = wave_sum(acc);
    if (lane == 0) d.rowbuf[i] = acc;
  }
}

// ---------------------------------------------------------------------------------------- //
// Row pass: s_i = sum_j K_ij x_j, one wave per row, 8 loads in flight per lane.
//   KNOPP: u_i = 1 / sum_j ((1/a_i) K_ij) v_j              (x = v[slot_in], out u[slot_out])
//   STAB : a_i = clamp((mu_i / s_i)^p_row)                  (x = b = v[slot_in])
// ---------------------------------------------------------------------------------------- //
template <bool KNOPP>
__device__ __forceinline__ bool knopp_stop(const SkArgs& a, SkDev& d, int it) {
  // the loop condition for iterate it-1 (err > stopThr), then the K^T u == 0 / inf / NaN break
  // of iteration it (flagged by its column update); every row workgroup takes the same decision
  __shared__ int stop;
  if (wave_id() == 0) {
    const int lane = lane_id();
    const int prev = it - 1;
    int st = 0;
    if (prev >= 0 && prev % 10 == 0) {
      double e = 0.0;
      for (int q = lane; q < a.nfin; q += 64) e += d.errpart[q];
      const double err = sqrt(wave_sum(e));
      if (!(err > d.sd[SD_TOL])) st = 1;
      if (blockIdx.x == 0 && lane == 0) {
        d.sd[SD_ERR] = err;
        if (st) mark_done(d.st, prev + 1, 1, prev & 1);
      }
    }
    if (!st && d.st[ST_FAIL]) {
      st = 1;
      if (blockIdx.x == 0 && lane == 0) mark_done(d.st, it, 2, (it + 1) & 1);
    }
    if (lane == 0) stop = st;
  }
  __syncthreads();
  return stop != 0;
}

// Sweep.  A workgroup of 8 waves owns rows [r0, r1); wave w owns the column slice
// c0 + 64 k + lane (k < nc) of every row.  Per group of G rows the wave loads its slice of all G
// rows at once (G * NCM independent loads), the next group's loads in flight while the current
// group is reduced (register double buffer; plain loads stay in flight across __syncthreads), and
//   PH1:  row sums s_r = sum_j K_rj x_j (x = v / b of slot_in) are reduced lane -> wave -> the 8
//         waves (LDS, fixed order) into the row update y_r (u or a, written to u[slot_out]);
//   !PH1: y_r = yin[r] (column sums of the final plan);
// then the same registers accumulate acc_j += y_r K_rj: part[wg][j] = sum over the workgroup's
// rows, in row order.  K is read exactly once.
// PW: the row exponent p_row may differ from 1 (GEN): only then does the sweep contain pow's
// out-of-line call, whose register saves would otherwise spill the K double buffer in the loop
template <bool KNOPP, bool PH1, int NCM, bool PW = false>
__global__ __launch_bounds__(64 * kSweepWaves) void k_sk_sweep(SkArgs a, SkDev d, int it,
                                                               int slot_in, int slot_out,
                                                               const double* __restrict__ yin,
                                                               int gate) {
  constexpr int G = NCM <= 8 ? 32 / NCM : (NCM <= 16 ? 2 : 1);  // rows per group
  // NCM > 16 (J > 8192): the wave's slice of the column scaling x lives in LDS (each lane reads
  // back only what it wrote: no barrier), which keeps K double-buffered in registers
  constexpr bool XL = NCM > 16;
  __shared__ double red[2][kSweepWaves][G];
  __shared__ double xsh[XL ? kSweepWaves * NCM * 64 : 1];
  const int w = wave_id(), lane = lane_id();
  const int wg = blockIdx.x;
  const int r0 = wg * a.rpw, r1 = min(a.I, r0 + a.rpw);
  const int cw = ((a.J + kSweepWaves - 1) / kSweepWaves + 63) & ~63;
  const int c0 = w * cw;
  bool ok[XL ? 1 : NCM];
  double xs[XL ? 1 : NCM], acc[NCM];
  const double* __restrict__ x = d.v + (int64_t)slot_in * a.J;
#pragma unroll
  for (int k = 0; k < NCM; ++k) {
    const int c = c0 + 64 * k + lane;
    const bool okk = 64 * k < cw && c < a.J;
    if constexpr (!XL) ok[k] = okk;
    const double xv = (PH1 && okk) ? x[c] : 0.0;
    if constexpr (XL) xsh[(w * NCM + k) * 64 + lane] = xv;
    else xs[k] = xv;
    acc[k] = 0.0;
  }
  auto xs_at = [&](int k) -> double {
    if constexpr (XL) return xsh[(w * NCM + k) * 64 + lane];
    else return xs[k];
  };
  // branch-free loads: out-of-range rows / columns read a clamped in-range address, then zero
  // (XL: indices and masks recomputed per load instead of held in 2 * NCM registers)
  int cidx[XL ? 1 : NCM];
  if constexpr (!XL) {
#pragma unroll
    for (int k = 0; k < NCM; ++k) cidx[k] = min(c0 + 64 * k + lane, a.J - 1);
  }
  // XL validity of column c0 + 64 k + lane as one compare: 64 k < lim (inside the wave's slice and J)
  const int lim = min(c0 + cw, a.J) - c0 - lane;
  auto load = [&](double (&kv)[G][NCM], int g0) {
#pragma unroll
    for (int r = 0; r < G; ++r) {
      const double* __restrict__ Kr = d.K + (int64_t)min(g0 + r, r1 - 1) * a.J;
#pragma unroll
      for (int k = 0; k < NCM; ++k) {
        if constexpr (XL) {  // unclamped: one base + immediate offsets (K is padded, sk_plan)
          const double t = Kr[c0 + 64 * k + lane];
          kv[r][k] = 64 * k < lim ? t : 0.0;
        } else {
          const double t = Kr[cidx[k]];
          kv[r][k] = ok[k] ? t : 0.0;
        }
      }
    }
  };
  auto process = [&](const double (&kv)[G][NCM], int g0, int par) {
    const int nr = min(G, r1 - g0);
    double yv[G];
    if (PH1) {
#pragma unroll
      for (int r = 0; r < G; ++r) {
        double p = 0.0;
        if (r < nr) {
          const double inva = KNOPP ? 1.0 / a.a[g0 + r] : 1.0;
#pragma unroll
          for (int k = 0; k < NCM; ++k) p = fma(KNOPP ? inva * kv[r][k] : kv[r][k], xs_at(k), p);
        }
        p = wave_sum_f64(p);
        if (lane == 0) red[par][w][r] = p;
      }
      // the only barrier of the group (red[par] is double-buffered).  STAB / GEN / RELAX: the
      // wave partials in LDS are complete (lgkmcnt(0)), then a raw s_barrier -- __syncthreads()
      // is a workgroup fence too, whose vmcnt(0) drained the next group's K loads (the prefetch)
      // at every group: sinkhorn_iteration at B = 15000 2,164 -> 2,385 iters/s.  KNOPP keeps
      // the fence (its row loads of 1/a sit behind the prefetch: 2,770 -> 2,628 without it)
      if constexpr (KNOPP) {
        __syncthreads();
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      // every wave reduces the 8 wave partials of each row itself (same order -> same y)
#pragma unroll
      for (int r = 0; r < G; ++r) {
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < kSweepWaves; ++q) sum += red[par][q][r];
        double y = 0.0;
        if (r < nr) {
          if (KNOPP) {
            y = 1.0 / sum;  // u = 1 / (Kp v)
          } else {
            const double qr = a.a[g0 + r] / sum;  // a = clamp((mu / K b)^p)
            y = myclamp(PW ? powp(qr, a.p_row) : qr);
          }
          if (w == 0 && lane == r) {
            d.u[(int64_t)slot_out * a.I + g0 + r] = y;
            if (KNOPP && (y != y || isinf(y))) {
              if (a.shard) atomicOr((unsigned long long*)&d.st[ST_UFAIL], 1ull);  // all ranks decide
              else mark_done(d.st, it, 2, (it + 1) & 1);
            }
            if (!KNOPP && y > kBig) atomicOr((unsigned long long*)&d.st[ST_BIG], 1ull);
          }
        }
        yv[r] = y;
      }
    } else {
#pragma unroll
      for (int r = 0; r < G; ++r) yv[r] = r < nr ? yin[g0 + r] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < G; ++r) {
      if (r < nr) {
#pragma unroll
        for (int k = 0; k < NCM; ++k) acc[k] = fma(yv[r], kv[r][k], acc[k]);
      }
    }
  };
  double kA[G][NCM], kB[G][NCM];
  int g0 = r0;
  // the first group's loads go out before the stop decisions (two dependent round trips on the
  // status block); loading K is harmless when the iteration turns out to be a no-op
  if (g0 < r1) load(kA, g0);
  if (gate && d.st[ST_DONE]) return;
  if (PH1 && KNOPP && knopp_stop<KNOPP>(a, d, it)) return;
  // STAB / GEN / RELAX: the next group's loads go out unconditionally (past the last group: the
  // last rows again, never used), so every path into a group's processing has the same loads
  // outstanding and the compiler's waits there cover only the group being processed (KNOPP: as
  // before, loads only for groups that exist)
  while (g0 < r1) {
    const int g1 = g0 + G;
    if (!KNOPP || g1 < r1) load(kB, g1);
    process(kA, g0, 0);
    if (g1 >= r1) break;
    const int g2 = g1 + G;
    if (!KNOPP || g2 < r1) load(kA, g2);
    process(kB, g1, 1);
    g0 = g2;
  }
  double* __restrict__ part = d.part + (int64_t)wg * a.J + c0 + lane;
#pragma unroll
  for (int k = 0; k < NCM; ++k)
    if (64 * k < cw && c0 + 64 * k + lane < a.J) part[64 * k] = acc[k];
}

// Column update: s_j = sum_q part[q][j], then
//   KNOPP: err^2 term of iterate it-1 (v_{it-1} s_j - b_j)^2, v_j = b_j / s_j, break flags
//   STAB : b_j = clamp((nu_j / s_j)^p_col), big flag
//   SUM  : col_sum_j = s_j (times v_j for a KNOPP plan)
// A 1024-thread workgroup owns kFinCols = 16 columns: lane & 15 is the column, the 64 (wave,
// lane >> 4) slots stride the partials (all loads of a thread in flight at once); the 64 slot sums
// of a column are added in slot order (deterministic).
enum { FIN_KNOPP = 0, FIN_STAB = 1, FIN_SUM = 2 };

template <int MODE>
__global__ __launch_bounds__(1024) void k_sk_colfin(SkArgs a, SkDev d, int slot_prev,
                                                    int slot_out, double* __restrict__ col_sum) {
  if (MODE != FIN_SUM && d.st[ST_DONE]) return;
  __shared__ double red[64][kFinCols];
  const int lane = lane_id(), w = wave_id();
  const int cl = lane & (kFinCols - 1), slot = w * 4 + (lane >> 4);
  const int j = blockIdx.x * kFinCols + cl;
  const int jc = min(j, a.J - 1);
  constexpr int kU = kMaxSweepWg / 64;
  double pv[kU];
#pragma unroll
  for (int k = 0; k < kU; ++k) {
    const int q = slot + 64 * k;
    const double t = d.part[(int64_t)min(q, a.ns - 1) * a.J + jc];
    pv[k] = q < a.ns ? t : 0.0;
  }
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int k = 0; k < kU; k += 2) {
    s0 += pv[k];
    s1 += pv[k + 1];
  }
  red[slot][cl] = s0 + s1;
  __syncthreads();
  if (w != 0 || lane >= kFinCols) return;
  double s = 0.0;
#pragma unroll 8
  for (int q = 0; q < 64; ++q) s += red[q][cl];
  double errp = 0.0;
  bool fail = false, big = false;
  if (j < a.J) {
    if (MODE == FIN_KNOPP) {
      const double t = d.v[(int64_t)slot_prev * a.J + j] * s - a.b[j];
      errp = t * t;
      const double vj = a.b[j] / s;
      fail = s == 0.0 || vj != vj || isinf(vj);
      d.v[(int64_t)slot_out * a.J + j] = vj;
    } else if (MODE == FIN_STAB) {
      const double bj = myclamp(powp(a.b[j] / s, a.p_col));
      big = bj > kBig;
      d.v[(int64_t)slot_out * a.J + j] = bj;
    } else {
      const int fs = (int)(d.st[ST_SLOT] & 1);
      col_sum[j] = a.mode == GNNEA_SK_KNOPP ? s * d.v[(int64_t)fs * a.J + j] : s;
    }
  }
  if (MODE == FIN_KNOPP) {
#pragma unroll
    for (int o = kFinCols / 2; o > 0; o >>= 1) errp += __shfl_xor(errp, o, 64);
    const unsigned long long anyf = __ballot(fail) & ((1ull << kFinCols) - 1);
    if (lane == 0) {
      d.errpart[blockIdx.x] = errp;
      if (anyf) atomicOr((unsigned long long*)&d.st[ST_FAIL], 1ull);
    }
  } else if (MODE == FIN_STAB) {
    const unsigned long long anyb = __ballot(big) & ((1ull << kFinCols) - 1);
    if (lane == 0 && anyb) atomicOr((unsigned long long*)&d.st[ST_BIG], 2ull);
  }
}

// ---------------------------------------------------------------------------------------- //
// STAB absorption: pu += eps log a, pv += eps log b, b = 1; then k_sk_kbuild<STAB> rebuilds K
// with the row sums of K C, and k_sk_absorb_final takes the transport / tolerance decision.
// ---------------------------------------------------------------------------------------- //
__global__ __launch_bounds__(256) void k_sk_absorb_vec(SkArgs a, SkDev d, int it, int slot,
                                                       int max_iter) {
  if (d.st[ST_DONE]) return;
  const bool absorb = (it % 10 == 0) || d.st[ST_BIG] || it == max_iter - 1;
  if (!absorb) return;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < a.I) d.pu[t] += a.eps * log(d.u[(int64_t)slot * a.I + t]);
  if (t < a.J) {
    double* b = d.v + (int64_t)slot * a.J;
    d.pv[t] += a.eps * log(b[t]);
    b[t] = 1.0;
  }
}

__global__ __launch_bounds__(1024) void k_sk_absorb_final(SkArgs a, SkDev d, int it, int slot,
                                                          int max_iter, int init) {
  if (d.st[ST_DONE]) return;
  const bool absorb = init || (it % 10 == 0) || d.st[ST_BIG] || it == max_iter - 1;
  __syncthreads();
  if (!absorb) return;
  __shared__ double red[1024];
  double s = 0.0;
  for (int i = threadIdx.x; i < a.I; i += 1024) s += d.rowbuf[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  const double tnew = red[0];
  d.st[ST_BIG] = 0;
  d.sd[SD_TNEW] = tnew;
  if (init) {
    d.sd[SD_TPREV] = tnew;
    return;
  }
  const double tprev = d.sd[SD_TPREV];
  if (fabs(tnew - tprev) / fabs(tprev) < d.sd[SD_TOL]) {
    mark_done(d.st, it, 1, slot);  // break: ii stays, `transport` keeps the previous value
    return;
  }
  d.sd[SD_TPREV] = tnew;
  if (it == max_iter - 1) mark_done(d.st, max_iter, 0, slot);
}

__global__ void k_sk_init(SkArgs a, SkDev d, double tol) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 32) {
    if (t < 8) d.st[t] = 0;
    else d.sd[t] = 0.0;
    if (t == SD_TOL) d.sd[SD_TOL] = tol;
  }
  const bool knopp = a.mode == GNNEA_SK_KNOPP;
  // KNOPP: u = 1/I, v = 1/J in slot 1 (the "previous" slot of iteration 0);
  // STAB: potentials 0 and b = 1 in slot 1
  for (int i = t; i < a.I; i += gridDim.x * blockDim.x) {
    d.pu[i] = 0.0;
    d.u[i] = 0.0;
    d.u[a.I + i] = knopp ? 1.0 / (double)a.ig : 1.0;
  }
  for (int j = t; j < a.J; j += gridDim.x * blockDim.x) {
    d.pv[j] = 0.0;
    d.v[j] = 0.0;
    d.v[a.J + j] = knopp ? 1.0 / (double)a.J : 1.0;
  }
}

// ---------------------------------------------------------------------------------------- //
// Finish: plan (KNOPP: P = u K v; STAB: K), its row sums, sum P M (KNOPP loss), column sums.
// ---------------------------------------------------------------------------------------- //
__device__ __forceinline__ int sk_final_slot(const SkDev& d, int iters_run) {
  if (d.st[ST_DONE]) return (int)(d.st[ST_SLOT] & 1);
  return iters_run > 0 ? ((iters_run - 1) & 1) : 1;
}

template <typename T, typename P>
__global__ __launch_bounds__(256) void k_sk_plan(const T* __restrict__ C, SkArgs a, SkDev d,
                                                 int iters_run, P* __restrict__ plan, int64_t ldp,
                                                 double* __restrict__ row_sum,
                                                 double* __restrict__ xcol) {
  const int slot = sk_final_slot(d, iters_run);
  const int i = blockIdx.x * 4 + wave_id();
  const bool knopp = a.mode == GNNEA_SK_KNOPP;
  if (blockIdx.x == 0 && threadIdx.x == 0) d.st[ST_SLOT] = slot;
  if (i >= a.I) return;
  const int lane = lane_id();
  const double ui = knopp ? d.u[(int64_t)slot * a.I + i] : 1.0;
  const double* v = d.v + (int64_t)slot * a.J;
  const double* Ki = d.K + (int64_t)i * a.J;
  const T* Ci = C + (int64_t)i * a.ldc;
  double rs = 0.0, loss = 0.0;
  for (int j = lane; j < a.J; j += 64) {
    const double pv = knopp ? (ui * Ki[j]) * v[j] : Ki[j];
    if (plan) plan[(int64_t)i * ldp + j] = (P)pv;
    rs += pv;
    if (knopp) loss += pv * (double)Ci[j];
  }
  rs = wave_sum(rs);
  loss = wave_sum(loss);
  if (lane == 0) {
    if (row_sum) row_sum[i] = rs;
    d.rowbuf[i] = loss;
    xcol[i] = ui;  // column-sum weights: u (KNOPP) or 1
  }
}

__global__ __launch_bounds__(1024) void k_sk_loss(SkArgs a, SkDev d, int iters_run) {
  __shared__ double red[1024];
  double s = 0.0;
  for (int i = threadIdx.x; i < a.I; i += 1024) s += d.rowbuf[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (a.mode == GNNEA_SK_KNOPP) d.sd[SD_LOSS] = red[0];
    if (!d.st[ST_DONE]) d.st[ST_ITERS] = iters_run;
  }
}

static bool sk_valid(const gnnea_sinkhorn* p) {
  if (!p || !p->C || !p->ws || !p->a || !p->b) return false;
  if (p->I < 1 || p->J < 1 || p->J > kMaxJ || p->ldc < p->J) return false;
  if (p->c_dtype != GNNEA_F32 && p->c_dtype != GNNEA_F64) return false;
  if (p->mode < GNNEA_SK_KNOPP || p->mode > GNNEA_SK_RELAX) return false;
  if (!(p->eps > 0.0)) return false;
  return true;
}

template <bool KNOPP, bool PH1, bool PW>
static void launch_sweep_pw(const SkArgs& a, const SkDev& d, int it, int si, int so,
                            const double* yin, int gate, hipStream_t s) {
  const dim3 g(a.ns), b(64 * kSweepWaves);
  const int nc = (((a.J + kSweepWaves - 1) / kSweepWaves + 63) & ~63) / 64;
  if (nc <= 4)
    hipLaunchKernelGGL((k_sk_sweep<KNOPP, PH1, 4, PW>), g, b, 0, s, a, d, it, si, so, yin, gate);
  else if (nc <= 8)
    hipLaunchKernelGGL((k_sk_sweep<KNOPP, PH1, 8, PW>), g, b, 0, s, a, d, it, si, so, yin, gate);
  else if (nc <= 16)
    hipLaunchKernelGGL((k_sk_sweep<KNOPP, PH1, 16, PW>), g, b, 0, s, a, d, it, si, so, yin, gate);
  else
    hipLaunchKernelGGL((k_sk_sweep<KNOPP, PH1, 32, PW>), g, b, 0, s, a, d, it, si, so, yin, gate);
}

template <bool KNOPP, bool PH1>
static void launch_sweep(const SkArgs& a, const SkDev& d, int it, int si, int so, const double* yin,
                         int gate, hipStream_t s) {
  if (!KNOPP && PH1 && a.p_row != 1.0)
    launch_sweep_pw<KNOPP, PH1, true>(a, d, it, si, so, yin, gate, s);
  else
    launch_sweep_pw<KNOPP, PH1, false>(a, d, it, si, so, yin, gate, s);
}

// ---------------------------------------------------------------------------------------- //
// KNOPP with K resident ON CHIP (utils/ot_loss.py:50-66 at the EA batch, B = 3000 and alike).
// At I * J <= ~9.4M the fp64 K fits the chip's registers + LDS: one workgroup per CU owns a
// block of at most 144 rows x 256 columns (P row blocks x Q column blocks, P * Q <= #CUs), keeps
// it in VGPRs (5 of 9 thread-tile rows) and LDS (the other 4) for a whole batch of iterations, and
// one persistent launch runs the batch.  Thread t = (ra, cb) = (t >> 4, t & 15) holds rows
// ra + 16 i (i < 9) and columns cb + 16 j (j < 16) of the block.  Per iteration `it`:
//   1. v_it = b / (K^T u_{it-1}) for the block's columns: the P row blocks' column partials of
//      K^T u_{it-1} summed in row-block order, and the err^2 terms of iterate it-1 (ot_loss.py:65);
//   2. row partials s_i = sum_j K_ij v_j over the block's columns (16-lane DPP sums, fixed order);
//   3. the Q column blocks' row partials summed in column-block order, u_it = 1 / ((1/a_i) s_i);
//      the stop decisions of knopp_stop (err of it-1, K^T u == 0 / bad v) taken identically by
//      every workgroup from the same published words;
//   4. column partials sum_i K_ij u_i over the block's rows for step 1 of iteration it + 1.
// K is read from HBM once per launch.  Hand-offs (cdna_hip_programming.md §6 Guideline 16, the
// all-sc1 form): payload words stored and loaded write-through (agent-scope relaxed atomics =
// global_store / global_load ... sc1), every storing wave drains (s_waitcnt vmcnt(0)), then a
// workgroup barrier and ONE lane's sc1 flag store carrying the phase epoch (row partials of
// iteration it: it + 1; column partials of iteration it: it + 2); a consumer's wave 0 polls the
// flags of the workgroups it reads (>= epoch, bounded spin), the other waves load after a
// workgroup barrier.  Payloads are double-buffered by iteration parity: a producer can run at
// most one iteration ahead of any consumer of the same buffer (it needs that consumer's next
// publication first).  Every spin is bounded (kResSpinTicks of the 100 MHz real-time counter):
// a timed-out workgroup sets GNNEA_SK_ST_TIMEOUT, marks the loop done and exits, and its peers
// time out in turn.  An entry barrier (monotonic arrival counter) separates every workgroup's read
// of ST_DONE from any write of it in the same launch, so all workgroups take the same decision.
// ---------------------------------------------------------------------------------------- //
constexpr uint64_t kResSpinTicks = 25000000ull;  // 250 ms at 100 MHz
enum { ST_TMO = GNNEA_SK_ST_TIMEOUT };

typedef __attribute__((address_space(1))) double res_gd;
typedef __attribute__((address_space(1))) unsigned int res_gu;

struct ResGeom {
  int P, Q, R, Cb;
  bool ok;
  uint64_t spin;  // bound of every inter-workgroup wait, real-time ticks (GNNEA_SK_DEBUG_SPIN: 0)
};

static ResGeom res_geom(int I, int J) {
  ResGeom g;
  g.P = div_up(I, kResRows);
  g.Q = div_up(J, kResCols);
  g.R = div_up(I, g.P);
  g.Cb = div_up(J, g.Q);
  g.ok = (int64_t)g.P * g.Q <= kResMaxWg;
  g.spin = kResSpinTicks;
  return g;
}

__device__ __forceinline__ void res_st(double* p, double x) {
  __hip_atomic_store((res_gd*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double res_ld(const double* p) {
  return __hip_atomic_load((res_gd*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned res_ldu(const unsigned* p) {
  return __hip_atomic_load((res_gu*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void res_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// sum_{k < n} p[k * stride] in a fixed order (even / odd k, then the two), every load of a chunk
// of 32 in flight at once: one round trip per chunk instead of one per partial
__device__ __forceinline__ double res_sum_strided(const double* p, int64_t stride, int n) {
  double s0 = 0.0, s1 = 0.0;
  for (int k0 = 0; k0 < n; k0 += 32) {
    double x[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = k0 + k < n ? res_ld(p + (int64_t)(k0 + k) * stride) : 0.0;
#pragma unroll
    for (int k = 0; k < 32; k += 2) {
      s0 += x[k];
      s1 += x[k + 1];
    }
  }
  return s0 + s1;
}

// one wave: until flags[base + k * stride] >= epoch for every k < n; false on timeout
__device__ bool res_wait(const unsigned* flags, int base, int stride, int n, unsigned epoch,
                         uint64_t spin) {
  const int lane = lane_id();
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
    for (int k = lane; k < n; k += 64) ok &= res_ldu(flags + base + k * stride) >= epoch;
    if (__all(ok)) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > spin) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

__device__ __forceinline__ void res_timeout(SkDev& d) {
  atomicOr((unsigned long long*)&d.st[ST_TMO], 1ull);
  mark_done(d.st, 0, 3, 0);
}

// workgroup sum in a fixed order (lanes by DPP, then waves 0..3): the same value on every
// workgroup that sums the same per-thread terms
__device__ __forceinline__ double res_block_sum(double x, double* red4) {
  x = wave_sum_f64(x);
  __syncthreads();  // red4 may still be read by the previous call
  if (lane_id() == 0) red4[wave_id()] = x;
  __syncthreads();
  return (red4[0] + red4[1]) + (red4[2] + red4[3]);
}

__global__ __launch_bounds__(256, 1) void k_sk_res(SkArgs a, SkDev d, ResGeom g, int first,
                                                   int count) {
  // K rows kResRR..kResRA-1 of the thread tile, column pairs as one 16-B word per lane
  __shared__ double2 klds[kResLR * (kResCA / 2) * 256];
  __shared__ double vsh[kResCols], ush[kResRows], colred[4][kResCols];
  __shared__ double red4[4], peer[kResMaxWg];
  __shared__ int peerf[kResMaxWg];
  __shared__ int sh_state;
  const int t = threadIdx.x, w = wave_id(), lane = lane_id();
  const int ra = t >> 4, cb = t & 15;
  const int wg = blockIdx.x, p = wg / g.Q, q = wg - (wg / g.Q) * g.Q;
  const unsigned nwg = (unsigned)(g.P * g.Q);
  const int r0 = p * g.R, c0 = q * g.Cb;
  const int nr = max(0, min(g.R, a.I - r0)), nc = max(0, min(g.Cb, a.J - c0));
  const int64_t J = a.J, I = a.I;
  double* rowpart = d.rowpart;  // [2][Q][I]
  double* colpart = d.colpart;  // [2][P][J]
  double* rowaux = d.rowaux;    // [2][P*Q][2]: err^2 of the column block, bad-v flag
  double* colaux = d.colaux;    // [2][P*Q]: bad-u flag of the row block
  // -- the K block (zeros outside the matrix) --
  double kr[kResRR][kResCA];
#pragma unroll
  for (int i = 0; i < kResRA; ++i) {
    const int lr = ra + 16 * i;
    const bool rok = lr < nr;
    const double* Kr = d.K + (int64_t)(r0 + (rok ? lr : 0)) * J + c0;
#pragma unroll
    for (int j = 0; j < kResCA; j += 2) {
      const int lc0 = cb + 16 * j, lc1 = lc0 + 16;
      const double k0 = rok && lc0 < nc ? Kr[lc0] : 0.0;
      const double k1 = rok && lc1 < nc ? Kr[lc1] : 0.0;
      if (i < kResRR) {
        kr[i][j] = k0;
        kr[i][j + 1] = k1;
      } else {
        klds[((i - kResRR) * (kResCA / 2) + j / 2) * 256 + t] = make_double2(k0, k1);
      }
    }
  }
  const double inva = t < nr ? 1.0 / a.a[r0 + t] : 0.0;  // row t of the block (step 3)
  const double bj = t < nc ? a.b[c0 + t] : 0.0;         // column t of the block (step 1)
  double vprev = t < nc ? d.v[(int64_t)((first + 1) & 1) * J + c0 + t] : 0.0;  // v_{first-1}
  // -- entry barrier: every workgroup reads ST_DONE before any can write it --
  if (t == 0) {
    const int64_t done = __hip_atomic_load(&d.st[ST_DONE], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    res_drain();
    const unsigned v = __hip_atomic_fetch_add((res_gu*)d.ecnt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    int st = done ? 1 : 0;
    if (!st) {
      const unsigned target = (v / nwg + 1) * nwg;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (res_ldu(d.ecnt) < target) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > g.spin) {
          st = 2;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    sh_state = st;
  }
  __syncthreads();
  if (sh_state) {
    if (sh_state == 2 && t == 0) res_timeout(d);
    return;
  }

  // column pass: colpart[par][p][c0 + c] = sum over the block's rows of K_rc u_r (ush), published
  // with the block's bad-u flag under epoch ep
  auto col_pass = [&](int par, unsigned ep, bool ufail) {
    double u[kResRA];
#pragma unroll
    for (int i = 0; i < kResRA; ++i) u[i] = ush[ra + 16 * i];
#pragma unroll
    for (int j = 0; j < kResCA; j += 2) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int i = 0; i < kResRA; ++i) {
        double k0, k1;
        if (i < kResRR) {
          k0 = kr[i][j];
          k1 = kr[i][j + 1];
        } else {
          const double2 kk = klds[((i - kResRR) * (kResCA / 2) + j / 2) * 256 + t];
          k0 = kk.x;
          k1 = kk.y;
        }
        s0 = fma(u[i], k0, s0);
        s1 = fma(u[i], k1, s1);
      }
      s0 += __shfl_xor(s0, 16, 64);
      s1 += __shfl_xor(s1, 16, 64);
      s0 += __shfl_xor(s0, 32, 64);
      s1 += __shfl_xor(s1, 32, 64);
      if (lane < 16) {
        colred[w][cb + 16 * j] = s0;
        colred[w][cb + 16 * (j + 1)] = s1;
      }
    }
    __syncthreads();
    if (t < nc)
      res_st(colpart + ((int64_t)par * g.P + p) * J + c0 + t,
             (colred[0][t] + colred[1][t]) + (colred[2][t] + colred[3][t]));
    if (t == 0) res_st(colaux + (int64_t)par * nwg + wg, ufail ? 1.0 : 0.0);
    res_drain();
    __syncthreads();
    if (t == 0) __hip_atomic_store((res_gu*)(d.cflag + wg), ep, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
  };

  if (first == 0) {  // K^T u_0, u_0 = 1 / I (ot_loss.py:39), published as iteration -1
    if (t < kResRows) ush[t] = t < nr ? 1.0 / (double)a.ig : 0.0;
    __syncthreads();
    col_pass(1, 1u, false);
  }
  for (int it = first; it < first + count; ++it) {
    const int cur = it & 1, prv = cur ^ 1;
    // 1. v_it from the column partials of iterate it-1 (wave 0 polls; then every load of the
    //    step -- the partials and the row blocks' bad-u flags -- goes out in one round trip)
    if (w == 0) {
      const bool ok = res_wait(d.cflag, q, g.Q, g.P, (unsigned)(it + 1), g.spin);
      if (lane == 0) sh_state = ok ? 0 : 2;
    }
    __syncthreads();
    if (sh_state) {
      if (t == 0) res_timeout(d);
      return;
    }
    double errp = 0.0, vj = 0.0;
    bool vfail = false;
    if (t < nc) {
      const double s = res_sum_strided(colpart + (int64_t)prv * g.P * J + c0 + t, J, g.P);
      const double tt = vprev * s - bj;  // err of iterate it-1 (ot_loss.py:65-66), s = K^T u_{it-1}
      errp = tt * tt;
      vj = bj / s;  // ot_loss.py:54
      vfail = s == 0.0 || vj != vj || isinf(vj);
    }
    vsh[t] = vj;
    if (w == 0) {
      bool uf = false;
      for (int k = lane; k < g.P; k += 64)
        uf |= res_ld(colaux + (int64_t)prv * nwg + k * g.Q + q) != 0.0;
      const bool any_uf = __any(uf);
      if (lane == 0) sh_state = any_uf ? 1 : 0;  // iteration it-1 broke on u (marked by its rows)
    }
    const double err2_blk = res_block_sum(errp, red4);  // barriers: vsh and sh_state published
    if (sh_state) return;
    const bool vfail_blk = __syncthreads_or(vfail);
    if (t < nc) {
      if (p == 0) d.v[(int64_t)cur * J + c0 + t] = vj;
      vprev = vj;
    }
    // 2. row partials over the block's columns
    double acc[kResRA];
#pragma unroll
    for (int i = 0; i < kResRA; ++i) acc[i] = 0.0;
#pragma unroll
    for (int j = 0; j < kResCA; j += 2) {
      const double v0 = vsh[cb + 16 * j], v1 = vsh[cb + 16 * (j + 1)];
#pragma unroll
      for (int i = 0; i < kResRA; ++i) {
        double k0, k1;
        if (i < kResRR) {
          k0 = kr[i][j];
          k1 = kr[i][j + 1];
        } else {
          const double2 kk = klds[((i - kResRR) * (kResCA / 2) + j / 2) * 256 + t];
          k0 = kk.x;
          k1 = kk.y;
        }
        acc[i] = fma(k0, v0, acc[i]);
        acc[i] = fma(k1, v1, acc[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < kResRA; ++i) {  // sum over the 16 lanes of a DPP row (same ra)
      double x = acc[i];
      x += mov_dpp_f64<0xB1>(x);
      x += mov_dpp_f64<0x4E>(x);
      x += mov_dpp_f64<0x141>(x);
      x += mov_dpp_f64<0x140>(x);
      const int lr = ra + 16 * i;
      if (cb == 0 && lr < nr) res_st(rowpart + ((int64_t)cur * g.Q + q) * I + r0 + lr, x);
    }
    if (t == 0) {
      res_st(rowaux + ((int64_t)cur * nwg + wg) * 2, err2_blk);
      res_st(rowaux + ((int64_t)cur * nwg + wg) * 2 + 1, vfail_blk ? 1.0 : 0.0);
    }
    res_drain();
    __syncthreads();
    if (t == 0) __hip_atomic_store((res_gu*)(d.rflag + wg), (unsigned)(it + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
    // 3. the row block's partials; the stop decisions of knopp_stop, identical everywhere
    if (w == 0) {
      const bool ok = res_wait(d.rflag, p * g.Q, 1, g.Q, (unsigned)(it + 1), g.spin);
      if (lane == 0) sh_state = ok ? 0 : 2;
    }
    __syncthreads();
    if (sh_state) {
      if (t == 0) res_timeout(d);
      return;
    }
    const double srow =
        t < nr ? res_sum_strided(rowpart + (int64_t)cur * g.Q * I + r0 + t, I, g.Q) : 0.0;
    if (w == 0) {
      for (int k = lane; k < g.Q; k += 64) {
        const double* ax = rowaux + ((int64_t)cur * nwg + p * g.Q + k) * 2;
        peer[k] = res_ld(ax);
        peerf[k] = res_ld(ax + 1) != 0.0;
      }
      if (lane == 0) {
        double e2 = 0.0;
        bool vf = false;
        int st = 0;
        for (int k = 0; k < g.Q; ++k) {  // column-block order: every workgroup the same sum
          vf |= peerf[k] != 0;
          e2 += peer[k];
        }
        const int prev = it - 1;
        if (prev >= 0 && prev % 10 == 0) {
          const double err = sqrt(e2);
          if (wg == 0) d.sd[SD_ERR] = err;
          if (!(err > d.sd[SD_TOL])) {
            st = 1;
            if (wg == 0) mark_done(d.st, prev + 1, 1, prev & 1);
          }
        }
        if (!st && vf) {
          st = 1;
          if (wg == 0) mark_done(d.st, it, 2, (it + 1) & 1);
        }
        sh_state = st;
      }
    }
    __syncthreads();
    if (sh_state) return;
    bool ufail = false;
    if (t < kResRows) {
      double u = 0.0;
      if (t < nr) {
        u = 1.0 / (inva * srow);  // u = 1 / (Kp v), Kp = (1/a) K   (ot_loss.py:45, :55)
        ufail = u != u || isinf(u);
        if (q == 0) d.u[(int64_t)cur * I + r0 + t] = u;
      }
      ush[t] = u;
    }
    const bool ufail_blk = __syncthreads_or(ufail);
    if (ufail_blk && t == 0) mark_done(d.st, it, 2, (it + 1) & 1);  // every later step stops
    // 4. column partials of K^T u_it for iteration it + 1
    col_pass(cur, (unsigned)(it + 2), ufail_blk);
  }
}

// the on-chip path serves KNOPP (variant 0, unsharded) when the blocks fit the device's CUs
// (flag GNNEA_SK_NO_ONCHIP disables it: the host's retry after a timeout, and A/B measurements)
static int res_num_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  return n;
}

static bool res_applies(const gnnea_sinkhorn* p) {
  if (p->mode != GNNEA_SK_KNOPP || (p->variant != 0 && p->variant != GNNEA_SK_AUTO) ||
      p->J > kMaxJ)
    return false;
  if (p->flags & GNNEA_SK_NO_ONCHIP) return false;
  const ResGeom g = res_geom(p->I, p->J);
  return g.ok && g.P * g.Q <= res_num_cus();
}

static int res_launch(const gnnea_sinkhorn* p, int first, int count, hipStream_t s) {
  SkArgs a = sk_args(p);
  SkDev d = sk_dev(p);
  ResGeom g = res_geom(p->I, p->J);
  // GNNEA_SK_DEBUG_SPIN: every wait's bound is 0 ticks, so a workgroup that finds a peer not yet
  // arrived times out at once -- the timeout path (ST_TIMEOUT, the host's re-solve on the sweep
  // path) exercised on the device by the tests
  if (p->flags & GNNEA_SK_DEBUG_SPIN) g.spin = 0;
  // a plain launch of at most one workgroup per CU (res_applies).  Not hipLaunchCooperativeKernel:
  // the HIP runtime then keeps a dedicated cooperative queue whose teardown at process exit
  // crashed inside libhsa-runtime64 under rocprofv3's kernel tracing (the queue destroyed after
  // the tool's finalisation).  Co-residency is not guaranteed by a plain launch when another
  // stream holds CUs: every inter-workgroup wait is bounded (kResSpinTicks), a timed-out solve
  // sets GNNEA_SK_ST_TIMEOUT and the host solves it again on the sweep path (gnnea/sinkhorn.py).
  hipLaunchKernelGGL(k_sk_res, dim3(g.P * g.Q), dim3(256), 0, s, a, d, g, first, count);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int sk_iter_t(const gnnea_sinkhorn* p, int first, int count, hipStream_t s) {
  const SkArgs a = sk_args(p);
  const SkDev d = sk_dev(p);
  const dim3 grow(div_up(p->I, 4)), gfin(a.nfin);
  const bool knopp = p->mode == GNNEA_SK_KNOPP;
  if (res_applies(p)) return res_launch(p, first, count, s);
  for (int it = first; it < first + count; ++it) {
    const int cur = it & 1, prev = cur ^ 1;
    if (knopp) {
      // partials of K^T u_{it-1} come from the previous sweep (or the init column pass)
      hipLaunchKernelGGL(k_sk_colfin<FIN_KNOPP>, gfin, dim3(1024), 0, s, a, d, prev, cur,
                         nullptr);
      launch_sweep<true, true>(a, d, it, cur, cur, nullptr, 1, s);  // u_it and K^T u_it
    } else {
      launch_sweep<false, true>(a, d, it, prev, cur, nullptr, 1, s);  // a_it and K^T a_it
      hipLaunchKernelGGL(k_sk_colfin<FIN_STAB>, gfin, dim3(1024), 0, s, a, d, prev, cur,
                         nullptr);
      hipLaunchKernelGGL(k_sk_absorb_vec, dim3(div_up(p->I > p->J ? p->I : p->J, 256)),
                         dim3(256), 0, s, a, d, it, cur, p->max_iter);
      hipLaunchKernelGGL((k_sk_kbuild<T, false>), grow, dim3(256), 0, s, (const T*)p->C, a, d,
                         it, p->max_iter, 0);
      hipLaunchKernelGGL(k_sk_absorb_final, dim3(1), dim3(1024), 0, s, a, d, it, cur,
                         p->max_iter, 0);
    }
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

// ---------------------------------------------------------------------------------------- //
// §8e, row-sharded KNOPP in the scaling form (the dispatch of gnnea_sinkhorn_shard_*,
// sinkhorn_shard.hip, for J <= kMaxJ): every rank keeps the fp64 K of its rows resident and runs
// the same fused sweep; the sweep's column partials of K^T u are summed over the rank's
// workgroups in order (k_sk_shard_combine) into one J-row, the rows of all ranks are all-gathered
// by the caller and summed in rank order (k_sk_shard_colfin), so v and every stop decision are
// bit-identical on all ranks.  A bad u (inf / NaN) is flagged (ST_UFAIL), travels with the
// rank's row and ends the loop one iteration later on every rank, reverting to iterate it-2 (the
// merge then leaves v's slot untouched).  Pair row: J sums, then the flag at J (J + 2 doubles).
// ---------------------------------------------------------------------------------------- //
__global__ __launch_bounds__(256) void k_sk_shard_combine(SkArgs a, SkDev d,
                                                          double* __restrict__ pair) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < a.J) {
    double s0 = 0.0, s1 = 0.0;
    int q = 0;
    for (; q + 2 <= a.ns; q += 2) {
      s0 += d.part[(int64_t)q * a.J + j];
      s1 += d.part[(int64_t)(q + 1) * a.J + j];
    }
    if (q < a.ns) s0 += d.part[(int64_t)q * a.J + j];
    pair[j] = s0 + s1;
  }
  if (j == 0) {
    pair[a.J] = (!d.st[ST_DONE] && d.st[ST_UFAIL]) ? 1.0 : 0.0;
    pair[a.J + 1] = 0.0;
  }
}

__device__ __forceinline__ bool shard_ufail(const double* __restrict__ pairs, int W,
                                            int64_t stride, int J) {
  bool u = false;
  for (int r = 0; r < W; ++r) u |= pairs[(int64_t)r * stride + J] != 0.0;
  return u;
}

// v_it from the W gathered rows (rank order), err^2 partials of iterate it-1, K^T u == 0 / bad v
// flags (read by the sweep's knopp_stop exactly as in the unsharded loop)
__global__ __launch_bounds__(256) void k_sk_shard_colfin(SkArgs a, SkDev d,
                                                         const double* __restrict__ pairs, int W,
                                                         int64_t stride, int it) {
  if (d.st[ST_DONE]) return;
  if (shard_ufail(pairs, W, stride, a.J)) {  // iteration it-1 broke on u: keep iterate it-2
    if (blockIdx.x == 0 && threadIdx.x == 0) mark_done(d.st, it - 1, 2, it & 1);
    return;
  }
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int cur = it & 1, prev = cur ^ 1;
  double errp = 0.0;
  bool fail = false;
  if (j < a.J) {
    double s = 0.0;
    for (int r = 0; r < W; ++r) s += pairs[(int64_t)r * stride + j];
    const double t = d.v[(int64_t)prev * a.J + j] * s - a.b[j];  // (utils/ot_loss.py:65-66)
    errp = t * t;
    const double vj = a.b[j] / s;  // (:54)
    fail = s == 0.0 || vj != vj || isinf(vj);
    d.v[(int64_t)cur * a.J + j] = vj;
  }
  errp = wave_sum(errp);
  __shared__ double red[4];
  if (lane_id() == 0) red[wave_id()] = errp;
  if (__any(fail) && lane_id() == 0) atomicOr((unsigned long long*)&d.st[ST_FAIL], 1ull);
  __syncthreads();
  if (threadIdx.x == 0) {
    d.errpart[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    if (blockIdx.x == 0) d.st[ST_UFAIL] = 0;  // consumed (it travelled in the gathered rows)
  }
}

namespace skscale {

bool shard_ok(const gnnea_sinkhorn* p) {  // (GNNEA_SK_AUTO: the scaling form when sharded)
  return p && (p->variant == 0 || p->variant == GNNEA_SK_AUTO) && p->mode == GNNEA_SK_KNOPP &&
         p->J <= kMaxJ && sk_valid(p);
}
int64_t shard_ws_bytes(int I, int J) {
  if (J > kMaxJ) return 0;
  const SkWs w = sk_plan(I, J);
  // the colfin's err partials (one per 256 columns) must fit the errpart slots (one per 16)
  return w.total;
}
int shard_pair_len(const gnnea_sinkhorn* p) { return p->J + 2; }

static SkArgs shard_args(const gnnea_sinkhorn* p, int I_global) {
  SkArgs a = sk_args(p);
  a.ig = I_global;
  a.shard = 1;
  return a;
}

int shard_init(const gnnea_sinkhorn* p, int I_global, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const SkArgs a = shard_args(p, I_global);
  const SkDev d = sk_dev(p);
  const int n = p->I > p->J ? p->I : p->J;
  hipLaunchKernelGGL(k_sk_init, dim3(div_up(n > 32 ? n : 32, 256)), dim3(256), 0, s, a, d,
                     p->tol);
  // the err partials the sharded colfin does not write (slots past ceil(J / 256)) stay zero
  if (hipMemsetAsync(d.errpart, 0, 8 * (size_t)a.nfin, s) != hipSuccess) return GNNEA_EINVAL;
  const dim3 grow(div_up(p->I, 4));
  if (p->c_dtype == GNNEA_F32)
    hipLaunchKernelGGL((k_sk_kbuild<float, true>), grow, dim3(256), 0, s, (const float*)p->C, a,
                       d, 0, p->max_iter, 1);
  else
    hipLaunchKernelGGL((k_sk_kbuild<double, true>), grow, dim3(256), 0, s, (const double*)p->C,
                       a, d, 0, p->max_iter, 1);
  launch_sweep<true, false>(a, d, 0, 1, 1, d.u + p->I, 0, s);  // K^T u0 partials (u0 in slot 1)
  GNNEA_LAUNCH_CHECK();
  return 0;
}

int shard_colpart(const gnnea_sinkhorn* p, double* pair, void* stream) {
  const SkArgs a = shard_args(p, p->I);
  hipLaunchKernelGGL(k_sk_shard_combine, dim3(div_up(p->J, 256)), dim3(256), 0,
                     (hipStream_t)stream, a, sk_dev(p), pair);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

int shard_step(const gnnea_sinkhorn* p, int it, const double* pairs, int W, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const SkArgs a = shard_args(p, p->I);
  const SkDev d = sk_dev(p);
  hipLaunchKernelGGL(k_sk_shard_colfin, dim3(div_up(p->J, 256)), dim3(256), 0, s, a, d, pairs, W,
                     (int64_t)shard_pair_len(p), it);
  const int cur = it & 1;
  launch_sweep<true, true>(a, d, it, cur, cur, nullptr, 1, s);  // u_it and K^T u_it partials
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// after the close step (the status block holds the final slot): plan rows, row sums, this
// rank's sum P.M (loss_part[0]) and column sums (col_part)
int shard_finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype, int64_t ldp,
                 double* row_sum, double* loss_part, double* col_part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const SkArgs a = shard_args(p, p->I);
  const SkDev d = sk_dev(p);
  const dim3 grow(div_up(p->I, 4));
  double* xcol = d.pu;
#define GNNEA_PLAN(T, PT)                                                                   \
  hipLaunchKernelGGL((k_sk_plan<T, PT>), grow, dim3(256), 0, s, (const T*)p->C, a, d,      \
                     p->iters_run, (PT*)plan, ldp, row_sum, xcol)
  if (p->c_dtype == GNNEA_F32) {
    if (plan_dtype == GNNEA_F32) GNNEA_PLAN(float, float);
    else GNNEA_PLAN(float, double);
  } else {
    if (plan_dtype == GNNEA_F32) GNNEA_PLAN(double, float);
    else GNNEA_PLAN(double, double);
  }
#undef GNNEA_PLAN
  hipLaunchKernelGGL(k_sk_loss, dim3(1), dim3(1024), 0, s, a, d, p->iters_run);
  GNNEA_LAUNCH_CHECK();
  if (hipMemcpyAsync(loss_part, d.sd + SD_LOSS, 8, hipMemcpyDeviceToDevice, s) != hipSuccess)
    return GNNEA_EINVAL;
  if (col_part) {
    launch_sweep<true, false>(a, d, 0, 0, 0, xcol, 0, s);
    hipLaunchKernelGGL(k_sk_colfin<FIN_SUM>, dim3(a.nfin), dim3(1024), 0, s, a, d, 0, 0,
                       col_part);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace skscale

// the memory-lean log-domain path (sinkhorn_log.hip)
namespace sklog {
int64_t ws_bytes(int I, int J);
int init(const gnnea_sinkhorn* p, void* stream);
int iterate(const gnnea_sinkhorn* p, int first, int count, void* stream);
int finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype, int64_t ldp, double* row_sum,
           double* col_sum, void* stream);
bool fused_ok(const gnnea_sinkhorn* p);
}  // namespace sklog

// variant 1, or J beyond the sweep's register tiles: log-domain passes, no I x J workspace;
// GNNEA_SK_AUTO: KNOPP that the on-chip kernel cannot hold takes the fused log-domain sweep (one
// pass over C per iteration against the resident K's I*J*8 bytes per iteration, and no K build)
static bool use_log(const gnnea_sinkhorn* p) {
  if (p->variant == 1 || p->J > kMaxJ) return true;
  return p->variant == GNNEA_SK_AUTO && p->mode == GNNEA_SK_KNOPP && sk_valid(p) &&
         !res_applies(p) && sklog::fused_ok(p);
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_sinkhorn_ws_bytes(int I, int J) {
  if (I < 1 || J < 1) return GNNEA_EINVAL;
  const int64_t lg = sklog::ws_bytes(I, J);
  if (J > kMaxJ) return lg;
  const int64_t sc = sk_plan(I, J).total;
  return sc > lg ? sc : lg;
}

extern "C" int gnnea_sinkhorn_path(const gnnea_sinkhorn* p) {
  if (p && use_log(p)) return GNNEA_SK_PATH_LOG;
  if (!sk_valid(p)) return GNNEA_EINVAL;
  return res_applies(p) ? GNNEA_SK_PATH_ONCHIP : GNNEA_SK_PATH_SWEEP;
}

extern "C" int gnnea_sinkhorn_init(const gnnea_sinkhorn* p, void* stream) {
  if (p && use_log(p)) return sklog::init(p, stream);
  if (!sk_valid(p)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const SkArgs a = sk_args(p);
  const SkDev d = sk_dev(p);
  const int n = p->I > p->J ? p->I : p->J;
  hipLaunchKernelGGL(k_sk_init, dim3(div_up(n > 32 ? n : 32, 256)), dim3(256), 0, s, a, d,
                     p->tol);
  GNNEA_LAUNCH_CHECK();
  const dim3 grow(div_up(p->I, 4));
  const bool f32 = p->c_dtype == GNNEA_F32;
  if (p->mode == GNNEA_SK_KNOPP) {
    if (f32)
      hipLaunchKernelGGL((k_sk_kbuild<float, true>), grow, dim3(256), 0, s, (const float*)p->C,
                         a, d, 0, p->max_iter, 1);
    else
      hipLaunchKernelGGL((k_sk_kbuild<double, true>), grow, dim3(256), 0, s,
                         (const double*)p->C, a, d, 0, p->max_iter, 1);
    if (res_applies(p)) {  // k_sk_res computes K^T u0 itself; its flags start at 0
      if (hipMemsetAsync(d.rflag, 0, kResFlagBytes, s) != hipSuccess) return GNNEA_EINVAL;
    } else {
      launch_sweep<true, false>(a, d, 0, 1, 1, d.u + p->I, 0, s);  // K^T u0, u0 = 1/I (slot 1)
    }
  } else {  // K0 with zero potentials and transport = sum K0 . C   (sinkhorn_loss.py:193-195)
    if (f32)
      hipLaunchKernelGGL((k_sk_kbuild<float, false>), grow, dim3(256), 0, s, (const float*)p->C,
                         a, d, 0, p->max_iter, 1);
    else
      hipLaunchKernelGGL((k_sk_kbuild<double, false>), grow, dim3(256), 0, s,
                         (const double*)p->C, a, d, 0, p->max_iter, 1);
    hipLaunchKernelGGL(k_sk_absorb_final, dim3(1), dim3(1024), 0, s, a, d, 0, 0, p->max_iter, 1);
  }
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_sinkhorn_iterate(const gnnea_sinkhorn* p, int first, int count,
                                      void* stream) {
  if (p && use_log(p)) return sklog::iterate(p, first, count, stream);
  if (!sk_valid(p) || first < 0 || count < 1) return GNNEA_EINVAL;
  if (p->c_dtype == GNNEA_F32) return sk_iter_t<float>(p, first, count, (hipStream_t)stream);
  return sk_iter_t<double>(p, first, count, (hipStream_t)stream);
}

extern "C" int gnnea_sinkhorn_finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype,
                                     int64_t ldp, double* row_sum, double* col_sum,
                                     void* stream) {
  if (p && use_log(p)) return sklog::finish(p, plan, plan_dtype, ldp, row_sum, col_sum, stream);
  if (!sk_valid(p)) return GNNEA_EINVAL;
  if (plan && plan_dtype != GNNEA_F32 && plan_dtype != GNNEA_F64) return GNNEA_EINVAL;
  if (plan && ldp < p->J) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const SkArgs a = sk_args(p);
  const SkDev d = sk_dev(p);
  const dim3 grow(div_up(p->I, 4));
  double* xcol = d.pu;  // free after the loop: column-sum weights (u or 1) for the colpart
#define GNNEA_PLAN(T, PT)                                                                   \
  hipLaunchKernelGGL((k_sk_plan<T, PT>), grow, dim3(256), 0, s, (const T*)p->C, a, d,      \
                     p->iters_run, (PT*)plan, ldp, row_sum, xcol)
  if (p->c_dtype == GNNEA_F32) {
    if (plan_dtype == GNNEA_F32) GNNEA_PLAN(float, float);
    else GNNEA_PLAN(float, double);
  } else {
    if (plan_dtype == GNNEA_F32) GNNEA_PLAN(double, float);
    else GNNEA_PLAN(double, double);
  }
#undef GNNEA_PLAN
  GNNEA_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sk_loss, dim3(1), dim3(1024), 0, s, a, d, p->iters_run);
  GNNEA_LAUNCH_CHECK();
  if (col_sum) {
    launch_sweep<true, false>(a, d, 0, 0, 0, xcol, 0, s);
    hipLaunchKernelGGL(k_sk_colfin<FIN_SUM>, dim3(a.nfin), dim3(1024), 0, s, a, d, 0, 0,
                       col_sum);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}
