// a9-a12. Fused log-domain Sinkhorn (fp64 arithmetic, fp32 or fp64 cost storage): the
// memory-lean path of gnnea_sinkhorn_* (variant 1, and any J beyond the sweep's register tiles),
// keeping no I x J state -- every pass recomputes its terms from C with fp64 exp.  Dispatched from
// sinkhorn.hip; the status block is shared with the scaling-form path.
//
// Reference semantics restated in potentials:
//   KNOPP (utils/ot_loss.py:5-76), f = log u, g = log v:
//       g_j = log b_j - LSE_i(f_i - M_ij/reg)      (v = b / K^T u,   :53-54)
//       f_i = log a_i - LSE_j(g_j - M_ij/reg)      (u = 1 / (K/a) v, :55)
//     K_ij = exp_f64(-M_ij/reg) underflows to 0 below -745.13 in fp64: such terms are dropped,
//     K^T u == 0 (column LSE below ln(DBL_TRUE_MIN)) or inf/NaN u, v break the loop with the
//     previous iterate (:57-62); err = ||v (K^T u) - b||_2 every 10th iteration (:64-66).
//   STAB / GEN / RELAX (SinkhornOT/sinkhorn_loss.py:159-356), potentials in units of eps,
//   ua / va = absorbed potentials u/eps, v/eps, f / g = full potentials (u + eps log a)/eps:
//       log s_i = LSE_j( min(ua_i + va_j - C_ij/eps, ln 1e30) + g_j - va_j )   (K b, clamped K)
//       f_i = ua_i + min(p_row (log mu_i - log s_i), ln 1e30)                  (a = clamp((mu/s)^p))
//     and symmetrically for g; absorption (ii%10==0, max(a|b) > 1e20, last iteration) sets
//     ua = f, va = g and evaluates transport = sum K.C for the relative-tolerance break.
// One iteration = row pass (one wave per row, coalesced 64-wide column sweep, chunked online
// LSE with 16 loads in flight per lane) + column pass fused with the column update (16 columns
// x 64 row groups per 1024-thread workgroup, merged through LDS).  Both passes are latency- and
// fp64-exp-bound at B = 3000 (C is L2 / Infinity-Cache resident).  A device status block gates
// every kernel so iterations after the stop condition are no-ops.
#include "common.h"

namespace gnnea {
namespace sklog {

constexpr double kLn1e20 = 46.051701859880914;   // log(1e20)  (sinkhorn_loss.py:11 big)
constexpr double kLn1e30 = 69.07755278982137;    // log(1e30)  (sinkhorn_loss.py:12 huge)
constexpr double kExpUnderflow = -745.1332191019412;  // exp_f64(x) == 0 in fp64 for x below
constexpr double kLnTrueMin = -744.4400719213812;     // log(DBL_TRUE_MIN)
constexpr double kExpOverflow = 709.782712893384;     // exp_f64(x) == inf above

struct SkWs {
  int64_t f, g, ua, va, rowbuf, errpart, part_m, part_s, la, lb, fs, gs, fpart, ftab, fbrows, fbcnt, total;
  int ncb, nsf;
};

static inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

constexpr int kMaxSplits = 16;  // row splits of the partial column pass

// fused KNOPP sweep (k_lsk_sweep): waves per workgroup, exp table size, widest J, workgroups
constexpr int kFW = 8, kFTab = 2048, kFMaxJ = 64 * kFW * 32, kFWgTarget = 256;
static int fused_rpw(int I) { return (I + kFWgTarget - 1) / kFWgTarget; }
static int fused_wgs(int I) { return (I + fused_rpw(I) - 1) / fused_rpw(I); }

static SkWs sk_plan(int I, int J) {
  SkWs w;
  int64_t o = GNNEA_SK_STATUS_BYTES;
  w.f = o; o = al256(o + 2 * 8ll * I);
  w.g = o; o = al256(o + 2 * 8ll * J);
  w.ua = o; o = al256(o + 8ll * I);
  w.va = o; o = al256(o + 8ll * J);
  w.rowbuf = o; o = al256(o + 8ll * I);
  w.ncb = (J + 7) / 8;  // errpart slots: enough for the narrowest column workgroup (8 cols)
  w.errpart = o; o = al256(o + 8ll * w.ncb);
  w.part_m = o; o = al256(o + 8ll * kMaxSplits * J);
  w.part_s = o; o = al256(o + 8ll * kMaxSplits * J);
  w.la = o; o = al256(o + 8ll * I);
  w.lb = o; o = al256(o + 8ll * J);
  w.fs = o; o = al256(o + 2 * 8ll * I);  // KNOPP fast path: f, g in units of ln2 / 64
  w.gs = o; o = al256(o + 2 * 8ll * J);
  // fused KNOPP sweep (J <= kFMaxJ): column partials of its workgroups and the 2^(j/2048) table
  w.nsf = fused_wgs(I);
  w.fpart = o; o = al256(o + 8ll * w.nsf * J);
  w.ftab = o; o = al256(o + 8ll * kFTab);
  w.fbrows = o; o = al256(o + 4ll * w.nsf * fused_rpw(I));  // rows listed for k_lsk_fix
  w.fbcnt = o; o = al256(o + 4ll * w.nsf);
  w.total = o;
  return w;
}

struct SkDev {
  int64_t* st;   // status ints
  double* sd;    // status doubles (sd[8] ...)
  double *f, *g, *ua, *va, *rowbuf, *errpart, *pm, *ps;
  double *fs, *gs;  // f, g scaled by 64 / ln 2 (KNOPP fast path)
  double *fpart, *ftab;  // fused KNOPP sweep: column partials [nsf][J], 2^(j/2048) table
  int *fbrows, *fbcnt;   // rows each sweep workgroup left for the exact update (k_lsk_fix)
  int ncb;  // errpart slots written by the column pass of the active variant
};

static SkDev sk_dev(const gnnea_sinkhorn* p) {
  SkWs w = sk_plan(p->I, p->J);
  char* b = (char*)p->ws;
  SkDev d;
  d.st = (int64_t*)b;
  d.sd = (double*)b;
  d.f = (double*)(b + w.f);
  d.g = (double*)(b + w.g);
  d.ua = (double*)(b + w.ua);
  d.va = (double*)(b + w.va);
  d.rowbuf = (double*)(b + w.rowbuf);
  d.errpart = (double*)(b + w.errpart);
  d.pm = (double*)(b + w.part_m);
  d.ps = (double*)(b + w.part_s);
  d.fs = (double*)(b + w.fs);
  d.gs = (double*)(b + w.gs);
  d.fpart = (double*)(b + w.fpart);
  d.ftab = (double*)(b + w.ftab);
  d.fbrows = (int*)(b + w.fbrows);
  d.fbcnt = (int*)(b + w.fbcnt);
  d.ncb = w.ncb;
  return d;
}

enum { ST_DONE = 0, ST_ITERS = 1, ST_REASON = 2, ST_SLOT = 3, ST_BIG = 4, ST_FAIL = 5 };
// set by init when C holds a non-finite value: the KNOPP passes then keep the NaN-propagating
// natural-unit terms instead of the scaled fast path (whose clamp would hide a NaN)
enum { ST_CNAN = 17 };
// set by init when some K entry underflows (-C / reg < kExpUnderflow: the reference's exp gives
// 0 there): only then does the fused sweep carry the per-element mask (a compare and a select)
enum { ST_CMASK = 18 };
enum { SD_ERR = GNNEA_SK_SD_ERR, SD_TPREV = GNNEA_SK_SD_TPREV, SD_LOSS = GNNEA_SK_SD_LOSS,
       SD_TOL = GNNEA_SK_SD_TOL, SD_TNEW = GNNEA_SK_SD_TNEW };

template <typename T>
__device__ __forceinline__ double ld_c(const T* C, int64_t idx) {
  return (double)C[idx];
}

// online log-sum-exp with one exp per element
struct Lse {
  double m, s;
  __device__ __forceinline__ void init() { m = -INFINITY; s = 0.0; }
  __device__ __forceinline__ void add(double x) {
    if (x == -INFINITY) return;
    if (x > m) {
      s = s * exp_f64(m - x) + 1.0;
      m = x;
    } else {
      s += exp_f64(x - m);
    }
  }
  __device__ __forceinline__ void merge(double m2, double s2) {
    if (m2 == -INFINITY) return;
    if (m == -INFINITY) { m = m2; s = s2; return; }
    if (m2 > m) { s = s * exp_f64(m - m2) + s2; m = m2; }
    else s += s2 * exp_f64(m2 - m);
  }
  __device__ __forceinline__ double value() const { return m == -INFINITY ? -INFINITY : m + log(s); }
};

__device__ __forceinline__ Lse wave_lse(Lse l) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double m2 = __shfl_xor(l.m, o, 64);
    const double s2 = __shfl_xor(l.s, o, 64);
    l.merge(m2, s2);
  }
  return l;
}

struct SkArgs {
  int mode, I, J;
  int64_t ldc;
  double inv_eps, p_row, p_col, kclamp;  // kclamp: ln 1e30 for STAB modes, +inf for KNOPP
  const double *la, *lb;
  const double *wa, *wb;  // the weights a, b themselves (the fused sweep's u_new / u_old, err)
};

__device__ __forceinline__ void mark_done(int64_t* st, int64_t iters, int64_t reason,
                                          int64_t slot) {
  if (atomicCAS((unsigned long long*)&st[ST_DONE], 0ull, 1ull) == 0ull) {
    st[ST_ITERS] = iters;
    st[ST_REASON] = reason;
    st[ST_SLOT] = slot;
  }
}

// exp(x) of the LSE terms (x <= 0, -inf for a masked term, NaN kept NaN) by the 64-entry table
// 2^(j/64) (exactly rounded, in LDS: lse_table) and a degree-5 polynomial on |r| <= ln2 / 128:
//   x = (64 t' + j) ln2/64 + r,  exp(x) = 2^t' * 2^(j/64) * (1 + (e^r - 1)),
// truncation r^6 / 720 < 3.5e-17, about 1 ulp in all -- 14 fp64 operations against exp_f64's 19,
// the inner-loop cost of both LSE passes (2 I J exponentials per iteration).
__device__ const double kExp2Tab64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951};

struct LseTable {
  double t[64];
};
// every thread of the workgroup calls it (a barrier inside)
__device__ __forceinline__ const double* lse_table(LseTable& sh) {
  if (threadIdx.x < 64) sh.t[threadIdx.x] = kExp2Tab64[threadIdx.x];
  __syncthreads();
  return sh.t;
}

__device__ __forceinline__ double exp_tab(double x, const double* __restrict__ tab) {
  constexpr double kInvL = 92.33248261689366;         // 64 / ln 2
  constexpr double kLHi = 0.010830424696249145;       // ln 2 / 64, high part
  constexpr double kLLo = 3.623510646634843e-19;      // ln 2 / 64 - kLHi
  const double xc = fmax(x, -1.0e4);  // -inf -> -1e4: 2^-14427 underflows to 0 below
  const double t = __builtin_rint(xc * kInvL);
  double r = __builtin_fma(-t, kLHi, xc);
  r = __builtin_fma(-t, kLLo, r);
  const int ti = (int)t;
  double p = __builtin_fma(r, 1.0 / 120.0, 1.0 / 24.0);
  p = __builtin_fma(p, r, 1.0 / 6.0);
  p = __builtin_fma(p, r, 0.5);
  p = __builtin_fma(p, r, 1.0);
  p *= r;  // e^r - 1
  const double tj = tab[ti & 63];
  const double y = __builtin_ldexp(__builtin_fma(tj, p, tj), ti >> 6);
  return x != x ? x : y;
}

// Chunked, branch-free online LSE: per chunk of CH values one rescale exp + one exp per value
// (a per-element "if (x > m)" diverges across lanes and costs two exps per element).
template <int CH>
__device__ __forceinline__ void lse_chunk(Lse& l, const double (&x)[CH],
                                          const double* __restrict__ tab) {
  double cm = x[0];
#pragma unroll
  for (int k = 1; k < CH; ++k) cm = fmax(cm, x[k]);
  if (cm == -INFINITY) return;  // whole chunk masked (K == 0)
  const double nm = fmax(l.m, cm);
  double acc = l.m == -INFINITY ? 0.0 : l.s * exp_tab(l.m - nm, tab);
#pragma unroll
  for (int k = 0; k < CH; ++k) acc += exp_tab(x[k] - nm, tab);  // exp_tab(-inf) == 0
  l.m = nm;
  l.s = acc;
}

// KNOPP fast path: terms in units of ln2 / 64 (x~ = x * 64 / ln 2), so the table exponential
// needs no range-reduction multiply: t = rint(x~), r = x~ - t (exact), 2^(x~/64) =
// 2^(t >> 6) * 2^((t & 63) / 64) * e^(r ln2/64), |r ln2 / 64| <= ln2 / 128 as in exp_tab.  A term
// x~ = fma(k, 64 / ln 2, g~) replaces k + g: 13 VALU per exponential against exp_tab's 17 (NaN
// guard and reduction multiply gone; C was checked finite by init, ST_CNAN).
constexpr double kScale = 92.33248261689366;     // 64 / ln 2
constexpr double kUnscale = 0.010830424696249145;  // ln 2 / 64
__device__ __forceinline__ double exp2t(double xs, const double* __restrict__ tab) {
  constexpr double c1 = 0.010830424696249145, c2 = 5.86490495505617e-05,
                   c3 = 2.1173137155464776e-07, c4 = 5.732851688640402e-10,
                   c5 = 1.2417843701716925e-12;  // (ln2/64)^k / k!
  const double xc = fmax(xs, -1.0e6);  // -inf -> 2^-15625: 0 below
  const double t = __builtin_rint(xc);
  const double r = xc - t;
  const int ti = (int)t;
  double p = __builtin_fma(r, c5, c4);
  p = __builtin_fma(p, r, c3);
  p = __builtin_fma(p, r, c2);
  p = __builtin_fma(p, r, c1);
  p *= r;  // e^(r ln2/64) - 1
  const double tj = tab[ti & 63];
  return __builtin_ldexp(__builtin_fma(tj, p, tj), ti >> 6);
}

// lse_chunk on scaled terms (l.m scaled too until lse_unscale)
template <int CH>
__device__ __forceinline__ void lse2_chunk(Lse& l, const double (&x)[CH],
                                           const double* __restrict__ tab) {
  double cm = x[0];
#pragma unroll
  for (int k = 1; k < CH; ++k) cm = fmax(cm, x[k]);
  if (cm == -INFINITY) return;
  const double nm = fmax(l.m, cm);
  double acc = l.m == -INFINITY ? 0.0 : l.s * exp2t(l.m - nm, tab);
#pragma unroll
  for (int k = 0; k < CH; ++k) acc += exp2t(x[k] - nm, tab);
  l.m = nm;
  l.s = acc;
}
__device__ __forceinline__ void lse_unscale(Lse& l) {
  if (l.m != -INFINITY) l.m *= kUnscale;
}

// KNOPP scaled term: -inf where K_ij underflows (the same test on k as sk_term)
__device__ __forceinline__ double sk_term_s(double c, double inv_eps, double pot_s) {
  const double k = -c * inv_eps;
  return k < kExpUnderflow ? -INFINITY : __builtin_fma(k, kScale, pot_s);
}

// logit of the reference's K_ij * scaling: -inf where K_ij underflows to 0 in fp64
template <bool KNOPP>
__device__ __forceinline__ double sk_term(double ua, double va, double c, double inv_eps,
                                          double kclamp, double pot_minus_abs) {
  const double k = KNOPP ? -c * inv_eps : ua + va - c * inv_eps;
  if (k < kExpUnderflow) return -INFINITY;
  return (KNOPP ? k : fmin(k, kclamp)) + pot_minus_abs;
}

// KNOPP loop decisions, in the reference's order (utils/ot_loss.py:50-72): the err test of
// iterate it-1 (when (it-1)%10 == 0), then the K^T u == 0 / inf / NaN break of iteration it
// flagged by this iteration's column pass.  Evaluated by wave 0 of every row workgroup (all
// take the same decision); returns true when the workgroup must stop.
__device__ __forceinline__ bool knopp_stop(SkDev& d, int it) {
  __shared__ int stop;
  const int lane = lane_id();
  if (wave_id() == 0) {
    const int prev = it - 1;
    int st = 0;
    if (prev >= 0 && prev % 10 == 0) {
      double e = 0.0;
      for (int b = lane; b < d.ncb; b += 64) e += d.errpart[b];
      const double err = sqrt(wave_sum(e));
      if (!(err > d.sd[SD_TOL])) st = 1;  // stopThr: the loop runs while err > stopThr
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

__device__ __forceinline__ void finish_row(const SkArgs& a, SkDev& d, int i, Lse l, int it,
                                           int slot_out, double uai, bool knopp) {
  const double ls = l.value();
  double la = a.p_row * (a.la[i] - ls);
  if (knopp) {
    d.f[(int64_t)slot_out * a.I + i] = la;  // u = 1/(Kp v)
    d.fs[(int64_t)slot_out * a.I + i] = la * kScale;
    if (!(la <= kExpOverflow)) mark_done(d.st, it, 2, (it + 1) & 1);  // u inf / NaN
  } else {
    if (la > kLn1e30) la = kLn1e30;  // a = clamp(., 0, 1e30)
    if (la > kLn1e20) atomicOr((unsigned long long*)&d.st[ST_BIG], 1ull);
    d.f[(int64_t)slot_out * a.I + i] = uai + la;  // F = u + eps log a
  }
}

// Row pass: f_out_i from g_in.  WPR waves per row (4/WPR rows per 256-thread workgroup); each
// lane keeps CH independent loads in flight per round; partial LSEs merged by shuffles + LDS.
template <typename T, bool KNOPP, int CH, int WPR>
__global__ __launch_bounds__(256) void k_sk_row(const T* __restrict__ C, SkArgs a, SkDev d,
                                                int it, int slot_in, int slot_out) {
  if (d.st[ST_DONE]) return;
  if (KNOPP && knopp_stop(d, it)) return;
  __shared__ double wm[4], ws[4];
  __shared__ LseTable tab_sh;
  const double* tab = lse_table(tab_sh);
  const int w = wave_id(), lane = lane_id();
  const int i = blockIdx.x * (4 / WPR) + w / WPR;
  const int t = (w % WPR) * 64 + lane;  // thread index inside the row's team
  constexpr int NT = 64 * WPR;
  Lse l;
  l.init();
  if (KNOPP && !d.st[ST_CNAN]) {  // fast path (uniform): scaled terms, unmasked full chunks
    if (i < a.I) {
      const double* __restrict__ gs = d.gs + (int64_t)slot_in * a.J;
      const T* __restrict__ Ci = C + (int64_t)i * a.ldc;
      int j0 = 0;
      for (; j0 + NT * CH <= a.J; j0 += NT * CH) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
          const int j = j0 + NT * k + t;
          x[k] = sk_term_s((double)Ci[j], a.inv_eps, gs[j]);
        }
        lse2_chunk<CH>(l, x, tab);
      }
      if (j0 < a.J) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
          const int j = j0 + NT * k + t;
          x[k] = j < a.J ? sk_term_s((double)Ci[j], a.inv_eps, gs[j]) : -INFINITY;
        }
        lse2_chunk<CH>(l, x, tab);
      }
      lse_unscale(l);
    }
  } else if (i < a.I) {
    const double* __restrict__ g = d.g + (int64_t)slot_in * a.J;
    const double* __restrict__ va = d.va;
    const double uai = KNOPP ? 0.0 : d.ua[i];
    const T* __restrict__ Ci = C + (int64_t)i * a.ldc;
    for (int j0 = 0; j0 < a.J; j0 += NT * CH) {
      double x[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int j = j0 + NT * k + t;
        x[k] = -INFINITY;
        if (j < a.J) {
          const double vj = KNOPP ? 0.0 : va[j];
          x[k] = sk_term<KNOPP>(uai, vj, (double)Ci[j], a.inv_eps, a.kclamp, g[j] - vj);
        }
      }
      lse_chunk<CH>(l, x, tab);
    }
  }
  l = wave_lse(l);
  if (WPR > 1) {
    if (lane == 0) {
      wm[w] = l.m;
      ws[w] = l.s;
    }
    __syncthreads();
    if (i >= a.I || (w % WPR) != 0 || lane != 0) return;
    for (int q = 1; q < WPR; ++q) l.merge(wm[w + q], ws[w + q]);
  } else if (i >= a.I || lane != 0) {
    return;
  }
  finish_row(a, d, i, l, it, slot_out, KNOPP ? 0.0 : d.ua[i], KNOPP);
}

// Finish column j from its LSE: g update, KNOPP err^2 term and break flags, STAB big flag.
__device__ __forceinline__ void finish_col(const SkArgs& a, SkDev& d, int j, double ls,
                                           int slot_g_prev, int slot_g_out, bool knopp,
                                           double& errp, bool& fail, bool& big) {
  if (knopp) {
    // err of the previous iterate: v_{k-1} * (K^T u_{k-1}) - b    (utils/ot_loss.py:65-66)
    const double t = exp_f64(d.g[(int64_t)slot_g_prev * a.J + j] + ls) - exp_f64(a.lb[j]);
    errp = t * t;
    fail = !(ls >= kLnTrueMin);  // K^T u == 0 (or NaN)     (:57)
    const double gj = a.lb[j] - ls;
    fail = fail || !(gj <= kExpOverflow);  // v inf / NaN   (:58-59)
    d.g[(int64_t)slot_g_out * a.J + j] = gj;
    d.gs[(int64_t)slot_g_out * a.J + j] = gj * kScale;
  } else {
    double lb = a.p_col * (a.lb[j] - ls);
    if (lb > kLn1e30) lb = kLn1e30;
    big = lb > kLn1e20;
    d.g[(int64_t)slot_g_out * a.J + j] = d.va[j] + lb;
  }
}

// Column pass, fused with the update: a 1024-thread workgroup owns COLS columns; thread
// (c = tid % COLS, rg = tid / COLS) runs an online LSE over rows rg, rg + RG, ... of column c
// with CH loads in flight, row groups merge through LDS, the first COLS threads finish.
template <typename T, bool KNOPP, int COLS, int CH>
__global__ __launch_bounds__(1024) void k_sk_col_fused(const T* __restrict__ C, SkArgs a, SkDev d,
                                                       int it, int slot_f, int slot_g_prev,
                                                       int slot_g_out) {
  if (d.st[ST_DONE]) return;
  constexpr int RG = 1024 / COLS;
  __shared__ double sm[RG][COLS], ss[RG][COLS];
  __shared__ LseTable tab_sh;
  const double* tab = lse_table(tab_sh);
  const int c = threadIdx.x % COLS, rg = threadIdx.x / COLS;
  const int j = blockIdx.x * COLS + c;
  const double* __restrict__ f = d.f + (int64_t)slot_f * a.I;
  const double* __restrict__ ua = d.ua;
  Lse l;
  l.init();
  if (KNOPP && !d.st[ST_CNAN]) {  // fast path: scaled terms
    if (j < a.J) {
      const double* __restrict__ fs = d.fs + (int64_t)slot_f * a.I;
      for (int i0 = rg; i0 < a.I; i0 += RG * CH) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
          const int i = i0 + RG * k;
          x[k] = i < a.I ? sk_term_s((double)C[(int64_t)i * a.ldc + j], a.inv_eps, fs[i])
                         : -INFINITY;
        }
        lse2_chunk<CH>(l, x, tab);
      }
      lse_unscale(l);
    }
  } else if (j < a.J) {
    const double vaj = KNOPP ? 0.0 : d.va[j];
    for (int i0 = rg; i0 < a.I; i0 += RG * CH) {
      double x[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int i = i0 + RG * k;
        x[k] = -INFINITY;
        if (i < a.I) {
          const double ui = KNOPP ? 0.0 : ua[i];
          x[k] = sk_term<KNOPP>(ui, vaj, (double)C[(int64_t)i * a.ldc + j], a.inv_eps, a.kclamp,
                                f[i] - ui);
        }
      }
      lse_chunk<CH>(l, x, tab);
    }
  }
  sm[rg][c] = l.m;
  ss[rg][c] = l.s;
  __syncthreads();
#pragma unroll
  for (int h = RG / 2; h > 0; h >>= 1) {
    if (rg < h) {
      l.merge(sm[rg + h][c], ss[rg + h][c]);
      sm[rg][c] = l.m;
      ss[rg][c] = l.s;
    }
    __syncthreads();
  }
  if (rg != 0) return;  // threads 0..COLS-1 (first lanes of wave 0)
  double errp = 0.0;
  bool fail = false, big = false;
  if (j < a.J) finish_col(a, d, j, l.value(), slot_g_prev, slot_g_out, KNOPP, errp, fail, big);
#pragma unroll
  for (int o = COLS / 2; o > 0; o >>= 1) errp += __shfl_xor(errp, o, 64);
  const unsigned long long lanes = COLS >= 64 ? ~0ull : (1ull << COLS) - 1;
  const unsigned long long anyfail = __ballot(fail) & lanes, anybig = __ballot(big) & lanes;
  if (threadIdx.x == 0) {
    if (KNOPP) {
      d.errpart[blockIdx.x] = errp;
      if (anyfail) atomicOr((unsigned long long*)&d.st[ST_FAIL], 1ull);
    } else if (anybig) {
      atomicOr((unsigned long long*)&d.st[ST_BIG], 2ull);
    }
  }
}

// Column pass, split: workgroup = 16 waves x 64 consecutive columns (full 256-B / 512-B rows)
// over one of NS row splits; partial (max, sum) pairs merged by k_sk_col_combine.
template <typename T, bool KNOPP, int CH>
__global__ __launch_bounds__(1024) void k_sk_col_part(const T* __restrict__ C, SkArgs a, SkDev d,
                                                      int slot_f, int rows_per_split) {
  if (d.st[ST_DONE]) return;
  __shared__ double sm[16][64], ss[16][64];
  __shared__ LseTable tab_sh;
  const double* tab = lse_table(tab_sh);
  const int lane = lane_id(), w = wave_id();
  const int j = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rows_per_split, r1 = min(a.I, r0 + rows_per_split);
  const double* __restrict__ f = d.f + (int64_t)slot_f * a.I;
  const double* __restrict__ ua = d.ua;
  Lse l;
  l.init();
  if (KNOPP && !d.st[ST_CNAN]) {  // fast path: scaled terms, unmasked full chunks
    if (j < a.J) {
      const double* __restrict__ fs = d.fs + (int64_t)slot_f * a.I;
      int i0 = r0 + w;
      for (; i0 + 16 * (CH - 1) < r1; i0 += 16 * CH) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
          const int i = i0 + 16 * k;
          x[k] = sk_term_s((double)C[(int64_t)i * a.ldc + j], a.inv_eps, fs[i]);
        }
        lse2_chunk<CH>(l, x, tab);
      }
      if (i0 < r1) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) {
          const int i = i0 + 16 * k;
          x[k] = i < r1 ? sk_term_s((double)C[(int64_t)i * a.ldc + j], a.inv_eps, fs[i])
                        : -INFINITY;
        }
        lse2_chunk<CH>(l, x, tab);
      }
      lse_unscale(l);
    }
  } else if (j < a.J) {
    const double vaj = KNOPP ? 0.0 : d.va[j];
    for (int i0 = r0 + w; i0 < r1; i0 += 16 * CH) {
      double x[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int i = i0 + 16 * k;
        x[k] = -INFINITY;
        if (i < r1) {
          const double ui = KNOPP ? 0.0 : ua[i];
          x[k] = sk_term<KNOPP>(ui, vaj, (double)C[(int64_t)i * a.ldc + j], a.inv_eps, a.kclamp,
                                f[i] - ui);
        }
      }
      lse_chunk<CH>(l, x, tab);
    }
  }
  sm[w][lane] = l.m;
  ss[w][lane] = l.s;
  __syncthreads();
  if (w != 0 || j >= a.J) return;
  for (int q = 1; q < 16; ++q) l.merge(sm[q][lane], ss[q][lane]);
  d.pm[(int64_t)blockIdx.y * a.J + j] = l.m;
  d.ps[(int64_t)blockIdx.y * a.J + j] = l.s;
}

template <bool KNOPP>
__global__ __launch_bounds__(256) void k_sk_col_combine(SkArgs a, SkDev d, int ns, int slot_g_prev,
                                                        int slot_g_out) {
  if (d.st[ST_DONE]) return;
  __shared__ double red[4];
  const int j = blockIdx.x * 256 + threadIdx.x;
  double errp = 0.0;
  bool fail = false, big = false;
  if (j < a.J) {
    double m[kMaxSplits], sv[kMaxSplits];
#pragma unroll
    for (int q = 0; q < kMaxSplits; ++q) {  // all loads first, then the merges
      m[q] = q < ns ? d.pm[(int64_t)q * a.J + j] : -INFINITY;
      sv[q] = q < ns ? d.ps[(int64_t)q * a.J + j] : 0.0;
    }
    Lse l;
    l.init();
#pragma unroll
    for (int q = 0; q < kMaxSplits; ++q) l.merge(m[q], sv[q]);
    finish_col(a, d, j, l.value(), slot_g_prev, slot_g_out, KNOPP, errp, fail, big);
  }
  if (KNOPP) {
    errp = wave_sum(errp);
    if (lane_id() == 0) red[wave_id()] = errp;
    if (__any(fail) && lane_id() == 0) atomicOr((unsigned long long*)&d.st[ST_FAIL], 1ull);
    __syncthreads();
    if (threadIdx.x == 0) d.errpart[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  } else if (__any(big) && lane_id() == 0) {
    atomicOr((unsigned long long*)&d.st[ST_BIG], 2ull);
  }
}

// STAB absorption, part A (one wave per row): decide, set ua = f, row sums of K.C.
template <typename T>
__global__ __launch_bounds__(256) void k_sk_absorb_rows(const T* __restrict__ C, SkArgs a, SkDev d,
                                                        int it, int slot, int max_iter,
                                                        int init) {
  if (d.st[ST_DONE]) return;
  const bool absorb = init || (it % 10 == 0) || d.st[ST_BIG] || it == max_iter - 1;
  if (!absorb) return;
  const int i = blockIdx.x * 4 + wave_id();
  if (i >= a.I) return;
  const int lane = lane_id();
  const double fi = init ? 0.0 : d.f[(int64_t)slot * a.I + i];
  const double* g = d.g + (int64_t)slot * a.J;
  const T* Ci = C + (int64_t)i * a.ldc;
  double acc = 0.0;
  for (int j = lane; j < a.J; j += 64) {
    const double c = ld_c(Ci, j);
    const double k = fmin(fi + (init ? 0.0 : g[j]) - c * a.inv_eps, a.kclamp);
    acc += exp_f64(k) * c;
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    d.rowbuf[i] = acc;
    d.ua[i] = fi;
  }
}

// STAB absorption, part B (single workgroup): va = g, transport, tolerance break, bookkeeping.
__global__ __launch_bounds__(1024) void k_sk_absorb_final(SkArgs a, SkDev d, int it, int slot,
                                                          int max_iter, int init, double tol) {
  if (d.st[ST_DONE]) return;
  const bool absorb = init || (it % 10 == 0) || d.st[ST_BIG] || it == max_iter - 1;
  __syncthreads();
  if (!absorb) return;
  __shared__ double red[1024];
  const double* g = d.g + (int64_t)slot * a.J;
  for (int j = threadIdx.x; j < a.J; j += 1024) d.va[j] = init ? 0.0 : g[j];
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
  if (init) {
    d.sd[SD_TPREV] = tnew;
    d.sd[SD_TNEW] = tnew;
    return;
  }
  const double tprev = d.sd[SD_TPREV];
  d.sd[SD_TNEW] = tnew;
  if (fabs(tnew - tprev) / fabs(tprev) < tol) {
    mark_done(d.st, it, 1, slot);  // break: ii stays, `transport` keeps the previous value
    return;
  }
  d.sd[SD_TPREV] = tnew;
  if (it == max_iter - 1) mark_done(d.st, max_iter, 0, slot);
}

// ST_CNAN: does C hold a NaN or an infinity (KNOPP: the passes then take the exact terms);
// ST_CMASK: does any term underflow (-C / reg < kExpUnderflow, the fused sweep's mask predicate)
template <typename T>
__global__ __launch_bounds__(256) void k_sk_cscan(const T* __restrict__ C, int I, int J,
                                                  int64_t ldc, double neg_s, int64_t* st) {
  bool bad = false, msk = false;
  const int64_t n = (int64_t)I * J;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t i = e / J, j = e - i * J;
    const double c = (double)C[i * ldc + j];
    bad |= !isfinite(c);
    msk |= c * neg_s < kExpUnderflow;
  }
  if (__any(bad) && lane_id() == 0) atomicOr((unsigned long long*)&st[ST_CNAN], 1ull);
  if (__any(msk) && lane_id() == 0) atomicOr((unsigned long long*)&st[ST_CMASK], 1ull);
}

__global__ void k_sk_logw(const double* __restrict__ wa, const double* __restrict__ wb, int I,
                          int J, double* __restrict__ la, double* __restrict__ lb) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < I) la[t] = log(wa[t]);
  if (t < J) lb[t] = log(wb[t]);
}

__global__ void k_sk_init(SkArgs a, SkDev d, double tol) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 32) {
    if (t < 8) d.st[t] = 0;
    else d.sd[t] = 0.0;
    if (t == SD_TOL) d.sd[SD_TOL] = tol;
  }
  const bool knopp = a.mode == GNNEA_SK_KNOPP;
  // KNOPP: u = 1/I, v = 1/J stored in slot 1 (the "previous" slot of iteration 0)
  for (int i = t; i < a.I; i += gridDim.x * blockDim.x) {
    d.ua[i] = 0.0;
    d.f[i] = 0.0;
    d.f[a.I + i] = knopp ? -log((double)a.I) : 0.0;
    d.fs[a.I + i] = knopp ? -log((double)a.I) * kScale : 0.0;
  }
  for (int j = t; j < a.J; j += gridDim.x * blockDim.x) {
    d.va[j] = 0.0;
    d.g[j] = 0.0;
    d.g[a.J + j] = knopp ? -log((double)a.J) : 0.0;
    d.gs[a.J + j] = knopp ? -log((double)a.J) * kScale : 0.0;
  }
}

// Final plan, one wave per row; also its row sums.
// final ping-pong slot: the break / tolerance slot, else the last iteration run (1 = initial)
__device__ __forceinline__ int sk_final_slot(const SkDev& d, int iters_run) {
  if (d.st[ST_DONE]) return (int)(d.st[ST_SLOT] & 1);
  return iters_run > 0 ? ((iters_run - 1) & 1) : 1;
}

template <typename T, typename P>
__global__ __launch_bounds__(256) void k_sk_plan(const T* __restrict__ C, SkArgs a, SkDev d,
                                                 int iters_run, P* __restrict__ plan, int64_t ldp,
                                                 double* __restrict__ row_sum) {
  const int slot = sk_final_slot(d, iters_run);
  const int i = blockIdx.x * 4 + wave_id();
  if (i >= a.I) return;
  const int lane = lane_id();
  const bool knopp = a.mode == GNNEA_SK_KNOPP;
  const double fi = knopp ? d.f[(int64_t)slot * a.I + i] : d.ua[i];
  const double* g = knopp ? d.g + (int64_t)slot * a.J : d.va;
  const T* Ci = C + (int64_t)i * a.ldc;
  double rs = 0.0, loss = 0.0;
  for (int j = lane; j < a.J; j += 64) {
    const double c = ld_c(Ci, j);
    double v;
    if (knopp) {
      // P = u * K * v with K = exp_f64(-M/reg) underflowing to 0 below -745.13
      const double k = -c * a.inv_eps;
      v = k < kExpUnderflow ? 0.0 : exp_f64(fi + g[j] + k);
    } else {
      v = exp_f64(fmin(fi + g[j] - c * a.inv_eps, a.kclamp));
    }
    if (plan) plan[(int64_t)i * ldp + j] = (P)v;
    rs += v;
    loss += v * c;
  }
  rs = wave_sum(rs);
  loss = wave_sum(loss);
  if (lane == 0) {
    if (row_sum) row_sum[i] = rs;
    d.rowbuf[i] = loss;
  }
}

// Column sums of the returned plan: kMaxSplits row ranges per 256-column block (one thread per
// column, partial sums into the workspace's split rows), then the splits added in order by
// k_sk_colsum_fin: deterministic.  (One thread per column over all I rows ran 59 workgroups for
// 7.6 ms at B = 15000.)
template <typename T>
__global__ __launch_bounds__(256) void k_sk_colsum(const T* __restrict__ C, SkArgs a, SkDev d,
                                                   int iters_run, double* __restrict__ part) {
  const int slot = sk_final_slot(d, iters_run);
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int ns = gridDim.y, sp = blockIdx.y;
  const int i0 = (int)((int64_t)a.I * sp / ns), i1 = (int)((int64_t)a.I * (sp + 1) / ns);
  if (j >= a.J) return;
  const bool knopp = a.mode == GNNEA_SK_KNOPP;
  const double gj = knopp ? d.g[(int64_t)slot * a.J + j] : d.va[j];
  const double* f = knopp ? d.f + (int64_t)slot * a.I : d.ua;
  double s0 = 0.0, s1 = 0.0;
  auto term = [&](int i) {
    const double c = ld_c(C, (int64_t)i * a.ldc + j);
    if (knopp) {
      const double k = -c * a.inv_eps;
      return k < kExpUnderflow ? 0.0 : exp_f64(f[i] + gj + k);
    }
    return exp_f64(fmin(f[i] + gj - c * a.inv_eps, a.kclamp));
  };
  int i = i0;
  for (; i + 1 < i1; i += 2) {  // two independent chains
    s0 += term(i);
    s1 += term(i + 1);
  }
  if (i < i1) s0 += term(i);
  part[(int64_t)sp * a.J + j] = s0 + s1;
}

__global__ __launch_bounds__(256) void k_sk_colsum_fin(const double* __restrict__ part, int ns,
                                                       int J, double* __restrict__ col_sum) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= J) return;
  double s = 0.0;
  for (int q = 0; q < ns; ++q) s += part[(int64_t)q * J + j];
  col_sum[j] = s;
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
    d.sd[SD_LOSS] = red[0];
    if (!d.st[ST_DONE]) {
      d.st[ST_ITERS] = iters_run;
      d.st[ST_SLOT] = sk_final_slot(d, iters_run);
    }
  }
}

static bool sk_valid(const gnnea_sinkhorn* p) {
  if (!p || !p->C || !p->ws || !p->a || !p->b) return false;
  if (p->I < 1 || p->J < 1 || p->ldc < p->J) return false;
  if (p->c_dtype != GNNEA_F32 && p->c_dtype != GNNEA_F64) return false;
  if (p->mode < GNNEA_SK_KNOPP || p->mode > GNNEA_SK_RELAX) return false;
  if (!(p->eps > 0.0)) return false;
  return true;
}

static SkArgs sk_args(const gnnea_sinkhorn* p) {
  SkArgs a;
  a.mode = p->mode;
  a.I = p->I;
  a.J = p->J;
  a.ldc = p->ldc;
  a.inv_eps = 1.0 / p->eps;
  const bool gen = p->mode == GNNEA_SK_GEN, relax = p->mode == GNNEA_SK_RELAX;
  a.p_row = gen ? p->p : 1.0;
  a.p_col = (gen || relax) ? p->p : 1.0;
  a.kclamp = p->mode == GNNEA_SK_KNOPP ? INFINITY : kLn1e30;
  const SkWs w = sk_plan(p->I, p->J);
  a.la = (const double*)((const char*)p->ws + w.la);  // log a, log b: filled by init
  a.lb = (const double*)((const char*)p->ws + w.lb);
  a.wa = p->a;
  a.wb = p->b;
  return a;
}

// ---------------------------------------------------------------------------------------- //
// Fused KNOPP sweep: ONE pass over C per iteration and ONE exponential per element.
//
// The reference's scaling-form iteration (utils/ot_loss.py:53-55, v = b / K^T u then
// u = 1 / (Kp v)) on potentials f = log u, g = log v, the kernel recomputed from C in the pass.
// Row i of iteration it (g = g_it complete, written by the column update before the sweep):
//   x_ij = g_j + k_ij (k_ij = -C_ij / reg, masked to -inf where exp_f64 underflows, as sk_term),
//   each wave w: M_w = max over its columns, e_ij = exp(x_ij - M_w) <= 1, s_w = sum e_ij;
//   the workgroup: M = max_w M_w, s = sum_w s_w exp(M_w - M), LSE_j(x_ij) = M + log s,
//   f_it,i = log a_i - LSE   (u = a / (K v)),
// and the same e_ij, scaled by exp(M_w - M) a_i / s, ARE the entries of P(u_it, v_it) =
// u_it K v_it (<= a_i: no overflow; an entry lost to underflow is below 2^-1022 a_i).
// Accumulated down the workgroup's rows they are its partial of S_j = v_it (K^T u_it)_j; the
// column update (k_lsk_colfin) sums the partials in fixed order:
//   err^2 term of iterate it   (S_j - b_j)^2                    (utils/ot_loss.py:64-66)
//   g_{it+1} = log b_j - log S_j + g_{it,j}                      (v = b / K^T u, :53-54)
// A column whose S_j is outside [2^-600, 2^600] (K^T u underflowing, an all-masked column, inf,
// NaN) is recomputed there from C and f with a running maximum, so the fast path never trades
// accuracy.  The breaks are the two-pass path's: K^T u == 0 (column LSE below ln DBL_TRUE_MIN)
// or v inf / NaN flagged by the column update, u inf / NaN by the row update, the err test of
// iterate it-1 at the start of sweep it.
//
// Layout (as k_sk_sweep of the scaling form): a 512-thread workgroup owns rows [r0, r1) (about
// one workgroup per CU); wave w owns the column slice c0 + 64 k + lane (k < NCM) of every row, the
// slice's g in LDS; the next row's C values are in flight (buffer loads: columns past J read 0,
// no clamp per column) while a row is reduced; one barrier per row.  Per element: the fp64 term
// (one multiply, the underflow mask, one fma), the running max, the table exponential
// (2^(x/2048): 2048-entry table in LDS + degree-3 polynomial, truncation 3.4e-17), the row sum
// and the column fma -- against two exponentials, two running maxima and two passes over C in the
// two-pass form.  C is read once per iteration: I J sizeof(T) bytes (0.9 GB fp32 at B = 15000).
constexpr double kFScale = 2954.639443740597;  // 2048 / ln 2
constexpr double kFLo = 0x1p-600, kFHi = 0x1p600;

__global__ void k_lsk_tab(double* __restrict__ tab) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < kFTab) tab[j] = exp2((double)j / (double)kFTab);
}

// 2^(x / 2048): t = rint(x), r = x - t in [-1/2, 1/2], 2^(t >> 11) * tab[t & 2047] * e^(r ln2/2048)
// (e^y - 1 to degree 3, |y| <= 1.7e-4).  x = -huge (a masked term) gives 0: t saturates in the
// int conversion, ldexp underflows.  NaN stays NaN.
__device__ __forceinline__ double exp2x(double x, const double* __restrict__ tab) {
  constexpr double c1 = 0.0003384507717577858, c2 = 5.72744624517204e-08,
                   c3 = 6.461528672932365e-12;  // (ln2/2048)^k / k!
  const double t = __builtin_rint(x);
  const double r = x - t;
  const int ti = (int)t;
  double p = __builtin_fma(r, c3, c2);
  p = __builtin_fma(p, r, c1);
  p *= r;
  const double tj = tab[ti & (kFTab - 1)];
  return __builtin_ldexp(__builtin_fma(tj, p, tj), ti >> 11);
}

// exp2x in two halves, so that a group of elements issues its table reads together and the reads'
// LDS latency runs under the group's polynomials (one element at a time, each read was waited
// for three instructions after its issue)
struct Exp2Part {
  double r;  // x - rint(x)
  int ti;    // rint(x) (saturated for a masked term)
};
__device__ __forceinline__ Exp2Part exp2x_split(double x) {
  const double t = __builtin_rint(x);
  return Exp2Part{x - t, (int)t};
}
__device__ __forceinline__ double exp2x_poly(double r) {  // e^(r ln2/2048) - 1
  constexpr double c1 = 0.0003384507717577858, c2 = 5.72744624517204e-08,
                   c3 = 6.461528672932365e-12;
  double p = __builtin_fma(r, c3, c2);
  p = __builtin_fma(p, r, c1);
  return p * r;
}
__device__ __forceinline__ double exp2x_finish(const Exp2Part& q, double tj) {
  constexpr double c1 = 0.0003384507717577858, c2 = 5.72744624517204e-08,
                   c3 = 6.461528672932365e-12;  // (ln2/2048)^k / k!
  double p = __builtin_fma(q.r, c3, c2);
  p = __builtin_fma(p, q.r, c1);
  p *= q.r;
  return __builtin_ldexp(__builtin_fma(tj, p, tj), q.ti >> 11);
}
constexpr int kExpGroup = 4;  // B = 15000: 4305-4402 iters/s (8: 4266, 1: 4095;
                              // profiles/r05_sinkhorn_egrp_ab.json)

// natural-unit logit of K_ij (masked: -inf where exp_f64(-C/reg) underflows, as sk_term)
__device__ __forceinline__ double lsk_k(double c, double inv_eps) {
  const double k = -c * inv_eps;
  return k < kExpUnderflow ? -INFINITY : k;
}

// The sweep's per-row barrier: the wave partials in LDS are complete (lgkmcnt(0)), then a raw
// s_barrier.  __syncthreads() is a workgroup fence as well, which waits vmcnt(0): it drained the
// next row's C loads (the prefetch) at every row.  The LDS hand-off needs no vector-memory wait.
__device__ __forceinline__ void row_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// PH0 (init): no row update, P(u_0, v_0) = exp(f_0 + g_0 + k) directly: the partials of
// v_0 K^T u_0 for the first column update.
// PAIR (fp32 C, J and ldc even): lane l owns the column PAIRS c0 + 128 p + 2 l + {0, 1}, read as
// one 8-B buffer load each (NCM / 2 loads per row instead of NCM: two rows in flight stay below
// the 63 outstanding loads vmcnt can count), g as one 16-B LDS read per pair.
template <typename T, int NCM, bool PH0, bool PAIR, int FW>
__global__ __launch_bounds__(64 * FW) void k_lsk_sweep(const T* __restrict__ C, SkArgs a, SkDev d,
                                                        int it, int slot_fp, int slot_g,
                                                        int slot_fo, int rpw) {
  __shared__ double tab[kFTab];
  __shared__ double gsh[FW * NCM * 64];
  __shared__ double reds[2][FW];
  if (!PH0 && d.st[ST_DONE]) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  {
    double tv[kFTab / (64 * FW)];
#pragma unroll
    for (int q = 0; q < kFTab / (64 * FW); ++q) tv[q] = d.ftab[tid + q * 64 * FW];
#pragma unroll
    for (int q = 0; q < kFTab / (64 * FW); ++q) tab[tid + q * 64 * FW] = tv[q];
  }
  const int r0 = blockIdx.x * rpw, r1 = min(a.I, r0 + rpw);
  const int cw = ((a.J + FW - 1) / FW + 63) & ~63;
  const int c0 = w * cw;
  const int lim = min(c0 + cw, a.J) - c0 - lane;  // column c0 + 64 k + lane is valid iff 64 k < lim
  const double* __restrict__ g = d.g + (int64_t)slot_g * a.J;
  {  // the wave's slice of g (scaled), column c0 + q at gsh[w NCM 64 + q]; every load issued
     // first from a clamped column (a load under the validity branch waited for each in turn)
    double* __restrict__ gf = gsh + w * NCM * 64 + lane;
    double gv[NCM];
#pragma unroll
    for (int k = 0; k < NCM; ++k) gv[k] = g[min(c0 + 64 * k + lane, a.J - 1)];
#pragma unroll
    for (int k = 0; k < NCM; ++k) gf[64 * k] = 64 * k < lim ? gv[k] * kFScale : -1e300;
  }
  __syncthreads();
  // element k of this lane: column c0 + lbase + eo(k)
  constexpr auto eo = [](int k) { return PAIR ? 128 * (k >> 1) + (k & 1) : 64 * k; };
  const int lbase = PAIR ? 2 * lane : lane;
  const int limv = min(c0 + cw, a.J) - c0 - lbase;  // element k valid iff eo(k) < limv
  const double* __restrict__ gl = gsh + w * NCM * 64 + lbase;
  T kA[NCM], kB[NCM], kC[NCM];
  // the row's two scalars (f_prev, a) ride with its C loads, issued FIRST: a row's scalars are
  // then older than the next row's C loads in flight, and waiting for them is a counted vmcnt
  // (loaded inside process() they were the newest loads, and the wait for them drained the next
  // row's prefetch every row)
  double fA = 0.0, fB = 0.0, fC = 0.0, wA = 0.0, wB = 0.0, wC = 0.0;
  // buffer loads over the row (J elements): one lane offset, the 64 k steps as scalar offsets;
  // columns past J read 0 (their g slice is -1e300: no contribution) without a clamp per column
  const uint32_t voff = (uint32_t)(c0 + lbase) * sizeof(T);
  auto load = [&](T (&kv)[NCM], double& fv, double& wv, int r) {
    fv = d.f[(int64_t)slot_fp * a.I + r];
    wv = a.wa[r];
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(C + (int64_t)r * a.ldc), (short)0, a.J * (int)sizeof(T), 0x00020000);
    if constexpr (PAIR) {
#pragma unroll
      for (int p = 0; p < NCM / 2; ++p) {
        const uint64_t v = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(
            rs, voff, 512 * p, 0));
        kv[2 * p] = __builtin_bit_cast(T, (uint32_t)v);
        kv[2 * p + 1] = __builtin_bit_cast(T, (uint32_t)(v >> 32));
      }
    } else {
#pragma unroll
      for (int k = 0; k < NCM; ++k) {
        if constexpr (sizeof(T) == 4)
          kv[k] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, voff, 256 * k, 0));
        else
          kv[k] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, 512 * k, 0));
      }
    }
  };
  // the first rows' loads go out before the stop decision (round trips on the status block)
  if (r0 < r1) {
    load(kA, fA, wA, r0);
    if (PAIR && FW == 8) load(kB, fB, wB, min(r0 + 1, r1 - 1));
  }
  if (!PH0 && knopp_stop(d, it)) return;
  double acc[NCM];
#pragma unroll
  for (int k = 0; k < NCM; ++k) acc[k] = 0.0;
  const double neg_s = -a.inv_eps;
  // fp32 C: the term is masked (the reference's K entry underflows to 0: -C/reg below
  // kExpUnderflow) exactly when C > cthr, the largest float that still gives a finite term --
  // one f32 compare per element; the masked element's C is replaced by 1e30 (x -> -huge ->
  // exp2x 0); the logit is one fma with the folded scale C * (-kFScale / reg)
  const double ncs = neg_s * kFScale;
  float cthr = (float)(kExpUnderflow / neg_s);
  while (!((double)cthr * neg_s >= kExpUnderflow)) cthr = nextafterf(cthr, -INFINITY);
  while ((double)nextafterf(cthr, INFINITY) * neg_s >= kExpUnderflow)
    cthr = nextafterf(cthr, INFINITY);
  // MT: the mask (std::true_type when init found an underflowing term, ST_CMASK; a uniform
  // choice for the whole launch): without it no element needs the compare and select
  auto logit = [&](T c, double gsum, auto mt) {
    if constexpr (sizeof(T) == 4) {
      float cm = (float)c;
      if constexpr (decltype(mt)::value) cm = c > cthr ? 1e30f : cm;
      return __builtin_fma((double)cm, ncs, gsum);
    } else {
      if constexpr (decltype(mt)::value) {
        const double kn = (double)c * neg_s;
        const double kk = kn < kExpUnderflow ? -1e300 : kn;
        return __builtin_fma(kk, kFScale, gsum);
      } else {
        return __builtin_fma((double)c, ncs, gsum);
      }
    }
  };
  int nfb = 0;  // rows listed for the exact update (k_lsk_fix)
  auto process = [&](const T (&kv)[NCM], const double fv, const double wv, int r, int par,
                     auto mt) {
    // x = (g_j + k_ij) in units of ln2 / 2048; masked terms -3e303 (exp2x -> 0).  The slice of g
    // is re-read from LDS per row (opaque to hoisting: held in registers it would cost 2 NCM)
    asm volatile("" ::: "memory");
    double e[NCM];
    if (PH0) {
      const double f0 = fv * kFScale;
#pragma unroll
      for (int k = 0; k < NCM; ++k) {
        e[k] = exp2x(logit(kv[k], gl[eo(k)] + f0, mt), tab);
        acc[k] += e[k];
      }
      return;
    }
    // shifted by f_prev: x + f_prev = log P(u_prev, v_it)_ij <= log b_j (v_it = b / K^T u_prev),
    // so e_ij = P(u_prev, v_it)_ij needs no running maximum; s_i = u_prev (K v_it)_i
    const double fps = fv * kFScale;
    double rsum = 0.0;
    // groups of EG elements: logits and table indices, the EG table reads, then the polynomials
    constexpr int EG = kExpGroup < NCM ? kExpGroup : NCM;
    static_assert(NCM % EG == 0, "group size");
    // phased: the group's table reads and the NEXT group's g reads are issued, then the group's
    // polynomials run under them, then the reads are consumed
    double gv[EG];
#pragma unroll
    for (int u = 0; u < EG; ++u) gv[u] = gl[eo(u)];
#pragma unroll
    for (int k0 = 0; k0 < NCM; k0 += EG) {
      Exp2Part q[EG];
      double tj[EG], pp[EG];
#pragma unroll
      for (int u = 0; u < EG; ++u) q[u] = exp2x_split(logit(kv[k0 + u], gv[u] + fps, mt));
#pragma unroll
      for (int u = 0; u < EG; ++u) tj[u] = tab[q[u].ti & (kFTab - 1)];
      if (k0 + EG < NCM) {
#pragma unroll
        for (int u = 0; u < EG; ++u) gv[u] = gl[eo(k0 + EG + u)];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < EG; ++u) pp[u] = exp2x_poly(q[u].r);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < EG; ++u) {
        e[k0 + u] = __builtin_ldexp(__builtin_fma(tj[u], pp[u], tj[u]), q[u].ti >> 11);
        rsum += e[k0 + u];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    rsum = wave_sum_f64(rsum);
    if (lane == 0) reds[par][w] = rsum;
    row_barrier();  // double-buffered by row parity: one barrier per row
    double sr = 0.0;
#pragma unroll
    for (int q = 0; q < FW; ++q) sr += reds[par][q];  // every wave, the same order
    // (NaN -- in C or a potential -- propagates through the fast path; the row update flags it)
    if ((sr >= kFLo && sr <= kFHi) || sr != sr) {  // u_it / u_prev = a / s
      const double wi = wv / sr;
      // f_it = f_prev + log a - log s, written by k_lsk_fix (no log in the streaming kernel)
      if (w == 0 && lane == 0) d.rowbuf[r] = sr;
#pragma unroll
      for (int k = 0; k < NCM; ++k) acc[k] = __builtin_fma(e[k], wi, acc[k]);
      return;
    }
    // out of range (uniform: every wave summed the same partials): the row is listed for
    // k_lsk_fix, which writes its exact update and adds its column contributions to this
    // workgroup's partial row after the sweep; nothing of it goes into acc
    if (w == 0 && lane == 0) {
      d.fbrows[(int64_t)blockIdx.x * rpw + nfb] = r;
      d.rowbuf[r] = -1.0;  // (k_lsk_fix: listed, not a row sum)
    }
    ++nfb;
    return;
  };
  // the next row's loads go out unconditionally (past the last row: the last row again), so
  // every path into a row's processing has the same loads outstanding and its waits are counted
  // vmcnt(NCM loads of the next row) -- a conditional load made the compiler wait for the
  // count of the path without it, i.e. for most of the next row's loads
  // PAIR: NCM / 2 + 2 loads per row, two rows ahead in flight (three register buffers, the
  // waits vmcnt(2 rows)); otherwise one row ahead
  auto rows = [&](auto mt) {
    int r = r0, par = 0;
    if constexpr (PAIR && FW == 8) {
      while (r < r1) {
        load(kC, fC, wC, min(r + 2, r1 - 1));
        process(kA, fA, wA, r, par, mt);
        if (r + 1 >= r1) break;
        load(kA, fA, wA, min(r + 3, r1 - 1));
        process(kB, fB, wB, r + 1, par ^ 1, mt);
        if (r + 2 >= r1) break;
        load(kB, fB, wB, min(r + 4, r1 - 1));
        process(kC, fC, wC, r + 2, par, mt);
        par ^= 1;
        r += 3;
      }
    } else {
      while (r < r1) {
        load(kB, fB, wB, min(r + 1, r1 - 1));
        process(kA, fA, wA, r, par, mt);
        if (r + 1 >= r1) break;
        load(kA, fA, wA, min(r + 2, r1 - 1));
        process(kB, fB, wB, r + 1, par ^ 1, mt);
        r += 2;
      }
    }
  };
  if (d.st[ST_CMASK])
    rows(std::true_type{});
  else
    rows(std::false_type{});
  double* __restrict__ part = d.fpart + (int64_t)blockIdx.x * a.J + c0 + lbase;
#pragma unroll
  for (int k = 0; k < NCM; ++k)
    if (eo(k) < limv) part[eo(k)] = acc[k];
  if (!PH0 && tid == 0) d.fbcnt[blockIdx.x] = nfb;
}

// The exact row update for the rows a fused sweep workgroup listed (k_lsk_sweep, SH): per row in
// list order, the LSE with a running maximum (natural units, the workgroup's waves over column
// slices, merged in fixed order), f_new = log a - LSE, and P(u_new, v)_ij = exp(f_new + g_j +
// k_ij) added to that workgroup's partial row.  A workgroup with an empty list returns at once.
template <typename T>
__global__ __launch_bounds__(64 * kFW) void k_lsk_fix(const T* __restrict__ C, SkArgs a, SkDev d,
                                                      int it, int slot_fp, int slot_g, int slot_fo,
                                                      int rpw) {
  if (d.st[ST_DONE]) return;
  {  // the row update of the workgroup's rows from their sums: f_it = f_prev + log a - log s
    const int r0 = blockIdx.x * rpw, r1 = min(a.I, r0 + rpw);
    bool bad = false;
    for (int r = r0 + (int)threadIdx.x; r < r1; r += 64 * kFW) {
      const double sr = d.rowbuf[r];
      if (sr == -1.0) continue;  // listed: the exact update below
      const double fnew = d.f[(int64_t)slot_fp * a.I + r] + (a.la[r] - log(sr));
      d.f[(int64_t)slot_fo * a.I + r] = fnew;
      bad |= !(fnew <= kExpOverflow);  // u inf / NaN
    }
    if (bad) mark_done(d.st, it, 2, (it + 1) & 1);
  }
  const int n = d.fbcnt[blockIdx.x];
  if (n == 0) return;
  __shared__ double fbm[kFW], fbs[kFW];
  const int w = wave_id(), lane = lane_id();
  const int cw = ((a.J + kFW - 1) / kFW + 63) & ~63;
  const int c0 = w * cw, c1 = min(c0 + cw, a.J);
  const double* __restrict__ g = d.g + (int64_t)slot_g * a.J;
  double* __restrict__ fb = d.fpart + (int64_t)blockIdx.x * a.J;
  for (int q = 0; q < n; ++q) {
    const int r = d.fbrows[(int64_t)blockIdx.x * rpw + q];
    const T* __restrict__ Cr = C + (int64_t)r * a.ldc;
    Lse l;
    l.init();
    for (int c = c0 + lane; c < c1; c += 64) l.add(lsk_k((double)Cr[c], a.inv_eps) + g[c]);
    l = wave_lse(l);
    if (lane == 0) {
      fbm[w] = l.m;
      fbs[w] = l.s;
    }
    __syncthreads();
    Lse t;
    t.init();
    for (int v = 0; v < kFW; ++v) t.merge(fbm[v], fbs[v]);
    __syncthreads();  // fbm / fbs read by every wave before the next row reuses them
    const double fnew = a.la[r] - t.value();  // u = a / (K v): +inf when K v == 0
    for (int c = c0 + lane; c < c1; c += 64) {
      const double kn = lsk_k((double)Cr[c], a.inv_eps);
      fb[c] += kn != -INFINITY ? exp_f64(fnew + g[c] + kn) : 0.0;
    }
    if (w == 0 && lane == 0) {
      d.f[(int64_t)slot_fo * a.I + r] = fnew;
      if (!(fnew <= kExpOverflow)) mark_done(d.st, it, 2, (it + 1) & 1);  // u inf / NaN
    }
  }
}

// Column update of the fused sweep: S_j = sum of the workgroup partials (fixed order), the
// err^2 term of the iterate the partials belong to, g = log b - log S + g_prev, the break flags.
// 16 columns per 1024-thread workgroup (errpart slots: div_up(J, 16)); a column whose S is out
// of [2^-600, 2^600] (or not finite) is recomputed from C and f exactly (running maximum).
template <typename T>
__global__ __launch_bounds__(1024) void k_lsk_colfin(const T* __restrict__ C, SkArgs a, SkDev d,
                                                     int ns, int slot_f, int slot_g_prev,
                                                     int slot_g_out) {
  if (d.st[ST_DONE]) return;
  constexpr int NC = 16;
  __shared__ double red[64][NC], lm[64][NC];
  __shared__ int need;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int cl = lane & (NC - 1), slot = w * 4 + (lane >> 4);
  const int j = blockIdx.x * NC + cl;
  const int jc = min(j, a.J - 1);
  if (tid == 0) need = 0;
  double s = 0.0;
  for (int q = slot; q < ns; q += 64) s += d.fpart[(int64_t)q * a.J + jc];
  red[slot][cl] = s;
  __syncthreads();
  double S = 0.0;
  bool slow = false;
  if (tid < NC) {
#pragma unroll 8
    for (int q = 0; q < 64; ++q) S += red[q][cl];
    slow = j < a.J && !(S >= kFLo && S <= kFHi);
    if (slow) need = 1;
  }
  __syncthreads();
  double L = 0.0;
  if (need) {  // uniform: the whole workgroup recomputes its flagged columns
    const double* __restrict__ f = d.f + (int64_t)slot_f * a.I;
    Lse l;
    l.init();
    for (int i = slot; i < a.I; i += 64) l.add(f[i] + lsk_k((double)C[(int64_t)i * a.ldc + jc], a.inv_eps));
    lm[slot][cl] = l.m;
    red[slot][cl] = l.s;
    __syncthreads();
    if (tid < NC) {
      Lse t;
      t.init();
      for (int q = 0; q < 64; ++q) t.merge(lm[q][cl], red[q][cl]);
      L = t.value();  // log K^T u_j
    }
  }
  if (tid >= 64) return;
  double errp = 0.0;
  bool fail = false;
  if (tid < NC && j < a.J) {
    const double gp = d.g[(int64_t)slot_g_prev * a.J + j];
    double gj;
    if (!slow) {
      const double t = S - a.wb[j];  // v_prev (K^T u) - b
      errp = t * t;
      gj = a.lb[j] - log(S) + gp;
    } else {
      const double t = exp_f64(gp + L) - a.wb[j];
      errp = t * t;
      fail = !(L >= kLnTrueMin);  // K^T u == 0 (or NaN)   (ot_loss.py:57)
      gj = a.lb[j] - L;
    }
    fail = fail || !(gj <= kExpOverflow);  // v inf / NaN   (:58-59)
    d.g[(int64_t)slot_g_out * a.J + j] = gj;
  }
#pragma unroll
  for (int o = NC / 2; o > 0; o >>= 1) errp += __shfl_xor(errp, o, 64);
  const unsigned long long anyfail = __ballot(fail) & ((1ull << NC) - 1);
  if (tid == 0) {
    d.errpart[blockIdx.x] = errp;
    if (anyfail) atomicOr((unsigned long long*)&d.st[ST_FAIL], 1ull);
  }
}

// the fused sweep serves KNOPP for J <= kFMaxJ (flag GNNEA_SK_TWO_PASS keeps the two passes: the
// parity tests compare the two)
static bool fused_applies(const gnnea_sinkhorn* p) {
  const bool on = !(p->flags & GNNEA_SK_TWO_PASS);
  // fp64 C: the slice's loads double, J <= kFMaxJ / 2 keeps them in registers
  return on && p->mode == GNNEA_SK_KNOPP &&
         p->J <= (p->c_dtype == GNNEA_F64 ? kFMaxJ / 2 : kFMaxJ);
}

bool fused_ok(const gnnea_sinkhorn* p) { return p && fused_applies(p); }

template <typename T, bool PH0, bool PAIR, int FW>
static void launch_fused_sweep_p(const T* C, const SkArgs& a, const SkDev& d, int it, int sfp,
                                 int sg, int sfo, hipStream_t s) {
  const int rpw = fused_rpw(a.I), ns = fused_wgs(a.I);
  const int nc = (((a.J + FW - 1) / FW + 63) & ~63) / 64;
  const dim3 g(ns), b(64 * FW);
  if (nc <= 4)
    hipLaunchKernelGGL((k_lsk_sweep<T, 4, PH0, PAIR, FW>), g, b, 0, s, C, a, d, it, sfp, sg, sfo,
                       rpw);
  else if (nc <= 8)
    hipLaunchKernelGGL((k_lsk_sweep<T, 8, PH0, PAIR, FW>), g, b, 0, s, C, a, d, it, sfp, sg, sfo,
                       rpw);
  else if (sizeof(T) == 8 || FW == 16 || nc <= 16)  // (fp64 C: fused_applies bounds nc by 16)
    hipLaunchKernelGGL((k_lsk_sweep<T, 16, PH0, PAIR, FW>), g, b, 0, s, C, a, d, it, sfp, sg, sfo,
                       rpw);
  else if constexpr (sizeof(T) == 4 && FW == 8)
    hipLaunchKernelGGL((k_lsk_sweep<T, 32, PH0, PAIR, FW>), g, b, 0, s, C, a, d, it, sfp, sg, sfo,
                       rpw);
}

// fp32 C whose rows start on 8-B boundaries and hold whole column pairs: the PAIR layout
template <typename T, bool PH0>
static void launch_fused_sweep(const T* C, const SkArgs& a, const SkDev& d, int it, int sfp,
                               int sg, int sfo, hipStream_t s) {
  if constexpr (sizeof(T) == 4) {
    if (a.J % 2 == 0 && a.ldc % 2 == 0 && ((uintptr_t)C & 7) == 0) {
      // wide rows: 16 waves of 16 columns per lane (four waves per SIMD) instead of 8 of 32
      if (a.J > 64 * 8 * 16)
        launch_fused_sweep_p<T, PH0, true, 16>(C, a, d, it, sfp, sg, sfo, s);
      else
        launch_fused_sweep_p<T, PH0, true, 8>(C, a, d, it, sfp, sg, sfo, s);
      return;
    }
  }
  launch_fused_sweep_p<T, PH0, false, 8>(C, a, d, it, sfp, sg, sfo, s);
}

// Launch configurations of the two passes (10*row + col); the path runs configuration 0, the
// others are kept from the round-1 A/B timing (profiles/r01_microbench_sk_variants.json).
//   row: 0 wave/row CH 8 | 1 wave/row CH 4 | 2 wave/row CH 16 | 3 4 waves/row CH 12 | 4 2 waves/row CH 8
//   col: 0 fused 16 cols CH 16 | 1 split 64-col CH 8 + combine | 2 fused 8 cols CH 12 | 3 split CH 4
// Row 0 = fastest measured at B = 3000 (profiles/r01_microbench_sk_variants.json); column 0 up
// to I = 4096, column 1 above (sk_iter_t).
template <typename T, bool KNOPP>
static void launch_row(int rv, const T* C, const SkArgs& a, const SkDev& d, int it, int si,
                       int so, hipStream_t s) {
  const int I = a.I;
  switch (rv) {
    case 1: hipLaunchKernelGGL((k_sk_row<T, KNOPP, 4, 1>), dim3(div_up(I, 4)), dim3(256), 0, s, C, a, d, it, si, so); break;
    case 2: hipLaunchKernelGGL((k_sk_row<T, KNOPP, 16, 1>), dim3(div_up(I, 4)), dim3(256), 0, s, C, a, d, it, si, so); break;
    case 3: hipLaunchKernelGGL((k_sk_row<T, KNOPP, 12, 4>), dim3(I), dim3(256), 0, s, C, a, d, it, si, so); break;
    case 4: hipLaunchKernelGGL((k_sk_row<T, KNOPP, 8, 2>), dim3(div_up(I, 2)), dim3(256), 0, s, C, a, d, it, si, so); break;
    default: hipLaunchKernelGGL((k_sk_row<T, KNOPP, 8, 1>), dim3(div_up(I, 4)), dim3(256), 0, s, C, a, d, it, si, so); break;
  }
}

static int col_splits(int I, int J) {
  const int strips = (J + 63) / 64;
  int ns = (512 + strips - 1) / strips;
  const int by_rows = (I + 63) / 64;
  ns = ns > by_rows ? by_rows : ns;
  ns = ns > kMaxSplits ? kMaxSplits : ns;
  return ns < 1 ? 1 : ns;
}

template <typename T, bool KNOPP>
static void launch_col(int cv, const T* C, const SkArgs& a, SkDev& d, int it, int sf, int sgp,
                       int sgo, hipStream_t s) {
  const int J = a.J;
  switch (cv) {
    case 0:
      d.ncb = div_up(J, 16);
      hipLaunchKernelGGL((k_sk_col_fused<T, KNOPP, 16, 16>), dim3(d.ncb), dim3(1024), 0, s, C, a, d, it, sf, sgp, sgo);
      break;
    case 2:
      d.ncb = div_up(J, 8);
      hipLaunchKernelGGL((k_sk_col_fused<T, KNOPP, 8, 12>), dim3(d.ncb), dim3(1024), 0, s, C, a, d, it, sf, sgp, sgo);
      break;
    default: {  // 1, 3: split + combine
      const int ns = col_splits(a.I, J);
      const int rps = (a.I + ns - 1) / ns;
      d.ncb = div_up(J, 256);
      if (cv == 3)
        hipLaunchKernelGGL((k_sk_col_part<T, KNOPP, 4>), dim3(div_up(J, 64), ns), dim3(1024), 0, s, C, a, d, sf, rps);
      else
        hipLaunchKernelGGL((k_sk_col_part<T, KNOPP, 8>), dim3(div_up(J, 64), ns), dim3(1024), 0, s, C, a, d, sf, rps);
      hipLaunchKernelGGL(k_sk_col_combine<KNOPP>, dim3(d.ncb), dim3(256), 0, s, a, d, ns, sgp, sgo);
    }
  }
}

template <typename T>
static int sk_iter_t(const gnnea_sinkhorn* p, int first, int count, hipStream_t s) {
  SkArgs a = sk_args(p);
  SkDev d = sk_dev(p);
  // default pass configuration: the fused column pass serialises I / 64 rows per thread, the
  // split pass (row splits + combine) fills the chip at large I: 1.065 -> 0.780 ms per KNOPP
  // iteration at B = 15000, equal within 5 % at B = 3000 (tools/dbg/sk_log_cfg.py)
  const int rv = 0, cv = p->I > 4096 ? 1 : 0;
  const dim3 gabs(div_up(p->I, 4));
  const T* C = (const T*)p->C;
  const bool fused = fused_applies(p);
  for (int it = first; it < first + count; ++it) {
    const int cur = it & 1, prev = (it + 1) & 1;
    if (p->mode == GNNEA_SK_KNOPP && fused) {
      // column update from the previous sweep's partials (P(u_prev, v_prev)), then the sweep
      d.ncb = div_up(a.J, 16);
      hipLaunchKernelGGL(k_lsk_colfin<T>, dim3(d.ncb), dim3(1024), 0, s, C, a, d,
                         fused_wgs(a.I), prev, prev, cur);
      launch_fused_sweep<T, false>(C, a, d, it, prev, cur, cur, s);
      hipLaunchKernelGGL(k_lsk_fix<T>, dim3(fused_wgs(a.I)), dim3(64 * kFW), 0, s, C, a, d, it,
                           prev, cur, cur, fused_rpw(a.I));
    } else if (p->mode == GNNEA_SK_KNOPP) {
      launch_col<T, true>(cv, C, a, d, it, prev, prev, cur, s);  // sets d.ncb for the row pass
      launch_row<T, true>(rv, C, a, d, it, cur, cur, s);
    } else {
      launch_row<T, false>(rv, C, a, d, it, prev, cur, s);
      launch_col<T, false>(cv, C, a, d, it, cur, prev, cur, s);
      hipLaunchKernelGGL(k_sk_absorb_rows<T>, gabs, dim3(256), 0, s, C, a, d, it, cur,
                         p->max_iter, 0);
      hipLaunchKernelGGL(k_sk_absorb_final, dim3(1), dim3(1024), 0, s, a, d, it, cur,
                         p->max_iter, 0, p->tol);
    }
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}


int64_t ws_bytes(int I, int J) {
  if (I < 1 || J < 1) return GNNEA_EINVAL;
  return sk_plan(I, J).total;
}

int init(const gnnea_sinkhorn* p, void* stream) {
  if (!sk_valid(p)) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  SkArgs a = sk_args(p);
  SkDev d = sk_dev(p);
  const int n = p->I > p->J ? p->I : p->J;
  hipLaunchKernelGGL(k_sk_logw, dim3(div_up(n, 256)), dim3(256), 0, s, p->a, p->b, p->I, p->J,
                     (double*)a.la, (double*)a.lb);
  hipLaunchKernelGGL(k_sk_init, dim3(div_up(n > 32 ? n : 32, 256)), dim3(256), 0, s, a, d,
                     p->tol);
  GNNEA_LAUNCH_CHECK();
  if (p->mode == GNNEA_SK_KNOPP) {
    const int nb = div_up((int64_t)p->I * p->J, 256) < 2048 ? div_up((int64_t)p->I * p->J, 256)
                                                             : 2048;
    if (p->c_dtype == GNNEA_F32)
      hipLaunchKernelGGL(k_sk_cscan<float>, dim3(nb), dim3(256), 0, s, (const float*)p->C, p->I,
                         p->J, p->ldc, -a.inv_eps, d.st);
    else
      hipLaunchKernelGGL(k_sk_cscan<double>, dim3(nb), dim3(256), 0, s, (const double*)p->C,
                         p->I, p->J, p->ldc, -a.inv_eps, d.st);
    GNNEA_LAUNCH_CHECK();
    if (fused_applies(p)) {  // the table, then the partials of v_0 K^T u_0 (slot 1: u_0, v_0)
      hipLaunchKernelGGL(k_lsk_tab, dim3(div_up(kFTab, 256)), dim3(256), 0, s, d.ftab);
      if (p->c_dtype == GNNEA_F32)
        launch_fused_sweep<float, true>((const float*)p->C, a, d, 0, 1, 1, 1, s);
      else
        launch_fused_sweep<double, true>((const double*)p->C, a, d, 0, 1, 1, 1, s);
      GNNEA_LAUNCH_CHECK();
    }
  }
  if (p->mode != GNNEA_SK_KNOPP) {  // initial transport = sum K0 . C   (sinkhorn_loss.py:195)
    const dim3 grow(div_up(p->I, 4));
    if (p->c_dtype == GNNEA_F32)
      hipLaunchKernelGGL(k_sk_absorb_rows<float>, grow, dim3(256), 0, s, (const float*)p->C, a,
                         d, 0, 0, p->max_iter, 1);
    else
      hipLaunchKernelGGL(k_sk_absorb_rows<double>, grow, dim3(256), 0, s, (const double*)p->C,
                         a, d, 0, 0, p->max_iter, 1);
    hipLaunchKernelGGL(k_sk_absorb_final, dim3(1), dim3(1024), 0, s, a, d, 0, 0, p->max_iter, 1,
                       p->tol);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

int iterate(const gnnea_sinkhorn* p, int first, int count, void* stream) {
  if (!sk_valid(p) || first < 0 || count < 1) return GNNEA_EINVAL;
  if (p->c_dtype == GNNEA_F32) return sk_iter_t<float>(p, first, count, (hipStream_t)stream);
  return sk_iter_t<double>(p, first, count, (hipStream_t)stream);
}

int finish(const gnnea_sinkhorn* p, void* plan, int plan_dtype, int64_t ldp, double* row_sum,
           double* col_sum, void* stream) {
  if (!sk_valid(p)) return GNNEA_EINVAL;
  if (plan && plan_dtype != GNNEA_F32 && plan_dtype != GNNEA_F64) return GNNEA_EINVAL;
  if (plan && ldp < p->J) return GNNEA_EINVAL;
  // final potentials: the status block's slot after a break, else those of iteration
  // iters_run-1 (iters_run == 0: the initial u = 1/I, v = 1/J)
  hipStream_t s = (hipStream_t)stream;
  SkArgs a = sk_args(p);
  SkDev d = sk_dev(p);
  const int slot = p->iters_run;
  const dim3 grow(div_up(p->I, 4));
#define GNNEA_PLAN(T, PT)                                                                   \
  hipLaunchKernelGGL((k_sk_plan<T, PT>), grow, dim3(256), 0, s, (const T*)p->C, a, d, slot, \
                     (PT*)plan, ldp, row_sum)
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
    const int ns = std::max(1, std::min(kMaxSplits, div_up(p->I, 256)));
    const dim3 gcs(div_up(p->J, 256), ns);
    if (p->c_dtype == GNNEA_F32)
      hipLaunchKernelGGL(k_sk_colsum<float>, gcs, dim3(256), 0, s, (const float*)p->C, a, d,
                         slot, d.pm);
    else
      hipLaunchKernelGGL(k_sk_colsum<double>, gcs, dim3(256), 0, s, (const double*)p->C, a, d,
                         slot, d.pm);
    GNNEA_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sk_colsum_fin, dim3(div_up(p->J, 256)), dim3(256), 0, s, d.pm, ns, p->J,
                       col_sum);
    GNNEA_LAUNCH_CHECK();
  }
  return 0;
}

}  // namespace sklog
}  // namespace gnnea
