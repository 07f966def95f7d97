// a2-a4. CSR neighbour aggregation  Y = epilogue(A · X)
// (replaces torch.spmm(adj, hidden) at layers/layers.py:35 and :64, the act at :38/:67 and the
//  HighWay blend at :69-76).
//
// Gather model: per SpMM the kernel must move
//     4(N+1) + 8E + 4·E·D + 4·N·D bytes,
// dominated by the E·D neighbour-row gathers.  Layout of the work:
//   * one wave (64 lanes) per destination row, 4 rows per 256-thread workgroup;
//   * lane l owns float4 chunks l, l+64, ... of the feature row (16 B per lane per load:
//     a wave-instruction moves up to 1 KiB of one neighbour row, fully coalesced);
//   * the row's (col, val) pairs are loaded 64 at a time, one per lane, and broadcast to the
//     wave with v_readlane (wave-uniform, no LDS);
//   * neighbours are unrolled by 4 so every lane keeps 4 x NCH independent 16-B loads in flight;
//   * workgroups are remapped XCD-contiguously so consecutive rows (ring neighbours, self loops)
//     hit the same XCD's L2.
// No atomics, no LDS; results are deterministic (fixed CSR order, fixed fma chain per lane).
#include "common.h"

namespace gnnea {

enum { EPI_ACT = 0, EPI_HIGHWAY = 1 };

// TX: storage of the gathered rows X and of gate_pre / resid; TY: storage of Y and the saved
// S / g (float or bf16_t; arithmetic is fp32 either way).
template <typename TX, typename TY>
struct HighwayArgs {
  const typename Vec4<TX>::raw* gate_pre;
  int64_t ldg4;
  const float4* bias4;  // fp32 bias_gate (nullable)
  const typename Vec4<TX>::raw* resid;
  int64_t ldr4;
  typename Vec4<TY>::raw* save_s;
  typename Vec4<TY>::raw* save_g;
  int64_t lds4;
  float beta;  // EPI_ACT: Y = act(A.X + beta*Y)  (partial aggregations, dist halo overlap)
};

template <int ACT>
__device__ __forceinline__ float4 act4(float4 v) {
  return make_float4(act_fwd<ACT>(v.x), act_fwd<ACT>(v.y), act_fwd<ACT>(v.z), act_fwd<ACT>(v.w));
}

__device__ __forceinline__ float sigm(float x) { return gate_sigmoid(x); }

template <int ACT, int EPI, int NCH, typename TX, typename TY>
__global__ __launch_bounds__(256) void k_spmm_v4(const int32_t* __restrict__ rowptr,
                                                 const int32_t* __restrict__ col,
                                                 const float* __restrict__ val, int n_rows, int D4,
                                                 const typename Vec4<TX>::raw* __restrict__ X,
                                                 int64_t ldx4,
                                                 typename Vec4<TY>::raw* __restrict__ Y,
                                                 int64_t ldy4, HighwayArgs<TX, TY> hw) {
  typedef typename Vec4<TX>::raw RX;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptr[row], end = rowptr[row + 1];

  float4 acc[NCH];
  bool own[NCH];
#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    acc[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    own[q] = lane + 64 * q < D4;
  }

  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int mc = lane < cnt ? col[base + lane] : 0;
    const float mv = lane < cnt ? val[base + lane] : 0.f;
    int k = 0;
    for (; k + 4 <= cnt; k += 4) {
      const int j0 = readlane_i(mc, k), j1 = readlane_i(mc, k + 1);
      const int j2 = readlane_i(mc, k + 2), j3 = readlane_i(mc, k + 3);
      const float v0 = readlane_f(mv, k), v1 = readlane_f(mv, k + 1);
      const float v2 = readlane_f(mv, k + 2), v3 = readlane_f(mv, k + 3);
      const RX* x0 = X + (int64_t)j0 * ldx4 + lane;
      const RX* x1 = X + (int64_t)j1 * ldx4 + lane;
      const RX* x2 = X + (int64_t)j2 * ldx4 + lane;
      const RX* x3 = X + (int64_t)j3 * ldx4 + lane;
      RX r0[NCH], r1[NCH], r2[NCH], r3[NCH];
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        if (own[q]) {
          r0[q] = x0[64 * q];
          r1[q] = x1[64 * q];
          r2[q] = x2[64 * q];
          r3[q] = x3[64 * q];
        }
      }
#pragma unroll
      for (int q = 0; q < NCH; ++q) {
        if (own[q]) {
          acc[q] = f4_fma(v0, Vec4<TX>::get(r0[q]), acc[q]);
          acc[q] = f4_fma(v1, Vec4<TX>::get(r1[q]), acc[q]);
          acc[q] = f4_fma(v2, Vec4<TX>::get(r2[q]), acc[q]);
          acc[q] = f4_fma(v3, Vec4<TX>::get(r3[q]), acc[q]);
        }
      }
    }
    for (; k < cnt; ++k) {
      const int j = readlane_i(mc, k);
      const float v = readlane_f(mv, k);
      const RX* xr = X + (int64_t)j * ldx4 + lane;
#pragma unroll
      for (int q = 0; q < NCH; ++q)
        if (own[q]) acc[q] = f4_fma(v, Vec4<TX>::get(xr[64 * q]), acc[q]);
    }
  }

#pragma unroll
  for (int q = 0; q < NCH; ++q) {
    if (!own[q]) continue;
    const int c = lane + 64 * q;
    if constexpr (EPI == EPI_ACT) {
      if (hw.beta != 0.f) {
        const float4 y = Vec4<TY>::get(Y[(int64_t)row * ldy4 + c]);
        acc[q].x = fmaf(hw.beta, y.x, acc[q].x);
        acc[q].y = fmaf(hw.beta, y.y, acc[q].y);
        acc[q].z = fmaf(hw.beta, y.z, acc[q].z);
        acc[q].w = fmaf(hw.beta, y.w, acc[q].w);
      }
    }
    float4 s = act4<ACT>(acc[q]);
    if constexpr (EPI == EPI_ACT) {
      Y[(int64_t)row * ldy4 + c] = Vec4<TY>::put(s);
    } else {
      float4 gp = Vec4<TX>::get(hw.gate_pre[(int64_t)row * hw.ldg4 + c]);
      if (hw.bias4) {
        const float4 b = hw.bias4[c];
        gp.x += b.x; gp.y += b.y; gp.z += b.z; gp.w += b.w;
      }
      const float4 g = make_float4(sigm(gp.x), sigm(gp.y), sigm(gp.z), sigm(gp.w));
      const float4 r = Vec4<TX>::get(hw.resid[(int64_t)row * hw.ldr4 + c]);
      // reference order: transform_gate * support + carry_gate * residual, carry = 1 - g
      float4 o;
      o.x = g.x * s.x + (1.f - g.x) * r.x;
      o.y = g.y * s.y + (1.f - g.y) * r.y;
      o.z = g.z * s.z + (1.f - g.z) * r.z;
      o.w = g.w * s.w + (1.f - g.w) * r.w;
      Y[(int64_t)row * ldy4 + c] = Vec4<TY>::put(o);
      if (hw.save_s) hw.save_s[(int64_t)row * hw.lds4 + c] = Vec4<TY>::put(s);
      if (hw.save_g) hw.save_g[(int64_t)row * hw.lds4 + c] = Vec4<TY>::put(g);
    }
  }
}

// Scalar path for any D / alignment: lane owns columns lane, lane+64, ...
template <int ACT, int EPI, typename TX, typename TY>
__global__ __launch_bounds__(256) void k_spmm_scalar(const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const float* __restrict__ val, int n_rows,
                                                     int D, const TX* __restrict__ X,
                                                     int64_t ldx, TY* __restrict__ Y,
                                                     int64_t ldy, const TX* gate_pre,
                                                     int64_t ldg, const float* bias,
                                                     const TX* resid, int64_t ldr,
                                                     TY* save_s, TY* save_g, int64_t lds,
                                                     float beta) {
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int row = blk * 4 + wave_id();
  if (row >= n_rows) return;
  const int lane = lane_id();
  const int beg = rowptr[row], end = rowptr[row + 1];
  for (int c0 = 0; c0 < D; c0 += 64) {
    const int c = c0 + lane;
    float acc = 0.f;
    for (int e = beg; e < end; ++e) {
      const int j = col[e];
      if (c < D) acc = fmaf(val[e], to_f32<TX>(X[(int64_t)j * ldx + c]), acc);
    }
    if (c >= D) continue;
    if (EPI == EPI_ACT && beta != 0.f) acc = fmaf(beta, to_f32<TY>(Y[(int64_t)row * ldy + c]), acc);
    const float s = act_fwd<ACT>(acc);
    if constexpr (EPI == EPI_ACT) {
      Y[(int64_t)row * ldy + c] = from_f32<TY>(s);
    } else {
      float gp = to_f32<TX>(gate_pre[(int64_t)row * ldg + c]) + (bias ? bias[c] : 0.f);
      const float g = sigm(gp);
      const float r = to_f32<TX>(resid[(int64_t)row * ldr + c]);
      Y[(int64_t)row * ldy + c] = from_f32<TY>(g * s + (1.f - g) * r);
      if (save_s) save_s[(int64_t)row * lds + c] = from_f32<TY>(s);
      if (save_g) save_g[(int64_t)row * lds + c] = from_f32<TY>(g);
    }
  }
}

template <typename T>
static inline bool alv(const void* p) {  // aligned for one Vec4<T> load
  return p == nullptr || (((uintptr_t)p) & (sizeof(typename Vec4<T>::raw) - 1)) == 0;
}

template <int ACT, int EPI, typename TX, typename TY>
static int launch_spmm(const int32_t* rowptr, const int32_t* col, const float* val, int n_rows,
                       int D, const TX* X, int64_t ldx, TY* Y, int64_t ldy,
                       const TX* gate_pre, int64_t ldg, const float* bias, const TX* resid,
                       int64_t ldr, TY* save_s, TY* save_g, int64_t lds, float beta,
                       hipStream_t stream) {
  const int nb = div_up(n_rows, 4);
  bool vec = (D % 4 == 0) && (ldx % 4 == 0) && (ldy % 4 == 0) && alv<TX>(X) && alv<TY>(Y);
  if (EPI == EPI_HIGHWAY)
    vec = vec && (ldg % 4 == 0) && (ldr % 4 == 0) && (lds % 4 == 0) && alv<TX>(gate_pre) &&
          alv<float>(bias) && alv<TX>(resid) && alv<TY>(save_s) && alv<TY>(save_g);
  const int D4 = D / 4;
  if (vec && D4 <= 256) {
    typedef typename Vec4<TX>::raw RX;
    typedef typename Vec4<TY>::raw RY;
    HighwayArgs<TX, TY> hw{(const RX*)gate_pre, ldg / 4, (const float4*)bias, (const RX*)resid,
                           ldr / 4, (RY*)save_s, (RY*)save_g, lds / 4, beta};
    const int nch = (D4 + 63) / 64;
#define GNNEA_SPMM_CASE(N)                                                                    \
  case N:                                                                                     \
    hipLaunchKernelGGL((k_spmm_v4<ACT, EPI, N, TX, TY>), dim3(nb), dim3(256), 0, stream,      \
                       rowptr, col, val, n_rows, D4, (const RX*)X, ldx / 4, (RY*)Y, ldy / 4,  \
                       hw);                                                                   \
    break;
    switch (nch) {
      GNNEA_SPMM_CASE(1)
      GNNEA_SPMM_CASE(2)
      GNNEA_SPMM_CASE(3)
      GNNEA_SPMM_CASE(4)
      default: break;
    }
#undef GNNEA_SPMM_CASE
  } else {
    hipLaunchKernelGGL((k_spmm_scalar<ACT, EPI, TX, TY>), dim3(nb), dim3(256), 0, stream, rowptr,
                       col, val, n_rows, D, X, ldx, Y, ldy, gate_pre, ldg, bias, resid, ldr,
                       save_s, save_g, lds, beta);
  }
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <int EPI, typename TX, typename TY>
static int dispatch_act(int act, const int32_t* rowptr, const int32_t* col, const float* val,
                        int n_rows, int D, const TX* X, int64_t ldx, TY* Y, int64_t ldy,
                        const TX* gate_pre, int64_t ldg, const float* bias, const TX* resid,
                        int64_t ldr, TY* save_s, TY* save_g, int64_t lds, float beta,
                        hipStream_t s) {
#define GNNEA_ACT_CASE(A)                                                                     \
  case A:                                                                                     \
    return launch_spmm<A, EPI, TX, TY>(rowptr, col, val, n_rows, D, X, ldx, Y, ldy, gate_pre, \
                                       ldg, bias, resid, ldr, save_s, save_g, lds, beta, s);
  switch (act) {
    GNNEA_ACT_CASE(GNNEA_ACT_IDENTITY)
    GNNEA_ACT_CASE(GNNEA_ACT_RELU)
    GNNEA_ACT_CASE(GNNEA_ACT_ELU)
    GNNEA_ACT_CASE(GNNEA_ACT_LEAKY_RELU)
    GNNEA_ACT_CASE(GNNEA_ACT_SIGMOID)
    GNNEA_ACT_CASE(GNNEA_ACT_TANH)
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_ACT_CASE
}

// ---- elementwise backward helpers ----------------------------------------------------------

template <int ACT, typename T>
__global__ void k_act_bwd(const T* __restrict__ dY, const T* __restrict__ Y, T* __restrict__ G,
                          int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride)
    G[i] = from_f32<T>(to_f32<T>(dY[i]) * act_grad_from_out<ACT>(to_f32<T>(Y[i])));
}

template <int ACT, typename T>
__global__ void k_highway_bwd(const T* __restrict__ dY, const T* __restrict__ S,
                              const T* __restrict__ Gt, const T* __restrict__ R, int64_t ld,
                              int64_t n_rows, int D, T* __restrict__ dS_pre, int64_t ld_ds,
                              int64_t cs_ds, T* __restrict__ dgate, int64_t ld_dg,
                              T* __restrict__ dresid, int64_t ld_dr) {
  const int64_t n = n_rows * (int64_t)D;
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; t < n; t += stride) {
    const int64_t r = t / D, c = t - r * D;
    const int64_t i = r * ld + c;
    const float dy = to_f32<T>(dY[i]), s = to_f32<T>(S[i]), g = to_f32<T>(Gt[i]);
    const float x = to_f32<T>(R[i]);
    // dS_pre at (c / 64)·cs_ds + r·ld_ds + c % 64: cs_ds = 64 row-major, or the slice-major
    // table the transposed sliced aggregation reads (ld_ds = 64, cs_ds = slice stride)
    dS_pre[(c >> 6) * cs_ds + r * ld_ds + (c & 63)] =
        from_f32<T>(dy * g * act_grad_from_out<ACT>(s));
    dgate[r * ld_dg + c] = from_f32<T>(dy * (s - x) * g * (1.f - g));
    if (dresid) dresid[r * ld_dr + c] = from_f32<T>(dy * (1.f - g));
  }
}

// Row-wise vector form (D, every ld and cs_ds % 4 == 0, 16-B / 8-B aligned bases): one wave per
// row, lane = 4-column chunk, no per-element 64-bit index division; 4 consecutive columns stay
// inside one 64-column slice of a slice-major dS_pre.
template <int ACT, typename T>
__global__ __launch_bounds__(256) void k_highway_bwd_v4(
    const T* __restrict__ dY, const T* __restrict__ S, const T* __restrict__ Gt,
    const T* __restrict__ R, int64_t ld, int64_t n_rows, int D, T* __restrict__ dS_pre,
    int64_t ld_ds, int64_t cs_ds, T* __restrict__ dgate, int64_t ld_dg, T* __restrict__ dresid,
    int64_t ld_dr) {
  typedef typename Vec4<T>::raw V;
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave_id(); r < n_rows; r += nw) {
    for (int c = 4 * lane; c < D; c += 256) {
      const int64_t i = r * ld + c;
      const float4 dy = Vec4<T>::get(*(const V*)(dY + i)), sv = Vec4<T>::get(*(const V*)(S + i));
      const float4 g = Vec4<T>::get(*(const V*)(Gt + i)), x = Vec4<T>::get(*(const V*)(R + i));
      const float dyv[4] = {dy.x, dy.y, dy.z, dy.w}, s4[4] = {sv.x, sv.y, sv.z, sv.w};
      const float g4[4] = {g.x, g.y, g.z, g.w}, x4[4] = {x.x, x.y, x.z, x.w};
      float ds[4], dg[4], dr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ds[e] = dyv[e] * g4[e] * act_grad_from_out<ACT>(s4[e]);
        dg[e] = dyv[e] * (s4[e] - x4[e]) * g4[e] * (1.f - g4[e]);
        dr[e] = dyv[e] * (1.f - g4[e]);
      }
      *(V*)(dS_pre + (c >> 6) * cs_ds + r * ld_ds + (c & 63)) =
          Vec4<T>::put(make_float4(ds[0], ds[1], ds[2], ds[3]));
      *(V*)(dgate + r * ld_dg + c) = Vec4<T>::put(make_float4(dg[0], dg[1], dg[2], dg[3]));
      if (dresid)
        *(V*)(dresid + r * ld_dr + c) = Vec4<T>::put(make_float4(dr[0], dr[1], dr[2], dr[3]));
    }
  }
}

// The fused HighWay layer's backward without a saved gate: g = sigmoid(gate_pre + bias_gate)
// recomputed from the slice-major projection table Zs (gate_pre at column goff + c, the same
// float operations as the forward epilogue, so the same g bit for bit) -- the forward then does
// not write G (N·D·4 bytes per layer).  dS_pre slice-major as gnnea_highway_bwd_sliced_f32.
template <int ACT>
__global__ __launch_bounds__(256) void k_highway_bwd_zg(
    const float* __restrict__ dY, const float* __restrict__ S, const float4* __restrict__ Zs,
    int64_t zs4, int goff, const float* __restrict__ bias, const float* __restrict__ R, int64_t ld,
    int64_t n_rows, int D, float* __restrict__ dS_s, int64_t cs_ds, float* __restrict__ dgate,
    int64_t ld_dg, float* __restrict__ dresid, int64_t ld_dr) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave_id(); r < n_rows; r += nw) {
    for (int c = 4 * lane; c < D; c += 256) {
      const int64_t i = r * ld + c;
      const int gc = goff + c;
      const float4 dy = *(const float4*)(dY + i), sv = *(const float4*)(S + i);
      const float4 x = *(const float4*)(R + i);
      float4 gp = Zs[(int64_t)(gc >> 6) * zs4 + r * 16 + ((gc & 63) >> 2)];
      if (bias) {
        const float4 bv = *(const float4*)(bias + c);
        gp.x += bv.x; gp.y += bv.y; gp.z += bv.z; gp.w += bv.w;
      }
      const float dyv[4] = {dy.x, dy.y, dy.z, dy.w}, s4[4] = {sv.x, sv.y, sv.z, sv.w};
      const float gp4[4] = {gp.x, gp.y, gp.z, gp.w}, x4[4] = {x.x, x.y, x.z, x.w};
      float ds[4], dg[4], dr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = gate_sigmoid(gp4[e]);  // as sigm_f in the forward epilogue
        ds[e] = dyv[e] * g * act_grad_from_out<ACT>(s4[e]);
        dg[e] = dyv[e] * (s4[e] - x4[e]) * g * (1.f - g);
        dr[e] = dyv[e] * (1.f - g);
      }
      *(float4*)(dS_s + (c >> 6) * cs_ds + r * 64 + (c & 63)) = make_float4(ds[0], ds[1], ds[2], ds[3]);
      *(float4*)(dgate + r * ld_dg + c) = make_float4(dg[0], dg[1], dg[2], dg[3]);
      if (dresid)
        *(float4*)(dresid + r * ld_dr + c) = make_float4(dr[0], dr[1], dr[2], dr[3]);
    }
  }
}

// The same backward without S: act' from the forward's relu sign mask (ACT relu; identity: 1)
// and S - x from the output, g (S - x) = out - x, so
//   dS_pre = dY g act',  dgate = dY (out - x)(1 - g),  dresid = dY (1 - g).
template <int ACT>
__global__ __launch_bounds__(256) void k_highway_bwd_zgm(
    const float* __restrict__ dY, const float* __restrict__ O, const float4* __restrict__ Zs,
    int64_t zs4, int goff, const float* __restrict__ bias, const float* __restrict__ R, int64_t ld,
    int64_t n_rows, int D, const uint8_t* __restrict__ mask, int64_t ldm,
    float* __restrict__ dS_s, int64_t cs_ds, float* __restrict__ dgate, int64_t ld_dg,
    float* __restrict__ dresid, int64_t ld_dr) {
  const int lane = lane_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave_id(); r < n_rows; r += nw) {
    for (int c = 4 * lane; c < D; c += 256) {
      const int64_t i = r * ld + c;
      const int gc = goff + c;
      const float4 dy = *(const float4*)(dY + i), ov = *(const float4*)(O + i);
      const float4 x = *(const float4*)(R + i);
      float4 gp = Zs[(int64_t)(gc >> 6) * zs4 + r * 16 + ((gc & 63) >> 2)];
      uint32_t mb = 15u;
      if constexpr (ACT == GNNEA_ACT_RELU) mb = mask[r * ldm + 16 * (c >> 6) + ((c & 63) >> 2)];
      if (bias) {
        const float4 bv = *(const float4*)(bias + c);
        gp.x += bv.x; gp.y += bv.y; gp.z += bv.z; gp.w += bv.w;
      }
      const float dyv[4] = {dy.x, dy.y, dy.z, dy.w}, o4[4] = {ov.x, ov.y, ov.z, ov.w};
      const float gp4[4] = {gp.x, gp.y, gp.z, gp.w}, x4[4] = {x.x, x.y, x.z, x.w};
      float ds[4], dg[4], dr[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float g = gate_sigmoid(gp4[e]);  // as sigm_f in the forward epilogue
        ds[e] = ((mb >> e) & 1u) ? dyv[e] * g : 0.f;
        dg[e] = dyv[e] * (o4[e] - x4[e]) * (1.f - g);
        dr[e] = dyv[e] * (1.f - g);
      }
      *(float4*)(dS_s + (c >> 6) * cs_ds + r * 64 + (c & 63)) = make_float4(ds[0], ds[1], ds[2], ds[3]);
      *(float4*)(dgate + r * ld_dg + c) = make_float4(dg[0], dg[1], dg[2], dg[3]);
      if (dresid)
        *(float4*)(dresid + r * ld_dr + c) = make_float4(dr[0], dr[1], dr[2], dr[3]);
    }
  }
}

template <typename T>
static int act_bwd_t(const T* dY, const T* Y, T* G, int64_t n, int act, hipStream_t s) {
  if (n < 0) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!dY || !Y || !G) return GNNEA_EINVAL;
  const int nb = (int)(n / 256 + 1 < 8192 ? n / 256 + 1 : 8192);
#define GNNEA_AB(A) hipLaunchKernelGGL((k_act_bwd<A, T>), dim3(nb), dim3(256), 0, s, dY, Y, G, n)
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_AB(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_AB(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_AB(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_AB(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_AB(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_AB(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_AB
  GNNEA_LAUNCH_CHECK();
  return 0;
}

template <typename T>
static int highway_bwd_t(const T* dY, const T* S, const T* G, const T* resid, int64_t ld,
                         int64_t n_rows, int32_t D, T* dS_pre, int64_t ld_ds, T* dgate,
                         int64_t ld_dg, T* dresid, int64_t ld_dr, int act, hipStream_t s,
                         int64_t cs_ds = 64) {
  if (n_rows < 0 || D < 0 || ld < D || ld_dg < D || (dresid && ld_dr < D)) return GNNEA_EINVAL;
  if (cs_ds == 64 ? ld_ds < D : (ld_ds != 64 || cs_ds < n_rows * 64)) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!dY || !S || !G || !resid || !dS_pre || !dgate) return GNNEA_EINVAL;
  const int64_t n = n_rows * (int64_t)D;
  const int nb = (int)(n / 256 + 1 < 8192 ? n / 256 + 1 : 8192);
  constexpr uintptr_t al = sizeof(typename Vec4<T>::raw) - 1;
  const bool v4 = D % 4 == 0 && ld % 4 == 0 && ld_ds % 4 == 0 && cs_ds % 4 == 0 &&
                  ld_dg % 4 == 0 && (!dresid || ld_dr % 4 == 0) &&
                  !(((uintptr_t)dY | (uintptr_t)S | (uintptr_t)G | (uintptr_t)resid |
                     (uintptr_t)dS_pre | (uintptr_t)dgate | (uintptr_t)dresid) & al);
  const int nbv = (int)((n_rows + 3) / 4 < 16384 ? (n_rows + 3) / 4 : 16384);
#define GNNEA_HWB(A)                                                                          \
  if (v4)                                                                                     \
    hipLaunchKernelGGL((k_highway_bwd_v4<A, T>), dim3(nbv), dim3(256), 0, s, dY, S, G, resid, \
                       ld, n_rows, D, dS_pre, ld_ds, cs_ds, dgate, ld_dg, dresid, ld_dr);     \
  else                                                                                        \
    hipLaunchKernelGGL((k_highway_bwd<A, T>), dim3(nb), dim3(256), 0, s, dY, S, G, resid, ld, \
                       n_rows, D, dS_pre, ld_ds, cs_ds, dgate, ld_dg, dresid, ld_dr)
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_HWB(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_HWB(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_HWB(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_HWB(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_HWB(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_HWB(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_HWB
  GNNEA_LAUNCH_CHECK();
  return 0;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_spmm_csr_f32(const int32_t* rowptr, const int32_t* col, const float* val,
                                  int32_t n_rows, int32_t D, const float* X, int64_t ldx,
                                  float* Y, int64_t ldy, int act, void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !X || !Y || ldx < D || ldy < D) return GNNEA_EINVAL;
  return dispatch_act<EPI_ACT, float, float>(act, rowptr, col, val, n_rows, D, X, ldx, Y, ldy,
                                             nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, 0,
                                             0.f, (hipStream_t)stream);
}

extern "C" int gnnea_spmm_csr_beta_f32(const int32_t* rowptr, const int32_t* col,
                                       const float* val, int32_t n_rows, int32_t D,
                                       const float* X, int64_t ldx, float beta, float* Y,
                                       int64_t ldy, int act, void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !X || !Y || ldx < D || ldy < D) return GNNEA_EINVAL;
  return dispatch_act<EPI_ACT, float, float>(act, rowptr, col, val, n_rows, D, X, ldx, Y, ldy,
                                             nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, 0,
                                             beta, (hipStream_t)stream);
}

extern "C" int gnnea_spmm_highway_f32(const int32_t* rowptr, const int32_t* col,
                                      const float* val, int32_t n_rows, int32_t D,
                                      const float* X, int64_t ldx, const float* gate_pre,
                                      int64_t ldg, const float* bias_gate, const float* resid,
                                      int64_t ldr, float* Y, int64_t ldy, float* save_s,
                                      float* save_g, int64_t lds, int act, void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !X || !Y || !gate_pre || !resid) return GNNEA_EINVAL;
  if (ldx < D || ldy < D || ldg < D || ldr < D || ((save_s || save_g) && lds < D))
    return GNNEA_EINVAL;
  return dispatch_act<EPI_HIGHWAY, float, float>(act, rowptr, col, val, n_rows, D, X, ldx, Y,
                                                 ldy, gate_pre, ldg, bias_gate, resid, ldr,
                                                 save_s, save_g, lds, 0.f, (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_f32(const float* dY, const float* Y, float* G, int64_t n, int act,
                                 void* stream) {
  return act_bwd_t<float>(dY, Y, G, n, act, (hipStream_t)stream);
}

extern "C" int gnnea_highway_bwd_f32(const float* dY, const float* S, const float* G,
                                     const float* resid, int64_t ld, int64_t n_rows, int32_t D,
                                     float* dS_pre, float* dgate, float* dresid, int act,
                                     void* stream) {
  return highway_bwd_t<float>(dY, S, G, resid, ld, n_rows, D, dS_pre, ld, dgate, ld, dresid, ld,
                              act, (hipStream_t)stream);
}

extern "C" int gnnea_highway_bwd_ld_f32(const float* dY, const float* S, const float* G,
                                        const float* resid, int64_t ld, int64_t n_rows, int32_t D,
                                        float* dS_pre, int64_t ld_ds, float* dgate, int64_t ld_dg,
                                        float* dresid, int64_t ld_dr, int act, void* stream) {
  return highway_bwd_t<float>(dY, S, G, resid, ld, n_rows, D, dS_pre, ld_ds, dgate, ld_dg,
                              dresid, ld_dr, act, (hipStream_t)stream);
}

// dS_pre written slice-major ([ceil(D/64)][n_rows][64], slice stride sstride): the input of the
// transposed sliced aggregation of the fused HighWay layer's backward
extern "C" int gnnea_highway_bwd_sliced_f32(const float* dY, const float* S, const float* G,
                                            const float* resid, int64_t ld, int64_t n_rows,
                                            int32_t D, float* dS_s, int64_t sstride,
                                            float* dgate, int64_t ld_dg, float* dresid,
                                            int64_t ld_dr, int act, void* stream) {
  if (sstride == 64) return GNNEA_EINVAL;  // 64 is the row-major code of the kernel
  return highway_bwd_t<float>(dY, S, G, resid, ld, n_rows, D, dS_s, 64, dgate, ld_dg, dresid,
                              ld_dr, act, (hipStream_t)stream, sstride);
}

// as gnnea_highway_bwd_sliced_zg_f32 without S: the forward's output and (relu) its sign mask
extern "C" int gnnea_highway_bwd_sliced_zgm_f32(const float* dY, const float* O, const float* Zs,
                                                int64_t zs_stride, int32_t goff,
                                                const float* bias_gate, const float* resid,
                                                int64_t ld, int64_t n_rows, int32_t D,
                                                const uint8_t* mask, int64_t ldm, float* dS_s,
                                                int64_t sstride, float* dgate, int64_t ld_dg,
                                                float* dresid, int64_t ld_dr, int act,
                                                void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!dY || !O || !Zs || !resid || !dS_s || !dgate) return GNNEA_EINVAL;
  if (act != GNNEA_ACT_RELU && act != GNNEA_ACT_IDENTITY) return GNNEA_EINVAL;
  if (act == GNNEA_ACT_RELU && (!mask || ldm < 16 * ((D + 63) / 64))) return GNNEA_EINVAL;
  const uintptr_t al = (uintptr_t)dY | (uintptr_t)O | (uintptr_t)Zs | (uintptr_t)resid |
                       (uintptr_t)dS_s | (uintptr_t)dgate | (uintptr_t)dresid |
                       (uintptr_t)bias_gate;
  if (D % 4 || ld % 4 || ld < D || goff < 0 || goff % 4 || zs_stride % 64 ||
      zs_stride < n_rows * 64 || sstride % 64 || sstride < n_rows * 64 || ld_dg % 4 ||
      ld_dg < D || (dresid && (ld_dr % 4 || ld_dr < D)) || (al & 15))
    return GNNEA_EINVAL;
  const int nbv = (int)((n_rows + 3) / 4 < 16384 ? (n_rows + 3) / 4 : 16384);
  hipStream_t s = (hipStream_t)stream;
  if (act == GNNEA_ACT_RELU)
    hipLaunchKernelGGL((k_highway_bwd_zgm<GNNEA_ACT_RELU>), dim3(nbv), dim3(256), 0, s, dY, O,
                       (const float4*)Zs, zs_stride / 4, goff, bias_gate, resid, ld, n_rows, D,
                       mask, ldm, dS_s, sstride, dgate, ld_dg, dresid, ld_dr);
  else
    hipLaunchKernelGGL((k_highway_bwd_zgm<GNNEA_ACT_IDENTITY>), dim3(nbv), dim3(256), 0, s, dY,
                       O, (const float4*)Zs, zs_stride / 4, goff, bias_gate, resid, ld, n_rows, D,
                       mask, ldm, dS_s, sstride, dgate, ld_dg, dresid, ld_dr);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// as gnnea_highway_bwd_sliced_f32 with the gate recomputed from the projection table (above)
extern "C" int gnnea_highway_bwd_sliced_zg_f32(const float* dY, const float* S, const float* Zs,
                                               int64_t zs_stride, int32_t goff,
                                               const float* bias_gate, const float* resid,
                                               int64_t ld, int64_t n_rows, int32_t D,
                                               float* dS_s, int64_t sstride, float* dgate,
                                               int64_t ld_dg, float* dresid, int64_t ld_dr, int act,
                                               void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!dY || !S || !Zs || !resid || !dS_s || !dgate) return GNNEA_EINVAL;
  const uintptr_t al = (uintptr_t)dY | (uintptr_t)S | (uintptr_t)Zs | (uintptr_t)resid |
                       (uintptr_t)dS_s | (uintptr_t)dgate | (uintptr_t)dresid |
                       (uintptr_t)bias_gate;
  if (D % 4 || ld % 4 || ld < D || goff < 0 || goff % 4 || zs_stride % 64 ||
      zs_stride < n_rows * 64 || sstride % 64 || sstride < n_rows * 64 || ld_dg % 4 ||
      ld_dg < D || (dresid && (ld_dr % 4 || ld_dr < D)) || (al & 15))
    return GNNEA_EINVAL;
  const int nbv = (int)((n_rows + 3) / 4 < 16384 ? (n_rows + 3) / 4 : 16384);
  hipStream_t s = (hipStream_t)stream;
#define GNNEA_HZ(A)                                                                            \
  hipLaunchKernelGGL((k_highway_bwd_zg<A>), dim3(nbv), dim3(256), 0, s, dY, S,                \
                     (const float4*)Zs, zs_stride / 4, goff, bias_gate, resid, ld, n_rows, D, \
                     dS_s, sstride, dgate, ld_dg, dresid, ld_dr)
  switch (act) {
    case GNNEA_ACT_IDENTITY: GNNEA_HZ(GNNEA_ACT_IDENTITY); break;
    case GNNEA_ACT_RELU: GNNEA_HZ(GNNEA_ACT_RELU); break;
    case GNNEA_ACT_ELU: GNNEA_HZ(GNNEA_ACT_ELU); break;
    case GNNEA_ACT_LEAKY_RELU: GNNEA_HZ(GNNEA_ACT_LEAKY_RELU); break;
    case GNNEA_ACT_SIGMOID: GNNEA_HZ(GNNEA_ACT_SIGMOID); break;
    case GNNEA_ACT_TANH: GNNEA_HZ(GNNEA_ACT_TANH); break;
    default: return GNNEA_EINVAL;
  }
#undef GNNEA_HZ
  GNNEA_LAUNCH_CHECK();
  return 0;
}

// ---- bf16 storage (cfg-5) ------------------------------------------------------------------

extern "C" int gnnea_spmm_csr_bf16(const int32_t* rowptr, const int32_t* col, const float* val,
                                   int32_t n_rows, int32_t D, const void* X, int64_t ldx,
                                   float beta, void* Y, int64_t ldy, int y_dtype, int act,
                                   void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !X || !Y || ldx < D || ldy < D) return GNNEA_EINVAL;
  if (y_dtype == GNNEA_BF16)
    return dispatch_act<EPI_ACT, bf16_t, bf16_t>(act, rowptr, col, val, n_rows, D,
                                                 (const bf16_t*)X, ldx, (bf16_t*)Y, ldy,
                                                 nullptr, 0, nullptr, nullptr, 0, nullptr,
                                                 nullptr, 0, beta, (hipStream_t)stream);
  if (y_dtype == GNNEA_F32)
    return dispatch_act<EPI_ACT, bf16_t, float>(act, rowptr, col, val, n_rows, D,
                                                (const bf16_t*)X, ldx, (float*)Y, ldy, nullptr,
                                                0, nullptr, nullptr, 0, nullptr, nullptr, 0,
                                                beta, (hipStream_t)stream);
  return GNNEA_EINVAL;
}

extern "C" int gnnea_spmm_highway_bf16(const int32_t* rowptr, const int32_t* col,
                                       const float* val, int32_t n_rows, int32_t D,
                                       const void* X, int64_t ldx, const void* gate_pre,
                                       int64_t ldg, const float* bias_gate, const void* resid,
                                       int64_t ldr, void* Y, int64_t ldy, void* save_s,
                                       void* save_g, int64_t lds, int act, void* stream) {
  if (n_rows < 0 || D < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || D == 0) return 0;
  if (!rowptr || !col || !val || !X || !Y || !gate_pre || !resid) return GNNEA_EINVAL;
  if (ldx < D || ldy < D || ldg < D || ldr < D || ((save_s || save_g) && lds < D))
    return GNNEA_EINVAL;
  return dispatch_act<EPI_HIGHWAY, bf16_t, bf16_t>(
      act, rowptr, col, val, n_rows, D, (const bf16_t*)X, ldx, (bf16_t*)Y, ldy,
      (const bf16_t*)gate_pre, ldg, bias_gate, (const bf16_t*)resid, ldr, (bf16_t*)save_s,
      (bf16_t*)save_g, lds, 0.f, (hipStream_t)stream);
}

extern "C" int gnnea_act_bwd_bf16(const void* dY, const void* Y, void* G, int64_t n, int act,
                                  void* stream) {
  return act_bwd_t<bf16_t>((const bf16_t*)dY, (const bf16_t*)Y, (bf16_t*)G, n, act,
                           (hipStream_t)stream);
}

extern "C" int gnnea_highway_bwd_bf16(const void* dY, const void* S, const void* G,
                                      const void* resid, int64_t ld, int64_t n_rows, int32_t D,
                                      void* dS_pre, void* dgate, void* dresid, int act,
                                      void* stream) {
  return highway_bwd_t<bf16_t>((const bf16_t*)dY, (const bf16_t*)S, (const bf16_t*)G,
                               (const bf16_t*)resid, ld, n_rows, D, (bf16_t*)dS_pre, ld,
                               (bf16_t*)dgate, ld, (bf16_t*)dresid, ld, act, (hipStream_t)stream);
}

extern "C" int gnnea_highway_bwd_ld_bf16(const void* dY, const void* S, const void* G,
                                         const void* resid, int64_t ld, int64_t n_rows,
                                         int32_t D, void* dS_pre, int64_t ld_ds, void* dgate,
                                         int64_t ld_dg, void* dresid, int64_t ld_dr, int act,
                                         void* stream) {
  return highway_bwd_t<bf16_t>((const bf16_t*)dY, (const bf16_t*)S, (const bf16_t*)G,
                               (const bf16_t*)resid, ld, n_rows, D, (bf16_t*)dS_pre, ld_ds,
                               (bf16_t*)dgate, ld_dg, (bf16_t*)dresid, ld_dr, act,
                               (hipStream_t)stream);
}
