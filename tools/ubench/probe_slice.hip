// Probe: column-sliced CSR SpMM with the feature table held slice-major ([S][n][w]) so that one
// slice (n*w*4 bytes) stays resident in the 256 MiB Infinity Cache while its gathers run.
// Compares against the row-major library kernel (gnnea_spmm_csr_f32) on one KG of the cfg-4
// generator shape (n = 1M, ring + uniform random edges, ~21 nnz per row).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench/probe_slice tools/ubench/probe_slice.hip \
//          -Lgnn-mtl_amd/gnnea -lgnnea -Wl,-rpath,$PWD/gnn-mtl_amd/gnnea
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <vector>
#include <algorithm>
#include <random>

extern "C" int gnnea_spmm_csr_f32(const int32_t*, const int32_t*, const float*, int32_t, int32_t,
                                  const float*, int64_t, float*, int64_t, int, void*);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// L lanes x float4 per gathered slice row (w = 4L columns); G = 64/L lane groups, group g takes
// neighbours g, g+G, ... of the wave's destination row; U neighbours per group in flight.
template <int L, int U, bool SLICED_Y>
__global__ __launch_bounds__(256) void k_slice(const int* __restrict__ rowptr,
                                               const int* __restrict__ col,
                                               const float* __restrict__ val, int n, int nbs,
                                               const float4* __restrict__ Xs, int S, int D,
                                               float* __restrict__ Y, int ldy) {
  constexpr int G = 64 / L;
  const int b = blockIdx.x;
  const int s = b / nbs;
  const int rb = xcd_remap(b - s * nbs, nbs);
  const int row = rb * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const int lane = threadIdx.x & 63;
  const int g = lane / L, c = lane % L;
  const float4* X = Xs + (int64_t)s * n * L + c;
  const int beg = rowptr[row], end = rowptr[row + 1];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int base = beg; base < end; base += 64) {
    const int cnt = min(64, end - base);
    const int mc = lane < cnt ? col[base + lane] : 0;
    const float mv = lane < cnt ? val[base + lane] : 0.f;
    for (int k = 0; k < cnt; k += G * U) {
      float4 r[U];
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = k + u * G + g;
        const int j = __shfl(mc, e & 63, 64);
        v[u] = __shfl(mv, e & 63, 64);
        if (e < cnt) r[u] = X[(int64_t)j * L];
        else { r[u] = make_float4(0.f, 0.f, 0.f, 0.f); v[u] = 0.f; }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc.x = fmaf(v[u], r[u].x, acc.x);
        acc.y = fmaf(v[u], r[u].y, acc.y);
        acc.z = fmaf(v[u], r[u].z, acc.z);
        acc.w = fmaf(v[u], r[u].w, acc.w);
      }
    }
  }
#pragma unroll
  for (int o = L; o < 64; o <<= 1) {
    acc.x += __shfl_xor(acc.x, o, 64);
    acc.y += __shfl_xor(acc.y, o, 64);
    acc.z += __shfl_xor(acc.z, o, 64);
    acc.w += __shfl_xor(acc.w, o, 64);
  }
  if (g == 0) {
    float4 o = make_float4(fmaxf(acc.x, 0.f), fmaxf(acc.y, 0.f), fmaxf(acc.z, 0.f),
                           fmaxf(acc.w, 0.f));
    if (SLICED_Y) {
      ((float4*)Y)[((int64_t)s * n + row) * L + c] = o;
    } else {
      const int c0 = s * 4 * L + 4 * c;
      float* y = Y + (int64_t)row * ldy + c0;
      if (c0 + 4 <= D) *(float4*)y = o;
      else {
        if (c0 < D) y[0] = o.x;
        if (c0 + 1 < D) y[1] = o.y;
        if (c0 + 2 < D) y[2] = o.z;
      }
    }
  }
}

template <int L, int U, bool SY>
static float run_slice(const int* rp, const int* cl, const float* vl, int n, const float* X,
                       float* Xs_buf, float* Y, int D, int reps, hipEvent_t e0, hipEvent_t e1,
                       std::vector<float>& hy, const std::vector<float>& href) {
  const int w = 4 * L, S = (D + w - 1) / w;
  // build the sliced table on the host side of the probe (zero padded)
  std::vector<float> hx((size_t)n * D);
  CK(hipMemcpy(hx.data(), X, hx.size() * 4, hipMemcpyDeviceToHost));
  std::vector<float> hs((size_t)S * n * w, 0.f);
  for (int s = 0; s < S; ++s)
    for (int i = 0; i < n; ++i)
      for (int q = 0; q < w && s * w + q < D; ++q)
        hs[((size_t)s * n + i) * w + q] = hx[(size_t)i * D + s * w + q];
  CK(hipMemcpy(Xs_buf, hs.data(), hs.size() * 4, hipMemcpyHostToDevice));
  const int nbs = (n + 3) / 4;
  std::vector<float> t;
  for (int r = 0; r < reps + 3; ++r) {
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_slice<L, U, SY>), dim3(nbs * S), dim3(256), 0, 0, rp, cl, vl, n, nbs,
                       (const float4*)Xs_buf, S, D, Y, D);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  double err = 0;
  if (!SY) {
    CK(hipMemcpy(hy.data(), Y, hy.size() * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < hy.size(); ++i) err = std::max(err, (double)fabsf(hy[i] - href[i]));
  }
  printf("  slice L=%2d w=%3d S=%2d U=%d Y=%s: %.4f ms  (table/slice %.0f MB)  maxerr %.2e\n", L,
         w, S, U, SY ? "sliced" : "rowmaj", t[t.size() / 2], (double)n * w * 4 / 1e6, err);
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 1000000;
  const int D = 300;
  const long extra = argc > 2 ? atol(argv[2]) : 9000000;  // random undirected pairs
  std::mt19937_64 rng(1);
  std::vector<int> deg(n, 0);
  std::vector<std::pair<int, int>> ed;
  ed.reserve(n * 3 + extra * 2);
  for (int i = 0; i < n; ++i) {
    ed.push_back({i, i});
    int j = (i + 1) % n;
    ed.push_back({i, j});
    ed.push_back({j, i});
  }
  for (long t = 0; t < extra; ++t) {
    int a = rng() % n, b = rng() % n;
    ed.push_back({a, b});
    ed.push_back({b, a});
  }
  std::sort(ed.begin(), ed.end());
  std::vector<int> rowptr(n + 1, 0), colv(ed.size());
  std::vector<float> valv(ed.size());
  for (size_t e = 0; e < ed.size(); ++e) {
    rowptr[ed[e].first + 1]++;
    colv[e] = ed[e].second;
    valv[e] = 0.05f + (float)((rng() >> 40) & 1023) / 1024.f * 0.1f;
  }
  for (int i = 0; i < n; ++i) rowptr[i + 1] += rowptr[i];
  const long E = ed.size();
  printf("n=%d E=%ld D=%d\n", n, E, D);
  std::vector<float> hx((size_t)n * D);
  for (auto& x : hx) x = (float)((int)(rng() >> 44) - (1 << 19)) / (1 << 19);
  int *rp, *cl;
  float *vl, *X, *Y, *Xs;
  CK(hipMalloc(&rp, (n + 1) * 4));
  CK(hipMalloc(&cl, E * 4));
  CK(hipMalloc(&vl, E * 4));
  CK(hipMalloc(&X, (size_t)n * D * 4));
  CK(hipMalloc(&Y, (size_t)n * 384 * 4 + 4096));
  CK(hipMalloc(&Xs, (size_t)n * 384 * 4 + 4096));
  CK(hipMemcpy(rp, rowptr.data(), (n + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(cl, colv.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(vl, valv.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 15;
  std::vector<float> t;
  for (int r = 0; r < reps + 3; ++r) {
    CK(hipEventRecord(e0));
    int rc = gnnea_spmm_csr_f32(rp, cl, vl, n, D, X, D, Y, D, 1, 0);
    if (rc) { printf("rc %d\n", rc); return 1; }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  const double gm = 4.0 * (n + 1) + 8.0 * E + 4.0 * E * D + 4.0 * n * D;
  printf("  library row-major: %.4f ms  gather-model %.1f GB/s\n", t[t.size() / 2],
         gm / t[t.size() / 2] / 1e6);
  std::vector<float> href((size_t)n * D), hy((size_t)n * D);
  CK(hipMemcpy(href.data(), Y, href.size() * 4, hipMemcpyDeviceToHost));
  float m;
  m = run_slice<16, 2, false>(rp, cl, vl, n, X, Xs, Y, D, reps, e0, e1, hy, href);
  m = run_slice<16, 4, false>(rp, cl, vl, n, X, Xs, Y, D, reps, e0, e1, hy, href);
  printf("      gather-model rate %.1f GB/s\n", gm / m / 1e6);
  m = run_slice<16, 4, true>(rp, cl, vl, n, X, Xs, Y, D, reps, e0, e1, hy, href);
  printf("      gather-model rate %.1f GB/s\n", gm / m / 1e6);
  m = run_slice<32, 2, false>(rp, cl, vl, n, X, Xs, Y, D, reps, e0, e1, hy, href);
  m = run_slice<32, 4, false>(rp, cl, vl, n, X, Xs, Y, D, reps, e0, e1, hy, href);
  printf("      per-300-col equivalent %.4f ms\n", m * 300.0 / 384.0);
  return 0;
}
