// Microbenchmark: fp64 FMA and exp throughput on gfx950 (diagnostic for the Sinkhorn passes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../gnn-mtl_amd/csrc/common.h"
using namespace gnnea;

__global__ void k_fma(double* out, int iters, double seed) {
  double a = seed + threadIdx.x, b = 1.0000001, c = 0.999999;
  double x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
  for (int i = 0; i < iters; ++i) {
    x0 = fma(x0, b, c); x1 = fma(x1, b, c); x2 = fma(x2, b, c); x3 = fma(x3, b, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
__global__ void k_myexp(double* out, int iters, double seed) {
  double x0 = -seed - threadIdx.x * 1e-3, s = 0;
  for (int i = 0; i < iters; ++i) {
    s += exp_f64(x0 - i * 1e-4) + exp_f64(x0 - i * 2e-4) + exp_f64(x0 - i * 3e-4) + exp_f64(x0 - i * 4e-4);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_libexp(double* out, int iters, double seed) {
  double x0 = -seed - threadIdx.x * 1e-3, s = 0;
  for (int i = 0; i < iters; ++i) {
    s += exp(x0 - i * 1e-4) + exp(x0 - i * 2e-4) + exp(x0 - i * 3e-4) + exp(x0 - i * 4e-4);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_f32exp(float* out, int iters, float seed) {
  float x0 = -seed - threadIdx.x * 1e-3f, s = 0;
  for (int i = 0; i < iters; ++i) {
    s += __expf(x0 - i * 1e-4f) + __expf(x0 - i * 2e-4f) + __expf(x0 - i * 3e-4f) + __expf(x0 - i * 4e-4f);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_empty(int* p) { if (p && threadIdx.x == 9999) p[0] = 1; }

#include <chrono>
int main() {
  const int blocks = 256 * 8, threads = 256, iters = 2000;
  double* d; float* f;
  hipMalloc(&d, sizeof(double) * blocks * threads);
  hipMalloc(&f, sizeof(float) * blocks * threads);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const double n = (double)blocks * threads * iters * 4;
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(a); hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("fp64 fma      : %8.3f ms  %8.2f T/s\n", ms, n / ms / 1e9);
    hipEventRecord(a); hipLaunchKernelGGL(k_myexp, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("exp_f64 (ours): %8.3f ms  %8.2f G/s\n", ms, n / ms / 1e6);
    hipEventRecord(a); hipLaunchKernelGGL(k_libexp, dim3(blocks), dim3(threads), 0, 0, d, iters, 1.0); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("exp (ocml)    : %8.3f ms  %8.2f G/s\n", ms, n / ms / 1e6);
    hipEventRecord(a); hipLaunchKernelGGL(k_f32exp, dim3(blocks), dim3(threads), 0, 0, f, iters, 1.0f); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms, a, b); printf("__expf f32    : %8.3f ms  %8.2f G/s\n", ms, n / ms / 1e6);
  }
  {
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int i = 0; i < 10000; ++i) hipLaunchKernelGGL(k_empty, dim3(750), dim3(256), 0, 0, (int*)nullptr);
    auto t1 = std::chrono::high_resolution_clock::now();
    (void)hipDeviceSynchronize();
    auto t2 = std::chrono::high_resolution_clock::now();
    printf("empty launches: host enqueue %.2f us/launch, wall %.2f us/launch\n",
           std::chrono::duration<double, std::micro>(t1 - t0).count() / 1e4,
           std::chrono::duration<double, std::micro>(t2 - t0).count() / 1e4);
  }
  return 0;
}
