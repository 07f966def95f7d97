// Checks the DPP / permlane wave sums of common.h against a serial sum (one wave per block).
#include <cstdio>
#include <vector>
#include "../../gnn-mtl_amd/csrc/common.h"
using namespace gnnea;
__global__ void k(const float* xf, const double* xd, float* of, double* od, float* osf) {
  const int t = threadIdx.x;
  const float f = wave_sum_f32(xf[blockIdx.x * 64 + t]);
  const double d = wave_sum_f64(xd[blockIdx.x * 64 + t]);
  const float s = wave_sum_shfl(xf[blockIdx.x * 64 + t]);
  of[blockIdx.x * 64 + t] = f;
  od[blockIdx.x * 64 + t] = d;
  osf[blockIdx.x * 64 + t] = s;
}
int main() {
  const int B = 4;
  std::vector<float> hf(64 * B);
  std::vector<double> hd(64 * B);
  for (int i = 0; i < 64 * B; ++i) { hf[i] = (float)(i % 64 + 1 + 100 * (i / 64)); hd[i] = hf[i]; }
  float *xf, *of, *osf; double *xd, *od;
  hipMalloc(&xf, 256 * 4); hipMalloc(&of, 256 * 4); hipMalloc(&osf, 256 * 4);
  hipMalloc(&xd, 256 * 8); hipMalloc(&od, 256 * 8);
  hipMemcpy(xf, hf.data(), 256 * 4, hipMemcpyHostToDevice);
  hipMemcpy(xd, hd.data(), 256 * 8, hipMemcpyHostToDevice);
  k<<<B, 64>>>(xf, xd, of, od, osf);
  std::vector<float> rf(256), rs(256); std::vector<double> rd(256);
  hipMemcpy(rf.data(), of, 256 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(rs.data(), osf, 256 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(rd.data(), od, 256 * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int b = 0; b < B; ++b) {
    double ref = 0; for (int t = 0; t < 64; ++t) ref += hd[b * 64 + t];
    for (int t = 0; t < 64; ++t) {
      if (rf[b * 64 + t] != (float)ref || rd[b * 64 + t] != ref || rs[b*64+t] != (float)ref) {
        if (bad++ < 8) printf("block %d lane %d: f32 %g f64 %g shfl %g ref %g\n", b, t, rf[b*64+t], rd[b*64+t], rs[b*64+t], ref);
      }
    }
  }
  printf("%s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  return bad != 0;
}
