// Probe: does a 16-B global_load_lds (LDS DMA) from an 8-B aligned (not 16-B aligned) global
// address deliver the right bytes on gfx950?  bf16 activation rows of 300 elements are 600 B, so
// every other row starts 8 B off a 16-B boundary.  Prints mismatches (0 expected if supported).
//   hipcc --offload-arch=gfx950 -O2 -o probe_glds probe_glds.hip && ./probe_glds
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

__global__ void k_probe(const uint16_t* src, int off_elems, uint32_t* out) {
  __shared__ __attribute__((aligned(1024))) uint32_t buf[256];
  const int lane = threadIdx.x;
  // lane l copies 16 B from src + off + 8 l (bf16 elements)
  __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + off_elems + 8 * lane), (lds_void_t*)buf, 16,
                                   0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 256; i += 64) out[i] = buf[i];
}

int main() {
  const int n = 4096;
  uint16_t h[n];
  for (int i = 0; i < n; ++i) h[i] = (uint16_t)(i * 7 + 3);
  uint16_t* d;
  uint32_t* o;
  hipMalloc(&d, n * 2);
  hipMalloc(&o, 1024);
  hipMemcpy(d, h, n * 2, hipMemcpyHostToDevice);
  int bad_total = 0;
  for (int off = 0; off < 8; off += 2) {  // 0: 16-B aligned; 4: 8-B aligned; 2, 6: 4-B aligned
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d, off, o);
    uint32_t r[256];
    hipMemcpy(r, o, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) {
      const uint32_t want = (uint32_t)h[off + 2 * i] | ((uint32_t)h[off + 2 * i + 1] << 16);
      if (r[i] != want) ++bad;
    }
    printf("offset %d elements (%d B): %d of 256 dwords wrong\n", off, 2 * off, bad);
    bad_total += bad;
  }
  printf("glds16 unaligned probe: %s\n", bad_total ? "MISMATCH" : "ok");
  return 0;
}
