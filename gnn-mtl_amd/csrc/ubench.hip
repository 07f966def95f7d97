// Bandwidth anchors for the roofline fractions bench.py quotes ("measure a
// device-copy bandwidth on the box and report it next to the datasheet value").  torch's copy_
// (5.0 TB/s) is one implementation's rate, not the hardware's; these two kernels are the
// reference points the gather-bound passes are judged against:
//   k_ub_copy    a streaming copy, 16 B per lane per access, every lane of a wave on consecutive
//                16-B chunks (1 KB per wave instruction), four or eight accesses in flight per
//                lane, plain or nontemporal, a grid of a few workgroups per CU striding over the
//                buffer; or the same loads alone (read only);
//   k_ub_gather  whole-row gathers: one wave per 64 rows of an index list, each row read by the
//                lanes of the wave as 8-B chunks (row_bytes % 8 == 0: a 600-B row is 75 chunks),
//                summed into one accumulator per lane (nothing is written per row, so only the
//                gathered bytes cross HBM) — the access pattern of the row-major GAT passes
//                (600-B bf16 rows at cfg-5) when the index list is uniform random over a table
//                much larger than the 256-MB Infinity Cache.
#include "common.h"

namespace gnnea {

// U accesses of 16 B in flight per lane; NT: nontemporal loads and stores; RO: read only (the
// loaded words xor-folded, one word per lane written at the end: a read-bandwidth anchor)
typedef unsigned int ub_u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT, bool RO>
__global__ __launch_bounds__(256) void k_ub_copy(const uint4* __restrict__ src,
                                                 uint4* __restrict__ dst, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t x = 0;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (NT) {
        const ub_u32x4 t = __builtin_nontemporal_load((const ub_u32x4*)(src + i + u * stride));
        v[u] = make_uint4(t.x, t.y, t.z, t.w);
      } else {
        v[u] = src[i + u * stride];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (RO) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
      else if constexpr (NT)
        __builtin_nontemporal_store(ub_u32x4{v[u].x, v[u].y, v[u].z, v[u].w},
                                    (ub_u32x4*)(dst + i + u * stride));
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n16; i += stride) {
    const uint4 v = src[i];
    if constexpr (RO) x ^= v.x ^ v.y ^ v.z ^ v.w;
    else dst[i] = v;
  }
  if constexpr (RO) ((uint32_t*)dst)[(int64_t)blockIdx.x * 256 + threadIdx.x] = x;
}

// wave w handles index entries [64 w, 64 w + 64): the 64 row ids are loaded once (one per lane)
// and broadcast; for each row every lane reads its 8-B chunk(s), U rows in flight
template <int NCH>
__global__ __launch_bounds__(256) void k_ub_gather(const unsigned char* __restrict__ table,
                                                   int64_t row_bytes, const int32_t* __restrict__ idx,
                                                   int64_t n, float* __restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * 4 + wave_id();
  const int64_t base = w * 64;
  if (base >= n) return;
  const int lane = lane_id();
  const int cnt = (int)min((int64_t)64, n - base);
  const int my = idx[base + min(lane, cnt - 1)];
  const int nfull = (int)(row_bytes / 8);
  uint32_t acc = 0;
  constexpr int U = 4;
  for (int k = 0; k < cnt; k += U) {
    uint2 v[U][NCH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = __shfl(my, min(k + u, cnt - 1), 64);
      const unsigned char* row = table + (int64_t)r * row_bytes;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const int ch = lane + 64 * c;
        // chunks past the row re-read the row's first chunk (no branch around the load)
        v[u][c] = *(const uint2*)(row + 8 * (ch < nfull ? ch : 0));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int c = 0; c < NCH; ++c) acc ^= v[u][c].x ^ v[u][c].y;
  }
  // one value per lane keeps the loads live; written once per wave
  if (lane == 0) out[w] = (float)(acc & 0xffff);
}

// The two access shapes of a row-major bf16 GAT pass over 300-column rows, as pure gathers:
//   WIN12  600-B rows (8-B aligned), lane l reads the 12-B dword window holding its 5 columns
//          5 l .. 5 l + 4 (byte offset (10 l) & ~3; 60 lanes), as k_gat_fwd_hg / k_gat_bwd_src_hg;
//   !WIN12 rows padded to row_bytes % 16 == 0 (608 B), 16 B per lane (38 lanes).
template <bool WIN12>
__global__ __launch_bounds__(256) void k_ub_gather_gat(const unsigned char* __restrict__ table,
                                                       int64_t row_bytes,
                                                       const int32_t* __restrict__ idx, int64_t n,
                                                       float* __restrict__ out) {
  const int64_t w = (int64_t)blockIdx.x * 4 + wave_id();
  const int64_t base = w * 64;
  if (base >= n) return;
  const int lane = lane_id();
  const int cnt = (int)min((int64_t)64, n - base);
  const int my = idx[base + min(lane, cnt - 1)];
  const int lanes = WIN12 ? 60 : (int)(row_bytes / 16);
  const int off = WIN12 ? ((10 * min(lane, lanes - 1)) & ~3) : 16 * min(lane, lanes - 1);
  uint32_t acc = 0;
  constexpr int U = 8;
  for (int k = 0; k < cnt; k += U) {
    uint32_t v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = __shfl(my, min(k + u, cnt - 1), 64);
      const unsigned char* p = table + (int64_t)r * row_bytes + off;
      if constexpr (WIN12) {
        const HIP_vector_type<unsigned int, 3> t = *(const HIP_vector_type<unsigned int, 3>*)p;
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = 0;
      } else {
        const uint4 t = *(const uint4*)p;
        v[u][0] = t.x; v[u][1] = t.y; v[u][2] = t.z; v[u][3] = t.w;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (lane == 0) out[w] = (float)(acc & 0xffff);
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int gnnea_ub_copy(const void* src, void* dst, int64_t bytes, int32_t blocks,
                             int32_t flags, void* stream) {
  if (bytes < 0 || bytes % 16 || blocks <= 0 || flags < 0 || flags > 7) return GNNEA_EINVAL;
  if (bytes == 0) return 0;
  if (!src || !dst || (((uintptr_t)src | (uintptr_t)dst) & 15)) return GNNEA_EALIGN;
  // read only: dst receives one word per thread of the grid
  if ((flags & GNNEA_UB_READ_ONLY) && (int64_t)blocks * 256 * 4 > bytes) return GNNEA_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint4* a = (const uint4*)src;
  uint4* b = (uint4*)dst;
  const int64_t n = bytes / 16;
  const dim3 g(blocks), t(256);
  switch (flags) {
    case 0: hipLaunchKernelGGL((k_ub_copy<4, false, false>), g, t, 0, s, a, b, n); break;
    case 1: hipLaunchKernelGGL((k_ub_copy<4, true, false>), g, t, 0, s, a, b, n); break;
    case 2: hipLaunchKernelGGL((k_ub_copy<8, false, false>), g, t, 0, s, a, b, n); break;
    case 3: hipLaunchKernelGGL((k_ub_copy<8, true, false>), g, t, 0, s, a, b, n); break;
    case 4: hipLaunchKernelGGL((k_ub_copy<4, false, true>), g, t, 0, s, a, b, n); break;
    case 5: hipLaunchKernelGGL((k_ub_copy<4, true, true>), g, t, 0, s, a, b, n); break;
    case 6: hipLaunchKernelGGL((k_ub_copy<8, false, true>), g, t, 0, s, a, b, n); break;
    default: hipLaunchKernelGGL((k_ub_copy<8, true, true>), g, t, 0, s, a, b, n); break;
  }
  GNNEA_LAUNCH_CHECK();
  return 0;
}

extern "C" int gnnea_ub_gather(const void* table, int64_t row_bytes, const int32_t* idx,
                               int64_t n, float* out, int32_t mode, void* stream) {
  if (mode == GNNEA_UB_GAT_WIN12 || mode == GNNEA_UB_GAT_V16) {  // the GAT access shapes
    if (n < 0 || !table || !idx || !out) return GNNEA_EINVAL;
    if (mode == GNNEA_UB_GAT_WIN12 ? row_bytes != 600 : (row_bytes % 16 || row_bytes > 1024 ||
                                                         row_bytes < 16))
      return GNNEA_EINVAL;
    if (((uintptr_t)table) & 15) return GNNEA_EALIGN;
    if (n == 0) return 0;
    const int64_t nb = ((n + 63) / 64 + 3) / 4;
    if (nb >= (1ll << 31)) return GNNEA_EINVAL;
    if (mode == GNNEA_UB_GAT_WIN12)
      hipLaunchKernelGGL(k_ub_gather_gat<true>, dim3((unsigned)nb), dim3(256), 0,
                         (hipStream_t)stream, (const unsigned char*)table, row_bytes, idx, n, out);
    else
      hipLaunchKernelGGL(k_ub_gather_gat<false>, dim3((unsigned)nb), dim3(256), 0,
                         (hipStream_t)stream, (const unsigned char*)table, row_bytes, idx, n, out);
    GNNEA_LAUNCH_CHECK();
    return 0;
  }
  if (mode != 0) return GNNEA_EINVAL;
  if (row_bytes <= 0 || row_bytes % 8 || row_bytes > 2 * 1024 || n < 0) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!table || !idx || !out || (((uintptr_t)table) & 7)) return GNNEA_EINVAL;
  const int64_t waves = (n + 63) / 64, nb = (waves + 3) / 4;
  if (nb >= (1ll << 31)) return GNNEA_EINVAL;
  const int nch = (int)((row_bytes / 8 + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  switch (nch) {
    case 1: hipLaunchKernelGGL(k_ub_gather<1>, dim3((unsigned)nb), dim3(256), 0, s,
                               (const unsigned char*)table, row_bytes, idx, n, out); break;
    case 2: hipLaunchKernelGGL(k_ub_gather<2>, dim3((unsigned)nb), dim3(256), 0, s,
                               (const unsigned char*)table, row_bytes, idx, n, out); break;
    case 3: hipLaunchKernelGGL(k_ub_gather<3>, dim3((unsigned)nb), dim3(256), 0, s,
                               (const unsigned char*)table, row_bytes, idx, n, out); break;
    default: hipLaunchKernelGGL(k_ub_gather<4>, dim3((unsigned)nb), dim3(256), 0, s,
                                (const unsigned char*)table, row_bytes, idx, n, out); break;
  }
  GNNEA_LAUNCH_CHECK();
  return 0;
}
