// a1. COO -> CSR on the device (replaces the coalesce hidden inside torch.spmm,
// layers/layers.py:35/64, and adj.coalesce().indices() at layers/att_layers.py:31).
//
// Pipeline (all on the caller's stream, all scratch in the caller's workspace):
//   key[e] = row[e] * n_cols + col[e]          (uint64; only the needed bits are sorted)
//   stable radix sort (key, e)                 (rocPRIM onesweep)
//   head[k] = key[k] != key[k-1]               -> inclusive scan -> output slot
//   heads sum their duplicate run in input order, write col / val / perm, count rows
//   rowptr = exclusive scan of row counts
#include "common.h"
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

namespace gnnea {

template <typename IDX>
__global__ void k_make_keys(const IDX* __restrict__ row, const IDX* __restrict__ col, int64_t nnz,
                            uint64_t n_cols, uint64_t* __restrict__ keys,
                            int64_t* __restrict__ idx, int* __restrict__ bad, int64_t n_rows) {
  int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nnz) return;
  const int64_t r = (int64_t)row[e], c = (int64_t)col[e];
  if (r < 0 || r >= n_rows || c < 0 || c >= (int64_t)n_cols) {
    atomicOr(bad, 1);
    keys[e] = 0;
  } else {
    keys[e] = (uint64_t)r * n_cols + (uint64_t)c;
  }
  idx[e] = e;
}

__global__ void k_heads(const uint64_t* __restrict__ keys, int64_t nnz, int* __restrict__ head) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) return;
  head[k] = (k == 0 || keys[k] != keys[k - 1]) ? 1 : 0;
}

__global__ void k_emit(const uint64_t* __restrict__ keys, const int64_t* __restrict__ idx,
                       const int* __restrict__ head, const int* __restrict__ slot, int64_t nnz,
                       uint64_t n_cols, const float* __restrict__ val,
                       int32_t* __restrict__ col_out, float* __restrict__ val_out,
                       int64_t* __restrict__ perm_out, int* __restrict__ row_count,
                       int64_t* __restrict__ nnz_out, const int* __restrict__ bad) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) return;
  // an out-of-range index is reported as *nnz_out = -1 (no host sync inside the ABI)
  if (k == nnz - 1) *nnz_out = *bad ? (int64_t)-1 : (int64_t)slot[k];
  if (!head[k]) return;
  const int64_t s = slot[k] - 1;
  const uint64_t key = keys[k];
  const int64_t r = (int64_t)(key / n_cols);
  col_out[s] = (int32_t)(key - (uint64_t)r * n_cols);
  if (perm_out) perm_out[s] = idx[k];
  if (val_out) {
    // duplicates are adjacent and, the sort being stable, in input order
    float acc = val ? val[idx[k]] : 1.f;
    for (int64_t q = k + 1; q < nnz && keys[q] == key; ++q) acc += val ? val[idx[q]] : 1.f;
    val_out[s] = acc;
  }
  atomicAdd(&row_count[r], 1);
}

static inline int64_t align_up(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct CsrWs {
  int64_t keys_a, keys_b, idx_a, idx_b, head, slot, count, bad, cub, total;
  size_t cub_sort, cub_scan, cub_scan_rows;
};

static int plan_ws(int64_t nnz, int64_t n_rows, int end_bit, CsrWs* w) {
  size_t sort_bytes = 0, scan_bytes = 0, scan_rows = 0;
  rocprim::double_buffer<uint64_t> kb(nullptr, nullptr);
  rocprim::double_buffer<int64_t> vb(nullptr, nullptr);
  GNNEA_HIP(rocprim::radix_sort_pairs(nullptr, sort_bytes, kb, vb, (size_t)nnz, 0, end_bit));
  GNNEA_HIP(rocprim::inclusive_scan(nullptr, scan_bytes, (int*)nullptr, (int*)nullptr,
                                    (size_t)nnz, rocprim::plus<int>()));
  GNNEA_HIP(rocprim::exclusive_scan(nullptr, scan_rows, (int*)nullptr, (int*)nullptr, 0,
                                    (size_t)(n_rows + 1), rocprim::plus<int>()));
  int64_t o = 0;
  w->keys_a = o; o = align_up(o + 8 * nnz);
  w->keys_b = o; o = align_up(o + 8 * nnz);
  w->idx_a = o; o = align_up(o + 8 * nnz);
  w->idx_b = o; o = align_up(o + 8 * nnz);
  w->head = o; o = align_up(o + 4 * nnz);
  w->slot = o; o = align_up(o + 4 * nnz);
  w->count = o; o = align_up(o + 4 * (n_rows + 1));
  w->bad = o; o = align_up(o + 16);
  w->cub = o;
  w->cub_sort = sort_bytes;
  w->cub_scan = scan_bytes;
  w->cub_scan_rows = scan_rows;
  size_t m = sort_bytes > scan_bytes ? sort_bytes : scan_bytes;
  m = m > scan_rows ? m : scan_rows;
  o = align_up(o + (int64_t)m);
  w->total = o;
  return 0;
}

static int key_bits(int64_t n_rows, int64_t n_cols) {
  const unsigned long long maxkey = (unsigned long long)n_rows * (unsigned long long)n_cols;
  int b = 1;
  while (b < 64 && (1ull << b) < maxkey) ++b;
  return b;
}

}  // namespace gnnea

using namespace gnnea;

extern "C" int64_t gnnea_coo_to_csr_ws_bytes(int64_t nnz, int64_t n_rows, int64_t n_cols) {
  if (nnz < 0 || n_rows < 0 || n_cols < 0) return GNNEA_EINVAL;
  CsrWs w;
  int rc = plan_ws(nnz > 0 ? nnz : 1, n_rows, key_bits(n_rows, n_cols), &w);
  if (rc) return GNNEA_EINVAL;
  return w.total;
}

extern "C" int gnnea_coo_to_csr(const void* row_idx, const void* col_idx, int index_bytes,
                                const float* val, int64_t nnz, int64_t n_rows, int64_t n_cols,
                                int32_t* rowptr, int32_t* col_out, float* val_out,
                                int64_t* perm_out, int64_t* nnz_out, void* ws, int64_t ws_bytes,
                                void* stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (nnz < 0 || n_rows < 0 || n_cols < 0 || !rowptr || !nnz_out) return GNNEA_EINVAL;
  if (index_bytes != 4 && index_bytes != 8) return GNNEA_EINVAL;
  if (nnz >= (1ll << 31) || n_rows >= (1ll << 31) || n_cols >= (1ll << 31)) return GNNEA_EINVAL;
  if (nnz > 0 && (!row_idx || !col_idx || !col_out || !ws)) return GNNEA_EINVAL;
  const int end_bit = key_bits(n_rows, n_cols);
  CsrWs w;
  if (plan_ws(nnz > 0 ? nnz : 1, n_rows, end_bit, &w)) return GNNEA_EINVAL;
  if (ws_bytes < w.total) return GNNEA_EWORKSPACE;
  char* base = (char*)ws;
  int* count = (int*)(base + w.count);
  GNNEA_HIP(hipMemsetAsync(count, 0, sizeof(int) * (n_rows + 1), stream));
  if (nnz == 0) {
    GNNEA_HIP(hipMemsetAsync(rowptr, 0, sizeof(int32_t) * (n_rows + 1), stream));
    GNNEA_HIP(hipMemsetAsync(nnz_out, 0, sizeof(int64_t), stream));
    return 0;
  }
  uint64_t* keys_a = (uint64_t*)(base + w.keys_a);
  uint64_t* keys_b = (uint64_t*)(base + w.keys_b);
  int64_t* idx_a = (int64_t*)(base + w.idx_a);
  int64_t* idx_b = (int64_t*)(base + w.idx_b);
  int* head = (int*)(base + w.head);
  int* slot = (int*)(base + w.slot);
  int* bad = (int*)(base + w.bad);
  void* cub = (void*)(base + w.cub);
  GNNEA_HIP(hipMemsetAsync(bad, 0, sizeof(int), stream));

  const int tpb = 256;
  const int nb = div_up(nnz, tpb);
  if (index_bytes == 8)
    hipLaunchKernelGGL(k_make_keys<int64_t>, dim3(nb), dim3(tpb), 0, stream,
                       (const int64_t*)row_idx, (const int64_t*)col_idx, nnz, (uint64_t)n_cols,
                       keys_a, idx_a, bad, n_rows);
  else
    hipLaunchKernelGGL(k_make_keys<int32_t>, dim3(nb), dim3(tpb), 0, stream,
                       (const int32_t*)row_idx, (const int32_t*)col_idx, nnz, (uint64_t)n_cols,
                       keys_a, idx_a, bad, n_rows);
  GNNEA_LAUNCH_CHECK();

  rocprim::double_buffer<uint64_t> kb(keys_a, keys_b);
  rocprim::double_buffer<int64_t> vb(idx_a, idx_b);
  size_t sort_bytes = w.cub_sort;
  GNNEA_HIP(rocprim::radix_sort_pairs(cub, sort_bytes, kb, vb, (size_t)nnz, 0, end_bit, stream));
  const uint64_t* keys = kb.current();
  const int64_t* idx = vb.current();

  hipLaunchKernelGGL(k_heads, dim3(nb), dim3(tpb), 0, stream, keys, nnz, head);
  GNNEA_LAUNCH_CHECK();
  size_t scan_bytes = w.cub_scan;
  GNNEA_HIP(rocprim::inclusive_scan(cub, scan_bytes, head, slot, (size_t)nnz,
                                    rocprim::plus<int>(), stream));
  hipLaunchKernelGGL(k_emit, dim3(nb), dim3(tpb), 0, stream, keys, idx, head, slot, nnz,
                     (uint64_t)n_cols, val, col_out, val_out, perm_out, count, nnz_out, bad);
  GNNEA_LAUNCH_CHECK();
  size_t scan_rows = w.cub_scan_rows;
  GNNEA_HIP(rocprim::exclusive_scan(cub, scan_rows, count, rowptr, 0, (size_t)(n_rows + 1),
                                    rocprim::plus<int>(), stream));
  return 0;
}

namespace gnnea {
// row id of every CSR entry (used to build the transpose from (col, row) pairs)
__global__ void k_expand_rows(const int32_t* __restrict__ rowptr, int32_t n_rows,
                              int32_t* __restrict__ row_out) {
  const int r = blockIdx.x * 4 + wave_id();
  if (r >= n_rows) return;
  const int beg = rowptr[r], end = rowptr[r + 1];
  for (int e = beg + lane_id(); e < end; e += 64) row_out[e] = r;
}
}  // namespace gnnea

extern "C" int gnnea_csr_expand_rows(const int32_t* rowptr, int32_t n_rows, int64_t nnz,
                                     int32_t* row_out, void* stream) {
  if (n_rows < 0 || nnz < 0) return GNNEA_EINVAL;
  if (n_rows == 0 || nnz == 0) return 0;
  if (!rowptr || !row_out) return GNNEA_EINVAL;
  hipLaunchKernelGGL(gnnea::k_expand_rows, dim3(gnnea::div_up(n_rows, 4)), dim3(256), 0,
                     (hipStream_t)stream, rowptr, n_rows, row_out);
  GNNEA_LAUNCH_CHECK();
  return 0;
}

namespace gnnea {
__global__ void k_perm_invert(const int64_t* __restrict__ perm, int64_t n,
                              int64_t* __restrict__ inv) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) inv[perm[k]] = k;
}
}  // namespace gnnea

extern "C" int gnnea_perm_invert(const int64_t* perm, int64_t n, int64_t* inv, void* stream) {
  if (n < 0) return GNNEA_EINVAL;
  if (n == 0) return 0;
  if (!perm || !inv) return GNNEA_EINVAL;
  hipLaunchKernelGGL(gnnea::k_perm_invert, dim3(gnnea::div_up(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, perm, n, inv);
  GNNEA_LAUNCH_CHECK();
  return 0;
}
