// Host-side KG ingestion, declared in include/gnnea_host.h.
//
//   gnnea_h_loadfile          utils/data_utils.py:362-372  loadfile(fn, num)
//   gnnea_h_adjacency         utils/data_utils.py:296-336  get_matrix + get_sparse_tensor
//   gnnea_h_relation_groups   utils/data_utils.py:272-293  rfunc's per-relation head/tail lists
//
// The reference walks Python dicts per line / per triple (minutes at 20M triples); here the file
// is parsed by chunks in parallel threads and the adjacency is built with counting sorts:
// candidates (h,t),(t,h) are bucketed by row, deduplicated per row keeping the first occurrence,
// and emitted in first-occurrence order (the dict-insertion order of the reference) or sorted.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../../include/gnnea_host.h"

namespace {

int n_threads() {
  const unsigned hc = std::thread::hardware_concurrency();
  const int t = hc ? (int)hc : 8;
  return std::min(t, 16);
}

template <typename F>
void parallel_for(int64_t n, F&& f) {
  const int T = (int)std::min<int64_t>(n_threads(), std::max<int64_t>(1, n / 65536));
  if (T <= 1) {
    f(0, n, 0);
    return;
  }
  std::vector<std::thread> ths;
  for (int k = 0; k < T; ++k) {
    const int64_t b = n * k / T, e = n * (k + 1) / T;
    ths.emplace_back([&, b, e, k] { f(b, e, k); });
  }
  for (auto& t : ths) t.join();
}

bool read_all(const char* path, std::vector<char>& buf) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return false;
  std::fseek(fp, 0, SEEK_END);
  const long sz = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  if (sz < 0) {
    std::fclose(fp);
    return false;
  }
  buf.resize((size_t)sz);
  const size_t got = sz ? std::fread(buf.data(), 1, (size_t)sz, fp) : 0;
  std::fclose(fp);
  return got == (size_t)sz;
}

// Python int() of one field: optional surrounding whitespace, sign, digits with single '_'
bool parse_field(const char* b, const char* e, int64_t& v) {
  auto ws = [](char c) { return c == ' ' || c == '\v' || c == '\f' || c == '\r' || c == '\n'; };
  while (b < e && ws(*b)) ++b;
  while (e > b && ws(e[-1])) --e;
  if (b == e) return false;
  bool neg = false;
  if (*b == '+' || *b == '-') {
    neg = *b == '-';
    ++b;
  }
  if (b == e || *b == '_' || e[-1] == '_') return false;
  int64_t x = 0;
  char prev = 0;
  for (const char* p = b; p < e; ++p) {
    if (*p == '_') {
      if (prev == '_') return false;
    } else if (*p >= '0' && *p <= '9') {
      x = x * 10 + (*p - '0');
    } else {
      return false;
    }
    prev = *p;
  }
  v = neg ? -x : x;
  return true;
}

// one logical line [b, e) (terminator excluded) minus its last character, as line[:-1]
bool parse_line(const char* b, const char* e, bool had_newline, int ncols, int64_t* out) {
  if (!had_newline && e > b) --e;  // no terminator: line[:-1] eats the last character
  const char* p = b;
  for (int c = 0; c < ncols; ++c) {
    if (p > e) return false;  // fewer fields than ncols (IndexError)
    const char* q = p;
    while (q < e && *q != '\t') ++q;
    if (!parse_field(p, q, out[c])) return false;
    p = q + 1;
  }
  return true;
}

}  // namespace

extern "C" int64_t gnnea_h_loadfile(const char* path, int32_t ncols, int64_t* out,
                                    int64_t cap_rows) {
  if (!path || ncols < 1) return GNNEA_H_EINVAL;
  std::vector<char> buf;
  if (!read_all(path, buf)) return GNNEA_H_EIO;
  // universal newlines: "\r\n" and "\r" end a line like "\n"
  const char* s = buf.data();
  const int64_t n = (int64_t)buf.size();
  std::vector<int64_t> starts;  // line starts
  starts.reserve(n / 16 + 2);
  int64_t i = 0;
  while (i < n) {
    starts.push_back(i);
    while (i < n && s[i] != '\n' && s[i] != '\r') ++i;
    if (i < n) i += (s[i] == '\r' && i + 1 < n && s[i + 1] == '\n') ? 2 : 1;
  }
  const int64_t rows = (int64_t)starts.size();
  if (!out) return rows;
  if (cap_rows < rows) return GNNEA_H_ESPACE;
  std::atomic<bool> bad(false);
  parallel_for(rows, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e && !bad.load(std::memory_order_relaxed); ++r) {
      const int64_t ls = starts[r];
      int64_t le = ls;
      while (le < n && s[le] != '\n' && s[le] != '\r') ++le;
      const bool nl = le < n;
      if (!parse_line(s + ls, s + le, nl, ncols, out + r * ncols)) bad = true;
    }
  });
  return bad ? GNNEA_H_EPARSE : rows;
}

extern "C" int64_t gnnea_h_adjacency(const int64_t* tr, int64_t nt, int64_t n_ent,
                                     int32_t reference_order, int64_t* row, int64_t* col,
                                     float* val, int64_t cap) {
  if (nt < 0 || n_ent < 0 || (nt > 0 && !tr)) return GNNEA_H_EINVAL;
  for (int64_t i = 0; i < nt; ++i) {
    const int64_t h = tr[3 * i], t = tr[3 * i + 2];
    if (h < 0 || h >= n_ent || t < 0 || t >= n_ent) return GNNEA_H_EINVAL;
  }
  // degrees and first-appearance order of entities
  std::vector<int64_t> deg((size_t)n_ent, 0);
  std::vector<int64_t> ents;
  std::vector<char> seen((size_t)n_ent, 0);
  int64_t m = 0;  // non-self triples
  for (int64_t i = 0; i < nt; ++i) {
    const int64_t h = tr[3 * i], t = tr[3 * i + 2];
    if (!seen[h]) { seen[h] = 1; deg[h] = 1; ents.push_back(h); }
    if (!seen[t]) { seen[t] = 1; deg[t] = 1; ents.push_back(t); }
    if (h != t) { ++deg[h]; ++deg[t]; ++m; }
  }
  // candidates p = 2k (h,t), 2k+1 (t,h) of the k-th non-self triple, bucketed by row
  std::vector<int64_t> crow(2 * m), ccol(2 * m);
  {
    int64_t k = 0;
    for (int64_t i = 0; i < nt; ++i) {
      const int64_t h = tr[3 * i], t = tr[3 * i + 2];
      if (h == t) continue;
      crow[2 * k] = h; ccol[2 * k] = t;
      crow[2 * k + 1] = t; ccol[2 * k + 1] = h;
      ++k;
    }
  }
  std::vector<int64_t> ptr((size_t)n_ent + 1, 0);
  for (int64_t p = 0; p < 2 * m; ++p) ++ptr[crow[p] + 1];
  for (int64_t r = 0; r < n_ent; ++r) ptr[r + 1] += ptr[r];
  std::vector<int64_t> bucket(2 * m);  // candidate positions, stable within a row
  {
    std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
    for (int64_t p = 0; p < 2 * m; ++p) bucket[fill[crow[p]]++] = p;
  }
  // per row: order by (col, position); the first of each col group is the dict entry
  std::vector<char> first(2 * m, 0);
  std::vector<int64_t> uniq_cnt((size_t)n_ent, 0);
  parallel_for(n_ent, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e; ++r) {
      int64_t* beg = bucket.data() + ptr[r];
      int64_t* end = bucket.data() + ptr[r + 1];
      std::sort(beg, end, [&](int64_t x, int64_t y) {
        return ccol[x] != ccol[y] ? ccol[x] < ccol[y] : x < y;
      });
      int64_t u = 0;
      for (int64_t* q = beg; q < end; ++q)
        if (q == beg || ccol[*q] != ccol[q[-1]]) { first[*q] = 1; ++u; }
      uniq_cnt[r] = u;
    }
  });
  int64_t nnz = (int64_t)ents.size();
  for (int64_t r = 0; r < n_ent; ++r) nnz += uniq_cnt[r];
  if (!row) return nnz;
  if (!col || !val || cap < nnz) return GNNEA_H_ESPACE;
  auto value = [&](int64_t a, int64_t b) {
    return (float)((1.0 / std::sqrt((double)deg[a])) / std::sqrt((double)deg[b]));
  };
  if (reference_order) {
    int64_t o = 0;
    for (int64_t p = 0; p < 2 * m; ++p)
      if (first[p]) { row[o] = crow[p]; col[o] = ccol[p]; ++o; }
    for (int64_t e : ents) { row[o] = e; col[o] = e; ++o; }
  } else {
    // row-major (row, col) order: each row's unique cols in ascending order, self loop merged
    std::vector<int64_t> off((size_t)n_ent + 1, 0);
    for (int64_t r = 0; r < n_ent; ++r) off[r + 1] = off[r] + uniq_cnt[r] + (seen[r] ? 1 : 0);
    parallel_for(n_ent, [&](int64_t b, int64_t e, int) {
      for (int64_t r = b; r < e; ++r) {
        int64_t o = off[r];
        bool self_done = !seen[r];
        for (int64_t q = ptr[r]; q < ptr[r + 1]; ++q) {
          const int64_t p = bucket[q];
          if (!first[p]) continue;
          if (!self_done && ccol[p] > r) { row[o] = r; col[o] = r; ++o; self_done = true; }
          row[o] = r; col[o] = ccol[p]; ++o;
        }
        if (!self_done) { row[o] = r; col[o] = r; ++o; }
      }
    });
  }
  parallel_for(nnz, [&](int64_t b, int64_t e, int) {
    for (int64_t k = b; k < e; ++k) val[k] = value(row[k], col[k]);
  });
  return nnz;
}

extern "C" int64_t gnnea_h_relation_groups(const int64_t* tr, int64_t nt, int64_t n_rel,
                                           int64_t* rel_ptr, int64_t* heads, int64_t* tails) {
  if (nt < 0 || n_rel < 0 || (nt > 0 && !tr) || !rel_ptr || (nt > 0 && (!heads || !tails)))
    return GNNEA_H_EINVAL;
  std::fill(rel_ptr, rel_ptr + n_rel + 1, 0);
  for (int64_t i = 0; i < nt; ++i) {
    const int64_t r = tr[3 * i + 1];
    if (r < 0 || r >= n_rel) return GNNEA_H_EINVAL;
    ++rel_ptr[r + 1];
  }
  int64_t distinct = 0;
  for (int64_t r = 0; r < n_rel; ++r) {
    distinct += rel_ptr[r + 1] > 0;
    rel_ptr[r + 1] += rel_ptr[r];
  }
  std::vector<int64_t> fill(rel_ptr, rel_ptr + n_rel);
  for (int64_t i = 0; i < nt; ++i) {
    const int64_t r = tr[3 * i + 1];
    heads[fill[r]] = tr[3 * i];
    tails[fill[r]] = tr[3 * i + 2];
    ++fill[r];
  }
  return distinct;
}
