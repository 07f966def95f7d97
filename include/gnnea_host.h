/*
 * gnnea_host.h — host-side (CPU, C++) KG ingestion of libgnnea_host.so.
 *
 * Replaces the per-line / per-triple Python loops of the reference's entity-alignment loaders:
 *   loadfile            utils/data_utils.py:362-372   (tab-separated integer columns)
 *   get_matrix +        utils/data_utils.py:296-336   (normalised two-KG adjacency, COO in the
 *   get_sparse_tensor                                   reference's dict-insertion order)
 *   rfunc               utils/data_utils.py:272-293   (relation head / tail incidence)
 * Plain pointers and sizes; host memory, caller-owned; return >= 0 on success (a count) or a
 * negative GNNEA_H_E* code.  Thread-safe, no global state.
 */
#ifndef GNNEA_HOST_H
#define GNNEA_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNNEA_H_EINVAL (-1)   /* bad argument */
#define GNNEA_H_EIO (-2)      /* file cannot be opened / read */
#define GNNEA_H_EPARSE (-3)   /* a line has fewer than ncols integer fields (int() would raise) */
#define GNNEA_H_ESPACE (-4)   /* output capacity too small */

/* Rows of a text file as the reference's loadfile(fn, num) reads them: each line minus its last
 * character (line[:-1], so a final line without a newline loses its last digit, as in the
 * reference), split on '\t', the first ncols fields parsed as integers (int(): surrounding
 * whitespace and a sign allowed).  out: rows x ncols int64, row-major, capacity cap_rows.
 * Returns the row count; with out == NULL only counts. */
int64_t gnnea_h_loadfile(const char* path, int32_t ncols, int64_t* out, int64_t cap_rows);

/* Normalised adjacency of a triple list (h, r, t) over n_ent entities, as get_sparse_tensor:
 *   entries (h,t), (t,h) of every triple with h != t, first occurrence order, then a self loop
 *   (e,e) for every entity in order of first appearance (h before t in each triple);
 *   value 1 / sqrt(deg_r) / sqrt(deg_c) in fp64 rounded to fp32, deg = 1 + #non-self triples
 *   touching the entity (multi-edges counted).
 * reference_order == 0 returns the same entries sorted by (row, col) instead.
 * Returns nnz; with row == NULL only counts (cap ignored).  Entity ids must be in [0, n_ent). */
int64_t gnnea_h_adjacency(const int64_t* triples, int64_t n_triples, int64_t n_ent,
                          int32_t reference_order, int64_t* row, int64_t* col, float* val,
                          int64_t cap);

/* Relation incidence of rfunc: for every relation r (ids in [0, n_rel)) the number of triples
 * and, grouped by relation in triple order, their heads and tails:
 *   rel_ptr[n_rel+1] (CSR offsets), heads[n_triples], tails[n_triples].
 * Returns the number of distinct relations that occur. */
int64_t gnnea_h_relation_groups(const int64_t* triples, int64_t n_triples, int64_t n_rel,
                                int64_t* rel_ptr, int64_t* heads, int64_t* tails);

#ifdef __cplusplus
}
#endif
#endif /* GNNEA_HOST_H */
