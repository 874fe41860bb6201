/*
 * ORACLE (test infrastructure only) — plain-C restatement of a variable-length MATCH item
 * (OMatchPathItem.executeTraversal with while/maxDepth, core/.../sql/parser/OMatchPathItem.java:79-105)
 * for the case where WHERE does not read $depth and `while` reads nothing but $depth. The reference
 * recurses over walks; a vertex v is in the result set of a start vertex iff some walk of length
 * d ≤ D reaches it (D = first depth where `while` is false, or maxDepth) and WHERE(v) holds, i.e. iff
 * its BFS distance is ≤ D. One start vertex per thread, a stamped distance array, level by level.
 * Used (1) as a second checker at scales the walk-enumerating Python oracle cannot reach and (2) as
 * bench.py's cpu_baseline leg for configs[2]. Never linked into the product.
 *
 * Edge accounting follows SURVEY §8(d): Σ over levels d < D of the degrees of the level's vertices.
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline int bm(const uint64_t *w, uint32_t v) { return (int)((w[v >> 6] >> (v & 63)) & 1ull); }

typedef struct {
  uint32_t *buf;
  uint64_t n, cap;
} pairs;

static void push_pair(pairs *p, uint32_t a, uint32_t b) {
  if (p->n == p->cap) {
    p->cap = p->cap ? p->cap * 2 : 1024;
    p->buf = (uint32_t *)realloc(p->buf, p->cap * 2 * sizeof(uint32_t));
  }
  p->buf[2 * p->n] = a;
  p->buf[2 * p->n + 1] = b;
  p->n++;
}

/* Returns the number of (root index, v) results; pairs in *out when emit != 0 (malloc'ed, 2 u32 per
 * pair). max_depth < 0 = unbounded. where_bm may be NULL. */
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* *digest (may be NULL): Σ over the (root, v) results of the row hash of (rid_base | roots[i],
 * rid_base | v) — the device's OMX_FLAG_DIGEST of `RETURN s, v` (oracle/dfs.py row_digest). */
int64_t bfs_varlen_ex(const uint64_t *rp, const uint32_t *col, uint32_t V, const uint32_t *roots, int64_t nroots,
                      int32_t max_depth, const uint64_t *where_bm, int32_t nthreads, int32_t emit, uint32_t **out,
                      uint64_t *out_pairs, uint64_t *edges, uint64_t rid_base, uint64_t *digest) {
  if (nthreads < 1) nthreads = 1;
  pairs *sinks = (pairs *)calloc(nthreads, sizeof(pairs));
  uint64_t *tedges = (uint64_t *)calloc(nthreads, sizeof(uint64_t));
  uint64_t *tcount = (uint64_t *)calloc(nthreads, sizeof(uint64_t));
  uint64_t *tdig = (uint64_t *)calloc(nthreads, sizeof(uint64_t));
#pragma omp parallel num_threads(nthreads)
  {
    const int t = omp_get_thread_num();
    uint32_t *stamp = (uint32_t *)calloc(V, sizeof(uint32_t));
    uint32_t *queue = (uint32_t *)malloc((size_t)V * sizeof(uint32_t));
#pragma omp for schedule(dynamic, 1)
    for (int64_t i = 0; i < nroots; ++i) {
      const uint32_t mark = (uint32_t)(i + 1);
      uint64_t head = 0, tail = 0;
      queue[tail++] = roots[i];
      stamp[roots[i]] = mark;
      for (int32_t d = 0;; ++d) {
        const uint64_t level_end = tail;
        for (uint64_t q = head; q < level_end; ++q) {
          const uint32_t v = queue[q];
          if (!where_bm || bm(where_bm, v)) {
            tcount[t]++;
            if (digest) tdig[t] += mix64(mix64(0x9E3779B97F4A7C15ull ^ (rid_base | roots[i])) ^ (rid_base | v));
            if (emit) push_pair(&sinks[t], (uint32_t)i, v);
          }
        }
        if ((max_depth >= 0 && d >= max_depth) || head == level_end) break;
        for (uint64_t q = head; q < level_end; ++q) {
          const uint32_t v = queue[q];
          tedges[t] += rp[v + 1] - rp[v];
          for (uint64_t j = rp[v]; j < rp[v + 1]; ++j) {
            const uint32_t w = col[j];
            if (stamp[w] != mark) {
              stamp[w] = mark;
              queue[tail++] = w;
            }
          }
        }
        head = level_end;
        if (head == tail) break;
      }
    }
    free(stamp);
    free(queue);
  }
  uint64_t total = 0, ed = 0, dg = 0;
  for (int t = 0; t < nthreads; ++t) {
    total += tcount[t];
    ed += tedges[t];
    dg += tdig[t];
  }
  if (digest) *digest = dg;
  if (emit) {
    uint32_t *buf = (uint32_t *)malloc((total ? total : 1) * 2 * sizeof(uint32_t));
    uint64_t off = 0;
    for (int t = 0; t < nthreads; ++t) {
      if (sinks[t].n) memcpy(buf + 2 * off, sinks[t].buf, sinks[t].n * 2 * sizeof(uint32_t));
      off += sinks[t].n;
      free(sinks[t].buf);
    }
    *out = buf;
    *out_pairs = total;
  }
  if (edges) *edges = ed;
  free(sinks);
  free(tedges);
  free(tcount);
  free(tdig);
  return (int64_t)total;
}

int64_t bfs_varlen(const uint64_t *rp, const uint32_t *col, uint32_t V, const uint32_t *roots, int64_t nroots,
                   int32_t max_depth, const uint64_t *where_bm, int32_t nthreads, int32_t emit, uint32_t **out,
                   uint64_t *out_pairs, uint64_t *edges) {
  return bfs_varlen_ex(rp, col, V, roots, nroots, max_depth, where_bm, nthreads, emit, out, out_pairs, edges, 0, NULL);
}
