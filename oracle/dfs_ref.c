/*
 * ORACLE (test infrastructure only) — plain-C restatement of the reference's MATCH DFS for
 * fixed-length patterns, used (1) as the parity checker at RMAT scales the Python oracle cannot
 * reach and (2) as bench.py's cpu_baseline leg ("port"). Never linked into the product.
 *
 * Restates OMatchStatement.processContext (core/.../sql/parser/OMatchStatement.java:412-568):
 * one recursion level per sorted pattern edge; for each neighbour r of the bound source
 *   - target already bound      → keep the branch iff r == bound (existence, `break` at :476)
 *   - target prefetched (< 20)  → bind r if r ∈ candidates (:478-490)
 *   - target free               → bind r (:491-497)
 * Forward edges filter neighbours with the target's WHERE inside OMatchPathItem.executeTraversal
 * (P/OMatchPathItem.java:63-78, a HashSet when filtered); reverse edges use executeReverse and apply
 * the WHERE only in the free branch (:553-554). Filters arrive as V-bit bitmaps evaluated by the
 * Python oracle. Complete bindings are emitted (de-duplication happens in the caller, as
 * OBasicCommandContext.addToUniqueResult does).
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -shared → oracle/_build/libdfsref.so)
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MAXP 4
#define MAXA 16
#define MODE_FREE 0
#define MODE_CAND 1
#define MODE_BOUND 2

typedef struct {
  int32_t src, dst;           /* alias indices */
  int32_t mode;               /* MODE_* */
  int32_t forward;            /* 1 = executeTraversal (WHERE applied), 0 = executeReverse */
  int32_t nparts;
  const uint64_t *rp[MAXP];
  const uint32_t *col[MAXP];
  const uint64_t *where_bm;   /* target WHERE (NULL = none) */
  const uint64_t *cand_bm;    /* candidate set (class ∧ WHERE) for MODE_CAND */
  int32_t need_dedup;         /* neighbour lists may repeat a vertex (several parts / parallel edges) */
  int32_t sorted;             /* every part's rows ascending */
} dfs_step;

typedef struct {
  int32_t nsteps, naliases;
  dfs_step steps[MAXA];
} dfs_plan;

typedef struct {
  uint32_t *buf;
  uint64_t n, cap;   /* rows */
  uint64_t edges;    /* adjacency entries read */
  uint64_t bindings;
  int emit;
  int k;
  /* whole-result checks at sizes where rows cannot be kept: the projected columns of every binding are
     hashed (digest of a result whose rows are distinct by construction), or, for a one-column
     projection, marked in a V-bit set (the distinct set, OBasicCommandContext.addToUniqueResult) */
  const int32_t *proj;
  int32_t nproj;
  uint64_t rid_base;
  uint64_t digest;
  uint64_t *seen;
} sink;

/* splitmix64 finalizer; the row hash chains it over the RIDs (same function as the device's
   OMX_FLAG_DIGEST and oracle/dfs.py row_digest) */
static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static inline int bm(const uint64_t *b, uint32_t v) { return (int)((b[v >> 6] >> (v & 63)) & 1ull); }

static void emit_row(sink *s, const uint32_t *bind) {
  s->bindings++;
  if (s->seen) {
    const uint32_t v = bind[s->proj[0]];
    __atomic_fetch_or(&s->seen[v >> 6], 1ull << (v & 63), __ATOMIC_RELAXED);
  } else if (s->nproj) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int c = 0; c < s->nproj; ++c) h = mix64(h ^ (s->rid_base | bind[s->proj[c]]));
    s->digest += h;
  }
  if (!s->emit) return;
  if (s->n == s->cap) {
    s->cap = s->cap ? s->cap * 2 : 1024;
    s->buf = (uint32_t *)realloc(s->buf, s->cap * s->k * sizeof(uint32_t));
  }
  memcpy(s->buf + s->n * s->k, bind, s->k * sizeof(uint32_t));
  s->n++;
}

static int contains(const uint32_t *a, uint64_t n, uint32_t x) {
  for (uint64_t i = 0; i < n; ++i)
    if (a[i] == x) return 1;
  return 0;
}

static void process(const dfs_plan *p, int e, uint32_t *bind, sink *s) {
  if (e == p->nsteps) {
    emit_row(s, bind);
    return;
  }
  const dfs_step *st = &p->steps[e];
  const uint32_t v = bind[st->src];
  /* neighbours of v; a filtered forward traversal returns a set (HashSet, OMatchPathItem.java:61,75) */
  uint32_t local[64];
  uint32_t *seen = local;
  uint64_t nseen = 0, capseen = 64;
  const int dedup = st->forward && st->where_bm != NULL && st->need_dedup;
  for (int q = 0; q < st->nparts; ++q) {
    const uint64_t lo = st->rp[q][v], hi = st->rp[q][v + 1];
    s->edges += hi - lo;
    for (uint64_t i = lo; i < hi; ++i) {
      const uint32_t r = st->col[q][i];
      if (st->forward && st->where_bm && !bm(st->where_bm, r)) continue;
      if (dedup) {
        if (contains(seen, nseen, r)) continue;
        if (nseen == capseen) {
          uint32_t *n2 = (uint32_t *)malloc(2 * capseen * sizeof(uint32_t));
          memcpy(n2, seen, nseen * sizeof(uint32_t));
          if (seen != local) free(seen);
          seen = n2;
          capseen *= 2;
        }
        seen[nseen++] = r;
      }
      if (st->mode == MODE_BOUND) {
        if (st->sorted && !dedup) {
          /* rows sorted: the first match is found by binary search (same branch taken as the
             linear scan + break of :468-477) */
          const uint32_t t = bind[st->dst];
          uint64_t a = lo, b = hi;
          while (a < b) {
            uint64_t m = (a + b) >> 1;
            if (st->col[q][m] < t) a = m + 1; else b = m;
          }
          if (a < hi && st->col[q][a] == t && (!st->forward || !st->where_bm || bm(st->where_bm, t))) {
            process(p, e + 1, bind, s);
            goto done;
          }
          break;
        }
        if (bind[st->dst] == r) {
          process(p, e + 1, bind, s);
          goto done; /* break (:476) */
        }
      } else if (st->mode == MODE_CAND) {
        if (bm(st->cand_bm, r)) {
          bind[st->dst] = r;
          process(p, e + 1, bind, s);
        }
      } else {
        if (!st->forward && st->where_bm && !bm(st->where_bm, r)) continue;
        bind[st->dst] = r;
        process(p, e + 1, bind, s);
      }
    }
  }
done:
  if (seen != local) free(seen);
}

/* Runs the DFS from every root (bound to alias `root_alias`) on `nthreads` threads.
 * Returns complete bindings; rows (naliases u32 per row) when emit != 0, in *out (malloc'ed). */
/* dfs_run_ex: proj[0..nproj) = the RETURN columns (alias indices); with nproj > 0 every binding's
 * projection is hashed into *digest (RIDs = rid_base | dense id), or, when seen != NULL (nproj == 1),
 * set in the V-bit set `seen` instead. */
int64_t dfs_run_ex(const dfs_plan *p, int32_t root_alias, const uint32_t *roots, int64_t nroots, int32_t nthreads,
                   int32_t emit, uint32_t **out, uint64_t *out_rows, uint64_t *edges, const int32_t *proj,
                   int32_t nproj, uint64_t rid_base, uint64_t *digest, uint64_t *seen) {
  if (nthreads < 1) nthreads = 1;
  sink *sinks = (sink *)calloc(nthreads, sizeof(sink));
  for (int t = 0; t < nthreads; ++t) {
    sinks[t].emit = emit;
    sinks[t].k = p->naliases;
    sinks[t].proj = proj;
    sinks[t].nproj = nproj;
    sinks[t].rid_base = rid_base;
    sinks[t].seen = nproj == 1 ? seen : NULL;
  }
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
  for (int64_t i = 0; i < nroots; ++i) {
    sink *s = &sinks[omp_get_thread_num()];
    uint32_t bind[MAXA];
    memset(bind, 0, sizeof(bind));
    bind[root_alias] = roots[i];
    process(p, 0, bind, s);
  }
  uint64_t total = 0, rows = 0, ed = 0, dg = 0;
  for (int t = 0; t < nthreads; ++t) {
    dg += sinks[t].digest;
    total += sinks[t].bindings;
    rows += sinks[t].n;
    ed += sinks[t].edges;
  }
  if (emit) {
    uint32_t *buf = (uint32_t *)malloc((rows ? rows : 1) * p->naliases * sizeof(uint32_t));
    uint64_t off = 0;
    for (int t = 0; t < nthreads; ++t) {
      if (sinks[t].n) memcpy(buf + off * p->naliases, sinks[t].buf, sinks[t].n * p->naliases * sizeof(uint32_t));
      off += sinks[t].n;
      free(sinks[t].buf);
    }
    *out = buf;
    *out_rows = rows;
  }
  if (edges) *edges = ed;
  if (digest) *digest = dg;
  free(sinks);
  return (int64_t)total;
}

int64_t dfs_run(const dfs_plan *p, int32_t root_alias, const uint32_t *roots, int64_t nroots, int32_t nthreads,
                int32_t emit, uint32_t **out, uint64_t *out_rows, uint64_t *edges) {
  return dfs_run_ex(p, root_alias, roots, nroots, nthreads, emit, out, out_rows, edges, NULL, 0, 0, NULL, NULL);
}

void dfs_free(void *p) { free(p); }
