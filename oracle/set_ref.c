/*
 * ORACLE (test infrastructure only) — a multithreaded, SET-BASED CPU restatement of the MATCH
 * bindings of fixed-length forward chains (a -> b -> c ...), the "multithreaded C++ set-based CPU path"
 * SURVEY §8(d) asks for beside the faithful DFS (oracle/dfs_ref.c). Used by bench.py's cpu_baseline leg
 * (`set_based`) and checked against dfs_ref.c in tests/test_oracle_set.py. Never linked into the product.
 *
 * Same bindings as OMatchStatement.processContext (core/.../sql/parser/OMatchStatement.java:412-568) for
 * a chain of free forward hops, computed with the algebra the device uses instead of a per-root walk:
 *   per hop, over the R rows of the binding table (one u32 column per alias, row-major here):
 *     1. the distinct sources of the hop's source column (a V-byte marker, then a listing);
 *     2. per distinct source u, its filtered list L(u) = {r in N(u) : WHERE(r)} — a HashSet when the hop
 *        has a WHERE (P/OMatchPathItem.java:61,71-78), so a neighbour repeated by parallel edges is kept
 *        once (rows are sorted, so repeats are adjacent); an unfiltered hop's list is N(u) itself;
 *     3. the rows: row i continues once per entry of L(src_i) (offsets = the scan of |L(src_i)|).
 *   E_t (edges) = Σ over the rows entering each hop of deg(src_i), as the reference iterates them.
 * The last hop of a one-column projection can mark the union of its lists into a V-bit set instead of
 * writing rows (the distinct set of OBasicCommandContext.addToUniqueResult; bindings still Σ |L(src_i)|).
 *
 * Buffers live in one static context and are reused by the next call (bench repetitions do not pay
 * first-touch page faults again). Not thread-safe; one caller at a time.
 *
 * Build: make -C oracle   (gcc -O2 -fopenmp -shared → oracle/_build/libdfsref.so)
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SET_MAXH 8

typedef struct {
  int32_t src;              /* column of the hop's source alias (0 = the root) */
  int32_t set_valued;       /* 1: a neighbour repeated in N(u) is kept once (WHERE + a multigraph) */
  const uint64_t *rp;       /* CSR, rows ascending */
  const uint32_t *col;
  const uint64_t *where_bm; /* target WHERE as a V-bit set, NULL = none */
} set_hop;

typedef struct {
  int32_t nhops;
  set_hop hops[SET_MAXH];
} set_plan;

typedef struct {
  uint32_t *tab[2];
  uint64_t cap[2];          /* u32 words */
  uint8_t *flag;
  uint32_t *idx;
  uint64_t V;
  uint32_t *ulist;
  uint64_t *loff;
  uint32_t *lcol;
  uint64_t ucap, lcap;
  uint64_t *roff;
  uint64_t rcap;
  uint64_t max_rows;         /* the most rows any hop of the last run wrote (set_max_rows) */
  /* the last result */
  const uint32_t *rows;
  uint64_t nrows;
  int32_t k;
} set_ctx;

static set_ctx C;

/* set when a host allocation failed: the run stops and set_run returns -1 (the bench then skips the
   set-based baseline instead of crashing) */
static int set_oom;

/* grows *pp to hold `need` elements; 0 (and set_oom) when realloc fails, *pp and *cap unchanged */
static int grow(void **pp, uint64_t *cap, uint64_t need, size_t elem) {
  if (need <= *cap) return 1;
  uint64_t c = *cap ? *cap : 1024;
  while (c < need) c *= 2;
  void *q = realloc(*pp, c * elem);
  if (!q) {
    set_oom = 1;
    return 0;
  }
  *pp = q;
  *cap = c;
  return 1;
}
#define GROW(p, cap, need, elem) grow((void **)&(p), (cap), (need), (elem))

static inline int bm(const uint64_t *b, uint32_t v) { return (int)((b[v >> 6] >> (v & 63)) & 1ull); }

/* exclusive scan of a[0..n) into out[0..n] (out[n] = total) on T threads */
static void scan_u64(const uint64_t *a, uint64_t n, uint64_t *out, int T) {
  uint64_t part[257];
  if (T > 256) T = 256;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num(), nt = omp_get_num_threads();
    const uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += a[i];
    part[t + 1] = s;
#pragma omp barrier
#pragma omp single
    {
      part[0] = 0;
      for (int j = 1; j <= nt; ++j) part[j] += part[j - 1];
    }
    s = part[t];
    for (uint64_t i = lo; i < hi; ++i) {
      out[i] = s;
      s += a[i];
    }
    if (t == nt - 1) out[n] = s;
  }
}

/* one hop over the R rows of width k in `in`; returns the rows written to `out` (width k + 1), or, with
   mark != NULL, marks the union of the sources' lists and returns Σ |L(src_i)| */
static uint64_t hop(const set_hop *h, uint32_t V, const uint32_t *in, uint64_t R, int k, int slot, uint64_t *mark,
                    uint64_t *edges, int T) {
  const int s = h->src;
  /* 1. distinct sources (only a filtered hop lists them: an unfiltered list is the adjacency row) */
  const int filt = h->where_bm != NULL;
  uint64_t U = 0;
  if (filt) {
    if (C.V < V) {
      free(C.flag);
      free(C.idx);
      C.flag = (uint8_t *)calloc(V, 1);
      C.idx = (uint32_t *)malloc((size_t)V * 4);
      C.V = V;
      if (!C.flag || !C.idx) {
        free(C.flag);
        free(C.idx);
        C.flag = NULL;
        C.idx = NULL;
        C.V = 0;
        set_oom = 1;
        return 0;
      }
    }
#pragma omp parallel for num_threads(T) schedule(static)
    for (uint64_t i = 0; i < R; ++i) C.flag[in[i * k + s]] = 1;
    /* listing: per-thread counts over V, scanned */
    uint64_t cnt[257] = {0};
    int nt = T > 256 ? 256 : T;
#pragma omp parallel num_threads(nt)
    {
      const int t = omp_get_thread_num(), n = omp_get_num_threads();
      const uint64_t lo = (uint64_t)V * t / n, hi = (uint64_t)V * (t + 1) / n;
      uint64_t c = 0;
      for (uint64_t v = lo; v < hi; ++v) c += C.flag[v];
      cnt[t + 1] = c;
#pragma omp barrier
#pragma omp single
      {
        for (int j = 1; j <= n; ++j) cnt[j] += cnt[j - 1];
        U = cnt[n];
        if (GROW(C.ulist, &C.ucap, U + 1, 4)) {
          uint64_t *lo2 = (uint64_t *)realloc(C.loff, (C.ucap + 1) * 8);
          if (lo2) C.loff = lo2;
          else set_oom = 1;
        }
      }
      /* (the single's implicit barrier: every thread sees set_oom) */
      uint64_t p = cnt[t];
      for (uint64_t v = lo; v < hi; ++v)
        if (C.flag[v]) {
          C.flag[v] = 0;
          if (set_oom) continue;
          C.idx[v] = (uint32_t)p;
          C.ulist[p++] = (uint32_t)v;
        }
    }
    if (set_oom) return 0;
    /* 2. filtered lists: count, scan, fill */
    uint64_t *len = C.loff;  /* counts in place, then scanned into roff scratch and copied back */
#pragma omp parallel for num_threads(T) schedule(dynamic, 256)
    for (uint64_t u = 0; u < U; ++u) {
      const uint32_t v = C.ulist[u];
      uint64_t c = 0;
      uint32_t last = UINT32_MAX;
      for (uint64_t e = h->rp[v]; e < h->rp[v + 1]; ++e) {
        const uint32_t r = h->col[e];
        if (!bm(h->where_bm, r)) continue;
        if (h->set_valued && r == last) continue;
        last = r;
        ++c;
      }
      len[u] = c;
    }
    if (!GROW(C.roff, &C.rcap, U + 1 > R + 1 ? U + 1 : R + 1, 8)) return 0;
    scan_u64(len, U, C.roff, T);
    memcpy(C.loff, C.roff, (U + 1) * 8);
    const uint64_t NL = C.loff[U];
    if (!GROW(C.lcol, &C.lcap, NL + 1, 4)) return 0;
#pragma omp parallel for num_threads(T) schedule(dynamic, 256)
    for (uint64_t u = 0; u < U; ++u) {
      const uint32_t v = C.ulist[u];
      uint64_t o = C.loff[u];
      uint32_t last = UINT32_MAX;
      for (uint64_t e = h->rp[v]; e < h->rp[v + 1]; ++e) {
        const uint32_t r = h->col[e];
        if (!bm(h->where_bm, r)) continue;
        if (h->set_valued && r == last) continue;
        last = r;
        C.lcol[o++] = r;
      }
    }
  }
  /* 3. rows: per row its list length (and its source's degree, E_t), scanned */
  uint64_t *rl = (uint64_t *)malloc((R + 1) * 8);
  if (!rl) {
    set_oom = 1;
    return 0;
  }
  uint64_t et = 0;
#pragma omp parallel for num_threads(T) schedule(static) reduction(+ : et)
  for (uint64_t i = 0; i < R; ++i) {
    const uint32_t v = in[i * k + s];
    et += h->rp[v + 1] - h->rp[v];
    if (filt) {
      const uint32_t u = C.idx[v];
      rl[i] = C.loff[u + 1] - C.loff[u];
    } else {
      rl[i] = h->rp[v + 1] - h->rp[v];
    }
  }
  *edges += et;
  if (mark) {
    /* the distinct set of the last column: the union of the sources' lists */
    uint64_t tot = 0;
#pragma omp parallel for num_threads(T) schedule(static) reduction(+ : tot)
    for (uint64_t i = 0; i < R; ++i) tot += rl[i];
    if (filt) {
#pragma omp parallel for num_threads(T) schedule(dynamic, 256)
      for (uint64_t u = 0; u < U; ++u)
        for (uint64_t e = C.loff[u]; e < C.loff[u + 1]; ++e) {
          const uint32_t r = C.lcol[e];
          if (!bm(mark, r)) __atomic_fetch_or(&mark[r >> 6], 1ull << (r & 63), __ATOMIC_RELAXED);
        }
    } else {
      /* unfiltered: the distinct sources' adjacency rows (each source once) */
      uint8_t *seen_src = (uint8_t *)calloc(V, 1);
      if (!seen_src) {
        set_oom = 1;
        free(rl);
        return 0;
      }
#pragma omp parallel for num_threads(T) schedule(dynamic, 1024)
      for (uint64_t i = 0; i < R; ++i) {
        const uint32_t v = in[i * k + s];
        if (seen_src[v] || __atomic_exchange_n(&seen_src[v], 1, __ATOMIC_RELAXED)) continue;
        for (uint64_t e = h->rp[v]; e < h->rp[v + 1]; ++e) {
          const uint32_t r = h->col[e];
          if (!bm(mark, r)) __atomic_fetch_or(&mark[r >> 6], 1ull << (r & 63), __ATOMIC_RELAXED);
        }
      }
      free(seen_src);
    }
    free(rl);
    return tot;
  }
  if (!GROW(C.roff, &C.rcap, R + 1, 8)) {
    free(rl);
    return 0;
  }
  scan_u64(rl, R, C.roff, T);
  free(rl);
  const uint64_t N = C.roff[R];
  const int k2 = k + 1;
  if (N > C.max_rows) C.max_rows = N;
  if (!GROW(C.tab[slot], &C.cap[slot], N * k2 + 1, 4)) return 0;
  uint32_t *out = C.tab[slot];
#pragma omp parallel for num_threads(T) schedule(dynamic, 1024)
  for (uint64_t i = 0; i < R; ++i) {
    const uint32_t *row = in + i * k;
    const uint32_t v = row[s];
    const uint32_t *l;
    uint64_t n;
    if (filt) {
      const uint32_t u = C.idx[v];
      l = C.lcol + C.loff[u];
      n = C.loff[u + 1] - C.loff[u];
    } else {
      l = h->col + h->rp[v];
      n = h->rp[v + 1] - h->rp[v];
    }
    uint32_t *o = out + C.roff[i] * k2;
    for (uint64_t j = 0; j < n; ++j, o += k2) {
      for (int c = 0; c < k; ++c) o[c] = row[c];
      o[k] = l[j];
    }
  }
  return N;
}

/* Runs the chain from `roots` (column 0). Returns the complete bindings; *edges = E_t. With mark != NULL
   the last hop marks its column's distinct set (a V-bit set) instead of writing rows; otherwise the rows
   stay in the context (set_rows). */
int64_t set_run(const set_plan *p, uint32_t V, const uint32_t *roots, int64_t nroots, int32_t nthreads, uint64_t *mark,
                uint64_t *edges) {
  const int T = nthreads < 1 ? 1 : nthreads;
  *edges = 0;
  set_oom = 0;
  C.max_rows = 0;
  C.rows = NULL;
  C.nrows = 0;
  C.k = 0;
  if (!GROW(C.tab[0], &C.cap[0], (uint64_t)nroots + 1, 4)) return -1;
  memcpy(C.tab[0], roots, (size_t)nroots * 4);
  const uint32_t *in = C.tab[0];
  uint64_t R = (uint64_t)nroots;
  int k = 1, slot = 1;
  for (int h = 0; h < p->nhops; ++h) {
    const int last = h == p->nhops - 1;
    if (last && mark) {
      const uint64_t b = hop(&p->hops[h], V, in, R, k, slot, mark, edges, T);
      return set_oom ? -1 : (int64_t)b;
    }
    R = hop(&p->hops[h], V, in, R, k, slot, NULL, edges, T);
    if (set_oom) return -1;
    in = C.tab[slot];
    slot ^= 1;
    ++k;
  }
  C.rows = in;
  C.nrows = R;
  C.k = k;
  return (int64_t)R;
}

static inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* Σ over the last result's rows of the splitmix64 chain of the projected columns' RIDs (the digest of
   oracle/dfs.py row_digest and the device's OMX_FLAG_DIGEST when the rows are distinct) */
uint64_t set_digest(const int32_t *proj, int32_t nproj, uint64_t rid_base, int32_t nthreads) {
  uint64_t d = 0;
  const int k = C.k;
#pragma omp parallel for num_threads(nthreads < 1 ? 1 : nthreads) schedule(static) reduction(+ : d)
  for (uint64_t i = 0; i < C.nrows; ++i) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int c = 0; c < nproj; ++c) h = mix64(h ^ (rid_base | C.rows[i * k + proj[c]]));
    d += h;
  }
  return d;
}

/* the last result: rows (row-major, *k u32 each), valid until the next set_run */
/* the most rows one hop of the last set_run wrote (the run's peak table, rows of width ≤ 9) */
uint64_t set_max_rows(void) { return C.max_rows; }

const uint32_t *set_rows(uint64_t *n, int32_t *k) {
  *n = C.nrows;
  *k = C.k;
  return C.rows;
}
