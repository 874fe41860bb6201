// gen.cpp — deterministic synthetic inputs and host CSR utilities.
//
// Graph500 RMAT (A=.57, B=.19, C=.19, D=.05), edge factor 16. Every edge is a pure function of
// (seed, edge index) through splitmix64, so the same graph is produced by any thread count and by
// the numpy restatement in the tests; vertex ids are scrambled by a seeded bijection of [0, 2^scale)
// so hubs are spread over the id space (and over GPUs under a modulo partition).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <thread>
#include <unordered_set>
#include <vector>

#include "common.h"

namespace {

template <class F>
void par(uint64_t n, F f) {
  unsigned nt = omx::host_threads();
  if (n < (1u << 16)) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t) th.emplace_back([=] { f(n * t / nt, n * (t + 1) / nt); });
  for (auto &x : th) x.join();
}

struct Rmat {
  int scale;
  uint64_t seed, mask, m1, m2, c1, c2;
  // thresholds on a 32-bit uniform: A, A+B, A+B+C
  static constexpr uint32_t TA = (uint32_t)(0.57 * 4294967296.0);
  static constexpr uint32_t TB = (uint32_t)(0.76 * 4294967296.0);
  static constexpr uint32_t TC = (uint32_t)(0.95 * 4294967296.0);
  Rmat(int s, uint64_t sd) : scale(s), seed(sd) {
    mask = (scale >= 64) ? ~0ull : ((1ull << scale) - 1);
    m1 = omx::splitmix64(seed ^ 0x1111) | 1;
    m2 = omx::splitmix64(seed ^ 0x2222) | 1;
    c1 = omx::splitmix64(seed ^ 0x3333);
    c2 = omx::splitmix64(seed ^ 0x4444);
  }
  // bijection of [0, 2^scale): odd multiply, add, xor-shift (each invertible mod 2^scale)
  uint64_t scramble(uint64_t x) const {
    int h = scale / 2 + 1;
    x = (x * m1 + c1) & mask;
    x ^= x >> h;
    x = (x * m2 + c2) & mask;
    x ^= x >> h;
    return x & mask;
  }
  void edge(uint64_t i, uint32_t &u, uint32_t &v) const {
    uint64_t a = 0, b = 0, st = seed * 0x9E3779B97F4A7C15ull + i * 0xD1B54A32D192ED03ull;
    uint64_t r = 0;
    for (int lvl = 0; lvl < scale; ++lvl) {
      if ((lvl & 1) == 0) r = omx::splitmix64(st + (uint64_t)lvl);
      uint32_t x = (lvl & 1) ? (uint32_t)(r >> 32) : (uint32_t)r;
      int q = x < TA ? 0 : x < TB ? 1 : x < TC ? 2 : 3;
      a = (a << 1) | (q >> 1);
      b = (b << 1) | (q & 1);
    }
    u = (uint32_t)scramble(a);
    v = (uint32_t)scramble(b);
  }
};

}  // namespace

namespace omx {
unsigned host_threads() {
  unsigned n = std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
  if (const char *e = std::getenv("OMP_NUM_THREADS")) {
    const long k = std::strtol(e, nullptr, 10);
    if (k > 0) n = std::min<unsigned>(n, (unsigned)k);
  }
  return n;
}
}  // namespace omx

extern "C" {

void omx_host_free(void *p) { std::free(p); }

int omx_csr_transpose(uint32_t V, const uint64_t *rp, const uint32_t *col, uint64_t **trp, uint32_t **tcol) {
  const uint64_t E = rp[V];
  std::vector<std::atomic<uint64_t>> deg(V);
  for (auto &d : deg) d.store(0, std::memory_order_relaxed);
  par(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v)
      for (uint64_t e = rp[v]; e < rp[v + 1]; ++e) deg[col[e]].fetch_add(1, std::memory_order_relaxed);
  });
  uint64_t *orp = (uint64_t *)std::malloc(sizeof(uint64_t) * ((size_t)V + 1));
  uint32_t *ocol = (uint32_t *)std::malloc(sizeof(uint32_t) * std::max<uint64_t>(E, 1));
  if (!orp || !ocol) return OMX_E_OOM;
  orp[0] = 0;
  for (uint32_t v = 0; v < V; ++v) orp[v + 1] = orp[v] + deg[v].load(std::memory_order_relaxed);
  for (uint32_t v = 0; v < V; ++v) deg[v].store(orp[v], std::memory_order_relaxed);
  par(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v)
      for (uint64_t e = rp[v]; e < rp[v + 1]; ++e) ocol[deg[col[e]].fetch_add(1, std::memory_order_relaxed)] = (uint32_t)v;
  });
  par(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v) std::sort(ocol + orp[v], ocol + orp[v + 1]);
  });
  *trp = orp;
  *tcol = ocol;
  return OMX_OK;
}

int omx_rmat_generate(int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple, uint64_t **out_rp,
                      uint32_t **out_col, uint64_t *n_edges) {
  if (scale < 1 || scale > 31 || edge_factor < 1 || !out_rp || !out_col || !n_edges) return OMX_E_INVALID;
  const uint64_t V = 1ull << scale, M = (uint64_t)edge_factor * V;
  Rmat g(scale, seed);
  std::vector<std::atomic<uint64_t>> deg(V);
  for (auto &d : deg) d.store(0, std::memory_order_relaxed);
  par(M, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t u, v;
      g.edge(i, u, v);
      deg[u].fetch_add(1, std::memory_order_relaxed);
    }
  });
  std::vector<uint64_t> rp(V + 1, 0);
  for (uint64_t v = 0; v < V; ++v) rp[v + 1] = rp[v] + deg[v].load(std::memory_order_relaxed);
  for (uint64_t v = 0; v < V; ++v) deg[v].store(rp[v], std::memory_order_relaxed);
  uint32_t *col = (uint32_t *)std::malloc(sizeof(uint32_t) * std::max<uint64_t>(M, 1));
  if (!col) return OMX_E_OOM;
  par(M, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t u, v;
      g.edge(i, u, v);
      col[deg[u].fetch_add(1, std::memory_order_relaxed)] = v;
    }
  });
  // sort rows; optionally drop self loops and parallel edges (SURVEY §8(d) headline runs)
  std::vector<uint64_t> keep(V, 0);
  par(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v) {
      uint32_t *b = col + rp[v], *e = col + rp[v + 1];
      std::sort(b, e);
      if (simple) {
        uint32_t *w = b;
        for (uint32_t *x = b; x < e; ++x)
          if (*x != (uint32_t)v && (w == b || *(w - 1) != *x)) *w++ = *x;
        keep[v] = (uint64_t)(w - b);
      } else {
        keep[v] = (uint64_t)(e - b);
      }
    }
  });
  uint64_t *orp = (uint64_t *)std::malloc(sizeof(uint64_t) * (V + 1));
  if (!orp) {
    std::free(col);
    return OMX_E_OOM;
  }
  orp[0] = 0;
  for (uint64_t v = 0; v < V; ++v) orp[v + 1] = orp[v] + keep[v];
  const uint64_t E = orp[V];
  if (simple) {  // compact in place (destination never passes the source)
    for (uint64_t v = 0; v < V; ++v)
      if (orp[v] != rp[v]) std::memmove(col + orp[v], col + rp[v], keep[v] * sizeof(uint32_t));
    uint32_t *shrunk = (uint32_t *)std::realloc(col, sizeof(uint32_t) * std::max<uint64_t>(E, 1));
    if (shrunk) col = shrunk;
  }
  *out_rp = orp;
  *out_col = col;
  *n_edges = E;
  return OMX_OK;
}

// One 1-D partition of the same RMAT graph: every rank replays all M edge draws (they are pure
// functions of the edge index) and keeps the out-edges of its sources and the in-edges of its
// destinations; each row is then sorted (and, for the simple graph, deduplicated and stripped of the
// self loop) exactly like the full generator's rows and the rows of their transpose.
static int rmat_rows(uint64_t M, const Rmat &g, uint32_t lo, uint32_t hi, bool by_dst, int32_t simple,
                     uint64_t **out_rp, uint32_t **out_col, uint64_t *n_edges) {
  const uint64_t VL = (uint64_t)hi - lo;
  std::vector<std::atomic<uint64_t>> deg(VL);
  for (auto &d : deg) d.store(0, std::memory_order_relaxed);
  auto key = [&](uint32_t u, uint32_t v) { return by_dst ? v : u; };
  par(M, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      uint32_t u, v;
      g.edge(i, u, v);
      const uint32_t k = key(u, v);
      if (k >= lo && k < hi) deg[k - lo].fetch_add(1, std::memory_order_relaxed);
    }
  });
  std::vector<uint64_t> rp(VL + 1, 0);
  for (uint64_t x = 0; x < VL; ++x) rp[x + 1] = rp[x] + deg[x].load(std::memory_order_relaxed);
  for (uint64_t x = 0; x < VL; ++x) deg[x].store(rp[x], std::memory_order_relaxed);
  uint32_t *col = (uint32_t *)std::malloc(sizeof(uint32_t) * std::max<uint64_t>(rp[VL], 1));
  if (!col) return OMX_E_OOM;
  par(M, [&](uint64_t a, uint64_t b) {
    for (uint64_t i = a; i < b; ++i) {
      uint32_t u, v;
      g.edge(i, u, v);
      const uint32_t k = key(u, v);
      if (k >= lo && k < hi) col[deg[k - lo].fetch_add(1, std::memory_order_relaxed)] = by_dst ? u : v;
    }
  });
  std::vector<uint64_t> keep(VL, 0);
  par(VL, [&](uint64_t a, uint64_t b) {
    for (uint64_t x = a; x < b; ++x) {
      uint32_t *s = col + rp[x], *e = col + rp[x + 1];
      std::sort(s, e);
      if (simple) {
        uint32_t *w = s;
        for (uint32_t *y = s; y < e; ++y)
          if (*y != (uint32_t)(lo + x) && (w == s || *(w - 1) != *y)) *w++ = *y;
        keep[x] = (uint64_t)(w - s);
      } else {
        keep[x] = (uint64_t)(e - s);
      }
    }
  });
  uint64_t *orp = (uint64_t *)std::malloc(sizeof(uint64_t) * (VL + 1));
  if (!orp) {
    std::free(col);
    return OMX_E_OOM;
  }
  orp[0] = 0;
  for (uint64_t x = 0; x < VL; ++x) orp[x + 1] = orp[x] + keep[x];
  if (simple)
    for (uint64_t x = 0; x < VL; ++x)
      if (orp[x] != rp[x]) std::memmove(col + orp[x], col + rp[x], keep[x] * sizeof(uint32_t));
  *out_rp = orp;
  *out_col = col;
  *n_edges = orp[VL];
  return OMX_OK;
}

int omx_rmat_generate_part(int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple, uint32_t lo, uint32_t hi,
                           uint64_t **out_rp, uint32_t **out_col, uint64_t *n_out, uint64_t **in_rp, uint32_t **in_col,
                           uint64_t *n_in) {
  if (scale < 1 || scale > 31 || edge_factor < 1 || lo > hi || hi > (1ull << scale) || !out_rp || !out_col ||
      !n_out || !in_rp || !in_col || !n_in)
    return OMX_E_INVALID;
  const uint64_t M = (uint64_t)edge_factor << scale;
  Rmat g(scale, seed);
  int rc = rmat_rows(M, g, lo, hi, false, simple, out_rp, out_col, n_out);
  if (rc != OMX_OK) return rc;
  rc = rmat_rows(M, g, lo, hi, true, simple, in_rp, in_col, n_in);
  if (rc != OMX_OK) {
    std::free(*out_rp);
    std::free(*out_col);
  }
  return rc;
}

// LDBC-SNB-like Knows graph (configs[3]). LDBC Datagen creates knows edges between persons that are
// close in a correlation dimension (university, interests, random), so the graph has a skewed degree
// distribution and many triangles. Restated here: target degrees from a log-normal scaled to
// 2·target_edges endpoint slots; three passes (45 % / 45 % / 10 % of every person's slots) each sort
// the persons by a key — community id with a skewed size distribution + random, twice, then random —
// and connect each person to the following ones in that order with a probability decaying with the
// distance, while both have slots left. Pairs are unique (no self loops); each undirected pair gets
// one directed Knows edge, oriented by a hash of the pair. Deterministic in (n_persons, edges, seed).
int omx_ldbc_knows_generate(uint32_t n_persons, uint64_t target_edges, uint64_t seed, uint64_t **out_rp,
                            uint32_t **out_col, uint64_t *n_edges) {
  if (n_persons < 2 || !out_rp || !out_col || !n_edges) return OMX_E_INVALID;
  const uint32_t N = n_persons;
  auto u01 = [](uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); };
  std::vector<double> t(N);
  double tsum = 0;
  for (uint32_t i = 0; i < N; ++i) {
    double z = 0;  // ≈ N(0,1): Irwin–Hall of 12 uniforms
    for (int k = 0; k < 12; ++k) z += u01(omx::splitmix64(seed ^ (0xD6E8FEB86659FD93ull * (i * 12ull + k + 1))));
    z -= 6.0;
    t[i] = std::exp(1.1 * z);
    tsum += t[i];
  }
  const double scale = 2.0 * (double)target_edges / tsum;
  std::vector<uint32_t> slots(N);
  for (uint32_t i = 0; i < N; ++i) slots[i] = (uint32_t)std::min<double>(std::max(1.0, std::round(t[i] * scale)), N / 4.0);
  std::unordered_set<uint64_t> pairs;
  pairs.reserve(target_edges * 2);
  const double share[3] = {0.45, 0.45, 0.10};
  const uint32_t ncomm[2] = {std::max<uint32_t>(1, N / 120), std::max<uint32_t>(1, N / 400)};
  std::vector<uint32_t> order(N), cap(N);
  std::vector<uint64_t> key(N);
  for (int pass = 0; pass < 3; ++pass) {
    for (uint32_t i = 0; i < N; ++i) {
      const uint64_t h = omx::splitmix64(seed * 31 + (uint64_t)pass * 0x100000001ull + i);
      if (pass < 2) {
        const double u = u01(omx::splitmix64(h ^ 0xC0FFEE));
        const uint64_t c = (uint64_t)(ncomm[pass] * u * u);  // low ids = large communities
        key[i] = (c << 32) | (h & 0xffffffffull);
      } else {
        key[i] = h;
      }
      cap[i] = (uint32_t)std::round(slots[i] * share[pass]);
    }
    std::iota(order.begin(), order.end(), 0u);
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return key[a] < key[b] || (key[a] == key[b] && a < b); });
    for (uint32_t k = 0; k < N; ++k) {
      const uint32_t i = order[k];
      const double lambda = 4.0 * (cap[i] + 1);
      for (uint32_t d = 1; cap[i] > 0 && d <= 4000 && k + d < N; ++d) {
        const uint32_t j = order[k + d];
        if (!cap[j]) continue;
        const uint64_t a = std::min(i, j), b = std::max(i, j), pk = (a << 32) | b;
        const double p = 0.9 * std::exp(-(double)d / lambda);
        if (u01(omx::splitmix64(pk ^ (seed + 0x51ED27u * (pass + 1)))) >= p) continue;
        if (pairs.insert(pk).second) {
          --cap[i];
          --cap[j];
        }
      }
    }
  }
  std::vector<uint64_t> deg(N + 1, 0);
  std::vector<std::pair<uint32_t, uint32_t>> edges;
  edges.reserve(pairs.size());
  for (uint64_t pk : pairs) {
    const uint32_t a = (uint32_t)(pk >> 32), b = (uint32_t)pk;
    if (omx::splitmix64(pk ^ seed ^ 0xABCDEFull) & 1) edges.emplace_back(a, b);
    else edges.emplace_back(b, a);
  }
  std::sort(edges.begin(), edges.end());
  const uint64_t E = edges.size();
  uint64_t *rp = (uint64_t *)std::malloc(sizeof(uint64_t) * ((size_t)N + 1));
  uint32_t *col = (uint32_t *)std::malloc(sizeof(uint32_t) * std::max<uint64_t>(E, 1));
  if (!rp || !col) {
    std::free(rp);
    std::free(col);
    return OMX_E_OOM;
  }
  std::memset(rp, 0, sizeof(uint64_t) * ((size_t)N + 1));
  for (uint64_t e = 0; e < E; ++e) {
    rp[edges[e].first + 1]++;
    col[e] = edges[e].second;
  }
  for (uint32_t v = 0; v < N; ++v) rp[v + 1] += rp[v];
  *out_rp = rp;
  *out_col = col;
  *n_edges = E;
  return OMX_OK;
}

int omx_synthetic_int_column(uint32_t V, uint64_t seed, int32_t modulo, int32_t **out) {
  if (modulo <= 0 || !out) return OMX_E_INVALID;
  int32_t *c = (int32_t *)std::malloc(sizeof(int32_t) * std::max<uint32_t>(V, 1));
  if (!c) return OMX_E_OOM;
  par(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v) c[v] = (int32_t)(omx::splitmix64(seed ^ (v * 0xA24BAED4963EE407ull)) % (uint64_t)modulo);
  });
  *out = c;
  return OMX_OK;
}

}  // extern "C"
