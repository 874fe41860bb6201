// bfs.hip — multi-source level-synchronous BFS for variable-length MATCH items.
//
// OMatchPathItem.executeTraversal with while/maxDepth (P/OMatchPathItem.java:79-105) enumerates
// walks depth-first without a visited set. When WHERE does not read $depth and `while` is either
// depth-free or reads nothing but $depth, the reference's result set for one start vertex is exactly
// {v : BFS distance(start, v) ≤ D in the graph restricted to expandable nodes, WHERE(v)} — so it is
// computed here by BFS, 64 binding rows at a time: every vertex holds a u64 lane mask (bit i = row i
// of the batch), and one level is
//     next[w] = OR_{v→w} (frontier[v] ∧ while(v)) ∧ ¬visited[w]
// evaluated top-down (push: atomicOr over the frontier's edges, for small frontiers) or bottom-up
// (pull: merge-path tiles over the reversed adjacency of the vertices that still miss a lane — the
// RMAT levels that cover most of the graph). The result is emitted once per batch from the visited
// masks.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "devutil.h"
#include "graph.h"
#include "kernels.h"

namespace omx {

namespace {
constexpr int kB = 256;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}
}  // namespace

// seeds: lane i of the batch starts at src[row0 + i]
// touched (optional): each distinct seed vertex once (the first level's sparse prologue)
__global__ void k_bfs_seed(const uint32_t *src, uint64_t row0, int nl, uint64_t *frontier, uint32_t *touched,
                           unsigned long long *touched_n) {
  int i = threadIdx.x;
  if (i < nl) {
    const uint32_t v = src[row0 + i];
    const uint64_t old = atomicOr((unsigned long long *)&frontier[v], 1ull << i);
    if (touched && old == 0) touched[atomicAdd(touched_n, 1ull)] = v;
  }
}
void launch_bfs_seed(const uint32_t *src, uint64_t row0, int nl, uint64_t *frontier, hipStream_t s, uint32_t *touched,
                     unsigned long long *touched_n) {
  hipLaunchKernelGGL(k_bfs_seed, dim3(1), dim3(64), 0, s, src, row0, nl, frontier, touched, touched_n);
  KCHECK("k_bfs_seed");
}

// Level prologue over every vertex (grid-stride): m = frontier ∧ ¬visited (the level's new vertices) is
// merged into visited; if the level expands, m is cut to the `while` bitmap and the frontier's
// statistics are accumulated (one atomic per block and counter): stats[0] = Σ popc(m)·deg (the edges
// the reference traverses, SURVEY §8(d) E_t), stats[1] = Σ deg over active vertices (push work),
// stats[2] = active vertices, stats[3] = OR of m (the live lanes: a lane whose frontier is empty
// reaches nothing more, so the pull does not wait for it); with hub_bm (the pull's hubs, V bits)
// stats[4] / stats[5] = the same push work / count over the active vertices that are not hubs (what a
// hubs-only pull leaves to a push).
__global__ __launch_bounds__(kB) void k_bfs_prep(uint64_t *frontier, uint64_t *visited, uint32_t vlo, uint32_t V,
                                                 const uint64_t *while_bm, int expand, DAdj adj,
                                                 unsigned long long *stats, uint64_t *fbm, const uint64_t *hub_bm,
                                                 uint64_t *zero, int first, int zfull) {
  __shared__ uint64_t s_r[6][kB / 64];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t te = 0, td = 0, tn = 0, tl = 0, hd = 0, hn = 0;
  // kPrepU block-strides per round, their frontier words loaded together (clamped, unconditional)
  // before any store: one iteration at a time waited a memory round trip per 256 vertices, since each
  // iteration's load came after the previous one's stores (vector memory completes in order)
  constexpr int kPrepU = 4;
  for (uint64_t b0 = vlo + (uint64_t)blockIdx.x * kB * kPrepU; b0 < V; b0 += (uint64_t)gridDim.x * kB * kPrepU) {
    uint64_t fu[kPrepU], ou[kPrepU];
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const uint64_t v = b0 + (uint64_t)u * kB + threadIdx.x;
      const uint64_t x = frontier[v < V ? v : V - 1];
      fu[u] = v < V ? x : 0;
      // the previous level's frontier bits (before this level's ballot overwrites them): the next-mask
      // array is the previous frontier array, non-zero only there
      const uint64_t wi = (b0 + (uint64_t)u * kB) / 64 + wave;
      ou[u] = (zero && !zfull && wi * 64 < V) ? fbm[wi] : ~0ull;
    }
#pragma unroll
    for (int u = 0; u < kPrepU; ++u) {
      const uint64_t v0 = b0 + (uint64_t)u * kB;
      const uint64_t v = v0 + threadIdx.x;
      const uint64_t f = fu[u];
      if (zero && v < V && ((ou[u] >> lane) & 1ull)) zero[v] = 0;
      if (first && v < V) visited[v] = f;  // (a batch's first level: visited is written, never read)
      uint64_t m = 0;
      if (f) {
        const uint64_t vis = first ? 0ull : visited[v];
        m = f & ~vis;
        if (m && !first) visited[v] = vis | m;
        if (expand && while_bm && !bm_test(while_bm, (uint32_t)v)) m = 0;
        if (m != f) frontier[v] = m;
        if (m && expand) {
          const uint64_t d = adj_degree(adj, (uint32_t)v);
          te += (uint64_t)__popcll(m) * d;
          td += d;
          tn += 1;
          tl |= m;
          if (hub_bm && !bm_test(hub_bm, (uint32_t)v)) {
            hd += d;
            hn += 1;
          }
        }
      }
      const uint64_t word = __ballot(m != 0);  // bit v of fbm: v's frontier mask is non-empty
      if (fbm && lane == 0 && v0 + wave * 64 < V) fbm[(v0 >> 6) + wave] = word;
    }
  }
  if (!expand) return;
  te = wave_sum_u64(te);
  td = wave_sum_u64(td);
  tn = wave_sum_u64(tn);
  hd = wave_sum_u64(hd);
  hn = wave_sum_u64(hn);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) tl |= __shfl_xor(tl, off, 64);
  if (lane == 0) {
    s_r[0][wave] = te;
    s_r[1][wave] = td;
    s_r[2][wave] = tn;
    s_r[3][wave] = tl;
    s_r[4][wave] = hd;
    s_r[5][wave] = hn;
  }
  __syncthreads();
  if (threadIdx.x < 3 || (hub_bm && (threadIdx.x == 4 || threadIdx.x == 5))) {
    uint64_t x = 0;
    for (int w = 0; w < kB / 64; ++w) x += s_r[threadIdx.x][w];
    if (x) atomicAdd(&stats[threadIdx.x], (unsigned long long)x);
  } else if (threadIdx.x == 3) {
    uint64_t x = 0;
    for (int w = 0; w < kB / 64; ++w) x |= s_r[3][w];
    if (x) atomicOr(&stats[3], (unsigned long long)x);
  }
}
void launch_bfs_prep(uint64_t *frontier, uint64_t *visited, uint32_t V, const uint64_t *while_bm, bool expand,
                     const DAdj &adj, unsigned long long *stats, uint64_t *fbm, int cus, hipStream_t s, uint32_t vlo,
                     const uint64_t *hub_bm, uint64_t *zero, bool first, bool zero_all) {
  if (vlo && fbm) fail(OMX_E_INVALID, "internal: the frontier bitmap covers whole words from vertex 0");
  if (V <= vlo) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(V - vlo, kB * 4), (uint64_t)cus * 8);
  hipLaunchKernelGGL(k_bfs_prep, dim3(g), dim3(kB), 0, s, frontier, visited, vlo, V, while_bm, (int)expand, adj, stats,
                     fbm, hub_bm, zero, (int)first, (int)(zero_all || !fbm));
  KCHECK("k_bfs_prep");
}

// Sparse level prologue: when the previous level was a push, the vertices its atomics touched first
// (k_bfs_push's touched list) are the only ones whose frontier mask can be non-zero, so the prologue runs
// over that list instead of every vertex (C3's second and third levels: thousands of vertices, against a
// 16.8 M-vertex sweep of frontier + visited at ≈5.5 TB/s, 0.12 ms each). Two launches:
//   k_bfs_sparse_clear over the previous level's active list: the next-mask array (the previous level's
//     frontier array) zeroed and the frontier bitmap's bits cleared where they were set — what the full
//     prologue's `zero` / ballot do for every vertex;
//   k_bfs_prep_sparse over the touched list: the full prologue's per-vertex body (visited merge, while
//     cut, statistics, frontier bitmap bit) and the level's active list for the push (no k_bfs_list sweep).
// The lists' lengths live on the device (grid-stride loops over *n): no host round trip decides a grid.
__global__ __launch_bounds__(kB) void k_bfs_sparse_clear(const uint32_t *prev, const unsigned long long *n,
                                                         uint64_t *zero, uint64_t *fbm) {
  const uint64_t cnt = *n;
  for (uint64_t i = (uint64_t)blockIdx.x * kB + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * kB) {
    const uint32_t v = prev[i];
    zero[v] = 0;
    atomicAnd((unsigned long long *)&fbm[v >> 6], ~(1ull << (v & 63)));
  }
}
__global__ __launch_bounds__(kB) void k_bfs_prep_sparse(const uint32_t *touched, const unsigned long long *n,
                                                        uint64_t *frontier, uint64_t *visited,
                                                        const uint64_t *while_bm, int expand, DAdj adj,
                                                        unsigned long long *stats, uint64_t *fbm,
                                                        const uint64_t *hub_bm, uint32_t *act,
                                                        unsigned long long *act_n) {
  __shared__ uint64_t s_r[6][kB / 64];
  __shared__ uint32_t s_w[kB / 64];
  __shared__ uint32_t s_base;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t te = 0, td = 0, tn = 0, tl = 0, hd = 0, hn = 0;
  const uint64_t cnt = *n;
  for (uint64_t i0 = (uint64_t)blockIdx.x * kB; i0 < cnt; i0 += (uint64_t)gridDim.x * kB) {
    const uint64_t i = i0 + threadIdx.x;
    uint32_t v = 0;
    uint64_t m = 0;
    if (i < cnt) {
      v = touched[i];
      const uint64_t f = frontier[v];
      const uint64_t vis = visited[v];
      m = f & ~vis;
      if (m) visited[v] = vis | m;
      if (expand && while_bm && !bm_test(while_bm, v)) m = 0;
      if (m != f) frontier[v] = m;
      if (m && expand) {
        const uint64_t d = adj_degree(adj, v);
        te += (uint64_t)__popcll(m) * d;
        td += d;
        tn += 1;
        tl |= m;
        if (hub_bm && !bm_test(hub_bm, v)) {
          hd += d;
          hn += 1;
        }
        atomicOr((unsigned long long *)&fbm[v >> 6], 1ull << (v & 63));
      }
    }
    if (!expand) continue;
    const uint32_t a = (m != 0) ? 1u : 0u;
    uint32_t tot;
    const uint32_t off = block_excl_scan<kB>(a, s_w, &tot);
    if (threadIdx.x == 0 && tot) s_base = (uint32_t)atomicAdd(act_n, (unsigned long long)tot);
    __syncthreads();
    if (a) act[s_base + off] = v;
    __syncthreads();
  }
  if (!expand) return;
  (void)lane;
  te = wave_sum_u64(te);
  td = wave_sum_u64(td);
  tn = wave_sum_u64(tn);
  hd = wave_sum_u64(hd);
  hn = wave_sum_u64(hn);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) tl |= __shfl_xor(tl, off, 64);
  if ((threadIdx.x & 63) == 0) {
    s_r[0][wave] = te;
    s_r[1][wave] = td;
    s_r[2][wave] = tn;
    s_r[3][wave] = tl;
    s_r[4][wave] = hd;
    s_r[5][wave] = hn;
  }
  __syncthreads();
  if (threadIdx.x < 3 || (hub_bm && (threadIdx.x == 4 || threadIdx.x == 5))) {
    uint64_t x = 0;
    for (int w = 0; w < kB / 64; ++w) x += s_r[threadIdx.x][w];
    if (x) atomicAdd(&stats[threadIdx.x], (unsigned long long)x);
  } else if (threadIdx.x == 3) {
    uint64_t x = 0;
    for (int w = 0; w < kB / 64; ++w) x |= s_r[3][w];
    if (x) atomicOr(&stats[3], (unsigned long long)x);
  }
}
void launch_bfs_prep_sparse(const uint32_t *prev, const unsigned long long *prev_n, const uint32_t *touched,
                            const unsigned long long *touched_n, uint64_t bound, uint64_t *frontier, uint64_t *visited,
                            const uint64_t *while_bm, bool expand, const DAdj &adj, unsigned long long *stats,
                            uint64_t *fbm, const uint64_t *hub_bm, uint64_t *zero, uint32_t *act,
                            unsigned long long *act_n, int cus, hipStream_t s) {
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nblocks(bound, kB), (uint64_t)cus * 8));
  hipLaunchKernelGGL(k_bfs_sparse_clear, dim3(g), dim3(kB), 0, s, prev, prev_n, zero, fbm);
  KCHECK("k_bfs_sparse_clear");
  hipLaunchKernelGGL(k_bfs_prep_sparse, dim3(g), dim3(kB), 0, s, touched, touched_n, frontier, visited, while_bm,
                     (int)expand, adj, stats, fbm, hub_bm, act, act_n);
  KCHECK("k_bfs_prep_sparse");
}

// active vertices (non-zero frontier mask) → list, one atomic per block and iteration (push levels only)
__global__ __launch_bounds__(kB) void k_bfs_list(const uint64_t *frontier, uint32_t V, uint32_t *list,
                                                 unsigned long long *count) {
  __shared__ uint32_t s_w[kB / 64];
  __shared__ uint32_t s_base;
  // 4 block-strides per round: their words loaded together, one scan and one atomic for all (the list's
  // order inside a round is thread-major; the push does not depend on it)
  constexpr int kListU = 4;
  for (uint64_t b0 = (uint64_t)blockIdx.x * kB * kListU; b0 < V; b0 += (uint64_t)gridDim.x * kB * kListU) {
    uint64_t fu[kListU];
#pragma unroll
    for (int u = 0; u < kListU; ++u) {
      const uint64_t v = b0 + (uint64_t)u * kB + threadIdx.x;
      fu[u] = frontier[v < V ? v : V - 1];
    }
    uint32_t n = 0;
#pragma unroll
    for (int u = 0; u < kListU; ++u) n += (b0 + (uint64_t)u * kB + threadIdx.x < V && fu[u] != 0) ? 1u : 0u;
    uint32_t tot;
    uint32_t off = block_excl_scan<kB>(n, s_w, &tot);
    if (threadIdx.x == 0 && tot) s_base = (uint32_t)atomicAdd(count, (unsigned long long)tot);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kListU; ++u) {
      const uint64_t v = b0 + (uint64_t)u * kB + threadIdx.x;
      if (v < V && fu[u] != 0) list[s_base + off++] = (uint32_t)v;
    }
    __syncthreads();
  }
}
void launch_bfs_list(const uint64_t *frontier, uint32_t V, uint32_t *list, unsigned long long *count, int cus,
                     hipStream_t s) {
  if (!V) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(V, kB * 4), (uint64_t)cus * 8);
  hipLaunchKernelGGL(k_bfs_list, dim3(g), dim3(kB), 0, s, frontier, V, list, count);
  KCHECK("k_bfs_list");
}

// the frontier vertices that are not hubs, listed for a push beside a hubs-only pull: one thread per
// 64-vertex word of the frontier bitmap (fbm & ~hub_bm, 2 MB each at RMAT-24 instead of the V·8-B
// masks), one atomic per block (a block per 256 vertices made 65 K atomics on one counter: 0.78 ms)
__global__ __launch_bounds__(kB) void k_bfs_list_nonhub(const uint64_t *fbm, const uint64_t *hub_bm, uint32_t V,
                                                        uint32_t *list, unsigned long long *count) {
  __shared__ uint32_t s_w[kB / 64];
  __shared__ uint32_t s_base;
  const uint64_t nw = ((uint64_t)V + 63) / 64;
  for (uint64_t w0 = (uint64_t)blockIdx.x * kB; w0 < nw; w0 += (uint64_t)gridDim.x * kB) {
    const uint64_t w = w0 + threadIdx.x;
    uint64_t bits = 0;
    if (w < nw) {
      bits = fbm[w] & ~hub_bm[w];
      if (w == nw - 1 && (V & 63u)) bits &= (1ull << (V & 63u)) - 1ull;
    }
    uint32_t tot;
    uint32_t off = block_excl_scan<kB>((uint32_t)__popcll(bits), s_w, &tot);
    if (threadIdx.x == 0 && tot) s_base = (uint32_t)atomicAdd(count, (unsigned long long)tot);
    __syncthreads();
    for (; bits; bits &= bits - 1) list[s_base + off++] = (uint32_t)(w * 64 + __builtin_ctzll(bits));
    __syncthreads();
  }
}
void launch_bfs_list_nonhub(const uint64_t *fbm, const uint64_t *hub_bm, uint32_t V, uint32_t *list,
                            unsigned long long *count, int cus, hipStream_t s) {
  if (!V) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(((uint64_t)V + 63) / 64, kB), (uint64_t)cus * 8);
  hipLaunchKernelGGL(k_bfs_list_nonhub, dim3(g), dim3(kB), 0, s, fbm, hub_bm, V, list, count);
  KCHECK("k_bfs_list_nonhub");
}

// partitioned sparse levels: the rank's frontier as (vertex, mask low word, mask high word) triples
// (list: owned vertices relative to vlo, from k_bfs_list over fr + vlo), and their scatter on the peers
__global__ void k_bfs_frontier_pack(uint32_t *list, uint64_t n, uint32_t vlo, const uint64_t *fr, uint32_t *mlo,
                                    uint32_t *mhi) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t v = list[i] + vlo;
  const uint64_t m = fr[v];
  list[i] = v;
  mlo[i] = (uint32_t)m;
  mhi[i] = (uint32_t)(m >> 32);
}
__global__ void k_bfs_frontier_scatter(const uint32_t *v, const uint32_t *mlo, const uint32_t *mhi, uint64_t n,
                                       uint64_t *fr) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fr[v[i]] = ((uint64_t)mhi[i] << 32) | mlo[i];
}
void launch_bfs_frontier_pack(uint32_t *list, uint64_t n, uint32_t vlo, const uint64_t *fr, uint32_t *mlo, uint32_t *mhi,
                              hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_bfs_frontier_pack, dim3(nblocks(n, kB)), dim3(kB), 0, s, list, n, vlo, fr, mlo, mhi);
  KCHECK("k_bfs_frontier_pack");
}
void launch_bfs_frontier_scatter(const uint32_t *v, const uint32_t *mlo, const uint32_t *mhi, uint64_t n, uint64_t *fr,
                                 hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_bfs_frontier_scatter, dim3(nblocks(n, kB)), dim3(kB), 0, s, v, mlo, mhi, n, fr);
  KCHECK("k_bfs_frontier_scatter");
}

// degree of every listed vertex in one adjacency part (+ a trailing 0 for the exclusive scan)
__global__ void k_bfs_list_deg(const uint32_t *list, uint64_t nl, const uint64_t *rp, uint64_t *deg) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nl) deg[i] = rp[list[i] + 1] - rp[list[i]];
  else if (i == nl) deg[nl] = 0;
}
void launch_bfs_list_deg(const uint32_t *list, uint64_t nl, const uint64_t *rp, uint64_t *deg, hipStream_t s) {
  hipLaunchKernelGGL(k_bfs_list_deg, dim3(nblocks(nl + 1, kB)), dim3(kB), 0, s, list, nl, rp, deg);
  KCHECK("k_bfs_list_deg");
}

// Top-down: one thread per frontier edge (consecutive threads → consecutive col[] entries); the
// owning list entry is found by binary search in the degree prefix.
// top-down level: every out-edge of the listed frontier pushes its source's mask. A block takes
// kPushIT·kB consecutive edges; their sources' list offsets are staged in LDS (two global searches a
// block), so an edge finds its source with an LDS binary search (a global search per edge was ≈20
// dependent loads); a range over more than kPushStage sources searches the global offsets.
constexpr int kPushIT = 8, kPushStage = 2048;
__global__ __launch_bounds__(kB) void k_bfs_push(const uint32_t *list, const uint64_t *loffs, uint64_t nl,
                                                 uint64_t etot, const uint64_t *rp, const uint32_t *col,
                                                 const uint64_t *frontier, const uint64_t *visited, uint64_t *next,
                                                 uint32_t *touched, unsigned long long *touched_n) {
  __shared__ uint64_t s_off[kPushStage + 1];
  __shared__ uint64_t s_lo, s_hi;
  __shared__ uint32_t s_t[kB * kPushIT];  // this range's first touches (LDS appends, one global atomic a range)
  __shared__ uint32_t s_tn, s_tbase;
  auto search = [&](uint64_t lo, uint64_t hi, uint64_t e) {  // largest i in [lo, hi] with loffs[i] <= e
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) >> 1;
      if (loffs[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  constexpr uint64_t per = (uint64_t)kB * kPushIT;
  for (uint64_t e0 = (uint64_t)blockIdx.x * per; e0 < etot; e0 += (uint64_t)gridDim.x * per) {
    const uint64_t e1 = e0 + per < etot ? e0 + per : etot;
    if (threadIdx.x == 0) {
      const uint64_t lo = search(0, nl - 1, e0);
      s_lo = lo;
      s_hi = search(lo, nl - 1, e1 - 1);
      s_tn = 0;
    }
    __syncthreads();
    const uint64_t lo = s_lo, hi = s_hi, n = hi - lo + 1;
    const bool staged = n + 1 <= (uint64_t)kPushStage;
    if (staged)
      for (uint64_t i = threadIdx.x; i <= n; i += kB) s_off[i] = loffs[lo + i];
    __syncthreads();
    for (int k = 0; k < kPushIT; ++k) {
      const uint64_t e = e0 + (uint64_t)k * kB + threadIdx.x;
      if (e >= e1) break;
      uint64_t j, base;
      if (staged) {
        uint32_t a = 0, b = (uint32_t)(n - 1);
        while (a < b) {
          const uint32_t mid = (a + b + 1) >> 1;
          if (s_off[mid] <= e) a = mid;
          else b = mid - 1;
        }
        j = lo + a;
        base = s_off[a];
      } else {
        j = search(lo, hi, e);
        base = loffs[j];
      }
      const uint32_t v = list[j];
      const uint32_t w = col[rp[v] + (e - base)];
      const uint64_t m = frontier[v] & ~visited[w];
      bool first = false;
      if (m && (next[w] & m) != m) {
        const uint64_t old = atomicOr((unsigned long long *)&next[w], (unsigned long long)m);
        first = old == 0;  // the first bits w receives at this level
      }
      if (touched && first) s_t[atomicAdd(&s_tn, 1u)] = w;  // w joins the next level's touched list, once
    }
    __syncthreads();
    if (touched) {  // the range's touches: one counter atomic, then a coalesced copy
      if (threadIdx.x == 0 && s_tn) s_tbase = (uint32_t)atomicAdd(touched_n, (unsigned long long)s_tn);
      __syncthreads();
      for (uint32_t i = threadIdx.x; i < s_tn; i += kB) touched[s_tbase + i] = s_t[i];
    }
    __syncthreads();  // s_off, s_lo and s_t are restaged by the next range
  }
}
void launch_bfs_push(const uint32_t *list, const uint64_t *loffs, uint64_t nl, uint64_t etot, const uint64_t *rp,
                     const uint32_t *col, const uint64_t *frontier, const uint64_t *visited, uint64_t *next,
                     int cus, hipStream_t s, uint32_t *touched, unsigned long long *touched_n) {
  if (!etot || !nl) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(etot, (uint64_t)kB * kPushIT), (uint64_t)cus * 16);
  hipLaunchKernelGGL(k_bfs_push, dim3(g), dim3(kB), 0, s, list, loffs, nl, etot, rp, col, frontier, visited, next,
                     touched, touched_n);
  KCHECK("k_bfs_push");
}

__global__ void k_pull_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part);

// Bottom-up over one reversed adjacency part: merge-path tiles of kPullTile items over (vertices +
// in-edges), partitioned once per traversal from the part's row_ptr (k_pull_partition with offs = rp).
// Consecutive lanes take consecutive in-edges (coalesced col[] loads); the in-edges of a vertex that
// misses no live lane are skipped; each edge gathers its source's frontier mask. The col array is the
// hub-annotated copy (k_pull_annotate): in RMAT most in-edges come from a few hundred thousand
// high-degree sources, whose masks scattered over the V·8-B frontier cost one cache line each; their
// copies in the dense hub array (k_hub_gather) mostly hit L2 (C3: pull 7.5 → 5.6 ms).
// PROBE (levels whose frontier is sparse): a non-hub mask is gathered only if its bit in the frontier
// bitmap (V bits, L2-resident) is set. On the dense level the probe costs more than it saves, and a
// probe of the hubs' bitmap before a hub mask was slower on both (profiles/r02/c3probe, c3hbm).
// Masks are OR-reduced per vertex in LDS (ds_or_b64) and written with one atomicOr per vertex and tile
// (next[] is zeroed first; k_bfs_prep masks out visited lanes).
// Measured and rejected (profiles/r02/c3var, c3pipe, c3direct, c3flat): non-temporal loads of the
// streamed arrays (no change); the next tile's loads issued before this tile's gathers (no change,
// fewer waves); a flat kernel without tiles (a per-edge owner array, segmented DPP OR, global atomics:
// 4.0 against 3.3 ms per C3 step).
#ifndef OMX_PULL_B
#define OMX_PULL_B 256
#endif
#ifndef OMX_PULL_IPT
#define OMX_PULL_IPT 4
#endif
constexpr int kPullB = OMX_PULL_B, kPullIPT = OMX_PULL_IPT, kPullTile = kPullB * kPullIPT;
static_assert(kPullTile <= 65535, "s_seg holds tile-local row indices in 16 bits");

template <bool PROBE>
__global__ __launch_bounds__(kPullB) void k_bfs_pull(uint32_t V, const uint64_t *rp, const uint32_t *col,
                                                     const uint64_t *part, uint64_t E, uint64_t ntiles,
                                                     uint64_t lanes, const uint64_t *frontier,
                                                     const uint64_t *hub_fr, const uint64_t *fbm,
                                                     const uint64_t *visited, uint64_t *next) {
  constexpr int B = kPullB, IPT = kPullIPT, T = kPullTile, W = B / 64;
  // tile item jl is in-edge j0 + jl (merge-path tiles cover consecutive edges), so a row needs only
  // its lane mask and accumulator here: 18 B per row + 2 B per item → 8 workgroups per CU
  __shared__ uint64_t s_need[T + 1];
  __shared__ unsigned long long s_acc[T + 1];
  __shared__ uint16_t s_seg[T];
  __shared__ uint32_t s_wmax[W];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t d0 = t * (uint64_t)T;
    const uint64_t d1 = min(d0 + (uint64_t)T, (uint64_t)V + E);
    const uint64_t i0 = part[t], i1 = part[t + 1];
    const uint64_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t ne = (uint32_t)(j1 - j0);
    if (ne == 0) continue;  // uniform: only edge-less vertices in this tile
    const uint64_t rlast = min(i1, (uint64_t)V - 1);
    const uint32_t nr = (uint32_t)(rlast - i0 + 1);
    // the tile's col words are requested first, so their round trip overlaps the row setup's
    // (C3 pull 3.69 → 3.48 ms per step, profiles/r02/c3var)
    uint32_t xk[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const uint32_t jl = k * B + tid;
      xk[k] = jl < ne ? col[j0 + jl] : 0u;
    }
    for (uint32_t x = tid; x < ne; x += B) s_seg[x] = 0;
    __syncthreads();
    for (uint32_t lr = tid; lr < nr; lr += B) {
      const uint64_t r = i0 + lr;
      const uint64_t rs = rp[r], re = rp[r + 1];
      const uint64_t s = rs > j0 ? rs - j0 : 0;
      const uint64_t e = re < j1 ? (re > j0 ? re - j0 : 0) : ne;
      if (e > s && s < ne) s_seg[s] = (uint16_t)lr;
      s_need[lr] = (e > s) ? (lanes & ~visited[r]) : 0;
      s_acc[lr] = 0;
    }
    __syncthreads();
    {  // inclusive max-scan of s_seg → owning vertex of every tile edge
      uint32_t vals[IPT];
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t idx = tid * IPT + i;
        const uint32_t x = idx < ne ? s_seg[idx] : 0;
        m = m > x ? m : x;
        vals[i] = m;
      }
      uint32_t incl = m;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl = incl > y ? incl : y;
      }
      if (lane == 63) s_wmax[wave] = incl;
      uint32_t excl = __shfl_up(incl, 1, 64);
      if (lane == 0) excl = 0;
      __syncthreads();
      uint32_t wp = 0;
      for (uint32_t w = 0; w < wave; ++w) wp = wp > s_wmax[w] ? wp : s_wmax[w];
      const uint32_t pre = excl > wp ? excl : wp;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t idx = tid * IPT + i;
        if (idx < ne) s_seg[idx] = (uint16_t)(pre > vals[i] ? pre : vals[i]);
      }
    }
    __syncthreads();
    // all IPT gathers are issued before the first merge consumes one (IPT independent chains in
    // flight per lane); every non-empty mask is merged by its own LDS atomic (a segmented wave scan
    // first measured 1-2% slower)
    uint64_t fk[IPT];
    uint32_t lrk[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const uint32_t jl = k * B + tid;
      const uint32_t lr = jl < ne ? s_seg[jl] : 0u;
      uint64_t f = 0;
      if (jl < ne) {
        const uint64_t need = s_need[lr];
        const uint32_t x = xk[k];
        if (need) {
          if (x >> 31) f = hub_fr[x & 0x7FFFFFFFu] & need;
          else if (!PROBE || ((fbm[x >> 6] >> (x & 63)) & 1)) f = frontier[x] & need;
        }
      }
      fk[k] = f;
      lrk[k] = lr;
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k)
      if (fk[k]) atomicOr(&s_acc[lrk[k]], (unsigned long long)fk[k]);
    __syncthreads();
    for (uint32_t lr = tid; lr < nr; lr += B) {
      const unsigned long long a = s_acc[lr];
      if (a) atomicOr((unsigned long long *)&next[i0 + lr], a);
    }
    __syncthreads();
  }
}
uint64_t bfs_pull_tiles(uint32_t V, uint64_t E) { return ((uint64_t)V + E + kPullTile - 1) / kPullTile; }
void launch_bfs_pull_partition(const uint64_t *rp, uint32_t V, uint64_t E, uint64_t *part, hipStream_t s) {
  // merge path over A = row ends and B = edges with tiles of kPullTile (same split as k_mp_partition)
  const uint64_t ntiles = bfs_pull_tiles(V, E);
  hipLaunchKernelGGL(k_pull_partition, dim3(nblocks(ntiles + 1, kB)), dim3(kB), 0, s, rp, (uint64_t)V, E, ntiles, part);
  KCHECK("k_pull_partition");
}
void launch_bfs_pull(uint32_t V, const uint64_t *rp, const uint32_t *col, const uint64_t *part, uint64_t E,
                     uint64_t lanes, const uint64_t *frontier, const uint64_t *hub_fr, const uint64_t *fbm,
                     const uint64_t *visited, uint64_t *next, int cus, hipStream_t s) {
  const uint64_t ntiles = bfs_pull_tiles(V, E);
  if (!ntiles || !lanes) return;
  const auto kern = fbm ? k_bfs_pull<true> : k_bfs_pull<false>;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kPullB, 0) != hipSuccess || per < 1) per = 2;
  // resident workgroups per CU: 7 of the 8 that fit measured fastest at C3 (4.26 ms against 5.54 ms
  // at 8 and 4.60 at 5: with a full CU the random gathers thrash L2)
  per = std::min(per, 7);
  const unsigned g = (unsigned)std::min<uint64_t>(ntiles, (uint64_t)cus * per);
  hipLaunchKernelGGL(kern, dim3(g), dim3(kPullB), 0, s, V, rp, col, part, E, ntiles, lanes, frontier, hub_fr, fbm,
                     visited, next);
  KCHECK("k_bfs_pull");
}

// ---- wave-tiled bottom-up level (k_bfs_pull_w) ----------------------------------------------------
// The same level as k_bfs_pull over the same hub-annotated reversed CSR, tiled by waves over the in-edge
// space: every wave owns tiles of kPwTile consecutive in-edges (tile i → wave i mod W; no workgroup
// barriers). A tile's vertices (≤ kPwRows; a tile over more, or the partial last one, goes to
// k_bfs_pull_w_slow) sit in the wave's own LDS table — lane mask still needed and accumulator — and mark
// their first in-edge in a byte array spread by a max-scan, so an in-edge's vertex is one LDS byte. Lane l
// takes in-edges l + 64j: coalesced col[] words; each mask gathered (LDS copy of the first hubs' masks,
// the hub array, or the frontier after the bitmap probe) is merged into its vertex's accumulator by an
// LDS atomic, and every non-zero accumulator goes to next[] with one atomicOr.
// One 16-wave workgroup per CU, so the hub masks staged in LDS (the ≈10 K highest-degree sources, staged
// once per launch) serve every wave of the CU. Measured at C3's sparse level (profiles/r03/pullw): the
// level is bound by its L2 traffic (248 M TCP→TCC requests, 36 % missing, per launch; profiles/r03/
// pmc_c3), not by the tiles' latency — wave tiles alone 1.70-1.99 ms against k_bfs_pull's 1.72-1.74; the
// LDS hubs take 8 % of the requests' worth off: 1.59 ms.
#ifndef OMX_PW_WAVES
#define OMX_PW_WAVES 16
#endif
#ifndef OMX_PW_ROWS
#define OMX_PW_ROWS 256
#endif
constexpr int kPwTile = 1024, kPwJ = kPwTile / 64, kPwRows = OMX_PW_ROWS, kPwWaves = OMX_PW_WAVES;
// the first hub masks (highest degree) staged in LDS once per launch: one workgroup per CU, the rest of
// its LDS after the waves' tables
constexpr int kPwLdsHubs = (160 * 1024 - kPwWaves * (kPwTile + 16 * kPwRows) - 64) / 8;

struct PwTable {
  uint32_t mk[kPwTile / 4];  // kPwTile u8: table entry of every in-edge of the tile
  uint64_t need[kPwRows];
  unsigned long long acc[kPwRows];
};

// HUBS (a sparse level whose non-hub frontier is pushed instead, exec.hip varlen_msbfs): non-hub in-edges
// are skipped without any memory access
template <bool PROBE, bool HUBS>
__global__ __launch_bounds__(64 * kPwWaves) void k_bfs_pull_w(const uint64_t *rp, const uint32_t *col,
                                                             const uint32_t *__restrict__ tiles,
                                                             const uint64_t *__restrict__ rb, uint64_t n,
                                                             uint64_t lanes, const uint64_t *frontier,
                                                             const uint64_t *hub_fr, const uint64_t *fbm,
                                                             const uint64_t *visited, uint64_t *next, uint32_t nlds) {
  __shared__ PwTable s_tb[kPwWaves];
  __shared__ uint64_t s_hub[kPwLdsHubs];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  PwTable &tb = s_tb[wv];
  for (uint32_t h = threadIdx.x; h < nlds; h += blockDim.x) s_hub[h] = hub_fr[h];
  __syncthreads();
  const uint64_t W = (uint64_t)gridDim.x * kPwWaves;
  for (uint64_t i = (uint64_t)blockIdx.x * kPwWaves + wv; i < n; i += W) {
    const uint64_t t = tiles[i], t0 = t * kPwTile, r0 = rb[2 * t];
    const uint32_t nr = (uint32_t)(rb[2 * t + 1] - r0 + 1);  // ≤ kPwRows (a regular tile)
    uint32_t x[kPwJ];
#pragma unroll
    for (int j = 0; j < kPwJ; ++j) x[j] = col[t0 + 64 * j + lane];
    uint32_t *mk = tb.mk + lane * (kPwJ / 4);
#pragma unroll
    for (int q = 0; q < kPwJ / 4; ++q) mk[q] = 0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kPwRows / 64; ++q) {
      const uint32_t k = lane + 64 * q;
      if (k < nr) {
        const uint64_t rs = rp[r0 + k], re = rp[r0 + k + 1];
        if (re > rs && rs > t0 && rs < t0 + kPwTile) reinterpret_cast<uint8_t *>(tb.mk)[rs - t0] = (uint8_t)k;
        tb.need[k] = re > rs ? lanes & ~visited[r0 + k] : 0ull;
        tb.acc[k] = 0;
      }
    }
    __builtin_amdgcn_wave_barrier();
    {  // max-scan of the marks: lane l holds bytes 16l … 16l + 15
      uint32_t wd[kPwJ / 4];
      uint32_t m = 0;
#pragma unroll
      for (int q = 0; q < kPwJ / 4; ++q) {
        wd[q] = mk[q];
#pragma unroll
        for (int b = 0; b < 4; ++b) m = max(m, (wd[q] >> (8 * b)) & 0xFFu);
      }
      uint32_t incl = m;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl = max(incl, y);
      }
      uint32_t run = __shfl_up(incl, 1, 64);
      if (lane == 0) run = 0;
#pragma unroll
      for (int q = 0; q < kPwJ / 4; ++q) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          run = max(run, (wd[q] >> (8 * b)) & 0xFFu);
          o |= run << (8 * b);
        }
        mk[q] = o;
      }
    }
    __builtin_amdgcn_wave_barrier();
    const uint8_t *mb = reinterpret_cast<const uint8_t *>(tb.mk);
    uint64_t f[kPwJ];
    uint32_t kk[kPwJ];
#pragma unroll
    for (int j = 0; j < kPwJ; ++j) {  // every gather requested before the first merge
      const uint32_t k = mb[64 * j + lane];
      const uint64_t nd = tb.need[k];
      const uint32_t xv = x[j];
      uint64_t g = 0;
      if (nd) {
        const uint32_t hx = xv & 0x7FFFFFFFu;
        if ((xv >> 31) && hx < nlds) g = s_hub[hx] & nd;
        else if (xv >> 31) g = hub_fr[hx] & nd;
        else if (!HUBS && (!PROBE || ((fbm[xv >> 6] >> (xv & 63)) & 1))) g = frontier[xv] & nd;
      }
      f[j] = g;
      kk[j] = k;
    }
#pragma unroll
    for (int j = 0; j < kPwJ; ++j)
      if (f[j]) atomicOr(&tb.acc[kk[j]], (unsigned long long)f[j]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < kPwRows / 64; ++q) {
      const uint32_t k = lane + 64 * q;
      if (k < nr) {
        const unsigned long long a = tb.acc[k];
        if (a) atomicOr((unsigned long long *)&next[r0 + k], a);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the table is rebuilt for the next tile
  }
}

// the other tiles: one thread per in-edge, its vertex by a search of the row pointers
template <bool PROBE, bool HUBS>
__global__ __launch_bounds__(256) void k_bfs_pull_w_slow(const uint64_t *rp, const uint32_t *col, uint64_t E,
                                                        const uint32_t *tiles, const uint64_t *rb, uint64_t n,
                                                        uint64_t lanes, const uint64_t *frontier,
                                                        const uint64_t *hub_fr, const uint64_t *fbm,
                                                        const uint64_t *visited, uint64_t *next) {
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t t = tiles[i], t0 = t * kPwTile, t1 = min(t0 + (uint64_t)kPwTile, E);
    for (uint64_t e = t0 + threadIdx.x; e < t1; e += blockDim.x) {
      uint64_t lo = rb[2 * t], hi = rb[2 * t + 1];  // last row with rp[r] <= e
      while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (rp[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      const uint64_t nd = lanes & ~visited[lo];
      if (!nd) continue;
      const uint32_t xv = col[e];
      uint64_t g = 0;
      if (xv >> 31) g = hub_fr[xv & 0x7FFFFFFFu] & nd;
      else if (!HUBS && (!PROBE || ((fbm[xv >> 6] >> (xv & 63)) & 1))) g = frontier[xv] & nd;
      if (g) atomicOr((unsigned long long *)&next[lo], (unsigned long long)g);
    }
  }
}

// first / last vertex of every in-edge tile and whether the tile is regular (full, ≤ kPwRows vertices)
__global__ void k_pull_w_bounds(const uint64_t *rp, uint32_t V, uint64_t E, uint64_t ntiles, uint64_t *rb,
                                uint8_t *regular) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t e0 = t * kPwTile, e1 = min(e0 + (uint64_t)kPwTile, E) - 1;
  auto last_le = [&](uint64_t lo, uint64_t hi, uint64_t e) {
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) >> 1;
      if (rp[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  const uint64_t r0 = last_le(0, V - 1, e0), r1 = last_le(r0, V - 1, e1);
  rb[2 * t] = r0;
  rb[2 * t + 1] = r1;
  regular[t] = r1 - r0 < (uint64_t)kPwRows && e0 + kPwTile <= E;
}

uint64_t bfs_pull_w_tiles(uint64_t E) { return (E + kPwTile - 1) / kPwTile; }
void launch_pull_w_bounds(const uint64_t *rp, uint32_t V, uint64_t E, uint64_t *rb, uint8_t *regular, hipStream_t s) {
  const uint64_t nt = bfs_pull_w_tiles(E);
  if (!nt) return;
  hipLaunchKernelGGL(k_pull_w_bounds, dim3(nblocks(nt, kB)), dim3(kB), 0, s, rp, V, E, nt, rb, regular);
  KCHECK("k_pull_w_bounds");
}
void launch_bfs_pull_w(const uint64_t *rp, const uint32_t *col, uint64_t E, const uint32_t *tiles, uint64_t nreg,
                       const uint64_t *rb, uint64_t lanes, const uint64_t *frontier, const uint64_t *hub_fr,
                       uint32_t nhubs, const uint64_t *fbm, const uint64_t *visited, uint64_t *next, int cus,
                       hipStream_t s, bool hubs_only) {
  const uint64_t nt = bfs_pull_w_tiles(E);
  if (!nt || !lanes) return;
  constexpr int per = 1;  // workgroups per CU (16 waves each: one LDS copy of the hub masks a CU)
  const uint32_t nlds = std::min(nhubs, (uint32_t)kPwLdsHubs);
  const char *slow_env = std::getenv("OMX_PULLW_SLOW");  // 1: every tile through k_bfs_pull_w_slow (tests)
  const bool slow_all = slow_env && std::strcmp(slow_env, "0") != 0;
  if (slow_all) nreg = 0;
  if (nreg) {
    const dim3 g((unsigned)std::min<uint64_t>((nreg + kPwWaves - 1) / kPwWaves, (uint64_t)cus * per));
    if (hubs_only) hipLaunchKernelGGL((k_bfs_pull_w<false, true>), g, dim3(64 * kPwWaves), 0, s, rp, col, tiles, rb, nreg, lanes, frontier, hub_fr, fbm, visited, next, nlds);
    else if (fbm) hipLaunchKernelGGL((k_bfs_pull_w<true, false>), g, dim3(64 * kPwWaves), 0, s, rp, col, tiles, rb, nreg, lanes, frontier, hub_fr, fbm, visited, next, nlds);
    else hipLaunchKernelGGL((k_bfs_pull_w<false, false>), g, dim3(64 * kPwWaves), 0, s, rp, col, tiles, rb, nreg, lanes, frontier, hub_fr, fbm, visited, next, nlds);
    KCHECK("k_bfs_pull_w");
  }
  if (nt > nreg) {
    const dim3 g((unsigned)std::min<uint64_t>(nt - nreg, (uint64_t)cus * 8));
    if (hubs_only) hipLaunchKernelGGL((k_bfs_pull_w_slow<false, true>), g, dim3(256), 0, s, rp, col, E, tiles + nreg, rb, nt - nreg, lanes, frontier, hub_fr, fbm, visited, next);
    else if (fbm) hipLaunchKernelGGL((k_bfs_pull_w_slow<true, false>), g, dim3(256), 0, s, rp, col, E, tiles + nreg, rb, nt - nreg, lanes, frontier, hub_fr, fbm, visited, next);
    else hipLaunchKernelGGL((k_bfs_pull_w_slow<false, false>), g, dim3(256), 0, s, rp, col, E, tiles + nreg, rb, nt - nreg, lanes, frontier, hub_fr, fbm, visited, next);
    KCHECK("k_bfs_pull_w_slow");
  }
}

// Dense levels with an early exit: one thread per vertex walks its in-edges in the annotated col's
// hub-first order (the first alone, then four at a time) and stops as soon as the gathered masks cover the lanes the vertex
// still needs. Once the frontier holds a large share of V, most vertices are covered by their first
// in-edge (a hub every live lane has reached): C3's dense level reads 10 M of its 208 M in-edges
// (tools/c3_exit_stats.c). A vertex still uncovered after kExitScan in-edges is listed for
// k_bfs_pull_rest (one wave per vertex). next[] may hold an earlier part's lanes: they are not needed
// again and are kept. scanned accumulates the in-edges read (for the algorithmic bytes).
constexpr uint32_t kExitScan = 16;
__global__ __launch_bounds__(kB) void k_bfs_pull_exit(uint32_t vlo, uint32_t V, const uint64_t *rp, const uint32_t *col,
                                                      uint64_t lanes, const uint64_t *frontier,
                                                      const uint64_t *hub_fr, const uint64_t *visited,
                                                      uint64_t *next, uint32_t *rest, unsigned long long *counts) {
  const uint32_t lane = threadIdx.x & 63;
  uint64_t scanned = 0;
  // persistent grid-stride: the in-edge count is added once per wave (one atomic per vertex wave on a
  // single counter serialised the launch: 3.2 ms)
  for (uint64_t v0 = vlo + (uint64_t)blockIdx.x * kB; v0 < V; v0 += (uint64_t)gridDim.x * kB) {
    const uint64_t v = v0 + threadIdx.x;
    bool more = false;
    if (v < V) {
      const uint64_t old = next[v];
      const uint64_t need = lanes & ~visited[v] & ~old;
      const uint64_t s = rp[v], e = rp[v + 1];
      if (need && e > s) {
        // the first in-edge alone (the top hub covers most vertices), then four at a time
        const uint32_t x0 = col[s];
        uint64_t acc = (x0 >> 31) ? hub_fr[x0 & 0x7FFFFFFFu] : frontier[x0];
        uint64_t i = s + 1;
        const uint64_t stop = e - s > kExitScan ? s + kExitScan : e;
        while (i < stop && (acc & need) != need) {
          uint32_t x[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) x[k] = i + k < stop ? col[i + k] : 0u;
          uint64_t m[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            m[k] = 0;
            if (i + k < stop) m[k] = (x[k] >> 31) ? hub_fr[x[k] & 0x7FFFFFFFu] : frontier[x[k]];
          }
          acc |= m[0] | m[1] | m[2] | m[3];
          i = i + 4 < stop ? i + 4 : stop;
        }
        scanned += i - s;
        acc &= need;
        if (acc) next[v] = old | acc;
        more = acc != need && i < e;
      }
    }
    // the uncovered vertices with in-edges left: one slot per wave, then one per lane (rare)
    const uint64_t mm = __ballot(more);
    if (mm) {
      unsigned long long base = 0;
      const uint32_t first = (uint32_t)__builtin_ctzll(mm);
      if (lane == first) base = atomicAdd(&counts[1], (unsigned long long)__popcll(mm));
      base = __shfl(base, (int)first, 64);
      if (more) rest[base + lane_prefix(mm)] = (uint32_t)v;
    }
  }
  scanned = wave_sum_u64(scanned);
  if (lane == 0 && scanned) atomicAdd(&counts[0], (unsigned long long)scanned);
}

// the remaining in-edges of the listed vertices: one wave per vertex, 64 in-edges per step, OR-reduced
// across the wave, until the vertex's needed lanes are covered or its list ends
__global__ __launch_bounds__(kB) void k_bfs_pull_rest(const uint32_t *rest, const unsigned long long *counts,
                                                      const uint64_t *rp, const uint32_t *col, uint64_t lanes,
                                                      const uint64_t *frontier, const uint64_t *hub_fr,
                                                      const uint64_t *visited, uint64_t *next,
                                                      unsigned long long *scanned_out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t n = counts[1];
  const uint64_t nw = (uint64_t)gridDim.x * (kB / 64);
  uint64_t scanned = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * (kB / 64) + (threadIdx.x >> 6); w < n; w += nw) {
    const uint32_t v = rest[w];
    const uint64_t old = next[v];
    const uint64_t need = lanes & ~visited[v] & ~old;
    const uint64_t e = rp[v + 1];
    uint64_t acc = 0;
    for (uint64_t i = rp[v] + kExitScan; i < e; i += 64) {
      uint64_t m = 0;
      if (i + lane < e) {
        const uint32_t x = col[i + lane];
        m = (x >> 31) ? hub_fr[x & 0x7FFFFFFFu] : frontier[x];
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m |= __shfl_xor(m, off, 64);
      acc |= m;
      scanned += e - i < 64 ? e - i : 64;
      if ((acc & need) == need) break;
    }
    acc &= need;
    if (lane == 0 && acc) next[v] = old | acc;
  }
  if (lane == 0 && scanned) atomicAdd(scanned_out, (unsigned long long)scanned);
}

void launch_bfs_pull_exit(uint32_t V, const uint64_t *rp, const uint32_t *col, uint64_t lanes,
                          const uint64_t *frontier, const uint64_t *hub_fr, const uint64_t *visited, uint64_t *next,
                          uint32_t *rest, unsigned long long *counts, int cus, hipStream_t s, uint32_t vlo) {
  if (V <= vlo || !lanes) return;
  hipLaunchKernelGGL(k_bfs_pull_exit, dim3((unsigned)std::min<uint64_t>(nblocks(V - vlo, kB), (uint64_t)cus * 8)), dim3(kB),
                     0, s, vlo, V, rp, col, lanes, frontier, hub_fr, visited, next, rest, counts);
  KCHECK("k_bfs_pull_exit");
  hipLaunchKernelGGL(k_bfs_pull_rest, dim3((unsigned)cus * 8), dim3(kB), 0, s, rest, counts, rp, col, lanes, frontier,
                     hub_fr, visited, next, counts);
  KCHECK("k_bfs_pull_rest");
}

__global__ void k_pull_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  uint64_t d = t * (uint64_t)kPullTile;
  if (d > R + E) d = R + E;
  uint64_t lo = d > E ? d - E : 0, hi = d < R ? d : R;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (offs[mid + 1] <= d - 1 - mid) lo = mid + 1;
    else hi = mid;
  }
  part[t] = lo;
}

// Result emission from the visited masks: (row0 + lane, v) for every set lane of v with emit(v).
// last: the final level's frontier, not merged into visited by a prologue (a level that does not expand
// only merges): merged here, so the emission reads visited alone
__global__ __launch_bounds__(kB) void k_bfs_emit_count(uint64_t *visited, const uint64_t *emit_bm, uint32_t V,
                                                       uint32_t *blk, const uint64_t *last) {
  __shared__ uint32_t s_w[kB / 64];
  const uint64_t v = (uint64_t)blockIdx.x * kB + threadIdx.x;
  uint32_t c = 0;
  uint64_t vis = 0;
  if (v < V) {
    vis = visited[v];
    if (last) {
      const uint64_t x = last[v];
      if (x & ~vis) {
        vis |= x;
        visited[v] = vis;
      }
    }
  }
  if (v < V && (!emit_bm || bm_test(emit_bm, (uint32_t)v))) c = (uint32_t)__popcll(vis);
  uint32_t tot;
  block_excl_scan<kB>(c, s_w, &tot);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}
// The block's output range is written through LDS in windows of kEmitWin entries: every thread
// drops its (lane, vertex) pairs that fall in the window into LDS, then the block flushes the window
// with coalesced stores (the same order as a thread-by-thread write: vertex-major, lanes ascending).
// With carried columns (cc.n > 0) the pair's binding row is written as its columns' values
// (cc.in[c][row0 + lane], staged once per block in LDS) instead of as a row index, so no row gather
// follows the emission.
constexpr uint32_t kEmitWin = 4096;
__global__ __launch_bounds__(kB) void k_bfs_emit_write(const uint64_t *visited, const uint64_t *emit_bm, uint32_t V,
                                                       const uint64_t *blk_offs, uint32_t row0, uint32_t *out_row,
                                                       uint32_t *out_v, BfsCarry cc) {
  // a staged pair is its lane and its thread (the vertex is the block's first + thread): 2 B of LDS,
  // so more blocks stay resident than with 4-B lane and vertex words
  __shared__ uint32_t s_w[kB / 64];
  __shared__ uint8_t s_row[kEmitWin];
  __shared__ uint8_t s_t[kEmitWin];
  __shared__ uint32_t s_cv[BfsCarry::kMax][64];
  static_assert(kB <= 256, "s_t holds a thread index in 8 bits");
  const uint64_t v = (uint64_t)blockIdx.x * kB + threadIdx.x;
  for (int c = 0; c < cc.n; ++c)
    if (threadIdx.x < cc.nl) s_cv[c][threadIdx.x] = cc.in[c][row0 + threadIdx.x];
  uint64_t m = 0;
  if (v < V && (!emit_bm || bm_test(emit_bm, (uint32_t)v))) m = visited[v];
  uint32_t tot;
  const uint32_t c = (uint32_t)__popcll(m);
  const uint32_t off = block_excl_scan<kB>(c, s_w, &tot);  // (its barrier also publishes s_cv)
  const uint64_t base = blk_offs[blockIdx.x];
  for (uint32_t w0 = 0; w0 < tot; w0 += kEmitWin) {
    const uint32_t w1 = min(w0 + kEmitWin, tot);
    if (off < w1 && off + c > w0) {
      uint64_t mm = m;
      uint32_t o = off;
      for (; o < w0; ++o) mm &= mm - 1;  // entries that belong to an earlier window
      for (; mm && o < w1; ++o) {
        s_row[o - w0] = (uint8_t)__builtin_ctzll(mm);
        s_t[o - w0] = (uint8_t)threadIdx.x;
        mm &= mm - 1;
      }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < w1 - w0; i += kB) {
      const uint32_t l = s_row[i];
      if (cc.n == 0) out_row[base + w0 + i] = row0 + l;
      for (int k = 0; k < cc.n; ++k) cc.out[k][base + w0 + i] = s_cv[k][l];
      out_v[base + w0 + i] = (uint32_t)((uint64_t)blockIdx.x * kB + s_t[i]);
    }
    __syncthreads();
  }
}
void launch_bfs_emit_count(uint64_t *visited, const uint64_t *emit_bm, uint32_t V, uint32_t *blk, hipStream_t s,
                           const uint64_t *last) {
  hipLaunchKernelGGL(k_bfs_emit_count, dim3(nblocks(V, kB)), dim3(kB), 0, s, visited, emit_bm, V, blk, last);
  KCHECK("k_bfs_emit_count");
}
void launch_bfs_emit_write(const uint64_t *visited, const uint64_t *emit_bm, uint32_t V, const uint64_t *blk_offs,
                           uint32_t row0, uint32_t *out_row, uint32_t *out_v, const BfsCarry &cc, hipStream_t s) {
  hipLaunchKernelGGL(k_bfs_emit_write, dim3(nblocks(V, kB)), dim3(kB), 0, s, visited, emit_bm, V, blk_offs, row0,
                     out_row, out_v, cc);
  KCHECK("k_bfs_emit_write");
}
unsigned bfs_blocks(uint32_t V) { return nblocks(V, kB); }

// T_BOUND: row r (lane r - row0) keeps its binding iff its bound target was reached and passes emit
__global__ void k_bfs_bound(const uint32_t *dst, uint64_t row0, int nl, const uint64_t *visited,
                            const uint64_t *emit_bm, uint8_t *flags, const uint64_t *last) {
  const int i = threadIdx.x;
  if (i >= nl) return;
  const uint32_t t = dst[row0 + i];
  const uint64_t vis = visited[t] | (last ? last[t] : 0ull);
  flags[row0 + i] = ((vis >> i) & 1ull) && (!emit_bm || bm_test(emit_bm, t));
}
void launch_bfs_bound(const uint32_t *dst, uint64_t row0, int nl, const uint64_t *visited, const uint64_t *emit_bm,
                      uint8_t *flags, hipStream_t s, const uint64_t *last) {
  hipLaunchKernelGGL(k_bfs_bound, dim3(1), dim3(64), 0, s, dst, row0, nl, visited, emit_bm, flags, last);
  KCHECK("k_bfs_bound");
}

// ---- hub annotation (once per CSR) -------------------------------------------------------------------
constexpr int kHist = 4096;  // degree histogram buckets (degrees ≥ 4095 share the last one)

__global__ __launch_bounds__(kB) void k_deg_hist(const uint64_t *rp, uint32_t V, uint32_t *hist) {
  __shared__ uint32_t s_h[kHist];
  for (int i = threadIdx.x; i < kHist; i += kB) s_h[i] = 0;
  __syncthreads();
  for (uint64_t v = (uint64_t)blockIdx.x * kB + threadIdx.x; v < V; v += (uint64_t)gridDim.x * kB) {
    const uint64_t d = rp[v + 1] - rp[v];
    atomicAdd(&s_h[d < kHist - 1 ? d : kHist - 1], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHist; i += kB)
    if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// hub_idx[v] = its hub index when deg(v) ≥ t (order of discovery; any order is a valid labelling)
__global__ __launch_bounds__(kB) void k_hub_mark(const uint64_t *rp, uint32_t V, uint64_t t, uint32_t *hub_idx,
                                                 uint32_t *hubs, unsigned long long *count) {
  __shared__ uint32_t s_w[kB / 64];
  __shared__ uint32_t s_base;
  for (uint64_t v0 = (uint64_t)blockIdx.x * kB; v0 < V; v0 += (uint64_t)gridDim.x * kB) {
    const uint64_t v = v0 + threadIdx.x;
    const bool hub = v < V && rp[v + 1] - rp[v] >= t;
    uint32_t tot;
    const uint32_t off = block_excl_scan<kB>(hub ? 1u : 0u, s_w, &tot);
    if (threadIdx.x == 0 && tot) s_base = (uint32_t)atomicAdd(count, (unsigned long long)tot);
    __syncthreads();
    if (v < V) hub_idx[v] = hub ? s_base + off : 0xFFFFFFFFu;
    if (hub) hubs[s_base + off] = (uint32_t)v;
    __syncthreads();
  }
}

// hub degrees (sort keys) and, after the sort, every hub's index = its rank by degree (densest first)
__global__ void k_hub_deg(const uint32_t *hubs, uint32_t n, const uint64_t *rp, uint32_t *deg) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) deg[i] = (uint32_t)min<uint64_t>(rp[hubs[i] + 1] - rp[hubs[i]], 0xFFFFFFFFull);
}
__global__ void k_hub_rank(const uint32_t *hubs, uint32_t n, uint32_t *hub_idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hub_idx[hubs[i]] = i;
}

// Rows of the annotated col re-ordered hub-first by rank (the pull ORs a row's masks in any order):
// the lanes of a wave then read the hottest hub masks, which share cache lines, before the rest.
// sort key per entry = row << 32 | (hub ? rank : 2^31 + vertex)
__global__ void k_row_heads(const uint64_t *rp, uint32_t V, uint32_t *head) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < V && rp[v + 1] > rp[v]) head[rp[v]] = (uint32_t)v;
}
__global__ void k_pull_keys(const uint32_t *row, const uint32_t *ann, uint64_t E, uint64_t *keys) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t x = ann[e];
    const uint32_t k = (x >> 31) ? (x & 0x7FFFFFFFu) : (0x80000000u | x);
    keys[e] = ((uint64_t)row[e] << 32) | k;
  }
}
__global__ void k_pull_unkey(const uint64_t *keys, uint64_t E, uint32_t *ann) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = (uint32_t)keys[e];
    ann[e] = (k >> 31) ? (k & 0x7FFFFFFFu) : (0x80000000u | k);
  }
}
struct MaxU32 {
  __device__ __forceinline__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};

__global__ void k_pull_annotate(const uint32_t *col, uint64_t E, const uint32_t *hub_idx, uint32_t *out) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t c = col[e];
    const uint32_t h = hub_idx[c];
    out[e] = h != 0xFFFFFFFFu ? (0x80000000u | h) : c;
  }
}

uint32_t build_pull_col(const uint64_t *rp_self, const uint64_t *rp_other, const uint32_t *col, uint32_t V, uint64_t E,
                        uint32_t max_hubs, uint32_t *hub_idx, uint32_t *hist, unsigned long long *count, uint32_t *hubs,
                        uint32_t *out, int cus, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(hist, 0, kHist * sizeof(uint32_t), s));
  HIP_CHECK(hipMemsetAsync(count, 0, sizeof(unsigned long long), s));
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(V, kB), (uint64_t)cus * 4);
  hipLaunchKernelGGL(k_deg_hist, dim3(g), dim3(kB), 0, s, rp_other, V, hist);
  KCHECK("k_deg_hist");
  std::vector<uint32_t> h(kHist);
  HIP_CHECK(hipMemcpyAsync(h.data(), hist, kHist * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  // the lowest degree threshold t ≥ 2 whose vertices (deg ≥ t) number at most max_hubs
  uint64_t cum = 0, t = kHist;
  for (int d = kHist - 1; d >= 2; --d) {
    if (cum + h[d] > max_hubs) break;
    cum += h[d];
    t = d;
  }
  if (cum == 0) t = ~0ull;  // no hubs: the copy is the plain col
  hipLaunchKernelGGL(k_hub_mark, dim3(g), dim3(kB), 0, s, rp_other, V, (uint64_t)t, hub_idx, hubs, count);
  KCHECK("k_hub_mark");
  // hub index = rank by degree (descending): the masks gathered most often share the first lines of
  // the packed array
  if (cum > 1) {
    const uint32_t n = (uint32_t)cum;
    uint32_t *deg = nullptr, *deg2 = nullptr, *h2 = nullptr;
    void *tmp = nullptr;
    size_t tb = 0;
    HIP_CHECK(hipMalloc((void **)&deg, (size_t)n * 4));
    HIP_CHECK(hipMalloc((void **)&deg2, (size_t)n * 4));
    HIP_CHECK(hipMalloc((void **)&h2, (size_t)n * 4));
    hipLaunchKernelGGL(k_hub_deg, dim3(nblocks(n, kB)), dim3(kB), 0, s, hubs, n, rp_other, deg);
    KCHECK("k_hub_deg");
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tb, deg, deg2, hubs, h2, (int)n, 0, 32, s));
    HIP_CHECK(hipMalloc(&tmp, std::max<size_t>(tb, 16)));
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairsDescending(tmp, tb, deg, deg2, hubs, h2, (int)n, 0, 32, s));
    HIP_CHECK(hipMemcpyAsync(hubs, h2, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_hub_rank, dim3(nblocks(n, kB)), dim3(kB), 0, s, hubs, n, hub_idx);
    KCHECK("k_hub_rank");
    HIP_CHECK(hipStreamSynchronize(s));
    (void)hipFree(deg);
    (void)hipFree(deg2);
    (void)hipFree(h2);
    (void)hipFree(tmp);
  }
  if (E) {
    const unsigned ge = (unsigned)std::min<uint64_t>(nblocks(E, kB), (uint64_t)cus * 16);
    hipLaunchKernelGGL(k_pull_annotate, dim3(ge), dim3(kB), 0, s, col, E, hub_idx, out);
    KCHECK("k_pull_annotate");
    if (cum > 0 && E < (1ull << 40)) {
      uint32_t *row = nullptr;
      uint64_t *k0 = nullptr, *k1 = nullptr;
      void *tmp = nullptr;
      size_t tb = 0;
      int vbits = 1;
      while (vbits < 32 && (1ull << vbits) < V) ++vbits;
      HIP_CHECK(hipMalloc((void **)&row, E * 4));
      HIP_CHECK(hipMalloc((void **)&k0, E * 8));
      HIP_CHECK(hipMalloc((void **)&k1, E * 8));
      HIP_CHECK(hipMemsetAsync(row, 0, E * 4, s));
      hipLaunchKernelGGL(k_row_heads, dim3(nblocks(V, kB)), dim3(kB), 0, s, rp_self, V, row);
      KCHECK("k_row_heads");
      HIP_CHECK(hipcub::DeviceScan::InclusiveScan(nullptr, tb, row, row, MaxU32(), (int64_t)E, s));
      HIP_CHECK(hipMalloc(&tmp, std::max<size_t>(tb, 16)));
      HIP_CHECK(hipcub::DeviceScan::InclusiveScan(tmp, tb, row, row, MaxU32(), (int64_t)E, s));
      hipLaunchKernelGGL(k_pull_keys, dim3(ge), dim3(kB), 0, s, row, out, E, k0);
      KCHECK("k_pull_keys");
      HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(tmp);
      tmp = nullptr;
      tb = 0;
      HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, k0, k1, (int64_t)E, 0, 32 + vbits, s));
      HIP_CHECK(hipMalloc(&tmp, std::max<size_t>(tb, 16)));
      HIP_CHECK(hipcub::DeviceRadixSort::SortKeys(tmp, tb, k0, k1, (int64_t)E, 0, 32 + vbits, s));
      hipLaunchKernelGGL(k_pull_unkey, dim3(ge), dim3(kB), 0, s, k1, E, out);
      KCHECK("k_pull_unkey");
      HIP_CHECK(hipStreamSynchronize(s));
      (void)hipFree(tmp);
      (void)hipFree(row);
      (void)hipFree(k0);
      (void)hipFree(k1);
    }
  }
  return (uint32_t)cum;
}

// per pull level: the hubs' frontier masks, packed
__global__ void k_hub_gather(const uint32_t *hubs, uint32_t n, const uint64_t *frontier, uint64_t *hub_fr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) hub_fr[i] = frontier[hubs[i]];
}
void launch_hub_gather(const uint32_t *hubs, uint32_t n, const uint64_t *frontier, uint64_t *hub_fr, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_hub_gather, dim3(nblocks(n, kB)), dim3(kB), 0, s, hubs, n, frontier, hub_fr);
  KCHECK("k_hub_gather");
}

}  // namespace omx
