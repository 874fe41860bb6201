// factor.hip — the filtered neighbour lists of a factorized hop (exec.hip Executor::expand_factorized).
//
// A filtered hop whose rows repeat their source vertices is expanded once per distinct source u: L(u) =
// the neighbours of u passing the target's WHERE bitmap (OMatchPathItem.executeTraversal with the
// filter, P/OMatchPathItem.java:63-78), grouped by source so that the rows are written over the lists.
// Here the distinct sources' adjacency entries are one flat range [0, EU) in source order (doff = the
// exclusive scan of their degrees), cut into tiles of kFlTile entries:
//   k_flist_tile   one workgroup per tile: each entry's source row from the tile's row range staged in
//                  LDS, the col word (coalesced: a wave reads 64 consecutive entries per step, so a hub
//                  row's sorted neighbours probe few bitmap lines), the bitmap probe (L2-resident
//                  V-bit bitmap), the survivors compacted in entry order into the tile's slot of a
//                  scratch buffer, and per-source survivor counts (LDS, then one global atomic per
//                  source and tile);
//   k_flist_gather the tiles' survivors moved to their final place (a scan of the tile counts).
// The lists come out grouped by source in source order, so their offsets are the scan of the counts —
// no key histogram / scatter, no arenas, no degree binning. Reads: 4 B per entry (+ the probe); writes:
// 4 B per survivor, twice.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "devutil.h"

namespace omx {

namespace {

constexpr int kFlB = 256, kFlSteps = 16, kFlTile = kFlB * kFlSteps, kFlRows = 1024;  // 20.5 KiB of LDS

// last r in [lo, hi] with off[r] <= e (off ascending, off[lo] <= e)
template <class T>
__device__ __forceinline__ uint64_t last_le_range(const T *off, uint64_t lo, uint64_t hi, uint64_t e) {
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// the first and last source row of every tile (one thread per tile: the searches run in parallel rather
// than as a dependent chain at the head of each tile)
__global__ void k_flist_bounds(const uint64_t *doff, uint64_t U, uint64_t EU, uint64_t ntiles, uint64_t *rb) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t t0 = t * kFlTile, t1 = min(t0 + (uint64_t)kFlTile, EU) - 1;
  rb[2 * t] = last_le_range(doff, 0, U - 1, t0);
  rb[2 * t + 1] = last_le_range(doff, rb[2 * t], U - 1, t1);
}

// degree and first col position of every distinct source (the tiles read both with coalesced loads)
__global__ void k_flist_prep(const uint32_t *ub, uint64_t U, const uint64_t *rp, uint64_t *deg, uint64_t *astart) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u > U) return;
  if (u == U) {
    deg[U] = 0;
    return;
  }
  const uint32_t v = ub[u];
  const uint64_t s = rp[v];
  deg[u] = rp[v + 1] - s;
  astart[u] = s;
}

// rowv (optional): the rows' vertices; with it every survivor's row vertex is written to tmp_row too.
// A tile's rows are staged in LDS (col position of entry e = s_base[row] + e) and every entry finds its
// row through s_seg: the rows mark their first entry in the tile, an inclusive max-scan spreads the mark
// (the merge-path trick of kernels.hip k_expand; no per-entry search). A tile over more than kFlRows rows
// (a run of short rows) searches the global offsets instead.
__global__ __launch_bounds__(kFlB) void k_flist_tile(const uint64_t *doff, const uint64_t *astart, uint64_t EU,
                                                     const uint64_t *rb, const uint32_t *col, const uint64_t *filter,
                                                     uint32_t *tmp, uint32_t *tile_cnt, unsigned long long *cnt,
                                                     const uint32_t *rowv, uint32_t *tmp_row) {
  constexpr int W = kFlB / 64, IPT = kFlSteps;
  __shared__ uint64_t s_base[kFlRows];  // col position of a row's entry e, minus e
  __shared__ uint32_t s_cnt[kFlRows];   // survivors per row in this tile
  __shared__ uint16_t s_seg[kFlTile];   // tile-local row of every entry
  __shared__ uint32_t s_w[kFlSteps][W];
  __shared__ uint32_t s_wmax[W];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t ntiles = (EU + kFlTile - 1) / kFlTile;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t t0 = tile * kFlTile, t1 = min(t0 + (uint64_t)kFlTile, EU) - 1;
    const uint32_t ne = (uint32_t)(t1 - t0 + 1);
    const uint64_t r0 = rb[2 * tile], nr = rb[2 * tile + 1] - r0 + 1;
    const bool staged = nr <= kFlRows;
    if (staged) {
      for (uint32_t x = tid; x < ne; x += kFlB) s_seg[x] = 0;
      __syncthreads();
      for (uint32_t lr = tid; lr < nr; lr += kFlB) {
        const uint64_t rs = doff[r0 + lr], re = doff[r0 + lr + 1];
        const uint64_t st = rs > t0 ? rs - t0 : 0;
        if (re > rs && st < ne) s_seg[st] = (uint16_t)lr;
        s_base[lr] = astart[r0 + lr] - rs;
        s_cnt[lr] = 0;
      }
      __syncthreads();
      uint32_t vals[IPT];
      uint32_t mx = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t idx = tid * IPT + i;
        const uint32_t v = idx < ne ? s_seg[idx] : 0;
        mx = mx > v ? mx : v;
        vals[i] = mx;
      }
      uint32_t incl = mx;
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
    // every step's col word and probe requested before any is consumed
    uint32_t x[kFlSteps];
    uint64_t r[kFlSteps];
#pragma unroll
    for (int k = 0; k < kFlSteps; ++k) {
      const uint32_t jl = (uint32_t)k * kFlB + tid;
      x[k] = 0;
      r[k] = ~0ull;
      if (jl < ne) {
        const uint64_t e = t0 + jl;
        uint64_t pos;
        if (staged) {
          r[k] = s_seg[jl];
          pos = s_base[r[k]] + e;
        } else {
          r[k] = last_le_range(doff, r0, r0 + nr - 1, e);
          pos = astart[r[k]] + (e - doff[r[k]]);
        }
        x[k] = col[pos];
      }
    }
    uint32_t keep = 0;
#pragma unroll
    for (int k = 0; k < kFlSteps; ++k)
      if (r[k] != ~0ull && bm_test(filter, x[k])) keep |= 1u << k;
    uint64_t m[kFlSteps];
#pragma unroll
    for (int k = 0; k < kFlSteps; ++k) {
      m[k] = __ballot((keep >> k) & 1u);
      if (lane == 0) s_w[k][wave] = (uint32_t)__popcll(m[k]);
    }
    __syncthreads();
    // survivors in entry order: step k's survivors follow all earlier steps' (wave totals in LDS)
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int k = 0; k < kFlSteps; ++k) {
      uint32_t kb = 0, kt = 0;
#pragma unroll
      for (int w = 0; w < kFlB / 64; ++w) {
        const uint32_t c = s_w[k][w];
        kb += (uint32_t)w < wave ? c : 0;
        kt += c;
      }
      if ((keep >> k) & 1u) {
        const uint64_t o = t0 + total + kb + lane_prefix(m[k]);
        tmp[o] = x[k];
        if (rowv) {
          tmp_row[o] = rowv[staged ? r0 + r[k] : r[k]];
        } else if (staged) {
          atomicAdd(&s_cnt[r[k]], 1u);
        } else {
          atomicAdd(&cnt[r[k]], 1ull);
        }
      }
      total += kt;
    }
    (void)before;
    if (threadIdx.x == 0) tile_cnt[tile] = total;
    __syncthreads();  // s_cnt complete
    if (staged && !rowv)
      for (uint32_t i = threadIdx.x; i < nr; i += kFlB)
        if (s_cnt[i]) atomicAdd(&cnt[r0 + i], (unsigned long long)s_cnt[i]);
    __syncthreads();  // the LDS tables are restaged by the next tile
  }
}

__global__ __launch_bounds__(kFlB) void k_flist_gather(const uint32_t *tmp, const uint32_t *tile_cnt,
                                                       const uint64_t *tile_off, uint64_t ntiles, uint32_t *out,
                                                       const uint32_t *tmp_row, uint32_t *out_row) {
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t n = tile_cnt[tile];
    const uint64_t src = tile * kFlTile, dst = tile_off[tile];
    for (uint32_t i = threadIdx.x; i < n; i += kFlB) out[dst + i] = tmp[src + i];
    if (tmp_row)
      for (uint32_t i = threadIdx.x; i < n; i += kFlB) out_row[dst + i] = tmp_row[src + i];
  }
}

// reverse lists: offsets of every distinct source's group among the keys sorted ascending
__global__ void k_flist_group_offsets(const uint32_t *keys, uint64_t n, const uint32_t *ub, uint64_t U, uint64_t *loff) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u > U) return;
  if (u == U) {
    loff[U] = n;
    return;
  }
  const uint32_t b = ub[u];
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (keys[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  loff[u] = lo;
}

}  // namespace

uint64_t flist_tiles(uint64_t EU) { return (EU + kFlTile - 1) / kFlTile; }

void launch_flist_prep(const uint32_t *ub, uint64_t U, const uint64_t *rp, uint64_t *deg, uint64_t *astart, hipStream_t s) {
  hipLaunchKernelGGL(k_flist_prep, dim3(nblocks(U + 1, 256)), dim3(256), 0, s, ub, U, rp, deg, astart);
  KCHECK("k_flist_prep");
}

void launch_flist_tile(uint64_t U, const uint64_t *doff, const uint64_t *astart, uint64_t EU, const uint32_t *col,
                       const uint64_t *filter, uint32_t *tmp, uint32_t *tile_cnt, unsigned long long *cnt, uint64_t *rb,
                       int cus, hipStream_t s, const uint32_t *rowv, uint32_t *tmp_row) {
  if (!EU || !U) return;
  const uint64_t nt = flist_tiles(EU);
  hipLaunchKernelGGL(k_flist_bounds, dim3(nblocks(nt, 256)), dim3(256), 0, s, doff, U, EU, nt, rb);
  KCHECK("k_flist_bounds");
  hipLaunchKernelGGL(k_flist_tile, dim3((unsigned)std::min<uint64_t>(nt, (uint64_t)cus * 8)), dim3(kFlB), 0, s, doff,
                     astart, EU, rb, col, filter, tmp, tile_cnt, cnt, rowv, tmp_row);
  KCHECK("k_flist_tile");
}

void launch_flist_gather(const uint32_t *tmp, const uint32_t *tile_cnt, const uint64_t *tile_off, uint64_t ntiles,
                         uint32_t *out, int cus, hipStream_t s, const uint32_t *tmp_row, uint32_t *out_row) {
  if (!ntiles) return;
  hipLaunchKernelGGL(k_flist_gather, dim3((unsigned)std::min<uint64_t>(ntiles, (uint64_t)cus * 8)), dim3(kFlB), 0, s, tmp,
                     tile_cnt, tile_off, ntiles, out, tmp_row, out_row);
  KCHECK("k_flist_gather");
}

void launch_flist_group_offsets(const uint32_t *keys, uint64_t n, const uint32_t *ub, uint64_t U, uint64_t *loff,
                                hipStream_t s) {
  hipLaunchKernelGGL(k_flist_group_offsets, dim3(nblocks(U + 1, 256)), dim3(256), 0, s, keys, n, ub, U, loff);
  KCHECK("k_flist_group_offsets");
}

}  // namespace omx
