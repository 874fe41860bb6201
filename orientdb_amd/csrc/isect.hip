// isect.hip — the fused closing check of a cyclic pattern as a sorted-list intersection (BASELINE
// north_star (4)).
//
// A pattern edge x → t followed by a closing check y → t (t bound by the expansion) keeps the rows
// (…, t) with t ∈ N_x(x) ∩ N_y(y): the reference iterates N_x(x) and, for each t, scans N_y(y) until it
// finds t (existence with break, P/OMatchStatement.java:468-477). Both lists are sorted in the snapshot,
// so the device intersects them:
//   - rows whose two lists have comparable lengths (the larger ≤ ratio × the smaller, m + n ≤ 1024) go
//     through k_isect_merge: a workgroup stages the two lists of every row of a tile in LDS with
//     independent coalesced loads, then walks the merged order of each row's pair with a merge path —
//     thread i takes positions [8i, 8i + 8) of the tile's concatenated merged sequences, finds its
//     split of the row's (A, B) pair by a binary search on the diagonal, and consumes one element a
//     step; an A element (the expansion's neighbour) matches when the last B element consumed equals
//     it (ties put B first, so an equal B element is always consumed before it). Parallel edges keep
//     their multiplicity on the A side (one row per edge x → t) and count once on the B side
//     (existence), as the reference's loop does;
//   - skewed pairs keep the binary-search probe of the shorter list into the longer one (the fused
//     expansion kernels, Executor::expand_check_isect).
//
// Tiles: merge row r weighs m + n + 8; tile t holds the rows whose weight offset lies in
// [t·1024, (t+1)·1024), so a tile stages < 2048 entries over ≤ 205 rows. The rows of tile t write their
// matches at boff[first row of t] (boff: the scan of the rows' output bounds, min(m, n) when N_x has no
// parallel edges, else m) and report the count: a block-segmented table, compacted by the caller.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "devutil.h"
#include "graph.h"
#include "kernels.h"

namespace omx {

namespace {

constexpr int kIsBlock = 256;
constexpr int kIsIPT = 8;
constexpr int kIsTile = kIsBlock * kIsIPT;

// one row's class (Executor::expand_check_isect): 0 nothing to intersect, 1 merge, 2 iterate N_x and
// probe N_y, 3 iterate N_y and probe N_x (swap); sums: [0] Σ m, [1] Σ m·n, [2 + c] rows of class c
__global__ __launch_bounds__(256) void k_isect_class(const uint32_t *xs, const uint32_t *ys, uint64_t R, DAdjPart ax,
                                                     DAdjPart ay, IsectPolicy pol, uint8_t *cls, uint32_t *w,
                                                     uint32_t *bnd, unsigned long long *sums) {
  __shared__ unsigned long long s_sum[6];
  if (threadIdx.x < 6) s_sum[threadIdx.x] = 0;
  __syncthreads();
  uint64_t sm = 0, smn = 0;
  uint32_t cc[4] = {0, 0, 0, 0};
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t x = xs[r], y = ys[r];
    const uint64_t m = ax.rp[x + 1] - ax.rp[x], n = ay.rp[y + 1] - ay.rp[y];
    const uint64_t lo = m < n ? m : n, hi = m < n ? n : m;
    uint8_t c;
    if (m == 0 || n == 0) c = 0;
    else if (pol.merge && m + n <= kIsRowCap && (pol.force || (double)hi <= pol.ratio * (double)lo)) c = 1;
    else if (pol.swap && m > n) c = 3;
    else c = 2;
    cls[r] = c;
    w[r] = c == 1 ? (uint32_t)(m + n) + kIsRowPad : 0u;
    bnd[r] = c == 1 ? (uint32_t)(pol.dup_free ? lo : m) : 0u;
    sm += m;
    smn += m * n;
    cc[0] += c == 0;
    cc[1] += c == 1;
    cc[2] += c == 2;
    cc[3] += c == 3;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sm += __shfl_xor(sm, off, 64);
    smn += __shfl_xor(smn, off, 64);
#pragma unroll
    for (int k = 0; k < 4; ++k) cc[k] += __shfl_xor(cc[k], off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&s_sum[0], (unsigned long long)sm);
    atomicAdd(&s_sum[1], (unsigned long long)smn);
#pragma unroll
    for (int k = 0; k < 4; ++k) atomicAdd(&s_sum[2 + k], (unsigned long long)cc[k]);
  }
  __syncthreads();
  if (threadIdx.x < 6 && s_sum[threadIdx.x]) atomicAdd(&sums[threadIdx.x], s_sum[threadIdx.x]);
}

// tile_row[t] = the first merge row whose weight offset reaches t·(kIsTile / 2); tile_row[ntiles] = nM
__global__ void k_isect_tiles(const uint64_t *woff, uint64_t nM, uint64_t ntiles, uint32_t *tile_row) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  if (t == ntiles) {
    tile_row[t] = (uint32_t)nM;
    return;
  }
  const uint64_t key = t * (uint64_t)(kIsTile / 2);
  uint64_t lo = 0, hi = nM;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (woff[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  tile_row[t] = (uint32_t)lo;
}

template <bool WRITE>
__global__ __launch_bounds__(kIsBlock) void k_isect_merge(IsectArgs a) {
  constexpr int B = kIsBlock, IPT = kIsIPT, T = kIsTile, W = B / 64;
  __shared__ uint32_t s_stage[T];  // per row: its A list, then its B list
  __shared__ uint8_t s_seg[T];     // tile row owning each staged entry / merged position
  __shared__ uint32_t s_ot[T];     // the tile's matches: value …
  __shared__ uint8_t s_or[T];      // … and tile row
  __shared__ uint16_t s_lo[B], s_m[B], s_n[B];
  __shared__ uint64_t s_a[B], s_b[B];
  __shared__ uint32_t s_ri[B];
  __shared__ uint32_t s_w[W], s_w2[W], s_wmax[W];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint64_t medges = 0, nrows = 0;
  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint32_t r0 = a.tile_row[t], r1 = a.tile_row[t + 1];
    const uint32_t nr = r1 - r0;  // ≤ 205 (weight ≥ 10 a row, < 2056 a tile)
    // 1. the tile's rows: their two lists and where they are staged
    uint32_t m = 0, n = 0, ri = 0;
    uint64_t as = 0, bs = 0;
    if (tid < nr) {
      ri = a.idx[r0 + tid];
      const uint32_t x = a.xs[ri], y = a.ys[ri];
      as = a.ax.rp[x];
      bs = a.ay.rp[y];
      m = (uint32_t)(a.ax.rp[x + 1] - as);
      n = (uint32_t)(a.ay.rp[y + 1] - bs);
    }
    uint32_t total;
    const uint32_t lo = block_excl_scan<B>(m + n, s_w, &total);
    if (tid < nr) {
      s_lo[tid] = (uint16_t)lo;
      s_m[tid] = (uint16_t)m;
      s_n[tid] = (uint16_t)n;
      s_a[tid] = as;
      s_b[tid] = bs;
      s_ri[tid] = ri;
    }
    for (uint32_t k = tid; k < total; k += B) s_seg[k] = 0;
    __syncthreads();
    if (tid < nr) s_seg[lo] = (uint8_t)tid;  // every row holds ≥ 2 entries: distinct starts
    __syncthreads();
    {  // inclusive max-scan of the row marks over the tile (IPT consecutive entries a thread)
      uint32_t vals[IPT];
      uint32_t mx = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        const uint32_t k = tid * IPT + i;
        const uint32_t v = k < total ? s_seg[k] : 0u;
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
        const uint32_t k = tid * IPT + i;
        if (k < total) s_seg[k] = (uint8_t)(pre > vals[i] ? pre : vals[i]);
      }
    }
    __syncthreads();
    // 2. stage both lists of every row: all loads issued before the first LDS store
    {
      uint32_t v[IPT];
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const uint32_t k = j * B + tid;
        v[j] = 0;
        if (k < total) {
          const uint32_t lr = s_seg[k], q = k - s_lo[lr], mm = s_m[lr];
          v[j] = q < mm ? a.ax.col[s_a[lr] + q] : a.ay.col[s_b[lr] + (q - mm)];
        }
      }
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const uint32_t k = j * B + tid;
        if (k < total) s_stage[k] = v[j];
      }
    }
    __syncthreads();
    // 3. merge path: positions [tid·IPT, tid·IPT + IPT) of the rows' merged sequences
    uint32_t mt[IPT];
    uint32_t mr[IPT];
    uint32_t found = 0;
    {
      const uint32_t p0 = tid * IPT;
      uint32_t lr = 0, rlo = 0, mm = 0, nn = 0, i = 0, j = 0, last = 0, rend = 0;
      bool has = false;
      if (p0 < total) {
        lr = s_seg[p0];
        rlo = s_lo[lr];
        mm = s_m[lr];
        nn = s_n[lr];
        rend = rlo + mm + nn;
        const uint32_t *A = s_stage + rlo, *Bv = s_stage + rlo + mm;
        const uint32_t d = p0 - rlo;
        uint32_t l = d > nn ? d - nn : 0, h = d < mm ? d : mm;
        while (l < h) {  // i = A elements among the first d merged positions (ties: B first)
          const uint32_t mid = (l + h) >> 1;
          if (A[mid] < Bv[d - 1 - mid]) l = mid + 1;
          else h = mid;
        }
        i = l;
        j = d - l;
        has = j > 0;
        last = has ? Bv[j - 1] : 0u;
      }
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const uint32_t p = p0 + k;
        mt[k] = 0;
        mr[k] = 0;
        if (p < total) {
          if (p == rend) {  // the next row starts where this one ends (rows are staged back to back)
            ++lr;
            rlo = rend;
            mm = s_m[lr];
            nn = s_n[lr];
            rend = rlo + mm + nn;
            i = j = 0;
            has = false;
          }
          const uint32_t *A = s_stage + rlo, *Bv = s_stage + rlo + mm;
          if (j < nn && (i >= mm || Bv[j] <= A[i])) {
            last = Bv[j++];
            has = true;
          } else {
            const uint32_t tv = A[i++];
            if (!a.xfilter || bm_test(a.xfilter, tv)) {
              medges += nn;  // the unfused check would scan N_y(y) for this t
              if (has && last == tv && (!a.yfilter || bm_test(a.yfilter, tv))) {
                mt[k] = tv;
                mr[k] = lr;
                found |= 1u << k;
              }
            }
          }
        }
      }
    }
    // 4. the matches: scanned over the block, staged in LDS, written as full-block runs
    uint32_t tot;
    const uint32_t off = block_excl_scan<B>((uint32_t)__popc(found), s_w2, &tot);
    if (WRITE) {
      uint32_t o = off;
#pragma unroll
      for (int k = 0; k < IPT; ++k)
        if ((found >> k) & 1u) {
          s_ot[o] = mt[k];
          s_or[o] = (uint8_t)mr[k];
          ++o;
        }
      __syncthreads();
      const uint64_t base = a.boff[r0];
      for (uint32_t k = tid; k < tot; k += B) {
        const uint32_t row = s_ri[s_or[k]];
        a.out_dst[base + k] = s_ot[k];
        for (int c = 0; c < a.ncarry; ++c) a.carry_out[c][base + k] = a.carry_in[c][row];
      }
      if (tid == 0) {
        a.seg_count[t] = tot;
        a.seg_start[t] = base;
      }
    } else if (tid == 0) {
      nrows += tot;
    }
    __syncthreads();  // LDS reuse by the next tile
  }
  // one atomic per block and counter
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) medges += __shfl_xor(medges, off, 64);
  __shared__ unsigned long long s_me[W];
  if (lane == 0) s_me[wave] = medges;
  __syncthreads();
  if (tid == 0) {
    unsigned long long tmed = 0;
    for (int w = 0; w < W; ++w) tmed += s_me[w];
    if (tmed) atomicAdd(a.counters, tmed);
    if (nrows) atomicAdd(a.counters + 1, (unsigned long long)nrows);
  }
}

}  // namespace

void launch_isect_class(const uint32_t *xs, const uint32_t *ys, uint64_t R, const DAdjPart &ax, const DAdjPart &ay,
                        const IsectPolicy &pol, uint8_t *cls, uint32_t *w, uint32_t *bnd, unsigned long long *sums,
                        int cus, hipStream_t s) {
  if (!R) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(R, 256), (uint64_t)cus * 4);
  hipLaunchKernelGGL(k_isect_class, dim3(g), dim3(256), 0, s, xs, ys, R, ax, ay, pol, cls, w, bnd, sums);
  KCHECK("k_isect_class");
}

uint64_t isect_tiles(uint64_t wtotal) { return (wtotal + kIsTile / 2 - 1) / (kIsTile / 2); }

void launch_isect_tiles(const uint64_t *woff, uint64_t nM, uint64_t ntiles, uint32_t *tile_row, hipStream_t s) {
  hipLaunchKernelGGL(k_isect_tiles, dim3(nblocks(ntiles + 1, 256)), dim3(256), 0, s, woff, nM, ntiles, tile_row);
  KCHECK("k_isect_tiles");
}

void launch_isect_merge(const IsectArgs &a, bool write, int cus, hipStream_t s) {
  if (!a.ntiles) return;
  if (a.ncarry > kMaxCols) fail(OMX_E_INVALID, "internal: k_isect_merge carries at most kMaxCols columns");
  int occ = 0;
  if (write) HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_isect_merge<true>, kIsBlock, 0));
  else HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_isect_merge<false>, kIsBlock, 0));
  const unsigned g = (unsigned)std::min<uint64_t>(a.ntiles, (uint64_t)cus * std::max(occ, 1));
  if (write) hipLaunchKernelGGL(k_isect_merge<true>, dim3(g), dim3(kIsBlock), 0, s, a);
  else hipLaunchKernelGGL(k_isect_merge<false>, dim3(g), dim3(kIsBlock), 0, s, a);
  KCHECK("k_isect_merge");
}

}  // namespace omx
