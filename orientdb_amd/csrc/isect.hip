// isect.hip — the fused closing check of a cyclic pattern as a sorted-list intersection (BASELINE
// north_star (4)).
//
// A pattern edge x → t followed by a closing check y → t (t bound by the expansion) keeps the rows
// (…, t) with t ∈ N_x(x) ∩ N_y(y): the reference iterates N_x(x) and, for each t, scans N_y(y) until it
// finds t (existence with break, P/OMatchStatement.java:468-477). Both lists are sorted in the snapshot,
// so the device intersects them:
//   - rows whose two lists have comparable lengths (the larger ≤ ratio × the smaller, m + n ≤ 256) go
//     through k_isect_merge_w: a wave stages the two lists of every row of its tile in LDS with
//     independent loads, then walks the merged order of each row's pair with a merge path — lane l takes
//     positions [8l, 8l + 8) of the tile's concatenated merged sequences, finds its split of the row's
//     (A, B) pair by a binary search on the diagonal, and consumes one element a step; an A element (the
//     expansion's neighbour) matches when the last B element consumed equals it (ties put B first, so an
//     equal B element is always consumed before it). Parallel edges keep their multiplicity on the A side
//     (one row per edge x → t) and count once on the B side (existence), as the reference's loop does;
//   - skewed pairs keep the binary-search probe of the shorter list into the longer one (the fused
//     expansion kernels, Executor::expand_check_isect).
//
// Tiles: merge row r weighs m + n + 8; tile t holds the rows whose weight offset lies in [t·256,
// (t+1)·256), so a tile stages ≤ 512 entries over ≤ 52 rows — one wave's: the waves of a workgroup share
// no tile and meet at no barrier (round 4: a first version with 2048-entry tiles per 256-thread workgroup
// waited a dependent load chain and four barriers per tile, 2.06 ms at C4 against the probe's 0.74).
// k_isect_prep lays every merged row's (list starts, lengths) out in merge order first, so a tile's row
// loads are coalesced and independent. The rows of tile t write their matches at boff[first row of t]
// (boff: the scan of the rows' output bounds, min(m, n) when N_x has no parallel edges, else m) and
// report the count: a block-segmented table, compacted by the caller.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "devutil.h"
#include "graph.h"
#include "kernels.h"

namespace omx {

namespace {

constexpr int kIwTile = 512;          // list entries a wave tile stages (8 a lane)
constexpr int kIwIPT = kIwTile / 64;  // merged positions a lane walks
constexpr int kIwRows = 64;           // rows a tile holds at most (≤ 52 with the weights below)
constexpr int kIwWaves = 4;           // waves of a workgroup (independent)
static_assert(kIsRowCap * 2 == kIwTile, "a tile's weight window is half its entries");

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

// tile_row[t] = the first merge row whose weight offset reaches t·kIsRowCap; tile_row[ntiles] = nM
__global__ void k_isect_tiles(const uint64_t *woff, uint64_t nM, uint64_t ntiles, uint32_t *tile_row) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  if (t == ntiles) {
    tile_row[t] = (uint32_t)nM;
    return;
  }
  const uint64_t key = t * (uint64_t)kIsRowCap;
  uint64_t lo = 0, hi = nM;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (woff[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  tile_row[t] = (uint32_t)lo;
}

// every merged row's list starts and lengths in merge order (one thread a row: the dependent loads of
// all rows in flight at once, not at the head of each tile)
__global__ void k_isect_prep(const uint32_t *idx, uint64_t nM, const uint32_t *xs, const uint32_t *ys, DAdjPart ax,
                             DAdjPart ay, uint64_t *pa, uint64_t *pb, uint32_t *pmn) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nM) return;
  const uint32_t r = idx[k], x = xs[r], y = ys[r];
  const uint64_t a0 = ax.rp[x], a1 = ax.rp[x + 1], b0 = ay.rp[y], b1 = ay.rp[y + 1];
  pa[k] = a0;
  pb[k] = b0;
  pmn[k] = (uint32_t)(a1 - a0) | ((uint32_t)(b1 - b0) << 16);  // m, n ≤ kIsRowCap
}

struct IwTable {
  uint32_t stage[kIwTile];  // per row: its A list, then its B list
  uint32_t ot[kIwTile];     // the tile's matches: value …
  uint8_t seg[kIwTile];     // tile row owning each staged entry / merged position
  uint8_t orow[kIwTile];    // … and tile row
  uint16_t lo[kIwRows], m[kIwRows], n[kIwRows];
  uint32_t ri[kIwRows];
  uint64_t as[kIwRows], bs[kIwRows];
};

template <bool WRITE>
__global__ __launch_bounds__(64 * kIwWaves) void k_isect_merge_w(IsectArgs a) {
  constexpr int IPT = kIwIPT;
  __shared__ IwTable s_tb[kIwWaves];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  IwTable &tb = s_tb[wv];
  uint64_t medges = 0, nrows = 0;
  const uint64_t W = (uint64_t)gridDim.x * kIwWaves;
  for (uint64_t t = (uint64_t)blockIdx.x * kIwWaves + wv; t < a.ntiles; t += W) {
    const uint32_t r0 = a.tile_row[t], r1 = a.tile_row[t + 1];
    const uint32_t nr = r1 - r0;  // ≤ 52 (weight ≥ 10 a row, < 520 a tile)
    // 1. the tile's rows (one a lane), their staging offsets by a wave scan
    uint32_t m = 0, n = 0, ri = 0;
    uint64_t as = 0, bs = 0;
    if (lane < nr) {
      ri = a.idx[r0 + lane];
      as = a.pa[r0 + lane];
      bs = a.pb[r0 + lane];
      const uint32_t mn = a.pmn[r0 + lane];
      m = mn & 0xFFFFu;
      n = mn >> 16;
    }
    uint32_t incl = m + n;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= (uint32_t)off) incl += y;
    }
    const uint32_t lo = incl - (m + n), total = __shfl(incl, 63, 64);
    if (lane < nr) {
      tb.lo[lane] = (uint16_t)lo;
      tb.m[lane] = (uint16_t)m;
      tb.n[lane] = (uint16_t)n;
      tb.ri[lane] = ri;
      tb.as[lane] = as;
      tb.bs[lane] = bs;
    }
    uint32_t *seg32 = reinterpret_cast<uint32_t *>(tb.seg) + lane * (IPT / 4);
#pragma unroll
    for (int q = 0; q < IPT / 4; ++q) seg32[q] = 0;
    __builtin_amdgcn_wave_barrier();
    if (lane < nr) tb.seg[lo] = (uint8_t)lane;  // every row holds ≥ 2 entries: distinct starts
    __builtin_amdgcn_wave_barrier();
    {  // inclusive max-scan of the row marks: lane l holds bytes 8l … 8l + 7
      uint32_t wd[IPT / 4];
      uint32_t mx = 0;
#pragma unroll
      for (int q = 0; q < IPT / 4; ++q) {
        wd[q] = seg32[q];
#pragma unroll
        for (int b = 0; b < 4; ++b) mx = max(mx, (wd[q] >> (8 * b)) & 0xFFu);
      }
      uint32_t sc = mx;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(sc, off, 64);
        if (lane >= (uint32_t)off) sc = max(sc, y);
      }
      uint32_t run = __shfl_up(sc, 1, 64);
      if (lane == 0) run = 0;
#pragma unroll
      for (int q = 0; q < IPT / 4; ++q) {
        uint32_t o = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          run = max(run, (wd[q] >> (8 * b)) & 0xFFu);
          o |= run << (8 * b);
        }
        seg32[q] = o;
      }
    }
    __builtin_amdgcn_wave_barrier();
    // 2. stage both lists of every row: all loads issued before the first LDS store
    {
      uint32_t v[IPT];
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const uint32_t p = j * 64 + lane;
        v[j] = 0;
        if (p < total) {
          const uint32_t lr = tb.seg[p], q = p - tb.lo[lr], mm = tb.m[lr];
          v[j] = q < mm ? a.ax.col[tb.as[lr] + q] : a.ay.col[tb.bs[lr] + (q - mm)];
        }
      }
#pragma unroll
      for (int j = 0; j < IPT; ++j) {
        const uint32_t p = j * 64 + lane;
        if (p < total) tb.stage[p] = v[j];
      }
    }
    __builtin_amdgcn_wave_barrier();
    // 3. merge path: positions [lane·IPT, lane·IPT + IPT) of the rows' merged sequences
    uint32_t mt[IPT];
    uint32_t mr[IPT];
    uint32_t found = 0;
    {
      const uint32_t p0 = lane * IPT;
      uint32_t lr = 0, rlo = 0, mm = 0, nn = 0, i = 0, j = 0, last = 0, rend = 0;
      bool has = false;
      if (p0 < total) {
        lr = tb.seg[p0];
        rlo = tb.lo[lr];
        mm = tb.m[lr];
        nn = tb.n[lr];
        rend = rlo + mm + nn;
        const uint32_t *A = tb.stage + rlo, *Bv = tb.stage + rlo + mm;
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
            mm = tb.m[lr];
            nn = tb.n[lr];
            rend = rlo + mm + nn;
            i = j = 0;
            has = false;
          }
          const uint32_t *A = tb.stage + rlo, *Bv = tb.stage + rlo + mm;
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
    // 4. the matches: a wave scan, staged in LDS, written as full-wave runs at the tile's slot
    const uint32_t c = (uint32_t)__popc(found);
    uint32_t oincl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(oincl, off, 64);
      if (lane >= (uint32_t)off) oincl += y;
    }
    const uint32_t tot = __shfl(oincl, 63, 64);
    if (WRITE) {
      uint32_t o = oincl - c;
#pragma unroll
      for (int k = 0; k < IPT; ++k)
        if ((found >> k) & 1u) {
          tb.ot[o] = mt[k];
          tb.orow[o] = (uint8_t)mr[k];
          ++o;
        }
      __builtin_amdgcn_wave_barrier();
      const uint64_t base = a.boff[r0];
      for (uint32_t k = lane; k < tot; k += 64) {
        const uint32_t row = tb.ri[tb.orow[k]];
        a.out_dst[base + k] = tb.ot[k];
        for (int cc = 0; cc < a.ncarry; ++cc) a.carry_out[cc][base + k] = a.carry_in[cc][row];
      }
      if (lane == 0) {
        a.seg_count[t] = tot;
        a.seg_start[t] = base;
      }
    } else if (lane == 0) {
      nrows += tot;
    }
    __builtin_amdgcn_wave_barrier();  // the table is rebuilt for the next tile
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) medges += __shfl_xor(medges, off, 64);
  if (lane == 0) {
    if (medges) atomicAdd(a.counters, (unsigned long long)medges);
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

uint64_t isect_tiles(uint64_t wtotal) { return (wtotal + kIsRowCap - 1) / kIsRowCap; }

void launch_isect_tiles(const uint64_t *woff, uint64_t nM, uint64_t ntiles, uint32_t *tile_row, hipStream_t s) {
  hipLaunchKernelGGL(k_isect_tiles, dim3(nblocks(ntiles + 1, 256)), dim3(256), 0, s, woff, nM, ntiles, tile_row);
  KCHECK("k_isect_tiles");
}

void launch_isect_prep(const uint32_t *idx, uint64_t nM, const uint32_t *xs, const uint32_t *ys, const DAdjPart &ax,
                       const DAdjPart &ay, uint64_t *pa, uint64_t *pb, uint32_t *pmn, hipStream_t s) {
  if (!nM) return;
  hipLaunchKernelGGL(k_isect_prep, dim3(nblocks(nM, 256)), dim3(256), 0, s, idx, nM, xs, ys, ax, ay, pa, pb, pmn);
  KCHECK("k_isect_prep");
}

void launch_isect_merge(const IsectArgs &a, bool write, int cus, hipStream_t s) {
  if (!a.ntiles) return;
  if (a.ncarry > kMaxCols) fail(OMX_E_INVALID, "internal: k_isect_merge_w carries at most kMaxCols columns");
  int occ = 0;
  if (write) HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_isect_merge_w<true>, 64 * kIwWaves, 0));
  else HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_isect_merge_w<false>, 64 * kIwWaves, 0));
  const uint64_t blocks = (a.ntiles + kIwWaves - 1) / kIwWaves;
  const unsigned g = (unsigned)std::min<uint64_t>(blocks, (uint64_t)cus * std::max(occ, 1));
  if (write) hipLaunchKernelGGL(k_isect_merge_w<true>, dim3(g), dim3(64 * kIwWaves), 0, s, a);
  else hipLaunchKernelGGL(k_isect_merge_w<false>, dim3(g), dim3(64 * kIwWaves), 0, s, a);
  KCHECK("k_isect_merge_w");
}

}  // namespace omx
