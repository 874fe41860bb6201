// factor.hip — the filtered neighbour lists of a factorized hop (exec.hip Executor::expand_factorized).
//
// A filtered hop whose rows repeat their source vertices is expanded once per distinct source u: L(u) =
// the neighbours of u passing the target's WHERE bitmap (OMatchPathItem.executeTraversal with the
// filter, P/OMatchPathItem.java:63-78), grouped by source so that the rows are written over the lists.
// The lists come from the generic filtered expansion and a key histogram / scatter (exec.hip); this file
// writes the rows over them (the factorized emission below).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "devutil.h"

namespace omx {

namespace {

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

// ---- the factorized emission: every row (…, u) written over L(u) -------------------------------------
// The result rows of a factorized hop are Σ_rows |L(g[r])| — known before anything is written — so they
// are laid out densely, row by row (roff = the exclusive scan of the rows' list lengths; the rows are
// grouped by source beforehand, so a list is re-read from L2 by its rows), and written by tiles of the
// OUTPUT space rather than by binned rows: no degree binning, no heavy/light split, no arenas — every
// output row costs the same whatever the length of its list.
//
// k_femit_w: every wave owns tiles of kEwTile consecutive output rows (tile i → wave i mod W). A tile over
// at most 64 binding rows (nearly all) is "regular": its rows are loaded one per lane into the wave's own
// LDS table (list base, carried values) and mark their first output in a byte array, which a max-scan
// spreads, so output row o's table entry is one LDS byte (no barriers: the table is the wave's). Lane l
// writes output rows l + 64j (j < 16): every store is a 256-byte run of dwords per column. The other tiles
// (more than 64 rows — a run of short lists — and the partial last tile) go to k_femit_slow.
// Software pipeline over a wave's tiles t, t', t'': while t is stored, the list entries of t' are already
// requested (its table in the second LDS buffer) and the rows of t''. Vector memory completes in issue
// order on CDNA, so a load issued after a store waits for it: nothing a store needs is issued after an
// earlier store, and every memory instruction of the loop body runs unconditionally (clamped indices)
// so the compiler's wait counts stay exact across iterations.
// Occupancy: 8 waves per CU (one 512-thread workgroup). Measured at M1 (profiles/r03/femit): 6 or 10
// waves per CU 2.8 ms, 8 waves 2.2-2.3 ms; 16-byte stores of 4 consecutive rows per lane 2.6-2.9 ms; a
// contiguous run of tiles per wave 2.7 ms; the binned heavy/merge-path kernels 3.2 ms.
#ifndef OMX_EW_TILE
#define OMX_EW_TILE 1024
#endif
#ifndef OMX_EW_WAVES
#define OMX_EW_WAVES 8
#endif
constexpr int kEwTile = OMX_EW_TILE, kEwWaves = OMX_EW_WAVES, kEwJ = kEwTile / 64;
static_assert(kEwTile <= 256 * 64, "a lane's mark bytes are read as u32 words");

// len[r] = |L(g[r])| for r < n, 0 for n ≤ r ≤ R; n = *nd when nd is given (a device count ≤ R), else R
__global__ void k_femit_len(const uint32_t *g, uint64_t R, const uint64_t *loff, uint64_t *len, const uint64_t *nd) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r > R) return;
  const uint64_t n = nd ? *nd : R;
  if (r >= n) {
    len[r] = 0;
    return;
  }
  const uint32_t u = g[r];
  len[r] = loff[u + 1] - loff[u];
}

__global__ void k_femit_base(const uint32_t *g, uint64_t R, const uint64_t *loff, const uint64_t *roff, uint64_t *rbase,
                             const uint64_t *nd) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < (nd ? *nd : R)) rbase[r] = loff[g[r]] - roff[r];
}

// first and last binding row of every output tile (the rows holding its first and last output): one
// thread per binding row writes the tiles whose first / last output row falls in it (rows are non-empty,
// so every tile gets exactly one of each); then whether the tile is regular (full, ≤ 64 rows; slow_all:
// every tile through k_femit_slow, tests). One pass over the rows instead of two binary searches per tile.
__global__ void k_femit_bounds(const uint64_t *roff, uint64_t R, uint64_t N, uint64_t *rb) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint64_t rs = roff[r], re = roff[r + 1];
  for (uint64_t t = (rs + kEwTile - 1) / kEwTile; t * kEwTile < re; ++t) rb[2 * t] = r;  // tiles starting here
  const uint64_t last = (N - 1) / kEwTile;
  for (uint64_t t = rs / kEwTile; t <= last; ++t) {  // tiles ending here
    const uint64_t te = min((t + 1) * (uint64_t)kEwTile, N) - 1;
    if (te >= re) break;
    if (te >= rs) rb[2 * t + 1] = r;
  }
}
__global__ void k_femit_classify(const uint64_t *rb, uint64_t N, uint64_t ntiles, uint8_t *regular, int slow_all) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  regular[t] = !slow_all && rb[2 * t + 1] - rb[2 * t] < 64 && (t + 1) * kEwTile <= N;
}

struct EwRows {  // lane k: binding row r0 + k of the tile, as loaded (put into the table one step later)
  uint64_t rs;   // its first output row
  uint64_t base; // list position of output row o = base + o
  uint32_t car[kFemitCols];
  uint64_t t;    // the tile (wave-uniform)
  uint32_t ok;   // lane < rows of the tile
};

// tiles and rb are read with scalar loads: __restrict__ lets the compiler prove nothing here writes them
template <int NL, int NC>
__device__ __forceinline__ EwRows ew_rows(const FemitArgs &a, const uint32_t *__restrict__ tiles,
                                          const uint64_t *__restrict__ rb, uint64_t i, uint32_t lane) {
  EwRows w;
  w.t = tiles[i];
  const uint64_t r0 = rb[2 * w.t], nr = rb[2 * w.t + 1] - r0 + 1;  // ≤ 64 (regular tile)
  w.ok = lane < nr;
  const uint64_t r = r0 + (w.ok ? lane : 0);  // every lane loads: no branch around the loads
  w.rs = a.roff[r];
  w.base = a.rbase[r];
#pragma unroll
  for (int c = 0; c < kFemitCols; ++c) w.car[c] = c < NC ? a.cin[c][r] : 0u;
  return w;
}

template <int NL, int NC>
struct EwTable {
  uint32_t mk[kEwTile / 4];  // kEwTile u8: the table entry of every output row of the tile
  uint64_t base[64];
  uint32_t car[NC > 0 ? NC : 1][64];
};

template <int NL, int NC>
__device__ __forceinline__ void ew_put(EwTable<NL, NC> &tb, const EwRows &w, uint32_t lane) {
  constexpr int BPL = kEwTile / 64;  // mark bytes per lane
  const uint64_t t0 = w.t * kEwTile;
  uint32_t *mk = tb.mk + lane * (BPL / 4);
#pragma unroll
  for (int i = 0; i < BPL / 4; ++i) mk[i] = 0;
  tb.base[lane] = w.base;
#pragma unroll
  for (int c = 0; c < NC; ++c) tb.car[c][lane] = w.car[c];
  __builtin_amdgcn_wave_barrier();
  // a row other than the tile's first starts inside the tile (the first starts at or before it; rows
  // have non-empty lists, so their starts are distinct)
  if (w.ok && w.rs > t0 && w.rs < t0 + kEwTile) reinterpret_cast<uint8_t *>(tb.mk)[w.rs - t0] = (uint8_t)lane;
  __builtin_amdgcn_wave_barrier();
  uint32_t wd[BPL / 4];
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < BPL / 4; ++i) {
    wd[i] = mk[i];
#pragma unroll
    for (int b = 0; b < 4; ++b) m = max(m, (wd[i] >> (8 * b)) & 0xFFu);
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
  for (int i = 0; i < BPL / 4; ++i) {
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      run = max(run, (wd[i] >> (8 * b)) & 0xFFu);
      o |= run << (8 * b);
    }
    mk[i] = o;
  }
  __builtin_amdgcn_wave_barrier();
}

template <int NL, int NC>
__device__ __forceinline__ void ew_resolve(const FemitArgs &a, const EwTable<NL, NC> &tb, uint64_t t, uint32_t lane,
                                           uint32_t (&x)[NL][kEwJ]) {
  const uint64_t t0 = t * kEwTile;
  const uint8_t *mk = reinterpret_cast<const uint8_t *>(tb.mk);
#pragma unroll
  for (int j = 0; j < kEwJ; ++j) {
    const uint32_t o = 64 * j + lane;
    const uint64_t p = tb.base[mk[o]] + t0 + o;
#pragma unroll
    for (int m = 0; m < NL; ++m) x[m][j] = a.lcol[m][p];
  }
}

template <int NL, int NC>
__device__ __forceinline__ void ew_store(const FemitArgs &a, const EwTable<NL, NC> &tb, uint64_t t, uint32_t lane,
                                         const uint32_t (&x)[NL][kEwJ]) {
  const uint64_t t0 = t * kEwTile;
  const uint8_t *mk = reinterpret_cast<const uint8_t *>(tb.mk);
#pragma unroll
  for (int j = 0; j < kEwJ; ++j) {
    const uint32_t o = 64 * j + lane, k = mk[o];
#pragma unroll
    for (int m = 0; m < NL; ++m) a.lout[m][t0 + o] = x[m][j];
#pragma unroll
    for (int c = 0; c < NC; ++c) a.cout[c][t0 + o] = tb.car[c][k];
  }
}

// tiles: the regular tiles, *nreg of them (a device count: the partition's, read by the kernel, so the
// host does not wait for it between the partition and the launch)
template <int NL, int NC>
__global__ __launch_bounds__(64 * kEwWaves) void k_femit_w(FemitArgs a, const uint32_t *__restrict__ tiles,
                                                          const uint64_t *__restrict__ rb,
                                                          const uint64_t *__restrict__ nreg) {
  __shared__ EwTable<NL, NC> s_tb[kEwWaves][2];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t n = *nreg;
  const uint64_t W = (uint64_t)gridDim.x * kEwWaves;
  uint64_t i = (uint64_t)blockIdx.x * kEwWaves + wv;
  if (i >= n) return;
  // prologue: tile i's table and list entries, tile i + W's rows (indices past the end are clamped:
  // loaded, never stored)
  EwRows r0 = ew_rows<NL, NC>(a, tiles, rb, i, lane), r1;
  ew_put<NL, NC>(s_tb[wv][0], r0, lane);
  uint32_t x0[NL][kEwJ], x1[NL][kEwJ];
  ew_resolve<NL, NC>(a, s_tb[wv][0], r0.t, lane, x0);
  uint64_t t_cur = r0.t;
  r0 = ew_rows<NL, NC>(a, tiles, rb, min(i + W, n - 1), lane);
  // drain the prologue: the loop's entry then has nothing outstanding, so the waits the compiler places
  // at its head are those of the back edge, not vmcnt(0)
  __builtin_amdgcn_s_waitcnt(0);
  // one step: rows of tile i + 2W requested (rn), tile i + W's table put (rp) and its list entries
  // requested (xl), tile i stored (xs); unrolled twice so the register sets alternate instead of being
  // copied (a copy would wait for its loads)
#define OMX_EW_STEP(rp, rn, xs, xl, bs)                                  \
  {                                                                     \
    rn = ew_rows<NL, NC>(a, tiles, rb, min(i + 2 * W, n - 1), lane);    \
    ew_put<NL, NC>(s_tb[wv][(bs) ^ 1], rp, lane);                       \
    ew_resolve<NL, NC>(a, s_tb[wv][(bs) ^ 1], rp.t, lane, xl);          \
    ew_store<NL, NC>(a, s_tb[wv][bs], t_cur, lane, xs);                 \
    __builtin_amdgcn_wave_barrier(); /* rewritten two tiles on */       \
    t_cur = rp.t;                                                       \
    i += W;                                                             \
  }
  for (;;) {
    OMX_EW_STEP(r0, r1, x0, x1, 0)
    if (i >= n) break;
    OMX_EW_STEP(r1, r0, x1, x0, 1)
    if (i >= n) break;
  }
#undef OMX_EW_STEP
}

// the other tiles (tiles[*nreg, nt)): one workgroup each, every output row's binding row by a search of
// the row offsets
__global__ __launch_bounds__(256) void k_femit_slow(FemitArgs a, const uint32_t *all_tiles, const uint64_t *nreg,
                                                    uint64_t nt) {
  const uint64_t nr = *nreg;
  const uint32_t *tiles = all_tiles + nr;
  const uint64_t n = nt - nr;
  for (uint64_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint64_t t = tiles[i], t0 = t * kEwTile, r0 = a.rb[2 * t], r1 = a.rb[2 * t + 1];
    const uint32_t ne = (uint32_t)min((uint64_t)kEwTile, a.N - t0);
    // 4 consecutive output rows per thread: one search, then the rows walked forward
    for (uint32_t e = 4 * threadIdx.x; e < ne; e += 4 * blockDim.x) {
      uint64_t r = last_le_range(a.roff, r0, r1, t0 + e);
      for (uint32_t k = e; k < min(e + 4, ne); ++k) {
        const uint64_t o = t0 + k;
        while (a.roff[r + 1] <= o) ++r;
        for (int m = 0; m < a.nl; ++m) a.lout[m][o] = a.lcol[m][a.rbase[r] + o];
        for (int c = 0; c < a.nc; ++c) a.cout[c][o] = a.cin[c][r];
      }
    }
  }
}

}  // namespace

uint64_t femit_tiles(uint64_t N) { return (N + kEwTile - 1) / kEwTile; }

// the (list columns, constants) instances of k_femit_w: (1, 0…4) the rows over their sources' lists
bool femit_supported(int nl, int nc) { return nl == 1 && nc <= 4; }

void launch_femit_len(const uint32_t *g, uint64_t R, const uint64_t *loff, uint64_t *len, hipStream_t s,
                      const uint64_t *nd) {
  hipLaunchKernelGGL(k_femit_len, dim3(nblocks(R + 1, 256)), dim3(256), 0, s, g, R, loff, len, nd);
  KCHECK("k_femit_len");
}

void launch_femit_base(const uint32_t *g, uint64_t R, const uint64_t *loff, const uint64_t *roff, uint64_t *rbase,
                       hipStream_t s, const uint64_t *nd) {
  if (!R) return;
  hipLaunchKernelGGL(k_femit_base, dim3(nblocks(R, 256)), dim3(256), 0, s, g, R, loff, roff, rbase, nd);
  KCHECK("k_femit_base");
}

void launch_femit_bounds(const FemitArgs &a, uint64_t *rb, uint8_t *regular, bool slow_all, hipStream_t s) {
  const uint64_t nt = femit_tiles(a.N);
  if (!nt || !a.R) return;
  hipLaunchKernelGGL(k_femit_bounds, dim3(nblocks(a.R, 256)), dim3(256), 0, s, a.roff, a.R, a.N, rb);
  KCHECK("k_femit_bounds");
  hipLaunchKernelGGL(k_femit_classify, dim3(nblocks(nt, 256)), dim3(256), 0, s, rb, a.N, nt, regular, (int)slow_all);
  KCHECK("k_femit_classify");
}

void launch_femit(const FemitArgs &a, const uint32_t *tiles, const uint64_t *nreg, uint64_t nt, int cus,
                  hipStream_t s) {
  if (a.nc > kFemitCols || a.nl < 1 || a.nl > kFemitLists || !femit_supported(a.nl, a.nc))
    fail(OMX_E_INVALID, "internal: no k_femit_w instance for these columns");
  if (!nt) return;
  // one workgroup per CU, all resident at once: the tiles are assigned statically (sized for all nt tiles;
  // waves past the regular count exit at once)
  const dim3 grid((unsigned)std::min<uint64_t>((nt + kEwWaves - 1) / kEwWaves, (uint64_t)cus)), blk(64 * kEwWaves);
#define OMX_FEMIT_CASE(L, C) \
  case L * 8 + C: hipLaunchKernelGGL((k_femit_w<L, C>), grid, blk, 0, s, a, tiles, a.rb, nreg); break;
  switch (a.nl * 8 + a.nc) {
    OMX_FEMIT_CASE(1, 0) OMX_FEMIT_CASE(1, 1) OMX_FEMIT_CASE(1, 2) OMX_FEMIT_CASE(1, 3) OMX_FEMIT_CASE(1, 4)
    default: break;
  }
#undef OMX_FEMIT_CASE
  KCHECK("k_femit_w");
  hipLaunchKernelGGL(k_femit_slow, dim3((unsigned)std::min<uint64_t>(nt, (uint64_t)cus * 4)), dim3(256), 0, s, a, tiles,
                     nreg, nt);
  KCHECK("k_femit_slow");
}

}  // namespace omx
