// factor.hip — the filtered neighbour lists of a factorized hop (exec.hip Executor::expand_factorized).
//
// A filtered hop whose rows repeat their source vertices is expanded once per distinct source u: L(u) =
// the neighbours of u passing the target's WHERE bitmap (OMatchPathItem.executeTraversal with the
// filter, P/OMatchPathItem.java:63-78), grouped by source so that the rows are written over the lists.
// This file builds the lists in one tiled pass over the sources' rows (k_flist + k_flist_copy, round 5;
// exec.hip falls back to the binned filtered expansion + key histogram / scatter for multigraph
// set-valued hops, several CSR parts, partitions, semi-joins and when the lists col does not fit) and
// writes the rows over them (the factorized emission, k_femit_w).
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

// ---- the filtered lists of the distinct sources (round 5) -------------------------------------------
// L(u) = {r in N(u) : filter(r)} for the U distinct sources of a factorized hop, grouped by source (CSR
// loff / lcol), in one pass over their rows plus a copy.
// The sources' rows are read as aligned 4-entry chunks of the CSR's hub-annotated col (one 16-byte load
// per chunk; a row's first and last chunk mask the entries outside it): the chunks of all sources, in
// source order, form the chunk space (coff = the scan of every source's chunk count), cut into tiles of
// kFlChunks chunks, tile t → wave t mod W.
// Filter: every entry probes one bit array with one buffer load per entry index of the lane: the filter's
// words, then the hubs' bits by rank (a hub — one of the CSR's kFlistHubs vertices of highest in-degree,
// bfs.hip build_pull_col — is entered in the lists col as vb + its rank, vb = the filter's bits: its bit
// index is its entry; the hubs' 128 KiB of bits sit in the workgroup's LDS). No entry is checked before its
// probe: a chunk's entries outside the source's row are other rows' entries (in range) or the col's
// zeroed padding.
// Output: a tile's survivors, in entry order — which is source order — are written to its own
// kFlChunks·4-entry scratch slot (staged in LDS, 16-byte stores), with their count; the sources starting
// strictly inside the tile get their offset inside the tile's survivors. A scan of the counts gives every
// tile its base in lcol, k_flist_copy moves the survivors there (hub ranks back to vertices) and
// k_flist_loff finishes the list offsets.
// Measured (round 5, PMC): the pass is bound by instruction issue, not bytes — so no per-entry branch or
// conditional LDS write: compactions write every lane, the ones that have nothing to write to a discard
// slot of their own.
// The pass is software-pipelined over a wave's tiles: step i requests tile i+4's bounds, tile i+3's
// sources, tile i+2's chunks (after its LDS table is built), tile i+1's filter probes, and consumes tile i.
// Every memory instruction of a step is unconditional (indices clamped, stores dropped by the buffer
// range check), so the compiler's wait counts are exact, and every wait is for an instruction issued in
// the previous step — never behind the stores that step ended with (vector memory completes in order).
constexpr int kFlChunks = 128, kFlQ = kFlChunks / 64, kFlE = 4 * kFlQ;  // chunks per tile / per lane, entries per lane
constexpr int kFlWaves = 8, kFlSlots = 128;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kFlDrop = 0x80000000u;     // a buffer offset past every range: the access is dropped
constexpr uint32_t kFlDeferred = 0xFFFFFFFFu;  // a tile's count when k_flist_wide handles it

// bits[i] = the filter's u32 word i (i < vb/32), then word vb/32 + w bit i = the filter bit of hubs[32w + i]
// (no filter: every bit set)
__global__ void k_probe_bits(const uint32_t *hubs, uint32_t nh, const uint64_t *filter, uint32_t vb, uint32_t *bits) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t fw = vb / 32, fwp = (fw + 63) & ~63u, lane = threadIdx.x & 63;
  if (r < fwp) {  // (whole waves: threads [0, fwp) copy, the rest ballot 64 hubs a wave)
    if (r < fw) bits[r] = filter ? reinterpret_cast<const uint32_t *>(filter)[r] : 0xFFFFFFFFu;
    return;
  }
  const uint64_t h = r - fwp;
  const bool b = h < nh && (!filter || bm_test(filter, hubs[h < nh ? h : 0]));
  const uint64_t m = __builtin_amdgcn_ballot_w64(b);
  const uint64_t w0 = (h - lane) / 32;
  if (lane < 2 && (w0 + lane) * 32 < nh) bits[fw + w0 + lane] = (uint32_t)(m >> (32 * lane));
}
// a hub-annotated col entry (0x80000000 | rank) as vb + rank
__global__ void k_list_col(uint32_t *col, uint64_t E, uint32_t vb) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < E) {
    const uint32_t x = col[i];
    if (x >> 31) col[i] = vb + (x & 0x7FFFFFFFu);
  } else if (i < E + 4) {
    col[i] = 0u;
  }
}

// a source's row as chunks: the 4-entry groups of the col it touches
__device__ __forceinline__ uint32_t fl_nch(uint64_t rs, uint64_t deg) {
  return deg ? (uint32_t)(((rs + deg + 3) >> 2) - (rs >> 2)) : 0u;
}
__global__ void k_flist_nch(const uint32_t *ub, const uint64_t *doff, uint64_t U, const uint64_t *rp, uint32_t *nch) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < U) nch[i] = fl_nch(rp[ub[i]], doff[i + 1] - doff[i]);
  else if (i == U) nch[U] = 0;  // (the scan's last entry)
}
// every source's chunk table entry {gbase, coff, pack}: chunk c of the space is col group gbase + c;
// pack = first-chunk skip | (last-chunk entries − 1) << 2 | chunks << 4
__global__ void k_flist_info(const uint32_t *ub, const uint64_t *doff, const uint64_t *coff, uint64_t U,
                             const uint64_t *rp, uint4 *info) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= U) return;
  const uint64_t rs = rp[ub[i]], deg = doff[i + 1] - doff[i], c = coff[i];
  const uint64_t gb = (rs >> 2) - c;
  const uint32_t n = fl_nch(rs, deg);
  const uint32_t pack = (uint32_t)(rs & 3) | (deg ? (uint32_t)((rs + deg - 1) & 3) << 2 : 0u) | (n << 4);
  info[i] = make_uint4((uint32_t)gb, (uint32_t)(gb >> 32), (uint32_t)c, pack);
}
// first / last source of every tile of the chunk space: the sources whose chunk ranges hold the tile's first
// and last chunk (the last source with coff ≤ c: an empty source shares its coff with the next one, so
// it is never the last) — one thread per tile, two binary searches
__device__ __forceinline__ uint64_t fl_source_of(const uint64_t *coff, uint64_t U, uint64_t c) {
  uint64_t lo = 0, hi = U;  // the first r with coff[r] > c, in (0, U]
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (coff[mid] <= c) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;
}
// (ntot: the tiles past the chunk space, up to the bound's ntb, get a zero count for the counts' scan —
// every real tile's count is written by k_flist)
__global__ void k_flist_bounds(const uint64_t *coff, uint64_t U, const uint64_t *ec, uint64_t *rb, uint32_t *ntot,
                               uint64_t ntb) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, N = *ec;
  if (t > ntb) return;
  if (t * kFlChunks >= N) {
    ntot[t] = 0;
    return;
  }
  rb[2 * t] = fl_source_of(coff, U, t * kFlChunks);
  rb[2 * t + 1] = fl_source_of(coff, U, min((t + 1) * (uint64_t)kFlChunks, N) - 1);
}

struct FlHdr {
  uint64_t s0, ns;
};
struct FlSlot {  // a non-empty source of the tile being set up
  uint64_t gbase;
  uint32_t coff, pack;
};
struct FlWave {  // one wave's LDS
  union {
    struct {
      FlSlot tbl[kFlSlots];            // setup: the tile's non-empty sources, in order
      uint8_t st[kFlChunks];           // setup: st[c] = a non-empty source starts at chunk c of the tile
    } s;
    uint32_t surv[kFlE * 64];          // consume: the tile's survivors, in entry order
  } u;
  uint32_t coff[3][kFlSlots];          // the tiles' sources' first chunks (ring of 3)
  FlHdr hdr[3];
  uint16_t qs[kFlQ][64];               // consume: survivors before each chunk
};

__global__ __launch_bounds__(64 * kFlWaves) void k_flist(FlistArgs a) {
  __shared__ uint32_t s_hub[kFlistHubs / 32];
  __shared__ FlWave s_w[kFlWaves];
  const uint32_t lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  {  // the hubs' bits, 8 words a thread in flight
    const uint32_t hw = (a.nh + 31) / 32, *hb = a.bits + a.vb / 32;
    for (uint32_t b0 = 0; b0 < hw; b0 += 8 * blockDim.x) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t i = b0 + u * blockDim.x + threadIdx.x;
        v[u] = hb[i < hw ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t i = b0 + u * blockDim.x + threadIdx.x;
        if (i < hw) s_hub[i] = v[u];
      }
    }
  }
  __syncthreads();
  FlWave &w = s_w[wv];
  const uint4 *const acol4 = reinterpret_cast<const uint4 *>(a.acol);
  const __amdgpu_buffer_rsrc_t fr = __builtin_amdgcn_make_buffer_rsrc((void *)a.bits, 0, (int32_t)a.bbytes, 0x00020000);
  const uint64_t EC = *a.ec;
  const uint64_t nt = (EC + kFlChunks - 1) / kFlChunks;
  const uint64_t W = (uint64_t)gridDim.x * kFlWaves;
  const uint64_t tw = (uint64_t)blockIdx.x * kFlWaves + wv;
  if (tw >= nt) return;
  const uint64_t ntw = (nt - tw + W - 1) / W;  // tiles of this wave
  auto tile = [&](uint64_t i) { return tw + (i < ntw ? i : ntw - 1) * W; };
  const uint64_t gmax = (a.E + 3) / 4 - 1;
  // stage a: a tile's first / last source (lanes 0, 1)
  auto ld_bounds = [&](uint64_t i) -> uint64_t { return a.rb[2 * tile(i) + (lane & 1)]; };
  // stage b: its sources' chunk table entries
  auto ld_src = [&](uint64_t bv, uint4 (&sv)[2], FlHdr &h) {
    h.s0 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(bv >> 32), 0) << 32) | __builtin_amdgcn_readlane((uint32_t)bv, 0);
    const uint64_t s1 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(bv >> 32), 1) << 32) | __builtin_amdgcn_readlane((uint32_t)bv, 1);
    h.ns = s1 - h.s0 + 1;
    const uint64_t smax = a.U - 1;
    // (only the tile's sources: lanes past them are dropped by the range, no cache lines touched)
    (void)smax;
    const uint32_t nr = (uint32_t)min<uint64_t>(h.ns, (uint64_t)kFlSlots) * 16;
    const __amdgpu_buffer_rsrc_t ir = __builtin_amdgcn_make_buffer_rsrc((void *)(a.info + h.s0), 0, (int32_t)nr, 0x00020000);
    const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(ir, 16 * lane, 0, 0);
    // (a tile over ≤ 64 sources — all of M1's — issues one load: the TA's cost is per instruction)
    u32x4 v1 = {0u, 0u, 0u, 0u};
    if (h.ns > 64) v1 = __builtin_amdgcn_raw_buffer_load_b128(ir, 16 * (64 + lane), 0, 0);
    sv[0] = make_uint4(v0.x, v0.y, v0.z, v0.w);
    sv[1] = make_uint4(v1.x, v1.y, v1.z, v1.w);
  };
  // stage c: the tile's LDS table (non-empty sources in order, the chunks where they start), then its
  // chunks requested; vm = the lane's valid entries (bit 4q + i: component i of its chunk q)
  auto setup = [&](uint64_t i, const uint4 (&sv)[2], const FlHdr &h, int r, uint32_t (&x)[kFlE], uint32_t &vm) {
    const uint64_t t = tile(i), c0 = t * kFlChunks;
    const uint32_t nc = (uint32_t)min<uint64_t>((uint64_t)kFlChunks, EC - c0);
    const bool reg = h.ns <= (uint64_t)kFlSlots;
    if (lane < kFlChunks / 4) reinterpret_cast<uint32_t *>(w.u.s.st)[lane] = 0u;
    if (lane == 0) w.hdr[r] = h;
    uint32_t rank0 = 0;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t k = 64 * c + lane;
      const uint32_t cf = sv[c].z, nchk = sv[c].w >> 4;
      w.coff[r][k] = cf;
      const bool live = k < h.ns && nchk > 0;
      const uint64_t bl = __builtin_amdgcn_ballot_w64(live);
      FlSlot sl;
      sl.gbase = ((uint64_t)sv[c].y << 32) | sv[c].x;
      sl.coff = cf;
      sl.pack = sv[c].w;
      const uint32_t rk = rank0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(bl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bl, 0u));
      if (live) w.u.s.tbl[rk] = sl;
      rank0 += (uint32_t)__popcll(bl);
      const uint32_t d = cf - (uint32_t)c0;  // (a start inside the tile: 0 < d < nc)
      const bool in = live & (cf > (uint32_t)c0) & (d < nc);
      if (in) w.u.s.st[d] = 1;
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t nval = reg ? nc : 0u;
    uint32_t cs = 0;
    vm = 0;
#pragma unroll
    for (int q = 0; q < kFlQ; ++q) {
      const uint32_t cl = 64 * q + lane;
      const uint64_t sb = __builtin_amdgcn_ballot_w64(w.u.s.st[cl] != 0);
      const uint32_t k = cs + __builtin_amdgcn_mbcnt_hi((uint32_t)(sb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sb, 0u)) +
                         (uint32_t)((sb >> lane) & 1u);
      cs += (uint32_t)__popcll(sb);
      const FlSlot sl = w.u.s.tbl[k];
      const uint64_t c = c0 + cl;
      const bool ok = cl < nval;
      const uint32_t cc = (uint32_t)c - sl.coff, n = sl.pack >> 4;
      const uint32_t from = cc == 0 ? (sl.pack & 3u) : 0u, to = cc + 1 == n ? ((sl.pack >> 2) & 3u) + 1u : 4u;
      const uint32_t m4 = ok ? ((0xFu << from) & (0xFu >> (4u - to))) : 0u;
      vm |= m4 << (4 * q);
      const uint4 v = acol4[ok ? min(sl.gbase + c, gmax) : 0];
      x[4 * q] = v.x;
      x[4 * q + 1] = v.y;
      x[4 * q + 2] = v.z;
      x[4 * q + 3] = v.w;
    }
  };
  // stage d: the filter words of the valid non-hub entries (one buffer load per entry index of the lane;
  // the other lanes' offsets are dropped: no cache line touched)
  auto probe = [&](const uint32_t (&x)[kFlE], uint32_t vm, uint32_t (&fw)[kFlE]) {
#pragma unroll
    for (int e = 0; e < kFlE; ++e) {
      const bool p = ((vm >> e) & 1u) && x[e] < a.vb;
      fw[e] = __builtin_amdgcn_raw_buffer_load_b32(fr, p ? (x[e] >> 3) & ~3u : kFlDrop, 0, 0);
    }
  };
  // stage e: the tile's survivors staged in entry order and stored to its scratch slot, its count, and
  // the offsets of the sources starting inside it
  auto consume = [&](uint64_t i, const uint32_t (&x)[kFlE], uint32_t vm, const uint32_t (&fw)[kFlE], int r) {
    const uint64_t t = tile(i), c0 = t * kFlChunks;
    // (read off the LDS into SGPRs: a buffer descriptor built from a VGPR value becomes a waterfall loop)
    FlHdr h;
    h.s0 = wave_bcast64(w.hdr[r].s0);
    h.ns = wave_bcast64(w.hdr[r].ns);
    const bool deferred = h.ns > (uint64_t)kFlSlots;
    // an entry's bit (a hub's from the LDS; vb is a multiple of 64: its bit index is x mod 32 too), kept
    // where the entry is valid
    uint32_t sv = 0;
#pragma unroll
    for (int e = 0; e < kFlE; ++e) {
      const bool hub = x[e] >= a.vb;
      const uint32_t lw = s_hub[hub && ((vm >> e) & 1u) ? (x[e] - a.vb) >> 5 : 0u];
      sv |= (((hub ? lw : fw[e]) >> (x[e] & 31)) & 1u) << e;
    }
    sv &= vm;
    // staging in entry order: row q of chunks (chunk 64q + lane) after rows < q; inside a row, the survivors
    // of lower lanes (per component, a ballot) and of this chunk's earlier components
    uint32_t qb = 0;
#pragma unroll
    for (int q = 0; q < kFlQ; ++q) {
      const uint32_t sq = (sv >> (4 * q)) & 0xFu;
      uint32_t before = 0, tq = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint64_t b = __builtin_amdgcn_ballot_w64((sq >> c) & 1u);
        before += __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        tq += (uint32_t)__popcll(b);
      }
      w.qs[q][lane] = (uint16_t)(qb + before);
      uint32_t o = qb + before;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t b = (sq >> c) & 1u;
        if (b) w.u.surv[o] = x[4 * q + c];
        o += b;
      }
      qb += tq;
    }
    __builtin_amdgcn_wave_barrier();
    // 16-byte stores of the staged survivors, rounded up to whole 16 bytes (the slot has room)
    const uint32_t tot = deferred ? 0u : qb;
    const __amdgpu_buffer_rsrc_t sr =
        __builtin_amdgcn_make_buffer_rsrc(a.scratch + t * (uint64_t)(kFlChunks * 4), 0, (int32_t)(((tot + 3) & ~3u) * 4), 0x00020000);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(w.u.surv);
#pragma unroll
    for (int q = 0; q < kFlQ; ++q) {
      const uint32_t k = 64 * q + lane;
      if (q > 0 && tot <= 256u * q) break;  // (uniform: no store instruction for an empty row of lanes)
      const uint4 v = s4[k];
      u32x4 vv;
      vv.x = v.x;
      vv.y = v.y;
      vv.z = v.z;
      vv.w = v.w;
      __builtin_amdgcn_raw_buffer_store_b128(vv, sr, 4 * k < tot ? 16 * k : kFlDrop, 0, 0);
    }
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(a.ntot + t, 0, 4, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(deferred ? kFlDeferred : qb, cr, lane == 0 ? 0u : kFlDrop, 0, 0);
    // sources whose first chunk lies strictly inside the tile: survivors of the tile before it
    const __amdgpu_buffer_rsrc_t lr = __builtin_amdgcn_make_buffer_rsrc(a.loc + h.s0, 0, 4 * kFlSlots, 0x00020000);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const uint32_t k = 64 * c + lane;
      if (c > 0 && h.ns <= 64) break;  // (uniform)
      const uint32_t cf = w.coff[r][k], d = cf - (uint32_t)c0;
      const bool in = !deferred & (k < h.ns) & (cf > (uint32_t)c0) & (d < (uint32_t)kFlChunks);
      const uint32_t cl = in ? d : 0u;
      const uint32_t v = w.qs[cl >> 6][cl & 63];
      __builtin_amdgcn_raw_buffer_store_b32(v, lr, in ? 4 * k : kFlDrop, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();  // the staging area is the next setup's table
  };
  // prologue: tiles 0 and 1 set up, tile 0 probed, tile 2's sources and tile 3's bounds loaded; drained
  uint64_t P0, P1;
  uint4 S0[2], S1[2];
  FlHdr H0, H1;
  uint32_t X0[kFlE], X1[kFlE], X2[kFlE], V0, V1, V2;
  uint32_t F0[kFlE], F1[kFlE];
  {
    uint4 sv[2];
    FlHdr hv;
    ld_src(ld_bounds(0), sv, hv);
    setup(0, sv, hv, 0, X0, V0);
    probe(X0, V0, F0);
    ld_src(ld_bounds(1), sv, hv);
    setup(1, sv, hv, 1, X1, V1);
    ld_src(ld_bounds(2), S0, H0);
    P0 = ld_bounds(3);
    __builtin_amdgcn_s_waitcnt(0);
  }
  // step i: a) tile i+4's bounds; b) tile i+3's sources; c) tile i+2 set up, its chunks requested;
  // d) tile i+1 probed; e) tile i consumed. The register sets rotate over six unrolled steps (three
  // chunk sets, two of everything else), so no set is copied while its loads are in flight.
#define OMX_FL_STEP(PA, PB, SA, HA, SB, HB, XA, VA, XB, VB, XC, VC, FA, FB, RE, RC) \
  {                                                                                \
    PB = ld_bounds(i + 4);                                                         \
    ld_src(PA, SB, HB);                                                            \
    setup(i + 2, SA, HA, RC, XC, VC);                                              \
    probe(XB, VB, FB);                                                             \
    consume(i, XA, VA, FA, RE);                                                    \
  }
  for (uint64_t i = 0;;) {
    OMX_FL_STEP(P0, P1, S0, H0, S1, H1, X0, V0, X1, V1, X2, V2, F0, F1, 0, 2)
    if (++i >= ntw) break;
    OMX_FL_STEP(P1, P0, S1, H1, S0, H0, X1, V1, X2, V2, X0, V0, F1, F0, 1, 0)
    if (++i >= ntw) break;
    OMX_FL_STEP(P0, P1, S0, H0, S1, H1, X2, V2, X0, V0, X1, V1, F0, F1, 2, 1)
    if (++i >= ntw) break;
    OMX_FL_STEP(P1, P0, S1, H1, S0, H0, X0, V0, X1, V1, X2, V2, F1, F0, 0, 2)
    if (++i >= ntw) break;
    OMX_FL_STEP(P0, P1, S0, H0, S1, H1, X1, V1, X2, V2, X0, V0, F0, F1, 1, 0)
    if (++i >= ntw) break;
    OMX_FL_STEP(P1, P0, S1, H1, S0, H0, X2, V2, X0, V0, X1, V1, F1, F0, 2, 1)
    if (++i >= ntw) break;
  }
#undef OMX_FL_STEP
}

__device__ __forceinline__ uint32_t wave_excl_add(uint32_t v, uint32_t lane, uint32_t *total) {
  uint32_t incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += y;
  }
  *total = __builtin_amdgcn_readlane(incl, 63);
  return incl - v;
}

// the deferred tiles (over more than kFlSlots sources): one wave per tile, every chunk's source by a binary search; the same outputs as k_flist
__global__ __launch_bounds__(256) void k_flist_wide(FlistArgs a) {
  __shared__ uint32_t s_q[4][kFlChunks + 1];  // survivors before every chunk of the tile
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t EC = *a.ec;
  const uint64_t nt = (EC + kFlChunks - 1) / kFlChunks;
  // (a wave takes 64 consecutive tiles' counts at once and walks the deferred ones: one round trip per
  // 64 tiles, not per tile — a scan one tile at a time took 36 µs at M1, which defers none)
  for (uint64_t g0 = ((uint64_t)blockIdx.x * 4 + wv) * 64; g0 < nt; g0 += (uint64_t)gridDim.x * 4 * 64) {
   const uint64_t tl = g0 + lane;
   uint64_t dm = __builtin_amdgcn_ballot_w64(tl < nt && a.ntot[tl < nt ? tl : 0] == kFlDeferred);
   for (; dm; dm &= dm - 1) {
    const uint64_t t = g0 + __builtin_ctzll(dm);
    const uint64_t s0 = a.rb[2 * t], s1 = a.rb[2 * t + 1], c0 = t * kFlChunks;
    const uint32_t nc = (uint32_t)min<uint64_t>((uint64_t)kFlChunks, EC - c0);
    uint32_t qb = 0;
    for (uint32_t q = 0; q < kFlQ; ++q) {
      const uint32_t cl = 64 * q + lane;
      uint32_t sq = 0;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (cl < nc) {
        // the source of chunk c0 + cl: the last with coff ≤ c (its chunk table entry holds coff)
        uint64_t lo = s0, hi = s1;
        while (lo < hi) {
          const uint64_t mid = (lo + hi + 1) >> 1;
          if ((uint64_t)a.info[mid].z <= c0 + cl) lo = mid;
          else hi = mid - 1;
        }
        const uint4 in = a.info[lo];
        const uint64_t gb = ((uint64_t)in.y << 32) | in.x;
        const uint32_t cc = (uint32_t)(c0 + cl - in.z), n = in.w >> 4;
        const uint32_t from = cc == 0 ? (in.w & 3u) : 0u, to = cc + 1 == n ? ((in.w >> 2) & 3u) + 1u : 4u;
        v = reinterpret_cast<const uint4 *>(a.acol)[gb + c0 + cl];
        const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
        for (uint32_t c = from; c < to; ++c) {
          const uint32_t x = xs[c];
          if ((a.bits[x >> 5] >> (x & 31)) & 1u) sq |= 1u << c;
        }
      }
      uint32_t tq;
      const uint32_t ex = wave_excl_add((uint32_t)__builtin_popcount(sq), lane, &tq);
      s_q[wv][cl] = qb + ex;
      uint32_t o = qb + ex;
      const uint32_t xs[4] = {v.x, v.y, v.z, v.w};
      for (int c = 0; c < 4; ++c)
        if ((sq >> c) & 1u) a.scratch[t * (uint64_t)(kFlChunks * 4) + o++] = xs[c];
      qb += tq;
    }
    if (lane == 0) s_q[wv][kFlChunks] = qb;
    __builtin_amdgcn_wave_barrier();
    for (uint64_t k = lane; k < s1 - s0 + 1; k += 64) {
      const uint64_t cf = a.info[s0 + k].z;
      if (cf > c0 && cf < c0 + kFlChunks) a.loc[s0 + k] = s_q[wv][cf - c0];
    }
    if (lane == 0) a.ntot[t] = qb;
    __builtin_amdgcn_wave_barrier();
   }
  }
}

// the survivors of every tile moved to its base in lcol, hub ranks mapped back to vertices: a wave takes
// kFlCopyT consecutive tiles at once (their first 64 survivors each: every load of the batch in flight
// together), then any longer tile's rest
constexpr int kFlCopyT = 8;
__global__ __launch_bounds__(256) void k_flist_copy(FlistArgs a, const uint64_t *base) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nt = (*a.ec + kFlChunks - 1) / kFlChunks;
  const uint64_t t0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * kFlCopyT;
  if (t0 >= nt) return;
  const uint64_t tl = t0 + (lane & (kFlCopyT - 1));
  const uint32_t nl = tl < nt ? a.ntot[tl] : 0u;
  const uint64_t bl = base[tl < nt ? tl : nt - 1];
  uint32_t n[kFlCopyT], x[kFlCopyT];
  uint64_t b[kFlCopyT];
#pragma unroll
  for (int j = 0; j < kFlCopyT; ++j) {
    n[j] = __builtin_amdgcn_readlane(nl, j);
    b[j] = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(bl >> 32), j) << 32) | __builtin_amdgcn_readlane((uint32_t)bl, j);
  }
  // rounds of 64 entries of every tile at once (a tile of a hub's row holds up to 512 survivors: one
  // tile at a time, its rounds were a chain of dependent round trips)
  uint32_t nmax = 0;
#pragma unroll
  for (int j = 0; j < kFlCopyT; ++j) nmax = max(nmax, n[j]);
  for (uint32_t k0 = 0; k0 < nmax; k0 += 64) {
    const uint32_t k = k0 + lane;
#pragma unroll
    for (int j = 0; j < kFlCopyT; ++j)  // (n = 0 past the end: entry 0 of the last tile, never stored)
      x[j] = a.scratch[min(t0 + j, nt - 1) * (uint64_t)(kFlChunks * 4) + (k < n[j] ? k : 0u)];
#pragma unroll
    for (int j = 0; j < kFlCopyT; ++j) {  // (an unused lane's word may be a stale scratch word: never an index)
      const bool hub = k < n[j] && x[j] >= a.vb && x[j] - a.vb < a.nh;
      const uint32_t v = a.hubs[hub ? x[j] - a.vb : 0u];
      x[j] = hub ? v : x[j];
    }
#pragma unroll
    for (int j = 0; j < kFlCopyT; ++j)
      if (k < n[j]) a.lcol[b[j] + k] = x[j];
  }
}

// every list offset: a source whose first chunk opens a tile (or lies at the end) starts at that tile's
// base, any other at its tile's base + its offset inside the tile (k_flist); loff[U] = the total
__global__ void k_flist_loff(const uint64_t *coff, uint64_t U, const uint64_t *ec, const uint64_t *base, const uint32_t *loc,
                             uint64_t *loff) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s > U) return;
  const uint64_t EC = *ec, nt = (EC + kFlChunks - 1) / kFlChunks;
  const uint64_t c = s == U ? EC : coff[s];
  if (c >= EC) loff[s] = base[nt];
  else if (c % kFlChunks == 0) loff[s] = base[c / kFlChunks];
  else loff[s] = base[c / kFlChunks] + loc[s];
}

}  // namespace

// an upper bound of the chunk space's tiles: Σ ⌈(deg + 3) / 4⌉ + 1 chunks per source
uint64_t flist_tiles_bound(uint64_t EU, uint64_t U) { return (EU / 4 + 2 * U + kFlChunks) / kFlChunks + 1; }
uint64_t flist_tile_entries() { return 4ull * kFlChunks; }

void launch_flist_nch(const uint32_t *ub, const uint64_t *doff, uint64_t U, const uint64_t *rp, uint32_t *nch,
                      hipStream_t s) {
  if (!U) return;
  hipLaunchKernelGGL(k_flist_nch, dim3(nblocks(U + 1, 256)), dim3(256), 0, s, ub, doff, U, rp, nch);
  KCHECK("k_flist_nch");
}

void launch_flist_prep(const uint32_t *ub, const uint64_t *doff, const uint64_t *coff, uint64_t U, const uint64_t *rp,
                       const uint64_t *ec, uint4 *info, uint64_t *rb, uint32_t *ntot, uint64_t nt_bound, hipStream_t s) {
  if (!U) return;
  if (info) {  // (nullptr: the chunk table came with the sources, launch_srcrows)
    hipLaunchKernelGGL(k_flist_info, dim3(nblocks(U, 256)), dim3(256), 0, s, ub, doff, coff, U, rp, info);
    KCHECK("k_flist_info");
  }
  hipLaunchKernelGGL(k_flist_bounds, dim3(nblocks(nt_bound + 1, 256)), dim3(256), 0, s, coff, U, ec, rb, ntot, nt_bound);
  KCHECK("k_flist_bounds");
}

void launch_probe_bits(const uint32_t *hubs, uint32_t nh, const uint64_t *filter, uint32_t vb, uint32_t *bits,
                       hipStream_t s) {
  const uint64_t n = ((vb / 32 + 63) & ~63ull) + ((nh + 63) & ~63ull);
  hipLaunchKernelGGL(k_probe_bits, dim3(nblocks(n, 256)), dim3(256), 0, s, hubs, nh, filter, vb, bits);
  KCHECK("k_probe_bits");
}

void launch_list_col(uint32_t *col, uint64_t E, uint32_t vb, hipStream_t s) {
  hipLaunchKernelGGL(k_list_col, dim3(nblocks(E + 4, 256)), dim3(256), 0, s, col, E, vb);
  KCHECK("k_list_col");
}

void launch_flist(const FlistArgs &a, uint64_t nt_bound, int cus, hipStream_t s) {
  if (a.nh > kFlistHubs) fail(OMX_E_INVALID, "internal: more hubs than the lists col holds");
  // grids sized for the bound; waves past the real tile count exit at once
  const dim3 grid((unsigned)std::min<uint64_t>((nt_bound + kFlWaves - 1) / kFlWaves, (uint64_t)cus)), blk(64 * kFlWaves);
  hipLaunchKernelGGL(k_flist, grid, blk, 0, s, a);
  KCHECK("k_flist");
  const dim3 gw((unsigned)std::min<uint64_t>((nt_bound + 255) / 256, (uint64_t)cus * 4)), bw(256);
  hipLaunchKernelGGL(k_flist_wide, gw, bw, 0, s, a);
  KCHECK("k_flist_wide");
}

void launch_flist_finish(const FlistArgs &a, const uint64_t *coff, const uint64_t *base, uint64_t *loff, uint64_t nt_bound,
                         int cus, hipStream_t s) {
  hipLaunchKernelGGL(k_flist_copy, dim3((unsigned)((nt_bound + 4 * kFlCopyT - 1) / (4 * kFlCopyT))), dim3(256), 0, s, a,
                     base);
  KCHECK("k_flist_copy");
  hipLaunchKernelGGL(k_flist_loff, dim3(nblocks(a.U + 1, 256)), dim3(256), 0, s, coff, a.U, a.ec, base, a.loc, loff);
  KCHECK("k_flist_loff");
}

// ---- the factorized hop's prologues in three launches each (round 6) ---------------------------------
// Both walk the hop's R rows (sorted by source) in tiles of kPtT rows, 8 consecutive rows a thread: a
// count pass writes per-tile totals, one workgroup scans them and posts the hop's totals to the host
// mailbox, a fill pass writes the per-row / per-source arrays at the scanned offsets. They replace chains
// of ~10-12 small kernels (run heads, flagged selects, scans, degree gathers, reduces: each a launch, most
// of them rocPRIM's lookback-state init + scan pair), which at M1 cost more in launch gaps than in work.
constexpr int kPtB = 256, kPtI = 8, kPtT = kPtB * kPtI;

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}
// block-wide exclusive scan of one u64 per thread (kPtB threads); *total = the block's sum
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t x, uint64_t *s_w, uint64_t *total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += y;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  uint64_t woff = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kPtB / 64; ++w) {
    const uint64_t t = s_w[w];
    woff += w < (int)wave ? t : 0;
    tot += t;
  }
  __syncthreads();  // (s_w is reused by the next scan)
  *total = tot;
  return woff + incl - x;
}

// (a) the sorted rows' sources. ss[R]: the rows' source vertices, ascending. Per tile: the run heads (a
// distinct source starts), Σ deg over the heads (EU), Σ deg over the rows (E_t).
// a thread's 8 consecutive rows (i0 a multiple of 8: two aligned 16-byte loads when all are in range)
__device__ __forceinline__ void load8(const uint32_t *a, uint64_t i0, uint64_t R, uint32_t (&v)[kPtI]) {
  if (i0 + kPtI <= R) {
    const uint4 x = *reinterpret_cast<const uint4 *>(a + i0), y = *reinterpret_cast<const uint4 *>(a + i0 + 4);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w; v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  } else {
#pragma unroll
    for (int k = 0; k < kPtI; ++k) v[k] = i0 + k < R ? a[i0 + k] : 0u;
  }
}

// CH (a one-part adjacency, the lists pass's input): also Σ over the heads of their row's 4-entry chunks
// (k_flist's chunk space), so the fill writes the sources' chunk offsets and chunk table entries too
template <bool CH>
__global__ __launch_bounds__(kPtB) void k_srcrows_count(const uint32_t *ss, uint64_t R, DAdj adj, uint64_t *tt) {
  constexpr int K = CH ? 4 : 3;
  __shared__ uint64_t s_w[K][kPtB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kPtT + (uint64_t)threadIdx.x * kPtI;
  uint32_t v[kPtI];
  load8(ss, i0, R, v);
  const uint32_t prev0 = (i0 > 0 && i0 <= R) ? ss[i0 - 1] : 0u;
  // the degree of every run's first row in the thread (a head, or the thread's first row): independent
  // loads, issued together
  uint64_t dg[kPtI], rs[kPtI];
  uint64_t h = 0;
#pragma unroll
  for (int k = 0; k < kPtI; ++k) {
    const uint64_t i = i0 + k;
    const uint32_t pv = k ? v[k - 1] : prev0;
    const bool head = i < R && (i == 0 || v[k] != pv);
    h += head;
    const bool need = i < R && (head || k == 0);
    if (CH) {
      rs[k] = need ? adj.p[0].rp[v[k]] : 0;
      dg[k] = need ? adj.p[0].rp[v[k] + 1] - rs[k] : UINT64_MAX;
    } else {
      dg[k] = need ? adj_degree(adj, v[k]) : UINT64_MAX;
    }
  }
  uint64_t eu = 0, et = 0, d = 0, ec = 0;
#pragma unroll
  for (int k = 0; k < kPtI; ++k) {
    const uint64_t i = i0 + k;
    if (i >= R) break;
    const uint32_t pv = k ? v[k - 1] : prev0;
    const bool head = i == 0 || v[k] != pv;
    if (dg[k] != UINT64_MAX) d = dg[k];
    eu += head ? d : 0;
    et += d;
    if (CH && head) ec += fl_nch(rs[k], d);
  }
  uint64_t x[4] = {h, eu, et, ec};
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    x[j] = wave_sum_u64(x[j]);
    if (lane == 0) s_w[j][wave] = x[j];
  }
  __syncthreads();
  if (threadIdx.x < K) {
    uint64_t t = 0;
    for (int w = 0; w < kPtB / 64; ++w) t += s_w[threadIdx.x][w];
    tt[K * (uint64_t)blockIdx.x + threadIdx.x] = t;
  }
}

// one workgroup: exclusive scans of the tiles' K counters (in place), the totals to tot[0..K) and the
// mailbox (words in the order `order` lists them)
// (extra: one more word appended to the mail, e.g. a count another kernel left on the device)
constexpr int kScanB = kPtB, kScanI = 4;  // a thread scans 4 consecutive tiles a round
template <int K>
__global__ __launch_bounds__(kScanB) void k_tiles_scan(uint64_t *tt, uint64_t nt, uint64_t *tot, Mail mail, int4 order,
                                                        const uint64_t *extra) {
  __shared__ uint64_t s_w[kScanB / 64];
  uint64_t carry[K];
#pragma unroll
  for (int j = 0; j < K; ++j) carry[j] = 0;
  for (uint64_t t0 = 0; t0 < nt; t0 += (uint64_t)kScanB * kScanI) {
    const uint64_t tb = t0 + (uint64_t)threadIdx.x * kScanI;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      uint64_t x[kScanI], sum = 0;
#pragma unroll
      for (int q = 0; q < kScanI; ++q) {
        x[q] = tb + q < nt ? tt[K * (tb + q) + j] : 0;
        sum += x[q];
      }
      uint64_t total;
      uint64_t ex = carry[j] + block_excl_scan_u64(sum, s_w, &total);
#pragma unroll
      for (int q = 0; q < kScanI; ++q) {
        if (tb + q < nt) tt[K * (tb + q) + j] = ex;
        ex += x[q];
      }
      carry[j] += total;
    }
  }
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) tot[j] = carry[j];
    const int ord[4] = {order.x, order.y, order.z, order.w};
    const int nm = K < 3 ? K : 3;  // (a fourth counter is not posted)
#pragma unroll
    for (int j = 0; j < nm; ++j) {
      uint64_t w = 0;  // carry[ord[j]] with static indices (a dynamic one would put carry in scratch)
#pragma unroll
      for (int q = 0; q < K; ++q) w = ord[j] == q ? carry[q] : w;
      mail.p[j] = w;
    }
    if (extra) mail.p[nm] = *extra;
    mail_post(mail);
  }
}

// CH: coff[u] = the chunks of the sources before u (coff[U] = all), info[u] = k_flist's chunk table entry
template <bool CH>
__global__ __launch_bounds__(kPtB) void k_srcrows_fill(const uint32_t *ss, uint64_t R, DAdj adj, const uint64_t *tt,
                                                        const uint64_t *tot, uint32_t *ub, uint32_t *g, uint64_t *doff,
                                                        uint64_t *coff, uint4 *info) {
  constexpr int K = CH ? 4 : 3;
  __shared__ uint64_t s_w[kPtB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kPtT + (uint64_t)threadIdx.x * kPtI;
  uint32_t v[kPtI];
  load8(ss, i0, R, v);
  const uint32_t prev0 = (i0 > 0 && i0 <= R) ? ss[i0 - 1] : 0u;
  uint64_t dg[kPtI], rs[kPtI];
  uint32_t hm = 0;  // head bits
  uint64_t h = 0, eu = 0, ec = 0;
#pragma unroll
  for (int k = 0; k < kPtI; ++k) {
    const uint64_t i = i0 + k;
    const uint32_t pv = k ? v[k - 1] : prev0;
    const bool head = i < R && (i == 0 || v[k] != pv);
    if (CH) {
      rs[k] = head ? adj.p[0].rp[v[k]] : 0;
      dg[k] = head ? adj.p[0].rp[v[k] + 1] - rs[k] : 0;
    } else {
      dg[k] = head ? adj_degree(adj, v[k]) : 0;
    }
    hm |= head ? 1u << k : 0u;
    h += head;
  }
#pragma unroll
  for (int k = 0; k < kPtI; ++k) {
    eu += dg[k];
    if (CH && ((hm >> k) & 1u)) ec += fl_nch(rs[k], dg[k]);
  }
  const uint64_t *tb = tt + K * (uint64_t)blockIdx.x;
  uint64_t th, te, tc;
  uint64_t hb = block_excl_scan_u64(h, s_w, &th) + tb[0];
  uint64_t eb = block_excl_scan_u64(eu, s_w, &te) + tb[1];
  uint64_t cb = CH ? block_excl_scan_u64(ec, s_w, &tc) + tb[3] : 0;
  // the run a thread's first row continues (when it is not a head) is the last one before: index hb − 1
  uint64_t u = hb - 1;
  uint32_t gv[kPtI];
#pragma unroll
  for (int k = 0; k < kPtI; ++k) {
    if ((hm >> k) & 1u) {
      u = hb++;
      ub[u] = v[k];
      doff[u] = eb;
      eb += dg[k];
      if (CH) {
        const uint32_t n = fl_nch(rs[k], dg[k]);
        const uint64_t gb = (rs[k] >> 2) - cb;
        const uint32_t pack = (uint32_t)(rs[k] & 3) | (dg[k] ? (uint32_t)((rs[k] + dg[k] - 1) & 3) << 2 : 0u) | (n << 4);
        coff[u] = cb;
        info[u] = make_uint4((uint32_t)gb, (uint32_t)(gb >> 32), (uint32_t)cb, pack);
        cb += n;
      }
    }
    gv[k] = (uint32_t)u;
  }
  if (i0 + kPtI <= R) {
    *reinterpret_cast<uint4 *>(g + i0) = make_uint4(gv[0], gv[1], gv[2], gv[3]);
    *reinterpret_cast<uint4 *>(g + i0 + 4) = make_uint4(gv[4], gv[5], gv[6], gv[7]);
  } else {
#pragma unroll
    for (int k = 0; k < kPtI; ++k)
      if (i0 + k < R) g[i0 + k] = gv[k];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    doff[tot[0]] = tot[1];
    if (CH) coff[tot[0]] = tot[3];
  }
}

// (b) the emission's rows: row r (sorted by source) writes |L(g[r])| output rows; the non-empty rows,
// compacted (their source index, carried values through perm, first output row and list base)
// (b uses tiles of kErT rows, 4 a thread: its fill stages a tile's compacted rows in LDS)
constexpr int kErI = 4, kErT = kPtB * kErI;
__global__ __launch_bounds__(kPtB) void k_emitrows_count(const uint32_t *g, uint64_t R, const uint64_t *loff,
                                                          uint64_t *tt) {
  __shared__ uint64_t s_w[2][kPtB / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * kErT + (uint64_t)threadIdx.x * kErI;
  uint32_t uu[kErI];
  if (i0 + kErI <= R) {
    const uint4 x = *reinterpret_cast<const uint4 *>(g + i0);
    uu[0] = x.x; uu[1] = x.y; uu[2] = x.z; uu[3] = x.w;
  } else {
#pragma unroll
    for (int k = 0; k < kErI; ++k) uu[k] = i0 + k < R ? g[i0 + k] : 0u;
  }
  uint64_t ln[kErI];
#pragma unroll
  for (int k = 0; k < kErI; ++k) ln[k] = i0 + k < R ? loff[uu[k] + 1] - loff[uu[k]] : 0;  // (independent loads)
  uint64_t c = 0, n = 0;
#pragma unroll
  for (int k = 0; k < kErI; ++k) {
    c += ln[k] != 0;
    n += ln[k];
  }
  c = wave_sum_u64(c);
  n = wave_sum_u64(n);
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    s_w[0][wave] = c;
    s_w[1][wave] = n;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint64_t t = 0;
    for (int w = 0; w < kPtB / 64; ++w) t += s_w[threadIdx.x][w];
    tt[2 * (uint64_t)blockIdx.x + threadIdx.x] = t;
  }
}

// tot = {Rn, N}: gs[j], out[c][j] = in[c][perm[r]], roff[j] (roff[Rn] = N), rbase[j] = loff[g[r]] − roff[j].
// A tile's non-empty rows are compacted into LDS, then written as block-wide runs (a thread writing its own
// rows' consecutive slots scattered every store over the wave: 158 against ≈30 µs at M1)
__global__ __launch_bounds__(kPtB) void k_emitrows_fill(FemitRows a, const uint64_t *tt, const uint64_t *tot) {
  __shared__ uint64_t s_w[kPtB / 64];
  __shared__ uint32_t s_gs[kErT];
  __shared__ uint64_t s_ro[kErT], s_lo[kErT];
  __shared__ uint32_t s_cv[kFemitCols][kErT];
  const uint64_t i0 = (uint64_t)blockIdx.x * kErT + (uint64_t)threadIdx.x * kErI;
  uint32_t uu[kErI];
  if (i0 + kErI <= a.R) {
    const uint4 x = *reinterpret_cast<const uint4 *>(a.g + i0);
    uu[0] = x.x; uu[1] = x.y; uu[2] = x.z; uu[3] = x.w;
  } else {
#pragma unroll
    for (int k = 0; k < kErI; ++k) uu[k] = i0 + k < a.R ? a.g[i0 + k] : 0u;
  }
  uint64_t ln[kErI], lo[kErI];
  uint64_t c = 0, n = 0;
#pragma unroll
  for (int k = 0; k < kErI; ++k) {
    lo[k] = i0 + k < a.R ? a.loff[uu[k]] : 0;
    ln[k] = i0 + k < a.R ? a.loff[uu[k] + 1] - lo[k] : 0;
  }
#pragma unroll
  for (int k = 0; k < kErI; ++k) {
    c += ln[k] != 0;
    n += ln[k];
  }
  // the carried values of the non-empty rows: every load issued before the LDS writes
  uint32_t cv[kFemitCols][kErI];
  uint32_t pr[kErI];
#pragma unroll
  for (int k = 0; k < kErI; ++k) pr[k] = ln[k] ? a.perm[i0 + k] : 0u;
#pragma unroll
  for (int cc = 0; cc < kFemitCols; ++cc)
#pragma unroll
    for (int k = 0; k < kErI; ++k) cv[cc][k] = (cc < a.nc && ln[k]) ? a.in[cc][pr[k]] : 0u;
  uint64_t tc, tn;
  uint64_t jl = block_excl_scan_u64(c, s_w, &tc);
  uint64_t o = block_excl_scan_u64(n, s_w, &tn) + tt[2 * (uint64_t)blockIdx.x + 1];
#pragma unroll
  for (int k = 0; k < kErI; ++k) {
    if (!ln[k]) continue;
    s_gs[jl] = uu[k];
    s_ro[jl] = o;
    s_lo[jl] = lo[k];
#pragma unroll
    for (int cc = 0; cc < kFemitCols; ++cc)
      if (cc < a.nc) s_cv[cc][jl] = cv[cc][k];
    ++jl;
    o += ln[k];
  }
  __syncthreads();
  const uint64_t jb = tt[2 * (uint64_t)blockIdx.x];
  for (uint32_t t = threadIdx.x; t < (uint32_t)tc; t += kPtB) {
    a.gs[jb + t] = s_gs[t];
    a.roff[jb + t] = s_ro[t];
    a.rbase[jb + t] = s_lo[t] - s_ro[t];
#pragma unroll
    for (int cc = 0; cc < kFemitCols; ++cc)
      if (cc < a.nc) a.out[cc][jb + t] = s_cv[cc][t];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) a.roff[tot[0]] = tot[1];
}

uint64_t prologue_tiles(uint64_t R) { return (R + kPtT - 1) / kPtT; }
uint64_t emitrows_tiles(uint64_t R) { return (R + kErT - 1) / kErT; }

void launch_srcrows(const uint32_t *ss, uint64_t R, const DAdj &adj, uint64_t *tt, uint64_t *tot, uint32_t *ub,
                    uint32_t *g, uint64_t *doff, const Mail &mail, hipStream_t s, uint64_t *coff, uint4 *info) {
  const uint64_t nt = prologue_tiles(R);
  if (!nt) fail(OMX_E_INVALID, "internal: launch_srcrows without rows");
  if (nt > 0xFFFFFFFFull) unsupported("a factorized hop over 2^43 or more rows");
  if (coff && adj.n != 1) fail(OMX_E_INVALID, "internal: the lists' chunk space over several adjacency parts");
  // tiles' counters (heads, EU, E_t[, chunks]) → tot = {U, EU, E_t[, EC]}; mail = {E_t, U, EU}
  if (coff) {
    hipLaunchKernelGGL(k_srcrows_count<true>, dim3((unsigned)nt), dim3(kPtB), 0, s, ss, R, adj, tt);
    KCHECK("k_srcrows_count");
    hipLaunchKernelGGL(k_tiles_scan<4>, dim3(1), dim3(kScanB), 0, s, tt, nt, tot, mail, make_int4(2, 0, 1, 0),
                       (const uint64_t *)nullptr);
    KCHECK("k_tiles_scan");
    hipLaunchKernelGGL(k_srcrows_fill<true>, dim3((unsigned)nt), dim3(kPtB), 0, s, ss, R, adj, tt, tot, ub, g, doff,
                       coff, info);
    KCHECK("k_srcrows_fill");
  } else {
    hipLaunchKernelGGL(k_srcrows_count<false>, dim3((unsigned)nt), dim3(kPtB), 0, s, ss, R, adj, tt);
    KCHECK("k_srcrows_count");
    hipLaunchKernelGGL(k_tiles_scan<3>, dim3(1), dim3(kScanB), 0, s, tt, nt, tot, mail, make_int4(2, 0, 1, 0),
                       (const uint64_t *)nullptr);
    KCHECK("k_tiles_scan");
    hipLaunchKernelGGL(k_srcrows_fill<false>, dim3((unsigned)nt), dim3(kPtB), 0, s, ss, R, adj, tt, tot, ub, g, doff,
                       (uint64_t *)nullptr, (uint4 *)nullptr);
    KCHECK("k_srcrows_fill");
  }
}

void launch_emitrows(const FemitRows &a, uint64_t *tt, uint64_t *tot, const Mail &mail, hipStream_t s,
                     const uint64_t *extra) {
  const uint64_t nt = emitrows_tiles(a.R);
  if (!nt) fail(OMX_E_INVALID, "internal: launch_emitrows without rows");
  if (nt > 0xFFFFFFFFull) unsupported("a factorized emission over 2^43 or more rows");
  if (a.nc < 0 || a.nc > kFemitCols) fail(OMX_E_INVALID, "internal: k_emitrows_fill columns");
  hipLaunchKernelGGL(k_emitrows_count, dim3((unsigned)nt), dim3(kPtB), 0, s, a.g, a.R, a.loff, tt);
  KCHECK("k_emitrows_count");
  // tiles' counters (non-empty rows, output rows) → tot = {Rn, N}; mail = {Rn, N}
  hipLaunchKernelGGL(k_tiles_scan<2>, dim3(1), dim3(kScanB), 0, s, tt, nt, tot, mail, make_int4(0, 1, 0, 0), extra);
  KCHECK("k_tiles_scan");
  hipLaunchKernelGGL(k_emitrows_fill, dim3((unsigned)nt), dim3(kPtB), 0, s, a, tt, tot);
  KCHECK("k_emitrows_fill");
}

uint64_t femit_tiles(uint64_t N) { return (N + kEwTile - 1) / kEwTile; }

// the (list columns, constants) instances of k_femit_w: (1, 0…4) the rows over their sources' lists
bool femit_supported(int nl, int nc) { return nl == 1 && nc <= 4; }

void launch_femit_len(const uint32_t *g, uint64_t R, const uint64_t *loff, uint64_t *len, hipStream_t s,
                      const uint64_t *nd) {
  hipLaunchKernelGGL(k_femit_len, dim3(nblocks(R + 1, 256)), dim3(256), 0, s, g, R, loff, len, nd);
  KCHECK("k_femit_len");
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
