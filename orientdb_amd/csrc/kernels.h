// kernels.h — host-side launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "devtypes.h"

namespace omx {

constexpr int kMaxCols = 16;       // binding-table columns (pattern aliases) a kernel carries
constexpr int kExpandBlock = 256;  // 4 waves
constexpr int kExpandIPT = 8;      // merge-path items per thread
constexpr int kExpandTile = kExpandBlock * kExpandIPT;

// Rows with at least kHeavyDeg neighbours are cut into chunks: one edge-set part of one row, inside
// one kChunk-aligned window of the col[] array (so every lane's dwordx4 load is 16-B aligned).
constexpr uint64_t kHeavyDeg = 1024;
constexpr int kChunk = 1024;                       // edges per chunk = one wave × 16 dword loads per lane
constexpr int kHeavyBlock = 256;                   // 4 independent waves
constexpr int kHeavySlots = kChunk / 64;           // lane l takes edge l of each 64-edge slot

// LDS-sliced heavy expansion (filtered hops): the target bitmap is cut into slices of kSliceBits
// vertices (128 KiB each) and each heavy row's sorted adjacency is cut at the slice boundaries, so a
// chunk's neighbours all probe one slice; one workgroup per CU holds a slice in LDS and pulls that
// slice's chunks in a static round-robin. Bitmap probes become LDS reads instead of L2 requests.
constexpr uint32_t kSliceBits = 1u << 20;
constexpr uint32_t kSliceWords = kSliceBits / 32;  // u32 words per slice
constexpr int kMaxSlices = 16;                     // V ≤ 16·2^20; beyond that the L2-probe kernel is used
constexpr uint64_t kHeavyDegSliced = 256;         // LDS probes make short chunks cheap: a lower cut
constexpr int kStage = 448;                        // staged survivors per wave (16 waves × 1.75 KiB of LDS)
constexpr int kSliceBlock = 1024;                  // 16 waves: one workgroup per CU (LDS-limited)

// per adjacency part: the CSR's slice-cut index (EdgeSet::d_cuts), P−1 offsets per vertex
struct DCuts {
  const uint32_t *c[kMaxAdjParts];
};

struct SliceArgs {
  const uint64_t *qb;            // [P+1] chunk index bounds of each slice
  uint32_t wg0[kMaxSlices + 1];  // workgroups [wg0[q], wg0[q+1]) own slice q
  uint32_t V;
  uint32_t nslices;
  uint32_t shift;  // slice = 2^shift vertices (6 ≤ shift ≤ 20; tests shrink it to cut small graphs)
  // sliced light kernel: the compacted light rows (k_bin_fill LightRows)
  const uint32_t *lrow;
  const uint32_t *lcuts;
  const uint32_t *lcarry[4];  // carried values of the light rows (LightRows::carry), ≤ 4 columns
  uint64_t nl;
};

// a chunk of the sliced kernel: ≤ kChunk edges of one row part inside one bitmap slice (16 B: one
// scalar dwordx4 load)
struct SliceChunk {
  uint64_t lo;    // first col[] index
  uint32_t row;   // binding row
  uint16_t n;     // edges (1…kChunk)
  uint16_t part;  // adjacency part
};
static_assert(sizeof(SliceChunk) == 16, "SliceChunk is one dwordx4");

// host mailbox: Graph::h_mail is fine-grained pinned host memory; a kernel writes its payload words,
// fences at system scope and then writes `seq` into the last word, which the host polls (no copy
// kernel, no stream synchronisation on the small host reads between launches)
constexpr int kMailWords = 64;
constexpr int kMailSeq = kMailWords - 1;
struct Mail {
  uint64_t *p;
  uint64_t seq;
};

struct ChunkDesc {
  uint64_t lo, hi;  // absolute col[] range of the chunk inside part `part` (one kChunk-aligned window)
  uint64_t dense;   // output index of edge lo in the dense (unfiltered) layout
  uint32_t row;
  uint32_t part;
};

struct ExpandArgs {
  const uint32_t *src;      // [R] source vertex of every binding row
  const uint64_t *offs;     // [R+1] exclusive prefix sum of the rows' LIGHT adjacency lengths
  const uint64_t *lbase;    // [R] single-part adjacency: rp[src[r]] (k_bin_fill), so rows need no src load
  const uint64_t *part;     // [ntiles+1] merge-path split: rows consumed before tile t
  uint64_t R, E;            // rows, Σ light adjacency length
  uint64_t ntiles;
  DAdj adj;
  const uint64_t *filter;   // target bitmap (V bits) or nullptr
  int32_t ncarry;
  const uint32_t *carry_in[kMaxCols];
  uint32_t *carry_out[kMaxCols];
  uint32_t *out_dst;        // new column (neighbour)
  uint64_t *mark;           // write = false: V-bit set of the neighbours (a one-column distinct projection)
  // output placement. Dense (no filter): index = dense_base + edge index (light) or
  // ChunkDesc::dense + position in the chunk (heavy). Arena (filter): each worker w of the launch
  // (a block for the light kernel, a wave for the heavy one) appends to [arena_base + w·arena_cap, …)
  // and reports its row count in seg_count[seg_base + w].
  uint64_t dense_base;
  uint64_t arena_base, arena_cap;
  uint32_t *seg_count;
  uint64_t *seg_start;
  uint32_t seg_base;
  // heavy chunks
  const ChunkDesc *chunks;
  const SliceChunk *schunks;  // sliced kernel
  uint64_t nchunks;
  uint32_t chunk_shift;       // unsliced chunks: (1 << chunk_shift)-aligned col windows (8, 9 or 10)
  // fused closing check of a cyclic pattern (sorted-adjacency intersection): neighbour n of row r is
  // kept only if n ∈ N_member(member_src[r]); member_edges accumulates Σ |N_member(member_src[r])| over
  // the (row, n) pairs that reach the check, i.e. the edges the unfused check step traverses.
  // member_filter: the check's own target bitmap, applied after the edges are counted (k_check order).
  const uint32_t *member_src;
  DAdj member_adj;
  const uint64_t *member_filter;
  unsigned long long *member_edges;  // [0] Σ |N_member| of checked pairs, [1] col[] probes of the checks
};

// ---- isect.hip: the fused closing check as a sorted-list intersection (Executor::expand_check_isect) ----
constexpr uint32_t kIsRowCap = 256;   // m + n of a merged row (its two lists staged in a wave's LDS tile)
constexpr uint32_t kIsRowPad = 8;     // a merged row's tile weight beyond m + n (bounds the rows a tile holds)
struct IsectPolicy {
  int32_t merge;     // merge rows of comparable lengths
  int32_t force;     // merge every row with m + n ≤ kIsRowCap (tests)
  int32_t swap;      // probe rows iterate the shorter list (simple adjacencies, no expansion filter)
  int32_t dup_free;  // N_x has no parallel edges: a merged row matches at most min(m, n) times
  double ratio;      // merge when max(m, n) ≤ ratio · min(m, n)
};
struct IsectArgs {
  const uint32_t *idx;       // [nM] the merged rows' binding-table indices
  const uint64_t *pa, *pb;   // [nM] their N_x and N_y list starts (launch_isect_prep)
  const uint32_t *pmn;       // [nM] m | n << 16
  const uint64_t *boff;      // [nM] scan of their output bounds (a tile writes at boff[its first row])
  const uint32_t *tile_row;  // [ntiles + 1] first merged row of each tile
  uint64_t nM, ntiles;
  const uint32_t *xs, *ys;   // binding columns: expansion source x, check source y
  DAdjPart ax, ay;           // N_x (iterated: the new column), N_y (membership)
  const uint64_t *xfilter;   // the expansion's target bitmap, or nullptr
  const uint64_t *yfilter;   // the check's target bitmap, or nullptr
  int32_t ncarry;
  const uint32_t *carry_in[kMaxCols];
  uint32_t *carry_out[kMaxCols];
  uint32_t *out_dst;
  uint32_t *seg_count;       // [ntiles] rows tile t wrote, from seg_start[t]
  uint64_t *seg_start;
  unsigned long long *counters;  // [0] Σ |N_y(y)| over the A elements passing xfilter; [1] rows (count only)
};
// cls[r] ∈ {0 nothing, 1 merge, 2 probe N_y, 3 probe N_x}; w[r] = tile weight, bnd[r] = output bound of a
// merged row (0 otherwise); sums (6 words, zeroed): Σ m, Σ m·n, rows of each class
void launch_isect_class(const uint32_t *xs, const uint32_t *ys, uint64_t R, const DAdjPart &ax, const DAdjPart &ay,
                        const IsectPolicy &pol, uint8_t *cls, uint32_t *w, uint32_t *bnd, unsigned long long *sums,
                        int cus, hipStream_t s);
uint64_t isect_tiles(uint64_t wtotal);
void launch_isect_tiles(const uint64_t *woff, uint64_t nM, uint64_t ntiles, uint32_t *tile_row, hipStream_t s);
void launch_isect_prep(const uint32_t *idx, uint64_t nM, const uint32_t *xs, const uint32_t *ys, const DAdjPart &ax,
                       const DAdjPart &ay, uint64_t *pa, uint64_t *pb, uint32_t *pmn, hipStream_t s);
void launch_isect_merge(const IsectArgs &a, bool write, int cus, hipStream_t s);

// predicate VM → V-bit bitmap (u64 words); depth = value of $depth
// nwords > ⌈V/64⌉ zero-fills the padding words (0: no padding)
void launch_bitmap_keep_range(uint64_t *words, uint64_t nwords, uint64_t lo, uint64_t hi, hipStream_t s);
void launch_eval_bitmap(const DPred &pred, uint32_t V, int64_t depth, uint64_t *words, hipStream_t s,
                        uint64_t nwords = 0);
// two single-comparison predicates over the same int32 / int64 column (no class test), evaluated in one
// pass into their two bitmaps; false (nothing launched) when they are not of that form
bool launch_eval_bitmap_pair(const DPred &a, const DPred &b, uint32_t V, uint64_t *wa, uint64_t *wb, hipStream_t s,
                             uint64_t nwords = 0);
// filter bitmaps (Executor::bitmap) are padded to a multiple of the largest slice, so the sliced
// kernels stage whole slices with unchecked 16-byte loads
constexpr uint64_t kBitmapPadWords = kSliceBits / 64;
void launch_bitmap_and(const uint64_t *a, uint64_t *b, uint64_t nwords, hipStream_t s);
// per-word popcount of the bits v with lo <= v < hi (optionally also v % world == rank)
void launch_word_popc(const uint64_t *words, uint64_t nwords, uint32_t V, int rank, int world, uint32_t lo,
                      uint32_t hi, uint32_t *counts, hipStream_t s);
void launch_word_scatter(const uint64_t *words, uint64_t nwords, uint32_t V, int rank, int world, uint32_t lo,
                         uint32_t hi, const uint32_t *offsets, uint32_t *out, hipStream_t s);
// partitioned execution (dist.h): dest[r] = destination rank of row r, hist[p] += rows to rank p
constexpr int kMaxRanks = 64;
void launch_route_owner(const uint32_t *v, uint64_t R, uint32_t block, uint32_t W, uint32_t *dest, uint64_t *hist,
                        hipStream_t s);
void launch_route_hash(int ncols, const uint32_t *const *cols, uint64_t R, uint32_t W, uint32_t *dest, uint64_t *hist,
                       hipStream_t s);
// dest[r] = p with bounds[p] <= id[r] < bounds[p+1] (host bounds[0..W])
void launch_route_bounds(const uint32_t *id, uint64_t R, const uint64_t *bounds, uint32_t W, uint32_t *dest,
                         uint64_t *hist, hipStream_t s);
void launch_add_u32(uint32_t *x, uint64_t n, int64_t delta, hipStream_t s);

void launch_row_degree(const uint32_t *src, uint64_t R, const DAdj &adj, uint64_t *deg, hipStream_t s);
// deg[v - lo] = degree of row v (u64: a multigraph row may hold 2^32 or more entries)
void launch_row_degree_range(const uint64_t *rp, uint32_t lo, uint32_t hi, uint64_t *deg, hipStream_t s);
void launch_mp_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part,
                         hipStream_t s);
// rows [vlo, vhi) (the owned rows of a partition; rp indexed by global vertex id)
void launch_build_cuts(const uint64_t *rp, const uint32_t *col, uint32_t vlo, uint32_t vhi, uint32_t nslices,
                       uint32_t shift, uint32_t *cuts, hipStream_t s);
// Degree binning of R rows in three launches (rows in tiles of kBinBlock): per tile, the sums of the
// rows' light degrees, heavy degrees, light rows and heavy chunks per slice (blk[k·nb + b]); one
// workgroup scans them (qb[q] = first chunk of slice q, qb[P] = chunks; mail = {Σ light, Σ heavy,
// chunks, light rows NL, qb[0..P]}); then every tile redoes its rows and writes the light offsets,
// the light rows' first col index and the heavy rows' chunks. Unsliced: P = 1, kChunk-aligned
// ChunkDesc windows; sliced: SliceChunk pieces cut at the slice boundaries (cuts).
// LightRows::row == nullptr: loffs[R+1] / lbase[R] indexed by row (merge-path light kernel); else the
// light rows are compacted in order: loffs[NL+1], lbase[NL], row[NL], cuts[(q−1)·NL + i] (the sliced
// light kernel, single-part adjacency).
struct LightRows {
  uint32_t *row;
  uint32_t *cuts;
  uint64_t nl;
  // the light rows' carried values, compacted alongside (carry[c][i] = cin[c][row i]) when ≤ 4 columns
  int nc;
  const uint32_t *cin[4];
  uint32_t *carry[4];
};
constexpr int kBinBlock = 256;
constexpr int kBinKeys = 3;  // keys before the per-slice chunk counts
inline unsigned bin_tiles(uint64_t R) { return (unsigned)((R + 1 + kBinBlock - 1) / kBinBlock); }
// chunk_shift: unsliced chunks are the (1 << chunk_shift)-aligned windows a heavy row touches
void launch_bin_count(bool sliced, const uint32_t *src, uint64_t R, const DAdj &adj, const DCuts &cuts,
                      uint64_t heavy_deg, uint32_t P, uint64_t *blk, hipStream_t s, uint32_t chunk_shift = 10);
// extra[0..nextra) (device words) are posted after the totals: mail[5 + P + i]
// qb: 2·P + 1 + kBinKeys words (the P + 1 chunk bounds, then scratch for the per-key scan's totals)
void launch_bin_scan(uint64_t *blk, uint64_t R, uint32_t P, uint64_t *qb, const Mail &mail, hipStream_t s,
                     const unsigned long long *extra = nullptr, uint32_t nextra = 0);
// out[q] = set bits of slice q (2^shift vertices) of a V-bit bitmap, q < P
void launch_slice_popc(const uint64_t *bm, uint32_t V, uint32_t shift, uint32_t P, unsigned long long *out,
                       hipStream_t s);
void launch_bin_fill(bool sliced, const uint32_t *src, uint64_t R, const DAdj &adj, const DCuts &cuts,
                     uint64_t heavy_deg, uint32_t P, const uint64_t *blk, const uint64_t *qb, uint64_t *loffs,
                     uint64_t *lbase, const LightRows &lr, ChunkDesc *chunks, SliceChunk *schunks, hipStream_t s,
                     uint32_t chunk_shift = 10);
// grid = sa.wg0[P] workgroups (one per CU); wave w appends to arena_base + w·arena_cap and reports
// seg_count/seg_start[seg_base + w]
void launch_expand_heavy_sliced(const ExpandArgs &a, const SliceArgs &sa, unsigned grid, bool write, hipStream_t s);
// light rows of a sliced single-part hop (ExpandArgs: offs / lbase of the compacted light rows, E = Σ
// light; sa.wg0 over the light grid, sa.lrow / lcuts / nl); wave w appends to arena_base + w·arena_cap, arena_cap ≥
// ⌈E / waves of the smallest slice⌉ + 64·heavy_deg
void launch_expand_light_sliced(const ExpandArgs &a, const SliceArgs &sa, unsigned grid, bool write, hipStream_t s);
// persistent launches: `grid` blocks loop over the tiles / chunks
void launch_expand(const ExpandArgs &a, unsigned grid, bool write, hipStream_t s);
void launch_expand_heavy(const ExpandArgs &a, unsigned grid, bool write, hipStream_t s);
int expand_blocks_per_cu(bool heavy, bool single, bool filter, bool write, bool member = false, uint32_t chunk_shift = 10);
void launch_compact_segments(int ncols, uint32_t *const *in, uint32_t *const *out, const uint64_t *seg_start,
                             const uint32_t *seg_count, const uint64_t *seg_offs, uint32_t nseg, hipStream_t s);

// two launches: the bitmap's vertices in [lo, hi) (and v % world == rank), in order, and their count;
// blk holds bitmap_list_blocks(nwords) words of scratch
unsigned bitmap_list_blocks(uint64_t nwords);
// configs[0] in four launches and one host round trip (kernels.hip k_fof2_a / k_fof2_b + the list):
// roots → hop 1 → hop 2 marked → the marked set's ascending list in out; the mailbox gets {m, E1, E_t, EU}
constexpr uint32_t kFof2Bits = 1u << 18;  // V bound: k_fof2_b stages two V-bit sets in LDS (64 KiB)
struct Fof2Args {
  DAdj a1, a2;            // hop 1 / hop 2 adjacency
  const uint64_t *roots;  // V-bit root set (the rank's share: v % world == rank)
  int32_t rank, world;
  uint64_t *ubm, *bm;     // [W] zeroed: hop 1's targets (hop 2's distinct sources), hop 2's targets
  uint32_t V;
  uint64_t W;             // words of a V-bit set
  uint64_t *acc;          // [3] zeroed: E1, E_t, EU
};
// phase 0: hop 1 (grid workgroups); 1: hop 2; 2: the list (blk: bitmap_list_blocks(W) words) and the mail
void launch_fof2(const Fof2Args &a, int phase, unsigned grid, uint32_t *blk, uint32_t *out, const Mail *mail,
                 hipStream_t s);
void launch_bitmap_list_2k(const uint64_t *words, uint64_t nwords, uint32_t V, int rank, int world, uint32_t lo,
                           uint32_t hi, uint32_t *blk, uint32_t *out, const Mail &count, hipStream_t s);
// one workgroup: soffs = inclusive prefix of cnt (soffs[0] = 0); mail = {soffs[nseg_h], soffs[nseg],
// member[0], member[1], overflow} (member may be nullptr → 0; overflow = some segment below nseg_h
// counted more than cap_h rows, or one above it more than cap_l)
void launch_seg_totals(const uint32_t *cnt, uint64_t nseg, uint64_t nseg_h, uint64_t *soffs,
                       const unsigned long long *member, uint64_t cap_h, uint64_t cap_l, const Mail &mail,
                       hipStream_t s);
// mail[i] = word i at p (words of `bytes` = 4 or 8, zero-extended), i < n < kMailSeq
void launch_post_words(const void *p, int n, const Mail &mail, hipStream_t s, int bytes = 8);
// mail word i = *p[i] (u64 words anywhere on the device, up to 4)
void launch_post_ptrs(const uint64_t *const *p, int n, const Mail &mail, hipStream_t s);

void launch_check(const uint32_t *src, const uint32_t *dst, uint64_t R, const DAdj &adj, const uint64_t *filter,
                  uint8_t *flags, hipStream_t s);
void launch_gather_cols(const uint32_t *idx, uint64_t n, int ncols, const uint32_t *const *in, uint32_t *const *out,
                        hipStream_t s);
void launch_cross(uint64_t R, int ncols, const uint32_t *const *in, uint32_t *const *out, const uint32_t *cand,
                  uint64_t ncand, uint32_t *out_dst, hipStream_t s);
void launch_flag_bitmap(const uint32_t *v, uint64_t n, const uint64_t *bm, uint8_t *flags, hipStream_t s);
void launch_swap_flags(const uint32_t *xs, const uint32_t *ys, uint64_t R, const DAdj &ax, const DAdj &ay,
                       uint8_t *flags, unsigned long long *sums, int cus, hipStream_t s);
void launch_flag_colcmp(const uint32_t *a, const uint32_t *b, uint64_t n, bool eq, uint8_t *flags, hipStream_t s);
void launch_iota(uint32_t *out, uint64_t n, hipStream_t s);
void launch_fill_u32(uint32_t *out, uint64_t n, uint32_t x, hipStream_t s);
// factorized expansion: position of each key in a sorted unique list; a key histogram; a scatter by key
void launch_index_of(const uint32_t *sorted, uint64_t n, const uint32_t *keys, uint64_t m, uint32_t *out, hipStream_t s);
// factor.hip: the factorized hop's rows written over their sources' lists, by tiles of the output space
// Binding row r owns the list entries [loff[g[r]], loff[g[r]+1]) of the list columns: output row o of it
// takes every list column's entry at rbase[r] + o and every constant's value of row r.
constexpr int kFemitCols = 4;   // constants per binding row
constexpr int kFemitLists = 1;  // list columns
struct FemitArgs {
  const uint32_t *g;     // [R] binding row → its list (group) index
  const uint64_t *roff;  // [R+1] first output row of every binding row (scan of its list length)
  const uint64_t *loff;  // [groups+1] list offsets
  const uint64_t *rbase; // [R] loff[g[r]] − roff[r]: list position of output row o of row r is rbase[r] + o
  const uint64_t *rb;    // [2·tiles] first / last binding row of every output tile (launch_femit_bounds)
  uint64_t R, N;         // binding rows (every list non-empty), output rows
  int32_t nl, nc;
  const uint32_t *lcol[kFemitLists];  // list columns …
  uint32_t *lout[kFemitLists];        // … and where each is written
  const uint32_t *cin[kFemitCols];    // constants of every binding row …
  uint32_t *cout[kFemitCols];         // … and where each is written
};
bool femit_supported(int nl, int nc);
uint64_t femit_tiles(uint64_t N);
// len[r] = |L(g[r])| for r < R, len[R] = 0
// nd: a device row count ≤ R (rows past it: length 0, no base); nullptr: all R rows
void launch_femit_len(const uint32_t *g, uint64_t R, const uint64_t *loff, uint64_t *len, hipStream_t s,
                      const uint64_t *nd = nullptr);
// The factorized hop's prologues in three launches each (factor.hip, round 6); tt: 3 (srcrows) or 2
// (emitrows) u64 counters per prologue_tiles(R) tile, tot: 3 / 2 u64 totals.
uint64_t prologue_tiles(uint64_t R);  // launch_srcrows' tiles
uint64_t emitrows_tiles(uint64_t R);  // launch_emitrows' tiles
// ss[R]: the rows' sources, sorted → ub[U] (distinct sources), g[R] (row → source index), doff[U + 1] (scan
// of the sources' degrees); tot = {U, EU, E_t}; mail = {E_t, U, EU}
// coff / info (a one-part adjacency; tt then 4 counters a tile, tot 4): the sources' chunk offsets in
// k_flist's chunk space (coff[U + 1], coff[U] = all chunks) and their chunk table entries
void launch_srcrows(const uint32_t *ss, uint64_t R, const DAdj &adj, uint64_t *tt, uint64_t *tot, uint32_t *ub,
                    uint32_t *g, uint64_t *doff, const Mail &mail, hipStream_t s, uint64_t *coff = nullptr,
                    uint4 *info = nullptr);
// rows r < R grouped by source g[r]: the non-empty ones (|L(g[r])| > 0) compacted to j < Rn: gs[j] = g[r],
// out[c][j] = in[c][perm[r]], roff[j] = their first output row (roff[Rn] = N), rbase[j] = loff[g[r]] − roff[j];
// tot = {Rn, N}; mail = {Rn, N[, *extra]}
struct FemitRows {
  const uint32_t *g, *perm;
  const uint64_t *loff;
  uint64_t R;
  uint32_t *gs;
  uint64_t *roff, *rbase;
  int32_t nc;
  const uint32_t *in[kFemitCols];
  uint32_t *out[kFemitCols];
};
void launch_emitrows(const FemitRows &a, uint64_t *tt, uint64_t *tot, const Mail &mail, hipStream_t s,
                     const uint64_t *extra = nullptr);
// rb[2·femit_tiles(N)]: first / last binding row of every output tile; regular[t] = the tile is full and
// spans at most 64 binding rows (slow_all: none is)
void launch_femit_bounds(const FemitArgs &a, uint64_t *rb, uint8_t *regular, bool slow_all, hipStream_t s);
// a.rb set: tiles[0, *nreg) (the regular ones) through k_femit_w, tiles[*nreg, nt) through k_femit_slow;
// nreg is a device count
void launch_femit(const FemitArgs &a, const uint32_t *tiles, const uint64_t *nreg, uint64_t nt, int cus,
                  hipStream_t s);
// factor.hip (round 5): the filtered lists of a factorized hop's distinct sources in one pass over their
// rows (as aligned 4-entry chunks of the CSR's lists col: a hub — one of the kFlistHubs vertices of
// highest in-degree — as vb + its rank, other vertices as themselves), every entry probing one bit array
// (the filter's words, then the hubs' bits by rank: the hubs' bits stay cache-resident); each tile of the
// chunk space writes its survivors to its own scratch slot with their count, a scan gives every tile its
// base, and a copy moves them to lcol (grouped by source: the tiles are in source order) — CSR loff / lcol.
constexpr uint32_t kFlistHubs = 1u << 20;  // (their bits: 128 KiB of a lists workgroup's LDS)
struct FlistArgs {
  const uint32_t *ub;        // [U] distinct sources
  uint64_t U;
  const uint4 *info;         // [U] per source: {chunk space → col group base (u64), first chunk, pack}
  const uint64_t *ec;        // the chunk space's size (device)
  const uint32_t *acol;      // the CSR's lists col (vb + hub rank, or the vertex), padded to 4
  uint64_t E;                // its entries
  const uint32_t *hubs;      // hub rank → vertex
  uint32_t nh;               // hubs (≤ kFlistHubs)
  uint32_t vb;               // a hub's first id in acol (the filter's words · 64 ≥ V)
  const uint32_t *bits;      // [vb/32 + ⌈nh/32⌉] the target filter's bits, then the hubs' by rank
  uint64_t bbytes;           // its bytes
  const uint64_t *rb;        // [2·tiles] first / last source of every tile
  uint32_t *scratch;         // [tiles · flist_tile_entries()] every tile's survivors
  uint32_t *ntot;            // [tiles] their counts
  uint32_t *loc;             // [U] a source's offset inside its first tile's survivors
  uint32_t *lcol;            // the lists, grouped by source
};
uint64_t flist_tiles_bound(uint64_t EU, uint64_t U);
uint64_t flist_tile_entries();
// nch[i] = chunks of source i's row
void launch_flist_nch(const uint32_t *ub, const uint64_t *doff, uint64_t U, const uint64_t *rp, uint32_t *nch,
                      hipStream_t s);
// info[U] and rb (tile bounds) from coff = the exclusive scan of nch (coff[U] = *ec)
void launch_flist_prep(const uint32_t *ub, const uint64_t *doff, const uint64_t *coff, uint64_t U, const uint64_t *rp,
                       const uint64_t *ec, uint4 *info, uint64_t *rb, uint32_t *ntot, uint64_t nt_bound, hipStream_t s);
// bits = the filter's vb/32 words, then word w bit i = the filter bit of hubs[32w + i]
void launch_probe_bits(const uint32_t *hubs, uint32_t nh, const uint64_t *filter, uint32_t vb, uint32_t *bits,
                       hipStream_t s);
// a hub-annotated col (0x80000000 | rank) as a lists col (vb + rank), its 4 padding entries zeroed
void launch_list_col(uint32_t *col, uint64_t E, uint32_t vb, hipStream_t s);
// the pass (scratch, ntot, loc)
void launch_flist(const FlistArgs &a, uint64_t nt_bound, int cus, hipStream_t s);
// base = exclusive scan of ntot: lcol and loff[U + 1]
void launch_flist_finish(const FlistArgs &a, const uint64_t *coff, const uint64_t *base, uint64_t *loff, uint64_t nt_bound,
                         int cus, hipStream_t s);
void launch_key_hist(const uint32_t *key, uint64_t n, unsigned long long *counts, hipStream_t s);
// the same over a block-segmented table (segment s: entries [seg_start[s], + seg_count[s]))
void launch_key_hist_seg(const uint32_t *key, const uint64_t *seg_start, const uint32_t *seg_count, uint32_t nseg,
                         unsigned long long *counts, hipStream_t s);
void launch_key_scatter_seg(const uint32_t *key, const uint32_t *val, const uint64_t *seg_start, const uint32_t *seg_count,
                            uint32_t nseg, unsigned long long *cursor, uint32_t *out, hipStream_t s);
// 32-bit counters and cursors (fewer than 2^32 entries)
void launch_key_hist_seg(const uint32_t *key, const uint64_t *seg_start, const uint32_t *seg_count, uint32_t nseg,
                         unsigned int *counts, hipStream_t s);
void launch_key_scatter_seg(const uint32_t *key, const uint32_t *val, const uint64_t *seg_start, const uint32_t *seg_count,
                            uint32_t nseg, unsigned int *cursor, uint32_t *out, hipStream_t s);
void launch_key_scatter(const uint32_t *key, const uint32_t *val, uint64_t n, unsigned long long *cursor, uint32_t *out,
                        hipStream_t s);
void launch_pack_pairs(const uint32_t *hi, const uint32_t *lo, uint64_t n, uint64_t *keys, hipStream_t s);
void launch_unpack_pairs(const uint64_t *keys, uint64_t n, uint32_t *hi, uint32_t *lo, hipStream_t s);
void launch_flag_not_in(const uint64_t *sorted, uint64_t nsorted, const uint64_t *keys, uint64_t n, uint8_t *flags,
                        hipStream_t s);
// v ≥ V (a null binding) is skipped
void launch_mark_bitmap(const uint32_t *v, uint64_t n, uint64_t *bm, uint32_t V, hipStream_t s);
// optional targets (exec.hip Executor::expand_step / check_step)
void launch_flag_no_neighbor(const uint32_t *src, uint64_t R, const DAdj &adj, const uint64_t *filter, uint8_t *flags,
                             hipStream_t s);
void launch_check_optional(const uint32_t *src, uint32_t *dst, uint64_t R, const DAdj &adj, const uint64_t *filter,
                           uint32_t V, unsigned int *npe, hipStream_t s);
void launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *out, hipStream_t s);
// out[i] = src[idx[i]] for i < *nd (a device count ≤ cap)
void launch_gather_u32_dev(const uint32_t *src, const uint32_t *idx, const uint64_t *nd, uint64_t cap, uint32_t *out,
                           hipStream_t s);
void launch_scatter_u32(const uint32_t *idx, const uint32_t *val, uint64_t n, uint32_t *out, hipStream_t s);
void launch_flag_row_change(int ncols, const uint32_t *const *cols, uint64_t n, uint8_t *flags, hipStream_t s);
// TRAVERSE: RID lookup of the target records; a level's history / WHILE filter with first-position
// claims (dedup); the accepted records into the history
void launch_find_rids(const uint64_t *rids, uint32_t V, const uint64_t *keys, uint32_t m, uint32_t *out, hipStream_t s);
void launch_trav_filter(const uint32_t *w, uint64_t n, const uint64_t *hist, const uint64_t *pred, uint32_t *first,
                        uint8_t *flags, bool dedup, hipStream_t s);
void launch_trav_accept(const uint32_t *w, uint64_t n, uint64_t *hist, uint32_t *first, hipStream_t s);
void launch_andnot_bitmap(const uint64_t *pred, const uint64_t *hist, uint64_t *out, uint64_t nwords, hipStream_t s);
void launch_post_u32_to_u64(const uint32_t *a, uint64_t *b, hipStream_t s);
// shortestPath: first position meeting the other side's visited set; a level's first discoveries
void launch_sp_meet(const uint32_t *w, uint64_t n, const uint64_t *other, unsigned long long *pos, hipStream_t s);
void launch_sp_accept(const uint64_t *keys, uint64_t n, const uint32_t *queue, uint32_t *parent, uint64_t *visited,
                      uint32_t *first, uint32_t *next, hipStream_t s);
// a null binding (dense id ≥ V: an unmatched optional node) maps to kNullRid
constexpr uint64_t kNullRid = ~0ull;
void launch_map_rids(int ncols, const uint32_t *const *cols, uint64_t n, const uint64_t *rids, uint64_t *out,
                     uint32_t V, hipStream_t s);
// *out += Σ_rows splitmix64-chain(RIDs of the row) (OMX_FLAG_DIGEST; rids == nullptr: dense ids)
void launch_digest(int ncols, const uint32_t *const *cols, uint64_t n, const uint64_t *rids, uint32_t V,
                   unsigned long long *out, int cus, hipStream_t s);
// host evaluation of a predicate program that reads no vertex data (constants and $depth only)
bool eval_pred_const(const DPred &pred, int64_t depth);

// multi-source BFS (bfs.hip): u64 lane mask per vertex, 64 binding rows per batch
void launch_bfs_seed(const uint32_t *src, uint64_t row0, int nl, uint64_t *frontier, hipStream_t s,
                     uint32_t *touched = nullptr, unsigned long long *touched_n = nullptr);
// vertices [vlo, V) (a partition's own rows: vlo = part_lo, V = part_hi; fbm only from vertex 0);
// zero: the next level's mask array — the previous level's frontier array — zeroed where the previous
// level's frontier bits (fbm, read before this level's overwrite) are set, or everywhere with zero_all (no
// separate memset); first: a batch's first level — visited is not read but written (= the frontier)
void launch_bfs_prep(uint64_t *frontier, uint64_t *visited, uint32_t V, const uint64_t *while_bm, bool expand,
                     const DAdj &adj, unsigned long long *stats, uint64_t *fbm, int cus, hipStream_t s,
                     uint32_t vlo = 0, const uint64_t *hub_bm = nullptr, uint64_t *zero = nullptr, bool first = false,
                     bool zero_all = true);
void launch_bfs_list(const uint64_t *frontier, uint32_t V, uint32_t *list, unsigned long long *count, int cus,
                     hipStream_t s);
void launch_bfs_list_deg(const uint32_t *list, uint64_t nl, const uint64_t *rp, uint64_t *deg, hipStream_t s);
// frontier vertices not in hub_bm (a sparse level's push beside a hubs-only pull)
void launch_bfs_list_nonhub(const uint64_t *fbm, const uint64_t *hub_bm, uint32_t V, uint32_t *list,
                            unsigned long long *count, int cus, hipStream_t s);
// partitioned sparse levels: list[i] (relative to vlo) → the vertex and its mask split into two words; and
// fr[v[i]] = the mask on the receiving rank
void launch_bfs_frontier_pack(uint32_t *list, uint64_t n, uint32_t vlo, const uint64_t *fr, uint32_t *mlo, uint32_t *mhi,
                              hipStream_t s);
void launch_bfs_frontier_scatter(const uint32_t *v, const uint32_t *mlo, const uint32_t *mhi, uint64_t n, uint64_t *fr,
                                 hipStream_t s);
// touched (optional): every vertex whose next mask this push turns non-zero, once (*touched_n counts)
void launch_bfs_push(const uint32_t *list, const uint64_t *loffs, uint64_t nl, uint64_t etot, const uint64_t *rp,
                     const uint32_t *col, const uint64_t *frontier, const uint64_t *visited, uint64_t *next,
                     int cus, hipStream_t s, uint32_t *touched = nullptr, unsigned long long *touched_n = nullptr);
// the level prologue over the previous push's touched list (bfs.hip: k_bfs_sparse_clear over the previous
// level's active list `prev`, then k_bfs_prep_sparse); the level's active list → act (*act_n, zeroed by
// the caller); bound: an upper bound of both lists' lengths (grid size; the lengths stay on the device)
void launch_bfs_prep_sparse(const uint32_t *prev, const unsigned long long *prev_n, const uint32_t *touched,
                            const unsigned long long *touched_n, uint64_t bound, uint64_t *frontier, uint64_t *visited,
                            const uint64_t *while_bm, bool expand, const DAdj &adj, unsigned long long *stats,
                            uint64_t *fbm, const uint64_t *hub_bm, uint64_t *zero, uint32_t *act,
                            unsigned long long *act_n, int cus, hipStream_t s);
uint64_t bfs_pull_tiles(uint32_t V, uint64_t E);
void launch_bfs_pull_partition(const uint64_t *rp, uint32_t V, uint64_t E, uint64_t *part, hipStream_t s);
void launch_bfs_pull(uint32_t V, const uint64_t *rp, const uint32_t *col, const uint64_t *part, uint64_t E,
                     uint64_t lanes, const uint64_t *frontier, const uint64_t *hub_fr, const uint64_t *fbm,
                     const uint64_t *visited, uint64_t *next, int cus, hipStream_t s);
// the same level tiled by waves over the in-edge space (k_bfs_pull_w): rb[2·tiles] first / last vertex of
// every tile, regular[tile] (≤ 256 vertices, full); tiles = the tile indices, the nreg regular ones first
uint64_t bfs_pull_w_tiles(uint64_t E);
void launch_pull_w_bounds(const uint64_t *rp, uint32_t V, uint64_t E, uint64_t *rb, uint8_t *regular, hipStream_t s);
void launch_bfs_pull_w(const uint64_t *rp, const uint32_t *col, uint64_t E, const uint32_t *tiles, uint64_t nreg,
                       const uint64_t *rb, uint64_t lanes, const uint64_t *frontier, const uint64_t *hub_fr,
                       uint32_t nhubs, const uint64_t *fbm, const uint64_t *visited, uint64_t *next, int cus,
                       hipStream_t s, bool hubs_only = false);
// dense levels: per-vertex pull with an early exit (k_bfs_pull_exit + k_bfs_pull_rest) over vertices
// [vlo, V); rest u32[V]
// scratch; counts[0] += in-edges read, counts[1] = vertices handed to the per-wave pass (zeroed by the caller)
void launch_bfs_pull_exit(uint32_t V, const uint64_t *rp, const uint32_t *col, uint64_t lanes,
                          const uint64_t *frontier, const uint64_t *hub_fr, const uint64_t *visited, uint64_t *next,
                          uint32_t *rest, unsigned long long *counts, int cus, hipStream_t s, uint32_t vlo = 0);
// hub-annotated col of a CSR for k_bfs_pull (returns the hub count; hub_idx u32[V], hist u32[4096] scratch)
// rp_self: the CSR's own row pointers (its rows are re-ordered hub-first)
uint32_t build_pull_col(const uint64_t *rp_self, const uint64_t *rp_other, const uint32_t *col, uint32_t V, uint64_t E,
                        uint32_t max_hubs,
                        uint32_t *hub_idx, uint32_t *hist, unsigned long long *count, uint32_t *hubs,
                        uint32_t *out, int cus, hipStream_t s);
void launch_hub_gather(const uint32_t *hubs, uint32_t n, const uint64_t *frontier, uint64_t *hub_fr, hipStream_t s);
unsigned bfs_blocks(uint32_t V);
// last (optional): the final level's frontier, merged into visited here (the level skipped its prologue)
void launch_bfs_emit_count(uint64_t *visited, const uint64_t *emit_bm, uint32_t V, uint32_t *blk, hipStream_t s,
                           const uint64_t *last = nullptr);
// binding columns the BFS emission writes directly (row0 + lane → the lane's values); n = 0 → row indices
struct BfsCarry {
  static constexpr int kMax = 4;
  int n = 0;
  uint32_t nl = 0;  // lanes of the batch
  const uint32_t *in[kMax] = {};
  uint32_t *out[kMax] = {};
};
void launch_bfs_emit_write(const uint64_t *visited, const uint64_t *emit_bm, uint32_t V, const uint64_t *blk_offs,
                           uint32_t row0, uint32_t *out_row, uint32_t *out_v, const BfsCarry &cc, hipStream_t s);
void launch_bfs_bound(const uint32_t *dst, uint64_t row0, int nl, const uint64_t *visited, const uint64_t *emit_bm,
                      uint8_t *flags, hipStream_t s, const uint64_t *last = nullptr);

}  // namespace omx
