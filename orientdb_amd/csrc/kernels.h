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

struct ExpandArgs {
  const uint32_t *src;      // [R] source vertex of every binding row
  const uint64_t *offs;     // [R+1] exclusive prefix sum of the rows' adjacency lengths
  const uint64_t *part;     // [ntiles+1] merge-path split: rows consumed before tile t
  uint64_t R, E;            // rows, Σ adjacency length (= edges traversed)
  DAdj adj;
  const uint64_t *filter;   // target bitmap (V bits) or nullptr
  int32_t ncarry;
  const uint32_t *carry_in[kMaxCols];
  uint32_t *carry_out[kMaxCols];
  uint32_t *out_dst;        // new column (neighbour)
  uint32_t *tile_count;     // [ntiles] rows emitted per tile
};

// predicate VM → V-bit bitmap (u64 words); depth = value of $depth
void launch_eval_bitmap(const DPred &pred, uint32_t V, int64_t depth, uint64_t *words, hipStream_t s);
void launch_bitmap_and(const uint64_t *a, uint64_t *b, uint64_t nwords, hipStream_t s);
// per-word popcount (optionally restricted to v % world == rank)
void launch_word_popc(const uint64_t *words, uint64_t nwords, uint32_t V, int rank, int world, uint32_t *counts,
                      hipStream_t s);
void launch_word_scatter(const uint64_t *words, uint64_t nwords, uint32_t V, int rank, int world,
                         const uint32_t *offsets, uint32_t *out, hipStream_t s);

void launch_row_degree(const uint32_t *src, uint64_t R, const DAdj &adj, uint64_t *deg, hipStream_t s);
void launch_mp_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part,
                         hipStream_t s);
void launch_expand(const ExpandArgs &a, uint64_t ntiles, bool write, hipStream_t s);
void launch_compact_tiles(int ncols, uint32_t *const *in, uint32_t *const *out, const uint64_t *part,
                          const uint32_t *tile_count, const uint64_t *tile_offs, uint64_t ntiles, hipStream_t s);

void launch_check(const uint32_t *src, const uint32_t *dst, uint64_t R, const DAdj &adj, const uint64_t *filter,
                  uint8_t *flags, hipStream_t s);
void launch_gather_cols(const uint32_t *idx, uint64_t n, int ncols, const uint32_t *const *in, uint32_t *const *out,
                        hipStream_t s);
void launch_cross(uint64_t R, int ncols, const uint32_t *const *in, uint32_t *const *out, const uint32_t *cand,
                  uint64_t ncand, uint32_t *out_dst, hipStream_t s);
void launch_flag_bitmap(const uint32_t *v, uint64_t n, const uint64_t *bm, uint8_t *flags, hipStream_t s);
void launch_iota(uint32_t *out, uint64_t n, hipStream_t s);
void launch_pack_pairs(const uint32_t *hi, const uint32_t *lo, uint64_t n, uint64_t *keys, hipStream_t s);
void launch_unpack_pairs(const uint64_t *keys, uint64_t n, uint32_t *hi, uint32_t *lo, hipStream_t s);
void launch_flag_not_in(const uint64_t *sorted, uint64_t nsorted, const uint64_t *keys, uint64_t n, uint8_t *flags,
                        hipStream_t s);
void launch_mark_bitmap(const uint32_t *v, uint64_t n, uint64_t *bm, hipStream_t s);
void launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *out, hipStream_t s);
void launch_flag_row_change(int ncols, const uint32_t *const *cols, uint64_t n, uint8_t *flags, hipStream_t s);
void launch_map_rids(int ncols, const uint32_t *const *cols, uint64_t n, const uint64_t *rids, uint64_t *out,
                     hipStream_t s);

}  // namespace omx
