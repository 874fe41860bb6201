// ridbag.hip — device decoding of serialized ridbags into a CSR (include/omx/match.h
// omx_ridbag_decode_csr).
//
// An OrientDB vertex keeps each edge class's adjacency in an out_<L> / in_<L> ridbag field. The record
// serializer writes an embedded bag as (C/db/record/ridbag/ORidBag.java:198-276 toStream,
// C/db/record/ridbag/embedded/OEmbeddedRidBag.java:424-460 serialize, C/serialization/serializer/
// binary/impl/OLinkSerializer.java:54-58, OIntegerSerializer.java:53-58 — all big-endian):
//   [1 B config: bit 0 embedded, bit 1 UUID follows][16 B UUID if bit 1]
//   [int32 count][count × (int16 cluster id, int64 cluster position)]
// An SBTree-bonsai bag (config bit 0 clear; every bag of >= 40 entries by default,
// C/config/OGlobalConfiguration.java:356-358) holds a pointer to a B+-tree in a collection file plus the
// pending changes (C/db/record/ridbag/sbtree/OSBTreeRidBag.java:855-880, 903-929):
//   [int64 fileId][int64 root pageIndex][int32 root pageOffset][int32 cached size]
//   [int32 n][n × (int16 cluster, int64 position, int8 type, int32 value)]          (big-endian)
// Its entries are decoded from the collection files' pages (omx_bonsai_file; C/index/sbtreebonsai/
// local/OSBTreeBonsaiBucket.java:44-60 bucket layout, :263-279 entries; native = little-endian page
// memory, except the RID position, which OLinkSerializer writes big-endian). Without the files such a
// bag is rejected. Pipeline (decode_trees below): the trees' buckets level by level from the roots —
// an internal bucket's children are its first entry's left child and every entry's right child, so the
// leaves come out in key order, exactly the leaves OSBTreeBonsaiLocal.loadEntriesMajor walks along the
// right siblings — then one thread per leaf entry, the changes merged per bag (RIDBagIterator,
// OSBTreeRidBag.java:256-425) and every RID written `count` times.
//
// With lightweight edges the entries are the neighbour vertices' RIDs. With edge records they are the
// edge documents' RIDs and the neighbour is the edge's opposite vertex field (`in` for an out_ bag);
// the caller passes that table. Both lookups are binary searches over RID-sorted copies, so any RID
// assignment works (not only the one-cluster-per-class canonical one).
//
// Layout in HBM: the streams as one byte array (the caller's concatenation), offsets[V+1] into it. One
// pass counts (one thread per vertex: header parse), a scan gives the row pointers, one pass decodes
// (one thread per entry, its vertex found by binary search over the row pointers): every entry is read
// once (10 B) and written once (4 B) — an HBM-bound byte-parsing pass, no MFMA work.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "devutil.h"
#include "graph.h"

namespace omx {

namespace {

enum BagError : uint32_t {
  kBagOk = 0,
  kBagTruncated = 1,     // a stream shorter than its header / count says
  kBagSBTree = 2,        // config bit 0 clear: an SBTree bag (entries on disk)
  kBagUnknownRid = 4,    // an entry (or its edge's target) is no vertex of the snapshot
  kBagPosition = 8,      // a cluster position ≥ 2^48 or a negative cluster id (not packable)
  kBagUnknownEdge = 16,  // an edge RID missing from the edge table
  kBagUnknownFile = 32,  // an SBTree bag whose collection file was not passed
  kBagBadBucket = 64,    // a bucket pointer / entry position outside its page, or a tree deeper than 64
  kBagChangeType = 128,  // a change of unknown type, or changes not in RID order
};

__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ uint64_t be64(const uint8_t *p) {
  return ((uint64_t)be32(p) << 32) | (uint64_t)be32(p + 4);
}

__device__ __forceinline__ uint16_t be16(const uint8_t *p) { return (uint16_t)(((uint32_t)p[0] << 8) | p[1]); }
__device__ __forceinline__ uint32_t le32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

// An SBTree bag's header (tree_* arrays indexed by vertex): file index (-1: no tree, fileId -1),
// root bucket, change count and the offset of its first change
struct TreeHdr {
  int32_t *file;
  uint64_t *root;   // pageIndex << 24 | pageOffset
  uint32_t *nchg;
  uint64_t *chg;
  uint8_t *is_tree;
  const int64_t *fids;  // sorted file ids
  const uint64_t *npages;
  int32_t nfiles;
  uint32_t page_size;
};

constexpr uint64_t kTreeRow = ~0ull;  // pay[] of a row decoded from a tree (skipped by k_bag_decode)

// header of vertex v's stream: payload offset and entry count (0 for an empty stream = no field)
__device__ __forceinline__ uint32_t bag_header(const uint8_t *s, const uint64_t *offs, uint32_t v, uint64_t *payload,
                                               uint32_t *err, const TreeHdr *th) {
  const uint64_t b = offs[v], e = offs[v + 1];
  *payload = b;
  if (th) th->is_tree[v] = 0;
  if (e <= b) return 0;
  const uint8_t cfg = s[b];
  if (!(cfg & 1)) {
    if (!th) {
      atomicOr(err, (uint32_t)kBagSBTree);
      return 0;
    }
    const uint64_t h = b + 1 + ((cfg & 2) ? 16 : 0);
    if (h + 28 > e) {
      atomicOr(err, (uint32_t)kBagTruncated);
      return 0;
    }
    const int64_t fid = (int64_t)be64(s + h), page = (int64_t)be64(s + h + 8);
    const int32_t off = (int32_t)be32(s + h + 16);
    const uint32_t n = be32(s + h + 24);
    if ((n >> 31) || h + 28 + 15ull * n > e) {
      atomicOr(err, (uint32_t)kBagTruncated);
      return 0;
    }
    int32_t fi = -1;
    if (fid != -1) {
      int32_t lo = 0, hi = th->nfiles;
      while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (th->fids[mid] < fid) lo = mid + 1;
        else hi = mid;
      }
      if (lo == th->nfiles || th->fids[lo] != fid) {
        atomicOr(err, (uint32_t)kBagUnknownFile);
        return 0;
      }
      if (page < 0 || (uint64_t)page >= th->npages[lo] || off < 0 || (uint32_t)off + 83u > th->page_size) {
        atomicOr(err, (uint32_t)kBagBadBucket);
        return 0;
      }
      fi = lo;
    }
    th->is_tree[v] = 1;
    th->file[v] = fi;
    th->root[v] = fi < 0 ? 0 : ((uint64_t)page << 24) | (uint32_t)off;
    th->nchg[v] = n;
    th->chg[v] = h + 28;
    *payload = kTreeRow;
    return 0;
  }
  const uint64_t h = b + 1 + ((cfg & 2) ? 16 : 0);
  if (h + 4 > e) {
    atomicOr(err, (uint32_t)kBagTruncated);
    return 0;
  }
  const uint32_t n = be32(s + h);
  if ((n >> 31) || h + 4 + 10ull * n > e) {
    atomicOr(err, (uint32_t)kBagTruncated);
    return 0;
  }
  *payload = h + 4;
  return n;
}

__global__ void k_bag_count(const uint8_t *s, const uint64_t *offs, uint32_t V, uint64_t *cnt, uint64_t *pay,
                            uint32_t *err, TreeHdr th, int trees) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v > V) return;
  if (v == V) {
    cnt[V] = 0;
    return;
  }
  uint64_t p;
  cnt[v] = bag_header(s, offs, (uint32_t)v, &p, err, trees ? &th : nullptr);
  pay[v] = p;
}

// index of key in sorted[0..n) (n if absent)
__device__ __forceinline__ uint64_t find_sorted(const uint64_t *sorted, uint64_t n, uint64_t key) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo < n && sorted[lo] == key ? lo : n;
}

// RID → value lookup. Direct: RIDs whose positions are compact per cluster (the usual case: records
// are appended) index a table, base[cluster] + position; otherwise a binary search over a RID-sorted copy.
template <class T>
struct RidIndex {
  const int64_t *base;   // [32768] table offset of each cluster, -1 if absent (direct mode); affine: value − position
  const uint64_t *lim;   // [32768] positions of the cluster are < lim
  const uint64_t *lo;    // [32768] affine mode: positions are ≥ lo
  const T *table;        // direct mode; sentinel ~0 = no record
  const uint64_t *keys;  // sorted mode
  const T *vals;
  uint64_t n;
  int direct;
  int affine;            // every cluster's records hold contiguous positions at consecutive values
  __device__ __forceinline__ bool find(uint64_t rid, T *out) const {
    if (affine) {  // dense layout of the clusters (records appended, none deleted): no table read
      const uint32_t c = (uint32_t)(rid >> 48);
      const uint64_t p = rid & ((1ull << 48) - 1);
      if (c >= 32768 || p < lo[c] || p >= lim[c]) return false;
      *out = (T)(base[c] + (int64_t)p);
      return true;
    }
    if (direct) {
      const uint32_t c = (uint32_t)(rid >> 48);
      const uint64_t p = rid & ((1ull << 48) - 1);
      const int64_t b = c < 32768 ? base[c] : -1;
      if (b < 0 || p >= lim[c]) return false;
      const T x = table[b + p];
      if (x == (T)~(T)0) return false;
      *out = x;
      return true;
    }
    const uint64_t i = find_sorted(keys, n, rid);
    if (i == n) return false;
    *out = vals[i];
    return true;
  }
};

template <class T>
__global__ void k_index_fill(const uint64_t *rids, const T *vals, uint64_t n, const int64_t *base, T *table) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = rids[i];
    table[base[r >> 48] + (r & ((1ull << 48) - 1))] = vals ? vals[i] : (T)i;
  }
}

// One block decodes kDecTile consecutive entries. Their rows lie between the rows of the tile's first
// and last entry (two searches per block); the tile's row pointers and payload offsets are staged in
// LDS, so an entry's row is an LDS search. Each thread then issues its entries' window loads together,
// and their index lookups together (independent chains in flight instead of one dependent chain).
constexpr int kDecB = 256, kDecIPT = 8, kDecTile = kDecB * kDecIPT, kDecRows = 1024;
__global__ __launch_bounds__(kDecB) void k_bag_decode(const uint8_t *s, const uint64_t *pay, uint32_t V,
                                                      const uint64_t *rp, uint64_t E, RidIndex<uint32_t> vix,
                                                      RidIndex<uint64_t> eix, int edges, uint32_t *col, uint32_t *err,
                                                      uint64_t *erid) {
  __shared__ uint64_t s_r[2];
  __shared__ uint64_t s_rp[kDecRows + 1];
  __shared__ uint64_t s_pay[kDecRows];
  for (uint64_t t0 = (uint64_t)blockIdx.x * kDecTile; t0 < E; t0 += (uint64_t)gridDim.x * kDecTile) {
    const uint64_t t1 = min(t0 + (uint64_t)kDecTile, E) - 1;
    if (threadIdx.x < 2) {  // last v with rp[v] <= e
      const uint64_t e = threadIdx.x ? t1 : t0;
      uint64_t lo = 0, hi = V;
      while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (rp[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      s_r[threadIdx.x] = lo;
    }
    __syncthreads();
    const uint64_t r0 = s_r[0], r1 = s_r[1];
    const uint64_t nr = r1 - r0 + 1;
    const bool staged = nr <= kDecRows;
    if (staged) {
      for (uint32_t i = threadIdx.x; i <= nr; i += kDecB) s_rp[i] = rp[r0 + i];
      for (uint32_t i = threadIdx.x; i < nr; i += kDecB) s_pay[i] = pay[r0 + i];
    }
    __syncthreads();
    uint64_t off[kDecIPT];
#pragma unroll
    for (int k = 0; k < kDecIPT; ++k) {
      const uint64_t e = t0 + (uint64_t)k * kDecB + threadIdx.x;
      off[k] = ~0ull;
      if (e > t1) continue;
      uint64_t lo = 0, hi = nr - 1;  // row index relative to r0
      if (staged) {
        while (lo < hi) {
          const uint64_t mid = (lo + hi + 1) >> 1;
          if (s_rp[mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        off[k] = s_pay[lo] == kTreeRow ? ~0ull : s_pay[lo] + 10ull * (e - s_rp[lo]);
      } else {
        while (lo < hi) {
          const uint64_t mid = (lo + hi + 1) >> 1;
          if (rp[r0 + mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        off[k] = pay[r0 + lo] == kTreeRow ? ~0ull : pay[r0 + lo] + 10ull * (e - rp[r0 + lo]);
      }
    }
    uint64_t rid[kDecIPT];
#pragma unroll
    for (int k = 0; k < kDecIPT; ++k) {  // the 10-byte entries from the aligned dwords around them
      rid[k] = ~0ull;
      if (off[k] == ~0ull) continue;
      const uint64_t o = off[k];
      const uint32_t *w = reinterpret_cast<const uint32_t *>(s + (o & ~3ull));
      const uint32_t sh = (uint32_t)(o & 3) * 8;
      const uint64_t wl = ((uint64_t)w[1] << 32) | w[0], wh = ((uint64_t)(sh ? w[3] : 0u) << 32) | w[2];
      const uint64_t b07 = sh ? (wl >> sh) | (wh << (64 - sh)) : wl;  // entry bytes 0..7, little-endian
      const uint64_t b89 = (wh >> sh) & 0xFFFFull;                     // entry bytes 8..9
      const int16_t cl = (int16_t)(((b07 & 0xFF) << 8) | ((b07 >> 8) & 0xFF));
      const uint64_t pos = __builtin_bswap64((b07 >> 16) | (b89 << 48));
      if (cl < 0 || (pos >> 48)) atomicOr(err, (uint32_t)kBagPosition);
      else rid[k] = ((uint64_t)(uint16_t)cl << 48) | pos;
    }
    if (erid) {  // the entries themselves: the edge records' RIDs
#pragma unroll
      for (int k = 0; k < kDecIPT; ++k)
        if (off[k] != ~0ull) erid[t0 + (uint64_t)k * kDecB + threadIdx.x] = rid[k];
    }
    if (edges) {  // edge records: their opposite vertices
#pragma unroll
      for (int k = 0; k < kDecIPT; ++k) {
        if (rid[k] == ~0ull) continue;
        uint64_t target;
        if (eix.find(rid[k], &target)) rid[k] = target;
        else {
          atomicOr(err, (uint32_t)kBagUnknownEdge);
          rid[k] = ~0ull;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kDecIPT; ++k) {
      if (off[k] == ~0ull) continue;
      uint32_t out = 0xFFFFFFFFu;
      if (rid[k] != ~0ull && !vix.find(rid[k], &out)) {
        atomicOr(err, (uint32_t)kBagUnknownRid);
        out = 0xFFFFFFFFu;
      }
      col[t0 + (uint64_t)k * kDecB + threadIdx.x] = out;
    }
    __syncthreads();
  }
}

template <class T>
struct DevArr {
  T *p = nullptr;
  explicit DevArr(size_t n) { HIP_CHECK(hipMalloc((void **)&p, std::max<size_t>(n, 1) * sizeof(T))); }
  DevArr(const DevArr &) = delete;
  ~DevArr() {
    if (p) (void)hipFree(p);
  }
};

// RID index on the device (RidIndex), built from host arrays: direct when every RID is packable and the
// per-cluster position ranges total at most 2n + 64 K slots, else RID-sorted (radix sort) for searches
template <class T>
struct HostIndex {
  std::unique_ptr<DevArr<int64_t>> base;
  std::unique_ptr<DevArr<uint64_t>> lim, lo, keys;
  std::unique_ptr<DevArr<T>> table, vals;
  RidIndex<T> dev{};
};
template <class T>
void build_index(HostIndex<T> &ix, const uint64_t *rids, const T *vals, uint64_t n, hipStream_t s) {
  std::vector<int64_t> hb(32768, -1);
  std::vector<uint64_t> hl(32768, 0);
  bool packable = true;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t c = rids[i] >> 48, p = rids[i] & ((1ull << 48) - 1);
    if (c >= 32768) {
      packable = false;
      break;
    }
    hl[c] = std::max(hl[c], p + 1);
  }
  // affine: values are the positions i (vertex table) and every cluster's RIDs are contiguous positions
  // p0 … p0 + k − 1 held by consecutive i (value = p + delta): the canonical snapshot order
  if (packable && !vals && n) {
    std::vector<int64_t> delta(32768, INT64_MIN);
    std::vector<uint64_t> cnt(32768, 0), mn(32768, UINT64_MAX);
    bool affine = true;
    for (uint64_t i = 0; i < n && affine; ++i) {
      const uint64_t c = rids[i] >> 48, p = rids[i] & ((1ull << 48) - 1);
      const int64_t d = (int64_t)i - (int64_t)p;
      if (delta[c] == INT64_MIN) delta[c] = d;
      else if (delta[c] != d) affine = false;
      ++cnt[c];
      mn[c] = std::min(mn[c], p);
    }
    for (int c = 0; c < 32768 && affine; ++c)
      if (cnt[c] && hl[c] - mn[c] != cnt[c]) affine = false;  // no holes, no repeats
    if (affine) {
      std::vector<uint64_t> hlo(32768, 0);
      for (int c = 0; c < 32768; ++c) {
        hlo[c] = cnt[c] ? mn[c] : 0;
        hb[c] = cnt[c] ? delta[c] : 0;
        if (!cnt[c]) hl[c] = 0;
      }
      ix.base.reset(new DevArr<int64_t>(32768));
      ix.lim.reset(new DevArr<uint64_t>(32768));
      ix.lo.reset(new DevArr<uint64_t>(32768));
      HIP_CHECK(hipMemcpyAsync(ix.base->p, hb.data(), 32768 * 8, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipMemcpyAsync(ix.lim->p, hl.data(), 32768 * 8, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipMemcpyAsync(ix.lo->p, hlo.data(), 32768 * 8, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipStreamSynchronize(s));
      ix.dev.base = ix.base->p;
      ix.dev.lim = ix.lim->p;
      ix.dev.lo = ix.lo->p;
      ix.dev.affine = 1;
      return;
    }
  }
  uint64_t total = 0;
  if (packable)
    for (int c = 0; c < 32768; ++c)
      if (hl[c]) {
        hb[c] = (int64_t)total;
        total += hl[c];
      }
  DevArr<uint64_t> dr(n);
  if (n) HIP_CHECK(hipMemcpyAsync(dr.p, rids, n * 8, hipMemcpyHostToDevice, s));
  std::unique_ptr<DevArr<T>> dv;
  if (vals && n) {
    dv.reset(new DevArr<T>(n));
    HIP_CHECK(hipMemcpyAsync(dv->p, vals, n * sizeof(T), hipMemcpyHostToDevice, s));
  }
  if (packable && total <= 2 * n + 65536) {
    ix.base.reset(new DevArr<int64_t>(32768));
    ix.lim.reset(new DevArr<uint64_t>(32768));
    ix.table.reset(new DevArr<T>(total));
    HIP_CHECK(hipMemcpyAsync(ix.base->p, hb.data(), 32768 * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(ix.lim->p, hl.data(), 32768 * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(ix.table->p, 0xFF, std::max<uint64_t>(total, 1) * sizeof(T), s));
    if (n) {
      hipLaunchKernelGGL(k_index_fill<T>, dim3((unsigned)std::min<uint64_t>(nblocks(n, 256), 65536)), dim3(256), 0, s,
                         dr.p, dv ? dv->p : nullptr, n, ix.base->p, ix.table->p);
      KCHECK("k_index_fill");
    }
    ix.dev.base = ix.base->p;
    ix.dev.lim = ix.lim->p;
    ix.dev.table = ix.table->p;
    ix.dev.direct = 1;
  } else {
    ix.keys.reset(new DevArr<uint64_t>(n));
    ix.vals.reset(new DevArr<T>(n));
    DevArr<T> iv(n);
    if (!dv) {  // values = positions
      std::vector<T> h(n);
      for (uint64_t i = 0; i < n; ++i) h[i] = (T)i;
      if (n) HIP_CHECK(hipMemcpyAsync(iv.p, h.data(), n * sizeof(T), hipMemcpyHostToDevice, s));
      HIP_CHECK(hipStreamSynchronize(s));
    }
    size_t sb = 0;
    const T *vin = dv ? dv->p : iv.p;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, dr.p, ix.keys->p, vin, ix.vals->p, (int64_t)n, 0, 64, s));
    DevArr<uint8_t> stmp(sb);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(stmp.p, sb, dr.p, ix.keys->p, vin, ix.vals->p, (int64_t)n, 0, 64, s));
    ix.dev.keys = ix.keys->p;
    ix.dev.vals = ix.vals->p;
    ix.dev.n = n;
    ix.dev.direct = 0;
  }
  HIP_CHECK(hipStreamSynchronize(s));  // the temporaries above leave scope
}

// ---- SBTree-bonsai bags ------------------------------------------------------------------------------
// OSBTreeBonsaiBucket.java:44-60 offsets inside a bucket
constexpr uint32_t kBkSize = 32, kBkFlags = 36, kBkPos = 83, kLeafEntry = 14, kNodeEntry = 34;

struct Pages {
  const uint8_t *p;       // every file's pages, file f's at base[f]
  const uint64_t *base;
  const uint64_t *npages;
  uint32_t page_size;
  __device__ __forceinline__ const uint8_t *bucket(int32_t f, uint64_t ptr) const {
    return p + base[f] + (ptr >> 24) * (uint64_t)page_size + (ptr & 0xFFFFFFu);
  }
  // room from the bucket start to the end of its page
  __device__ __forceinline__ uint32_t room(uint64_t ptr) const { return page_size - (uint32_t)(ptr & 0xFFFFFFu); }
};

// the trees that have a root (fileId != -1): their index t, in vertex order
__global__ void k_tree_roots(const uint32_t *tv, uint32_t nt, const int32_t *file, uint8_t *flag) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nt) flag[t] = file[tv[t]] >= 0;
}
__global__ void k_node_init(const uint32_t *sel, uint64_t n, const uint32_t *tv, const int32_t *file, const uint64_t *root,
                            uint32_t *ntree, int32_t *nfile, uint64_t *nptr) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t t = sel[i], v = tv[t];
  ntree[i] = t;
  nfile[i] = file[v];
  nptr[i] = root[v];
}

// children of one level's buckets: a leaf stands for itself; an internal bucket of k entries has k + 1
// children (first entry's left child, then every entry's right child: OSBTreeBonsaiBucket.java:355-413
// keeps entry i's right child = entry i + 1's left child). internal[0] counts the internal buckets.
__global__ void k_node_count(Pages pg, const int32_t *nfile, const uint64_t *nptr, uint64_t n, uint32_t *nch,
                             unsigned long long *internal, uint32_t *err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    nch[n] = 0;
    return;
  }
  const uint8_t *b = pg.bucket(nfile[i], nptr[i]);
  const int32_t size = (int32_t)le32(b + kBkSize);
  const bool leaf = b[kBkFlags] & 1;
  if (size < 0 || kBkPos + 4ull * (uint32_t)size > pg.room(nptr[i])) {
    atomicOr(err, (uint32_t)kBagBadBucket);
    nch[i] = 0;
    return;
  }
  nch[i] = leaf ? 1u : (size ? (uint32_t)size + 1u : 0u);
  if (!leaf && size) atomicAdd(internal, 1ull);
}

__device__ __forceinline__ bool child_ptr(const Pages &pg, int32_t f, const uint8_t *p, uint64_t *out) {
  const int64_t page = (int64_t)le64(p);
  const int32_t off = (int32_t)le32(p + 8);
  if (page < 0 || (uint64_t)page >= pg.npages[f] || off < 0 || (uint32_t)off + kBkPos > pg.page_size) return false;
  *out = ((uint64_t)page << 24) | (uint32_t)off;
  return true;
}

__global__ void k_node_emit(Pages pg, const uint32_t *ntree, const int32_t *nfile, const uint64_t *nptr, uint64_t n,
                            const uint64_t *coff, uint32_t *otree, int32_t *ofile, uint64_t *optr, uint32_t *err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = coff[i], k = coff[i + 1] - o;
  if (!k) return;
  const int32_t f = nfile[i];
  const uint8_t *b = pg.bucket(f, nptr[i]);
  if (b[kBkFlags] & 1) {  // a leaf: carried to the next level as it is
    otree[o] = ntree[i];
    ofile[o] = f;
    optr[o] = nptr[i];
    return;
  }
  const uint32_t room = pg.room(nptr[i]);
  for (uint64_t j = 0; j < k; ++j) {
    const uint32_t e = j ? (uint32_t)j - 1 : 0;  // entry e: its left child (j = 0) or right child
    const uint32_t pos = le32(b + kBkPos + 4 * e);
    uint64_t c = 0;
    if (pos + kNodeEntry > room || !child_ptr(pg, f, b + pos + (j ? 12 : 0), &c)) {
      atomicOr(err, (uint32_t)kBagBadBucket);
      c = nptr[i];  // (the result is discarded: the error fails the call)
    }
    otree[o + j] = ntree[i];
    ofile[o + j] = f;
    optr[o + j] = c;
  }
}

// leaf sizes (the nodes are all leaves now); the entries each tree holds
__global__ void k_leaf_sizes(Pages pg, const uint32_t *ntree, const int32_t *nfile, const uint64_t *nptr, uint64_t n,
                             uint64_t *lsize, unsigned long long *tree_n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  if (i == n) {
    lsize[n] = 0;
    return;
  }
  const uint32_t size = le32(pg.bucket(nfile[i], nptr[i]) + kBkSize);  // validated by k_node_count
  lsize[i] = size;
  if (size) atomicAdd(&tree_n[ntree[i]], (unsigned long long)size);
}

// last i in [0, n) with a[i] <= x (a ascending, a[0] <= x)
__device__ __forceinline__ uint64_t last_le(const uint64_t *a, uint64_t n, uint64_t x) {
  uint64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (a[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// one thread per leaf entry: OSBTreeBonsaiBucket.getEntry (:263-279) — the key (int16 cluster in native
// order, int64 position big-endian) and the int32 counter (native order)
__global__ void k_leaf_entries(Pages pg, const int32_t *nfile, const uint64_t *nptr, uint64_t nleaves,
                               const uint64_t *loff, uint64_t T, uint64_t *rid, int32_t *val, uint32_t *err) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = last_le(loff, nleaves, e);
    const uint32_t i = (uint32_t)(e - loff[l]);
    const uint8_t *b = pg.bucket(nfile[l], nptr[l]);
    const uint32_t pos = le32(b + kBkPos + 4 * i);
    uint64_t r = ~0ull;
    int32_t c = 0;
    if (pos + kLeafEntry > pg.room(nptr[l])) {
      atomicOr(err, (uint32_t)kBagBadBucket);
    } else {
      const uint8_t *q = b + pos;
      const int16_t cl = (int16_t)((uint16_t)q[0] | ((uint16_t)q[1] << 8));
      const uint64_t position = be64(q + 2);
      if (cl < 0 || (position >> 48)) atomicOr(err, (uint32_t)kBagPosition);
      else r = ((uint64_t)(uint16_t)cl << 48) | position;
      c = (int32_t)le32(q + 10);
    }
    rid[e] = r;
    val[e] = c;
  }
}

// runs (RID, count) of a tree without changes: its entries, each yielded max(1, counter) times
// (RIDBagIterator.next returns the RID before comparing the counter, OSBTreeRidBag.java:287-309)
__global__ void k_runs_copy(const uint64_t *rid, const int32_t *val, uint64_t T, const uint64_t *teoff, uint32_t nt,
                            const uint32_t *tv, const uint32_t *nchg, const uint64_t *roff, uint64_t *rrid,
                            uint64_t *rcnt) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t t = last_le(teoff, nt, e);
    if (nchg[tv[t]]) continue;  // merged by k_runs_merge
    const uint64_t r = roff[t] + (e - teoff[t]);
    rrid[r] = rid[e];
    rcnt[r] = val[e] > 0 ? (uint64_t)val[e] : 1ull;
  }
}

__device__ __forceinline__ int32_t apply_change(uint8_t type, int32_t delta, int32_t value) {
  return type == 0 ? value + delta : delta;  // DiffChange.applyTo / AbsoluteChange.applyTo (:118-195)
}

// one thread per tree with changes: the tree entries and the changes (RID order, as the skip list
// serialised them) merged like RIDBagIterator.next (:293-340); every slot of the tree's runs is written,
// the ones left over with count 0
__global__ void k_runs_merge(const uint8_t *s, const uint64_t *rid, const int32_t *val, const uint64_t *teoff,
                             const uint32_t *tv, uint32_t nt, const uint32_t *nchg, const uint64_t *chg,
                             const uint64_t *roff, uint64_t *rrid, uint64_t *rcnt, uint32_t *err) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;
  const uint32_t v = tv[t], nc = nchg[v];
  if (!nc) return;
  const uint64_t e0 = teoff[t], e1 = teoff[t + 1], c0 = chg[v];
  uint64_t w = roff[t];
  const uint64_t wend = roff[t + 1];
  uint64_t ei = e0;
  uint32_t ci = 0;
  uint64_t prev = 0;
  // the next change (key, type, value); key ~0 when none is left
  auto change = [&](uint32_t j, uint64_t *key, uint8_t *type, int32_t *x) {
    const uint8_t *q = s + c0 + 15ull * j;
    const int16_t cl = (int16_t)be16(q);
    const uint64_t pos = be64(q + 2);
    *type = q[10];
    *x = (int32_t)be32(q + 11);
    if (cl < 0 || (pos >> 48)) {
      atomicOr(err, (uint32_t)kBagPosition);
      *key = ~0ull - 1;
    } else {
      *key = ((uint64_t)(uint16_t)cl << 48) | pos;
    }
    if (*type > 1 || (j && *key <= prev)) atomicOr(err, (uint32_t)kBagChangeType);
    prev = *key;
  };
  uint64_t ck = ~0ull;
  uint8_t ct = 0;
  int32_t cx = 0;
  if (ci < nc) change(ci, &ck, &ct, &cx);
  while (ei < e1 || ci < nc) {
    const uint64_t tk = ei < e1 ? rid[ei] : ~0ull;
    uint64_t key;
    int64_t cnt;
    if (ci < nc && ck < tk) {  // a change-only RID: applyTo(0)
      key = ck;
      cnt = apply_change(ct, cx, 0);
      if (++ci < nc) change(ci, &ck, &ct, &cx);
    } else {  // a tree entry, with its change if there is one
      key = tk;
      const int32_t tv0 = val[ei++];
      if (ci < nc && ck == tk) {
        cnt = apply_change(ct, cx, tv0);
        if (++ci < nc) change(ci, &ck, &ct, &cx);
      } else {
        cnt = tv0 > 0 ? tv0 : 1;
      }
    }
    if (cnt > 0 && w < wend) {
      rrid[w] = key;
      rcnt[w] = (uint64_t)cnt;
      ++w;
    }
  }
  for (; w < wend; ++w) {
    rrid[w] = 0;
    rcnt[w] = 0;
  }
}

__global__ void k_tree_row_counts(const uint32_t *tv, uint32_t nt, const uint64_t *tsum, uint64_t *cnt) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < nt) cnt[tv[t]] = tsum[t];
}

// one thread per run: its RID → dense vertex id, written `count` times at the row's place
__global__ void k_runs_write(const uint64_t *rrid, const uint64_t *rcnt, uint64_t R, const uint64_t *ro,
                             const uint64_t *roff, uint32_t nt, const uint32_t *tv, const uint64_t *rp,
                             RidIndex<uint32_t> vix, RidIndex<uint64_t> eix, int edges, uint32_t *col, uint32_t *err,
                             uint64_t *erid) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = rcnt[r];
    if (!c) continue;
    const uint64_t t = last_le(roff, nt, r);
    const uint64_t out = rp[tv[t]] + (ro[r] - ro[roff[t]]);
    uint64_t id = rrid[r];
    if (erid)
      for (uint64_t k = 0; k < c; ++k) erid[out + k] = id;
    uint32_t x = 0xFFFFFFFFu;
    if (id != ~0ull && edges && !eix.find(id, &id)) {
      atomicOr(err, (uint32_t)kBagUnknownEdge);
      id = ~0ull;
    }
    if (id != ~0ull && !vix.find(id, &x)) {
      atomicOr(err, (uint32_t)kBagUnknownRid);
      x = 0xFFFFFFFFu;
    }
    for (uint64_t k = 0; k < c; ++k) col[out + k] = x;
  }
}

std::string bag_error_text(uint32_t e) {
  std::string m;
  if (e & kBagSBTree) m += " an SBTree ridbag without its collection files (omx_bonsai_file);";
  if (e & kBagUnknownFile) m += " an SBTree ridbag whose collection file was not passed;";
  if (e & kBagBadBucket) m += " an SBTree bucket pointer or entry outside its page (or a tree deeper than 64 levels);";
  if (e & kBagChangeType) m += " an SBTree ridbag change of unknown type or out of RID order;";
  if (e & kBagTruncated) m += " a stream shorter than its header and count;";
  if (e & kBagPosition) m += " a RID with a negative cluster or a position of 2^48 or more;";
  if (e & kBagUnknownEdge) m += " an edge RID missing from the edge table;";
  if (e & kBagUnknownRid) m += " a RID that is no vertex of the snapshot;";
  return m;
}

struct WidenU32 {
  __host__ __device__ uint64_t operator()(const uint32_t &x) const { return x; }
};

// The SBTree bags of a decode: their trees' leaves and runs (decode_trees), then their rows' counts
struct TreeRuns {
  uint32_t nt = 0;  // trees (vertices with an SBTree bag)
  std::unique_ptr<DevArr<uint32_t>> tv;
  std::unique_ptr<DevArr<uint64_t>> roff, rrid, rcnt;  // runs of tree t at [roff[t], roff[t+1])
  uint64_t R = 0;
};

template <class F>
void cub_call(hipStream_t s, F f) {
  size_t b = 0;
  HIP_CHECK(f(nullptr, b));
  DevArr<uint8_t> tmp(b);
  HIP_CHECK(f(tmp.p, b));
  HIP_CHECK(hipStreamSynchronize(s));
}

uint64_t read_u64(const uint64_t *p, hipStream_t s) {
  uint64_t x = 0;
  HIP_CHECK(hipMemcpyAsync(&x, p, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return x;
}

uint32_t read_err(const uint32_t *err, hipStream_t s) {
  uint32_t e = 0;
  HIP_CHECK(hipMemcpyAsync(&e, err, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return e;
}

// the trees' entries as runs (RID, count) in iteration order, and every tree row's count into cnt[v]
void decode_trees(hipStream_t s, const uint8_t *ds, uint32_t V, const TreeHdr &th, const uint8_t *is_tree,
                  const Pages &pg, uint64_t *cnt, uint32_t *err, TreeRuns &out) {
  // the vertices with an SBTree bag, in vertex order
  DevArr<uint32_t> tv(V), nsel(2);
  DevArr<unsigned long long> n64(2);
  hipcub::CountingInputIterator<uint32_t> iota(0);
  cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, iota, is_tree, tv.p, n64.p, (int64_t)V, s); });
  const uint32_t nt = (uint32_t)read_u64(reinterpret_cast<uint64_t *>(n64.p), s);
  out.nt = nt;
  if (!nt) return;
  // level 0: the roots of the trees that have one
  DevArr<uint8_t> hasroot(nt);
  hipLaunchKernelGGL(k_tree_roots, dim3(nblocks(nt, 256)), dim3(256), 0, s, tv.p, nt, th.file, hasroot.p);
  KCHECK("k_tree_roots");
  DevArr<uint32_t> sel(nt);
  cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, iota, hasroot.p, sel.p, n64.p, (int64_t)nt, s); });
  uint64_t n = read_u64(reinterpret_cast<uint64_t *>(n64.p), s);
  auto ntree = std::make_unique<DevArr<uint32_t>>(n);
  auto nfile = std::make_unique<DevArr<int32_t>>(n);
  auto nptr = std::make_unique<DevArr<uint64_t>>(n);
  if (n) {
    hipLaunchKernelGGL(k_node_init, dim3(nblocks(n, 256)), dim3(256), 0, s, sel.p, n, tv.p, th.file, th.root, ntree->p,
                       nfile->p, nptr->p);
    KCHECK("k_node_init");
  }
  // levels: every internal bucket replaced by its children (leaves carried) until only leaves are left
  for (int level = 0; n; ++level) {
    if (level > 64) {
      uint32_t e = kBagBadBucket;
      HIP_CHECK(hipMemcpyAsync(err, &e, 4, hipMemcpyHostToDevice, s));
      HIP_CHECK(hipStreamSynchronize(s));
      return;
    }
    DevArr<uint32_t> nch(n + 1);
    HIP_CHECK(hipMemsetAsync(n64.p, 0, 8, s));
    hipLaunchKernelGGL(k_node_count, dim3(nblocks(n + 1, 256)), dim3(256), 0, s, pg, nfile->p, nptr->p, n, nch.p, n64.p, err);
    KCHECK("k_node_count");
    if (read_err(err, s)) return;
    const uint64_t internal = read_u64(reinterpret_cast<uint64_t *>(n64.p), s);
    if (!internal) break;
    DevArr<uint64_t> coff(n + 1);
    hipcub::TransformInputIterator<uint64_t, WidenU32, const uint32_t *> nch64(nch.p, WidenU32());
    cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, nch64, coff.p, (int64_t)n + 1, s); });
    const uint64_t m = read_u64(coff.p + n, s);
    auto otree = std::make_unique<DevArr<uint32_t>>(m);
    auto ofile = std::make_unique<DevArr<int32_t>>(m);
    auto optr = std::make_unique<DevArr<uint64_t>>(m);
    hipLaunchKernelGGL(k_node_emit, dim3(nblocks(n, 256)), dim3(256), 0, s, pg, ntree->p, nfile->p, nptr->p, n, coff.p,
                       otree->p, ofile->p, optr->p, err);
    KCHECK("k_node_emit");
    if (read_err(err, s)) return;
    ntree = std::move(otree);
    nfile = std::move(ofile);
    nptr = std::move(optr);
    n = m;
  }
  // leaves → entries; entries per tree
  DevArr<uint64_t> lsize(n + 1), loff(n + 1);
  DevArr<unsigned long long> tree_n(nt + 1);
  HIP_CHECK(hipMemsetAsync(tree_n.p, 0, (nt + 1ull) * 8, s));
  uint64_t T = 0;
  if (n) {
    hipLaunchKernelGGL(k_leaf_sizes, dim3(nblocks(n + 1, 256)), dim3(256), 0, s, pg, ntree->p, nfile->p, nptr->p, n,
                       lsize.p, tree_n.p);
    KCHECK("k_leaf_sizes");
    cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, lsize.p, loff.p, (int64_t)n + 1, s); });
    T = read_u64(loff.p + n, s);
  }
  DevArr<uint64_t> erid(T);
  DevArr<int32_t> eval(T);
  if (T) {
    hipLaunchKernelGGL(k_leaf_entries, dim3((unsigned)std::min<uint64_t>(nblocks(T, 256), 65536)), dim3(256), 0, s, pg,
                       nfile->p, nptr->p, n, loff.p, T, erid.p, eval.p, err);
    KCHECK("k_leaf_entries");
  }
  DevArr<uint64_t> teoff(nt + 1);
  cub_call(s, [&](void *t, size_t &b) {
    return hipcub::DeviceScan::ExclusiveSum(t, b, reinterpret_cast<uint64_t *>(tree_n.p), teoff.p, (int64_t)nt + 1, s);
  });
  // runs: the tree's entries plus its changes (upper bound when changes merge)
  DevArr<uint64_t> nruns(nt + 1);
  {
    std::vector<uint32_t> htv(nt);
    std::vector<uint32_t> hn(V);
    std::vector<uint64_t> hte(nt + 1), hr(nt + 1);
    HIP_CHECK(hipMemcpyAsync(htv.data(), tv.p, nt * 4ull, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(hn.data(), th.nchg, V * 4ull, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(hte.data(), teoff.p, (nt + 1ull) * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    for (uint32_t t = 0; t < nt; ++t) hr[t] = hte[t + 1] - hte[t] + hn[htv[t]];
    hr[nt] = 0;
    HIP_CHECK(hipMemcpyAsync(nruns.p, hr.data(), (nt + 1ull) * 8, hipMemcpyHostToDevice, s));
  }
  out.roff = std::make_unique<DevArr<uint64_t>>(nt + 1);
  cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, nruns.p, out.roff->p, (int64_t)nt + 1, s); });
  const uint64_t R = read_u64(out.roff->p + nt, s);
  out.R = R;
  out.rrid = std::make_unique<DevArr<uint64_t>>(R);
  out.rcnt = std::make_unique<DevArr<uint64_t>>(R);
  if (T) {
    hipLaunchKernelGGL(k_runs_copy, dim3((unsigned)std::min<uint64_t>(nblocks(T, 256), 65536)), dim3(256), 0, s, erid.p,
                       eval.p, T, teoff.p, nt, tv.p, th.nchg, out.roff->p, out.rrid->p, out.rcnt->p);
    KCHECK("k_runs_copy");
  }
  hipLaunchKernelGGL(k_runs_merge, dim3(nblocks(nt, 64)), dim3(64), 0, s, ds, erid.p, eval.p, teoff.p, tv.p, nt, th.nchg,
                     th.chg, out.roff->p, out.rrid->p, out.rcnt->p, err);
  KCHECK("k_runs_merge");
  // every tree row's count: Σ of its runs' counts
  DevArr<uint64_t> tsum(nt);
  if (R) {
    cub_call(s, [&](void *t, size_t &b) {
      return hipcub::DeviceSegmentedReduce::Sum(t, b, out.rcnt->p, tsum.p, (int)nt, out.roff->p, out.roff->p + 1, s);
    });
  } else {
    HIP_CHECK(hipMemsetAsync(tsum.p, 0, nt * 8ull, s));
  }
  hipLaunchKernelGGL(k_tree_row_counts, dim3(nblocks(nt, 256)), dim3(256), 0, s, tv.p, nt, tsum.p, cnt);
  KCHECK("k_tree_row_counts");
  out.tv = std::make_unique<DevArr<uint32_t>>(nt);
  HIP_CHECK(hipMemcpyAsync(out.tv->p, tv.p, nt * 4ull, hipMemcpyDeviceToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace

void ridbag_decode_csr(int device, const uint8_t *streams, uint64_t nbytes, const uint64_t *offsets, uint32_t V,
                       const uint64_t *vertex_rids, const uint64_t *edge_rids, const uint64_t *edge_targets,
                       uint64_t nedges, const omx_bonsai_file *files, int32_t nfiles, uint32_t page_size,
                       uint64_t *row_ptr, uint32_t *col, uint64_t *n_entries, uint64_t *entry_rids) {
  if (device < 0) fail(OMX_E_INVALID, "ridbag decoding runs on a device");
  if (entry_rids && !edge_rids) fail(OMX_E_INVALID, "entry_rids needs the edge records (edge_rids, edge_targets)");
  if (!offsets || !n_entries || (V && !vertex_rids) || (nbytes && !streams)) fail(OMX_E_INVALID, "null argument");
  if ((edge_rids == nullptr) != (edge_targets == nullptr)) fail(OMX_E_INVALID, "edge_rids and edge_targets go together");
  if (offsets[0] > offsets[V] || offsets[V] > nbytes) fail(OMX_E_INVALID, "stream offsets out of range");
  for (uint32_t v = 0; v < V; ++v)
    if (offsets[v + 1] < offsets[v]) fail(OMX_E_INVALID, "stream offsets not ascending");
  const bool trees = files != nullptr;
  if (nfiles < 0 || (nfiles > 0 && !files)) fail(OMX_E_INVALID, "bad collection file list");
  if (trees && (page_size < 128 || page_size > (1u << 24))) fail(OMX_E_INVALID, "bad page size");
  // the collection files, by ascending file id (pages of file f at base[f] in one device buffer)
  std::vector<int32_t> order(std::max(nfiles, 0));
  for (int32_t f = 0; f < nfiles; ++f) order[f] = f;
  std::sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return files[a].file_id < files[b].file_id; });
  std::vector<int64_t> hfid(std::max(nfiles, 1), 0);
  std::vector<uint64_t> hbase(std::max(nfiles, 1), 0), hnp(std::max(nfiles, 1), 0);
  uint64_t pbytes = 0;
  for (int32_t k = 0; k < nfiles; ++k) {
    const omx_bonsai_file &f = files[order[k]];
    if (k && f.file_id == hfid[k - 1]) fail(OMX_E_INVALID, "duplicate collection file id");
    if (f.n_pages && !f.pages) fail(OMX_E_INVALID, "null collection file pages");
    if (f.n_pages >= (1ull << 40)) fail(OMX_E_INVALID, "collection file too large");
    hfid[k] = f.file_id;
    hbase[k] = pbytes;
    hnp[k] = f.n_pages;
    pbytes += f.n_pages * (uint64_t)page_size;
  }
  HIP_CHECK(hipSetDevice(device));
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } sg{s};
  DevArr<uint8_t> ds(nbytes + 16);  // padding: the decoder reads whole dwords around an entry
  DevArr<uint64_t> doffs(V + 1ull), cnt(V + 1ull), rp(V + 1ull), pay(V + 1ull);
  DevArr<uint32_t> err(1);
  if (nbytes) HIP_CHECK(hipMemcpyAsync(ds.p, streams, nbytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(doffs.p, offsets, (V + 1ull) * 8, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
  // SBTree headers and the collection files' pages
  std::unique_ptr<DevArr<int32_t>> tfile;
  std::unique_ptr<DevArr<uint64_t>> troot, tchg, dbase, dnp;
  std::unique_ptr<DevArr<uint32_t>> tnchg;
  std::unique_ptr<DevArr<uint8_t>> tis, dpages;
  std::unique_ptr<DevArr<int64_t>> dfid;
  TreeHdr th{};
  Pages pg{};
  if (trees) {
    tfile.reset(new DevArr<int32_t>(V));
    troot.reset(new DevArr<uint64_t>(V));
    tchg.reset(new DevArr<uint64_t>(V));
    tnchg.reset(new DevArr<uint32_t>(V));
    tis.reset(new DevArr<uint8_t>(V));
    dfid.reset(new DevArr<int64_t>(hfid.size()));
    dbase.reset(new DevArr<uint64_t>(hbase.size()));
    dnp.reset(new DevArr<uint64_t>(hnp.size()));
    dpages.reset(new DevArr<uint8_t>(pbytes));
    HIP_CHECK(hipMemsetAsync(tnchg->p, 0, V * 4ull, s));
    HIP_CHECK(hipMemcpyAsync(dfid->p, hfid.data(), hfid.size() * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(dbase->p, hbase.data(), hbase.size() * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(dnp->p, hnp.data(), hnp.size() * 8, hipMemcpyHostToDevice, s));
    for (int32_t k = 0; k < nfiles; ++k)
      if (hnp[k])
        HIP_CHECK(hipMemcpyAsync(dpages->p + hbase[k], files[order[k]].pages, hnp[k] * (uint64_t)page_size,
                                 hipMemcpyHostToDevice, s));
    th = TreeHdr{tfile->p, troot->p, tnchg->p, tchg->p, tis->p, dfid->p, dnp->p, nfiles, page_size};
    pg = Pages{dpages->p, dbase->p, dnp->p, page_size};
  }
  hipLaunchKernelGGL(k_bag_count, dim3(nblocks(V + 1ull, 256)), dim3(256), 0, s, ds.p, doffs.p, V, cnt.p, pay.p, err.p, th,
                     trees ? 1 : 0);
  KCHECK("k_bag_count");
  uint32_t herr = read_err(err.p, s);
  if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
  TreeRuns tr;
  if (trees) {
    decode_trees(s, ds.p, V, th, tis->p, pg, cnt.p, err.p, tr);
    herr = read_err(err.p, s);
    if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
  }
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.p, rp.p, (int64_t)V + 1, s));
  DevArr<uint8_t> tmp(tb);
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, cnt.p, rp.p, (int64_t)V + 1, s));
  uint64_t E = 0;
  HIP_CHECK(hipMemcpyAsync(&E, rp.p + V, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  *n_entries = E;
  if (row_ptr) HIP_CHECK(hipMemcpyAsync(row_ptr, rp.p, (V + 1ull) * 8, hipMemcpyDeviceToHost, s));
  if (!col) {
    HIP_CHECK(hipStreamSynchronize(s));
    return;
  }
  // RID indexes of the vertices (→ dense id) and of the edge records (→ opposite vertex RID)
  HostIndex<uint32_t> vix;
  build_index<uint32_t>(vix, vertex_rids, nullptr, V, s);
  HostIndex<uint64_t> eix;
  if (edge_rids) build_index<uint64_t>(eix, edge_rids, edge_targets, nedges, s);
  DevArr<uint32_t> dcol(E);
  std::unique_ptr<DevArr<uint64_t>> derid;
  if (entry_rids) derid.reset(new DevArr<uint64_t>(E));
  uint64_t *erp = entry_rids ? derid->p : nullptr;
  if (E) {
    const unsigned grid = (unsigned)std::min<uint64_t>((E + kDecTile - 1) / kDecTile, 65536);
    hipLaunchKernelGGL(k_bag_decode, dim3(grid), dim3(kDecB), 0, s, ds.p, pay.p, V, rp.p, E, vix.dev, eix.dev,
                       edge_rids ? 1 : 0, dcol.p, err.p, erp);
    KCHECK("k_bag_decode");
  }
  if (tr.R) {  // the SBTree rows: every run's RID `count` times at its place in the row
    DevArr<uint64_t> ro(tr.R + 1);
    cub_call(s, [&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, tr.rcnt->p, ro.p, (int64_t)tr.R, s); });
    hipLaunchKernelGGL(k_runs_write, dim3((unsigned)std::min<uint64_t>(nblocks(tr.R, 256), 65536)), dim3(256), 0, s,
                       tr.rrid->p, tr.rcnt->p, tr.R, ro.p, tr.roff->p, tr.nt, tr.tv->p, rp.p, vix.dev, eix.dev,
                       edge_rids ? 1 : 0, dcol.p, err.p, erp);
    KCHECK("k_runs_write");
  }
  if (E) HIP_CHECK(hipMemcpyAsync(col, dcol.p, E * 4, hipMemcpyDeviceToHost, s));
  if (E && entry_rids) HIP_CHECK(hipMemcpyAsync(entry_rids, erp, E * 8, hipMemcpyDeviceToHost, s));
  herr = read_err(err.p, s);
  if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
}

}  // namespace omx
