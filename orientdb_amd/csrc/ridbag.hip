// ridbag.hip — device decoding of serialized ridbags into a CSR (include/omx/match.h
// omx_ridbag_decode_csr).
//
// An OrientDB vertex keeps each edge class's adjacency in an out_<L> / in_<L> ridbag field. The record
// serializer writes an embedded bag as (C/db/record/ridbag/ORidBag.java:198-276 toStream,
// C/db/record/ridbag/embedded/OEmbeddedRidBag.java:424-460 serialize, C/serialization/serializer/
// binary/impl/OLinkSerializer.java:54-58, OIntegerSerializer.java:53-58 — all big-endian):
//   [1 B config: bit 0 embedded, bit 1 UUID follows][16 B UUID if bit 1]
//   [int32 count][count × (int16 cluster id, int64 cluster position)]
// An SBTree bag (config bit 0 clear) holds a pointer to an on-disk B-tree, not its entries: it cannot be
// decoded from the record bytes and is rejected.
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
};

__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}
__device__ __forceinline__ uint64_t be64(const uint8_t *p) {
  return ((uint64_t)be32(p) << 32) | (uint64_t)be32(p + 4);
}

// header of vertex v's stream: payload offset and entry count (0 for an empty stream = no field)
__device__ __forceinline__ uint32_t bag_header(const uint8_t *s, const uint64_t *offs, uint32_t v, uint64_t *payload,
                                               uint32_t *err) {
  const uint64_t b = offs[v], e = offs[v + 1];
  *payload = b;
  if (e <= b) return 0;
  const uint8_t cfg = s[b];
  if (!(cfg & 1)) {
    atomicOr(err, (uint32_t)kBagSBTree);
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
                            uint32_t *err) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v > V) return;
  if (v == V) {
    cnt[V] = 0;
    return;
  }
  uint64_t p;
  cnt[v] = bag_header(s, offs, (uint32_t)v, &p, err);
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
                                                      RidIndex<uint64_t> eix, int edges, uint32_t *col, uint32_t *err) {
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
        off[k] = s_pay[lo] + 10ull * (e - s_rp[lo]);
      } else {
        while (lo < hi) {
          const uint64_t mid = (lo + hi + 1) >> 1;
          if (rp[r0 + mid] <= e) lo = mid;
          else hi = mid - 1;
        }
        off[k] = pay[r0 + lo] + 10ull * (e - rp[r0 + lo]);
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

std::string bag_error_text(uint32_t e) {
  std::string m;
  if (e & kBagSBTree) m += " an SBTree (non-embedded) ridbag, whose entries are not in the record;";
  if (e & kBagTruncated) m += " a stream shorter than its header and count;";
  if (e & kBagPosition) m += " a RID with a negative cluster or a position of 2^48 or more;";
  if (e & kBagUnknownEdge) m += " an edge RID missing from the edge table;";
  if (e & kBagUnknownRid) m += " a RID that is no vertex of the snapshot;";
  return m;
}

}  // namespace

void ridbag_decode_csr(int device, const uint8_t *streams, uint64_t nbytes, const uint64_t *offsets, uint32_t V,
                       const uint64_t *vertex_rids, const uint64_t *edge_rids, const uint64_t *edge_targets,
                       uint64_t nedges, uint64_t *row_ptr, uint32_t *col, uint64_t *n_entries) {
  if (device < 0) fail(OMX_E_INVALID, "ridbag decoding runs on a device");
  if (!offsets || !n_entries || (V && !vertex_rids) || (nbytes && !streams)) fail(OMX_E_INVALID, "null argument");
  if ((edge_rids == nullptr) != (edge_targets == nullptr)) fail(OMX_E_INVALID, "edge_rids and edge_targets go together");
  if (offsets[0] > offsets[V] || offsets[V] > nbytes) fail(OMX_E_INVALID, "stream offsets out of range");
  for (uint32_t v = 0; v < V; ++v)
    if (offsets[v + 1] < offsets[v]) fail(OMX_E_INVALID, "stream offsets not ascending");
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
  hipLaunchKernelGGL(k_bag_count, dim3(nblocks(V + 1ull, 256)), dim3(256), 0, s, ds.p, doffs.p, V, cnt.p, pay.p, err.p);
  KCHECK("k_bag_count");
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt.p, rp.p, (int64_t)V + 1, s));
  DevArr<uint8_t> tmp(tb);
  HIP_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, cnt.p, rp.p, (int64_t)V + 1, s));
  uint64_t E = 0;
  uint32_t herr = 0;
  HIP_CHECK(hipMemcpyAsync(&E, rp.p + V, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
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
  if (E) {
    const unsigned grid = (unsigned)std::min<uint64_t>((E + kDecTile - 1) / kDecTile, 65536);
    hipLaunchKernelGGL(k_bag_decode, dim3(grid), dim3(kDecB), 0, s, ds.p, pay.p, V, rp.p, E, vix.dev, eix.dev,
                       edge_rids ? 1 : 0, dcol.p, err.p);
    KCHECK("k_bag_decode");
    HIP_CHECK(hipMemcpyAsync(col, dcol.p, E * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
}

}  // namespace omx
