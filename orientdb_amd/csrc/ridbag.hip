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
#include <cstring>
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

// payload offset of a stream the count pass accepted
__device__ __forceinline__ uint64_t bag_payload(const uint8_t *s, const uint64_t *offs, uint32_t v) {
  const uint64_t b = offs[v];
  return b + 1 + ((s[b] & 2) ? 16 : 0) + 4;
}

__global__ void k_bag_count(const uint8_t *s, const uint64_t *offs, uint32_t V, uint64_t *cnt, uint32_t *err) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v > V) return;
  if (v == V) {
    cnt[V] = 0;
    return;
  }
  uint64_t p;
  cnt[v] = bag_header(s, offs, (uint32_t)v, &p, err);
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

__global__ void k_bag_decode(const uint8_t *s, const uint64_t *offs, uint32_t V, const uint64_t *rp, uint64_t E,
                             const uint64_t *vrid, const uint32_t *vdense, const uint64_t *erid, const uint64_t *etarget,
                             uint64_t nedges, uint32_t *col, uint32_t *err) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    // the vertex whose row holds entry e: last v with rp[v] <= e
    uint64_t lo = 0, hi = V;
    while (lo < hi) {
      const uint64_t mid = (lo + hi + 1) >> 1;
      if (rp[mid] <= e) lo = mid;
      else hi = mid - 1;
    }
    const uint32_t v = (uint32_t)lo;
    const uint8_t *p = s + bag_payload(s, offs, v) + 10ull * (e - rp[v]);
    const int16_t cl = (int16_t)(((uint32_t)p[0] << 8) | p[1]);
    const uint64_t pos = be64(p + 2);
    uint32_t out = 0xFFFFFFFFu;
    if (cl < 0 || (pos >> 48)) {
      atomicOr(err, (uint32_t)kBagPosition);
    } else {
      uint64_t rid = ((uint64_t)(uint16_t)cl << 48) | pos;
      bool ok = true;
      if (erid) {  // an edge record: its opposite vertex
        const uint64_t i = find_sorted(erid, nedges, rid);
        if (i == nedges) {
          atomicOr(err, (uint32_t)kBagUnknownEdge);
          ok = false;
        } else {
          rid = etarget[i];
        }
      }
      if (ok) {
        const uint64_t i = find_sorted(vrid, V, rid);
        if (i == V) atomicOr(err, (uint32_t)kBagUnknownRid);
        else out = vdense[i];
      }
    }
    col[e] = out;
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
  DevArr<uint8_t> ds(nbytes);
  DevArr<uint64_t> doffs(V + 1ull), cnt(V + 1ull), rp(V + 1ull);
  DevArr<uint32_t> err(1);
  if (nbytes) HIP_CHECK(hipMemcpyAsync(ds.p, streams, nbytes, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(doffs.p, offsets, (V + 1ull) * 8, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
  hipLaunchKernelGGL(k_bag_count, dim3(nblocks(V + 1ull, 256)), dim3(256), 0, s, ds.p, doffs.p, V, cnt.p, err.p);
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
  // RID-sorted vertex table (and edge table): the decoder's binary searches
  DevArr<uint64_t> vr(V), vrs(V);
  DevArr<uint32_t> vd(V), vds(V);
  if (V) {
    HIP_CHECK(hipMemcpyAsync(vr.p, vertex_rids, (uint64_t)V * 8, hipMemcpyHostToDevice, s));
    std::vector<uint32_t> iota(V);
    for (uint32_t v = 0; v < V; ++v) iota[v] = v;
    HIP_CHECK(hipMemcpyAsync(vd.p, iota.data(), (uint64_t)V * 4, hipMemcpyHostToDevice, s));
    size_t sb = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, vr.p, vrs.p, vd.p, vds.p, (int64_t)V, 0, 64, s));
    DevArr<uint8_t> stmp(sb);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(stmp.p, sb, vr.p, vrs.p, vd.p, vds.p, (int64_t)V, 0, 64, s));
    HIP_CHECK(hipStreamSynchronize(s));  // iota leaves scope
  }
  DevArr<uint64_t> er(nedges), ers(nedges), et(nedges), ets(nedges);
  if (edge_rids && nedges) {
    HIP_CHECK(hipMemcpyAsync(er.p, edge_rids, nedges * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(et.p, edge_targets, nedges * 8, hipMemcpyHostToDevice, s));
    size_t sb = 0;
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sb, er.p, ers.p, et.p, ets.p, (int64_t)nedges, 0, 64, s));
    DevArr<uint8_t> stmp(sb);
    HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(stmp.p, sb, er.p, ers.p, et.p, ets.p, (int64_t)nedges, 0, 64, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  DevArr<uint32_t> dcol(E);
  if (E) {
    const unsigned grid = (unsigned)std::min<uint64_t>(nblocks(E, 256), 65536);
    hipLaunchKernelGGL(k_bag_decode, dim3(grid), dim3(256), 0, s, ds.p, doffs.p, V, rp.p, E, vrs.p, vds.p,
                       edge_rids ? ers.p : nullptr, edge_rids ? ets.p : nullptr, nedges, dcol.p, err.p);
    KCHECK("k_bag_decode");
    HIP_CHECK(hipMemcpyAsync(col, dcol.p, E * 4, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (herr) fail(OMX_E_INVALID, "ridbag streams:" + bag_error_text(herr));
}

}  // namespace omx
