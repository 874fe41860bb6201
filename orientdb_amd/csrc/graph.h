// graph.h — the immutable HBM snapshot of a database's vertices, ridbags and properties.
//
// Replaces the lazy record/ridbag reads of the reference's DFS (ORidBag.rawIterator
// C/db/record/ridbag/ORidBag.java:160, OrientVertex.getVertices B/OrientVertex.java:401-460,
// ODocument.field C/record/impl/ODocument.java:820) with one snapshot per database state:
//   * per edge class: out-CSR and in-CSR (u64 row_ptr, u32 dense vertex ids), rows sorted;
//   * class_id u16 per vertex, RID u64 per vertex;
//   * one column per property (int32 / int64 / double / dictionary-coded string) + presence bytes.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"
#include "devtypes.h"

#define HIP_CHECK(x)                                                                                    \
  do {                                                                                                  \
    hipError_t e_ = (x);                                                                                \
    if (e_ != hipSuccess) ::omx::fail(OMX_E_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_));     \
  } while (0)

namespace omx {

// Caching device allocator: execution buffers are recycled between queries so that a steady-state
// omx_execute issues no hipMalloc/hipFree (Guideline 9 of the CDNA HIP guide).
class DevicePool {
 public:
  void *alloc(size_t bytes);
  void release(void *p);
  void trim();
  ~DevicePool();
  size_t cached_bytes() const { return cached_; }
  // bytes of the live allocation starting at p (0 if p is not one)
  size_t size_of(const void *p) const {
    auto it = live_.find(const_cast<void *>(p));
    return it == live_.end() ? 0 : it->second;
  }

 private:
  std::multimap<size_t, void *> free_;
  std::unordered_map<void *, size_t> live_;
  size_t cached_ = 0;
};

// Process-wide pool of pinned host blocks that back result rows (omx_result_rows, SURVEY §8(b) Ownership:
// a library-owned pinned buffer released by omx_result_free). A block is never value-initialised; a freed
// one goes back to the pool (up to OMX_PINNED_CACHE_GB, default 64 GiB, cached) and the next result of
// a similar size reuses it, so a steady-state hand-over neither pins nor zeroes host pages. Process-wide
// rather than per graph: a result may outlive its snapshot. If pinning fails the block is pageable
// (malloc, also uninitialised); *pinned says which.
void *host_rows_acquire(size_t bytes, size_t *capacity, bool *pinned);
void host_rows_release(void *p);
size_t host_rows_cached_bytes();

// OMX_POOL_POISON=1 (debug): every buffer DevicePool::alloc hands out, fresh or reused, is filled with 0xFF
// bytes first, so a kernel that reads a scratch word it never wrote sees 0xFFFFFFFF, not a lucky zero
bool pool_poison();

template <class T>
struct DBuf {
  DevicePool *pool = nullptr;
  T *p = nullptr;
  size_t n = 0;
  DBuf() = default;
  DBuf(DevicePool *pl, size_t count) : pool(pl), n(count) {
    p = count ? (T *)pool->alloc(count * sizeof(T)) : nullptr;
  }
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  DBuf(DBuf &&o) noexcept { *this = std::move(o); }
  DBuf &operator=(DBuf &&o) noexcept {
    if (this != &o) {
      reset();
      pool = o.pool; p = o.p; n = o.n;
      o.p = nullptr; o.n = 0;
    }
    return *this;
  }
  ~DBuf() { reset(); }
  void reset() {
    if (p && pool) pool->release(p);
    p = nullptr;
    n = 0;
  }
};

struct ClassInfo {
  std::string name;
  int super = -1;
  bool is_edge = false;
  int cluster = 0;
  uint64_t exact_count = 0;     // vertices whose class is exactly this one
  std::vector<int> poly;        // this class and every subclass (polymorphic set)
};

struct EdgeSet {
  int cls = -1;
  // 0: an edge class's adjacency (vertex → vertex). Snapshots with edge records (Graph::edge_records) add
  // 1: that class's edge records (out: vertex → the ids of its out-edges, in: vertex → its in-edges) and
  // 2 (one set): every record's endpoints (out: edge → its out-vertex, outV(); in: edge → its in-vertex, inV())
  int pseudo = 0;
  uint64_t n_edges = 0;     // out CSR edges (of the owned rows)
  uint64_t n_in_edges = 0;  // in CSR edges (of the owned rows)
  bool out_sorted = true, in_sorted = true;  // rows ascending
  bool out_simple = true, in_simple = true;  // rows strictly ascending (no parallel edges)
  uint64_t max_deg[2] = {0, 0};               // the longest row of the out / in CSR (of the owned rows)
  uint64_t *d_out_rp = nullptr, *d_in_rp = nullptr;
  uint32_t *d_out_col = nullptr, *d_in_col = nullptr;
  // slice-cut index of a CSR (0 = out, 1 = in), per slice shift: for every vertex, the offsets inside
  // its sorted row where neighbours reach q·2^shift (q = 1…P−1); built on the first filtered hop
  // that uses the CSR (a property of the immutable snapshot, like the sort order)
  std::map<uint32_t, uint32_t *> d_cuts[2];
  // hub-annotated copy of a CSR's col (0 = out, 1 = in) for the bottom-up BFS (bfs.hip k_bfs_pull):
  // a neighbour that is one of the n_hubs vertices of highest degree in the opposite CSR is stored as
  // 0x80000000 | its hub index, so its frontier mask is read from a small L2-resident hub array;
  // built on the first pull level over the CSR
  uint32_t *d_pull_col[2] = {nullptr, nullptr};
  uint32_t *d_hubs[2] = {nullptr, nullptr};
  uint64_t *d_hub_bm[2] = {nullptr, nullptr};  // the hubs as a V-bit set (built with d_pull_col)
  uint32_t n_hubs[2] = {0, 0};
  uint64_t hub_entries[2] = {0, 0};     // entries of d_pull_col that name a hub (the hub CSR's size)
  uint32_t hubs_requested[2] = {0, 0};  // the hub budget d_pull_col was built with (rebuilt when it changes)
  // merge-path split of the CSR into pull tiles (bfs.hip k_pull_partition), built with d_pull_col
  uint64_t *d_pull_part[2] = {nullptr, nullptr};
  // in-edge wave tiles of the CSR (bfs.hip k_bfs_pull_w): first / last vertex of every tile, and the tile
  // indices with the regular tiles (full, ≤ 256 vertices) first
  uint64_t *d_pullw_rb[2] = {nullptr, nullptr};
  uint32_t *d_pullw_tiles[2] = {nullptr, nullptr};
  uint64_t pullw_nreg[2] = {0, 0};
  // the hub entries alone, as a CSR (row v: the entries of d_pull_col's row v that name a hub, in order)
  // with its own wave tiles: what a hubs-only pull level reads (built with d_pull_col)
  uint64_t *d_hub_rp[2] = {nullptr, nullptr};
  uint32_t *d_hub_col[2] = {nullptr, nullptr};
  uint64_t *d_hubw_rb[2] = {nullptr, nullptr};
  uint32_t *d_hubw_tiles[2] = {nullptr, nullptr};
  uint64_t hubw_nreg[2] = {0, 0};
  // lists col of a CSR for the factorized hop's filtered lists (factor.hip k_flists): as d_pull_col, with
  // the kFlistHubs vertices of highest degree in the opposite CSR as hubs, a hub's entry list_vb + its rank
  // (its filter bit is read from a small, cache-resident array); built on the first factorized hop over
  // the CSR
  uint32_t *d_list_col[2] = {nullptr, nullptr};
  uint32_t list_vb[2] = {0, 0};
  uint32_t *d_list_hubs[2] = {nullptr, nullptr};
  uint32_t n_list_hubs[2] = {0, 0};
  // partitioned snapshot: row pointers of every vertex's degree (V + 1 entries, the scan of all ranks'
  // degrees gathered once) — what out()/in()/both().size() in a WHERE reads (no col[] behind them)
  uint64_t *d_global_rp[2] = {nullptr, nullptr};
};

struct Property {
  std::string name;
  int type = 0;
  std::vector<std::string> dict;        // strings, sorted
  bool has_nulls = false;
  // absent on some vertex / some edge record (edge_records: a vertex field is absent on every edge)
  bool nulls_v = false, nulls_e = false;
  void *d_values = nullptr;
  uint8_t *d_present = nullptr;
  // host copy kept only for indexed properties (root estimation, OWhereClause.estimate)
  std::vector<int64_t> h_int;
  std::vector<double> h_dbl;
  std::vector<uint8_t> h_present;
};

struct IndexInfo {
  int cls;
  int prop;
  bool unique;
};

struct Graph {
  uint64_t uid = 0;  // process-unique id (plan caches key on it, not on the address)
  uint32_t V = 0;  // records: vertices, then (edge_records) the edge records, ids [vertices, V)
  uint32_t vertices = 0;
  bool edge_records = false;
  int device = -1;
  // 1-D partition: the CSR rows held are those of [part_lo, part_hi) (local row pointers); the
  // device row-pointer arrays are addressed with a global vertex id through rp(): base − part_lo
  uint32_t part_lo = 0, part_hi = 0;
  bool partitioned() const { return part_lo != 0 || part_hi != V; }
  std::vector<ClassInfo> classes;
  std::vector<EdgeSet> esets;
  std::vector<Property> props;
  std::vector<IndexInfo> indexes;
  std::vector<uint16_t> h_vclass;  // kept when indexes exist, or copied on the first RETURN expression
  std::vector<uint64_t> h_rids;    // copied on the first RETURN expression (project.cpp)
  // edge records: every record's out- / in-vertex (the edge document's `out` / `in` links), copied from
  // the endpoints set on the first RETURN expression that reads them (project.cpp)
  std::vector<uint32_t> h_etail, h_ehead;
  uint16_t *d_vclass = nullptr;
  uint64_t *d_rids = nullptr;
  DColumn *d_cols = nullptr;
  uint64_t device_bytes = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // side stream: light-row expansion runs beside the heavy-row one
  DevicePool pool;
  uint64_t *h_stage = nullptr;             // pinned host words for small device→host reads
  static constexpr int kStageWords = 512;
  uint64_t *h_mail = nullptr;              // fine-grained pinned host mailbox (kernels.h Mail)
  uint64_t mail_seq = 0;
  std::vector<hipEvent_t> event_pool;      // reusable timing events (OMX_FLAG_KERNEL_TIMING)

  // row pointers indexed by a global (owned) vertex id; dir 0 = out, 1 = in
  const uint64_t *rp(const EdgeSet &e, int dir) const { return (dir == 0 ? e.d_out_rp : e.d_in_rp) - part_lo; }
  const uint32_t *col(const EdgeSet &e, int dir) const { return dir == 0 ? e.d_out_col : e.d_in_col; }

  ~Graph();
  bool on_device() const { return device >= 0; }
  int class_id(const std::string &name) const;        // case-insensitive, -1 if absent
  int prop_id(const std::string &name) const;         // exact, -1 if absent
  bool is_subclass_of(int c, int sup) const;
  uint64_t count(int c) const;                         // OClassImpl.count() (polymorphic)
  void class_mask(int c, uint64_t mask[4]) const;      // polymorphic set as a 256-bit mask
  // index lookup size for prop == value over the polymorphic class (OWhereClause.estimateFromIndex)
  int64_t index_hits(int cls, int prop, const struct Value &v) const;
};

Graph *graph_create(const omx_graph_desc *d);
// ridbag.hip: omx_ridbag_decode_csr / omx_ridbag_decode_csr_ex (files = NULL: embedded bags only)
void ridbag_decode_csr(int device, const uint8_t *streams, uint64_t nbytes, const uint64_t *offsets, uint32_t V,
                       const uint64_t *vertex_rids, const uint64_t *edge_rids, const uint64_t *edge_targets,
                       uint64_t nedges, const omx_bonsai_file *files, int32_t nfiles, uint32_t page_size,
                       uint64_t *row_ptr, uint32_t *col, uint64_t *n_entries, uint64_t *entry_rids = nullptr);

}  // namespace omx
