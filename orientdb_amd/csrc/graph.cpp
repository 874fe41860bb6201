// graph.cpp — snapshot validation, host-side statistics and upload to HBM.
#include "graph.h"

#include <set>

#include <algorithm>
#include <atomic>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "kernels.h"
#include "sql.h"

namespace omx {

// ---- device pool -----------------------------------------------------------------------------------

static size_t round_size(size_t b) {
  if (b <= 4096) return 4096;
  if (b <= (1u << 20)) {  // power of two up to 1 MiB
    size_t r = 4096;
    while (r < b) r <<= 1;
    return r;
  }
  const size_t g = 2u << 20;  // 2 MiB granules above
  return (b + g - 1) / g * g;
}

bool pool_poison() {  // read on every allocation, so a test can switch it within one process
  const char *e = std::getenv("OMX_POOL_POISON");
  return e && std::strcmp(e, "0") != 0;
}

// the whole device is drained first: a reused buffer may still be read by a kernel queued on any stream
static void poison_fill(void *p, size_t bytes) {
  if (!pool_poison()) return;
  if (hipDeviceSynchronize() != hipSuccess || hipMemset(p, 0xFF, bytes) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
    fail(OMX_E_DEVICE, std::string("OMX_POOL_POISON fill failed: ") + hipGetErrorString(hipGetLastError()));
}

void *DevicePool::alloc(size_t bytes) {
  size_t sz = round_size(bytes);
  auto it = free_.lower_bound(sz);
  if (it != free_.end() && it->first <= sz + sz / 4 + (2u << 20)) {
    void *p = it->second;
    live_[p] = it->first;
    cached_ -= it->first;
    free_.erase(it);
    poison_fill(p, live_[p]);
    return p;
  }
  void *p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) {
    (void)hipGetLastError();
    trim();
    if (hipMalloc(&p, sz) != hipSuccess) {
      (void)hipGetLastError();
      fail(OMX_E_OOM, "device allocation of " + std::to_string(sz) + " bytes failed");
    }
  }
  live_[p] = sz;
  poison_fill(p, sz);
  return p;
}

void DevicePool::release(void *p) {
  auto it = live_.find(p);
  if (it == live_.end()) return;
  free_.emplace(it->second, p);
  cached_ += it->second;
  live_.erase(it);
}

void DevicePool::trim() {
  for (auto &kv : free_) (void)hipFree(kv.second);
  free_.clear();
  cached_ = 0;
}

DevicePool::~DevicePool() {
  trim();
  for (auto &kv : live_) (void)hipFree(kv.first);
}

// ---- host blocks for result rows -------------------------------------------------------------------

namespace {
struct HostRows {
  std::mutex mu;
  std::multimap<size_t, void *> free_;                         // capacity → block
  std::unordered_map<void *, std::pair<size_t, bool>> live_;  // block → (capacity, pinned)
  std::unordered_map<void *, bool> pinned_free_;               // cached block → pinned
  size_t cached = 0;
  size_t limit = [] {
    const char *e = std::getenv("OMX_PINNED_CACHE_GB");
    return (size_t)(e ? std::strtod(e, nullptr) : 64.0) << 30;
  }();
  static void drop(void *p, bool pinned) {
    if (pinned) (void)hipHostFree(p);
    else std::free(p);
  }
  ~HostRows() {
    for (auto &kv : free_) drop(kv.second, pinned_free_[kv.second]);
  }
};
HostRows &host_rows() {
  static HostRows *h = new HostRows;  // never destroyed: results may be freed during static teardown
  return *h;
}
}  // namespace

void *host_rows_acquire(size_t bytes, size_t *capacity, bool *pinned) {
  HostRows &h = host_rows();
  const size_t g = 2u << 20;
  const size_t sz = std::max<size_t>(g, (bytes + g - 1) / g * g);
  {
    std::lock_guard<std::mutex> lk(h.mu);
    // a cached block of at least sz and at most 2·sz (+64 MiB) bytes
    auto it = h.free_.lower_bound(sz);
    if (it != h.free_.end() && it->first <= 2 * sz + (64u << 20)) {
      void *p = it->second;
      const size_t cap = it->first;
      const bool pin = h.pinned_free_[p];
      h.pinned_free_.erase(p);
      h.live_[p] = {cap, pin};
      h.cached -= cap;
      h.free_.erase(it);
      *capacity = cap;
      *pinned = pin;
      return p;
    }
  }
  void *p = nullptr;
  bool pin = true;
  if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess || !p) {
    (void)hipGetLastError();
    // trim the cache and try again, then fall back to pageable memory
    {
      std::lock_guard<std::mutex> lk(h.mu);
      for (auto &kv : h.free_) HostRows::drop(kv.second, h.pinned_free_[kv.second]);
      h.free_.clear();
      h.pinned_free_.clear();
      h.cached = 0;
    }
    p = nullptr;
    if (hipHostMalloc(&p, sz, hipHostMallocDefault) != hipSuccess || !p) {
      (void)hipGetLastError();
      pin = false;
      p = std::malloc(sz);
      if (!p) fail(OMX_E_OOM, "host allocation of " + std::to_string(sz) + " result bytes failed");
    }
  }
  std::lock_guard<std::mutex> lk(h.mu);
  h.live_[p] = {sz, pin};
  *capacity = sz;
  *pinned = pin;
  return p;
}

void host_rows_release(void *p) {
  if (!p) return;
  HostRows &h = host_rows();
  std::lock_guard<std::mutex> lk(h.mu);
  auto it = h.live_.find(p);
  if (it == h.live_.end()) return;
  const size_t cap = it->second.first;
  const bool pin = it->second.second;
  h.live_.erase(it);
  if (cap > h.limit) {
    HostRows::drop(p, pin);
    return;
  }
  // evict the largest cached blocks until this one fits under the limit
  while (h.cached + cap > h.limit && !h.free_.empty()) {
    auto last = std::prev(h.free_.end());
    HostRows::drop(last->second, h.pinned_free_[last->second]);
    h.pinned_free_.erase(last->second);
    h.cached -= last->first;
    h.free_.erase(last);
  }
  h.free_.emplace(cap, p);
  h.pinned_free_[p] = pin;
  h.cached += cap;
}

size_t host_rows_cached_bytes() {
  HostRows &h = host_rows();
  std::lock_guard<std::mutex> lk(h.mu);
  return h.cached;
}

// ---- graph -----------------------------------------------------------------------------------------

Graph::~Graph() {
  if (device >= 0) {
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    auto f = [](void *p) { if (p) (void)hipFree(p); };
    f(d_vclass);
    f(d_rids);
    f(d_cols);
    for (auto &e : esets) {
      f(e.d_out_rp); f(e.d_in_rp); f(e.d_out_col); f(e.d_in_col);
      for (auto &m : e.d_cuts)
        for (auto &kv : m) f(kv.second);
      for (int d = 0; d < 2; ++d) {
        f(e.d_pull_col[d]); f(e.d_hubs[d]); f(e.d_hub_bm[d]); f(e.d_pull_part[d]); f(e.d_global_rp[d]);
        f(e.d_pullw_rb[d]); f(e.d_pullw_tiles[d]); f(e.d_hub_rp[d]); f(e.d_hub_col[d]); f(e.d_hubw_rb[d]); f(e.d_hubw_tiles[d]);
        f(e.d_list_col[d]); f(e.d_list_hubs[d]);
      }
    }
    for (auto &p : props) { f(p.d_values); f(p.d_present); }
    if (stream) (void)hipStreamDestroy(stream);
    if (stream2) (void)hipStreamDestroy(stream2);
    if (h_stage) (void)hipHostFree(h_stage);
    if (h_mail) (void)hipHostFree(h_mail);
    for (hipEvent_t e : event_pool) (void)hipEventDestroy(e);
  }
}

int Graph::class_id(const std::string &name) const {
  for (size_t i = 0; i < classes.size(); ++i)
    if (classes[i].name == name) return (int)i;
  for (size_t i = 0; i < classes.size(); ++i)
    if (ieq(classes[i].name, name)) return (int)i;
  return -1;
}

int Graph::prop_id(const std::string &name) const {
  for (size_t i = 0; i < props.size(); ++i)
    if (props[i].name == name) return (int)i;
  return -1;
}

bool Graph::is_subclass_of(int c, int sup) const {
  while (c >= 0) {
    if (c == sup) return true;
    c = classes[c].super;
  }
  return false;
}

uint64_t Graph::count(int c) const {
  uint64_t n = 0;
  for (int x : classes[c].poly) n += classes[x].exact_count;
  return n;
}

void Graph::class_mask(int c, uint64_t mask[4]) const {
  mask[0] = mask[1] = mask[2] = mask[3] = 0;
  for (int x : classes[c].poly) mask[x >> 6] |= 1ull << (x & 63);
}

int64_t Graph::index_hits(int cls, int prop, const Value &v) const {
  const Property &p = props[prop];
  int64_t n = 0;
  uint64_t mask[4];
  class_mask(cls, mask);
  for (uint32_t i = 0; i < V; ++i) {
    int c = h_vclass[i];
    if (!((mask[c >> 6] >> (c & 63)) & 1)) continue;
    if (!p.h_present.empty() && !p.h_present[i]) continue;
    bool eq = false;
    if (p.type == OMX_PROP_DOUBLE) {
      double x = p.h_dbl[i];
      eq = (v.kind == Value::INT && x == (double)v.i) || (v.kind == Value::DBL && x == v.d);
    } else if (p.type == OMX_PROP_STRING) {
      eq = v.kind == Value::STR && p.h_int[i] >= 0 && p.dict[p.h_int[i]] == v.s;
    } else {
      int64_t x = p.h_int[i];
      eq = (v.kind == Value::INT && x == v.i) || (v.kind == Value::DBL && (double)x == v.d) ||
           (v.kind == Value::BOOL && x == v.i);
    }
    n += eq;
  }
  return n;
}

// ---- creation --------------------------------------------------------------------------------------

template <class F>
static void parallel_for(uint64_t n, F f) {
  unsigned nt = host_threads();
  if (n < 65536) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([=]() {
      uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
      f(lo, hi);
    });
  for (auto &x : th) x.join();
}

// Checks row order; returns (sorted, simple).
static std::pair<bool, bool> scan_rows(uint32_t V, const uint64_t *rp, const uint32_t *col) {
  std::atomic<bool> sorted{true}, simple{true};
  parallel_for(V, [&](uint64_t lo, uint64_t hi) {
    bool so = true, si = true;
    for (uint64_t v = lo; v < hi; ++v)
      for (uint64_t e = rp[v] + 1; e < rp[v + 1]; ++e) {
        if (col[e - 1] > col[e]) so = false;
        if (col[e - 1] >= col[e]) si = false;
      }
    if (!so) sorted = false;
    if (!si) simple = false;
  });
  return {sorted.load(), simple.load()};
}

// the longest row of a CSR (EdgeSet::max_deg)
static uint64_t max_row(uint32_t V, const uint64_t *rp) {
  std::atomic<uint64_t> m{0};
  parallel_for(V, [&](uint64_t lo, uint64_t hi) {
    uint64_t x = 0;
    for (uint64_t v = lo; v < hi; ++v) x = std::max(x, rp[v + 1] - rp[v]);
    uint64_t cur = m.load();
    while (x > cur && !m.compare_exchange_weak(cur, x)) {
    }
  });
  return m.load();
}

static void sort_rows(uint32_t V, const uint64_t *rp, uint32_t *col) {
  parallel_for(V, [&](uint64_t lo, uint64_t hi) {
    for (uint64_t v = lo; v < hi; ++v) std::sort(col + rp[v], col + rp[v + 1]);
  });
}

template <class T>
static T *upload(const T *h, size_t n, uint64_t &acc) {
  if (n == 0) n = 1;
  T *d = nullptr;
  HIP_CHECK(hipMalloc(&d, n * sizeof(T)));
  if (h) HIP_CHECK(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
  else HIP_CHECK(hipMemset(d, 0, n * sizeof(T)));
  acc += n * sizeof(T);
  return d;
}

extern "C" int omx_csr_transpose(uint32_t, const uint64_t *, const uint32_t *, uint64_t **, uint32_t **);

static Graph *create_snapshot(const omx_graph_desc *d) {
  if (!d) fail(OMX_E_INVALID, "null graph descriptor");
  if (d->n_classes <= 0 || d->n_classes > 256) fail(OMX_E_INVALID, "n_classes must be in [1, 256]");
  if (d->n_vertices > 0 && (!d->vertex_class || !d->rids)) fail(OMX_E_INVALID, "vertex_class and rids required");
  auto g = std::make_unique<Graph>();
  static std::atomic<uint64_t> next_uid{1};
  g->uid = next_uid.fetch_add(1);
  g->V = d->n_vertices;
  g->device = d->device;
  uint32_t V = g->V;
  if (d->part_lo == 0 && d->part_hi == 0) {
    g->part_hi = V;
  } else {
    if (d->part_lo > d->part_hi || d->part_hi > V) fail(OMX_E_INVALID, "bad partition range");
    g->part_lo = d->part_lo;
    g->part_hi = d->part_hi;
  }
  const uint32_t VL = g->part_hi - g->part_lo;  // rows held

  for (int i = 0; i < d->n_classes; ++i) {
    ClassInfo c;
    c.name = d->classes[i].name ? d->classes[i].name : "";
    c.super = d->classes[i].superclass;
    c.is_edge = d->classes[i].is_edge_class != 0;
    c.cluster = d->classes[i].cluster_id;
    if (c.super < -1 || c.super >= d->n_classes) fail(OMX_E_INVALID, "bad superclass index for " + c.name);
    g->classes.push_back(c);
  }
  for (int i = 0; i < d->n_classes; ++i)
    for (int j = 0; j < d->n_classes; ++j)
      if (g->is_subclass_of(j, i)) g->classes[i].poly.push_back(j);
  std::vector<uint64_t> counts(d->n_classes, 0);
  for (uint32_t v = 0; v < V; ++v) {
    uint16_t c = d->vertex_class[v];
    if (c >= d->n_classes) fail(OMX_E_INVALID, "vertex_class out of range at vertex " + std::to_string(v));
    counts[c]++;
  }
  for (int i = 0; i < d->n_classes; ++i) g->classes[i].exact_count = counts[i];

  // properties
  for (int i = 0; i < d->n_properties; ++i) {
    const omx_property_desc &pd = d->properties[i];
    Property p;
    p.name = pd.name ? pd.name : "";
    p.type = pd.type;
    if (p.type < OMX_PROP_INT32 || p.type > OMX_PROP_BOOL) fail(OMX_E_INVALID, "bad property type for " + p.name);
    if (p.type == OMX_PROP_STRING) {
      for (int k = 0; k < pd.dict_size; ++k) p.dict.push_back(pd.dict[k]);
      for (int k = 1; k < pd.dict_size; ++k)
        if (!(p.dict[k - 1] < p.dict[k])) fail(OMX_E_INVALID, "string dictionary of " + p.name + " not sorted/unique");
    }
    if (pd.present)
      for (uint32_t v = 0; v < V && !p.has_nulls; ++v) p.has_nulls = pd.present[v] == 0;
    g->props.push_back(std::move(p));
  }
  for (int i = 0; i < d->n_indexes; ++i) {
    const omx_index_desc &x = d->indexes[i];
    int pid = g->prop_id(x.property ? x.property : "");
    if (x.class_id < 0 || x.class_id >= d->n_classes) fail(OMX_E_INVALID, "bad index class");
    if (pid < 0) continue;  // index on a property no vertex carries: never matches a condition
    g->indexes.push_back({x.class_id, pid, x.unique != 0});
    Property &p = g->props[pid];
    const omx_property_desc &pd = d->properties[pid];
    if (p.h_int.empty() && p.h_dbl.empty()) {
      if (p.type == OMX_PROP_DOUBLE) p.h_dbl.assign((const double *)pd.values, (const double *)pd.values + V);
      else if (p.type == OMX_PROP_INT64) p.h_int.assign((const int64_t *)pd.values, (const int64_t *)pd.values + V);
      else {
        const int32_t *s = (const int32_t *)pd.values;
        p.h_int.assign(s, s + V);
      }
      if (pd.present) p.h_present.assign(pd.present, pd.present + V);
    }
  }
  if (!g->indexes.empty()) g->h_vclass.assign(d->vertex_class, d->vertex_class + V);

  // edge sets: validate, sort rows if needed, build the transpose if absent
  std::vector<std::vector<uint32_t>> sorted_copies;
  struct Tmp { const uint64_t *orp, *irp; const uint32_t *ocol, *icol; uint64_t *own_rp = nullptr; uint32_t *own_col = nullptr; };
  std::vector<Tmp> tmp(d->n_edge_sets);
  for (int i = 0; i < d->n_edge_sets; ++i) {
    const omx_edge_set_desc &ed = d->edge_sets[i];
    EdgeSet es;
    es.cls = ed.edge_class;
    es.n_edges = ed.n_edges;
    es.n_in_edges = ed.n_in_edges ? ed.n_in_edges : ed.n_edges;
    if (es.cls < 0 || es.cls >= d->n_classes) fail(OMX_E_INVALID, "bad edge class index");
    if (!ed.out_row_ptr || (ed.n_edges && !ed.out_col)) fail(OMX_E_INVALID, "edge set without out CSR");
    if (ed.out_row_ptr[0] != 0 || ed.out_row_ptr[VL] != ed.n_edges) fail(OMX_E_INVALID, "out_row_ptr inconsistent");
    if (g->partitioned() && !(ed.in_row_ptr && ed.in_col))
      fail(OMX_E_INVALID, "a partition needs the in CSR of its rows (in_row_ptr / in_col)");
    Tmp &t = tmp[i];
    t.orp = ed.out_row_ptr;
    t.ocol = ed.out_col;
    for (uint64_t e = 0; e < ed.n_edges; e += std::max<uint64_t>(1, ed.n_edges / 4096))
      if (ed.out_col[e] >= V) fail(OMX_E_INVALID, "out_col out of range");
    auto so = scan_rows(VL, t.orp, t.ocol);
    if (!so.first) {
      sorted_copies.emplace_back(t.ocol, t.ocol + ed.n_edges);
      sort_rows(VL, t.orp, sorted_copies.back().data());
      t.ocol = sorted_copies.back().data();
      so = scan_rows(VL, t.orp, t.ocol);
    }
    es.out_sorted = so.first;
    es.out_simple = so.second;
    if (ed.in_row_ptr && ed.in_col) {
      if (ed.in_row_ptr[0] != 0 || ed.in_row_ptr[VL] != es.n_in_edges) fail(OMX_E_INVALID, "in_row_ptr inconsistent");
      t.irp = ed.in_row_ptr;
      t.icol = ed.in_col;
      auto si = scan_rows(VL, t.irp, t.icol);
      if (!si.first) {
        sorted_copies.emplace_back(t.icol, t.icol + es.n_in_edges);
        sort_rows(VL, t.irp, sorted_copies.back().data());
        t.icol = sorted_copies.back().data();
        si = scan_rows(VL, t.irp, t.icol);
      }
      es.in_sorted = si.first;
      es.in_simple = si.second;
    } else {
      if (es.n_in_edges != es.n_edges) fail(OMX_E_INVALID, "n_in_edges without an in CSR");
      omx_csr_transpose(V, t.orp, t.ocol, &t.own_rp, &t.own_col);
      t.irp = t.own_rp;
      t.icol = t.own_col;
      auto si = scan_rows(V, t.irp, t.icol);
      es.in_sorted = si.first;
      es.in_simple = si.second;
    }
    es.max_deg[0] = max_row(VL, t.orp);
    es.max_deg[1] = max_row(VL, t.irp);
    g->esets.push_back(es);
  }

  if (g->device >= 0) {
    HIP_CHECK(hipSetDevice(g->device));
    HIP_CHECK(hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&g->stream2, hipStreamNonBlocking));
    HIP_CHECK(hipHostMalloc((void **)&g->h_stage, Graph::kStageWords * sizeof(uint64_t), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc((void **)&g->h_mail, kMailWords * sizeof(uint64_t), hipHostMallocCoherent));
    std::memset(g->h_mail, 0, kMailWords * sizeof(uint64_t));
    uint64_t &acc = g->device_bytes;
    g->d_vclass = upload(d->vertex_class, V, acc);
    g->d_rids = upload(d->rids, V, acc);
    for (int i = 0; i < d->n_edge_sets; ++i) {
      EdgeSet &es = g->esets[i];
      es.d_out_rp = upload(tmp[i].orp, (size_t)VL + 1, acc);
      es.d_out_col = upload(tmp[i].ocol, es.n_edges, acc);
      es.d_in_rp = upload(tmp[i].irp, (size_t)VL + 1, acc);
      es.d_in_col = upload(tmp[i].icol, es.n_in_edges, acc);
    }
    std::vector<DColumn> cols;
    for (int i = 0; i < d->n_properties; ++i) {
      Property &p = g->props[i];
      const omx_property_desc &pd = d->properties[i];
      size_t w = (p.type == OMX_PROP_INT64 || p.type == OMX_PROP_DOUBLE) ? 8 : 4;
      void *dv = nullptr;
      HIP_CHECK(hipMalloc(&dv, std::max<size_t>(1, (size_t)V * w)));
      if (V) HIP_CHECK(hipMemcpy(dv, pd.values, (size_t)V * w, hipMemcpyHostToDevice));
      acc += (size_t)V * w;
      p.d_values = dv;
      if (p.has_nulls) p.d_present = upload(pd.present, V, acc);
      cols.push_back({p.d_values, p.d_present, p.type, 0});
    }
    if (!cols.empty()) g->d_cols = upload(cols.data(), cols.size(), acc);
  }
  for (auto &t : tmp) {
    omx_host_free(t.own_rp);
    omx_host_free(t.own_col);
  }
  return g.release();
}

namespace {
// property values of one record kind, widened to the merged column (codes of a string remapped)
void merge_prop(const omx_property_desc *pd, uint64_t n, uint64_t at, size_t w, const std::vector<std::string> &dict,
                std::vector<uint8_t> &vals, std::vector<uint8_t> &pres) {
  if (!pd) return;
  std::vector<int32_t> remap;
  if (pd->type == OMX_PROP_STRING)
    for (int k = 0; k < pd->dict_size; ++k)
      remap.push_back((int32_t)(std::lower_bound(dict.begin(), dict.end(), std::string(pd->dict[k])) - dict.begin()));
  for (uint64_t i = 0; i < n; ++i) {
    pres[at + i] = pd->present ? pd->present[i] : 1;
    if (!remap.empty()) {
      int32_t c = ((const int32_t *)pd->values)[i];
      if (pres[at + i] && (c < 0 || c >= (int32_t)remap.size())) fail(OMX_E_INVALID, std::string("string code out of range in ") + pd->name);
      c = pres[at + i] ? remap[c] : 0;
      std::memcpy(vals.data() + (at + i) * w, &c, 4);
    } else {
      std::memcpy(vals.data() + (at + i) * w, (const uint8_t *)pd->values + i * w, w);
    }
  }
}
}  // namespace

// Edge records (every edge set given with edge_rids): one id space of records — the vertices [0, V), then
// the edge records [V, V + E) (set 0's out entries in the given order, then set 1's, ...) — so a MATCH
// edge node binds a record id like any alias (classes, RIDs and fields are per record, as ODocument's).
// Per edge class a second set holds its records' ids (outE()/inE() as CSRs), and one set the records'
// endpoints (outV()/inV()); vertex rows of those are the records' ridbags, edge rows of the vertex sets
// are empty (out()/in() of an edge record yields nothing, GF/OSQLFunctionMove.java:66-91).
Graph *graph_create(const omx_graph_desc *d) {
  if (!d) fail(OMX_E_INVALID, "null graph descriptor");
  bool erec = d->n_edge_sets > 0;
  for (int i = 0; i < d->n_edge_sets; ++i) erec = erec && d->edge_sets[i].edge_rids != nullptr;
  if (!erec) {
    Graph *g = create_snapshot(d);
    g->vertices = g->V;
    for (auto &p : g->props) p.nulls_v = p.has_nulls;
    return g;
  }
  if (!(d->part_lo == 0 && (d->part_hi == 0 || d->part_hi == d->n_vertices)))
    fail(OMX_E_INVALID, "edge records (edge_rids) on a partitioned snapshot");
  if (d->n_vertices > 0 && (!d->vertex_class || !d->rids)) fail(OMX_E_INVALID, "vertex_class and rids required");
  const uint64_t V = d->n_vertices;
  const int ns = d->n_edge_sets;
  std::vector<uint64_t> base(ns + 1, 0);
  for (int i = 0; i < ns; ++i) {
    const omx_edge_set_desc &ed = d->edge_sets[i];
    if (!ed.out_row_ptr || (ed.n_edges && !ed.out_col)) fail(OMX_E_INVALID, "edge set without an out CSR");
    if (ed.out_row_ptr[0] != 0 || ed.out_row_ptr[V] != ed.n_edges) fail(OMX_E_INVALID, "out_row_ptr inconsistent");
    if (ed.edge_class < 0 || ed.edge_class >= d->n_classes) fail(OMX_E_INVALID, "bad edge class index");
    base[i + 1] = base[i] + ed.n_edges;
  }
  const uint64_t E = base[ns], N = V + E;
  if (N >= 0xFFFFFFFFull) fail(OMX_E_INVALID, "2^32 - 1 or more vertex and edge records");
  // records: class and RID
  std::vector<uint16_t> vclass(N);
  std::vector<uint64_t> rids(N);
  std::copy(d->vertex_class, d->vertex_class + V, vclass.begin());
  std::copy(d->rids, d->rids + V, rids.begin());
  std::vector<uint32_t> head(E), tail(E);
  for (int i = 0; i < ns; ++i) {
    const omx_edge_set_desc &ed = d->edge_sets[i];
    for (uint64_t o = 0; o < ed.n_edges; ++o) {
      vclass[V + base[i] + o] = (uint16_t)ed.edge_class;
      rids[V + base[i] + o] = ed.edge_rids[o];
    }
    for (uint64_t u = 0; u < V; ++u)
      for (uint64_t o = ed.out_row_ptr[u]; o < ed.out_row_ptr[u + 1]; ++o) {
        if (ed.out_col[o] >= V) fail(OMX_E_INVALID, "out_col entry out of range");
        tail[base[i] + o] = (uint32_t)u;
        head[base[i] + o] = ed.out_col[o];
      }
  }
  // fields: one column per name over every record (absent where the record kind lacks it)
  struct MP {
    std::string name;
    int type;
    const omx_property_desc *v = nullptr, *e = nullptr;
    std::vector<std::string> dict;
    std::vector<uint8_t> vals, pres;
    std::vector<const char *> dict_p;
  };
  std::vector<MP> mps;
  auto find = [&](const std::string &n) -> MP * {
    for (auto &m : mps)
      if (m.name == n) return &m;
    return nullptr;
  };
  for (int k = 0; k < d->n_properties; ++k) {
    const omx_property_desc &pd = d->properties[k];
    mps.push_back(MP{pd.name ? pd.name : "", pd.type});
    mps.back().v = &pd;
  }
  for (int k = 0; k < d->n_edge_properties; ++k) {
    const omx_property_desc &pd = d->edge_properties[k];
    const std::string n = pd.name ? pd.name : "";
    MP *m = find(n);
    if (!m) {
      mps.push_back(MP{n, pd.type});
      m = &mps.back();
    } else if (m->type != pd.type) {
      fail(OMX_E_INVALID, "field " + n + " has different types on vertices and edges");
    }
    m->e = &pd;
  }
  for (auto &m : mps) {
    if (m.type < OMX_PROP_INT32 || m.type > OMX_PROP_BOOL) fail(OMX_E_INVALID, "bad property type for " + m.name);
    const size_t w = (m.type == OMX_PROP_INT64 || m.type == OMX_PROP_DOUBLE) ? 8 : 4;
    if (m.type == OMX_PROP_STRING) {
      std::set<std::string> all;
      for (const omx_property_desc *pd : {m.v, m.e})
        if (pd)
          for (int k = 0; k < pd->dict_size; ++k) all.insert(pd->dict[k]);
      m.dict.assign(all.begin(), all.end());
      for (auto &x : m.dict) m.dict_p.push_back(x.c_str());
    }
    m.vals.assign(std::max<size_t>(1, N * w), 0);
    m.pres.assign(N, 0);
    merge_prop(m.v, V, 0, w, m.dict, m.vals, m.pres);
    if (m.e) {
      merge_prop(m.e, E, V, w, m.dict, m.vals, m.pres);
    }
  }
  std::vector<omx_property_desc> props;
  for (auto &m : mps)
    props.push_back(omx_property_desc{m.name.c_str(), m.type, m.vals.data(), m.pres.data(), (int32_t)m.dict.size(),
                                      m.dict_p.empty() ? nullptr : m.dict_p.data()});
  // edge sets: the classes' adjacency over N rows, their records, the endpoints
  std::vector<std::vector<uint64_t>> rps;
  std::vector<std::vector<uint32_t>> cols;
  auto ext = [&](const uint64_t *rp) {  // V + 1 row pointers → N + 1 (edge rows empty)
    rps.emplace_back(N + 1);
    std::copy(rp, rp + V + 1, rps.back().begin());
    std::fill(rps.back().begin() + V + 1, rps.back().end(), rp[V]);
    return rps.back().data();
  };
  std::vector<omx_edge_set_desc> sets(2 * ns + 1);
  for (int i = 0; i < ns; ++i) {
    const omx_edge_set_desc &ed = d->edge_sets[i];
    omx_edge_set_desc &a = sets[i], &r = sets[ns + i];
    a = omx_edge_set_desc{};
    a.edge_class = r.edge_class = ed.edge_class;
    a.n_edges = r.n_edges = ed.n_edges;
    a.out_row_ptr = r.out_row_ptr = ext(ed.out_row_ptr);
    a.out_col = ed.out_col;
    cols.emplace_back(ed.n_edges);
    for (uint64_t o = 0; o < ed.n_edges; ++o) cols.back()[o] = (uint32_t)(V + base[i] + o);
    r.out_col = cols.back().data();
    if (ed.in_row_ptr && ed.in_col) {
      if (!ed.in_edge_index) fail(OMX_E_INVALID, "in_edge_index is required with edge_rids and an in CSR");
      const uint64_t ni = ed.n_in_edges ? ed.n_in_edges : ed.n_edges;
      if (ni != ed.n_edges || ed.in_row_ptr[0] != 0 || ed.in_row_ptr[V] != ni) fail(OMX_E_INVALID, "in_row_ptr inconsistent");
      a.in_row_ptr = r.in_row_ptr = ext(ed.in_row_ptr);
      a.in_col = ed.in_col;
      a.n_in_edges = r.n_in_edges = ni;
      cols.emplace_back(ni);
      for (uint64_t q = 0; q < ni; ++q) {
        const uint64_t o = ed.in_edge_index[q];
        if (o >= ed.n_edges) fail(OMX_E_INVALID, "in_edge_index out of range");
        cols.back()[q] = (uint32_t)(V + base[i] + o);
      }
      r.in_col = cols.back().data();
    } else {
      // the transpose of the records: an in row lists its edges in out order
      rps.emplace_back(N + 1, 0);
      std::vector<uint64_t> &irp = rps.back();
      for (uint64_t o = 0; o < ed.n_edges; ++o) irp[ed.out_col[o] + 1]++;
      for (uint64_t v = 0; v < N; ++v) irp[v + 1] += irp[v];
      std::vector<uint64_t> cur(irp.begin(), irp.end() - 1);
      cols.emplace_back(ed.n_edges);
      std::vector<uint32_t> &ic = cols.back();
      for (uint64_t o = 0; o < ed.n_edges; ++o) ic[cur[ed.out_col[o]]++] = (uint32_t)(V + base[i] + o);
      r.in_row_ptr = irp.data();
      r.in_col = ic.data();
      r.n_in_edges = ed.n_edges;
    }
  }
  {
    omx_edge_set_desc &q = sets[2 * ns];
    q = omx_edge_set_desc{};
    q.edge_class = d->edge_sets[0].edge_class;
    q.n_edges = q.n_in_edges = E;
    rps.emplace_back(N + 1, 0);
    for (uint64_t k = 0; k < E; ++k) rps.back()[V + k + 1] = k + 1;
    q.out_row_ptr = q.in_row_ptr = rps.back().data();
    q.out_col = tail.data();
    q.in_col = head.data();
  }
  omx_graph_desc nd = *d;
  nd.n_vertices = (uint32_t)N;
  nd.vertex_class = vclass.data();
  nd.rids = rids.data();
  nd.n_edge_sets = (int32_t)sets.size();
  nd.edge_sets = sets.data();
  nd.n_properties = (int32_t)props.size();
  nd.properties = props.data();
  nd.part_lo = nd.part_hi = 0;
  nd.n_edge_properties = 0;
  nd.edge_properties = nullptr;
  Graph *g = create_snapshot(&nd);
  g->vertices = (uint32_t)V;
  g->edge_records = true;
  for (size_t k = 0; k < mps.size(); ++k) {
    const std::vector<uint8_t> &pr = mps[k].pres;
    Property &p = g->props[k];
    p.nulls_v = std::find(pr.begin(), pr.begin() + V, 0) != pr.begin() + V;
    p.nulls_e = std::find(pr.begin() + V, pr.end(), 0) != pr.end();
  }
  for (int i = 0; i < ns; ++i) g->esets[ns + i].pseudo = 1;
  g->esets[2 * ns].pseudo = 2;
  return g;
}

}  // namespace omx
