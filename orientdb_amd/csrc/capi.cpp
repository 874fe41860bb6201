// capi.cpp — the extern "C" boundary (include/omx/match.h).
#include <algorithm>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dist.h"
#include "exec.h"
#include "graph.h"
#include "plan.h"
#include "projdev.h"
#include "sql.h"

struct omx_graph {
  std::unique_ptr<omx::Graph> g;
  // a snapshot may be executed from several host threads (OrientDB sessions): its stream, scratch pool,
  // host mailbox and lazily built adjacency caches are per graph, so executions are serialised
  std::mutex m;
};
struct omx_statement {
  std::unique_ptr<omx::Statement> st;
  std::string text;
  // the last compiled plan, reused while the graph and the parameters are the same (the reference's
  // statement cache keeps parsed statements; a plan here is the parse + planner output)
  uint64_t plan_graph = 0;
  std::string plan_key;
  std::unique_ptr<omx::Plan> plan;
};
struct omx_comm {
  std::unique_ptr<omx::Transport> t;
};

namespace {
thread_local std::string g_last_error;

template <class F>
int guard(F f) {
  try {
    f();
    g_last_error.clear();
    return OMX_OK;
  } catch (const omx::OmxError &e) {
    g_last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc &) {
    g_last_error = "host out of memory";
    return OMX_E_OOM;
  } catch (const std::exception &e) {
    g_last_error = e.what();
    return OMX_E_EXECUTION;
  }
}

omx::Params make_params(const omx_value *vals, int32_t n) {
  omx::Params p;
  for (int32_t i = 0; i < n; ++i) {
    const omx_value &v = vals[i];
    omx::Value x;
    switch (v.type) {
      case OMX_VAL_NULL: break;
      case OMX_VAL_INT: x = omx::Value::Int(v.i); break;
      case OMX_VAL_DOUBLE: x = omx::Value::Dbl(v.d); break;
      case OMX_VAL_STRING: x = omx::Value::Str(v.s ? v.s : ""); break;
      case OMX_VAL_BOOL: x = omx::Value::Bool(v.i != 0); break;
      default: omx::fail(OMX_E_INVALID, "bad parameter type");
    }
    if (v.name) {
      p.named.emplace_back(v.name, x);
    } else {
      if (v.index < 0) omx::fail(OMX_E_INVALID, "negative parameter index");
      if ((size_t)v.index >= p.positional.size()) p.positional.resize(v.index + 1);
      p.positional[v.index] = x;
    }
  }
  return p;
}
// identity of a parameter list (type, position/name, value) for the plan cache
std::string params_key(const omx_value *vals, int32_t n) {
  std::string k;
  for (int32_t i = 0; i < n; ++i) {
    const omx_value &v = vals[i];
    k += std::to_string(v.type) + ":" + std::to_string(v.index) + ":" + (v.name ? v.name : "") + "=";
    switch (v.type) {
      case OMX_VAL_INT: case OMX_VAL_BOOL: k += std::to_string(v.i); break;
      case OMX_VAL_DOUBLE: {
        char b[32];
        std::snprintf(b, sizeof(b), "%a", v.d);
        k += b;
        break;
      }
      case OMX_VAL_STRING: k += std::to_string(v.s ? std::strlen(v.s) : 0) + ":" + (v.s ? v.s : ""); break;
      default: break;
    }
    k += ";";
  }
  return k;
}
// ---- pointer-free buffers (omx_graph_create_blob / omx_execute_packed) ------------------------------
static_assert(sizeof(omx_graph_blob) == 112 && offsetof(omx_graph_blob, edge_records_off) == 88, "omx_graph_blob layout");
static_assert(sizeof(omx_class_rec) == 24 && sizeof(omx_edge_set_rec) == 56 && sizeof(omx_property_rec) == 40 &&
                  sizeof(omx_index_rec) == 16 && sizeof(omx_param_rec) == 40 && sizeof(omx_edge_records_rec) == 16,
              "blob record layouts");
constexpr uint64_t kBlobV1Header = 88;  // a version-1 header ends at indexes_off

class Blob {
 public:
  Blob(const void *p, uint64_t size) : p_(static_cast<const uint8_t *>(p)), size_(size) {
    if (!p_) omx::fail(OMX_E_INVALID, "null buffer");
  }
  // `count` elements of T at byte offset `off` (nullptr when off == 0 and optional)
  template <class T>
  const T *array(uint64_t off, uint64_t count, const char *what, bool optional = false) const {
    if (off == 0) {
      if (optional || count == 0) return nullptr;
      omx::fail(OMX_E_INVALID, std::string("buffer: missing ") + what);
    }
    if (off % alignof(T) != 0) omx::fail(OMX_E_INVALID, std::string("buffer: misaligned ") + what);
    if (off > size_ || count > (size_ - off) / sizeof(T)) omx::fail(OMX_E_INVALID, std::string("buffer: ") + what + " out of range");
    return reinterpret_cast<const T *>(p_ + off);
  }
  const char *str(uint64_t off, const char *what, bool optional = false) const {
    if (off == 0) {
      if (optional) return nullptr;
      omx::fail(OMX_E_INVALID, std::string("buffer: missing ") + what);
    }
    if (off >= size_) omx::fail(OMX_E_INVALID, std::string("buffer: ") + what + " out of range");
    const void *z = std::memchr(p_ + off, 0, size_ - off);
    if (!z) omx::fail(OMX_E_INVALID, std::string("buffer: unterminated ") + what);
    return reinterpret_cast<const char *>(p_ + off);
  }

 private:
  const uint8_t *p_;
  uint64_t size_;
};

// the blob's contents, not only its extents: a stale or malformed snapshot fails here with
// OMX_E_INVALID instead of sending out-of-range ids to the kernels (a parallel host scan, cheap next to
// the upload that follows)
template <class F>
bool parallel_all(uint64_t n, F ok) {
  const uint64_t kMin = 1u << 22;
  const unsigned nt = n < kMin ? 1u : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<char> good(nt, 1);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      const uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
      for (uint64_t i = lo; i < hi; ++i)
        if (!ok(i)) { good[t] = 0; return; }
    });
  for (auto &x : th) x.join();
  for (char c : good)
    if (!c) return false;
  return true;
}
void check_csr(const uint64_t *rp, const uint32_t *col, uint64_t rows, uint64_t V, const char *what) {
  if (!rp) return;
  if (rp[0] != 0) omx::fail(OMX_E_INVALID, std::string("buffer: ") + what + " row_ptr[0] != 0");
  if (!parallel_all(rows, [&](uint64_t i) { return rp[i] <= rp[i + 1]; }))
    omx::fail(OMX_E_INVALID, std::string("buffer: ") + what + " row_ptr is not non-decreasing");
  if (!parallel_all(rp[rows], [&](uint64_t i) { return col[i] < V; }))
    omx::fail(OMX_E_INVALID, std::string("buffer: ") + what + " col holds a vertex id >= n_vertices");
}

}  // namespace

extern "C" {

int omx_graph_create_blob(const void *blob, uint64_t size, omx_graph **out) {
  return guard([&] {
    if (!out) omx::fail(OMX_E_INVALID, "null out pointer");
    const Blob b(blob, size);
    if (size < kBlobV1Header) omx::fail(OMX_E_INVALID, "buffer smaller than its header");
    if (reinterpret_cast<uintptr_t>(blob) % 8) omx::fail(OMX_E_INVALID, "buffer not 8-byte aligned");
    const omx_graph_blob *h = static_cast<const omx_graph_blob *>(blob);
    if (h->magic != OMX_BLOB_MAGIC || (h->version != 1 && h->version != OMX_BLOB_VERSION))
      omx::fail(OMX_E_INVALID, "buffer: bad magic/version");
    const bool v2 = h->version >= 2;
    if (v2 && size < sizeof(omx_graph_blob)) omx::fail(OMX_E_INVALID, "buffer smaller than its header");
    if (h->n_classes < 0 || h->n_edge_sets < 0 || h->n_properties < 0 || h->n_indexes < 0)
      omx::fail(OMX_E_INVALID, "buffer: negative count");
    const uint64_t V = h->n_vertices;
    const uint32_t VL = (h->part_lo == 0 && h->part_hi == 0) ? h->n_vertices : h->part_hi - h->part_lo;
    if (h->part_hi < h->part_lo) omx::fail(OMX_E_INVALID, "buffer: bad partition range");
    omx_graph_desc d{};
    d.n_vertices = h->n_vertices;
    d.device = h->device;
    d.part_lo = h->part_lo;
    d.part_hi = h->part_hi;
    d.vertex_class = b.array<uint16_t>(h->vertex_class_off, V, "vertex_class");
    d.rids = b.array<uint64_t>(h->rids_off, V, "rids");
    std::vector<omx_class_desc> cls(h->n_classes);
    const omx_class_rec *cr = b.array<omx_class_rec>(h->classes_off, h->n_classes, "classes");
    for (int i = 0; i < h->n_classes; ++i)
      cls[i] = omx_class_desc{b.str(cr[i].name_off, "class name"), cr[i].superclass, cr[i].is_edge_class, cr[i].cluster_id};
    d.n_classes = h->n_classes;
    d.classes = cls.data();
    std::vector<omx_edge_set_desc> es(h->n_edge_sets);
    const omx_edge_set_rec *er = b.array<omx_edge_set_rec>(h->edge_sets_off, h->n_edge_sets, "edge sets");
    for (int i = 0; i < h->n_edge_sets; ++i) {
      const omx_edge_set_rec &r = er[i];
      const uint64_t nin = r.n_in_edges ? r.n_in_edges : r.n_edges;
      es[i].edge_class = r.edge_class;
      es[i].n_edges = r.n_edges;
      es[i].out_row_ptr = b.array<uint64_t>(r.out_row_ptr_off, (uint64_t)VL + 1, "out_row_ptr");
      es[i].out_col = b.array<uint32_t>(r.out_col_off, r.n_edges, "out_col");
      es[i].in_row_ptr = b.array<uint64_t>(r.in_row_ptr_off, (uint64_t)VL + 1, "in_row_ptr", true);
      es[i].in_col = es[i].in_row_ptr ? b.array<uint32_t>(r.in_col_off, nin, "in_col") : nullptr;
      es[i].n_in_edges = r.n_in_edges;
      if (es[i].out_row_ptr && es[i].out_row_ptr[VL] != r.n_edges) omx::fail(OMX_E_INVALID, "buffer: out_row_ptr[V] != n_edges");
      if (es[i].in_row_ptr && es[i].in_row_ptr[VL] != nin) omx::fail(OMX_E_INVALID, "buffer: in_row_ptr[V] != n_in_edges");
      check_csr(es[i].out_row_ptr, es[i].out_col, VL, V, "out");
      check_csr(es[i].in_row_ptr, es[i].in_col, VL, V, "in");
    }
    d.n_edge_sets = h->n_edge_sets;
    d.edge_sets = es.data();
    uint64_t n_erec = 0;
    if (v2 && h->edge_records_off) {
      const omx_edge_records_rec *xr = b.array<omx_edge_records_rec>(h->edge_records_off, h->n_edge_sets, "edge records");
      for (int i = 0; i < h->n_edge_sets; ++i) {
        es[i].edge_rids = b.array<uint64_t>(xr[i].edge_rids_off, es[i].n_edges, "edge_rids");
        es[i].in_edge_index = es[i].in_row_ptr ? b.array<uint64_t>(xr[i].in_edge_index_off, es[i].n_in_edges ? es[i].n_in_edges : es[i].n_edges, "in_edge_index")
                                               : nullptr;
        n_erec += es[i].n_edges;
      }
    }
    if (v2 && (h->n_edge_properties < 0 || (h->n_edge_properties > 0 && !h->edge_records_off)))
      omx::fail(OMX_E_INVALID, "buffer: edge properties without edge records");
    const int n_eprops = v2 ? h->n_edge_properties : 0;
    std::vector<std::vector<const char *>> dicts(h->n_properties + n_eprops);
    auto props = [&](uint64_t off, int n, uint64_t rows, int d0) {
      std::vector<omx_property_desc> pr(n);
      const omx_property_rec *prr = b.array<omx_property_rec>(off, n, "properties");
      for (int i = 0; i < n; ++i) {
        const omx_property_rec &r = prr[i];
        pr[i].name = b.str(r.name_off, "property name");
        pr[i].type = r.type;
        const size_t w = r.type == OMX_PROP_INT64 || r.type == OMX_PROP_DOUBLE ? 8 : 4;
        pr[i].values = w == 8 ? (const void *)b.array<uint64_t>(r.values_off, rows, "property values")
                              : (const void *)b.array<uint32_t>(r.values_off, rows, "property values");
        pr[i].present = b.array<uint8_t>(r.present_off, rows, "present", true);
        if (r.dict_size < 0) omx::fail(OMX_E_INVALID, "buffer: negative dictionary size");
        if (r.type == OMX_PROP_STRING) {
          const uint64_t *doff = b.array<uint64_t>(r.dict_off, (uint64_t)r.dict_size, "dictionary");
          for (int k = 0; k < r.dict_size; ++k) dicts[d0 + i].push_back(b.str(doff[k], "dictionary string"));
        }
        pr[i].dict_size = r.dict_size;
        pr[i].dict = dicts[d0 + i].empty() ? nullptr : dicts[d0 + i].data();
      }
      return pr;
    };
    std::vector<omx_property_desc> pr = props(h->properties_off, h->n_properties, V, 0);
    std::vector<omx_property_desc> epr = props(v2 ? h->edge_properties_off : 0, n_eprops, n_erec, h->n_properties);
    d.n_properties = h->n_properties;
    d.properties = pr.data();
    d.n_edge_properties = n_eprops;
    d.edge_properties = epr.data();
    std::vector<omx_index_desc> ix(h->n_indexes);
    const omx_index_rec *ir = b.array<omx_index_rec>(h->indexes_off, h->n_indexes, "indexes");
    for (int i = 0; i < h->n_indexes; ++i) ix[i] = omx_index_desc{ir[i].class_id, b.str(ir[i].property_off, "index property"), ir[i].unique};
    d.n_indexes = h->n_indexes;
    d.indexes = ix.data();
    auto g = std::make_unique<omx_graph>();
    g->g.reset(omx::graph_create(&d));
    *out = g.release();
  });
}

int omx_execute_packed(omx_graph *g, omx_statement *s, int32_t mode, int32_t flags, int64_t limit, int32_t shard_rank,
                       int32_t shard_world, omx_comm *comm, const void *param_blob, uint64_t param_blob_size,
                       omx_result **out) {
  std::vector<omx_value> vals;
  const int rc = guard([&] {
    if (!param_blob) return;
    const Blob b(param_blob, param_blob_size);
    if (param_blob_size < 8) omx::fail(OMX_E_INVALID, "parameter buffer smaller than its header");
    if (reinterpret_cast<uintptr_t>(param_blob) % 8) omx::fail(OMX_E_INVALID, "parameter buffer not 8-byte aligned");
    const uint32_t *n = static_cast<const uint32_t *>(param_blob);
    const omx_param_rec *r = b.array<omx_param_rec>(8, n[0], "parameters");
    for (uint32_t i = 0; i < n[0]; ++i) {
      omx_value v{};
      v.type = r[i].type;
      v.index = r[i].index;
      v.i = r[i].i;
      v.d = r[i].d;
      v.name = b.str(r[i].name_off, "parameter name", true);
      v.s = r[i].type == OMX_VAL_STRING ? b.str(r[i].s_off, "parameter string") : nullptr;
      vals.push_back(v);
    }
  });
  if (rc != OMX_OK) return rc;
  omx_exec_options o;
  omx_exec_options_init(&o);
  o.mode = mode;
  o.flags = flags;
  o.limit = limit;
  o.shard_rank = shard_rank;
  o.shard_world = shard_world;
  o.comm = comm;
  o.params = vals.empty() ? nullptr : vals.data();
  o.n_params = (int32_t)vals.size();
  return omx_execute(g, s, &o, out);
}

int omx_graph_create(const omx_graph_desc *desc, omx_graph **out) {
  return guard([&] {
    if (!out) omx::fail(OMX_E_INVALID, "null out pointer");
    auto h = std::make_unique<omx_graph>();
    h->g.reset(omx::graph_create(desc));
    *out = h.release();
  });
}

void omx_graph_destroy(omx_graph *g) { delete g; }

int omx_graph_class_count(const omx_graph *g, const char *name, uint64_t *count) {
  return guard([&] {
    if (!g || !name || !count) omx::fail(OMX_E_INVALID, "null argument");
    int c = g->g->class_id(name);
    if (c < 0) omx::fail(OMX_E_INVALID, std::string("class not defined: ") + name);
    *count = g->g->count(c);
  });
}

uint64_t omx_graph_device_bytes(const omx_graph *g) { return g ? g->g->device_bytes : 0; }

int omx_statement_parse(const char *text, omx_statement **out) {
  return guard([&] {
    if (!text || !out) omx::fail(OMX_E_INVALID, "null argument");
    auto s = std::make_unique<omx_statement>();
    s->text = text;
    s->st = omx::parse_match(text);
    *out = s.release();
  });
}

void omx_statement_free(omx_statement *s) { delete s; }

int omx_statement_explain(omx_statement *s, const omx_graph *g, const omx_value *params, int32_t n_params, char *buf,
                          size_t len) {
  return guard([&] {
    if (!s || !g || !buf || !len) omx::fail(OMX_E_INVALID, "null argument");
    omx::Params p = make_params(params, n_params);
    std::string reason;
    auto plan = omx::build_plan(*s->st, *g->g, p, true, &reason);
    std::string j = omx::plan_json(*plan, reason);
    std::strncpy(buf, j.c_str(), len - 1);
    buf[len - 1] = 0;
  });
}

void omx_exec_options_init(omx_exec_options *o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->mode = OMX_MODE_MATERIALIZE;
  o->limit = -1;
  o->shard_world = 1;
  o->comm = nullptr;
}

int omx_execute(omx_graph *g, omx_statement *s, const omx_exec_options *opts, omx_result **out) {
  omx::Transport *t = opts && opts->comm ? opts->comm->t.get() : nullptr;
  bool running = false;
  const int rc = guard([&] {
    if (!g || !s || !out) omx::fail(OMX_E_INVALID, "null argument");
    omx_exec_options o;
    omx_exec_options_init(&o);
    if (opts) o = *opts;
    if (o.shard_world < 1 || o.shard_rank < 0 || o.shard_rank >= o.shard_world) omx::fail(OMX_E_INVALID, "bad shard");
    const std::string key = params_key(o.params, o.n_params);
    if (!s->plan || s->plan_graph != g->g->uid || s->plan_key != key) {
      omx::Params p = make_params(o.params, o.n_params);
      s->plan.reset();
      s->plan = omx::build_plan(*s->st, *g->g, p, false);
      s->plan_graph = g->g->uid;
      s->plan_key = key;
    }
    std::lock_guard<std::mutex> lk(g->m);
    *out = omx::execute_plan(*g->g, *s->plan, o, t, &running);
  });
  // A rank that fails releases the peers waiting for it in an exchange; the communicator is unusable
  // afterwards. The exception is OMX_E_UNSUPPORTED raised by the planner or the plan's partition checks,
  // before execution starts: they see the same statement, parameters and replicated schema on every
  // rank, so every rank refused alike, nobody waits, the host falls back to the reference engine and the
  // communicator stays usable for the next query. A refusal raised during execution may depend on the
  // rank's own rows (a size limit), so it aborts like any other failure.
  if (rc != OMX_OK && t && (rc != OMX_E_UNSUPPORTED || running)) t->abort();
  return rc;
}

int omx_comm_unique_id(uint8_t *id) {
  return guard([&] {
    if (!id) omx::fail(OMX_E_INVALID, "null argument");
    omx::rccl_unique_id(id);
  });
}

int omx_comm_create_rccl(int32_t rank, int32_t world, int32_t device, const uint8_t *id, omx_comm **out) {
  return guard([&] {
    if (!id || !out) omx::fail(OMX_E_INVALID, "null argument");
    auto c = std::make_unique<omx_comm>();
    c->t = omx::make_rccl_transport(rank, world, device, id);
    *out = c.release();
  });
}

int omx_comm_create_threads(int32_t world, omx_comm **out) {
  return guard([&] {
    if (!out || world < 1) omx::fail(OMX_E_INVALID, "bad argument");
    auto hub = std::make_shared<omx::ThreadHub>(world);
    std::vector<std::unique_ptr<omx_comm>> cs;
    for (int r = 0; r < world; ++r) {
      cs.push_back(std::make_unique<omx_comm>());
      cs.back()->t = omx::make_thread_transport(hub, r);
    }
    for (int r = 0; r < world; ++r) out[r] = cs[r].release();
  });
}

int omx_comm_create_host(int32_t rank, int32_t world, const omx_host_collectives *hc, omx_comm **out) {
  return guard([&] {
    if (!hc || !out) omx::fail(OMX_E_INVALID, "null argument");
    auto c = std::make_unique<omx_comm>();
    c->t = omx::make_host_transport(rank, world, omx::HostCollectives{hc->ctx, hc->allgather, hc->alltoallv, hc->abort});
    *out = c.release();
  });
}

int32_t omx_comm_rank(const omx_comm *c) { return c ? c->t->rank() : -1; }
int32_t omx_comm_world(const omx_comm *c) { return c ? c->t->world() : 0; }
void omx_comm_destroy(omx_comm *c) { delete c; }

int omx_result_info_get(const omx_result *r, omx_result_info *info) {
  return guard([&] {
    if (!r || !info) omx::fail(OMX_E_INVALID, "null argument");
    *info = r->info;
  });
}

const char *omx_result_column_name(const omx_result *r, int32_t col) {
  if (!r || col < 0 || (size_t)col >= r->names.size()) return nullptr;
  return r->names[col].c_str();
}

const uint64_t *omx_result_rows(const omx_result *r) {
  if (!r || !r->rows || !r->info.n_rows) return nullptr;
  return r->rows;
}

int omx_result_kernel_stat(const omx_result *r, int32_t i, const char **name, int64_t *launches, double *total_ms,
                           uint64_t *alg_bytes) {
  if (!r || i < 0 || (size_t)i >= r->kstats.size()) return OMX_E_INVALID;
  const auto &k = r->kstats[i];
  if (name) *name = k.name.c_str();
  if (launches) *launches = k.launches;
  if (total_ms) *total_ms = k.ms;
  if (alg_bytes) *alg_bytes = k.bytes;
  return OMX_OK;
}

int omx_result_kernel_launch(const omx_result *r, int32_t i, const char **name, double *ms, uint64_t *alg_bytes) {
  if (!r || i < 0 || (size_t)i >= r->klaunches.size()) return OMX_E_INVALID;
  const auto &k = r->klaunches[i];
  if (name) *name = k.name.c_str();
  if (ms) *ms = k.ms;
  if (alg_bytes) *alg_bytes = k.bytes;
  return OMX_OK;
}

int omx_result_kernel_launch_bytes(const omx_result *r, int32_t i, uint64_t *alg_bytes, uint64_t *hbm_bytes) {
  if (!r || i < 0 || (size_t)i >= r->klaunches.size()) return OMX_E_INVALID;
  const auto &k = r->klaunches[i];
  if (alg_bytes) *alg_bytes = k.bytes;
  if (hbm_bytes) *hbm_bytes = k.hbm;
  return OMX_OK;
}

void omx_result_free(omx_result *r) { delete r; }

int omx_result_cell(const omx_result *r, uint64_t row, int32_t col, omx_cell *out) {
  if (r && out && !r->pcols.empty()) {  // documents evaluated on the device (projdev.hip): columnar cells
    if (row >= r->n_pcol_rows || col < 0 || (size_t)col >= r->pcols.size()) return OMX_E_INVALID;
    const omx_result::PCol &pc = r->pcols[col];
    const uint64_t x = pc.val[row];
    std::memset(out, 0, sizeof(*out));
    switch (pc.kind[row]) {
      case omx::PJ_K_INT: out->type = OMX_CELL_INT; out->i = (int64_t)x; break;
      case omx::PJ_K_DBL: out->type = OMX_CELL_DOUBLE; std::memcpy(&out->d, &x, 8); break;
      case omx::PJ_K_STR: out->type = OMX_CELL_STRING; out->s = pc.strs.at(x).c_str(); break;
      case omx::PJ_K_BOOL: out->type = OMX_CELL_BOOL; out->i = (int64_t)x; break;
      case omx::PJ_K_RID: out->type = OMX_CELL_RID; out->rid = x; break;
      default: out->type = OMX_CELL_NULL; break;
    }
    return OMX_OK;
  }
  if (!r || !out || row >= r->docs.size() || col < 0 || (size_t)col >= r->docs[row].size()) return OMX_E_INVALID;
  const omx::HVal &v = r->docs[row][col];
  std::memset(out, 0, sizeof(*out));
  switch (v.k) {
    case omx::HVal::NUL: out->type = OMX_CELL_NULL; break;
    case omx::HVal::INT: out->type = OMX_CELL_INT; out->i = v.i; break;
    case omx::HVal::DBL: out->type = OMX_CELL_DOUBLE; out->d = v.d; break;
    case omx::HVal::STR: out->type = OMX_CELL_STRING; out->s = v.s.c_str(); break;
    case omx::HVal::BOOL: out->type = OMX_CELL_BOOL; out->i = v.i; break;
    case omx::HVal::RID: out->type = OMX_CELL_RID; out->rid = v.rid; break;
    case omx::HVal::LIST: out->type = OMX_CELL_LIST; out->n = (int32_t)v.items.size(); out->s = v.json.c_str(); break;
    case omx::HVal::MAP: out->type = OMX_CELL_MAP; out->n = (int32_t)v.items.size(); out->s = v.json.c_str(); break;
  }
  return OMX_OK;
}

int omx_result_column(const omx_result *r, int32_t col, int32_t *types, uint64_t *bits) {
  if (!r || !types || !bits || col < 0) return OMX_E_INVALID;
  if (!r->pcols.empty()) {
    if ((size_t)col >= r->pcols.size()) return OMX_E_INVALID;
    const omx_result::PCol &pc = r->pcols[col];
    for (uint64_t i = 0; i < r->n_pcol_rows; ++i) {
      switch (pc.kind[i]) {
        case omx::PJ_K_INT: types[i] = OMX_CELL_INT; bits[i] = pc.val[i]; break;
        case omx::PJ_K_DBL: types[i] = OMX_CELL_DOUBLE; bits[i] = pc.val[i]; break;
        case omx::PJ_K_STR: types[i] = OMX_CELL_STRING; bits[i] = 0; break;
        case omx::PJ_K_BOOL: types[i] = OMX_CELL_BOOL; bits[i] = pc.val[i]; break;
        case omx::PJ_K_RID: types[i] = OMX_CELL_RID; bits[i] = pc.val[i]; break;
        default: types[i] = OMX_CELL_NULL; bits[i] = 0; break;
      }
    }
    return OMX_OK;
  }
  if (!r->docs.empty() && (size_t)col >= r->docs[0].size()) return OMX_E_INVALID;
  for (size_t i = 0; i < r->docs.size(); ++i) {
    if ((size_t)col >= r->docs[i].size()) return OMX_E_INVALID;
    const omx::HVal &v = r->docs[i][col];
    bits[i] = 0;
    switch (v.k) {
      case omx::HVal::NUL: types[i] = OMX_CELL_NULL; break;
      case omx::HVal::INT: types[i] = OMX_CELL_INT; bits[i] = (uint64_t)v.i; break;
      case omx::HVal::DBL: types[i] = OMX_CELL_DOUBLE; std::memcpy(&bits[i], &v.d, 8); break;
      case omx::HVal::STR: types[i] = OMX_CELL_STRING; break;
      case omx::HVal::BOOL: types[i] = OMX_CELL_BOOL; bits[i] = (uint64_t)v.i; break;
      case omx::HVal::RID: types[i] = OMX_CELL_RID; bits[i] = v.rid; break;
      case omx::HVal::LIST: types[i] = OMX_CELL_LIST; break;
      case omx::HVal::MAP: types[i] = OMX_CELL_MAP; break;
    }
  }
  return OMX_OK;
}

int omx_ridbag_decode_csr(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                          uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                          const uint64_t *edge_targets, uint64_t n_edge_records, uint64_t *row_ptr, uint32_t *col,
                          uint64_t *n_entries) {
  return guard([&] {
    omx::ridbag_decode_csr(device, streams, stream_bytes, offsets, n_vertices, vertex_rids, edge_rids, edge_targets,
                           n_edge_records, nullptr, 0, 0, row_ptr, col, n_entries);
  });
}

int omx_ridbag_decode_csr_ex(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                             uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                             const uint64_t *edge_targets, uint64_t n_edge_records, const omx_bonsai_file *files,
                             int32_t n_files, uint32_t page_size, uint64_t *row_ptr, uint32_t *col,
                             uint64_t *n_entries) {
  return guard([&] {
    omx::ridbag_decode_csr(device, streams, stream_bytes, offsets, n_vertices, vertex_rids, edge_rids, edge_targets,
                           n_edge_records, files, files ? n_files : 0,
                           page_size ? page_size : OMX_BONSAI_PAGE_SIZE, row_ptr, col, n_entries);
  });
}

int omx_ridbag_decode_edges(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                            uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                            const uint64_t *edge_targets, uint64_t n_edge_records, const omx_bonsai_file *files,
                            int32_t n_files, uint32_t page_size, uint64_t *row_ptr, uint32_t *col,
                            uint64_t *entry_rids, uint64_t *n_entries) {
  return guard([&] {
    if (!edge_rids || !edge_targets) omx::fail(OMX_E_INVALID, "omx_ridbag_decode_edges decodes bags of edge records");
    omx::ridbag_decode_csr(device, streams, stream_bytes, offsets, n_vertices, vertex_rids, edge_rids, edge_targets,
                           n_edge_records, files, files ? n_files : 0,
                           page_size ? page_size : OMX_BONSAI_PAGE_SIZE, row_ptr, col, n_entries,
                           col ? entry_rids : nullptr);
  });
}

const char *omx_last_error(void) { return g_last_error.c_str(); }

const char *omx_version(void) { return "omx 0.1 (gfx950)"; }

}  // extern "C"
