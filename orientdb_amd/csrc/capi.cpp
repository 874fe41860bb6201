// capi.cpp — the extern "C" boundary (include/omx/match.h).
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>

#include "dist.h"
#include "exec.h"
#include "graph.h"
#include "plan.h"
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
}  // namespace

extern "C" {

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
    *out = omx::execute_plan(*g->g, *s->plan, o, o.comm ? o.comm->t.get() : nullptr);
  });
  // a rank that fails (planning included) releases the peers waiting for it in an exchange
  if (rc != OMX_OK && opts && opts->comm) opts->comm->t->abort();
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
  if (!r || r->rows.empty()) return nullptr;
  return r->rows.data();
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

void omx_result_free(omx_result *r) { delete r; }

int omx_result_cell(const omx_result *r, uint64_t row, int32_t col, omx_cell *out) {
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

const char *omx_last_error(void) { return g_last_error.c_str(); }

const char *omx_version(void) { return "omx 0.1 (gfx950)"; }

}  // extern "C"
