// project.cpp — result documents of RETURN expressions / JSON (see project.h).
//
// The evaluator restates the reference's expression semantics for what a RETURN item of MATCH reads:
//   field of a record / map / list         OSuffixIdentifier.execute (P/OSuffixIdentifier.java:40-58)
//   + - * / %, string concatenation          OMathExpression (P/OMathExpression.java)
//   = != < <= > >=                           OQueryOperatorEquals.equals (S/operator/OQueryOperatorEquals.java:67-97),
//                                            OGtOperator/OLtOperator/OGeOperator/OLeOperator (NPE on a null left
//                                            operand except <)
//   out()/in()/both() of a vertex            OSQLFunctionMove (GF/OSQLFunctionMove.java:66-144)
//   [i] [a-b] [i, j] [condition]             OArraySelector / OArrayRangeSelector / OArraySingleValuesSelector /
//                                            OArrayConditionSelector (P/OModifier.java)
//   size() toUpperCase() toLowerCase()       OSQLMethodSize / OSQLMethodToUpperCase / OSQLMethodToLowerCase
#include "project.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_set>

namespace omx {
namespace {

// ---- host mirrors of the snapshot columns (copied once per graph; the snapshot is immutable) ---------
void ensure_rids(Graph &g) {
  if (g.h_rids.size() == g.V) return;
  std::vector<uint64_t> r(g.V);
  if (g.V) HIP_CHECK(hipMemcpy(r.data(), g.d_rids, (size_t)g.V * 8, hipMemcpyDeviceToHost));
  g.h_rids.swap(r);
}
void ensure_vclass(Graph &g) {
  if (g.h_vclass.size() == g.V) return;
  std::vector<uint16_t> c(g.V);
  if (g.V) HIP_CHECK(hipMemcpy(c.data(), g.d_vclass, (size_t)g.V * 2, hipMemcpyDeviceToHost));
  g.h_vclass.swap(c);
}
// the edge records' `out` / `in` links, from the endpoints set (EdgeSet::pseudo == 2)
void ensure_links(Graph &g) {
  const uint64_t E = (uint64_t)g.V - g.vertices;
  if (g.h_etail.size() == E) return;
  for (const EdgeSet &es : g.esets)
    if (es.pseudo == 2) {
      std::vector<uint32_t> t(E), h(E);
      if (E) {
        HIP_CHECK(hipMemcpy(t.data(), es.d_out_col, E * 4, hipMemcpyDeviceToHost));
        HIP_CHECK(hipMemcpy(h.data(), es.d_in_col, E * 4, hipMemcpyDeviceToHost));
      }
      g.h_etail.swap(t);
      g.h_ehead.swap(h);
      return;
    }
  fail(OMX_E_INVALID, "internal: edge records without an endpoints set");
}
void ensure_prop(Graph &g, Property &p) {
  if (!p.h_int.empty() || !p.h_dbl.empty() || g.V == 0) return;
  if (p.type == OMX_PROP_DOUBLE) {
    p.h_dbl.resize(g.V);
    HIP_CHECK(hipMemcpy(p.h_dbl.data(), p.d_values, (size_t)g.V * 8, hipMemcpyDeviceToHost));
  } else if (p.type == OMX_PROP_INT64) {
    p.h_int.resize(g.V);
    HIP_CHECK(hipMemcpy(p.h_int.data(), p.d_values, (size_t)g.V * 8, hipMemcpyDeviceToHost));
  } else {
    std::vector<int32_t> t(g.V);
    HIP_CHECK(hipMemcpy(t.data(), p.d_values, (size_t)g.V * 4, hipMemcpyDeviceToHost));
    p.h_int.assign(t.begin(), t.end());
  }
  if (p.d_present) {
    p.h_present.resize(g.V);
    HIP_CHECK(hipMemcpy(p.h_present.data(), p.d_present, g.V, hipMemcpyDeviceToHost));
  }
}

bool is_num(const HVal &x) { return x.k == HVal::INT || x.k == HVal::DBL; }
double dbl(const HVal &x) { return x.k == HVal::DBL ? x.d : (double)x.i; }
HVal mk_int(int64_t i) { HVal v; v.k = HVal::INT; v.i = i; return v; }
HVal mk_dbl(double d) { HVal v; v.k = HVal::DBL; v.d = d; return v; }
HVal mk_str(std::string s) { HVal v; v.k = HVal::STR; v.s = std::move(s); return v; }
HVal mk_bool(bool b) { HVal v; v.k = HVal::BOOL; v.i = b; return v; }
HVal mk_rid(uint32_t x) { HVal v; v.k = HVal::RID; v.v = x; return v; }

std::string num_str(const HVal &x) {
  if (x.k == HVal::INT) return std::to_string(x.i);
  char b[64];
  std::snprintf(b, sizeof(b), "%.17g", x.d);
  return b;
}
std::string to_str(const HVal &x) {  // String.valueOf for concatenation
  switch (x.k) {
    case HVal::NUL: return "";
    case HVal::STR: return x.s;
    case HVal::BOOL: return x.i ? "true" : "false";
    case HVal::INT:
    case HVal::DBL: return num_str(x);
    default: return "";
  }
}

class Evaluator {
 public:
  Evaluator(Graph &g, const Plan &p) : g_(g), p_(p) {}

  HVal value(const ExprP &e, const HVal &rec) {
    switch (e->kind) {
      case Expr::LIT: return lit(e->value);
      case Expr::PARAM: {
        const Value *v = p_.params.get(*e);
        if (!v) fail(OMX_E_EXECUTION, "missing value for query parameter " + expr_text(e));
        return lit(*v);
      }
      case Expr::FIELD: return field(rec, e->name);
      case Expr::MATH: return math(e->name, value(e->kids[0], rec), value(e->kids[1], rec));
      case Expr::CHAIN: {
        if (e->kids[0]->kind == Expr::CALL) fail(OMX_E_UNSUPPORTED, "function call in a RETURN expression");
        HVal cur = value(e->kids[0], rec);
        for (const Suffix &s : e->suffixes) cur = suffix(cur, s, rec);
        return cur;
      }
      case Expr::JSON: {
        HVal m;
        m.k = HVal::MAP;
        for (size_t i = 0; i < e->kids.size(); ++i) {
          m.keys.push_back(e->json_keys[i]);
          m.items.push_back(value(e->kids[i], rec));
        }
        return m;
      }
      case Expr::ARRAY: {
        HVal l;
        l.k = HVal::LIST;
        for (auto &k : e->kids) l.items.push_back(value(k, rec));
        return l;
      }
      case Expr::OR:
      case Expr::AND:
      case Expr::NOT:
      case Expr::CMP:
      case Expr::TRUTH: return mk_bool(boolean(e, rec));
      default: fail(OMX_E_UNSUPPORTED, "expression " + expr_text(e) + " in a RETURN item");
    }
  }

  bool boolean(const ExprP &c, const HVal &rec) {
    switch (c->kind) {
      case Expr::OR:
        for (auto &k : c->kids)
          if (boolean(k, rec)) return true;
        return false;
      case Expr::AND:
        for (auto &k : c->kids)
          if (!boolean(k, rec)) return false;
        return true;
      case Expr::NOT: return !boolean(c->kids[0], rec);
      case Expr::TRUTH: {
        HVal v = value(c->kids[0], rec);
        return v.k == HVal::BOOL && v.i;
      }
      case Expr::CMP: {
        HVal l = value(c->kids[0], rec), r = value(c->kids[1], rec);
        if (c->name == "=") return equals(l, r);
        if (c->name == "!=") return !equals(l, r);
        return compare(c->name, l, r);
      }
      default: {
        HVal v = value(c, rec);
        return v.k == HVal::BOOL && v.i;
      }
    }
  }

 private:
  Graph &g_;
  const Plan &p_;
  std::map<std::pair<const Suffix *, uint32_t>, std::vector<uint32_t>> adj_cache_;

 public:
  const RetAdj *fetched_ = nullptr;

  static HVal lit(const Value &v) {
    switch (v.kind) {
      case Value::INT: return mk_int(v.i);
      case Value::DBL: return mk_dbl(v.d);
      case Value::STR: return mk_str(v.s);
      case Value::BOOL: return mk_bool(v.i != 0);
      default: return HVal();
    }
  }

  HVal field(const HVal &base, const std::string &name) {
    switch (base.k) {
      case HVal::RID: {
        if (ieq(name, "@rid")) return base;
        if (ieq(name, "@class")) {
          ensure_vclass(g_);
          return mk_str(g_.classes[g_.h_vclass[base.v]].name);
        }
        // an edge record's `out` / `in` field: the vertex it links (the edge document's LINK fields)
        if (g_.edge_records && base.v >= g_.vertices && base.v < g_.V && (name == "out" || name == "in")) {
          ensure_links(g_);
          return mk_rid((name == "out" ? g_.h_etail : g_.h_ehead)[base.v - g_.vertices]);
        }
        const int pid = g_.prop_id(name);
        if (pid < 0) return HVal();
        Property &p = g_.props[pid];
        ensure_prop(g_, p);
        if (!p.h_present.empty() && !p.h_present[base.v]) return HVal();
        switch (p.type) {
          case OMX_PROP_DOUBLE: return mk_dbl(p.h_dbl[base.v]);
          case OMX_PROP_STRING: {
            const int64_t c = p.h_int[base.v];
            return c >= 0 && (size_t)c < p.dict.size() ? mk_str(p.dict[c]) : HVal();
          }
          case OMX_PROP_BOOL: return mk_bool(p.h_int[base.v] != 0);
          default: return mk_int(p.h_int[base.v]);
        }
      }
      case HVal::MAP:
        for (size_t i = 0; i < base.keys.size(); ++i)
          if (base.keys[i] == name) return base.items[i];
        return HVal();
      case HVal::LIST: {
        HVal l;
        l.k = HVal::LIST;
        for (auto &x : base.items) l.items.push_back(field(x, name));
        return l;
      }
      default: return HVal();
    }
  }

  HVal math(const std::string &op, const HVal &a, const HVal &b) {
    if (op == "+" && (a.k == HVal::STR || b.k == HVal::STR)) return mk_str(to_str(a) + to_str(b));
    if (a.k == HVal::NUL || b.k == HVal::NUL) return HVal();
    if (!is_num(a) || !is_num(b)) fail(OMX_E_EXECUTION, "arithmetic on non-numeric values in a RETURN expression");
    if (a.k == HVal::INT && b.k == HVal::INT) {
      const int64_t x = a.i, y = b.i;
      if (op == "+") return mk_int(x + y);
      if (op == "-") return mk_int(x - y);
      if (op == "*") return mk_int(x * y);
      if (y == 0) fail(OMX_E_EXECUTION, "division by zero in a RETURN expression");
      if (op == "/") return mk_int(x / y);
      return mk_int(x % y);
    }
    const double x = dbl(a), y = dbl(b);
    if (op == "+") return mk_dbl(x + y);
    if (op == "-") return mk_dbl(x - y);
    if (op == "*") return mk_dbl(x * y);
    if (op == "/") return mk_dbl(x / y);
    return mk_dbl(std::fmod(x, y));
  }

  // OQueryOperatorEquals.equals: null → false; records by identity; numbers by value; string vs number
  // by parsing the string as the number's type
  static bool equals(const HVal &a, const HVal &b) {
    if (a.k == HVal::NUL || b.k == HVal::NUL) return false;
    if (a.k == HVal::RID || b.k == HVal::RID) return a.k == b.k && a.v == b.v;
    if (is_num(a) && is_num(b)) return a.k == HVal::INT && b.k == HVal::INT ? a.i == b.i : dbl(a) == dbl(b);
    if (a.k == HVal::STR && is_num(b)) return str_num_eq(a.s, b);
    if (is_num(a) && b.k == HVal::STR) return str_num_eq(b.s, a);
    if (a.k != b.k) return false;
    if (a.k == HVal::STR) return a.s == b.s;
    if (a.k == HVal::BOOL) return a.i == b.i;
    return key(a) == key(b);
  }
  static bool str_num_eq(const std::string &s, const HVal &n) {
    char *end = nullptr;
    if (n.k == HVal::INT) {
      const long long x = std::strtoll(s.c_str(), &end, 10);
      return !s.empty() && end && *end == 0 && x == n.i;
    }
    const double x = std::strtod(s.c_str(), &end);
    return !s.empty() && end && *end == 0 && x == n.d;
  }
  static bool compare(const std::string &op, HVal a, HVal b) {
    if (a.k == HVal::NUL) {
      if (op == "<") return false;
      fail(OMX_E_EXECUTION, "NullPointerException: null left operand of " + op);
    }
    // a non-null left operand: iLeft.getClass() != iRight.getClass() dereferences the right one first
    // (P/OGtOperator.java:22-33, P/OLtOperator.java:22-36, P/OGeOperator.java:43-54, P/OLeOperator.java:22-33)
    if (b.k == HVal::NUL) fail(OMX_E_EXECUTION, "NullPointerException: null right operand of " + op);
    int c;
    if (is_num(a) && is_num(b)) {
      if (a.k == HVal::INT && b.k == HVal::INT) c = a.i < b.i ? -1 : a.i > b.i;
      else c = dbl(a) < dbl(b) ? -1 : dbl(a) > dbl(b);
    } else if (a.k == HVal::STR && is_num(b)) {
      const std::string bs = num_str(b);
      c = a.s < bs ? -1 : a.s > bs;
    } else if (is_num(a) && b.k == HVal::STR) {
      char *end = nullptr;
      const double y = std::strtod(b.s.c_str(), &end);
      if (b.s.empty() || !end || *end) return false;
      c = dbl(a) < y ? -1 : dbl(a) > y;
    } else if (a.k == HVal::STR && b.k == HVal::STR) {
      c = a.s < b.s ? -1 : a.s > b.s;
    } else {
      return false;
    }
    if (op == "<") return c < 0;
    if (op == "<=") return c <= 0;
    if (op == ">") return c > 0;
    return c >= 0;
  }

  // out()/in()/both() of one vertex: the adjacency parts of the plan's AdjSpec, read from the device CSR
  std::vector<uint32_t> neighbours(const Suffix *s, uint32_t v) {
    auto key = std::make_pair(s, v);
    if (fetched_) {  // a partitioned run: every list the expressions read was fetched from its owner
      auto f = fetched_->find(key);
      if (f == fetched_->end()) fail(OMX_E_INVALID, "internal: a RETURN adjacency list was not fetched");
      return f->second;
    }
    auto it = adj_cache_.find(key);
    if (it != adj_cache_.end()) return it->second;
    std::vector<uint32_t> out;
    const AdjSpec &a = p_.ret_adj.at(s);
    for (auto &part : a.parts) {
      const EdgeSet &es = g_.esets[part.first];
      uint64_t rp[2];
      HIP_CHECK(hipMemcpy(rp, g_.rp(es, part.second) + v, 16, hipMemcpyDeviceToHost));
      if (rp[1] > rp[0]) {
        const size_t off = out.size();
        out.resize(off + (rp[1] - rp[0]));
        HIP_CHECK(hipMemcpy(out.data() + off, g_.col(es, part.second) + rp[0], (rp[1] - rp[0]) * 4, hipMemcpyDeviceToHost));
      }
    }
    adj_cache_[key] = out;
    return out;
  }

  HVal suffix(const HVal &cur, const Suffix &s, const HVal &rec) {
    if (s.kind == Suffix::FIELD) return field(cur, s.name);
    if (s.kind == Suffix::METHOD) {
      const std::string m = lower(s.name);
      if (m == "out" || m == "in" || m == "both") {
        HVal l;
        l.k = HVal::LIST;
        auto add = [&](const HVal &x) {
          if (x.k != HVal::RID) return;
          for (uint32_t n : neighbours(&s, x.v)) l.items.push_back(mk_rid(n));
        };
        if (cur.k == HVal::LIST) {
          for (auto &x : cur.items) add(x);
        } else {
          add(cur);
        }
        return l;
      }
      if (m == "size") {
        if (cur.k == HVal::NUL) return mk_int(0);
        if (cur.k == HVal::LIST || cur.k == HVal::MAP) return mk_int((int64_t)cur.items.size());
        if (cur.k == HVal::STR) return mk_int((int64_t)cur.s.size());
        return mk_int(1);
      }
      if (m == "touppercase" || m == "tolowercase") {
        if (cur.k == HVal::NUL) return HVal();
        std::string t = cur.k == HVal::STR ? cur.s : to_str(cur);
        for (auto &ch : t) ch = (char)(m == "touppercase" ? std::toupper((unsigned char)ch) : std::tolower((unsigned char)ch));
        return mk_str(t);
      }
      fail(OMX_E_UNSUPPORTED, "method " + s.name + "() in a RETURN expression");
    }
    // selectors
    std::vector<HVal> lst;
    if (cur.k == HVal::LIST) lst = cur.items;
    else lst.push_back(cur);
    auto idx = [&](const ExprP &x) -> int64_t {
      HVal v = value(x, rec);
      return v.k == HVal::INT ? v.i : INT64_MIN;
    };
    HVal l;
    l.k = HVal::LIST;
    switch (s.sel) {
      case Suffix::SEL_RANGE: {
        const int64_t n = (int64_t)lst.size();
        int64_t a = idx(s.index), b = idx(s.index2);
        a = std::max<int64_t>(0, std::min(a, n));
        b = std::max<int64_t>(a, std::min(b, n));
        for (int64_t i = a; i < b; ++i) l.items.push_back(lst[i]);
        return l;
      }
      case Suffix::SEL_MULTI:
        for (auto &x : s.items) {
          const int64_t i = idx(x);
          if (i >= 0 && i < (int64_t)lst.size()) l.items.push_back(lst[i]);
        }
        return l;
      case Suffix::SEL_COND:
        for (auto &x : lst)
          if (boolean(s.index, x)) l.items.push_back(x);
        return l;
      default: {
        const int64_t i = idx(s.index);
        return i >= 0 && i < (int64_t)lst.size() ? lst[i] : HVal();
      }
    }
  }

 public:
  // canonical content of a value (ODocumentEqualityWrapper: documents equal by content, records by
  // identity); maps compare by key set, lists in order
  static std::string key(const HVal &x) {
    switch (x.k) {
      case HVal::NUL: return "n";
      case HVal::INT: return "i" + std::to_string(x.i);
      case HVal::DBL: {
        uint64_t b;
        std::memcpy(&b, &x.d, 8);
        return "d" + std::to_string(b);
      }
      case HVal::STR: return "s" + std::to_string(x.s.size()) + ":" + x.s;
      case HVal::BOOL: return x.i ? "b1" : "b0";
      case HVal::RID: return "r" + std::to_string(x.v);
      case HVal::LIST: {
        std::string o = "l" + std::to_string(x.items.size()) + "[";
        for (auto &y : x.items) o += key(y) + ",";
        return o + "]";
      }
      case HVal::MAP: {
        std::vector<size_t> ord(x.keys.size());
        for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return x.keys[a] < x.keys[b]; });
        std::string o = "m{";
        for (size_t i : ord) o += std::to_string(x.keys[i].size()) + ":" + x.keys[i] + "=" + key(x.items[i]) + ",";
        return o + "}";
      }
    }
    return "";
  }
};

// RIDs of the result (and JSON text of list / map cells, RIDs as "#cluster:position")
void finish(HVal &x, const Graph &g) {
  if (x.k == HVal::RID) x.rid = g.h_rids[x.v];
  for (auto &y : x.items) finish(y, g);
}
std::string jesc(const std::string &s) {
  std::string o = "\"";
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') { o += '\\'; o += (char)c; }
    else if (c < 0x20) { char b[8]; std::snprintf(b, sizeof(b), "\\u%04x", c); o += b; }
    else o += (char)c;
  }
  return o + "\"";
}
std::string to_json(const HVal &x) {
  switch (x.k) {
    case HVal::NUL: return "null";
    case HVal::INT:
    case HVal::DBL: return num_str(x);
    case HVal::STR: return jesc(x.s);
    case HVal::BOOL: return x.i ? "true" : "false";
    case HVal::RID: return jesc("#" + std::to_string(x.rid >> 48) + ":" + std::to_string(x.rid & ((1ull << 48) - 1)));
    case HVal::LIST: {
      std::string o = "[";
      for (size_t i = 0; i < x.items.size(); ++i) o += (i ? "," : "") + to_json(x.items[i]);
      return o + "]";
    }
    case HVal::MAP: {
      std::string o = "{";
      for (size_t i = 0; i < x.items.size(); ++i) o += (i ? "," : "") + jesc(x.keys[i]) + ":" + to_json(x.items[i]);
      return o + "}";
    }
  }
  return "null";
}

}  // namespace

std::vector<Document> build_documents(Graph &g, const Plan &p, const std::vector<const uint32_t *> &cols, uint64_t n,
                                      int64_t limit, hipStream_t s, const RetAdj *fetched) {
  const size_t k = cols.size();
  std::vector<uint32_t> h(n * k);
  for (size_t c = 0; c < k; ++c)
    if (n) HIP_CHECK(hipMemcpyAsync(h.data() + c * n, cols[c], n * 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  ensure_rids(g);
  Evaluator ev(g, p);
  ev.fetched_ = fetched;
  std::vector<Document> docs;
  std::unordered_set<std::string> seen;
  const uint64_t cap = limit > -1 ? (uint64_t)std::max<int64_t>(limit, 1) : UINT64_MAX;
  for (uint64_t r = 0; r < n && docs.size() < cap; ++r) {
    // the matched map as a document: alias → record (null for an unmatched optional node)
    HVal mapdoc;
    mapdoc.k = HVal::MAP;
    for (size_t c = 0; c < k; ++c) {
      mapdoc.keys.push_back(p.aliases[p.out_aliases[c]]);
      const uint32_t v = h[c * n + r];
      mapdoc.items.push_back(v < g.V ? mk_rid(v) : HVal());
    }
    Document d;
    if (p.proj == Plan::PROJ_JSON) {
      HVal m = ev.value(p.returns[0].expr, mapdoc);
      d = m.items;
    } else {
      for (auto &ri : p.returns)
        d.push_back(ri.expr->kind == Expr::FIELD ? [&] {  // a bare identifier reads the matched map
          for (size_t c = 0; c < k; ++c)
            if (mapdoc.keys[c] == ri.expr->name) return mapdoc.items[c];
          return HVal();
        }()
                                                 : ev.value(ri.expr, mapdoc));
    }
    std::string key;
    for (size_t i = 0; i < d.size(); ++i) key += std::to_string(p.out_names[i].size()) + ":" + p.out_names[i] + "=" + Evaluator::key(d[i]) + ";";
    if (!seen.insert(key).second) continue;
    for (auto &x : d) {
      finish(x, g);
      if (x.k == HVal::LIST || x.k == HVal::MAP) x.json = to_json(x);
    }
    docs.push_back(std::move(d));
  }
  return docs;
}

}  // namespace omx
