// plan.cpp — restates the reference's MATCH planning and compiles it to device steps.
//
//   parse-time      OMatchStatement.parse (P/OMatchStatement.java:129-178): assignDefaultAliases
//                   :202-218, Pattern.addExpression (P/Pattern.java:15-27), addAliases :905-948,
//                   rebindFilters :185-195, Pattern.validate (P/Pattern.java:48-65)
//   estimates       estimateRootEntries :874-903, OWhereClause.estimate (P/OWhereClause.java:57-95)
//   edge order      sortEdges :272-325 (stable sort of OPair by estimate, CM/util/OPair.java:97-99)
//   candidates      calculateMatch :334-386 (prefetch below threshold 20, getNextAlias :858-872)
//   per-edge rules  processContext :412-568 — forward: OMatchPathItem.executeTraversal applies the
//                   target's WHERE (P/OMatchPathItem.java:49-107); reverse: executeReverse, WHERE only
//                   in the free branch (:553-554); bound target → existence (:468-477); prefetched
//                   target → candidate membership (:478-490), free → bind (:491-497)
//   cartesian       expandCartesianProduct :620-650
//   projection      addResult :661-729 ($elements, $pathElements, $patterns/$matches, $paths, aliases)
#include "plan.h"

#include <algorithm>
#include <cmath>
#include <map>
#include <optional>
#include <set>
#include <sstream>

namespace omx {

const Value *Params::get(const Expr &p) const {
  if (!p.name.empty()) {
    for (auto &kv : named)
      if (kv.first == p.name) return &kv.second;
    return nullptr;
  }
  if (p.param_index >= 0 && (size_t)p.param_index < positional.size()) return &positional[p.param_index];
  return nullptr;
}

namespace {

const std::string kDefaultPrefix = "$ORIENT_DEFAULT_ALIAS_";
const int64_t kThreshold = 20;  // OMatchStatement.threshold (:35)
const int64_t kLongMax = INT64_MAX;

struct PNode {
  std::string alias;
  std::vector<int> out, in;  // edge indices, insertion order (LinkedHashSet)
  bool optional = false;
};
struct PEdge {
  const PathItem *item;
  int out, in;
};

bool is_num(const Value &v) { return v.kind == Value::INT || v.kind == Value::DBL; }
double as_dbl(const Value &v) { return v.kind == Value::DBL ? v.d : (double)v.i; }

// OQueryOperatorEquals.equals (S/operator/OQueryOperatorEquals.java:67-97) on constants.
bool const_equals(const Value &a, const Value &b) {
  if (a.kind == Value::NUL || b.kind == Value::NUL) return false;
  if (is_num(a) && is_num(b)) {
    if (a.kind == Value::INT && b.kind == Value::INT) return a.i == b.i;
    return as_dbl(a) == as_dbl(b);
  }
  if (a.kind == Value::STR && b.kind == Value::STR) return a.s == b.s;
  if (a.kind == Value::BOOL && b.kind == Value::BOOL) return a.i == b.i;
  if (a.kind == Value::STR && is_num(b)) return a.s == (b.kind == Value::INT ? std::to_string(b.i) : std::to_string(b.d));
  if (is_num(a) && b.kind == Value::STR) {
    char *end = nullptr;
    double x = std::strtod(b.s.c_str(), &end);
    return end && *end == 0 && !b.s.empty() && x == as_dbl(a);
  }
  return false;
}

class Planner {
 public:
  Planner(const Statement &st, const Graph &g, const Params &params) : st_(st), g_(g), params_(params) {}

  std::unique_ptr<Plan> run(bool logical_only) {
    plan_ = std::make_unique<Plan>();
    exprs_ = st_.expressions;  // private copy: default aliases / rebound filters are assigned here
    assign_default_aliases();
    // the logical plan (explain) keeps the reference's edge nodes; the device plan fuses them
    // (with edge records, $paths / $pathElements read the edge nodes: those are kept)
    if (!logical_only && !(g_.edge_records && (returns_has("$paths") || returns_has("$pathElements")))) fuse_edge_items();
    for (auto &e : exprs_) add_expression(e);
    for (auto &e : exprs_) {
      add_aliases(e.origin);
      for (auto &it : e.items) add_aliases(it.filter);
    }
    validate();
    if (!logical_only) type_nodes();
    for (auto &n : nodes_) {
      plan_->aliases.push_back(n.alias);
      plan_->explicit_alias.push_back(n.alias.rfind(kDefaultPrefix, 0) != 0);
    }
    estimate_root_entries();
    for (auto &kv : plan_->estimates)
      if (kv.second == 0) plan_->empty = true;
    sort_edges();
    choose_prefetch_and_root();
    if (logical_only) return std::move(plan_);
    plan_->params = params_;
    compile_steps();
    compile_projection();
    plan_->limit = st_.has_limit ? st_.limit : -1;
    return std::move(plan_);
  }

  // TRAVERSE ... STRATEGY BREADTH_FIRST / SELECT expand(<chain>) FROM <target> (ChainSpec)
  std::unique_ptr<Plan> run_chain(bool logical_only) {
    plan_ = std::make_unique<Plan>();
    Plan &p = *plan_;
    const bool trav = st_.kind == Statement::TRAVERSE;
    p.kind = trav ? Plan::TRAVERSE : Plan::SELECT;
    if (!trav && st_.fields[0]->kind == Expr::CALL && ieq(st_.fields[0]->name, "shortestPath")) p.kind = Plan::SHORTEST_PATH;
    p.out_names = {"@rid"};
    p.limit = st_.has_limit ? st_.limit : -1;
    if (logical_only) return std::move(plan_);
    p.params = params_;
    if (!st_.unsupported.empty()) unsupported(st_.unsupported);
    const Target &t = st_.target;
    if (!t.other.empty()) unsupported("target " + t.other + " (only records and classes on the device)");
    ChainSpec &c = p.chain;
    if (!t.class_name.empty()) {
      c.root_class = g_.class_id(t.class_name);
      if (c.root_class < 0) fail(OMX_E_EXECUTION, "Class '" + t.class_name + "' was not found in current database");
      if (g_.classes[c.root_class].is_edge) unsupported("a target of edge records");
    }
    for (auto &r : t.rids)
      if (r.first >= 0 && r.second >= 0) c.root_rids.push_back(((uint64_t)r.first << 48) | (uint64_t)r.second);
    legacy_ = true;
    if (trav) {
      // OTraverse runs the BREADTH_FIRST work list level by level; DEPTH_FIRST is a sequential stack walk
      if (!st_.breadth_first) unsupported("TRAVERSE with the DEPTH_FIRST strategy (only BREADTH_FIRST on the device)");
      AdjSpec cat;
      std::set<std::string> seen;  // traverse.fields(Set): a field given twice is traversed once
      for (auto &f : st_.fields) {
        if (!seen.insert(lower(expr_text(f))).second) continue;
        AdjSpec a = move_call(f, "traverse field");
        cat.parts.insert(cat.parts.end(), a.parts.begin(), a.parts.end());
        cat.sorted = cat.sorted && a.sorted;
      }
      if (seen.size() > 1)
        unsupported("TRAVERSE of several fields (the reference keeps them in a HashSet: their order is unspecified)");
      if ((int)cat.parts.size() > kMaxAdjParts) unsupported("too many edge classes in one traversal");
      c.hops.push_back(cat);
      c.pred_prog = add_prog(st_.where, true);
      c.max_depth = st_.max_depth;
    } else if (st_.fields[0]->kind == Expr::CALL && ieq(st_.fields[0]->name, "shortestPath")) {
      compile_shortest_path(st_.fields[0]);
    } else {
      // expand(f0(...).f1(...)...): every call moves the whole list (OSQLEngine.foreachRecord keeps the
      // order and the duplicates); outE('L').inV() / inE('L').outV() pairs are one hop
      if (!st_.expand) unsupported("a SELECT projection other than shortestPath()");
      if (t.rids.empty() && t.class_name.empty()) unsupported("SELECT expand() without a FROM target");
      const ExprP &x = st_.fields[0];
      std::vector<std::pair<std::string, std::vector<ExprP>>> calls;
      if (x->kind == Expr::CALL) {
        calls.emplace_back(x->name, x->kids);
      } else if (x->kind == Expr::CHAIN && x->kids[0]->kind == Expr::CALL) {
        calls.emplace_back(x->kids[0]->name, x->kids[0]->kids);
        for (auto &sfx : x->suffixes) {
          if (sfx.kind != Suffix::METHOD) unsupported("expand() argument " + expr_text(x));
          calls.emplace_back(sfx.name, sfx.args);
        }
      } else {
        unsupported("expand() argument " + expr_text(x));
      }
      for (size_t i = 0; i < calls.size(); ++i) {
        const std::string m = lower(calls[i].first);
        const std::vector<std::string> labels = labels_of(calls[i].second);
        if ((m == "oute" || m == "ine") && i + 1 < calls.size() && calls[i + 1].second.empty() &&
            lower(calls[i + 1].first) == (m == "oute" ? "inv" : "outv")) {
          c.hops.push_back(adjacency(m == "oute" ? "out" : "in", labels));
          ++i;
          continue;
        }
        if (m != "out" && m != "in" && m != "both") unsupported("function " + calls[i].first + "() in expand() on the device");
        c.hops.push_back(adjacency(m, labels));
      }
      c.pred_prog = add_prog(st_.where, false);
    }
    return std::move(plan_);
  }

 private:
  // a record argument: a RID literal, or a string / parameter holding "#c:p" (graph.getVertex(Object))
  uint64_t rid_arg(const ExprP &e, const char *what) const {
    if (e->kind == Expr::RID) return (uint64_t)e->value.i;
    auto v = fold(e);
    if (v && v->kind == Value::STR) {
      const std::string &x = v->s;
      const size_t c = x.find(':');
      if (!x.empty() && x[0] == '#' && c != std::string::npos) {
        char *e1 = nullptr, *e2 = nullptr;
        const long long cl = std::strtoll(x.c_str() + 1, &e1, 10), pos = std::strtoll(x.c_str() + c + 1, &e2, 10);
        if (e1 == x.c_str() + c && e2 && *e2 == 0 && cl >= 0 && pos >= 0) return ((uint64_t)cl << 48) | (uint64_t)pos;
      }
    }
    unsupported(std::string("shortestPath() ") + what + " " + expr_text(e) + " (a record id on the device)");
  }

  // shortestPath(<source>, <destination>[, <direction>[, <edge class>[, {maxDepth: n}]]]): the
  // bidirectional BFS of OSQLFunctionShortestPath.execute (GF/OSQLFunctionShortestPath.java:85-200)
  void compile_shortest_path(const ExprP &f) {
    Plan &p = *plan_;
    p.kind = Plan::SHORTEST_PATH;
    ChainSpec &c = p.chain;
    c.expand_rows = st_.expand;
    if (!st_.expand) p.out_names = {st_.alias.empty() ? std::string("shortestPath") : st_.alias};
    const Target &t = st_.target;
    if (!t.rids.empty() || !t.class_name.empty() || !t.other.empty())
      unsupported("shortestPath() evaluated per record of a FROM target");
    const auto &a = f->kids;
    if (a.size() < 2 || a.size() > 5) fail(OMX_E_PARSE, "Syntax error: shortestPath(<sourceVertex>, <destinationVertex>, [<direction>, [ <edgeTypeAsString> ]])");
    c.sp_src = rid_arg(a[0], "source");
    c.sp_dst = rid_arg(a[1], "destination");
    std::string left = "both";
    if (a.size() > 2) {
      auto v = fold(a[2]);
      if (!v) unsupported("non-constant shortestPath() direction");
      if (v->kind != Value::NUL) {  // Direction.valueOf(toUpperCase): OUT / IN / BOTH
        if (v->kind != Value::STR) fail(OMX_E_EXECUTION, "No enum constant for direction " + expr_text(a[2]));
        left = lower(v->s);
        if (left != "out" && left != "in" && left != "both")
          fail(OMX_E_EXECUTION, "No enum constant com.tinkerpop.blueprints.Direction." + v->s);
      }
    }
    const std::string right = left == "out" ? "in" : left == "in" ? "out" : "both";
    std::vector<std::string> labels;
    if (a.size() > 3) {
      auto v = fold(a[3]);
      if (!v) unsupported("non-constant shortestPath() edge class");
      if (v->kind == Value::STR) labels.push_back(v->s);
      else if (v->kind != Value::NUL) labels.push_back(expr_text(a[3]));
    }
    c.sp_left = adjacency(left, labels);
    c.sp_right = adjacency(right, labels);
    if (a.size() > 4 && a[4]->kind == Expr::JSON) {  // bindAdditionalParams: {maxDepth: n}
      for (size_t i = 0; i < a[4]->json_keys.size(); ++i)
        if (a[4]->json_keys[i] == "maxDepth") {
          auto v = fold(a[4]->kids[i]);
          if (v && v->kind == Value::INT) c.sp_max_depth = (int)v->i;
          else if (v && v->kind == Value::DBL) c.sp_max_depth = (int)v->d;
          else if (v && v->kind == Value::STR) {
            char *e = nullptr;
            const long x = std::strtol(v->s.c_str(), &e, 10);
            if (e && *e == 0 && !v->s.empty()) c.sp_max_depth = (int)x;
          }
        }
    } else if (a.size() > 4 && !(fold(a[4]) && fold(a[4])->kind == Value::NUL)) {
      unsupported("shortestPath() additional parameters other than a {maxDepth: n} map");
    }
  }

  std::vector<std::string> labels_of(const std::vector<ExprP> &args) const {
    std::vector<std::string> labels;
    for (auto &a : args) {
      auto v = fold(a);
      if (!v || v->kind != Value::STR) unsupported("non-constant edge label");
      labels.push_back(v->s);
    }
    return labels;
  }
  // out('L', ...) / in(...) / both(...) as a field of TRAVERSE
  AdjSpec move_call(const ExprP &f, const char *what) const {
    if (f->kind != Expr::CALL) unsupported(std::string(what) + " " + expr_text(f) + " (only out()/in()/both() on the device)");
    const std::string m = lower(f->name);
    if (m != "out" && m != "in" && m != "both")
      unsupported(std::string(what) + " " + expr_text(f) + " (only out()/in()/both() on the device)");
    return adjacency(m, labels_of(f->kids));
  }

  const Statement &st_;
  bool legacy_ = false;  // compiling a legacy-SQL condition (TRAVERSE WHILE, SELECT WHERE)
  const Graph &g_;
  const Params &params_;
  std::unique_ptr<Plan> plan_;
  std::vector<MatchExpression> exprs_;
  std::vector<PNode> nodes_;
  std::map<std::string, int> alias_idx_;
  std::vector<PEdge> edges_;
  std::vector<std::string> class_order_, filter_order_;  // LinkedHashMap insertion orders
  std::map<std::string, std::string> alias_class_;
  std::map<std::string, std::vector<ExprP>> alias_where_;
  std::vector<std::pair<int, bool>> sorted_;  // (edge index, forward)
  std::set<int> prefetched_;
  int root_ = -1;

  // ---- parse-time -------------------------------------------------------------------------------
  void assign_default_aliases() {
    int counter = 0;
    for (auto &e : exprs_) {
      if (e.origin.alias.empty()) e.origin.alias = kDefaultPrefix + std::to_string(counter++);
      for (auto &it : e.items)
        if (it.filter.alias.empty()) it.filter.alias = kDefaultPrefix + std::to_string(counter++);
    }
  }
  // `outE('L').inV()` / `inE('L').outV()` whose edge step has no filter: its node is an anonymous edge
  // alias that no other item and no $matches/$patterns/explicit RETURN reads, and OSQLFunctionMove's e2v
  // yields one vertex per edge (GF/OSQLFunctionMove.java:122-143), so the pair is out('L') / in('L') with
  // the edge multiplicity, which the distinct result rows absorb. $paths / $pathElements would expose
  // the edge records: compile_projection leaves those to the reference engine.
  bool fused_edges_ = false;
  void fuse_edge_items() {
    for (auto &e : exprs_) {
      std::vector<PathItem> items;
      for (size_t i = 0; i < e.items.size(); ++i) {
        const PathItem &a = e.items[i];
        const std::string m = lower(a.method);
        if (!a.is_multi && !a.has_filter && (m == "oute" || m == "ine") && i + 1 < e.items.size()) {
          const PathItem &b = e.items[i + 1];
          const std::string v = lower(b.method);
          if (!b.is_multi && b.labels.empty() && ((m == "oute" && v == "inv") || (m == "ine" && v == "outv")) &&
              !b.filter.while_ && !b.filter.has_max_depth) {
            PathItem f = b;
            f.method = m == "oute" ? "out" : "in";
            f.labels = a.labels;
            items.push_back(f);
            fused_edges_ = true;
            ++i;
            continue;
          }
        }
        items.push_back(a);
      }
      e.items.swap(items);
    }
  }
  bool returns_has(const char *name) const {
    for (auto &r : st_.returns)
      if (ieq(r.text, name)) return true;
    return false;
  }
  // the record kind each pattern node binds (OSQLFunctionMove: out/in/both and outE/inE/bothE start at a
  // vertex, outV/inV/bothV at an edge record; GF/OSQLFunctionMove.java:66-144): a node reached both ways,
  // or whose class is of the other kind, matches no record in the reference; the device leaves it to the
  // reference engine
  std::vector<char> edge_node_;  // per node: 1 = binds edge records
  void type_nodes() {
    std::vector<int> kind(nodes_.size(), 0);  // 0 unknown, 1 vertex, 2 edge
    auto set = [&](int n, int k) {
      if (kind[n] && kind[n] != k)
        unsupported("pattern node " + nodes_[n].alias + " reached both as a vertex and as an edge record");
      kind[n] = k;
    };
    for (auto &e : edges_) {
      const PathItem &it = *e.item;
      const std::string m = it.is_multi ? std::string() : lower(it.method);
      if (m == "oute" || m == "ine" || m == "bothe") {
        set(e.out, 1);
        set(e.in, 2);
      } else if (m == "outv" || m == "inv" || m == "bothv") {
        set(e.out, 2);
        set(e.in, 1);
      } else {
        set(e.out, 1);
        set(e.in, 1);
      }
    }
    edge_node_.assign(nodes_.size(), 0);
    for (size_t n = 0; n < nodes_.size(); ++n) {
      auto c = alias_class_.find(nodes_[n].alias);
      if (c != alias_class_.end()) {
        const int ci = g_.class_id(c->second);
        if (ci >= 0) {
          const int k = g_.classes[ci].is_edge ? 2 : 1;
          if (kind[n] && kind[n] != k)
            unsupported("pattern node " + nodes_[n].alias + " of class " + c->second + " reached as a" +
                        (kind[n] == 2 ? "n edge record" : " vertex"));
          kind[n] = k;
        }
      }
      edge_node_[n] = kind[n] == 2;
      if (edge_node_[n] && !g_.edge_records)
        unsupported("edge node " + nodes_[n].alias + " on a snapshot without edge records (lightweight edges)");
    }
  }
  int node(const MatchFilter &f) {
    auto it = alias_idx_.find(f.alias);
    int id;
    if (it == alias_idx_.end()) {
      id = (int)nodes_.size();
      nodes_.push_back(PNode{f.alias});
      alias_idx_[f.alias] = id;
    } else {
      id = it->second;
    }
    if (f.optional) nodes_[id].optional = true;
    return id;
  }
  void add_expression(const MatchExpression &e) {
    int origin = node(e.origin);
    for (auto &it : e.items) {
      int nxt = node(it.filter);
      edges_.push_back(PEdge{&it, origin, nxt});
      nodes_[origin].out.push_back((int)edges_.size() - 1);
      nodes_[nxt].in.push_back((int)edges_.size() - 1);
      origin = nxt;
    }
  }
  void add_aliases(const MatchFilter &f) {
    if (f.where) {
      if (!alias_where_.count(f.alias)) filter_order_.push_back(f.alias);
      alias_where_[f.alias].push_back(f.where);
    }
    if (!f.class_name.empty()) {
      auto it = alias_class_.find(f.alias);
      if (it == alias_class_.end()) {
        alias_class_[f.alias] = f.class_name;
        class_order_.push_back(f.alias);
      } else {
        int a = g_.class_id(f.class_name), b = g_.class_id(it->second);
        if (a < 0 || b < 0) fail(OMX_E_EXECUTION, "class not defined: " + (a < 0 ? f.class_name : it->second));
        if (g_.is_subclass_of(a, b)) it->second = f.class_name;
        else if (!g_.is_subclass_of(b, a))
          fail(OMX_E_EXECUTION, "classes defined for alias " + f.alias + " (" + f.class_name + ", " + it->second +
                                    ") are not in the same hierarchy");
      }
    }
  }
  void validate() {
    for (auto &n : nodes_)
      if (n.optional) {
        if (!n.out.empty())
          fail(OMX_E_PARSE, "In current MATCH version, optional nodes are allowed only on right terminal nodes");
        if (n.in.empty()) fail(OMX_E_PARSE, "In current MATCH version, optional nodes must have at least one incoming pattern edge");
      }
  }
  // the alias's whole WHERE (AND of its fragments): what the estimates see (OWhereClause.estimate)
  ExprP where_of(const std::string &alias) const {
    auto it = alias_where_.find(alias);
    if (it == alias_where_.end()) return nullptr;
    auto a = std::make_shared<Expr>();
    a->kind = Expr::AND;
    a->kids = it->second;
    return a;
  }

  // `$matched.X op $currentMatch` (either order, op = / == / != / <>): a row-level conjunct
  static bool row_cmp(const ExprP &e, std::string *alias, bool *eq) {
    if (!e || e->kind != Expr::CMP) return false;
    const std::string &op = e->name;
    if (op != "=" && op != "==" && op != "!=" && op != "<>") return false;
    auto is_cur = [](const ExprP &x) { return x->kind == Expr::VAR && ieq(x->name, "$currentMatch"); };
    auto matched = [](const ExprP &x, std::string *a) {
      if (x->kind != Expr::CHAIN || x->suffixes.size() != 1 || x->suffixes[0].kind != Suffix::FIELD) return false;
      if (x->kids[0]->kind != Expr::VAR || !ieq(x->kids[0]->name, "$matched")) return false;
      *a = x->suffixes[0].name;
      return true;
    };
    const ExprP &L = e->kids[0], &R = e->kids[1];
    if (!((is_cur(R) && matched(L, alias)) || (is_cur(L) && matched(R, alias)))) return false;
    *eq = op == "=" || op == "==";
    return true;
  }
  static void flatten_and(const ExprP &e, std::vector<ExprP> &out) {
    if (e->kind == Expr::AND) {
      for (auto &k : e->kids) flatten_and(k, out);
    } else {
      out.push_back(e);
    }
  }
  // the alias's WHERE without its row-level conjuncts (what a per-vertex bitmap can hold), and those
  // conjuncts as (alias, equal)
  ExprP vertex_where_of(const std::string &alias, std::vector<std::pair<std::string, bool>> *rows = nullptr) const {
    ExprP w = where_of(alias);
    if (!w) return nullptr;
    std::vector<ExprP> conj, keep;
    flatten_and(w, conj);
    for (auto &c : conj) {
      std::string a;
      bool eq;
      if (row_cmp(c, &a, &eq)) {
        if (rows) rows->emplace_back(a, eq);
      } else {
        keep.push_back(c);
      }
    }
    if (keep.empty()) return nullptr;
    auto a = std::make_shared<Expr>();
    a->kind = Expr::AND;
    a->kids = keep;
    return a;
  }
  bool has_row_conds(const std::string &alias) const {
    std::vector<std::pair<std::string, bool>> r;
    vertex_where_of(alias, &r);
    return !r.empty();
  }

  // ---- estimates -------------------------------------------------------------------------------
  std::optional<Value> fold(const ExprP &e) const {
    if (!e) return std::nullopt;
    switch (e->kind) {
      case Expr::LIT: return e->value;
      case Expr::PARAM: {
        const Value *v = params_.get(*e);
        if (!v) fail(OMX_E_EXECUTION, "missing value for query parameter " + expr_text(e));
        return *v;
      }
      case Expr::MATH: {
        auto a = fold(e->kids[0]), b = fold(e->kids[1]);
        if (!a || !b) return std::nullopt;
        if (e->name == "+" && (a->kind == Value::STR || b->kind == Value::STR)) {
          auto str = [](const Value &v) {
            return v.kind == Value::STR ? v.s : v.kind == Value::INT ? std::to_string(v.i)
                                                : v.kind == Value::NUL ? std::string() : std::to_string(v.d);
          };
          return Value::Str(str(*a) + str(*b));
        }
        if (!is_num(*a) || !is_num(*b)) return Value();
        if (a->kind == Value::INT && b->kind == Value::INT) {
          int64_t x = a->i, y = b->i;
          if (e->name == "+") return Value::Int(x + y);
          if (e->name == "-") return Value::Int(x - y);
          if (e->name == "*") return Value::Int(x * y);
          if (y == 0) unsupported("integer division by zero in a constant expression");
          if (e->name == "/") return Value::Int(x / y);
          return Value::Int(x % y);
        }
        double x = as_dbl(*a), y = as_dbl(*b);
        if (e->name == "+") return Value::Dbl(x + y);
        if (e->name == "-") return Value::Dbl(x - y);
        if (e->name == "*") return Value::Dbl(x * y);
        if (e->name == "/") return Value::Dbl(x / y);
        return Value::Dbl(std::fmod(x, y));
      }
      case Expr::CMP: {
        auto a = fold(e->kids[0]), b = fold(e->kids[1]);
        if (!a || !b) return std::nullopt;
        const std::string &op = e->name;
        if (op == "=") return Value::Bool(const_equals(*a, *b));
        if (op == "!=") return Value::Bool(!const_equals(*a, *b));
        if (a->kind == Value::NUL) {
          if (op == "<") return Value::Bool(false);
          unsupported("comparison with a null left operand (NullPointerException in the reference)");
        }
        if (b->kind == Value::NUL) unsupported("comparison with a null right operand (NullPointerException in the reference)");
        int c;
        if (is_num(*a) && is_num(*b)) {
          if (a->kind == Value::INT && b->kind == Value::INT) c = a->i < b->i ? -1 : a->i > b->i;
          else c = as_dbl(*a) < as_dbl(*b) ? -1 : as_dbl(*a) > as_dbl(*b);
        } else if (a->kind == Value::STR && b->kind == Value::STR) {
          c = a->s < b->s ? -1 : a->s > b->s;
        } else {
          unsupported("comparison of constants of different types");
        }
        if (op == "<") return Value::Bool(c < 0);
        if (op == "<=") return Value::Bool(c <= 0);
        if (op == ">") return Value::Bool(c > 0);
        return Value::Bool(c >= 0);
      }
      case Expr::AND:
      case Expr::OR: {
        bool all = true, any = false;
        for (auto &k : e->kids) {
          auto v = fold(k);
          if (!v) return std::nullopt;
          bool b = v->kind == Value::BOOL && v->i;
          all = all && b;
          any = any || b;
        }
        return Value::Bool(e->kind == Expr::AND ? all : any);
      }
      case Expr::NOT: {
        auto v = fold(e->kids[0]);
        if (!v) return std::nullopt;
        return Value::Bool(!(v->kind == Value::BOOL && v->i));
      }
      case Expr::TRUTH: {
        auto v = fold(e->kids[0]);
        if (!v) return std::nullopt;
        return Value::Bool(v->kind == Value::BOOL && v->i);
      }
      default: return std::nullopt;
    }
  }

  // OBooleanExpression.flatten: disjunctive normal form as a list of AND blocks.
  std::vector<std::vector<ExprP>> flatten(const ExprP &e) const {
    if (e->kind == Expr::OR) {
      std::vector<std::vector<ExprP>> out;
      for (auto &k : e->kids) {
        auto f = flatten(k);
        out.insert(out.end(), f.begin(), f.end());
      }
      return out;
    }
    if (e->kind == Expr::AND) {
      std::vector<std::vector<ExprP>> blocks{{}};
      for (auto &k : e->kids) {
        auto f = flatten(k);
        std::vector<std::vector<ExprP>> nb;
        for (auto &b : blocks)
          for (auto &x : f) {
            auto y = b;
            y.insert(y.end(), x.begin(), x.end());
            nb.push_back(y);
          }
        blocks.swap(nb);
      }
      return blocks;
    }
    return {{e}};
  }

  int64_t estimate(int cls, const ExprP &where) const {
    int64_t count = (int64_t)g_.count(cls);
    if (count > 1) count /= 2;
    if (count < kThreshold) return count;
    int64_t indexes_count = 0;
    for (auto &block : flatten(where)) {
      std::vector<std::pair<std::string, Value>> conds;  // getEqualityOperations (P/OWhereClause.java:222-236)
      for (auto &b : block)
        if (b->kind == Expr::CMP && b->name == "=" && b->kids[0]->kind == Expr::FIELD &&
            (b->kids[1]->kind == Expr::LIT || b->kids[1]->kind == Expr::PARAM))
          conds.emplace_back(b->kids[0]->name, *fold(b->kids[1]));
      int64_t est = kLongMax;
      for (auto &ix : g_.indexes) {
        if (!g_.is_subclass_of(cls, ix.cls)) continue;
        const Value *key = nullptr;
        for (auto &c : conds)
          if (c.first == g_.props[ix.prop].name) key = &c.second;
        if (!key) continue;
        int64_t hits = g_.index_hits(ix.cls, ix.prop, *key);
        int64_t n = ix.unique ? (hits > 0 ? 1 : kLongMax) : hits;
        if (n < est) est = n;
      }
      if (est > count) return count;
      indexes_count += est;
    }
    return std::min(indexes_count, count);
  }

  void estimate_root_entries() {
    std::vector<std::string> all = class_order_;
    for (auto &a : filter_order_)
      if (std::find(all.begin(), all.end(), a) == all.end()) all.push_back(a);
    for (auto &alias : all) {
      auto it = alias_class_.find(alias);
      if (it == alias_class_.end()) continue;
      int c = g_.class_id(it->second);
      if (c < 0) fail(OMX_E_EXECUTION, "class not defined: " + it->second);
      ExprP w = where_of(alias);
      plan_->estimates.emplace_back(alias, w ? estimate(c, w) : (int64_t)g_.count(c));
    }
  }

  void sort_edges() {
    std::vector<std::pair<int64_t, std::string>> weights;
    for (auto &kv : plan_->estimates) weights.emplace_back(kv.second, kv.first);
    std::stable_sort(weights.begin(), weights.end(),
                     [](const std::pair<int64_t, std::string> &a, const std::pair<int64_t, std::string> &b) {
                       return a.first < b.first;
                     });
    std::set<int> tedges, tnodes;
    std::vector<int> next;
    auto in_next = [&](int n) { return std::find(next.begin(), next.end(), n) != next.end(); };
    while (sorted_.size() < edges_.size()) {
      for (auto &w : weights) {
        int root = alias_idx_.at(w.second);
        if (nodes_[root].optional) continue;
        if (!tnodes.count(root)) {
          next.push_back(root);
          break;
        }
      }
      if (next.empty()) break;
      while (!next.empty()) {
        int n = next.front();
        next.erase(next.begin());
        tnodes.insert(n);
        for (int e : nodes_[n].out)
          if (!tedges.count(e)) {
            sorted_.emplace_back(e, true);
            tedges.insert(e);
            if (!tnodes.count(edges_[e].in) && !in_next(edges_[e].in)) next.push_back(edges_[e].in);
          }
        for (int e : nodes_[n].in)
          if (!tedges.count(e) && edges_[e].item->bidirectional()) {
            sorted_.emplace_back(e, false);
            tedges.insert(e);
            if (!tnodes.count(edges_[e].out) && !in_next(edges_[e].out)) next.push_back(edges_[e].out);
          }
      }
    }
    for (auto &s : sorted_)
      plan_->sorted_edges.emplace_back(nodes_[edges_[s.first].out].alias, nodes_[edges_[s.first].in].alias, s.second);
  }

  void choose_prefetch_and_root() {
    bool found = false;
    for (auto &kv : plan_->estimates)
      if (kv.second < kThreshold) {
        prefetched_.insert(alias_idx_.at(kv.first));
        plan_->prefetched.push_back(kv.first);
        found = true;
      }
    if (!found && !plan_->estimates.empty()) {  // getNextAlias (:858-872): first strict minimum
      const std::pair<std::string, int64_t> *lo = nullptr;
      for (auto &kv : plan_->estimates)
        if (!lo || lo->second > kv.second) lo = &kv;
      prefetched_.insert(alias_idx_.at(lo->first));
      plan_->prefetched.push_back(lo->first);
    }
    if (!sorted_.empty()) {
      const PEdge &e = edges_[sorted_[0].first];
      root_ = sorted_[0].second ? e.out : e.in;
    } else {
      root_ = 0;
    }
    plan_->root = nodes_[root_].alias;
  }

  // ---- predicate compiler ----------------------------------------------------------------------
  enum CT { C_NUL, C_INT, C_DBL, C_BOOL };
  struct ProgBuilder {
    PredProgram p;
    int depth = 0, max_depth = 0;
    void emit(int32_t op, int32_t arg = 0, int64_t i = 0, double d = 0, int dstack = 0) {
      if (p.code.size() >= (size_t)kMaxPred) unsupported("predicate program too long for the device VM");
      p.code.push_back(DPredInstr{op, arg, i, d});
      depth += dstack;
      max_depth = std::max(max_depth, depth);
      if (max_depth > 16) unsupported("predicate expression too deep for the device VM");
    }
  };

  static bool shadowed(const std::string &n) {
    std::string l = lower(n);
    return l == "depth" || l == "matched" || l == "currentmatch" || l == "current" || l == "parent" ||
           l == "paths" || l == "patterns" || l == "matches" || l == "elements" || l == "pathelements";
  }

  CT push_const(ProgBuilder &b, const Value &v) {
    switch (v.kind) {
      case Value::NUL: b.emit(P_PUSH_NULL, 0, 0, 0, 1); return C_NUL;
      case Value::INT: b.emit(P_PUSH_INT, 0, v.i, 0, 1); return C_INT;
      case Value::DBL: b.emit(P_PUSH_DBL, 0, 0, v.d, 1); return C_DBL;
      case Value::BOOL: b.emit(P_PUSH_BOOL, 0, v.i, 0, 1); return C_BOOL;
      case Value::STR: unsupported("string value outside a comparison with a string property");
    }
    return C_NUL;
  }

  // records: the edge methods bind edge records (outE/inE/bothE → the record sets, outV/inV/bothV → the
  // endpoints set; Graph::edge_records); otherwise outE/inE/bothE stand for their vertices' adjacency (a
  // fused pair, a degree)
  AdjSpec adjacency(const std::string &method_in, const std::vector<std::string> &labels_in, bool records = false) const {
    std::string m = lower(method_in);
    if (records && (m == "outv" || m == "inv" || m == "bothv")) {
      AdjSpec a;
      for (size_t i = 0; i < g_.esets.size(); ++i)
        if (g_.esets[i].pseudo == 2) {
          if (m != "inv") a.parts.emplace_back((int)i, 0);
          if (m != "outv") a.parts.emplace_back((int)i, 1);
        }
      a.sorted = true;
      a.dup_free = a.parts.size() == 1;
      return a;
    }
    const int want = records && (m == "oute" || m == "ine" || m == "bothe") ? 1 : 0;
    if (m == "oute") m = "out";
    else if (m == "ine") m = "in";
    else if (m == "bothe") m = "both";
    if (m != "out" && m != "in" && m != "both") unsupported("traversal method " + method_in + "() on the device");
    std::vector<std::string> labels = labels_in;
    if (labels.size() == 1 && ieq(labels[0], "E")) labels.clear();  // OrientVertex.getFieldNames :1036-1038
    // the set of edge classes (label + all subclasses; B/OrientVertex.java:1048-1060)
    std::vector<int> classes;
    if (labels.empty()) {
      for (auto &es : g_.esets)
        if (!es.pseudo && std::find(classes.begin(), classes.end(), es.cls) == classes.end()) classes.push_back(es.cls);
    } else {
      for (auto &l : labels) {
        int c = g_.class_id(l);
        if (c < 0) continue;  // no out_<label> field on any vertex
        for (int s : g_.classes[c].poly)
          if (std::find(classes.begin(), classes.end(), s) == classes.end()) classes.push_back(s);
      }
    }
    AdjSpec a;
    for (int c : classes)
      for (size_t i = 0; i < g_.esets.size(); ++i) {
        if (g_.esets[i].cls != c || g_.esets[i].pseudo != want) continue;
        if (m == "out" || m == "both") a.parts.emplace_back((int)i, 0);
        if (m == "in" || m == "both") a.parts.emplace_back((int)i, 1);
      }
    if ((int)a.parts.size() > kMaxAdjParts) unsupported("too many edge classes in one traversal");
    a.sorted = true;
    for (auto &p : a.parts) a.sorted = a.sorted && (p.second == 0 ? g_.esets[p.first].out_sorted : g_.esets[p.first].in_sorted);
    a.dup_free = a.parts.size() <= 1 &&
                 (a.parts.empty() || (a.parts[0].second == 0 ? g_.esets[a.parts[0].first].out_simple
                                                             : g_.esets[a.parts[0].first].in_simple));
    return a;
  }

  CT compile_value(ProgBuilder &b, const ExprP &e, bool allow_depth) {
    if (auto v = fold(e)) return push_const(b, *v);
    switch (e->kind) {
      case Expr::FIELD: {
        if (shadowed(e->name)) unsupported("field name shadowed by a context variable: " + e->name);
        if (e->name[0] == '@') unsupported("record attribute " + e->name + " in a device predicate");
        int p = g_.prop_id(e->name);
        if (p < 0) {  // no vertex has the field: always null
          b.emit(P_PUSH_NULL, 0, 0, 0, 1);
          return C_NUL;
        }
        int t = g_.props[p].type;
        if (t == OMX_PROP_STRING) unsupported("string property " + e->name + " outside a comparison with a constant");
        b.emit(P_PUSH_COL, p, 0, 0, 1);
        return t == OMX_PROP_DOUBLE ? C_DBL : t == OMX_PROP_BOOL ? C_BOOL : C_INT;
      }
      case Expr::VAR: {
        if (ieq(e->name, "$depth") && allow_depth) {
          b.p.uses_depth = true;
          b.emit(P_PUSH_DEPTH, 0, 0, 0, 1);
          return C_INT;
        }
        unsupported("context variable " + e->name + " in a device predicate");
      }
      case Expr::MATH: {
        CT l = compile_value(b, e->kids[0], allow_depth);
        CT r = compile_value(b, e->kids[1], allow_depth);
        if (l == C_BOOL || r == C_BOOL) unsupported("arithmetic on booleans");
        int32_t op = e->name == "+" ? P_ADD : e->name == "-" ? P_SUB : e->name == "*" ? P_MUL : e->name == "/" ? P_DIV : P_MOD;
        b.emit(op, 0, 0, 0, -1);
        return (l == C_DBL || r == C_DBL) ? C_DBL : C_INT;
      }
      case Expr::CHAIN: {
        // <out|in|both|outE|inE|bothE>('L', ...).size()  →  degree of the current vertex
        const ExprP &base = e->kids[0];
        if (base->kind == Expr::CALL && e->suffixes.size() == 1 && e->suffixes[0].kind == Suffix::METHOD &&
            ieq(e->suffixes[0].name, "size") && e->suffixes[0].args.empty()) {
          std::vector<std::string> labels;
          for (auto &a : base->kids) {
            auto v = fold(a);
            if (!v || v->kind != Value::STR) unsupported("non-constant edge label");
            labels.push_back(v->s);
          }
          AdjSpec adj = adjacency(base->name, labels);
          if (b.p.deg.size() >= (size_t)kMaxDegAdj) unsupported("too many degree terms in one predicate");
          b.p.deg.push_back(adj);
          b.emit(P_PUSH_DEG, (int)b.p.deg.size() - 1, 0, 0, 1);
          return C_INT;
        }
        unsupported("expression " + expr_text(e) + " in a device predicate");
      }
      default: unsupported("expression " + expr_text(e) + " in a device predicate");
    }
  }

  // the records a predicate is compiled for: edge records (an edge node's WHERE) or vertices
  bool pred_edges_ = false;
  bool prop_nulls(int p) const { return pred_edges_ ? g_.props[p].nulls_e : g_.props[p].nulls_v; }
  // can the value be null for some vertex of the snapshot (a property with absent values, a field no
  // vertex has, arithmetic over either)
  bool may_be_null(const ExprP &e) const {
    if (fold(e)) return false;
    switch (e->kind) {
      case Expr::FIELD: {
        const int p = g_.prop_id(e->name);
        return p < 0 || prop_nulls(p);
      }
      case Expr::MATH: return may_be_null(e->kids[0]) || may_be_null(e->kids[1]);
      default: return false;  // $depth, out()/in()/both().size()
    }
  }

  static std::string flip(const std::string &op) {
    if (op == "<") return ">";
    if (op == ">") return "<";
    if (op == "<=") return ">=";
    if (op == ">=") return "<=";
    return op;
  }

  bool string_may_be_null(const ExprP &e) const {
    int p;
    return string_field(e, &p) && prop_nulls(p);
  }

  bool string_field(const ExprP &e, int *prop) const {
    if (e->kind != Expr::FIELD || shadowed(e->name)) return false;
    int p = g_.prop_id(e->name);
    if (p < 0 || g_.props[p].type != OMX_PROP_STRING) return false;
    *prop = p;
    return true;
  }

  // string property vs string constant → comparison of dictionary codes (the dictionary is sorted)
  void emit_string_cmp(ProgBuilder &b, int prop, const std::string &op, const std::string &s) {
    const auto &dict = g_.props[prop].dict;
    int64_t lb = std::lower_bound(dict.begin(), dict.end(), s) - dict.begin();
    bool found = (size_t)lb < dict.size() && dict[lb] == s;
    int64_t ub = lb + (found ? 1 : 0);
    if (op == "=" || op == "!=") {
      if (!found) {
        b.emit(P_PUSH_BOOL, 0, op == "!=", 0, 1);
        return;
      }
      b.emit(P_PUSH_COL, prop, 0, 0, 1);
      b.emit(P_PUSH_INT, 0, lb, 0, 1);
      b.emit(op == "=" ? P_EQ : P_NE, 0, 0, 0, -1);
      return;
    }
    b.emit(P_PUSH_COL, prop, 0, 0, 1);
    if (op == "<") { b.emit(P_PUSH_INT, 0, lb, 0, 1); b.emit(P_LT, 0, 0, 0, -1); }
    else if (op == "<=") { b.emit(P_PUSH_INT, 0, ub, 0, 1); b.emit(P_LT, 0, 0, 0, -1); }
    else if (op == ">") { b.emit(P_PUSH_INT, 0, ub, 0, 1); b.emit(P_GE, 0, 0, 0, -1); }
    else { b.emit(P_PUSH_INT, 0, lb, 0, 1); b.emit(P_GE, 0, 0, 0, -1); }
  }

  void compile_bool(ProgBuilder &b, const ExprP &e, bool allow_depth) {
    if (auto v = fold(e)) {
      b.emit(P_PUSH_BOOL, 0, v->kind == Value::BOOL && v->i, 0, 1);
      return;
    }
    switch (e->kind) {
      case Expr::OR:
      case Expr::AND:
        for (size_t i = 0; i < e->kids.size(); ++i) {
          compile_bool(b, e->kids[i], allow_depth);
          if (i) b.emit(e->kind == Expr::OR ? P_OR : P_AND, 0, 0, 0, -1);
        }
        return;
      case Expr::NOT:
        compile_bool(b, e->kids[0], allow_depth);
        b.emit(P_NOT);
        return;
      case Expr::TRUTH: {
        CT t = compile_value(b, e->kids[0], allow_depth);
        if (t != C_BOOL) {  // only a boolean true is "true"
          b.emit(P_PUSH_BOOL, 0, 0, 0, 1);
          b.emit(P_AND, 0, 0, 0, -1);
          return;
        }
        b.emit(P_TRUTH);
        return;
      }
      case Expr::CMP: {
        const ExprP &L = e->kids[0], &R = e->kids[1];
        std::string op = e->name;
        int prop;
        auto fl = fold(L), fr = fold(R);
        if (legacy_) {
          // legacy operators (S/operator/OQueryOperatorEqualityNotNulls.java:50-56): a null operand makes
          // every comparison false, != included; the right operand is converted to the left one's type
          // (OQueryOperatorMajor.java:63-69: OType.convert), which truncates a fractional constant
          if ((fl && fl->kind == Value::NUL) || (fr && fr->kind == Value::NUL)) {
            b.emit(P_PUSH_BOOL, 0, 0, 0, 1);
            return;
          }
          if (op == "!=" && (may_be_null(L) || may_be_null(R) || string_may_be_null(L) || string_may_be_null(R)))
            unsupported("!= with a possibly-null operand in a legacy condition (false in the reference, true on the device)");
          if (string_field(L, &prop) && fr && fr->kind == Value::STR) return emit_string_cmp(b, prop, op, fr->s);
          if (string_field(R, &prop) && fl && fl->kind == Value::STR) return emit_string_cmp(b, prop, flip(op), fl->s);
          CT l = compile_value(b, L, allow_depth);
          CT r = compile_value(b, R, allow_depth);
          if (l == C_INT && r == C_DBL) unsupported("an integer compared with a fractional value in a legacy condition (converted)");
          if ((l == C_BOOL) != (r == C_BOOL)) unsupported("comparison of a boolean with a number");
          if (l == C_BOOL && op != "=" && op != "!=") unsupported("ordering comparison of booleans");
          int32_t code = op == "=" ? P_EQ : op == "!=" ? P_NE : op == "<" ? P_LT : op == "<=" ? P_LE : op == ">" ? P_GT : P_GE;
          b.emit(code, 0, 0, 0, -1);
          return;
        }
        if (string_field(L, &prop) && fr && fr->kind == Value::STR) {
          if ((op == ">" || op == ">=" || op == "<=") && prop_nulls(prop))
            unsupported("a possibly-null left operand of " + op + " (NullPointerException in the reference): " + expr_text(L));
          return emit_string_cmp(b, prop, op, fr->s);
        }
        const bool ordering = op == "<" || op == "<=" || op == ">" || op == ">=";
        if (string_field(R, &prop) && fl && fl->kind == Value::STR) {
          // a constant left operand: a null right one is the reference's NPE for every ordering operator
          if (ordering && prop_nulls(prop))
            unsupported("a possibly-null right operand of " + op + " (NullPointerException in the reference): " + expr_text(R));
          return emit_string_cmp(b, prop, flip(op), fl->s);
        }
        if (fr && fr->kind == Value::NUL) {
          if (!ordering) {
            b.emit(P_PUSH_BOOL, 0, op == "!=", 0, 1);
            return;
          }
          // null < null is false (OLtOperator tests the left operand first); anything else throws
          if (op == "<" && fl && fl->kind == Value::NUL) {
            b.emit(P_PUSH_BOOL, 0, 0, 0, 1);
            return;
          }
          unsupported("null right operand of " + op + " (NullPointerException in the reference)");
        }
        if (fl && fl->kind == Value::NUL) {
          if (op == "=" || op == "!=" || op == "<") {
            b.emit(P_PUSH_BOOL, 0, op == "!=", 0, 1);
            return;
          }
          unsupported("null left operand of " + op);
        }
        // OGtOperator / OGeOperator / OLeOperator throw NullPointerException on a null left operand
        // (P/OGtOperator.java:22-33, P/OGeOperator.java:43-54, P/OLeOperator.java:22-33); whether it is
        // thrown depends on which records the DFS reaches, so a left operand that can be null on this
        // snapshot is left to the reference engine instead of being compared false
        if ((op == ">" || op == ">=" || op == "<=") && may_be_null(L))
          unsupported("a possibly-null left operand of " + op + " (NullPointerException in the reference): " + expr_text(L));
        // all four ordering operators dereference a null right operand once the left one is non-null
        // (`iLeft.getClass() != iRight.getClass()`): compared false on the device, thrown by the reference
        if (ordering && (may_be_null(R) || string_may_be_null(R)))
          unsupported("a possibly-null right operand of " + op + " (NullPointerException in the reference): " + expr_text(R));
        CT l = compile_value(b, L, allow_depth);
        CT r = compile_value(b, R, allow_depth);
        if ((l == C_BOOL) != (r == C_BOOL) && l != C_NUL && r != C_NUL)
          unsupported("comparison of a boolean with a number");
        if (l == C_BOOL && op != "=" && op != "!=") unsupported("ordering comparison of booleans");
        int32_t code = op == "=" ? P_EQ : op == "!=" ? P_NE : op == "<" ? P_LT : op == "<=" ? P_LE : op == ">" ? P_GT : P_GE;
        b.emit(code, 0, 0, 0, -1);
        return;
      }
      default: unsupported("condition " + expr_text(e) + " in a device predicate");
    }
  }

  int add_prog(const ExprP &e, bool allow_depth) {
    if (!e) return -1;
    ProgBuilder b;
    compile_bool(b, e, allow_depth);
    if (b.p.code.size() == 1 && b.p.code[0].op == P_PUSH_BOOL) {
      if (b.p.code[0].i) return -1;  // statically true
      b.p.const_false = true;
    }
    plan_->progs.push_back(b.p);
    return (int)plan_->progs.size() - 1;
  }

  std::map<std::pair<std::string, int>, int> bm_cache_;  // (alias, kind) → bitmap
  // kind 0: WHERE of the alias (traversal filter, $currentMatch = neighbour)
  // kind 1: candidate set = polymorphic class ∧ WHERE (fetchAliasCandidates :401-410)
  int bitmap(const std::string &alias, int kind) {
    auto key = std::make_pair(alias, kind);
    auto it = bm_cache_.find(key);
    if (it != bm_cache_.end()) return it->second;
    BitmapSpec s;
    if (kind == 1 && has_row_conds(alias))
      unsupported("$matched in the WHERE of a root, prefetched or cartesian alias (" + alias + ")");
    auto ai = alias_idx_.find(alias);
    pred_edges_ = ai != alias_idx_.end() && (size_t)ai->second < edge_node_.size() && edge_node_[ai->second];
    s.prog = add_prog(vertex_where_of(alias), false);
    if (g_.edge_records && ai != alias_idx_.end()) s.records = pred_edges_ ? 2 : 1;
    pred_edges_ = false;
    if (kind == 1) {
      auto c = alias_class_.find(alias);
      if (c == alias_class_.end()) fail(OMX_E_EXECUTION, "Cannot execute MATCH statement on alias " + alias + ": class not defined");
      s.class_id = g_.class_id(c->second);
    }
    int id = -1;
    if (s.prog >= 0 || s.class_id >= 0) {
      plan_->bitmaps.push_back(s);
      id = (int)plan_->bitmaps.size() - 1;
    }
    bm_cache_[key] = id;
    return id;
  }

  // ---- steps -----------------------------------------------------------------------------------
  void compile_steps() {
    for (auto &n : nodes_) plan_->optional.push_back(n.optional);
    // candidate sets that must be non-empty (calculateMatch :340-357, :359-367)
    for (int a : prefetched_) plan_->must_be_nonempty.push_back(bitmap(nodes_[a].alias, 1));
    if (!prefetched_.count(root_))
      fail(OMX_E_EXECUTION, "NullPointerException: no candidates for root alias " + nodes_[root_].alias);

    std::vector<bool> bound(nodes_.size(), false);
    Step r;
    r.kind = S_ROOT;
    r.dst = root_;
    r.cand_bm = bitmap(nodes_[root_].alias, 1);
    r.desc = "root " + nodes_[root_].alias;
    plan_->steps.push_back(r);
    bound[root_] = true;
    for (auto &se : sorted_) {
      const PEdge &pe = edges_[se.first];
      bool fwd = se.second;
      const PathItem &it = *pe.item;
      int s = fwd ? pe.out : pe.in, t = fwd ? pe.in : pe.out;
      if (!bound[s]) {
        if (fwd && prefetched_.count(s)) {  // restart from candidates (:434-445)
          Step n;
          n.kind = S_NEWROOT;
          n.dst = s;
          n.cand_bm = bitmap(nodes_[s].alias, 1);
          n.desc = "new component root " + nodes_[s].alias;
          plan_->steps.push_back(n);
          bound[s] = true;
        } else {
          Step k;
          k.kind = S_KILL;
          k.desc = "unbound start " + nodes_[s].alias + " without candidates: no results";
          plan_->steps.push_back(k);
          return;
        }
      }
      Step st;
      st.src = s;
      st.dst = t;
      st.mode = bound[t] ? T_BOUND : prefetched_.count(t) ? T_CAND : T_FREE;
      bool varlen = it.filter.while_ || it.filter.has_max_depth;
      if (nodes_[s].optional) unsupported("a traversal starting from the optional node " + nodes_[s].alias);
      if (nodes_[t].optional) {
        if (varlen || it.is_multi) unsupported("an optional variable-length or multi-step item");
        if (!fwd) unsupported("a reversed traversal into an optional node");
        st.optional = true;
        st.where_bm = bitmap(nodes_[t].alias, 0);
      }
      std::string m = lower(it.method);
      const bool erec = m == "oute" || m == "ine" || m == "bothe" || m == "outv" || m == "inv" || m == "bothv";
      if (!it.is_multi && m != "out" && m != "in" && m != "both" && !(erec && g_.edge_records))
        unsupported("traversal method " + it.method + "() on the device");
      if (erec && varlen) unsupported("a variable-length item over edge records (" + it.method + "())");
      std::vector<std::pair<std::string, bool>> rconds;
      vertex_where_of(nodes_[t].alias, &rconds);
      // a reversed traversal into a bound or prefetched target applies no WHERE (executeReverse's
      // branches :468-490 test existence / candidates only); a forward one into a bound target filters
      // the traversal with the WHERE, $matched included (:468-477 after executeTraversal), so the
      // row-level conjuncts follow the check
      if (!fwd && st.mode != T_FREE) rconds.clear();
      // (a variable-length or multi-step item: the WHERE selects the walk's outputs and never steers the
      // walk — the while condition / maxDepth do, P/OMatchPathItem.java:79-105 — so the row-level
      // conjuncts filter its output rows as they filter a single hop's)
      if (!rconds.empty()) {
        if (st.mode == T_CAND || st.optional)
          unsupported("$matched in the WHERE of a prefetched or optional target (" + nodes_[t].alias + ")");
        for (auto &rc : rconds) {
          auto ai = alias_idx_.find(rc.first);
          if (ai == alias_idx_.end() || !bound[ai->second] || ai->second == t)
            unsupported("$matched." + rc.first + " is not bound when " + nodes_[t].alias + " is matched");
        }
      }
      if (it.is_multi) {  // never reversed: OMultiMatchPathItem.isBidirectional is false
        st.kind = S_MULTI;
        st.trav.multi = true;
        st.trav.subs = compile_subs(it.multi);
        st.trav.varlen = varlen;
        st.trav.where_prog = add_prog(vertex_where_of(nodes_[t].alias), varlen);  // the rebound alias filter (:185-195)
        st.trav.while_prog = add_prog(it.filter.while_, true);
        st.trav.has_max_depth = it.filter.has_max_depth;
        st.trav.max_depth = it.filter.max_depth;
        if (st.mode == T_CAND) st.cand_bm = bitmap(nodes_[t].alias, 1);
      } else if (varlen) {
        st.kind = S_VARLEN;
        st.adj = adjacency(m, it.labels);
        st.where_prog = add_prog(vertex_where_of(nodes_[t].alias), true);
        st.while_prog = add_prog(it.filter.while_, true);
        st.has_max_depth = it.filter.has_max_depth;
        st.max_depth = it.filter.max_depth;
        if (st.mode == T_CAND) st.cand_bm = bitmap(nodes_[t].alias, 1);
      } else {
        // executeReverse (P/OMethodCall.java:92-126): outE ↔ outV, inE ↔ inV
        static const std::map<std::string, std::string> kRev = {{"out", "in"}, {"in", "out"}, {"both", "both"},
                                                                {"oute", "outv"}, {"outv", "oute"},
                                                                {"ine", "inv"}, {"inv", "ine"}};
        std::string rm = m;
        if (!fwd) {
          auto r = kRev.find(m);
          if (r == kRev.end()) unsupported("a reversed " + it.method + "() item");
          rm = r->second;
        }
        st.adj = adjacency(rm, it.labels, erec);
        if (st.mode == T_BOUND) {
          st.kind = S_CHECK;
          st.filter_bm = fwd ? bitmap(nodes_[t].alias, 0) : -1;
        } else {
          st.kind = S_EXPAND;
          st.filter_bm = st.mode == T_CAND ? bitmap(nodes_[t].alias, 1) : bitmap(nodes_[t].alias, 0);
          st.distinct_nb = fwd && where_of(nodes_[t].alias) != nullptr;
        }
      }
      st.desc = std::string(st.kind == S_VARLEN ? "varlen " : st.kind == S_MULTI ? "multi " : st.kind == S_CHECK ? "check " : "expand ") +
                nodes_[s].alias + (fwd ? " -" : " <-") + it.method + "- " + nodes_[t].alias +
                (st.mode == T_BOUND ? " [bound]" : st.mode == T_CAND ? " [candidates]" : " [free]");
      plan_->steps.push_back(st);
      bound[t] = true;
      for (auto &rc : rconds) {
        Step c;
        c.kind = S_ROWCMP;
        c.src = alias_idx_.at(rc.first);
        c.dst = t;
        c.row_eq = rc.second;
        c.desc = "rows where $matched." + rc.first + (rc.second ? " = " : " != ") + nodes_[t].alias;
        plan_->steps.push_back(c);
      }
    }
    for (size_t a = 0; a < nodes_.size(); ++a)
      if (!bound[a]) {  // expandCartesianProduct (:620-650)
        Step c;
        c.kind = S_CARTESIAN;
        c.dst = (int)a;
        c.cand_bm = bitmap(nodes_[a].alias, 1);
        c.desc = "cartesian " + nodes_[a].alias;
        plan_->steps.push_back(c);
        bound[a] = true;
      }
  }

  // The sub-items of a multi item .( ... ): their own filters (not rebound: they are not pattern nodes),
  // `outE('L').inV()` and `inE('L').outV()` pairs as the vertex sets of out('L') / in('L')
  std::vector<TravSpec> compile_subs(const std::vector<PathItem> &items) {
    std::vector<TravSpec> out;
    for (size_t i = 0; i < items.size(); ++i) {
      const PathItem &s = items[i];
      const PathItem *fi = &s;  // the item whose filter applies
      TravSpec t;
      if (s.is_multi) {
        t.multi = true;
        t.subs = compile_subs(s.multi);
      } else {
        const std::string m = lower(s.method);
        if (m == "oute" || m == "ine") {
          if (s.filter.where || s.filter.while_ || s.filter.has_max_depth || s.filter.optional)
            unsupported("a filter on the edge step " + s.method + "() inside .( ... )");
          const std::string v = i + 1 < items.size() && !items[i + 1].is_multi ? lower(items[i + 1].method) : "";
          if (!((m == "oute" && v == "inv") || (m == "ine" && v == "outv")) || !items[i + 1].labels.empty())
            unsupported("edge step " + s.method + "() not followed by its vertex step inside .( ... )");
          t.adj = adjacency(m == "oute" ? "out" : "in", s.labels);
          fi = &items[++i];
        } else {
          if (m != "out" && m != "in" && m != "both") unsupported("traversal method " + s.method + "() inside .( ... )");
          t.adj = adjacency(m, s.labels);
        }
      }
      const MatchFilter &f = fi->filter;
      if (f.optional) unsupported("optional inside .( ... )");
      t.varlen = f.while_ || f.has_max_depth;
      t.where_prog = add_prog(f.where, t.varlen);
      t.while_prog = add_prog(f.while_, true);
      t.has_max_depth = f.has_max_depth;
      t.max_depth = f.max_depth;
      out.push_back(std::move(t));
    }
    return out;
  }

  // OExpression.getDefaultAlias: the item's text without spaces, every run of other characters than
  // letters, digits, '_' and '$' → '_' ('friend.name' → 'friend_name')
  static std::string default_alias(const std::string &raw) {
    std::string s, o;
    for (char c : raw)
      if (c != ' ') s += c;
    bool run = false;
    for (char c : s) {
      if (std::isalnum((unsigned char)c) || c == '_' || c == '$') {
        o += c;
        run = false;
      } else if (!run) {
        o += '_';
        run = true;
      }
    }
    size_t a = o.find_first_not_of('_'), b = o.find_last_not_of('_');
    return a == std::string::npos ? std::string() : o.substr(a, b - a + 1);
  }

  // what the result builder (project.cpp) evaluates: literals, parameters, aliases and their fields,
  // arithmetic / string concatenation, comparisons, JSON and arrays, out()/in()/both() of a vertex,
  // size() / toUpperCase() / toLowerCase(), and [i] / [a-b] / [i, j] / [condition] selectors
  void check_return(const ExprP &e, std::vector<int> &refs) {
    if (!e) return;
    switch (e->kind) {
      case Expr::LIT:
      case Expr::PARAM: return;
      case Expr::FIELD: {
        auto it = alias_idx_.find(e->name);
        if (it != alias_idx_.end() && std::find(refs.begin(), refs.end(), it->second) == refs.end())
          refs.push_back(it->second);
        return;
      }
      case Expr::VAR: unsupported("context variable " + e->name + " in a RETURN expression");
      case Expr::CALL: unsupported("function call " + e->name + "() in a RETURN expression");
      case Expr::CHAIN:
        check_return(e->kids[0], refs);
        for (size_t si = 0; si < e->suffixes.size(); ++si) {
          const Suffix &s = e->suffixes[si];
          if (s.kind == Suffix::METHOD) {
            const std::string m = lower(s.name);
            if (m == "out" || m == "in" || m == "both") {
              std::vector<std::string> labels;
              for (auto &a : s.args) {
                auto v = fold(a);
                if (!v || v->kind != Value::STR) unsupported("non-constant edge label in a RETURN expression");
                labels.push_back(v->s);
              }
              plan_->ret_adj[&s] = adjacency(m, labels);
              auto ai = e->kids[0] && e->kids[0]->kind == Expr::FIELD ? alias_idx_.find(e->kids[0]->name)
                                                                          : alias_idx_.end();
              if (si == 0 && ai != alias_idx_.end()) plan_->ret_adj_alias.emplace_back(&s, ai->second);
              else plan_->ret_adj_deep = true;
            } else if (!((m == "size" || m == "touppercase" || m == "tolowercase") && s.args.empty())) {
              unsupported("method " + s.name + "() in a RETURN expression");
            }
          } else if (s.kind == Suffix::INDEX) {
            for (const ExprP &x : {s.index, s.index2}) check_return(x, refs);
            for (auto &x : s.items) check_return(x, refs);
          }
        }
        return;
      default:
        for (auto &k : e->kids) check_return(k, refs);
    }
  }

  void compile_projection() {
    auto has = [&](const char *name) {
      for (auto &r : st_.returns)
        if (ieq(r.text, name)) return true;
      return false;
    };
    Plan &p = *plan_;
    if (fused_edges_ && (has("$paths") || has("$pathElements")))
      unsupported("$paths / $pathElements of a pattern with edge steps (the edge records are returned)");
    if (has("$elements") || has("$pathElements")) {
      p.proj = Plan::PROJ_ELEMENTS;
      bool all = has("$elements") ? false : true;
      for (size_t a = 0; a < nodes_.size(); ++a)
        if (all || p.explicit_alias[a]) p.out_aliases.push_back((int)a);
      p.out_names.push_back(all ? "$pathElements" : "$elements");
    } else if (has("$patterns") || has("$matches") || has("$paths")) {
      bool all = !(has("$patterns") || has("$matches"));
      for (size_t a = 0; a < nodes_.size(); ++a)
        if (all || p.explicit_alias[a]) {
          p.out_aliases.push_back((int)a);
          p.out_names.push_back(nodes_[a].alias);
        }
    } else {
      bool plain = true;
      for (auto &r : st_.returns)
        plain = plain && r.expr->kind == Expr::FIELD && alias_idx_.count(r.expr->name);
      if (plain) {
        for (auto &r : st_.returns) {
          p.out_aliases.push_back(alias_idx_.at(r.expr->name));
          p.out_names.push_back(r.alias.empty() ? r.expr->name : r.alias);
        }
      } else {
        // expressions / JSON (addResult :698-719, jsonToDoc :791-806): evaluated per distinct tuple of the
        // aliases they read
        const bool json = st_.returns.size() == 1 && st_.returns[0].expr->kind == Expr::JSON && st_.returns[0].alias.empty();
        p.proj = json ? Plan::PROJ_JSON : Plan::PROJ_EXPR;
        p.returns = st_.returns;
        std::vector<int> refs;
        for (auto &r : st_.returns) check_return(r.expr, refs);
        p.out_aliases = refs;
        if (json) {
          p.out_names = st_.returns[0].expr->json_keys;
        } else {
          for (auto &r : st_.returns) p.out_names.push_back(r.alias.empty() ? default_alias(r.raw) : r.alias);
        }
      }
    }
    bool dup_free = !std::any_of(p.optional.begin(), p.optional.end(), [](char o) { return o != 0; });
    for (auto &s : p.steps)
      if (s.kind == S_EXPAND && !s.adj.dup_free) dup_free = false;
    std::set<int> cover(p.out_aliases.begin(), p.out_aliases.end());
    p.unique_by_construction = p.proj == Plan::PROJ_ALIASES && dup_free && cover.size() == nodes_.size() &&
                               p.out_aliases.size() == nodes_.size();
    // liveness of the binding columns, backwards from the projection
    std::vector<char> live(nodes_.size(), 0);
    for (int a : p.out_aliases) live[a] = 1;
    p.live_before.assign(p.steps.size(), {});
    for (size_t i = p.steps.size(); i-- > 0;) {
      const Step &s = p.steps[i];
      auto use = [&](int a) {
        if (a >= 0) live[a] = 1;
      };
      switch (s.kind) {
        case S_EXPAND: use(s.src); break;
        case S_CHECK:
        case S_ROWCMP: use(s.src); use(s.dst); break;
        case S_VARLEN:
        case S_MULTI:
          use(s.src);
          if (s.mode == T_BOUND) use(s.dst);
          break;
        default: break;
      }
      p.live_before[i] = live;
    }
  }
};

std::string jstr(const std::string &s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    o += c;
  }
  return o + "\"";
}

}  // namespace

std::unique_ptr<Plan> build_plan(const Statement &st, const Graph &g, const Params &params, bool logical_only,
                                 std::string *reason) {
  const bool chain = st.kind != Statement::MATCH;
  if (!logical_only) return chain ? Planner(st, g, params).run_chain(false) : Planner(st, g, params).run(false);
  auto p = chain ? Planner(st, g, params).run_chain(true) : Planner(st, g, params).run(true);
  if (reason) {
    try {
      if (chain) Planner(st, g, params).run_chain(false);
      else Planner(st, g, params).run(false);
      reason->clear();
    } catch (const OmxError &e) {
      if (e.code != OMX_E_UNSUPPORTED) throw;
      *reason = e.what();
    }
  }
  return p;
}

std::string plan_json(const Plan &p, const std::string &reason) {
  std::ostringstream o;
  o << "{\"kind\":"
    << jstr(p.kind == Plan::MATCH ? "MATCH" : p.kind == Plan::TRAVERSE ? "TRAVERSE" : p.kind == Plan::SELECT ? "SELECT" : "SHORTEST_PATH");
  o << ",\"aliases\":[";
  for (size_t i = 0; i < p.aliases.size(); ++i) o << (i ? "," : "") << jstr(p.aliases[i]);
  o << "],\"estimates\":{";
  for (size_t i = 0; i < p.estimates.size(); ++i)
    o << (i ? "," : "") << jstr(p.estimates[i].first) << ":" << p.estimates[i].second;
  o << "},\"prefetched\":[";
  for (size_t i = 0; i < p.prefetched.size(); ++i) o << (i ? "," : "") << jstr(p.prefetched[i]);
  o << "],\"root\":" << jstr(p.root) << ",\"edges\":[";
  for (size_t i = 0; i < p.sorted_edges.size(); ++i)
    o << (i ? "," : "") << "[" << jstr(std::get<0>(p.sorted_edges[i])) << "," << jstr(std::get<1>(p.sorted_edges[i]))
      << "," << (std::get<2>(p.sorted_edges[i]) ? "true" : "false") << "]";
  o << "],\"empty\":" << (p.empty ? "true" : "false");
  o << ",\"supported\":" << (reason.empty() ? "true" : "false") << ",\"unsupported_reason\":" << jstr(reason) << "}";
  return o.str();
}

}  // namespace omx
