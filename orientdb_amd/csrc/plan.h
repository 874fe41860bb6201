// plan.h — logical MATCH plan (the reference's planner) and its compilation to device steps.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "devtypes.h"
#include "graph.h"
#include "sql.h"

namespace omx {

// Parameters of OCommandSQL.execute(args): positional or named.
struct Params {
  std::vector<Value> positional;
  std::vector<std::pair<std::string, Value>> named;
  const Value *get(const Expr &p) const;
};

// Neighbour list of a traversal: concatenation of (edge set, direction) parts.
struct AdjSpec {
  std::vector<std::pair<int, int>> parts;  // (edge set index, 0 = out CSR, 1 = in CSR)
  bool dup_free = false;                   // neighbours of a vertex are distinct
  bool sorted = true;                      // every part's rows sorted
};

struct PredProgram {
  std::vector<DPredInstr> code;  // empty = always true
  std::vector<AdjSpec> deg;      // adjacency referenced by P_PUSH_DEG
  bool uses_depth = false;
  bool const_false = false;      // statically false (e.g. name = 'absent')
};

struct BitmapSpec {
  int prog = -1;      // predicate (-1 = none)
  int class_id = -1;  // polymorphic class test (-1 = none)
  // edge-records snapshots: the records the alias binds (1 vertices, 2 edge records; 0 = any): the bitmap
  // is evaluated over that id range only (the rest zero), which lets a field present on every record of
  // that kind take the null-free fast path
  int records = 0;
};

// S_ROWCMP: keep the rows where col[src] (=|!=) col[dst]: a WHERE conjunct `$matched.X op $currentMatch`
// of the alias the previous step bound (OMatchPathItem.executeTraversal evaluates it per neighbour
// with $matched = the row's bindings, P/OMatchPathItem.java:49-78; identity comparison of records)
// S_MULTI: a multi-step item .( ... ) (OMultiMatchPathItem, P/OMultiMatchPathItem.java:41-61), over
// (row, vertex) pair sets (Step::trav)
enum StepKind { S_ROOT, S_EXPAND, S_CHECK, S_VARLEN, S_NEWROOT, S_CARTESIAN, S_KILL, S_ROWCMP, S_MULTI };
enum TargetMode { T_FREE, T_CAND, T_BOUND };
// an optional target (OMatchStatement.java:448-458): no match → the row continues with the alias null
// (dense id V); a bound optional target that is not reached is overwritten with null

// One item's traversal as a set-valued function of a start vertex, OMatchPathItem.executeTraversal
// (P/OMatchPathItem.java:49-107): single-hop items expand `adj` and keep the neighbours passing `where`
// (a HashSet); variable-length items (while / maxDepth) run level by level from the start vertex with
// $depth; multi items compose `subs`, each applied to every vertex of the previous step's set (a set
// per step, OMultiMatchPathItem.traversePatternEdge). `outE('L').inV()` / `inE('L').outV()` pairs
// inside a multi item are the vertex sets of out('L') / in('L').
struct TravSpec {
  bool multi = false;
  AdjSpec adj;                  // single-method item
  std::vector<TravSpec> subs;   // multi item
  bool varlen = false;          // while or maxDepth given
  int where_prog = -1, while_prog = -1;
  bool has_max_depth = false;
  int max_depth = 0;
};

struct Step {
  StepKind kind = S_EXPAND;
  TargetMode mode = T_FREE;
  int src = -1, dst = -1;  // alias indices (binding-table columns)
  AdjSpec adj;
  int filter_bm = -1;      // bitmap applied to a FREE/CAND target, or to the bound target of a forward S_CHECK
  int cand_bm = -1;        // candidate bitmap (S_ROOT, S_NEWROOT, S_CARTESIAN, S_VARLEN in CAND mode)
  int where_prog = -1, while_prog = -1;  // S_VARLEN
  bool has_max_depth = false;
  int max_depth = 0;
  bool row_eq = false;     // S_ROWCMP: = (true) or != (false)
  TravSpec trav;           // S_MULTI
  bool optional = false;   // S_EXPAND / S_CHECK into an optional node
  int where_bm = -1;       // optional target: the node's WHERE alone (the emptiness test of the traversal)
  // S_EXPAND: the traversal returns a set (a forward single hop into a node with a WHERE: the HashSet of
  // P/OMatchPathItem.java:61,71-78), so a neighbour reached over several edges (parallel edges, or both()
  // over u → v and v → u) binds once; reverse traversals and hops without a WHERE keep every edge
  bool distinct_nb = false;
  std::string desc;
};

// TRAVERSE (C/command/traverse/OTraverse.java, STRATEGY BREADTH_FIRST) and SELECT expand(<chain>)
// (GF/OSQLFunctionMove.java:66-91 via OSQLEngine.foreachRecord, S/OSQLEngine.java:264-290): an ordered
// list of records, kept in the reference's emission order.
struct ChainSpec {
  // TRAVERSE: one entry, the fields' neighbour lists concatenated in field order (the reference pushes one
  // OTraverseMultiValueProcess per field, OTraverseRecordProcess.java:136-160); SELECT: one per chained call
  std::vector<AdjSpec> hops;
  int pred_prog = -1;       // TRAVERSE WHILE (reads $depth; legacy null semantics) / SELECT WHERE
  int max_depth = -1;       // TRAVERSE MAXDEPTH
  int root_class = -1;      // FROM <class>: its vertices (polymorphic) in snapshot order
  std::vector<uint64_t> root_rids;  // FROM #c:p / [#c:p, ...] (packed c << 48 | p), in the order written
  // shortestPath(src, dst[, direction[, edge class[, {maxDepth: n}]]]) (GF/OSQLFunctionShortestPath.java)
  uint64_t sp_src = 0, sp_dst = 0;  // packed RIDs
  AdjSpec sp_left, sp_right;        // the source side's direction and the destination side's opposite
  int sp_max_depth = -1;            // -1: none
  bool expand_rows = true;          // expand(shortestPath(...)): one row per vertex; else one document
};

struct Plan {
  enum Kind { MATCH, TRAVERSE, SELECT, SHORTEST_PATH } kind = MATCH;
  ChainSpec chain;  // TRAVERSE / SELECT / SHORTEST_PATH
  // logical plan (what the reference computes; also reported by omx_statement_explain)
  std::vector<std::string> aliases;  // pattern nodes, insertion order (Pattern.aliasToNode)
  std::vector<bool> explicit_alias;
  std::vector<std::pair<std::string, int64_t>> estimates;  // estimateRootEntries order
  std::vector<std::string> prefetched;
  std::string root;
  std::vector<std::tuple<std::string, std::string, bool>> sorted_edges;  // (out alias, in alias, forward)
  bool empty = false;  // some estimate is 0 → empty result (OMatchStatement.java:249-251)

  // physical plan
  std::vector<PredProgram> progs;
  std::vector<BitmapSpec> bitmaps;
  std::vector<int> must_be_nonempty;  // candidate bitmaps of prefetched aliases (calculateMatch :340-357)
  std::vector<Step> steps;
  // PROJ_EXPR: RETURN expressions (addResult :700-720), PROJ_JSON: one JSON RETURN (:791-806). Both are
  // evaluated per distinct tuple of the aliases they read (out_aliases), then de-duplicated by content
  enum Projection { PROJ_ALIASES, PROJ_ELEMENTS, PROJ_EXPR, PROJ_JSON } proj = PROJ_ALIASES;
  std::vector<int> out_aliases;
  std::vector<std::string> out_names;
  std::vector<ReturnItem> returns;                 // PROJ_EXPR / PROJ_JSON
  std::map<const Suffix *, AdjSpec> ret_adj;       // out()/in()/both() suffixes inside RETURN expressions
  // the ones applied to an alias directly (`a.out('L')…`), in RETURN order (the same on every rank): a
  // partitioned run fetches those vertices' lists from their owners; ret_adj_deep: some out()/in()/both()
  // applies to a list or a field (its vertices are only known while the expression is evaluated)
  std::vector<std::pair<const Suffix *, int>> ret_adj_alias;
  bool ret_adj_deep = false;
  std::vector<char> optional;                      // per alias: an optional pattern node (null when unmatched)
  Params params;                                   // the query parameters (RETURN expressions read them)
  bool unique_by_construction = false;
  // live_before[i][a]: alias a is read by step i or a later step, or projected; a bound column that is
  // not live is dropped before step i (expansions then carry only what is still read)
  std::vector<std::vector<char>> live_before;
  int64_t limit = -1;  // LIMIT clause (-1 = none)
};

// Builds the plan. Throws OmxError(OMX_E_UNSUPPORTED) when the statement is valid MATCH but outside
// what the device engine executes (the host then falls back to the reference OMatchStatement);
// `logical_only` stops after the reference's planning steps (used by explain).
std::unique_ptr<Plan> build_plan(const Statement &st, const Graph &g, const Params &params, bool logical_only,
                                 std::string *unsupported_reason = nullptr);

std::string plan_json(const Plan &p, const std::string &unsupported_reason);

}  // namespace omx
