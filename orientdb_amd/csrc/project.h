// project.h — result documents of RETURN expressions and JSON RETURNs (the OResultSet fill).
//
// The reference builds one ODocument per complete binding (OMatchStatement.addResult,
// P/OMatchStatement.java:698-719: every RETURN item evaluated against the matched map; jsonToDoc
// :791-806) and keeps it if no equal document was kept before (OBasicCommandContext.addToUniqueResult,
// C/command/OBasicCommandContext.java:347-353, ODocumentEqualityWrapper: equality by content).
//
// Here the device produces the distinct tuples of the aliases the RETURN items read (a projection is a
// function of those bindings, so de-duplicating them first keeps the result set); this file turns each
// tuple into a document on the host — the work the Java side does when it fills the OResultSet — and
// de-duplicates the documents by content. Property values, RIDs and classes come from host mirrors of
// the snapshot's columns (copied once per graph), out()/in()/both() lists from the device CSR.
#pragma once
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "graph.h"
#include "plan.h"

namespace omx {

// a value of a result document: null, number, string, boolean, a record (vertex), a list or a map
struct HVal {
  enum Kind { NUL, INT, DBL, STR, BOOL, RID, LIST, MAP } k = NUL;
  int64_t i = 0;
  double d = 0;
  std::string s;
  uint32_t v = 0;    // RID: dense vertex id
  uint64_t rid = 0;  // RID: (cluster << 48) | position (filled for the result)
  std::vector<HVal> items;
  std::vector<std::string> keys;  // MAP
  std::string json;               // LIST / MAP cells of a result: the value as JSON (RIDs as "#c:p")
};
using Document = std::vector<HVal>;  // one value per Plan::out_names

// the lists of out()/in()/both() suffixes of RETURN expressions, per (suffix, vertex)
using RetAdj = std::map<std::pair<const Suffix *, uint32_t>, std::vector<uint32_t>>;

// cols: n distinct tuples of Plan::out_aliases (device columns, dense ids; V = null). limit: LIMIT
// (after content de-duplication; -1 none; 0 keeps one, as addSingleResult does). fetched: a partitioned
// run's lists fetched from their owners (Executor::fetch_return_adjacency); every list is then read from
// it (a partition's CSR holds its own rows only), else from the device CSR.
std::vector<Document> build_documents(Graph &g, const Plan &p, const std::vector<const uint32_t *> &cols, uint64_t n,
                                      int64_t limit, hipStream_t s, const RetAdj *fetched = nullptr);

}  // namespace omx
