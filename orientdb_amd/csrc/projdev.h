// projdev.h — RETURN expressions evaluated on the device (projdev.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "graph.h"
#include "plan.h"

struct omx_result;

namespace omx {

// kinds of a device-evaluated result cell
enum PjKind : uint8_t { PJ_K_NUL = 0, PJ_K_INT, PJ_K_DBL, PJ_K_STR, PJ_K_BOOL, PJ_K_RID };
constexpr int kPjMaxItems = 8, kPjMaxCols = 8;

// every RETURN item is in the device subset (alias, alias.property, literals, parameters, + - * / % over
// numbers); otherwise *why names the first item that is not
bool device_projection_ok(const Graph &g, const Plan &p, std::string *why);

// cols: n distinct tuples of Plan::out_aliases (dense ids, V = null). Fills res.pcols / res.n_pcol_rows
// with the content-distinct documents (at most max(limit, 1) when limit > -1).
void device_project(Graph &g, const Plan &p, const std::vector<const uint32_t *> &cols, uint64_t n, int64_t limit,
                    int cus, hipStream_t s, omx_result &res);

}  // namespace omx
