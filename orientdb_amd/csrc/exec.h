// exec.h — runs a compiled Plan on the device and produces the distinct RETURN rows.
#pragma once
#include <string>
#include <vector>

#include "graph.h"
#include "plan.h"
#include "project.h"

struct omx_result {
  omx_result_info info{};
  std::vector<std::string> names;
  std::vector<uint64_t> rows;  // row-major n_rows × n_cols
  std::vector<omx::Document> docs;  // RETURN expressions / JSON: one document per row (info.documents)
  struct KStat {
    std::string name;
    int64_t launches = 0;
    double ms = 0;
    uint64_t bytes = 0;
  };
  std::vector<KStat> kstats;
  std::vector<KStat> klaunches;  // every timed launch in issue order (launches = 1 each)
};

namespace omx {
class Transport;
// tr: the ranks' communicator for a partitioned snapshot (nullptr otherwise)
omx_result *execute_plan(Graph &g, const Plan &p, const omx_exec_options &opts, Transport *tr = nullptr);
}
