// exec.h — runs a compiled Plan on the device and produces the distinct RETURN rows.
#pragma once
#include <string>
#include <unordered_map>
#include <vector>

#include "graph.h"
#include "plan.h"
#include "project.h"

struct omx_result {
  omx_result_info info{};
  std::vector<std::string> names;
  // row-major n_rows × n_cols RIDs in a library-owned host block (graph.h host_rows_acquire: pinned,
  // pooled, never value-initialised), returned to the pool by omx_result_free
  uint64_t *rows = nullptr;
  size_t rows_capacity = 0;  // bytes of the block
  bool rows_pinned = false;
  omx_result() = default;
  omx_result(const omx_result &) = delete;
  omx_result &operator=(const omx_result &) = delete;
  ~omx_result() { omx::host_rows_release(rows); }
  std::vector<omx::Document> docs;  // RETURN expressions / JSON: one document per row (info.documents)
  struct KStat {
    std::string name;
    int64_t launches = 0;
    double ms = 0;
    uint64_t bytes = 0;
    uint64_t hbm = 0;  // the bytes HBM must move at least (each distinct byte once; L2 re-reads excluded)
  };
  std::vector<KStat> kstats;
  std::vector<KStat> klaunches;  // every timed launch in issue order (launches = 1 each)
  // documents evaluated on the device (projdev.hip): one column per RETURN item, n_pcol_rows cells each
  struct PCol {
    std::vector<uint8_t> kind;                        // omx::PJ_K_*
    std::vector<uint64_t> val;                        // int64 / double bits / dictionary code / bool / RID
    std::unordered_map<uint64_t, std::string> strs;  // dictionary code → string (string columns)
  };
  std::vector<PCol> pcols;
  uint64_t n_pcol_rows = 0;
};

namespace omx {
class Transport;
// tr: the ranks' communicator for a partitioned snapshot (nullptr otherwise)
// *running (if given) is set once the plan's partition checks passed and execution started
omx_result *execute_plan(Graph &g, const Plan &p, const omx_exec_options &opts, Transport *tr = nullptr,
                         bool *running = nullptr);
}
