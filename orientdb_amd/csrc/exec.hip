// exec.hip — device execution of a compiled MATCH plan.
//
// The reference enumerates bindings depth-first, one MatchContext copy per traversed edge
// (P/OMatchStatement.java:412-568). Here the same bindings are produced level by level: a
// binding table (one u32 column of dense vertex ids per bound alias, SoA in HBM) is expanded one
// sorted pattern edge at a time, with the reference's per-edge filter rules (see plan.cpp), and
// de-duplicated at the end like OBasicCommandContext.addToUniqueResult
// (C/command/OBasicCommandContext.java:347-353). Scans, radix sorts and flagged selects are hipCUB
// (rocPRIM) device primitives; the traversal kernels are hand-written (kernels.hip).
#include "exec.h"
#include "projdev.h"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>

#include "dist.h"
#include "kernels.h"
#include "project.h"

namespace omx {
namespace {
// rocPRIM's radix sort takes its merge-sort path up to 2^20 items: at C2's 0.7 M rows that is 21 launches,
// ≈0.14 ms. With a merge-sort limit of 0 every size above one block runs onesweep (one histogram pass and
// ⌈bits / 8⌉ scatter passes): C2 0.920 → 0.888 ms, R1 1.573 → 1.495 ms, M1 and C4 unchanged (one box,
// interleaved, `gpurun_out/rs1`, `rs2`).
using OnesweepSort = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
template <class K, class V>
hipError_t sort_pairs(void *t, size_t &b, const K *ki, K *ko, const V *vi, V *vo, uint64_t n, int bits, hipStream_t s) {
  return rocprim::radix_sort_pairs<OnesweepSort>(t, b, ki, ko, vi, vo, (size_t)n, 0u, (unsigned)bits, s);
}
template <class K>
hipError_t sort_keys(void *t, size_t &b, const K *ki, K *ko, uint64_t n, int bits, hipStream_t s) {
  return rocprim::radix_sort_keys<OnesweepSort>(t, b, ki, ko, (size_t)n, 0u, (unsigned)bits, s);
}
}  // namespace
}  // namespace omx

namespace omx {
namespace {

struct CastU64 {
  __host__ __device__ uint64_t operator()(const uint32_t &x) const { return x; }
};
struct NonZeroU64 {
  __host__ __device__ uint8_t operator()(const uint64_t &x) const { return x != 0; }
};
struct CastU8U32 {
  __host__ __device__ uint32_t operator()(const uint8_t &x) const { return x; }
};
// a hub-annotated col entry (bit 31: the entry names a hub)
struct HubFlag {
  __host__ __device__ uint64_t operator()(const uint32_t &x) const { return x >> 31; }
};
struct HubFlag8 {
  __host__ __device__ uint8_t operator()(const uint32_t &x) const { return (uint8_t)(x >> 31); }
};

class Timer {
 public:
  Timer(bool on, bool hot_only, hipStream_t s, std::vector<hipEvent_t> *pool)
      : on_(on), hot_only_(hot_only), s_(s), pool_(pool) {
    // OMX_TIME_ONLY=<timer name> with OMX_FLAG_TIME_HOT: only that traversal kernel is timed — a benchmark's
    // timed steps measure their dominant kernel with two events a launch, not every hot kernel (bench.py)
    if (hot_only_)
      if (const char *o = std::getenv("OMX_TIME_ONLY")) only_ = o;
  }
  ~Timer() {
    for (auto &r : recs_) {
      pool_->push_back(r.a);
      pool_->push_back(r.b);
    }
  }
  // the traversal kernels (what OMX_FLAG_TIME_HOT keeps)
  static bool hot(const char *name) {
    static const char *const kHot[] = {"k_expand_heavy", "k_expand_heavy_sliced", "k_expand_light",
                                       "k_expand_light_sliced", "k_expand_light_check", "k_expand_heavy_check",
                                       "k_check", "k_bfs_pull", "k_bfs_pull_sparse", "k_bfs_pull_exit", "k_bfs_push",
                                       "k_bfs_emit", "k_trav_filter", "trav_select", "k_femit",
                                       "k_isect_merge", "k_flists", "k_flist_copy", "k_fof2_a", "k_fof2_b"};
    for (const char *h : kHot)
      if (std::strcmp(name, h) == 0) return true;
    return false;
  }
  // regions nest (a span such as "dedup" may hold a timed kernel): begin pushes, end closes the
  // innermost open region
  void begin(const char *name, hipStream_t st = nullptr) {
    if (!on_ || (hot_only_ && (!hot(name) || (!only_.empty() && only_ != name)))) {
      open_.push_back(SIZE_MAX);
      return;
    }
    Rec r;
    r.name = name;
    r.s = st ? st : s_;
    r.a = event();
    r.b = event();
    HIP_CHECK(hipEventRecord(r.a, r.s));
    recs_.push_back(r);
    open_.push_back(recs_.size() - 1);
  }
  // bytes: the algorithmic bytes; hbm: the bytes HBM must move at least, when a kernel
  // re-reads data it shares between work items from L2 (default: the algorithmic bytes)
  void end(uint64_t bytes = 0, uint64_t hbm = UINT64_MAX) {
    if (open_.empty()) return;
    last_ = open_.back();
    open_.pop_back();
    if (last_ == SIZE_MAX) return;
    recs_[last_].bytes = bytes;
    recs_[last_].hbm = hbm == UINT64_MAX ? bytes : hbm;
    HIP_CHECK(hipEventRecord(recs_[last_].b, recs_[last_].s));
  }
  // algorithmic bytes of the region just closed, when they are only known after the launch
  void amend(uint64_t bytes, uint64_t hbm = UINT64_MAX) {
    if (last_ != SIZE_MAX) {
      recs_[last_].bytes = bytes;
      recs_[last_].hbm = hbm == UINT64_MAX ? bytes : hbm;
    }
  }
  // index of the region just closed (SIZE_MAX when it was not recorded)
  size_t last() const { return last_; }
  bool on() const { return on_; }
  void amend_at(size_t i, uint64_t bytes, uint64_t hbm = UINT64_MAX) {
    if (i < recs_.size()) {
      recs_[i].bytes = bytes;
      recs_[i].hbm = hbm == UINT64_MAX ? bytes : hbm;
    }
  }
  // precondition: the stream has completed (Executor::run waits for its end event first)
  void collect(std::vector<omx_result::KStat> &out, std::vector<omx_result::KStat> &each) {
    if (!on_) return;
    for (auto &r : recs_) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
      each.push_back({r.name, 1, ms, r.bytes, r.hbm});
      auto it = std::find_if(out.begin(), out.end(), [&](const omx_result::KStat &k) { return k.name == r.name; });
      if (it == out.end()) {
        out.push_back({r.name, 0, 0, 0, 0});
        it = out.end() - 1;
      }
      it->launches++;
      it->ms += ms;
      it->bytes += r.bytes;
      it->hbm += r.hbm;
    }
  }

 private:
  hipEvent_t event() {
    hipEvent_t e;
    if (!pool_->empty()) {
      e = pool_->back();
      pool_->pop_back();
    } else {
      HIP_CHECK(hipEventCreate(&e));
    }
    return e;
  }
  struct Rec {
    std::string name;
    hipEvent_t a, b;
    hipStream_t s;
    uint64_t bytes = 0, hbm = 0;
  };
  bool on_, hot_only_;
  std::string only_;
  std::vector<size_t> open_;
  size_t last_ = SIZE_MAX;
  hipStream_t s_;
  std::vector<hipEvent_t> *pool_;
  std::vector<Rec> recs_;
};

// out[i] = src[idx[i]] (u64 values at u64 positions: a CSR's row pointers mapped through a scan)
__global__ void k_gather_u64_at(const uint64_t *src, const uint64_t *idx, uint64_t n, uint64_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}
static void launch_gather_u64_at(const uint64_t *src, const uint64_t *idx, uint64_t n, uint64_t *out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_gather_u64_at, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, idx, n, out);
}

// out[id[i]] = lo[i] | hi[i] << 32 (a fetched adjacency's degrees placed at their vertices)
__global__ void k_scatter_deg(const uint32_t *id, const uint32_t *lo, const uint32_t *hi, uint64_t n, uint64_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[id[i]] = (uint64_t)lo[i] | (uint64_t)hi[i] << 32;
}
static void launch_scatter_deg(const uint32_t *id, const uint32_t *lo, const uint32_t *hi, uint64_t n, uint64_t *out,
                               hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_scatter_deg, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, id, lo, hi, n, out);
}

// lo[i], hi[i] = the two words of in[i]: a u64 column as two u32 columns for a row exchange (a multigraph
// row may hold 2^32 or more entries)
__global__ void k_u64_split(const uint64_t *in, uint64_t n, uint32_t *lo, uint32_t *hi) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    lo[i] = (uint32_t)in[i];
    hi[i] = (uint32_t)(in[i] >> 32);
  }
}
static void launch_u64_split(const uint64_t *in, uint64_t n, uint32_t *lo, uint32_t *hi, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_u64_split, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, n, lo, hi);
}

// a partition's CSR as V + 1 global row pointers (rows outside [lo, hi) empty): what the lists col's
// hub-first row reordering (build_pull_col) walks
__global__ void k_full_rp(const uint64_t *rp_local, uint32_t lo, uint32_t hi, uint32_t V, uint64_t *out) {
  const uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v <= V) out[v] = v < lo ? 0 : v <= hi ? rp_local[v - lo] : rp_local[hi - lo];
}
// occurrences of every vertex in a col (a partition's stand-in for the opposite CSR's degrees: the hubs of
// its lists col are the targets its own rows name most)
__global__ void k_col_occurrences(const uint32_t *col, uint64_t E, uint32_t *cnt) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[col[e]], 1u);
}

// head[i] = 1 where a run of equal sorted keys starts
__global__ void k_u64_heads(const uint64_t *k, uint64_t n, uint8_t *head) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) head[i] = i == 0 || k[i] != k[i - 1];
}
static void launch_u64_heads(const uint64_t *k, uint64_t n, uint8_t *head, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_u64_heads, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k, n, head);
}

__global__ void k_invert_flags(const uint8_t *in, uint8_t *out, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = in[i] ? 0 : 1;
}

__global__ void k_pack_tuple(const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, int k, int vbits, uint64_t n,
                             uint64_t *keys);
__global__ void k_unpack_tuple(const uint64_t *keys, uint64_t n, int k, int vbits, uint32_t *c0, uint32_t *c1,
                               uint32_t *c2);

class Executor {
 public:
  Executor(Graph &g, const Plan &p, const omx_exec_options &o, Transport *tr)
      : g_(g), p_(p), o_(o), tr_(tr), s_(g.stream), pool_(g.pool), tm_((o.flags & OMX_FLAG_KERNEL_TIMING) != 0, (o.flags & OMX_FLAG_TIME_HOT) != 0, g.stream, &g.event_pool) {
    nwords_ = ((uint64_t)g.V + 63) / 64;
    // rows with at least this many neighbours take the chunked kernel (tests lower it to force the path)
    if (const char *h = std::getenv("OMX_HEAVY_DEG")) {
      heavy_deg_ = std::max<uint64_t>(1, std::strtoull(h, nullptr, 10));
      heavy_deg_sliced_ = heavy_deg_;
      heavy_deg_fixed_ = true;
    }
    if (const char *uc = std::getenv("OMX_UNF_CHUNK")) {
      const unsigned long c = std::strtoul(uc, nullptr, 10);
      unf_chunk_shift_ = c == 256 ? 8u : c == 512 ? 9u : c == 2048 ? 11u : 10u;
    }
    if (const char *h = std::getenv("OMX_HEAVY_DEG_UNFILTERED")) {
      heavy_deg_unfiltered_ = std::max<uint64_t>(1, std::strtoull(h, nullptr, 10));
      heavy_deg_unfiltered_set_ = true;
    }
    // variable-length strategy: "bfs" (multi-source BFS whenever exact), "pairs" ((row, v) levels), auto
    if (const char *v = std::getenv("OMX_VARLEN")) varlen_mode_ = v;
    if (const char *sl = std::getenv("OMX_SLICED")) sliced_ = std::strcmp(sl, "0") != 0;
    if (const char *sh = std::getenv("OMX_SLICE_SHIFT"))
      slice_shift_ = (uint32_t)std::min<long>(20, std::max<long>(6, std::strtol(sh, nullptr, 10)));
    if (const char *f = std::getenv("OMX_FUSE_CHECK")) fuse_mode_ = f;  // "0" disables the intersection
    if (const char *sw = std::getenv("OMX_SWAP_CHECK")) swap_ = std::strcmp(sw, "0") != 0;
    if (const char *de = std::getenv("OMX_DENSE_EXCHANGE")) dense_exchange_ = std::strcmp(de, "0") != 0;
    if (const char *hp = std::getenv("OMX_HUB_PUSH")) hub_push_ = std::strcmp(hp, "force") == 0 ? 2 : std::strcmp(hp, "0") != 0 ? 1 : 0;
    // OMX_MERGE: "0" keeps every closing check a binary-search probe; "force" merges every row whose two
    // lists fit a tile (tests); merge_ratio_: merge when the longer list is ≤ ratio × the shorter
    if (const char *mg = std::getenv("OMX_MERGE")) merge_ = std::strcmp(mg, "force") == 0 ? 2 : std::strcmp(mg, "0") != 0 ? 1 : 0;
    if (const char *hb = std::getenv("OMX_PULL_HUBS")) pull_hubs_ = (uint32_t)std::strtoul(hb, nullptr, 10);
    if (const char *d = std::getenv("OMX_BFS_PULL_DIV")) pull_div_ = std::max(1e-9, std::strtod(d, nullptr));
    if (const char *lv = std::getenv("OMX_PULL_LIVE")) pull_live_ = std::strcmp(lv, "0") != 0;
    if (const char *pr = std::getenv("OMX_PULL_PROBE")) pull_probe_ = std::strtod(pr, nullptr);
    if (const char *px = std::getenv("OMX_PULL_EXIT")) pull_exit_ = std::strcmp(px, "0") != 0;
    if (const char *pw = std::getenv("OMX_PULL_WAVE")) pull_wave_ = std::strcmp(pw, "0") != 0;
    if (const char *sp = std::getenv("OMX_SPARSE_PREP")) {
      sparse_prep_ = std::strcmp(sp, "0") != 0;
      if (std::atoi(sp) > 1) sparse_div_ = (uint64_t)std::atoi(sp);
    }
    bms_.resize(p.bitmaps.size());
    col_.resize(p.aliases.size());
    bound_.assign(p.aliases.size(), 0);
    if (const char *r = std::getenv("OMX_ROUTE_SELF")) route_self_ = std::strcmp(r, "0") != 0;
    debug_expand_ = std::getenv("OMX_HOST_TRACE") != nullptr;  // + one stderr line per expansion
    if (const char *ls = std::getenv("OMX_LIGHT_SLICED")) light_sliced_ = std::strcmp(ls, "0") != 0;
    if (const char *fz = std::getenv("OMX_FACTOR")) {  // "0": never; "force": every filtered hop (tests)
      factor_ = std::strcmp(fz, "0") != 0;
      if (std::strcmp(fz, "force") == 0) factor_min_rows_ = 1, factor_min_ratio_ = 0;
    }
    if (const char *fe = std::getenv("OMX_FEMIT")) femit_ = std::strcmp(fe, "force") == 0 ? 2 : std::strcmp(fe, "0") != 0 ? 1 : 0;
    if (const char *fl = std::getenv("OMX_FEMIT_SLOW")) femit_slow_ = std::strcmp(fl, "0") != 0;
    if (const char *sj = std::getenv("OMX_SEMI")) semi_ok_ = std::strcmp(sj, "0") != 0;
    if (const char *gq = std::getenv("OMX_GRP32")) grp32_ = std::strcmp(gq, "0") != 0;
    if (const char *fl = std::getenv("OMX_FLISTS")) flists_ = std::strcmp(fl, "0") != 0;  // "0": the sliced path
    if (const char *dp = std::getenv("OMX_DEVPROJ")) devproj_ = std::strcmp(dp, "0") != 0;
    if (const char *mf = std::getenv("OMX_MARK_FUSE")) mark_fuse_ = std::strcmp(mf, "0") != 0;
    if (const char *am = std::getenv("OMX_ARENA_MARGIN")) arena_margin_ = std::max(0.0, std::strtod(am, nullptr));
    dist_setup();
  }

  omx_result *run() {
    auto t0 = std::chrono::steady_clock::now();
    // OMX_HOST_TRACE=1: host-side phase times of each execute on stderr (µs; "gap" = since the
    // previous execute returned)
    static const bool host_trace = std::getenv("OMX_HOST_TRACE") != nullptr;
    static std::chrono::steady_clock::time_point last_exit;
    std::vector<std::pair<const char *, std::chrono::steady_clock::time_point>> marks;
    auto mark = [&](const char *n) {
      if (host_trace) marks.emplace_back(n, std::chrono::steady_clock::now());
    };
    mark("run");
    trace_waits_ = host_trace;
    last_wait_end_ = t0;
    auto res = std::make_unique<omx_result>();
    // the execute's bracketing events come from the graph's event pool (no create / destroy per execute)
    auto pooled_event = [&] {
      hipEvent_t e;
      if (!g_.event_pool.empty()) {
        e = g_.event_pool.back();
        g_.event_pool.pop_back();
      } else {
        HIP_CHECK(hipEventCreate(&e));
      }
      return e;
    };
    hipEvent_t ea = pooled_event(), eb = pooled_event();
    HIP_CHECK(hipEventRecord(ea, s_));
    mark("events");
    const bool chain = p_.kind != Plan::MATCH;
    if (dist_) gather_global_degrees();  // (degree predicates; a chain's WHERE / WHILE too)
    bool empty = !chain && (p_.empty || !check_candidates());
    bool counted_only = false;
    std::vector<DBuf<uint32_t>> chain_out;
    if (chain && dist_ && tr_->rank() != 0) {
      // a partitioned chain runs on rank 0; the others serve the adjacency lists it asks for
      serve_chain();
      R_ = 0;
      chain_out.push_back(DBuf<uint32_t>(&pool_, 1));
    } else if (chain) {
      chain_out.push_back(p_.kind == Plan::TRAVERSE ? traverse_bfs()
                          : p_.kind == Plan::SELECT ? select_expand()
                                                    : shortest_path());
      if (dist_) tr_->allgather_n({0, 0}, s_);  // the servers stop
    } else if (!empty && fof2_ok()) {
      fof2();
    } else if (!empty) {
      // a partitioned run keeps stepping with no local rows: every rank takes part in every exchange
      for (size_t i = 0; i < p_.steps.size() && (R_ > 0 || dist_); ++i) {
        const Step &st = p_.steps[i];
        bool last = i + 1 == p_.steps.size();
        bool count_only = last && o_.mode == OMX_MODE_COUNT && p_.unique_by_construction && st.kind == S_EXPAND;
        // the last expansion of a plan whose rows are distinct by construction may stay block-
        // segmented in HBM when the rows are not copied to the host
        bool seg_ok = last && p_.unique_by_construction && p_.proj == Plan::PROJ_ALIASES && !gather0_ &&
                      (o_.flags & OMX_FLAG_KEEP_DEVICE) && !(o_.flags & OMX_FLAG_DIGEST);
        // expansion + closing check fused into one intersection pass
        const Step *fuse = nullptr;
        if (st.kind == S_EXPAND && i + 1 < p_.steps.size() && fuse_ok(st, p_.steps[i + 1])) {
          prune(p_.live_before[i]);
          fuse = &p_.steps[i + 1];
          const bool last2 = i + 2 == p_.steps.size();
          count_only = last2 && o_.mode == OMX_MODE_COUNT && p_.unique_by_construction;
          seg_ok = last2 && p_.unique_by_construction && p_.proj == Plan::PROJ_ALIASES && !gather0_ &&
                   (o_.flags & OMX_FLAG_KEEP_DEVICE) && !(o_.flags & OMX_FLAG_DIGEST);
          expand_step(st, !count_only, seg_ok, fuse);
          counted_only = count_only;
          ++i;
          continue;
        }
        prune(p_.live_before[i]);
        if (last && st.kind == S_EXPAND && mark_ok(st)) {
          expand_mark(st);
          continue;
        }
        semi_ = last && !count_only && semi_for(st);
        switch (st.kind) {
          case S_ROOT: root(st); break;
          case S_EXPAND: expand_step(st, !count_only, seg_ok); counted_only = count_only; break;
          case S_CHECK: check_step(st); break;
          case S_VARLEN: varlen_step(st); break;
          case S_NEWROOT:
          case S_CARTESIAN: cross_step(st); break;
          case S_KILL: R_ = 0; break;
          case S_ROWCMP: rowcmp_step(st); break;
          case S_MULTI: multi_step(st); break;
        }
      }
      if (p_.steps.empty()) R_ = 0;
    } else {
      R_ = 0;
    }
    if (!chain) bindings_ = marked_ ? marked_bindings_ : semi_hops_ ? semi_bindings_ : R_;
    uint64_t n = 0;
    int ncols = 0;
    std::vector<DBuf<uint32_t>> out;
    // partitioned + distinct projection: equal tuples meet on one rank first (a chain's records are
    // on rank 0 already, in their order)
    if (dist_ && !chain && !empty && !counted_only && gather0_) {
      pre_rank0_distinct();
      route_rank0();
    }
    else if (dist_ && !chain && !empty && !counted_only && !p_.unique_by_construction) route_hash(p_.out_aliases);
    const bool sp_doc = p_.kind == Plan::SHORTEST_PATH && !p_.chain.expand_rows;
    const bool docs = p_.proj == Plan::PROJ_EXPR || p_.proj == Plan::PROJ_JSON || sp_doc;
    // partitioned: the lists out()/in()/both() read in RETURN expressions, from the vertices' owners
    RetAdj fetched;
    if (dist_ && !empty && !counted_only && docs && !p_.ret_adj_alias.empty()) fetch_return_adjacency(fetched);
    if (sp_doc) {  // SELECT shortestPath(...): one document whose field is the list of the path's RIDs
      HVal list;
      list.k = HVal::LIST;
      std::vector<uint64_t> rids(R_);
      if (R_) {
        DBuf<uint64_t> d(&pool_, R_);
        const uint32_t *cp = chain_out[0].p;
        launch_map_rids(1, &cp, R_, g_.d_rids, d.p, g_.V, s_);
        HIP_CHECK(hipMemcpyAsync(rids.data(), d.p, R_ * 8, hipMemcpyDeviceToHost, s_));
        HIP_CHECK(hipStreamSynchronize(s_));
      }
      list.json = "[";
      for (uint64_t i = 0; i < R_; ++i) {
        HVal r;
        r.k = HVal::RID;
        r.rid = rids[i];
        list.items.push_back(r);
        list.json += (i ? ",\"#" : "\"#") + std::to_string(rids[i] >> 48) + ":" + std::to_string(rids[i] & ((1ull << 48) - 1)) + "\"";
      }
      list.json += "]";
      res->docs.push_back(Document{list});
      n = 1;
      ncols = 1;
    } else if (chain) {  // the records in emission order (duplicates are the reference's: not de-duplicated)
      n = R_;
      ncols = 1;
      out = std::move(chain_out);
    } else if (R_ > 0 && !counted_only && docs) {
      // RETURN expressions / JSON: distinct tuples of the aliases they read (device), then one document
      // per tuple, de-duplicated by content (project.cpp: the OResultSet fill of addResult :698-719)
      if (!p_.out_aliases.empty()) project_dedup(out, n);
      else n = 1;  // constant expressions: the same document for every binding
      std::vector<const uint32_t *> cp;
      for (auto &c : out) cp.push_back(c.p);
      int64_t lim = p_.limit >= 0 ? p_.limit : o_.limit;
      // with LIMIT the host evaluator runs: it stops at the limit-th distinct document, as
      // addSingleResult :737-750 does, so an error in a later row is never raised (the device evaluates
      // every row); row indices are u32 in the device dedup table
      if (devproj_ && lim < 0 && n < UINT32_MAX && !p_.out_aliases.empty() && device_projection_ok(g_, p_, nullptr)) {
        // scalar items: evaluated and de-duplicated by content on the device (projdev.hip)
        tm_.begin("k_pj_eval");
        device_project(g_, p_, cp, n, lim, cus(), s_, *res);
        tm_.end(n * (4ull * cp.size() + 9ull * p_.returns.size()) * 2);
        n = res->n_pcol_rows;
      } else {
        tm_.begin("documents");
        res->docs = build_documents(g_, p_, cp, n, lim, s_, dist_ ? &fetched : nullptr);
        tm_.end();
        n = res->docs.size();
      }
      ncols = (int)p_.out_names.size();
      dedup_ran_ = 1;
    } else if (R_ > 0 && !counted_only) {
      project_dedup(out, n);
      ncols = (int)out.size();
    } else if (counted_only) {
      n = R_;
      ncols = (int)p_.out_aliases.size();
    }
    int64_t limit = p_.limit >= 0 ? p_.limit : o_.limit;
    if (dist_ && counted_only && limit > -1) {
      // COUNT with LIMIT over a partitioned snapshot: the ranks' counted rows are disjoint (distinct by
      // construction), so the result is min(Σ ranks, max(LIMIT, 1)), reported by rank 0
      uint64_t total = 0;
      for (uint64_t x : tr_->allgather(n, s_)) total += x;
      n = tr_->rank() == 0 ? total : 0;
    }
    if (limit > -1 && n > (uint64_t)std::max<int64_t>(limit, 1)) n = (uint64_t)std::max<int64_t>(limit, 1);
    if (n > 0 && !counted_only && !docs && (o_.flags & OMX_FLAG_DIGEST)) {
      std::vector<const uint32_t *> cp;
      for (auto &c : out) cp.push_back(c.p);
      DBuf<unsigned long long> d(&pool_, 1);
      HIP_CHECK(hipMemsetAsync(d.p, 0, 8, s_));
      launch_digest(ncols, cp.data(), n, (o_.flags & OMX_FLAG_NO_RID_MAP) ? nullptr : g_.d_rids, g_.V, d.p, cus(), s_);
      digest_ = read1(reinterpret_cast<const uint64_t *>(d.p));
    }
    if (n > 0 && !counted_only && !docs && !(o_.flags & OMX_FLAG_KEEP_DEVICE)) deliver_rows(out, n, ncols, *res);
    mark("launched");
    HIP_CHECK(hipEventRecord(eb, s_));
    // spin on the end event (the stream is usually idle by now: the last mailbox read waited for the
    // kernels) instead of a blocking synchronisation, whose wake-up costs ~10 µs per execute
    for (;;) {
      const hipError_t e = hipEventQuery(eb);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) fail(OMX_E_DEVICE, std::string("stream failed: ") + hipGetErrorString(e));
      __builtin_ia32_pause();
    }
    mark("synced");
    float dms = 0;
    HIP_CHECK(hipEventElapsedTime(&dms, ea, eb));
    g_.event_pool.push_back(ea);
    g_.event_pool.push_back(eb);
    tm_.collect(res->kstats, res->klaunches);
    res->info.n_rows = n;
    res->info.n_cols = n ? ncols : 0;
    res->info.deduplicated = dedup_ran_;
    res->info.edges_traversed = edges_;
    res->info.edges_read = edges_iter_;
    res->info.factorized_hops = (int32_t)factorized_hops_;
    res->info.rows_gathered = rows_gathered_;
    res->info.digest = digest_;
    res->info.documents = docs ? 1 : 0;
    res->info.bindings = bindings_;
    res->info.alg_bytes = alg_bytes_;
    res->info.device_ms = dms;
    res->names = p_.out_names;
    res->info.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    mark("done");
    if (host_trace) {
      auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::micro>(b - a).count();
      };
      std::fprintf(stderr, "[omx host] gap %.1f", last_exit.time_since_epoch().count() ? us(last_exit, t0) : 0.0);
      for (size_t i = 1; i < marks.size(); ++i) std::fprintf(stderr, " %s %.1f", marks[i].first, us(marks[i - 1].second, marks[i].second));
      std::fprintf(stderr, " | waits %zu:", waits_.size());
      for (auto &w : waits_) std::fprintf(stderr, " +%.0f/%.0f", w.first, w.second);
      std::fprintf(stderr, "\n");
      last_exit = std::chrono::steady_clock::now();
    }
    return res.release();
  }

 private:
  // The rows' hand-over to the host (SURVEY §8(b) Ownership, §8(d): reported apart from the step): the
  // dense ids are mapped to RIDs chunk by chunk into a ring of two device staging slots (k_map_rids on the
  // executor's stream) and each chunk is copied by DMA into the result's pinned host block on the side
  // stream, so chunk i+1's map runs under chunk i's copy and the device never holds the whole RID table.
  // The block comes from the process-wide pool (host_rows_acquire): no pinning, no zeroing once warm.
  void deliver_rows(const std::vector<DBuf<uint32_t>> &out, uint64_t n, int ncols, omx_result &res) {
    const uint64_t row_bytes = 8ull * (uint64_t)ncols, total = n * row_bytes;
    res.rows = static_cast<uint64_t *>(host_rows_acquire(total, &res.rows_capacity, &res.rows_pinned));
    res.info.host_rows_bytes = res.rows_capacity;
    res.info.host_rows_pinned = res.rows_pinned ? 1 : 0;
    // chunks of 1/8 of the table, between 256 KiB and 256 MiB: a mid-size result still overlaps
    const uint64_t chunk_bytes = std::min<uint64_t>(256ull << 20, std::max<uint64_t>(256ull << 10, total / 8));
    const uint64_t chunk_rows = std::max<uint64_t>(1, chunk_bytes / row_bytes);
    const uint64_t nslot = std::min<uint64_t>(n, chunk_rows);
    DBuf<uint64_t> stage(&pool_, 2 * nslot * ncols);
    const uint64_t *rid_map = (o_.flags & OMX_FLAG_NO_RID_MAP) ? nullptr : g_.d_rids;
    hipStream_t cs = g_.stream2;
    hipEvent_t mapped[2], copied[2], fin;
    for (int j = 0; j < 2; ++j) {
      HIP_CHECK(hipEventCreateWithFlags(&mapped[j], hipEventDisableTiming));
      HIP_CHECK(hipEventCreateWithFlags(&copied[j], hipEventDisableTiming));
    }
    HIP_CHECK(hipEventCreateWithFlags(&fin, hipEventDisableTiming));
    tm_.begin("deliver_d2h");
    std::vector<const uint32_t *> cp(ncols);
    uint64_t c = 0;
    for (uint64_t r0 = 0; r0 < n; r0 += chunk_rows, ++c) {
      const int slot = (int)(c & 1);
      const uint64_t nr = std::min(chunk_rows, n - r0);
      uint64_t *dst = stage.p + (uint64_t)slot * nslot * ncols;
      if (c >= 2) HIP_CHECK(hipStreamWaitEvent(s_, copied[slot], 0));  // the slot's previous copy is done
      for (int k = 0; k < ncols; ++k) cp[k] = out[k].p + r0;
      tm_.begin("k_map_rids");
      launch_map_rids(ncols, cp.data(), nr, rid_map, dst, g_.V, s_);
      tm_.end(nr * (uint64_t)ncols * 12);
      HIP_CHECK(hipEventRecord(mapped[slot], s_));
      HIP_CHECK(hipStreamWaitEvent(cs, mapped[slot], 0));
      HIP_CHECK(hipMemcpyAsync(res.rows + r0 * ncols, dst, nr * row_bytes, hipMemcpyDeviceToHost, cs));
      HIP_CHECK(hipEventRecord(copied[slot], cs));
    }
    HIP_CHECK(hipEventRecord(fin, cs));
    HIP_CHECK(hipStreamWaitEvent(s_, fin, 0));  // the executor's end event waits for the last copy
    tm_.end(total);
    for (int j = 0; j < 2; ++j) {
      (void)hipEventDestroy(mapped[j]);
      (void)hipEventDestroy(copied[j]);
    }
    (void)hipEventDestroy(fin);
  }

  Graph &g_;
  const Plan &p_;
  omx_exec_options o_;
  Transport *tr_ = nullptr;
  bool dist_ = false;        // partitioned execution: rows routed between ranks (dist.h)
  bool route_self_ = false;  // OMX_ROUTE_SELF=1: route through the transport even with one rank (tests)
  int owner_col_ = -1;       // rows currently sit on the owner of this column's vertex
  uint32_t block_ = 0;       // vertices per rank (block partition)
  std::vector<char> bound_;  // aliases bound so far (the same on every rank, whatever its row count)
  hipStream_t s_;
  DevicePool &pool_;
  Timer tm_;
  uint64_t nwords_;
  std::vector<DBuf<uint64_t>> bms_;
  std::vector<DBuf<uint32_t>> col_;
  uint64_t R_ = 1;
  uint64_t edges_ = 0, alg_bytes_ = 0, bindings_ = 0;
  // adjacency entries iterated one by one (omx_result_info.edges_read): E_t minus count-only hops summed
  // from degrees and minus the E_t of closing checks answered by binary search
  uint64_t edges_iter_ = 0;
  uint64_t digest_ = 0;  // OMX_FLAG_DIGEST
  int dedup_ran_ = 0;
  int cus_ = 0;
  uint64_t heavy_deg_ = kHeavyDeg;
  uint64_t heavy_deg_sliced_ = kHeavyDegSliced;
  bool heavy_deg_fixed_ = false;  // OMX_HEAVY_DEG given
  uint32_t unf_chunk_shift_ = 11;  // heavy chunk windows of unfiltered writes (OMX_UNF_CHUNK; 2048: profiles/r02/chunkwin)
  uint64_t heavy_deg_unfiltered_ = kHeavyDeg;  // unfiltered hops (OMX_HEAVY_DEG_UNFILTERED, over OMX_HEAVY_DEG)
  bool heavy_deg_unfiltered_set_ = false;
  bool debug_expand_ = false;
  bool light_sliced_ = true;  // LDS-sliced light kernel for sliced single-part hops (OMX_LIGHT_SLICED=0: merge path)
  bool sliced_ = true;  // LDS-sliced heavy kernel for filtered hops (OMX_SLICED=0 disables)
  uint32_t slice_shift_ = 20;  // log2 vertices per slice (OMX_SLICE_SHIFT, 6..20: tests cut small graphs)
  std::string varlen_mode_ = "auto";
  std::string fuse_mode_ = "1";
  bool swap_ = true;  // fused closing check iterates the shorter of the two lists (OMX_SWAP_CHECK=0: off)
  // fused closing check: merge path for lists of comparable lengths (isect.hip). Off by default: at C4
  // (LDBC SF10, lists of ≈ 30) the binary-search probe of an L1-resident list takes 0.74 ms a step and the
  // wave-tiled merge 1.38 ms (it reads both lists, 210 M entries against 65 M iterated; round 4,
  // profiles/r04/isect); OMX_MERGE=1 merges rows by the ratio rule, =force every row that fits a tile
  int merge_ = 0;
  double merge_ratio_ = 8;
  // hub masks packed for the pull kernel in degree-rank order (4 MiB: one XCD's L2); 0 = plain col. 2^20
  // measured best of 2^17…2^22 at C3 in round 2 (profiles/r02/c3rank); with the LDS hubs and the frontier
  // probe of round 3, 2^19 (sparse level 1.546 ms) edges out 2^20 (1.598) and 2^18 (1.594) (r04/c3h)
  uint32_t pull_hubs_ = 1u << 19;
  double pull_div_ = 20;  // bottom-up when the frontier's edges exceed 1/pull_div_ of the adjacency
  bool pull_live_ = true;  // the pull waits only for lanes whose frontier is non-empty
  // levels whose frontier holds fewer than this fraction of the vertices pull through the frontier bitmap
  double pull_probe_ = 0.1;
  bool pull_wave_ = true;  // OMX_PULL_WAVE=0: the workgroup-tiled k_bfs_pull for the tiled bottom-up levels
  bool pull_exit_ = true;  // denser levels pull per vertex with an early exit (OMX_PULL_EXIT=0: tiles)
  // sparse levels: hubs-only pull + push of the non-hub frontier when that pushes under 1/8 of the pull's
  // entries (OMX_HUB_PUSH=0: off, =force: at every sparse level; tests)
  int hub_push_ = 1;
  // partitioned BFS: levels whose frontier holds fewer than V/12 vertices exchange (vertex, mask) triples
  // instead of the frontier blocks (OMX_DENSE_EXCHANGE=1: always the blocks)
  bool dense_exchange_ = false;
  bool segmented_ = false;  // the final table is block-segmented (see expand_core)
  // sliced hops size their arenas from the target bitmap's density (OMX_ARENA_MARGIN scales the
  // estimate, 0 forces the short-arena re-run in tests)
  double arena_margin_ = 1.25;
  bool factor_ = true;           // factorized expansion of filtered hops (OMX_FACTOR=0: direct)
  bool sparse_prep_ = true;      // BFS level prologues over a push's touched list (OMX_SPARSE_PREP=0: full sweeps)
  uint64_t sparse_div_ = 8;      // (OMX_SPARSE_PREP=<n>: the push's edge bound V / n; 1 = every push)
  uint64_t factorized_hops_ = 0;
  uint64_t semi_hops_ = 0;  // last hops written as a semi-join (Executor::semi_join)
  uint64_t arena_retries_ = 0;
  bool trace_waits_ = false;  // OMX_HOST_TRACE
  std::vector<std::pair<double, double>> waits_;
  std::chrono::steady_clock::time_point last_wait_end_;

  // ---- helpers -----------------------------------------------------------------------------------
  template <class F>
  void cub(F f) {
    size_t bytes = 0;
    HIP_CHECK(f((void *)nullptr, bytes));
    DBuf<uint8_t> tmp(&pool_, std::max<size_t>(bytes, 16));
    HIP_CHECK(f((void *)tmp.p, bytes));
  }
  // the next mailbox a kernel posts to (kernels.h Mail), and the host side of it: spin on the
  // sequence word; every few thousand spins ask the stream whether it ended (or faulted) without
  // posting, so a failed launch surfaces as an error rather than a hang
  Mail mail() { return Mail{g_.h_mail, ++g_.mail_seq}; }
  const uint64_t *wait_mail() {
    volatile uint64_t *f = g_.h_mail + kMailSeq;
    const uint64_t seq = g_.mail_seq;
    // OMX_HOST_TRACE: each host wait's (µs since the previous wait ended, µs waited)
    struct WaitMark {
      std::vector<std::pair<double, double>> *w;
      std::chrono::steady_clock::time_point t0;
      std::chrono::steady_clock::time_point *last;
      ~WaitMark() {
        if (!w) return;
        const auto t1 = std::chrono::steady_clock::now();
        w->emplace_back(std::chrono::duration<double, std::micro>(t0 - *last).count(),
                        std::chrono::duration<double, std::micro>(t1 - t0).count());
        *last = t1;
      }
    } wm{trace_waits_ ? &waits_ : nullptr, std::chrono::steady_clock::now(), &last_wait_end_};
    for (uint32_t spins = 1; *f != seq; ++spins) {
      if (spins % 4096 == 0) {
        const hipError_t e = hipStreamQuery(s_);
        if (e == hipErrorNotReady) continue;
        if (e != hipSuccess) fail(OMX_E_DEVICE, std::string("stream failed: ") + hipGetErrorString(e));
        if (*f == seq) break;
        fail(OMX_E_DEVICE, "a device mailbox was not posted");
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return g_.h_mail;
  }
  // two u64 words in one host round trip (dptr[0], dptr[1])
  std::pair<uint64_t, uint64_t> read2(const uint64_t *dptr) {
    launch_post_words(dptr, 2, mail(), s_, 8);
    const uint64_t *w = wait_mail();
    return {w[0], w[1]};
  }
  template <class T>
  T read1(const T *dptr) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "read1 reads one 4- or 8-byte word");
    launch_post_words(dptr, 1, mail(), s_, (int)sizeof(T));
    const uint64_t w = wait_mail()[0];
    T v;
    if (sizeof(T) == 8) std::memcpy(&v, &w, 8);
    else { const uint32_t lo = (uint32_t)w; std::memcpy(&v, &lo, sizeof(T)); }
    return v;
  }

  DAdj make_adj(const AdjSpec &a) const {
    DAdj d{};
    d.n = (int32_t)a.parts.size();
    d.sorted = a.sorted;
    for (size_t i = 0; i < a.parts.size(); ++i) {
      const EdgeSet &es = g_.esets[a.parts[i].first];
      d.p[i].rp = g_.rp(es, a.parts[i].second);
      d.p[i].col = g_.col(es, a.parts[i].second);
    }
    return d;
  }

  // partitioned: out()/in()/both().size() of any vertex, through the gathered degree row pointers
  DAdj global_degree_adj(const AdjSpec &a) const {
    DAdj d = make_adj(a);
    for (size_t i = 0; i < a.parts.size(); ++i) {
      const uint64_t *g = g_.esets[a.parts[i].first].d_global_rp[a.parts[i].second];
      if (!g) fail(OMX_E_INVALID, "internal: global degrees not gathered");
      d.p[i].rp = g;
      d.p[i].col = nullptr;  // a degree term never reads neighbours
    }
    return d;
  }
  // every rank's degrees of the CSRs a degree predicate reads, gathered once per snapshot: each rank
  // sends the degrees of its rows to all ranks (all-to-all-v), the scan gives V + 1 row pointers
  void gather_global_degrees() {
    std::vector<std::pair<int, int>> need;
    for (const PredProgram &pp : p_.progs)
      for (const AdjSpec &a : pp.deg)
        for (const auto &part : a.parts)
          if (!g_.esets[part.first].d_global_rp[part.second] &&
              std::find(need.begin(), need.end(), part) == need.end())
            need.push_back(part);
    if (need.empty()) return;
    const int W = tr_->world();
    const std::vector<uint64_t> lohi = tr_->allgather_n({g_.part_lo, g_.part_hi}, s_);
    std::vector<uint64_t> plo(W), phi(W);
    for (int p = 0; p < W; ++p) {
      plo[p] = lohi[2 * p];
      phi[p] = lohi[2 * p + 1];
    }
    const uint32_t V = g_.V, lo = g_.part_lo, hi = g_.part_hi;
    for (const auto &part : need) {
      EdgeSet &es = g_.esets[part.first];
      // degrees travel as u64, two u32 words per vertex (the transport moves u32 columns)
      DBuf<uint64_t> mine(&pool_, std::max<uint32_t>(hi - lo, 1)), all(&pool_, std::max<uint32_t>(V, 1));
      if (hi > lo) launch_row_degree_range(g_.rp(es, part.second), lo, hi, mine.p, s_);
      std::vector<uint64_t> send(W, 2ull * (hi - lo)), sdispl(W, 0), recv(W), rdispl(W);
      for (int p = 0; p < W; ++p) {
        recv[p] = 2 * (phi[p] - plo[p]);
        rdispl[p] = 2 * plo[p];
      }
      tm_.begin("exchange");
      tr_->alltoallv({reinterpret_cast<const uint32_t *>(mine.p)}, send, sdispl,
                     {reinterpret_cast<uint32_t *>(all.p)}, recv, rdispl, s_);
      tm_.end(16ull * V);
      uint64_t *grp = nullptr;
      HIP_CHECK(hipMalloc((void **)&grp, ((uint64_t)V + 1) * 8));
      try {
        HIP_CHECK(hipMemsetAsync(grp, 0, 8, s_));
        cub([&](void *t, size_t &b) { return hipcub::DeviceScan::InclusiveSum(t, b, all.p, grp + 1, (int64_t)V, s_); });
        HIP_CHECK(hipStreamSynchronize(s_));
      } catch (...) {
        (void)hipFree(grp);
        throw;
      }
      es.d_global_rp[part.second] = grp;
      g_.device_bytes += ((uint64_t)V + 1) * 8;
    }
  }

  // records (BitmapSpec::records): the bitmap is kept to that kind's id range afterwards (keep_records)
  DPred make_pred(int prog, int class_id, int records = 0) const {
    DPred d{};
    d.cols = g_.d_cols;
    d.vclass = g_.d_vclass;
    // (a class whose polymorphic set holds every vertex of the snapshot — configs' class:Person — tests
    // nothing: the bitmap kernels then read no class ids; nor does one holding every record of the kind
    // the bitmap is kept to)
    const uint64_t kind_n = records == 1 ? g_.vertices : records == 2 ? (uint64_t)g_.V - g_.vertices : (uint64_t)g_.V;
    if (class_id >= 0 && g_.count(class_id) < kind_n) {
      d.use_class = 1;
      g_.class_mask(class_id, d.class_mask);
    }
    if (prog >= 0) {
      const PredProgram &pp = p_.progs[prog];
      d.n = (int32_t)pp.code.size();
      for (size_t i = 0; i < pp.code.size(); ++i) d.code[i] = pp.code[i];
      for (size_t i = 0; i < pp.deg.size(); ++i) d.deg[i] = dist_ ? global_degree_adj(pp.deg[i]) : make_adj(pp.deg[i]);
      match_atoms(pp, d);
      // a field present on every record of the kind: no presence test (the other kind's bits are cleared)
      for (int a = 0; a < d.n_atoms && records; ++a)
        if (!(records == 1 ? g_.props[d.atom_col[a]].nulls_v : g_.props[d.atom_col[a]].nulls_e)) d.atom_c[a].present = nullptr;
    }
    return d;
  }
  void keep_records(uint64_t *words, int records) {
    if (records == 1) launch_bitmap_keep_range(words, nwords_, 0, g_.vertices, s_);
    else if (records == 2) launch_bitmap_keep_range(words, nwords_, g_.vertices, g_.V, s_);
  }

  // [COL c, INT/DBL k, CMP] (AND|OR [COL, INT/DBL, CMP])* → DPred atoms (evaluated without the VM)
  void match_atoms(const PredProgram &pp, DPred &d) const {
    const auto &c = pp.code;
    if (c.size() < 3 || c.size() > 4 * 3 + 3) return;
    int n = 0, conj = -1;
    size_t i = 0;
    while (i < c.size()) {
      if (i + 2 >= c.size() || c[i].op != P_PUSH_COL || (c[i + 1].op != P_PUSH_INT && c[i + 1].op != P_PUSH_DBL) ||
          c[i + 2].op < P_EQ || c[i + 2].op > P_GE || n >= 4)
        return;
      const int col = c[i].arg;
      const bool dcol = g_.props[col].type == OMX_PROP_DOUBLE, dk = c[i + 1].op == P_PUSH_DBL;
      d.atom_col[n] = col;
      d.atom_c[n] = DColumn{g_.props[col].d_values, g_.props[col].d_present, g_.props[col].type, 0};
      d.atom_op[n] = c[i + 2].op;
      d.atom_dbl[n] = dcol || dk;
      d.atom_i[n] = c[i + 1].i;
      d.atom_d[n] = dk ? c[i + 1].d : (double)c[i + 1].i;
      ++n;
      i += 3;
      if (n > 1) {
        if (i >= c.size() || (c[i].op != P_AND && c[i].op != P_OR)) return;
        int cj = c[i].op == P_AND;
        if (conj >= 0 && cj != conj) return;
        conj = cj;
        ++i;
      } else if (i < c.size()) {
        // the second atom follows; its connective comes after it
      }
    }
    d.n_atoms = n;
    d.conj = conj < 0 ? 1 : conj;
  }

  void eval_bitmap(int prog, int class_id, int64_t depth, uint64_t *words, uint64_t nwords = 0, int records = 0) {
    tm_.begin("k_eval_bitmap");
    if (prog >= 0 && p_.progs[prog].const_false) {
      HIP_CHECK(hipMemsetAsync(words, 0, std::max(nwords, nwords_) * 8, s_));
    } else {
      // (vertices: the ids [0, vertices) evaluated, the words above written zero; edge records: every id, the
      // vertices' bits cleared after)
      launch_eval_bitmap(make_pred(prog, class_id, records), records == 1 ? g_.vertices : g_.V, depth, words, s_, nwords);
      if (records == 2) keep_records(words, records);
    }
    tm_.end((uint64_t)g_.V * 4 + nwords_ * 8);
    alg_bytes_ += (uint64_t)g_.V * 4;
  }

  // words of a filter bitmap: padded to whole slices (the sliced kernels stage slices unchecked)
  uint64_t padded_words() const { return (nwords_ + kBitmapPadWords - 1) / kBitmapPadWords * kBitmapPadWords; }

  const uint64_t *bitmap(int id) {
    if (id < 0) return nullptr;
    if (!bms_[id].p) {
      bms_[id] = DBuf<uint64_t>(&pool_, padded_words());
      // another bitmap of the plan that is one comparison over the same column (M1: the root's `age < 1`
      // and the last hop's `age >= 90`) is evaluated in the same pass over the column (round 6)
      const BitmapSpec &b = p_.bitmaps[id];
      const bool cf = b.prog >= 0 && p_.progs[b.prog].const_false;
      for (size_t j = 0; j < bms_.size() && !cf && b.prog >= 0; ++j) {
        const BitmapSpec &c = p_.bitmaps[j];
        if ((int)j == id || bms_[j].p || c.prog < 0 || p_.progs[c.prog].const_false) continue;
        const DPred pa = make_pred(b.prog, b.class_id, b.records), pb = make_pred(c.prog, c.class_id, c.records);
        DBuf<uint64_t> other(&pool_, padded_words());
        tm_.begin("k_eval_bitmap");
        const bool verts = b.records == 1 && c.records == 1;
        if (!launch_eval_bitmap_pair(pa, pb, verts ? g_.vertices : g_.V, bms_[id].p, other.p, s_, padded_words())) {
          tm_.end();
          continue;
        }
        if (!verts) {
          keep_records(bms_[id].p, b.records);
          keep_records(other.p, c.records);
        }
        tm_.end((uint64_t)g_.V * 4 + 2 * nwords_ * 8);
        alg_bytes_ += (uint64_t)g_.V * 4;
        bms_[j] = std::move(other);
        return bms_[id].p;
      }
      eval_bitmap(b.prog, b.class_id, 0, bms_[id].p, padded_words(), b.records);
    }
    return bms_[id].p;
  }

  uint64_t bitmap_count(const uint64_t *words, int rank, int world) {
    DBuf<uint32_t> cnt(&pool_, nwords_);
    launch_word_popc(words, nwords_, g_.V, rank, world, 0, g_.V, cnt.p, s_);
    DBuf<uint64_t> sum(&pool_, 1);
    hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> it(cnt.p, CastU64());
    cub([&](void *t, size_t &b) { return hipcub::DeviceReduce::Sum(t, b, it, sum.p, (int)nwords_, s_); });
    return read1(sum.p);
  }

  // vertices of a bitmap as a list, restricted to [lo, hi) (and to v % world == rank)
  DBuf<uint32_t> bitmap_list(const uint64_t *words, int rank, int world, uint64_t &n, uint32_t lo = 0,
                             uint32_t hi = UINT32_MAX) {
    hi = std::min(hi, g_.V);
    if (bitmap_list_blocks(nwords_) <= 4096) {  // two launches (≤ 64 M vertices)
      DBuf<uint32_t> out(&pool_, std::max<uint64_t>(hi > lo ? hi - lo : 0, 1));
      DBuf<uint32_t> blk(&pool_, bitmap_list_blocks(nwords_));
      tm_.begin("k_bitmap_to_list");
      launch_bitmap_list_2k(words, nwords_, g_.V, rank, world, lo, hi, blk.p, out.p, mail(), s_);
      n = wait_mail()[0];
      tm_.end(nwords_ * 8 + n * 4);
      return out;
    }
    DBuf<uint32_t> cnt(&pool_, nwords_ + 1);
    DBuf<uint32_t> offs(&pool_, nwords_ + 1);
    tm_.begin("k_bitmap_to_list");
    launch_word_popc(words, nwords_, g_.V, rank, world, lo, hi, cnt.p, s_);
    HIP_CHECK(hipMemsetAsync(cnt.p + nwords_, 0, 4, s_));
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, cnt.p, offs.p, (int)(nwords_ + 1), s_); });
    n = read1(offs.p + nwords_);
    DBuf<uint32_t> out(&pool_, std::max<uint64_t>(n, 1));
    launch_word_scatter(words, nwords_, g_.V, rank, world, lo, hi, offs.p, out.p, s_);
    tm_.end(nwords_ * 8 + n * 4);
    return out;
  }

  // calculateMatch (:340-357): an empty candidate set of a prefetched alias → empty result
  bool check_candidates() {
    // the root's own candidate set needs no separate count: an empty root list already yields no row
    const int root_bm = !p_.steps.empty() && p_.steps[0].kind == S_ROOT ? p_.steps[0].cand_bm : -1;
    for (int bm : p_.must_be_nonempty)
      if (bm >= 0 && bm != root_bm && bitmap_count(bitmap(bm), 0, 1) == 0) return false;
    return true;
  }

  // drop the bound columns no later step reads and the projection does not return
  void prune(const std::vector<char> &live) {
    for (size_t a = 0; a < col_.size(); ++a)
      if (!live[a] && (dist_ ? bound_[a] != 0 : col_[a].p != nullptr)) {
        col_[a].reset();
        bound_[a] = 0;
      }
  }

  std::vector<int> bound_cols() const {
    std::vector<int> c;
    for (size_t a = 0; a < col_.size(); ++a)
      if (dist_ ? bound_[a] != 0 : col_[a].p != nullptr) c.push_back((int)a);
    return c;
  }

  // ---- 1-D partitioned execution (dist.h) ----------------------------------------------------------
  void dist_setup() {
    if (p_.kind != Plan::MATCH && o_.shard_world > 1)
      unsupported("TRAVERSE / SELECT expand() / shortestPath() with root shards");
    if (!tr_) {
      if (g_.partitioned())
        fail(OMX_E_INVALID, "partitioned snapshot executed without a communicator (omx_exec_options.comm)");
      return;
    }
    const int W = tr_->world(), r = tr_->rank();
    if (W < 1 || W > kMaxRanks) fail(OMX_E_INVALID, "communicator world must be in [1, 64]");
    if (o_.shard_world > 1) fail(OMX_E_INVALID, "root shards and a partitioned communicator are exclusive");
    block_ = (uint32_t)(((uint64_t)g_.V + W - 1) / W);
    const uint32_t lo = (uint32_t)std::min<uint64_t>(g_.V, (uint64_t)r * block_);
    const uint32_t hi = (uint32_t)std::min<uint64_t>(g_.V, (uint64_t)(r + 1) * block_);
    if (g_.part_lo != lo || g_.part_hi != hi)
      fail(OMX_E_INVALID, "snapshot rows [" + std::to_string(g_.part_lo) + ", " + std::to_string(g_.part_hi) +
                              ") are not rank " + std::to_string(r) + "'s block of " + std::to_string(W));
    // disconnected patterns: a new root's candidates are every vertex (replicated classes and columns),
    // crossed with the rank's own rows, so the product stays partitioned by those rows. Degree
    // predicates read the gathered degrees (gather_global_degrees, at the start of run()).
    // RETURN expressions read the replicated property columns, but out()/in()/both() inside them read
    // adjacency rows a partition may not hold
    // out()/in()/both() applied to an alias is fetched from the owners before the projection
    // (fetch_return_adjacency); applied to a list or a field its vertices are only known while rank 0
    // evaluates the expression
    if (p_.ret_adj_deep)
      unsupported("out()/in()/both() of a list or a field in a RETURN expression is not supported on a partitioned snapshot");
    const bool limited = p_.limit >= 0 || o_.limit >= 0;
    // optional nodes need nothing more: a row is flagged or checked on the owner of the vertex whose
    // adjacency it reads (a traversal never starts from an optional alias, plan.cpp); RETURN expressions,
    // $elements / $pathElements and LIMIT are evaluated over the content-distinct result as a whole, so
    // the rows of every rank meet on rank 0 first (route_rank0)
    gather0_ = p_.proj != Plan::PROJ_ALIASES || limited;
    dist_ = true;
  }
  bool gather0_ = false;  // partitioned: the final rows go to rank 0 (projection over the whole result)
  bool devproj_ = true;   // OMX_DEVPROJ=0: every RETURN expression through the host evaluator

  // every rank's rows to rank 0 (before a projection that needs the whole result: documents by content,
  // $elements, LIMIT); the other ranks end with no rows
  void route_rank0() {
    owner_col_ = -1;
    if (tr_->world() == 1 && !route_self_) return;
    const int W = tr_->world();
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(R_, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    if (R_) {
      const uint64_t h0 = R_;
      HIP_CHECK(hipMemsetAsync(dest.p, 0, R_ * sizeof(uint32_t), s_));
      HIP_CHECK(hipMemcpyAsync(hist.p, &h0, sizeof(uint64_t), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipStreamSynchronize(s_));  // (h0 is a local)
    }
    route_rows(dest, hist);
    rows_gathered_ = R_;
  }
  uint64_t rows_gathered_ = 0;  // rows this rank received in route_rank0 (omx_result_info.rows_gathered)

  // before the rows meet on rank 0: equal tuples of the projected aliases meet on one rank
  // (hash(tuple) % N) and each rank keeps its distinct ones, so rank 0 receives only distinct tuples;
  // with LIMIT over plain alias rows (a distinct tuple is a distinct result row) a rank sends at most
  // max(LIMIT, 1) of them (addSingleResult :737-750 keeps that many)
  void pre_rank0_distinct() {
    if (p_.out_aliases.empty()) return;
    std::vector<int> al;
    for (int a : p_.out_aliases)
      if (std::find(al.begin(), al.end(), a) == al.end()) al.push_back(a);
    // columns no projection reads do not travel
    for (size_t a = 0; a < col_.size(); ++a)
      if (std::find(al.begin(), al.end(), (int)a) == al.end() && bound_[a]) {
        col_[a].reset();
        bound_[a] = 0;
      }
    if (!p_.unique_by_construction && !marked_) {
      route_hash(al);
      std::vector<DBuf<uint32_t>> cs;
      bool may_null = false;
      for (int a : al) {
        cs.push_back(std::move(col_[a]));
        may_null = may_null || p_.optional[a];
      }
      uint64_t n = R_ ? distinct_rows(cs, (int)al.size(), may_null) : 0;
      for (size_t i = 0; i < al.size(); ++i) col_[al[i]] = std::move(cs[i]);
      R_ = n;
      pre_distinct_ = true;
    }
    const int64_t limit = p_.limit >= 0 ? p_.limit : o_.limit;
    if (limit >= 0 && p_.proj == Plan::PROJ_ALIASES) R_ = std::min<uint64_t>(R_, (uint64_t)std::max<int64_t>(limit, 1));
  }
  bool pre_distinct_ = false;  // pre_rank0_distinct de-duplicated the rows (rank 0 receives disjoint sets)

  // every rank's rows (cols, n of them) to rank 0; returns the rows this rank holds afterwards
  uint64_t to_rank0(const std::vector<DBuf<uint32_t> *> &cols, uint64_t n) {
    const int W = tr_->world();
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(n, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    if (n) {
      HIP_CHECK(hipMemsetAsync(dest.p, 0, n * sizeof(uint32_t), s_));
      HIP_CHECK(hipMemcpyAsync(hist.p, &n, sizeof(uint64_t), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipStreamSynchronize(s_));  // (n is a local)
    }
    return exchange_cols(cols, n, dest, hist);
  }

  // out()/in()/both() applied to an alias in a RETURN expression, on a partitioned snapshot: rank 0
  // (which holds every row after route_rank0) sends the alias's distinct vertices to their owners, each
  // owner answers with their degrees and lists (the ordered expansion: parts in the AdjSpec's order, as
  // OrientVertex.getVertices iterates its fields), and rank 0 keeps them for the document builder. Every
  // rank takes part, in the plan's order of the suffixes.
  void fetch_return_adjacency(RetAdj &out) {
    const int W = tr_->world();
    for (const auto &sa : p_.ret_adj_alias) {
      const AdjSpec &as = p_.ret_adj.at(sa.first);
      // 1. the distinct vertices of the alias (rank 0; nulls skipped)
      uint64_t n = 0;
      DBuf<uint32_t> ids;
      if (R_ && col_[sa.second].p) {
        DBuf<uint64_t> bm(&pool_, std::max<uint64_t>(nwords_, 1));
        HIP_CHECK(hipMemsetAsync(bm.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
        launch_mark_bitmap(col_[sa.second].p, R_, bm.p, g_.V, s_);
        ids = bitmap_list(bm.p, 0, 1, n);
      } else {
        ids = DBuf<uint32_t>(&pool_, 1);
      }
      // 2. to their owners
      DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(n, 1));
      DBuf<uint64_t> hist(&pool_, W);
      HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
      if (n) launch_route_owner(ids.p, n, block_, (uint32_t)W, dest.p, hist.p, s_);
      n = exchange_cols({&ids}, n, dest, hist);
      // 3. the owners' degrees and lists, in id order
      DBuf<uint32_t> dlo(&pool_, std::max<uint64_t>(n, 1)), dhi(&pool_, std::max<uint64_t>(n, 1)), lists;
      uint64_t nl = 0;
      if (n) {
        DBuf<uint64_t> deg(&pool_, n + 1);
        launch_row_degree(ids.p, n, make_adj(as), deg.p, s_);
        launch_u64_split(deg.p, n, dlo.p, dhi.p, s_);
        ExpandOut o = expand_core(ids.p, n, as, nullptr, {}, true, false, nullptr, nullptr, nullptr, nullptr, true);
        nl = o.n;
        lists = nl ? std::move(o.dst) : DBuf<uint32_t>(&pool_, 1);
      } else {
        lists = DBuf<uint32_t>(&pool_, 1);
      }
      // 4. back to rank 0: (vertex, degree) rows, then the lists (both in rank order, then id order)
      n = to_rank0({&ids, &dlo, &dhi}, n);
      nl = to_rank0({&lists}, nl);
      if (tr_->rank() != 0 || n == 0) continue;
      std::vector<uint32_t> hid(n), hlo(n), hhi(n), hl(nl);
      HIP_CHECK(hipMemcpyAsync(hid.data(), ids.p, n * 4, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipMemcpyAsync(hlo.data(), dlo.p, n * 4, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipMemcpyAsync(hhi.data(), dhi.p, n * 4, hipMemcpyDeviceToHost, s_));
      if (nl) HIP_CHECK(hipMemcpyAsync(hl.data(), lists.p, nl * 4, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      uint64_t at = 0;
      for (uint64_t i = 0; i < n; ++i) {
        const uint64_t d = (uint64_t)hlo[i] | (uint64_t)hhi[i] << 32;
        if (at + d > nl) fail(OMX_E_INVALID, "internal: fetched adjacency lists are short");
        out[{sa.first, hid[i]}] = std::vector<uint32_t>(hl.begin() + at, hl.begin() + at + d);
        at += d;
      }
    }
  }

  // (row, vertex) pairs of an item's result sets (see traverse)
  struct PairSet {
    DBuf<uint32_t> row, v;
    uint64_t n = 0;
  };

  // rows travel to dest[r]; hist[p] = rows for rank p (both on the device)
  void route_rows(DBuf<uint32_t> &dest, DBuf<uint64_t> &hist) {
    std::vector<DBuf<uint32_t> *> cs;
    for (int c : bound_cols()) cs.push_back(&col_[c]);
    R_ = exchange_cols(cs, R_, dest, hist);
    segmented_ = false;
  }

  // columns of R rows travel to dest[r] (hist[p] = rows for rank p): a one-pass radix sort by
  // destination, an all-to-all of the counts, an all-to-all-v per column; returns the rows received
  uint64_t exchange_cols(const std::vector<DBuf<uint32_t> *> &cols, uint64_t R, DBuf<uint32_t> &dest,
                         DBuf<uint64_t> &hist) {
    const int W = tr_->world();
    DBuf<uint32_t> perm;
    if (R) {
      DBuf<uint32_t> iota(&pool_, R), sdest(&pool_, R);
      perm = DBuf<uint32_t>(&pool_, R);
      launch_iota(iota.p, R, s_);
      const int bits = std::max(1, bits_for((uint64_t)W - 1));
      cub([&](void *t, size_t &b) {
        return sort_pairs(t, b, dest.p, sdest.p, iota.p, perm.p, R, bits, s_);
      });
    }
    std::vector<uint64_t> send, recv;
    tr_->counts(hist.p, send, recv, s_);
    std::vector<uint64_t> sdispl(W, 0), rdispl(W, 0);
    uint64_t Rn = 0;
    for (int p = 0; p < W; ++p) {
      if (p) sdispl[p] = sdispl[p - 1] + send[p - 1];
      rdispl[p] = Rn;
      Rn += recv[p];
    }
    std::vector<DBuf<uint32_t>> sb, rb;
    std::vector<const uint32_t *> sp;
    std::vector<uint32_t *> rp;
    tm_.begin("k_route_gather");
    for (DBuf<uint32_t> *c : cols) {
      if (R && !c->p) fail(OMX_E_INVALID, "internal: an exchanged column is not materialized");
      sb.emplace_back(&pool_, std::max<uint64_t>(R, 1));
      if (R) launch_gather_u32(c->p, perm.p, R, sb.back().p, s_);
      rb.emplace_back(&pool_, std::max<uint64_t>(Rn, 1));
      sp.push_back(sb.back().p);
      rp.push_back(rb.back().p);
    }
    tm_.end(R * 12ull * cols.size());
    tm_.begin("exchange");
    tr_->alltoallv(sp, send, sdispl, rp, recv, rdispl, s_);
    tm_.end((R + Rn) * 4ull * cols.size());
    for (size_t i = 0; i < cols.size(); ++i) *cols[i] = std::move(rb[i]);
    return Rn;
  }

  // Σ over ranks (a partitioned run's loops must end on every rank at the same level)
  uint64_t global_sum(uint64_t x) {
    if (!dist_) return x;
    uint64_t t = 0;
    for (uint64_t y : tr_->allgather(x, s_)) t += y;
    return t;
  }
  // pairs travel to the owner of their vertex (partitioned: its adjacency is local there)
  void route_pairs_owner(PairSet &p) {
    if (!dist_ || (tr_->world() == 1 && !route_self_)) return;
    const int W = tr_->world();
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(p.n, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    if (p.n) launch_route_owner(p.v.p, p.n, block_, (uint32_t)W, dest.p, hist.p, s_);
    p.n = exchange_cols({&p.row, &p.v}, p.n, dest, hist);
  }

  // before a step that reads column c's adjacency: rows go to the rank that owns row[c]
  void route_owner(int c) {
    if (!dist_ || owner_col_ == c) return;
    owner_col_ = c;
    if (tr_->world() == 1 && !route_self_) return;
    const int W = tr_->world();
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(R_, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    tm_.begin("k_route_owner");
    launch_route_owner(col_[c].p, R_, block_, (uint32_t)W, dest.p, hist.p, s_);
    tm_.end(R_ * 8);
    route_rows(dest, hist);
  }

  // before a distinct projection: rows go to the rank given by a hash of the projected tuple
  void route_hash(const std::vector<int> &aliases) {
    owner_col_ = -1;
    if (tr_->world() == 1 && !route_self_) return;
    const int W = tr_->world();
    std::vector<const uint32_t *> cs;
    for (int a : aliases) cs.push_back(col_[a].p);
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(R_, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    tm_.begin("k_route_hash");
    launch_route_hash((int)cs.size(), cs.data(), R_, (uint32_t)W, dest.p, hist.p, s_);
    tm_.end(R_ * (4ull * cs.size() + 4));
    route_rows(dest, hist);
  }

  // ---- steps -------------------------------------------------------------------------------------
  void root(const Step &st) {
    uint64_t n = 0;
    int world = std::max(1, o_.shard_world);
    // a partition starts the rows of the roots it owns (their adjacency is local)
    col_[st.dst] = bitmap_list(bitmap(st.cand_bm), world > 1 ? o_.shard_rank : 0, world, n, g_.part_lo, g_.part_hi);
    R_ = n;
    bound_[st.dst] = 1;
    owner_col_ = st.dst;
  }

  struct ExpandOut {
    DBuf<uint32_t> dst;
    std::vector<DBuf<uint32_t>> carry;
    uint64_t n = 0;
    uint64_t E = 0;
    uint64_t E_member = 0;  // edges of a fused closing check
    bool counted_from_degrees = false;  // count-only unfiltered hop: no col[] read
    // block-segmented result (filtered expansion left un-compacted)
    bool segmented = false;
    DBuf<uint64_t> seg_start;
    DBuf<uint32_t> seg_count;
    DBuf<uint64_t> seg_offs;  // the segments' dense offsets (their counts' scan)
    uint32_t nseg = 0;
  };

  int cus() {
    if (!cus_) {
      hipDeviceProp_t prop;
      HIP_CHECK(hipGetDeviceProperties(&prop, g_.device));
      cus_ = prop.multiProcessorCount;
    }
    return cus_;
  }

  // the pull tiles' merge-path split of one CSR (built once per CSR: the snapshot is immutable)
  const uint64_t *pull_part_of(int eset, int dir, const uint64_t *rp, uint64_t E, uint64_t ntiles) {
    EdgeSet &es = g_.esets[eset];
    if (!es.d_pull_part[dir]) {  // built into a local buffer, published once complete
      uint64_t *part = nullptr;
      HIP_CHECK(hipMalloc((void **)&part, (ntiles + 1) * sizeof(uint64_t)));
      try {
        launch_bfs_pull_partition(rp, g_.V, E, part, s_);
        HIP_CHECK(hipStreamSynchronize(s_));
      } catch (...) {
        (void)hipFree(part);
        throw;
      }
      es.d_pull_part[dir] = part;
      g_.device_bytes += (ntiles + 1) * sizeof(uint64_t);
    }
    return es.d_pull_part[dir];
  }

  // the in-edge wave tiles of one CSR for k_bfs_pull_w (built once per CSR): tile bounds and the tile
  // indices, regular tiles first (*nreg of them)
  const uint32_t *pullw_of(int eset, int dir, const uint64_t *rp, uint64_t E, const uint64_t **rb, uint64_t *nreg) {
    EdgeSet &es = g_.esets[eset];
    if (!es.d_pullw_tiles[dir]) pullw_build(rp, E, es.d_pullw_rb[dir], es.d_pullw_tiles[dir], es.pullw_nreg[dir]);
    *rb = es.d_pullw_rb[dir];
    *nreg = es.pullw_nreg[dir];
    return es.d_pullw_tiles[dir];
  }
  // wave tiles of one CSR's in-edges: the tile bounds and the tile list, regular tiles first (built into
  // local buffers, published once complete)
  void pullw_build(const uint64_t *rp, uint64_t E, uint64_t *&rb_out, uint32_t *&tiles_out, uint64_t &nreg_out) {
    const uint64_t nt = bfs_pull_w_tiles(E);
    if (nt > 0xFFFFFFFFull) unsupported("a bottom-up level over 2^42 or more in-edges");
    uint64_t *b = nullptr;
    uint32_t *tl = nullptr;
    HIP_CHECK(hipMalloc((void **)&b, std::max<uint64_t>(2 * nt, 1) * sizeof(uint64_t)));
    if (hipMalloc((void **)&tl, std::max<uint64_t>(nt, 1) * sizeof(uint32_t)) != hipSuccess) {
      (void)hipFree(b);
      fail(OMX_E_OOM, "pull tiles");
    }
    uint64_t nr = 0;
    try {
      DBuf<uint8_t> reg(&pool_, std::max<uint64_t>(nt, 1));
      DBuf<uint64_t> cnt(&pool_, 1);
      launch_pull_w_bounds(rp, g_.V, E, b, reg.p, s_);
      hipcub::CountingInputIterator<uint32_t> it(0);
      cub([&](void *t, size_t &bytes) { return hipcub::DevicePartition::Flagged(t, bytes, it, reg.p, tl, cnt.p, (int64_t)nt, s_); });
      nr = read1(cnt.p);
    } catch (...) {
      (void)hipFree(b);
      (void)hipFree(tl);
      throw;
    }
    rb_out = b;
    nreg_out = nr;
    tiles_out = tl;
    g_.device_bytes += nt * 20;
  }

  // the hub entries of a pull col as their own CSR (EdgeSet::d_hub_rp / d_hub_col) and its wave tiles
  struct HubCsr {
    const uint64_t *rp = nullptr;
    const uint32_t *col = nullptr;
    uint64_t E = 0;
    const uint32_t *tiles = nullptr;
    const uint64_t *rb = nullptr;
    uint64_t nreg = 0;
  };
  HubCsr hub_csr_of(int eset, int dir) {
    EdgeSet &es = g_.esets[eset];
    HubCsr h;
    if (!es.d_pull_col[dir]) return h;
    const uint64_t E = dir == 0 ? es.n_edges : es.n_in_edges;
    if (!es.d_hub_col[dir]) {
      // every field is built into locals and published only once all six exist (a throw in the tile
      // build would otherwise leave d_hub_col set with no tiles for the next level to read)
      uint64_t *hrp = nullptr, *wrb = nullptr;
      uint32_t *hcol = nullptr, *wtiles = nullptr;
      uint64_t nh = 0, wnreg = 0;
      try {
        HIP_CHECK(hipMalloc((void **)&hrp, ((uint64_t)g_.V + 1) * 8));
        // excl[e] = hub entries before e (u32 when E < 2^32), then hub_rp[v] = excl[rp[v]]
        DBuf<uint64_t> ex(&pool_, E + 1);
        HIP_CHECK(hipMemsetAsync(ex.p, 0, 8, s_));
        hipcub::TransformInputIterator<uint64_t, HubFlag, const uint32_t *> fl(es.d_pull_col[dir], HubFlag());
        if (E) cub([&](void *t, size_t &b) { return hipcub::DeviceScan::InclusiveSum(t, b, fl, ex.p + 1, (int64_t)E, s_); });
        launch_gather_u64_at(ex.p, g_.rp(es, dir), (uint64_t)g_.V + 1, hrp, s_);
        nh = read1(ex.p + E);
        HIP_CHECK(hipMalloc((void **)&hcol, std::max<uint64_t>(nh, 1) * 4));
        DBuf<uint64_t> nsel(&pool_, 1);
        hipcub::TransformInputIterator<uint8_t, HubFlag8, const uint32_t *> f8(es.d_pull_col[dir], HubFlag8());
        if (E) cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, es.d_pull_col[dir], f8, hcol, nsel.p, (int64_t)E, s_); });
        HIP_CHECK(hipStreamSynchronize(s_));
        pullw_build(hrp, nh, wrb, wtiles, wnreg);
      } catch (...) {
        if (hrp) (void)hipFree(hrp);
        if (hcol) (void)hipFree(hcol);
        throw;
      }
      es.d_hub_rp[dir] = hrp;
      es.d_hub_col[dir] = hcol;
      es.hub_entries[dir] = nh;
      es.d_hubw_rb[dir] = wrb;
      es.d_hubw_tiles[dir] = wtiles;
      es.hubw_nreg[dir] = wnreg;
      g_.device_bytes += ((uint64_t)g_.V + 1) * 8 + nh * 4;
    }
    h.rp = es.d_hub_rp[dir];
    h.col = es.d_hub_col[dir];
    h.E = es.hub_entries[dir];
    h.tiles = es.d_hubw_tiles[dir];
    h.rb = es.d_hubw_rb[dir];
    h.nreg = es.hubw_nreg[dir];
    return h;
  }

  // the hub-annotated col of one CSR for the bottom-up BFS (built once per CSR, bfs.hip)
  const uint32_t *pull_col_of(int eset, int dir, uint32_t *nhubs, const uint32_t **hubs,
                              const uint64_t **hub_bm = nullptr) {
    EdgeSet &es = g_.esets[eset];
    *nhubs = 0;
    *hubs = nullptr;
    if (hub_bm) *hub_bm = nullptr;
    // k_bfs_pull reads bit 31 of a col entry as the hub tag: vertex ids must stay below 2^31
    if (g_.V >= 0x80000000u) unsupported("variable-length traversal over 2^31 or more vertices");
    if (pull_hubs_ == 0 || g_.partitioned()) return g_.col(es, dir);
    if (es.d_pull_col[dir] && es.hubs_requested[dir] != pull_hubs_) {  // another hub budget (OMX_PULL_HUBS)
      HIP_CHECK(hipStreamSynchronize(s_));
      (void)hipFree(es.d_pull_col[dir]);
      (void)hipFree(es.d_hubs[dir]);
      if (es.d_hub_bm[dir]) (void)hipFree(es.d_hub_bm[dir]);
      for (void *x : {(void *)es.d_hub_rp[dir], (void *)es.d_hub_col[dir], (void *)es.d_hubw_rb[dir], (void *)es.d_hubw_tiles[dir]})
        if (x) (void)hipFree(x);
      es.d_pull_col[dir] = nullptr;
      es.d_hubs[dir] = nullptr;
      es.d_hub_bm[dir] = nullptr;
      es.d_hub_rp[dir] = nullptr;
      es.d_hub_col[dir] = nullptr;
      es.d_hubw_rb[dir] = nullptr;
      es.d_hubw_tiles[dir] = nullptr;
    }
    if (!es.d_pull_col[dir]) {  // built into local buffers, published once complete
      const uint64_t E = dir == 0 ? es.n_edges : es.n_in_edges;
      uint32_t *pcol = nullptr, *hubs = nullptr, nh = 0;
      uint64_t *hbm = nullptr;
      try {
        HIP_CHECK(hipMalloc((void **)&pcol, std::max<size_t>(E * 4, 4)));
        HIP_CHECK(hipMalloc((void **)&hubs, std::max<size_t>((size_t)pull_hubs_ * 4, 4)));
        HIP_CHECK(hipMalloc((void **)&hbm, std::max<size_t>(nwords_ * 8, 8)));
        DBuf<uint32_t> hub_idx(&pool_, g_.V), hist(&pool_, 4096);
        DBuf<unsigned long long> cnt(&pool_, 1);
        nh = build_pull_col(g_.rp(es, dir), g_.rp(es, dir ^ 1), g_.col(es, dir), g_.V, E, pull_hubs_, hub_idx.p, hist.p,
                            cnt.p, hubs, pcol, cus(), s_);
        HIP_CHECK(hipMemsetAsync(hbm, 0, std::max<size_t>(nwords_ * 8, 8), s_));
        if (nh) launch_mark_bitmap(hubs, nh, hbm, g_.V, s_);
        HIP_CHECK(hipStreamSynchronize(s_));
      } catch (...) {
        if (pcol) (void)hipFree(pcol);
        if (hubs) (void)hipFree(hubs);
        if (hbm) (void)hipFree(hbm);
        throw;
      }
      es.d_pull_col[dir] = pcol;
      es.d_hubs[dir] = hubs;
      es.d_hub_bm[dir] = hbm;
      g_.device_bytes += nwords_ * 8;
      es.n_hubs[dir] = nh;
      es.hubs_requested[dir] = pull_hubs_;
      g_.device_bytes += E * 4 + (uint64_t)pull_hubs_ * 4;
    }
    *nhubs = es.n_hubs[dir];
    *hubs = es.d_hubs[dir];
    if (hub_bm) *hub_bm = es.d_hub_bm[dir];
    return es.d_pull_col[dir];
  }

  // the lists col of one CSR for the filtered lists (k_flists): the kFlistHubs vertices of highest degree
  // in the opposite CSR are hubs, entered as vb + rank (built once per CSR, into locals, published when
  // complete)
  const uint32_t *list_col_of(int eset, int dir, uint32_t *nhubs, const uint32_t **hubs, uint32_t *vb) {
    EdgeSet &es = g_.esets[eset];
    if (!es.d_list_col[dir]) {
      const uint64_t E = dir == 0 ? es.n_edges : es.n_in_edges;
      uint32_t *lcol = nullptr, *lh = nullptr, nh = 0;
      // the cached col stays for the snapshot's lifetime: built only when it and a pass's scratch over
      // every entry (lcol + survivors, 8 B an entry) leave 1 GiB of the device free (OMX_E_OOM otherwise:
      // the caller takes the binned lists)
      size_t free_b = 0, total_b = 0;
      HIP_CHECK(hipMemGetInfo(&free_b, &total_b));
      if ((uint64_t)free_b + pool_.cached_bytes() < (E + 4) * 4 + 8 * E + (1ull << 30))
        fail(OMX_E_OOM, "no room for the lists col of a " + std::to_string(E) + "-entry CSR");
      try {
        // padded: the lists kernel reads whole aligned 16-byte groups
        if (hipMalloc((void **)&lcol, (E + 4) * 4) != hipSuccess || hipMalloc((void **)&lh, (size_t)kFlistHubs * 4) != hipSuccess) {
          (void)hipGetLastError();
          fail(OMX_E_OOM, "device allocation of the lists col failed");
        }
        DBuf<uint32_t> hub_idx(&pool_, g_.V), hist(&pool_, 4096);
        DBuf<unsigned long long> cnt(&pool_, 1);
        const uint64_t *rp_self = g_.rp(es, dir), *rp_other = g_.rp(es, dir ^ 1);
        DBuf<uint64_t> full, occ_rp;
        if (g_.partitioned()) {
          // a partition holds its own rows only: the rows as V + 1 global row pointers, and hubs ranked
          // by how often the rank's own col names them (the opposite CSR's rows of other ranks are absent)
          const uint64_t V1 = (uint64_t)g_.V + 1;
          full = DBuf<uint64_t>(&pool_, V1);
          occ_rp = DBuf<uint64_t>(&pool_, V1);
          DBuf<uint32_t> occ(&pool_, V1);
          hipLaunchKernelGGL(k_full_rp, dim3((unsigned)((V1 + 255) / 256)), dim3(256), 0, s_,
                             dir == 0 ? es.d_out_rp : es.d_in_rp, g_.part_lo, g_.part_hi, g_.V, full.p);
          HIP_CHECK(hipMemsetAsync(occ.p, 0, V1 * 4, s_));
          if (E) hipLaunchKernelGGL(k_col_occurrences, dim3((unsigned)std::min<uint64_t>((E + 255) / 256, 16ull * cus())), dim3(256), 0, s_,
                                    g_.col(es, dir), E, occ.p);
          hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> it(occ.p, CastU64());
          cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, it, occ_rp.p, (int64_t)V1, s_); });
          HIP_CHECK(hipStreamSynchronize(s_));
          rp_self = full.p;
          rp_other = occ_rp.p;
        }
        nh = build_pull_col(rp_self, rp_other, g_.col(es, dir), g_.V, E, kFlistHubs, hub_idx.p, hist.p, cnt.p, lh,
                            lcol, cus(), s_);
        launch_list_col(lcol, E, (uint32_t)(nwords_ * 64), s_);
        HIP_CHECK(hipStreamSynchronize(s_));
      } catch (...) {
        if (lcol) (void)hipFree(lcol);
        if (lh) (void)hipFree(lh);
        throw;
      }
      es.d_list_col[dir] = lcol;
      es.d_list_hubs[dir] = lh;
      es.n_list_hubs[dir] = nh;
      es.list_vb[dir] = (uint32_t)(nwords_ * 64);
      g_.device_bytes += E * 4 + (uint64_t)kFlistHubs * 4;
    }
    *vb = es.list_vb[dir];
    *nhubs = es.n_list_hubs[dir];
    *hubs = es.d_list_hubs[dir];
    return es.d_list_col[dir];
  }

  // the filtered lists L(u) of the U distinct sources ub (doff: the scan of their degrees, EU = doff[U])
  // as a CSR (loff[U+1], lcol) through k_flists; the list entries stay on the device (loff[U]): lcol is
  // sized for all EU, so no host round trip
  // (pre_coff / pre_info: the sources' chunk offsets and chunk table entries from launch_srcrows)
  void filtered_lists(const uint32_t *ub, uint64_t U, const uint64_t *doff, uint64_t EU, const AdjSpec &adjs,
                      const uint64_t *filter, DBuf<uint64_t> &loff, DBuf<uint32_t> &lcol,
                      const uint64_t *pre_coff = nullptr, const uint4 *pre_info = nullptr) {
    const int es = adjs.parts[0].first, dir = adjs.parts[0].second;
    uint32_t nh = 0;
    const uint32_t *hubs = nullptr;
    uint32_t vb = 0;
    const uint32_t *acol = list_col_of(es, dir, &nh, &hubs, &vb);
    if ((uint64_t)vb != nwords_ * 64) fail(OMX_E_INVALID, "internal: lists col built for another filter width");
    const uint64_t *rp = g_.rp(g_.esets[es], dir);
    // the chunk space: every source's row as aligned 4-entry chunks of the col, in source order
    const uint64_t ntb = flist_tiles_bound(EU, U);
    DBuf<uint64_t> coffb, rb(&pool_, 2 * ntb), base(&pool_, ntb + 1);
    DBuf<uint4> infob;
    const uint64_t *coff = pre_coff;
    const uint4 *info = pre_info;
    if (!pre_coff) {
      DBuf<uint32_t> nch(&pool_, U + 1);
      coffb = DBuf<uint64_t>(&pool_, U + 1);
      launch_flist_nch(ub, doff, U, rp, nch.p, s_);  // (nch[U] = 0 included)
      hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> it(nch.p, CastU64());
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, it, coffb.p, (int64_t)(U + 1), s_); });
      infob = DBuf<uint4>(&pool_, std::max<uint64_t>(U, 1));
      coff = coffb.p;
      info = infob.p;
    }
    DBuf<uint32_t> ntot(&pool_, ntb + 1);
    // (ntot past the tiles zeroed)
    launch_flist_prep(ub, doff, coff, U, rp, coff + U, pre_coff ? nullptr : infob.p, rb.p, ntot.p, ntb, s_);
    const uint64_t nbits = vb / 32 + (nh + 31) / 32;
    DBuf<uint32_t> bits(&pool_, nbits), loc(&pool_, std::max<uint64_t>(U, 1));
    DBuf<uint32_t> scratch(&pool_, ntb * flist_tile_entries());
    launch_probe_bits(hubs, nh, filter, vb, bits.p, s_);
    FlistArgs a{};
    a.ub = ub;
    a.U = U;
    a.info = info;
    a.ec = coff + U;
    a.acol = acol;
    a.E = dir == 0 ? g_.esets[es].n_edges : g_.esets[es].n_in_edges;
    a.hubs = hubs;
    a.nh = nh;
    a.vb = vb;
    a.bits = bits.p;
    a.bbytes = nbits * 4;
    a.rb = rb.p;
    a.scratch = scratch.p;
    a.ntot = ntot.p;
    a.loc = loc.p;
    tm_.begin("k_flists");
    launch_flist(a, ntb, cus(), s_);
    tm_.end(4ull * EU + 16ull * U);
    {
      hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> it(ntot.p, CastU64());
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, it, base.p, (int64_t)(ntb + 1), s_); });
    }
    lcol = DBuf<uint32_t>(&pool_, std::max<uint64_t>(EU, 1));
    loff = DBuf<uint64_t>(&pool_, U + 1);
    a.lcol = lcol.p;
    tm_.begin("k_flist_copy");
    launch_flist_finish(a, coff, base.p, loff.p, ntb, cus(), s_);
    tm_.end(16ull * U);  // (+ 8 bytes a list entry: amended when the count is read)
    flist_copy_rec_ = tm_.last();
  }

  // the slice-cut index of every part of an adjacency (built once per CSR and slice size)
  DCuts slice_cuts_of(const AdjSpec &adjs, uint32_t P) {
    DCuts c{};
    if (P < 2) return c;
    for (size_t i = 0; i < adjs.parts.size(); ++i) {
      EdgeSet &es = g_.esets[adjs.parts[i].first];
      const int dir = adjs.parts[i].second;
      uint32_t *&d = es.d_cuts[dir][slice_shift_];
      if (!d) {
        const size_t bytes = (size_t)g_.V * (P - 1) * sizeof(uint32_t);
        HIP_CHECK(hipMalloc((void **)&d, std::max<size_t>(bytes, 4)));
        g_.device_bytes += bytes;
        launch_build_cuts(g_.rp(es, dir), g_.col(es, dir), g_.part_lo, g_.part_hi, P, slice_shift_, d, s_);
      }
      c.c[i] = d;
    }
    return c;
  }

  // One pattern-edge expansion of R rows (src column) with an optional target bitmap, carrying the
  // listed columns. write=false only counts. allow_segmented leaves a filtered result as per-block
  // segments (the final step of a plan whose rows are distinct by construction).
  // member_src/member_adj: fused closing check (ExpandArgs::member_src); the edges it stands for are
  // returned in ExpandOut::E_member.
  // raw_adj: an adjacency that is not a snapshot CSR (the factorized expansion's grouped lists)
  ExpandOut expand_core(const uint32_t *src, uint64_t R, const AdjSpec &adjs, const uint64_t *filter,
                        const std::vector<const uint32_t *> &carry, bool write, bool allow_segmented = false,
                        const uint32_t *member_src = nullptr, const AdjSpec *member_adj = nullptr,
                        const uint64_t *member_filter = nullptr, const DAdj *raw_adj = nullptr, bool ordered = false,
                        uint64_t *mark = nullptr) {
    ExpandOut o;
    if (mark && (write || filter || member_src || ordered))
      fail(OMX_E_INVALID, "internal: a marking expansion is unfiltered and writes no rows");
    DAdj adj = raw_adj ? *raw_adj : make_adj(adjs);
    if (adj.n == 0 || R == 0) return o;
    const bool member = member_src != nullptr;
    DBuf<unsigned long long> medges;
    if (member) {
      medges = DBuf<unsigned long long>(&pool_, 2);
      HIP_CHECK(hipMemsetAsync(medges.p, 0, 2 * sizeof(unsigned long long), s_));
    }
    if (!write && filter == nullptr && !member && !mark && !ordered) {
      // counting an unfiltered hop: its bindings are Σ degree — a degree reduction, no binning and no
      // col[] reads (C5's last hop over 7 M rows: 0.33 ms of binning count + scan before, round 5;
      // omx_result_info.edges_read excludes these edges)
      o.E = o.n = degree_sum(src, R, adjs, raw_adj);
      o.counted_from_degrees = true;
      alg_bytes_ += 8 * R;
      return o;
    }
    // 1. degree binning + scans (light edges: merge path; heavy rows: chunks). A filtered hop over a
    // sorted adjacency cuts the heavy rows' chunks at bitmap-slice boundaries (LDS-sliced kernel).
    const bool sliced = filter != nullptr && !member && !raw_adj && !ordered && adj.sorted && sliced_ &&
                        (uint64_t)g_.V <= ((uint64_t)kMaxSlices << slice_shift_);
    const uint32_t P = sliced ? (uint32_t)(((uint64_t)g_.V + (1ull << slice_shift_) - 1) >> slice_shift_) : 1;
    const DCuts cuts = sliced ? slice_cuts_of(adjs, P) : DCuts{};
    // the sliced kernels stage whole bitmap slices with unchecked loads: the filter must be padded
    if (sliced && pool_.size_of(filter) < padded_words() * 8)
      fail(OMX_E_INVALID, "internal: a sliced expansion's filter bitmap is not padded to whole slices");
    // sliced: a heavy row is cut into P pieces, one chunk each; below ~128 edges per piece a chunk issues
    // its 16 loads for a few live slots, so the cut grows with P (RMAT-24, P = 16: 2048 measured best of
    // 256…4096, profiles/r02/hd_sweep; RMAT-22, P = 4: 512 against 256, 1.80 against 1.83 ms per step)
    // ordered (TRAVERSE / SELECT expand): every row through the merge-path kernel, whose dense output is
    // in row order (the heavy kernel's rows would come first); filtered, one tile per block (below)
    const uint64_t hd = ordered ? UINT64_MAX
                        : (!filter && !member && (!heavy_deg_fixed_ || heavy_deg_unfiltered_set_)) ? heavy_deg_unfiltered_
                        : !sliced ? heavy_deg_
                        : heavy_deg_fixed_ ? heavy_deg_sliced_
                                           : std::max<uint64_t>(heavy_deg_sliced_, 128ull * P);
    if (ordered && member) fail(OMX_E_INVALID, "internal: an ordered expansion has no fused check");
    // per-tile sums → one-workgroup scan (posts the totals to the host) → per-tile offsets and chunks
    // (qb: the P + 1 chunk bounds, then the keys' totals of the per-key scan, launch_bin_scan)
    DBuf<uint64_t> blk(&pool_, (uint64_t)(kBinKeys + P) * bin_tiles(R)), qb(&pool_, 2ull * P + 1 + kBinKeys);
    // a sliced hop that writes rows sizes its arenas from the target bitmap's density per slice
    // (posted with the binning totals); an arena found short re-runs the hop with the exact bound
    const bool estimate = sliced && write;
    DBuf<unsigned long long> spop;
    if (estimate) {
      spop = DBuf<unsigned long long>(&pool_, P);
      launch_slice_popc(filter, g_.V, slice_shift_, P, spop.p, s_);
    }
    // unfiltered writes may cut heavy rows into other aligned windows (OMX_UNF_CHUNK: 256, 512, 1024, 2048)
    const uint32_t cs = (!filter && !member && write && !sliced) ? unf_chunk_shift_ : 10u;
    tm_.begin("k_bin_rows");
    launch_bin_count(sliced, src, R, adj, cuts, hd, P, blk.p, s_, cs);
    launch_bin_scan(blk.p, R, P, qb.p, mail(), s_, spop.p, estimate ? P : 0);
    const uint64_t *m = wait_mail();
    const uint64_t EL = m[0], EH = m[1], nchunks = m[2], NL = m[3];
    std::vector<uint64_t> hqb(m + 4, m + 5 + P);
    std::vector<double> dens(P, 1.0);  // fraction of each slice's vertices the target bitmap holds
    if (estimate)
      for (uint32_t q = 0; q < P; ++q) {
        const uint64_t lo = (uint64_t)q << slice_shift_, hi = std::min<uint64_t>(g_.V, (uint64_t)(q + 1) << slice_shift_);
        dens[q] = hi > lo ? std::min(1.0, (double)m[5 + P + q] / (double)(hi - lo)) : 0.0;
      }
    tm_.end(R * (4 + 16ull * adj.n + (sliced ? 4ull * (P - 1) * adj.n : 0)));
    const uint64_t E = EL + EH;
    o.E = E;
    if (E == 0) return o;
    if (!write && filter == nullptr && !member && !mark) {
      // counting an unfiltered hop: its bindings are Σ degree, known from the scan — no col[] reads
      // (reported apart: omx_result_info.edges_read excludes these edges)
      o.n = E;
      o.counted_from_degrees = true;
      alg_bytes_ += 8 * R;
      return o;
    }
    DBuf<ChunkDesc> chunks;
    DBuf<SliceChunk> schunks;
    if (sliced) schunks = DBuf<SliceChunk>(&pool_, std::max<uint64_t>(nchunks, 1));
    else chunks = DBuf<ChunkDesc>(&pool_, std::max<uint64_t>(nchunks, 1));
    tm_.begin("k_bin_fill");
    // light rows of a sliced single-part hop: the LDS-sliced light kernel over the compacted light rows
    // (no merge-path partition); otherwise light data indexed by row for the merge-path kernel
    const bool lsliced = sliced && adj.n == 1 && light_sliced_ && EL > 0;
    DBuf<uint64_t> loffs(&pool_, (lsliced ? NL : R) + 1), lbase;
    DBuf<uint32_t> lrow, lcuts;
    std::vector<DBuf<uint32_t>> lcarry;
    LightRows lr{};
    if (lsliced) {
      lbase = DBuf<uint64_t>(&pool_, NL);
      lrow = DBuf<uint32_t>(&pool_, NL);
      if (P > 1) lcuts = DBuf<uint32_t>(&pool_, (uint64_t)(P - 1) * NL);
      lr = LightRows{lrow.p, lcuts.p, NL, 0, {}, {}};
      if (write && carry.size() <= 4) {
        lr.nc = (int)carry.size();
        for (size_t c = 0; c < carry.size(); ++c) {
          lcarry.emplace_back(&pool_, NL);
          lr.cin[c] = carry[c];
          lr.carry[c] = lcarry.back().p;
        }
      }
    } else if (adj.n == 1) {
      lbase = DBuf<uint64_t>(&pool_, R);
    }
    launch_bin_fill(sliced, src, R, adj, cuts, hd, P, blk.p, qb.p, loffs.p, lbase.p, lr, chunks.p, schunks.p, s_, cs);
    tm_.end(R * (4 + 16ull * adj.n + 8 + (adj.n == 1 ? 8 : 0)) +
            nchunks * (sliced ? sizeof(SliceChunk) : sizeof(ChunkDesc)));
    const uint64_t ntiles = EL && !lsliced ? (R + EL + kExpandTile - 1) / kExpandTile : 0;
    DBuf<uint64_t> part;
    if (ntiles) {
      part = DBuf<uint64_t>(&pool_, ntiles + 1);
      tm_.begin("k_mp_partition");
      launch_mp_partition(loffs.p, R, EL, ntiles, part.p, s_);
      tm_.end((ntiles + 1) * 8 * 20);
    }
    // 2. persistent grids and output placement
    const bool single = adj.n == 1, filt = filter != nullptr || member;
    // heavy kernel: a worker is a wave (4 per block); light kernel: a worker is a block
    constexpr unsigned WPB = kHeavyBlock / 64;
    const uint64_t hblocks = (nchunks + WPB - 1) / WPB;
    // persistent grids: every resident slot. (Running the two kernels side by side on split grids
    // was measured slower: the light kernel is latency-bound per tile and needs the whole chip.)
    const uint64_t sh = (uint64_t)cus() * expand_blocks_per_cu(true, single, filt, write, member, cs);
    const uint64_t sl = (uint64_t)cus() * expand_blocks_per_cu(false, single, filt, write, member);
    constexpr unsigned SWPB = kSliceBlock / 64;
    // sliced: one workgroup per CU, split over the slices in proportion to their chunk counts
    SliceArgs sa{};
    uint64_t caph_sliced = 0;
    double caph_est = 0;  // expected rows of the fullest heavy wave (estimate mode)
    if (sliced && nchunks) {
      const uint64_t G = std::min<uint64_t>((uint64_t)cus(), (nchunks + SWPB - 1) / SWPB);
      sa.qb = qb.p;
      sa.V = g_.V;
      sa.nslices = P;
      sa.shift = slice_shift_;
      uint32_t w = 0;
      for (uint32_t q = 0; q < P; ++q) {
        const uint64_t nq = hqb[q + 1] - hqb[q];
        uint64_t k = nq ? std::max<uint64_t>(1, (G * nq + nchunks / 2) / nchunks) : 0;
        k = std::min<uint64_t>(k, (nq + SWPB - 1) / SWPB);
        sa.wg0[q] = w;
        w += (uint32_t)k;
        // + a 64-row tail pad (k_expand_heavy_sliced may write one dropped row past a wave's count)
        if (k) {
          const uint64_t cpw = (nq + k * SWPB - 1) / (k * SWPB);  // chunks of the fullest wave of slice q
          caph_sliced = std::max<uint64_t>(caph_sliced, cpw * (uint64_t)kChunk + 64);
          caph_est = std::max(caph_est, (double)cpw * ((double)EH / (double)nchunks) * dens[q]);
        }
      }
      sa.wg0[P] = w;
    }
    const unsigned gh = !nchunks ? 0 : sliced ? sa.wg0[P] : (unsigned)std::min<uint64_t>(hblocks, sh);
    // ordered + filtered: one merge-path tile per block, so the per-block segments are in entry order
    const unsigned gl = ntiles ? (unsigned)std::min<uint64_t>(ntiles, ordered && filt ? ntiles : sl) : 0;
    if (ordered && filt && ntiles > 0x7FFFFFFFull) unsupported("an ordered filtered expansion of 2^31 or more tiles");
    // sliced light kernel: one workgroup per CU, split evenly over the slices (light edges spread
    // over V like the heavy ones); a wave's arena holds its share of EL plus one 64-row group
    SliceArgs la{};
    unsigned gls = 0;
    uint64_t capls = 0;
    if (lsliced) {
      const uint32_t G = std::max<uint32_t>((uint32_t)cus(), P);
      uint32_t w = 0, kmin = UINT32_MAX;
      for (uint32_t q = 0; q < P; ++q) {
        const uint32_t k = G / P + (q < G % P ? 1u : 0u);
        la.wg0[q] = w;
        w += k;
        kmin = std::min(kmin, k);
      }
      la.wg0[P] = w;
      la.V = g_.V;
      la.nslices = P;
      la.shift = slice_shift_;
      la.lrow = lrow.p;
      la.lcuts = lcuts.p;
      for (int c = 0; c < lr.nc; ++c) la.lcarry[c] = lr.carry[c];
      la.nl = NL;
      gls = w;
      const uint64_t wmin = (uint64_t)kmin * SWPB;
      capls = (EL + wmin - 1) / wmin + 64 * hd;
    }
    const uint64_t lw = lsliced ? (uint64_t)gls * SWPB : gl;  // light workers (output segments)
    if (debug_expand_)
      std::fprintf(stderr, "[omx expand] R=%llu EL=%llu EH=%llu chunks=%llu P=%u ntiles=%llu gl=%u gls=%u gh=%u filt=%d\n",
                   (unsigned long long)R, (unsigned long long)EL, (unsigned long long)EH,
                   (unsigned long long)nchunks, P, (unsigned long long)ntiles, gl, gls, gh, (int)filt);
    // heavy output: one arena per wave, sized for the most chunks a wave of the launch owns
    const uint64_t wh = (uint64_t)gh * (sliced ? SWPB : WPB);
    const uint64_t caph_exact = !gh ? 0 : sliced ? caph_sliced : (nchunks + wh - 1) / wh * (1ull << cs);
    const uint64_t nseg_h = wh;
    const uint64_t capl_exact = lsliced ? capls : gl ? (ntiles + gl - 1) / gl * (uint64_t)kExpandTile : 0;
    double capl_est = 0;
    if (lsliced) {
      double dmax = 0;
      for (double d : dens) dmax = std::max(dmax, d);
      capl_est = (double)(capls - 64 * hd) * dmax;
    }
    // estimated arenas: 25 % over the expected rows plus 4096 (binomial spread of a wave's survivors)
    const double margin = arena_margin_;
    auto est_cap = [margin](double expect, uint64_t exact) {
      return std::min<uint64_t>(exact, (uint64_t)(expect * margin) + (margin > 0 ? 4096 : 0));
    };
    ExpandArgs a{};
    a.src = src;
    a.offs = loffs.p;
    a.lbase = lbase.p;
    a.part = part.p;
    a.R = R;
    a.E = EL;
    a.ntiles = ntiles;
    a.adj = adj;
    a.filter = filter;
    a.ncarry = (int32_t)carry.size();
    a.chunks = chunks.p;
    a.schunks = schunks.p;
    a.nchunks = nchunks;
    a.chunk_shift = cs;
    a.mark = mark;
    a.dense_base = EH;
    if (member) {
      a.member_src = member_src;
      a.member_adj = make_adj(*member_adj);
      a.member_filter = member_filter;
      a.member_edges = medges.p;
    }
    std::vector<DBuf<uint32_t>> outc;
    DBuf<uint32_t> odst;
    DBuf<uint64_t> soffs;
    if (filt) {
      o.nseg = (uint32_t)(nseg_h + lw);
      soffs = DBuf<uint64_t>(&pool_, o.nseg + 1);
      o.seg_start = DBuf<uint64_t>(&pool_, o.nseg);
      o.seg_count = DBuf<uint32_t>(&pool_, o.nseg);
      a.seg_start = o.seg_start.p;
      a.seg_count = o.seg_count.p;
    }
    // algorithmic bytes: 8 B row_ptr pair per row + 4 B col per edge (+ 4 B × columns
    // per emitted row, added below)
    uint64_t kb = 8 * R + 4 * E;
    // per-kernel algorithmic bytes (amended below once the emitted rows are known): heavy = 4·EH + out,
    // light = 8·R + 4·EL + out, out = 4 B × written columns × rows the kernel emitted
    const uint64_t outw = write ? 4ull * (carry.size() + 1) : 0;
    size_t rec_h = SIZE_MAX, rec_l = SIZE_MAX;
    uint64_t caph = caph_exact, capl = capl_exact, heavy_rows_cap = 0;
    const uint64_t *mt = nullptr;
    for (int attempt = 0;; ++attempt) {
      const bool est = estimate && attempt == 0;
      caph = est ? est_cap(caph_est, caph_exact) : caph_exact;
      capl = est && lsliced ? est_cap(capl_est, capl_exact) : capl_exact;
      heavy_rows_cap = wh * caph;
      const uint64_t cap = filt ? heavy_rows_cap + lw * capl : E;
      if (write) {
        odst = DBuf<uint32_t>(&pool_, std::max<uint64_t>(cap, 1));
        a.out_dst = odst.p;
        outc.clear();
        for (size_t c = 0; c < carry.size(); ++c) {
          outc.emplace_back(&pool_, std::max<uint64_t>(cap, 1));
          a.carry_in[c] = carry[c];
          a.carry_out[c] = outc.back().p;
        }
      }
      if (gh) {
        a.arena_base = 0;
        a.arena_cap = caph;
        a.seg_base = 0;
        if (sliced) {
          tm_.begin("k_expand_heavy_sliced");
          launch_expand_heavy_sliced(a, sa, gh, write, s_);
        } else {
          tm_.begin(member ? "k_expand_heavy_check" : "k_expand_heavy");
          launch_expand_heavy(a, gh, write, s_);
        }
        tm_.end(4 * EH + outw * (filt ? 0 : EH));
        rec_h = tm_.last();
      }
      if (gl || gls) {
        a.arena_base = heavy_rows_cap;
        a.arena_cap = capl;
        a.seg_base = (uint32_t)nseg_h;
        tm_.begin(lsliced ? "k_expand_light_sliced" : member ? "k_expand_light_check" : "k_expand_light");
        if (lsliced) launch_expand_light_sliced(a, la, gls, write, s_);
        else launch_expand(a, gl, write, s_);
        tm_.end(8 * R + 4 * EL + outw * (filt ? 0 : EL));
        rec_l = tm_.last();
      }
      if (!filt) break;
      // rows per block segment → total (and dense compaction when required); segment offsets + rows
      // emitted by the heavy kernel's segments, all rows, member words, arena overflow: one workgroup,
      // one host read
      launch_seg_totals(o.seg_count.p, o.nseg, nseg_h, soffs.p, member ? medges.p : nullptr,
                        gh ? caph : UINT64_MAX, (gl || gls) ? capl : UINT64_MAX, mail(), s_);
      mt = wait_mail();
      if (!mt[4]) break;
      if (!est) fail(OMX_E_INVALID, "internal: an exact expansion arena overflowed");
      ++arena_retries_;
      if (debug_expand_) std::fprintf(stderr, "[omx expand] estimated arena short: re-running with exact caps\n");
    }
    tm_.begin("expand_total");
    if (!filt) {
      o.n = E;
      if (write) kb += 4ull * (carry.size() + 1) * E;
      tm_.end(kb);
      alg_bytes_ += kb;
      if (write) {
        o.dst = std::move(odst);
        o.carry = std::move(outc);
      }
      return o;
    }
    // filtered: rows per block segment (mt: the seg-totals mail of the final attempt)
    const uint64_t nh_n[3] = {mt[0], mt[1], mt[2]};
    const uint64_t probes = mt[3];  // col[] probes of a fused closing check (4 B each, §8(d))
    o.E_member = nh_n[2];
    if (debug_expand_)
      std::fprintf(stderr, "[omx expand] rows out=%llu (heavy %llu) member edges=%llu probes=%llu\n",
                   (unsigned long long)nh_n[1], (unsigned long long)nh_n[0], (unsigned long long)nh_n[2],
                   (unsigned long long)mt[3]);
    const uint64_t n = nh_n[1];
    // the probes are split between the kernels in proportion to their edges (one counter for both)
    const uint64_t ph = E ? (uint64_t)((double)probes * (double)EH / (double)E) : 0;
    if (rec_h != SIZE_MAX) tm_.amend_at(rec_h, 4 * EH + outw * nh_n[0] + 4 * ph);
    if (rec_l != SIZE_MAX) tm_.amend_at(rec_l, 8 * R + 4 * EL + outw * (n - nh_n[0]) + 4 * (probes - ph));
    kb += 4 * probes;
    o.n = n;
    if (write) kb += 4ull * (carry.size() + 1) * n;
    tm_.end(kb);
    alg_bytes_ += kb;
    if (!write || n == 0) return o;
    if (allow_segmented) {
      o.segmented = true;
      o.dst = std::move(odst);
      o.carry = std::move(outc);
      o.seg_offs = std::move(soffs);
      return o;
    }
    o.dst = DBuf<uint32_t>(&pool_, n);
    std::vector<uint32_t *> ins{odst.p}, outs{o.dst.p};
    for (size_t c = 0; c < carry.size(); ++c) {
      o.carry.emplace_back(&pool_, n);
      ins.push_back(outc[c].p);
      outs.push_back(o.carry.back().p);
    }
    tm_.begin("k_compact_segments");
    launch_compact_segments((int)ins.size(), ins.data(), outs.data(), o.seg_start.p, o.seg_count.p, soffs.p, o.nseg, s_);
    tm_.end(8ull * ins.size() * n);
    return o;
  }

  // fused: the following S_CHECK closes a cycle on this step's new column (sorted-
  // adjacency intersection instead of materialising the wedges and probing each)
  void expand_step(const Step &st, bool write, bool allow_segmented, const Step *check = nullptr) {
    if (check && isect_ok(st, *check)) {
      expand_check_isect(st, *check, write);
      return;
    }
    if (check && swap_ok(st, *check)) {
      expand_check_swapped(st, *check, write);
      return;
    }
    route_owner(st.src);
    // optional target: rows whose traversal returns nothing continue with the target null (dense id V);
    // taken before the expansion replaces the columns (P/OMatchStatement.java:448-458)
    std::vector<DBuf<uint32_t>> empty_rows;
    uint64_t n_empty = 0;
    if (st.optional && R_) {
      DBuf<uint8_t> fl(&pool_, R_);
      launch_flag_no_neighbor(col_[st.src].p, R_, make_adj(st.adj), bitmap(st.where_bm), fl.p, s_);
      DBuf<uint32_t> idx(&pool_, R_);
      DBuf<uint64_t> nsel(&pool_, 1);
      hipcub::CountingInputIterator<uint32_t> cnt(0);
      cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, cnt, fl.p, idx.p, nsel.p, (int64_t)R_, s_); });
      n_empty = read1(nsel.p);
      for (int c : bound_cols()) {
        empty_rows.emplace_back(&pool_, std::max<uint64_t>(n_empty, 1));
        if (n_empty) launch_gather_u32(col_[c].p, idx.p, n_empty, empty_rows.back().p, s_);
      }
    }
    std::vector<int> cols = bound_cols();  // the carried columns (st.dst is not bound yet)
    if (!check && !st.optional && st.filter_bm >= 0 && factor_ && R_ >= factor_min_rows_ && expand_factorized(st, write, cols)) {
      bound_[st.dst] = 1;
      return;
    }
    bound_[st.dst] = 1;
    std::vector<const uint32_t *> carry;
    for (int c : cols) carry.push_back(col_[c].p);
    // a set-valued hop over an adjacency that may repeat a neighbour: the input row index rides along
    // and the (row, neighbour) pairs are made distinct (a count-only hop writes its rows for that)
    const bool nbset = st.distinct_nb && !st.adj.dup_free && !check;
    DBuf<uint32_t> rid;
    if (nbset) {
      write = true;
      allow_segmented = false;
      rid = DBuf<uint32_t>(&pool_, std::max<uint64_t>(R_, 1));
      launch_iota(rid.p, R_, s_);
      carry.push_back(rid.p);
    }
    ExpandOut o = expand_core(col_[st.src].p, R_, st.adj, bitmap(st.filter_bm), carry, write, allow_segmented,
                              check ? col_[check->src].p : nullptr, check ? &check->adj : nullptr,
                              check ? bitmap(check->filter_bm) : nullptr);
    edges_ += o.E + o.E_member;
    if (!o.counted_from_degrees) edges_iter_ += o.E;
    R_ = o.n;
    // (an expansion with no rows or no adjacency returns no carried columns at all)
    if (nbset && o.carry.size() > cols.size()) {
      DBuf<uint32_t> orid = std::move(o.carry.back());
      o.carry.pop_back();
      if (o.n) {
        std::vector<DBuf<uint32_t> *> oc;
        for (auto &c : o.carry) oc.push_back(&c);
        R_ = o.n = distinct_pairs(orid, o.dst, oc, o.n);
      }
    }
    if (n_empty) {  // append the null-target rows
      const uint64_t n = R_ + n_empty;
      auto cat = [&](DBuf<uint32_t> *a, const uint32_t *b) {
        DBuf<uint32_t> o2(&pool_, n);
        if (a && R_) HIP_CHECK(hipMemcpyAsync(o2.p, a->p, R_ * 4, hipMemcpyDeviceToDevice, s_));
        if (b) HIP_CHECK(hipMemcpyAsync(o2.p + R_, b, n_empty * 4, hipMemcpyDeviceToDevice, s_));
        else launch_fill_u32(o2.p + R_, n_empty, g_.V, s_);
        return o2;
      };
      for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = cat(R_ ? &o.carry[i] : nullptr, empty_rows[i].p);
      col_[st.dst] = cat(R_ ? &o.dst : nullptr, nullptr);
      R_ = n;
      segmented_ = false;
      return;
    }
    if (!write || R_ == 0) return;
    segmented_ = o.segmented;
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(o.carry[i]);
    col_[st.dst] = std::move(o.dst);
  }

  // The last hop of a plan that returns only its new alias, de-duplicated (configs[0]: `RETURN fof`):
  // every row's neighbours are marked in a V-bit set as the kernels read them, instead of being written
  // as rows and then marked (addToUniqueResult keeps one row per distinct value, C/command/
  // OBasicCommandContext.java:347-353). All Σ deg adjacency entries are still read; the bindings are
  // that sum. Unfiltered hops on one GPU, no LIMIT, no optional target, not a variable-length item.
  bool marked_ = false;
  uint64_t marked_bindings_ = 0;
  bool mark_fuse_ = true;  // OMX_MARK_FUSE=0: write the rows and mark them in the projection
  bool mark_ok(const Step &st) const {
    return mark_fuse_ && !dist_ && st.filter_bm < 0 && !st.optional && p_.kind == Plan::MATCH && !g_.edge_records &&
           p_.proj == Plan::PROJ_ALIASES && !p_.unique_by_construction && p_.out_aliases.size() == 1 &&
           p_.out_aliases[0] == st.dst && !p_.optional[st.dst] && p_.limit < 0 && o_.limit < 0 &&
           o_.mode == OMX_MODE_MATERIALIZE;
  }
  // configs[0]'s shape — root, an unfiltered hop, the marked last hop — on a graph of ≤ kFof2Bits vertices:
  // four launches (kernels.hip k_fof2_a / _b + the list) and one host round trip for the whole MATCH. The same
  // distinct set and accounting as root() + expand_step() + expand_mark()'s factorized branch: E_t = E1
  // + Σ over hop 1's rows of deg2, bindings = that sum, edges read = E1 + the distinct sources' entries.
  // (edges_read and factorized_hops are diagnostics of what ran: this path always reads the distinct
  // sources' entries only, so they say so even where the general path's thresholds — factor_min_rows_,
  // factor_min_ratio_ — would have read Σ deg2 one row at a time; E_t and bindings are path-independent)
  bool fof2_ok() {
    if (!mark_fuse_ || !factor_ || dist_ || g_.partitioned() || p_.kind != Plan::MATCH || p_.steps.size() != 3 ||
        g_.V > kFof2Bits || g_.V == 0 || g_.edge_records)
      return false;
    const Step &r = p_.steps[0], &h1 = p_.steps[1], &h2 = p_.steps[2];
    return r.kind == S_ROOT && r.cand_bm >= 0 && h1.kind == S_EXPAND && h2.kind == S_EXPAND && h1.src == r.dst && h2.src == h1.dst &&
           h1.filter_bm < 0 && !h1.optional && !h1.distinct_nb && !h1.adj.parts.empty() && !h2.adj.parts.empty() &&
           mark_ok(h2);
  }
  void fof2() {
    const Step &r = p_.steps[0], &h1 = p_.steps[1], &h2 = p_.steps[2];
    const uint64_t W = (g_.V + 63) / 64;
    DBuf<uint64_t> z(&pool_, 2 * W + 4);  // ubm, bm, acc: one memset
    DBuf<uint32_t> blk(&pool_, bitmap_list_blocks(W)), out(&pool_, g_.V);
    HIP_CHECK(hipMemsetAsync(z.p, 0, (2 * W + 4) * 8, s_));
    // ≥ 16 Ki edges a workgroup: its flush (W words, into the global set at agent scope) stays small beside
    // its marking (measured at RMAT-16: 4 Ki edges a workgroup, 4× the flushes, took 0.085 ms against 0.046)
    auto edges = [&](const AdjSpec &as) {
      uint64_t E = 0;
      for (auto &pt : as.parts) E += pt.second == 0 ? g_.esets[pt.first].n_edges : g_.esets[pt.first].n_in_edges;
      return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus(), E / 16384));
    };
    Fof2Args a{};
    a.a1 = make_adj(h1.adj);
    a.a2 = make_adj(h2.adj);
    a.roots = bitmap(r.cand_bm);
    a.rank = o_.shard_world > 1 ? o_.shard_rank : 0;
    a.world = std::max(1, o_.shard_world);
    a.ubm = z.p;
    a.bm = z.p + W;
    a.acc = z.p + 2 * W;
    a.V = g_.V;
    a.W = W;
    // (algorithmic bytes, amended once the counts are back: hop 1 reads the roots' words, its row pointers
    // and entries and the targets' row pointers (E_t); hop 2 the distinct sources' words, row pointers and
    // entries; the list the marked words and the vertices written)
    tm_.begin("k_fof2_a");
    launch_fof2(a, 0, edges(h1.adj), nullptr, nullptr, nullptr, s_);
    tm_.end();
    const size_t ra = tm_.last();
    tm_.begin("k_fof2_b");
    launch_fof2(a, 1, edges(h2.adj), nullptr, nullptr, nullptr, s_);
    tm_.end();
    const size_t rb = tm_.last();
    const Mail ml = mail();
    tm_.begin("k_bitmap_to_list");
    launch_fof2(a, 2, 0, blk.p, out.p, &ml, s_);
    tm_.end();
    const size_t rl = tm_.last();
    const uint64_t *m = wait_mail();
    const uint64_t n = m[0], e1 = m[1], et = m[2], eu = m[3];
    const uint64_t ba = W * 8 + 8ull * g_.V * a.a1.n + 4 * e1 + 16 * e1, bb = W * 16 + 8ull * g_.V * a.a2.n + 4 * eu,
                   bl = W * 8 + 4 * n;
    tm_.amend_at(ra, ba);
    tm_.amend_at(rb, bb);
    tm_.amend_at(rl, bl);
    alg_bytes_ += ba + bb + bl;
    edges_ += e1 + et;
    edges_iter_ += e1 + eu;
    marked_bindings_ = et;
    marked_ = true;
    factorized_hops_++;
    bound_[r.dst] = bound_[h1.dst] = bound_[h2.dst] = 1;
    col_[h2.dst] = std::move(out);
    R_ = n;
    segmented_ = false;
  }

  void expand_mark(const Step &st) {
    route_owner(st.src);
    DBuf<uint64_t> bm(&pool_, std::max<uint64_t>(nwords_, 1));
    HIP_CHECK(hipMemsetAsync(bm.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
    // rows whose sources repeat (C1: every Person a root, each b reached from all its in-neighbours) mark
    // each distinct source's neighbours once: the marked set is a union, so it is the same; E_t and the
    // bindings stay Σ over the rows of deg(src); edges_read counts what was iterated
    if (factor_ && R_ >= factor_min_rows_) {
      uint64_t U = 0;
      DBuf<uint32_t> ub;
      {
        DBuf<uint64_t> ubm(&pool_, std::max<uint64_t>(nwords_, 1));
        HIP_CHECK(hipMemsetAsync(ubm.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
        tm_.begin("k_mark_bitmap");
        launch_mark_bitmap(col_[st.src].p, R_, ubm.p, g_.V, s_);
        tm_.end(4ull * R_ + 8ull * nwords_);
        ub = bitmap_list(ubm.p, 0, 1, U);
      }
      const uint64_t Et = degree_sum(col_[st.src].p, R_, st.adj), EU = degree_sum(ub.p, U, st.adj);
      if (Et >= factor_min_ratio_ * EU) {
        ExpandOut o = expand_core(ub.p, U, st.adj, nullptr, {}, false, false, nullptr, nullptr, nullptr, nullptr, false,
                                  bm.p);
        edges_ += Et;
        edges_iter_ += o.E;
        marked_bindings_ = Et;
        factorized_hops_++;
        bound_[st.dst] = 1;
        marked_ = true;
        uint64_t m = 0;
        col_[st.dst] = bitmap_list(bm.p, 0, 1, m);
        R_ = m;
        segmented_ = false;
        return;
      }
    }
    ExpandOut o = expand_core(col_[st.src].p, R_, st.adj, nullptr, {}, false, false, nullptr, nullptr, nullptr, nullptr,
                              false, bm.p);
    edges_ += o.E;
    edges_iter_ += o.E;
    bound_[st.dst] = 1;
    marked_ = true;
    marked_bindings_ = o.E;
    uint64_t m = 0;
    col_[st.dst] = bitmap_list(bm.p, 0, 1, m);
    R_ = m;
    segmented_ = false;
  }

  // Factorized expansion of a filtered hop whose rows repeat their source vertices (hubs reached from
  // many roots: C2's second hop reads each distinct b's adjacency 31× over at RMAT-22, 50× at RMAT-24):
  //   1. the distinct sources U (V-bit bitmap + list) and each row's index into them;
  //   2. the filtered neighbour list L(u) of every distinct source: one filtered expansion of U rows;
  //   3. L grouped by source into a CSR (histogram, scan, scatter);
  //   4. an unfiltered expansion of the rows over L: dense output of exactly the result rows.
  // The rows are the direct expansion's (same multiset, processContext :491-497 per row); E_t still
  // counts Σ_rows deg; edges_read counts what was iterated (Σ_U deg + the L entries).
  // Returns false (nothing done) when the rows repeat their sources less than kFactorMinRatio-fold.
  uint64_t factor_min_rows_ = 4096, factor_min_ratio_ = 4;
  // Measured and removed (round 4, after rounds 2-3 kept them as options): the lists by ordered tiles of
  // the flat entry space, from the sources' side (1.6 ms for M1's 200 M entries) or the targets' in-rows
  // (0.25 ms + a 0.6 ms pair sort), the targets' (b, c) pairs written over the rows grouped by source
  // (5.22 against 4.35 ms per step: the pairs re-read their groups from MALL), the entries placed by a
  // rank written in the histogram pass (within box noise of the cursor scatter); profiles/r03/flist,
  // femit/reverse.txt, rank2.
  // OMX_FEMIT=0: write the rows with the generic unfiltered expansion (binned heavy / merge-path rows)
  // instead of k_femit's output tiles; k_femit's rows are grouped by source, so each list is re-read from
  // L2 by its rows (in row order they came from HBM / MALL: 4.35 against 5.2 ms per M1 step, round 3)
  // OMX_FEMIT: 0 = never, 1 = when the hop traverses at least femit_min_et_ edges (E_t), force = always
  // (tests). Below that its fixed costs (the row sort, selections, tile lists: ≈ 0.2 ms) outweigh the
  // faster writes. Round 3: C2 (RMAT-22, E_t 1.5e9) 1.21 ms against 1.15 binned (profiles/r03/femit/
  // c2ab.txt), so 4e9; round 5, with the lists from k_flists: C2 1.02 against 1.16-1.27 binned, one box
  // interleaved (gpurun_out/r5c2), so 1e9
  int femit_ = 1;
  static constexpr uint64_t kOnDevice = UINT64_MAX;  // a count left on the device (emit_factorized's nlist)
  size_t flist_copy_rec_ = SIZE_MAX;                  // the timing record of the last k_flist_copy
  static constexpr uint64_t femit_min_et_ = 1000000000ull;
  bool femit_slow_ = false;  // OMX_FEMIT_SLOW=1: every output tile through k_femit_slow (tests)

  // step 4 of expand_factorized when the rows are written: the output space Σ_rows |L(g[r])| is laid out
  // row by row and written by tiles of output rows (factor.hip k_femit)
  // The last hop of a plan whose projection never reads its new alias (RETURN a.uid, b.age over
  // a-->b-->c): every document of a row (…, b, c) is the document of (…, b), so the result is that of
  // the rows whose source has a non-empty filtered list — a semi-join, no (…, b, c) row is written. The
  // bindings (complete matches before de-duplication) are still Σ_rows |L(b)|; E_t is the hop's.
  // OMX_SEMI=0: write the rows as any other hop.
  bool semi_ = false, semi_ok_ = true;
  bool grp32_ = true;  // OMX_GRP32=0: 64-bit counters in the factorized grouping
  // the distinct sources' filtered lists through the hub-annotated col (factor.hip k_flists, round 5);
  // OMX_FLISTS=0: the sliced expansion + grouping (still the path for multigraph set-valued hops, several
  // CSR parts and partitioned snapshots)
  bool flists_ = true;
  uint64_t semi_bindings_ = 0;
  bool semi_for(const Step &st) const {
    if (!semi_ok_ || p_.kind != Plan::MATCH || st.kind != S_EXPAND || st.optional || p_.optional[st.dst] ||
        o_.mode != OMX_MODE_MATERIALIZE)
      return false;
    if (p_.proj != Plan::PROJ_ALIASES && p_.proj != Plan::PROJ_EXPR && p_.proj != Plan::PROJ_JSON) return false;
    return std::find(p_.out_aliases.begin(), p_.out_aliases.end(), st.dst) == p_.out_aliases.end();
  }
  void semi_join(const DBuf<uint32_t> &g, uint64_t R, const DBuf<uint64_t> &loff, const std::vector<int> &cols) {
    DBuf<uint64_t> len(&pool_, R + 1), nsel(&pool_, 2);  // nsel: {kept rows, bindings}
    launch_femit_len(g.p, R, loff.p, len.p, s_);
    cub([&](void *t, size_t &b) { return hipcub::DeviceReduce::Sum(t, b, len.p, nsel.p + 1, (int64_t)(R + 1), s_); });
    DBuf<uint32_t> idx(&pool_, std::max<uint64_t>(R, 1));
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    hipcub::TransformInputIterator<uint8_t, NonZeroU64, const uint64_t *> fl(len.p, NonZeroU64());
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, cnt, fl, idx.p, nsel.p, (int64_t)R, s_); });
    const auto kb = read2(nsel.p);
    const uint64_t Rn = kb.first;
    semi_bindings_ = kb.second;
    for (int c : cols) {
      DBuf<uint32_t> o(&pool_, std::max<uint64_t>(Rn, 1));
      if (Rn) launch_gather_u32(col_[c].p, idx.p, Rn, o.p, s_);
      col_[c] = std::move(o);
    }
    R_ = Rn;
    segmented_ = false;
    factorized_hops_++;
    semi_hops_++;
    if (debug_expand_)
      std::fprintf(stderr, "[omx factorized] semi-join R=%llu kept=%llu bindings=%llu\n", (unsigned long long)R,
                   (unsigned long long)Rn, (unsigned long long)semi_bindings_);
  }

  // perm_sorted: the rows sorted by source (g in that order); perm_sorted[i] = the row at sorted
  // position i. nlist: the entries of all U lists (each read from HBM once, then from L2 by its rows);
  // kOnDevice: loff[U] holds them (read with the emission's own round trip)
  void emit_factorized(DBuf<uint32_t> &g, uint64_t R, uint64_t U, DBuf<uint64_t> &loff, DBuf<uint32_t> &lcol,
                       uint64_t nlist, const std::vector<int> &cols, const Step &st, const uint32_t *perm_sorted) {
    // 1. the rows whose list is not empty (the others write nothing), in row order or grouped by source.
    // Their count Rn stays on the device until the output size N is known: the kernels in between run
    // over R rows and read Rn, so one host round trip returns both
    // (the rows are grouped by source already: the non-empty rows keep their sorted order; their source
    // indices and carried columns, first output rows and list bases in three launches, one mail:
    // factor.hip k_emitrows_*, round 6)
    DBuf<uint32_t> gs(&pool_, std::max<uint64_t>(R, 1));
    std::vector<DBuf<uint32_t>> sc;
    if (cols.size() > (size_t)kFemitCols) fail(OMX_E_INVALID, "internal: emission over more carried columns than k_femit_w takes");
    // 2. output rows of every binding row: the scan of its list length (roff[Rn] = N); list position of
    // output o
    DBuf<uint64_t> roff(&pool_, R + 1), rbase(&pool_, std::max<uint64_t>(R, 1));
    FemitRows fr{};
    fr.g = g.p;
    fr.perm = perm_sorted;
    fr.loff = loff.p;
    fr.R = R;
    fr.gs = gs.p;
    fr.roff = roff.p;
    fr.rbase = rbase.p;
    fr.nc = (int32_t)cols.size();
    for (size_t c = 0; c < cols.size(); ++c) {
      sc.emplace_back(&pool_, std::max<uint64_t>(R, 1));
      fr.in[c] = col_[cols[c]].p;
      fr.out[c] = sc.back().p;
    }
    DBuf<uint64_t> tt(&pool_, 2 * emitrows_tiles(R)), tot(&pool_, 2);
    tm_.begin("k_emitrows");
    launch_emitrows(fr, tt.p, tot.p, mail(), s_, nlist == kOnDevice ? loff.p + U : nullptr);
    tm_.end(28ull * R);
    const uint64_t *m = wait_mail();
    const uint64_t Rn = m[0], N = m[1];
    if (nlist == kOnDevice) {
      nlist = m[2];
      tm_.amend_at(flist_copy_rec_, 8ull * nlist + 16ull * U);
    }
    edges_iter_ += N;
    alg_bytes_ += 8ull * R + 4ull * N * (cols.size() + 2);  // as expand_core's unfiltered written hop
    R_ = N;
    factorized_hops_++;
    if (debug_expand_)
      std::fprintf(stderr, "[omx factorized] emission R=%llu (non-empty %llu) U=%llu rows=%llu\n",
                   (unsigned long long)R, (unsigned long long)Rn, (unsigned long long)U, (unsigned long long)N);
    if (N == 0) return;
    // 3. the output tiles (factor.hip k_femit_w): the rows' list entries → the new column, their
    // carried values → their columns
    FemitArgs a{};
    a.g = gs.p;
    a.roff = roff.p;
    a.rbase = rbase.p;
    a.loff = loff.p;
    a.R = Rn;
    a.N = N;
    a.nl = 1;
    a.lcol[0] = lcol.p;
    DBuf<uint32_t> dst(&pool_, N);
    a.lout[0] = dst.p;
    a.nc = (int32_t)cols.size();
    std::vector<DBuf<uint32_t>> outc;
    for (size_t c = 0; c < cols.size(); ++c) {
      outc.emplace_back(&pool_, N);
      a.cin[c] = sc[c].p;
      a.cout[c] = outc.back().p;
    }
    femit_run(a, nlist);
    segmented_ = false;
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(outc[i]);
    col_[st.dst] = std::move(dst);
  }

  // the output tiles of a factorized emission (a's rows, offsets, lists and columns set): regular tiles
  // (full, ≤ 64 binding rows) through k_femit_w, the others through k_femit_slow
  // list_entries: the entries of a.lcol[0]'s lists when each is re-read from L2 by its rows (0: unknown,
  // the HBM-necessary bytes are then the algorithmic ones)
  void femit_run(FemitArgs &a, uint64_t list_entries = 0) {
    const uint64_t nt = femit_tiles(a.N);
    if (nt > 0xFFFFFFFFull) unsupported("a factorized emission of 2^42 or more rows");
    DBuf<uint64_t> rb(&pool_, 2 * nt), nreg(&pool_, 1);
    DBuf<uint8_t> reg(&pool_, nt);
    DBuf<uint32_t> lists(&pool_, nt);
    a.rb = rb.p;
    launch_femit_bounds(a, rb.p, reg.p, femit_slow_, s_);
    hipcub::CountingInputIterator<uint32_t> it(0);
    cub([&](void *t, size_t &b) { return hipcub::DevicePartition::Flagged(t, b, it, reg.p, lists.p, nreg.p, (int64_t)nt, s_); });
    if (debug_expand_) {
      const uint64_t nr = read1(nreg.p);
      std::fprintf(stderr, "[omx factorized] emission tiles %llu: regular %llu, other %llu\n", (unsigned long long)nt,
                   (unsigned long long)nr, (unsigned long long)(nt - nr));
    }
    tm_.begin("k_femit");
    launch_femit(a, lists.p, nreg.p, nt, cus(), s_);  // the kernels read the partition's count (no host wait)
    // every list column read and every column written per output row; per binding row its offsets and
    // constants
    const uint64_t alg = a.N * 4ull * (2ull * a.nl + a.nc) + a.R * (24ull + 4ull * a.nc);
    // HBM-necessary: every column written per output row, each list entry and binding row read once
    tm_.end(alg, list_entries && a.nl == 1 ? a.N * 4ull * (a.nl + a.nc) + 4ull * list_entries + a.R * (24ull + 4ull * a.nc)
                                           : alg);
  }

  // an adjacency over edge records (the snapshot's record or endpoint sets, Graph::edge_records)
  bool records_adj(const AdjSpec &a) const {
    for (auto &p : a.parts)
      if (g_.esets[p.first].pseudo) return true;
    return false;
  }
  bool expand_factorized(const Step &st, bool write, const std::vector<int> &cols) {
    if (records_adj(st.adj)) return false;  // edge-record hops: the direct expansion
    const uint64_t R = R_;
    const uint32_t *src = col_[st.src].p;
    uint64_t U = 0, Et = 0, EU = 0;
    DBuf<uint32_t> ub, g, perm_s;
    DBuf<uint64_t> ubm, doffb;  // doffb: the scan of the distinct sources' degrees (doffb[U] = EU)
    const DAdj adj = make_adj(st.adj);
    // rows emitted by k_femit_w from the sources' lists: the rows are sorted by source here (the emission
    // wants them grouped), so the distinct sources are the sorted runs' heads and a row's source index
    // is its run — no bitmap, position map or second sort. Whether the emission runs depends on E_t (its
    // threshold), which the device computes beside the sort: E_t, the distinct sources U and their
    // adjacency total EU come back in one host round trip (three before: 0.06-0.09 ms of idle device)
    const bool femit_ok = write && !semi_ && femit_ && cols.size() <= (size_t)kFemitCols && R > 0 && adj.n > 0;
    bool femit = false;
    const bool nbset = st.distinct_nb && !st.adj.dup_free;
    // the lists pass's conditions known before the sources are (its EU bounds are checked after)
    // (k_flist_info packs a source's chunk count in 28 bits: rows under 2^30 entries)
    const bool fl_ok = flists_ && !(write && semi_) && !nbset && st.adj.parts.size() == 1 && g_.V < 0x80000000u &&
                       g_.esets[st.adj.parts[0].first].max_deg[st.adj.parts[0].second] < (1ull << 30);
    DBuf<uint64_t> ccoff;  // the sources' chunk offsets and chunk table (launch_srcrows, for k_flist)
    DBuf<uint4> cinfo;
    if (femit_ok) {
      DBuf<uint32_t> iota(&pool_, R), ss(&pool_, R);
      perm_s = DBuf<uint32_t>(&pool_, R);
      ub = DBuf<uint32_t>(&pool_, R);
      g = DBuf<uint32_t>(&pool_, R);
      launch_iota(iota.p, R, s_);
      // the key bits of the largest source id: V − 1, or V for a null (optional) binding — at RMAT-24 24
      // bits, three 8-bit onesweep passes instead of four for bits_for(V) = 25 (round 6)
      const int kbits = std::max(1, bits_for(p_.optional[st.src] ? (uint64_t)g_.V : (uint64_t)g_.V - 1));
      tm_.begin("femit_row_sort");
      // (rocPRIM onesweep configurations of 8-bit digits measured against hipCUB's default: within noise,
      // round 6, gpurun_out/r6i)
      cub([&](void *t, size_t &b) {
        return sort_pairs(t, b, src, ss.p, iota.p, perm_s.p, R, kbits, s_);
      });
      tm_.end(16ull * R * ((kbits + 7) / 8));
      // the sorted rows' distinct sources (run heads), each row's source index, the sources' degree scan
      // and E_t = Σ_rows deg(source): three launches, one mail {E_t, U, EU} (factor.hip k_srcrows_*)
      doffb = DBuf<uint64_t>(&pool_, R + 1);
      DBuf<uint64_t> tt(&pool_, 4 * prologue_tiles(R)), tot(&pool_, 4);
      if (fl_ok) {
        ccoff = DBuf<uint64_t>(&pool_, R + 1);
        cinfo = DBuf<uint4>(&pool_, R);
      }
      tm_.begin("k_srcrows");
      launch_srcrows(ss.p, R, adj, tt.p, tot.p, ub.p, g.p, doffb.p, mail(), s_, ccoff.p, cinfo.p);
      tm_.end(12ull * R + 16ull * R);
      const uint64_t *m = wait_mail();
      Et = m[0], U = m[1], EU = m[2];
      femit = femit_ == 2 || Et >= femit_min_et_;
      if (!femit) {  // below the threshold: the rows' source indices back in row order
        DBuf<uint32_t> gr(&pool_, R);
        launch_scatter_u32(perm_s.p, g.p, R, gr.p, s_);
        g = std::move(gr);
      }
    } else {
      Et = degree_sum(src, R, st.adj);
      // the distinct sources, ascending: marked in a V-bit bitmap and listed (no sort of the R rows)
      ubm = DBuf<uint64_t>(&pool_, std::max<uint64_t>(nwords_, 1));
      HIP_CHECK(hipMemsetAsync(ubm.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
      tm_.begin("k_mark_bitmap");
      launch_mark_bitmap(src, R, ubm.p, g_.V, s_);
      tm_.end(4ull * R + 8ull * nwords_);
      ub = bitmap_list(ubm.p, 0, 1, U);
      // the distinct sources' degrees, scanned
      DBuf<uint64_t> udeg(&pool_, U + 1);
      doffb = DBuf<uint64_t>(&pool_, U + 1);
      tm_.begin("k_row_degree");
      launch_row_degree(ub.p, U, adj, udeg.p, s_);
      tm_.end(U * (4ull + 16ull * st.adj.parts.size()));
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, udeg.p, doffb.p, (int64_t)(U + 1), s_); });
      EU = read1(doffb.p + U);
    }
    if (Et < factor_min_ratio_ * EU) return false;
    edges_ += Et;
    // 1. row → distinct source index: a V-sized position map scattered from the list, gathered per row
    // (sorted rows have theirs from the runs)
    DBuf<uint32_t> iu(&pool_, std::max<uint64_t>(U, 1));
    launch_iota(iu.p, U, s_);
    if (!g.p) {
      g = DBuf<uint32_t>(&pool_, R);
      DBuf<uint32_t> pos(&pool_, std::max<uint64_t>(g_.V, 1));
      tm_.begin("k_scatter_u32");
      launch_scatter_u32(ub.p, iu.p, U, pos.p, s_);
      tm_.end(12ull * U);
      tm_.begin("k_gather_u32");
      launch_gather_u32(pos.p, src, R, g.p, s_);
      tm_.end(12ull * R);
    }
    // 2.-3. the filtered lists of the distinct sources, grouped by source (CSR loff / lcol)
    DBuf<uint64_t> loff;
    DBuf<uint32_t> lcol;
    uint64_t nlist = 0;
    // (the chunk space's offsets are u32: EU / 4 + 2U chunks below 2^32; a semi-join needs the lists'
    // lengths only, which the binned path counts without grouping them: R1 1.66 against 1.81 ms through
    // the tiled pass without its copy, one box, `r05pmc2`)
    bool use_fl = fl_ok && EU > 0 && EU / 4 + 2 * U < 0xFFFFFF00ull;
    if (use_fl) {
      try {
        filtered_lists(ub.p, U, doffb.p, EU, st.adj, bitmap(st.filter_bm), loff, lcol, ccoff.p, cinfo.p);
        nlist = kOnDevice;
        edges_iter_ += EU;
      } catch (const OmxError &e) {
        // the lists col (E entries) or the pass's scratch (≈ 2 EU entries) did not fit: the binned lists
        // below size their buffers by the filtered count instead
        if (e.code != OMX_E_OOM) throw;
        (void)hipGetLastError();
        use_fl = false;
        loff = DBuf<uint64_t>();
        lcol = DBuf<uint32_t>();
      }
    }
    if (!use_fl) {
      DBuf<unsigned long long> cnt(&pool_, U + 1);
      loff = DBuf<uint64_t>(&pool_, U + 1);
      HIP_CHECK(hipMemsetAsync(cnt.p, 0, (U + 1) * 8, s_));
      // 2. filtered lists of the distinct sources: (source index, neighbour) pairs
      // (the filtered lists stay in the expansion's per-worker segments: grouping reads them in place)
      // (a set-valued hop over an adjacency that may repeat a neighbour: each list made distinct first)
      ExpandOut l = expand_core(ub.p, U, st.adj, bitmap(st.filter_bm), {iu.p}, true, !nbset);
      edges_iter_ += l.E;
      if (nbset && l.n) l.n = distinct_pairs(l.carry[0], l.dst, {}, l.n);
      nlist = l.n;
      // 3. grouped by source: offsets (U + 1) and the neighbours in group order (segmented lists under
      // 2^32 entries: 32-bit counters and cursors, half the atomics' footprint)
      const bool c32 = l.segmented && l.n < (1ull << 32) && grp32_;
      DBuf<uint32_t> h32;
      if (c32) {
        h32 = DBuf<uint32_t>(&pool_, U + 1);
        HIP_CHECK(hipMemsetAsync(h32.p, 0, (U + 1) * 4, s_));
      }
      if (l.n) {
        tm_.begin("k_key_hist");
        if (c32) launch_key_hist_seg(l.carry[0].p, l.seg_start.p, l.seg_count.p, l.nseg, h32.p, s_);
        else if (l.segmented) launch_key_hist_seg(l.carry[0].p, l.seg_start.p, l.seg_count.p, l.nseg, cnt.p, s_);
        else launch_key_hist(l.carry[0].p, l.n, cnt.p, s_);
        tm_.end(4ull * l.n + (c32 ? 4ull : 8ull) * U);
      }
      if (c32) {
        hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> hc(h32.p, CastU64());
        cub([&](void *t, size_t &b) {
          return hipcub::DeviceScan::ExclusiveSum(t, b, hc, loff.p, (int64_t)(U + 1), s_);
        });
      } else {
        cub([&](void *t, size_t &b) {
          return hipcub::DeviceScan::ExclusiveSum(t, b, cnt.p, reinterpret_cast<unsigned long long *>(loff.p), (int64_t)(U + 1), s_);
        });
      }
      if (write && semi_) {  // the new alias is never read again: the rows whose source has a list
        semi_join(g, R, loff, cols);
        return true;
      }
      lcol = DBuf<uint32_t>(&pool_, std::max<uint64_t>(l.n, 1));
      if (l.n && c32) {
        DBuf<uint32_t> cur(&pool_, U + 1);
        cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, h32.p, cur.p, (int64_t)(U + 1), s_); });
        tm_.begin("k_key_scatter");
        launch_key_scatter_seg(l.carry[0].p, l.dst.p, l.seg_start.p, l.seg_count.p, l.nseg, cur.p, lcol.p, s_);
        tm_.end(12ull * l.n + 4ull * U);
      } else if (l.n) {
        HIP_CHECK(hipMemcpyAsync(cnt.p, loff.p, (U + 1) * 8, hipMemcpyDeviceToDevice, s_));
        tm_.begin("k_key_scatter");
        if (l.segmented)
          launch_key_scatter_seg(l.carry[0].p, l.dst.p, l.seg_start.p, l.seg_count.p, l.nseg, cnt.p, lcol.p, s_);
        else launch_key_scatter(l.carry[0].p, l.dst.p, l.n, cnt.p, lcol.p, s_);
        tm_.end(12ull * l.n + 8ull * U);
      }
    }
    // 4. the rows over their sources' lists
    if (femit) {
      emit_factorized(g, R, U, loff, lcol, nlist, cols, st, perm_s.p);
      return true;
    }
    if (nlist == kOnDevice && (debug_expand_ || tm_.on())) {  // (diagnostics only: one more host read)
      nlist = read1(loff.p + U);
      tm_.amend_at(flist_copy_rec_, 8ull * nlist + 16ull * U);
    }
    DAdj ladj{};
    ladj.n = 1;
    ladj.sorted = 0;
    ladj.p[0].rp = loff.p;
    ladj.p[0].col = lcol.p;
    std::vector<const uint32_t *> carry;
    for (int c : cols) carry.push_back(col_[c].p);
    ExpandOut o = expand_core(g.p, R, st.adj, nullptr, carry, write, false, nullptr, nullptr, nullptr, &ladj);
    if (!o.counted_from_degrees) edges_iter_ += o.E;
    R_ = o.n;
    factorized_hops_++;
    if (debug_expand_)
      std::fprintf(stderr, "[omx factorized] R=%llu U=%llu Et=%llu EU=%llu lists=%llu rows=%llu\n", (unsigned long long)R,
                   (unsigned long long)U, (unsigned long long)Et, (unsigned long long)EU, (unsigned long long)nlist,
                   (unsigned long long)o.n);
    if (!write || R_ == 0) return true;
    segmented_ = false;
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(o.carry[i]);
    col_[st.dst] = std::move(o.dst);
    return true;
  }

  // ---- TRAVERSE / SELECT expand(): ordered record lists (Plan::chain) ------------------------------
  // the FROM records in target order: a class's vertices in snapshot order, or the listed RIDs that
  // name a vertex (an unknown RID is skipped, like a record that does not load); `where` filters them
  DBuf<uint32_t> chain_roots(uint64_t &n, int where) {
    const ChainSpec &c = p_.chain;
    DBuf<uint64_t> wscratch;
    if (c.root_class >= 0) {
      DBuf<uint64_t> bm(&pool_, padded_words());
      eval_bitmap(where, c.root_class, 0, bm.p, padded_words());
      return bitmap_list(bm.p, 0, 1, n);
    }
    n = 0;
    const uint64_t m = c.root_rids.size();
    if (!m) return DBuf<uint32_t>(&pool_, 1);
    DBuf<uint64_t> keys(&pool_, m);
    DBuf<uint32_t> ids(&pool_, m);
    HIP_CHECK(hipMemcpyAsync(keys.p, c.root_rids.data(), m * 8, hipMemcpyHostToDevice, s_));
    launch_fill_u32(ids.p, m, UINT32_MAX, s_);
    launch_find_rids(g_.d_rids, g_.V, keys.p, (uint32_t)m, ids.p, s_);
    std::vector<uint32_t> h(m);
    HIP_CHECK(hipMemcpyAsync(h.data(), ids.p, m * 4, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    std::vector<uint32_t> found;
    for (uint32_t v : h)
      if (v != UINT32_MAX) found.push_back(v);
    DBuf<uint32_t> r(&pool_, std::max<size_t>(found.size(), 1));
    n = found.size();
    if (n) {
      HIP_CHECK(hipMemcpyAsync(r.p, found.data(), n * 4, hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipStreamSynchronize(s_));  // `found` leaves scope
    }
    const uint64_t *wb = prog_bitmap(where, 0, wscratch);
    if (!n || !wb) return r;
    DBuf<uint8_t> flags(&pool_, n);
    launch_flag_bitmap(r.p, n, wb, flags.p, s_);
    DBuf<uint32_t> sel(&pool_, n);
    DBuf<uint64_t> nsel(&pool_, 1);
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, r.p, flags.p, sel.p, nsel.p, (int64_t)n, s_); });
    n = read1(nsel.p);
    return sel;
  }

  // one move of an ordered list: every entry's neighbours, entries in order (duplicates kept); with a
  // filter, only the neighbours in it (still in order)
  DBuf<uint32_t> ordered_hop(const uint32_t *cur, uint64_t n, const AdjSpec &adj, uint64_t &out_n,
                             const uint64_t *filter = nullptr) {
    out_n = 0;
    FetchedAdj f;
    if (dist_) chain_fetch(adj, cur, n, f);  // (every call, n = 0 included: the servers count on it)
    if (!n) return DBuf<uint32_t>(&pool_, 1);
    ExpandOut o = expand_core(cur, n, adj, filter, {}, true, false, nullptr, nullptr, nullptr, dist_ ? &f.adj : nullptr, true);
    edges_ += o.E;
    edges_iter_ += o.E;
    out_n = o.n;
    if (!o.n) return DBuf<uint32_t>(&pool_, 1);
    return std::move(o.dst);
  }

  int64_t chain_limit() const { return p_.limit >= 0 ? p_.limit : o_.limit; }

  // ---- partitioned TRAVERSE / SELECT / shortestPath: rank 0 walks, the owners serve adjacency lists ---
  // Before each ordered move rank 0 asks for the lists of the move's vertices (chain_fetch): the request
  // (1, the AdjSpec's index in chain_specs) travels in an allgather_n round, the vertices go to their
  // owners, which answer with degrees and lists (the ordered expansion: parts in the AdjSpec's order), and
  // rank 0 lays them out as a V-row CSR (zero rows for the vertices not asked for) that the unchanged
  // single-GPU code expands. A (0, 0) round ends the service. The work list, history, WHILE / WHERE
  // bitmaps (replicated columns) and the result stay on rank 0.
  struct FetchedAdj {
    DBuf<uint64_t> rp;
    DBuf<uint32_t> col;
    DAdj adj{};
  };
  std::vector<const AdjSpec *> chain_specs() const {
    std::vector<const AdjSpec *> v;
    for (const AdjSpec &h : p_.chain.hops) v.push_back(&h);
    v.push_back(&p_.chain.sp_left);
    v.push_back(&p_.chain.sp_right);
    return v;
  }
  void chain_fetch(const AdjSpec &as, const uint32_t *list, uint64_t n, FetchedAdj &f) {
    const std::vector<const AdjSpec *> specs = chain_specs();
    const uint64_t id = (uint64_t)(std::find(specs.begin(), specs.end(), &as) - specs.begin());
    if (id >= specs.size()) fail(OMX_E_INVALID, "internal: a chain adjacency outside the plan");
    tr_->allgather_n({1, id}, s_);
    fetch_lists(as, list, n, &f);
  }
  void serve_chain() {
    const std::vector<const AdjSpec *> specs = chain_specs();
    for (;;) {
      const std::vector<uint64_t> w = tr_->allgather_n({0, 0}, s_);
      if (w[0] == 0) return;  // rank 0's word: the walk ended
      if (w[1] >= specs.size()) fail(OMX_E_INVALID, "internal: a chain adjacency request out of range");
      fetch_lists(*specs[w[1]], nullptr, 0, nullptr);
    }
  }
  // collective: rank 0's vertices (list, n) → their lists from the owners; out (rank 0) gets the CSR
  void fetch_lists(const AdjSpec &as, const uint32_t *list, uint64_t n, FetchedAdj *out) {
    const int W = tr_->world();
    DBuf<uint32_t> ids;
    uint64_t m = 0;
    if (n) {  // distinct, ascending (so the owners' answers concatenate in vertex order)
      DBuf<uint64_t> bm(&pool_, std::max<uint64_t>(nwords_, 1));
      HIP_CHECK(hipMemsetAsync(bm.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
      launch_mark_bitmap(list, n, bm.p, g_.V, s_);
      ids = bitmap_list(bm.p, 0, 1, m);
    } else {
      ids = DBuf<uint32_t>(&pool_, 1);
    }
    DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(m, 1));
    DBuf<uint64_t> hist(&pool_, W);
    HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
    if (m) launch_route_owner(ids.p, m, block_, (uint32_t)W, dest.p, hist.p, s_);
    m = exchange_cols({&ids}, m, dest, hist);
    DBuf<uint32_t> dlo(&pool_, std::max<uint64_t>(m, 1)), dhi(&pool_, std::max<uint64_t>(m, 1)), lists;
    uint64_t nl = 0;
    if (m) {
      DBuf<uint64_t> deg(&pool_, m + 1);
      launch_row_degree(ids.p, m, make_adj(as), deg.p, s_);
      launch_u64_split(deg.p, m, dlo.p, dhi.p, s_);
      ExpandOut o = expand_core(ids.p, m, as, nullptr, {}, true, false, nullptr, nullptr, nullptr, nullptr, true);
      nl = o.n;
      lists = nl ? std::move(o.dst) : DBuf<uint32_t>(&pool_, 1);
    } else {
      lists = DBuf<uint32_t>(&pool_, 1);
    }
    m = to_rank0({&ids, &dlo, &dhi}, m);
    nl = to_rank0({&lists}, nl);
    if (!out) return;
    // rank 0: rp[v + 1] - rp[v] = the fetched degree of v (0 for the others), col = the lists in order
    DBuf<uint64_t> dv(&pool_, (uint64_t)g_.V + 1);
    HIP_CHECK(hipMemsetAsync(dv.p, 0, ((uint64_t)g_.V + 1) * 8, s_));
    if (m) launch_scatter_deg(ids.p, dlo.p, dhi.p, m, dv.p, s_);
    out->rp = DBuf<uint64_t>(&pool_, (uint64_t)g_.V + 1);
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, dv.p, out->rp.p, (int64_t)g_.V + 1, s_); });
    out->col = std::move(lists);
    out->adj = DAdj{};
    out->adj.n = 1;
    out->adj.sorted = as.parts.size() == 1 && as.sorted;
    out->adj.p[0].rp = out->rp.p;
    out->adj.p[0].col = out->col.p;
  }

  // TRAVERSE <fields> FROM <target> [WHILE <cond>] [MAXDEPTH d] [LIMIT n] STRATEGY BREADTH_FIRST.
  // OTraverse's queue (OTraverseContext.QueueMemory) holds, level by level, the records the previous
  // level's fields pushed, in push order; a record is emitted when it is processed, is not in the
  // history and passes WHILE with $depth = its level (OTraverseRecordProcess.process :49-105). A
  // processed record below MAXDEPTH stays in the history, so it is emitted once, at its first entry;
  // one at MAXDEPTH is popped with its history entry removed (:66-69, OTraverseContext.pop :58-70), so
  // every entry of the MAXDEPTH level that is not in the history is emitted, repeats included. LIMIT
  // stops the work list after n results (OTraverse.hasNext :68-70).
  DBuf<uint32_t> traverse_bfs() {
    const ChainSpec &c = p_.chain;
    uint64_t n = 0;
    DBuf<uint32_t> cur = chain_roots(n, -1);
    DBuf<uint64_t> hist(&pool_, std::max<uint64_t>(nwords_, 1)), pscratch, keep(&pool_, std::max<uint64_t>(nwords_, 1));
    DBuf<uint32_t> first(&pool_, std::max<uint64_t>(g_.V, 1));
    HIP_CHECK(hipMemsetAsync(hist.p, 0, std::max<uint64_t>(nwords_, 1) * 8, s_));
    launch_fill_u32(first.p, g_.V, UINT32_MAX, s_);
    const int64_t limit = chain_limit();
    std::vector<DBuf<uint32_t>> parts;
    std::vector<uint64_t> pn;
    uint64_t total = 0;
    // level 0 is the FROM list itself; the entries of a later level come from the ordered expansion of
    // the previous level's records filtered by ¬history ∧ WHILE($depth), so only records that will be
    // processed are written; what is left per level is the first-entry claim of each record
    bool filtered = false;
    for (int64_t d = 0; n > 0; ++d) {
      if (n >= UINT32_MAX) unsupported("a TRAVERSE level of 2^32 or more work-list entries");
      const bool last = c.max_depth >= 0 && d == c.max_depth;
      const uint64_t *pred = filtered ? nullptr : prog_bitmap(c.pred_prog, d, pscratch);
      uint64_t k = n;
      DBuf<uint32_t> acc;
      if (!last || !filtered) {
        DBuf<uint8_t> flags(&pool_, n);
        tm_.begin("k_trav_filter");
        launch_trav_filter(cur.p, n, filtered ? nullptr : hist.p, pred, first.p, flags.p, !last, s_);
        tm_.end(n * 6);
        acc = DBuf<uint32_t>(&pool_, n);
        DBuf<uint64_t> nsel(&pool_, 1);
        tm_.begin("trav_select");
        select_flagged(cur.p, flags.p, acc.p, nsel.p, n);
        tm_.end(n * 9);
        k = read1(nsel.p);
      } else {
        acc = std::move(cur);  // the MAXDEPTH level keeps every entry the expansion let through
      }
      if (!last) launch_trav_accept(acc.p, k, hist.p, first.p, s_);
      if (k) {
        parts.push_back(std::move(acc));
        pn.push_back(k);
        total += k;
      }
      if (last || k == 0 || (limit > 0 && total >= (uint64_t)limit)) break;
      // next level's filter: ¬history ∧ WHILE($depth = d + 1)
      const uint64_t *np = prog_bitmap(c.pred_prog, d + 1, pscratch);
      launch_andnot_bitmap(np, hist.p, keep.p, nwords_, s_);
      cur = ordered_hop(parts.back().p, k, c.hops[0], n, keep.p);
      filtered = true;
    }
    R_ = limit > 0 ? std::min<uint64_t>(total, (uint64_t)limit) : total;
    bindings_ = total;
    return concat_batches(parts, pn, total);
  }

  // DeviceSelect::Flagged with 32-bit item counts when they fit (the 64-bit path measured ~10× slower)
  template <class T>
  void select_flagged(const T *in, const uint8_t *flags, T *out, uint64_t *nsel, uint64_t n) {
    if (n < 0x7FFFFFFFull) {
      DBuf<uint32_t> n32(&pool_, 1);
      cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, in, flags, out, n32.p, (int)n, s_); });
      launch_post_u32_to_u64(n32.p, nsel, s_);
    } else {
      cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, in, flags, out, nsel, (int64_t)n, s_); });
    }
  }

  // SELECT expand(m0(...).m1(...)...) FROM <target> [WHERE <cond>] [LIMIT n]: each call moves the whole
  // list, every record's result concatenated in order (OSQLEngine.foreachRecord, S/OSQLEngine.java:264-290)
  DBuf<uint32_t> select_expand() {
    const ChainSpec &c = p_.chain;
    uint64_t n = 0;
    DBuf<uint32_t> cur = chain_roots(n, c.pred_prog);
    for (const AdjSpec &h : c.hops) {
      if (!n) break;
      uint64_t m = 0;
      cur = ordered_hop(cur.p, n, h, m);
      n = m;
    }
    const int64_t limit = chain_limit();
    bindings_ = n;
    R_ = limit > 0 ? std::min<uint64_t>(n, (uint64_t)limit) : n;
    return cur;
  }

  // shortestPath(src, dst, direction, edge class, {maxDepth}) — OSQLFunctionShortestPath.execute
  // (GF/OSQLFunctionShortestPath.java:85-200): a bidirectional BFS from both ends, each round walking the
  // side with the shorter queue one whole level first (walkLeft / walkRight :232-292). A walk scans its
  // queue in order and every queue entry's neighbours in order; the first neighbour the other side has
  // visited ends the search (computePath :294-313: previouses back to the source, nexts on to the
  // destination); otherwise a neighbour not yet visited on this side is remembered with the entry that
  // discovered it first and queued, in discovery order.
  struct SpSide {
    DBuf<uint32_t> queue, parent;
    DBuf<uint64_t> visited;
    uint64_t n = 0;
    const AdjSpec *adj = nullptr;
  };
  bool sp_walk(SpSide &A, SpSide &B, DBuf<uint32_t> &first, uint32_t *meet_w, uint32_t *meet_cur) {
    if (!A.n) return false;
    if (A.n >= UINT32_MAX) unsupported("a shortestPath() level of 2^32 or more vertices");
    DBuf<uint32_t> rows(&pool_, A.n);
    launch_iota(rows.p, A.n, s_);
    FetchedAdj f;
    if (dist_) chain_fetch(*A.adj, A.queue.p, A.n, f);
    ExpandOut o = expand_core(A.queue.p, A.n, *A.adj, nullptr, {rows.p}, true, false, nullptr, nullptr, nullptr,
                              dist_ ? &f.adj : nullptr, true);
    edges_ += o.E;
    edges_iter_ += o.E;
    if (!o.n) {
      A.n = 0;
      return false;
    }
    if (o.n >= UINT32_MAX) unsupported("a shortestPath() level of 2^32 or more neighbours");
    DBuf<unsigned long long> pos(&pool_, 1);
    HIP_CHECK(hipMemsetAsync(pos.p, 0xFF, 8, s_));
    launch_sp_meet(o.dst.p, o.n, B.visited.p, pos.p, s_);
    const uint64_t e = read1(reinterpret_cast<const uint64_t *>(pos.p));
    if (e != ~0ull) {
      *meet_w = read1(o.dst.p + e);
      *meet_cur = read1(A.queue.p + read1(o.carry[0].p + e));
      return true;
    }
    DBuf<uint8_t> flags(&pool_, o.n);
    launch_trav_filter(o.dst.p, o.n, A.visited.p, nullptr, first.p, flags.p, true, s_);
    DBuf<uint64_t> keys(&pool_, o.n), sel(&pool_, o.n), nsel(&pool_, 1);
    launch_pack_pairs(o.carry[0].p, o.dst.p, o.n, keys.p, s_);
    select_flagged(keys.p, flags.p, sel.p, nsel.p, o.n);
    const uint64_t k = read1(nsel.p);
    DBuf<uint32_t> next(&pool_, std::max<uint64_t>(k, 1));
    launch_sp_accept(sel.p, k, A.queue.p, A.parent.p, A.visited.p, first.p, next.p, s_);
    A.queue = std::move(next);
    A.n = k;
    return false;
  }

  DBuf<uint32_t> shortest_path() {
    const ChainSpec &c = p_.chain;
    DBuf<uint64_t> keys(&pool_, 2);
    DBuf<uint32_t> ids(&pool_, 2);
    const uint64_t hk[2] = {c.sp_src, c.sp_dst};
    HIP_CHECK(hipMemcpyAsync(keys.p, hk, 16, hipMemcpyHostToDevice, s_));
    launch_fill_u32(ids.p, 2, UINT32_MAX, s_);
    launch_find_rids(g_.d_rids, g_.V, keys.p, 2, ids.p, s_);
    uint32_t h[2];
    HIP_CHECK(hipMemcpyAsync(h, ids.p, 8, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int i = 0; i < 2; ++i)
      if (h[i] == UINT32_MAX)  // graph.getVertex(...) is null: the reference fails on it
        fail(OMX_E_EXECUTION, std::string("shortestPath(): ") + (i ? "destination" : "source") + " vertex #" +
                                  std::to_string(hk[i] >> 48) + ":" + std::to_string(hk[i] & ((1ull << 48) - 1)) + " not found");
    std::vector<uint32_t> path;
    if (h[0] == h[1]) {
      path.push_back(h[0]);
    } else {
      SpSide L, R;
      const uint64_t W = std::max<uint64_t>(nwords_, 1);
      for (SpSide *x : {&L, &R}) {
        x->visited = DBuf<uint64_t>(&pool_, W);
        x->parent = DBuf<uint32_t>(&pool_, g_.V);
        x->queue = DBuf<uint32_t>(&pool_, 1);
        x->n = 1;
        HIP_CHECK(hipMemsetAsync(x->visited.p, 0, W * 8, s_));
        launch_fill_u32(x->parent.p, g_.V, UINT32_MAX, s_);
      }
      L.adj = &c.sp_left;
      R.adj = &c.sp_right;
      launch_fill_u32(L.queue.p, 1, h[0], s_);
      launch_fill_u32(R.queue.p, 1, h[1], s_);
      launch_mark_bitmap(L.queue.p, 1, L.visited.p, g_.V, s_);
      launch_mark_bitmap(R.queue.p, 1, R.visited.p, g_.V, s_);
      DBuf<uint32_t> first(&pool_, g_.V);
      launch_fill_u32(first.p, g_.V, UINT32_MAX, s_);
      const int maxd = c.sp_max_depth;
      bool met = false, met_left = false;
      uint32_t mw = 0, mc = 0;
      for (int depth = 1;;) {
        if (maxd >= 0 && maxd <= depth) break;
        if (!L.n || !R.n) break;
        const bool left_first = L.n <= R.n;
        SpSide &A = left_first ? L : R, &B = left_first ? R : L;
        if (sp_walk(A, B, first, &mw, &mc)) {
          met = true;
          met_left = left_first;
          break;
        }
        ++depth;
        if (maxd >= 0 && maxd <= depth) break;
        if (!A.n) break;
        if (sp_walk(B, A, first, &mw, &mc)) {
          met = true;
          met_left = !left_first;
          break;
        }
        ++depth;
      }
      if (met) {  // computePath: previouses back from the meeting vertex, then its nexts
        path.push_back(mw);
        for (uint32_t x = met_left ? mc : read1(L.parent.p + mw); x != UINT32_MAX; x = read1(L.parent.p + x))
          path.insert(path.begin(), x);
        for (uint32_t x = met_left ? read1(R.parent.p + mw) : mc; x != UINT32_MAX; x = read1(R.parent.p + x))
          path.push_back(x);
      }
    }
    const int64_t limit = chain_limit();
    bindings_ = path.size();
    R_ = limit > 0 && c.expand_rows ? std::min<uint64_t>(path.size(), (uint64_t)limit) : path.size();
    DBuf<uint32_t> out(&pool_, std::max<size_t>(path.size(), 1));
    if (!path.empty()) {
      HIP_CHECK(hipMemcpyAsync(out.p, path.data(), path.size() * 4, hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipStreamSynchronize(s_));  // the host vector goes out of scope
    }
    return out;
  }

  // WHERE conjunct `$matched.X op $currentMatch` of the alias the previous step bound
  void rowcmp_step(const Step &st) {
    if (R_ == 0) return;
    DBuf<uint8_t> flags(&pool_, R_);
    launch_flag_colcmp(col_[st.src].p, col_[st.dst].p, R_, st.row_eq, flags.p, s_);
    select_rows(flags.p, R_);
  }

  // The fused intersection N_x(x) ∩ N_y(y) of an expansion x → t and a closing check y → t iterates
  // the shorter list and binary-searches the longer one. On simple adjacencies with no target filter
  // on the expansion the result rows are the same either way (no multiplicity, the check's own filter
  // applies to t on both sides), so rows are split by which list is shorter and each group runs the
  // fused kernel with its roles in that order. E_t stays the reference's: Σ|N_x(x)| for the hop and
  // Σ|N_x(x)|·|N_y(y)| for the check (k_swap_flags).
  bool swap_ok(const Step &ex, const Step &ck) const {
    return swap_ && !dist_ && ex.filter_bm < 0 && ex.adj.parts.size() == 1 && ck.adj.parts.size() == 1 &&
           ex.adj.dup_free && ck.adj.dup_free && ex.adj.sorted && ck.adj.sorted;
  }
  void expand_check_swapped(const Step &ex, const Step &ck, bool write) {
    require_u32_rows("a cycle-closing intersection");
    const std::vector<int> cols = bound_cols();  // carried columns (ex.dst is not bound yet)
    bound_[ex.dst] = 1;
    const uint64_t R = R_;
    const int ix = (int)(std::find(cols.begin(), cols.end(), ex.src) - cols.begin());
    const int iy = (int)(std::find(cols.begin(), cols.end(), ck.src) - cols.begin());
    DBuf<uint8_t> fl(&pool_, R);
    DBuf<unsigned long long> sums(&pool_, 2);
    HIP_CHECK(hipMemsetAsync(sums.p, 0, 2 * sizeof(unsigned long long), s_));
    launch_swap_flags(col_[ex.src].p, col_[ck.src].p, R, make_adj(ex.adj), make_adj(ck.adj), fl.p, sums.p, cus(), s_);
    // swapped rows first, the others after them (reversed: order is irrelevant)
    DBuf<uint32_t> idx(&pool_, R);
    DBuf<uint64_t> nsel(&pool_, 1);
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    cub([&](void *t, size_t &b) { return hipcub::DevicePartition::Flagged(t, b, cnt, fl.p, idx.p, nsel.p, (int64_t)R, s_); });
    const uint64_t *words[3] = {reinterpret_cast<const uint64_t *>(sums.p), reinterpret_cast<const uint64_t *>(sums.p) + 1,
                                nsel.p};
    launch_post_ptrs(words, 3, mail(), s_);  // (the sums and the swapped count in one round trip)
    const uint64_t *h = wait_mail();
    edges_ += h[0] + h[1];
    const uint64_t nsw = h[2];
    ExpandOut og[2];
    const uint64_t gn[2] = {nsw, R - nsw};
    const uint32_t *gi[2] = {idx.p, idx.p + nsw};
    const uint64_t *cfilter = bitmap(ck.filter_bm);
    for (int g = 0; g < 2; ++g) {
      if (gn[g] == 0) continue;
      std::vector<DBuf<uint32_t>> gc;
      std::vector<const uint32_t *> in, carry;
      std::vector<uint32_t *> out;
      for (int c : cols) {
        gc.emplace_back(&pool_, gn[g]);
        in.push_back(col_[c].p);
        out.push_back(gc.back().p);
      }
      launch_gather_cols(gi[g], gn[g], (int)cols.size(), in.data(), out.data(), s_);
      for (auto &b : gc) carry.push_back(b.p);
      // (left block-segmented: both groups are compacted straight into one table below)
      if (g == 0)  // |N_x(x)| > |N_y(y)|: iterate N_y(y), probe N_x(x)
        og[g] = expand_core(gc[iy].p, gn[g], ck.adj, nullptr, carry, write, write, gc[ix].p, &ex.adj, cfilter);
      else
        og[g] = expand_core(gc[ix].p, gn[g], ex.adj, nullptr, carry, write, write, gc[iy].p, &ck.adj, cfilter);
    }
    edges_iter_ += og[0].E + og[1].E;  // the iterated lists (the probed ones are binary-searched)
    R_ = og[0].n + og[1].n;
    if (!write || R_ == 0) return;
    segmented_ = false;
    // each group's segments compacted into its part of one table (round 6: the groups' compactions into
    // their own buffers and a concatenation of every column cost 47 µs more at C4)
    std::vector<DBuf<uint32_t>> cat;
    for (size_t i = 0; i <= cols.size(); ++i) cat.emplace_back(&pool_, R_);
    uint64_t base = 0;
    for (int g = 0; g < 2; ++g) {
      ExpandOut &o = og[g];
      if (!o.n) continue;
      std::vector<uint32_t *> ins, outs;
      for (size_t i = 0; i <= cols.size(); ++i) {
        ins.push_back(i < cols.size() ? o.carry[i].p : o.dst.p);
        outs.push_back(cat[i].p + base);
      }
      tm_.begin("k_compact_segments");
      launch_compact_segments((int)ins.size(), ins.data(), outs.data(), o.seg_start.p, o.seg_count.p, o.seg_offs.p, o.nseg, s_);
      tm_.end(8ull * ins.size() * o.n);
      base += o.n;
    }
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(cat[i]);
    col_[ex.dst] = std::move(cat.back());
  }

  // The fused intersection N_x(x) ∩ N_y(y) with a merge path (isect.hip) for the rows whose lists have
  // comparable lengths; the other rows probe: the shorter list iterated, the longer binary-searched
  // (swapped only where that yields the same rows, see swap_ok), as expand_check_swapped. One part on
  // each side, sorted rows, one GPU; the expansion's target filter and parallel edges are allowed (the
  // merge keeps N_x's multiplicity, N_y is existence).
  bool isect_ok(const Step &ex, const Step &ck) const {
    return merge_ && !dist_ && ex.adj.parts.size() == 1 && ck.adj.parts.size() == 1 && ex.adj.sorted && ck.adj.sorted;
  }
  void expand_check_isect(const Step &ex, const Step &ck, bool write) {
    require_u32_rows("a cycle-closing intersection");
    const std::vector<int> cols = bound_cols();  // carried columns (ex.dst is not bound yet)
    bound_[ex.dst] = 1;
    const uint64_t R = R_;
    const int ix = (int)(std::find(cols.begin(), cols.end(), ex.src) - cols.begin());
    const int iy = (int)(std::find(cols.begin(), cols.end(), ck.src) - cols.begin());
    const DAdj ax = make_adj(ex.adj), ay = make_adj(ck.adj);
    const uint64_t *xfilter = bitmap(ex.filter_bm), *yfilter = bitmap(ck.filter_bm);
    IsectPolicy pol{};
    pol.merge = 1;
    pol.force = merge_ == 2;
    pol.swap = swap_ok(ex, ck);
    pol.dup_free = ex.adj.dup_free;
    pol.ratio = merge_ratio_;
    // 1. each row's class, the E_t sums and the class sizes
    DBuf<uint8_t> cls(&pool_, std::max<uint64_t>(R, 1));
    DBuf<uint32_t> w(&pool_, std::max<uint64_t>(R, 1)), bnd(&pool_, std::max<uint64_t>(R, 1));
    DBuf<unsigned long long> sums(&pool_, 6);
    HIP_CHECK(hipMemsetAsync(sums.p, 0, 6 * sizeof(unsigned long long), s_));
    tm_.begin("k_isect_class");
    launch_isect_class(col_[ex.src].p, col_[ck.src].p, R, ax.p[0], ay.p[0], pol, cls.p, w.p, bnd.p, sums.p, cus(), s_);
    tm_.end(R * (8ull + 32ull + 9ull));
    launch_post_words(sums.p, 6, mail(), s_);
    const uint64_t *hm = wait_mail();
    const uint64_t hopE = hm[0], checkE = hm[1], nc[4] = {hm[2], hm[3], hm[4], hm[5]};
    // 2. rows grouped by class (stable: each group keeps the row order)
    DBuf<uint32_t> idx(&pool_, std::max<uint64_t>(R, 1));
    if (R) {
      DBuf<uint32_t> iota(&pool_, R);
      DBuf<uint8_t> scls(&pool_, R);
      launch_iota(iota.p, R, s_);
      cub([&](void *t, size_t &b) { return sort_pairs(t, b, cls.p, scls.p, iota.p, idx.p, R, 2, s_); });
    }
    const uint64_t nM = nc[1];
    const uint32_t *gi[3] = {idx.p + nc[0], idx.p + nc[0] + nc[1], idx.p + nc[0] + nc[1] + nc[2]};
    // 3. the merged rows
    uint64_t medges = 0, nmerged = 0, wtotal = 0;
    DBuf<uint32_t> mdst;
    std::vector<DBuf<uint32_t>> mcarry;
    if (nM) {
      DBuf<uint32_t> wm(&pool_, nM + 1), bm(&pool_, nM + 1);
      launch_gather_u32(w.p, gi[0], nM, wm.p, s_);
      launch_gather_u32(bnd.p, gi[0], nM, bm.p, s_);
      DBuf<uint64_t> woff(&pool_, nM + 1), boff(&pool_, nM + 1), tot(&pool_, 2);
      HIP_CHECK(hipMemsetAsync(wm.p + nM, 0, 4, s_));
      HIP_CHECK(hipMemsetAsync(bm.p + nM, 0, 4, s_));
      hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> w64(wm.p, CastU64()), b64(bm.p, CastU64());
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, w64, woff.p, (int64_t)(nM + 1), s_); });
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, b64, boff.p, (int64_t)(nM + 1), s_); });
      HIP_CHECK(hipMemcpyAsync(tot.p, woff.p + nM, 8, hipMemcpyDeviceToDevice, s_));
      HIP_CHECK(hipMemcpyAsync(tot.p + 1, boff.p + nM, 8, hipMemcpyDeviceToDevice, s_));
      const auto wb = read2(tot.p);
      wtotal = wb.first - (uint64_t)kIsRowPad * nM;  // the list entries the merge reads
      const uint64_t cap = wb.second, ntiles = isect_tiles(wb.first);
      if (ntiles > 0xFFFFFFFFull) unsupported("a merged intersection of 2^32 or more tiles");
      DBuf<uint32_t> trow(&pool_, ntiles + 1), segc(&pool_, std::max<uint64_t>(ntiles, 1));
      DBuf<uint64_t> segs(&pool_, std::max<uint64_t>(ntiles, 1));
      DBuf<unsigned long long> ctr(&pool_, 2);
      HIP_CHECK(hipMemsetAsync(ctr.p, 0, 2 * sizeof(unsigned long long), s_));
      launch_isect_tiles(woff.p, nM, ntiles, trow.p, s_);
      DBuf<uint64_t> pa(&pool_, nM), pb(&pool_, nM);
      DBuf<uint32_t> pmn(&pool_, nM);
      launch_isect_prep(gi[0], nM, col_[ex.src].p, col_[ck.src].p, ax.p[0], ay.p[0], pa.p, pb.p, pmn.p, s_);
      IsectArgs a{};
      a.idx = gi[0];
      a.pa = pa.p;
      a.pb = pb.p;
      a.pmn = pmn.p;
      a.boff = boff.p;
      a.tile_row = trow.p;
      a.nM = nM;
      a.ntiles = ntiles;
      a.xs = col_[ex.src].p;
      a.ys = col_[ck.src].p;
      a.ax = ax.p[0];
      a.ay = ay.p[0];
      a.xfilter = xfilter;
      a.yfilter = yfilter;
      a.counters = ctr.p;
      a.seg_count = segc.p;
      a.seg_start = segs.p;
      DBuf<uint32_t> odst;
      std::vector<DBuf<uint32_t>> ocar;
      if (write) {
        odst = DBuf<uint32_t>(&pool_, std::max<uint64_t>(cap, 1));
        a.out_dst = odst.p;
        a.ncarry = (int32_t)cols.size();
        for (size_t c = 0; c < cols.size(); ++c) {
          ocar.emplace_back(&pool_, std::max<uint64_t>(cap, 1));
          a.carry_in[c] = col_[cols[c]].p;
          a.carry_out[c] = ocar.back().p;
        }
      }
      tm_.begin("k_isect_merge");
      launch_isect_merge(a, write, cus(), s_);
      // per merged row: its index, x and y, two row_ptr pairs; its lists; 4 B × columns per written row
      // (amended below)
      tm_.end(nM * 44ull + 4ull * wtotal);
      const size_t rec = tm_.last();
      if (write) {
        DBuf<uint64_t> soffs(&pool_, ntiles + 1);
        launch_seg_totals(segc.p, ntiles, ntiles, soffs.p, ctr.p, 0, 0, mail(), s_);
        const uint64_t *mw = wait_mail();
        nmerged = mw[1];
        medges = mw[2];
        mdst = DBuf<uint32_t>(&pool_, std::max<uint64_t>(nmerged, 1));
        std::vector<uint32_t *> ins{odst.p}, outs{mdst.p};
        for (size_t c = 0; c < cols.size(); ++c) {
          mcarry.emplace_back(&pool_, std::max<uint64_t>(nmerged, 1));
          ins.push_back(ocar[c].p);
          outs.push_back(mcarry.back().p);
        }
        tm_.begin("k_compact_segments");
        launch_compact_segments((int)ins.size(), ins.data(), outs.data(), segs.p, segc.p, soffs.p, (uint32_t)ntiles, s_);
        tm_.end(8ull * ins.size() * nmerged);
      } else {
        const auto mr = read2(reinterpret_cast<const uint64_t *>(ctr.p));
        medges = mr.first;
        nmerged = mr.second;
      }
      tm_.amend_at(rec, nM * 44ull + 4ull * wtotal + 4ull * (cols.size() + 1) * (write ? nmerged : 0));
    }
    // 4. the probed rows: class 2 iterates N_x(x) and probes N_y(y), class 3 the other way round
    ExpandOut og[2];
    const uint64_t gn[2] = {nc[2], nc[3]};
    for (int g = 0; g < 2; ++g) {
      if (gn[g] == 0) continue;
      std::vector<DBuf<uint32_t>> gc;
      std::vector<const uint32_t *> in, carry;
      std::vector<uint32_t *> out;
      for (int c : cols) {
        gc.emplace_back(&pool_, gn[g]);
        in.push_back(col_[c].p);
        out.push_back(gc.back().p);
      }
      launch_gather_cols(gi[1 + g], gn[g], (int)cols.size(), in.data(), out.data(), s_);
      for (auto &b : gc) carry.push_back(b.p);
      if (g == 0)
        og[g] = expand_core(gc[ix].p, gn[g], ex.adj, xfilter, carry, write, false, gc[iy].p, &ck.adj, yfilter);
      else  // (swapped rows exist only without an expansion filter: swap_ok)
        og[g] = expand_core(gc[iy].p, gn[g], ck.adj, nullptr, carry, write, false, gc[ix].p, &ex.adj, yfilter);
    }
    // E_t: Σ|N_x(x)| for the hop, and for the check Σ|N_y(y)| over the hop's rows that
    // reach it — every N_x entry without an expansion filter, else the entries passing it (counted by the
    // merge kernel and the probing kernels)
    edges_ += hopE + (xfilter ? medges + og[0].E_member : checkE);
    edges_iter_ += wtotal + og[0].E + og[1].E;  // the merged lists (both read) and the iterated lists
    R_ = nmerged + og[0].n + og[1].n;
    if (!write || R_ == 0) return;
    segmented_ = false;
    // the three groups back to back
    auto cat3 = [&](DBuf<uint32_t> *parts[3], const uint64_t *ns) {
      const uint64_t n = ns[0] + ns[1] + ns[2];
      for (int k = 0; k < 3; ++k)
        if (ns[k] == n) return std::move(*parts[k]);
      DBuf<uint32_t> o(&pool_, n);
      uint64_t at = 0;
      for (int k = 0; k < 3; ++k) {
        if (ns[k]) HIP_CHECK(hipMemcpyAsync(o.p + at, parts[k]->p, ns[k] * 4, hipMemcpyDeviceToDevice, s_));
        at += ns[k];
      }
      return o;
    };
    const uint64_t ns[3] = {nmerged, og[0].n, og[1].n};
    for (size_t i = 0; i < cols.size(); ++i) {
      DBuf<uint32_t> e0, e1, e2;
      DBuf<uint32_t> *parts[3] = {nmerged ? &mcarry[i] : &e0, og[0].n ? &og[0].carry[i] : &e1, og[1].n ? &og[1].carry[i] : &e2};
      col_[cols[i]] = cat3(parts, ns);
    }
    DBuf<uint32_t> e0, e1, e2;
    DBuf<uint32_t> *parts[3] = {nmerged ? &mdst : &e0, og[0].n ? &og[0].dst : &e1, og[1].n ? &og[1].dst : &e2};
    col_[ex.dst] = cat3(parts, ns);
  }

  // The rows (…, n) of a set-valued hop (Step::distinct_nb) over an adjacency that may repeat a neighbour:
  // one row per distinct (input row, n) — rid is the input row index carried through the expansion.
  // Radix sort of the packed pairs, run heads, then every column (rid and dst included) gathered.
  // Returns the rows kept.
  uint64_t distinct_pairs(DBuf<uint32_t> &rid, DBuf<uint32_t> &dst, std::vector<DBuf<uint32_t> *> others, uint64_t n) {
    if (n <= 1) return n;
    const int vb = std::max(bits_for(g_.V), bits_for(n));  // (rid < n, dst ≤ V: both below 2^32)
    tm_.begin("distinct_pairs");
    DBuf<uint64_t> keys(&pool_, n), skeys(&pool_, n);
    std::vector<DBuf<uint32_t>> kc;
    kc.push_back(std::move(rid));
    kc.push_back(std::move(dst));
    const uint64_t R0 = R_;
    R_ = n;  // pack_tuple reads R_ rows
    pack_tuple(kc, 2, vb, keys.p);
    R_ = R0;
    rid = std::move(kc[0]);
    dst = std::move(kc[1]);
    DBuf<uint32_t> iota(&pool_, n), perm(&pool_, n);
    launch_iota(iota.p, n, s_);
    cub([&](void *t, size_t &b) { return sort_pairs(t, b, keys.p, skeys.p, iota.p, perm.p, n, 2 * vb, s_); });
    DBuf<uint8_t> head(&pool_, n);
    launch_u64_heads(skeys.p, n, head.p, s_);
    DBuf<uint32_t> sel(&pool_, n);
    DBuf<uint64_t> nsel(&pool_, 1);
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, perm.p, head.p, sel.p, nsel.p, (int64_t)n, s_); });
    const uint64_t m = read1(nsel.p);
    others.push_back(&dst);
    others.push_back(&rid);
    std::vector<DBuf<uint32_t>> nc;
    std::vector<const uint32_t *> in;
    std::vector<uint32_t *> out;
    for (DBuf<uint32_t> *c : others) {
      nc.emplace_back(&pool_, std::max<uint64_t>(m, 1));
      in.push_back(c->p);
      out.push_back(nc.back().p);
    }
    launch_gather_cols(sel.p, m, (int)in.size(), in.data(), out.data(), s_);
    for (size_t i = 0; i < others.size(); ++i) *others[i] = std::move(nc[i]);
    tm_.end(n * 40ull + m * 8ull * others.size());
    return m;
  }

  // keep the rows whose flag is set (all bound columns)
  void select_rows(const uint8_t *flags, uint64_t R) {
    if (R == 0) {  // (a partitioned rank without rows: nothing to select)
      R_ = 0;
      return;
    }
    require_u32_rows("a row selection");
    DBuf<uint32_t> idx(&pool_, R);
    DBuf<uint64_t> nsel(&pool_, 1);
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, cnt, flags, idx.p, nsel.p, (int64_t)R, s_); });
    const uint64_t n = read1(nsel.p);
    gather_rows(idx.p, n);
  }

  void gather_rows(const uint32_t *idx, uint64_t n) {
    std::vector<int> cols = bound_cols();
    for (int c : cols)
      if (!col_[c].p && R_) fail(OMX_E_INVALID, "internal: bound column " + p_.aliases[c] + " is not materialized");
    std::vector<DBuf<uint32_t>> nc;
    std::vector<const uint32_t *> in;
    std::vector<uint32_t *> out;
    for (int c : cols) {
      nc.emplace_back(&pool_, std::max<uint64_t>(n, 1));
      in.push_back(col_[c].p);
      out.push_back(nc.back().p);
    }
    tm_.begin("k_gather_cols");
    launch_gather_cols(idx, n, (int)cols.size(), in.data(), out.data(), s_);
    tm_.end(n * (4 + 8ull * cols.size()));
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(nc[i]);
    R_ = n;
  }

  // S_EXPAND (x → t) followed by S_CHECK (y → t, t bound by the expansion): the check keeps a row iff
  // t ∈ N(y), which a sorted adjacency answers by binary search inside the expansion kernels
  bool fuse_ok(const Step &ex, const Step &ck) const {
    if (fuse_mode_ == "0" || dist_) return false;  // partitioned: N(y) of the check may live on another rank
    if (ck.kind != S_CHECK || ck.dst != ex.dst || ck.src == ex.dst || !col_[ck.src].p) return false;
    if (ex.optional || ck.optional) return false;
    if (!ck.adj.sorted || ck.adj.parts.empty()) return false;
    if (ex.distinct_nb && !ex.adj.dup_free) return false;  // the expansion's neighbours form a set first
    return true;
  }

  uint64_t degree_sum(const uint32_t *src, uint64_t R, const AdjSpec &adjs, const DAdj *raw_adj = nullptr) {
    DAdj adj = raw_adj ? *raw_adj : make_adj(adjs);
    if (adj.n == 0 || R == 0) return 0;
    DBuf<uint64_t> deg(&pool_, R + 1), sum(&pool_, 1);
    tm_.begin("k_row_degree");
    launch_row_degree(src, R, adj, deg.p, s_);
    tm_.end(R * (4ull + 8ull * adj.n + 8ull));  // source id + row_ptr pair per part, 8-B degree written
    cub([&](void *t, size_t &b) { return hipcub::DeviceReduce::Sum(t, b, deg.p, sum.p, (int64_t)(R + 1), s_); });
    return read1(sum.p);
  }

  void check_step(const Step &st) {
    route_owner(st.src);
    if (R_ == 0) return;  // (a partitioned rank with no local rows after the exchange)
    const uint64_t R = R_;
    const uint64_t E = degree_sum(col_[st.src].p, R, st.adj);
    edges_ += E;
    if (st.optional) {  // a bound optional target not reached becomes null; no row is dropped
      DBuf<unsigned int> npe(&pool_, 1);
      HIP_CHECK(hipMemsetAsync(npe.p, 0, 4, s_));
      launch_check_optional(col_[st.src].p, col_[st.dst].p, R, make_adj(st.adj), bitmap(st.where_bm), g_.V, npe.p, s_);
      if (read1(npe.p))
        fail(OMX_E_EXECUTION, "NullPointerException: optional alias " + p_.aliases[st.dst] + " is null and reached again");
      return;
    }
    DBuf<uint8_t> flags(&pool_, R);
    tm_.begin("k_check");
    launch_check(col_[st.src].p, col_[st.dst].p, R, make_adj(st.adj), bitmap(st.filter_bm), flags.p, s_);
    // 8 B row_ptr pair + 4 B per binary-search probe
    const double avg = R ? (double)E / (double)R : 0.0;
    const uint64_t kb = 8 * R + 4 * R * (uint64_t)std::ceil(std::log2(avg + 1.0) + 1.0);
    tm_.end(kb);
    alg_bytes_ += kb;
    select_rows(flags.p, R);
  }

  void cross_step(const Step &st) {
    uint64_t nc = 0;
    DBuf<uint32_t> cand = bitmap_list(bitmap(st.cand_bm), 0, 1, nc);
    std::vector<int> cols = bound_cols();
    const uint64_t n = R_ * nc;
    std::vector<DBuf<uint32_t>> ncol;
    std::vector<const uint32_t *> in;
    std::vector<uint32_t *> out;
    for (int c : cols) {
      ncol.emplace_back(&pool_, std::max<uint64_t>(n, 1));
      in.push_back(col_[c].p);
      out.push_back(ncol.back().p);
    }
    DBuf<uint32_t> dst(&pool_, std::max<uint64_t>(n, 1));
    tm_.begin("k_cross");
    launch_cross(R_, (int)cols.size(), in.data(), out.data(), cand.p, nc, dst.p, s_);
    tm_.end(n * 4 * (cols.size() + 1));
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(ncol[i]);
    col_[st.dst] = std::move(dst);
    R_ = n;
  }

  // sorted unique u64 keys
  uint64_t sort_unique_keys(DBuf<uint64_t> &keys, uint64_t n, int end_bit = 64) {
    if (n == 0) return 0;
    DBuf<uint64_t> sorted(&pool_, n), uniq(&pool_, n), nsel(&pool_, 1);
    cub([&](void *t, size_t &b) {
      return sort_keys(t, b, keys.p, sorted.p, n, end_bit, s_);
    });
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Unique(t, b, sorted.p, uniq.p, nsel.p, (int64_t)n, s_); });
    uint64_t m = read1(nsel.p);
    keys = std::move(uniq);
    return m;
  }

  static int bits_for(uint64_t x) {
    int b = 1;
    while (b < 64 && (1ull << b) <= x) ++b;
    return b;
  }

  // Variable-length edge (while / maxDepth), OMatchPathItem.executeTraversal (P/OMatchPathItem.java:79-105):
  // level-synchronous over (row, vertex) pairs; level d keeps F_d ∩ where_d, expands F_d ∩ while_d
  // while d < maxDepth. Without $depth in where/while a visited set per row is exact and
  // terminates on cycles.
  void varlen_step(const Step &st) {
    bool depth_only_while = false;
    // partitioned: the multi-source BFS with the frontier blocks allgathered every level (a free or
    // candidate target, ≤ BfsCarry::kMax bound columns, few batches as below), else (row, vertex) pairs
    // routed to the owner of their vertex every level
    if (dist_ && varlen_mode_ != "pairs" && bfs_exact(st, depth_only_while) && st.mode != T_BOUND &&
        bound_cols().size() <= (size_t)BfsCarry::kMax) {
      const uint64_t nb = (global_sum(R_) + 63) / 64;  // the same choice on every rank
      if (varlen_mode_ == "bfs" || nb <= 64 || nb * (uint64_t)g_.V <= (1ull << 30)) {
        varlen_msbfs(st, depth_only_while);
        return;
      }
    }
    if (!dist_ && varlen_mode_ != "pairs" && bfs_exact(st, depth_only_while)) {
      const uint64_t nb = (R_ + 63) / 64;
      if (varlen_mode_ == "bfs" || nb <= 64 || nb * (uint64_t)g_.V <= (1ull << 30)) {
        varlen_msbfs(st, depth_only_while);
        return;
      }
    }
    varlen_pairs(st);
  }

  // The walk semantics of P/OMatchPathItem.java:79-105 equal BFS distance (bfs.hip) when WHERE does not
  // read $depth and `while` either does not read $depth or reads nothing else (then it is a constant
  // per level: the first depth where it is false ends the expansion).
  bool bfs_exact(const Step &st, bool &depth_only_while) const {
    if (st.where_prog >= 0 && p_.progs[st.where_prog].uses_depth) return false;
    depth_only_while = false;
    if (st.while_prog < 0 || !p_.progs[st.while_prog].uses_depth) return true;
    const PredProgram &w = p_.progs[st.while_prog];
    for (const auto &in : w.code)
      if (in.op == P_PUSH_COL || in.op == P_PUSH_DEG) return false;
    depth_only_while = true;
    return true;
  }

  // binding-row indices are u32 in the gathers, selects and (row, vertex) pair keys
  void require_u32_rows(const char *what) const {
    if (R_ >= (1ull << 32))
      unsupported(std::string(what) + " over 2^32 or more binding rows (u32 row indices)");
  }

  // Multi-source BFS over 64-row batches (bfs.hip). Rows (row, v) come out distinct per row.
  void varlen_msbfs(const Step &st, bool depth_only_while) {
    require_u32_rows("a variable-length item");
    // the pull kernels read bit 31 of an in-CSR entry as a hub tag (pull_col_of), and the partitioned
    // pull reads the raw col: ids must stay below 2^31 (checked before any exchange: V is replicated)
    if (g_.V >= 0x80000000u) unsupported("variable-length traversal over 2^31 or more vertices");
    uint64_t R = R_;
    const uint32_t V = g_.V;
    // Partitioned (SURVEY §8(e) "Variable-length: ... when the frontier is dense, an allgather"): every
    // rank runs every 64-row batch of the global rows, whose bound columns are first gathered to every
    // rank; prep, pull and visited cover the rank's own vertices [vlo, vhi), whose in-CSR rows it
    // holds, and each level's frontier blocks are allgathered so that the pull reads any in-neighbour's
    // mask. Every level pulls (per vertex, early exit). A rank emits the rows of its own vertices (the
    // rows then live at owner(dst)).
    const std::vector<int> bcols = bound_cols();
    const uint32_t *srcc = col_[st.src].p;
    std::vector<const uint32_t *> cin;
    for (int c : bcols) cin.push_back(col_[c].p);
    std::vector<DBuf<uint32_t>> grow;
    std::vector<uint64_t> plo, phi;
    uint32_t vlo = 0, vhi = V;
    if (dist_) {
      const int W = tr_->world(), me = tr_->rank();
      const std::vector<uint64_t> g3 = tr_->allgather_n({R_, g_.part_lo, g_.part_hi}, s_);
      std::vector<uint64_t> rs(W);
      plo.assign(W, 0);
      phi.assign(W, 0);
      for (int p = 0; p < W; ++p) {
        rs[p] = g3[3 * p];
        plo[p] = g3[3 * p + 1];
        phi[p] = g3[3 * p + 2];
      }
      vlo = g_.part_lo;
      vhi = g_.part_hi;
      std::vector<uint64_t> send(W, R_), sdispl(W, 0), recv(rs), rdispl(W, 0);
      R = 0;
      for (int p = 0; p < W; ++p) {
        rdispl[p] = R;
        R += rs[p];
      }
      if (R >= (1ull << 32)) unsupported("a partitioned variable-length item over 2^32 or more rows");
      std::vector<const uint32_t *> sb;
      std::vector<uint32_t *> rb;
      DBuf<uint32_t> dummy(&pool_, 1);
      for (size_t k = 0; k < bcols.size(); ++k) {
        grow.emplace_back(&pool_, std::max<uint64_t>(R, 1));
        sb.push_back(R_ ? col_[bcols[k]].p : dummy.p);
        rb.push_back(grow.back().p);
      }
      tm_.begin("exchange");
      tr_->alltoallv(sb, send, sdispl, rb, recv, rdispl, s_);
      tm_.end(4ull * bcols.size() * (R_ * W + R));
      (void)me;
      for (size_t k = 0; k < bcols.size(); ++k) {
        cin[k] = grow[k].p;
        if (bcols[k] == st.src) srcc = grow[k].p;
      }
      if (!R) {
        for (int c : bcols) col_[c] = DBuf<uint32_t>(&pool_, 1);
        col_[st.dst] = DBuf<uint32_t>(&pool_, 1);
        R_ = 0;
        owner_col_ = st.dst;
        return;
      }
    }
    const DAdj adj = make_adj(st.adj);
    AdjSpec rspec = st.adj;
    for (auto &p : rspec.parts) p.second ^= 1;
    const DAdj radj = make_adj(rspec);
    uint64_t eadj = 0;
    for (const auto &p : st.adj.parts) eadj += g_.esets[p.first].n_edges;
    // emission bitmap = WHERE (depth-free) ∧ candidates (prefetched target)
    DBuf<uint64_t> emit;
    const uint64_t *emit_bm = nullptr;
    if (st.where_prog >= 0) {
      emit = DBuf<uint64_t>(&pool_, nwords_);
      eval_bitmap(st.where_prog, -1, 0, emit.p);
      emit_bm = emit.p;
    }
    if (st.mode == T_CAND) {
      const uint64_t *c = bitmap(st.cand_bm);
      if (emit_bm) launch_bitmap_and(c, emit.p, nwords_, s_);
      else emit_bm = c;
    }
    DBuf<uint64_t> wbm;
    const uint64_t *while_bm = nullptr;
    DPred wconst{};
    if (st.while_prog >= 0 && !depth_only_while) {
      wbm = DBuf<uint64_t>(&pool_, nwords_);
      eval_bitmap(st.while_prog, -1, 0, wbm.p);
      while_bm = wbm.p;
    }
    const bool while_never = depth_only_while && p_.progs[st.while_prog].const_false;
    if (depth_only_while) wconst = make_pred(st.while_prog, -1);
    DBuf<uint64_t> fr(&pool_, V), nx(&pool_, V), vis(&pool_, V), fbm(&pool_, nwords_);
    DBuf<uint32_t> list;
    // the level prologue's six words (k_bfs_prep) and, in stats[6], the push level's list counter
    DBuf<unsigned long long> stats(&pool_, 7);
    // bottom-up partitions of every reversed part (once per traversal; built on the first pull level)
    std::vector<DBuf<uint64_t>> hub_fr(radj.n);
    // sparse levels pull over the hub entries only and push the non-hub frontier (one GPU, one part): the
    // hubs' V-bit set lets the level prologue count that frontier and its out-edges (OMX_HUB_PUSH=0: off)
    const uint64_t *hub_bm = nullptr;
    if (!dist_ && pull_wave_ && hub_push_ && radj.n == 1) {
      uint32_t nh = 0;
      const uint32_t *hb = nullptr;
      pull_col_of(rspec.parts[0].first, rspec.parts[0].second, &nh, &hb, &hub_bm);
      if (!nh) hub_bm = nullptr;
    }
    std::vector<const uint64_t *> pull_part(radj.n, nullptr);
    std::vector<const uint32_t *> pull_col(radj.n, nullptr), pull_hubs(radj.n, nullptr);
    std::vector<uint32_t> pull_nh(radj.n, 0);
    std::vector<uint64_t> pull_E(radj.n);
    for (int p = 0; p < radj.n; ++p) pull_E[p] = g_.esets[rspec.parts[p].first].n_edges;
    DBuf<uint32_t> rest;  // dense pull levels: vertices left to the per-wave pass
    DBuf<unsigned long long> exit_counts;
    std::vector<size_t> exit_recs;  // their timer records
    DBuf<uint8_t> bflags;
    if (st.mode == T_BOUND) bflags = DBuf<uint8_t>(&pool_, R);
    const unsigned nb = bfs_blocks(V);
    DBuf<uint32_t> blk(&pool_, nb);
    DBuf<uint64_t> blk_offs(&pool_, nb + 1);
    std::vector<DBuf<uint32_t>> orow, ov;
    std::vector<uint64_t> on;
    // up to BfsCarry::kMax bound columns are written by the emission itself (no row gather after it)
    const bool carry = bcols.size() <= (size_t)BfsCarry::kMax;
    std::vector<std::vector<DBuf<uint32_t>>> oc(carry ? bcols.size() : 0);
    uint64_t ntotal = 0;
    // sparse level prologues (bfs.hip k_bfs_prep_sparse): after a push level, the vertices its atomics
    // touched first are the next level's only candidates; the level's active lists ping-pong between two
    // slots (the previous level's list clears its bits while this level's is written); lcnt = {touched,
    // slot 0, slot 1} counts, on the device
    const bool sparse_ok = sparse_prep_ && !dist_ && vlo == 0 && vhi == V;
    // a push of fewer than V / kSparsePrepDiv edges records what it touches (at most that many vertices):
    // the next prologue visits those at a few random words each instead of sweeping V
    const uint64_t kSparsePrepDiv = sparse_div_;
    DBuf<uint32_t> touched, act[2];
    DBuf<unsigned long long> lcnt;
    if (sparse_ok) {
      touched = DBuf<uint32_t>(&pool_, V);
      act[0] = DBuf<uint32_t>(&pool_, V);
      act[1] = DBuf<uint32_t>(&pool_, V);
      lcnt = DBuf<unsigned long long>(&pool_, 3);
    }
    for (uint64_t row0 = 0; row0 < R; row0 += 64) {
      const int nl = (int)std::min<uint64_t>(64, R - row0);
      // the previous level: a push with its touched list (t_bound ≥ its length: the push's edges) and its
      // active list in act[prev_slot] (prev_n vertices)
      bool t_ok = false;
      uint64_t t_bound = 0, prev_n = 0;
      int prev_slot = -1;
      const uint64_t lanes = nl == 64 ? ~0ull : ((1ull << nl) - 1);
      // (one GPU: visited is zeroed by the first level's prologue, which covers every vertex)
      const bool whole = !dist_ && vlo == 0 && vhi == V;
      HIP_CHECK(hipMemsetAsync(fr.p, 0, (size_t)V * 8, s_));
      if (!whole) HIP_CHECK(hipMemsetAsync(vis.p, 0, (size_t)V * 8, s_));
      if (sparse_ok) {
        // the first level's prologue over the distinct seeds: visited, the next masks and the frontier
        // bitmap zeroed by memsets (write-only streams) instead of the full sweep that also reads the frontier
        HIP_CHECK(hipMemsetAsync(lcnt.p, 0, 3 * sizeof(unsigned long long), s_));
        launch_bfs_seed(srcc, row0, nl, fr.p, s_, touched.p, lcnt.p);
        HIP_CHECK(hipMemsetAsync(vis.p, 0, (size_t)V * 8, s_));
        HIP_CHECK(hipMemsetAsync(nx.p, 0, (size_t)V * 8, s_));
        HIP_CHECK(hipMemsetAsync(fbm.p, 0, (size_t)nwords_ * 8, s_));
        t_ok = true;
        t_bound = (uint64_t)nl;
        prev_slot = 0;  // (slot 0's count is 0: nothing to clear)
        prev_n = 0;
      } else {
        launch_bfs_seed(srcc, row0, nl, fr.p, s_);
      }
      const uint64_t *last = nullptr;  // a final level left unmerged: the emission merges it into visited
      for (int64_t d = 0;; ++d) {
        if (d > 100000) fail(OMX_E_EXECUTION, "variable-length traversal did not terminate");
        bool expand = !(st.has_max_depth && d >= st.max_depth);
        if (expand && depth_only_while) expand = !while_never && eval_pred_const(wconst, d);
        // a level that does not expand only merges its frontier into visited: with one GPU the emission's
        // counting pass does that (one sweep of V fewer); a sparse one still runs over its short list
        // (visited must hold something by then: a previous level's prologue, or the sparse first level's
        // memset — a batch's first full prologue is what writes it)
        if (!expand && whole && (d > 0 || sparse_ok) &&
            !(sparse_ok && t_ok && prev_slot >= 0 && t_bound * kSparsePrepDiv < (uint64_t)V)) {
          last = fr.p;
          break;
        }
        HIP_CHECK(hipMemsetAsync(stats.p, 0, 7 * sizeof(unsigned long long), s_));
        // (one GPU: the prologue zeroes the next level's masks as it streams the frontier, no memset)
        const bool zero_nx = whole;
        const bool sparse = sparse_ok && t_ok && prev_slot >= 0 && (d == 0 || t_bound * kSparsePrepDiv < (uint64_t)V);
        int cur_slot = -1;  // this level's active list, when the sparse prologue wrote it
        if (sparse) {
          cur_slot = prev_slot ^ 1;
          HIP_CHECK(hipMemsetAsync(lcnt.p + 1 + cur_slot, 0, sizeof(unsigned long long), s_));
          tm_.begin("k_bfs_prep_sparse");
          launch_bfs_prep_sparse(act[prev_slot].p, lcnt.p + 1 + prev_slot, touched.p, lcnt.p,
                                 std::max<uint64_t>(t_bound, prev_n), fr.p, vis.p, while_bm, expand, adj, stats.p, fbm.p,
                                 hub_bm, nx.p, act[cur_slot].p, lcnt.p + 1 + cur_slot, cus(), s_);
          tm_.end(12ull * prev_n + 40ull * t_bound);
        } else {
          tm_.begin("k_bfs_prep");
          launch_bfs_prep(fr.p, vis.p, vhi, while_bm, expand, adj, stats.p, dist_ ? nullptr : fbm.p, cus(), s_, vlo, hub_bm,
                          zero_nx ? nx.p : nullptr, whole && d == 0, d == 0);
          tm_.end(8ull * (vhi - vlo));
        }
        t_ok = false;
        if (!expand) break;
        launch_post_words(stats.p, 6, mail(), s_);
        const uint64_t *hm = wait_mail();
        uint64_t h[6] = {hm[0], hm[1], hm[2], hm[3], hm[4], hm[5]};
        // frontier scan + visited and row_ptr pair of the active vertices (sparse: the touched list's)
        if (!sparse) tm_.amend(8ull * (vhi - vlo) + 24ull * h[2]);
        uint64_t live_or = h[3];
        uint64_t active = h[2];
        std::vector<uint64_t> al;
        if (dist_) {  // every rank continues while any rank has an active vertex; live lanes over all ranks
          al = tr_->allgather_n({h[2], h[3]}, s_);
          active = 0;
          live_or = 0;
          for (int p = 0; p < tr_->world(); ++p) {
            active += al[2 * p];
            live_or |= al[2 * p + 1];
          }
          if (active == 0) break;
        } else if (h[2] == 0) {
          break;
        }
        // lanes with an empty frontier receive nothing at this level (OMX_PULL_LIVE=0: wait for all lanes)
        const uint64_t live = pull_live_ ? live_or : ~0ull;
        // E_t: the frontier's adjacency summed per row (lane); edges_iter_ counts the adjacency entries the
        // level's kernels actually read (push: the frontier's out-edges once for all lanes; tiled pull:
        // every in-edge; early-exit pull: the in-edges walked, added when the traversal ends)
        edges_ += h[0];
        if (!zero_nx) HIP_CHECK(hipMemsetAsync(nx.p, 0, (size_t)V * 8, s_));
        if (debug_expand_)
          std::fprintf(stderr, "[omx bfs] batch %llu level %lld: %s active=%llu push_edges=%llu E_t=%llu\n",
                       (unsigned long long)row0, (long long)d, (double)h[1] * pull_div_ > (double)eadj ? "pull" : "push",
                       (unsigned long long)h[2], (unsigned long long)h[1], (unsigned long long)h[0]);
        if (dist_) {
          const int W = tr_->world(), me = tr_->rank();
          if (12 * active < (uint64_t)V && !dense_exchange_) {
            // a sparse level: every rank sends its frontier vertices with their masks (12 B each) to every
            // peer instead of its whole block (8 B per owned vertex); the peers' entries of fr are zero
            // before they are scattered in (a rank's pull writes only its own vertices)
            const uint64_t n = h[2];
            DBuf<uint32_t> lv(&pool_, std::max<uint64_t>(n, 1)), mlo(&pool_, std::max<uint64_t>(n, 1)),
                mhi(&pool_, std::max<uint64_t>(n, 1));
            DBuf<unsigned long long> lc(&pool_, 1);
            HIP_CHECK(hipMemsetAsync(lc.p, 0, sizeof(unsigned long long), s_));
            if (n) launch_bfs_list(fr.p + vlo, vhi - vlo, lv.p, lc.p, cus(), s_);
            launch_bfs_frontier_pack(lv.p, n, vlo, fr.p, mlo.p, mhi.p, s_);
            std::vector<uint64_t> send(W, n), sdispl(W, 0), recv(W), rdispl(W);
            uint64_t nr = 0;
            for (int p = 0; p < W; ++p) {
              recv[p] = p == me ? 0 : al[2 * p];
              rdispl[p] = nr;
              nr += recv[p];
            }
            send[me] = 0;
            DBuf<uint32_t> rv(&pool_, std::max<uint64_t>(nr, 1)), rlo(&pool_, std::max<uint64_t>(nr, 1)),
                rhi(&pool_, std::max<uint64_t>(nr, 1));
            tm_.begin("exchange");
            tr_->alltoallv({lv.p, mlo.p, mhi.p}, send, sdispl, {rv.p, rlo.p, rhi.p}, recv, rdispl, s_);
            tm_.end(12ull * (n * (W - 1) + nr));
            if (vlo) HIP_CHECK(hipMemsetAsync(fr.p, 0, (size_t)vlo * 8, s_));
            if (vhi < V) HIP_CHECK(hipMemsetAsync(fr.p + vhi, 0, (size_t)(V - vhi) * 8, s_));
            launch_bfs_frontier_scatter(rv.p, rlo.p, rhi.p, nr, fr.p, s_);
          } else {
            // the frontier blocks of every rank (u64 masks sent as u32 word pairs; nothing to itself)
            std::vector<uint64_t> send(W, 2ull * (vhi - vlo)), sdispl(W, 0), recv(W), rdispl(W);
            for (int p = 0; p < W; ++p) {
              recv[p] = 2ull * (phi[p] - plo[p]);
              rdispl[p] = 2ull * plo[p];
            }
            send[me] = recv[me] = 0;
            tm_.begin("exchange");
            tr_->alltoallv({reinterpret_cast<const uint32_t *>(fr.p + vlo)}, send, sdispl,
                           {reinterpret_cast<uint32_t *>(fr.p)}, recv, rdispl, s_);
            tm_.end(8ull * V);
          }
          for (int p = 0; p < radj.n; ++p) {
            if (!rest.p) {
              rest = DBuf<uint32_t>(&pool_, V);
              exit_counts = DBuf<unsigned long long>(&pool_, 2);
              HIP_CHECK(hipMemsetAsync(exit_counts.p, 0, sizeof(unsigned long long), s_));
            }
            HIP_CHECK(hipMemsetAsync(exit_counts.p + 1, 0, sizeof(unsigned long long), s_));
            tm_.begin("k_bfs_pull_exit");
            // a partition's col has no hub tags (pull_col_of): the hub array is never read
            launch_bfs_pull_exit(vhi, radj.p[p].rp, radj.p[p].col, lanes & live, fr.p, fr.p, vis.p, nx.p, rest.p,
                                 exit_counts.p, cus(), s_, vlo);
            tm_.end(32ull * (vhi - vlo));
            if (tm_.last() != SIZE_MAX) exit_recs.push_back(tm_.last());
          }
        } else if ((double)h[1] * pull_div_ > (double)eadj) {
          for (int p = 0; p < radj.n; ++p) {
            const uint64_t nt = bfs_pull_tiles(V, pull_E[p]);
            if (!pull_part[p]) {
              pull_part[p] = pull_part_of(rspec.parts[p].first, rspec.parts[p].second, radj.p[p].rp, pull_E[p], nt);
              pull_col[p] = pull_col_of(rspec.parts[p].first, rspec.parts[p].second, &pull_nh[p], &pull_hubs[p]);
              hub_fr[p] = DBuf<uint64_t>(&pool_, std::max<uint32_t>(pull_nh[p], 1));
            }
            launch_hub_gather(pull_hubs[p], pull_nh[p], fr.p, hub_fr[p].p, s_);
            const bool probe = (double)h[2] < pull_probe_ * (double)V;
            if (!probe && pull_exit_) {
              // dense level: per-vertex walks that stop once the needed lanes are covered
              if (!rest.p) {
                rest = DBuf<uint32_t>(&pool_, V);
                exit_counts = DBuf<unsigned long long>(&pool_, 2);
                HIP_CHECK(hipMemsetAsync(exit_counts.p, 0, sizeof(unsigned long long), s_));
              }
              HIP_CHECK(hipMemsetAsync(exit_counts.p + 1, 0, sizeof(unsigned long long), s_));
              tm_.begin("k_bfs_pull_exit");
              launch_bfs_pull_exit(V, radj.p[p].rp, pull_col[p], lanes & live, fr.p, hub_fr[p].p, vis.p, nx.p, rest.p,
                                   exit_counts.p, cus(), s_);
              // per vertex: row_ptr pair + visited + next; per in-edge read: col + the source's frontier mask
              // (exit_counts[0] sums the in-edges read over the traversal; added once it has ended)
              tm_.end(32ull * V);
              if (tm_.last() != SIZE_MAX) exit_recs.push_back(tm_.last());
              continue;
            }
            // A sparse level whose frontier is mostly hubs (C3's third level: 1.2 K of its 54 M non-hub
            // in-edges come from frontier vertices) gathers masks for the hub entries only — a non-hub entry
            // costs its col word, no frontier-bitmap probe — and the non-hub frontier (h[5] vertices, h[4]
            // out-edges: counted by the prologue, no host round trip) pushes its out-edges instead, when
            // those are under 1/8 of the level's in-edges
            bool hubs_only = false;
            if (probe && hub_bm && (hub_push_ == 2 || h[4] * 8 < pull_E[p])) {
              hubs_only = true;
              const uint64_t nn = h[5], etot = h[4];
              if (etot) {
                if (!list.p) list = DBuf<uint32_t>(&pool_, V);
                DBuf<unsigned long long> nc(&pool_, 1);
                HIP_CHECK(hipMemsetAsync(nc.p, 0, sizeof(unsigned long long), s_));
                tm_.begin("k_bfs_list");
                launch_bfs_list_nonhub(fbm.p, hub_bm, V, list.p, nc.p, cus(), s_);
                tm_.end(V / 4);
                DBuf<uint64_t> deg(&pool_, nn + 1), loffs(&pool_, nn + 1);
                launch_bfs_list_deg(list.p, nn, adj.p[p].rp, deg.p, s_);
                cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, deg.p, loffs.p, (int64_t)(nn + 1), s_); });
                tm_.begin("k_bfs_push");
                launch_bfs_push(list.p, loffs.p, nn, etot, adj.p[p].rp, adj.p[p].col, fr.p, vis.p, nx.p, cus(), s_);
                tm_.end(20ull * etot + 24ull * nn);
                edges_iter_ += etot;
              }
            }
            // (hubs-only: the tiles run over the hub entries' own CSR, EdgeSet::d_hub_rp / d_hub_col)
            const HubCsr hc = hubs_only ? hub_csr_of(rspec.parts[p].first, rspec.parts[p].second) : HubCsr{};
            tm_.begin(probe ? "k_bfs_pull_sparse" : "k_bfs_pull");
            if (hubs_only && hc.col) {
              launch_bfs_pull_w(hc.rp, hc.col, hc.E, hc.tiles, hc.nreg, hc.rb, lanes & live, fr.p, hub_fr[p].p,
                                pull_nh[p], nullptr, vis.p, nx.p, cus(), s_, true);
            } else if (pull_wave_) {  // wave tiles over the in-edges
              const uint64_t *wrb = nullptr;
              uint64_t nreg = 0;
              const uint32_t *wt = pullw_of(rspec.parts[p].first, rspec.parts[p].second, radj.p[p].rp, pull_E[p], &wrb, &nreg);
              launch_bfs_pull_w(radj.p[p].rp, pull_col[p], pull_E[p], wt, nreg, wrb, lanes & live, fr.p, hub_fr[p].p,
                                pull_nh[p], probe && !hubs_only ? fbm.p : nullptr, vis.p, nx.p, cus(), s_, hubs_only);
            } else {
              launch_bfs_pull(V, radj.p[p].rp, pull_col[p], pull_part[p], pull_E[p], lanes & live, fr.p, hub_fr[p].p,
                              probe ? fbm.p : nullptr, vis.p, nx.p, cus(), s_);
            }
            // per vertex: row_ptr pair + visited (+ next); per in-edge: col + the source's frontier mask.
            // HBM-necessary: the masks are shared by all the in-edges of a source, so each is needed once
            // (probe levels: the frontier's masks and the frontier bitmap; else every vertex's mask)
            // (hubs-only over the hub CSR: its col words and a mask per entry)
            const uint64_t pe = hubs_only && hc.col ? hc.E : pull_E[p];
            tm_.end(16ull * V + 12ull * pe, 16ull * V + 4ull * pe + (probe ? 8ull * h[2] + (hubs_only ? 0 : V / 8) : 8ull * V));
            edges_iter_ += pe;
          }
        } else {
          // the level's active vertices: the sparse prologue's list, or a sweep of the frontier (into the
          // slot the previous level's list does not hold, with its count on the device for the next clear)
          const uint32_t *lp;
          int slot = -1;
          if (cur_slot >= 0) {
            slot = cur_slot;
            lp = act[slot].p;
          } else if (sparse_ok) {
            slot = prev_slot == 0 ? 1 : 0;
            HIP_CHECK(hipMemsetAsync(lcnt.p + 1 + slot, 0, sizeof(unsigned long long), s_));
            tm_.begin("k_bfs_list");
            launch_bfs_list(fr.p, V, act[slot].p, lcnt.p + 1 + slot, cus(), s_);
            tm_.end(8ull * V + 4ull * h[2]);
            lp = act[slot].p;
          } else {
            if (!list.p) list = DBuf<uint32_t>(&pool_, V);
            tm_.begin("k_bfs_list");
            launch_bfs_list(fr.p, V, list.p, stats.p + 6, cus(), s_);
            tm_.end(8ull * V + 4ull * h[2]);
            lp = list.p;
          }
          const uint64_t nl_act = h[2];
          if (sparse_ok) HIP_CHECK(hipMemsetAsync(lcnt.p, 0, sizeof(unsigned long long), s_));
          uint64_t pushed = 0;
          bool rec = false;  // this push records its touched list (a small push: the next prologue is sparse)
          DBuf<uint64_t> deg(&pool_, nl_act + 1), loffs(&pool_, nl_act + 1);
          for (int p = 0; p < adj.n; ++p) {
            launch_bfs_list_deg(lp, nl_act, adj.p[p].rp, deg.p, s_);
            cub([&](void *t, size_t &b) {
              return hipcub::DeviceScan::ExclusiveSum(t, b, deg.p, loffs.p, (int64_t)(nl_act + 1), s_);
            });
            // (one part: the prologue's Σ deg over the active vertices is this scan's total — no read-back)
            const uint64_t etot = adj.n == 1 ? h[1] : read1(loffs.p + nl_act);
            rec = sparse_ok && adj.n == 1 && etot * kSparsePrepDiv < (uint64_t)V;
            tm_.begin("k_bfs_push");
            launch_bfs_push(lp, loffs.p, nl_act, etot, adj.p[p].rp, adj.p[p].col, fr.p, vis.p, nx.p, cus(), s_,
                            rec ? touched.p : nullptr, rec ? lcnt.p : nullptr);
            // per frontier edge: col + visited + next (+ row_ptr and frontier mask per listed vertex)
            tm_.end(20ull * etot + 24ull * nl_act);
            edges_iter_ += etot;
            pushed += etot;
          }
          if (rec) {  // the next level runs its prologue over what this push touched
            t_ok = true;
            t_bound = pushed;
            prev_slot = slot;
            prev_n = nl_act;
          }
        }
        std::swap(fr, nx);
      }
      if (st.mode == T_BOUND) {
        launch_bfs_bound(col_[st.dst].p, row0, nl, vis.p, emit_bm, bflags.p, s_, last);
        continue;
      }
      tm_.begin("k_bfs_emit");
      launch_bfs_emit_count(vis.p, emit_bm, V, blk.p, s_, last);
      HIP_CHECK(hipMemsetAsync(blk_offs.p, 0, 8, s_));
      hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> bit(blk.p, CastU64());
      cub([&](void *t, size_t &b) { return hipcub::DeviceScan::InclusiveSum(t, b, bit, blk_offs.p + 1, (int64_t)nb, s_); });
      const uint64_t n = read1(blk_offs.p + nb);
      if (n) {
        BfsCarry cc;
        cc.nl = (uint32_t)nl;
        if (carry) {
          cc.n = (int)bcols.size();
          for (size_t k = 0; k < bcols.size(); ++k) {
            oc[k].emplace_back(&pool_, n);
            cc.in[k] = cin[k];
            cc.out[k] = oc[k].back().p;
          }
        } else {
          orow.emplace_back(&pool_, n);
        }
        ov.emplace_back(&pool_, n);
        on.push_back(n);
        launch_bfs_emit_write(vis.p, emit_bm, V, blk_offs.p, (uint32_t)row0, carry ? nullptr : orow.back().p,
                              ov.back().p, cc, s_);
        ntotal += n;
      }
      // visited + emission bitmap scans (two passes) + 4 B per written column per row
      tm_.end(16ull * V + 4ull * n * (carry ? bcols.size() + 1 : 2));
    }
    if (exit_counts.p) {
      const uint64_t walked = read1(exit_counts.p);
      edges_iter_ += walked;
      if (!exit_recs.empty()) tm_.amend_at(exit_recs[0], 32ull * (vhi - vlo) + 12ull * walked);
    }
    if (dist_) owner_col_ = st.dst;  // the rows were emitted by the owners of their new vertex
    if (st.mode == T_BOUND) {
      select_rows(bflags.p, R);
      return;
    }
    if (carry) {
      for (size_t k = 0; k < bcols.size(); ++k) col_[bcols[k]] = concat_batches(oc[k], on, ntotal);
      R_ = ntotal;
    } else {
      DBuf<uint32_t> rrow = concat_batches(orow, on, ntotal);
      gather_rows(rrow.p, ntotal);
    }
    col_[st.dst] = concat_batches(ov, on, ntotal);
  }

  // one column from per-batch pieces (moved when there is one piece)
  DBuf<uint32_t> concat_batches(std::vector<DBuf<uint32_t>> &parts, const std::vector<uint64_t> &n, uint64_t total) {
    if (parts.size() == 1) return std::move(parts[0]);
    DBuf<uint32_t> out(&pool_, std::max<uint64_t>(total, 1));
    uint64_t off = 0;
    for (size_t i = 0; i < parts.size(); ++i) {
      HIP_CHECK(hipMemcpyAsync(out.p + off, parts[i].p, n[i] * 4, hipMemcpyDeviceToDevice, s_));
      off += n[i];
    }
    parts.clear();
    return out;
  }

  // ---- (row, vertex) pair sets: the general traversal (any $depth use, multi items) -----------------
  // A pair set holds, per binding row, the set of vertices an item's executeTraversal returned so far
  // (P/OMatchPathItem.java:49-107): distinct (row, v) pairs, kept as two u32 columns. Sets of rows with
  // the same start vertex are the same, so per-row sets equal the reference's per-start-vertex HashSets.

  int pair_key_bits() const { return 32 + bits_for(g_.V); }

  // distinct (row, v) pairs of n packed keys (sorted)
  PairSet pairs_from_keys(DBuf<uint64_t> &keys, uint64_t n, bool unique_sorted = false) {
    PairSet o;
    if (!unique_sorted) n = sort_unique_keys(keys, n, pair_key_bits());
    o.n = n;
    o.row = DBuf<uint32_t>(&pool_, std::max<uint64_t>(n, 1));
    o.v = DBuf<uint32_t>(&pool_, std::max<uint64_t>(n, 1));
    if (n) launch_unpack_pairs(keys.p, n, o.row.p, o.v.p, s_);
    return o;
  }
  DBuf<uint64_t> pair_keys(const PairSet &p) {
    DBuf<uint64_t> k(&pool_, std::max<uint64_t>(p.n, 1));
    if (p.n) launch_pack_pairs(p.row.p, p.v.p, p.n, k.p, s_);
    return k;
  }
  // the pairs whose vertex is in bitmap bm
  PairSet filter_pairs(const PairSet &in, const uint64_t *bm) {
    if (!bm || in.n == 0) {
      DBuf<uint64_t> k = pair_keys(in);
      return pairs_from_keys(k, in.n, true);
    }
    DBuf<uint8_t> flags(&pool_, in.n);
    launch_flag_bitmap(in.v.p, in.n, bm, flags.p, s_);
    DBuf<uint64_t> all = pair_keys(in), sel(&pool_, in.n), nsel(&pool_, 1);
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, all.p, flags.p, sel.p, nsel.p, (int64_t)in.n, s_); });
    return pairs_from_keys(sel, read1(nsel.p), true);  // a subsequence of sorted keys stays sorted
  }
  // bitmap of a predicate program at $depth = depth (cached when it does not read $depth)
  std::map<int, DBuf<uint64_t>> prog_bms_;
  // (padded: a traversal's WHERE bitmap filters expansions, so the sliced kernels may stage it)
  const uint64_t *prog_bitmap(int prog, int64_t depth, DBuf<uint64_t> &scratch) {
    if (prog < 0) return nullptr;
    if (p_.progs[prog].uses_depth) {
      if (!scratch.p) scratch = DBuf<uint64_t>(&pool_, padded_words());
      eval_bitmap(prog, -1, depth, scratch.p, padded_words());
      return scratch.p;
    }
    DBuf<uint64_t> &b = prog_bms_[prog];
    if (!b.p) {
      b = DBuf<uint64_t>(&pool_, padded_words());
      eval_bitmap(prog, -1, 0, b.p, padded_words());
    }
    return b.p;
  }

  // one hop of a single-method item over a pair set (target bitmap optional), distinct pairs out
  PairSet hop_pairs(const PairSet &in_, const AdjSpec &adj, const uint64_t *filter) {
    const PairSet *in = &in_;
    PairSet routed;
    if (dist_) {  // expand where the vertex's rows are; new pairs meet at their vertex's owner for the dedup
      DBuf<uint64_t> k = pair_keys(in_);
      routed = pairs_from_keys(k, in_.n, true);
      route_pairs_owner(routed);
      in = &routed;
    }
    if (in->n == 0 && !dist_) return PairSet{};
    ExpandOut ex = in->n ? expand_core(in->v.p, in->n, adj, filter, {in->row.p}, true) : ExpandOut{};
    edges_ += ex.E;
    edges_iter_ += ex.E;
    PairSet out;
    if (ex.n) {
      out.n = ex.n;
      out.row = std::move(ex.carry[0]);
      out.v = std::move(ex.dst);
    }
    route_pairs_owner(out);
    if (out.n == 0) return PairSet{};
    DBuf<uint64_t> keys = pair_keys(out);
    return pairs_from_keys(keys, out.n);
  }

  // traversePatternEdge of an item (P/OMatchPathItem.java:109-126): the neighbour set without the
  // item's own filter; a multi item composes its sub-items (P/OMultiMatchPathItem.java:41-61)
  PairSet pattern_edge(const TravSpec &t, const PairSet &in) {
    if (!t.multi) return hop_pairs(in, t.adj, nullptr);
    PairSet cur;
    {
      DBuf<uint64_t> k = pair_keys(in);
      cur = pairs_from_keys(k, in.n, true);
    }
    for (const TravSpec &sub : t.subs) {
      if (global_sum(cur.n) == 0) break;
      cur = traverse(sub, cur);
    }
    return cur;
  }

  // executeTraversal (P/OMatchPathItem.java:49-107) from every pair's vertex at depth 0
  PairSet traverse(const TravSpec &t, const PairSet &in) {
    DBuf<uint64_t> where_scratch, while_scratch;
    if (!t.varlen) {  // one level; the item's WHERE filters the neighbours (a HashSet, :63-78)
      const uint64_t *w = prog_bitmap(t.where_prog, 0, where_scratch);
      if (!t.multi) return hop_pairs(in, t.adj, w);
      PairSet n = pattern_edge(t, in);
      return filter_pairs(n, w);
    }
    // level-synchronous: level d keeps F_d ∩ where_d and expands F_d ∩ while_d while d < maxDepth.
    // Without $depth in where/while the per-row visited set is exact and terminates on cycles.
    const bool dep = (t.where_prog >= 0 && p_.progs[t.where_prog].uses_depth) ||
                     (t.while_prog >= 0 && p_.progs[t.while_prog].uses_depth);
    const int kb = pair_key_bits();
    PairSet F;
    {
      DBuf<uint64_t> k = pair_keys(in);
      F = pairs_from_keys(k, in.n, true);
    }
    DBuf<uint64_t> visited;
    uint64_t nvisited = 0;
    if (!dep) {
      visited = pair_keys(F);
      nvisited = F.n;
    }
    std::vector<DBuf<uint64_t>> res_parts;
    std::vector<uint64_t> res_n;
    for (int64_t d = 0; global_sum(F.n); ++d) {
      if (d > 100000) fail(OMX_E_EXECUTION, "variable-length traversal did not terminate (the reference recurses without bound)");
      {  // include F_d ∩ where_d
        PairSet inc = filter_pairs(F, prog_bitmap(t.where_prog, d, where_scratch));
        if (inc.n) {
          res_parts.push_back(pair_keys(inc));
          res_n.push_back(inc.n);
        }
      }
      if (t.has_max_depth && d >= t.max_depth) break;
      PairSet G = filter_pairs(F, prog_bitmap(t.while_prog, d, while_scratch));  // F_d ∩ while_d
      if (global_sum(G.n) == 0) break;
      PairSet N = pattern_edge(t, G);
      if (!dep && N.n) {  // drop the pairs seen at an earlier level
        DBuf<uint64_t> keys = pair_keys(N);
        DBuf<uint8_t> flags(&pool_, N.n);
        launch_flag_not_in(visited.p, nvisited, keys.p, N.n, flags.p, s_);
        DBuf<uint64_t> fresh(&pool_, N.n), nsel(&pool_, 1);
        cub([&](void *tt, size_t &b) { return hipcub::DeviceSelect::Flagged(tt, b, keys.p, flags.p, fresh.p, nsel.p, (int64_t)N.n, s_); });
        const uint64_t nk = read1(nsel.p);
        if (nk) {
          DBuf<uint64_t> merged(&pool_, nvisited + nk);
          HIP_CHECK(hipMemcpyAsync(merged.p, visited.p, nvisited * 8, hipMemcpyDeviceToDevice, s_));
          HIP_CHECK(hipMemcpyAsync(merged.p + nvisited, fresh.p, nk * 8, hipMemcpyDeviceToDevice, s_));
          nvisited = sort_unique_keys(merged, nvisited + nk, kb);
          visited = std::move(merged);
        }
        N = pairs_from_keys(fresh, nk, true);
      }
      F = std::move(N);
    }
    // union of the levels' results (HashSet union, P/OMatchPathItem.java:61,96-101)
    uint64_t total = 0;
    for (auto n : res_n) total += n;
    DBuf<uint64_t> res(&pool_, std::max<uint64_t>(total, 1));
    uint64_t off = 0;
    for (size_t i = 0; i < res_parts.size(); ++i) {
      HIP_CHECK(hipMemcpyAsync(res.p + off, res_parts[i].p, res_n[i] * 8, hipMemcpyDeviceToDevice, s_));
      off += res_n[i];
    }
    return pairs_from_keys(res, total);
  }

  // the binding rows' start pairs (row index, source vertex)
  // (partitioned: row ids are global, rank r's rows from row_bounds_[r]; pairs are routed to the owners
  // of their vertices by the hops and back to the rows' ranks by bind_pairs)
  std::vector<uint64_t> row_bounds_;
  PairSet start_pairs(int src) {
    require_u32_rows("a variable-length or multi-step item");
    uint64_t base = 0;
    if (dist_) {
      const std::vector<uint64_t> rs = tr_->allgather(R_, s_);
      row_bounds_.assign(rs.size() + 1, 0);
      for (size_t p = 0; p < rs.size(); ++p) row_bounds_[p + 1] = row_bounds_[p] + rs[p];
      if (row_bounds_.back() >= (1ull << 32)) unsupported("a partitioned variable-length item over 2^32 or more rows");
      base = row_bounds_[tr_->rank()];
    }
    PairSet p;
    p.n = R_;
    p.row = DBuf<uint32_t>(&pool_, std::max<uint64_t>(R_, 1));
    p.v = DBuf<uint32_t>(&pool_, std::max<uint64_t>(R_, 1));
    launch_iota(p.row.p, R_, s_);
    launch_add_u32(p.row.p, R_, (int64_t)base, s_);
    if (R_) HIP_CHECK(hipMemcpyAsync(p.v.p, col_[src].p, R_ * 4, hipMemcpyDeviceToDevice, s_));
    return p;
  }

  // processContext's three branches (:468-497) over an item's (row, v) result set
  void bind_pairs(const Step &st, PairSet &res) {
    if (dist_) {  // the result pairs return to the ranks of their rows (local row ids)
      const int W = tr_->world();
      DBuf<uint32_t> dest(&pool_, std::max<uint64_t>(res.n, 1));
      DBuf<uint64_t> hist(&pool_, W);
      HIP_CHECK(hipMemsetAsync(hist.p, 0, W * sizeof(uint64_t), s_));
      if (res.n) launch_route_bounds(res.row.p, res.n, row_bounds_.data(), (uint32_t)W, dest.p, hist.p, s_);
      res.n = exchange_cols({&res.row, &res.v}, res.n, dest, hist);
      launch_add_u32(res.row.p, res.n, -(int64_t)row_bounds_[tr_->rank()], s_);
      DBuf<uint64_t> k = pair_keys(res);
      res = pairs_from_keys(k, res.n);  // sorted again (bound targets are looked up by binary search)
      owner_col_ = -1;                  // the rows are back on their own ranks
    }
    const uint64_t R = R_;
    if (st.mode == T_BOUND) {  // keep a row iff its bound target is in its set (existence)
      DBuf<uint64_t> rk = pair_keys(res);
      DBuf<uint32_t> idx(&pool_, std::max<uint64_t>(R, 1));
      launch_iota(idx.p, R, s_);
      DBuf<uint64_t> keys(&pool_, std::max<uint64_t>(R, 1));
      launch_pack_pairs(idx.p, col_[st.dst].p, R, keys.p, s_);
      DBuf<uint8_t> flags(&pool_, std::max<uint64_t>(R, 1)), keep(&pool_, std::max<uint64_t>(R, 1));
      launch_flag_not_in(rk.p, res.n, keys.p, R, flags.p, s_);
      invert_flags(flags.p, keep.p, R);
      select_rows(keep.p, R);
      return;
    }
    if (st.mode == T_CAND) res = filter_pairs(res, bitmap(st.cand_bm));
    gather_rows(res.row.p, res.n);  // (before dst is marked bound: gather_rows moves the bound columns)
    col_[st.dst] = std::move(res.v);
    bound_[st.dst] = 1;
  }

  // variable-length item over (row, vertex) pairs (any $depth use)
  void varlen_pairs(const Step &st) {
    TravSpec t;
    t.adj = st.adj;
    t.varlen = true;
    t.where_prog = st.where_prog;
    t.while_prog = st.while_prog;
    t.has_max_depth = st.has_max_depth;
    t.max_depth = st.max_depth;
    PairSet res = traverse(t, start_pairs(st.src));
    bind_pairs(st, res);
  }

  // multi-step item .( ... ) (OMultiMatchPathItem)
  void multi_step(const Step &st) {
    PairSet res = traverse(st.trav, start_pairs(st.src));
    bind_pairs(st, res);
  }

  void invert_flags(const uint8_t *in, uint8_t *out, uint64_t n) {
    if (!n) return;
    hipLaunchKernelGGL(k_invert_flags, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s_, in, out, n);
  }

  // Projection + distinct rows (addResult :661-729 → addToUniqueResult)
  void project_dedup(std::vector<DBuf<uint32_t>> &out, uint64_t &n) {
    n = R_;
    if (p_.proj == Plan::PROJ_ELEMENTS) {
      DBuf<uint64_t> bm(&pool_, nwords_);
      HIP_CHECK(hipMemsetAsync(bm.p, 0, nwords_ * 8, s_));
      tm_.begin("k_mark_bitmap");
      for (int a : p_.out_aliases) launch_mark_bitmap(col_[a].p, R_, bm.p, g_.V, s_);
      tm_.end(R_ * 4 * p_.out_aliases.size());
      uint64_t m = 0;
      out.push_back(bitmap_list(bm.p, 0, 1, m));
      n = m;
      dedup_ran_ = 1;
      return;
    }
    const int k = (int)p_.out_aliases.size();
    std::vector<int> taken(col_.size(), -1);
    for (int a : p_.out_aliases) {
      if (taken[a] < 0) {  // move the binding column (no copy); an alias returned twice is copied
        taken[a] = (int)out.size();
        out.push_back(std::move(col_[a]));
      } else {
        out.emplace_back(&pool_, R_);
        HIP_CHECK(hipMemcpyAsync(out.back().p, out[taken[a]].p, R_ * 4, hipMemcpyDeviceToDevice, s_));
      }
    }
    if (p_.unique_by_construction || marked_ || pre_distinct_) return;  // (marked_ / pre_distinct_: the rows are already the distinct set)
    bool may_null = false;
    for (int a : p_.out_aliases) may_null = may_null || p_.optional[a];
    n = distinct_rows(out, k, may_null);
  }

  // the distinct tuples of the k columns `out` (R_ rows each, rewritten in place); returns their count
  uint64_t distinct_rows(std::vector<DBuf<uint32_t>> &out, int k, bool may_null) {
    if (segmented_) fail(OMX_E_INVALID, "internal: segmented table reached dedup");
    uint64_t n = R_;
    dedup_ran_ = 1;
    tm_.begin("dedup");
    const int vbits = bits_for(g_.V);
    if (k == 1 && !may_null) {
      // one column: the distinct vertices are the set bits of a V-bit bitmap (no sort)
      DBuf<uint64_t> bm(&pool_, nwords_);
      HIP_CHECK(hipMemsetAsync(bm.p, 0, nwords_ * 8, s_));
      launch_mark_bitmap(out[0].p, R_, bm.p, g_.V, s_);
      uint64_t m = 0;
      DBuf<uint32_t> lst = bitmap_list(bm.p, 0, 1, m);
      out[0] = std::move(lst);
      n = m;
      tm_.end(R_ * 4 + nwords_ * 16 + m * 4);
      return n;
    }
    if (k <= 3 && k * vbits <= 64) {
      // pack the tuple into one u64 key
      DBuf<uint64_t> keys(&pool_, R_);
      pack_tuple(out, k, vbits, keys.p);
      n = sort_unique_keys(keys, R_, k * vbits);
      unpack_tuple(keys.p, n, out, k, vbits);
    } else {
      // LSD: stable radix sort of a row permutation by each column, last column first
      DBuf<uint32_t> order(&pool_, R_), order2(&pool_, R_), kin(&pool_, R_), kout(&pool_, R_);
      launch_iota(order.p, R_, s_);
      for (int c = k - 1; c >= 0; --c) {
        launch_gather_u32(out[c].p, order.p, R_, kin.p, s_);
        cub([&](void *t, size_t &b) {
          return sort_pairs(t, b, kin.p, kout.p, order.p, order2.p, R_, vbits, s_);
        });
        std::swap(order.p, order2.p);
      }
      std::vector<DBuf<uint32_t>> sorted;
      std::vector<const uint32_t *> sp;
      for (int c = 0; c < k; ++c) {
        sorted.emplace_back(&pool_, R_);
        launch_gather_u32(out[c].p, order.p, R_, sorted.back().p, s_);
        sp.push_back(sorted.back().p);
      }
      DBuf<uint8_t> flags(&pool_, R_);
      launch_flag_row_change(k, sp.data(), R_, flags.p, s_);
      DBuf<uint32_t> idx(&pool_, R_);
      DBuf<uint64_t> nsel(&pool_, 1);
      hipcub::CountingInputIterator<uint32_t> cnt(0);
      cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, cnt, flags.p, idx.p, nsel.p, (int64_t)R_, s_); });
      n = read1(nsel.p);
      for (int c = 0; c < k; ++c) launch_gather_u32(sorted[c].p, idx.p, n, out[c].p, s_);
    }
    tm_.end(R_ * 4ull * k * 4);
    return n;
  }

  void pack_tuple(std::vector<DBuf<uint32_t>> &cols, int k, int vbits, uint64_t *keys);
  void unpack_tuple(const uint64_t *keys, uint64_t n, std::vector<DBuf<uint32_t>> &cols, int k, int vbits);
};

__global__ void k_pack_tuple(const uint32_t *c0, const uint32_t *c1, const uint32_t *c2, int k, int vbits, uint64_t n,
                             uint64_t *keys) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t key = c0[i];
  if (k > 1) key = (key << vbits) | c1[i];
  if (k > 2) key = (key << vbits) | c2[i];
  keys[i] = key;
}
__global__ void k_unpack_tuple(const uint64_t *keys, uint64_t n, int k, int vbits, uint32_t *c0, uint32_t *c1,
                               uint32_t *c2) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t key = keys[i], m = (vbits >= 64) ? ~0ull : ((1ull << vbits) - 1);
  if (k > 2) { c2[i] = (uint32_t)(key & m); key >>= vbits; }
  if (k > 1) { c1[i] = (uint32_t)(key & m); key >>= vbits; }
  c0[i] = (uint32_t)key;
}

void Executor::pack_tuple(std::vector<DBuf<uint32_t>> &cols, int k, int vbits, uint64_t *keys) {
  if (k > 3) fail(OMX_E_INVALID, "pack_tuple: k > 3");
  uint64_t n = R_;
  hipLaunchKernelGGL(k_pack_tuple, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s_, cols[0].p,
                     k > 1 ? cols[1].p : nullptr, k > 2 ? cols[2].p : nullptr, k, vbits, n, keys);
}
void Executor::unpack_tuple(const uint64_t *keys, uint64_t n, std::vector<DBuf<uint32_t>> &cols, int k, int vbits) {
  if (!n) return;
  hipLaunchKernelGGL(k_unpack_tuple, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s_, keys, n, k, vbits, cols[0].p,
                     k > 1 ? cols[1].p : nullptr, k > 2 ? cols[2].p : nullptr);
}

}  // namespace

omx_result *execute_plan(Graph &g, const Plan &p, const omx_exec_options &opts, Transport *tr, bool *running) {
  if (running) *running = false;
  if (!g.on_device()) fail(OMX_E_DEVICE, "graph snapshot is host-only (device = -1)");
  HIP_CHECK(hipSetDevice(g.device));
  // a failure releases the peers waiting in an exchange with this rank: omx_execute (capi.cpp) aborts the
  // communicator unless the failure is a refusal of the plan or of its partition checks (the constructor:
  // the same statement and replicated schema on every rank, so every rank refused alike). Anything
  // raised once run() started may depend on this rank's own rows, so its peers must be released.
  Executor ex(g, p, opts, tr);
  if (running) *running = true;
  return ex.run();
}

}  // namespace omx
