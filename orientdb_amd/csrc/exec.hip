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

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>

#include "kernels.h"

namespace omx {
namespace {

struct CastU64 {
  __host__ __device__ uint64_t operator()(const uint32_t &x) const { return x; }
};

class Timer {
 public:
  Timer(bool on, hipStream_t s) : on_(on), s_(s) {}
  ~Timer() {
    for (auto &r : recs_) {
      (void)hipEventDestroy(r.a);
      (void)hipEventDestroy(r.b);
    }
  }
  void begin(const char *name, hipStream_t st = nullptr) {
    if (!on_) return;
    Rec r;
    r.name = name;
    r.s = st ? st : s_;
    HIP_CHECK(hipEventCreate(&r.a));
    HIP_CHECK(hipEventCreate(&r.b));
    HIP_CHECK(hipEventRecord(r.a, r.s));
    recs_.push_back(r);
  }
  void end(uint64_t bytes = 0) {
    if (!on_) return;
    recs_.back().bytes = bytes;
    HIP_CHECK(hipEventRecord(recs_.back().b, recs_.back().s));
  }
  void collect(std::vector<omx_result::KStat> &out) {
    if (!on_) return;
    HIP_CHECK(hipStreamSynchronize(s_));
    for (auto &r : recs_) {
      float ms = 0;
      HIP_CHECK(hipEventElapsedTime(&ms, r.a, r.b));
      auto it = std::find_if(out.begin(), out.end(), [&](const omx_result::KStat &k) { return k.name == r.name; });
      if (it == out.end()) {
        out.push_back({r.name, 0, 0, 0});
        it = out.end() - 1;
      }
      it->launches++;
      it->ms += ms;
      it->bytes += r.bytes;
    }
  }

 private:
  struct Rec {
    std::string name;
    hipEvent_t a, b;
    hipStream_t s;
    uint64_t bytes = 0;
  };
  bool on_;
  hipStream_t s_;
  std::vector<Rec> recs_;
};

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
  Executor(Graph &g, const Plan &p, const omx_exec_options &o)
      : g_(g), p_(p), o_(o), s_(g.stream), s2_(g.stream2), pool_(g.pool), tm_((o.flags & OMX_FLAG_KERNEL_TIMING) != 0, g.stream) {
    nwords_ = ((uint64_t)g.V + 63) / 64;
    // rows with at least this many neighbours take the chunked kernel (tests lower it to force the path)
    if (const char *h = std::getenv("OMX_HEAVY_DEG")) heavy_deg_ = std::max<uint64_t>(1, std::strtoull(h, nullptr, 10));
    bms_.resize(p.bitmaps.size());
    col_.resize(p.aliases.size());
  }

  omx_result *run() {
    auto t0 = std::chrono::steady_clock::now();
    auto res = std::make_unique<omx_result>();
    hipEvent_t ea, eb;
    HIP_CHECK(hipEventCreate(&ea));
    HIP_CHECK(hipEventCreate(&eb));
    HIP_CHECK(hipEventRecord(ea, s_));
    bool empty = p_.empty || !check_candidates();
    bool counted_only = false;
    if (!empty) {
      for (size_t i = 0; i < p_.steps.size() && R_ > 0; ++i) {
        const Step &st = p_.steps[i];
        bool last = i + 1 == p_.steps.size();
        bool count_only = last && o_.mode == OMX_MODE_COUNT && p_.unique_by_construction && st.kind == S_EXPAND;
        // the last expansion of a plan whose rows are distinct by construction may stay block-
        // segmented in HBM when the rows are not copied to the host
        bool seg_ok = last && p_.unique_by_construction && p_.proj == Plan::PROJ_ALIASES &&
                      (o_.flags & OMX_FLAG_KEEP_DEVICE);
        switch (st.kind) {
          case S_ROOT: root(st); break;
          case S_EXPAND: expand_step(st, !count_only, seg_ok); counted_only = count_only; break;
          case S_CHECK: check_step(st); break;
          case S_VARLEN: varlen_step(st); break;
          case S_NEWROOT:
          case S_CARTESIAN: cross_step(st); break;
          case S_KILL: R_ = 0; break;
        }
      }
      if (p_.steps.empty()) R_ = 0;
    } else {
      R_ = 0;
    }
    bindings_ = R_;
    uint64_t n = 0;
    int ncols = 0;
    std::vector<DBuf<uint32_t>> out;
    if (R_ > 0 && !counted_only) {
      project_dedup(out, n);
      ncols = (int)out.size();
    } else if (counted_only) {
      n = R_;
      ncols = (int)p_.out_aliases.size();
    }
    int64_t limit = p_.limit >= 0 ? p_.limit : o_.limit;
    if (limit > -1 && n > (uint64_t)std::max<int64_t>(limit, 1)) n = (uint64_t)std::max<int64_t>(limit, 1);
    if (n > 0 && !counted_only && !(o_.flags & OMX_FLAG_KEEP_DEVICE)) {
      DBuf<uint64_t> rids(&pool_, n * ncols);
      std::vector<const uint32_t *> cp;
      for (auto &c : out) cp.push_back(c.p);
      tm_.begin("k_map_rids");
      launch_map_rids(ncols, cp.data(), n, (o_.flags & OMX_FLAG_NO_RID_MAP) ? nullptr : g_.d_rids, rids.p, s_);
      tm_.end(n * ncols * 12);
      res->rows.resize(n * ncols);
      HIP_CHECK(hipMemcpyAsync(res->rows.data(), rids.p, n * ncols * sizeof(uint64_t), hipMemcpyDeviceToHost, s_));
    }
    HIP_CHECK(hipEventRecord(eb, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    float dms = 0;
    HIP_CHECK(hipEventElapsedTime(&dms, ea, eb));
    (void)hipEventDestroy(ea);
    (void)hipEventDestroy(eb);
    tm_.collect(res->kstats);
    res->info.n_rows = n;
    res->info.n_cols = n ? ncols : 0;
    res->info.deduplicated = dedup_ran_;
    res->info.edges_traversed = edges_;
    res->info.bindings = bindings_;
    res->info.alg_bytes = alg_bytes_;
    res->info.device_ms = dms;
    res->names = p_.out_names;
    res->info.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return res.release();
  }

 private:
  Graph &g_;
  const Plan &p_;
  omx_exec_options o_;
  hipStream_t s_, s2_;
  DevicePool &pool_;
  Timer tm_;
  uint64_t nwords_;
  std::vector<DBuf<uint64_t>> bms_;
  std::vector<DBuf<uint32_t>> col_;
  uint64_t R_ = 1;
  uint64_t edges_ = 0, alg_bytes_ = 0, bindings_ = 0;
  int dedup_ran_ = 0;
  int cus_ = 0;
  uint64_t heavy_deg_ = kHeavyDeg;
  bool segmented_ = false;  // the final table is block-segmented (see expand_core)

  // ---- helpers -----------------------------------------------------------------------------------
  template <class F>
  void cub(F f) {
    size_t bytes = 0;
    HIP_CHECK(f((void *)nullptr, bytes));
    DBuf<uint8_t> tmp(&pool_, std::max<size_t>(bytes, 16));
    HIP_CHECK(f((void *)tmp.p, bytes));
  }
  template <class T>
  T read1(const T *dptr) {
    T v;
    HIP_CHECK(hipMemcpyAsync(&v, dptr, sizeof(T), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    return v;
  }

  DAdj make_adj(const AdjSpec &a) const {
    DAdj d{};
    d.n = (int32_t)a.parts.size();
    d.sorted = a.sorted;
    for (size_t i = 0; i < a.parts.size(); ++i) {
      const EdgeSet &es = g_.esets[a.parts[i].first];
      d.p[i].rp = a.parts[i].second == 0 ? es.d_out_rp : es.d_in_rp;
      d.p[i].col = a.parts[i].second == 0 ? es.d_out_col : es.d_in_col;
    }
    return d;
  }

  DPred make_pred(int prog, int class_id) const {
    DPred d{};
    d.cols = g_.d_cols;
    d.vclass = g_.d_vclass;
    if (class_id >= 0) {
      d.use_class = 1;
      g_.class_mask(class_id, d.class_mask);
    }
    if (prog >= 0) {
      const PredProgram &pp = p_.progs[prog];
      d.n = (int32_t)pp.code.size();
      for (size_t i = 0; i < pp.code.size(); ++i) d.code[i] = pp.code[i];
      for (size_t i = 0; i < pp.deg.size(); ++i) d.deg[i] = make_adj(pp.deg[i]);
      match_atoms(pp, d);
    }
    return d;
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

  void eval_bitmap(int prog, int class_id, int64_t depth, uint64_t *words) {
    tm_.begin("k_eval_bitmap");
    if (prog >= 0 && p_.progs[prog].const_false) {
      HIP_CHECK(hipMemsetAsync(words, 0, nwords_ * 8, s_));
    } else {
      launch_eval_bitmap(make_pred(prog, class_id), g_.V, depth, words, s_);
    }
    tm_.end((uint64_t)g_.V * 4 + nwords_ * 8);
    alg_bytes_ += (uint64_t)g_.V * 4;
  }

  const uint64_t *bitmap(int id) {
    if (id < 0) return nullptr;
    if (!bms_[id].p) {
      bms_[id] = DBuf<uint64_t>(&pool_, nwords_);
      eval_bitmap(p_.bitmaps[id].prog, p_.bitmaps[id].class_id, 0, bms_[id].p);
    }
    return bms_[id].p;
  }

  uint64_t bitmap_count(const uint64_t *words, int rank, int world) {
    DBuf<uint32_t> cnt(&pool_, nwords_);
    launch_word_popc(words, nwords_, g_.V, rank, world, cnt.p, s_);
    DBuf<uint64_t> sum(&pool_, 1);
    hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> it(cnt.p, CastU64());
    cub([&](void *t, size_t &b) { return hipcub::DeviceReduce::Sum(t, b, it, sum.p, (int)nwords_, s_); });
    return read1(sum.p);
  }

  DBuf<uint32_t> bitmap_list(const uint64_t *words, int rank, int world, uint64_t &n) {
    DBuf<uint32_t> cnt(&pool_, nwords_ + 1);
    DBuf<uint32_t> offs(&pool_, nwords_ + 1);
    tm_.begin("k_bitmap_to_list");
    launch_word_popc(words, nwords_, g_.V, rank, world, cnt.p, s_);
    HIP_CHECK(hipMemsetAsync(cnt.p + nwords_, 0, 4, s_));
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, cnt.p, offs.p, (int)(nwords_ + 1), s_); });
    n = read1(offs.p + nwords_);
    DBuf<uint32_t> out(&pool_, std::max<uint64_t>(n, 1));
    launch_word_scatter(words, nwords_, g_.V, rank, world, offs.p, out.p, s_);
    tm_.end(nwords_ * 8 + n * 4);
    return out;
  }

  // calculateMatch (:340-357): an empty candidate set of a prefetched alias → empty result
  bool check_candidates() {
    for (int bm : p_.must_be_nonempty)
      if (bm >= 0 && bitmap_count(bitmap(bm), 0, 1) == 0) return false;
    return true;
  }

  std::vector<int> bound_cols() const {
    std::vector<int> c;
    for (size_t a = 0; a < col_.size(); ++a)
      if (col_[a].p) c.push_back((int)a);
    return c;
  }

  // ---- steps -------------------------------------------------------------------------------------
  void root(const Step &st) {
    uint64_t n = 0;
    int world = std::max(1, o_.shard_world);
    col_[st.dst] = bitmap_list(bitmap(st.cand_bm), world > 1 ? o_.shard_rank : 0, world, n);
    R_ = n;
  }

  struct ExpandOut {
    DBuf<uint32_t> dst;
    std::vector<DBuf<uint32_t>> carry;
    uint64_t n = 0;
    uint64_t E = 0;
    // block-segmented result (filtered expansion left un-compacted)
    bool segmented = false;
    DBuf<uint64_t> seg_start;
    DBuf<uint32_t> seg_count;
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

  // One pattern-edge expansion of R rows (src column) with an optional target bitmap, carrying the
  // listed columns. write=false only counts. allow_segmented leaves a filtered result as per-block
  // segments (the final step of a plan whose rows are distinct by construction).
  ExpandOut expand_core(const uint32_t *src, uint64_t R, const AdjSpec &adjs, const uint64_t *filter,
                        const std::vector<const uint32_t *> &carry, bool write, bool allow_segmented = false) {
    ExpandOut o;
    DAdj adj = make_adj(adjs);
    if (adj.n == 0 || R == 0) return o;
    // 1. degree binning + scans (light edges: merge path; heavy rows: chunks)
    DBuf<uint64_t> light(&pool_, R + 1), heavy(&pool_, R + 1), loffs(&pool_, R + 1), hoffs(&pool_, R + 1);
    DBuf<uint32_t> nch(&pool_, R + 1);
    DBuf<uint64_t> choffs(&pool_, R + 1);
    tm_.begin("k_row_split");
    launch_row_split(src, R, adj, heavy_deg_, light.p, heavy.p, nch.p, s_);
    tm_.end(R * (4 + 16ull * adj.n) + (R + 1) * 20);
    tm_.begin("scan_degrees");
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, light.p, loffs.p, (int64_t)(R + 1), s_); });
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, heavy.p, hoffs.p, (int64_t)(R + 1), s_); });
    hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> nit(nch.p, CastU64());
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::ExclusiveSum(t, b, nit, choffs.p, (int64_t)(R + 1), s_); });
    tm_.end((R + 1) * 40);
    uint64_t tot[3];
    HIP_CHECK(hipMemcpyAsync(&tot[0], loffs.p + R, 8, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(&tot[1], hoffs.p + R, 8, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(&tot[2], choffs.p + R, 8, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    const uint64_t EL = tot[0], EH = tot[1], nchunks = tot[2];
    const uint64_t E = EL + EH;
    o.E = E;
    if (E == 0) return o;
    DBuf<ChunkDesc> chunks;
    if (nchunks) {
      chunks = DBuf<ChunkDesc>(&pool_, nchunks);
      tm_.begin("k_fill_chunks");
      launch_fill_chunks(src, R, adj, choffs.p, hoffs.p, chunks.p, s_);
      tm_.end(nchunks * sizeof(ChunkDesc));
    }
    const uint64_t ntiles = EL ? (R + EL + kExpandTile - 1) / kExpandTile : 0;
    DBuf<uint64_t> part;
    if (ntiles) {
      part = DBuf<uint64_t>(&pool_, ntiles + 1);
      tm_.begin("k_mp_partition");
      launch_mp_partition(loffs.p, R, EL, ntiles, part.p, s_);
      tm_.end((ntiles + 1) * 8 * 20);
    }
    // 2. persistent grids and output placement
    const bool single = adj.n == 1, filt = filter != nullptr;
    // heavy kernel: a worker is a wave (4 per block); light kernel: a worker is a block
    constexpr unsigned WPB = kHeavyBlock / 64;
    const uint64_t hblocks = (nchunks + WPB - 1) / WPB;
    // persistent grids: every resident slot. (Running the two kernels side by side on split grids
    // was measured slower: the light kernel is latency-bound per tile and needs the whole chip.)
    const uint64_t sh = (uint64_t)cus() * expand_blocks_per_cu(true, single, filt, write);
    const uint64_t sl = (uint64_t)cus() * expand_blocks_per_cu(false, single, filt, write);
    const unsigned gh = nchunks ? (unsigned)std::min<uint64_t>(hblocks, sh) : 0;
    const unsigned gl = ntiles ? (unsigned)std::min<uint64_t>(ntiles, sl) : 0;
    const uint64_t wh = (uint64_t)gh * WPB;
    const uint64_t caph = gh ? (nchunks + wh - 1) / wh * (uint64_t)kChunk : 0;
    const uint64_t capl = gl ? (ntiles + gl - 1) / gl * (uint64_t)kExpandTile : 0;
    const uint64_t cap = filt ? wh * caph + gl * capl : E;
    ExpandArgs a{};
    a.src = src;
    a.offs = loffs.p;
    a.part = part.p;
    a.R = R;
    a.E = EL;
    a.ntiles = ntiles;
    a.adj = adj;
    a.filter = filter;
    a.ncarry = (int32_t)carry.size();
    a.chunks = chunks.p;
    a.nchunks = nchunks;
    a.hoffs = hoffs.p;
    a.dense_base = EH;
    std::vector<DBuf<uint32_t>> outc;
    DBuf<uint32_t> odst;
    if (write) {
      odst = DBuf<uint32_t>(&pool_, std::max<uint64_t>(cap, 1));
      a.out_dst = odst.p;
      for (size_t c = 0; c < carry.size(); ++c) {
        outc.emplace_back(&pool_, std::max<uint64_t>(cap, 1));
        a.carry_in[c] = carry[c];
        a.carry_out[c] = outc.back().p;
      }
    }
    if (filt) {
      o.nseg = (uint32_t)(wh + gl);
      o.seg_start = DBuf<uint64_t>(&pool_, o.nseg);
      o.seg_count = DBuf<uint32_t>(&pool_, o.nseg);
      a.seg_start = o.seg_start.p;
      a.seg_count = o.seg_count.p;
    }
    // algorithmic bytes: 8 B row_ptr pair per row + 4 B col per edge (+ 4 B × columns
    // per emitted row, added below)
    uint64_t kb = 8 * R + 4 * E;
    // per-kernel algorithmic bytes: heavy rows carry EH edges, light rows EL (+ 8 B per row each)
    if (gh) {
      a.arena_base = 0;
      a.arena_cap = caph;
      a.seg_base = 0;
      tm_.begin("k_expand_heavy");
      launch_expand_heavy(a, gh, write, s_);
      tm_.end(4 * EH + 24 * nchunks);
    }
    if (gl) {
      a.arena_base = wh * caph;
      a.arena_cap = capl;
      a.seg_base = (uint32_t)wh;
      tm_.begin("k_expand_light");
      launch_expand(a, gl, write, s_);
      tm_.end(8 * R + 4 * EL);
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
    // filtered: rows per block segment → total (and dense compaction when required)
    DBuf<uint64_t> soffs(&pool_, o.nseg + 1);
    hipcub::TransformInputIterator<uint64_t, CastU64, const uint32_t *> sit(o.seg_count.p, CastU64());
    cub([&](void *t, size_t &b) { return hipcub::DeviceScan::InclusiveSum(t, b, sit, soffs.p + 1, (int64_t)o.nseg, s_); });
    HIP_CHECK(hipMemsetAsync(soffs.p, 0, 8, s_));
    const uint64_t n = read1(soffs.p + o.nseg);
    o.n = n;
    if (write) kb += 4ull * (carry.size() + 1) * n;
    tm_.end(kb);
    alg_bytes_ += kb;
    if (!write || n == 0) return o;
    if (allow_segmented) {
      o.segmented = true;
      o.dst = std::move(odst);
      o.carry = std::move(outc);
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

  void expand_step(const Step &st, bool write, bool allow_segmented) {
    std::vector<int> cols = bound_cols();
    std::vector<const uint32_t *> carry;
    for (int c : cols) carry.push_back(col_[c].p);
    ExpandOut o = expand_core(col_[st.src].p, R_, st.adj, bitmap(st.filter_bm), carry, write, allow_segmented);
    edges_ += o.E;
    R_ = o.n;
    if (!write || R_ == 0) return;
    segmented_ = o.segmented;
    for (size_t i = 0; i < cols.size(); ++i) col_[cols[i]] = std::move(o.carry[i]);
    col_[st.dst] = std::move(o.dst);
  }

  // keep the rows whose flag is set (all bound columns)
  void select_rows(const uint8_t *flags, uint64_t R) {
    DBuf<uint32_t> idx(&pool_, R);
    DBuf<uint64_t> nsel(&pool_, 1);
    hipcub::CountingInputIterator<uint32_t> cnt(0);
    cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, cnt, flags, idx.p, nsel.p, (int64_t)R, s_); });
    const uint64_t n = read1(nsel.p);
    gather_rows(idx.p, n);
  }

  void gather_rows(const uint32_t *idx, uint64_t n) {
    std::vector<int> cols = bound_cols();
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

  uint64_t degree_sum(const uint32_t *src, uint64_t R, const AdjSpec &adjs) {
    DAdj adj = make_adj(adjs);
    if (adj.n == 0 || R == 0) return 0;
    DBuf<uint64_t> deg(&pool_, R + 1), sum(&pool_, 1);
    launch_row_degree(src, R, adj, deg.p, s_);
    cub([&](void *t, size_t &b) { return hipcub::DeviceReduce::Sum(t, b, deg.p, sum.p, (int64_t)(R + 1), s_); });
    return read1(sum.p);
  }

  void check_step(const Step &st) {
    const uint64_t R = R_;
    const uint64_t E = degree_sum(col_[st.src].p, R, st.adj);
    edges_ += E;
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
      return hipcub::DeviceRadixSort::SortKeys(t, b, keys.p, sorted.p, (int64_t)n, 0, end_bit, s_);
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
    const uint64_t R = R_;
    const bool dep_where = st.where_prog >= 0 && p_.progs[st.where_prog].uses_depth;
    const bool dep_while = st.while_prog >= 0 && p_.progs[st.while_prog].uses_depth;
    const bool use_visited = !dep_where && !dep_while;
    const int vbits = bits_for(g_.V);
    const int key_bits = 32 + vbits;
    DBuf<uint32_t> frow(&pool_, R), fv(&pool_, R);
    launch_iota(frow.p, R, s_);
    HIP_CHECK(hipMemcpyAsync(fv.p, col_[st.src].p, R * 4, hipMemcpyDeviceToDevice, s_));
    uint64_t nf = R;
    DBuf<uint64_t> visited;
    uint64_t nvisited = 0;
    if (use_visited) {
      visited = DBuf<uint64_t>(&pool_, R);
      launch_pack_pairs(frow.p, fv.p, R, visited.p, s_);
      nvisited = sort_unique_keys(visited, R, key_bits);
    }
    std::vector<DBuf<uint64_t>> res_parts;
    std::vector<uint64_t> res_n;
    DBuf<uint64_t> where_bm(&pool_, nwords_), while_bm(&pool_, nwords_);
    bool where_ready = false, while_ready = false;
    for (int64_t d = 0;; ++d) {
      if (d > 100000) fail(OMX_E_EXECUTION, "variable-length traversal did not terminate (the reference recurses without bound)");
      // include F_d ∩ where_d
      {
        DBuf<uint64_t> keys(&pool_, std::max<uint64_t>(nf, 1));
        uint64_t nk = nf;
        if (st.where_prog >= 0) {
          if (!where_ready || dep_where) {
            eval_bitmap(st.where_prog, -1, d, where_bm.p);
            where_ready = true;
          }
          DBuf<uint8_t> flags(&pool_, nf);
          launch_flag_bitmap(fv.p, nf, where_bm.p, flags.p, s_);
          DBuf<uint64_t> all(&pool_, nf), nsel(&pool_, 1);
          launch_pack_pairs(frow.p, fv.p, nf, all.p, s_);
          cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, all.p, flags.p, keys.p, nsel.p, (int64_t)nf, s_); });
          nk = read1(nsel.p);
        } else {
          launch_pack_pairs(frow.p, fv.p, nf, keys.p, s_);
        }
        if (nk) {
          res_parts.push_back(std::move(keys));
          res_n.push_back(nk);
        }
      }
      if (st.has_max_depth && d >= st.max_depth) break;
      // G = F_d ∩ while_d
      uint64_t ng = nf;
      DBuf<uint32_t> grow, gv;
      const uint32_t *gr = frow.p, *gvp = fv.p;
      if (st.while_prog >= 0) {
        if (!while_ready || dep_while) {
          eval_bitmap(st.while_prog, -1, d, while_bm.p);
          while_ready = true;
        }
        DBuf<uint8_t> flags(&pool_, nf);
        launch_flag_bitmap(fv.p, nf, while_bm.p, flags.p, s_);
        DBuf<uint64_t> all(&pool_, nf), sel(&pool_, nf), nsel(&pool_, 1);
        launch_pack_pairs(frow.p, fv.p, nf, all.p, s_);
        cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, all.p, flags.p, sel.p, nsel.p, (int64_t)nf, s_); });
        ng = read1(nsel.p);
        grow = DBuf<uint32_t>(&pool_, std::max<uint64_t>(ng, 1));
        gv = DBuf<uint32_t>(&pool_, std::max<uint64_t>(ng, 1));
        launch_unpack_pairs(sel.p, ng, grow.p, gv.p, s_);
        gr = grow.p;
        gvp = gv.p;
      }
      if (ng == 0) break;
      ExpandOut ex = expand_core(gvp, ng, st.adj, nullptr, {gr}, true);
      edges_ += ex.E;
      if (ex.n == 0) break;
      DBuf<uint64_t> keys(&pool_, ex.n);
      launch_pack_pairs(ex.carry[0].p, ex.dst.p, ex.n, keys.p, s_);
      uint64_t nk = sort_unique_keys(keys, ex.n, key_bits);
      if (use_visited) {
        DBuf<uint8_t> flags(&pool_, nk);
        launch_flag_not_in(visited.p, nvisited, keys.p, nk, flags.p, s_);
        DBuf<uint64_t> fresh(&pool_, nk), nsel(&pool_, 1);
        cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, keys.p, flags.p, fresh.p, nsel.p, (int64_t)nk, s_); });
        nk = read1(nsel.p);
        if (nk) {
          DBuf<uint64_t> merged(&pool_, nvisited + nk);
          HIP_CHECK(hipMemcpyAsync(merged.p, visited.p, nvisited * 8, hipMemcpyDeviceToDevice, s_));
          HIP_CHECK(hipMemcpyAsync(merged.p + nvisited, fresh.p, nk * 8, hipMemcpyDeviceToDevice, s_));
          nvisited = sort_unique_keys(merged, nvisited + nk, key_bits);
          visited = std::move(merged);
        }
        keys = std::move(fresh);
      }
      if (nk == 0) break;
      frow = DBuf<uint32_t>(&pool_, nk);
      fv = DBuf<uint32_t>(&pool_, nk);
      launch_unpack_pairs(keys.p, nk, frow.p, fv.p, s_);
      nf = nk;
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
    res_parts.clear();
    uint64_t nres = sort_unique_keys(res, total, key_bits);
    DBuf<uint32_t> rrow(&pool_, std::max<uint64_t>(nres, 1)), rv(&pool_, std::max<uint64_t>(nres, 1));
    launch_unpack_pairs(res.p, nres, rrow.p, rv.p, s_);
    if (st.mode == T_BOUND) {
      DBuf<uint32_t> idx(&pool_, std::max<uint64_t>(R, 1));
      launch_iota(idx.p, R, s_);
      DBuf<uint64_t> keys(&pool_, std::max<uint64_t>(R, 1));
      launch_pack_pairs(idx.p, col_[st.dst].p, R, keys.p, s_);
      DBuf<uint8_t> flags(&pool_, std::max<uint64_t>(R, 1));
      launch_flag_not_in(res.p, nres, keys.p, R, flags.p, s_);
      // flags = "not in" → invert by selecting on the complement
      DBuf<uint8_t> keep(&pool_, std::max<uint64_t>(R, 1));
      invert_flags(flags.p, keep.p, R);
      select_rows(keep.p, R);
      return;
    }
    if (st.mode == T_CAND && nres) {
      DBuf<uint8_t> flags(&pool_, nres);
      launch_flag_bitmap(rv.p, nres, bitmap(st.cand_bm), flags.p, s_);
      DBuf<uint64_t> sel(&pool_, nres), nsel(&pool_, 1);
      cub([&](void *t, size_t &b) { return hipcub::DeviceSelect::Flagged(t, b, res.p, flags.p, sel.p, nsel.p, (int64_t)nres, s_); });
      nres = read1(nsel.p);
      launch_unpack_pairs(sel.p, nres, rrow.p, rv.p, s_);
    }
    gather_rows(rrow.p, nres);
    col_[st.dst] = std::move(rv);
  }

  void invert_flags(const uint8_t *in, uint8_t *out, uint64_t n) {
    hipLaunchKernelGGL(k_invert_flags, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s_, in, out, n);
  }

  // Projection + distinct rows (addResult :661-729 → addToUniqueResult)
  void project_dedup(std::vector<DBuf<uint32_t>> &out, uint64_t &n) {
    n = R_;
    if (p_.proj == Plan::PROJ_ELEMENTS) {
      DBuf<uint64_t> bm(&pool_, nwords_);
      HIP_CHECK(hipMemsetAsync(bm.p, 0, nwords_ * 8, s_));
      tm_.begin("k_mark_bitmap");
      for (int a : p_.out_aliases) launch_mark_bitmap(col_[a].p, R_, bm.p, s_);
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
    if (p_.unique_by_construction) return;
    if (segmented_) fail(OMX_E_INVALID, "internal: segmented table reached dedup");
    dedup_ran_ = 1;
    tm_.begin("dedup");
    const int vbits = bits_for(g_.V);
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
          return hipcub::DeviceRadixSort::SortPairs(t, b, kin.p, kout.p, order.p, order2.p, (int64_t)R_, 0, vbits, s_);
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

omx_result *execute_plan(Graph &g, const Plan &p, const omx_exec_options &opts) {
  if (!g.on_device()) fail(OMX_E_DEVICE, "graph snapshot is host-only (device = -1)");
  HIP_CHECK(hipSetDevice(g.device));
  Executor ex(g, p, opts);
  return ex.run();
}

}  // namespace omx
