// projdev.hip — RETURN expressions evaluated on the device (the scalar subset of project.cpp).
//
// A RETURN item that reads only an alias (its record), one property of an alias's vertex, literals,
// parameters and + - * / % over numbers is compiled to a short stack program. One thread per distinct
// alias tuple (the device's distinct rows of the aliases the items read) evaluates every item into a
// (kind, 64-bit payload) cell; the documents are then de-duplicated by content on the device (an open-
// addressing table of row indices, equal = same kinds and payloads, which is project.cpp's content key:
// ODocumentEqualityWrapper, C/command/ODocumentEqualityWrapper.java:19-35) and only the distinct
// documents' cells travel to the host, where omx_result_cell reads them column by column. Semantics are
// project.cpp's Evaluator (field :169-191, math :206-225): a null operand makes a null result, integer
// arithmetic wraps, an integer division by zero and arithmetic on a non-number fail the execution.
// Strings (dictionary codes of one property per item), booleans and RIDs pass through; string
// concatenation, comparisons, lists, maps, methods and @class stay with the host evaluator.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstring>
#include <unordered_map>

#include "devutil.h"
#include "exec.h"
#include "graph.h"
#include "plan.h"
#include "projdev.h"

namespace omx {

namespace {

enum PjOp : int32_t { PJ_NULL, PJ_INT, PJ_DBL, PJ_BOOL, PJ_RID, PJ_PROP, PJ_ADD, PJ_SUB, PJ_MUL, PJ_DIV, PJ_MOD };

struct PjInstr {
  int32_t op;
  int32_t col;      // PJ_RID / PJ_PROP: index of the alias column
  int64_t i;        // PJ_INT / PJ_BOOL value; PJ_PROP: dictionary size of a string property
  double d;         // PJ_DBL
  DColumn c;        // PJ_PROP
};
constexpr int kPjMaxInstr = 16, kPjMaxStack = 8;
struct PjProgram {
  PjInstr code[kPjMaxInstr];
  int32_t n;
  int32_t pad;
};

enum PjErr : uint32_t { kPjNonNumeric = 1, kPjDivZero = 2 };

// ---- compilation (host) --------------------------------------------------------------------------------
// kinds a compiled sub-expression may produce (bit per PjKind)
constexpr uint32_t M(int k) { return 1u << k; }

struct Compiler {
  const Graph &g;
  const Plan &p;
  PjProgram prog{};
  std::string why;

  int alias_col(const std::string &name) const {
    for (size_t c = 0; c < p.out_aliases.size(); ++c)
      if (p.aliases[p.out_aliases[c]] == name) return (int)c;
    return -1;
  }
  bool emit(const PjInstr &in) {
    if (prog.n >= kPjMaxInstr) {
      why = "expression too long";
      return false;
    }
    prog.code[prog.n++] = in;
    return true;
  }
  bool literal(const Value &v, uint32_t *kinds) {
    PjInstr in{};
    switch (v.kind) {
      case Value::NUL: in.op = PJ_NULL; *kinds = M(PJ_K_NUL); break;
      case Value::INT: in.op = PJ_INT; in.i = v.i; *kinds = M(PJ_K_INT); break;
      case Value::DBL: in.op = PJ_DBL; in.d = v.d; *kinds = M(PJ_K_DBL); break;
      case Value::BOOL: in.op = PJ_BOOL; in.i = v.i; *kinds = M(PJ_K_BOOL); break;
      default: why = "a string literal"; return false;
    }
    return emit(in);
  }
  // compiles e; *kinds: the kinds it may produce; false (why set) when the host evaluator must run
  bool expr(const ExprP &e, uint32_t *kinds, int depth) {
    if (depth >= kPjMaxStack) {
      why = "expression too deep";
      return false;
    }
    switch (e->kind) {
      case Expr::LIT: return literal(e->value, kinds);
      case Expr::PARAM: {
        const Value *v = p.params.get(*e);
        if (!v) {
          why = "missing parameter";
          return false;
        }
        return literal(*v, kinds);
      }
      case Expr::FIELD: {  // a bare alias: its record
        const int c = alias_col(e->name);
        if (c < 0) {
          why = "identifier " + e->name;
          return false;
        }
        PjInstr in{};
        in.op = PJ_RID;
        in.col = c;
        *kinds = M(PJ_K_RID) | M(PJ_K_NUL);
        return emit(in);
      }
      case Expr::CHAIN: {  // alias.field
        if (e->kids[0]->kind != Expr::FIELD || e->suffixes.size() != 1 || e->suffixes[0].kind != Suffix::FIELD) {
          why = "chain " + expr_text(e);
          return false;
        }
        const int c = alias_col(e->kids[0]->name);
        const std::string &f = e->suffixes[0].name;
        // (an edge record's `out` / `in` link is resolved on the host, project.cpp)
        if (c < 0 || (!f.empty() && f[0] == '@' && !ieq(f, "@rid")) || (g.edge_records && (f == "out" || f == "in"))) {
          why = "chain " + expr_text(e);
          return false;
        }
        PjInstr in{};
        in.col = c;
        if (ieq(f, "@rid")) {
          in.op = PJ_RID;
          *kinds = M(PJ_K_RID) | M(PJ_K_NUL);
          return emit(in);
        }
        const int pid = g.prop_id(f);
        if (pid < 0) {  // no such property on any vertex: null (project.cpp field :177-178)
          in.op = PJ_NULL;
          *kinds = M(PJ_K_NUL);
          return emit(in);
        }
        const Property &pr = g.props[pid];
        in.op = PJ_PROP;
        in.c = DColumn{pr.d_values, pr.d_present, pr.type, 0};
        in.i = (int64_t)pr.dict.size();
        const int k = pr.type == OMX_PROP_DOUBLE ? PJ_K_DBL : pr.type == OMX_PROP_STRING ? PJ_K_STR
                      : pr.type == OMX_PROP_BOOL ? PJ_K_BOOL : PJ_K_INT;
        *kinds = M(k) | M(PJ_K_NUL);
        return emit(in);
      }
      case Expr::MATH: {
        uint32_t a = 0, b = 0;
        if (!expr(e->kids[0], &a, depth) || !expr(e->kids[1], &b, depth + 1)) return false;
        const uint32_t num = M(PJ_K_NUL) | M(PJ_K_INT) | M(PJ_K_DBL);
        if ((a | b) & ~num) {  // string concatenation, or the host's "arithmetic on non-numeric" error
          why = "arithmetic over non-numbers";
          return false;
        }
        PjInstr in{};
        const std::string &op = e->name;
        in.op = op == "+" ? PJ_ADD : op == "-" ? PJ_SUB : op == "*" ? PJ_MUL : op == "/" ? PJ_DIV : PJ_MOD;
        *kinds = M(PJ_K_NUL) | (((a | b) & M(PJ_K_DBL)) ? M(PJ_K_DBL) : 0) |
                 (((a & M(PJ_K_INT)) && (b & M(PJ_K_INT))) ? M(PJ_K_INT) : 0);
        return emit(in);
      }
      default: why = "expression " + expr_text(e); return false;
    }
  }
};

// ---- evaluation (device) -------------------------------------------------------------------------------
struct PjArgs {
  const PjProgram *progs;
  int32_t nitems;
  const uint32_t *col[kPjMaxCols];
  uint32_t V;
  const uint64_t *rids;
  uint8_t *kind;   // [item][n]
  uint64_t *val;   // [item][n]
  uint32_t *err;
};

__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double bdbl(uint64_t b) { return __longlong_as_double((long long)b); }

__global__ void k_pj_eval(PjArgs a, uint64_t n) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    for (int it = 0; it < a.nitems; ++it) {
      const PjProgram &pg = a.progs[it];
      uint8_t sk[kPjMaxStack];
      uint64_t sv[kPjMaxStack];
      int sp = 0;
      for (int ip = 0; ip < pg.n; ++ip) {
        const PjInstr &in = pg.code[ip];
        switch (in.op) {
          case PJ_NULL: sk[sp] = PJ_K_NUL; sv[sp++] = 0; break;
          case PJ_INT: sk[sp] = PJ_K_INT; sv[sp++] = (uint64_t)in.i; break;
          case PJ_DBL: sk[sp] = PJ_K_DBL; sv[sp++] = dbits(in.d); break;
          case PJ_BOOL: sk[sp] = PJ_K_BOOL; sv[sp++] = in.i ? 1 : 0; break;
          case PJ_RID: {
            const uint32_t v = a.col[in.col][r];
            if (v >= a.V) { sk[sp] = PJ_K_NUL; sv[sp++] = 0; }
            else { sk[sp] = PJ_K_RID; sv[sp++] = a.rids[v]; }
            break;
          }
          case PJ_PROP: {
            const uint32_t v = a.col[in.col][r];
            uint8_t k = PJ_K_NUL;
            uint64_t x = 0;
            if (v < a.V && (!in.c.present || in.c.present[v])) {
              switch (in.c.type) {
                case OMX_PROP_INT64: k = PJ_K_INT; x = (uint64_t)static_cast<const int64_t *>(in.c.values)[v]; break;
                case OMX_PROP_DOUBLE: k = PJ_K_DBL; x = dbits(static_cast<const double *>(in.c.values)[v]); break;
                case OMX_PROP_BOOL: k = PJ_K_BOOL; x = static_cast<const int32_t *>(in.c.values)[v] != 0; break;
                case OMX_PROP_STRING: {
                  const int32_t code = static_cast<const int32_t *>(in.c.values)[v];
                  if (code >= 0 && code < in.i) { k = PJ_K_STR; x = (uint64_t)code; }
                  break;
                }
                default: k = PJ_K_INT; x = (uint64_t)(int64_t)static_cast<const int32_t *>(in.c.values)[v]; break;
              }
            }
            sk[sp] = k;
            sv[sp++] = x;
            break;
          }
          default: {  // arithmetic: b = top, a = below
            const uint8_t kb = sk[sp - 1], ka = sk[sp - 2];
            const uint64_t vb = sv[sp - 1], va = sv[sp - 2];
            sp -= 2;
            uint8_t k = PJ_K_NUL;
            uint64_t x = 0;
            if (ka != PJ_K_NUL && kb != PJ_K_NUL) {
              if ((ka != PJ_K_INT && ka != PJ_K_DBL) || (kb != PJ_K_INT && kb != PJ_K_DBL)) {
                atomicOr(a.err, (uint32_t)kPjNonNumeric);
              } else if (ka == PJ_K_INT && kb == PJ_K_INT) {
                k = PJ_K_INT;
                const int64_t xa = (int64_t)va, xb = (int64_t)vb;
                switch (in.op) {
                  case PJ_ADD: x = va + vb; break;
                  case PJ_SUB: x = va - vb; break;
                  case PJ_MUL: x = va * vb; break;
                  default:
                    if (xb == 0) {
                      atomicOr(a.err, (uint32_t)kPjDivZero);
                    } else if (xb == -1) {  // Java: MIN / -1 wraps to MIN, MIN % -1 is 0
                      x = in.op == PJ_DIV ? (uint64_t)0 - va : 0;
                    } else {
                      x = (uint64_t)(in.op == PJ_DIV ? xa / xb : xa % xb);
                    }
                }
              } else {
                k = PJ_K_DBL;
                const double xa = ka == PJ_K_DBL ? bdbl(va) : (double)(int64_t)va;
                const double xb = kb == PJ_K_DBL ? bdbl(vb) : (double)(int64_t)vb;
                switch (in.op) {
                  case PJ_ADD: x = dbits(xa + xb); break;
                  case PJ_SUB: x = dbits(xa - xb); break;
                  case PJ_MUL: x = dbits(xa * xb); break;
                  case PJ_DIV: x = dbits(xa / xb); break;
                  default: x = dbits(fmod(xa, xb)); break;
                }
              }
            }
            sk[sp] = k;
            sv[sp++] = x;
          }
        }
      }
      a.kind[(uint64_t)it * n + r] = sk[0];
      a.val[(uint64_t)it * n + r] = sv[0];
    }
  }
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// content de-duplication: the first row to claim a slot with its content keeps it; an equal row found
// on the probe path is a duplicate
__global__ void k_pj_unique(const uint8_t *kind, const uint64_t *val, int nitems, uint64_t n, uint32_t *tab,
                            uint64_t mask, uint8_t *uniq) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int it = 0; it < nitems; ++it) h = mix(h ^ mix(((uint64_t)kind[(uint64_t)it * n + r] << 56) ^ val[(uint64_t)it * n + r]));
    uint64_t s = h & mask;
    uint8_t u = 0;
    for (;;) {
      const uint32_t cur = atomicCAS(&tab[s], 0xFFFFFFFFu, (uint32_t)r);
      if (cur == 0xFFFFFFFFu) {
        u = 1;
        break;
      }
      bool eq = true;
      for (int it = 0; it < nitems && eq; ++it)
        eq = kind[(uint64_t)it * n + cur] == kind[(uint64_t)it * n + r] && val[(uint64_t)it * n + cur] == val[(uint64_t)it * n + r];
      if (eq) break;
      s = (s + 1) & mask;
    }
    uniq[r] = u;
  }
}

template <class T>
__global__ void k_pj_gather(const T *in, const uint32_t *idx, uint64_t m, uint64_t n, int nitems, T *out) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x)
    for (int it = 0; it < nitems; ++it) out[(uint64_t)it * m + j] = in[(uint64_t)it * n + idx[j]];
}

}  // namespace

bool device_projection_ok(const Graph &g, const Plan &p, std::string *why) {
  if (p.proj != Plan::PROJ_EXPR || p.out_aliases.empty() || p.out_aliases.size() > (size_t)kPjMaxCols ||
      p.returns.size() > (size_t)kPjMaxItems) {
    if (why) *why = "not a scalar RETURN projection";
    return false;
  }
  for (const ReturnItem &ri : p.returns) {
    Compiler c{g, p};
    uint32_t k = 0;
    if (!c.expr(ri.expr, &k, 0)) {
      if (why) *why = c.why;
      return false;
    }
  }
  return true;
}

void device_project(Graph &g, const Plan &p, const std::vector<const uint32_t *> &cols, uint64_t n, int64_t limit,
                    int cus, hipStream_t s, omx_result &res) {
  const int nitems = (int)p.returns.size();
  if (n >= UINT32_MAX) fail(OMX_E_INVALID, "internal: device projection of 2^32 or more tuples (u32 table slots)");
  if (limit >= 0) fail(OMX_E_INVALID, "internal: device projection with LIMIT (the host evaluator stops at the limit)");
  std::vector<PjProgram> progs;
  for (const ReturnItem &ri : p.returns) {
    Compiler c{g, p};
    uint32_t k = 0;
    if (!c.expr(ri.expr, &k, 0)) fail(OMX_E_INVALID, "internal: device projection compile: " + c.why);
    progs.push_back(c.prog);
  }
  DBuf<PjProgram> dprog(&g.pool, progs.size());
  HIP_CHECK(hipMemcpyAsync(dprog.p, progs.data(), progs.size() * sizeof(PjProgram), hipMemcpyHostToDevice, s));
  DBuf<uint8_t> kind(&g.pool, std::max<uint64_t>(n * nitems, 1));
  DBuf<uint64_t> val(&g.pool, std::max<uint64_t>(n * nitems, 1));
  DBuf<uint32_t> err(&g.pool, 1);
  HIP_CHECK(hipMemsetAsync(err.p, 0, 4, s));
  PjArgs a{};
  a.progs = dprog.p;
  a.nitems = nitems;
  for (size_t c = 0; c < cols.size(); ++c) a.col[c] = cols[c];
  a.V = g.V;
  a.rids = g.d_rids;
  a.kind = kind.p;
  a.val = val.p;
  a.err = err.p;
  const unsigned grid = (unsigned)std::min<uint64_t>(nblocks(std::max<uint64_t>(n, 1), 256), (uint64_t)cus * 16);
  hipLaunchKernelGGL(k_pj_eval, dim3(grid), dim3(256), 0, s, a, n);
  KCHECK("k_pj_eval");
  // the distinct documents: a table of 2^k ≥ 2n slots
  uint64_t cap = 1;
  while (cap < 2 * n) cap <<= 1;
  DBuf<uint32_t> tab(&g.pool, cap);
  DBuf<uint8_t> uniq(&g.pool, std::max<uint64_t>(n, 1));
  HIP_CHECK(hipMemsetAsync(tab.p, 0xFF, cap * 4, s));
  hipLaunchKernelGGL(k_pj_unique, dim3(grid), dim3(256), 0, s, kind.p, val.p, nitems, n, tab.p, cap - 1, uniq.p);
  KCHECK("k_pj_unique");
  DBuf<uint32_t> idx(&g.pool, std::max<uint64_t>(n, 1));
  DBuf<uint64_t> nsel(&g.pool, 1);
  hipcub::CountingInputIterator<uint32_t> iota(0);
  size_t tb = 0;
  HIP_CHECK(hipcub::DeviceSelect::Flagged(nullptr, tb, iota, uniq.p, idx.p, nsel.p, (int64_t)n, s));
  {
    DBuf<uint8_t> tmp(&g.pool, std::max<size_t>(tb, 1));
    HIP_CHECK(hipcub::DeviceSelect::Flagged(tmp.p, tb, iota, uniq.p, idx.p, nsel.p, (int64_t)n, s));
  }
  uint64_t m = 0;
  uint32_t herr = 0;
  HIP_CHECK(hipMemcpyAsync(&m, nsel.p, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (herr & kPjDivZero) fail(OMX_E_EXECUTION, "division by zero in a RETURN expression");
  if (herr & kPjNonNumeric) fail(OMX_E_EXECUTION, "arithmetic on non-numeric values in a RETURN expression");
  // LIMIT after the content de-duplication (0 keeps one, as addSingleResult :737-750)
  if (limit > -1) m = std::min<uint64_t>(m, (uint64_t)std::max<int64_t>(limit, 1));
  DBuf<uint8_t> ok(&g.pool, std::max<uint64_t>(m * nitems, 1));
  DBuf<uint64_t> ov(&g.pool, std::max<uint64_t>(m * nitems, 1));
  if (m) {
    const unsigned g2 = (unsigned)std::min<uint64_t>(nblocks(m, 256), (uint64_t)cus * 16);
    hipLaunchKernelGGL(k_pj_gather<uint8_t>, dim3(g2), dim3(256), 0, s, kind.p, idx.p, m, n, nitems, ok.p);
    hipLaunchKernelGGL(k_pj_gather<uint64_t>, dim3(g2), dim3(256), 0, s, val.p, idx.p, m, n, nitems, ov.p);
    KCHECK("k_pj_gather");
  }
  res.pcols.assign(nitems, omx_result::PCol{});
  std::vector<uint8_t> hk(m * nitems);
  std::vector<uint64_t> hv(m * nitems);
  if (m) {
    HIP_CHECK(hipMemcpyAsync(hk.data(), ok.p, m * nitems, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(hv.data(), ov.p, m * nitems * 8, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  for (int it = 0; it < nitems; ++it) {
    omx_result::PCol &pc = res.pcols[it];
    pc.kind.assign(hk.begin() + (size_t)it * m, hk.begin() + (size_t)(it + 1) * m);
    pc.val.assign(hv.begin() + (size_t)it * m, hv.begin() + (size_t)(it + 1) * m);
    // the strings this column returns (dictionary codes of its property)
    const ReturnItem &ri = p.returns[it];
    if (ri.expr->kind == Expr::CHAIN) {
      const int pid = g.prop_id(ri.expr->suffixes[0].name);
      if (pid >= 0 && g.props[pid].type == OMX_PROP_STRING)
        for (uint64_t j = 0; j < m; ++j)
          if (pc.kind[j] == PJ_K_STR) pc.strs.emplace(pc.val[j], g.props[pid].dict[pc.val[j]]);
    }
  }
  res.n_pcol_rows = m;
}

}  // namespace omx
