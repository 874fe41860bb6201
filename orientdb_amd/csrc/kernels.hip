// kernels.hip — gfx950 (MI355X / CDNA4) kernels of the MATCH executor.
//
// None of this is a dense contraction: every kernel is HBM/L2-bound integer work (no MFMA). The
// hot path is the frontier expansion of one pattern edge over the binding table
// (OMatchStatement.processContext P/OMatchStatement.java:412-568 → OMatchPathItem.executeTraversal
// P/OMatchPathItem.java:49-78 → OrientVertex.getVertices B/OrientVertex.java:401-460), split by degree:
//   * heavy rows (≥ kHeavyDeg neighbours, the RMAT hubs that carry most edges) → k_expand_heavy:
//     chunks of ≤ 4096 edges of one row in one aligned col window; per lane 4 × dwordx4 loads, 16
//     independent bitmap probes, block scan, LDS-staged coalesced stores; row columns are constants;
//   * light rows → k_expand: merge-path tiles over (rows + edges) of 256 threads × 8 items; row
//     ownership of every edge resolved in LDS (scatter of row starts + block max-scan) so col[] loads
//     stay coalesced; compaction by wave64 ballot + mbcnt with wave totals scanned in LDS;
//   * both are persistent (grid = resident blocks) and append to a private per-block arena, so the
//     filtered output needs no global atomics and no compaction pass; the table is block-segmented
//     (k_compact_segments makes it dense only when a consumer needs it). Without a filter both write
//     straight to the dense position of each edge.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include "common.h"
#include "devutil.h"
#include "kernels.h"

namespace omx {

bool sync_launches() {
  static const bool on = [] {
    const char *e = std::getenv("OMX_SYNC_LAUNCH");
    return e && *e && *e != '0';
  }();
  return on;
}

// ---- predicate VM (compiled WHERE / while; P/OWhereClause.java:36-41, operators P/O*Operator.java) ----

struct VmVal {
  int64_t i;
  double d;
  int32_t t;  // 0 null, 1 int, 2 double, 3 bool
};

__host__ __device__ __forceinline__ VmVal vm_col(const DColumn &c, uint32_t v) {
  VmVal x{0, 0.0, 0};
  if (c.present && !c.present[v]) return x;
  switch (c.type) {
    case OMX_PROP_INT64: x.i = ((const int64_t *)c.values)[v]; x.t = 1; break;
    case OMX_PROP_DOUBLE: x.d = ((const double *)c.values)[v]; x.t = 2; break;
    case OMX_PROP_BOOL: x.i = ((const int32_t *)c.values)[v] != 0; x.t = 3; break;
    case OMX_PROP_STRING: {
      int32_t code = ((const int32_t *)c.values)[v];
      if (code < 0) return x;
      x.i = code;
      x.t = 1;
      break;
    }
    default: x.i = ((const int32_t *)c.values)[v]; x.t = 1; break;
  }
  return x;
}

__host__ __device__ __forceinline__ int vm_cmp(const VmVal &a, const VmVal &b) {
  if (a.t != 2 && b.t != 2) return a.i < b.i ? -1 : (a.i > b.i ? 1 : 0);
  double x = a.t == 2 ? a.d : (double)a.i, y = b.t == 2 ? b.d : (double)b.i;
  return x < y ? -1 : (x > y ? 1 : 0);
}

__host__ __device__ __forceinline__ bool vm_truthy(const VmVal &a) { return a.t == 3 && a.i != 0; }

__host__ __device__ __forceinline__ bool atom_cmp(int op, int c) {
  return op == P_EQ ? c == 0 : op == P_NE ? c != 0 : op == P_LT ? c < 0 : op == P_LE ? c <= 0 : op == P_GT ? c > 0 : c >= 0;
}

__host__ __device__ bool eval_pred(const DPred &P, uint32_t v, int64_t depth) {
  if (P.use_class) {
    uint32_t c = P.vclass[v];
    if (!((P.class_mask[c >> 6] >> (c & 63)) & 1ull)) return false;
  }
  if (P.n == 0) return true;
  if (P.n_atoms) {  // column OP constant atoms: no interpreter stack (no scratch)
    bool acc = P.conj != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= P.n_atoms) break;
      const VmVal x = vm_col(P.cols[P.atom_col[k]], v);
      bool r;
      if (x.t == 0) {
        r = P.atom_op[k] == P_NE;  // null: = < <= > >= false, != true
      } else if (P.atom_dbl[k]) {
        const double a = x.t == 2 ? x.d : (double)x.i, b = P.atom_d[k];
        r = atom_cmp(P.atom_op[k], a < b ? -1 : (a > b ? 1 : 0));
      } else {
        const int64_t b = P.atom_i[k];
        r = atom_cmp(P.atom_op[k], x.i < b ? -1 : (x.i > b ? 1 : 0));
      }
      acc = P.conj ? (acc && r) : (acc || r);
    }
    return acc;
  }
  VmVal st[16];
  int sp = 0;
  for (int pc = 0; pc < P.n; ++pc) {
    const DPredInstr in = P.code[pc];
    switch (in.op) {
      case P_PUSH_COL: st[sp++] = vm_col(P.cols[in.arg], v); break;
      case P_PUSH_INT: st[sp++] = VmVal{in.i, 0.0, 1}; break;
      case P_PUSH_DBL: st[sp++] = VmVal{0, in.d, 2}; break;
      case P_PUSH_NULL: st[sp++] = VmVal{0, 0.0, 0}; break;
      case P_PUSH_BOOL: st[sp++] = VmVal{in.i != 0, 0.0, 3}; break;
      case P_PUSH_DEPTH: st[sp++] = VmVal{depth, 0.0, 1}; break;
      case P_PUSH_DEG: {
        const DAdj &a = P.deg[in.arg];
        int64_t d = 0;
        for (int p = 0; p < a.n; ++p) d += (int64_t)(a.p[p].rp[v + 1] - a.p[p].rp[v]);
        st[sp++] = VmVal{d, 0.0, 1};
        break;
      }
      case P_ADD: case P_SUB: case P_MUL: case P_DIV: case P_MOD: {
        VmVal b = st[--sp], a = st[--sp];
        VmVal r{0, 0.0, 0};
        if (a.t != 0 && b.t != 0) {
          if (a.t != 2 && b.t != 2) {
            r.t = 1;
            switch (in.op) {
              case P_ADD: r.i = a.i + b.i; break;
              case P_SUB: r.i = a.i - b.i; break;
              case P_MUL: r.i = a.i * b.i; break;
              case P_DIV: if (b.i) r.i = a.i / b.i; else r.t = 0; break;
              default: if (b.i) r.i = a.i % b.i; else r.t = 0; break;
            }
          } else {
            double x = a.t == 2 ? a.d : (double)a.i, y = b.t == 2 ? b.d : (double)b.i;
            r.t = 2;
            switch (in.op) {
              case P_ADD: r.d = x + y; break;
              case P_SUB: r.d = x - y; break;
              case P_MUL: r.d = x * y; break;
              case P_DIV: r.d = x / y; break;
              default: r.d = fmod(x, y); break;
            }
          }
        }
        st[sp++] = r;
        break;
      }
      case P_EQ: case P_NE: {
        VmVal b = st[--sp], a = st[--sp];
        bool eq = a.t != 0 && b.t != 0 && vm_cmp(a, b) == 0;
        st[sp++] = VmVal{in.op == P_EQ ? eq : !eq, 0.0, 3};
        break;
      }
      case P_LT: case P_LE: case P_GT: case P_GE: {
        VmVal b = st[--sp], a = st[--sp];
        bool r = false;
        if (a.t != 0 && b.t != 0) {
          int c = vm_cmp(a, b);
          r = in.op == P_LT ? c < 0 : in.op == P_LE ? c <= 0 : in.op == P_GT ? c > 0 : c >= 0;
        }
        st[sp++] = VmVal{r, 0.0, 3};
        break;
      }
      case P_AND: case P_OR: {
        VmVal b = st[--sp], a = st[--sp];
        bool r = in.op == P_AND ? (vm_truthy(a) && vm_truthy(b)) : (vm_truthy(a) || vm_truthy(b));
        st[sp++] = VmVal{r, 0.0, 3};
        break;
      }
      case P_NOT: st[sp - 1] = VmVal{!vm_truthy(st[sp - 1]), 0.0, 3}; break;
      case P_TRUTH: st[sp - 1] = VmVal{vm_truthy(st[sp - 1]), 0.0, 3}; break;
      default: break;
    }
  }
  return vm_truthy(st[0]);
}

// host evaluation of a program that reads no vertex data (only constants and $depth)
bool eval_pred_const(const DPred &pred, int64_t depth) { return eval_pred(pred, 0, depth); }

// one lane per vertex, 64 vertices per wave → one u64 bitmap word per wave via ballot
// words [⌈V/64⌉, nwords) (padding) are written as zero
__global__ __launch_bounds__(256) void k_eval_bitmap(DPred P, uint32_t V, int64_t depth, uint64_t *words,
                                                     uint64_t nwords) {
  uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool b = v < V && eval_pred(P, (uint32_t)v, depth);
  uint64_t m = __ballot(b);
  if ((threadIdx.x & 63) == 0 && (v >> 6) < nwords) words[v >> 6] = m;
}

// "column OP constant" atoms (and the class test): EV bitmap words per wave, every load of the EV
// vertices (class id, presence, value; column descriptors from the kernel arguments) issued before
// any is used; loads are unconditional (index clamped) so none waits inside a branch
constexpr int kEvalWords = 4;
__device__ __forceinline__ uint64_t raw_col(const DColumn &c, uint64_t v) {
  return (c.type == OMX_PROP_INT64 || c.type == OMX_PROP_DOUBLE) ? ((const uint64_t *)c.values)[v]
                                                                 : (uint64_t)((const uint32_t *)c.values)[v];
}
__device__ __forceinline__ bool atom_true(const DPred &P, int k, uint64_t raw, bool present) {
  const DColumn &c = P.atom_c[k];
  if (!present || (c.type == OMX_PROP_STRING && (int32_t)(uint32_t)raw < 0)) return P.atom_op[k] == P_NE;
  if (P.atom_dbl[k]) {
    double a;
    if (c.type == OMX_PROP_DOUBLE) a = __longlong_as_double((long long)raw);
    else if (c.type == OMX_PROP_INT64) a = (double)(int64_t)raw;
    else if (c.type == OMX_PROP_BOOL) a = (uint32_t)raw != 0;
    else a = (double)(int32_t)(uint32_t)raw;
    const double b = P.atom_d[k];
    return atom_cmp(P.atom_op[k], a < b ? -1 : (a > b ? 1 : 0));
  }
  int64_t x;
  if (c.type == OMX_PROP_INT64) x = (int64_t)raw;
  else if (c.type == OMX_PROP_BOOL) x = (uint32_t)raw != 0;
  else x = (int32_t)(uint32_t)raw;
  const int64_t b = P.atom_i[k];
  return atom_cmp(P.atom_op[k], x < b ? -1 : (x > b ? 1 : 0));
}
// class c ∈ the predicate's polymorphic class set: the 4 mask words selected in registers (an index
// into the kernel-argument array by a lane value is a memory load, and the wave waits for it)
struct ClassMask {
  uint64_t m[4];
};
__device__ __forceinline__ ClassMask class_mask_regs(const DPred &P) {
  ClassMask r;
#pragma unroll
  for (int k = 0; k < 4; ++k)  // readfirstlane: values in SGPRs (a select of them cannot become a load)
    r.m[k] = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(P.class_mask[k] >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)P.class_mask[k]);
  return r;
}
__device__ __forceinline__ bool class_in_mask(const ClassMask &cm, uint32_t c) {
  const uint32_t w = c >> 6;
  // masks, not selects (a select chain is turned back into an indexed load)
  const uint64_t m = (cm.m[0] & (0ull - (uint64_t)(w == 0))) | (cm.m[1] & (0ull - (uint64_t)(w == 1))) |
                     (cm.m[2] & (0ull - (uint64_t)(w == 2))) | (cm.m[3] & (0ull - (uint64_t)(w == 3)));
  return (m >> (c & 63)) & 1ull;
}
__global__ __launch_bounds__(256) void k_eval_atoms(DPred P, uint32_t V, uint64_t *words, uint64_t nwords) {
  constexpr int EV = kEvalWords;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64 * EV;
  const ClassMask cm = class_mask_regs(P);
  uint64_t vv[EV];
  uint32_t cls[EV];
  uint64_t raw[4][EV];
  uint32_t pres[4][EV];
#pragma unroll
  for (int e = 0; e < EV; ++e) {
    const uint64_t v = (w0 + e) * 64 + lane;
    vv[e] = v < V ? v : V - 1;
    cls[e] = P.use_class ? P.vclass[vv[e]] : 0u;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k >= P.n_atoms) break;  // uniform
    const DColumn &c = P.atom_c[k];
#pragma unroll
    for (int e = 0; e < EV; ++e) {
      raw[k][e] = raw_col(c, vv[e]);
      pres[k][e] = c.present ? c.present[vv[e]] : 1u;
    }
  }
#pragma unroll
  for (int e = 0; e < EV; ++e) {
    const uint64_t v = (w0 + e) * 64 + lane;
    bool b = v < V;
    if (P.use_class) b = b && class_in_mask(cm, cls[e]);
    bool acc = P.conj != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= P.n_atoms) break;
      const bool r = atom_true(P, k, raw[k][e], pres[k][e] != 0);
      acc = P.conj ? (acc && r) : (acc || r);
    }
    const uint64_t m = __ballot(b && acc);
    if (lane == 0 && w0 + e < nwords) words[w0 + e] = m;
  }
}

// The same for atoms over 4-byte columns without absent values (the common WHERE: `age < 1`): a lane
// takes 4 consecutive vertices with one 16-byte load per column (and 8 bytes of class ids), so a wave
// instruction moves 1 KiB instead of 256 B; a word's 16 nibbles are OR-reduced across 16 lanes.
__global__ __launch_bounds__(256) void k_eval_atoms4(DPred P, uint32_t V, uint64_t *words, uint64_t nwords) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64 * 4;  // 4 words (256 vertices) per wave
  const uint64_t v0 = w0 * 64 + 4 * lane;
  const ClassMask cm = class_mask_regs(P);
  uint32_t cls[4] = {0, 0, 0, 0};
  uint32_t raw[4][4] = {};
  // wave-uniform: every wave but the last takes 16-byte column loads and 8-byte class loads, all issued
  // before any is used (a per-lane test made the compiler select between both forms and wait in between)
  const bool full = __builtin_amdgcn_readfirstlane((int)((w0 + 4) * 64 <= (uint64_t)V)) != 0;
  if (full) {
    uint2 c2 = make_uint2(0, 0);
    if (P.use_class) c2 = *reinterpret_cast<const uint2 *>(P.vclass + v0);
    uint4 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < P.n_atoms) x[k] = *reinterpret_cast<const uint4 *>((const uint32_t *)P.atom_c[k].values + v0);
    cls[0] = c2.x & 0xFFFFu, cls[1] = c2.x >> 16, cls[2] = c2.y & 0xFFFFu, cls[3] = c2.y >> 16;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < P.n_atoms) raw[k][0] = x[k].x, raw[k][1] = x[k].y, raw[k][2] = x[k].z, raw[k][3] = x[k].w;
  } else {
    if (P.use_class) {
#pragma unroll
      for (int j = 0; j < 4; ++j) cls[j] = P.vclass[v0 + j < V ? v0 + j : (uint64_t)V - 1];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= P.n_atoms) break;  // uniform
      const uint32_t *c = (const uint32_t *)P.atom_c[k].values;
#pragma unroll
      for (int j = 0; j < 4; ++j) raw[k][j] = c[v0 + j < V ? v0 + j : (uint64_t)V - 1];
    }
  }
  uint64_t nib = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bool b = v0 + j < V;
    if (P.use_class) b = b && class_in_mask(cm, cls[j]);
    bool acc = P.conj != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= P.n_atoms) break;
      const bool r = atom_true(P, k, raw[k][j], true);
      acc = P.conj ? (acc && r) : (acc || r);
    }
    nib |= (uint64_t)(b && acc) << j;
  }
  uint64_t x = nib << (4 * (lane & 15));
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) x |= __shfl_xor(x, off, 64);
  if ((lane & 15) == 0 && w0 + lane / 16 < nwords) words[w0 + lane / 16] = x;
}

// One comparison of an int32 column with an integer constant, no class test (M1's `age < 1`, `age >=
// 90`): the comparison is a range test lo <= x <= hi (negated for !=), and a wave takes 16 words (1,024
// vertices) a round with four 16-byte loads a lane in flight. The general kernel above holds 150 VGPRs
// when compiled for four groups a wave (3 waves a SIMD: 55 µs for RMAT-24's 67 MB column); this one
// holds few.
// (T = int64_t: the same over an int64 column, C5's `uid < 64` — 8 bytes a vertex, two 16-byte loads a
// group: 131 µs through the general kernel at RMAT-26, round 5)
constexpr int kAtom1U = 4;
// (words2: a second range test lo2…hi2 over the same column into its own bitmap — two predicates of a
// plan on one column, M1's root `age < 1` and last-hop `age >= 90`, in one pass over it)
template <class T>
__global__ __launch_bounds__(256) void k_eval_atom1(const T *col, int64_t lo, int64_t hi, int neg, uint32_t V,
                                                    uint64_t *words, uint64_t nwords, int64_t lo2, int64_t hi2, int neg2,
                                                    uint64_t *words2) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) / 64, nwv = (uint64_t)gridDim.x * 4;
  const uint64_t nrounds = (nwords + 4 * kAtom1U - 1) / (4 * kAtom1U);
  for (uint64_t rd = wave; rd < nrounds; rd += nwv) {
    const uint64_t w0 = rd * 4 * kAtom1U;
    const bool full = (w0 + 4 * kAtom1U) * 64 <= (uint64_t)V;  // wave-uniform
    T x[kAtom1U][4];
#pragma unroll
    for (int u = 0; u < kAtom1U; ++u) {
      const uint64_t v0 = (w0 + 4 * u) * 64 + 4 * lane;
      if (full) {
        if (sizeof(T) == 4) {
          const int4 q = *reinterpret_cast<const int4 *>(col + v0);
          x[u][0] = (T)q.x, x[u][1] = (T)q.y, x[u][2] = (T)q.z, x[u][3] = (T)q.w;
        } else {
          const longlong2 *p = reinterpret_cast<const longlong2 *>(col + v0);
          const longlong2 a = p[0], b = p[1];
          x[u][0] = (T)a.x, x[u][1] = (T)a.y, x[u][2] = (T)b.x, x[u][3] = (T)b.y;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) x[u][j] = col[v0 + j < V ? v0 + j : V - 1];
      }
    }
#pragma unroll
    for (int u = 0; u < kAtom1U; ++u) {
      const uint64_t v0 = (w0 + 4 * u) * 64 + 4 * lane;
      const T *e = x[u];
      uint64_t nib = 0, nib2 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool r = ((int64_t)e[j] >= lo && (int64_t)e[j] <= hi) != (neg != 0);
        nib |= (uint64_t)(r && v0 + j < V) << j;
        const bool r2 = ((int64_t)e[j] >= lo2 && (int64_t)e[j] <= hi2) != (neg2 != 0);
        nib2 |= (uint64_t)(r2 && v0 + j < V) << j;
      }
      uint64_t w = nib << (4 * (lane & 15)), w2 = nib2 << (4 * (lane & 15));
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) w |= __shfl_xor(w, off, 64);
      const uint64_t wi = w0 + 4 * u + lane / 16;
      if ((lane & 15) == 0 && wi < nwords) words[wi] = w;
      if (words2) {  // (wave-uniform)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) w2 |= __shfl_xor(w2, off, 64);
        if ((lane & 15) == 0 && wi < nwords) words2[wi] = w2;
      }
    }
  }
}

// pred is one int32 / int64 comparison with an integer constant, no class test: its range lo…hi (negated
// for !=)
static bool atom1_range(const DPred &pred, int64_t *plo, int64_t *phi, int *pneg) {
  const bool one = pred.n > 0 && pred.n_atoms == 1 && !pred.use_class && pred.atom_c[0].present == nullptr &&
                   (pred.atom_c[0].type == OMX_PROP_INT32 || pred.atom_c[0].type == OMX_PROP_INT64) &&
                   !pred.atom_dbl[0] && pred.atom_op[0] >= P_EQ && pred.atom_op[0] <= P_GE;
  if (!one) return false;
  const int64_t b = pred.atom_i[0];
  int64_t lo = INT64_MIN, hi = INT64_MAX;
  int neg = 0;
  switch (pred.atom_op[0]) {
    case P_EQ: lo = hi = b; break;
    case P_NE: lo = hi = b; neg = 1; break;
    case P_LT: if (b == INT64_MIN) lo = 1, hi = 0; else hi = b - 1; break;  // (lo > hi: nothing)
    case P_LE: hi = b; break;
    case P_GT: if (b == INT64_MAX) lo = 1, hi = 0; else lo = b + 1; break;
    default: lo = b; break;  // P_GE
  }
  *plo = lo, *phi = hi, *pneg = neg;
  return true;
}

static void launch_atom1(const DPred &pred, int64_t lo, int64_t hi, int neg, uint64_t *words, uint64_t *words2,
                         int64_t lo2, int64_t hi2, int neg2, uint32_t V, uint64_t nwords, hipStream_t s) {
  static int cus_of[64] = {};  // CUs of each device (queried once)
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    if (!cus_of[dev] && hipDeviceGetAttribute(&cus_of[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus_of[dev] = 256;
    cus = cus_of[dev];
  }
  const uint64_t rounds = (nwords + 4 * kAtom1U - 1) / (4 * kAtom1U);
  const uint64_t waves = std::min<uint64_t>(rounds, (uint64_t)std::max(cus, 1) * 32);
  if (pred.atom_c[0].type == OMX_PROP_INT32)
    hipLaunchKernelGGL(k_eval_atom1<int32_t>, dim3(nblocks(waves * 64, 256)), dim3(256), 0, s,
                       (const int32_t *)pred.atom_c[0].values, lo, hi, neg, V, words, nwords, lo2, hi2, neg2, words2);
  else
    hipLaunchKernelGGL(k_eval_atom1<int64_t>, dim3(nblocks(waves * 64, 256)), dim3(256), 0, s,
                       (const int64_t *)pred.atom_c[0].values, lo, hi, neg, V, words, nwords, lo2, hi2, neg2, words2);
  KCHECK("k_eval_atom1");
}

bool launch_eval_bitmap_pair(const DPred &a, const DPred &b, uint32_t V, uint64_t *wa, uint64_t *wb, hipStream_t s,
                             uint64_t nwords) {
  int64_t la, ha, lb, hb;
  int na, nb;
  if (!V || !atom1_range(a, &la, &ha, &na) || !atom1_range(b, &lb, &hb, &nb) ||
      a.atom_c[0].values != b.atom_c[0].values || a.atom_c[0].type != b.atom_c[0].type)
    return false;
  if (!nwords) nwords = ((uint64_t)V + 63) / 64;
  launch_atom1(a, la, ha, na, wa, wb, lb, hb, nb, V, nwords, s);
  return true;
}

// bits outside [lo, hi) cleared (a bitmap of an edge-records snapshot kept to one kind of record)
__global__ void k_bitmap_keep_range(uint64_t *words, uint64_t nwords, uint64_t lo, uint64_t hi) {
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b0 = w * 64;
    uint64_t m = 0;
    if (b0 + 64 > lo && b0 < hi) {
      m = ~0ull;
      if (b0 < lo) m &= ~0ull << (lo - b0);
      if (b0 + 64 > hi) m &= (1ull << (hi - b0)) - 1;
    }
    if (m != ~0ull) words[w] &= m;
  }
}
void launch_bitmap_keep_range(uint64_t *words, uint64_t nwords, uint64_t lo, uint64_t hi, hipStream_t s) {
  if (!nwords) return;
  hipLaunchKernelGGL(k_bitmap_keep_range, dim3((unsigned)std::min<uint64_t>(nblocks(nwords, 256), 4096)), dim3(256), 0, s,
                     words, nwords, lo, hi);
  KCHECK("k_bitmap_keep_range");
}

void launch_eval_bitmap(const DPred &pred, uint32_t V, int64_t depth, uint64_t *words, hipStream_t s,
                        uint64_t nwords) {
  if (!V) return;
  if (!nwords) nwords = ((uint64_t)V + 63) / 64;
  bool four = pred.n > 0 && pred.n_atoms > 0;
  for (int k = 0; four && k < pred.n_atoms; ++k)
    four = pred.atom_c[k].present == nullptr && pred.atom_c[k].type != OMX_PROP_INT64 &&
           pred.atom_c[k].type != OMX_PROP_DOUBLE;
  // one int32 / int64 comparison with an integer constant, no class test: the range-test kernel
  int64_t lo, hi;
  int neg;
  if (atom1_range(pred, &lo, &hi, &neg)) {
    launch_atom1(pred, lo, hi, neg, words, nullptr, 0, 0, 0, V, nwords, s);
    return;
  }
  if (four) {
    const uint64_t groups = (nwords + 3) / 4;
    hipLaunchKernelGGL(k_eval_atoms4, dim3(nblocks(groups * 64, 256)), dim3(256), 0, s, pred, V, words, nwords);
    KCHECK("k_eval_atoms4");
    return;
  }
  if (pred.n > 0 && pred.n_atoms > 0) {
    const uint64_t waves = (nwords + kEvalWords - 1) / kEvalWords;
    hipLaunchKernelGGL(k_eval_atoms, dim3(nblocks(waves * 64, 256)), dim3(256), 0, s, pred, V, words, nwords);
    KCHECK("k_eval_atoms");
    return;
  }
  hipLaunchKernelGGL(k_eval_bitmap, dim3(nblocks(nwords * 64, 256)), dim3(256), 0, s, pred, V, depth, words, nwords);
  KCHECK("k_eval_bitmap");
}

__global__ void k_bitmap_and(const uint64_t *a, uint64_t *b, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] &= a[i];
}
void launch_bitmap_and(const uint64_t *a, uint64_t *b, uint64_t n, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_bitmap_and, dim3(nblocks(n, 256)), dim3(256), 0, s, a, b, n);
  KCHECK("k_bitmap_and");
}

__device__ __forceinline__ uint64_t range_mask(uint64_t base, uint32_t lo, uint32_t hi) {
  // bits b of the word with lo <= base + b < hi
  if (base + 64 <= lo || base >= hi) return 0;
  uint64_t m = ~0ull;
  if (base < lo) m &= ~0ull << (lo - base);
  if (base + 64 > hi) m &= (hi - base >= 64) ? ~0ull : ((1ull << (hi - base)) - 1);
  return m;
}

__device__ __forceinline__ uint64_t shard_word(uint64_t w, uint64_t word, uint32_t V, int rank, int world,
                                               uint32_t lo, uint32_t hi) {
  uint64_t base = word * 64;
  w &= range_mask(base, lo, hi < V ? hi : V);
  if (world > 1) {
    uint64_t m = 0;
    for (int b = 0; b < 64; ++b)
      if ((base + b) % (uint64_t)world == (uint64_t)rank) m |= 1ull << b;
    w &= m;
  }
  return w;
}

__global__ void k_word_popc(const uint64_t *words, uint64_t n, uint32_t V, int rank, int world, uint32_t lo,
                            uint32_t hi, uint32_t *counts) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) counts[i] = __popcll(shard_word(words[i], i, V, rank, world, lo, hi));
}
void launch_word_popc(const uint64_t *words, uint64_t n, uint32_t V, int rank, int world, uint32_t lo, uint32_t hi,
                      uint32_t *counts, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_word_popc, dim3(nblocks(n, 256)), dim3(256), 0, s, words, n, V, rank, world, lo, hi, counts);
  KCHECK("k_word_popc");
}

__global__ void k_word_scatter(const uint64_t *words, uint64_t n, uint32_t V, int rank, int world, uint32_t lo,
                               uint32_t hi, const uint32_t *offsets, uint32_t *out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t w = shard_word(words[i], i, V, rank, world, lo, hi);
  uint32_t o = offsets[i];
  while (w) {
    int b = __builtin_ctzll(w);
    out[o++] = (uint32_t)(i * 64 + b);
    w &= w - 1;
  }
}
void launch_word_scatter(const uint64_t *words, uint64_t n, uint32_t V, int rank, int world, uint32_t lo, uint32_t hi,
                         const uint32_t *offsets, uint32_t *out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_word_scatter, dim3(nblocks(n, 256)), dim3(256), 0, s, words, n, V, rank, world, lo, hi, offsets,
                     out);
  KCHECK("k_word_scatter");
}

// ---- expansion ------------------------------------------------------------------------------------


__global__ void k_row_degree(const uint32_t *src, uint64_t R, DAdj adj, uint64_t *deg) {
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) deg[r] = adj_degree(adj, src[r]);
  else if (r == R) deg[R] = 0;
}
void launch_row_degree(const uint32_t *src, uint64_t R, const DAdj &adj, uint64_t *deg, hipStream_t s) {
  hipLaunchKernelGGL(k_row_degree, dim3(nblocks(R + 1, 256)), dim3(256), 0, s, src, R, adj, deg);
  KCHECK("k_row_degree");
}

// degrees of the rows [lo, hi) of one CSR (u32: a row of 2^32 or more entries does not occur in a
// partition's snapshot)
__global__ void k_row_degree_range(const uint64_t *rp, uint32_t lo, uint32_t hi, uint64_t *deg) {
  const uint64_t v = (uint64_t)lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v < hi) deg[v - lo] = rp[v + 1] - rp[v];
}
void launch_row_degree_range(const uint64_t *rp, uint32_t lo, uint32_t hi, uint64_t *deg, hipStream_t s) {
  if (hi <= lo) return;
  hipLaunchKernelGGL(k_row_degree_range, dim3(nblocks(hi - lo, 256)), dim3(256), 0, s, rp, lo, hi, deg);
  KCHECK("k_row_degree_range");
}

// merge path over A = row ends (offs[r+1]) and B = edge indices 0..E-1; a row end is consumed
// before edge j when offs[r+1] <= j.
__global__ void k_mp_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  uint64_t d = t * (uint64_t)kExpandTile;
  if (d > R + E) d = R + E;
  uint64_t lo = d > E ? d - E : 0, hi = d < R ? d : R;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (offs[mid + 1] <= d - 1 - mid) lo = mid + 1;
    else hi = mid;
  }
  part[t] = lo;
}
void launch_mp_partition(const uint64_t *offs, uint64_t R, uint64_t E, uint64_t ntiles, uint64_t *part,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_mp_partition, dim3(nblocks(ntiles + 1, 256)), dim3(256), 0, s, offs, R, E, ntiles, part);
  KCHECK("k_mp_partition");
}


// t ∈ N(v) for a sorted adjacency (lower_bound per part)
__device__ __forceinline__ bool adj_contains(const DAdj &a, uint32_t v, uint32_t t) {
  for (int p = 0; p < a.n; ++p) {
    uint64_t lo = a.p[p].rp[v], hi = a.p[p].rp[v + 1];
    const uint64_t end = hi;
    const uint32_t *col = a.p[p].col;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (col[mid] < t) lo = mid + 1;
      else hi = mid;
    }
    if (lo < end && col[lo] == t) return true;
  }
  return false;
}

__device__ __forceinline__ void wave_add_u64(unsigned long long *dst, uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if ((threadIdx.x & 63) == 0 && x) atomicAdd(dst, (unsigned long long)x);
}

// Light rows: merge-path tiles of kExpandTile (rows + edges) items, persistent blocks.
// MEMBER (implies FILTER): fused closing check, see ExpandArgs::member_src.
// set bit v, reading the word first: hub neighbours are marked again and again, and an atomic on a word
// that already holds the bit is wasted (a stale read only costs a redundant atomic)
__device__ __forceinline__ void mark_vertex(uint64_t *bm, uint32_t v) {
  const uint64_t bit = 1ull << (v & 63);
  if (!(__hip_atomic_load(&bm[v >> 6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
    atomicOr((unsigned long long *)&bm[v >> 6], (unsigned long long)bit);
}

template <bool SINGLE, bool FILTER, bool WRITE, bool MEMBER>
__global__ __launch_bounds__(kExpandBlock) void k_expand(ExpandArgs a) {
  constexpr int B = kExpandBlock, IPT = kExpandIPT, T = kExpandTile, W = B / 64;
  __shared__ uint64_t s_base[T + 1];  // SINGLE: first col index of the row's remaining edges; else [0] = skip of row 0
  __shared__ uint32_t s_vtx[SINGLE ? 1 : T + 1];
  __shared__ uint16_t s_ls[T + 1];    // local start of each row inside the tile
  __shared__ uint16_t s_seg[T];       // local row owning each tile edge
  __shared__ uint32_t s_wave[IPT * W];
  __shared__ uint32_t s_wmax[W];
  __shared__ uint32_t s_total;
  __shared__ uint32_t s_y[MEMBER ? T + 1 : 1];     // member source vertex of each tile row
  __shared__ uint32_t s_ydeg[MEMBER ? T + 1 : 1];  // its member-adjacency length

  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t arena = a.arena_base + (uint64_t)blockIdx.x * a.arena_cap;
  uint64_t acc = 0;
  uint64_t medges = 0, mprobes = 0;  // member-adjacency edges the check stands for, col[] probes made
  for (uint64_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) {
    const uint64_t d0 = t * (uint64_t)T;
    const uint64_t d1 = min(d0 + (uint64_t)T, a.R + a.E);
    const uint64_t i0 = a.part[t], i1 = a.part[t + 1];
    const uint64_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t ne = (uint32_t)(j1 - j0);
    if (ne == 0) continue;  // uniform
    const uint64_t rlast = min(i1, a.R - 1);
    const uint32_t nr = (uint32_t)(rlast - i0 + 1);

    for (uint32_t x = tid; x < ne; x += B) s_seg[x] = 0;
    __syncthreads();
    for (uint32_t lr = tid; lr < nr; lr += B) {
      const uint64_t r = i0 + lr;
      const uint64_t rs = a.offs[r], re = a.offs[r + 1];
      const uint64_t s = rs > j0 ? rs - j0 : 0;
      const uint64_t e = re < j1 ? (re > j0 ? re - j0 : 0) : ne;
      s_ls[lr] = (uint16_t)(s < ne ? s : ne);
      if (e > s && s < ne) s_seg[s] = (uint16_t)lr;
      const uint64_t skip = rs < j0 ? j0 - rs : 0;
      if (MEMBER) {
        const uint32_t y = a.member_src[r];
        s_y[lr] = y;
        s_ydeg[lr] = (uint32_t)adj_degree(a.member_adj, y);
      }
      if (SINGLE) {  // the row's first col index, precomputed by k_bin_fill (no dependent rp[src] load)
        s_base[lr] = a.lbase[r] + skip;
      } else {
        const uint32_t v = a.src[r];
        s_vtx[lr] = v;
        if (lr == 0) s_base[0] = skip;
      }
    }
    __syncthreads();
    // inclusive max-scan of s_seg (row index of the latest row starting at or before each edge)
    {
      uint32_t vals[IPT];
      uint32_t m = 0;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        uint32_t idx = tid * IPT + i;
        uint32_t x = idx < ne ? s_seg[idx] : 0;
        m = m > x ? m : x;
        vals[i] = m;
      }
      uint32_t incl = m;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= (uint32_t)off) incl = incl > y ? incl : y;
      }
      if (lane == 63) s_wmax[wave] = incl;
      uint32_t excl = __shfl_up(incl, 1, 64);
      if (lane == 0) excl = 0;
      __syncthreads();
      uint32_t wp = 0;
      for (uint32_t w = 0; w < wave; ++w) wp = wp > s_wmax[w] ? wp : s_wmax[w];
      uint32_t pre = excl > wp ? excl : wp;
#pragma unroll
      for (int i = 0; i < IPT; ++i) {
        uint32_t idx = tid * IPT + i;
        if (idx < ne) s_seg[idx] = (uint16_t)(pre > vals[i] ? pre : vals[i]);
      }
    }
    __syncthreads();

    uint32_t nb[IPT];
    uint16_t lrs[IPT];
    uint32_t passmask = 0;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      const uint32_t jl = k * B + tid;
      nb[k] = 0;
      lrs[k] = 0;
      if (jl < ne) {
        const uint32_t lr = s_seg[jl];
        uint64_t kk = jl - s_ls[lr];
        uint32_t n;
        if (SINGLE) {
          n = a.adj.p[0].col[s_base[lr] + kk];
        } else {
          const uint32_t v = s_vtx[lr];
          if (lr == 0) kk += s_base[0];
          n = 0;
          for (int p = 0; p < a.adj.n; ++p) {
            const uint64_t b0 = a.adj.p[p].rp[v], dp = a.adj.p[p].rp[v + 1] - b0;
            if (kk < dp) {
              n = a.adj.p[p].col[b0 + kk];
              break;
            }
            kk -= dp;
          }
        }
        nb[k] = n;
        lrs[k] = (uint16_t)lr;
        bool pass = FILTER ? (!a.filter || bm_test(a.filter, n)) : true;
        if (MEMBER && pass) {
          medges += s_ydeg[lr];
          pass = !a.member_filter || bm_test(a.member_filter, n);
          if (pass && a.member_adj.n != 1) pass = adj_contains(a.member_adj, s_y[lr], n);
        }
        passmask |= (uint32_t)pass << k;
      }
    }
    if (MEMBER && a.member_adj.n == 1) {
      // closing check n ∈ N(y) for the thread's IPT items at once: the binary searches advance in
      // lockstep, so each round issues up to IPT independent loads instead of one dependent chain
      const uint64_t *mrp = a.member_adj.p[0].rp;
      const uint32_t *mcol = a.member_adj.p[0].col;
      uint64_t lo[IPT], hi[IPT], end[IPT];
      uint32_t act = passmask;
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        lo[k] = hi[k] = end[k] = 0;
        if ((act >> k) & 1u) {
          const uint32_t y = s_y[lrs[k]];
          lo[k] = mrp[y];
          hi[k] = end[k] = mrp[y + 1];
        }
      }
      uint32_t srch = act;
      while (srch) {
        mprobes += (uint64_t)__popc(srch);
        uint32_t x[IPT];
        uint64_t mid[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          mid[k] = (lo[k] + hi[k]) >> 1;
          x[k] = ((srch >> k) & 1u) ? mcol[mid[k]] : 0u;
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          if ((srch >> k) & 1u) {
            if (x[k] < nb[k]) lo[k] = mid[k] + 1;
            else hi[k] = mid[k];
            if (lo[k] >= hi[k]) srch &= ~(1u << k);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < IPT; ++k)
        if (((act >> k) & 1u) && !(lo[k] < end[k] && mcol[lo[k]] == nb[k])) passmask &= ~(1u << k);
    }

    // the items' first kCvRegs carried values are all requested before the first store: loaded next to
    // the store that consumes it, each one waited for its own round trip (8 items × columns per thread);
    // two columns in registers (M1's a, b) keep the kernel at 5 waves per SIMD
    constexpr int kCvRegs = 2;
    uint32_t cv[WRITE ? IPT : 1][kCvRegs];
    if (WRITE) {
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        const uint64_t r = i0 + lrs[k];
        const bool live = k * B + tid < ne && (FILTER ? ((passmask >> k) & 1u) != 0 : true);
#pragma unroll
        for (int c = 0; c < kCvRegs; ++c) cv[k][c] = live && c < a.ncarry ? a.carry_in[c][r] : 0u;
      }
    }
    if (!FILTER) {
      if (WRITE) {
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
          const uint32_t jl = k * B + tid;
          if (jl < ne) {
            const uint64_t o = a.dense_base + j0 + jl;
            const uint64_t r = i0 + lrs[k];
            a.out_dst[o] = nb[k];
#pragma unroll
            for (int c = 0; c < kCvRegs; ++c)
              if (c < a.ncarry) a.carry_out[c][o] = cv[k][c];
            for (int c = kCvRegs; c < a.ncarry; ++c) a.carry_out[c][o] = a.carry_in[c][r];
          }
        }
      } else if (a.mark) {
#pragma unroll
        for (int k = 0; k < IPT; ++k)
          if (k * B + tid < ne) mark_vertex(a.mark, nb[k]);
      }
      __syncthreads();  // LDS reuse by the next tile
      continue;
    }

    // compaction: wave ballots per item row k, wave totals scanned in LDS (edge order preserved)
    uint64_t masks[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
      masks[k] = __ballot((passmask >> k) & 1u);
      if (lane == 0) s_wave[k * W + wave] = (uint32_t)__popcll(masks[k]);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (int x = 0; x < IPT * W; ++x) {
        uint32_t c = s_wave[x];
        s_wave[x] = run;
        run += c;
      }
      s_total = run;
    }
    __syncthreads();
    if (WRITE) {
#pragma unroll
      for (int k = 0; k < IPT; ++k) {
        if ((passmask >> k) & 1u) {
          const uint64_t o = arena + acc + s_wave[k * W + wave] + lane_prefix(masks[k]);
          const uint64_t r = i0 + lrs[k];
          a.out_dst[o] = nb[k];
#pragma unroll
          for (int c = 0; c < kCvRegs; ++c)
            if (c < a.ncarry) a.carry_out[c][o] = cv[k][c];
          for (int c = kCvRegs; c < a.ncarry; ++c) a.carry_out[c][o] = a.carry_in[c][r];
        }
      }
    }
    acc += s_total;
    __syncthreads();  // LDS reuse by the next tile
  }
  if (MEMBER) {  // one atomic per block and counter (per-wave atomics on one address serialise)
    __shared__ uint64_t s_mc[2][W];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      medges += __shfl_xor(medges, off, 64);
      mprobes += __shfl_xor(mprobes, off, 64);
    }
    if (lane == 0) {
      s_mc[0][wave] = medges;
      s_mc[1][wave] = mprobes;
    }
    __syncthreads();
    if (tid < 2) {
      uint64_t t = 0;
      for (int w = 0; w < W; ++w) t += s_mc[tid][w];
      if (t) atomicAdd(a.member_edges + tid, (unsigned long long)t);
    }
  }
  if (FILTER && tid == 0) {
    a.seg_count[a.seg_base + blockIdx.x] = (uint32_t)acc;
    a.seg_start[a.seg_base + blockIdx.x] = arena;
  }
}

// Heavy rows: one chunk = ≤ kChunk edges of one row inside one kChunk-aligned col window, owned by
// ONE wave (the 4 waves of a block are independent: no LDS, no barriers). Lane l takes edge l of
// each of the 16 64-edge slots: col[] loads are fully coalesced dwords, and since a row's adjacency
// is sorted, the 64 bitmap probes of one slot cover 64 consecutive neighbours — for hub rows a
// handful of cache lines instead of one line per lane. Compaction by one ballot + mbcnt per slot, so
// each slot's survivors land contiguously (coalesced stores) in the wave's private arena; the row's
// carried columns are chunk constants. The next chunk's descriptor and col[] words are loaded before
// the current chunk is filtered (software pipeline).
__device__ __forceinline__ bool bm_test32(const uint32_t *bm, uint32_t v) { return (bm[v >> 5] >> (v & 31)) & 1u; }

template <bool FILTER, bool WRITE, bool MEMBER, int NS = kHeavySlots>
__global__ __launch_bounds__(kHeavyBlock) void k_expand_heavy(ExpandArgs a) {
  constexpr int WPB = kHeavyBlock / 64;
  constexpr uint64_t CH = 64 * NS;  // the chunk window
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wid = (uint64_t)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * WPB;
  const uint64_t arena = a.arena_base + wid * a.arena_cap;
  const uint32_t *bm32 = reinterpret_cast<const uint32_t *>(a.filter);
  uint64_t acc = 0;
  uint64_t medges = 0, mprobes = 0;
  auto load = [&](const ChunkDesc &d, uint32_t (&q)[NS]) {
    const uint64_t win = d.lo / CH * CH;
    const uint32_t *col = a.adj.p[d.part].col + win;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint64_t idx = win + i * 64 + lane;
      q[i] = (idx >= d.lo && idx < d.hi) ? col[i * 64 + lane] : 0u;
    }
  };
  // the carried values of a chunk's row are loaded with its descriptor's prefetch (one chunk ahead)
  auto carry_load = [&](const ChunkDesc &dd, uint32_t (&cv)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) cv[k] = WRITE && k < a.ncarry ? a.carry_in[k][dd.row] : 0u;
  };
  uint64_t c = wid;
  ChunkDesc d{};
  uint32_t q[NS], cv[4] = {0, 0, 0, 0};
  if (c < a.nchunks) {
    d = a.chunks[c];
    load(d, q);
    carry_load(d, cv);
  }
  while (c < a.nchunks) {
    const uint64_t cn = c + nw;
    const uint64_t win = d.lo / CH * CH;
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const uint64_t idx = win + i * 64 + lane;
      bool ok = idx >= d.lo && idx < d.hi;
      if (FILTER && ok && bm32) ok = bm_test32(bm32, q[i]);
      mask |= (uint32_t)ok << i;
    }
    if (MEMBER) {  // the chunk's row has one member source: every lane searches the same sorted list
      const uint32_t y = a.member_src[d.row];
      const uint64_t ydeg = adj_degree(a.member_adj, y);
      medges += (uint64_t)__popc(mask) * ydeg;
      mprobes += (uint64_t)__popc(mask) * (uint64_t)(64 - __builtin_clzll(ydeg | 1));  // ⌈log₂⌉-ish steps
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if ((mask >> i) & 1u) {
          const bool keep = (!a.member_filter || bm_test(a.member_filter, q[i])) && adj_contains(a.member_adj, y, q[i]);
          mask &= ~((uint32_t)!keep << i);
        }
    }
    // prefetch the next chunk
    ChunkDesc dn = d;
    uint32_t qn[NS], cvn[4] = {0, 0, 0, 0};
    if (cn < a.nchunks) {
      dn = a.chunks[cn];
      load(dn, qn);
      carry_load(dn, cvn);
    }
    const uint32_t r = d.row;
    if (WRITE) {
      const int nc = a.ncarry;
      uint64_t base = FILTER ? arena + acc : 0;
#pragma unroll
      for (int i = 0; i < NS; ++i) {
        const bool bit = (mask >> i) & 1u;
        uint64_t o;
        if (FILTER) {
          const uint64_t m = __ballot(bit);
          o = base + lane_prefix(m);
          base += __popcll(m);
        } else {
          o = d.dense + (win + i * 64 + lane - d.lo);
        }
        // (measured alternatives, slower here: non-temporal stores 1.6×, profiles/r02/nt; loads shifted
        // so every dense store is 256-B aligned, 17 slots per chunk, +9 %, profiles/r02/aligned)
        if (bit) {
          a.out_dst[o] = q[i];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (k < nc) a.carry_out[k][o] = cv[k];
          for (int k = 4; k < nc; ++k) a.carry_out[k][o] = a.carry_in[k][r];
        }
      }
      if (FILTER) acc = base - arena;
    } else if (!FILTER && a.mark) {
#pragma unroll
      for (int i = 0; i < NS; ++i)
        if ((mask >> i) & 1u) mark_vertex(a.mark, q[i]);
    } else if (FILTER) {
      uint32_t cnt = __popc(mask);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
      acc += cnt;
    }
    c = cn;
    d = dn;
#pragma unroll
    for (int i = 0; i < NS; ++i) q[i] = qn[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) cv[k] = cvn[k];
  }
  if (MEMBER) {
    wave_add_u64(a.member_edges, medges);
    wave_add_u64(a.member_edges + 1, mprobes);
  }
  if (FILTER && lane == 0) {
    a.seg_count[a.seg_base + wid] = (uint32_t)acc;
    a.seg_start[a.seg_base + wid] = arena;
  }
}

// ---- LDS-sliced heavy expansion ---------------------------------------------------------------------
// The L2-probe kernel above issues one L1→L2 request per filtered edge whenever a 64-neighbour slot
// spans more than a few cache lines (rows of degree ~1K–100K on a V = 4M graph), and that request rate,
// not HBM, bounds it. Here the V-bit target bitmap is cut into 128 KiB slices (2^20 vertices) that a
// workgroup stages in LDS, and every heavy row's sorted adjacency is cut at the slice boundaries, so a
// chunk's probes all land in the slice its workgroup holds. HBM then only streams col[] (coalesced
// dwords, next chunk prefetched) and the surviving rows.

// sliced chunks need no window alignment (buffer loads with a per-chunk base): ⌈len / kChunk⌉ pieces
__device__ __forceinline__ uint32_t chunk_pieces(uint64_t lo, uint64_t hi) {
  return hi > lo ? (uint32_t)((hi - lo + kChunk - 1) / kChunk) : 0u;
}

// cut[q] = first index in col[b, e) whose neighbour is ≥ q·2^shift (cut[0] = b, cut[P] = e); the P−1
// binary searches run side by side so their loads overlap. MAXP ≥ P is a compile-time bound so the
// per-slice arrays stay in registers; positions are kept relative to b (a row has < 2^32 edges).
template <int MAXP>
__device__ __forceinline__ void slice_cuts(const uint32_t *col, uint64_t b, uint64_t e, uint32_t P, uint32_t shift,
                                           uint32_t (&cut)[MAXP + 1]) {
  const uint32_t n = (uint32_t)(e - b);
  const uint32_t *c = col + b;
  uint32_t hi[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q) {
    cut[q] = 0;
    hi[q] = q > 0 && (uint32_t)q < P ? n : 0;
  }
  bool any = n > 0;
  while (any) {
    any = false;
    uint32_t x[MAXP], mid[MAXP];
#pragma unroll
    for (int q = 1; q < MAXP; ++q) {
      mid[q] = (cut[q] + hi[q]) >> 1;
      x[q] = cut[q] < hi[q] ? c[mid[q]] : 0u;
    }
#pragma unroll
    for (int q = 1; q < MAXP; ++q) {
      if (cut[q] < hi[q]) {
        if ((uint64_t)x[q] < ((uint64_t)q << shift)) cut[q] = mid[q] + 1;
        else hi[q] = mid[q];
        any |= cut[q] < hi[q];
      }
    }
  }
#pragma unroll
  for (int q = 1; q <= MAXP; ++q)
    if ((uint32_t)q >= P) cut[q] = n;
}

// slice-cut index of one CSR: cuts[v·(P−1) + q−1] = cut[q] of row v (relative to the row start)
template <int MAXP>
__global__ __launch_bounds__(256) void k_build_cuts(const uint64_t *rp, const uint32_t *col, uint32_t vlo, uint32_t vhi,
                                                    uint32_t P, uint32_t shift, uint32_t *cuts) {
  const uint64_t v = vlo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= vhi) return;
  uint32_t cut[MAXP + 1];
  slice_cuts<MAXP>(col, rp[v], rp[v + 1], P, shift, cut);
#pragma unroll
  for (int q = 1; q < MAXP; ++q)
    if ((uint32_t)q < P) cuts[v * (P - 1) + q - 1] = cut[q];
}

// the slice bounds of row v in part p (cut[0] = 0, cut[P] = degree)
template <int MAXP>
__device__ __forceinline__ void load_cuts(const uint32_t *c, uint32_t v, uint32_t n, uint32_t P,
                                          uint32_t (&cut)[MAXP + 1]) {
  cut[0] = 0;
#pragma unroll
  for (int q = 1; q <= MAXP; ++q) cut[q] = (uint32_t)q < P ? c[(uint64_t)v * (P - 1) + q - 1] : n;
}

#define OMX_BY_MAXP(P, CALL) \
  do {                       \
    if ((P) <= 1) CALL(1);   \
    else if ((P) <= 2) CALL(2); \
    else if ((P) <= 4) CALL(4); \
    else if ((P) <= 8) CALL(8); \
    else CALL(16);           \
  } while (0)

void launch_build_cuts(const uint64_t *rp, const uint32_t *col, uint32_t vlo, uint32_t vhi, uint32_t nslices,
                       uint32_t shift, uint32_t *cuts, hipStream_t s) {
  if (vhi <= vlo || nslices < 2) return;
#define OMX_BC(M) hipLaunchKernelGGL(k_build_cuts<M>, dim3(nblocks(vhi - vlo, 256)), dim3(256), 0, s, rp, col, vlo, vhi, \
                                     nslices, shift, cuts)
  OMX_BY_MAXP(nslices, OMX_BC);
#undef OMX_BC
  KCHECK("k_build_cuts");
}

// ---- degree binning ---------------------------------------------------------------------------------
// Keys of row r (all 0 for r ≥ R): x[0] = light degree (0 < d < heavy_deg), x[1] = heavy degree,
// x[2] = 1 for a light row, x[3 + q] = heavy chunks in slice q. Unsliced (MAXP = 1): chunks are the
// kChunk-aligned windows the row's parts touch.
template <bool SLICED, int MAXP>
__device__ __forceinline__ void row_bins(const uint32_t *src, uint64_t r, uint64_t R, const DAdj &adj,
                                         const DCuts &cuts, uint64_t heavy_deg, uint32_t P,
                                         uint64_t (&x)[kBinKeys + MAXP], uint32_t cs = 10) {
#pragma unroll
  for (int k = 0; k < kBinKeys + MAXP; ++k) x[k] = 0;
  if (r >= R) return;
  const uint32_t v = src[r];
  const uint64_t d = adj_degree(adj, v);
  if (d < heavy_deg) {
    x[0] = d;
    x[2] = d > 0;
    return;
  }
  x[1] = d;
  for (int p = 0; p < adj.n; ++p) {
    const uint64_t b = adj.p[p].rp[v], e = adj.p[p].rp[v + 1];
    if (SLICED) {
      uint32_t cut[MAXP + 1];
      load_cuts<MAXP>(cuts.c[p], v, (uint32_t)(e - b), P, cut);
#pragma unroll
      for (int q = 0; q < MAXP; ++q) x[kBinKeys + q] += chunk_pieces(cut[q], cut[q + 1]);
    } else if (e > b) {
      x[kBinKeys] += ((e - 1) >> cs) - (b >> cs) + 1;
    }
  }
}

// block-wide exclusive scans of K u64 values per thread in one pass; x becomes exclusive, tot the sums
template <int B, int K>
__device__ __forceinline__ void block_excl_scan_k(uint64_t (&x)[K], uint64_t (&tot)[K], uint64_t *s_w) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t incl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    incl[k] = x[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(incl[k], off, 64);
      if (lane >= (uint32_t)off) incl[k] += y;
    }
    if (lane == 63) s_w[k * (B / 64) + wave] = incl[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    uint64_t woff = 0, t = 0;
#pragma unroll
    for (int w = 0; w < B / 64; ++w) {
      const uint64_t y = s_w[k * (B / 64) + w];
      woff += w < (int)wave ? y : 0;
      t += y;
    }
    tot[k] = t;
    x[k] = woff + incl[k] - x[k];
  }
}

// The binning keys' block scan with the per-slice chunk counts packed two to a u64 (lo, hi halves):
// 3 + MAXP/2 scans instead of 3 + MAXP, so the 16-slice kernels hold half the registers (226 VGPRs, 2
// waves per SIMD, before). A half cannot carry into the other: a block's chunks of one slice stay far
// below 2^32 (that would take > 2^41 edges in 256 rows).
template <int MAXP>
constexpr int bin_scan_keys() { return kBinKeys + (MAXP + 1) / 2; }
template <int B, int MAXP>
__device__ __forceinline__ void bin_block_scan(uint64_t (&x)[kBinKeys + MAXP], uint64_t (&tot)[kBinKeys + MAXP],
                                               uint64_t *s_w) {
  constexpr int NP = (MAXP + 1) / 2, K2 = kBinKeys + NP;
  uint64_t y[K2], t2[K2];
#pragma unroll
  for (int k = 0; k < kBinKeys; ++k) y[k] = x[k];
#pragma unroll
  for (int i = 0; i < NP; ++i)
    y[kBinKeys + i] = x[kBinKeys + 2 * i] | (2 * i + 1 < MAXP ? x[kBinKeys + 2 * i + 1] << 32 : 0ull);
  block_excl_scan_k<B, K2>(y, t2, s_w);
#pragma unroll
  for (int k = 0; k < kBinKeys; ++k) x[k] = y[k], tot[k] = t2[k];
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    x[kBinKeys + 2 * i] = (uint32_t)y[kBinKeys + i];
    tot[kBinKeys + 2 * i] = (uint32_t)t2[kBinKeys + i];
    if (2 * i + 1 < MAXP) {
      x[kBinKeys + 2 * i + 1] = y[kBinKeys + i] >> 32;
      tot[kBinKeys + 2 * i + 1] = t2[kBinKeys + i] >> 32;
    }
  }
}

template <bool SLICED, int MAXP>
__global__ __launch_bounds__(kBinBlock) void k_bin_count(const uint32_t *src, uint64_t R, DAdj adj, DCuts cuts,
                                                          uint64_t heavy_deg, uint32_t P, uint64_t *blk, uint32_t cs) {
  constexpr int K = kBinKeys + MAXP;
  __shared__ uint64_t s_w[bin_scan_keys<MAXP>() * (kBinBlock / 64)];
  const uint64_t r = (uint64_t)blockIdx.x * kBinBlock + threadIdx.x;
  uint64_t x[K], tot[K];
  row_bins<SLICED, MAXP>(src, r, R, adj, cuts, heavy_deg, P, x, cs);
  bin_block_scan<kBinBlock, MAXP>(x, tot, s_w);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if ((uint32_t)k < kBinKeys + P) blk[(uint64_t)k * gridDim.x + blockIdx.x] = tot[k];
  }
}

// one workgroup: exclusive scan of every key's tile sums in place (all keys' loads issued together),
// the slices' chunk bounds and the mail {EL, EH, chunks, light rows, qb[0..P]}
// PER > 0: every thread owns PER consecutive tiles (nb ≤ 1024·PER), loaded all at once (clamped
// indices, no branches) and kept in registers for the write-back; PER = 0: a loop per key
template <int MAXP, int PER>
__global__ __launch_bounds__(1024) void k_bin_scan(uint64_t *blk, uint32_t nb, uint32_t P, uint64_t *qb, Mail mail,
                                                   const unsigned long long *extra, uint32_t nextra) {
  constexpr int K = kBinKeys + MAXP, PV = PER > 0 ? PER : 1;
  __shared__ unsigned long long s_w[K][16];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t per = PER > 0 ? PER : (nb + 1023) / 1024;
  const uint32_t i0 = min(nb, threadIdx.x * per), i1 = min(nb, i0 + per);
  unsigned long long c[K], incl[K];
  uint64_t v[K][PV];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    c[k] = 0;
    if (PER > 0) {
#pragma unroll
      for (int p = 0; p < PV; ++p) {
        const uint32_t i = i0 + p;
        const uint64_t x = blk[(uint64_t)((uint32_t)k < kBinKeys + P ? k : 0) * nb + (i < nb ? i : nb - 1)];
        // a mask, not a select: the load stays unconditional (a select lets it sink into a branch,
        // and every branch then waits for its load)
        v[k][p] = x & (0ull - (uint64_t)(i < i1 && (uint32_t)k < kBinKeys + P));
        c[k] += v[k][p];
      }
    } else if ((uint32_t)k < kBinKeys + P) {
      for (uint32_t i = i0; i < i1; ++i) c[k] += blk[(uint64_t)k * nb + i];
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    incl[k] = c[k];
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const unsigned long long y = __shfl_up(incl[k], off, 64);
      if (lane >= (uint32_t)off) incl[k] += y;
    }
    if (lane == 63) s_w[k][wave] = incl[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if ((uint32_t)k >= kBinKeys + P) continue;
    unsigned long long run = 0;
    for (uint32_t w = 0; w < wave; ++w) run += s_w[k][w];
    run += incl[k] - c[k];
    uint64_t *a = blk + (uint64_t)k * nb;
    if (PER > 0) {
#pragma unroll
      for (int p = 0; p < PV; ++p) {
        if (i0 + p < i1) a[i0 + p] = run;
        run += v[k][p];
      }
    } else {
      for (uint32_t i = i0; i < i1; ++i) {
        const uint64_t y = a[i];
        a[i] = run;
        run += y;
      }
    }
  }
  if (threadIdx.x == 0) {
    unsigned long long tot[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      tot[k] = 0;
      for (int w = 0; w < 16; ++w) tot[k] += s_w[k][w];
    }
    uint64_t q0 = 0;
    mail.p[0] = tot[0];
    mail.p[1] = tot[1];
    mail.p[3] = tot[2];
#pragma unroll
    for (int q = 0; q < MAXP; ++q) {
      if ((uint32_t)q >= P) break;
      qb[q] = q0;
      mail.p[4 + q] = q0;
      q0 += tot[kBinKeys + q];
    }
    qb[P] = q0;
    mail.p[4 + P] = q0;
    mail.p[2] = q0;
    for (uint32_t i = 0; i < nextra; ++i) mail.p[5 + P + i] = extra[i];
    mail_post(mail);
  }
}

// The same scan with one workgroup per key (nb ≤ 4096: four tiles a thread, in registers): the keys'
// scans run side by side instead of one after another in a single workgroup (52 µs at M1's 3.6 K
// tiles × 19 keys), and k_bin_scan_post turns the keys' totals into the slices' chunk bounds and the
// same mail as k_bin_scan's.
__global__ __launch_bounds__(1024) void k_bin_scan_key(uint64_t *blk, uint32_t nb, uint64_t *tot) {
  constexpr int PER = 4;
  __shared__ unsigned long long s_w[16];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t *a = blk + (uint64_t)blockIdx.x * nb;
  const uint32_t i0 = threadIdx.x * PER;
  uint64_t v[PER];
  unsigned long long c = 0;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const uint32_t i = i0 + p;
    const uint64_t x = a[i < nb ? i : nb - 1];
    v[p] = x & (0ull - (uint64_t)(i < nb));  // a mask, not a select: the load stays unconditional
    c += v[p];
  }
  unsigned long long incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += y;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  unsigned long long run = incl - c, all = 0;
  for (uint32_t w = 0; w < 16; ++w) {
    if (w < wave) run += s_w[w];
    all += s_w[w];
  }
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    if (i0 + p < nb) a[i0 + p] = run;
    run += v[p];
  }
  if (threadIdx.x == 0) tot[blockIdx.x] = all;
}
__global__ void k_bin_scan_post(const uint64_t *tot, uint32_t P, uint64_t *qb, Mail mail,
                                const unsigned long long *extra, uint32_t nextra) {
  if (threadIdx.x != 0) return;
  uint64_t q0 = 0;
  mail.p[0] = tot[0];
  mail.p[1] = tot[1];
  mail.p[3] = tot[2];
  for (uint32_t q = 0; q < P; ++q) {
    qb[q] = q0;
    mail.p[4 + q] = q0;
    q0 += tot[kBinKeys + q];
  }
  qb[P] = q0;
  mail.p[4 + P] = q0;
  mail.p[2] = q0;
  for (uint32_t i = 0; i < nextra; ++i) mail.p[5 + P + i] = extra[i];
  mail_post(mail);
}

// Every tile redoes its rows' keys, adds the tile prefixes and writes the light offsets, the light
// rows' first col index and the heavy rows' chunks. lr.row == nullptr: light data indexed by row
// (loffs[R+1], lbase[R]: merge-path kernel); else compacted to the light rows in order (loffs[NL+1],
// lbase, lr.row, lr.cuts[(q−1)·NL + i] = slice cut q of light row i: sliced light kernel).
template <bool SLICED, int MAXP>
__global__ __launch_bounds__(kBinBlock) void k_bin_fill(const uint32_t *src, uint64_t R, DAdj adj, DCuts cuts,
                                                         uint64_t heavy_deg, uint32_t P, const uint64_t *blk,
                                                         const uint64_t *qb, uint64_t *loffs, uint64_t *lbase,
                                                         LightRows lr, ChunkDesc *chunks, SliceChunk *schunks,
                                                         uint32_t cs) {
  constexpr int K = kBinKeys + MAXP;
  __shared__ uint64_t s_w[bin_scan_keys<MAXP>() * (kBinBlock / 64)];
  const uint64_t r = (uint64_t)blockIdx.x * kBinBlock + threadIdx.x;
  const uint32_t nb = gridDim.x;
  uint64_t x[K], tot[K];
  row_bins<SLICED, MAXP>(src, r, R, adj, cuts, heavy_deg, P, x, cs);
  const uint64_t heavy = x[1], light = x[2];
  bin_block_scan<kBinBlock, MAXP>(x, tot, s_w);
  if (r > R) return;
  const uint64_t lo = x[0] + blk[blockIdx.x];
  if (lr.row) {
    const uint64_t i = x[2] + blk[2ull * nb + blockIdx.x];  // compact index of a light row
    if (r == R) {
      loffs[i] = lo;  // i = NL
      return;
    }
    if (light) {
      // every load before the first store: vector memory completes in order, so a load issued after
      // a store would wait for it (the loop of load/store pairs cost 0.2 ms a hop at M1)
      const uint32_t v = src[r];
      const uint64_t base = adj.p[0].rp[v];
      uint32_t cv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) cv[c] = c < lr.nc ? lr.cin[c][r] : 0;
      uint32_t cut[MAXP + 1];
      if (SLICED) load_cuts<MAXP>(cuts.c[0], v, 0u, P, cut);
      loffs[i] = lo;
      lbase[i] = base;
      lr.row[i] = (uint32_t)r;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < lr.nc) lr.carry[c][i] = cv[c];
      if (SLICED) {
#pragma unroll
        for (int q = 1; q < MAXP; ++q)
          if ((uint32_t)q < P) lr.cuts[(uint64_t)(q - 1) * lr.nl + i] = cut[q];
      }
      return;
    }
  } else {
    loffs[r] = lo;
    if (r == R) return;
    if (adj.n == 1) lbase[r] = adj.p[0].rp[src[r]];  // (an L1 hit: row_bins just read it)
  }
  if (!heavy) return;
  const uint32_t v = src[r];
  if (!SLICED) {
    uint64_t o = x[kBinKeys] + blk[(uint64_t)kBinKeys * nb + blockIdx.x];
    uint64_t pos = x[1] + blk[(uint64_t)nb + blockIdx.x];  // dense output index of the row's first edge
    for (int p = 0; p < adj.n; ++p) {
      const uint64_t b = adj.p[p].rp[v], e = adj.p[p].rp[v + 1];
      const uint64_t ch = 1ull << cs;
      for (uint64_t w = b >> cs << cs; e > b && w < e; w += ch) {  // an empty part has no chunk
        const uint64_t clo = w > b ? w : b, chi = w + ch < e ? w + ch : e;
        chunks[o++] = ChunkDesc{clo, chi, pos + (clo - b), (uint32_t)r, (uint32_t)p};
      }
      pos += e - b;
    }
    return;
  }
  uint64_t o[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q)
    o[q] = (uint32_t)q < P ? x[kBinKeys + q] + blk[(uint64_t)(kBinKeys + q) * nb + blockIdx.x] + qb[q] : 0;
  for (int p = 0; p < adj.n; ++p) {
    const uint64_t b = adj.p[p].rp[v], e = adj.p[p].rp[v + 1];
    uint32_t cut[MAXP + 1];
    load_cuts<MAXP>(cuts.c[p], v, (uint32_t)(e - b), P, cut);
#pragma unroll
    for (int q = 0; q < MAXP; ++q) {
      for (uint32_t clo = cut[q]; clo < cut[q + 1]; clo += kChunk) {  // as chunk_pieces
        const uint32_t chi = clo + kChunk < cut[q + 1] ? clo + kChunk : cut[q + 1];
        schunks[o[q]++] = SliceChunk{b + clo, (uint32_t)r, (uint16_t)(chi - clo), (uint16_t)p};
      }
    }
  }
}

void launch_bin_count(bool sliced, const uint32_t *src, uint64_t R, const DAdj &adj, const DCuts &cuts,
                      uint64_t heavy_deg, uint32_t P, uint64_t *blk, hipStream_t s, uint32_t chunk_shift) {
  const unsigned nb = bin_tiles(R);
  if (!sliced) {
    hipLaunchKernelGGL((k_bin_count<false, 1>), dim3(nb), dim3(kBinBlock), 0, s, src, R, adj, cuts, heavy_deg, 1u, blk,
                       chunk_shift);
  } else {
#define OMX_BN(M) hipLaunchKernelGGL((k_bin_count<true, M>), dim3(nb), dim3(kBinBlock), 0, s, src, R, adj, cuts, \
                                     heavy_deg, P, blk, 10u)
    OMX_BY_MAXP(P, OMX_BN);
#undef OMX_BN
  }
  KCHECK("k_bin_count");
}
void launch_bin_scan(uint64_t *blk, uint64_t R, uint32_t P, uint64_t *qb, const Mail &mail, hipStream_t s,
                     const unsigned long long *extra, uint32_t nextra) {
  const unsigned nb = bin_tiles(R);
  if (5 + P + nextra >= (uint32_t)kMailSeq) fail(OMX_E_INVALID, "internal: bin-scan mail overflows");
  if (nb <= 4096 && P > 4) {  // one workgroup per key, then the bounds and the mail
    uint64_t *tot = qb + P + 1;  // (qb holds P + 1 + kBinKeys + P words, launch_bin_scan's contract)
    hipLaunchKernelGGL(k_bin_scan_key, dim3(kBinKeys + P), dim3(1024), 0, s, blk, nb, tot);
    KCHECK("k_bin_scan_key");
    hipLaunchKernelGGL(k_bin_scan_post, dim3(1), dim3(64), 0, s, tot, P, qb, mail, extra, nextra);
    KCHECK("k_bin_scan_post");
    return;
  }
  if (nb <= 4096 && P <= 4) {  // registers for (3 + P) keys × 4 tiles
#define OMX_BS(M) hipLaunchKernelGGL((k_bin_scan<M, 4>), dim3(1), dim3(1024), 0, s, blk, nb, P, qb, mail, extra, nextra)
    if (P <= 1) OMX_BS(1);
    else if (P <= 2) OMX_BS(2);
    else OMX_BS(4);
#undef OMX_BS
  } else {
#define OMX_BS(M) hipLaunchKernelGGL((k_bin_scan<M, 0>), dim3(1), dim3(1024), 0, s, blk, nb, P, qb, mail, extra, nextra)
    OMX_BY_MAXP(P, OMX_BS);
#undef OMX_BS
  }
  KCHECK("k_bin_scan");
}
void launch_bin_fill(bool sliced, const uint32_t *src, uint64_t R, const DAdj &adj, const DCuts &cuts,
                     uint64_t heavy_deg, uint32_t P, const uint64_t *blk, const uint64_t *qb, uint64_t *loffs,
                     uint64_t *lbase, const LightRows &lr, ChunkDesc *chunks, SliceChunk *schunks, hipStream_t s,
                     uint32_t chunk_shift) {
  const unsigned nb = bin_tiles(R);
  if (!sliced) {
    hipLaunchKernelGGL((k_bin_fill<false, 1>), dim3(nb), dim3(kBinBlock), 0, s, src, R, adj, cuts, heavy_deg, 1u, blk,
                       qb, loffs, lbase, lr, chunks, schunks, chunk_shift);
  } else {
#define OMX_BF(M) hipLaunchKernelGGL((k_bin_fill<true, M>), dim3(nb), dim3(kBinBlock), 0, s, src, R, adj, cuts, \
                                     heavy_deg, P, blk, qb, loffs, lbase, lr, chunks, schunks, 10u)
    OMX_BY_MAXP(P, OMX_BF);
#undef OMX_BF
  }
  KCHECK("k_bin_fill");
}

// out[q] = set bits of bitmap slice q (2^shift vertices): the slices' densities size the arenas of the
// sliced expansion kernels (Executor::expand_core)
__global__ __launch_bounds__(256) void k_slice_popc(const uint64_t *bm, uint64_t nwords, uint32_t shift,
                                                    unsigned long long *out) {
  const uint64_t wps = shift >= 6 ? (1ull << (shift - 6)) : 1;
  const uint64_t w0 = (uint64_t)blockIdx.x * wps, w1 = min(nwords, w0 + wps);
  unsigned long long c = 0;
  for (uint64_t w = w0 + threadIdx.x; w < w1; w += blockDim.x) c += __popcll(bm[w]);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
  __shared__ unsigned long long s_c[4];
  if ((threadIdx.x & 63) == 0) s_c[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = s_c[0] + s_c[1] + s_c[2] + s_c[3];
}
void launch_slice_popc(const uint64_t *bm, uint32_t V, uint32_t shift, uint32_t P, unsigned long long *out,
                       hipStream_t s) {
  if (!P) return;
  hipLaunchKernelGGL(k_slice_popc, dim3(P), dim3(256), 0, s, bm, ((uint64_t)V + 63) / 64, shift, out);
  KCHECK("k_slice_popc");
}

// Copy bitmap slice q (2^shift bits) into LDS: 16-byte loads, eight per thread in flight before the
// LDS stores (a plain loop waits for each load before its store: 32 serial round trips per thread)
__device__ __forceinline__ void stage_slice(uint32_t *s_bm, const uint32_t *bm, uint32_t V, uint32_t q, uint32_t shift) {
  const uint64_t nw = ((uint64_t)V + 63) / 64 * 2;  // u32 words of the bitmap (before the padding)
  const uint32_t sw = (1u << shift) / 32;
  const uint64_t w0 = (uint64_t)q * sw;
  if (sw % (4 * kSliceBlock) == 0) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *src = reinterpret_cast<const u32x4 *>(bm + w0);
    u32x4 *dst = reinterpret_cast<u32x4 *>(s_bm);
    const uint32_t n4 = sw / 4;
    for (uint32_t i0 = 0; i0 < n4; i0 += 8 * kSliceBlock) {
      u32x4 t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // no range check: filter bitmaps are padded (kBitmapPadWords)
        const uint32_t i = i0 + k * kSliceBlock + threadIdx.x;
        t[k] = src[i < n4 ? i : 0];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t i = i0 + k * kSliceBlock + threadIdx.x;
        if (i < n4) dst[i] = t[k];
      }
    }
  } else {  // small slices (tests)
    for (uint32_t i = threadIdx.x; i < sw; i += kSliceBlock) s_bm[i] = w0 + i < nw ? bm[w0 + i] : 0u;
  }
  __syncthreads();
}

// Workgroups [wg0[q], wg0[q+1]) own slice q (the host sizes each range by the slice's chunk count);
// wave j of those takes the slice's chunks j, j + NW_q, … (static: a device-wide work counter would
// be one hot address that every XCD's atomics serialise on). Each wave appends its survivors to a
// private arena, like k_expand_heavy.
// load through the constant address space: a wave-uniform address becomes an s_load (the data must
// not change during the kernel)
template <typename T>
__device__ __forceinline__ T sload(const T *p) {
  return *(const __attribute__((address_space(4))) T *)(p);
}

// chunk descriptor through scalar loads (wave-uniform address; chunks are read-only in the kernel).
// The compiler turns a plain load here into a vector load whose wait would also drain the
// in-flight col[] prefetch (vmcnt is in order), so the two s_loads are explicit.
__device__ __forceinline__ SliceChunk sload_chunk(const SliceChunk *p) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const SliceChunk *pu = (const SliceChunk *)wave_bcast64((uint64_t)p);
  u32x4 a;
  asm volatile(
      "s_load_dwordx4 %0, %1, 0x0\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(a)  // early-clobber: the load lands after the base is read
      : "s"(pu)
      : "memory");
  SliceChunk d;
  d.lo = ((uint64_t)a.y << 32) | a.x;
  d.row = a.z;
  d.n = (uint16_t)(a.w & 0xffffu);
  d.part = (uint16_t)(a.w >> 16);
  return d;
}

// NC = carried columns stored through per-wave buffer descriptors (0…4); NC = -1: any count, plain
// global stores (more than 4 bound aliases). Per chunk: the next chunk's descriptor, carried values
// and 16 col dwords are issued first, then the current chunk's 16 LDS probes, then one ballot and the
// stores per 64-edge slot.
template <bool WRITE, int NC>
__global__ __launch_bounds__(kSliceBlock) void k_expand_heavy_sliced(ExpandArgs a, SliceArgs sa) {
  constexpr int NS = kHeavySlots, WPB = kSliceBlock / 64, NCV = NC < 0 ? 4 : (NC > 0 ? NC : 1);
  __shared__ uint32_t s_bm[kSliceBits / 32];
  // per-wave staging of a chunk's surviving neighbours: flushed with full-wave coalesced stores (the
  // chunk's carried columns are constants), instead of one partial store per column and 64-edge slot
  __shared__ uint32_t s_stage[WPB * (kStage + 1)];  // +1: a masked-off lane's probe may stage one row past
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t gw = blockIdx.x * WPB + wave;
  uint32_t qs = 0;
  while (qs + 1 < sa.nslices && blockIdx.x >= sa.wg0[qs + 1]) ++qs;
  stage_slice(s_bm, reinterpret_cast<const uint32_t *>(a.filter), sa.V, qs, sa.shift);
  const uint64_t qend = sa.qb[qs + 1];
  const uint32_t nwq = (sa.wg0[qs + 1] - sa.wg0[qs]) * WPB;
  const uint64_t arena = a.arena_base + (uint64_t)gw * a.arena_cap;
  const int nc = NC < 0 ? a.ncarry : NC;
  // per-wave output descriptors (arena-relative byte offsets fit 32 bits: arena_cap·4 < 2 GiB)
  const int32_t arena_bytes = WRITE ? (int32_t)(a.arena_cap * 4 < 0x7fffffffull ? a.arena_cap * 4 : 0x7fffffffull) : 0;
  static_assert(kChunk * 4 <= 0x7fffffff, "in-range store offsets stay below the 0x80000000 drop marker");
  auto out_rsrc = [&](int k) {
    uint32_t *p = k < 0 ? a.out_dst : (k < nc ? a.carry_out[k] : a.out_dst);
    return __builtin_amdgcn_make_buffer_rsrc(p + arena, 0, arena_bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t od = out_rsrc(-1), oc0 = out_rsrc(0), oc1 = out_rsrc(1), oc2 = out_rsrc(2),
                               oc3 = out_rsrc(3);
  uint32_t acc = 0;
  // chunk descriptors and carried values are read through the constant address space (scalar loads:
  // they stay in SGPRs, so the col[] buffer descriptor needs no waterfall loop, and they wait on
  // lgkmcnt instead of queueing behind the in-flight col[] loads on vmcnt)
  struct Cur {
    uint64_t lo;
    uint32_t n, row, part;
    uint32_t cv[NCV];
    uint32_t q[NS];
  };
  // unconditional (a past-the-end chunk becomes an empty copy of the last one): a skipped load
  // would make the waitcnt pass assume the worst at the join and drain the prefetch
  auto load = [&](uint64_t c, Cur &x) {
    const bool live = c < qend;
    const SliceChunk d = sload_chunk(a.schunks + (live ? c : qend - 1));
    x.lo = d.lo;
    x.n = live ? (uint32_t)d.n : 0u;
    x.row = d.row;
    x.part = d.part;
    if (WRITE) {
#pragma unroll
      for (int k = 0; k < NCV; ++k) x.cv[k] = k < nc ? sload(a.carry_in[k] + x.row) : 0u;
    }
    // lanes past the chunk end read 0 through the descriptor's range check
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint32_t *>(a.adj.p[x.part].col + x.lo), 0, (int32_t)(x.n * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < NS; ++i) x.q[i] = __builtin_amdgcn_raw_buffer_load_b32(cr, (i * 64 + lane) * 4, 0, 0);
  };
  // per 64-edge slot: 2 VALU for the LDS word (a neighbour of the slice, so its low bits are the
  // offset), one bit-field extract, the ballot, a lane prefix, and exec-masked compacted stores
  const uint32_t wbits = sa.shift - 5;  // bitmap words per slice = 2^wbits
  uint32_t *const stage = s_stage + wave * (kStage + 1);
  auto cvk = [](const Cur &x, int k) { return k < NCV ? x.cv[k < NCV ? k : 0] : 0u; };
  // writes the `n` staged rows (neighbour from LDS, carried columns constant) at the arena's acc
  // an estimated arena may be short (Executor::expand_core): rows past arena_cap are counted, not
  // written (an explicit bound: the buffer range check does not cover the scalar offset)
  const uint64_t cap = a.arena_cap;
  auto flush = [&](const Cur &x, uint32_t n) {
    const int32_t so = (int32_t)(acc * 4);
    for (uint32_t k = 0; k < n; k += 64) {
      const uint32_t idx = k + lane;
      if (idx < n && acc + idx < cap) {
        const uint32_t off = idx * 4;
        __builtin_amdgcn_raw_buffer_store_b32(stage[idx], od, off, so, 0);
        if (nc > 0) __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 0), oc0, off, so, 0);
        if (nc > 1) __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 1), oc1, off, so, 0);
        if (nc > 2) __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 2), oc2, off, so, 0);
        if (nc > 3) __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 3), oc3, off, so, 0);
      }
    }
    acc += n;
  };
  auto process = [&](const Cur &x) {
    uint32_t w[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) w[i] = s_bm[__builtin_amdgcn_ubfe(x.q[i], 5, wbits)];
    // all 16 probes are in flight before the first is used (one LDS wait, not one per slot)
#pragma unroll
    for (int i = 0; i < NS; ++i) asm volatile("" : "+v"(w[i]));
    uint32_t st = 0;  // rows staged for this chunk
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if ((uint32_t)(i * 64) >= x.n) break;  // uniform: slice cuts leave chunks short (≈600 of 1024 edges)
      const uint32_t v = x.q[i];
      // v_bfe_u32 reads the low 5 bits of its offset operand. Lanes past the chunk end (last slot
      // only) are cut from the ballot on the scalar side (a set probe there stages one row past the
      // counted ones, never flushed).
      const bool bit = __builtin_amdgcn_ubfe(w[i], v, 1) != 0;
      uint64_t m = __builtin_amdgcn_ballot_w64(bit);
      const uint32_t rem = x.n - (uint32_t)(i * 64);
      if (rem < 64) m &= (1ull << rem) - 1;
      const uint32_t cnt = (uint32_t)__popcll(m);
      if (WRITE) {
        if (NC >= 0) {
          if (bit) stage[st + lane_prefix(m)] = v;
          st += cnt;
          if (st > kStage - 64) {  // uniform: room for one more slot
            flush(x, st);
            st = 0;
          }
        } else if (bit && acc + lane_prefix(m) < cap) {  // more than 4 carried columns: direct stores
          const uint32_t pre = lane_prefix(m);
          const uint32_t off = pre * 4;
          const int32_t so = (int32_t)(acc * 4);
          __builtin_amdgcn_raw_buffer_store_b32(v, od, off, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 0), oc0, off, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 1), oc1, off, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 2), oc2, off, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(cvk(x, 3), oc3, off, so, 0);
          for (int kk = 4; kk < nc; ++kk) a.carry_out[kk][arena + acc + pre] = a.carry_in[kk][x.row];
        }
      }
      if (!WRITE || NC < 0) acc += cnt;
    }
    if (WRITE && NC >= 0 && st) flush(x, st);
  };
  // three register sets in rotation, two chunks in flight while one is filtered (no copy of in-flight
  // load destinations: the waitcnt pass then only waits for the chunk it processes)
  const uint64_t c0 = sa.qb[qs] + (uint64_t)(blockIdx.x - sa.wg0[qs]) * WPB + wave;
  if (c0 < qend) {
    const uint64_t K = (qend - c0 + nwq - 1) / nwq;  // chunks of this wave
    Cur A, B, C;
    load(c0, A);
    load(c0 + nwq, B);
    for (uint64_t k = 0;; k += 3) {
      load(c0 + (k + 2) * nwq, C);
      process(A);
      if (k + 1 >= K) break;
      load(c0 + (k + 3) * nwq, A);
      process(B);
      if (k + 2 >= K) break;
      load(c0 + (k + 4) * nwq, B);
      process(C);
      if (k + 3 >= K) break;
    }
  }
  if (lane == 0) {
    a.seg_count[a.seg_base + gw] = acc;
    a.seg_start[a.seg_base + gw] = arena;
  }
}

void launch_expand_heavy_sliced(const ExpandArgs &a, const SliceArgs &sa, unsigned grid, bool write, hipStream_t s) {
  if (!grid) return;
  const dim3 g(grid), b(kSliceBlock);
  if (!write) {
    hipLaunchKernelGGL((k_expand_heavy_sliced<false, 0>), g, b, 0, s, a, sa);
  } else {
    switch (a.ncarry) {
      case 0: hipLaunchKernelGGL((k_expand_heavy_sliced<true, 0>), g, b, 0, s, a, sa); break;
      case 1: hipLaunchKernelGGL((k_expand_heavy_sliced<true, 1>), g, b, 0, s, a, sa); break;
      case 2: hipLaunchKernelGGL((k_expand_heavy_sliced<true, 2>), g, b, 0, s, a, sa); break;
      case 3: hipLaunchKernelGGL((k_expand_heavy_sliced<true, 3>), g, b, 0, s, a, sa); break;
      case 4: hipLaunchKernelGGL((k_expand_heavy_sliced<true, 4>), g, b, 0, s, a, sa); break;
      default: hipLaunchKernelGGL((k_expand_heavy_sliced<true, -1>), g, b, 0, s, a, sa); break;
    }
  }
  KCHECK("k_expand_heavy_sliced");
}

// ---- LDS-sliced light rows ---------------------------------------------------------------------------
// The merge-path kernel probes the target bitmap through L2: one L1→L2 request per edge (a light row's
// few sorted neighbours spread over all of V), and that request rate bounds it. Here, as for the heavy
// rows, workgroups [wg0[q], wg0[q+1]) hold slice q of the bitmap in LDS. The light rows come compacted
// by k_bin_fill (offsets, first col index, row, slice cuts: coalesced, no dependent loads). Wave j of
// slice q owns the 64-light-row groups whose first edge offset lies in [EL·j/W_q, EL·(j+1)/W_q) (a
// 64-ary search over the offsets) and per group packs the 64 rows' slice-q pieces into 64-edge slots:
// each lane finds the row owning its edge with a 6-step search over the wave's piece offsets
// (cross-lane reads), loads the neighbour and probes LDS. U slots are in flight per step and the next
// group's row data (with the carried values, compacted by k_bin_fill for ≤ 4 columns, so a survivor's
// columns come from a cross-lane read, not a gather) is loaded while the current one is filtered. Survivors go to the wave's arena (cap
// ⌈EL/W_q⌉ + 64·heavy_deg rows), compacted by ballot.
// Round 3: a slot's owners come from a per-wave byte table instead of a 6-step cross-lane search per
// slot: per round of 64·U entries the pieces mark their first entry (the round's first entry's owner from
// one search), a max-scan spreads the marks, and each entry reads its owner's lane as one LDS byte
// (the search cost 40 of the ≈ 67 VALU operations per entry, PMC profiles/r03/pmc_light).
constexpr int kLightStage = 256;  // staged survivors per wave (16 waves × 1.25 KiB beside the slice)
template <bool WRITE, int U, int NC>
__global__ __launch_bounds__(kSliceBlock) void k_expand_light_sliced(ExpandArgs a, SliceArgs sa) {
  constexpr int NCV = NC > 0 ? NC : 1;
  constexpr int WPB = kSliceBlock / 64;
  constexpr int RB = U;  // mark bytes per lane and round
  static_assert(RB % 4 == 0, "a lane's marks are whole words");
  __shared__ uint32_t s_bm[kSliceBits / 32];
  __shared__ uint32_t s_stv[WRITE ? WPB * kLightStage : 1];
  __shared__ uint8_t s_stj[WRITE ? WPB * kLightStage : 1];
  __shared__ uint32_t s_mk[WPB * 64 * U / 4];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t gw = blockIdx.x * WPB + wave;
  uint32_t qs = 0;
  while (qs + 1 < sa.nslices && blockIdx.x >= sa.wg0[qs + 1]) ++qs;
  stage_slice(s_bm, reinterpret_cast<const uint32_t *>(a.filter), sa.V, qs, sa.shift);
  const uint32_t P = sa.nslices, wbits = sa.shift - 5;
  const uint64_t NL = sa.nl, EL = a.E, G = (NL + 63) / 64;
  const uint32_t nwq = (sa.wg0[qs + 1] - sa.wg0[qs]) * WPB;
  const uint32_t wq = (blockIdx.x - sa.wg0[qs]) * WPB + wave;
  const uint64_t *offs = a.offs;
  // first group g ∈ [0, G] whose first edge offset is ≥ target (offs[min(64g, NL)]; g = G → EL)
  auto group_lb = [&](uint64_t target) -> uint64_t {
    uint64_t lo = 0, hi = G;
    while (lo < hi) {
      const uint64_t step = (hi - lo + 63) / 64;
      const uint64_t p = lo + (uint64_t)lane * step;
      const bool f = p >= hi || offs[p * 64 < NL ? p * 64 : NL] >= target;
      const uint64_t m = __builtin_amdgcn_ballot_w64(f);
      if (m == 0) {
        lo += 63 * step + 1;
      } else {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        if (l == 0) break;  // lo itself
        hi = lo + (uint64_t)l * step;
        lo += (uint64_t)(l - 1) * step + 1;
      }
    }
    return lo;
  };
  const uint64_t g0 = group_lb(EL * wq / nwq);
  const uint64_t g1 = wq + 1 == nwq ? G : group_lb(EL * (wq + 1) / nwq);
  const uint64_t arena = a.arena_base + (uint64_t)gw * a.arena_cap;
  const uint32_t *col = a.adj.p[0].col;
  const uint32_t *clo_p = qs > 0 ? sa.lcuts + (uint64_t)(qs - 1) * NL : nullptr;
  const uint32_t *chi_p = qs + 1 < P ? sa.lcuts + (uint64_t)qs * NL : nullptr;
  const int nc = a.ncarry;
  // row data of one group (loads unconditional, index clamped: a skipped load would make the waitcnt
  // pass drain the prefetch at the join)
  struct Grp {
    uint64_t o0, o1, lb;
    uint32_t clo, chi, row;
    uint32_t cv[NCV];
  };
  auto gload = [&](uint64_t g, Grp &m) {
    const uint64_t i = g * 64 + lane;
    const uint64_t ii = i < NL ? i : NL - 1;
    m.o0 = offs[ii];
    m.o1 = i < NL ? offs[ii + 1] : m.o0;  // a lane past NL gets an empty piece
    m.lb = a.lbase[ii];
    m.clo = clo_p ? clo_p[ii] : 0u;
    m.chi = chi_p ? chi_p[ii] : 0xffffffffu;
    m.row = WRITE && NC < 0 ? sa.lrow[ii] : 0u;
#pragma unroll
    for (int c = 0; c < NCV; ++c) m.cv[c] = WRITE && c < NC ? sa.lcarry[c][ii] : 0u;
  };
  uint64_t acc = 0;
  // per-wave LDS staging of the group's survivors (neighbour, owning lane), written out with
  // full-wave coalesced stores once per group: no stores between the col[] loads of a group's steps
  // (gfx9 counts stores on vmcnt, so each partial store would hold up the next step's load wait)
  uint32_t *const stv = s_stv + wave * kLightStage;
  uint8_t *const stj = s_stj + wave * kLightStage;
  uint32_t st = 0;
  auto flush = [&](const Grp &m) {
    for (uint32_t k = 0; k < st; k += 64) {
      const uint32_t idx = k + lane;
      const uint32_t j = idx < st ? stj[idx] : 0u;
      const uint32_t v = idx < st ? stv[idx] : 0u;
      uint32_t cv[NCV];
#pragma unroll
      for (int c = 0; c < NCV; ++c) cv[c] = c < NC ? (uint32_t)__shfl(m.cv[c], (int)j, 64) : 0u;
      const uint32_t rr = NC < 0 ? (uint32_t)__shfl(m.row, (int)j, 64) : 0u;
      if (idx < st && acc + idx < a.arena_cap) {  // an estimated arena may be short: counted, not written
        const uint64_t o = arena + acc + idx;
        a.out_dst[o] = v;
        if (NC < 0) {
          for (int c = 0; c < nc; ++c) a.carry_out[c][o] = a.carry_in[c][rr];
        } else {
#pragma unroll
          for (int c = 0; c < NCV; ++c)
            if (c < NC) a.carry_out[c][o] = cv[c];
        }
      }
    }
    acc += st;
    st = 0;
  };
  auto process = [&](uint64_t g, const Grp &m) {
    const uint32_t dl = (uint32_t)(m.o1 - m.o0);
    const uint32_t clo = dl ? m.clo : 0u, chi = dl ? (m.chi < dl ? m.chi : dl) : 0u;
    const uint32_t len = chi - clo;
    const uint64_t start = m.lb + clo;
    uint32_t incl = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(incl, off, 64);
      if (lane >= (uint32_t)off) incl += y;
    }
    const uint32_t pre = incl - len;
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    uint32_t *const mkt = s_mk + wave * (64 * U / 4);
    uint8_t *const mb = reinterpret_cast<uint8_t *>(mkt);
    for (uint32_t base = 0; base < T; base += 64 * U) {
      // owner of entry base: the last lane j with pre_j ≤ base (zero-length pieces share their
      // successor's offset); the pieces starting inside the round mark their first entry
      uint32_t j0 = 0;
#pragma unroll
      for (int st = 32; st > 0; st >>= 1)
        if ((uint32_t)__shfl(pre, (int)(j0 + st), 64) <= base) j0 += st;
#pragma unroll
      for (int i = 0; i < RB / 4; ++i) mkt[lane * (RB / 4) + i] = 0;
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) mb[0] = (uint8_t)j0;
      if (len && pre > base && pre < base + 64 * U) mb[pre - base] = (uint8_t)lane;
      __builtin_amdgcn_wave_barrier();
      {  // max-scan of the marks: lane l holds bytes RB·l … RB·l + RB − 1
        uint32_t wd[RB / 4];
        uint32_t mx = 0;
#pragma unroll
        for (int i = 0; i < RB / 4; ++i) {
          wd[i] = mkt[lane * (RB / 4) + i];
#pragma unroll
          for (int b = 0; b < 4; ++b) mx = max(mx, (wd[i] >> (8 * b)) & 0xFFu);
        }
        uint32_t sc = mx;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const uint32_t y = __shfl_up(sc, off, 64);
          if (lane >= (uint32_t)off) sc = max(sc, y);
        }
        uint32_t run = __shfl_up(sc, 1, 64);
        if (lane == 0) run = 0;
#pragma unroll
        for (int i = 0; i < RB / 4; ++i) {
          uint32_t o = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            run = max(run, (wd[i] >> (8 * b)) & 0xFFu);
            o |= run << (8 * b);
          }
          mkt[lane * (RB / 4) + i] = o;
        }
      }
      __builtin_amdgcn_wave_barrier();
      uint32_t nb[U], jj[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = base + u * 64 + lane;
        const uint32_t j = mb[u * 64 + lane];
        const uint64_t sj = ((uint64_t)(uint32_t)__shfl((uint32_t)(start >> 32), (int)j, 64) << 32) |
                            (uint32_t)__shfl((uint32_t)start, (int)j, 64);
        const uint32_t pj = (uint32_t)__shfl(pre, (int)j, 64);
        jj[u] = j;
        // unconditional load (lanes past T read the piece start and are masked below)
        nb[u] = col[e < T ? sj + (e - pj) : sj];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t e = base + u * 64 + lane;
        const uint32_t v = nb[u];
        const bool bit = e < T && ((s_bm[__builtin_amdgcn_ubfe(v, 5, wbits)] >> (v & 31)) & 1u);
        const uint64_t mk = __builtin_amdgcn_ballot_w64(bit);
        if (WRITE) {
          if (bit) {
            const uint32_t o = st + lane_prefix(mk);
            stv[o] = v;
            stj[o] = (uint8_t)jj[u];
          }
          st += (uint32_t)__popcll(mk);
          if (st > kLightStage - 64) flush(m);  // uniform: room for one more slot
        } else {
          acc += (uint64_t)__popcll(mk);
        }
      }
      __builtin_amdgcn_wave_barrier();  // the round's marks are rewritten by the next round
    }
    if (WRITE && st) flush(m);
  };
  if (g0 < g1) {
    Grp A, B;
    gload(g0, A);
    for (uint64_t g = g0;; g += 2) {
      gload(g + 1 < g1 ? g + 1 : g, B);
      process(g, A);
      if (g + 1 >= g1) break;
      gload(g + 2 < g1 ? g + 2 : g + 1, A);
      process(g + 1, B);
      if (g + 2 >= g1) break;
    }
  }
  if (lane == 0) {
    a.seg_count[a.seg_base + gw] = (uint32_t)acc;
    a.seg_start[a.seg_base + gw] = arena;
  }
}

void launch_expand_light_sliced(const ExpandArgs &a, const SliceArgs &sa, unsigned grid, bool write, hipStream_t s) {
  if (!grid) return;
  const dim3 g(grid), b(kSliceBlock);
  if (!write) {
    hipLaunchKernelGGL((k_expand_light_sliced<false, 8, 0>), g, b, 0, s, a, sa);
  } else {
    switch (a.ncarry) {
      case 0: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, 0>), g, b, 0, s, a, sa); break;
      case 1: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, 1>), g, b, 0, s, a, sa); break;
      case 2: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, 2>), g, b, 0, s, a, sa); break;
      case 3: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, 3>), g, b, 0, s, a, sa); break;
      case 4: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, 4>), g, b, 0, s, a, sa); break;
      default: hipLaunchKernelGGL((k_expand_light_sliced<true, 8, -1>), g, b, 0, s, a, sa); break;
    }
  }
  KCHECK("k_expand_light_sliced");
}

void launch_expand(const ExpandArgs &a, unsigned grid, bool write, hipStream_t s) {
  if (!grid) return;
  const bool single = a.adj.n == 1, member = a.member_src != nullptr, filter = a.filter != nullptr || member;
  dim3 g(grid), b(kExpandBlock);
  // (unfiltered rows: a wave-per-output-window kernel without the LDS row bookkeeping measured 1.6×
  // slower than these merge-path tiles, profiles/r02/dense)
#define OMX_EXP(S, F, Wr, M) hipLaunchKernelGGL((k_expand<S, F, Wr, M>), g, b, 0, s, a)
#define OMX_EXP_W(S, F, M) { if (write) OMX_EXP(S, F, true, M); else OMX_EXP(S, F, false, M); }
  if (single) {
    if (member) OMX_EXP_W(true, true, true)
    else if (filter) OMX_EXP_W(true, true, false)
    else OMX_EXP_W(true, false, false)
  } else {
    if (member) OMX_EXP_W(false, true, true)
    else if (filter) OMX_EXP_W(false, true, false)
    else OMX_EXP_W(false, false, false)
  }
#undef OMX_EXP_W
#undef OMX_EXP
  KCHECK("k_expand");
}

void launch_expand_heavy(const ExpandArgs &a, unsigned grid, bool write, hipStream_t s) {
  if (!grid) return;
  const bool member = a.member_src != nullptr, filter = a.filter != nullptr || member;
  dim3 g(grid), b(kHeavyBlock);
  // smaller chunk windows only for unfiltered writes (the dense emission of medium rows)
  if ((filter || !write) && a.chunk_shift != 10) fail(OMX_E_INVALID, "internal: heavy chunks below 1024 only for dense writes");
#define OMX_EXH(F, Wr, M) hipLaunchKernelGGL((k_expand_heavy<F, Wr, M>), g, b, 0, s, a)
  if (member) { if (write) OMX_EXH(true, true, true); else OMX_EXH(true, false, true); }
  else if (filter) { if (write) OMX_EXH(true, true, false); else OMX_EXH(true, false, false); }
  else if (!write) OMX_EXH(false, false, false);
  else if (a.chunk_shift == 8) hipLaunchKernelGGL((k_expand_heavy<false, true, false, 4>), g, b, 0, s, a);
  else if (a.chunk_shift == 9) hipLaunchKernelGGL((k_expand_heavy<false, true, false, 8>), g, b, 0, s, a);
  else if (a.chunk_shift == 10) OMX_EXH(false, true, false);
  else if (a.chunk_shift == 11) hipLaunchKernelGGL((k_expand_heavy<false, true, false, 32>), g, b, 0, s, a);
  else fail(OMX_E_INVALID, "internal: heavy chunk windows of 256, 512, 1024 or 2048 entries");
#undef OMX_EXH
  KCHECK("k_expand_heavy");
}

int expand_blocks_per_cu(bool heavy, bool single, bool filter, bool write, bool member, uint32_t chunk_shift) {
  // the occupancy query costs a host round trip into the runtime: answer each variant once
  static int cache[128];
  static std::mutex cache_m;
  filter = filter || member;
  const int cs = heavy && !filter && write ? (int)(chunk_shift - 8) & 3 : 2;  // 0..3: 256..2048 entries
  const int key = (int)heavy | (int)single << 1 | (int)filter << 2 | (int)write << 3 | (int)member << 4 | cs << 5;
  {
    std::lock_guard<std::mutex> lk(cache_m);
    if (cache[key]) return cache[key];
  }
  int n = 0;
  hipError_t e;
#define OCC(K, BS) hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, K, BS, 0)
  if (heavy) {
    if (member) e = write ? OCC((k_expand_heavy<true, true, true>), kHeavyBlock) : OCC((k_expand_heavy<true, false, true>), kHeavyBlock);
    else if (filter) e = write ? OCC((k_expand_heavy<true, true, false>), kHeavyBlock) : OCC((k_expand_heavy<true, false, false>), kHeavyBlock);
    else if (!write) e = OCC((k_expand_heavy<false, false, false>), kHeavyBlock);
    else if (cs == 0) e = OCC((k_expand_heavy<false, true, false, 4>), kHeavyBlock);
    else if (cs == 1) e = OCC((k_expand_heavy<false, true, false, 8>), kHeavyBlock);
    else if (cs == 3) e = OCC((k_expand_heavy<false, true, false, 32>), kHeavyBlock);
    else e = OCC((k_expand_heavy<false, true, false>), kHeavyBlock);
  } else if (single) {
    e = member ? OCC((k_expand<true, true, true, true>), kExpandBlock)
               : filter ? OCC((k_expand<true, true, true, false>), kExpandBlock) : OCC((k_expand<true, false, true, false>), kExpandBlock);
  } else {
    e = member ? OCC((k_expand<false, true, true, true>), kExpandBlock)
               : filter ? OCC((k_expand<false, true, true, false>), kExpandBlock) : OCC((k_expand<false, false, true, false>), kExpandBlock);
  }
#undef OCC
  if (e != hipSuccess || n < 1) n = 2;
  std::lock_guard<std::mutex> lk(cache_m);
  cache[key] = n;
  return n;
}

struct ColPtrs {
  const uint32_t *in[kMaxCols];
  uint32_t *out[kMaxCols];
};

__global__ void k_compact_segments(int ncols, ColPtrs cp, const uint64_t *seg_start, const uint32_t *seg_count,
                                   const uint64_t *seg_offs) {
  const uint32_t b = blockIdx.x;
  const uint32_t cnt = seg_count[b];
  const uint64_t src = seg_start[b], dst = seg_offs[b];
  for (int c = 0; c < ncols; ++c)
    for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) cp.out[c][dst + i] = cp.in[c][src + i];
}
void launch_compact_segments(int ncols, uint32_t *const *in, uint32_t *const *out, const uint64_t *seg_start,
                             const uint32_t *seg_count, const uint64_t *seg_offs, uint32_t nseg, hipStream_t s) {
  if (!nseg) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) {
    cp.in[c] = in[c];
    cp.out[c] = out[c];
  }
  hipLaunchKernelGGL(k_compact_segments, dim3(nseg), dim3(256), 0, s, ncols, cp, seg_start, seg_count, seg_offs);
  KCHECK("k_compact_segments");
}

// ---- optional targets (P/OMatchStatement.java:448-458) ------------------------------------------------
// flags[r] = 1 iff no neighbour of src[r] passes `filter` (the traversal returned nothing)
__global__ void k_flag_no_neighbor(const uint32_t *src, uint64_t R, DAdj adj, const uint64_t *filter, uint8_t *flags) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint32_t v = src[r];
  bool any = false;
  for (int p = 0; p < adj.n && !any; ++p)
    for (uint64_t e = adj.p[p].rp[v], h = adj.p[p].rp[v + 1]; e < h && !any; ++e)
      any = !filter || bm_test(filter, adj.p[p].col[e]);
  flags[r] = any ? 0 : 1;
}
void launch_flag_no_neighbor(const uint32_t *src, uint64_t R, const DAdj &adj, const uint64_t *filter, uint8_t *flags,
                             hipStream_t s) {
  if (!R) return;
  hipLaunchKernelGGL(k_flag_no_neighbor, dim3(nblocks(R, 256)), dim3(256), 0, s, src, R, adj, filter, flags);
  KCHECK("k_flag_no_neighbor");
}
// A bound optional target t of row r: t ∉ traversal(src[r]) → t := null (V). A null t with a non-empty
// traversal is the reference's NullPointerException (matched.get(t).getIdentity(), :468): *npe = 1.
__global__ void k_check_optional(const uint32_t *src, uint32_t *dst, uint64_t R, DAdj adj, const uint64_t *filter,
                                 uint32_t V, unsigned int *npe) {
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint32_t v = src[r], t = dst[r];
  bool found = false, any = false;
  for (int p = 0; p < adj.n; ++p)
    for (uint64_t e = adj.p[p].rp[v], h = adj.p[p].rp[v + 1]; e < h; ++e) {
      const uint32_t x = adj.p[p].col[e];
      if (filter && !bm_test(filter, x)) continue;
      any = true;
      found = found || x == t;
    }
  if (t >= V) {
    if (any) atomicOr(npe, 1u);
  } else if (!found) {
    dst[r] = V;
  }
}
void launch_check_optional(const uint32_t *src, uint32_t *dst, uint64_t R, const DAdj &adj, const uint64_t *filter,
                           uint32_t V, unsigned int *npe, hipStream_t s) {
  if (!R) return;
  hipLaunchKernelGGL(k_check_optional, dim3(nblocks(R, 256)), dim3(256), 0, s, src, dst, R, adj, filter, V, npe);
  KCHECK("k_check_optional");
}

// ---- bound-target check (existence of dst[r] in N(src[r]); P/OMatchStatement.java:468-477) ----------

__global__ void k_check(const uint32_t *src, const uint32_t *dst, uint64_t R, DAdj adj, const uint64_t *filter,
                        uint8_t *flags) {
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const uint32_t v = src[r], t = dst[r];
  bool found = false;
  if (!filter || bm_test(filter, t)) {
    for (int p = 0; p < adj.n && !found; ++p) {
      uint64_t lo = adj.p[p].rp[v], hi = adj.p[p].rp[v + 1];
      const uint32_t *col = adj.p[p].col;
      if (adj.sorted) {
        while (lo < hi) {
          uint64_t mid = (lo + hi) >> 1;
          uint32_t x = col[mid];
          if (x < t) lo = mid + 1;
          else hi = mid;
        }
        found = lo < adj.p[p].rp[v + 1] && col[lo] == t;
      } else {
        for (uint64_t e = lo; e < hi && !found; ++e) found = col[e] == t;
      }
    }
  }
  flags[r] = found;
}
void launch_check(const uint32_t *src, const uint32_t *dst, uint64_t R, const DAdj &adj, const uint64_t *filter,
                  uint8_t *flags, hipStream_t s) {
  if (!R) return;
  hipLaunchKernelGGL(k_check, dim3(nblocks(R, 256)), dim3(256), 0, s, src, dst, R, adj, filter, flags);
  KCHECK("k_check");
}

// ---- partitioned execution: destination rank of every binding row (dist.h) -----------------------
__device__ __forceinline__ void route_count(uint32_t d, bool live, uint32_t W, unsigned long long *s_h,
                                            unsigned long long *hist) {
  if (live) atomicAdd(&s_h[d], 1ull);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x)
    if (s_h[i]) atomicAdd(&hist[i], s_h[i]);
}

// owner of the row's vertex under the block partition: min(v / block, W − 1)
__global__ void k_route_owner(const uint32_t *v, uint64_t R, uint32_t block, uint32_t W, uint32_t *dest,
                              unsigned long long *hist) {
  __shared__ unsigned long long s_h[kMaxRanks];
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) s_h[i] = 0;
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0;
  if (r < R) {
    d = min(v[r] / block, W - 1);
    dest[r] = d;
  }
  route_count(d, r < R, W, s_h, hist);
}
void launch_route_owner(const uint32_t *v, uint64_t R, uint32_t block, uint32_t W, uint32_t *dest, uint64_t *hist,
                        hipStream_t s) {
  if (!R) return;
  hipLaunchKernelGGL(k_route_owner, dim3(nblocks(R, 256)), dim3(256), 0, s, v, R, block, W, dest,
                     reinterpret_cast<unsigned long long *>(hist));
  KCHECK("k_route_owner");
}

// a row id's origin: the rank p with bounds[p] <= id < bounds[p+1] (global row ids of a pair set)
struct RankBounds {
  uint64_t b[kMaxRanks + 1];
};
__global__ void k_route_bounds(const uint32_t *id, uint64_t R, RankBounds rb, uint32_t W, uint32_t *dest,
                               unsigned long long *hist) {
  __shared__ unsigned long long s_h[kMaxRanks];
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) s_h[i] = 0;
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0;
  if (r < R) {
    const uint64_t x = id[r];
    while (d + 1 < W && rb.b[d + 1] <= x) ++d;
    dest[r] = d;
  }
  route_count(d, r < R, W, s_h, hist);
}
void launch_route_bounds(const uint32_t *id, uint64_t R, const uint64_t *bounds, uint32_t W, uint32_t *dest,
                         uint64_t *hist, hipStream_t s) {
  if (!R) return;
  RankBounds rb{};
  for (uint32_t i = 0; i <= W; ++i) rb.b[i] = bounds[i];
  hipLaunchKernelGGL(k_route_bounds, dim3(nblocks(R, 256)), dim3(256), 0, s, id, R, rb, W, dest,
                     reinterpret_cast<unsigned long long *>(hist));
  KCHECK("k_route_bounds");
}
__global__ void k_add_u32(uint32_t *x, uint64_t n, int64_t delta) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = (uint32_t)((int64_t)x[i] + delta);
}
void launch_add_u32(uint32_t *x, uint64_t n, int64_t delta, hipStream_t s) {
  if (!n || !delta) return;
  hipLaunchKernelGGL(k_add_u32, dim3(nblocks(n, 256)), dim3(256), 0, s, x, n, delta);
  KCHECK("k_add_u32");
}

// a hash of the projected tuple: equal rows meet on one rank for the distinct pass
__global__ void k_route_hash(int ncols, ColPtrs cp, uint64_t R, uint32_t W, uint32_t *dest, unsigned long long *hist) {
  __shared__ unsigned long long s_h[kMaxRanks];
  for (uint32_t i = threadIdx.x; i < W; i += blockDim.x) s_h[i] = 0;
  __syncthreads();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t d = 0;
  if (r < R) {
    uint64_t h = 0x243F6A8885A308D3ull;
    for (int c = 0; c < ncols; ++c) {
      h = (h ^ cp.in[c][r]) * 0x9E3779B97F4A7C15ull;
      h ^= h >> 29;
    }
    d = (uint32_t)((h >> 32) % W);
    dest[r] = d;
  }
  route_count(d, r < R, W, s_h, hist);
}
void launch_route_hash(int ncols, const uint32_t *const *cols, uint64_t R, uint32_t W, uint32_t *dest, uint64_t *hist,
                       hipStream_t s) {
  if (!R) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) cp.in[c] = cols[c];
  hipLaunchKernelGGL(k_route_hash, dim3(nblocks(R, 256)), dim3(256), 0, s, ncols, cp, R, W, dest,
                     reinterpret_cast<unsigned long long *>(hist));
  KCHECK("k_route_hash");
}

// ---- one-workgroup scans (few elements; saves the launches of a device-wide scan) ----------------

// the vertices of a bitmap (range/shard restricted) in order, and their count, in two launches:
// per-block popcounts, then every block adds the counts of the blocks before it (≤ a few hundred
// words, read in parallel) to its own scan and scatters; the last block writes the total
constexpr int kListB = 256;
__global__ __launch_bounds__(kListB) void k_list_counts(const uint64_t *words, uint64_t n, uint32_t V, int rank,
                                                        int world, uint32_t lo, uint32_t hi, uint32_t *blk) {
  __shared__ uint32_t s_w[kListB / 64];
  const uint64_t i = (uint64_t)blockIdx.x * kListB + threadIdx.x;
  const uint32_t c = i < n ? __popcll(shard_word(words[i], i, V, rank, world, lo, hi)) : 0;
  uint32_t tot;
  block_excl_scan<kListB>(c, s_w, &tot);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kListB) void k_list_scatter(const uint64_t *words, uint64_t n, uint32_t V, int rank,
                                                         int world, uint32_t lo, uint32_t hi, const uint32_t *blk,
                                                         uint32_t *out, Mail mail, const uint64_t *extra, int nextra) {
  __shared__ uint32_t s_w[kListB / 64];
  __shared__ unsigned long long s_pre[kListB / 64];
  // prefix of the blocks before this one
  unsigned long long p = 0;
  for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kListB) p += blk[b];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) p += __shfl_xor(p, off, 64);
  if ((threadIdx.x & 63) == 0) s_pre[threadIdx.x >> 6] = p;
  __syncthreads();
  unsigned long long pre = 0;
#pragma unroll
  for (int w = 0; w < kListB / 64; ++w) pre += s_pre[w];
  const uint64_t i = (uint64_t)blockIdx.x * kListB + threadIdx.x;
  uint64_t w = i < n ? shard_word(words[i], i, V, rank, world, lo, hi) : 0;
  uint32_t tot;
  uint64_t o = pre + block_excl_scan<kListB>((uint32_t)__popcll(w), s_w, &tot);
  while (w) {
    out[o++] = (uint32_t)(i * 64 + __builtin_ctzll(w));
    w &= w - 1;
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the host only needs the count (and extra's words)
    mail.p[0] = pre + tot;
    for (int j = 0; j < nextra; ++j) mail.p[1 + j] = extra[j];
    mail_post(mail);
  }
}
void launch_bitmap_list_2k(const uint64_t *words, uint64_t n, uint32_t V, int rank, int world, uint32_t lo,
                           uint32_t hi, uint32_t *blk, uint32_t *out, const Mail &mail, hipStream_t s) {
  const unsigned g = nblocks(n, kListB);
  hipLaunchKernelGGL(k_list_counts, dim3(g), dim3(kListB), 0, s, words, n, V, rank, world, lo, hi, blk);
  KCHECK("k_list_counts");
  hipLaunchKernelGGL(k_list_scatter, dim3(g), dim3(kListB), 0, s, words, n, V, rank, world, lo, hi, blk, out, mail,
                     (const uint64_t *)nullptr, 0);
  KCHECK("k_list_scatter");
}
unsigned bitmap_list_blocks(uint64_t nwords) { return nblocks(nwords, kListB); }

// ---- configs[0] in four launches (round 5) ----------------------------------------------------------
// MATCH {class:Person}-Knows->{}-Knows->{as:fof} RETURN fof on a small graph (V ≤ kFof2Bits): the roots'
// hop, the marked last hop (Executor::expand_mark's factorized branch: each distinct middle vertex's
// adjacency read once) and the list of the marked set, queued back to back with one host round trip —
// the general path's 15-odd launches and four round trips cost more than the work at RMAT-16.
//   k_fof2_a: every edge (v, b) of hop 1 with v a root: b marked (LDS bitmap, flushed to ubm once per
//             workgroup); E1 += 1; E_t += deg2(b)
//   k_fof2_b: every edge (b, c) of hop 2 with b in ubm (staged in LDS): c marked (likewise, into bm);
//             EU += 1
//   then bm's ascending list (k_list_counts / k_list_scatter), whose last workgroup posts {m, E1, E_t,
//   EU}. (A single cooperative launch with grid barriers measured 0.57 ms: the in-kernel cross-XCD
//   bitmap traffic at agent scope costs more than the launches it saves.)
// every edge of one part, a wave per contiguous range of 64-edge groups (balanced over edges, not
// vertices): f(ok, v, x) for the lane's edge (v → x)
template <class F>
__device__ __forceinline__ void fof2_edges(const DAdjPart &p, uint32_t V, F &&f) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const uint64_t E = p.rp[V];
  const uint64_t chunk = ((E + nw - 1) / nw + 63) & ~63ull;
  const uint64_t e0 = w * chunk, e1 = min(E, e0 + chunk);
  if (e0 >= e1) return;
  uint32_t lo = 0, hi = V;  // the source of e0: the last v with rp[v] ≤ e0 (rp[V] = E > e0)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (p.rp[mid] <= e0) lo = mid;
    else hi = mid;
  }
  uint32_t v0 = lo;
  for (uint64_t g = e0; g < e1; g += 64) {
    const uint64_t e = g + lane;
    const bool ok = e < e1;
    uint32_t v = v0;
    if (ok) {  // galloping from the group's first source
      uint32_t a = v0, b = v0 + 1, step = 1;
      while (b < V && p.rp[b] <= e) {
        a = b;
        step <<= 1;
        b = a + step;
      }
      if (b > V) b = V;
      while (b - a > 1) {
        const uint32_t mid = (a + b) >> 1;
        if (p.rp[mid] <= e) a = mid;
        else b = mid;
      }
      v = a;
    }
    f(ok, v, ok ? p.col[e] : 0u);
    v0 = __builtin_amdgcn_readlane(v, 63);
  }
}
__device__ __forceinline__ void fof2_add(unsigned long long *acc, uint64_t x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  if ((threadIdx.x & 63) == 0 && x) atomicAdd(acc, (unsigned long long)x);
}
// a workgroup's LDS marks into the global set (only words with a new bit)
__device__ __forceinline__ void fof2_flush(const unsigned long long *s_bm, uint64_t *bm, uint64_t W) {
  __syncthreads();
  for (uint64_t w = threadIdx.x; w < W; w += blockDim.x) {
    const unsigned long long m = s_bm[w];
    if (m && (__hip_atomic_load(&bm[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & m) != m)
      atomicOr((unsigned long long *)&bm[w], m);
  }
}
__global__ __launch_bounds__(1024) void k_fof2_a(Fof2Args a) {
  extern __shared__ unsigned long long s_fof[];
  for (uint64_t w = threadIdx.x; w < a.W; w += blockDim.x) s_fof[w] = 0;
  __syncthreads();
  uint64_t e1 = 0, et = 0;
  for (int q = 0; q < a.a1.n; ++q)
    fof2_edges(a.a1.p[q], a.V, [&](bool ok, uint32_t v, uint32_t b) {
      if (ok && ((a.roots[v >> 6] >> (v & 63)) & 1ull) && (a.world <= 1 || v % (uint32_t)a.world == (uint32_t)a.rank)) {
        e1 += 1;
        et += adj_degree(a.a2, b);
        atomicOr(&s_fof[b >> 6], 1ull << (b & 63));
      }
    });
  unsigned long long *acc = reinterpret_cast<unsigned long long *>(a.acc);
  fof2_add(acc + 0, e1);
  fof2_add(acc + 1, et);
  fof2_flush(s_fof, a.ubm, a.W);
}
__global__ __launch_bounds__(1024) void k_fof2_b(Fof2Args a) {
  extern __shared__ unsigned long long s_fof[];
  unsigned long long *s_ub = s_fof, *s_bm = s_fof + a.W;
  for (uint64_t w = threadIdx.x; w < a.W; w += blockDim.x) {
    s_ub[w] = a.ubm[w];
    s_bm[w] = 0;
  }
  __syncthreads();
  uint64_t eu = 0;
  for (int q = 0; q < a.a2.n; ++q)
    fof2_edges(a.a2.p[q], a.V, [&](bool ok, uint32_t b, uint32_t c) {
      if (ok && ((s_ub[b >> 6] >> (b & 63)) & 1ull)) {
        eu += 1;
        atomicOr(&s_bm[c >> 6], 1ull << (c & 63));
      }
    });
  fof2_add(reinterpret_cast<unsigned long long *>(a.acc) + 2, eu);
  fof2_flush(s_bm, a.bm, a.W);
}

void launch_fof2(const Fof2Args &a, int phase, unsigned grid, uint32_t *blk, uint32_t *out, const Mail *mail,
                 hipStream_t s) {
  if (a.V > kFof2Bits || a.W != (a.V + 63) / 64) fail(OMX_E_INVALID, "internal: k_fof2 over a set its LDS cannot hold");
  if (phase == 0) {
    hipLaunchKernelGGL(k_fof2_a, dim3(std::max(1u, grid)), dim3(1024), a.W * 8, s, a);
    KCHECK("k_fof2_a");
  } else if (phase == 1) {
    hipLaunchKernelGGL(k_fof2_b, dim3(std::max(1u, grid)), dim3(1024), a.W * 16, s, a);
    KCHECK("k_fof2_b");
  } else {
    const unsigned g = nblocks(a.W, kListB);
    hipLaunchKernelGGL(k_list_counts, dim3(g), dim3(kListB), 0, s, (const uint64_t *)a.bm, a.W, a.V, 0, 1, 0u, a.V, blk);
    KCHECK("k_list_counts");
    hipLaunchKernelGGL(k_list_scatter, dim3(g), dim3(kListB), 0, s, (const uint64_t *)a.bm, a.W, a.V, 0, 1, 0u, a.V,
                       blk, out, *mail, (const uint64_t *)a.acc, 3);
    KCHECK("k_list_scatter");
  }
}

// inclusive prefix of the segments' row counts (soffs[0] = 0, soffs[i+1] = Σ_{j<=i}) and the four
// words a filtered expansion reads back: rows of the first nseg_h segments, all rows, member words
// PER > 0: PER consecutive segments per thread (nseg ≤ 1024·PER), loaded at once and kept in registers
template <int PER>
__global__ __launch_bounds__(1024) void k_seg_totals(const uint32_t *cnt, uint64_t nseg, uint64_t nseg_h,
                                                     uint64_t *soffs, const unsigned long long *member,
                                                     uint64_t cap_h, uint64_t cap_l, Mail mail) {
  constexpr int PV = PER > 0 ? PER : 1;
  __shared__ unsigned long long s_w[16];
  __shared__ uint32_t s_over;
  if (threadIdx.x == 0) s_over = 0;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t per = PER > 0 ? PER : (nseg + 1023) / 1024;
  const uint64_t i0 = min(nseg, (uint64_t)threadIdx.x * per), i1 = min(nseg, i0 + per);
  unsigned long long c = 0;
  uint32_t v[PV];
  uint32_t over = 0;  // a segment counted more rows than its arena holds (estimated caps)
  if (PER > 0) {
#pragma unroll
    for (int p = 0; p < PV; ++p) {
      const uint64_t i = i0 + p;
      const uint32_t x = cnt[i < nseg ? i : nseg - 1];
      v[p] = x & (0u - (uint32_t)(i < i1));  // mask, not select (see k_bin_scan)
      c += v[p];
      over |= (uint32_t)(v[p] > (i < nseg_h ? cap_h : cap_l));
    }
  } else {
    for (uint64_t i = i0; i < i1; ++i) {
      c += cnt[i];
      over |= (uint32_t)(cnt[i] > (i < nseg_h ? cap_h : cap_l));
    }
  }
  if (over) atomicOr(&s_over, 1u);
  unsigned long long incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(incl, off, 64);
    if (lane >= (uint32_t)off) incl += y;
  }
  if (lane == 63) s_w[wave] = incl;
  __syncthreads();
  unsigned long long base = 0;
  for (uint32_t w = 0; w < wave; ++w) base += s_w[w];
  unsigned long long run = base + incl - c;
  if (threadIdx.x == 0) soffs[0] = 0;
  if (PER > 0) {
#pragma unroll
    for (int p = 0; p < PV; ++p) {
      run += v[p];
      if (i0 + p < i1) soffs[i0 + p + 1] = run;
    }
  } else {
    for (uint64_t i = i0; i < i1; ++i) {
      run += cnt[i];
      soffs[i + 1] = run;
    }
  }
  __threadfence_block();
  __syncthreads();
  if (threadIdx.x == 0) {
    mail.p[0] = soffs[nseg_h];
    mail.p[1] = soffs[nseg];
    mail.p[2] = member ? member[0] : 0;
    mail.p[3] = member ? member[1] : 0;
    mail.p[4] = s_over;
    mail_post(mail);
  }
}
void launch_seg_totals(const uint32_t *cnt, uint64_t nseg, uint64_t nseg_h, uint64_t *soffs,
                       const unsigned long long *member, uint64_t cap_h, uint64_t cap_l, const Mail &mail,
                       hipStream_t s) {
  if (nseg == 0) {
    hipLaunchKernelGGL((k_seg_totals<0>), dim3(1), dim3(1024), 0, s, cnt, nseg, nseg_h, soffs, member, cap_h, cap_l, mail);
  } else if (nseg <= 8 * 1024) {
    hipLaunchKernelGGL((k_seg_totals<8>), dim3(1), dim3(1024), 0, s, cnt, nseg, nseg_h, soffs, member, cap_h, cap_l, mail);
  } else {
    hipLaunchKernelGGL((k_seg_totals<0>), dim3(1), dim3(1024), 0, s, cnt, nseg, nseg_h, soffs, member, cap_h, cap_l, mail);
  }
  KCHECK("k_seg_totals");
}

// ---- small host reads ------------------------------------------------------------------------------
__global__ void k_post_words(const void *p, int n, int bytes, Mail mail) {
  for (int i = 0; i < n; ++i) mail.p[i] = bytes == 8 ? ((const uint64_t *)p)[i] : (uint64_t)((const uint32_t *)p)[i];
  mail_post(mail);
}
struct PostPtrs {
  const uint64_t *p[4];
};
__global__ void k_post_ptrs(PostPtrs pp, int n, Mail mail) {
  for (int i = 0; i < n; ++i) mail.p[i] = *pp.p[i];
  mail_post(mail);
}
void launch_post_ptrs(const uint64_t *const *p, int n, const Mail &mail, hipStream_t s) {
  if (n <= 0 || n > 4) fail(OMX_E_INVALID, "post_ptrs: bad word count");
  PostPtrs pp{};
  for (int i = 0; i < n; ++i) pp.p[i] = p[i];
  hipLaunchKernelGGL(k_post_ptrs, dim3(1), dim3(1), 0, s, pp, n, mail);
  KCHECK("k_post_ptrs");
}
void launch_post_words(const void *p, int n, const Mail &mail, hipStream_t s, int bytes) {
  if (n <= 0 || n >= kMailSeq) fail(OMX_E_INVALID, "post_words: bad word count");
  hipLaunchKernelGGL(k_post_words, dim3(1), dim3(1), 0, s, p, n, bytes, mail);
  KCHECK("k_post_words");
}

// ---- helpers ----------------------------------------------------------------------------------------

__global__ void k_gather_cols(const uint32_t *idx, uint64_t n, int ncols, ColPtrs cp) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t r = idx[i];
  for (int c = 0; c < ncols; ++c) cp.out[c][i] = cp.in[c][r];
}
void launch_gather_cols(const uint32_t *idx, uint64_t n, int ncols, const uint32_t *const *in, uint32_t *const *out,
                        hipStream_t s) {
  if (!n || !ncols) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) {
    cp.in[c] = in[c];
    cp.out[c] = out[c];
  }
  hipLaunchKernelGGL(k_gather_cols, dim3(nblocks(n, 256)), dim3(256), 0, s, idx, n, ncols, cp);
  KCHECK("k_gather_cols");
}

__global__ void k_cross(uint64_t R, int ncols, ColPtrs cp, const uint32_t *cand, uint64_t ncand, uint32_t *out_dst) {
  uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= R * ncand) return;
  const uint64_t r = o / ncand, c = o % ncand;
  out_dst[o] = cand[c];
  for (int k = 0; k < ncols; ++k) cp.out[k][o] = cp.in[k][r];
}
void launch_cross(uint64_t R, int ncols, const uint32_t *const *in, uint32_t *const *out, const uint32_t *cand,
                  uint64_t ncand, uint32_t *out_dst, hipStream_t s) {
  if (!R || !ncand) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) {
    cp.in[c] = in[c];
    cp.out[c] = out[c];
  }
  hipLaunchKernelGGL(k_cross, dim3(nblocks(R * ncand, 256)), dim3(256), 0, s, R, ncols, cp, cand, ncand, out_dst);
  KCHECK("k_cross");
}

__global__ void k_flag_bitmap(const uint32_t *v, uint64_t n, const uint64_t *bm, uint8_t *flags) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = bm_test(bm, v[i]);
}
void launch_flag_bitmap(const uint32_t *v, uint64_t n, const uint64_t *bm, uint8_t *flags, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_flag_bitmap, dim3(nblocks(n, 256)), dim3(256), 0, s, v, n, bm, flags);
  KCHECK("k_flag_bitmap");
}

// Fused closing check, shorter side first: row r (x = xs[r] expanded over ax, y = ys[r] whose list ay
// is probed) is flagged when |ax(x)| > |ay(y)|, so the intersection iterates ay(y) and probes ax(x)
// instead. sums[0] += Σ |ax(x)| (the hop's E_t), sums[1] += Σ |ax(x)|·|ay(y)| (the check's E_t: every
// wedge (x, y, n) traverses ay(y)); one atomic per wave.
__global__ __launch_bounds__(256) void k_swap_flags(const uint32_t *xs, const uint32_t *ys, uint64_t R, DAdj ax,
                                                    DAdj ay, uint8_t *flags, unsigned long long *sums) {
  __shared__ uint64_t s_p[2][4];
  uint64_t dx = 0, dxy = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = adj_degree(ax, xs[r]);
    const uint64_t b = adj_degree(ay, ys[r]);
    flags[r] = a > b;
    dx += a;
    dxy += a * b;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    dx += __shfl_xor(dx, off, 64);
    dxy += __shfl_xor(dxy, off, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_p[0][w] = dx;
    s_p[1][w] = dxy;
  }
  __syncthreads();
  if (threadIdx.x < 2) {  // one atomic per block and sum: a few hundred, not one per wave
    const uint64_t t = s_p[threadIdx.x][0] + s_p[threadIdx.x][1] + s_p[threadIdx.x][2] + s_p[threadIdx.x][3];
    if (t) atomicAdd(&sums[threadIdx.x], (unsigned long long)t);
  }
}
void launch_swap_flags(const uint32_t *xs, const uint32_t *ys, uint64_t R, const DAdj &ax, const DAdj &ay,
                       uint8_t *flags, unsigned long long *sums, int cus, hipStream_t s) {
  if (!R) return;
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(R, 256), (uint64_t)cus * 2);
  hipLaunchKernelGGL(k_swap_flags, dim3(g), dim3(256), 0, s, xs, ys, R, ax, ay, flags, sums);
  KCHECK("k_swap_flags");
}

// S_ROWCMP: flags[i] = (a[i] == b[i]) == eq (record identity of two bound aliases)
__global__ void k_flag_colcmp(const uint32_t *a, const uint32_t *b, uint64_t n, int eq, uint8_t *flags) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) flags[i] = (a[i] == b[i]) == (eq != 0);
}
void launch_flag_colcmp(const uint32_t *a, const uint32_t *b, uint64_t n, bool eq, uint8_t *flags, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_flag_colcmp, dim3(nblocks(n, 256)), dim3(256), 0, s, a, b, n, (int)eq, flags);
  KCHECK("k_flag_colcmp");
}

// ---- factorized expansion (Executor::expand_factorized) ---------------------------------------------
// out[i] = index of keys[i] in the sorted, duplicate-free sorted[0..n) (every key is present)
__global__ void k_index_of(const uint32_t *sorted, uint64_t n, const uint32_t *keys, uint64_t m, uint32_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t k = keys[i];
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  out[i] = (uint32_t)lo;
}
void launch_index_of(const uint32_t *sorted, uint64_t n, const uint32_t *keys, uint64_t m, uint32_t *out, hipStream_t s) {
  if (!m) return;
  hipLaunchKernelGGL(k_index_of, dim3(nblocks(m, 256)), dim3(256), 0, s, sorted, n, keys, m, out);
  KCHECK("k_index_of");
}
// counts[key[i]] += 1
// Keys arrive in runs (an expansion writes one source's survivors contiguously), and a hub's run would
// serialise on one counter: every wave combines its runs of equal keys and issues one atomic per run.
__device__ __forceinline__ uint64_t key_runs(uint32_t k, bool valid, int lane) {
  const uint32_t prev = __shfl_up(k, 1, 64);
  return __ballot(valid && (lane == 0 || prev != k));
}
__global__ void k_key_hist(const uint32_t *key, uint64_t n, unsigned long long *counts) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = i < n;
  const uint32_t k = valid ? key[i] : 0xFFFFFFFFu;
  const uint64_t heads = key_runs(k, valid, lane);
  const int nvalid = __popcll(__ballot(valid));  // the valid lanes are a prefix of the wave
  if (valid && ((heads >> lane) & 1)) {
    const uint64_t later = lane == 63 ? 0 : heads & (~0ull << (lane + 1));
    const int nxt = later ? __ffsll((unsigned long long)later) - 1 : 64;
    atomicAdd(&counts[k], (unsigned long long)(min(nxt, nvalid) - lane));
  }
}
void launch_key_hist(const uint32_t *key, uint64_t n, unsigned long long *counts, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_key_hist, dim3(nblocks(n, 256)), dim3(256), 0, s, key, n, counts);
  KCHECK("k_key_hist");
}
// out[cursor[key[i]]++] = val[i] (cursor starts at the groups' offsets; order inside a group is free):
// the head of each run reserves the run's slots, its lanes write at the head's base + their rank
__global__ void k_key_scatter(const uint32_t *key, const uint32_t *val, uint64_t n, unsigned long long *cursor,
                              uint32_t *out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool valid = i < n;
  const uint32_t k = valid ? key[i] : 0xFFFFFFFFu;
  const uint64_t heads = key_runs(k, valid, lane);
  const int nvalid = __popcll(__ballot(valid));
  unsigned long long base = 0;
  if (valid && ((heads >> lane) & 1)) {
    const uint64_t later = lane == 63 ? 0 : heads & (~0ull << (lane + 1));
    const int nxt = later ? __ffsll((unsigned long long)later) - 1 : 64;
    base = atomicAdd(&cursor[k], (unsigned long long)(min(nxt, nvalid) - lane));
  }
  const uint64_t upto = heads & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
  const int hl = upto ? 63 - __clzll((long long)upto) : lane;  // this lane's run head
  base = __shfl(base, hl, 64);
  if (valid) out[base + (uint64_t)(lane - hl)] = val[i];
}
void launch_key_scatter(const uint32_t *key, const uint32_t *val, uint64_t n, unsigned long long *cursor, uint32_t *out,
                        hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_key_scatter, dim3(nblocks(n, 256)), dim3(256), 0, s, key, val, n, cursor, out);
  KCHECK("k_key_scatter");
}

// head[i] = 1 where a sorted key run starts
// the same over a block-segmented table (an expansion's per-worker arenas, ExpandArgs::seg_start /
// seg_count) without compacting it first: one wave per segment, kSegU × 64 entries a round. A round
// issues all its loads, then all its atomics, then its stores: vector memory completes in order, so
// one 64-entry step at a time (load, atomic, store) paid a full memory round trip per atomic.
// T = unsigned int when the entries fit 32 bits: half the counter array (0.91 M sources at M1: 3.6
// instead of 7.3 MB), so more of the atomics hit L2.
constexpr int kSegU = 4;
template <typename T>
__global__ __launch_bounds__(256) void k_key_hist_seg(const uint32_t *__restrict__ key,
                                                      const uint64_t *__restrict__ seg_start,
                                                      const uint32_t *__restrict__ seg_count, uint32_t nseg,
                                                      T *counts) {
  const uint32_t sg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= nseg) return;
  const int lane = threadIdx.x & 63;
  const uint64_t b = seg_start[sg];
  const uint32_t n = seg_count[sg];
  for (uint32_t j = 0; j < n; j += 64 * kSegU) {
    uint32_t k[kSegU];
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const uint32_t jj = j + 64u * u + lane;
      k[u] = key[b + (jj < n ? jj : 0)];  // clamped, unconditional
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const uint32_t j0 = j + 64u * u;
      const bool valid = j0 + lane < n;
      const uint32_t kk = valid ? k[u] : 0xFFFFFFFFu;
      const uint64_t heads = key_runs(kk, valid, lane);
      const int nvalid = j0 < n ? (int)min(64u, n - j0) : 0;
      if (valid && ((heads >> lane) & 1)) {
        const uint64_t later = lane == 63 ? 0 : heads & (~0ull << (lane + 1));
        const int nxt = later ? __ffsll((unsigned long long)later) - 1 : 64;
        atomicAdd(&counts[kk], (T)(min(nxt, nvalid) - lane));
      }
    }
  }
}
template <typename T>
__global__ __launch_bounds__(256) void k_key_scatter_seg(const uint32_t *__restrict__ key,
                                                         const uint32_t *__restrict__ val,
                                                         const uint64_t *__restrict__ seg_start,
                                                         const uint32_t *__restrict__ seg_count, uint32_t nseg,
                                                         T *cursor, uint32_t *out) {
  const uint32_t sg = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (sg >= nseg) return;
  const int lane = threadIdx.x & 63;
  const uint64_t b = seg_start[sg];
  const uint32_t n = seg_count[sg];
  for (uint32_t j = 0; j < n; j += 64 * kSegU) {
    uint32_t k[kSegU], v[kSegU];
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const uint32_t jj = j + 64u * u + lane;
      const uint64_t i = b + (jj < n ? jj : 0);
      k[u] = key[i];
      v[u] = val[i];
    }
    T base[kSegU];
    uint64_t heads[kSegU];
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const uint32_t j0 = j + 64u * u;
      const bool valid = j0 + lane < n;
      const uint32_t kk = valid ? k[u] : 0xFFFFFFFFu;
      heads[u] = key_runs(kk, valid, lane);
      const int nvalid = j0 < n ? (int)min(64u, n - j0) : 0;
      base[u] = 0;
      if (valid && ((heads[u] >> lane) & 1)) {
        const uint64_t later = lane == 63 ? 0 : heads[u] & (~0ull << (lane + 1));
        const int nxt = later ? __ffsll((unsigned long long)later) - 1 : 64;
        base[u] = atomicAdd(&cursor[kk], (T)(min(nxt, nvalid) - lane));
      }
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const uint32_t j0 = j + 64u * u;
      const uint64_t upto = heads[u] & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
      const int hl = upto ? 63 - __clzll((long long)upto) : lane;
      const T bs = __shfl(base[u], hl, 64);
      if (j0 + lane < n) out[bs + (uint64_t)(lane - hl)] = v[u];
    }
  }
}
template <typename T>
static void key_hist_seg(const uint32_t *key, const uint64_t *seg_start, const uint32_t *seg_count, uint32_t nseg,
                         T *counts, hipStream_t s) {
  if (!nseg) return;
  hipLaunchKernelGGL(k_key_hist_seg<T>, dim3(nblocks(nseg, 4)), dim3(256), 0, s, key, seg_start, seg_count, nseg, counts);
  KCHECK("k_key_hist_seg");
}
template <typename T>
static void key_scatter_seg(const uint32_t *key, const uint32_t *val, const uint64_t *seg_start, const uint32_t *seg_count,
                            uint32_t nseg, T *cursor, uint32_t *out, hipStream_t s) {
  if (!nseg) return;
  hipLaunchKernelGGL(k_key_scatter_seg<T>, dim3(nblocks(nseg, 4)), dim3(256), 0, s, key, val, seg_start, seg_count, nseg,
                     cursor, out);
  KCHECK("k_key_scatter_seg");
}
void launch_key_hist_seg(const uint32_t *key, const uint64_t *seg_start, const uint32_t *seg_count, uint32_t nseg,
                         unsigned long long *counts, hipStream_t s) {
  key_hist_seg(key, seg_start, seg_count, nseg, counts, s);
}
void launch_key_hist_seg(const uint32_t *key, const uint64_t *seg_start, const uint32_t *seg_count, uint32_t nseg,
                         unsigned int *counts, hipStream_t s) {
  key_hist_seg(key, seg_start, seg_count, nseg, counts, s);
}
void launch_key_scatter_seg(const uint32_t *key, const uint32_t *val, const uint64_t *seg_start, const uint32_t *seg_count,
                            uint32_t nseg, unsigned long long *cursor, uint32_t *out, hipStream_t s) {
  key_scatter_seg(key, val, seg_start, seg_count, nseg, cursor, out, s);
}
void launch_key_scatter_seg(const uint32_t *key, const uint32_t *val, const uint64_t *seg_start, const uint32_t *seg_count,
                            uint32_t nseg, unsigned int *cursor, uint32_t *out, hipStream_t s) {
  key_scatter_seg(key, val, seg_start, seg_count, nseg, cursor, out, s);
}


// ---- TRAVERSE (exec.hip Executor::traverse_bfs) -----------------------------------------------------
// out[j] = the vertex whose RID is keys[j] (left untouched when no vertex has it; RIDs are unique)
__global__ void k_find_rids(const uint64_t *rids, uint32_t V, const uint64_t *keys, uint32_t m, uint32_t *out) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < V; v += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = rids[v];
    for (uint32_t j = 0; j < m; ++j)
      if (keys[j] == r) out[j] = (uint32_t)v;
  }
}
void launch_find_rids(const uint64_t *rids, uint32_t V, const uint64_t *keys, uint32_t m, uint32_t *out, hipStream_t s) {
  if (!V || !m) return;
  hipLaunchKernelGGL(k_find_rids, dim3((unsigned)std::min<uint64_t>(nblocks(V, 256), 4096)), dim3(256), 0, s, rids, V,
                     keys, m, out);
  KCHECK("k_find_rids");
}
// A level's work-list entries w[e] in queue order: an entry is processed when its record is not in the
// history H and passes the WHILE bitmap (OTraverseRecordProcess.process :49-63); `dedup` levels claim
// each record's first position (a later entry of an accepted record meets it in the history)
__global__ void k_trav_filter(const uint32_t *w, uint64_t n, const uint64_t *hist, const uint64_t *pred,
                              uint32_t *first, uint8_t *flags, int dedup) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint32_t v = w[e];
  bool keep = !hist || !((hist[v >> 6] >> (v & 63)) & 1);
  if (keep && pred) keep = (pred[v >> 6] >> (v & 63)) & 1;
  // a repeated record (a hub reached from many entries) would serialise on one address: the claim is
  // skipped once an earlier position holds it (blocks run roughly in position order)
  if (keep && dedup && first[v] > (uint32_t)e) atomicMin(&first[v], (uint32_t)e);
  flags[e] = keep;
}
__global__ void k_trav_first(const uint32_t *w, uint64_t n, const uint32_t *first, uint8_t *flags) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n && flags[e] && first[w[e]] != (uint32_t)e) flags[e] = 0;
}
void launch_trav_filter(const uint32_t *w, uint64_t n, const uint64_t *hist, const uint64_t *pred, uint32_t *first,
                        uint8_t *flags, bool dedup, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_trav_filter, dim3(nblocks(n, 256)), dim3(256), 0, s, w, n, hist, pred, first, flags, (int)dedup);
  KCHECK("k_trav_filter");
  if (!dedup) return;
  hipLaunchKernelGGL(k_trav_first, dim3(nblocks(n, 256)), dim3(256), 0, s, w, n, first, flags);
  KCHECK("k_trav_first");
}
// out = (pred or all ones) ∧ ¬hist: the next TRAVERSE level's expansion filter
__global__ void k_andnot_bitmap(const uint64_t *pred, const uint64_t *hist, uint64_t *out, uint64_t nwords) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nwords) out[i] = (pred ? pred[i] : ~0ull) & ~hist[i];
}
void launch_andnot_bitmap(const uint64_t *pred, const uint64_t *hist, uint64_t *out, uint64_t nwords, hipStream_t s) {
  if (!nwords) return;
  hipLaunchKernelGGL(k_andnot_bitmap, dim3(nblocks(nwords, 256)), dim3(256), 0, s, pred, hist, out, nwords);
  KCHECK("k_andnot_bitmap");
}
__global__ void k_u32_to_u64(const uint32_t *a, uint64_t *b) { *b = *a; }
void launch_post_u32_to_u64(const uint32_t *a, uint64_t *b, hipStream_t s) {
  hipLaunchKernelGGL(k_u32_to_u64, dim3(1), dim3(1), 0, s, a, b);
  KCHECK("k_u32_to_u64");
}
// accepted records join the history; their first-position claims are released
__global__ void k_trav_accept(const uint32_t *w, uint64_t n, uint64_t *hist, uint32_t *first) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint32_t v = w[e];
  atomicOr((unsigned long long *)&hist[v >> 6], 1ull << (v & 63));
  first[v] = 0xFFFFFFFFu;
}
void launch_trav_accept(const uint32_t *w, uint64_t n, uint64_t *hist, uint32_t *first, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_trav_accept, dim3(nblocks(n, 256)), dim3(256), 0, s, w, n, hist, first);
  KCHECK("k_trav_accept");
}

// ---- shortestPath (exec.hip Executor::shortest_path) -------------------------------------------------
// *pos = the first work-list position whose vertex the other side has visited
__global__ void k_sp_meet(const uint32_t *w, uint64_t n, const uint64_t *other, unsigned long long *pos) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool hit = e < n && ((other[w[e] >> 6] >> (w[e] & 63)) & 1);
  const uint64_t b = __ballot(hit);
  if (b && (threadIdx.x & 63) == (uint32_t)(__ffsll((unsigned long long)b) - 1)) atomicMin(pos, (unsigned long long)e);
}
void launch_sp_meet(const uint32_t *w, uint64_t n, const uint64_t *other, unsigned long long *pos, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sp_meet, dim3(nblocks(n, 256)), dim3(256), 0, s, w, n, other, pos);
  KCHECK("k_sp_meet");
}
// the level's first discoveries (row << 32 | vertex, in discovery order): previous / next of the vertex
// = the queue entry that discovered it, the vertex joins the side's visited set and its next queue
__global__ void k_sp_accept(const uint64_t *keys, uint64_t n, const uint32_t *queue, uint32_t *parent, uint64_t *visited,
                            uint32_t *first, uint32_t *next) {
  const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const uint32_t v = (uint32_t)keys[e], row = (uint32_t)(keys[e] >> 32);
  parent[v] = queue[row];
  atomicOr((unsigned long long *)&visited[v >> 6], 1ull << (v & 63));
  first[v] = 0xFFFFFFFFu;
  next[e] = v;
}
void launch_sp_accept(const uint64_t *keys, uint64_t n, const uint32_t *queue, uint32_t *parent, uint64_t *visited,
                      uint32_t *first, uint32_t *next, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_sp_accept, dim3(nblocks(n, 256)), dim3(256), 0, s, keys, n, queue, parent, visited, first, next);
  KCHECK("k_sp_accept");
}

__global__ void k_fill_u32(uint32_t *out, uint64_t n, uint32_t x) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = x;
}
void launch_fill_u32(uint32_t *out, uint64_t n, uint32_t x, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_fill_u32, dim3(nblocks(n, 256)), dim3(256), 0, s, out, n, x);
  KCHECK("k_fill_u32");
}

__global__ void k_iota(uint32_t *out, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (uint32_t)i;
}
void launch_iota(uint32_t *out, uint64_t n, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_iota, dim3(nblocks(n, 256)), dim3(256), 0, s, out, n);
  KCHECK("k_iota");
}

__global__ void k_pack_pairs(const uint32_t *hi, const uint32_t *lo, uint64_t n, uint64_t *keys) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = ((uint64_t)hi[i] << 32) | lo[i];
}
void launch_pack_pairs(const uint32_t *hi, const uint32_t *lo, uint64_t n, uint64_t *keys, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_pack_pairs, dim3(nblocks(n, 256)), dim3(256), 0, s, hi, lo, n, keys);
  KCHECK("k_pack_pairs");
}

__global__ void k_unpack_pairs(const uint64_t *keys, uint64_t n, uint32_t *hi, uint32_t *lo) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    hi[i] = (uint32_t)(keys[i] >> 32);
    lo[i] = (uint32_t)keys[i];
  }
}
void launch_unpack_pairs(const uint64_t *keys, uint64_t n, uint32_t *hi, uint32_t *lo, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_unpack_pairs, dim3(nblocks(n, 256)), dim3(256), 0, s, keys, n, hi, lo);
  KCHECK("k_unpack_pairs");
}

__global__ void k_flag_not_in(const uint64_t *sorted, uint64_t ns, const uint64_t *keys, uint64_t n, uint8_t *flags) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = keys[i];
  uint64_t lo = 0, hi = ns;
  while (lo < hi) {
    uint64_t mid = (lo + hi) >> 1;
    if (sorted[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  flags[i] = !(lo < ns && sorted[lo] == k);
}
void launch_flag_not_in(const uint64_t *sorted, uint64_t ns, const uint64_t *keys, uint64_t n, uint8_t *flags,
                        hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_flag_not_in, dim3(nblocks(n, 256)), dim3(256), 0, s, sorted, ns, keys, n, flags);
  KCHECK("k_flag_not_in");
}

// grid-stride; a bit already set is only read (a one-column distinct of 4e8 rows over 4e4 vertices
// would otherwise serialise on a few hundred words' atomics)
__global__ __launch_bounds__(256) void k_mark_bitmap(const uint32_t *v, uint64_t n, uint64_t *bm, uint32_t V) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t x = v[i];
    if (x >= V) continue;
    const uint64_t bit = 1ull << (x & 63);
    if (!(__hip_atomic_load(&bm[x >> 6], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bit))
      atomicOr((unsigned long long *)&bm[x >> 6], (unsigned long long)bit);
  }
}
// small V (the whole bitmap fits LDS): every workgroup marks a private copy and ORs its non-zero words
// into the global one — C1 (RMAT-16: 1024 words, 9.6e5 rows) spent 145 µs in hub-word contention with
// the global atomics above
constexpr uint32_t kMarkLdsWords = 8192;  // 64 KiB: V ≤ 2^19
__global__ __launch_bounds__(1024) void k_mark_bitmap_lds(const uint32_t *v, uint64_t n, uint64_t *bm, uint32_t V) {
  __shared__ unsigned long long s_bm[kMarkLdsWords];
  const uint32_t nw = (V + 63) / 64;
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) s_bm[w] = 0;
  __syncthreads();
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x, lo = blockIdx.x * per, hi = min(n, lo + per);
  for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    const uint32_t x = v[i];
    if (x < V) atomicOr(&s_bm[x >> 6], 1ull << (x & 63));
  }
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < nw; w += blockDim.x) {
    const unsigned long long m = s_bm[w];
    if (m && (__hip_atomic_load(&bm[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & m) != m)
      atomicOr((unsigned long long *)&bm[w], m);
  }
}
void launch_mark_bitmap(const uint32_t *v, uint64_t n, uint64_t *bm, uint32_t V, hipStream_t s) {
  if (!n) return;
  if (V <= kMarkLdsWords * 64) {
    // ≥ 8192 rows per workgroup, so the flush (V/64 words per workgroup) stays small beside the marking
    const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(n / 8192, 512));
    hipLaunchKernelGGL(k_mark_bitmap_lds, dim3(g), dim3(1024), 0, s, v, n, bm, V);
    KCHECK("k_mark_bitmap_lds");
    return;
  }
  hipLaunchKernelGGL(k_mark_bitmap, dim3((unsigned)std::min<uint64_t>(nblocks(n, 256), 256 * 64)), dim3(256), 0, s, v, n,
                     bm, V);
  KCHECK("k_mark_bitmap");
}

// out[idx[i]] = val[i]
__global__ void k_scatter_u32(const uint32_t *idx, const uint32_t *val, uint64_t n, uint32_t *out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[idx[i]] = val[i];
}
void launch_scatter_u32(const uint32_t *idx, const uint32_t *val, uint64_t n, uint32_t *out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_scatter_u32, dim3(nblocks(n, 256)), dim3(256), 0, s, idx, val, n, out);
  KCHECK("k_scatter_u32");
}
__global__ void k_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = src[idx[i]];
}
void launch_gather_u32(const uint32_t *src, const uint32_t *idx, uint64_t n, uint32_t *out, hipStream_t s) {
  if (!n) return;
  hipLaunchKernelGGL(k_gather_u32, dim3(nblocks(n, 256)), dim3(256), 0, s, src, idx, n, out);
  KCHECK("k_gather_u32");
}
// the same for a device count *nd ≤ cap (threads for cap entries)
__global__ void k_gather_u32_dev(const uint32_t *src, const uint32_t *idx, const uint64_t *nd, uint32_t *out) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < *nd) out[i] = src[idx[i]];
}
void launch_gather_u32_dev(const uint32_t *src, const uint32_t *idx, const uint64_t *nd, uint64_t cap, uint32_t *out,
                           hipStream_t s) {
  if (!cap) return;
  hipLaunchKernelGGL(k_gather_u32_dev, dim3(nblocks(cap, 256)), dim3(256), 0, s, src, idx, nd, out);
  KCHECK("k_gather_u32_dev");
}

__global__ void k_flag_row_change(int ncols, ColPtrs cp, uint64_t n, uint8_t *flags) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool change = i == 0;
  for (int c = 0; c < ncols && !change; ++c) change = cp.in[c][i] != cp.in[c][i - 1];
  flags[i] = change;
}
void launch_flag_row_change(int ncols, const uint32_t *const *cols, uint64_t n, uint8_t *flags, hipStream_t s) {
  if (!n) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) cp.in[c] = cols[c];
  hipLaunchKernelGGL(k_flag_row_change, dim3(nblocks(n, 256)), dim3(256), 0, s, ncols, cp, n, flags);
  KCHECK("k_flag_row_change");
}

// a null binding (an unmatched optional node: dense id V) maps to kNullRid
__device__ __forceinline__ uint64_t rid_of(const uint64_t *rids, uint32_t v, uint32_t V) {
  return v >= V ? kNullRid : rids ? rids[v] : (uint64_t)v;
}
__global__ void k_map_rids(int ncols, ColPtrs cp, uint64_t n, const uint64_t *rids, uint64_t *out, uint32_t V) {
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for (int c = 0; c < ncols; ++c) out[i * ncols + c] = rid_of(rids, cp.in[c][i], V);
}
void launch_map_rids(int ncols, const uint32_t *const *cols, uint64_t n, const uint64_t *rids, uint64_t *out,
                     uint32_t V, hipStream_t s) {
  if (!n || !ncols) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) cp.in[c] = cols[c];
  hipLaunchKernelGGL(k_map_rids, dim3(nblocks(n, 256)), dim3(256), 0, s, ncols, cp, n, rids, out, V);
  KCHECK("k_map_rids");
}

// ---- order-independent digest of a result table (OMX_FLAG_DIGEST) --------------------------------------
// digest = Σ_rows h(row) mod 2^64, h = splitmix64 chained over the row's RIDs in column order (the same
// function as oracle/dfs.py row_digest): the parity tests compare whole result sets of ~1e9 rows
// without copying them to the host.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_digest(int ncols, ColPtrs cp, uint64_t n, const uint64_t *rids, uint32_t V,
                                                unsigned long long *out) {
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int c = 0; c < ncols; ++c) {
      h = mix64(h ^ rid_of(rids, cp.in[c][i], V));
    }
    acc += h;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}
void launch_digest(int ncols, const uint32_t *const *cols, uint64_t n, const uint64_t *rids, uint32_t V,
                   unsigned long long *out, int cus, hipStream_t s) {
  if (!n || !ncols) return;
  ColPtrs cp;
  for (int c = 0; c < ncols; ++c) cp.in[c] = cols[c];
  const unsigned g = (unsigned)std::min<uint64_t>(nblocks(n, 256), (uint64_t)cus * 8);
  hipLaunchKernelGGL(k_digest, dim3(g), dim3(256), 0, s, ncols, cp, n, rids, V, out);
  KCHECK("k_digest");
}

}  // namespace omx
