// devtypes.h — plain structs shared by host code and gfx950 kernels (passed by value as kernel args).
#pragma once
#include <cstdint>

namespace omx {

// One adjacency "part": the CSR of one edge class in one direction (out_<E> or in_<E> ridbags of every
// vertex, B/OrientVertex.java:401-460). A traversal over several labels / both() concatenates parts,
// exactly like OrientVertex.getVertices iterates several out_X/in_X fields in turn.
struct DAdjPart {
  const uint64_t *rp;   // [V+1]
  const uint32_t *col;  // [E]
};

constexpr int kMaxAdjParts = 8;
struct DAdj {
  DAdjPart p[kMaxAdjParts];
  int32_t n;
  int32_t sorted;  // every part's rows sorted ascending (binary-searchable)
};

// Device view of one property column (C/record/impl/ODocument.java field values, columnar).
struct DColumn {
  const void *values;      // int32 / int64 / double / int32 dictionary codes
  const uint8_t *present;  // 1 = field present; nullptr = always present
  int32_t type;            // OMX_PROP_*
  int32_t pad;
};

// Predicate program (WHERE / while compiled to a stack machine; P/OWhereClause.java:36-41).
enum PredOp : int32_t {
  P_PUSH_COL = 1,  // arg = column index
  P_PUSH_INT,      // i
  P_PUSH_DBL,      // d
  P_PUSH_NULL,
  P_PUSH_BOOL,     // i
  P_PUSH_DEPTH,    // $depth
  P_PUSH_DEG,      // arg = adjacency index in DPred::deg (out/in/both('L').size())
  P_ADD, P_SUB, P_MUL, P_DIV, P_MOD,
  P_EQ, P_NE, P_LT, P_LE, P_GT, P_GE,
  P_AND, P_OR, P_NOT,
  P_TRUTH,         // value is boolean true
};

struct DPredInstr {
  int32_t op;
  int32_t arg;
  int64_t i;
  double d;
};

constexpr int kMaxPred = 40;
constexpr int kMaxDegAdj = 3;
struct DPred {
  DPredInstr code[kMaxPred];
  int32_t n;          // 0 = no program (always true)
  int32_t use_class;  // 1 = also require class_id ∈ class_mask (polymorphic class test)
  uint64_t class_mask[4];
  DAdj deg[kMaxDegAdj];
  const DColumn *cols;
  const uint16_t *vclass;
  // fast path (no interpreter): n_atoms comparisons "column OP constant", all AND (conj=1) or all OR
  int32_t n_atoms;
  int32_t conj;
  int32_t atom_col[4];
  int32_t atom_op[4];
  int64_t atom_i[4];
  double atom_d[4];
  int32_t atom_dbl[4];  // compare as double (double column or double constant)
  DColumn atom_c[4];    // the atoms' column descriptors (kernel-argument copies: no dependent load)
};

}  // namespace omx
