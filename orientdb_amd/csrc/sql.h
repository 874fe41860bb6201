// sql.h — AST of the MATCH statement subset the engine parses.
//
// Grammar restated from core/src/main/grammar/OrientSQL.jjt:1138-1170 (MatchStatement),
// :3277-3560 (MatchExpression, MatchPathItem, MatchFilter, arrows) of the reference; node classes
// mirror P/OMatchStatement.java, P/OMatchExpression.java, P/OMatchPathItem.java,
// P/OMultiMatchPathItem.java, P/OMatchFilter.java (P/ = core/src/main/java/.../core/sql/parser/).
#pragma once
#include <memory>
#include <string>
#include <vector>

namespace omx {

struct Expr;
using ExprP = std::shared_ptr<Expr>;

// Values of literals and parameters.
struct Value {
  enum Kind { NUL, INT, DBL, STR, BOOL } kind = NUL;
  int64_t i = 0;
  double d = 0;
  std::string s;
  static Value Int(int64_t v) { Value x; x.kind = INT; x.i = v; return x; }
  static Value Dbl(double v) { Value x; x.kind = DBL; x.d = v; return x; }
  static Value Str(const std::string &v) { Value x; x.kind = STR; x.s = v; return x; }
  static Value Bool(bool v) { Value x; x.kind = BOOL; x.i = v; return x; }
};

struct Suffix {
  enum Kind { FIELD, METHOD, INDEX } kind;
  std::string name;
  std::vector<ExprP> args;
  // INDEX selectors (OArraySelector / OArrayRangeSelector / OArraySingleValuesSelector / a condition):
  // [i] → index; [a-b] → index..index2 (exclusive); [i, j, …] → items; [cond] → index (a condition)
  enum Sel { SEL_ONE, SEL_RANGE, SEL_MULTI, SEL_COND } sel = SEL_ONE;
  ExprP index, index2;
  std::vector<ExprP> items;
};

struct Expr {
  enum Kind {
    LIT,    // value
    PARAM,  // ? (index) or :name
    FIELD,  // identifier (field of the current record, or a context variable of that name)
    VAR,    // $depth, $matched, $currentMatch, $current, $matches, ...
    MATH,   // op + - * / % ; kids[0], kids[1]
    CALL,   // function call name(args) on the current record, e.g. in('ManagerOf')
    CHAIN,  // kids[0] followed by suffixes
    JSON,   // {'k': expr, ...}
    ARRAY,  // [expr, ...]
    OR, AND, NOT,
    CMP,    // op = == != <> < <= > >= ; kids[0], kids[1]
    TRUTH,  // boolean value of kids[0]
    RID,    // record id literal #c:p: value.i = (c << 48) | p
  } kind;
  Value value;
  std::string name;  // FIELD/VAR/CALL name, PARAM name, MATH/CMP operator
  int param_index = -1;
  std::vector<ExprP> kids;
  std::vector<Suffix> suffixes;
  std::vector<std::string> json_keys;
};

struct MatchFilter {
  std::string alias;
  std::string class_name;
  ExprP where, while_;
  bool has_max_depth = false;
  int max_depth = 0;
  bool optional = false;
};

struct PathItem {
  std::string method;              // out/in/both/outE/inE/bothE/outV/inV/bothV ("" for a multi item)
  std::vector<std::string> labels; // edge class labels; empty = any
  MatchFilter filter;
  bool has_filter = false;
  bool is_multi = false;
  std::vector<PathItem> multi;     // sub-items of .( ... )
  // OMatchPathItem.isBidirectional (P/OMatchPathItem.java:29-40)
  bool bidirectional() const;
};

struct MatchExpression {
  MatchFilter origin;
  std::vector<PathItem> items;
};

struct ReturnItem {
  ExprP expr;
  std::string alias;  // AS alias ("" if none)
  std::string text;   // canonical text, for $matches/$paths detection
  std::string raw;    // the item's tokens joined by spaces (string literals unquoted): its default alias
};

// FROM target of a legacy TRAVERSE / SELECT (S/filter/OSQLTarget.java): records by RID, or a class
struct Target {
  std::vector<std::pair<int64_t, int64_t>> rids;  // #c:p or [#c:p, ...], in the order written
  std::string class_name;                         // FROM <class> (polymorphic)
  std::string other;                              // anything else (sub-query, cluster:, index:): its text
};

struct Statement {
  // MATCH (P/OMatchStatement.java); TRAVERSE (S/OCommandExecutorSQLTraverse.java:64-139);
  // SELECT expand(<chain>) (S/OCommandExecutorSQLSelect.java, GF/OSQLFunctionMove.java:66-91)
  enum Kind { MATCH, TRAVERSE, SELECT } kind = MATCH;
  std::vector<MatchExpression> expressions;
  std::vector<ReturnItem> returns;
  bool has_limit = false;
  int64_t limit = -1;
  int n_positional = 0;
  // TRAVERSE / SELECT
  Target target;
  std::vector<ExprP> fields;  // TRAVERSE: the fields to traverse, as written; SELECT: the expand() argument
  ExprP where;                // TRAVERSE: WHILE (or the deprecated WHERE); SELECT: WHERE
  int max_depth = -1;         // TRAVERSE MAXDEPTH (-1: none)
  bool breadth_first = false; // TRAVERSE STRATEGY BREADTH_FIRST (default DEPTH_FIRST, OTraverse.java)
  bool expand = true;         // SELECT: expand(fields[0]) (rows) or the projection fields[0] [AS alias]
  std::string alias;          // SELECT projection alias ("" = the default)
  std::string unsupported;    // a clause the device engine does not execute (reported by the planner)
};

// Parses a MATCH, TRAVERSE or SELECT statement; throws OmxError(OMX_E_PARSE) on syntax errors.
std::unique_ptr<Statement> parse_statement(const std::string &text);
inline std::unique_ptr<Statement> parse_match(const std::string &text) { return parse_statement(text); }

// Canonical text of an expression (used for default return aliases and diagnostics).
std::string expr_text(const ExprP &e);

}  // namespace omx
