// sql.cpp — lexer and recursive-descent parser for the MATCH statement subset.
//
// Follows the MATCH productions of core/src/main/grammar/OrientSQL.jjt (:1138-1170 MatchStatement,
// :3277-3560 match expressions / path items / filters / arrow forms) of the reference. Arrow items:
//   -L->  ≡ .out('L')     <-L-  ≡ .in('L')     -L-  ≡ .both('L')     -->, <--, --  = any label.
#include "sql.h"

#include <cctype>
#include <cstdlib>

#include "common.h"

namespace omx {

bool PathItem::bidirectional() const {
  if (is_multi) return false;  // OMultiMatchPathItem.isBidirectional (P/OMultiMatchPathItem.java:27-29)
  if (filter.while_ || filter.has_max_depth || filter.optional) return false;
  // OMethodCall.bidirectionalMethods (P/OMethodCall.java:21)
  std::string m = lower(method);
  return m == "out" || m == "in" || m == "both" || m == "oute" || m == "ine" || m == "inv" || m == "outv";
}

namespace {

struct Tok {
  enum Kind { ID, NUM, STR, OP, RID, END } kind;  // RID: "#c:p" → v = "c:p"
  std::string v;
};

std::vector<Tok> tokenize(const std::string &s) {
  std::vector<Tok> out;
  size_t i = 0, n = s.size();
  static const char *ops2[] = {"<>", "!=", "<=", ">=", "==", "->", "<-", "--"};
  while (i < n) {
    char c = s[i];
    if (isspace((unsigned char)c)) { ++i; continue; }
    if (isdigit((unsigned char)c)) {
      size_t j = i;
      while (j < n && isdigit((unsigned char)s[j])) ++j;
      if (j + 1 < n && s[j] == '.' && isdigit((unsigned char)s[j + 1])) {
        ++j;
        while (j < n && isdigit((unsigned char)s[j])) ++j;
      }
      out.push_back({Tok::NUM, s.substr(i, j - i)});
      i = j;
      continue;
    }
    if (c == '\'' || c == '"') {
      std::string v;
      size_t j = i + 1;
      while (j < n && s[j] != c) {
        if (s[j] == '\\' && j + 1 < n) { v += s[j + 1]; j += 2; continue; }
        v += s[j++];
      }
      if (j >= n) fail(OMX_E_PARSE, "unterminated string literal");
      out.push_back({Tok::STR, v});
      i = j + 1;
      continue;
    }
    if (isalpha((unsigned char)c) || c == '_' || ((c == '$' || c == '@') && i + 1 < n &&
                                                  (isalpha((unsigned char)s[i + 1]) || s[i + 1] == '_'))) {
      size_t j = i + 1;
      while (j < n && (isalnum((unsigned char)s[j]) || s[j] == '_')) ++j;
      out.push_back({Tok::ID, s.substr(i, j - i)});
      i = j;
      continue;
    }
    if (c == '#' && i + 1 < n && (isdigit((unsigned char)s[i + 1]) || s[i + 1] == '-')) {  // record id #c:p
      size_t j = i + 1;
      if (s[j] == '-') ++j;
      while (j < n && isdigit((unsigned char)s[j])) ++j;
      if (j >= n || s[j] != ':') fail(OMX_E_PARSE, "malformed record id at offset " + std::to_string(i));
      ++j;
      if (j < n && s[j] == '-') ++j;
      while (j < n && isdigit((unsigned char)s[j])) ++j;
      out.push_back({Tok::RID, s.substr(i + 1, j - i - 1)});
      i = j;
      continue;
    }
    if (c == '`') {  // quoted identifier
      size_t j = s.find('`', i + 1);
      if (j == std::string::npos) fail(OMX_E_PARSE, "unterminated quoted identifier");
      out.push_back({Tok::ID, s.substr(i + 1, j - i - 1)});
      i = j + 1;
      continue;
    }
    bool two = false;
    if (i + 1 < n) {
      for (auto *o : ops2)
        if (s[i] == o[0] && s[i + 1] == o[1]) {
          out.push_back({Tok::OP, std::string(o, 2)});
          i += 2;
          two = true;
          break;
        }
    }
    if (two) continue;
    if (std::string("-+*/%=<>{}()[],:.?").find(c) != std::string::npos) {
      out.push_back({Tok::OP, std::string(1, c)});
      ++i;
      continue;
    }
    fail(OMX_E_PARSE, std::string("unexpected character '") + c + "' at offset " + std::to_string(i));
  }
  out.push_back({Tok::END, ""});
  return out;
}

ExprP mk(Expr::Kind k) {
  auto e = std::make_shared<Expr>();
  e->kind = k;
  return e;
}

class Parser {
 public:
  explicit Parser(const std::string &text) : t_(tokenize(text)) {}

  std::unique_ptr<Statement> statement() {
    if (kw("traverse")) return traverse();
    if (kw("select")) return select();
    if (!kw("match")) fail(OMX_E_PARSE, "MATCH, TRAVERSE or SELECT expected");
    ++i_;
    auto st = std::make_unique<Statement>();
    st->expressions.push_back(match_expression());
    while (op(",")) {
      ++i_;
      st->expressions.push_back(match_expression());
    }
    if (!kw("return")) fail(OMX_E_PARSE, "RETURN expected");
    ++i_;
    for (;;) {
      ReturnItem ri;
      const size_t start = i_;
      ri.expr = expr();
      ri.text = expr_text(ri.expr);
      for (size_t k = start; k < i_; ++k) ri.raw += (k > start ? " " : "") + t_[k].v;
      if (kw("as")) {
        ++i_;
        ri.alias = next().v;
      }
      st->returns.push_back(ri);
      if (op(",")) { ++i_; continue; }
      break;
    }
    if (kw("limit")) limit(*st);
    if (t_[i_].kind != Tok::END) fail(OMX_E_PARSE, "unexpected token '" + t_[i_].v + "'");
    st->n_positional = nparam_;
    return st;
  }

  // TRAVERSE <field>[, <field>]* FROM <target> [WHILE <cond>] [LIMIT n] [MAXDEPTH n] [STRATEGY s]
  // (OCommandExecutorSQLTraverse.parse / parseFields, S/OCommandExecutorSQLTraverse.java:64-139,212-247)
  std::unique_ptr<Statement> traverse() {
    ++i_;
    auto st = std::make_unique<Statement>();
    st->kind = Statement::TRAVERSE;
    if (kw("from")) fail(OMX_E_PARSE, "Missed field list to cross in TRAVERSE");
    for (;;) {
      if (op("*")) {
        ++i_;
        auto all = mk(Expr::FIELD);
        all->name = "*";
        st->fields.push_back(all);
      } else {
        st->fields.push_back(expr());
      }
      if (!op(",")) break;
      ++i_;
    }
    if (!kw("from")) fail(OMX_E_PARSE, "Missed FROM in TRAVERSE");
    ++i_;
    target(*st);
    if (kw("while") || kw("where")) {  // WHERE: the deprecated spelling of WHILE (:93-102)
      ++i_;
      st->where = or_expr();
    }
    while (t_[i_].kind != Tok::END) {
      if (kw("limit")) {
        limit(*st);
        if (st->limit == 0 || st->limit < -1) fail(OMX_E_PARSE, "Limit must be > 0 or = -1 (no limit)");
      } else if (kw("maxdepth")) {
        ++i_;
        Tok n = next();
        if (n.kind != Tok::NUM && !(n.kind == Tok::OP && n.v == "-")) fail(OMX_E_PARSE, "Invalid MAXDEPTH value");
        if (n.kind != Tok::NUM) fail(OMX_E_PARSE, "Invalid MAXDEPTH: value set minor than ZERO");
        st->max_depth = std::atoi(n.v.c_str());
      } else if (kw("strategy")) {
        ++i_;
        const std::string w = lower(next().v);
        if (w == "breadth_first") st->breadth_first = true;
        else if (w == "depth_first") st->breadth_first = false;
        else fail(OMX_E_PARSE, "Invalid STRATEGY. Use one between [DEPTH_FIRST, BREADTH_FIRST]");
      } else if (kw("skip") || kw("offset") || kw("timeout")) {
        st->unsupported = lower(next().v) + " in TRAVERSE";
        next();
      } else {
        fail(OMX_E_PARSE, "unexpected token '" + t_[i_].v + "'");
      }
    }
    st->n_positional = nparam_;
    return st;
  }

  // SELECT expand(<chain>) FROM <target> [WHERE <cond>] [LIMIT n]: the rows of the expanded chain;
  // SELECT shortestPath(...) [AS a] / SELECT expand(shortestPath(...)) (no FROM). Other SELECT forms are
  // the legacy SQL executor's and stay there.
  std::unique_ptr<Statement> select() {
    ++i_;
    auto st = std::make_unique<Statement>();
    st->kind = Statement::SELECT;
    if (kw("expand") && op("(", 1)) {
      ++i_;
      expect("(");
      st->fields.push_back(expr());
      expect(")");
    } else if (kw("shortestPath") && op("(", 1)) {
      st->expand = false;
      st->fields.push_back(expr());
      if (kw("as")) {
        ++i_;
        st->alias = next().v;
      }
    } else {
      fail(OMX_E_UNSUPPORTED, "SELECT without expand() or shortestPath(): the legacy SQL executor's");
    }
    if (op(",")) fail(OMX_E_UNSUPPORTED, "SELECT with several projections on the device");
    if (!kw("from")) {
      if (t_[i_].kind != Tok::END && !kw("limit")) fail(OMX_E_UNSUPPORTED, "SELECT clause '" + t_[i_].v + "' on the device");
      st->target.other = "";
      if (kw("limit")) limit(*st);
      if (t_[i_].kind != Tok::END) fail(OMX_E_UNSUPPORTED, "SELECT clause '" + t_[i_].v + "' on the device");
      st->n_positional = nparam_;
      return st;
    }
    ++i_;
    target(*st);
    if (kw("where")) {
      ++i_;
      st->where = or_expr();
    }
    if (kw("limit")) limit(*st);
    if (t_[i_].kind != Tok::END) fail(OMX_E_UNSUPPORTED, "SELECT clause '" + t_[i_].v + "' on the device");
    st->n_positional = nparam_;
    return st;
  }

  void limit(Statement &st) {
    ++i_;
    bool neg = false;
    if (op("-")) { ++i_; neg = true; }
    Tok n = next();
    if (n.kind != Tok::NUM) fail(OMX_E_PARSE, "LIMIT expects an integer");
    st.has_limit = true;
    st.limit = std::strtoll(n.v.c_str(), nullptr, 10) * (neg ? -1 : 1);
  }

  static std::pair<int64_t, int64_t> rid_of(const std::string &v) {
    const size_t c = v.find(':');
    return {std::strtoll(v.substr(0, c).c_str(), nullptr, 10), std::strtoll(v.substr(c + 1).c_str(), nullptr, 10)};
  }

  // OSQLTarget (S/filter/OSQLTarget.java): a record id, a list of them, a class; other forms are kept as
  // text (the planner reports them unsupported)
  void target(Statement &st) {
    if (peek().kind == Tok::RID) {
      st.target.rids.push_back(rid_of(next().v));
    } else if (op("[")) {
      ++i_;
      while (!op("]")) {
        Tok t = next();
        if (t.kind != Tok::RID) fail(OMX_E_PARSE, "record id expected in the target list");
        st.target.rids.push_back(rid_of(t.v));
        if (op(",")) ++i_;
      }
      ++i_;
    } else if (op("(")) {
      int depth = 0;
      do {
        if (t_[i_].kind == Tok::END) fail(OMX_E_PARSE, "unbalanced parentheses in the target");
        if (op("(")) ++depth;
        if (op(")")) --depth;
        st.target.other += t_[i_++].v + " ";
      } while (depth > 0);
    } else if (peek().kind == Tok::ID && op(":", 1)) {  // cluster:x, index:x, metadata:x
      st.target.other = next().v;
      st.target.other += ":" + (++i_, next().v);
    } else if (peek().kind == Tok::ID) {
      st.target.class_name = next().v;
    } else {
      fail(OMX_E_PARSE, "target expected after FROM");
    }
  }

 private:
  std::vector<Tok> t_;
  size_t i_ = 0;
  int nparam_ = 0;

  const Tok &peek(size_t k = 0) const { return t_[std::min(i_ + k, t_.size() - 1)]; }
  Tok next() { return t_[std::min(i_++, t_.size() - 1)]; }
  bool op(const char *v, size_t k = 0) const { return peek(k).kind == Tok::OP && peek(k).v == v; }
  bool kw(const char *v, size_t k = 0) const { return peek(k).kind == Tok::ID && ieq(peek(k).v, v); }
  void expect(const char *v) {
    Tok t = next();
    if (!(t.kind == Tok::OP && t.v == v)) fail(OMX_E_PARSE, std::string("expected '") + v + "', got '" + t.v + "'");
  }

  MatchExpression match_expression() {
    MatchExpression me;
    me.origin = match_filter();
    for (;;) {
      if (op(".")) me.items.push_back(method_item());
      else if (op("-") || op("<-") || op("--")) me.items.push_back(arrow_item());
      else break;
    }
    return me;
  }

  MatchFilter match_filter() {
    expect("{");
    MatchFilter f;
    bool first = true;
    while (!op("}")) {
      if (!first) expect(",");
      first = false;
      std::string key = lower(next().v);
      expect(":");
      if (key == "class") {
        f.class_name = next().v;
      } else if (key == "as") {
        f.alias = next().v;
      } else if (key == "where") {
        expect("(");
        f.where = or_expr();
        expect(")");
      } else if (key == "while") {
        expect("(");
        f.while_ = or_expr();
        expect(")");
      } else if (key == "maxdepth") {
        Tok n = next();
        if (n.kind != Tok::NUM) fail(OMX_E_PARSE, "maxDepth expects an integer");
        f.has_max_depth = true;
        f.max_depth = std::atoi(n.v.c_str());
      } else if (key == "optional") {
        f.optional = ieq(next().v, "true");
      } else {
        fail(OMX_E_PARSE, "unknown match filter item '" + key + "'");
      }
    }
    expect("}");
    return f;
  }

  std::vector<std::string> labels() {
    expect("(");
    std::vector<std::string> out;
    while (!op(")")) {
      Tok t = next();
      if (t.kind != Tok::STR && t.kind != Tok::ID) fail(OMX_E_PARSE, "edge label expected");
      out.push_back(t.v);
      if (op(",")) ++i_;
    }
    expect(")");
    return out;
  }

  PathItem method_item() {
    expect(".");
    PathItem it;
    if (op("(")) {
      ++i_;
      it.is_multi = true;
      while (!op(")")) {
        if (op(".")) {
          it.multi.push_back(method_item());
        } else if (peek().kind == Tok::ID) {  // OMatchPathItemFirst (P/OMatchPathItemFirst.java)
          PathItem sub;
          sub.method = next().v;
          sub.labels = labels();
          if (op("{")) { sub.filter = match_filter(); sub.has_filter = true; }
          it.multi.push_back(sub);
        } else {
          it.multi.push_back(arrow_item());
        }
      }
      expect(")");
      if (op("{")) { it.filter = match_filter(); it.has_filter = true; }
      return it;
    }
    it.method = next().v;
    it.labels = labels();
    if (op("{")) { it.filter = match_filter(); it.has_filter = true; }
    return it;
  }

  PathItem arrow_item() {
    PathItem it;
    if (op("--")) {  // "-->" (tokenised "--" ">") or "--"
      ++i_;
      if (op(">")) { ++i_; it.method = "out"; }
      else it.method = "both";
    } else if (op("<-")) {
      ++i_;
      if (op("-")) ++i_;
      else { it.labels.push_back(next().v); expect("-"); }
      it.method = "in";
    } else {
      expect("-");
      if (op("->")) { ++i_; it.method = "out"; }
      else if (op("-")) { ++i_; it.method = "both"; }
      else {
        it.labels.push_back(next().v);
        if (op("->")) { ++i_; it.method = "out"; }
        else { expect("-"); it.method = "both"; }
      }
    }
    it.filter = match_filter();
    it.has_filter = true;
    return it;
  }

  // boolean expressions (OWhereClause → OOrBlock → OAndBlock → ONotBlock → OBinaryCondition)
  ExprP or_expr() {
    ExprP a = and_expr();
    if (!kw("or")) return a;
    auto o = mk(Expr::OR);
    o->kids.push_back(a);
    while (kw("or")) { ++i_; o->kids.push_back(and_expr()); }
    return o;
  }
  ExprP and_expr() {
    ExprP a = not_expr();
    if (!kw("and")) return a;
    auto o = mk(Expr::AND);
    o->kids.push_back(a);
    while (kw("and")) { ++i_; o->kids.push_back(not_expr()); }
    return o;
  }
  ExprP not_expr() {
    if (kw("not")) {
      ++i_;
      auto n = mk(Expr::NOT);
      n->kids.push_back(not_expr());
      return n;
    }
    return cmp_expr();
  }
  ExprP cmp_expr() {
    ExprP l = expr();
    const Tok &t = peek();
    if (t.kind == Tok::OP && (t.v == "=" || t.v == "==" || t.v == "!=" || t.v == "<>" || t.v == "<" || t.v == "<=" ||
                              t.v == ">" || t.v == ">=")) {
      ++i_;
      auto c = mk(Expr::CMP);
      c->name = t.v == "==" ? "=" : (t.v == "<>" ? "!=" : t.v);
      c->kids.push_back(l);
      c->kids.push_back(expr());
      return c;
    }
    // a parenthesised condition is already boolean: `(a and b) or c`
    if (l->kind == Expr::OR || l->kind == Expr::AND || l->kind == Expr::NOT || l->kind == Expr::CMP) return l;
    auto tr = mk(Expr::TRUTH);
    tr->kids.push_back(l);
    return tr;
  }
  ExprP expr() {
    ExprP l = term();
    while (op("+") || op("-")) {
      auto m = mk(Expr::MATH);
      m->name = next().v;
      m->kids.push_back(l);
      m->kids.push_back(term());
      l = m;
    }
    return l;
  }
  ExprP term() {
    ExprP l = unary();
    while (op("*") || op("/") || op("%")) {
      auto m = mk(Expr::MATH);
      m->name = next().v;
      m->kids.push_back(l);
      m->kids.push_back(unary());
      l = m;
    }
    return l;
  }
  ExprP unary() {
    if (op("-")) {
      ++i_;
      auto m = mk(Expr::MATH);
      m->name = "-";
      auto z = mk(Expr::LIT);
      z->value = Value::Int(0);
      m->kids.push_back(z);
      m->kids.push_back(unary());
      return m;
    }
    return postfix();
  }
  std::vector<ExprP> call_args() {
    expect("(");
    std::vector<ExprP> a;
    while (!op(")")) {
      a.push_back(expr());
      if (op(",")) ++i_;
    }
    expect(")");
    return a;
  }
  ExprP postfix() {
    ExprP base = primary();
    std::vector<Suffix> sfx;
    for (;;) {
      if (op(".")) {
        ++i_;
        Suffix s;
        s.name = next().v;
        if (op("(")) { s.kind = Suffix::METHOD; s.args = call_args(); }
        else s.kind = Suffix::FIELD;
        sfx.push_back(s);
      } else if (op("[")) {
        ++i_;
        Suffix s;
        s.kind = Suffix::INDEX;
        if (peek().kind == Tok::NUM && peek(1).kind == Tok::OP && peek(1).v == "-" && peek(2).kind == Tok::NUM &&
            peek(3).kind == Tok::OP && peek(3).v == "]") {  // [a-b]: a range, not a subtraction
          s.sel = Suffix::SEL_RANGE;
          s.index = mk(Expr::LIT);
          s.index->value = Value::Int(std::strtoll(next().v.c_str(), nullptr, 10));
          ++i_;
          s.index2 = mk(Expr::LIT);
          s.index2->value = Value::Int(std::strtoll(next().v.c_str(), nullptr, 10));
        } else {
          ExprP sel = or_expr();
          if (op("-")) {
            ++i_;
            s.sel = Suffix::SEL_RANGE;
            s.index = sel->kind == Expr::TRUTH ? sel->kids[0] : sel;
            s.index2 = expr();
          } else if (op(",")) {
            s.sel = Suffix::SEL_MULTI;
            s.items.push_back(sel->kind == Expr::TRUTH ? sel->kids[0] : sel);
            while (op(",")) {
              ++i_;
              s.items.push_back(expr());
            }
          } else if (sel->kind == Expr::TRUTH) {
            s.sel = Suffix::SEL_ONE;
            s.index = sel->kids[0];
          } else {
            s.sel = Suffix::SEL_COND;
            s.index = sel;
          }
        }
        expect("]");
        sfx.push_back(s);
      } else {
        break;
      }
    }
    if (sfx.empty()) return base;
    auto c = mk(Expr::CHAIN);
    c->kids.push_back(base);
    c->suffixes = sfx;
    return c;
  }
  ExprP primary() {
    Tok t = next();
    if (t.kind == Tok::NUM) {
      auto e = mk(Expr::LIT);
      if (t.v.find('.') != std::string::npos) e->value = Value::Dbl(std::strtod(t.v.c_str(), nullptr));
      else e->value = Value::Int(std::strtoll(t.v.c_str(), nullptr, 10));
      return e;
    }
    if (t.kind == Tok::STR) {
      auto e = mk(Expr::LIT);
      e->value = Value::Str(t.v);
      return e;
    }
    if (t.kind == Tok::OP && t.v == "(") {
      ExprP e = or_expr();
      expect(")");
      if (e->kind == Expr::TRUTH) return e->kids[0];  // a parenthesised value
      return e;
    }
    if (t.kind == Tok::RID) {
      auto e = mk(Expr::RID);
      const auto r = rid_of(t.v);
      e->value = Value::Int((int64_t)(((uint64_t)r.first << 48) | ((uint64_t)r.second & ((1ull << 48) - 1))));
      e->name = "#" + t.v;
      return e;
    }
    if (t.kind == Tok::OP && t.v == "?") {
      auto e = mk(Expr::PARAM);
      e->param_index = nparam_++;
      return e;
    }
    if (t.kind == Tok::OP && t.v == ":") {
      auto e = mk(Expr::PARAM);
      e->name = next().v;
      return e;
    }
    if (t.kind == Tok::OP && t.v == "{") {
      auto e = mk(Expr::JSON);
      while (!op("}")) {
        e->json_keys.push_back(next().v);
        expect(":");
        e->kids.push_back(expr());
        if (op(",")) ++i_;
      }
      expect("}");
      return e;
    }
    if (t.kind == Tok::OP && t.v == "[") {
      auto e = mk(Expr::ARRAY);
      while (!op("]")) {
        e->kids.push_back(expr());
        if (op(",")) ++i_;
      }
      expect("]");
      return e;
    }
    if (t.kind == Tok::ID) {
      std::string l = lower(t.v);
      if (l == "true" || l == "false") {
        auto e = mk(Expr::LIT);
        e->value = Value::Bool(l == "true");
        return e;
      }
      if (l == "null") return mk(Expr::LIT);
      if (op("(")) {
        auto e = mk(Expr::CALL);
        e->name = t.v;
        e->kids = call_args();
        return e;
      }
      auto e = mk(t.v[0] == '$' ? Expr::VAR : Expr::FIELD);
      e->name = t.v;
      return e;
    }
    fail(OMX_E_PARSE, "unexpected token '" + t.v + "'");
  }
};

}  // namespace

std::string expr_text(const ExprP &e) {
  if (!e) return "";
  switch (e->kind) {
    case Expr::LIT:
      switch (e->value.kind) {
        case Value::NUL: return "null";
        case Value::INT: return std::to_string(e->value.i);
        case Value::DBL: return std::to_string(e->value.d);
        case Value::STR: return "'" + e->value.s + "'";
        case Value::BOOL: return e->value.i ? "true" : "false";
      }
      return "";
    case Expr::PARAM: return e->name.empty() ? "?" : ":" + e->name;
    case Expr::FIELD:
    case Expr::VAR: return e->name;
    case Expr::MATH: return expr_text(e->kids[0]) + " " + e->name + " " + expr_text(e->kids[1]);
    case Expr::CALL: {
      std::string s = e->name + "(";
      for (size_t i = 0; i < e->kids.size(); ++i) s += (i ? ", " : "") + expr_text(e->kids[i]);
      return s + ")";
    }
    case Expr::CHAIN: {
      std::string s = expr_text(e->kids[0]);
      for (auto &x : e->suffixes) {
        if (x.kind == Suffix::FIELD) s += "." + x.name;
        else if (x.kind == Suffix::METHOD) {
          s += "." + x.name + "(";
          for (size_t i = 0; i < x.args.size(); ++i) s += (i ? ", " : "") + expr_text(x.args[i]);
          s += ")";
        } else s += "[" + expr_text(x.index) + "]";
      }
      return s;
    }
    case Expr::JSON: return "{json}";
    case Expr::ARRAY: return "[array]";
    case Expr::OR:
    case Expr::AND: {
      std::string s = "(";
      for (size_t i = 0; i < e->kids.size(); ++i)
        s += (i ? (e->kind == Expr::OR ? " or " : " and ") : "") + expr_text(e->kids[i]);
      return s + ")";
    }
    case Expr::NOT: return "not " + expr_text(e->kids[0]);
    case Expr::CMP: return expr_text(e->kids[0]) + " " + e->name + " " + expr_text(e->kids[1]);
    case Expr::TRUTH: return expr_text(e->kids[0]);
    case Expr::RID: return e->name;
  }
  return "";
}

std::unique_ptr<Statement> parse_statement(const std::string &text) { return Parser(text).statement(); }

}  // namespace omx
