"""ORACLE (test infrastructure only) — a faithful CPU restatement of OrientDB 2.2.8 SQL MATCH.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only
as the checker. The product path (orientdb_amd/) never imports it.

Everything below restates the reference's behaviour, read as text from /root/reference (the Java
reference cannot be built or run here: no JVM, SURVEY.md §0 finding 5). Path prefixes:
  P/  = core/src/main/java/com/orientechnologies/orient/core/sql/parser/
  C/  = core/src/main/java/com/orientechnologies/orient/core/
  GF/ = graphdb/src/main/java/com/orientechnologies/orient/graph/sql/functions/
  B/  = graphdb/src/main/java/com/tinkerpop/blueprints/impls/orient/

Pinned by: every known-answer assertion of
graphdb/src/test/java/com/orientechnologies/orient/graph/sql/OMatchStatementExecutionTest.java
(tests/test_oracle_known_answers.py), on the graph restated in tests/golden/make_match_test_db.py.

Parts:
  * RefDB         — records, classes (polymorphic counts), per-vertex ridbags out_<E>/in_<E> of edge
                    records in insertion order (C/db/record/ridbag/embedded/OEmbeddedRidBag.java:46).
  * parse()       — MATCH grammar subset (core/src/main/grammar/OrientSQL.jjt:1138-1170,3277-3560):
                    {class,as,where,while,maxDepth,optional}, .out/.in/.both/.outE/.inE/.bothE/.outV/
                    .inV/.bothV(labels), arrows -L-> <-L- -L-, multi-items .( ... ), RETURN items
                    (aliases, expressions, $matches/$patterns/$paths/$elements/$pathElements, JSON), LIMIT.
  * MatchOracle   — OMatchStatement.parse (:129-218, :905-948), execute (:244-267), estimateRootEntries
                    (:874-903), sortEdges (:272-325), calculateMatch (:334-386), processContext
                    (:412-568), expandCartesianProduct (:620-650), addResult/addSingleResult (:661-750).
"""
from __future__ import annotations

import json
import re
from collections import OrderedDict

# ----------------------------------------------------------------------------------------------------
# database model
# ----------------------------------------------------------------------------------------------------


class Record:
    """A vertex or edge record. Identity = RID (C/id/ORecordId.java:158-160)."""

    __slots__ = ("rid", "cls", "props", "is_edge", "out_v", "in_v", "bags", "idx")

    def __init__(self, rid, cls, props, is_edge=False):
        self.rid = rid
        self.cls = cls
        self.props = props
        self.is_edge = is_edge
        self.out_v = None
        self.in_v = None
        self.bags = {}  # field name (out_X / in_X) -> list of edge records, insertion order
        self.idx = -1  # dense index among vertices (vertices only)

    def __hash__(self):
        return hash(self.rid)

    def __eq__(self, other):
        return isinstance(other, Record) and other.rid == self.rid

    def __repr__(self):
        return "#%d:%d" % self.rid


class OracleError(Exception):
    """OCommandExecutionException / NullPointerException raised by the reference."""


class RefDB:
    """In-memory database holding what the MATCH path reads."""

    def __init__(self):
        self.classes = OrderedDict()  # name -> dict(superclass, is_edge, cluster)
        self.records = []
        self.vertices = []
        self.by_class = {}  # exact class -> list of records
        self.indexes = []  # (class, property, unique)
        self._next_cluster = 11

    # schema -----------------------------------------------------------------------------------------
    def create_class(self, name, superclass=None, is_edge=False, cluster=None):
        if cluster is None:
            cluster = self._next_cluster
        self.classes[name] = {"superclass": superclass, "is_edge": is_edge, "cluster": cluster}
        self._next_cluster = max(self._next_cluster, cluster) + 1
        self.by_class[name] = []

    def class_name(self, name):
        """Schema class lookup is case-insensitive (OSchemaShared.getClass)."""
        if name in self.classes:
            return name
        for c in self.classes:
            if c.lower() == name.lower():
                return c
        return None

    def is_subclass_of(self, c, sup):
        """OClassImpl.isSubClassOf: c == sup or sup is an ancestor of c."""
        while c is not None:
            if c == sup:
                return True
            c = self.classes[c]["superclass"]
        return False

    def subclasses(self, c):
        return [x for x in self.classes if self.is_subclass_of(x, c)]

    def count(self, c):
        """OClassImpl.count() = polymorphic count (C/metadata/schema/OClassImpl.java:1485-1499)."""
        return sum(len(self.by_class[x]) for x in self.subclasses(c))

    def browse(self, c):
        out = []
        for x in self.subclasses(c):
            out.extend(self.by_class[x])
        return out

    # data -------------------------------------------------------------------------------------------
    def add_vertex(self, cls, props):
        r = Record((self.classes[cls]["cluster"], len(self.by_class[cls])), cls, dict(props))
        r.idx = len(self.vertices)
        self.records.append(r)
        self.vertices.append(r)
        self.by_class[cls].append(r)
        return r

    def add_edge(self, cls, out_v, in_v, props=None):
        """Regular (heavyweight) edge: an edge record linked from out_<cls> of out_v and in_<cls> of in_v
        (B/OrientVertex.java:109-180, createLink), with its own fields."""
        e = Record((self.classes[cls]["cluster"], len(self.by_class[cls])), cls, dict(props or {}), is_edge=True)
        e.out_v, e.in_v = out_v, in_v
        self.records.append(e)
        self.by_class[cls].append(e)
        out_v.bags.setdefault("out_" + cls, []).append(e)
        in_v.bags.setdefault("in_" + cls, []).append(e)
        return e

    @staticmethod
    def from_json(obj):
        if isinstance(obj, str):
            with open(obj) as f:
                obj = json.load(f)
        db = RefDB()
        for c in obj["classes"]:
            db.create_class(c["name"], c["superclass"], c["is_edge"])
        for v in obj["vertices"]:
            db.add_vertex(v["class"], v["props"])
        for e in obj["edges"]:
            db.add_edge(e["class"], db.vertices[e["out"]], db.vertices[e["in"]], e.get("props"))
        for ix in obj.get("indexes", []):
            db.indexes.append((ix["class"], ix["property"], bool(ix["unique"])))
        return db

    # graph functions ----------------------------------------------------------------------------------
    def field_names(self, direction, labels):
        """OrientVertex.getFieldNames (B/OrientVertex.java:1035-1088): a single label 'E' or no label
        means every edge field; otherwise the label classes and all their subclasses."""
        if labels is not None and len(labels) == 1 and labels[0].lower() == "e":
            labels = None
        if labels is None or len(labels) == 0:
            return None
        names = []
        for lab in labels:
            c = self.class_name(lab)
            cands = [lab] if c is None else [c] + [s for s in self.subclasses(c) if s != c]
            for x in cands:
                if x not in names:
                    names.append(x)
        out = []
        for x in names:
            if direction in ("out", "both"):
                out.append("out_" + x)
            if direction in ("in", "both"):
                out.append("in_" + x)
        return out

    def connections(self, v, direction, labels):
        """Edge records of v (OrientVertex.getEdges / getVertices iteration over the ridbag fields)."""
        names = self.field_names(direction, labels)
        res = []
        if names is None:
            for f in v.bags:
                if (direction in ("out", "both") and f.startswith("out_")) or (
                        direction in ("in", "both") and f.startswith("in_")):
                    res.extend((f, e) for e in v.bags[f])
        else:
            for f in names:
                for e in v.bags.get(f, []):
                    res.append((f, e))
        return res

    def move(self, rec, fn, labels):
        """out/in/both/outE/inE/bothE/outV/inV/bothV on one record (GF/OSQLFunctionMove.java:66-144)."""
        fn = fn.lower()
        if rec is None:
            return []
        if rec.is_edge:
            if fn == "outv":
                return [rec.out_v]
            if fn == "inv":
                return [rec.in_v]
            if fn == "bothv":
                return [rec.out_v, rec.in_v]
            return []
        if fn in ("out", "in", "both"):
            res = []
            for f, e in self.connections(rec, fn, labels):
                res.append(e.in_v if f.startswith("out_") else e.out_v)
            return res
        if fn in ("oute", "ine", "bothe"):
            d = fn[:-1]
            return [e for f, e in self.connections(rec, d, labels)]
        return []


# ----------------------------------------------------------------------------------------------------
# parser (restates the MATCH part of core/src/main/grammar/OrientSQL.jjt)
# ----------------------------------------------------------------------------------------------------


class ParseError(Exception):
    """OCommandSQLParsingException."""


class MatchFilter:
    def __init__(self):
        self.alias = None
        self.class_name = None
        self.where = None
        self.while_ = None
        self.max_depth = None
        self.optional = False


class PathItem:
    def __init__(self, method, labels, flt, multi=None):
        self.method = method  # 'out', 'in', 'both', 'outE', ... or None for multi
        self.labels = labels  # list of label strings or None
        self.filter = flt
        self.multi = multi  # list[PathItem] for .( ... )

    def is_bidirectional(self):
        """OMatchPathItem.isBidirectional (P/OMatchPathItem.java:29-40), OMethodCall.isBidirectional
        (P/OMethodCall.java:21,56-58); multi items are never bidirectional (P/OMultiMatchPathItem.java)."""
        if self.multi is not None:
            return False
        if self.filter.while_ is not None or self.filter.max_depth is not None or self.filter.optional:
            return False
        return self.method.lower() in ("out", "in", "both", "oute", "ine", "inv", "outv")


class MatchExpression:
    def __init__(self, origin, items):
        self.origin = origin
        self.items = items


class Statement:
    def __init__(self):
        self.expressions = []
        self.return_items = []  # list of (expr, alias or None, text)
        self.limit = None


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>\d+\.\d+|\d+)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<id>[$@]?[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op><>|!=|<=|>=|==|->|<-|--|[-+*/%=<>{}()\[\],:.?])
""", re.X)


def _tokenize(text):
    toks = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            raise ParseError("unexpected character at %d: %r" % (pos, text[pos:pos + 10]))
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        val = m.group(kind)
        if kind == "str":
            val = val[1:-1].replace("\\'", "'").replace('\\"', '"')
        toks.append((kind, val))
    toks.append(("eof", None))
    return toks


class _Parser:
    def __init__(self, text):
        self.toks = _tokenize(text)
        self.i = 0
        self.nparam = 0

    # token helpers
    def peek(self, k=0):
        return self.toks[self.i + k]

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def at(self, val, k=0):
        t = self.toks[self.i + k]
        return t[0] in ("op",) and t[1] == val

    def at_kw(self, kw, k=0):
        t = self.toks[self.i + k]
        return t[0] == "id" and t[1].lower() == kw

    def expect(self, val):
        t = self.next()
        if t[1] != val:
            raise ParseError("expected %r, got %r" % (val, t[1]))
        return t

    # statement
    def statement(self):
        if not self.at_kw("match"):
            raise ParseError("MATCH expected")
        self.next()
        st = Statement()
        st.expressions.append(self.match_expression())
        while self.at(","):
            self.next()
            st.expressions.append(self.match_expression())
        if not self.at_kw("return"):
            raise ParseError("RETURN expected")
        self.next()
        while True:
            start = self.i
            e = self.expr()
            text = " ".join(str(t[1]) for t in self.toks[start:self.i])
            alias = None
            if self.at_kw("as"):
                self.next()
                alias = self.next()[1]
            st.return_items.append((e, alias, text))
            if self.at(","):
                self.next()
                continue
            break
        if self.at_kw("limit"):
            self.next()
            neg = False
            if self.at("-"):
                self.next()
                neg = True
            t = self.next()
            if t[0] != "num":
                raise ParseError("LIMIT expects a number")
            st.limit = -int(t[1]) if neg else int(t[1])
        if self.peek()[0] != "eof":
            raise ParseError("unexpected token %r" % (self.peek()[1],))
        return st

    def match_expression(self):
        origin = self.match_filter()
        items = []
        while True:
            if self.at("."):
                items.append(self.method_item())
            elif self.at("-") or self.at("<-") or self.at("--"):
                items.append(self.arrow_item())
            else:
                break
        return MatchExpression(origin, items)

    def match_filter(self):
        self.expect("{")
        f = MatchFilter()
        first = True
        while not self.at("}"):
            if not first:
                self.expect(",")
            first = False
            key = self.next()[1].lower()
            self.expect(":")
            if key == "class":
                t = self.next()
                f.class_name = t[1]
            elif key == "as":
                f.alias = self.next()[1]
            elif key == "where":
                self.expect("(")
                f.where = self.or_expr()
                self.expect(")")
            elif key == "while":
                self.expect("(")
                f.while_ = self.or_expr()
                self.expect(")")
            elif key == "maxdepth":
                f.max_depth = int(self.next()[1])
            elif key == "optional":
                f.optional = self.next()[1].lower() == "true"
            else:
                raise ParseError("unknown match filter item %r" % key)
        self.expect("}")
        return f

    def labels(self):
        self.expect("(")
        labs = []
        while not self.at(")"):
            t = self.next()
            if t[0] not in ("str", "id"):
                raise ParseError("label expected")
            labs.append(t[1])
            if self.at(","):
                self.next()
        self.expect(")")
        return labs if labs else None

    def method_item(self):
        self.expect(".")
        if self.at("("):
            self.next()
            subs = []
            while not self.at(")"):
                if self.at("."):
                    subs.append(self.method_item())
                elif self.peek()[0] == "id":
                    # OMatchPathItemFirst: the first item of a multi path may be a bare function call
                    # (P/OMatchPathItemFirst.java:35-39)
                    name = self.next()[1]
                    labs = self.labels()
                    flt = self.match_filter() if self.at("{") else MatchFilter()
                    subs.append(PathItem(name, labs, flt))
                else:
                    subs.append(self.arrow_item())
            self.expect(")")
            flt = self.match_filter() if self.at("{") else MatchFilter()
            return PathItem(None, None, flt, multi=subs)
        name = self.next()[1]
        labs = self.labels()
        flt = self.match_filter() if self.at("{") else MatchFilter()
        return PathItem(name, labs, flt)

    def arrow_item(self):
        """-L-> = .out('L'), <-L- = .in('L'), -L- = .both('L'); bare arrows mean any label
        (OrientSQL.jjt:3438-3467)."""
        if self.at("--"):  # "--" then "{" (both, no label) or "-->"(tokenized as -- >)
            self.next()
            if self.at(">"):
                self.next()
                method, labs = "out", None
            else:
                method, labs = "both", None
        elif self.at("<-"):
            self.next()
            labs = None
            if self.at("-"):
                self.next()
            elif self.at("--"):
                raise ParseError("bad arrow")
            else:
                labs = [self.next()[1]]
                self.expect("-")
            method = "in"
        else:
            self.expect("-")
            labs = None
            if self.at("->"):
                self.next()
                method = "out"
            elif self.at("-"):
                self.next()
                method = "both"
            else:
                labs = [self.next()[1]]
                if self.at("->"):
                    self.next()
                    method = "out"
                else:
                    self.expect("-")
                    method = "both"
        flt = self.match_filter()
        return PathItem(method, labs, flt)

    # boolean / value expressions
    def or_expr(self):
        parts = [self.and_expr()]
        while self.at_kw("or"):
            self.next()
            parts.append(self.and_expr())
        return parts[0] if len(parts) == 1 else ("or", parts)

    def and_expr(self):
        parts = [self.not_expr()]
        while self.at_kw("and"):
            self.next()
            parts.append(self.not_expr())
        return parts[0] if len(parts) == 1 else ("and", parts)

    def not_expr(self):
        if self.at_kw("not"):
            self.next()
            return ("not", self.not_expr())
        return self.cmp_expr()

    def cmp_expr(self):
        left = self.expr()
        t = self.peek()
        if t[0] == "op" and t[1] in ("=", "==", "!=", "<>", "<", "<=", ">", ">="):
            self.next()
            right = self.expr()
            return ("cmp", t[1], left, right)
        return ("truth", left)

    def expr(self):
        left = self.term()
        while self.at("+") or self.at("-"):
            op = self.next()[1]
            left = ("math", op, left, self.term())
        return left

    def term(self):
        left = self.unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = self.next()[1]
            left = ("math", op, left, self.unary())
        return left

    def unary(self):
        if self.at("-"):
            self.next()
            return ("math", "-", ("lit", 0), self.unary())
        return self.postfix()

    def postfix(self):
        base = self.primary()
        suffixes = []
        while True:
            if self.at("."):
                self.next()
                name = self.next()[1]
                if self.at("("):
                    suffixes.append(("method", name, self.call_args()))
                else:
                    suffixes.append(("field", name))
            elif self.at("["):
                self.next()
                if self.peek()[0] == "num" and self.at("-", 1) and self.peek(2)[0] == "num" and self.at("]", 3):
                    lo = int(self.next()[1])
                    self.next()
                    hi = int(self.next()[1])
                    self.expect("]")
                    suffixes.append(("index", ("range", ("lit", lo), ("lit", hi))))
                    continue
                sel = self.or_expr()
                if self.at("-"):
                    self.next()
                    sel = ("range", sel, self.expr())
                elif self.at(","):
                    items = [sel]
                    while self.at(","):
                        self.next()
                        items.append(self.expr())
                    sel = ("multi", items)
                self.expect("]")
                suffixes.append(("index", sel))
            else:
                break
        return base if not suffixes else ("chain", base, suffixes)

    def call_args(self):
        self.expect("(")
        args = []
        while not self.at(")"):
            args.append(self.expr())
            if self.at(","):
                self.next()
        self.expect(")")
        return args

    def primary(self):
        t = self.next()
        kind, val = t
        if kind == "num":
            return ("lit", float(val) if "." in val else int(val))
        if kind == "str":
            return ("lit", val)
        if kind == "op" and val == "(":
            e = self.or_expr()
            self.expect(")")
            if e[0] == "truth":  # a parenthesised value, not a condition
                return ("paren", e[1])
            return ("paren", e)
        if kind == "op" and val == "?":
            p = ("param", self.nparam)
            self.nparam += 1
            return p
        if kind == "op" and val == ":":
            return ("param", self.next()[1])
        if kind == "op" and val == "{":
            return self.json_body()
        if kind == "op" and val == "[":
            items = []
            while not self.at("]"):
                items.append(self.expr())
                if self.at(","):
                    self.next()
            self.expect("]")
            return ("array", items)
        if kind == "id":
            low = val.lower()
            if low in ("true", "false"):
                return ("lit", low == "true")
            if low == "null":
                return ("lit", None)
            if self.at("("):
                return ("call", val, self.call_args())
            if val.startswith("$"):
                return ("var", val)
            return ("field", val)
        raise ParseError("unexpected token %r" % (val,))

    def json_body(self):
        pairs = []
        while not self.at("}"):
            k = self.next()
            self.expect(":")
            pairs.append((k[1], self.expr()))
            if self.at(","):
                self.next()
        self.expect("}")
        return ("json", pairs)


def parse(text):
    return _Parser(text).statement()


# ----------------------------------------------------------------------------------------------------
# expression evaluation (P/OWhereClause.java:36-41, P/OBinaryCondition.java:34-36, operators)
# ----------------------------------------------------------------------------------------------------

def _num(x):
    return isinstance(x, (int, float)) and not isinstance(x, bool)


def _equals(a, b):
    """OQueryOperatorEquals.equals (S/operator/OQueryOperatorEquals.java:67-97)."""
    if a is None or b is None:
        return False
    if isinstance(a, Record) or isinstance(b, Record):
        return isinstance(a, Record) and isinstance(b, Record) and a.rid == b.rid
    if _num(a) and _num(b):
        return a == b
    if isinstance(a, str) and _num(b):
        try:
            return type(b)(a) == b
        except ValueError:
            return False
    if _num(a) and isinstance(b, str):
        try:
            return a == type(a)(b)
        except ValueError:
            return False
    return a == b


def _compare(op, a, b):
    """OGtOperator/OGeOperator/OLeOperator throw NPE on a null left operand, OLtOperator returns false
    (P/OGtOperator.java:22-33, P/OLtOperator.java:22-36, P/OGeOperator.java:43-54, P/OLeOperator.java:22-33).
    With a non-null left operand, all four evaluate `iLeft.getClass() != iRight.getClass()` first, so a
    null right operand is a NullPointerException too (the `iRight == null` test after OType.convert is
    never reached with a null)."""
    if a is None:
        if op == "<":
            return False
        raise OracleError("NullPointerException: null left operand of %s" % op)
    if b is None:
        raise OracleError("NullPointerException: null right operand of %s" % op)
    if _num(a) and _num(b):
        pass
    elif isinstance(a, str) and _num(b):
        try:
            b = str(b)
        except Exception:
            return False
    elif _num(a) and isinstance(b, str):
        try:
            b = type(a)(b)
        except ValueError:
            return False
    elif type(a) != type(b):
        return False
    if op == "<":
        return a < b
    if op == "<=":
        return a <= b
    if op == ">":
        return a > b
    return a >= b


class Ctx:
    """OBasicCommandContext variables ($matched, $currentMatch, $depth, $current) and parameters."""

    def __init__(self, params=None):
        self.vars = {}
        self.params = params or {}


class Evaluator:
    def __init__(self, db, ctx):
        self.db = db
        self.ctx = ctx

    def matches(self, cond, rec):
        if cond is None:
            return True
        return bool(self.boolean(cond, rec))

    def boolean(self, c, rec):
        k = c[0]
        if k == "or":
            return any(self.boolean(x, rec) for x in c[1])
        if k == "and":
            return all(self.boolean(x, rec) for x in c[1])
        if k == "not":
            return not self.boolean(c[1], rec)
        if k == "paren":
            return self.boolean(c[1], rec)
        if k == "cmp":
            op, l, r = c[1], self.value(c[2], rec), self.value(c[3], rec)
            if op in ("=", "=="):
                return _equals(l, r)
            if op in ("!=", "<>"):
                return not _equals(l, r)
            return _compare(op, l, r)
        if k == "truth":
            v = self.value(c[1], rec)
            return v is True
        raise OracleError("bad condition %r" % (c,))

    def field(self, base, name):
        if base is None:
            return None
        if isinstance(base, Record):
            if name.lower() == "@rid":
                return base
            if name.lower() == "@class":
                return base.cls
            if base.is_edge and name in ("out", "in"):
                return base.out_v if name == "out" else base.in_v
            return base.props.get(name)
        if isinstance(base, dict):
            return base.get(name)
        if isinstance(base, list):
            return [self.field(x, name) for x in base]
        return None

    def value(self, e, rec):
        k = e[0]
        if k == "lit":
            return e[1]
        if k == "paren":
            return self.value(e[1], rec)
        if k in ("or", "and", "not", "cmp", "truth"):
            return self.boolean(e, rec)
        if k == "param":
            return self.ctx.params[e[1]]
        if k == "var":
            name = e[1]
            return self.ctx.vars.get(name)
        if k == "field":
            # OSuffixIdentifier.execute: a context variable of the same name shadows the field
            # (P/OSuffixIdentifier.java:40-58)
            if e[1] in self.ctx.vars:
                return self.ctx.vars[e[1]]
            return self.field(rec, e[1])
        if k == "math":
            a, b = self.value(e[2], rec), self.value(e[3], rec)
            op = e[1]
            if op == "+":
                if isinstance(a, str) or isinstance(b, str):
                    return ("" if a is None else str(a)) + ("" if b is None else str(b))
                if a is None or b is None:
                    return None
                return a + b
            if a is None or b is None:
                return None
            if op == "-":
                return a - b
            if op == "*":
                return a * b
            # Java arithmetic (P/OMathExpression.java:105-147): integer / truncates toward zero and % takes
            # the dividend's sign (Python's // and % floor); a double % is fmod
            if op == "/":
                if isinstance(a, int) and isinstance(b, int):
                    q = abs(a) // abs(b)
                    return -q if (a < 0) != (b < 0) else q
                return a / b
            if op == "%":
                if isinstance(a, int) and isinstance(b, int):
                    r = abs(a) % abs(b)
                    return -r if a < 0 else r
                import math
                return math.fmod(a, b)
        if k == "call":
            return self.call(e[1], e[2], rec, rec)
        if k == "chain":
            cur = self.value(e[1], rec) if e[1][0] != "call" else self.call(e[1][1], e[1][2], rec, rec)
            for s in e[2]:
                cur = self.suffix(cur, s, rec)
            return cur
        if k == "json":
            return {key: self.value(x, rec) for key, x in e[1]}
        if k == "array":
            return [self.value(x, rec) for x in e[1]]
        raise OracleError("bad expression %r" % (e,))

    def call(self, name, args, target, rec):
        low = name.lower()
        if low in ("out", "in", "both", "oute", "ine", "bothe", "outv", "inv", "bothv"):
            labs = [self.value(a, rec) for a in args] or None
            if isinstance(target, list):
                res = []
                for t in target:
                    res.extend(self.db.move(t, low, labs))
                return res
            return self.db.move(target, low, labs)
        raise OracleError("unsupported function %s" % name)

    def suffix(self, cur, s, rec):
        if s[0] == "field":
            return self.field(cur, s[1])
        if s[0] == "method":
            name = s[1].lower()
            if name in ("out", "in", "both", "oute", "ine", "bothe", "outv", "inv", "bothv"):
                return self.call(name, s[2], cur, rec)
            if name == "size":
                if cur is None:
                    return 0
                return len(cur) if isinstance(cur, (list, tuple, set, str)) else 1
            if name == "touppercase":
                return None if cur is None else str(cur).upper()
            if name == "tolowercase":
                return None if cur is None else str(cur).lower()
            raise OracleError("unsupported method %s" % name)
        if s[0] == "index":
            sel = s[1]
            lst = cur if isinstance(cur, list) else [cur]
            if sel[0] == "range":
                a, b = self.value(sel[1], rec), self.value(sel[2], rec)
                return lst[a:b]
            if sel[0] == "multi":
                return [lst[self.value(x, rec)] for x in sel[1] if self.value(x, rec) < len(lst)]
            if sel[0] in ("cmp", "or", "and", "not"):
                return [x for x in lst if self.boolean(sel, x)]
            i = self.value(sel, rec)
            return lst[i] if isinstance(i, int) and 0 <= i < len(lst) else None
        raise OracleError("bad suffix")


# ----------------------------------------------------------------------------------------------------
# the MATCH engine (P/OMatchStatement.java)
# ----------------------------------------------------------------------------------------------------

DEFAULT_ALIAS_PREFIX = "$ORIENT_DEFAULT_ALIAS_"
THRESHOLD = 20  # OMatchStatement.threshold (:35)


class PatternNode:
    def __init__(self, alias):
        self.alias = alias
        self.out = []  # PatternEdge, insertion ordered (LinkedHashSet)
        self.in_ = []
        self.optional = False


class PatternEdge:
    def __init__(self, item, out_node, in_node):
        self.item = item
        self.out = out_node
        self.in_ = in_node


class MatchContext:
    """OMatchStatement.MatchContext (:38-65)."""

    def __init__(self):
        self.current_edge = 0
        self.candidates = OrderedDict()
        self.matched = OrderedDict()
        self.matched_edges = set()

    def copy(self, alias, value):
        r = MatchContext()
        r.candidates = OrderedDict(self.candidates)
        r.candidates.pop(alias, None)
        r.matched = OrderedDict(self.matched)
        r.matched[alias] = value
        r.matched_edges = set(self.matched_edges)
        r.current_edge = self.current_edge
        return r


class _LimitReached(Exception):
    pass


class MatchOracle:
    """One parsed MATCH statement bound to a RefDB."""

    def __init__(self, db, text):
        self.db = db
        self.text = text
        self.st = parse(text)
        self._assign_default_aliases()
        self.nodes = OrderedDict()
        self.edges = []
        for ex in self.st.expressions:
            self._add_expression(ex)
        self.alias_filters = OrderedDict()
        self.alias_classes = OrderedDict()
        for ex in self.st.expressions:
            self._add_aliases(ex.origin)
            for it in ex.items:
                self._add_aliases(it.filter)
        self._rebind_filters()
        self._validate()

    # parse-time (OMatchStatement.parse :129-178) -------------------------------------------------
    def _assign_default_aliases(self):
        counter = 0
        for ex in self.st.expressions:
            if ex.origin.alias is None:
                ex.origin.alias = DEFAULT_ALIAS_PREFIX + str(counter)
                counter += 1
            for it in ex.items:
                if it.filter.alias is None:
                    it.filter.alias = DEFAULT_ALIAS_PREFIX + str(counter)
                    counter += 1

    def _node(self, flt):
        n = self.nodes.get(flt.alias)
        if n is None:
            n = PatternNode(flt.alias)
            self.nodes[flt.alias] = n
        if flt.optional:
            n.optional = True
        return n

    def _add_expression(self, ex):
        """Pattern.addExpression (P/Pattern.java:15-27)."""
        origin = self._node(ex.origin)
        for it in ex.items:
            nxt = self._node(it.filter)
            e = PatternEdge(it, origin, nxt)
            origin.out.append(e)
            nxt.in_.append(e)
            self.edges.append(e)
            origin = nxt

    def _add_aliases(self, flt):
        """addAliases (:905-948): AND of every where fragment of an alias, lowest subclass."""
        alias = flt.alias
        if flt.where is not None:
            self.alias_filters.setdefault(alias, [])
            self.alias_filters[alias].append(flt.where)
        if flt.class_name is not None:
            prev = self.alias_classes.get(alias)
            if prev is None:
                self.alias_classes[alias] = flt.class_name
            else:
                a, b = self.db.class_name(flt.class_name), self.db.class_name(prev)
                if a is not None and b is not None and self.db.is_subclass_of(a, b):
                    self.alias_classes[alias] = flt.class_name
                elif a is not None and b is not None and self.db.is_subclass_of(b, a):
                    self.alias_classes[alias] = prev
                else:
                    raise OracleError("classes defined for alias %s (%s, %s) are not in the same hierarchy"
                                      % (alias, flt.class_name, prev))

    def where_of(self, alias):
        w = self.alias_filters.get(alias)
        if not w:
            return None
        return ("and", list(w))

    def _rebind_filters(self):
        """rebindFilters (:185-195): every filter of an alias evaluates the merged WHERE."""
        for ex in self.st.expressions:
            ex.origin.where = self.where_of(ex.origin.alias)
            for it in ex.items:
                it.filter.where = self.where_of(it.filter.alias)

    def _validate(self):
        """Pattern.validate (P/Pattern.java:48-65)."""
        for n in self.nodes.values():
            if n.optional:
                if n.out:
                    raise ParseError("optional nodes are allowed only on right terminal nodes")
                if not n.in_:
                    raise ParseError("optional nodes must have at least one incoming pattern edge")

    # planning ----------------------------------------------------------------------------------------
    def _flatten(self, c):
        """OBooleanExpression.flatten: disjunctive normal form as a list of AND blocks (lists)."""
        k = c[0]
        if k == "paren" and c[1][0] in ("or", "and", "not", "cmp", "truth"):
            return self._flatten(c[1])
        if k == "or":
            out = []
            for x in c[1]:
                out.extend(self._flatten(x))
            return out
        if k == "and":
            blocks = [[]]
            for x in c[1]:
                fx = self._flatten(x)
                blocks = [b + f for b in blocks for f in fx]
            return blocks
        return [[c]]

    def _estimate(self, cls, where, ctx):
        """OWhereClause.estimate (P/OWhereClause.java:57-95)."""
        count = self.db.count(cls)
        if count > 1:
            count //= 2
        if count < THRESHOLD:
            return count
        indexes = [(p, u) for (c, p, u) in self.db.indexes if self.db.is_subclass_of(cls, c)]
        total = 0
        for block in self._flatten(where):
            conds = {}
            for b in block:
                if b[0] == "cmp" and b[1] in ("=", "==") and b[2][0] == "field" and b[3][0] in ("lit", "param"):
                    conds[b[2][1]] = b[3][1] if b[3][0] == "lit" else ctx.params[b[3][1]]
            est = None
            for (p, unique) in indexes:
                if p in conds:
                    key = conds[p]
                    hits = [r for r in self.db.browse(cls) if _equals(r.props.get(p), key)]
                    if unique:
                        n = 1 if hits else None
                    else:
                        n = len(hits)
                    if n is not None and (est is None or n < est):
                        est = n
            if est is None or est > count:
                return count
            total += est
        return min(total, count)

    def estimate_root_entries(self, ctx):
        """estimateRootEntries (:874-903)."""
        aliases = list(self.alias_classes.keys()) + [a for a in self.alias_filters if a not in self.alias_classes]
        res = OrderedDict()
        for alias in aliases:
            cname = self.alias_classes.get(alias)
            if cname is None:
                continue
            c = self.db.class_name(cname)
            if c is None:
                raise OracleError("class not defined: " + cname)
            where = self.where_of(alias)
            res[alias] = self._estimate(c, where, ctx) if where is not None else self.db.count(c)
        return res

    def sort_edges(self, estimates):
        """sortEdges (:272-325): BFS over the pattern from the cheapest non-optional root, stable sort
        by estimate only (CM/util/OPair.java:97-99)."""
        weights = sorted(estimates.items(), key=lambda kv: kv[1])
        result = []
        traversed_edges = set()
        traversed_nodes = set()
        next_nodes = []
        while len(result) < len(self.edges):
            for alias, _ in weights:
                root = self.nodes[alias]
                if root.optional:
                    continue
                if alias not in traversed_nodes:
                    next_nodes.append(root)
                    break
            if not next_nodes:
                break
            while next_nodes:
                node = next_nodes.pop(0)
                traversed_nodes.add(node.alias)
                for e in node.out:
                    if id(e) not in traversed_edges:
                        result.append((e, True))
                        traversed_edges.add(id(e))
                        if e.in_.alias not in traversed_nodes and e.in_ not in next_nodes:
                            next_nodes.append(e.in_)
                for e in node.in_:
                    if id(e) not in traversed_edges and e.item.is_bidirectional():
                        result.append((e, False))
                        traversed_edges.add(id(e))
                        if e.out.alias not in traversed_nodes and e.out not in next_nodes:
                            next_nodes.append(e.out)
        return result

    def plan(self, params=None):
        """The execution plan (estimates, prefetched aliases, root, sorted edges) — compared with
        omx_statement_explain in the tests."""
        ctx = Ctx(self._param_map(params))
        est = self.estimate_root_entries(ctx)
        sorted_edges = self.sort_edges(est)
        pre = [a for a, v in est.items() if v < THRESHOLD]
        if not pre and est:
            pre = [self._next_alias(est, MatchContext())]
        if sorted_edges:
            e, fwd = sorted_edges[0]
            root = e.out.alias if fwd else e.in_.alias
        else:
            root = next(iter(self.nodes))
        return {
            "estimates": dict(est),
            "prefetched": pre,
            "root": root,
            "edges": [(e.out.alias, e.in_.alias, fwd) for e, fwd in sorted_edges],
        }

    # execution ---------------------------------------------------------------------------------------
    @staticmethod
    def _param_map(params):
        if params is None:
            return {}
        if isinstance(params, dict):
            return dict(params)
        return {i: v for i, v in enumerate(params)}

    def _query(self, alias, ctx):
        """fetchAliasCandidates → query (:401-410, :815-840): (select from Class where <where>)."""
        c = self.db.class_name(self.alias_classes[alias])
        where = self.where_of(alias)
        ev = Evaluator(self.db, Ctx(ctx.params))
        out = []
        for r in self.db.browse(c):
            try:
                ok = ev.matches(where, r)
            except OracleError:
                ok = False  # legacy SELECT operators compare null as false
            if ok:
                out.append(r)
        return out

    @staticmethod
    def _next_alias(est, mctx):
        """getNextAlias (:858-872)."""
        lower = None
        for alias, v in est.items():
            if alias in mctx.matched:
                continue
            if lower is None or lower[1] > v:
                lower = (alias, v)
        return lower[0]

    def execute(self, params=None, limit=None, stats=None):
        """OMatchStatement.execute (:244-267). Returns the list of result documents (dicts) or records,
        in emission order, de-duplicated by content. `limit` is limitFromProtocol (setLimit)."""
        self.ctx = Ctx(self._param_map(params))
        self.ev = Evaluator(self.db, self.ctx)
        self.results = []
        self.unique = set()
        self.limit_protocol = -1 if limit is None else limit
        self.stats = stats if stats is not None else {}
        self.stats.setdefault("bindings", 0)
        est = self.estimate_root_entries(self.ctx)
        if 0 in est.values():
            return []
        self.sorted_edges = self.sort_edges(est)
        try:
            self._calculate_match(est, MatchContext())
        except _LimitReached:
            pass
        return self.results

    def _calculate_match(self, est, mctx):
        """calculateMatch (:334-386)."""
        root_found = False
        for alias, v in est.items():
            if v < THRESHOLD:
                matches = self._query(alias, self.ctx)
                if not matches:
                    if self.nodes[alias].optional:
                        continue
                    return
                mctx.candidates[alias] = matches
                root_found = True
        if not root_found:
            alias = self._next_alias(est, mctx)
            matches = self._query(alias, self.ctx)
            if not matches:
                return
            mctx.candidates[alias] = matches
        if self.sorted_edges:
            e, fwd = self.sorted_edges[0]
            smallest = e.out.alias if fwd else e.in_.alias
        else:
            smallest = next(iter(self.nodes))
        cands = mctx.candidates.get(smallest)
        if cands is None:
            raise OracleError("NullPointerException: no candidates for root alias " + smallest)
        self._from_candidates(mctx, cands, smallest, 0)

    def _from_candidates(self, mctx, cands, alias, start_edge):
        """processContextFromCandidates (:388-399)."""
        for r in list(cands):
            child = mctx.copy(alias, r)
            child.current_edge = start_edge
            self._process(child)

    def _all_nodes_calculated(self, mctx):
        return all(a in mctx.matched for a in self.nodes)

    def _traverse_edge(self, item, mctx, start, depth):
        """OMatchPathItem.executeTraversal (P/OMatchPathItem.java:49-107); multi items restate
        OMultiMatchPathItem.traversePatternEdge (P/OMultiMatchPathItem.java:41-61)."""
        flt = item.filter
        where, while_, max_depth = flt.where, flt.while_, flt.max_depth
        ctx, ev = self.ctx, self.ev
        if while_ is None and max_depth is None:
            qr = self._traverse_pattern_edge(item, mctx, start)
            if where is None:
                return qr
            result = []
            seen = set()
            for origin in qr:
                prev = ctx.vars.get("$currentMatch")
                ctx.vars["$currentMatch"] = origin
                if ev.matches(where, origin) and origin not in seen:
                    seen.add(origin)
                    result.append(origin)
                ctx.vars["$currentMatch"] = prev
            return result
        result = []
        seen = set()
        ctx.vars["$depth"] = depth
        prev = ctx.vars.get("$currentMatch")
        ctx.vars["$currentMatch"] = start
        if where is None or ev.matches(where, start):
            if start not in seen:
                seen.add(start)
                result.append(start)
        if (max_depth is None or depth < max_depth) and (while_ is None or ev.matches(while_, start)):
            qr = self._traverse_pattern_edge(item, mctx, start)
            for origin in qr:
                sub = self._traverse_edge(item, mctx, origin, depth + 1)
                for x in sub:
                    if x not in seen:
                        seen.add(x)
                        result.append(x)
        ctx.vars["$currentMatch"] = prev
        return result

    def _traverse_pattern_edge(self, item, mctx, start):
        """traversePatternEdge (P/OMatchPathItem.java:109-126): the method applied to one record; the
        possibleResults hint only matters for the supernode+edge-index shortcut
        (GF/OSQLFunctionOut.java:66-79), which returns the same records."""
        if item.multi is not None:
            result = [start]
            for sub in item.multi:
                nxt = []
                seen = set()
                for sp in result:
                    for x in self._traverse_edge(sub, mctx, sp, 0):
                        if x not in seen:
                            seen.add(x)
                            nxt.append(x)
                result = nxt
            return result
        res = self.db.move(start, item.method, item.labels)
        self.stats["edges"] = self.stats.get("edges", 0) + len(res)
        return res

    def _reverse(self, item, rec):
        """OMethodCall.executeReverse (P/OMethodCall.java:92-126)."""
        m = item.method.lower()
        rev = {"out": "in", "in": "out", "both": "both", "oute": "outv", "outv": "oute", "ine": "inv",
               "inv": "ine"}[m]
        res = self.db.move(rec, rev, item.labels)
        self.stats["edges"] = self.stats.get("edges", 0) + len(res)
        return res

    def _process(self, mctx):
        """processContext (:412-568)."""
        self.ctx.vars["$matched"] = mctx.matched
        if len(self.edges) == len(mctx.matched_edges) and self._all_nodes_calculated(mctx):
            self._add_result(mctx)
            return
        if len(self.sorted_edges) == mctx.current_edge:
            self._expand_cartesian(mctx)
            return
        edge, fwd = self.sorted_edges[mctx.current_edge]
        if fwd:
            if id(edge) in mctx.matched_edges:
                return
            start = mctx.matched.get(edge.out.alias)
            if start is None:
                right = mctx.candidates.get(edge.out.alias)
                if right is not None:
                    self._from_candidates(mctx, right, edge.out.alias, mctx.current_edge)
                return
            values = self._traverse_edge(edge.item, mctx, start, 0)
            tgt = edge.in_.alias
            if edge.in_.optional and (not [x for x in values if x is not None] or
                                      (mctx.matched.get(tgt) is not None and mctx.matched.get(tgt) not in values)):
                child = mctx.copy(tgt, None)
                child.current_edge = mctx.current_edge + 1
                child.matched_edges.add(id(edge))
                self._process(child)
            for rv in values:
                if rv is None:
                    continue
                prev = mctx.candidates.get(tgt)
                if tgt in mctx.matched:
                    bound = mctx.matched[tgt]
                    if bound is None:
                        raise OracleError("NullPointerException: optional alias re-bound")
                    if bound == rv:
                        child = mctx.copy(tgt, rv)
                        child.current_edge = mctx.current_edge + 1
                        child.matched_edges.add(id(edge))
                        self._process(child)
                        break
                elif prev:
                    for cid in prev:
                        if cid == rv:
                            child = mctx.copy(tgt, cid)
                            child.current_edge = mctx.current_edge + 1
                            child.matched_edges.add(id(edge))
                            self._process(child)
                else:
                    child = mctx.copy(tgt, rv)
                    child.current_edge = mctx.current_edge + 1
                    child.matched_edges.add(id(edge))
                    self._process(child)
        else:
            if id(edge) in mctx.matched_edges:
                return
            if not edge.item.is_bidirectional():
                raise OracleError("Invalid pattern to match!")
            values = self._reverse(edge.item, mctx.matched.get(edge.in_.alias))
            tgt = edge.out.alias
            if edge.out.optional and (not values or
                                      (mctx.matched.get(tgt) is not None and mctx.matched.get(tgt) not in values)):
                child = mctx.copy(tgt, None)
                child.current_edge = mctx.current_edge + 1
                child.matched_edges.add(id(edge))
                self._process(child)
            for lv in values:
                if lv is None:
                    continue
                prev = mctx.candidates.get(tgt)
                if tgt in mctx.matched:
                    bound = mctx.matched[tgt]
                    if bound is None:
                        raise OracleError("NullPointerException: optional alias re-bound")
                    if bound == lv:
                        child = mctx.copy(tgt, lv)
                        child.current_edge = mctx.current_edge + 1
                        child.matched_edges.add(id(edge))
                        self._process(child)
                        break
                elif prev:
                    for cid in prev:
                        if cid == lv:
                            child = mctx.copy(tgt, cid)
                            child.current_edge = mctx.current_edge + 1
                            child.matched_edges.add(id(edge))
                            self._process(child)
                else:
                    where = self.where_of(tgt)
                    if where is None or self.ev.matches(where, lv):
                        child = mctx.copy(tgt, lv)
                        child.current_edge = mctx.current_edge + 1
                        child.matched_edges.add(id(edge))
                        self._process(child)

    def _expand_cartesian(self, mctx):
        """expandCartesianProduct (:620-650)."""
        for alias in self.nodes:
            if alias not in mctx.matched:
                if alias not in self.alias_classes:
                    raise OracleError("Cannot execute MATCH statement on alias %s: class not defined" % alias)
                for r in self._query(alias, self.ctx):
                    child = mctx.copy(alias, r)
                    if self._all_nodes_calculated(child):
                        self._add_result(child)
                    else:
                        self._expand_cartesian(child)
                break

    # results -----------------------------------------------------------------------------------------
    def _returns(self, name):
        return any(text.replace(" ", "").lower() == name.lower() for _, _, text in self.st.return_items)

    @staticmethod
    def is_explicit(alias):
        return not alias.startswith(DEFAULT_ALIAS_PREFIX)

    def _add_result(self, mctx):
        """addResult (:661-729)."""
        self.stats["bindings"] += 1
        if self._returns("$elements"):
            for alias, v in mctx.matched.items():
                if self.is_explicit(alias) and v is not None:
                    self._add_single(v)
            return
        if self._returns("$pathElements"):
            for alias, v in mctx.matched.items():
                if v is not None:
                    self._add_single(v)
            return
        if self._returns("$patterns") or self._returns("$matches"):
            doc = OrderedDict((a, v) for a, v in mctx.matched.items() if self.is_explicit(a))
        elif self._returns("$paths"):
            doc = OrderedDict(mctx.matched)
        elif len(self.st.return_items) == 1 and self.st.return_items[0][0][0] == "json" and \
                self.st.return_items[0][1] is None:
            ev = Evaluator(self.db, self.ctx)
            doc = ev.value(self.st.return_items[0][0], dict(mctx.matched))
        else:
            doc = OrderedDict()
            ev = Evaluator(self.db, Ctx(self.ctx.params))
            mapdoc = dict(mctx.matched)
            for e, alias, text in self.st.return_items:
                name = alias if alias is not None else self._default_alias(e, text)
                doc[name] = self._eval_return(ev, e, mapdoc)
        self._add_single(doc)

    def _eval_return(self, ev, e, mapdoc):
        """RETURN items are evaluated against a document holding the matched map
        (ODocument.fromMap, :705-718)."""
        if e[0] == "field":
            return mapdoc.get(e[1])
        return ev.value(e, mapdoc)

    @staticmethod
    def _default_alias(e, text):
        """OExpression.getDefaultAlias: 'friend.name' → 'friend_name'."""
        return re.sub(r"[^A-Za-z0-9_$]+", "_", text.replace(" ", "")).strip("_")

    @staticmethod
    def _content_key(doc):
        """ODocumentEqualityWrapper (C/command/ODocumentEqualityWrapper.java:19-35): records compare by
        identity, documents by content."""
        if isinstance(doc, Record):
            return ("rec", doc.rid)

        def norm(x):
            if isinstance(x, Record):
                return ("r", x.rid)
            if isinstance(x, dict):
                return ("d", tuple(sorted((k, norm(v)) for k, v in x.items())))
            if isinstance(x, (list, tuple)):
                return ("l", tuple(norm(v) for v in x))
            return ("v", x)

        return norm(doc)

    def _add_single(self, doc):
        """addSingleResult (:737-750) → OBasicCommandContext.addToUniqueResult (:347-353)."""
        key = self._content_key(doc)
        if key in self.unique:
            return
        self.unique.add(key)
        self.results.append(doc)
        limit = self.limit_protocol
        if self.st.limit is not None:
            limit = self.st.limit
        if limit > -1 and limit <= len(self.results):
            raise _LimitReached()


def run(db, text, params=None, limit=None):
    """Convenience: parse + execute one MATCH statement on `db`."""
    return MatchOracle(db, text).execute(params, limit)


def rid_tuples(results, aliases):
    """Sorted tuples of packed RIDs ((cluster << 48) | position) for alias-projection results."""
    out = []
    for d in results:
        row = []
        for a in aliases:
            v = d[a] if isinstance(d, dict) else d
            row.append(-1 if v is None else (v.rid[0] << 48) | v.rid[1])
        out.append(tuple(row))
    return sorted(out)
