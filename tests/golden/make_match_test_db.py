"""Generate tests/golden/match_test_db.json — the graph of the reference's MATCH execution test.

Restates, as data, the database built in @BeforeClass of
/root/reference/graphdb/src/test/java/com/orientechnologies/orient/graph/sql/OMatchStatementExecutionTest.java:26-220:
  Person/Friend            :32-47
  MathOp                   :49-51
  OrgChart                 :93-187  (Department, Employee, ParentDepartment, WorksAt, ManagerOf)
  TriangleV/TriangleE      :189-205 (UNIQUE_HASH_INDEX on TriangleV.uid)
  IndexedVertex/IndexedEdge:62-91   (NOTUNIQUE index on IndexedVertex.uid, edge index on (out,in))
  DiamondV/DiamondE        :207-220

Vertices are listed in creation order; every class has one cluster (cluster ids assigned in class
creation order starting at 11), so a vertex's RID is #cluster:position with position = its rank
within its class. The reference DB uses `class.minimumClusters` clusters per class, so its RIDs are
not pinned; the known-answer tests assert counts and names only, which is what the
oracle is checked against.

Run:  python tests/golden/make_match_test_db.py   (writes the JSON next to this file)
"""
import json
import os

classes = []  # (name, superclass or None, is_edge)
vertices = []  # {"class": c, "props": {...}}
edges = []  # {"class": c, "out": vidx, "in": vidx}
indexes = []  # {"class": c, "property": p, "unique": bool}


def cls(name, sup, is_edge=False):
    classes.append({"name": name, "superclass": sup, "is_edge": is_edge})


def vertex(klass, **props):
    vertices.append({"class": klass, "props": props})
    return len(vertices) - 1


def edge(c, a, b):
    edges.append({"class": c, "out": a, "in": b})


def find(klass, **props):
    out = []
    for i, v in enumerate(vertices):
        if v["class"] == klass and all(v["props"].get(k) == x for k, x in props.items()):
            out.append(i)
    return out


cls("V", None)
cls("E", None, True)

# Person / Friend (:32-47)
cls("Person", "V")
cls("Friend", "E", True)
for n in ["n1", "n2", "n3", "n4", "n5", "n6"]:
    vertex("Person", name=n)
for a, b in [("n1", "n2"), ("n1", "n3"), ("n2", "n4"), ("n4", "n5"), ("n4", "n6")]:
    edge("Friend", find("Person", name=a)[0], find("Person", name=b)[0])

# MathOp (:49-51)
cls("MathOp", "V")
vertex("MathOp", a=1, b=3, c=2)
vertex("MathOp", a=5, b=3, c=2)

# OrgChart (:93-187)
cls("Employee", "V")
cls("Department", "V")
cls("ParentDepartment", "E", True)
cls("WorksAt", "E", True)
cls("ManagerOf", "E", True)
dept_hierarchy = [[1, 2], [3, 4], [5, 6], [7, 8], [], [], [], [9], [], []]
dept_managers = ["a", "b", "d", None, None, None, None, "c", None, None]
employees = [["p1"], ["p2", "p3"], ["p4", "p5"], ["p6"], ["p7"], ["p8"], ["p9"], ["p10"], ["p11"], ["p12", "p13"]]
for i in range(10):
    vertex("Department", name="department%d" % i)
for parent, children in enumerate(dept_hierarchy):
    for child in children:
        edge("ParentDepartment", find("Department", name="department%d" % child)[0],
             find("Department", name="department%d" % parent)[0])
for dept, manager in enumerate(dept_managers):
    if manager is not None:
        m = vertex("Employee", name=manager)
        edge("ManagerOf", m, find("Department", name="department%d" % dept)[0])
for dept, emps in enumerate(employees):
    for e in emps:
        v = vertex("Employee", name=e)
        edge("WorksAt", v, find("Department", name="department%d" % dept)[0])

# Triangle (:189-205)
cls("TriangleV", "V")
indexes.append({"class": "TriangleV", "property": "uid", "unique": True})
cls("TriangleE", "E", True)
for i in range(10):
    vertex("TriangleV", uid=i)
for a, b in [(0, 1), (0, 2), (1, 2), (1, 3), (2, 4), (3, 4), (3, 5), (4, 0), (4, 7), (6, 7), (7, 8), (7, 9), (8, 9),
             (9, 1), (8, 3), (8, 4)]:
    edge("TriangleE", find("TriangleV", uid=a)[0], find("TriangleV", uid=b)[0])

# IndexedVertex / IndexedEdge (:62-91); the reference creates this after the triangle graph.
cls("IndexedVertex", "V")
indexes.append({"class": "IndexedVertex", "property": "uid", "unique": False})
cls("IndexedEdge", "E", True)
nodes = 1000
first = len(vertices)
for i in range(nodes):
    vertex("IndexedVertex", uid=i)
for i in range(100):
    lo, hi = i * nodes // 100, (i + 1) * nodes // 100
    for u in range(nodes):
        if lo < u < hi:
            edge("IndexedEdge", first + 0, first + u)
for i in range(100):
    lo, hi = (i * nodes // 100) + 1, ((i + 1) * nodes // 100) + 1
    for u in range(nodes):
        if lo < u < hi:
            edge("IndexedEdge", first + u, first + 1)

# Diamond (:207-220)
cls("DiamondV", "V")
cls("DiamondE", "E", True)
for i in range(4):
    vertex("DiamondV", uid=i)
for a, b in [(0, 1), (0, 2), (1, 3), (2, 3)]:
    edge("DiamondE", find("DiamondV", uid=a)[0], find("DiamondV", uid=b)[0])

if __name__ == "__main__":
    out = {"classes": classes, "vertices": vertices, "edges": edges, "indexes": indexes}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "match_test_db.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=None, separators=(",", ":"))
    print("wrote", path, len(vertices), "vertices", len(edges), "edges")
