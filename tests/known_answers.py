"""Known-answer MATCH cases of the reference, as data.

Every entry restates one assertion of
/root/reference/graphdb/src/test/java/com/orientechnologies/orient/graph/sql/OMatchStatementExecutionTest.java
(line numbers given), on the graph of tests/golden/match_test_db.json. `outer` restates the wrapping
legacy `select ... from (match ...)` where the test has one:
  ("names", alias)       select <alias>.name as name from (...)   → multiset of names
  ("expand", alias)      select expand(<alias>) from (...)        → list of records
`expect` is (count, names or None): names is the expected set of `name`/value strings when the test
asserts them. `gpu` marks cases the MI355X engine is expected to execute (the rest must come back
OMX_E_UNSUPPORTED and fall back to the reference engine).
"""

KNOWN = [
    # id, line, query, params, outer, expect(count, values), gpu
    ("testSimple", 232, "match {class:Person, as: person} return person", None, None, (6, None), True),
    ("testSimpleWhere", 246,
     "match {class:Person, as: person, where: (name = 'n1' or name = 'n2')} return person", None,
     ("names", "person"), (2, {"n1", "n2"}), True),
    ("testSimpleLimit", 261,
     "match {class:Person, as: person, where: (name = 'n1' or name = 'n2')} return person limit 1", None, None,
     (1, None), True),
    ("testSimpleLimit2", 269,
     "match {class:Person, as: person, where: (name = 'n1' or name = 'n2')} return person limit -1", None, None,
     (2, None), True),
    ("testSimpleLimit3", 277,
     "match {class:Person, as: person, where: (name = 'n1' or name = 'n2')} return person limit 3", None, None,
     (2, None), True),
    ("testSimpleUnnamedParams", 285,
     "match {class:Person, as: person, where: (name = ? or name = ?)} return person", ["n1", "n2"],
     ("names", "person"), (2, {"n1", "n2"}), True),
    ("testCommonFriends", 300,
     "match {class:Person, where:(name = 'n1')}.both('Friend'){as:friend}.both('Friend'){class: Person, where:(name = 'n4')} return $matches",
     None, ("names", "friend"), (1, {"n2"}), True),
    ("testCommonFriendsArrows", 312,
     "match {class:Person, where:(name = 'n1')}-Friend-{as:friend}-Friend-{class: Person, where:(name = 'n4')} return $matches",
     None, ("names", "friend"), (1, {"n2"}), True),
    ("testCommonFriends2", 324,
     "match {class:Person, where:(name = 'n1')}.both('Friend'){as:friend}.both('Friend'){class: Person, where:(name = 'n4')} return friend.name as name",
     None, ("field", "name"), (1, {"n2"}), True),
    ("testCommonFriends2Arrows", 336,
     "match {class:Person, where:(name = 'n1')}-Friend-{as:friend}-Friend-{class: Person, where:(name = 'n4')} return friend.name as name",
     None, ("field", "name"), (1, {"n2"}), True),
    ("testReturnMethod", 348,
     "match {class:Person, where:(name = 'n1')}.both('Friend'){as:friend}.both('Friend'){class: Person, where:(name = 'n4')} return friend.name.toUppercase() as name",
     None, ("field", "name"), (1, {"N2"}), True),
    ("testReturnMethodArrows", 360,
     "match {class:Person, where:(name = 'n1')}-Friend-{as:friend}-Friend-{class: Person, where:(name = 'n4')} return friend.name.toUppercase() as name",
     None, ("field", "name"), (1, {"N2"}), True),
    ("testReturnExpression", 372,
     "match {class:Person, where:(name = 'n1')}.both('Friend'){as:friend}.both('Friend'){class: Person, where:(name = 'n4')} return friend.name + ' ' +friend.name as name",
     None, ("field", "name"), (1, {"n2 n2"}), True),
    ("testReturnExpressionArrows", 384,
     "match {class:Person, where:(name = 'n1')}-Friend-{as:friend}-Friend-{class: Person, where:(name = 'n4')} return friend.name + ' ' +friend.name as name",
     None, ("field", "name"), (1, {"n2 n2"}), True),
    ("testReturnDefaultAlias", 396,
     "match {class:Person, where:(name = 'n1')}.both('Friend'){as:friend}.both('Friend'){class: Person, where:(name = 'n4')} return friend.name",
     None, ("field", "friend_name"), (1, {"n2"}), True),
    ("testReturnDefaultAliasArrows", 408,
     "match {class:Person, where:(name = 'n1')}-Friend-{as:friend}-Friend-{class: Person, where:(name = 'n4')} return friend.name",
     None, ("field", "friend_name"), (1, {"n2"}), True),
    ("testFriendsOfFriends", 414,
     "match {class:Person, where:(name = 'n1')}.out('Friend').out('Friend'){as:friend} return $matches", None,
     ("names", "friend"), (1, {"n4"}), True),
    ("testFriendsOfFriendsArrows", 426,
     "match {class:Person, where:(name = 'n1')}-Friend->{}-Friend->{as:friend} return $matches", None,
     ("names", "friend"), (1, {"n4"}), True),
    ("testFriendsOfFriends2", 438,
     "match {class:Person, where:(name = 'n1'), as: me}.both('Friend').both('Friend'){as:friend, where: ($matched.me != $currentMatch)} return $matches",
     None, ("names_not", "friend"), (None, {"n1"}), True),
    ("testFriendsOfFriends2Arrows", 452,
     "match {class:Person, where:(name = 'n1'), as: me}-Friend-{}-Friend-{as:friend, where: ($matched.me != $currentMatch)} return $matches",
     None, ("names_not", "friend"), (None, {"n1"}), True),
    ("testFriendsWithName", 466,
     "match {class:Person, where:(name = 'n1' and 1 + 1 = 2)}.out('Friend'){as:friend, where:(name = 'n2' and 1 + 1 = 2)} return friend",
     None, ("names", "friend"), (1, {"n2"}), True),
    ("testFriendsWithNameArrows", 478,
     "match {class:Person, where:(name = 'n1' and 1 + 1 = 2)}-Friend->{as:friend, where:(name = 'n2' and 1 + 1 = 2)} return friend",
     None, ("names", "friend"), (1, {"n2"}), True),
    ("testWhile.1", 493,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, while: ($depth < 1)} return friend", None,
     ("names", "friend"), (3, None), True),
    ("testWhile.2", 501,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, while: ($depth < 2), where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testWhile.3", 509,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, while: ($depth < 4), where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testWhile.4", 517,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, while: (true) } return friend", None,
     ("names", "friend"), (6, None), True),
    ("testWhile.5", 525,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, while: (true) } return friend limit 3", None,
     ("names", "friend"), (3, None), True),
    ("testWhileArrows.1", 540,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, while: ($depth < 1)} return friend", None,
     ("names", "friend"), (3, None), True),
    ("testWhileArrows.2", 548,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, while: ($depth < 2), where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testWhileArrows.3", 556,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, while: ($depth < 4), where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testWhileArrows.4", 564,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, while: (true) } return friend", None,
     ("names", "friend"), (6, None), True),
    ("testMaxDepth.1", 573,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, maxDepth: 1, where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testMaxDepth.2", 580,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, maxDepth: 1 } return friend", None,
     ("names", "friend"), (3, None), True),
    ("testMaxDepth.3", 587,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, maxDepth: 0 } return friend", None,
     ("names", "friend"), (1, None), True),
    ("testMaxDepth.4", 594,
     "match {class:Person, where:(name = 'n1')}.out('Friend'){as:friend, maxDepth: 1, where: ($depth > 0) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testMaxDepthArrow.1", 604,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, maxDepth: 1, where: ($depth=1) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testMaxDepthArrow.2", 611,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, maxDepth: 1 } return friend", None,
     ("names", "friend"), (3, None), True),
    ("testMaxDepthArrow.3", 618,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, maxDepth: 0 } return friend", None,
     ("names", "friend"), (1, None), True),
    ("testMaxDepthArrow.4", 625,
     "match {class:Person, where:(name = 'n1')}-Friend->{as:friend, maxDepth: 1, where: ($depth > 0) } return friend",
     None, ("names", "friend"), (2, None), True),
    ("testTriangle1", 891,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}.out('TriangleE'){as: friend2}.out('TriangleE'){as: friend3},{class:TriangleV, as: friend1}.out('TriangleE'){as: friend3}return $matches",
     None, None, (1, None), True),
    ("testTriangle1Arrows", 905,
     "match {class:TriangleV, as: friend1, where: (uid = 0)} -TriangleE-> {as: friend2} -TriangleE-> {as: friend3},{class:TriangleV, as: friend1} -TriangleE-> {as: friend3}return $matches",
     None, None, (1, None), True),
    ("testTriangle2Old", 917,
     "match {class:TriangleV, as: friend1}.out('TriangleE'){class:TriangleV, as: friend2, where: (uid = 1)}.out('TriangleE'){as: friend3},{class:TriangleV, as: friend1}.out('TriangleE'){as: friend3}return $matches",
     None, ("uids", ("friend1", "friend2", "friend3")), (1, {(0, 1, 2)}), True),
    ("testTriangle2", 939,
     "match {class:TriangleV, as: friend1}.out('TriangleE'){class:TriangleV, as: friend2, where: (uid = 1)}.out('TriangleE'){as: friend3},{class:TriangleV, as: friend1}.out('TriangleE'){as: friend3}return $patterns",
     None, ("uids", ("friend1", "friend2", "friend3")), (1, {(0, 1, 2)}), True),
    ("testTriangle2Arrows", 961,
     "match {class:TriangleV, as: friend1}-TriangleE->{class:TriangleV, as: friend2, where: (uid = 1)}-TriangleE->{as: friend3},{class:TriangleV, as: friend1}-TriangleE->{as: friend3}return $matches",
     None, ("uids", ("friend1", "friend2", "friend3")), (1, {(0, 1, 2)}), True),
    ("testTriangle3", 983,
     "match {class:TriangleV, as: friend1}-TriangleE->{as: friend2}-TriangleE->{as: friend3, where: (uid = 2)},{class:TriangleV, as: friend1}-TriangleE->{as: friend3}return $matches",
     None, None, (1, None), True),
    ("testTriangle4", 998,
     "match {class:TriangleV, as: friend1}.out('TriangleE'){as: friend2, where: (uid = 1)}.out('TriangleE'){as: friend3},{class:TriangleV, as: friend1}.out('TriangleE'){as: friend3}return $matches",
     None, None, (1, None), True),
    ("testTriangle4Arrows", 1013,
     "match {class:TriangleV, as: friend1}-TriangleE->{as: friend2, where: (uid = 1)}-TriangleE->{as: friend3},{class:TriangleV, as: friend1}-TriangleE->{as: friend3}return $matches",
     None, None, (1, None), True),
    ("testTriangleWithEdges4", 1028,
     "match {class:TriangleV, as: friend1}.outE('TriangleE').inV(){as: friend2, where: (uid = 1)}.outE('TriangleE').inV(){as: friend3},{class:TriangleV, as: friend1}.outE('TriangleE').inV(){as: friend3}return $matches",
     None, None, (1, None), True),
    ("testCartesianProduct", 1048,
     "match {class:TriangleV, as: friend1, where:(uid = 1)},{class:TriangleV, as: friend2, where:(uid = 2 or uid = 3)}return $matches",
     None, ("uid_of", "friend1"), (2, {1}), True),
    ("testCartesianProductLimit", 1063,
     "match {class:TriangleV, as: friend1, where:(uid = 1)},{class:TriangleV, as: friend2, where:(uid = 2 or uid = 3)}return $matches LIMIT 1",
     None, ("uid_of", "friend1"), (1, {1}), True),
    ("testArrayNumber", 1078,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[0] as foo", None,
     ("field_kind", "foo"), (1, "vertex"), True),
    ("testArraySingleSelectors2", 1092,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[0,1] as foo", None,
     ("field_len", "foo"), (1, 2), True),
    ("testArrayRangeSelectors1", 1107,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[0-1] as foo", None,
     ("field_len", "foo"), (1, 1), True),
    ("testArrayRange2", 1122,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[0-2] as foo", None,
     ("field_len", "foo"), (1, 2), True),
    ("testArrayRange3", 1137,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[0-3] as foo", None,
     ("field_len", "foo"), (1, 2), True),
    ("testConditionInSquareBrackets", 1152,
     "match {class:TriangleV, as: friend1, where: (uid = 0)}return friend1.out('TriangleE')[uid = 2] as foo", None,
     ("list_uids", "foo"), (1, [2]), True),  # :1168-1171: one vertex, uid == 2
    ("testIndexedEdge", 1175,
     "match {class:IndexedVertex, as: one, where: (uid = 0)}.out('IndexedEdge'){class:IndexedVertex, as: two, where: (uid = 1)}return one, two",
     None, None, (1, None), True),
    ("testIndexedEdgeArrows", 1187,
     "match {class:IndexedVertex, as: one, where: (uid = 0)}-IndexedEdge->{class:IndexedVertex, as: two, where: (uid = 1)}return one, two",
     None, None, (1, None), True),
    ("testJson", 1199, "match {class:IndexedVertex, as: one, where: (uid = 0)} return {'name':'foo', 'uuid':one.uid}",
     None, None, (1, None), True),
    ("testJson2", 1213,
     "match {class:IndexedVertex, as: one, where: (uid = 0)} return {'name':'foo', 'sub': {'uuid':one.uid}}", None,
     None, (1, None), True),
    ("testJson3", 1227,
     "match {class:IndexedVertex, as: one, where: (uid = 0)} return {'name':'foo', 'sub': [{'uuid':one.uid}]}", None,
     None, (1, None), True),
    ("testUnique.1", 1241,
     "match {class:DiamondV, as: one, where: (uid = 0)}.out('DiamondE').out('DiamondE'){as: two} return one, two",
     None, None, (1, None), True),
    ("testUnique.2", 1250,
     "match {class:DiamondV, as: one, where: (uid = 0)}.out('DiamondE').out('DiamondE'){as: two} return one.uid, two.uid",
     None, None, (1, None), True),
    ("testOptional", 1323,
     "match {class:Person, as: person} -NonExistingEdge-> {as:b, optional:true} return person, b.name", None, None,
     (6, None), True),
    ("testOptional2", 1336,
     "match {class:Person, as: person} --> {as:b, optional:true, where:(nonExisting = 12)} return person, b.name",
     None, None, (6, None), True),
    ("testOptional3", 1349,
     "match {class:Person, as:a, where:(name = 'n1' and 1 + 1 = 2)}.out('Friend'){as:friend, where:(name = 'n2' and 1 + 1 = 2)},{as:a}.out(){as:b, where:(nonExisting = 12), optional:true},{as:friend}.out(){as:b, optional:true} return friend",
     None, ("names", "friend"), (1, {"n2"}), True),
    ("testAliasesWithSubquery", 1365, "match {class:Person, as:A} return A.name as namexx", None,
     ("field_prefix", "namexx"), (6, "n"), True),
]


def _manager(person, arrows, multi):
    if multi:
        body = ("  .( -WorksAt->{}-ParentDepartment->{      while: (in('ManagerOf').size() == 0),"
                "      where: (in('ManagerOf').size() > 0)     }   )<-ManagerOf-{as: manager}") if arrows else (
            "   .( out('WorksAt')     .out('ParentDepartment'){       while: (in('ManagerOf').size() == 0),"
            "       where: (in('ManagerOf').size() > 0)     }   )  .in('ManagerOf'){as: manager}")
    else:
        body = ("  -WorksAt->{}-ParentDepartment->{      while: (in('ManagerOf').size() == 0),"
                "      where: (in('ManagerOf').size() > 0)  }<-ManagerOf-{as: manager}") if arrows else (
            "  .out('WorksAt')  .out('ParentDepartment'){      while: (in('ManagerOf').size() == 0),"
            "      where: (in('ManagerOf').size() > 0)  }  .in('ManagerOf'){as: manager}")
    return "  match {class:Employee, where: (name = '%s')}%s  return manager" % (person, body)


def _managed(manager, arrows, multi, ret="managed"):
    cond = "$depth = 0 or in('ManagerOf').size() = 0"
    if multi:
        mid = ("  -ManagerOf->{}  .(inE('ParentDepartment').outV()){      while: (%s),      where: (%s)  }<-WorksAt-{as: managed}"
               if arrows else
               "  .out('ManagerOf')  .(inE('ParentDepartment').outV()){      while: (%s),      where: (%s)  }  .in('WorksAt'){as: managed}")
    else:
        mid = ("  -ManagerOf->{}<-ParentDepartment-{      while: (%s),      where: (%s)  }<-WorksAt-{as: managed}"
               if arrows else
               "  .out('ManagerOf')  .in('ParentDepartment'){      while: (%s),      where: (%s)  }  .in('WorksAt'){as: managed}")
    boss = ", as:boss" if ret != "managed" else ""
    return "  match {class:Employee%s, where: (name = '%s')}%s  return %s" % (boss, manager, mid % (cond, cond), ret)


for _p, _m in [("p10", "c"), ("p12", "c"), ("p6", "b"), ("p11", "b")]:
    for _arrows in (False, True):
        for _multi in (False, True):
            KNOWN.append(("testManager%s%s.%s" % ("2" if _multi else "", "Arrows" if _arrows else "", _p),
                          660 if not _multi else 710, _manager(_p, _arrows, _multi), None, ("names", "manager"),
                          (1, {_m}), True))
for _arrows in (False, True):
    for _multi in (False, True):
        tag = "testManaged%s%s" % ("2" if _multi else "", "Arrows" if _arrows else "")
        KNOWN.append((tag + ".a", 734, _managed("a", _arrows, _multi), None, ("names", "managed"), (1, {"p1"}), True))
        KNOWN.append((tag + ".b", 734, _managed("b", _arrows, _multi), None, ("names", "managed"),
                      (5, {"p2", "p3", "p6", "p7", "p11"}), True))
KNOWN.append(("testManagedElements", 1264, _managed("b", True, False, "$elements"), None, ("record_names", None),
              (6, {"b", "p2", "p3", "p6", "p7", "p11"}), True))
KNOWN.append(("testManagedPathElements", 1299, _managed("b", True, False, "$pathElements"), None,
              ("record_names", None),
              (10, {"department1", "department3", "department4", "department8", "b", "p2", "p3", "p6", "p7", "p11"}),
              True))
