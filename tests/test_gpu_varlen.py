"""Variable-length MATCH items (while / maxDepth; P/OMatchPathItem.java:79-105, SURVEY §8 a9, configs[2]).

Every case runs through both device strategies — the multi-source BFS (bfs.hip, 64 rows per lane mask,
push/pull levels) and the (row, vertex) level expansion — and must equal the oracle's walk enumeration
(oracle/match_ref.py _traverse_edge, the reference's recursion restated) bit for bit.
"""
import pytest

from tests.test_gpu_parity import _parity, rmat10, rmat10_raw  # noqa: F401  (fixtures)

pytestmark = pytest.mark.gpu

VARLEN = [
    ("depth_only", "MATCH {class:Person,as:s,where:(uid = 14)}-Knows->{as:v, while:($depth < 3)} RETURN s, v"),
    ("two_batches", "MATCH {class:Person,as:s,where:(uid < 70)}-Knows->{as:v, while:($depth < 2)} RETURN s, v"),
    ("shared_sources", "MATCH {class:Person,as:a,where:(uid < 10)}-Knows->{as:b}-Knows->{as:c, while:($depth < 2)} RETURN a, b, c"),
    ("where_target", "MATCH {class:Person,as:s,where:(uid < 6)}-Knows->{as:v, while:($depth < 3), where:(age < 30)} RETURN s, v"),
    ("maxdepth", "MATCH {class:Person,as:s,where:(uid = 16)}-Knows->{as:v, maxDepth: 2, where:(age < 50)} RETURN s, v"),
    ("maxdepth0", "MATCH {class:Person,as:s,where:(uid < 4)}-Knows->{as:v, maxDepth: 0} RETURN s, v"),
    ("while_prop", "MATCH {class:Person,as:s,where:(uid < 18)}-Knows->{as:v, maxDepth: 3, while:(age < 60)} RETURN s, v"),
    ("while_false_at_1", "MATCH {class:Person,as:s,where:(uid < 8)}-Knows->{as:v, while:($depth != 1)} RETURN s, v"),
    ("in_dir", "MATCH {class:Person,as:s,where:(uid < 5)}<-Knows-{as:v, while:($depth < 3), where:(age > 40)} RETURN s, v"),
    ("both_dir", "MATCH {class:Person,as:s,where:(uid = 3)}-Knows-{as:v, maxDepth: 2} RETURN s, v"),
    ("method_form", "MATCH {class:Person,as:s,where:(uid = 17)}.out('Knows'){as:v, while:($depth < 3)} RETURN v"),
    ("depth_and_prop", "MATCH {class:Person,as:s,where:(uid < 18)}-Knows->{as:v, while:($depth < 3 and age < 70)} RETURN s, v"),
    ("where_depth", "MATCH {class:Person,as:s,where:(uid < 4)}-Knows->{as:v, while:($depth < 3), where:($depth = 2)} RETURN s, v"),
    ("bound_target", "MATCH {class:Person,as:a,where:(uid < 8)}-Knows->{as:b}, {as:a}-Knows->{as:b, while:($depth < 2)} RETURN a, b"),
]


def _cols(q):
    ret = q.split("RETURN")[1]
    return [c.strip() for c in ret.split(",")]


# environment per mode: auto push/pull, every level top-down, every level bottom-up gathering every
# mask, the same through the frontier bitmap, the same waiting for every lane (not only the live ones)
_PULL = {"OMX_VARLEN": "bfs", "OMX_BFS_PULL_DIV": "1000000000000"}
MODES = {
    "bfs_auto": {"OMX_VARLEN": "bfs"},
    "bfs_push": {"OMX_VARLEN": "bfs", "OMX_BFS_PULL_DIV": "1"},
    "bfs_pull": dict(_PULL, OMX_PULL_PROBE="0"),  # dense levels: per-vertex early-exit pull
    "bfs_pull_tiles": dict(_PULL, OMX_PULL_PROBE="0", OMX_PULL_EXIT="0"),  # dense levels: in-edge wave tiles
    "bfs_pull_tiles_slow": dict(_PULL, OMX_PULL_PROBE="0", OMX_PULL_EXIT="0", OMX_PULLW_SLOW="1"),  # the long-row path
    "bfs_full_preps": {"OMX_VARLEN": "bfs", "OMX_SPARSE_PREP": "0"},  # every level prologue a full sweep
    "bfs_pull_probe": dict(_PULL, OMX_PULL_PROBE="2", OMX_HUB_PUSH="0"),
    # sparse levels: the hub entries pulled, the non-hub frontier pushed (every level: OMX_PULL_PROBE=2)
    "bfs_pull_hubs_push": dict(_PULL, OMX_PULL_PROBE="2", OMX_HUB_PUSH="force"),
    # the workgroup-tiled k_bfs_pull, and every wave tile through the slow path
    "bfs_pull_tiles_wg": dict(_PULL, OMX_PULL_PROBE="0", OMX_PULL_EXIT="0", OMX_PULL_WAVE="0"),
    "bfs_pull_probe_wg": dict(_PULL, OMX_PULL_PROBE="2", OMX_PULL_WAVE="0"),
    "bfs_pull_all_lanes": dict(_PULL, OMX_PULL_LIVE="0"),
    "pairs": {"OMX_VARLEN": "pairs"},
}


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("q", VARLEN, ids=[q[0] for q in VARLEN])
def test_varlen_parity(rmat10, q, mode, monkeypatch):
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    g, ref = rmat10
    _parity(g, ref, q[1], _cols(q[1]))


@pytest.mark.parametrize("q", [q for q in VARLEN if q[0] in ("two_batches", "both_dir", "while_prop")], ids=lambda q: q[0])
def test_varlen_parity_multigraph(rmat10_raw, q, monkeypatch):
    monkeypatch.setenv("OMX_VARLEN", "bfs")
    g, ref = rmat10_raw
    _parity(g, ref, q[1], _cols(q[1]))


@pytest.mark.parametrize("q", [q for q in VARLEN if q[0] in ("two_batches", "where_target", "while_prop", "both_dir")
                               and "$depth" not in q[1]], ids=lambda q: q[0])
def test_bfs_edge_count_matches_visited_levels(rmat10, q, monkeypatch):
    """With a depth-free while the (row, vertex) path also keeps a visited set, so both strategies
    traverse exactly the same frontier edges (SURVEY §8(d) E_t: Σ over levels of the frontier degree sum).
    (A depth-reading while walks without a visited set on the pair path: only the row sets agree.)"""
    import orientdb_amd as o
    g, _ = rmat10
    out = {}
    for mode in ("bfs", "pairs"):
        monkeypatch.setenv("OMX_VARLEN", mode)
        out[mode] = o.OMatchStatement(q[1]).execute(g).info
    assert out["bfs"]["edges_traversed"] == out["pairs"]["edges_traversed"]
    assert out["bfs"]["n_rows"] == out["pairs"]["n_rows"]


def test_bfs_kernels_reported(rmat10, monkeypatch):
    import orientdb_amd as o
    g, _ = rmat10
    monkeypatch.setenv("OMX_VARLEN", "bfs")
    rs = o.OMatchStatement(VARLEN[1][1]).execute(g, flags=o.OMX_FLAG_KERNEL_TIMING)
    names = {k["name"] for k in rs.kernel_stats}
    assert "k_bfs_prep" in names and "k_bfs_emit" in names
    assert names & {"k_bfs_push", "k_bfs_pull", "k_bfs_pull_sparse", "k_bfs_pull_exit"}


@pytest.mark.parametrize("exit_", ["exit", "tiles"])
@pytest.mark.parametrize("hubs", ["16", "0"], ids=["partial_hubs", "no_hubs"])
@pytest.mark.parametrize("q", [q for q in VARLEN if q[0] in ("two_batches", "where_target", "in_dir", "both_dir")],
                         ids=lambda q: q[0])
def test_varlen_pull_hub_threshold(rmat10, q, hubs, exit_, monkeypatch):
    """Bottom-up levels with only the 16 highest-degree sources annotated as hubs (the degree threshold
    then picks a strict subset, as at C3's scale), or none (plain col), through the per-vertex
    early-exit pull or the merge-path tiles."""
    monkeypatch.setenv("OMX_VARLEN", "bfs")
    monkeypatch.setenv("OMX_BFS_PULL_DIV", "1000000000000")
    monkeypatch.setenv("OMX_PULL_PROBE", "0")
    monkeypatch.setenv("OMX_PULL_EXIT", "1" if exit_ == "exit" else "0")
    monkeypatch.setenv("OMX_PULL_HUBS", hubs)
    g, ref = rmat10
    _parity(g, ref, q[1], _cols(q[1]))


@pytest.fixture(scope="module")
def rmat14():
    import orientdb_amd as o
    return o.GraphSnapshot.rmat(14, device=0, keep_csr=True)


@pytest.mark.parametrize("pull", ["auto", "pull", "pull_tiles", "pull_probe", "pull_hubs_push", "pull_tiles_wg",
                                  "pull_probe_wg"])
def test_varlen_rmat14_hub_root_vs_c_bfs(rmat14, pull, monkeypatch):
    """RMAT-14 from the highest-degree vertex and 63 others (rows straddle pull tiles; the hub
    threshold picks a strict subset of the sources) against oracle/bfs_ref.c, all levels bottom-up
    in the "pull" modes ("pull_probe": every level through the frontier bitmap)."""
    import numpy as np
    import orientdb_amd as o
    from oracle import dfs
    monkeypatch.setenv("OMX_VARLEN", "bfs")
    monkeypatch.setenv("OMX_PULL_HUBS", "512")
    if pull != "auto":
        monkeypatch.setenv("OMX_BFS_PULL_DIV", "1000000000000")
    monkeypatch.setenv("OMX_PULL_PROBE", "2" if pull.startswith(("pull_probe", "pull_hubs")) else "0")
    monkeypatch.setenv("OMX_HUB_PUSH", "force" if pull == "pull_hubs_push" else "0")
    monkeypatch.setenv("OMX_PULL_EXIT", "0" if pull.startswith("pull_tiles") else "1")
    monkeypatch.setenv("OMX_PULL_WAVE", "0" if pull.endswith("_wg") else "1")
    g = rmat14
    rp, col = g.csr
    top = int(np.argmax(np.diff(rp)))
    roots = np.unique(np.concatenate([[top], np.arange(63)])).astype(np.uint32)
    q = "MATCH {class:Person,as:s,where:(uid = %d or uid < 63)}-Knows->{as:v, while:($depth < 3)} RETURN s, v" % top
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_NO_RID_MAP)
    ref = dfs.bfs_varlen(rp, col, roots, max_depth=3, nthreads=8)
    assert rs.info["n_rows"] == ref["n"]
    assert rs.info["edges_traversed"] == ref["edges"]
    got = np.sort(rs.rows[:, 0].astype(np.uint64) << np.uint64(32) | rs.rows[:, 1].astype(np.uint64))
    want = np.sort(roots[ref["pairs"][:, 0]].astype(np.uint64) << np.uint64(32) | ref["pairs"][:, 1].astype(np.uint64))
    assert np.array_equal(got, want)


@pytest.fixture(scope="module")
def rmat16():
    import orientdb_amd as o
    return o.GraphSnapshot.rmat(16, device=0, keep_csr=True)


@pytest.mark.parametrize("depth,nroots", [(4, 64), (3, 200)])
def test_c3_shape_rmat16_vs_c_bfs(rmat16, depth, nroots):
    """configs[2] query shape at RMAT-16 against oracle/bfs_ref.c: identical (s, v) rows and the same
    traversed-edge count (Σ over levels of the frontier degree sum)."""
    import numpy as np
    import orientdb_amd as o
    from oracle import dfs
    g = rmat16
    q = "MATCH {class:Person,as:s,where:(uid < %d)}-Knows->{as:v, while:($depth < %d)} RETURN s, v" % (nroots, depth)
    rs = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_NO_RID_MAP)
    ref = dfs.bfs_varlen(g.csr[0], g.csr[1], np.arange(nroots, dtype=np.uint32), max_depth=depth, nthreads=8)
    assert rs.info["n_rows"] == ref["n"]
    assert rs.info["edges_traversed"] == ref["edges"]
    si, vi = rs.columns.index("s"), rs.columns.index("v")
    got = np.sort(rs.rows[:, si].astype(np.uint64) << np.uint64(32) | rs.rows[:, vi].astype(np.uint64))
    want = np.sort(ref["pairs"][:, 0].astype(np.uint64) << np.uint64(32) | ref["pairs"][:, 1].astype(np.uint64))
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", ["bfs_auto", "bfs_full_preps", "bfs_push", "bfs_pull_hubs_push"])
@pytest.mark.parametrize("q", [q for q in VARLEN if q[0] in ("maxdepth0", "two_batches", "while_prop", "where_target")],
                         ids=lambda q: q[0])
def test_varlen_poisoned_pool(rmat10, q, mode, monkeypatch):
    """The BFS levels under OMX_POOL_POISON=1 (every pooled buffer 0xFF-filled first): a level prologue,
    a touched / active list or an emission that read a word nobody wrote would differ. Round 6 found
    one this way: maxDepth 0 with full prologues skipped the first level's prologue, the one that writes
    visited, and emitted from the poisoned words."""
    monkeypatch.setenv("OMX_POOL_POISON", "1")
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    g, ref = rmat10
    _parity(g, ref, q[1], _cols(q[1]))
