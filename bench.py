"""Benchmark: MATCH edges traversed/sec (GTEPS) + bindings/sec on a synthetic RMAT Person/Knows graph.

Default workload = BASELINE.json's metric config, "RMAT-24 2-hop" (`--query m1`): RMAT scale-24
(V = 16,777,216, 16·V raw edges, simple: 263 M edges) with configs[1]'s 2-hop query,
  MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c
(root window 1 %, target window 10 %: 168 K roots, E_t ≈ 1.03e10 edges, ≈ 1.03e9 distinct rows per step,
SURVEY §8(d) "adjust to keep ≤ ~1e9 rows"). `--query c2` is configs[1] itself (the same query at scale 22);
c1/c3/c4/c5 are the other configs. One "step" = one full execution of the MATCH (root scan → expansions
→ distinct rows in HBM; inputs resident in HBM before the timed region).

N GPUs (one process per GPU, torch.distributed.run): by default the graph is 1-D PARTITIONED (SURVEY
§8(e), BASELINE north_star): rank r generates and holds the CSR rows of the vertices [r·B, (r+1)·B),
starts from the roots it owns, and binding rows travel to the owner of the vertex whose adjacency the
next hop reads (RCCL all-to-all over xGMI). The query is the same at every N: scaling is "strong".
`--replicated`: the graph is replicated, roots sharded v % N == rank, no data-path collective, and the
root window widens to `age < N` so per-GPU work is fixed ("weak"). The barrier and the max-over-ranks
reduction go over gloo (CPU); torch never touches the GPU here (libomx owns it).

Prints ONE JSON line (rank 0).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "MATCH edges traversed/sec (GTEPS) + bindings/sec, RMAT-24 2-hop, 1-8 GPUs"
# name → (workload, query, default RMAT scale)
QUERIES = {
    "m1": ("M1: RMAT-24 2-hop MATCH with WHERE on both ends (the metric's own config; configs[1]'s query at scale 24)",
           "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c", 24),
    "c2": ("C2: RMAT 2-hop MATCH with WHERE property filter on both ends",
           "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c", 22),
    "c1": ("C1: RMAT 2-hop MATCH friends-of-friends", "MATCH {class:Person}-Knows->{}-Knows->{as:fof} RETURN fof", 16),
    "c3": ("C3: variable-length MATCH out('Knows'){while:($depth<4)} from 64 roots (multi-source BFS)",
           "MATCH {class:Person,as:s,where:(uid < 64)}-Knows->{as:v, while:($depth < 4)} RETURN s, v", 24),
    "c4": ("C4: cyclic triangle MATCH (a->b->c->a) via sorted-adjacency intersection, LDBC-SNB-like SF10 Knows",
           "MATCH {class:Person,as:a}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c", "ldbc"),
    "c5": ("C5: RMAT 3-hop MATCH (COUNT), 1-D partitioned graph, per-hop all-to-all row exchange (RCCL)",
           "MATCH {class:Person,as:a,where:(uid < 64)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:d} RETURN a,b,c,d", 26),
    "r1": ("R1: configs[1]'s 2-hop at RMAT-22 returning RETURN expressions (documents by content, evaluated on the device)",
           "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a.uid, b.age", 22),
    # edge nodes (round 6): configs[1]'s shape with the Knows edges as records and a filter on their field w
    "e1": ("E1: configs[1]'s 2-hop at RMAT-22 through edge nodes, outE('Knows'){as: e, where: (w < 10)}.inV()",
           "MATCH {class:Person,as:a,where:(age < 1)}.outE('Knows'){as:e, where:(w < 10)}.inV(){as:b,where:(age >= 90)} "
           "RETURN a, e, b", 22),
    # SURVEY §8(f) rows (not the metric): {hub} = the vertex of highest out-degree
    "t1": ("T1: TRAVERSE out('Knows') STRATEGY BREADTH_FIRST from the highest-degree vertex (its whole reach)",
           "TRAVERSE out('Knows') FROM #11:{hub} STRATEGY BREADTH_FIRST", 24),
    "s1": ("S1: SELECT expand(out('Knows').out('Knows')) from the highest-degree vertex (rows with repeats)",
           "SELECT expand(out('Knows').out('Knows')) FROM #11:{hub}", 22),
    "p1": ("P1: shortestPath() over out('Knows') from the lowest-id vertex of out-degree 1 to the highest-degree vertex",
           "SELECT expand(shortestPath(#11:{leaf}, #11:{hub}, 'OUT', 'Knows'))", 24),
}
CHAIN = {"t1", "s1", "p1"}
# Weak scaling over roots on the replicated graph (each root's DFS subtree is independent):
# at N ranks the root window widens N-fold and every rank keeps ≈ the N=1 share (roots v % N == rank),
# so per-GPU work is fixed as N grows. At N=1 the query is exactly configs[1]'s.
WEAK_ROOTS = {"c2": ("age < 1", "age < %d"), "m1": ("age < 1", "age < %d")}


def scaled_query(name, query, world, partitioned):
    """The query a run at `world` ranks executes, and its scaling kind."""
    if world > 1 and name in WEAK_ROOTS and not partitioned:
        old, new = WEAK_ROOTS[name]
        assert old in query
        return query.replace(old, new % world), "weak"
    return query, "strong"


REPLICATED_ONLY = {"c1", "c4", "t1", "s1", "p1", "e1"}
EDGE_RECORDS = {"e1"}  # snapshots built with the edges as records (GraphSnapshot.rmat(edge_records=True))  # C4 LDBC replica; C1 all-root fof; TRAVERSE / SELECT / shortestPath
COUNT_MODE = {"c5"}   # the last hop counts its rows (count mode)
LDBC_SF10 = dict(n_persons=70000, target_edges=2_000_000, seed=10)  # ≈7e4 Person, ≈2e6 Knows
# kernels that can be the dominant one (pseudo-records like expand_total / dedup are spans, not kernels)
HOT_KERNELS = ("k_femit", "k_flists", "k_fof2_a", "k_fof2_b", "k_isect_merge", "k_expand_heavy", "k_expand_heavy_sliced", "k_expand_light", "k_expand_light_sliced", "k_trav_filter",
               "k_expand_light_check", "k_expand_heavy_check", "k_check", "k_bfs_pull", "k_bfs_pull_sparse", "k_bfs_pull_exit", "k_bfs_push", "k_bfs_prep", "k_bfs_emit",
               "k_gather_cols", "k_compact_segments")
# timer records that are spans over other records or move no HBM bytes (not summed into a step)
SPAN_RECORDS = ("expand_total", "documents", "exchange", "deliver_d2h")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md §Chip-level parameters)


def hip_sync():
    """hipDeviceSynchronize on the runtime libomx uses (torch is kept off the GPU in this process)."""
    ctypes.CDLL("libamdhip64.so.7").hipDeviceSynchronize()


def cpu_baseline_varlen(g, nroots, depth, target_s, threads):
    """configs[2]: the oracle's C BFS restatement (oracle/bfs_ref.c), one root per thread."""
    import numpy as np
    from oracle import dfs
    rp, col = g.csr
    roots = np.arange(nroots, dtype=np.uint32)
    edges = pairs = 0
    secs = 0.0
    reps = 0
    while secs < target_s and reps < 1000:
        r = dfs.bfs_varlen(rp, col, roots, max_depth=depth, nthreads=threads, emit=False)
        edges += r["edges"]
        pairs += r["n"]
        secs += r["seconds"]
        reps += 1
    return {"value": edges / secs / 1e9, "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": "all %d roots x %d repetitions (%.1f s, %d edges, %d result rows; oracle/bfs_ref.c BFS, %d threads)" % (
                nroots, reps, secs, edges, pairs, threads),
            "bindings_per_s": pairs / secs}


def host_threads():
    """Threads for the CPU baseline: the host cores this job may use. On the GPU box that is its CPU
    share per GPU, which the harness exports as OMP_NUM_THREADS (16); os.cpu_count() there reports the
    whole machine, whose other cores belong to other jobs. Returns (threads, cores visible)."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(share, visible) if share > 0 else visible), visible


def cpu_baseline_chain(g, query, target_s):
    """TRAVERSE / SELECT expand: the oracle's restatement (oracle/traverse_ref.py, pure Python, one core)
    on a bounded sample of the same kind of work, GTEPS = adjacency entries it iterated / its time.
    TRAVERSE: the work list FROM the first K vertices MAXDEPTH 1 (every root's out-list pushed and
    processed); SELECT: the two-call chain over the first K vertices. K doubles until ≈ target_s / 4."""
    from oracle.traverse_ref import BREADTH_FIRST, expand_chain, traverse
    rp, col = g.csr
    seen = [0]

    def out(v):
        row = col[rp[v]:rp[v + 1]].tolist()
        seen[0] += len(row)
        return row
    k = 256
    while True:
        seen[0] = 0
        roots = list(range(min(k, g.V)))
        t0 = time.perf_counter()
        if query.startswith("TRAVERSE"):
            traverse(roots, lambda v: [out(v)], max_depth=1, strategy=BREADTH_FIRST)
            what = "the work list from vertices 0..%d, MAXDEPTH 1" % (len(roots) - 1)
        else:
            expand_chain(roots, [out, out])
            what = "the chain out().out() from vertices 0..%d" % (len(roots) - 1)
        secs = time.perf_counter() - t0
        if secs > target_s / 4 or k >= g.V:
            break
        k *= 2
    return {"value": seen[0] / secs / 1e9, "unit": "GTEPS", "cores": 1, "kind": "port",
            "sample": "%s (%.1f s, %d adjacency entries; oracle/traverse_ref.py, pure Python, 1 thread)" % (
                what, secs, seen[0])}


def cpu_baseline_shortest(g, query, target_s):
    """shortestPath: the oracle's restatement (oracle/shortest_path_ref.py, pure Python, one core) on the
    same pair, repeated to ≈ target_s / 4; GTEPS = adjacency entries its walks iterated / its time."""
    import re
    from oracle.shortest_path_ref import shortest_path
    from orientdb_amd.graph import csr_transpose
    rp, col = g.csr
    a, b = (int(x) for x in re.findall(r"#11:(\d+)", query)[:2])
    irp, icol = csr_transpose(g.V, rp, col)
    seen = [0]

    def nb(r, c):
        def f(v):
            row = c[r[v]:r[v + 1]].tolist()
            seen[0] += len(row)
            return row
        return f
    secs, reps = 0.0, 0
    while secs < target_s / 4 and reps < 100:
        t0 = time.perf_counter()
        shortest_path(a, b, nb(rp, col), nb(irp, icol))
        secs += time.perf_counter() - t0
        reps += 1
    return {"value": seen[0] / secs / 1e9, "unit": "GTEPS", "cores": 1, "kind": "port",
            "sample": "the same pair x %d (%.1f s, %d adjacency entries; oracle/shortest_path_ref.py, pure Python, "
                      "1 thread)" % (reps, secs, seen[0])}


def cpu_baseline_edges(g, query, target_s):
    """E1: the edge-node 2-hop restated over the CSR with numpy (oracle/edge_ref.py, one core, pinned to
    oracle/match_ref.py) on a bounded sample of the roots, doubled until ≈ target_s / 4."""
    import re
    import numpy as np
    from oracle.edge_ref import edge_two_hop
    rp, col = g.csr
    amax, wmax, bmin = (int(x) for x in re.search(r"age < (\d+).*w < (\d+).*age >= (\d+)", query).groups())
    roots = np.nonzero(g.age < amax)[0]
    emask, bmask = g.w < wmax, g.age >= bmin
    k = 1024
    while True:
        sample = roots[:k]
        t0 = time.perf_counter()
        r, edges = edge_two_hop(rp, col, sample, emask, bmask)
        secs = time.perf_counter() - t0
        if secs > target_s / 4 or k >= len(roots):
            break
        k *= 2
    reps = 1
    while secs < target_s / 4 and reps < 1000:  # the whole root set is a short run: repeat it
        t0 = time.perf_counter()
        edge_two_hop(rp, col, sample, emask, bmask)
        secs += time.perf_counter() - t0
        reps += 1
    return {"value": edges * reps / secs / 1e9, "unit": "GTEPS", "cores": 1, "kind": "port",
            "sample": "%d of %d roots x %d (%.1f s, %d edges and %d rows each; oracle/edge_ref.py, numpy, 1 thread)" % (
                len(sample), len(roots), reps, secs, edges, len(r[0]))}


def cpu_baseline(g, query, target_s=12.0, single_thread_too=False):
    """The oracle's C DFS restatement (oracle/dfs_ref.c) on the host cores, on a bounded sample of
    the same workload's roots; GTEPS over the sampled roots."""
    import numpy as np
    from oracle import dfs
    if "shortestPath" in query:
        return cpu_baseline_shortest(g, query, target_s)
    if query.startswith(("TRAVERSE", "SELECT")):
        return cpu_baseline_chain(g, query, target_s)
    if ".outE(" in query:
        return cpu_baseline_edges(g, query, target_s)
    threads, visible = host_threads()
    if "while:($depth < 4)" in query:
        r = cpu_baseline_varlen(g, 64, 4, target_s, threads)
        r["cores_visible"] = visible
        return r
    rp, col = g.csr
    cg = dfs.CsrGraph(rp, col, {"uid": np.arange(g.V, dtype=np.int64), "age": g.age})
    head, ret = query.split("RETURN")
    if "." in ret:  # RETURN expressions: the DFS enumerates the same bindings of the aliases they read
        import re as _re
        query = head + "RETURN " + ",".join(sorted(set(_re.findall(r"\b([a-z]+)\.", ret))))
    import re
    m = re.search(r"\((age|uid) < (\d+)\)", query.split("-")[0])
    nroots_total = int(np.count_nonzero(cg.columns[m.group(1)] < int(m.group(2)))) if m else g.V
    out = dfs_sample(dfs, cg, query, threads, target_s, nroots_total)
    out["cores_visible"] = visible
    try:  # the same bindings set-at-a-time (the set-based CPU path beside the DFS)
        sb = set_sample(dfs, cg, query, threads, target_s, nroots_total, out.pop("bindings_per_root"))
        if sb is not None:
            out["set_based"] = sb
    except NotImplementedError:
        pass
    if single_thread_too:  # configs[0]: the faithful one-thread DFS beside the port on the job's cores
        one = dfs_sample(dfs, cg, query, 1, target_s / 2, nroots_total)
        out["single_thread"] = {k: one[k] for k in ("value", "unit", "cores", "kind", "sample", "bindings_per_s")}
    return out


def dfs_sample(dfs, cg, query, threads, target_s, nroots_total):
    """oracle/dfs_ref.c over a bounded root sample, repeated until ≈ target_s of CPU work is timed."""
    probe = dfs.run(cg, query, nthreads=threads, emit=False, root_sample=64)
    per_root = max(probe["seconds"] / max(probe["nroots"], 1), 1e-7)
    sample = int(min(nroots_total, max(64, target_s / per_root)))
    edges = bindings = 0
    secs = 0.0
    reps = 0
    while secs < target_s and reps < 1000:
        r = dfs.run(cg, query, nthreads=threads, emit=False, root_sample=sample)
        edges += r["edges"]
        bindings += r["bindings"]
        secs += r["seconds"]
        reps += 1
    return {"value": edges / secs / 1e9, "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": "%d of %d roots x %d repetitions (%.1f s, %d edges, %d bindings; oracle/dfs_ref.c DFS, %d "
                      "thread%s)" % (sample, nroots_total, reps, secs, edges, bindings, threads,
                                     "" if threads == 1 else "s = the job's host-core share (OMP_NUM_THREADS)"),
            "bindings_per_s": bindings / secs, "bindings_per_root": bindings / max(sample * reps, 1)}


# rows the set-based CPU path may hold at once (it writes every hop's rows: ~16 B a row and column)
SET_MAX_ROWS = 1.5e8


def set_sample(dfs, cg, query, threads, target_s, nroots_total, bindings_per_root):
    """oracle/set_ref.c (the device's algebra on the host cores: per hop the distinct sources' filtered
    lists once, then every row written) over the whole root set when it fits ≈ target_s / 3 per run, else a
    bounded root sample; repeated until ≈ target_s is timed. The sample is capped so that its rows
    (bindings per root from the DFS sample) stay under SET_MAX_ROWS; None when one root alone exceeds it
    (C5's 3-hop: 4e8 rows a root)."""
    cap = int(SET_MAX_ROWS / max(bindings_per_root, 1e-9))
    if cap < 1:
        return None
    try:
        probe = dfs.set_run(cg, query, nthreads=threads, root_sample=min(nroots_total, 4096, cap))
    except MemoryError:
        return None
    # an intermediate hop may write more rows than the last (a selective last hop): the sample is also
    # bounded by the probe's largest per-hop table, per root
    cap = min(cap, int(SET_MAX_ROWS / max(probe["max_rows"] / max(probe["nroots"], 1), 1e-9)))
    if cap < 1:
        return None
    per_root = max(probe["seconds"] / max(probe["nroots"], 1), 1e-9)
    sample = int(min(nroots_total, cap, max(4096, target_s / 3 / per_root)))
    edges = bindings = 0
    secs = 0.0
    reps = 0
    while secs < target_s and reps < 1000:
        try:
            r = dfs.set_run(cg, query, nthreads=threads, root_sample=sample)
        except MemoryError:
            return None
        if reps:  # the first run pays the buffers' first touch
            edges += r["edges"]
            bindings += r["bindings"]
            secs += r["seconds"]
        reps += 1
    return {"value": edges / secs / 1e9, "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": "%d of %d roots x %d timed repetitions (%.1f s, %d edges, %d rows written; oracle/set_ref.c "
                      "set-at-a-time: distinct sources' filtered lists, then the rows, %d threads)" % (
                          sample, nroots_total, reps - 1, secs, edges, bindings, threads),
            "bindings_per_s": bindings / secs}


def reduce_over_ranks(dist, dt, edges, bindings, rows):
    """Whole-job totals from per-rank step statistics: time = MAX over ranks (the slowest rank ends the
    job), edges/bindings/rows = SUM (roots are sharded v % N == rank, so every root's rows live on
    exactly one rank and the per-rank results are disjoint). dist=None → single process."""
    if dist is None:
        return float(dt), float(edges), float(bindings), float(rows)
    import torch
    t = torch.tensor([float(dt)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(edges), float(bindings), float(rows)], dtype=torch.float64)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return t.item(), s[0].item(), s[1].item(), s[2].item()


def with_heartbeat(label, fn, every=20.0):
    """Run fn() while a child process prints a progress line to stderr every `every` s (a long
    RMAT-26 build would otherwise look hung to a silence watchdog; a child is immune to the GIL)."""
    import subprocess
    code = ("import sys, time\nt0 = time.time()\nwhile True:\n    time.sleep(%f)\n"
            "    print('[bench] %s: %%.0f s' %% (time.time() - t0), file=sys.stderr, flush=True)\n" % (every, label))
    hb = subprocess.Popen([sys.executable, "-c", code])
    try:
        return fn()
    finally:
        hb.kill()
        hb.wait()


def measured_traffic(args, dom, default_scale, world):
    """HBM bytes per launch of the dominant kernel from the committed PMC passes (tools/pmc_traffic.py
    writes profiles/traffic.json) — only for the exact default workload they were collected on."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "traffic.json")
    if world != 1 or args.count or str(args.scale) != str(default_scale) or not os.path.exists(path):
        return None
    rec = json.load(open(path)).get(args.query)
    return rec if rec and rec.get("kernel") == dom else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", default=None, help="RMAT scale or 'ldbc' (default: the query's config)")
    ap.add_argument("--query", default="m1", choices=sorted(QUERIES))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--count", action="store_true", help="COUNT mode (the last hop counts its rows)")
    ap.add_argument("--no-deliver", action="store_true", help="skip the RID map + D2H hand-over measurement")
    ap.add_argument("--replicated", action="store_true",
                    help="N > 1: replicate the graph and shard roots (weak scaling) instead of 1-D partitioning it")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of N ranks on a one-GPU box: every rank on that device (the driver's runs leave it unset)
    local = int(os.environ.get("OMX_BENCH_DEVICE", local))
    import orientdb_amd as o  # loads libomx (and the system HIP runtime) before torch

    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    workload, query, default_scale = QUERIES[args.query]
    if args.scale is None:
        args.scale = default_scale
    partitioned = world > 1 and not args.replicated and args.query not in REPLICATED_ONLY and args.scale != "ldbc"
    query, scaling = scaled_query(args.query, query, world, partitioned)
    t_build = time.perf_counter()
    keep = (rank == 0 and world == 1 and not args.no_cpu_baseline) or "{hub}" in query
    comm = None
    if args.scale == "ldbc":
        g = o.GraphSnapshot.ldbc_like(device=local, keep_csr=keep, **LDBC_SF10)
        graph_desc = {"graph": "LDBC-SNB-like Knows (gen.cpp omx_ldbc_knows_generate)", **LDBC_SF10}
    elif partitioned and world > 1:
        # every rank generates and uploads only the rows it owns; the RCCL unique id travels over gloo
        args.scale = int(args.scale)
        g = with_heartbeat("graph build", lambda: o.GraphSnapshot.rmat(args.scale, device=local,
                                                                        partition=(rank, world)))
        uid = [o.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = o.Comm.rccl(rank, world, local, uid[0])
        graph_desc = {"graph": "RMAT, 1-D partitioned (block of ceil(V/N) vertices per GPU)", "scale": args.scale,
                      "edge_factor": 16, "rows_owned": list(g.part)}
    else:
        args.scale = int(args.scale)
        erec = args.query in EDGE_RECORDS
        g = with_heartbeat("graph build", lambda: o.GraphSnapshot.rmat(args.scale, device=local, keep_csr=keep,
                                                                        edge_records=erec))
        graph_desc = {"graph": "RMAT" + (" with edge records (field w)" if erec else ""), "scale": args.scale,
                      "edge_factor": 16}
    t_build = time.perf_counter() - t_build
    if "{hub}" in query:  # the vertex of highest out-degree (lowest id on ties)
        import numpy as np
        deg = np.diff(g.csr[0].astype(np.int64))
        query = query.replace("{hub}", str(int(np.argmax(deg))))
        query = query.replace("{leaf}", str(int(np.argmax(deg == 1))))
    st = o.OMatchStatement(query)
    flags = o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING | o.OMX_FLAG_TIME_HOT
    mode = o.OMX_MODE_COUNT if (args.query in COUNT_MODE or args.count) else o.OMX_MODE_MATERIALIZE
    # replicated graph: roots sharded v % N == rank; partitioned: each rank starts from the roots it owns
    shard = (0, 1) if comm is not None else (rank, world)
    run_kw = dict(flags=flags, shard=shard, documents=False, mode=mode, comm=comm)
    wrs = None
    for _ in range(args.warmup):
        wrs = st.execute(g, **run_kw)
    # the timed steps record their dominant kernel only (two HIP events a launch, OMX_TIME_ONLY): the hot
    # kernel with the most device time in the last warmup execution, where every hot kernel was timed
    hot = {k["name"]: k["ms"] for k in wrs.kernel_stats if k["name"] in HOT_KERNELS} if wrs is not None else {}
    if hot:
        os.environ["OMX_TIME_ONLY"] = max(hot, key=hot.get)
    barrier()
    hip_sync()
    t0 = time.perf_counter()
    infos = []
    kst = {}
    step_launches = []
    for _ in range(args.steps):
        rs = st.execute(g, **run_kw)
        infos.append(rs.info)
        step_launches.append(rs.kernel_launches)
        for k in rs.kernel_stats:
            a = kst.setdefault(k["name"], {"launches": 0, "ms": 0.0, "alg_bytes": 0})
            a["launches"] += k["launches"]
            a["ms"] += k["ms"]
            a["alg_bytes"] += k["alg_bytes"]
    hip_sync()
    barrier()
    dt = time.perf_counter() - t0
    os.environ.pop("OMX_TIME_ONLY", None)
    # one more execution, untimed by the step clock, with every instrumented kernel timed: the
    # algorithmic bytes of a whole step (SURVEY §8(d) per kernel; spans that wrap other records or move
    # no HBM bytes excluded) for the step-level roofline
    prof = st.execute(g, **dict(run_kw, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING))
    step_bytes = sum(k["alg_bytes"] for k in prof.kernel_launches if k["name"] not in SPAN_RECORDS)
    step_kernel_ms = sum(k["ms"] for k in prof.kernel_launches if k["name"] not in SPAN_RECORDS)
    deliver = None
    if world == 1 and mode == o.OMX_MODE_MATERIALIZE and not args.no_deliver and not infos[-1]["documents"]:
        # the dense → RID map and the D2H hand-over of the rows, reported apart from the
        # step: executions without KEEP_DEVICE (the rows mapped to RIDs on the device chunk by chunk and
        # copied by DMA into libomx's pooled pinned host block, as an OResultSet fill would read them).
        # The first one pins the block (cold); the second reuses it (steady state, the reported wall_ms).
        walls = []
        for _ in range(2):
            t1 = time.perf_counter()
            d = st.execute(g, **dict(run_kw, flags=o.OMX_FLAG_KERNEL_TIMING, fetch_rows=False))
            walls.append((time.perf_counter() - t1) * 1e3)
            ks = {k["name"]: k for k in d.kernel_stats}
            info = d.info
            del d
        wall = walls[-1]
        nrows, ncols = info["n_rows"], info["n_cols"]
        mp, d2h = ks.get("k_map_rids", {"ms": 0.0}), ks.get("deliver_d2h", {"ms": 0.0})
        deliver = {"rows": nrows, "cols": ncols, "bytes": nrows * ncols * 8, "wall_ms": wall,
                   "first_wall_ms": walls[0], "map_rids_ms": mp["ms"], "d2h_ms": d2h["ms"],
                   "d2h_GBps": nrows * ncols * 8 / (d2h["ms"] / 1e3) / 1e9 if d2h["ms"] > 0 else None,
                   "host_rows_bytes": info["host_rows_bytes"], "host_rows_pinned": bool(info["host_rows_pinned"]),
                   "note": "executions outside the timed steps without OMX_FLAG_KEEP_DEVICE: rows mapped to u64 "
                           "RIDs on the device in chunks (k_map_rids) and copied by DMA into a pooled pinned host "
                           "block, chunk i+1's map under chunk i's copy (deliver_d2h spans both); wall_ms is the "
                           "whole execute including the step, on the second execution (the block reused); "
                           "first_wall_ms includes pinning the block"}
    edges = sum(i["edges_traversed"] for i in infos)
    edges_read = sum(i["edges_read"] for i in infos)
    bindings = sum(i["bindings"] for i in infos)
    rows = infos[-1]["n_rows"]
    dt_max, edges_all, bindings_all, rows_all = reduce_over_ranks(dist, dt, edges, bindings, rows)
    edges_read_all = reduce_over_ranks(dist, dt, edges_read, 0, 0)[1]
    step_bytes_all = reduce_over_ranks(dist, dt, step_bytes, 0, 0)[1]
    if comm is not None:
        comm.close()
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    # the dominant kernel: the hot-path kernel with the most device time
    cands = {k: v for k, v in kst.items() if k in HOT_KERNELS}
    dom = max(cands, key=lambda k: cands[k]["ms"]) if cands else "k_expand_heavy"
    exp = cands.get(dom, {"launches": 1, "ms": 0.0, "alg_bytes": 0})
    # the dominant kernel launch by launch: slot j = its j-th launch in a step (M1: the first hop, then
    # the row emission); the roofline is taken on the slot with the most device time, averaged over the
    # timed steps, so achieved = that launch's algorithmic bytes ÷ its duration
    per_step = [[k for k in sl if k["name"] == dom] for sl in step_launches]
    nslots = min((len(x) for x in per_step), default=0)
    slots = [{"ms": sum(x[j]["ms"] for x in per_step) / len(per_step),
              "alg_bytes": sum(x[j]["alg_bytes"] for x in per_step) / len(per_step),
              "hbm_bytes": sum(x[j].get("hbm_bytes", x[j]["alg_bytes"]) for x in per_step) / len(per_step)}
             for j in range(nslots)]
    main_slot = max(range(nslots), key=lambda j: slots[j]["ms"]) if nslots else None
    if main_slot is not None and slots[main_slot]["ms"] > 0:
        launch = slots[main_slot]
    else:
        launch = {"ms": exp["ms"] / max(exp["launches"], 1), "alg_bytes": exp["alg_bytes"] / max(exp["launches"], 1)}
        launch["hbm_bytes"] = launch["alg_bytes"]
    achieved = launch["alg_bytes"] / (launch["ms"] / 1e3) / 1e9 if launch["ms"] > 0 else 0.0
    # the bytes HBM must move at least (each distinct byte once: a factorized hop's lists and a pull
    # level's frontier masks are re-read from L2 by the rows / in-edges sharing them) per launch time
    hbm_gbs = launch["hbm_bytes"] / (launch["ms"] / 1e3) / 1e9 if launch["ms"] > 0 else 0.0
    ms_step = dt_max / args.steps * 1e3
    out = {
        "metric": METRIC,
        "value": edges_all / dt_max / 1e9,
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (%s, deterministic splitmix64 generator in libomx)" % graph_desc["graph"],
        "config": {"workload": workload, "query": query, **graph_desc,
                   "V": g.V, "E": g.n_edges, "rows_per_step": int(rows_all),
                   "edges_per_step": int(edges_all / args.steps), "bindings_per_step": int(bindings_all / args.steps),
                   # adjacency entries a kernel iterated (omx_result_info.edges_read): E_t minus a COUNT
                   # run's unfiltered last hop (summed from degrees) and minus the E_t of cycle-closing
                   # checks answered by binary search (E_t per SURVEY §8(d) still counts both)
                   "edges_read_per_step": int(edges_read_all / args.steps),
                   "parallelism": ("1-D partitioned graph over %d GPUs, rows exchanged per hop (RCCL all-to-all)"
                                   % world) if comm is not None else
                                  ("1 GPU" if world == 1 else
                                   "roots sharded v%%N across %d GPUs, graph replicated" % world),
                   "mode": "count" if mode == o.OMX_MODE_COUNT else "materialize (rows kept in HBM)",
                   "graph_build_s": round(t_build, 2)},
        "bindings_per_s": bindings_all / dt_max,
        # distinct result rows (documents for RETURN expressions) per second
        "rows_per_s": rows_all * args.steps / dt_max,
        # adjacency entries the kernels actually iterated per second (GTEPS counts E_t)
        "read_rate": {"value": edges_read_all / dt_max / 1e9, "unit": "G adjacency entries read/s"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "launch": ("launch %d of %d per step (the one with the most device time)" % (main_slot + 1, nslots)
                                if main_slot is not None else "all launches"),
                     "alg_bytes_per_launch": launch["alg_bytes"], "avg_launch_ms": launch["ms"],
                     # achieved/frac count SURVEY §8(d)'s algorithmic bytes, L2 re-reads included; hbm_frac
                     # counts each distinct byte once; pmc_frac is the measured PMC traffic (below)
                     "hbm_bytes_per_launch": launch["hbm_bytes"], "hbm_achieved": hbm_gbs,
                     "hbm_frac": hbm_gbs / HBM_PEAK_GBS, "pmc_frac": None,
                     "launches_per_step": slots,
                     "kernel_total": {"alg_bytes_per_step": exp["alg_bytes"] / args.steps,
                                      "ms_per_step": exp["ms"] / args.steps},
                     # whole step: Σ algorithmic bytes of every instrumented kernel of one execution ÷ the
                     # step wall time ÷ the HBM peak of the GPUs taking part
                     "step_alg_bytes": step_bytes_all, "step_kernel_ms": step_kernel_ms,
                     "step_frac": step_bytes_all / (ms_step / 1e3) / 1e9 / (HBM_PEAK_GBS * world),
                     "traffic": None},
        # every instrumented kernel of one execution after the timed steps (those time their dominant
        # kernel only)
        "kernels": {k["name"]: {"launches": k["launches"], "ms_per_step": k["ms"],
                                "GBps": (k["alg_bytes"] / (k["ms"] / 1e3) / 1e9) if k["ms"] > 0 else None}
                    for k in sorted(prof.kernel_stats, key=lambda k: -k["ms"])},
        "cpu_baseline": None,
        "deliver": deliver,
    }
    tr = measured_traffic(args, dom, default_scale, world)
    if tr is not None:
        out["roofline"]["traffic"] = tr["bytes_per_launch"]
        out["roofline"]["traffic_source"] = tr["source"] + " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, per launch)"
        if launch["ms"] > 0:  # the PMC pass's bytes over this run's launch time
            out["roofline"]["pmc_frac"] = tr["bytes_per_launch"] / (launch["ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(g, query, args.cpu_seconds, single_thread_too=args.query == "c1")
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
