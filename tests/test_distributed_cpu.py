"""The N>1 path on CPU: two gloo ranks, roots sharded v % N == rank (bench.py).

Each rank runs the oracle DFS (oracle/dfs_ref.c) over its shard of the same RMAT graph and reduces its
step statistics through bench.reduce_over_ranks — the exact code the multi-GPU bench uses. Rank 0 checks
that the shards are disjoint, that their union equals the unsharded result, and that the reduced totals
equal the single-process totals. (The GPU shard path itself is covered by test_gpu_parity's shard test.)
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

QUERIES = [
    "MATCH {class:Person,as:a,where:(age < 10)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
    "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c}-Knows->{as:a} RETURN a,b,c",
]


def _graph():
    import orientdb_amd as o
    from oracle import dfs
    rp, col = o.rmat_csr(10, 16, 10)
    age = o.synthetic_int_column(1 << 10, 10 ^ 0xA9E, 100).astype(np.int64)
    return dfs.CsrGraph(rp, col, {"uid": np.arange(1 << 10, dtype=np.int64), "age": age})


def _worker(rank, world, port, q, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import bench
    from oracle import dfs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _graph()
        r = dfs.run(g, q, emit=True, shard=(rank, world))
        rows = r["rows"]
        dt, edges, bindings, nrows = bench.reduce_over_ranks(dist, r["seconds"] + rank, r["edges"], r["bindings"],
                                                             len(rows))
        gathered = [None] * world
        dist.all_gather_object(gathered, rows.tolist())
        if rank == 0:
            out.put({"dt": dt, "edges": edges, "bindings": bindings, "rows": nrows, "shards": gathered,
                     "local_dt": r["seconds"]})
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("q", QUERIES)
def test_two_rank_sharded_match(q):
    from oracle import dfs
    world = 2
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, out)) for r in range(world)]
    for p in procs:
        p.start()
    res = out.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = dfs.run(_graph(), q, emit=True)
    want = {tuple(r) for r in full["rows"].tolist()}
    shards = [{tuple(r) for r in s} for s in res["shards"]]
    assert not (shards[0] & shards[1])                       # disjoint: a row's root lives on one rank
    assert shards[0] | shards[1] == want                      # union = unsharded result
    assert all(len(s) > 0 for s in shards)
    assert res["rows"] == len(want)
    assert res["edges"] == full["edges"] and res["bindings"] == full["bindings"]
    assert res["dt"] >= 1.0                                   # MAX over ranks (rank 1 reported +1 s)


def test_reduce_single_process_is_identity():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.reduce_over_ranks(None, 0.5, 10, 20, 3) == (0.5, 10.0, 20.0, 3.0)


def test_bench_scaling_modes():
    """bench.py: N=1 runs the config verbatim; N > 1 on the (default) partitioned graph keeps the query
    (strong scaling); --replicated widens the root window N-fold (weak scaling)."""
    import bench
    assert bench.QUERIES["m1"][1] == bench.QUERIES["c2"][1] and bench.QUERIES["m1"][2] == 24
    for name in ("m1", "c2"):
        q = bench.QUERIES[name][1]
        assert bench.scaled_query(name, q, 1, False) == (q, "strong")
        assert bench.scaled_query(name, q, 8, True) == (q, "strong")
        q8, kind = bench.scaled_query(name, q, 8, False)
        assert kind == "weak" and "age < 8" in q8 and "age >= 90" in q8
    assert bench.scaled_query("c5", bench.QUERIES["c5"][1], 8, True) == (bench.QUERIES["c5"][1], "strong")


def test_bench_host_threads():
    import bench
    threads, visible = bench.host_threads()
    assert 1 <= threads <= visible
