"""Probe: two processes on ONE GPU driving the partitioned MATCH through RCCL (world 2).

RCCL may refuse two ranks on one device; the probe reports that instead of failing. When it runs,
both ranks' rows are checked against a single-snapshot run of the same query.
usage: python tools/rccl_two_ranks.py
"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
Q = "MATCH {class:Person,as:a,where:(age < 5)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c"


def worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import orientdb_amd as o
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        uid = [o.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        part = o.GraphSnapshot.rmat(12, device=0, partition=(rank, world))
        comm = o.Comm.rccl(rank, world, 0, uid[0])
        rs = o.OMatchStatement(Q).execute(part, comm=comm, documents=False)
        rows = [tuple(int(x) for x in r) for r in rs.rows]
        g = [None] * world
        dist.all_gather_object(g, rows)
        if rank == 0:
            out.put(("ok", g))
        comm.close()
    except Exception as e:  # noqa: BLE001
        out.put(("error", "rank %d: %s" % (rank, e)))
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    status, payload = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
    if status != "ok":
        print("RCCL two ranks on one GPU: not available here:", payload)
        return
    import orientdb_amd as o
    full = o.OMatchStatement(Q).execute(o.GraphSnapshot.rmat(12, device=0), documents=False)
    want = {tuple(int(x) for x in r) for r in full.rows}
    got = set().union(*[set(x) for x in payload])
    print("RCCL two ranks on one GPU: rows %d/%d, equal=%s" % (len(got), len(want), got == want))
    assert got == want


if __name__ == "__main__":
    main()
