"""One rank of a multi-process partitioned MATCH over host collectives (tests/test_gpu_dist_host.py):
`python tests/dist_host_worker.py RANK WORLD PORT SCALE QUERIES_JSON` joins a gloo group on 127.0.0.1,
builds its RMAT partition on cuda:0, executes every query through orientdb_amd.dist.host_comm and prints
one JSON line per query: its share's rows, digest (OMX_FLAG_DIGEST, additive over disjoint shares),
E_t and bindings, plus the COUNT-mode rows."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world, port, scale = (int(x) for x in sys.argv[1:5])
    queries = json.loads(sys.argv[5])
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import orientdb_amd as o
    from orientdb_amd.dist import host_comm
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = o.GraphSnapshot.rmat(scale, device=0, partition=(rank, world))
    comm = host_comm(rank, world)
    for name, q in queries:
        rs = o.OMatchStatement(q).execute(g, comm=comm, flags=o.OMX_FLAG_DIGEST | o.OMX_FLAG_KEEP_DEVICE,
                                          documents=False)
        rc = o.OMatchStatement(q).execute(g, comm=comm, mode=o.OMX_MODE_COUNT, flags=o.OMX_FLAG_KEEP_DEVICE,
                                          documents=False)
        print(json.dumps({"name": name, "rows": rs.info["n_rows"], "digest": rs.info["digest"],
                          "edges": rs.info["edges_traversed"], "bindings": rs.info["bindings"],
                          "count_rows": rc.info["n_rows"]}), flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
