"""The partitioned MATCH across PROCESSES: `world` processes, each holding one 1-D
partition of the same RMAT graph on the box's GPU, joined by torch.distributed gloo through
orientdb_amd.dist.host_comm (include/omx/match.h omx_comm_create_host). Every routed hop's count exchange
and all-to-all-v of the binding columns crosses process boundaries — the routing code the RCCL transport
runs, with the bytes staged through host memory instead of xGMI. The ranks' shares must add up to the
unpartitioned run: rows, the additive digest of the distinct rows, E_t and the COUNT-mode rows."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.test_gpu_parity import RMAT_QUERIES

pytestmark = pytest.mark.gpu

IDS = ("c2_both_ends", "c1_fof", "two_cols_dedup", "in_dir", "both_dir", "three_hop", "triangle", "paths",
       "bound_candidate", "matches")
QUERIES = [(q[0], q[1]) for q in RMAT_QUERIES if q[0] in IDS]
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_host_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, scale, queries):
    port = _port()
    procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(world), str(port), str(scale), json.dumps(queries)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=150)
            assert p.returncode == 0, err[-3000:]
            outs.append([json.loads(x) for x in out.splitlines() if x.startswith("{")])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.mark.parametrize("world", [2, 3])
def test_processes_over_host_collectives(world):
    import orientdb_amd as o
    scale = 10
    g = o.GraphSnapshot.rmat(scale, device=0)
    outs = _run(world, scale, QUERIES)
    assert all(len(x) == len(QUERIES) for x in outs)
    for i, (name, q) in enumerate(QUERIES):
        ref = o.OMatchStatement(q).execute(g, flags=o.OMX_FLAG_DIGEST | o.OMX_FLAG_KEEP_DEVICE, documents=False)
        refc = o.OMatchStatement(q).execute(g, mode=o.OMX_MODE_COUNT, flags=o.OMX_FLAG_KEEP_DEVICE, documents=False)
        shares = [x[i] for x in outs]
        assert all(s["name"] == name for s in shares)
        assert sum(s["rows"] for s in shares) == ref.info["n_rows"], name
        assert sum(s["digest"] for s in shares) % (1 << 64) == ref.info["digest"], name
        assert sum(s["edges"] for s in shares) == ref.info["edges_traversed"], name
        assert sum(s["count_rows"] for s in shares) == refc.info["n_rows"], name
