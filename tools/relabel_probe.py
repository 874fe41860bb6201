"""Development aid (run on the GPU box): what a degree-ordered vertex relabel would give M1 / C3, measured
without changing the engine. The same RMAT graph is built twice — dense ids as generated, and dense ids
in descending in-degree order (hubs first; RIDs, uid and age travel with their vertex, so every MATCH
answers the same RID tuples) — and the metric's query runs on both: per-step time, rows, E_t and the
digest (equal by construction), plus the per-kernel times of one execution each.

usage: python tools/relabel_probe.py [scale] [steps] [query: m1|c3]
"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import orientdb_amd as o  # noqa: E402
from orientdb_amd import _native as N  # noqa: E402
from orientdb_amd.graph import RID_POS_BITS, rmat_csr, synthetic_int_column  # noqa: E402

Q = {"m1": "MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} RETURN a,b,c",
     "c3": "MATCH {class:Person,as:s,where:(uid < 64)}-Knows->{as:v, while:($depth < 4)} RETURN s, v"}


def snapshot(V, rp, col, uid, age, rids):
    classes = [("V", -1, False, 9), ("E", -1, True, 10), ("Person", 0, False, 11), ("Knows", 1, True, 12)]
    props = [{"name": "uid", "type": N.OMX_PROP_INT64, "values": uid},
             {"name": "age", "type": N.OMX_PROP_INT32, "values": age}]
    return o.GraphSnapshot(V, classes, np.full(V, 2, np.uint16), rids, [{"cls": 3, "out_rp": rp, "out_col": col}],
                           props, [], 0)


def relabel(V, rp, col):
    """new id = rank by descending in-degree (ties by old id); rows re-sorted"""
    indeg = np.bincount(col, minlength=V)
    perm = np.argsort(-indeg.astype(np.int64), kind="stable").astype(np.uint32)  # new → old
    newid = np.empty(V, np.uint32)
    newid[perm] = np.arange(V, dtype=np.uint32)
    deg = np.diff(rp.astype(np.int64))
    src_new = np.repeat(newid, deg)  # entries in old order, their new row
    key = (src_new.astype(np.uint64) << np.uint64(32)) | newid[col].astype(np.uint64)
    del src_new
    key.sort()
    ncol = (key & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    ndeg = deg[perm]
    nrp = np.zeros(V + 1, np.uint64)
    nrp[1:] = np.cumsum(ndeg)
    return perm, nrp, ncol


def run(g, q, steps):
    st = o.OMatchStatement(q)
    kw = dict(flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING | o.OMX_FLAG_TIME_HOT, documents=False)
    for _ in range(3):
        st.execute(g, **kw)
    t = time.perf_counter()
    for _ in range(steps):
        rs = st.execute(g, **kw)
    ms = (time.perf_counter() - t) / steps * 1e3
    dg = st.execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_DIGEST, documents=False)
    prof = st.execute(g, flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING, documents=False)
    ks = sorted(((k["name"], k["ms"]) for k in prof.kernel_stats), key=lambda x: -x[1])[:12]
    return ms, rs.info["n_rows"], rs.info["edges_traversed"], dg.info.get("digest"), ks


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    q = Q[sys.argv[3] if len(sys.argv) > 3 else "m1"]
    V = 1 << scale
    rp, col = rmat_csr(scale, 16, scale, True, device=0)
    age = synthetic_int_column(V, scale ^ 0xA9E, 100)
    uid = np.arange(V, dtype=np.int64)
    rids = (np.uint64(11) << np.uint64(RID_POS_BITS)) | np.arange(V, dtype=np.uint64)
    t = time.perf_counter()
    perm, nrp, ncol = relabel(V, rp, col)
    print("relabel %.1f s" % (time.perf_counter() - t), flush=True)
    for name, args in (("original", (rp, col, uid, age, rids)),
                       ("degree-ordered", (nrp, ncol, uid[perm], age[perm], rids[perm]))):
        g = snapshot(V, *args)
        ms, n, et, dg, ks = run(g, q, steps)
        print("%-15s %.3f ms/step rows %d E_t %d digest %s" % (name, ms, n, et, dg), flush=True)
        print("   " + ", ".join("%s %.3f" % k for k in ks), flush=True)
        g.close()


if __name__ == "__main__":
    main()
