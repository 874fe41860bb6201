"""Ridbag ingest throughput: RMAT-<scale> out-bags written as embedded ridbag streams (the record
serializer's bytes), decoded on the device by omx_ridbag_decode_csr. Prints one JSON line: entries,
stream bytes, wall time of the decode call (host → device copies included: the boundary hands over host
buffers) and the decoded CSR's equality with the source. Run under `rocprofv3 --kernel-trace --stats`
for the kernels' own times (k_bag_count, k_bag_decode).

usage: python tools/ridbag_bench.py [--scale 22] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def streams_of(rp, col, cluster=11):
    """[cfg=1][count BE32][(cluster BE16, position BE64) × count] per vertex, vectorised."""
    V = len(rp) - 1
    deg = np.diff(rp.astype(np.int64))
    offs = np.zeros(V + 1, np.uint64)
    offs[1:] = np.cumsum(5 + 10 * deg)
    blob = np.zeros(int(offs[-1]), np.uint8)
    starts = offs[:-1].astype(np.int64)
    blob[starts] = 1
    cnt = deg.astype(">u4").view(np.uint8).reshape(V, 4)
    for k in range(4):
        blob[starts + 1 + k] = cnt[:, k]
    base = np.repeat(starts + 5, deg) + 10 * (np.arange(len(col)) - np.repeat(rp[:-1].astype(np.int64), deg))
    blob[base + 1] = cluster
    pos = col.astype(">u8").view(np.uint8).reshape(-1, 8)
    for k in range(8):
        blob[base + 2 + k] = pos[:, k]
    return blob.tobytes(), offs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from orientdb_amd.graph import rmat_csr
    from orientdb_amd.ridbag import decode_ridbag_blob
    rp, col = rmat_csr(a.scale, seed=2)
    V = len(rp) - 1
    blob, offs = streams_of(rp, col)
    vr = (np.uint64(11) << np.uint64(48)) | np.arange(V, dtype=np.uint64)
    decode_ridbag_blob(blob, offs, vr)  # warm-up (context, allocations)
    times = []
    ok = True
    for _ in range(a.reps):
        t0 = time.perf_counter()
        grp, gcol = decode_ridbag_blob(blob, offs, vr)
        times.append(time.perf_counter() - t0)
        ok = ok and np.array_equal(gcol, col) and np.array_equal(grp, rp.astype(np.uint64))
    best = min(times)
    print(json.dumps({"scale": a.scale, "vertices": V, "entries": int(len(col)), "stream_bytes": len(blob),
                      "decode_wall_s": best, "entries_per_s_pcie_inclusive": len(col) / best, "csr_equal": bool(ok)}))


if __name__ == "__main__":
    main()
