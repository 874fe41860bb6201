"""Host time of one bench step outside the device work: omx_execute's call, the Python result read-out
(_collect) and omx_result_free, per phase (`python3 tools/hostgap.py [query] [steps]`)."""
import ctypes as C
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import bench  # noqa: E402
import orientdb_amd as o
from orientdb_amd import _native as N


def main():
    q = sys.argv[1] if len(sys.argv) > 1 else "m1"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    desc, query, scale = bench.QUERIES[q][:3]
    g = o.GraphSnapshot.rmat(scale, device=0) if isinstance(scale, int) else o.GraphSnapshot.ldbc_like(device=0)
    st = o.OMatchStatement(query)
    flags = o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING | o.OMX_FLAG_TIME_HOT
    if len(sys.argv) > 3 and sys.argv[3] == "untimed":  # no HIP events at all
        flags = o.OMX_FLAG_KEEP_DEVICE
    for _ in range(3):
        st.execute(g, flags=flags, documents=False)
    L = N.lib()
    for _ in range(steps):
        t0 = time.perf_counter()
        arr, n = o.match._values((), {})
        opt = N.omx_exec_options()
        L.omx_exec_options_init(C.byref(opt))
        opt.flags = flags
        opt.shard_world = 1
        r = C.c_void_p()
        t1 = time.perf_counter()
        N.check(L.omx_execute(g.handle, st._h, C.byref(opt), C.byref(r)))
        t2 = time.perf_counter()
        rs = o.OMatchStatement._collect(r, False)
        t3 = time.perf_counter()
        L.omx_result_free(r)
        t4 = time.perf_counter()
        print("prep %.3f  execute %.3f  collect %.3f (%d launches)  free %.3f ms" % (
            (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, len(rs.kernel_launches), (t4 - t3) * 1e3), flush=True)


if __name__ == "__main__":
    main()
