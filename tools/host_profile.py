"""Where the host time of a bench step goes: cProfile over repeated executes of the C2 statement on
RMAT-22 (development aid; run on the GPU box)."""
import cProfile
import pstats
import sys
import time

sys.path.insert(0, ".")
import orientdb_amd as o  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
g = o.GraphSnapshot.rmat(scale, device=0)
q = ("MATCH {class:Person,as:a,where:(age < 1)}-Knows->{as:b}-Knows->{as:c,where:(age >= 90)} "
     "RETURN a,b,c")
st = o.OMatchStatement(q)
kw = dict(flags=o.OMX_FLAG_KEEP_DEVICE | o.OMX_FLAG_KERNEL_TIMING | o.OMX_FLAG_TIME_HOT, documents=False)
for _ in range(3):
    st.execute(g, **kw)
n = 20
t = time.perf_counter()
for _ in range(n):
    st.execute(g, **kw)
print("ms per execute %.3f" % ((time.perf_counter() - t) / n * 1e3))
pr = cProfile.Profile()
pr.enable()
for _ in range(n):
    st.execute(g, **kw)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
