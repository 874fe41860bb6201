"""Probe: time the RMAT generator and the host-only snapshot at one scale, phase by phase."""
import sys
import time

sys.path.insert(0, ".")
import orientdb_amd as o  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
t = time.time()
rp, col = o.rmat_csr(scale, 16, scale)
print("generate %.1f s, E=%d" % (time.time() - t, len(col)), flush=True)
t = time.time()
trp, tcol = o.csr_transpose(1 << scale, rp, col)
print("transpose %.1f s" % (time.time() - t), flush=True)
