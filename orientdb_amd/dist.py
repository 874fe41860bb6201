"""Communicators of a 1-D partitioned MATCH (include/omx/match.h).

A partitioned snapshot (GraphSnapshot.rmat(..., partition=(rank, world))) holds the CSR rows of the
vertices one rank owns. OMatchStatement.execute(graph, comm=c) then routes binding rows between the
ranks before every step that reads an adjacency (and by tuple hash before a distinct projection); each
rank returns its share of the rows.

  Comm.rccl(rank, world, device, uid)   one process per GPU, RCCL over xGMI; uid = Comm.unique_id()
                                        made on one rank and shared (e.g. torch.distributed over gloo)
  Comm.threads(world)                   `world` ranks that are threads of this process (one GPU is
                                        enough): the exchange is device-to-device copies
  host_comm(rank, world[, group])       one process per rank joined by torch.distributed host
                                        collectives (gloo): the exchange staged through host memory
"""
import ctypes as C

from . import _native as N


class Comm:
    def __init__(self, handle):
        self._h = handle

    @property
    def handle(self):
        if self._h is None:
            raise RuntimeError("communicator closed")
        return self._h

    @property
    def rank(self):
        return N.lib().omx_comm_rank(self.handle)

    @property
    def world(self):
        return N.lib().omx_comm_world(self.handle)

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * N.OMX_COMM_ID_BYTES)()
        N.check(N.lib().omx_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def rccl(cls, rank, world, device, uid):
        if len(uid) != N.OMX_COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be %d bytes" % N.OMX_COMM_ID_BYTES)
        buf = (C.c_uint8 * N.OMX_COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        N.check(N.lib().omx_comm_create_rccl(rank, world, device, buf, C.byref(h)))
        return cls(h)

    @classmethod
    def threads(cls, world):
        hs = (C.c_void_p * world)()
        N.check(N.lib().omx_comm_create_threads(world, hs))
        return [cls(C.c_void_p(h)) for h in hs]

    def close(self):
        if getattr(self, "_h", None) is not None:
            N.lib().omx_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- ranks joined by the caller's host collectives (omx_comm_create_host) ----------------------------
_ALLG = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)
_A2AV = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_void_p,
                    C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
_ABRT = C.CFUNCTYPE(None, C.c_void_p)


class _HostCollectives(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("allgather", _ALLG), ("alltoallv", _A2AV), ("abort", _ABRT)]


def host_comm(rank, world, group=None):
    """A communicator whose exchange runs over torch.distributed host collectives (gloo: all_gather and
    all_to_all_single of byte tensors) — one process per rank, any GPUs (one shared GPU included). The
    process group must be initialised; every rank calls this with the same world."""
    import torch
    import torch.distributed as dist

    def _bytes(addr, n):
        return torch.frombuffer((C.c_uint8 * n).from_address(addr), dtype=torch.uint8) if n else torch.empty(0, dtype=torch.uint8)

    def allgather(_ctx, send, n, recv):
        try:
            out = torch.empty(world * n, dtype=torch.uint8)
            dist.all_gather_into_tensor(out, _bytes(send, n).clone(), group=group)
            C.memmove(recv, out.data_ptr(), world * n)
            return 0
        except Exception:  # an error code, never an exception through the C frames
            return 1

    def alltoallv(_ctx, send, sc, sd, recv, rc, rd):
        try:
            scl = [int(sc[p]) for p in range(world)]
            rcl = [int(rc[p]) for p in range(world)]
            ns, nr = sum(scl), sum(rcl)
            if any(int(sd[p]) != sum(scl[:p]) for p in range(world)) or any(int(rd[p]) != sum(rcl[:p]) for p in range(world)):
                return 2  # (libomx packs the peers' parts back to back)
            out = torch.empty(nr, dtype=torch.uint8)
            dist.all_to_all_single(out, _bytes(send, ns).clone(), rcl, scl, group=group)
            if nr:
                C.memmove(recv, out.data_ptr(), nr)
            return 0
        except Exception:
            return 1

    cbs = (_ALLG(allgather), _A2AV(alltoallv), _ABRT(lambda _ctx: None))
    hc = _HostCollectives(None, *cbs)
    h = C.c_void_p()
    N.check(N.lib().omx_comm_create_host(rank, world, C.byref(hc), C.byref(h)))
    c = Comm(h)
    c._keep = (cbs, hc)  # the callbacks live as long as the communicator
    return c
