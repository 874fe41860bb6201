"""Communicators of a 1-D partitioned MATCH (include/omx/match.h).

A partitioned snapshot (GraphSnapshot.rmat(..., partition=(rank, world))) holds the CSR rows of the
vertices one rank owns. OMatchStatement.execute(graph, comm=c) then routes binding rows between the
ranks before every step that reads an adjacency (and by tuple hash before a distinct projection); each
rank returns its share of the rows.

  Comm.rccl(rank, world, device, uid)   one process per GPU, RCCL over xGMI; uid = Comm.unique_id()
                                        made on one rank and shared (e.g. torch.distributed over gloo)
  Comm.threads(world)                   `world` ranks that are threads of this process (one GPU is
                                        enough): the exchange is device-to-device copies
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
