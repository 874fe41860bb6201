"""orientdb_amd — an MI355X-native (gfx950) executor for OrientDB 2.2.8 SQL MATCH.

The product is the HIP library orientdb_amd/_lib/libomx.so behind the C ABI of include/omx/match.h;
this package is its host-side mirror of the reference's command interface (see match.py).
"""
from . import _native
from ._native import (OmxError, OmxExecutionError, OmxParseError, OmxUnsupported, OMX_MODE_COUNT,
                      OMX_MODE_MATERIALIZE, OMX_FLAG_KERNEL_TIMING, OMX_FLAG_NO_RID_MAP, OMX_FLAG_KEEP_DEVICE, OMX_FLAG_TIME_HOT,
                      OMX_FLAG_DIGEST)
from .graph import (GraphSnapshot, pack_rid, unpack_rid, rmat_csr, ldbc_csr, csr_transpose, synthetic_int_column,
                    partition_range, rmat_partition)
from .dist import Comm
from .match import (GraphDatabase, OCommandSQL, OMatchStatement, OCommandExecutorSQLTraverse,
                    OCommandExecutorSQLSelectExpand, OResultSet, ODocument, ORecordId)

__all__ = ["GraphSnapshot", "GraphDatabase", "OCommandSQL", "OMatchStatement", "OCommandExecutorSQLTraverse",
           "OCommandExecutorSQLSelectExpand", "OResultSet", "ODocument",
           "ORecordId", "Comm", "partition_range", "rmat_partition", "OmxError", "OmxExecutionError", "OmxParseError", "OmxUnsupported", "pack_rid",
           "unpack_rid", "rmat_csr", "ldbc_csr", "csr_transpose", "synthetic_int_column", "OMX_MODE_COUNT",
           "OMX_MODE_MATERIALIZE", "OMX_FLAG_KERNEL_TIMING", "OMX_FLAG_NO_RID_MAP", "OMX_FLAG_KEEP_DEVICE", "OMX_FLAG_TIME_HOT",
           "OMX_FLAG_DIGEST"]


def version():
    return _native.lib().omx_version().decode()
