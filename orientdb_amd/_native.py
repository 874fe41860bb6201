"""ctypes binding of include/omx/match.h (orientdb_amd/_lib/libomx.so).

The shared library is the product: every MATCH executed through this package runs in its HIP
kernels. There is no Python or CPU fallback; a missing library raises immediately.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OMX_LIB: an alternative build of the same library (A/B experiments under tools/)
LIB_PATH = os.environ.get("OMX_LIB") or os.path.join(_HERE, "_lib", "libomx.so")

OMX_OK, OMX_E_UNSUPPORTED, OMX_E_INVALID, OMX_E_OOM, OMX_E_DEVICE, OMX_E_PARSE, OMX_E_EXECUTION = range(7)
OMX_PROP_INT32, OMX_PROP_INT64, OMX_PROP_DOUBLE, OMX_PROP_STRING, OMX_PROP_BOOL = 1, 2, 3, 4, 5
OMX_VAL_NULL, OMX_VAL_INT, OMX_VAL_DOUBLE, OMX_VAL_STRING, OMX_VAL_BOOL = 0, 1, 2, 3, 4
OMX_MODE_MATERIALIZE, OMX_MODE_COUNT = 0, 1
OMX_FLAG_KERNEL_TIMING, OMX_FLAG_NO_RID_MAP, OMX_FLAG_KEEP_DEVICE, OMX_FLAG_TIME_HOT, OMX_FLAG_DIGEST = 1, 2, 4, 8, 16


class omx_class_desc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("superclass", C.c_int32), ("is_edge_class", C.c_int32),
                ("cluster_id", C.c_int32)]


class omx_edge_set_desc(C.Structure):
    _fields_ = [("edge_class", C.c_int32), ("n_edges", C.c_uint64),
                ("out_row_ptr", C.POINTER(C.c_uint64)), ("out_col", C.POINTER(C.c_uint32)),
                ("in_row_ptr", C.POINTER(C.c_uint64)), ("in_col", C.POINTER(C.c_uint32)), ("n_in_edges", C.c_uint64),
                ("edge_rids", C.POINTER(C.c_uint64)), ("in_edge_index", C.POINTER(C.c_uint64))]


class omx_property_desc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", C.c_int32), ("values", C.c_void_p),
                ("present", C.POINTER(C.c_uint8)), ("dict_size", C.c_int32), ("dict", C.POINTER(C.c_char_p))]


class omx_index_desc(C.Structure):
    _fields_ = [("class_id", C.c_int32), ("property", C.c_char_p), ("unique", C.c_int32)]


class omx_graph_desc(C.Structure):
    _fields_ = [("n_vertices", C.c_uint32), ("n_classes", C.c_int32), ("classes", C.POINTER(omx_class_desc)),
                ("vertex_class", C.POINTER(C.c_uint16)), ("rids", C.POINTER(C.c_uint64)),
                ("n_edge_sets", C.c_int32), ("edge_sets", C.POINTER(omx_edge_set_desc)),
                ("n_properties", C.c_int32), ("properties", C.POINTER(omx_property_desc)),
                ("n_indexes", C.c_int32), ("indexes", C.POINTER(omx_index_desc)), ("device", C.c_int32),
                ("part_lo", C.c_uint32), ("part_hi", C.c_uint32),
                ("n_edge_properties", C.c_int32), ("edge_properties", C.POINTER(omx_property_desc))]


class omx_value(C.Structure):
    _fields_ = [("type", C.c_int32), ("index", C.c_int32), ("name", C.c_char_p), ("i", C.c_int64),
                ("d", C.c_double), ("s", C.c_char_p)]


class omx_exec_options(C.Structure):
    _fields_ = [("mode", C.c_int32), ("flags", C.c_int32), ("limit", C.c_int64), ("shard_rank", C.c_int32),
                ("shard_world", C.c_int32), ("params", C.POINTER(omx_value)), ("n_params", C.c_int32),
                ("comm", C.c_void_p)]


class omx_result_info(C.Structure):
    _fields_ = [("n_rows", C.c_uint64), ("n_cols", C.c_int32), ("deduplicated", C.c_int32),
                ("edges_traversed", C.c_uint64), ("bindings", C.c_uint64), ("alg_bytes", C.c_uint64),
                ("device_ms", C.c_double), ("total_ms", C.c_double), ("edges_read", C.c_uint64),
                ("digest", C.c_uint64), ("documents", C.c_int32), ("factorized_hops", C.c_int32),
                ("rows_gathered", C.c_uint64), ("host_rows_bytes", C.c_uint64), ("host_rows_pinned", C.c_int32),
                ("reserved0", C.c_int32)]


OMX_NULL_RID = (1 << 64) - 1  # a null binding (unmatched optional node)
OMX_CELL_NULL, OMX_CELL_INT, OMX_CELL_DOUBLE, OMX_CELL_STRING, OMX_CELL_BOOL, OMX_CELL_RID, OMX_CELL_LIST, \
    OMX_CELL_MAP = range(8)


class omx_cell(C.Structure):
    _fields_ = [("type", C.c_int32), ("n", C.c_int32), ("i", C.c_int64), ("d", C.c_double), ("rid", C.c_uint64),
                ("s", C.c_char_p)]


# every exported symbol of include/omx/match.h: name -> (restype, argtypes)
SIGNATURES = {
    "omx_graph_create": (C.c_int, [C.POINTER(omx_graph_desc), C.POINTER(C.c_void_p)]),
    "omx_graph_destroy": (None, [C.c_void_p]),
    "omx_graph_class_count": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_uint64)]),
    "omx_graph_device_bytes": (C.c_uint64, [C.c_void_p]),
    "omx_statement_parse": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "omx_statement_free": (None, [C.c_void_p]),
    "omx_statement_explain": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(omx_value), C.c_int32, C.c_char_p,
                                        C.c_size_t]),
    "omx_exec_options_init": (None, [C.POINTER(omx_exec_options)]),
    "omx_execute": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(omx_exec_options), C.POINTER(C.c_void_p)]),
    "omx_result_info_get": (C.c_int, [C.c_void_p, C.POINTER(omx_result_info)]),
    "omx_result_column_name": (C.c_char_p, [C.c_void_p, C.c_int32]),
    "omx_result_rows": (C.POINTER(C.c_uint64), [C.c_void_p]),
    "omx_result_kernel_stat": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_char_p), C.POINTER(C.c_int64),
                                         C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "omx_result_kernel_launch": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                                          C.POINTER(C.c_uint64)]),
    "omx_result_kernel_launch_bytes": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "omx_result_free": (None, [C.c_void_p]),
    "omx_result_cell": (C.c_int, [C.c_void_p, C.c_uint64, C.c_int32, C.POINTER(omx_cell)]),
    "omx_result_column": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]),
    "omx_graph_create_blob": (C.c_int, [C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "omx_execute_packed": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                     C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_void_p)]),
    "omx_last_error": (C.c_char_p, []),
    "omx_version": (C.c_char_p, []),
    "omx_rmat_generate": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int32,
                                    C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)),
                                    C.POINTER(C.c_uint64)]),
    "omx_ldbc_knows_generate": (C.c_int, [C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.POINTER(C.c_uint64)),
                                          C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64)]),
    "omx_csr_transpose": (C.c_int, [C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                    C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32))]),
    "omx_synthetic_int_column": (C.c_int, [C.c_uint32, C.c_uint64, C.c_int32, C.POINTER(C.POINTER(C.c_int32))]),
    "omx_host_free": (None, [C.c_void_p]),
    "omx_rmat_generate_part": (C.c_int, [C.c_int32, C.c_int32, C.c_uint64, C.c_int32, C.c_uint32, C.c_uint32,
                                         C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)),
                                         C.POINTER(C.c_uint64), C.POINTER(C.POINTER(C.c_uint64)),
                                         C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64)]),
    "omx_rmat_generate_dev": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_uint64, C.c_int32,
                                        C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)),
                                        C.POINTER(C.c_uint64)]),
    "omx_rmat_generate_part_dev": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.c_uint64, C.c_int32, C.c_uint32,
                                             C.c_uint32, C.POINTER(C.POINTER(C.c_uint64)),
                                             C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_uint64),
                                             C.POINTER(C.POINTER(C.c_uint64)), C.POINTER(C.POINTER(C.c_uint32)),
                                             C.POINTER(C.c_uint64)]),
    "omx_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "omx_comm_create_rccl": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.POINTER(C.c_void_p)]),
    "omx_comm_create_threads": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    "omx_comm_create_host": (C.c_int, [C.c_int32, C.c_int32, C.c_void_p, C.POINTER(C.c_void_p)]),
    "omx_comm_rank": (C.c_int32, [C.c_void_p]),
    "omx_comm_world": (C.c_int32, [C.c_void_p]),
    "omx_comm_destroy": (None, [C.c_void_p]),
    "omx_ridbag_decode_csr": (C.c_int, [C.c_int32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32,
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64)]),
    "omx_ridbag_decode_csr_ex": (C.c_int, [C.c_int32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32,
                                           C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                           C.c_uint64, C.c_void_p, C.c_int32, C.c_uint32, C.POINTER(C.c_uint64),
                                           C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "omx_ridbag_decode_edges": (C.c_int, [C.c_int32, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64), C.c_uint32,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                          C.c_uint64, C.c_void_p, C.c_int32, C.c_uint32, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
}


class omx_bonsai_file(C.Structure):
    _fields_ = [("file_id", C.c_int64), ("pages", C.c_void_p), ("n_pages", C.c_uint64)]
OMX_COMM_ID_BYTES = 128

_lib = None


def lib():
    """The loaded libomx.so. Raises if the extension was not built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("orientdb_amd native library missing: %s — run __graft_entry__.build() "
                              "(make -C orientdb_amd/csrc)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class OmxError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (omx status %d)" % (msg, code))
        self.code = code


class OmxUnsupported(OmxError):
    """OMX_E_UNSUPPORTED: valid MATCH the device engine does not execute (the reference executor
    would run it instead)."""


class OmxParseError(OmxError):
    """OCommandSQLParsingException."""


class OmxExecutionError(OmxError):
    """OCommandExecutionException."""


def check(code):
    if code == OMX_OK:
        return
    msg = lib().omx_last_error().decode("utf-8", "replace")
    cls = {OMX_E_UNSUPPORTED: OmxUnsupported, OMX_E_PARSE: OmxParseError,
           OMX_E_EXECUTION: OmxExecutionError}.get(code, OmxError)
    raise cls(code, msg)
