/*
 * omx/match.h — C ABI of the MI355X-native OrientDB SQL MATCH executor.
 *
 * This is the drop-in boundary described in SURVEY.md §8(b). Every entry point replaces one piece of
 * the reference's MATCH execution (OrientDB 2.2.8, paths relative to /root/reference):
 *
 *   omx_graph_create        ← the record/ridbag reads the DFS performs lazily:
 *                             ORidBag.rawIterator      core/.../db/record/ridbag/ORidBag.java:160
 *                             OrientVertex.getVertices graphdb/.../blueprints/impls/orient/OrientVertex.java:401-460
 *                             ODocument.field          core/.../record/impl/ODocument.java:820
 *                             (the snapshot is built once; it is immutable afterwards)
 *   omx_statement_parse     ← OMatchStatement.parse    core/.../sql/parser/OMatchStatement.java:129-178
 *                             (assignDefaultAliases :202-218, addAliases :905-948, Pattern.validate Pattern.java:48-65)
 *   omx_statement_explain   ← estimateRootEntries :874-903 + sortEdges :272-325 (the execution plan, as JSON)
 *   omx_execute             ← OMatchStatement.execute  :244-267 → calculateMatch :334-386 → processContext :412-568
 *                             → addResult :661-729 → OBasicCommandContext.addToUniqueResult
 *                               core/.../command/OBasicCommandContext.java:347-353
 *   omx_result_*            ← OSQLSynchQuery.getResult core/.../sql/query/OSQLSynchQuery.java:111-113 (the OResultSet)
 *   omx_last_error          ← the message of OCommandExecutionException / OCommandSQLParsingException
 *
 * Conventions: plain C types only; every function returns an int status (OMX_OK = 0) unless it is
 * a getter; on failure omx_last_error() (thread-local) describes the error. OMX_E_UNSUPPORTED means
 * "valid MATCH, but not executable by this engine": the host (the Java OMatchStatement strategy) falls
 * back to the reference executor. A graph may be executed from several host threads: omx_execute
 * serialises the executions of one graph (its stream, scratch pool and adjacency caches are per graph).
 * A statement handle belongs to one thread at a time (it caches its compiled plan).
 */
#ifndef OMX_MATCH_H
#define OMX_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------------------------------- */
#define OMX_OK            0
#define OMX_E_UNSUPPORTED 1 /* valid query, not supported by the GPU engine → host falls back        */
#define OMX_E_INVALID     2 /* bad argument / bad snapshot / unknown class                             */
#define OMX_E_OOM         3 /* device or host allocation failed                                        */
#define OMX_E_DEVICE      4 /* HIP runtime error (no device, launch failure, ...)                      */
#define OMX_E_PARSE       5 /* OCommandSQLParsingException equivalent                                  */
#define OMX_E_EXECUTION   6 /* OCommandExecutionException equivalent                                   */

/* ---- snapshot description ------------------------------------------------------------------------ */
#define OMX_PROP_INT32  1 /* values: const int32_t[V]                                                 */
#define OMX_PROP_INT64  2 /* values: const int64_t[V]                                                 */
#define OMX_PROP_DOUBLE 3 /* values: const double[V]                                                  */
#define OMX_PROP_STRING 4 /* values: const int32_t[V] codes into dict (sorted, unique, UTF-8)         */
#define OMX_PROP_BOOL   5 /* values: const int32_t[V] 0/1                                              */

typedef struct omx_class_desc {
  const char *name;      /* class name, e.g. "Person"                                              */
  int32_t superclass;    /* index of the superclass in the class array, -1 for a root class         */
  int32_t is_edge_class; /* 1 for E and its subclasses                                              */
  int32_t cluster_id;    /* cluster of the class (RID = cluster:position), informational           */
} omx_class_desc;

/* Adjacency of one edge class (regular or lightweight edges alike): for every vertex v the multiset of
 * neighbours of v through out_<Class> (out CSR) and in_<Class> (in CSR). Duplicates (parallel edges)
 * must be kept: they are the ridbag multiplicity (OSBTreeRidBag.java:292-295). Within a row the order
 * is free; omx sorts rows it finds unsorted. */
typedef struct omx_edge_set_desc {
  int32_t edge_class;           /* index into classes[]                                            */
  uint64_t n_edges;             /* E (of the owned rows, for a partition)                          */
  const uint64_t *out_row_ptr;  /* [V+1] ([part_hi − part_lo + 1] for a partition)                 */
  const uint32_t *out_col;      /* [E] dense vertex ids                                            */
  const uint64_t *in_row_ptr;   /* [V+1] (the transpose); may be NULL → built by omx (required for */
                                /* a partition: the in-rows of the owned vertices)                 */
  const uint32_t *in_col;       /* [n_in_edges]                                                    */
  uint64_t n_in_edges;          /* edges of the in CSR; 0 = n_edges (always equal when unpartitioned) */
  /* Regular (heavyweight) edges: the edge records behind the CSR entries, which MATCH binds to edge   */
  /* nodes (outE('L'){as: e, where: (...)}.inV(), OSQLFunctionMove.java:109-144). NULL: lightweight     */
  /* edges (no records: such patterns are OMX_E_UNSUPPORTED). Not on a partitioned snapshot.            */
  const uint64_t *edge_rids;    /* [n_edges] RID of the edge record of out_col entry i               */
  const uint64_t *in_edge_index;/* [n_in_edges] the out_col entry of the same edge record, for every  */
                                /* in_col entry; required with edge_rids when in_row_ptr is given      */
} omx_edge_set_desc;

typedef struct omx_property_desc {
  const char *name;             /* property name (field name)                                      */
  int32_t type;                 /* OMX_PROP_*                                                      */
  const void *values;           /* [V]                                                             */
  const uint8_t *present;       /* [V] 1 = field present, 0 = null/absent; NULL = all present       */
  int32_t dict_size;            /* OMX_PROP_STRING only                                            */
  const char *const *dict;      /* OMX_PROP_STRING only: sorted by byte order, unique              */
} omx_property_desc;

/* A schema index (CREATE INDEX ... ON Class (prop)). Only used for root estimation, exactly as
 * OWhereClause.estimate uses indexes (OWhereClause.java:57-95). */
typedef struct omx_index_desc {
  int32_t class_id;
  const char *property;
  int32_t unique; /* 1 = UNIQUE / UNIQUE_HASH_INDEX, 0 = NOTUNIQUE                                   */
} omx_index_desc;

typedef struct omx_graph_desc {
  uint32_t n_vertices;                 /* V                                                       */
  int32_t n_classes;
  const omx_class_desc *classes;
  const uint16_t *vertex_class;        /* [V] class index of every vertex                         */
  const uint64_t *rids;                /* [V] RID packed (cluster << 48) | position               */
  int32_t n_edge_sets;
  const omx_edge_set_desc *edge_sets;
  int32_t n_properties;
  const omx_property_desc *properties;
  int32_t n_indexes;
  const omx_index_desc *indexes;
  int32_t device;                      /* HIP device ordinal; -1 = host-only (plan/explain only)   */
  /* 1-D partition: this snapshot holds the out/in CSR rows of the vertices
   * [part_lo, part_hi) only; classes, RIDs and properties stay replicated for all V vertices. Rank r of
   * a world of N owns [r·B, min(V, (r+1)·B)) with B = ⌈V/N⌉. part_lo = part_hi = 0: every row. */
  uint32_t part_lo, part_hi;
  /* Properties of the edge records (edge sets with edge_rids): values indexed by edge id = the edge   */
  /* sets' out_col entries one after the other (set 0's entries, then set 1's, ...), as given.         */
  int32_t n_edge_properties;
  const omx_property_desc *edge_properties;
} omx_graph_desc;

typedef struct omx_graph omx_graph;
typedef struct omx_statement omx_statement;
typedef struct omx_result omx_result;
typedef struct omx_comm omx_comm;

/* ---- graph snapshot --------------------------------------------------------------------------- */
int omx_graph_create(const omx_graph_desc *desc, omx_graph **out);
void omx_graph_destroy(omx_graph *g);
/* Host-side introspection of a snapshot (counts are the OClassImpl.count(polymorphic) of a class). */
int omx_graph_class_count(const omx_graph *g, const char *class_name, uint64_t *count);
uint64_t omx_graph_device_bytes(const omx_graph *g);

/* ---- statement (parse + pattern) -------------------------------------------------------------- */
int omx_statement_parse(const char *text, omx_statement **out);
void omx_statement_free(omx_statement *s);

/* Query parameters (OCommandSQL.execute(args...)): positional (name == NULL, index = position) or
 * named (":name"). */
#define OMX_VAL_NULL   0
#define OMX_VAL_INT    1
#define OMX_VAL_DOUBLE 2
#define OMX_VAL_STRING 3
#define OMX_VAL_BOOL   4
typedef struct omx_value {
  int32_t type;
  int32_t index;       /* positional index (0-based) when name == NULL                             */
  const char *name;    /* named parameter (without ':') or NULL                                    */
  int64_t i;
  double d;
  const char *s;
} omx_value;

/* Writes the MATCH plan as JSON into buf (NUL-terminated, truncated to len): aliases with classes,
 * estimates, prefetched aliases, root alias and the sorted edge list. Works on host-only graphs. */
int omx_statement_explain(omx_statement *s, const omx_graph *g, const omx_value *params, int32_t n_params,
                          char *buf, size_t len);

/* ---- execution -------------------------------------------------------------------------------- */
#define OMX_MODE_MATERIALIZE 0 /* distinct RETURN rows (the OResultSet)                            */
#define OMX_MODE_COUNT       1 /* counts only (edges traversed, bindings, distinct rows if cheap)   */

#define OMX_FLAG_KERNEL_TIMING 1 /* time every kernel with HIP events (omx_result_kernel_stat)     */
#define OMX_FLAG_NO_RID_MAP    2 /* return dense vertex ids instead of RIDs                         */
#define OMX_FLAG_KEEP_DEVICE   4 /* do not copy rows to the host (benchmarking; rows stay in HBM)   */
#define OMX_FLAG_TIME_HOT      8 /* with KERNEL_TIMING: time only the traversal kernels (expansion,  */
                                 /* check, BFS levels), so the events do not stretch a timed step     */
#define OMX_FLAG_DIGEST       16 /* compute omx_result_info.digest on the device (works with         */
                                 /* KEEP_DEVICE: whole-result parity checks without a host copy)      */

typedef struct omx_exec_options {
  int32_t mode;          /* OMX_MODE_*                                                            */
  int32_t flags;         /* OMX_FLAG_*                                                            */
  int64_t limit;         /* OMatchStatement.setLimit (limitFromProtocol); -1 = none               */
  int32_t shard_rank;    /* root shard of this process (multi-GPU): roots v with v % world == rank */
  int32_t shard_world;   /* 1 = no sharding                                                       */
  const omx_value *params;
  int32_t n_params;
  omx_comm *comm;        /* partitioned snapshot: the ranks' communicator (NULL otherwise)        */
} omx_exec_options;

void omx_exec_options_init(omx_exec_options *o);
int omx_execute(omx_graph *g, omx_statement *s, const omx_exec_options *opts, omx_result **out);

typedef struct omx_result_info {
  uint64_t n_rows;           /* distinct RETURN rows (after LIMIT)                                 */
  int32_t n_cols;            /* RID columns per row (0 for an empty result)                        */
  int32_t deduplicated;      /* 1 if a dedup pass ran, 0 if rows were distinct by construction     */
  uint64_t edges_traversed;  /* Σ_h E_t(h), SURVEY §8(d)                                           */
  uint64_t bindings;         /* complete matches before dedup (a parallel edge into a filtered     */
                             /* target binds once per edge; the reference HashSet binds it once)   */
  uint64_t alg_bytes;        /* algorithmic HBM bytes, SURVEY §8(d)                                */
  double device_ms;          /* wall time of the device part (root scan → last kernel)             */
  double total_ms;           /* wall time of omx_execute                                           */
  uint64_t edges_read;       /* adjacency entries a kernel iterated one by one: edges_traversed     */
                             /* minus the hops a COUNT run sums from degrees (an unfiltered last    */
                             /* hop) and minus the E_t a cycle-closing check stands for (answered   */
                             /* by binary searches into the sorted adjacency, never iterated)       */
  uint64_t digest;           /* OMX_FLAG_DIGEST: Σ over the distinct rows of h(row) mod 2^64, h =   */
                             /* splitmix64 chained over the row's RIDs in column order (h0 =        */
                             /* 0x9E3779B97F4A7C15, h = mix(h ^ rid)); 0 otherwise                  */
  int32_t documents;         /* 1: rows are documents of RETURN expressions / JSON (omx_result_cell); */
                             /* 0: rows are RID tuples (omx_result_rows)                             */
  int32_t factorized_hops;   /* filtered hops run through the factorized expansion (distinct       */
                             /* sources → grouped filtered lists → rows over the lists; diagnostic) */
  uint64_t rows_gathered;    /* partitioned runs whose projection needs the whole result (RETURN     */
                             /* expressions, $elements, LIMIT): rows this rank received when the     */
                             /* rows met on rank 0 — distinct tuples only, each rank de-duplicates   */
                             /* its hash share first; 0 elsewhere (diagnostic)                       */
  uint64_t host_rows_bytes;  /* bytes of the library-owned host block holding omx_result_rows (0 with  */
                             /* KEEP_DEVICE or for documents); released to a pooled cache by         */
                             /* omx_result_free and reused by the next result of a similar size      */
  int32_t host_rows_pinned;  /* 1: that block is pinned (page-locked) host memory, so the rows came   */
                             /* over PCIe by DMA; 0: pageable (pinning failed) or no block            */
  int32_t reserved0;
} omx_result_info;

/* A null binding (an unmatched optional node, P/OMatchStatement.java:448-458) in omx_result_rows. */
#define OMX_NULL_RID UINT64_MAX

int omx_result_info_get(const omx_result *r, omx_result_info *info);
const char *omx_result_column_name(const omx_result *r, int32_t col);
/* Row-major n_rows × n_cols RIDs ((cluster << 48) | position), or dense ids with NO_RID_MAP.
 * Library-owned pinned host memory (info.host_rows_bytes / host_rows_pinned); valid until omx_result_free,
 * which returns the block to the library's pool. NULL with KEEP_DEVICE. */
const uint64_t *omx_result_rows(const omx_result *r);
/* Per-kernel device timing (OMX_FLAG_KERNEL_TIMING): i-th kernel name, launches, total ms, and the
 * algorithmic bytes the launches of that kernel moved. Returns OMX_E_INVALID past the end. */
int omx_result_kernel_stat(const omx_result *r, int32_t i, const char **name, int64_t *launches, double *total_ms,
                           uint64_t *alg_bytes);
/* The same timing launch by launch, in issue order (a kernel launched several times per execution,
 * e.g. a first hop and a row emission, is reported per launch). Returns OMX_E_INVALID past the end. */
int omx_result_kernel_launch(const omx_result *r, int32_t i, const char **name, double *ms, uint64_t *alg_bytes);
/* Launch i's byte counts: alg_bytes as above, and hbm_bytes, the bytes HBM must move at least — each
 * distinct byte once, so data a kernel shares between work items and re-reads from L2 (a factorized
 * hop's lists, a pull level's frontier masks) counts once. Returns OMX_E_INVALID past the end. */
int omx_result_kernel_launch_bytes(const omx_result *r, int32_t i, uint64_t *alg_bytes, uint64_t *hbm_bytes);
void omx_result_free(omx_result *r);

/* One field of a result document (info.documents = 1): the value of RETURN item `col` (or of JSON key
 * `col`) in row `row`, as ODocument.field would hold it. LIST / MAP values come as JSON text in `s`
 * (records as "#cluster:position" strings); `s` stays valid until omx_result_free. */
#define OMX_CELL_NULL   0
#define OMX_CELL_INT    1
#define OMX_CELL_DOUBLE 2
#define OMX_CELL_STRING 3
#define OMX_CELL_BOOL   4
#define OMX_CELL_RID    5
#define OMX_CELL_LIST   6
#define OMX_CELL_MAP    7
typedef struct omx_cell {
  int32_t type;   /* OMX_CELL_*                                                                     */
  int32_t n;      /* LIST / MAP: elements                                                           */
  int64_t i;      /* INT, BOOL (0/1)                                                                */
  double d;       /* DOUBLE                                                                         */
  uint64_t rid;   /* RID: (cluster << 48) | position                                                */
  const char *s;  /* STRING (UTF-8), LIST / MAP (JSON)                                              */
} omx_cell;
int omx_result_cell(const omx_result *r, uint64_t row, int32_t col, omx_cell *out);
/* Column `col` of a document result in bulk: types[row] = OMX_CELL_* and bits[row] = the INT / BOOL
 * value, the DOUBLE's IEEE-754 bits or the packed RID (0 for NULL; STRING / LIST / MAP cells are read
 * with omx_result_cell). Both arrays hold info.n_rows entries. One call per column replaces n_rows
 * omx_result_cell calls when a host binding converts the rows (JNI: one long[] per column). */
int omx_result_column(const omx_result *r, int32_t col, int32_t *types, uint64_t *bits);

const char *omx_last_error(void);
const char *omx_version(void);

/* ---- pointer-free variants (JNI / Panama: one caller-owned direct buffer) ---------------------- */
/* The same snapshot and parameters as omx_graph_desc / omx_value, laid out in ONE buffer the Java side
 * fills (a direct ByteBuffer, native byte order) with every pointer replaced by a byte offset from the
 * start of the buffer (0 = none). Arrays are naturally aligned; strings are NUL-terminated UTF-8. omx
 * validates every offset and length against `size` (OMX_E_INVALID otherwise) and copies what it keeps. */
#define OMX_BLOB_MAGIC   0x47584D4Fu /* "OMXG" */
#define OMX_BLOB_VERSION 2u          /* version 1 buffers (the header up to indexes_off) are accepted too */
typedef struct omx_graph_blob {       /* at offset 0 of the buffer                                       */
  uint32_t magic, version;
  uint32_t n_vertices;
  int32_t n_classes, n_edge_sets, n_properties, n_indexes;
  int32_t device;
  uint32_t part_lo, part_hi;
  uint64_t classes_off;      /* omx_class_rec[n_classes]                                               */
  uint64_t vertex_class_off; /* uint16_t[V]                                                            */
  uint64_t rids_off;         /* uint64_t[V]                                                            */
  uint64_t edge_sets_off;    /* omx_edge_set_rec[n_edge_sets]                                          */
  uint64_t properties_off;   /* omx_property_rec[n_properties]                                         */
  uint64_t indexes_off;      /* omx_index_rec[n_indexes]                                               */
  /* version 2: edge records (omx_edge_set_desc.edge_rids / in_edge_index, omx_graph_desc.edge_properties) */
  uint64_t edge_records_off; /* omx_edge_records_rec[n_edge_sets], 0 = lightweight edges             */
  int32_t n_edge_properties, reserved;
  uint64_t edge_properties_off; /* omx_property_rec[n_edge_properties], values over the edge records  */
} omx_graph_blob;
typedef struct omx_edge_records_rec {
  uint64_t edge_rids_off;      /* uint64_t[n_edges]                                                   */
  uint64_t in_edge_index_off;  /* uint64_t[n_in_edges]; 0 when the set has no in CSR                  */
} omx_edge_records_rec;
typedef struct omx_class_rec {
  uint64_t name_off;
  int32_t superclass, is_edge_class, cluster_id, reserved;
} omx_class_rec;
typedef struct omx_edge_set_rec {
  int32_t edge_class, reserved;
  uint64_t n_edges, out_row_ptr_off, out_col_off, in_row_ptr_off, in_col_off, n_in_edges;
} omx_edge_set_rec;
typedef struct omx_property_rec {
  uint64_t name_off;
  int32_t type, dict_size;
  uint64_t values_off, present_off;
  uint64_t dict_off;         /* uint64_t[dict_size] offsets of the dictionary strings                  */
} omx_property_rec;
typedef struct omx_index_rec {
  uint64_t property_off;
  int32_t class_id, unique;
} omx_index_rec;
int omx_graph_create_blob(const void *blob, uint64_t size, omx_graph **out);

/* ---- ridbag ingest ------------------------------------------------------------------------------
 * Decodes, on `device`, the vertices' serialized out_<L> (or in_<L>) ridbag fields into one CSR of dense
 * vertex ids, each bag's entry order kept (the reference's iteration order). Replaces iterating
 * ORidBag.rawIterator per vertex on the Java side (C/db/record/ridbag/ORidBag.java:160) when a snapshot
 * is built from the stored records. Stream format (ORidBag.toStream, ORidBag.java:198-276;
 * OEmbeddedRidBag.serialize, .../ridbag/embedded/OEmbeddedRidBag.java:424-460; big-endian):
 *   [1 B config: bit 0 embedded, bit 1 UUID][16 B UUID if bit 1][int32 count][count × (int16 cluster,
 *   int64 position)]
 * streams: the vertices' streams concatenated; vertex v's is [offsets[v], offsets[v+1]) (empty: no
 * field). vertex_rids[V]: every vertex's packed RID (dense order). Lightweight edges: the entries are
 * vertex RIDs (edge_rids = edge_targets = NULL). Edge records: the entries are edge RIDs and
 * edge_targets[i] is the opposite vertex RID of edge record edge_rids[i] (its `in` field for out_
 * bags, `out` for in_ bags). Fills row_ptr[V+1] (may be NULL) and *n_entries; col[*n_entries] when
 * col != NULL (call once with col = NULL to size it). OMX_E_INVALID: malformed stream, an SBTree
 * (non-embedded) bag, or an entry that resolves to no vertex. */
int omx_ridbag_decode_csr(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                          uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                          const uint64_t *edge_targets, uint64_t n_edge_records, uint64_t *row_ptr, uint32_t *col,
                          uint64_t *n_entries);

/* SBTree-bonsai ridbags (config bit 0 clear: every bag of >= 40 entries by default,
 * C/config/OGlobalConfiguration.java:356-358) keep their entries in a collection file
 * (collections_<cluster>.sbc). Stream (C/db/record/ridbag/sbtree/OSBTreeRidBag.java:855-880, big-endian):
 * [config][UUID?][int64 fileId][int64 root pageIndex][int32 root pageOffset][int32 cached size]
 * [int32 n][n × (int16 cluster, int64 position, int8 change type, int32 value)]. The host passes each
 * collection file's pages as stored (OSBTreeBonsaiBucket layout, C/index/sbtreebonsai/local/
 * OSBTreeBonsaiBucket.java:44-60,263-279): the bag's entries are decoded on the device in the order
 * OSBTreeRidBag's iterator yields them (tree entries in RID order merged with the changes, each RID
 * `counter` times, :256-425). files = NULL: as omx_ridbag_decode_csr. page_size 0: 64 KiB
 * (DISK_CACHE_PAGE_SIZE). OMX_E_INVALID also for a bag whose file is missing, a bucket pointer or
 * entry outside its page, a tree deeper than 64 levels, or changes out of RID order. */
#define OMX_BONSAI_PAGE_SIZE 65536u
typedef struct omx_bonsai_file {
  int64_t file_id;       /* the fileId an SBTree bag's stream names                                   */
  const uint8_t *pages;  /* n_pages × page_size bytes: page i at i × page_size                         */
  uint64_t n_pages;
} omx_bonsai_file;
int omx_ridbag_decode_csr_ex(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                             uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                             const uint64_t *edge_targets, uint64_t n_edge_records, const omx_bonsai_file *files,
                             int32_t n_files, uint32_t page_size, uint64_t *row_ptr, uint32_t *col,
                             uint64_t *n_entries);

/* omx_ridbag_decode_csr_ex for bags of edge records (edge_rids / edge_targets required) that also returns
 * entry_rids[*n_entries] (may be NULL), the edge record RID of every CSR entry — the edge_rids of an
 * omx_edge_set_desc built from the same out_ bags, so edge nodes can bind those records. */
int omx_ridbag_decode_edges(int32_t device, const uint8_t *streams, uint64_t stream_bytes, const uint64_t *offsets,
                            uint32_t n_vertices, const uint64_t *vertex_rids, const uint64_t *edge_rids,
                            const uint64_t *edge_targets, uint64_t n_edge_records, const omx_bonsai_file *files,
                            int32_t n_files, uint32_t page_size, uint64_t *row_ptr, uint32_t *col,
                            uint64_t *entry_rids, uint64_t *n_entries);

/* Parameters as one buffer: uint32_t n, uint32_t reserved, omx_param_rec[n], then the strings. */
typedef struct omx_param_rec {
  int32_t type, index;       /* OMX_VAL_*, positional index (when name_off == 0)                       */
  int64_t i;
  double d;
  uint64_t name_off;         /* named parameter (without ':'), 0 = positional                          */
  uint64_t s_off;            /* OMX_VAL_STRING                                                          */
} omx_param_rec;
/* omx_execute with plain option fields and the parameter buffer (param_blob may be NULL: none). */
int omx_execute_packed(omx_graph *g, omx_statement *s, int32_t mode, int32_t flags, int64_t limit, int32_t shard_rank,
                       int32_t shard_world, omx_comm *comm, const void *param_blob, uint64_t param_blob_size,
                       omx_result **out);

/* ---- multi-GPU: communicator of a 1-D partitioned MATCH ------------------------ */
/* With a partitioned snapshot, omx_execute routes binding rows to the rank owning the vertex whose
 * adjacency the next step reads (an all-to-all of counts, then of every bound column), and before a
 * de-duplicating projection routes rows by a hash of the projected tuple. Every rank returns its share
 * of the distinct rows; their union is the result. All ranks must execute the same statements in the
 * same order. The reference has no counterpart (OMatchStatement.isLocalExecution, :1009-1011). */
#define OMX_COMM_ID_BYTES 128
/* RCCL unique id (ncclGetUniqueId) created on one rank and shared with the others by the caller. */
int omx_comm_unique_id(uint8_t id[OMX_COMM_ID_BYTES]);
/* One process per GPU: RCCL over xGMI (ncclCommInitRank on `device`). */
int omx_comm_create_rccl(int32_t rank, int32_t world, int32_t device, const uint8_t id[OMX_COMM_ID_BYTES],
                         omx_comm **out);
/* Ranks that are threads of this process (any devices, one GPU included): out[0..world-1]. The exchange
 * is device-to-device copies behind a barrier; each rank's omx_execute runs on its own thread. */
int omx_comm_create_threads(int32_t world, omx_comm **out);
/* Ranks that are processes joined by the caller's own host collectives (e.g. torch.distributed over gloo,
 * MPI): the exchange is staged through host memory — counts and rows copied to the host, exchanged by the
 * callbacks, copied back. For hosts without RCCL between the ranks' GPUs (or one GPU shared by several
 * processes); the routing code is the one the RCCL transport runs. Callbacks return 0 on success. */
typedef struct omx_host_collectives {
  void *ctx;
  /* every rank's `nbytes` bytes of `send`, rank-major, into recv (world × nbytes bytes) */
  int (*allgather)(void *ctx, const void *send, uint64_t nbytes, void *recv);
  /* byte all-to-all-v: send[sdispl[p], +scount[p]) goes to rank p; what rank p sends lands at
   * recv[rdispl[p], +rcount[p]) (counts and displacements in bytes, world entries each) */
  int (*alltoallv)(void *ctx, const void *send, const uint64_t *scount, const uint64_t *sdispl, void *recv,
                   const uint64_t *rcount, const uint64_t *rdispl);
  void (*abort)(void *ctx); /* may be NULL */
} omx_host_collectives;
int omx_comm_create_host(int32_t rank, int32_t world, const omx_host_collectives *c, omx_comm **out);
int32_t omx_comm_rank(const omx_comm *c);
int32_t omx_comm_world(const omx_comm *c);
void omx_comm_destroy(omx_comm *c);

/* ---- synthetic graphs (benchmark / test inputs) -------------------------------- */
/* Graph500 RMAT (a=.57,b=.19,c=.19), V = 2^scale, edge_factor·V raw directed edges, deterministic
 * counter-based RNG (splitmix64), vertex ids scrambled by a bijection. simple != 0 removes self loops
 * and parallel edges. Outputs are host arrays owned by the library (omx_host_free). */
int omx_rmat_generate(int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple, uint64_t **out_row_ptr,
                      uint32_t **out_col, uint64_t *n_edges);
/* LDBC-SNB-like Knows graph (configs[3]): n_persons vertices, ≈ target_edges directed
 * edges (unique pairs, one direction each), skewed degrees and high clustering from correlated
 * windows; rows sorted. Deterministic in (n_persons, target_edges, seed). */
int omx_ldbc_knows_generate(uint32_t n_persons, uint64_t target_edges, uint64_t seed, uint64_t **out_row_ptr,
                            uint32_t **out_col, uint64_t *n_edges);
/* The partition [lo, hi) of the same RMAT graph: out rows and in rows (the transpose's rows) of the
 * owned vertices, local row pointers of hi − lo + 1 entries, rows sorted; identical to the rows of
 * omx_rmat_generate (+ omx_csr_transpose) for those vertices. */
int omx_rmat_generate_part(int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple, uint32_t lo, uint32_t hi,
                           uint64_t **out_row_ptr, uint32_t **out_col, uint64_t *n_out, uint64_t **in_row_ptr,
                           uint32_t **in_col, uint64_t *n_in);
/* The same two generators run on GPU `device` (every edge drawn in parallel, the CSR built by a radix
 * sort of (row, neighbour) keys): identical output arrays, host-owned (omx_host_free); seconds for
 * RMAT-26 where the host generators take minutes. */
int omx_rmat_generate_dev(int32_t device, int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple,
                          uint64_t **out_row_ptr, uint32_t **out_col, uint64_t *n_edges);
int omx_rmat_generate_part_dev(int32_t device, int32_t scale, int32_t edge_factor, uint64_t seed, int32_t simple,
                               uint32_t lo, uint32_t hi, uint64_t **out_row_ptr, uint32_t **out_col, uint64_t *n_out,
                               uint64_t **in_row_ptr, uint32_t **in_col, uint64_t *n_in);
/* CSR transpose (host, multi-threaded); rows of the output are sorted. */
int omx_csr_transpose(uint32_t n_vertices, const uint64_t *row_ptr, const uint32_t *col, uint64_t **t_row_ptr,
                      uint32_t **t_col);
/* age property of the synthetic Person vertices: uniform [0,100) from splitmix64(seed ^ v). */
int omx_synthetic_int_column(uint32_t n_vertices, uint64_t seed, int32_t modulo, int32_t **out);
void omx_host_free(void *p);

#ifdef __cplusplus
}
#endif
#endif /* OMX_MATCH_H */
