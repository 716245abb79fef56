/*
 * lancedb_hip.h — the drop-in C-ABI of the MI355X-native k-NN path.
 *
 * Every symbol below replaces the export of the same name in the reference's
 * Rust library (rust_lib/src/ffi.rs), consumed unchanged by the reference's C++
 * shim src/rust_ffi.cpp:7-42 (paths relative to /root/reference).  Conventions
 * kept from ffi.rs:
 *   - handle = opaque pointer owning all state (ffi.rs:51), freed only by
 *     lance_free_detached (null-safe, ffi.rs:137-142);
 *   - errors: NULL / -1 return plus a NUL-terminated message truncated to
 *     err_buf_len-1 bytes (ffi.rs:15-24); a NULL handle reports "null handle";
 *   - every output buffer is caller-allocated; strings are borrowed;
 *   - calls may arrive from any thread; search may run concurrently with
 *     add/delete (the handle serialises internally).
 * Symbols marked NEW have no counterpart in the shipped ffi.rs.
 */
#ifndef LANCEDB_HIP_H
#define LANCEDB_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- create / open / free ------------------------------------------------ */

/* ffi.rs:37-57 (called from rust_ffi.cpp:47).  Creates (replacing any existing
 * table of that name, lance_manager.rs:42) an empty vector-only table.
 * metric: "l2" (default) | "dot" | "ip" | "cosine".  db_path "" = in-memory. */
void *lance_create_detached(const char *db_path, int32_t dimension, const char *metric, const char *table_name,
                            char *err_buf, int err_buf_len);

/* ffi.rs:62-89 (rust_ffi.cpp:58), lance_manager.rs:62-126.  Multi-column
 * table from an Arrow C Data Interface schema (struct of the table's columns,
 * borrowed): the first FixedSizeList<float32>[dim] column is the vector, every
 * other column metadata (filterable by a search predicate, persisted in the
 * table log, carried by merge and compact).  NULL with an error otherwise. */
void *lance_create_detached_from_arrow(const char *db_path, void *arrow_schema, const char *metric,
                                       const char *table_name, char *err_buf, int err_buf_len);

/* ffi.rs:92-111 (rust_ffi.cpp:68).  Re-opens a table persisted under db_path;
 * next label = max(label)+1 (lance_manager.rs:157-158). */
void *lance_open_detached(const char *db_path, const char *table_name, const char *metric, char *err_buf,
                          int err_buf_len);

/* ffi.rs:137-142 (rust_ffi.cpp:76).  Null-safe. */
void lance_free_detached(void *handle);

/* ffi.rs:114-123 / :126-135 (rust_ffi.cpp:80,84).  0 for a null handle. */
int32_t lance_detached_has_extra_columns(void *handle);
int32_t lance_detached_dimension(void *handle);

/* ---- ingest --------------------------------------------------------------- */

/* ffi.rs:228-250 (rust_ffi.cpp:88).  Returns the new label or -1. */
int64_t lance_detached_add(void *handle, const float *vector, int32_t dimension, char *err_buf, int err_buf_len);

/* ffi.rs:252-289 (rust_ffi.cpp:97).  vectors: num x dim row-major f32 (DuckDB
 * ARRAY child buffer, lance_index.cpp:940-946).  Labels are dense consecutive
 * [next_label, next_label+num) (lance_manager.rs:232-233).  Returns num or -1. */
int32_t lance_detached_add_batch(void *handle, const float *vectors, int32_t num, int32_t dim, int64_t *out_labels,
                                 char *err_buf, int err_buf_len);

/* ffi.rs:147-180 (rust_ffi.cpp:108), lance_manager.rs:251-301.  A struct
 * array of the table's columns [vector FixedSizeList<float32>[dim], extra...]
 * (Arrow C Data Interface); the callee takes the array over (its release is
 * called, the caller's struct is left released), the schema stays borrowed.
 * Extra columns: integers, float, double, boolean, utf8 / large utf8, NULLs
 * allowed.  Labels dense as add_batch.  Returns num or -1. */
int32_t lance_detached_add_batch_arrow(void *handle, void *arrow_schema, void *arrow_array, int64_t *out_labels,
                                       char *err_buf, int err_buf_len);

/* ffi.rs:186-222 (rust_ffi.cpp:118).  Copies the listed live rows of source
 * into target under fresh target labels; writes the (old,new) label pairs. */
int32_t lance_detached_merge(void *target_handle, void *source_handle, const int64_t *live_source_labels,
                             int32_t live_count, int64_t *out_old_labels, int64_t *out_new_labels, char *err_buf,
                             int err_buf_len);

/* ---- search --------------------------------------------------------------- */

/* ffi.rs:295-329 (rust_ffi.cpp:130-139).  Exact top-k of one query over all
 * live rows, ascending distance (ties: the handle's tie rule, label
 * descending by default — option "tie" below); writes n <= k
 * (label, distance) pairs, returns n or -1.  dim != index dim is an error here
 * (lance_manager.rs:401-407); the C++ caller returns {} before calling
 * (lance_index.cpp:444-446).  nprobes / refine_factor only matter once an
 * IVF index exists (lance_index.hpp:91-92 defaults 20 / 1). */
int32_t lance_detached_search(void *handle, const float *query, int32_t dim, int32_t k, int32_t nprobes,
                              int32_t refine_factor, int64_t *out_labels, float *out_distances, char *err_buf,
                              int err_buf_len);

/* NEW — the form the reference's C++ already calls (lance_index.cpp:452-453):
 * a nullable Lance-SQL predicate inserted after refine_factor (NULL or "" =
 * unfiltered), as lance_optimizer.cpp:204-344 writes it: column op constant,
 * AND / OR, NOT (..), IS [NOT] NULL, [NOT] IN (..), BETWEEN; string literals
 * '..' ('' escapes), numbers, true / false, NULL.  Columns: the table's extra
 * columns and the implicit int64 `label`.  Prefilter semantics (LanceDB
 * only_if): top-k over the live rows whose predicate is TRUE (SQL three-valued
 * logic).  Unknown column / syntax error: -1. */
int32_t lance_detached_search_with_predicate(void *handle, const float *query, int32_t dim, int32_t k,
                                             int32_t nprobes, int32_t refine_factor, const char *predicate,
                                             int64_t *out_labels, float *out_distances, char *err_buf,
                                             int err_buf_len);

/* NEW — batched search.  queries: nq x dim row-major f32;
 * out_labels / out_distances: nq x k (unused slots: label -1, distance NaN);
 * out_counts: nq.  Returns nq or -1. */
int32_t lance_detached_search_batch(void *handle, const float *queries, int32_t nq, int32_t dim, int32_t k,
                                    int32_t nprobes, int32_t refine_factor, const char *predicate,
                                    int64_t *out_labels, float *out_distances, int32_t *out_counts, char *err_buf,
                                    int err_buf_len);

/* ---- count / delete ------------------------------------------------------- */

/* ffi.rs:335-353 (rust_ffi.cpp:141).  Live rows, or -1. */
int64_t lance_detached_count(void *handle, char *err_buf, int err_buf_len);

/* ffi.rs:355-374 / :376-397 (rust_ffi.cpp:150,159).  0 or -1.  Unknown or
 * already-deleted labels are a no-op (a SQL `label IN (..)` delete). */
int32_t lance_detached_delete(void *handle, int64_t label, char *err_buf, int err_buf_len);
int32_t lance_detached_delete_batch(void *handle, const int64_t *labels, int32_t count, char *err_buf,
                                    int err_buf_len);

/* ---- ANN index / maintenance --------------------------------------------- */

/* ffi.rs:403-423 (rust_ffi.cpp:168), lance_manager.rs:483-515.  Trains and
 * builds an IVF index over the live rows (replace = true): IVF_PQ (default, as
 * the reference builds) or IVF_FLAT (option "index_type").  num_partitions /
 * num_sub_vectors <= 0 take LanceDB's defaults (sqrt(rows); dim/16, dim/8 or 1).
 * Later searches probe `nprobes` partitions and re-rank k*refine_factor PQ
 * candidates exactly; rows added afterwards are searched exactly until
 * lance_detached_compact (= optimize) indexes them.  0 or -1. */
int32_t lance_detached_create_index(void *handle, int32_t num_partitions, int32_t num_sub_vectors, char *err_buf,
                                    int err_buf_len);

/* The call lance_index.cpp:481-486 already makes (LanceDetachedCreateScalarIndex,
 * never declared nor exported by the reference): a scalar
 * index ("BTREE" default, or "BITMAP") on a metadata column of a multi-column
 * table; search predicates comparing the column with a literal use it.
 * Persisted in the table log.  0 or -1. */
int32_t lance_detached_create_scalar_index(void *handle, const char *column, const char *index_type, char *err_buf,
                                           int err_buf_len);

/* ffi.rs:425-445 (rust_ffi.cpp:176).  HNSW is out of scope:
 * returns 0 and keeps serving exact flat search (lance_hnsw.test pins only
 * result counts). */
int32_t lance_detached_create_hnsw_index(void *handle, int32_t m, int32_t ef_construction, char *err_buf,
                                          int err_buf_len);

/* ffi.rs:447-465 (rust_ffi.cpp:184).  Drops tombstoned rows from the device
 * store (labels are preserved).  0 or -1. */
int32_t lance_detached_compact(void *handle, char *err_buf, int err_buf_len);

/* ffi.rs:471-500 (rust_ffi.cpp:192).  Copies the vector of a live label into
 * out_vec (capacity floats); returns dim or -1 ("output buffer too small",
 * "label N not found"). */
int32_t lance_detached_get_vector(void *handle, int64_t label, float *out_vec, int32_t capacity, char *err_buf,
                                  int err_buf_len);

/* ffi.rs:510-541 (rust_ffi.cpp:201).  With out_labels/out_vectors NULL only
 * *out_count is written.  Rows in ascending label order. */
int32_t lance_detached_get_all_vectors(void *handle, int64_t *out_labels, float *out_vectors, int64_t *out_count,
                                       char *err_buf, int err_buf_len);

/* ---- NEW: device / sharding / introspection -------------------------------- */

/* Library version string (static storage). */
const char *lance_hip_version(void);

/* Number of HIP devices visible to the library (0 when none / no driver). */
int32_t lance_hip_device_count(void);

/* Per-handle options, key/value strings (unknown keys: error, -1):
 *   "tie"          "label_desc" (default) | "label_asc": which of several rows
 *                  at an equal exact distance come first (and so which make the
 *                  k-th place).  label_desc is what the reference's golden
 *                  shows (test/sql/lance_optimizer_filter.test:36-44: ids 3 and
 *                  4 tie at d = 2.0 and LanceDB returns 4); the default of a new
 *                  handle comes from LANCE_HIP_TIE in the process environment
 *                  (a DuckDB process has no option channel)
 *   "metric_quirk" "1" = rank every search by squared L2 whatever the index
 *                  metric, exactly as the reference does (lance_manager.rs:
 *                  411-418 never sets distance_type); default "0"
 *   "reserve_rows" pre-size the device store for this many rows
 *   "storage"      "f32" (default) | "bf16": element type of the device store;
 *                  bf16 keeps the nearest-even bf16 of each added row and every
 *                  result is exact with respect to those stored rows.  Only
 *                  while the table holds no rows.
 *   "scan_i8"      "on" (default) | "off": a store (f32 or bf16) with dim padded
 *                  to a multiple of 128 (<= 1024) also keeps an int8 copy of its
 *                  rows (one scale per 256-row tile, 1 B per element + 16 B of
 *                  row terms) that the flat scans stream when there is no
 *                  predicate and no metric_quirk (any k on the threshold path of
 *                  > 65536 slots, k <= 32 on the dense path of smaller stores);
 *                  results are unchanged (exact re-rank + certificate).  Built on
 *                  the first search or by "prepare".
 *   "prepare"      "1": build the int8 scan copy now (outside any timing)
 *   "scan_copy"    "on" (default) | "off": an f32 store may keep a bf16 copy of
 *                  its rows for the scans the int8 copy does not serve (k > 32,
 *                  a predicate, metric_quirk) and the IVF_FLAT bound scan; built
 *                  on the first search that needs it; refine and get_vector read
 *                  the f32 rows, results are unchanged
 *   "sample_div"   the threshold sample pass covers ~1/sample_div of the row
 *                  tiles (at least 32 tiles); default "0" = auto (16 up to 8192
 *                  tiles of 256 rows, 32 past that)
 *   "split_div"    int8 append pass over >= 128 * split_div tiles: the first
 *                  1/split_div of the tiles with the sample's threshold, the rest
 *                  with the tighter one their candidates give (e.g. "8"); "0"
 *                  or "1" = one pass, the default (results unchanged either way)
 *   "cand_extra"   small stores (dense path, <= 65536 rows): exact candidates
 *                  re-ranked per query beyond k: max(k * refine_factor, k +
 *                  max(cand_extra, k)), default "32"; the threshold path re-ranks
 *                  in bound order until its certificate holds (no fixed count)
 *   "cand_extra_i8" the same for the dense path on the int8 copy; "0" = auto (96)
 *   "small_exact"  "1" (default) | "0": <= 8 queries over <= 32768 slots
 *                  (k <= 64, dim <= 4096) take one launch of exact f64
 *                  distances + merge instead of the bound/refine pipeline
 *   "retry_pass"   "1" (default) | "0": rerun uncertified threshold-path
 *                  queries with a tightened tau before the exact fallback
 *   "index_type"   "ivf_pq" (default) | "ivf_flat": what create_index builds
 *   "kmeans_iters" k-means iterations (coarse and PQ), default "50"
 *   "ivf_seed"     seed of the k-means training sample, default 24301
 *   "ivf_flat_scan" "bound" (default) | "exact": IVF_FLAT list scan by MFMA bf16
 *                  lower bounds + certified exact re-rank, or exact f64 distances
 *   "pq_scan"      "fast" (default) | "exact_lut": IVF_PQ list-major 8-bit-LUT
 *                  scan, or the query-major f32-LUT scan
 *   "pq_seed"      "1" (default) | "0": the fast scan's per-query bound starts
 *                  at the kk-th smallest key of the query's nearest probed list
 *                  (kk = k * refine_factor; results unchanged, less work)
 *   "pq_query"     "f32" (default) | "fp8": IVF_PQ distance tables from e4m3
 *                  (fp8) queries (BASELINE.json configs[4]); coarse search and
 *                  re-rank keep the f32 query
 *   "pq_lut"       "fused" (default) | "split": the fast scan's per-query
 *                  tables in one launch or three (bit-identical)
 *   "pq_merge_bound" "1" (default) | "0": the fast scan's run merge keeps only
 *                  keys at or below the scan's final bound (same lists)
 *   "ivf_coarse"   "fused" (default) | "flat": IVF coarse search by the fused
 *                  MFMA-bound + exact-refine kernels or by the flat path over
 *                  the centroid store (same probes)
 *   "s8_couple"    "0" (default) | lag: int8 append scan pair coupling
 *   "time_kernels" "1" = record HIP events around scan launches
 *                  (lance_hip_kernel_times); default "0"
 *   "scan8_variant" geometry of the int8 append kernel at dim 768: "0" (the
 *                  default) is the only value a release build accepts; other
 *                  geometries and timing ablations exist only in development
 *                  builds (LHIP_ABLATION_BUILD) and are rejected here (-1)
 *   "pr_first"     bounds refined in the first chunk of the final
 *                  threshold-path refine, this handle only: "0" = the default
 *                  (96), else 8..1024; results are exact for every value
 *   "devices"      "0,1,..." (two or more ids, repeats allowed): this empty
 *                  handle row-shards its table over one store per listed
 *                  device; searches run on every store and the per-store top-k
 *                  lists merge on the first device (results as one store)
 * The handle is bound to the HIP device current when it was created, or, with
 * LANCE_HIP_DEVICES=0,1,... in the process environment at create / open time,
 * is a multi-device handle over those devices (one id: that device).  Every
 * option of a multi-device handle applies to each of its stores.
 * Returns 0 or -1. */
int32_t lance_hip_set_option(void *handle, const char *key, const char *value, char *err_buf, int err_buf_len);

/* Statistics of the last search on this handle (for benches/tests):
 * out[0] = queries whose exactness certificate failed and took the exact
 * fallback, out[1] = total candidates refined (first pass), out[2] = max pool
 * size,
 * out[3] = 1 if the dense (small-N) path ran, 2 if the one-launch small exact
 * search ran (option "small_exact", default on: <= 8 queries, <= 32768 slots,
 * k <= 64, dim <= 4096), out[4] = queries rerun by the
 * second threshold pass (option "retry_pass", default on: an uncertified
 * query is rescanned with tau = its first-pass k-th exact distance and
 * full-size segments before it may take the exact fallback), out[5] = launches
 * of the threshold append scan in the first pass (2 with option "split_div").
 * Returns 0 or -1. */
int32_t lance_hip_last_search_stats(void *handle, int64_t *out, int32_t n);

/* Per-handle HIP-event timings of the scan kernels (enable with option
 * "time_kernels"="1"; events recorded on the handle's stream around each launch):
 * out[0] total ms of threshold-scan launches, out[1] their count, out[2] rows
 * per launch, out[3] padded queries per launch, out[4] total ms of small-store
 * dense scans, out[5] their count, out[6] bytes per element the scan streams
 * (1 with the int8 scan copy, 2 with a bf16 store or scan copy, else 4),
 * out[7] total ms of IVF list-scan launches, out[8] their count, out[9] their
 * algorithmic bytes (every probed list's rows or codes once + each query's PQ
 * table, summed), out[10] (query, row) pairs scored (summed), out[11] total ms
 * of the IVF coarse searches, out[12] which kernel ran the last timed threshold
 * scan: 2 the int8 scan8_kernel, 0 the LDS-staged scan_kernel.
 * Returns 0 or -1. */
int32_t lance_hip_kernel_times(void *handle, double *out, int32_t n);

/* Device-pointer ingest: num x dim row-major f32 already on the handle's device.
 * Labels [returned, returned+num).  Returns the first label or -1. */
int64_t lance_hip_add_batch_device(void *handle, const float *d_vectors, int64_t num, int32_t dim, char *err_buf,
                                   int err_buf_len);

/* Device-pointer batched search (inputs resident in HBM; synchronous: returns
 * once the device outputs are written).  Same semantics as
 * lance_detached_search_batch.  Returns nq or -1. */
int32_t lance_hip_search_batch_device(void *handle, const float *d_queries, int32_t nq, int32_t dim, int32_t k,
                                      int32_t nprobes, int32_t refine_factor, int64_t *d_out_labels,
                                      float *d_out_distances, int32_t *d_out_counts, char *err_buf, int err_buf_len);

/* NEW — asynchronous device-pointer search (a serving loop that keeps the GPU
 * busy while the host prepares the next batch).  Same arguments and results as
 * lance_hip_search_batch_device, but the call only enqueues the search on the
 * handle's stream and returns a ticket (>= 1) or -1; the results are final —
 * certified, reruns and exact fallbacks done — once lance_hip_search_wait
 * returns for that ticket.  d_queries must be ready on entry (stream-ordered
 * before the call); it and the outputs must stay valid until the wait.  At
 * most two searches are in flight per handle (a third call first completes
 * the oldest); every other call that touches the device or the handle's
 * options (search, add, delete, compact, create_index, get_vector,
 * lance_hip_set_option, ...) first completes every pending one; count,
 * dimension and the statistics getters only read host state.  An IVF search
 * that fits one pass (<= 2048 queries) is enqueued whole (round 6; its
 * coarse-search flags and any rerun at the wait); flat searches that are not a single
 * threshold-path pass (small stores, > 2048 queries) and every search with a
 * predicate or option time_kernels run synchronously inside the call. */
int64_t lance_hip_search_batch_device_async(void *handle, const float *d_queries, int32_t nq, int32_t dim, int32_t k,
                                            int32_t nprobes, int32_t refine_factor, int64_t *d_out_labels,
                                            float *d_out_distances, int32_t *d_out_counts, char *err_buf,
                                            int err_buf_len);

/* NEW — orders the handle's later searches after everything enqueued so far on
 * `caller_stream` (a hipStream_t of the handle's device, NULL = the null stream),
 * without a host wait: an event recorded there that the handle's stream waits on.
 * For a caller that writes the queries (or reads a previous batch's outputs, e.g.
 * an all-gather of them) on its own stream before lance_hip_search_batch_device_async.
 * Multi-device handles wait on the host instead.  0 or -1. */
int32_t lance_hip_stream_after(void *handle, void *caller_stream, char *err_buf, int err_buf_len);

/* NEW — completes every asynchronous search of the handle up to `ticket`
 * (<= 0: all of them).  0 or -1. */
int32_t lance_hip_search_wait(void *handle, int64_t ticket, char *err_buf, int err_buf_len);

/* Device-pointer variant of lance_hip_merge_topk (current device): enqueued on
 * the null stream behind whatever the caller put there (e.g. the all-gather of
 * the partial lists) and returns without waiting; the outputs are ready in that
 * stream's order (a host read through the null stream, or a synchronize, sees
 * them).  Returns nq or -1 (launch errors only). */
int32_t lance_hip_merge_topk_device(int32_t nshard, int32_t nq, int32_t k, const int64_t *d_part_labels,
                                    const float *d_part_dists, const int32_t *d_part_counts, int64_t *d_out_labels,
                                    float *d_out_dists, int32_t *d_out_counts, char *err_buf, int err_buf_len);

/* NEW — the exchange's merge in one launch: nshard packed rows exactly as one
 * all-gather of every rank's row delivers them.  Row s starts at
 * d_gathered + s * row_stride (int32 words, 8-byte aligned, row_stride even and
 * >= lance_hip_merge_packed_stride(nq, k)): labels int64[nq*k] (shard-local),
 * dists f32[nq*k], counts i32[nq], and in the row's last two words the shard's
 * label offset (int64); labels >= 0 are shifted by it before the merge.  Same
 * order, stream and return as lance_hip_merge_topk_device. */
int64_t lance_hip_merge_packed_stride(int32_t nq, int32_t k);
int32_t lance_hip_merge_topk_packed(int32_t nshard, int32_t nq, int32_t k, const int32_t *d_gathered,
                                    int64_t row_stride, int64_t *d_out_labels, float *d_out_dists,
                                    int32_t *d_out_counts, char *err_buf, int err_buf_len);

/* Merge per-shard partial top-k lists into a global top-k, on the device of
 * the handle (multi-GPU path: shards all-gathered over RCCL).
 * part_labels / part_dists: nshard x nq x k (host pointers), part_counts:
 * nshard x nq.  Order (distance asc, label under LANCE_HIP_TIE: descending
 * unless it says label_asc).  Returns nq or -1. */
int32_t lance_hip_merge_topk(int32_t nshard, int32_t nq, int32_t k, const int64_t *part_labels,
                             const float *part_dists, const int32_t *part_counts, int64_t *out_labels,
                             float *out_dists, int32_t *out_counts, char *err_buf, int err_buf_len);

/* NEW — the filtered-search predicate evaluator on a host Arrow batch (struct
 * of [vector, extra...] as lance_detached_add_batch_arrow takes; nothing is
 * taken over, no device needed): out_mask[r] = live[r] && predicate TRUE for
 * row r with label labels[r]; indexed_columns (nullable, comma-separated) are
 * evaluated through a scalar index as lance_detached_create_scalar_index builds
 * it.  Returns the selected count or -1. */
int64_t lance_hip_predicate_mask(void *arrow_schema, void *arrow_array, const int64_t *labels, const uint8_t *live,
                                 const char *predicate, const char *indexed_columns, uint8_t *out_mask, char *err_buf,
                                 int err_buf_len);

/* NEW — IVF state: out[0] type (-1 none, 0 IVF_FLAT, 1 IVF_PQ), out[1] nlist,
 * out[2] m, out[3] dsub, out[4] rows indexed, out[5] slots.  0 or -1. */
int32_t lance_hip_ivf_info(void *handle, int64_t *out, int32_t n);

/* NEW — host copy of the IVF model and per-slot layout (any pointer may be
 * NULL): centroids [nlist][dim], codebook [m][256][dsub], and for every slot
 * (the ascending-label storage order, deleted rows included until compaction):
 * label, live flag, list (-1 = not indexed yet), codes [m].  0 or -1. */
int32_t lance_hip_ivf_export(void *handle, float *centroids, float *codebook, int64_t *slot_labels,
                             uint8_t *slot_live, int32_t *slot_list, uint8_t *slot_codes, char *err_buf,
                             int err_buf_len);

/* NEW — install a trained model (multi-GPU: rank 0 trains, every rank indexes
 * its shard with the same centroids / codebook).  index_type 0 IVF_FLAT, 1
 * IVF_PQ; codebook [m][256][dim/m] (NULL for IVF_FLAT).  0 or -1. */
int32_t lance_hip_ivf_set_model(void *handle, int32_t index_type, int32_t num_partitions, int32_t num_sub_vectors,
                                const float *centroids, const float *codebook, char *err_buf, int err_buf_len);

#ifdef __cplusplus
}
#endif

#endif /* LANCEDB_HIP_H */
