// Internal launcher API between the C-ABI layer (lance_hip_abi.cpp) and the
// gfx950 kernels (knn_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lhip {

enum Metric : int { METRIC_L2 = 0, METRIC_DOT = 1, METRIC_COSINE = 2 };

// Scan tile geometry (see DESIGN.md "Scan kernel").
constexpr int SCAN_BR = 256;  // base rows per workgroup tile (MFMA M)
constexpr int I8_CHUNK_STRIDE = SCAN_BR * 64;  // int8 copy (k-major tiles): bytes between a tile's 64-B k-chunks
constexpr int SCAN_BQ = 256;  // queries per workgroup tile   (MFMA N)
constexpr int SCAN_BK = 64;   // k-step
constexpr int DPAD = 64;      // row stride of the device store is a multiple of this
constexpr int MAX_CAND = 256; // max refined candidates per query per pass
constexpr int MAX_PASS_Q = 2048; // queries per search pipeline pass (SCAN_BQ-query tiles per scan launch)

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// Per-row auxiliary data kept beside the rows (16 B per slot, tile-blocked SoA):
//   x = alpha (f32 |x|^2 for l2, 0 otherwise; +inf = tombstone / padding)
//   y = xn    (|x| for l2/dot, 0 for cosine)
//   z = ux    (upper bound of |bf16(x)| + |x - bf16(x)|; cosine: divided by |x|)
//   w = sc    (1 for l2/dot, 1/|x| for cosine)
struct StoreView {
	const void *X;           // [n_slots][ld] rows, zero padded to ld: f32, or bf16 bits when xbf16
	const float4 *rowaux;    // [n_slots rounded up to SCAN_BR], tile-blocked SoA (raix() in knn_kernels.hip)
	const int64_t *labels;   // [n_slots] slot -> label
	int64_t n_slots;
	int ld;                  // padded row stride (floats), multiple of DPAD
	int dim;
	int metric;
	int xbf16;               // base stored as bf16 (storage option "bf16")
	// What the scan kernels stream: the bf16 scan copy of an f32 store, the
	// bf16 store itself, or (scan_copy off) the f32 rows.  The row aux bounds
	// hold for either: ux covers |x - bf16(x)| with the same RNE rounding.
	const void *Xscan;
	int scan_bf16;
	// int8 scan copy (option scan_i8): Xscan = int8 rows (stride ld bytes) and the
	// scan kernels read scan_aux, its own row terms (alpha, |e_x|, |x~|, scale),
	// instead of rowaux; null / 0 = rowaux and the bf16 / f32 rows above
	const float4 *scan_aux = nullptr;
	int scan_i8 = 0;
	// int8 scan copy: per row tile (s_T, max |e_x|, max |x~|, 0)
	const float4 *tstat = nullptr;
	// per-handle tuning (results exact for every accepted value): pool_refine's
	// first final-mode chunk (0 = default), the ld = 768 scan8 geometry (0 =
	// default; other values only in LHIP_ABLATION_BUILD builds)
	int pr_first = 0;
	int s8_variant = 0;
	// tie rule of the final order (option "tie"): 0 = (distance, label asc),
	// 1 = (distance, label desc) (device_common.h tie_x64)
	int tie_desc = 0;
	// scan8 pair coupling (option "s8_couple", speed only): a workgroup of a pair
	// does not start a 32-row unit more than s8_couple units ahead of its
	// partner's progress (s8_prog: one word per workgroup, epoch-tagged, owned by
	// the pass's stream); 0 = off
	unsigned long long *s8_prog = nullptr;
	int s8_couple = 0;
};

// Per-query constants for the lower-bound epilogue:
//   LB = alpha + xn*B + ux*A + (s*sc)*S + C      (s = bf16 MFMA dot)
struct QueryView {
	const float *Qf;         // [nq_pad][ld] f32 queries, zero padded
	const uint16_t *Qb;      // [nq_pad][ld] bf16 queries (int8 scan: int8 in the first ld bytes of each row)
	const float4 *qaux;      // [nq_pad] (S, A, B, C)
	int nq;
	int nq_pad;              // multiple of SCAN_BQ
};

// ---- ingest ------------------------------------------------------------------
// Computes rowaux for slots [s0, s0+n) of a store (f64 norms, bf16 error norms),
// and folds max(alpha), max(ux) into stats[0], stats[1] (as float bits).
// X holds f32 rows, or bf16 bits when xbf16.
void launch_rowaux(const void *X, int xbf16, int ld, int dim, int metric, int64_t s0, int64_t n, float4 *rowaux,
                   unsigned *stats, hipStream_t st);

// Rounds n f32 rows (stride src_ld) to bf16 (round to nearest even) into
// dst rows of stride ld, zero-filling columns [dim, ld).
void launch_rows_to_bf16(const float *src, int64_t src_ld, int64_t n, int dim, int ld, uint16_t *dst, hipStream_t st);

// int8 scan copy of the row tiles [t0, t1) (SCAN_BR rows each) of an f32 store
// holding n_slots rows: one scale per tile, int8 rows Xq (stride ld bytes, zero
// padded; rows past n_slots zero), their row terms aux8 (tombstones copied from
// rowaux, rows past n_slots +inf) and per-tile terms tstat[t] = (s_T, max |e_x|,
// max |x~|, 0); folds max |alpha| and max(xn, ux) into stats[0], stats[1] (float bits).
void launch_tiles_to_i8(const void *X, int xbf16, int ld, int dim, int metric, int64_t n_slots, int64_t t0,
                        int64_t t1, const float4 *rowaux, int8_t *Xq, float4 *aux8, float4 *tstat, unsigned *stats,
                        hipStream_t st);

// rowaux[from, to) = (+inf, 0, 0, 0): padding rows past the last slot.
void launch_fill_rowaux(float4 *rowaux, int64_t from, int64_t to, hipStream_t st);

// Marks the listed slots dead (rowaux.x = +inf).
void launch_tombstone(float4 *rowaux, const int64_t *slots, int n, hipStream_t st);
// dst = src with alpha = +inf on slots [0, n_slots) whose mask byte is 0
// (filtered search); rows [0, cap) copied
void launch_filter_rowaux(const float4 *src, const uint8_t *mask, int64_t n_slots, int64_t cap, float4 *dst,
                          hipStream_t st);

// ---- search ------------------------------------------------------------------
// int8 scan (scan_i8): int8 queries (one scale for the batch) into Qb's rows
// (first ld bytes of each 2*ld-byte row) and the int8 bound's constants; Qf and
// zero3 as below; qm = nq scratch float2 (per-query maxima).
void launch_prep_queries_i8(const float *Q, int nq, int dim, int ld, int nq_pad, int metric, float max_alpha,
                            float max_x, float2 *qm, float *Qf, uint16_t *Qb, float4 *qaux, int *zero3,
                            hipStream_t st);
// Also zeroes zero3[0 .. 3*nq) when non-null (the search's status words).
void launch_prep_queries(const float *Q, int nq, int dim, int ld, int nq_pad, int metric, float max_alpha,
                         float max_ux, float *Qf, uint16_t *Qb, float4 *qaux, int *zero3, hipStream_t st);

// Dense lower-bound scan over row tiles t*tile_stride, t < n_tiles:
// out[q][t*BR + r] = LB(q, slot) (+inf for tombstones / rows past n_slots).
void launch_scan_dense(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, float *out,
                       int64_t ld_out, hipStream_t st);

// Threshold scan over all rows (persistent: scan_grid(n_tiles) workgroups):
// workgroup g appends (orderedkey(LB), slot) for LB <= tau[q] into its own
// segment seg_pool[(g*nq + q)*seg_cap ..], count in seg_cnt[g*nq + q] (may
// exceed seg_cap: overflow is reported by select).  seg_pool holds scan_grid(n_tiles) *
// (nq_pad / SCAN_BQ) more entries past the segments: per-workgroup sink words.
void launch_scan_append(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                        int seg_cap, hipStream_t st);

// Sample scan over row tiles t*tile_stride, t < n_tiles (persistent, scan_grid(n_tiles)
// workgroups): for every tile, each 64-row quarter appends its smallest lower
// bound per query, (orderedkey(LB), slot), to the workgroup's segment as
// launch_scan_append does (4 entries per tile and query; +inf bounds skipped).
void launch_scan_tilemin(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, uint2 *seg_pool,
                         int *seg_cnt, int seg_cap, hipStream_t st);

// Workgroups a scan over n_tiles tiles launches (= min(n_tiles, CUs)).
int scan_grid(int64_t n_tiles);

// The int8 append pass by scan8_kernel (scan8_kernels.hip): workgroup PAIRS,
// each half of a 256-query tile resident in LDS, rows HBM -> registers, bounds
// screened in exact integers (tile / batch common scales).  Applies to an int8
// scan copy with ld in [512, 1024]; writes scan8_segments(n_tiles) segments per
// query (one per pair) in launch_scan_append's format.  A tile range [t0, t1)
// (t1 < 0: to the end) writes its segments from segment seg_base on, so two
// launches over disjoint ranges fill disjoint segment sets of one pool.
bool scan8_fits(const StoreView &s);
int scan8_segments(int64_t n_tiles);
int scan8_prog_words();  // StoreView::s8_prog words (pair coupling)
bool scan8_variant_ok(int v);  // a geometry this build carries (release: 0 only)
void launch_scan8_append(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                         int seg_cap, hipStream_t st, int64_t t0 = 0, int64_t t1 = -1, int seg_base = 0);
// The sample pass on the int8 copy (scan8_kernel, tilemin mode): row tiles
// t * tile_stride, t < n_tiles; per tile, query and 32-row unit the row of
// smallest bound -> (orderedkey(LB), slot) into scan8_segments(n_tiles)
// segments per query of capacity >= scan8_tilemin_cap(n_tiles) (+inf / NaN
// bounds skipped), launch_scan_tilemin's format.
int scan8_tilemin_cap(int64_t n_tiles);
void launch_scan8_tilemin(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, uint2 *seg_pool,
                          int *seg_cnt, int seg_cap, hipStream_t st);
// Segments per query launch_scan_append writes for this store.
int scan_append_segments(const StoreView &s, int64_t n_tiles);

// Per-query top-M selection by LB.  Writes cand_slot[q][0..M), cand_cnt[q] and
// the cut cut[q] = a lower bound on the true distance of every live row not
// selected (+inf when nothing live was left out; -inf when unknown -> the
// certificate fails).  Dense source: n_entries per query, entry i -> slot
// (i/BR)*stride*BR + i%BR.  Segment source: the append scan's output;
// pool_total[q] = entries seen (-1 on overflow); tau may be null (= +inf).
// tie_desc: equal keys straddling the M-th place are taken by slot descending
// (the exact fallback under the label-descending tie rule), else ascending.
void launch_select_dense(const float *dense, int64_t ld_dense, int64_t n_entries, int64_t tile_stride, int nq, int M,
                         uint32_t *cand_slot, int *cand_cnt, float *cut, hipStream_t st, int tie_desc);
void launch_select_segments(const uint2 *seg_pool, const int *seg_cnt, int seg_cap, int n_seg, const float *tau,
                            int nq, int M, uint32_t *cand_slot, int *cand_cnt, float *cut, int *pool_total,
                            int *big, hipStream_t st);

// Select + refine + finalize of a threshold pass in one launch: per query the
// segments (every row with LB <= tau) sorted by (LB, slot) and refined in that
// order.  mode 1 (final): until the next bound exceeds the k-th exact distance;
// writes top-k L / D / C and the certificate (as finalize, incl. the live-count
// check; tau may be null = +inf).  mode 0 (sample): refines the m_tau smallest
// bounds, tau_out[q] = their k-th smallest exact distance (+inf when fewer,
// NaN when any is NaN).  refined[q] = rows refined, pool_total[q] = pool size
// (-1 on overflow); both may be null.  n_seg <= 512, k <= MAX_CAND.
// first chunk of pool_refine's final mode: StoreView::pr_first (handle option
// "pr_first"), clamped to [8, pool_refine_max_first()]
int pool_refine_max_first();
void launch_pool_refine(const StoreView &s, const QueryView &q, const uint2 *seg_pool, const int *seg_cnt,
                        int seg_cap, int n_seg, const float *tau, int k, int mode, int m_tau, int64_t live,
                        float *tau_out, int64_t *L, float *D, int *C, int *cert, int *refined, int *pool_total,
                        hipStream_t st);

// Exact distances (f64 accumulation, rounded to f32) of the candidates.
void launch_refine(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt, int M,
                   float *cand_dist, hipStream_t st);

// refine + finalize mode 0 in one launch: tau[q] = the need-th smallest exact
// distance of the candidates (+inf when fewer, NaN when any is NaN).
void launch_refine_tau(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt, int M,
                       int need, float *tau, hipStream_t st);

// Sort candidates by (distance, label).  mode 0 (TAU): tau[q] = largest exact
// distance among the candidates when at least need_for_tau of them exist, else
// +inf.  mode 1 (FINAL): writes top-k, counts and the certificate ok[q] (false when
// live >= 0 and fewer than min(k, live) hits came out).
void launch_finalize(const StoreView &s, const uint32_t *cand_slot, const int *cand_cnt, const float *cand_dist,
                     const float *cut, int nq, int M, int k, int mode, int need_for_tau, float *tau,
                     int64_t *out_labels, float *out_dists, int *out_counts, int *cert_ok, hipStream_t st,
                    int64_t live = -1);

// Exact fallback for one query: exact distance of every slot into keys[n_slots]
// (dead slots -> NaN with all-ones payload so they sort last), labels into vals;
// under the label-descending tie rule in reverse slot order (entry n-1-slot),
// so that a stable ascending sort puts equal distances in label-descending order.
void launch_exact_all(const StoreView &s, const QueryView &q, int qi, float *keys, int64_t *vals, hipStream_t st);

// Batched exact fallback: keys[i][r] (row stride ld_keys >= n_slots) = exact
// distance of slot r to query i of q (the value refine computes), +inf for
// dead / filtered slots; feeds launch_select_dense with tile_stride 1.
void launch_exact_dense(const StoreView &s, const QueryView &q, float *keys, int64_t ld_keys, hipStream_t st);

// Radix sort (key f32 asc, stable) of n pairs; temp sized by the first call with
// temp == nullptr.  Returns hipError_t as int.
int sort_pairs(void *temp, size_t &temp_bytes, const float *keys_in, float *keys_out, const int64_t *vals_in,
               int64_t *vals_out, int64_t n, hipStream_t st);

// Small exact search (one launch): nq <= SMALL_MAX_Q queries (Q = [nq][dim]
// f32, unpadded, device) over a store of <= SMALL_MAX_ROWS slots; exact f64
// distances, per-workgroup top-k, last-workgroup merge.  part = 16 B x nq x
// small_exact_grid(n_slots) x k scratch; counter = nq zeroed words (left
// zeroed).  Writes labels/distances/counts like finalize.
constexpr int SMALL_THREADS = 256;
constexpr int SMALL_MAX_ROWS = 32768;
constexpr int SMALL_MAX_DIM = 4096;
constexpr int SMALL_MAX_Q = 8;
constexpr int SMALL_MAX_K = 64;
constexpr int SMALL_MAX_PART = 4096;
bool small_exact_fits(int64_t n_slots, int dim, int nq, int k);
int small_exact_grid(int64_t n_slots);
void launch_small_exact(const StoreView &s, const float *Q, int nq, int k, void *part, unsigned *counter, int64_t *L,
                        float *D, int *C, hipStream_t st);

// Second threshold pass of failed queries fq[0..nf): packs their prepared
// query rows into Qf2/Qb2/qaux2 (nf_pad rows, pads zero), tau2[i] = min(tau,
// first-pass k-th exact distance) (keep_tau: tau itself — a rerun that only
// widens the selection), zeroes status2 = [cert | cnt | pool] x nf.
void launch_retry_gather(const int *fq, int nf, int nf_pad, int ld, int k, const QueryView &q, const float *tau,
                         const float *dists, float *Qf2, uint16_t *Qb2, float4 *qaux2, float *tau2, int *status2,
                         hipStream_t st, int keep_tau = 0);
// Writes back the rerun results of the queries the rerun certified; for the
// others tau[q] = min(tau2, rerun k-th exact distance) for a further rerun.
void launch_retry_scatter(const int *fq, int nf, int k, const int64_t *L2, const float *D2, const int *C2,
                          const int *cert2, const float *tau2, int64_t *L, float *D, int *C, int *cert, float *tau,
                          hipStream_t st);

// Merge nshard partial top-k lists (device pointers) into the global top-k,
// (distance, label) order under the tie rule tie_desc.
void launch_merge_topk(int nshard, int nq, int k, const int64_t *part_labels, const float *part_dists,
                       const int *part_counts, int64_t *out_labels, float *out_dists, int *out_counts,
                       hipStream_t st, int tie_desc);

// The same merge over nshard packed rows of one all-gather (row s at
// gathered + s * stride int32 words: labels int64[nq*k], dists f32[nq*k],
// counts i32[nq], the shard's label offset int64 in the last two words);
// local labels >= 0 are shifted by their shard's offset.  stride is even.
void launch_merge_packed(int nshard, int nq, int k, const int32_t *gathered, int64_t stride, int64_t *out_labels,
                         float *out_dists, int *out_counts, hipStream_t st, int tie_desc);

// Copies the first n_live entries of a sorted fallback result into the outputs.
void launch_copy_fallback(const float *keys, const int64_t *vals, int64_t n_live, int k, int qi,
                          int64_t *out_labels, float *out_dists, int *out_counts, hipStream_t st);

// Gathers slots idx[0..n) of a store into a new store (same ld), in order.
// Used by lance_detached_compact (drops tombstones, keeps label order).
void launch_gather_rows(const void *X, int xbf16, const float4 *rowaux, const int64_t *labels, const int64_t *idx,
                        int64_t n, int ld, void *Xo, float4 *rowaux_o, int64_t *labels_o, hipStream_t st);

}  // namespace lhip
