// IVF_FLAT / IVF_PQ indexes of the MI355X-native path (internal; not public ABI).
//
// Replaces what lance_manager.rs:483-515 (create_ann_index -> lancedb 0.15
// IvfPqIndexBuilder -> lance-index 0.22 k-means + PQ training) builds and what
// lance_manager.rs:411-418 (vector_search(..).nprobes(n).refine_factor(r))
// searches, paths relative to /root/reference.  Layout and kernels: DESIGN.md
// "IVF".  Canonical numerics (restated by oracle/ivf.py):
//   coarse   exact distances to the centroids (f64 accumulate, f32 result),
//            top-nprobe by (distance, list id)
//   IVF_FLAT exact distance of every live row of the probed lists,
//            top-k by (distance, label)
//   IVF_PQ   ADC(q, row) = (d0 + tau_row) + sum_j LUT[j][code_j], summed in f32
//            in j order, d0 = the coarse distance of the row's list, LUT =
//            -2 P[q] and tau_row = sum_j T[list][j][code_j] (f32, j order, from
//            0) for L2 / cosine (residual PQ); LUT = -P[q], tau = 0 for dot; with
//              P[q][j][c] = sum_t q_{j,t} * y_{j,c,t}
//              T[l][j][c] = sum_t y_{j,c,t} * (y_{j,c,t} + 2 c_{l,j,t})
//            (f32, t in order, no fused multiply-add); top-(k*refine_factor)
//            by (ADC, label) -> exact re-rank -> top-k by (distance, label)
//   rows added after the build (slots >= n_indexed) are searched exactly and
//   merged (LanceDB searches unindexed fragments flat); cosine works in the
//   row-normalised space (k-means, residuals, P), exact cosine at the end.
#pragma once
#include "index.h"

namespace lhip {

enum IvfType : int { IVF_FLAT = 0, IVF_PQ = 1 };
constexpr int PQ_K = 256;          // 8-bit codes (nbits = 8)
constexpr int PQ_MAX_M = 128;      // LUT of m x 256 f32 must fit in LDS with the top-k buffer
constexpr int PQ_MAX_DSUB = 64;    // codebook slice of one sub-space in LDS
constexpr int IVF_TOPK_CAP = 2048; // LDS top-k buffer of the list scans / merges
constexpr int IVF_MAX_K = 1024;    // k (and k * refine_factor) bound of the IVF path
constexpr int FLAT_BLK = 256;      // rows per IVF_FLAT list-scan work item
constexpr uint32_t SLOT_NONE = 0xFFFFFFFFu;
// IVF_PQ fast scan (pq_fast_scan_kernel): FQ_G queries share one LUT lookup
constexpr int FQ_G = 4;             // queries per work item (4 byte lanes of a u32)
constexpr int FQ_THREADS = 512;
constexpr int FQ_CAP = 1024;        // LDS candidate buffer per query of an item
constexpr int FQ_CHUNK = 8192;      // list positions per work item
constexpr int FQ_MAX_M = 96;        // LUT u32 [m][256] + FQ_G x FQ_CAP keys in LDS
constexpr int FQ_MAX_KK = 512;      // k * refine_factor bound of the fast scan
constexpr int FL_KEYS = 16;         // IVF_FLAT bound scan: (LB, slot) keys per (query, item); k <= FL_KEYS - 1

struct IvfState {
	int type = IVF_PQ;
	int nlist = 0, m = 0, dsub = 0, mp = 0;  // mp = code bytes per row, multiple of 16
	int metric = METRIC_L2;                  // index metric
	int64_t n_indexed = 0;                   // slots [0, n_indexed) are in the lists
	Index *coarse = nullptr;                 // centroid store (exact top-nprobe)
	DevBuf<float> centroids;                 // [nlist][ld] f32, zero padded
	DevBuf<float> codebook;                  // [m][256][dsub]
	DevBuf<float> T;                         // [nlist][m][256] (L2 / cosine)
	DevBuf<int> assign;                      // [n_indexed] list of each indexed slot
	DevBuf<uint8_t> codes;                   // [n_indexed][mp] slot-major codes
	// list layout (rebuilt when dirty): positions padded to 64 per list
	bool dirty = true;
	std::vector<int64_t> h_loff;             // [nlist+1]
	std::vector<int64_t> h_lcnt;             // [nlist] rows per list (unpadded)
	DevBuf<int64_t> loff;
	DevBuf<uint32_t> lslot;                  // [npos] slot, SLOT_NONE for padding
	DevBuf<uint8_t> lcodes;                  // [npos][mp] codes, row-major in list order
	DevBuf<float> ltau;                      // [npos] row term of the L2 / cosine ADC (list order)
	DevBuf<int> blk_list, lblk0;             // IVF_FLAT work items (256 positions each)
	// IVF_FLAT bound scan: the bf16 (RNE) rows in list position order, [npos + 256][ld]
	// (zero rows for padding): an item's 256 rows are one contiguous 256 x ld block
	DevBuf<uint16_t> lrows;
	DevBuf<float4> lterms;  // [npos + FLAT_BLK] row terms in list order at layout time (with lrows)
	bool lrows_ok = false;
	DevBuf<int64_t> blk_pos0;
	int nblk = 0, maxb = 1;
	// search workspace
	DevBuf<float> Qf, Qn, P, probe_d, tmpf;
	DevBuf<double> Qd, qn2;
	DevBuf<int64_t> probe_l, pref;
	DevBuf<int> probe_c, lcnt, pstart, pairs;
	DevBuf<uint64_t> keys, tkeys, cand_a, cand_b, best;
	DevBuf<uint8_t> tmpb;
	// fast PQ scan workspace
	DevBuf<float> Qq;                        // fp8-rounded queries (option pq_query = fp8)
	DevBuf<uint8_t> lut8;                    // [nq][m][256]
	DevBuf<float> qpar;                      // [nq] (D, L0) pairs
	DevBuf<int> item_off, work, ocnt, xbeg;
	DevBuf<int4> itab;  // fast-scan item table (launch_pq_fast_items)
	DevBuf<int> boff, btot;  // IVF_FLAT bound scan: work items per block, their total
	DevBuf<int> itb;         // IVF_FLAT bound scan: item -> block table (flat_lb_table_kernel)
	DevBuf<uint32_t> live_bits;  // IVF_FLAT bound scan: live slots of the search (1 bit each)
	DevBuf<uint64_t> thrq, okeys;
	// IVF_FLAT bound scan workspace
	DevBuf<float> lbQf, cut;
	DevBuf<uint16_t> lbQb;
	DevBuf<float4> lbqaux;
	DevBuf<int> cert;
	std::vector<int> h_cert;
	// fused coarse search (coarse_kernels.hip): per (query, partition) bounds, per-query fallback flags
	DevBuf<float2> cbnd;
	DevBuf<int> cflag;
	// pinned, 2 x MAX_PASS_Q: the flags' copy is enqueued with the pass and read
	// after its completion (two slots: two asynchronous searches in flight)
	int *h_cflag = nullptr;
	int cflag_slot = 0;
	~IvfState();
};

// ---- fused coarse search (coarse_kernels.hip) ----------------------------------
// top-nprobe partitions of nq queries Q [nq][dim] (device, unpadded) over the
// centroid rows C [nc][ld] f32, exact (the flat path's order and distances):
// probe_l / probe_d [nq][nprobe], probe_c [nq]; flag[q] = 1 when query q must
// take the flat path instead (non-finite bounds, candidate overflow); such a
// query's probes are written as -1 / NaN / count 0, so the rest of the pass can
// run before the host reads the flags.
// bnd: nq * nc float2 scratch.
bool coarse_fused_fits(int dim, int nc, int nprobe);
void launch_coarse_search(const float *Q, int nq, int dim, const float *C, int ld, int nc, int metric, int nprobe,
                          float2 *bnd, int64_t *probe_l, float *probe_d, int *probe_c, int *flag, hipStream_t st);

// ---- host API (ivf_index.cpp) -----------------------------------------------
// lance_detached_create_index: train (k-means on a seeded sample, PQ on the
// residuals) and index every live row.  num_partitions / num_sub_vectors <= 0
// take LanceDB's defaults (sqrt(rows); dim/16, dim/8 or 1).
void ivf_build(Index *ix, int type, int num_partitions, int num_sub_vectors);
// Install a given model (multi-GPU: rank 0 trains, every rank indexes its own
// shard with the same centroids / codebook).  codebook may be null for IVF_FLAT.
void ivf_set_model(Index *ix, int type, int nlist, int m, const float *centroids, const float *codebook);
// lance_detached_compact (= optimize(All)): index the rows added since the build.
void ivf_optimize(Index *ix);
// Batched IVF search; device pointers.  Synchronous, unless `defer` is given
// and the search is one pass: then everything is enqueued on the handle's
// stream, defer->ivf is set, and ivf_finish completes it once the stream has
// passed it (the fused coarse flags' check, a rerun on the flat coarse path).
void ivf_search(Index *ix, const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD, int *dC,
                PendingPass *defer = nullptr);
void ivf_finish(Index *ix, PendingPass &p);

// Host copies of the model (centroids [nlist][dim], codebook [m][256][dsub]) and
// of the per-slot list / codes (slots >= n_indexed: list -1, codes 0).
void ivf_export_model(Index *ix, float *centroids, float *codebook);
void ivf_export_slots(Index *ix, int32_t *slot_list, uint8_t *slot_codes);

// ---- kernel launchers (ivf_kernels.hip) -------------------------------------
void launch_gather_sample(const void *X, int xbf16, int ld, int dim, const int64_t *slots, int64_t n, int normalize,
                          float *out_f32, uint16_t *out_bf16, hipStream_t st);
void launch_centroid_prep(const float *C, int nc, int nc_pad, int ld, uint16_t *Cb, float *cnorm, hipStream_t st);
// best[r] = min over centroids of (orderedkey(|c|^2 - 2 s_r x_r.c) << 32 | c), bf16 MFMA dot products.
// Rows: X (f32 or bf16 bits, stride ld) rows r0 + r for r < n; s_r = 1 or the
// row scale (rowaux w, cosine).  best must be pre-set to ~0.
void launch_kmeans_assign(const void *X, int xbf16, int ld, int64_t r0, int64_t n, const float *row_scale_aux,
                          const uint16_t *Cb, const float *cnorm, int nc_pad, uint64_t *best, hipStream_t st);
// same with f32 centroids [nc_pad][ld] and exact-f32 MFMA products (row placement)
void launch_kmeans_assign_f32(const void *X, int xbf16, int ld, int64_t r0, int64_t n, const float *row_scale_aux,
                              const float *Cf, const float *cnorm, int nc_pad, uint64_t *best, hipStream_t st);
// sum over rows of the winning score (f64, for the k-means stopping rule)
void launch_score_sum(const uint64_t *best, int64_t n, double *out, hipStream_t st);
void launch_sq_sum(const float *v, int64_t n, double *out, hipStream_t st);
void launch_gather_bytes(const uint8_t *src, const int64_t *idx, int64_t n, int row_bytes, uint8_t *dst,
                         hipStream_t st);
void launch_best_to_assign(const uint64_t *best, int64_t n, int *assign, uint32_t *keys, uint32_t *vals,
                           hipStream_t st);
int sort_u32_pairs(void *temp, size_t &temp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                   uint32_t *vout, int64_t n, int end_bit, hipStream_t st);
void launch_segments(const uint32_t *sorted_keys, int64_t n, int nseg, int *seg_start, hipStream_t st);
void launch_centroid_mean(const float *S, int ld, int dim, const uint32_t *sorted_idx, const int *seg_start, int nc,
                          float *C, hipStream_t st);
void launch_residuals(const float *S, const int *assign, const float *C, int ld, int64_t n, float *R,
                      hipStream_t st);
void launch_pq_assign(const float *R, int ld, int64_t n, int m, int dsub, const float *cb, uint32_t *keys,
                      uint32_t *vals, hipStream_t st);
void launch_pq_mean(const float *R, int ld, const uint32_t *sorted_idx, const int *seg_start, int m, int dsub,
                    float *cb, hipStream_t st);
void launch_pq_encode(const void *X, int xbf16, int ld, int dim, int64_t s0, int64_t n, const float *rowaux_f,
                      int normalize, const int *assign, const float *C, const float *cb, int m, int dsub, int mp,
                      uint8_t *codes, hipStream_t st);
void launch_pq_tables_T(const float *C, int ld, const float *cb, int nlist, int m, int dsub, float *T,
                        hipStream_t st);
void launch_pq_layout(const uint8_t *codes, const uint32_t *lslot, int64_t npos, int mp, uint8_t *lcodes,
                      hipStream_t st);
// search side
void launch_ivf_prep(const float *Q, int nq, int dim, int ld, int normalize, float *Qf, float *Qn, hipStream_t st);
// probes -> per-list query sets (pstart [nlist + 1], pairs).  With loff (needs
// invert_fused_fits): also the fast scan's item_off / xbeg, as launch_pq_fast_items
// would lay them out (then call it with offsets_done)
bool invert_fused_fits(int nlist);
void launch_invert(const int64_t *probe_l, int nq, int nprobe, int nlist, int *lcnt, int *pstart, int *pairs,
                   hipStream_t st, const int64_t *loff = nullptr, int *item_off = nullptr, int *xbeg = nullptr);
void launch_flat_list_scan(const StoreView &s, const int *blk_list, const int64_t *blk_pos0, const int *lblk0,
                           const int64_t *loff, const uint32_t *lslot, int nblk, const int *pstart, const int *pairs,
                           int nprobe, int maxb, int64_t tail_s0, int64_t tail_n, int nq, const double *Qd,
                           const double *qn2, int kk, uint64_t *out, hipStream_t st);
// IVF_FLAT bound scan (MFMA bf16 lower bounds): out [pair][maxb][16] (LB, slot) keys per (query, item);
// rows from lrows (list order, launch_list_rows_bf16) or, when null, from the store's bf16 scan rows by slot
void launch_flat_list_lb(const StoreView &s, const int *blk_list, const int64_t *blk_pos0, const int *lblk0,
                         const int64_t *loff, const uint32_t *lslot, int nblk, const int *pstart, const int *pairs,
                         int nprobe, int maxb, const uint16_t *Qb, const float4 *qaux, uint64_t *out, hipStream_t st,
                         const uint16_t *lrows, const float4 *lterms, uint32_t *live_bits /* [n_slots / 32 + 1] */,
                         int *boff /* [nblk + 1] */, int *tot /* [1] */,
                         int *itb = nullptr /* item -> block table, itb_cap entries */, int itb_cap = 0);
// out [npos] = (xn, ux, sc, 0) of the row at each list position (the bound scan's list-order row terms)
void launch_list_terms(const float4 *rowaux, const uint32_t *lslot, int64_t npos, float4 *out, hipStream_t st);
// out [npos][ld] = bf16 (RNE) of the row at each list position (f32 or bf16 store X), zero for padding
void launch_list_rows_bf16(const void *X, int xbf16, int ld, int dim, const uint32_t *lslot, int64_t npos,
                           uint16_t *out, hipStream_t st);
// per query: top-M bound candidates of its probed lists and the cut (every other row has LB >= cut)
void launch_flat_lb_merge(int nq, int nprobe, const int64_t *probe_l, const int *lblk0, int maxb, const uint64_t *keys,
                          int M, uint64_t *cand, float *cut, hipStream_t st);
// exact re-rank + tail merge + certificate (cert[q] = 1 when no left-out row can enter the top k)
void launch_flat_lb_refine(const StoreView &s, const float *Qf, const uint64_t *ca, int M, const uint64_t *cb, int kb,
                           const float *cut, int nq, int k, int64_t *outL, float *outD, int *outC, int *cert,
                           hipStream_t st);
// Qd [nq][ld] f64 copy of the padded f32 queries Qf, qn2 [nq] = sum of q^2 in element order
void launch_ivf_qd(const float *Qf, int nq, int ld, int dim, double *Qd, double *qn2, hipStream_t st);
void launch_pq_P(const float *Q, int qld, int nq, const float *cb, int m, int dsub, float *P, hipStream_t st);
// pref [nq][nprobe+1]: exclusive prefix of the probed lists' padded lengths
void launch_probe_prefix(const int64_t *probe_l, int nq, int nprobe, const int64_t *loff, int64_t *pref,
                         hipStream_t st);
// segments per query of the IVF_PQ scan (grid S x nq)
int pq_segments(int nq);
// out [nq][S][kk]: per (query, segment) top-kk (ADC, slot) keys
void launch_pq_query_scan(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                          const float *rowaux_f, int nq, int nprobe, const int64_t *probe_l, const float *probe_d,
                          const float *ltau, const float *P, const int64_t *pref, int S, int kk, uint64_t *out,
                          hipStream_t st);
// fp8 (OCP e4m3fn) queries for the ADC tables: Qo = e4m3(Q / s) * s, s = absmax / 448 per query
void launch_pq_query_fp8(const float *Q, int qld, int nq, int dim, float *Qo, hipStream_t st);
// 8-bit LUTs lut8 [nq][m][256] and qpar [nq] = (D, L0) from P (see pq_lut_u8_kernel)
void launch_pq_lut_u8(const float *P, int nq, int m, float sP, uint8_t *lut8, float2 *qpar, hipStream_t st);
// fp8 rounding (fp8 != 0) + ADC table + 8-bit LUT of each query in one launch
// (pq_query_fp8 + pq_P + pq_lut_u8, bit-identical); Q [nq][qld], dim = m * dsub
bool pq_lut_fused_fits(int m, int dim);
void launch_pq_lut_fused(const float *Q, int qld, int nq, int dim, int fp8, const float *cb, int m, int dsub, float sP,
                         uint8_t *lut8, float2 *qpar, hipStream_t st);
// item_off [nlist+1]: work items of the fast scan per list (query groups x row chunks), lists in
// XCD-major order; xbeg [9]: each XCD's item range
// itab [2 x items] (when non-null): per item (list, row chunk, -, -), (pair ids of its query group)
void launch_pq_fast_items(const int *pstart, const int64_t *loff, const int *pairs, int nlist, int *item_off,
                          int *xbeg, int4 *itab, int itab_cap, hipStream_t st, bool offsets_done = false);
// per query: the kk-th smallest fast-scan key of its nearest probed list -> thrq (atomicMin)
void launch_pq_seed(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                    const float *rowaux_f, int nq, int nprobe, const int64_t *probe_l, const float *probe_d,
                    const float *ltau, const uint8_t *lut8, const float2 *qpar, int kk, uint64_t *thrq, hipStream_t st);
int pq_fast_lds_bytes(int m);
// list-major 8-bit-LUT scan: per query its candidate run out [nq][ocap] (count ocnt[q]);
// work (8 ints: one claim counter per XCD), thrq [nq] (~0) and ocnt [nq] (0) must be initialised
void launch_pq_fast_scan(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                         const float *rowaux_f, int nlist, int nprobe, const int *pstart, const int *pairs,
                         const int *item_off, const int *xbeg, const float *probe_d, const float *ltau,
                         const uint8_t *lut8, const float2 *qpar, int kk, int *work, uint64_t *thrq, int *ocnt,
                         uint64_t *out, int ocap, const int4 *itab, int grid, hipStream_t st);
void launch_pq_run_merge(const uint64_t *keys, const int *ocnt, int nq, int ocap, int K, uint64_t *out,
                         hipStream_t st,
                         const uint64_t *thrq = nullptr);
// ltau [npos]: per list position sum_j T[l][j][c_j] (f32, j ascending), 0 for padding
void launch_pq_tau(const uint8_t *codes, const uint32_t *lslot, const int64_t *loff, int nlist, int64_t npos, int m,
                   int mp, const float *T, float *ltau, hipStream_t st);
// per query: top-K keys over the list-scan outputs of its probes (nblk_of
// lists via lblk0, or 1 per probe when lblk0 is null) and/or a tail output.
void launch_ivf_merge(int nq, int nprobe, const int64_t *probe_l, const int *lblk0, int maxb, int kk,
                      const uint64_t *keys, int tail_nb, const uint64_t *tkeys, int K, uint64_t *out, hipStream_t st);
void launch_keys_to_output(const uint64_t *keys, int nq, int K, int k, const int64_t *labels, int64_t *outL,
                           float *outD, int *outC, hipStream_t st, int tie_desc);
void launch_ivf_refine_final(const StoreView &s, const float *Qf, const uint64_t *ca, int ka, const uint64_t *cb,
                             int kb, int nq, int k, int64_t *outL, float *outD, int *outC, hipStream_t st);

}  // namespace lhip
