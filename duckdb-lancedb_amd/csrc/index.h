// Internal: the handle behind the C-ABI (lhip::Index), its device store and
// workspace.  Shared by lance_hip_abi.cpp (flat path, C-ABI) and ivf_index.cpp
// (IVF_FLAT / IVF_PQ, lance_manager.rs:483-515).  Not part of the public ABI.
#pragma once
#include "knn_kernels.h"
#include "meta.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <vector>

namespace lhip {

struct IvfState;            // ivf_index.cpp
struct Index;
void ivf_free(IvfState *s);  // ivf_index.cpp
// compaction keeps slots `keep` (ascending old slots): carry the IVF list
// assignment / PQ codes of the kept indexed rows over to their new slots
void ivf_remap(Index *ix, const std::vector<int64_t> &keep);

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
struct Error : std::runtime_error {
	using std::runtime_error::runtime_error;
};

#define HIPCHK(expr)                                                                                                   \
	do {                                                                                                               \
		hipError_t _e = (expr);                                                                                        \
		if (_e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " #expr);          \
	} while (0)

// Completion wait of a search: spins on the stream (a blocking wait costs tens
// of microseconds of wake-up per call, ~10% of a C2 batch).
inline void spin_sync(hipStream_t st) {
	hipError_t e;
	while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
	}
	if (e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e) + " at stream completion");
}

inline void write_err(char *buf, int len, const std::string &msg) {
	if (!buf || len <= 0) return;
	size_t n = std::min(msg.size(), (size_t)(len - 1));
	memcpy(buf, msg.data(), n);
	buf[n] = 0;
}

inline int metric_id(const std::string &m) {
	// lance_manager.rs:493-497: cosine -> Cosine, dot|ip -> Dot, else L2
	if (m == "cosine") return METRIC_COSINE;
	if (m == "dot" || m == "ip") return METRIC_DOT;
	return METRIC_L2;
}

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
template <typename T>
struct DevBuf {
	T *p = nullptr;
	size_t n = 0;  // capacity in elements
	~DevBuf() { release(); }
	void release() {
		if (p) (void)hipFree(p);
		p = nullptr;
		n = 0;
	}
	// grow without preserving contents
	void need(size_t m) {
		if (m <= n) return;
		release();
		size_t c = std::max(m, (size_t)1);
		HIPCHK(hipMalloc(&p, c * sizeof(T)));
		n = c;
	}
};

// Per-pass buffers of the flat pipeline: the prepared queries, tau and the
// status words [cert | cand_cnt | pool_cnt] x nq (pinned host memory the
// threshold path's kernels write in place; the dense path's copy in HBM).
// Two sets: an asynchronous pass still in flight keeps its own while the next
// pass is enqueued (Index::search_async).
struct PassBufs {
	DevBuf<float> Qf, tau;
	DevBuf<uint16_t> Qb;
	DevBuf<float4> qaux;
	DevBuf<float2> qm;  // int8 queries: per-query maxima (the batch scale)
	DevBuf<int> status;
	DevBuf<uint2> seg_pool;       // threshold path: per-(workgroup, query) segments of this pass
	DevBuf<int> seg_cnt;
	DevBuf<unsigned long long> s8prog;  // scan8 pair-coupling progress words (epoch-tagged: zeroed once)
	int *h_status = nullptr;      // pinned
	int *d_status_map = nullptr;  // its device-visible address
	size_t h_status_n = 0;
	hipEvent_t done = nullptr;    // end of an asynchronous pass
	PassBufs() = default;
	PassBufs(const PassBufs &) = delete;
	PassBufs &operator=(const PassBufs &) = delete;
	~PassBufs() {
		if (h_status) (void)hipHostFree(h_status);
		if (done) (void)hipEventDestroy(done);
	}
	void need_host_status(size_t n) {
		if (n <= h_status_n) return;
		if (h_status) HIPCHK(hipHostFree(h_status));
		h_status = nullptr;
		HIPCHK(hipHostMalloc(&h_status, n * sizeof(int)));
		h_status_n = n;
		void *dv = nullptr;
		HIPCHK(hipHostGetDevicePointer(&dv, h_status, 0));
		d_status_map = static_cast<int *>(dv);
	}
};

// A sharded search enqueued on every shard (shards.cpp shard_submit): the
// shards' tickets, merged at shard_finish_oldest into the caller's outputs.
struct ShardPending {
	int64_t ticket = 0;
	int slot = 0, nq = 0, k = 0, odev = -1;  // odev: device of the outputs (-1: host / unknown)
	bool out_host = false;
	std::vector<int64_t> st;
	std::vector<char> empty;
	int64_t *L = nullptr;
	float *D = nullptr;
	int *C = nullptr;
};

// An enqueued pass whose completion check (certificates, reruns, fallback)
// is still to run (Index::finish_chunk).
struct PendingPass {
	int slot = 0, nq = 0, k = 0;
	int64_t *dL = nullptr;
	float *dD = nullptr;
	int *dC = nullptr;
	StoreView sv{};
	QueryView qv{};
	bool hmap = false, fast_ok = false, dense = false, two_append = false, async = false;
	int64_t n_tiles = 0, ticket = 0, st3 = 0, st5 = 0;
	// an asynchronous IVF search (ivf_search enqueued without its end wait): the
	// pinned slot of its fused coarse flags, and what a rerun on the flat coarse
	// path needs (ivf_finish)
	bool ivf = false, ivf_fused = false;
	int ivf_flag_slot = 0, nprobes = 0, refine = 0;
	const float *dQ = nullptr;
};

struct Workspace {
	DevBuf<float> Qin, cut, dense, cand_dist, out_d, fb_keys, fb_keys2, stage;
	DevBuf<int> out_c;
	DevBuf<int> selbig;         // per query: pool too large for the small select
	// small exact search (search_chunk): per-workgroup partial top-k lists and
	// the per-query completion counters (zeroed at allocation, left zeroed)
	DevBuf<uint4> spart;
	DevBuf<unsigned> scnt;
	// second threshold pass of uncertified queries (search_chunk)
	DevBuf<float> rQf, rtau, rD;
	DevBuf<uint16_t> rQb;
	DevBuf<float4> rqaux;
	DevBuf<int> rfq, rstat, rC;
	DevBuf<int64_t> rL;
	DevBuf<uint32_t> cand_slot;
	DevBuf<int64_t> out_l, fb_vals, fb_vals2, idx;
	DevBuf<uint8_t> sort_tmp, out_blk;
	uint8_t *h_io = nullptr;    // pinned staging of the host-buffer API (queries in, results out)
	size_t h_io_n = 0;
	~Workspace() {
		if (h_io) (void)hipHostFree(h_io);
	}
	uint8_t *need_host_io(size_t bytes) {
		if (bytes > h_io_n) {
			if (h_io) HIPCHK(hipHostFree(h_io));
			h_io = nullptr;
			HIPCHK(hipHostMalloc(&h_io, bytes));
			h_io_n = bytes;
		}
		return h_io;
	}
};

// ---------------------------------------------------------------------------
// the handle
// ---------------------------------------------------------------------------
struct Index {
	std::string db_path, table, metric_name;
	int metric = METRIC_L2;
	int dim = 0;
	int ld = 0;  // padded row stride
	int device = 0;
	bool metric_quirk = false;  // rank by L2 whatever the metric (reference behaviour)

	std::mutex mu;
	int64_t next_label = 0;

	// host bookkeeping (slot order == ascending label order, always)
	std::vector<int64_t> slot_label;
	std::vector<uint8_t> live;
	int64_t n_live = 0;

	// device store: rows of `ld` elements, f32, or bf16 bits with storage "bf16"
	void *X = nullptr;
	bool xbf16 = false;
	size_t xes() const { return xbf16 ? 2 : 4; }
	uint8_t *xrow(int64_t s) const { return static_cast<uint8_t *>(X) + (size_t)s * ld * xes(); }
	// bf16 scan copy of an f32 store (option scan_copy, default on): built on the
	// first search that streams bf16 rows (ensure_xs: the flat scans when the int8
	// copy does not apply, the IVF_FLAT bound scan), never when the int8 copy
	// serves every search (10M x 768: 15 GB not held); then the scan
	// streams 2 B per element; refine, get_vector and compact use the f32 rows
	uint16_t *Xs = nullptr;
	bool scan_copy = true;
	bool has_scan_copy() const { return !xbf16 && scan_copy; }
	float4 *rowaux = nullptr;  // aux for `metric`
	// int8 scan copy (option scan_i8): derived from X on demand (ensure_i8) and
	// rebuilt after any change of the rows or tombstones (mut_ver); the flat
	// scans stream it with rowaux8 as their row terms, everything else uses X
	bool scan_i8 = true;
	int last_scan_esz = 0;  // bytes per element the last flat search's scan streamed (1 int8, 2 bf16, 4 f32)
	int8_t *Xq = nullptr;
	float4 *rowaux8 = nullptr;
	float4 *tstat8 = nullptr;  // per row tile: (s_T, max |e_x|, max |x~|, 0) of the int8 copy
	int64_t q8_cap = 0;
	uint64_t mut_ver = 1, q8_ver = 0;
	DevBuf<unsigned> stats8;
	float max_alpha8 = 0.f, max_x8 = 0.f;
	// refined candidates with the int8 scan: k + max(cand_extra_i8, k) (looser bounds put more rows below the
	// k-th distance: 1M x 768 up to ~80, 10M x 768 up to ~110); 0 = auto: 96 up to 4M slots, 192 past that
	int cand_extra_i8 = 0;
	int cand_extra_i8_eff() const { return cand_extra_i8 ? cand_extra_i8 : (n_slots > (4 << 20) ? 192 : 96); }
	float4 *rowaux_l2 = nullptr;  // aux for L2 when metric_quirk is on and metric != l2
	int64_t *dlabels = nullptr;
	int64_t cap = 0, n_slots = 0;
	DevBuf<unsigned> stats;  // [0]=max alpha bits, [1]=max ux bits, [2],[3] for rowaux_l2
	float max_alpha = 0.f, max_ux = 0.f, max_alpha_l2 = 0.f, max_ux_l2 = 0.f;
	hipStream_t stream = nullptr;
	// asynchronous passes run on their pass-buffer set's own stream (ordered after
	// the handle's stream by ev_order): pass i+1's first kernels overlap pass i's last
	hipStream_t pstream[2] = {nullptr, nullptr};
	hipEvent_t ev_order = nullptr;
	hipEvent_t ev_caller = nullptr;  // (lance_hip_stream_after: the caller's stream, recorded)
	hipStream_t pass_stream(int slot) {
		if (!pstream[slot]) HIPCHK(hipStreamCreateWithFlags(&pstream[slot], hipStreamNonBlocking));
		if (!ev_order) HIPCHK(hipEventCreateWithFlags(&ev_order, hipEventDisableTiming));
		return pstream[slot];
	}
	Workspace ws;
	PassBufs pb[2];
	std::deque<PendingPass> pending;  // asynchronous passes not finished yet (<= 2)
	int64_t next_ticket = 1;

	// persistence
	FILE *log = nullptr;

	// IVF index (lance_detached_create_index, ivf_index.cpp); null = flat search.
	// Options: index_type (IVF_PQ as lance_manager.rs:483-515 builds, or
	// IVF_FLAT), k-means iterations and sampling seed.
	IvfState *ivf = nullptr;

	// metadata columns of a multi-column table (lance_create_detached_from_arrow;
	// null for vector-only tables) and the filtered-search state: a search with
	// a predicate runs with `faux` = the row aux with alpha = +inf on every slot
	// the predicate does not select (the scan, refine, fallback and IVF list
	// scans already skip such rows as tombstones) and filter_live in place of
	// n_live
	std::unique_ptr<MetaStore> meta;
	bool filter_on = false;
	int64_t filter_live = 0;
	DevBuf<uint8_t> fmask;
	DevBuf<float4> faux;
	int64_t live_rows() const { return filter_on ? filter_live : n_live; }
	// the row aux a search reads: `base`, or its filtered copy
	const float4 *search_aux(const float4 *base) {
		if (!filter_on) return base;
		faux.need((size_t)cap);
		launch_filter_rowaux(base, fmask.p, n_slots, cap, faux.p, stream);
		return faux.p;
	}
	int ivf_type_opt = 1;  // 0 IVF_FLAT, 1 IVF_PQ
	int kmeans_iters = 50;  // lance k-means max_iters default
	uint64_t ivf_seed = 0x5eedULL;
	bool pq_fast = true;    // IVF_PQ list-major 8-bit-LUT scan (option "pq_scan" = "fast"; "exact_lut": f32 LUT, query-major)
	bool pq_seed = true;    // fast scan: per-query bound seeded from the nearest probed list (option "pq_seed")
	bool pq_lut_fused = true;    // fast scan: fp8 + ADC table + 8-bit LUT in one launch (option "pq_lut" = fused | split)
	bool pq_merge_bound = true;  // fast scan: the run merge skips keys above the scan's final bound (option "pq_merge_bound")
	bool ivf_coarse_fused = true;      // IVF coarse search by coarse_kernels.hip (option "ivf_coarse" = fused | flat)
	int64_t ivf_coarse_fallbacks = 0;  // passes the fused coarse search sent to the flat path
	bool pq_fp8 = false;         // IVF_PQ ADC tables from e4m3 (fp8) queries (option "pq_query" = "fp8" | "f32")
	bool ivf_flat_bound = true;  // IVF_FLAT list scan by MFMA bf16 lower bounds + certified exact re-rank (option "ivf_flat_scan" = "bound" | "exact")
	int64_t ivf_flat_fallbacks = 0;  // batches the bound scan could not certify (rerun exactly)

	int64_t last_stats[6] = {0, 0, 0, 0, 0, 0};

	// multi-device handle (env LANCE_HIP_DEVICES or option "devices", shards.cpp):
	// the rows live in `shards`, one Index per device holding whole ingest batches
	// under their global labels; this handle keeps next_label, the live count and
	// the table log, and merges the shards' top-k lists on the first device
	std::vector<std::unique_ptr<Index>> shards;
	bool sharded() const { return !shards.empty(); }
	// per in-flight search slot (two sharded searches may be in flight): the
	// shards' partial lists on the first device, the merged lists when the
	// caller's outputs live elsewhere (host, another device)
	DevBuf<int64_t> m_pl[2];
	DevBuf<float> m_pd[2];
	DevBuf<int> m_pc[2];
	DevBuf<uint8_t> m_out[2];
	std::deque<ShardPending> spending;  // sharded searches enqueued, not merged yet (<= 2)
	// as a shard: its queries / partial lists per parent slot, and the event its
	// peer copies of a slot's lists end at (the merge stream waits on it)
	DevBuf<float> sh_q[2];
	DevBuf<uint8_t> sh_out[2];
	hipEvent_t sh_ev[2] = {nullptr, nullptr};
	// option calls made before the handle became multi-device, replayed on each
	// shard by shard_init (so `devices` may come after other options)
	std::vector<std::pair<std::string, std::string>> opt_log;

	// optional HIP-event timing of the scan kernels, on the stream they run on
	bool time_kernels = false;
	// sample pass covers ~1/sample_div of the tiles (>= 32 tiles); 0 = auto: 16 up to
	// 8192 tiles (2M rows: a tighter tau, fewer appended bounds; C2 790k vs 762k q/s,
	// r04h), 32 past that (10M rows: the larger sample costs more than it saves, r03x)
	int sample_div = 0;
	int sample_div_eff(int64_t n_tiles) const { return sample_div > 0 ? sample_div : (n_tiles <= 8192 ? 16 : 32); }
	bool small_exact = true;  // one-launch exact search for <= 8 queries over <= 32768 slots
	bool defer_sync = false;  // caller synchronizes the stream itself (host-buffer search)
	bool retry_pass = true;  // rerun uncertified queries with a tighter tau before the exact fallback
	int cand_extra = 32;  // refined candidates: max(k * refine_factor, k + max(cand_extra, k))
	hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
	// progressive threshold (int8 append pass): the first 1/split_div of the tiles
	// with the sample's tau, then the rest with the tau their pool gives (0: one pass)
	int split_div = 0;
	int pr_first = 0;    // option "pr_first": pool_refine's first final-mode chunk (0 = the kernel's default)
	int s8_variant = 0;  // option "scan8_variant": scan8 geometry (release builds: 0 only)
	int tie_desc = 1;    // option "tie" / LANCE_HIP_TIE: 1 = (distance, label desc), 0 = (distance, label asc)
	int s8_couple = 0;   // option "s8_couple": scan8 pair coupling lag in 32-row units (0 = off; speed only)
	double kt_append_ms = 0.0, kt_dense_ms = 0.0;
	int64_t kt_append_n = 0, kt_dense_n = 0;
	int64_t kt_append_rows = 0, kt_append_qpad = 0;
	int kt_append_kernel = 0;  // 2: the last timed append pass ran scan8_kernel, 0: scan_kernel
	// IVF list scans (ivf_search): launches, ms, and their algorithmic work:
	// bytes = rows of every probed list once (row data or codes) + per-pair
	// tables; pair_rows = sum over (query, list) pairs of the list's rows
	double kt_ivf_ms = 0.0, kt_ivf_bytes = 0.0, kt_ivf_pair_rows = 0.0, kt_ivf_coarse_ms = 0.0;
	int64_t kt_ivf_n = 0;

	~Index() {
		if (stream) (void)hipStreamSynchronize(stream);  // (pending passes: their kernels end first)
		for (auto &ps : pstream)
			if (ps) (void)hipStreamSynchronize(ps);
		if (log) fclose(log);
		ivf_free(ivf);
		(void)hipSetDevice(device);
		if (X) (void)hipFree(X);
		if (Xs) (void)hipFree(Xs);
		if (Xq) (void)hipFree(Xq);
		if (rowaux8) (void)hipFree(rowaux8);
		if (tstat8) (void)hipFree(tstat8);
		if (rowaux) (void)hipFree(rowaux);
		if (rowaux_l2) (void)hipFree(rowaux_l2);
		if (dlabels) (void)hipFree(dlabels);
		for (auto &e : ev)
			if (e) (void)hipEventDestroy(e);
		for (auto &e : sh_ev)
			if (e) (void)hipEventDestroy(e);
		if (stream) (void)hipStreamDestroy(stream);
		for (auto &ps : pstream)
			if (ps) (void)hipStreamDestroy(ps);
		if (ev_order) (void)hipEventDestroy(ev_order);
		if (ev_caller) (void)hipEventDestroy(ev_caller);
	}

	void tic(int i) {
		if (time_kernels) HIPCHK(hipEventRecord(ev[i], stream));
	}
	float toc_ms(int a, int b) {
		float ms = 0.f;
		HIPCHK(hipEventSynchronize(ev[b]));
		HIPCHK(hipEventElapsedTime(&ms, ev[a], ev[b]));
		return ms;
	}

	void init_device(int dev) {
		int n = 0;
		if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw Error("no HIP device available");
		if (dev < 0) HIPCHK(hipGetDevice(&dev));
		if (dev >= n) throw Error("HIP device " + std::to_string(dev) + " out of range");
		device = dev;
		HIPCHK(hipSetDevice(device));
		HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
		stats.need(4);
		HIPCHK(hipMemsetAsync(stats.p, 0, 4 * sizeof(unsigned), stream));
		HIPCHK(hipStreamSynchronize(stream));
	}

	// every entry point that touches the device: the handle's device current,
	// and no asynchronous search pending (finished first: a mutation or another
	// search never runs under one)
	void bind() {
		HIPCHK(hipSetDevice(device));
		drain();
	}
	void bind_nodrain() { HIPCHK(hipSetDevice(device)); }

	// grow the device store to hold at least `want` slots (contents preserved)
	void reserve(int64_t want) {
		if (want <= cap) return;
		++mut_ver;
		// capacity is a multiple of the scan tile and the tail past n_slots is
		// zero: the scan kernel streams whole tiles without clamping rows
		int64_t c = round_up(std::max<int64_t>(want, std::max<int64_t>(4096, cap * 2)), SCAN_BR);
		void *nX = nullptr;
		uint16_t *nXs = nullptr;
		float4 *na = nullptr, *na2 = nullptr;
		int64_t *nl = nullptr;
		HIPCHK(hipMalloc(&nX, (size_t)c * ld * xes()));
		if (Xs) HIPCHK(hipMalloc(&nXs, (size_t)c * ld * 2));
		HIPCHK(hipMalloc(&na, (size_t)c * sizeof(float4)));
		HIPCHK(hipMalloc(&nl, (size_t)c * sizeof(int64_t)));
		if (rowaux_l2 || (metric_quirk && metric != METRIC_L2)) HIPCHK(hipMalloc(&na2, (size_t)c * sizeof(float4)));
		if (n_slots > 0) {
			HIPCHK(hipMemcpyAsync(nX, X, (size_t)n_slots * ld * xes(), hipMemcpyDeviceToDevice, stream));
			if (nXs) HIPCHK(hipMemcpyAsync(nXs, Xs, (size_t)n_slots * ld * 2, hipMemcpyDeviceToDevice, stream));
			// row aux is tile-blocked SoA: move whole tile blocks (cap is a
			// multiple of SCAN_BR, so they exist in the old buffer)
			const size_t aux_bytes = (size_t)round_up(n_slots, SCAN_BR) * sizeof(float4);
			HIPCHK(hipMemcpyAsync(na, rowaux, aux_bytes, hipMemcpyDeviceToDevice, stream));
			HIPCHK(hipMemcpyAsync(nl, dlabels, (size_t)n_slots * sizeof(int64_t), hipMemcpyDeviceToDevice, stream));
			if (na2 && rowaux_l2) HIPCHK(hipMemcpyAsync(na2, rowaux_l2, aux_bytes, hipMemcpyDeviceToDevice, stream));
		}
		HIPCHK(hipMemsetAsync(static_cast<uint8_t *>(nX) + (size_t)n_slots * ld * xes(), 0,
		                      (size_t)(c - n_slots) * ld * xes(), stream));
		if (nXs) HIPCHK(hipMemsetAsync(nXs + (size_t)n_slots * ld, 0, (size_t)(c - n_slots) * ld * 2, stream));
		launch_fill_rowaux(na, n_slots, c, stream);
		if (na2) launch_fill_rowaux(na2, n_slots, c, stream);
		HIPCHK(hipStreamSynchronize(stream));
		if (X) HIPCHK(hipFree(X));
		if (Xs) HIPCHK(hipFree(Xs));
		Xs = nXs;
		if (rowaux) HIPCHK(hipFree(rowaux));
		if (dlabels) HIPCHK(hipFree(dlabels));
		if (rowaux_l2) HIPCHK(hipFree(rowaux_l2));
		X = nX;
		rowaux = na;
		dlabels = nl;
		rowaux_l2 = na2;
		cap = c;
	}

	void refresh_stats() {
		unsigned h[4];
		HIPCHK(hipMemcpyAsync(h, stats.p, sizeof(h), hipMemcpyDeviceToHost, stream));
		HIPCHK(hipStreamSynchronize(stream));
		memcpy(&max_alpha, &h[0], 4);
		memcpy(&max_ux, &h[1], 4);
		memcpy(&max_alpha_l2, &h[2], 4);
		memcpy(&max_ux_l2, &h[3], 4);
	}

	// scan copy rows [s0, s0+n) = bf16 (RNE) of the f32 rows of X (padding
	// columns stay zero)
	void fill_scan_copy(int64_t s0, int64_t n, uint16_t *dst) {
		if (n > 0)
			launch_rows_to_bf16(reinterpret_cast<const float *>(xrow(s0)), ld, n, dim, ld, dst + (size_t)s0 * ld,
			                    stream);
	}

	// option scan_copy: build or drop the bf16 scan copy of an f32 store
	void set_scan_copy(bool on) {
		if (on == scan_copy) return;
		scan_copy = on;
		if (!on) {
			if (Xs) HIPCHK(hipFree(Xs));
			Xs = nullptr;
		}
	}
	// the bf16 scan copy, built now if the store keeps one and it is not there yet
	void ensure_xs() {
		if (!has_scan_copy() || Xs || !X || cap == 0) return;
		HIPCHK(hipMalloc(&Xs, (size_t)cap * ld * 2));
		HIPCHK(hipMemsetAsync(Xs, 0, (size_t)cap * ld * 2, stream));
		fill_scan_copy(0, n_slots, Xs);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(stream));
	}

	// the int8 scan applies: an f32 or bf16 store whose rows fit the int8 stages
	// (ld a multiple of 128, exact integer dot products up to ld = 1024), no
	// filter, ranking by the index metric
	bool i8_usable() const {
		return scan_i8 && X && n_slots > 0 && ld % 128 == 0 && ld <= 1024 && !filter_on &&
		       !(metric_quirk && metric != METRIC_L2);
	}
	// whether a flat search of nq queries for k streams the int8 copy: any k on
	// the threshold path (pool_refine refines as far as its certificate needs),
	// k <= 32 on the dense path of small stores (a fixed candidate count)
	bool scan_uses_i8(int nq, int k) const {
		(void)nq;
		return i8_usable() && (k <= 32 || (n_slots > 65536 && k + 8 <= MAX_CAND));
	}
	// (re)build the int8 scan copy and its row terms from X when stale
	void ensure_i8() {
		if (Xq && q8_ver == mut_ver && q8_cap == cap) return;
		if (!Xq || q8_cap != cap) {
			drop_i8();
			HIPCHK(hipMalloc(&Xq, (size_t)cap * ld));
			HIPCHK(hipMalloc(&rowaux8, (size_t)cap * sizeof(float4)));
			HIPCHK(hipMalloc(&tstat8, (size_t)(cap / SCAN_BR) * sizeof(float4)));
			q8_cap = cap;
		}
		stats8.need(2);
		HIPCHK(hipMemsetAsync(stats8.p, 0, 2 * sizeof(unsigned), stream));
		// whole tiles up to the last row; past them: zero rows, +inf row terms
		const int64_t t1 = (n_slots + SCAN_BR - 1) / SCAN_BR, r1 = t1 * SCAN_BR;
		HIPCHK(hipMemsetAsync(Xq + (size_t)r1 * ld, 0, (size_t)(cap - r1) * ld, stream));
		launch_tiles_to_i8(X, xbf16 ? 1 : 0, ld, dim, metric, n_slots, 0, t1, rowaux, Xq, rowaux8, tstat8,
		                   stats8.p, stream);
		launch_fill_rowaux(rowaux8, r1, cap, stream);
		HIPCHK(hipGetLastError());
		unsigned h[2];
		HIPCHK(hipMemcpyAsync(h, stats8.p, sizeof(h), hipMemcpyDeviceToHost, stream));
		HIPCHK(hipStreamSynchronize(stream));
		memcpy(&max_alpha8, &h[0], 4);
		memcpy(&max_x8, &h[1], 4);
		q8_ver = mut_ver;
	}
	void drop_i8() {
		if (Xq) HIPCHK(hipFree(Xq));
		if (rowaux8) HIPCHK(hipFree(rowaux8));
		if (tstat8) HIPCHK(hipFree(tstat8));
		Xq = nullptr;
		rowaux8 = nullptr;
		tstat8 = nullptr;
		q8_cap = 0;
	}

	// append rows already resident on the device at X[n_slots .. n_slots+num)
	int64_t commit_rows(int64_t num) {
		// a current int8 scan copy (same capacity) takes the new rows in place
		const bool i8_cur = Xq && q8_ver == mut_ver && q8_cap == cap;
		++mut_ver;
		const int64_t first = next_label;
		std::vector<int64_t> labs((size_t)num);
		for (int64_t i = 0; i < num; ++i) labs[(size_t)i] = first + i;
		HIPCHK(hipMemcpyAsync(dlabels + n_slots, labs.data(), (size_t)num * sizeof(int64_t), hipMemcpyHostToDevice,
		                      stream));
		if (Xs) fill_scan_copy(n_slots, num, Xs);
		launch_rowaux(X, xbf16, ld, dim, metric, n_slots, num, rowaux, stats.p, stream);
		if (rowaux_l2) launch_rowaux(X, xbf16, ld, dim, METRIC_L2, n_slots, num, rowaux_l2, stats.p + 2, stream);
		// (the tile the new rows start in is re-quantised whole: its scale may grow)
		if (i8_cur)
			launch_tiles_to_i8(X, xbf16 ? 1 : 0, ld, dim, metric, n_slots + num, n_slots / SCAN_BR,
			                   (n_slots + num + SCAN_BR - 1) / SCAN_BR, rowaux, Xq, rowaux8, tstat8, stats8.p, stream);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(stream));
		refresh_stats();
		if (i8_cur) {
			unsigned h8[2];
			HIPCHK(hipMemcpy(h8, stats8.p, sizeof(h8), hipMemcpyDeviceToHost));
			memcpy(&max_alpha8, &h8[0], 4);
			memcpy(&max_x8, &h8[1], 4);
			q8_ver = mut_ver;
		}
		slot_label.insert(slot_label.end(), labs.begin(), labs.end());
		live.insert(live.end(), (size_t)num, 1);
		if (meta && meta->cols.size() && meta->cols[0].size() < (size_t)(n_slots + num))
			meta->append_nulls(n_slots + num - (int64_t)meta->cols[0].size());
		n_slots += num;
		n_live += num;
		next_label = first + num;
		return first;
	}

	int64_t add_host(const float *v, int64_t num) {
		reserve(n_slots + num);
		if (!xbf16) {
			float *dst = reinterpret_cast<float *>(xrow(n_slots));
			if (ld != dim) HIPCHK(hipMemsetAsync(dst, 0, (size_t)num * ld * sizeof(float), stream));
			HIPCHK(hipMemcpy2DAsync(dst, (size_t)ld * sizeof(float), v, (size_t)dim * sizeof(float),
			                        (size_t)dim * sizeof(float), (size_t)num, hipMemcpyHostToDevice, stream));
		} else {
			// bf16 store: f32 rows through a bounded device staging buffer
			const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(num, (int64_t)(64 << 20) / (dim * 4)));
			ws.stage.need((size_t)chunk * dim);
			for (int64_t i = 0; i < num; i += chunk) {
				const int64_t m = std::min<int64_t>(chunk, num - i);
				HIPCHK(hipMemcpyAsync(ws.stage.p, v + i * dim, (size_t)m * dim * sizeof(float), hipMemcpyHostToDevice,
				                      stream));
				launch_rows_to_bf16(ws.stage.p, dim, m, dim, ld, reinterpret_cast<uint16_t *>(xrow(n_slots + i)),
				                    stream);
				HIPCHK(hipStreamSynchronize(stream));  // staging buffer reused
			}
		}
		return commit_rows(num);
	}

	int64_t add_device(const float *v, int64_t num) {
		reserve(n_slots + num);
		if (!xbf16) {
			float *dst = reinterpret_cast<float *>(xrow(n_slots));
			if (ld != dim) HIPCHK(hipMemsetAsync(dst, 0, (size_t)num * ld * sizeof(float), stream));
			HIPCHK(hipMemcpy2DAsync(dst, (size_t)ld * sizeof(float), v, (size_t)dim * sizeof(float),
			                        (size_t)dim * sizeof(float), (size_t)num, hipMemcpyDeviceToDevice, stream));
		} else {
			launch_rows_to_bf16(v, dim, num, dim, ld, reinterpret_cast<uint16_t *>(xrow(n_slots)), stream);
		}
		return commit_rows(num);
	}

	// rows [s0, s0+n) as f32 (dim columns) into host memory
	void read_rows(int64_t s0, int64_t n, float *out) {
		if (n <= 0) return;
		if (!xbf16) {
			HIPCHK(hipMemcpy2D(out, (size_t)dim * sizeof(float), xrow(s0), (size_t)ld * sizeof(float),
			                   (size_t)dim * sizeof(float), (size_t)n, hipMemcpyDeviceToHost));
			return;
		}
		std::vector<uint16_t> b((size_t)n * dim);
		HIPCHK(hipMemcpy2D(b.data(), (size_t)dim * 2, xrow(s0), (size_t)ld * 2, (size_t)dim * 2, (size_t)n,
		                   hipMemcpyDeviceToHost));
		for (size_t i = 0; i < b.size(); ++i) {
			const uint32_t u = (uint32_t)b[i] << 16;
			memcpy(out + i, &u, 4);
		}
	}

	// storage "f32" | "bf16"; only while the store holds no rows
	void set_storage(bool bf16) {
		if (n_slots > 0) throw Error("storage can only be changed on an empty table");
		if (bf16 == xbf16) return;
		++mut_ver;
		if (X) {
			HIPCHK(hipFree(X));
			if (Xs) HIPCHK(hipFree(Xs));
			Xs = nullptr;
			HIPCHK(hipFree(rowaux));
			HIPCHK(hipFree(dlabels));
			if (rowaux_l2) HIPCHK(hipFree(rowaux_l2));
			X = nullptr;
			rowaux = rowaux_l2 = nullptr;
			dlabels = nullptr;
			cap = 0;
		}
		xbf16 = bf16;
	}

	int64_t slot_of(int64_t label) const {
		auto it = std::lower_bound(slot_label.begin(), slot_label.end(), label);
		if (it == slot_label.end() || *it != label) return -1;
		return (int64_t)(it - slot_label.begin());
	}

	// returns the labels actually deleted (live before the call)
	std::vector<int64_t> remove(const int64_t *labels, int64_t n) {
		std::vector<int64_t> slots, done;
		for (int64_t i = 0; i < n; ++i) {
			int64_t s = slot_of(labels[i]);
			if (s < 0 || !live[(size_t)s]) continue;
			live[(size_t)s] = 0;
			--n_live;
			slots.push_back(s);
			done.push_back(labels[i]);
		}
		if (!slots.empty()) {
			// a current int8 scan copy takes the tombstones in place (no rebuild)
			const bool i8_cur = Xq && q8_ver == mut_ver && q8_cap == cap;
			++mut_ver;
			ws.idx.need(slots.size());
			HIPCHK(hipMemcpyAsync(ws.idx.p, slots.data(), slots.size() * sizeof(int64_t), hipMemcpyHostToDevice,
			                      stream));
			launch_tombstone(rowaux, ws.idx.p, (int)slots.size(), stream);
			if (i8_cur) {
				launch_tombstone(rowaux8, ws.idx.p, (int)slots.size(), stream);
				q8_ver = mut_ver;
			}
			if (rowaux_l2) launch_tombstone(rowaux_l2, ws.idx.p, (int)slots.size(), stream);
			HIPCHK(hipGetLastError());
			HIPCHK(hipStreamSynchronize(stream));
		}
		return done;
	}

	void compact() {
		if (n_live == n_slots) return;
		++mut_ver;
		std::vector<int64_t> keep;
		keep.reserve((size_t)n_live);
		for (int64_t s = 0; s < n_slots; ++s)
			if (live[(size_t)s]) keep.push_back(s);
		const int64_t n = (int64_t)keep.size();
		if (ivf) ivf_remap(this, keep);
		if (meta) meta->keep_slots(keep);
		const int64_t c = round_up(std::max<int64_t>(4096, n), SCAN_BR);
		void *nX = nullptr;
		float4 *na = nullptr, *na2 = nullptr;
		int64_t *nl = nullptr;
		HIPCHK(hipMalloc(&nX, (size_t)c * ld * xes()));
		HIPCHK(hipMalloc(&na, (size_t)c * sizeof(float4)));
		HIPCHK(hipMalloc(&nl, (size_t)c * sizeof(int64_t)));
		if (rowaux_l2) HIPCHK(hipMalloc(&na2, (size_t)c * sizeof(float4)));
		if (n > 0) {
			ws.idx.need((size_t)n);
			HIPCHK(hipMemcpyAsync(ws.idx.p, keep.data(), (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, stream));
			launch_gather_rows(X, xbf16, rowaux, dlabels, ws.idx.p, n, ld, nX, na, nl, stream);
			if (rowaux_l2) launch_gather_rows(X, xbf16, rowaux_l2, dlabels, ws.idx.p, n, ld, nX, na2, nl, stream);
			HIPCHK(hipGetLastError());
		}
		HIPCHK(hipMemsetAsync(static_cast<uint8_t *>(nX) + (size_t)n * ld * xes(), 0, (size_t)(c - n) * ld * xes(),
		                      stream));
		launch_fill_rowaux(na, n, c, stream);
		if (na2) launch_fill_rowaux(na2, n, c, stream);
		uint16_t *nXs = nullptr;
		if (Xs) {
			HIPCHK(hipMalloc(&nXs, (size_t)c * ld * 2));
			HIPCHK(hipMemsetAsync(nXs, 0, (size_t)c * ld * 2, stream));
			if (n > 0)
				launch_rows_to_bf16(static_cast<const float *>(nX), ld, n, dim, ld, nXs, stream);
			HIPCHK(hipGetLastError());
		}
		HIPCHK(hipStreamSynchronize(stream));
		if (Xs) HIPCHK(hipFree(Xs));
		Xs = nXs;
		HIPCHK(hipFree(X));
		HIPCHK(hipFree(rowaux));
		HIPCHK(hipFree(dlabels));
		if (rowaux_l2) HIPCHK(hipFree(rowaux_l2));
		X = nX;
		rowaux = na;
		dlabels = nl;
		rowaux_l2 = na2;
		cap = c;
		std::vector<int64_t> nsl;
		nsl.reserve((size_t)n);
		for (int64_t s : keep) nsl.push_back(slot_label[(size_t)s]);
		slot_label.swap(nsl);
		live.assign((size_t)n, 1);
		n_slots = n;
		n_live = n;
	}

	// ---- persistence: append-only log <db_path>/<table>.lancehip ----------
	std::string log_path() const { return db_path + "/" + table + ".lancehip"; }

	void log_open(bool truncate) {
		if (db_path.empty()) return;
		// mkdir -p db_path
		std::string acc;
		for (size_t i = 0; i <= db_path.size(); ++i) {
			if (i == db_path.size() || db_path[i] == '/') {
				if (!acc.empty() && acc != "/") (void)mkdir(acc.c_str(), 0755);
			}
			if (i < db_path.size()) acc.push_back(db_path[i]);
		}
		log = fopen(log_path().c_str(), truncate ? "wb" : "ab");
		if (!log) throw Error("cannot open " + log_path() + ": " + strerror(errno));
		if (truncate) {
			fwrite("LHIPLOG1", 1, 8, log);
			int32_t d = dim;
			fwrite(&d, 4, 1, log);
			fflush(log);
		}
	}
	void log_add(int64_t first, const float *v, int64_t num) {
		if (!log) return;
		uint8_t tag = 1;
		fwrite(&tag, 1, 1, log);
		fwrite(&first, 8, 1, log);
		fwrite(&num, 8, 1, log);
		fwrite(v, sizeof(float), (size_t)num * dim, log);
		fflush(log);
	}
	// multi-column tables: schema record (tag 6, right after the header) and
	// the metadata rows of each ingest batch (tag 7, after its tag-1 record)
	void log_meta_schema() {
		if (!log || !meta) return;
		std::vector<uint8_t> b;
		meta->serialize_schema(b);
		uint8_t tag = 6;
		int64_t n = (int64_t)b.size();
		fwrite(&tag, 1, 1, log);
		fwrite(&n, 8, 1, log);
		fwrite(b.data(), 1, b.size(), log);
		fflush(log);
	}
	void log_meta_rows(int64_t s0, int64_t num, const MetaStore *from = nullptr) {
		if (!from) from = meta.get();
		if (!log || !from) return;
		std::vector<uint8_t> b;
		from->serialize_rows(s0, num, b);
		uint8_t tag = 7;
		int64_t n = (int64_t)b.size();
		fwrite(&tag, 1, 1, log);
		fwrite(&n, 8, 1, log);
		fwrite(b.data(), 1, b.size(), log);
		fflush(log);
	}
	void log_scalar_index(const std::string &col, const std::string &ty) {
		if (!log) return;
		uint8_t tag = 8;
		uint32_t a = (uint32_t)col.size(), b = (uint32_t)ty.size();
		fwrite(&tag, 1, 1, log);
		fwrite(&a, 4, 1, log);
		fwrite(col.data(), 1, a, log);
		fwrite(&b, 4, 1, log);
		fwrite(ty.data(), 1, b, log);
		fflush(log);
	}
	void log_storage() {
		if (!log) return;
		uint8_t tag = 3, v = xbf16 ? 1 : 0;
		fwrite(&tag, 1, 1, log);
		fwrite(&v, 1, 1, log);
		fflush(log);
	}
	void log_del(const std::vector<int64_t> &labs) {
		if (!log || labs.empty()) return;
		uint8_t tag = 2;
		int64_t n = (int64_t)labs.size();
		fwrite(&tag, 1, 1, log);
		fwrite(&n, 8, 1, log);
		fwrite(labs.data(), 8, labs.size(), log);
		fflush(log);
	}

	// IVF model record (tag 4: type, nlist, m, centroids [nlist][dim], codebook)
	// of `src`'s model (default: this handle's) and optimize record (tag 5);
	// bodies in ivf_index.cpp
	void log_model(Index *src = nullptr);
	void log_optimize();

	// ---- search ------------------------------------------------------------
	// IVF search when an index exists, else the exact flat path
	void search_any(const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD, int *dC);
	// Device-side batched search; dQ [nq][dim] (device), outputs device.
	void search_device(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC);
	void search_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC);
	bool enqueue_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC, int slot,
	                   bool async, PendingPass &p);
	void finish_chunk(PendingPass &p);
	int pb_free_slot() const;
	// asynchronous search: enqueue (returns a ticket), complete at wait_ticket
	int64_t search_async(const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD, int *dC);
	void wait_ticket(int64_t ticket);  // <= 0: every pending search
	void finish_oldest();
	void drain();
};

// ---- multi-device handles (shards.cpp) ---------------------------------------
std::vector<int> parse_devices(const std::string &spec);
std::vector<int> env_devices();
// tie rule of the final order: "label_desc" (1, the default: the reference's
// golden at lance_optimizer_filter.test:36-44) or "label_asc" (0); the handle's
// default comes from LANCE_HIP_TIE, option "tie" sets it per handle
int parse_tie(const std::string &v);
int env_tie();
void shard_init(Index *ix, const std::vector<int> &devs);
Index *shard_for_add(Index *ix);
int64_t shard_live(const Index *ix);
int64_t shard_add(Index *ix, const float *v, int64_t num, int vdev, Index **into, Index *force = nullptr);
std::vector<int64_t> shard_remove(Index *ix, const int64_t *labels, int64_t n);
void shard_search(Index *ix, const float *Q, int qdev, int nq, int k, int nprobes, int refine, const char *pred,
                  int64_t *L, float *D, int *C, bool out_host);
// asynchronous sharded search (no predicate): every shard's pass enqueued, a
// ticket back; shard_finish_oldest completes the oldest (certificates on every
// shard, peer copies, the merge on the first device into the outputs on device
// odev, -1 = host)
int64_t shard_submit(Index *ix, const float *Q, int qdev, int nq, int k, int nprobes, int refine, int64_t *L,
                     float *D, int *C, bool out_host, int odev);
void shard_finish_oldest(Index *ix);
Index *shard_of_label(Index *ix, int64_t label, int64_t *slot);
void shard_all_rows(Index *ix, std::vector<int64_t> &labels, std::vector<float> &vecs);
void shard_compact(Index *ix);
void shard_create_index(Index *ix, int type, int num_partitions, int num_sub_vectors);
void shard_counts(Index *ix);

// A search with a predicate: evaluates it over the slots (host, vectorised),
// uploads the mask and turns filtering on for the scope of the search call.
struct FilterScope {
	Index *ix;
	FilterScope(Index *i, const char *predicate) : ix(i) {
		if (!predicate || !predicate[0]) return;
		std::vector<uint8_t> mask;
		ix->filter_live = eval_predicate(predicate, ix->meta.get(), ix->slot_label, ix->live, mask);
		ix->bind();
		ix->fmask.need(std::max<size_t>(mask.size(), 1));
		if (!mask.empty())
			HIPCHK(hipMemcpyAsync(ix->fmask.p, mask.data(), mask.size(), hipMemcpyHostToDevice, ix->stream));
		HIPCHK(hipStreamSynchronize(ix->stream));
		ix->filter_on = true;
	}
	~FilterScope() { ix->filter_on = false; }
};

}  // namespace lhip
