// C-ABI of the MI355X-native k-NN path: the symbols of
// /root/reference/rust_lib/src/ffi.rs, re-implemented over a device-resident
// vector store and the gfx950 kernels of knn_kernels.hip.
//
// Layering: the reference's C++ shim src/rust_ffi.cpp calls
// these extern "C" functions; in the reference they enter Rust (ffi.rs ->
// lance_manager.rs -> lancedb/lance).  Here they enter this file, which owns:
//   * the handle (ffi.rs:51 Box<LanceIndex>) = lhip::Index,
//   * the label bookkeeping of lance_manager.rs (dense labels from next_label,
//     :227-242; delete by label, :461-471; count, :474-478; reopen with
//     next_label = max(label)+1, :136-169/:662-696),
//   * a write-ahead log replacing the Lance dataset directory (persistence),
//   * the device store (f32 rows padded to a multiple of 64 floats + per-row
//     aux) and the search pipeline.
// Error convention of ffi.rs:15-24: NULL / -1 and a NUL-terminated message.
#include "../../include/lancedb_hip.h"
#include "knn_kernels.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/stat.h>
#include <vector>

namespace lhip {

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
static void spin_sync(hipStream_t st) {
	hipError_t e;
	while ((e = hipStreamQuery(st)) == hipErrorNotReady) {
	}
	if (e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e) + " at stream completion");
}

static void write_err(char *buf, int len, const std::string &msg) {
	if (!buf || len <= 0) return;
	size_t n = std::min(msg.size(), (size_t)(len - 1));
	memcpy(buf, msg.data(), n);
	buf[n] = 0;
}

static int metric_id(const std::string &m) {
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

struct Workspace {
	DevBuf<float> Qin, Qf, tau, cut, dense, cand_dist, out_d, fb_keys, fb_keys2, stage;
	DevBuf<uint16_t> Qb;
	DevBuf<float4> qaux;
	DevBuf<uint2> seg_pool;
	DevBuf<int> seg_cnt;
	DevBuf<int> status, out_c;  // status = [cert | cand_cnt | pool_cnt] x nq
	int *h_status = nullptr;    // pinned mirror of status
	size_t h_status_n = 0;
	DevBuf<uint32_t> cand_slot;
	DevBuf<int64_t> out_l, fb_vals, fb_vals2, idx;
	DevBuf<uint8_t> sort_tmp;
	~Workspace() {
		if (h_status) (void)hipHostFree(h_status);
	}
	void need_host_status(size_t n) {
		if (n <= h_status_n) return;
		if (h_status) HIPCHK(hipHostFree(h_status));
		h_status = nullptr;
		HIPCHK(hipHostMalloc(&h_status, n * sizeof(int)));
		h_status_n = n;
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
	// bf16 scan copy of an f32 store (option scan_copy, default on): the scan
	// streams 2 B per element; refine, get_vector and compact use the f32 rows
	uint16_t *Xs = nullptr;
	bool scan_copy = true;
	bool has_scan_copy() const { return !xbf16 && scan_copy; }
	float4 *rowaux = nullptr;  // aux for `metric`
	float4 *rowaux_l2 = nullptr;  // aux for L2 when metric_quirk is on and metric != l2
	int64_t *dlabels = nullptr;
	int64_t cap = 0, n_slots = 0;
	DevBuf<unsigned> stats;  // [0]=max alpha bits, [1]=max ux bits, [2],[3] for rowaux_l2
	float max_alpha = 0.f, max_ux = 0.f, max_alpha_l2 = 0.f, max_ux_l2 = 0.f;
	hipStream_t stream = nullptr;
	Workspace ws;

	// persistence
	FILE *log = nullptr;

	// ANN parameters recorded by create_index (flat search stays exact)
	int32_t ivf_partitions = 0, ivf_sub_vectors = 0;

	int64_t last_stats[4] = {0, 0, 0, 0};

	// optional HIP-event timing of the scan kernels, on the stream they run on
	bool time_kernels = false;
	int sample_div = 32;  // sample pass covers ~1/sample_div of the tiles (>= 32 tiles)
	hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
	double kt_append_ms = 0.0, kt_dense_ms = 0.0;
	int64_t kt_append_n = 0, kt_dense_n = 0;
	int64_t kt_append_rows = 0, kt_append_qpad = 0;

	~Index() {
		if (log) fclose(log);
		(void)hipSetDevice(device);
		if (X) (void)hipFree(X);
		if (Xs) (void)hipFree(Xs);
		if (rowaux) (void)hipFree(rowaux);
		if (rowaux_l2) (void)hipFree(rowaux_l2);
		if (dlabels) (void)hipFree(dlabels);
		for (auto &e : ev)
			if (e) (void)hipEventDestroy(e);
		if (stream) (void)hipStreamDestroy(stream);
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

	void bind() { HIPCHK(hipSetDevice(device)); }

	// grow the device store to hold at least `want` slots (contents preserved)
	void reserve(int64_t want) {
		if (want <= cap) return;
		// capacity is a multiple of the scan tile and the tail past n_slots is
		// zero: the scan kernel streams whole tiles without clamping rows
		int64_t c = round_up(std::max<int64_t>(want, std::max<int64_t>(4096, cap * 2)), SCAN_BR);
		void *nX = nullptr;
		uint16_t *nXs = nullptr;
		float4 *na = nullptr, *na2 = nullptr;
		int64_t *nl = nullptr;
		HIPCHK(hipMalloc(&nX, (size_t)c * ld * xes()));
		if (has_scan_copy()) HIPCHK(hipMalloc(&nXs, (size_t)c * ld * 2));
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
			return;
		}
		if (xbf16 || !X) return;  // allocated with the store
		HIPCHK(hipMalloc(&Xs, (size_t)cap * ld * 2));
		HIPCHK(hipMemsetAsync(Xs, 0, (size_t)cap * ld * 2, stream));
		fill_scan_copy(0, n_slots, Xs);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(stream));
	}

	// append rows already resident on the device at X[n_slots .. n_slots+num)
	int64_t commit_rows(int64_t num) {
		const int64_t first = next_label;
		std::vector<int64_t> labs((size_t)num);
		for (int64_t i = 0; i < num; ++i) labs[(size_t)i] = first + i;
		HIPCHK(hipMemcpyAsync(dlabels + n_slots, labs.data(), (size_t)num * sizeof(int64_t), hipMemcpyHostToDevice,
		                      stream));
		if (Xs) fill_scan_copy(n_slots, num, Xs);
		launch_rowaux(X, xbf16, ld, dim, metric, n_slots, num, rowaux, stats.p, stream);
		if (rowaux_l2) launch_rowaux(X, xbf16, ld, dim, METRIC_L2, n_slots, num, rowaux_l2, stats.p + 2, stream);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(stream));
		refresh_stats();
		slot_label.insert(slot_label.end(), labs.begin(), labs.end());
		live.insert(live.end(), (size_t)num, 1);
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
			ws.idx.need(slots.size());
			HIPCHK(hipMemcpyAsync(ws.idx.p, slots.data(), slots.size() * sizeof(int64_t), hipMemcpyHostToDevice,
			                      stream));
			launch_tombstone(rowaux, ws.idx.p, (int)slots.size(), stream);
			if (rowaux_l2) launch_tombstone(rowaux_l2, ws.idx.p, (int)slots.size(), stream);
			HIPCHK(hipGetLastError());
			HIPCHK(hipStreamSynchronize(stream));
		}
		return done;
	}

	void compact() {
		if (n_live == n_slots) return;
		std::vector<int64_t> keep;
		keep.reserve((size_t)n_live);
		for (int64_t s = 0; s < n_slots; ++s)
			if (live[(size_t)s]) keep.push_back(s);
		const int64_t n = (int64_t)keep.size();
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

	// ---- search ------------------------------------------------------------
	// Device-side batched search; dQ [nq][dim] (device), outputs device.
	void search_device(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC);
	void search_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC);
};

void Index::search_device(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC) {
	last_stats[0] = last_stats[1] = last_stats[2] = last_stats[3] = 0;
	// one pipeline pass covers up to MAX_PASS_Q queries (several query tiles
	// per scan launch): the per-pass fixed cost is paid once per pass
	for (int s = 0; s < nq; s += MAX_PASS_Q) {
		int c = std::min(MAX_PASS_Q, nq - s);
		search_chunk(dQ + (int64_t)s * dim, c, k, refine, dL + (int64_t)s * k, dD + (int64_t)s * k, dC + s);
	}
}

void Index::search_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC) {
	const int eff_metric = metric_quirk ? METRIC_L2 : metric;
	const float4 *aux = (metric_quirk && metric != METRIC_L2) ? rowaux_l2 : rowaux;
	const float ma = (metric_quirk && metric != METRIC_L2) ? max_alpha_l2 : max_alpha;
	const float mu = (metric_quirk && metric != METRIC_L2) ? max_ux_l2 : max_ux;
	StoreView sv{X, aux, dlabels, n_slots, ld, dim, eff_metric, xbf16 ? 1 : 0,
	             Xs ? static_cast<const void *>(Xs) : X, (xbf16 || Xs) ? 1 : 0};
	const int nq_pad = (int)round_up(nq, SCAN_BQ);
	ws.Qf.need((size_t)nq_pad * ld);
	ws.Qb.need((size_t)nq_pad * ld);
	ws.qaux.need(nq_pad);
	ws.tau.need(nq);
	ws.cut.need(nq);
	ws.cand_slot.need((size_t)nq * MAX_CAND);
	ws.cand_dist.need((size_t)nq * MAX_CAND);
	ws.status.need((size_t)3 * nq);
	ws.need_host_status((size_t)3 * nq);
	int *d_cert = ws.status.p, *d_cand_cnt = ws.status.p + nq, *d_pool_cnt = ws.status.p + 2 * nq;
	launch_prep_queries(dQ, nq, dim, ld, nq_pad, eff_metric, ma, mu, ws.Qf.p, ws.Qb.p, ws.qaux.p, ws.status.p, stream);
	QueryView qv{ws.Qf.p, ws.Qb.p, ws.qaux.p, nq, nq_pad};

	// refined candidates: k + max(32, k) — past k the bound slack (bf16 query
	// rounding) spans more ranks as the neighbour distances crowd (C3: k = 100)
	const int Mfinal = std::min(MAX_CAND, std::max(k * std::max(refine, 1), k + std::max(32, k)));
	const int64_t n_tiles = (n_slots + SCAN_BR - 1) / SCAN_BR;
	const bool fast_ok = (k + 8 <= MAX_CAND) && n_live > 0;
	bool all_fallback = !fast_ok;
	constexpr int64_t DENSE_MAX_ROWS = 65536;

	if (fast_ok && n_slots <= DENSE_MAX_ROWS) {
		// small store: dense lower bounds for every row, one selection
		last_stats[3] = 1;
		const int64_t cols = n_tiles * SCAN_BR;
		ws.dense.need((size_t)nq * cols);
		tic(0);
		launch_scan_dense(sv, qv, n_tiles, 1, ws.dense.p, cols, stream);
		tic(1);
		launch_select_dense(ws.dense.p, cols, cols, 1, nq, Mfinal, ws.cand_slot.p, d_cand_cnt, ws.cut.p, stream);
		launch_refine(sv, qv, ws.cand_slot.p, d_cand_cnt, Mfinal, ws.cand_dist.p, stream);
		launch_finalize(sv, ws.cand_slot.p, d_cand_cnt, ws.cand_dist.p, ws.cut.p, nq, Mfinal, k, 1, 0, nullptr, dL,
		                dD, dC, d_cert, stream);
		if (time_kernels) {
			kt_dense_ms += toc_ms(0, 1);
			kt_dense_n += 1;
		}
	} else if (fast_ok) {
		// 1) sample pass over every stride-th tile (~1/sample_div of them, at
		//    least 32 and (k+8)/2): per tile, query and 64-row quarter the row
		//    of smallest bound -> top-(k+8) of those by bound -> exact
		//    distances -> tau[q] = the k-th smallest (an upper bound on the
		//    k-th nearest distance: k real rows lie within it)
		const int64_t n_sample = std::min<int64_t>(
		    n_tiles, std::max<int64_t>({(n_tiles + sample_div - 1) / sample_div, 32, (k + 9) / 2}));
		const int64_t stride = std::max<int64_t>(1, n_tiles / n_sample);
		const int Ms = k + 8;
		const int n_seg_s = scan_grid(n_sample);
		const int cap_s = (int)round_up(4 * ((n_sample + n_seg_s - 1) / n_seg_s), 4);
		ws.seg_pool.need((size_t)n_seg_s * nq * cap_s + (size_t)n_seg_s * (nq_pad / SCAN_BQ));
		ws.seg_cnt.need((size_t)n_seg_s * nq);
		launch_scan_tilemin(sv, qv, n_sample, stride, ws.seg_pool.p, ws.seg_cnt.p, cap_s, stream);
		launch_select_segments(ws.seg_pool.p, ws.seg_cnt.p, cap_s, n_seg_s, nullptr, nq, Ms, ws.cand_slot.p,
		                       d_cand_cnt, ws.cut.p, nullptr, stream);
		launch_refine(sv, qv, ws.cand_slot.p, d_cand_cnt, Ms, ws.cand_dist.p, stream);
		launch_finalize(sv, ws.cand_slot.p, d_cand_cnt, ws.cand_dist.p, ws.cut.p, nq, Ms, k, 0, k, ws.tau.p,
		                nullptr, nullptr, nullptr, nullptr, stream);
		// 2) threshold scan over every row into per-(workgroup, query) segments;
		//    a segment holds ~4x its expected share of the (k+8)*N/sample pool
		const int n_seg = scan_grid(n_tiles);
		const int64_t expect = (int64_t)(k + 4) * ((n_tiles + n_sample - 1) / n_sample);
		const int seg_cap = (int)std::min<int64_t>(1024, round_up(std::max<int64_t>(64, 4 * expect / n_seg), 32));
		ws.seg_pool.need((size_t)n_seg * nq * seg_cap + (size_t)n_seg * (nq_pad / SCAN_BQ));  // + per-workgroup sink
		ws.seg_cnt.need((size_t)n_seg * nq);
		tic(2);
		launch_scan_append(sv, qv, ws.tau.p, ws.seg_pool.p, ws.seg_cnt.p, seg_cap, stream);
		tic(3);
		// 3) top-M by LB, exact refine, certificate
		launch_select_segments(ws.seg_pool.p, ws.seg_cnt.p, seg_cap, n_seg, ws.tau.p, nq, Mfinal, ws.cand_slot.p,
		                       d_cand_cnt, ws.cut.p, d_pool_cnt, stream);
		launch_refine(sv, qv, ws.cand_slot.p, d_cand_cnt, Mfinal, ws.cand_dist.p, stream);
		launch_finalize(sv, ws.cand_slot.p, d_cand_cnt, ws.cand_dist.p, ws.cut.p, nq, Mfinal, k, 1, 0, nullptr, dL,
		                dD, dC, d_cert, stream);
	}
	HIPCHK(hipGetLastError());

	// one pinned readback of [cert | cand_cnt | pool_cnt]
	HIPCHK(hipMemcpyAsync(ws.h_status, ws.status.p, (size_t)3 * nq * sizeof(int), hipMemcpyDeviceToHost, stream));
	spin_sync(stream);
	if (time_kernels && !all_fallback && last_stats[3] == 0) {
		kt_append_ms += toc_ms(2, 3);
		kt_append_n += 1;
		kt_append_rows = n_slots;
		kt_append_qpad = nq_pad;
	}
	const int *h_cert = ws.h_status;
	for (int q = 0; q < nq; ++q) {
		last_stats[1] += ws.h_status[nq + q];
		last_stats[2] = std::max<int64_t>(last_stats[2], ws.h_status[2 * nq + q]);
	}
	// exact fallback for every query whose certificate failed
	for (int q = 0; q < nq; ++q) {
		if (!all_fallback && h_cert[q]) continue;
		last_stats[0] += 1;
		ws.fb_keys.need((size_t)n_slots);
		ws.fb_keys2.need((size_t)n_slots);
		ws.fb_vals.need((size_t)n_slots);
		ws.fb_vals2.need((size_t)n_slots);
		launch_exact_all(sv, qv, q, ws.fb_keys.p, ws.fb_vals.p, stream);
		size_t tb = 0;
		HIPCHK((hipError_t)sort_pairs(nullptr, tb, ws.fb_keys.p, ws.fb_keys2.p, ws.fb_vals.p, ws.fb_vals2.p, n_slots,
		                              stream));
		ws.sort_tmp.need(tb);
		HIPCHK((hipError_t)sort_pairs(ws.sort_tmp.p, tb, ws.fb_keys.p, ws.fb_keys2.p, ws.fb_vals.p, ws.fb_vals2.p,
		                              n_slots, stream));
		launch_copy_fallback(ws.fb_keys2.p, ws.fb_vals2.p, n_live, k, q, dL, dD, dC, stream);
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipStreamSynchronize(stream));
}

// ---------------------------------------------------------------------------
// replay a persisted log (lance_manager.rs:136-169 open semantics)
// ---------------------------------------------------------------------------
static void replay_log(Index *ix, const std::string &path) {
	FILE *f = fopen(path.c_str(), "rb");
	if (!f) throw Error("table not found: " + path);
	char magic[8];
	int32_t d = 0;
	if (fread(magic, 1, 8, f) != 8 || memcmp(magic, "LHIPLOG1", 8) != 0 || fread(&d, 4, 1, f) != 1 || d <= 0) {
		fclose(f);
		throw Error("corrupt table log: " + path);
	}
	ix->dim = d;
	ix->ld = (int)round_up(d, DPAD);
	std::vector<float> buf;
	for (;;) {
		uint8_t tag;
		if (fread(&tag, 1, 1, f) != 1) break;
		if (tag == 1) {
			int64_t first, num;
			if (fread(&first, 8, 1, f) != 1 || fread(&num, 8, 1, f) != 1) break;
			buf.resize((size_t)num * d);
			if (fread(buf.data(), sizeof(float), buf.size(), f) != buf.size()) break;  // torn tail: ignore
			// a label at or below an existing slot label can only follow a reopen
			// that reused labels of deleted rows: drop the tombstones first so the
			// slot -> label order stays strictly ascending
			if (ix->n_slots > 0 && first <= ix->slot_label.back()) ix->compact();
			ix->next_label = first;
			ix->add_host(buf.data(), num);
		} else if (tag == 3) {
			uint8_t v;
			if (fread(&v, 1, 1, f) != 1) break;
			ix->set_storage(v == 1);
		} else if (tag == 2) {
			int64_t n;
			if (fread(&n, 8, 1, f) != 1) break;
			std::vector<int64_t> labs((size_t)n);
			if (fread(labs.data(), 8, (size_t)n, f) != (size_t)n) break;
			ix->remove(labs.data(), n);
		} else {
			break;
		}
	}
	fclose(f);
	ix->compact();
	// next_label = MAX(label)+1 over live rows, 0 when empty (lance_manager.rs:157-158, :662-696)
	int64_t mx = -1;
	for (int64_t s = 0; s < ix->n_slots; ++s)
		if (ix->live[(size_t)s]) mx = std::max(mx, ix->slot_label[(size_t)s]);
	ix->next_label = mx + 1;
}

}  // namespace lhip

using lhip::Error;
using lhip::Index;

static Index *as_index(void *h) { return reinterpret_cast<Index *>(h); }
static std::string cstr(const char *p) { return p ? std::string(p) : std::string(); }

#define API_GUARD(errprefix, failval)                                                                                  \
	catch (const std::exception &e) {                                                                                  \
		lhip::write_err(err_buf, err_buf_len, std::string(errprefix) + e.what());                                      \
		return failval;                                                                                                \
	}                                                                                                                  \
	catch (...) {                                                                                                      \
		lhip::write_err(err_buf, err_buf_len, std::string(errprefix) + "unknown error");                               \
		return failval;                                                                                                \
	}

extern "C" {

const char *lance_hip_version(void) { return "lancedb-hip 0.1.0 (gfx950)"; }

int32_t lance_hip_device_count(void) {
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return 0;
	return n;
}

void *lance_create_detached(const char *db_path, int32_t dimension, const char *metric, const char *table_name,
                            char *err_buf, int err_buf_len) {
	try {
		if (dimension <= 0) throw Error("dimension must be positive, got " + std::to_string(dimension));
		auto ix = new Index();
		try {
			ix->db_path = cstr(db_path);
			ix->table = cstr(table_name);
			if (ix->table.empty()) ix->table = "vectors";
			ix->metric_name = cstr(metric);
			ix->metric = lhip::metric_id(ix->metric_name);
			ix->dim = dimension;
			ix->ld = (int)lhip::round_up(dimension, lhip::DPAD);
			ix->init_device(-1);
			ix->log_open(true);  // drop any existing table of that name (lance_manager.rs:42)
		} catch (...) {
			delete ix;
			throw;
		}
		return ix;
	}
	API_GUARD("create failed: ", nullptr)
}

void *lance_create_detached_from_arrow(const char *db_path, void *arrow_schema, const char *metric,
                                       const char *table_name, char *err_buf, int err_buf_len) {
	if (!arrow_schema) {
		lhip::write_err(err_buf, err_buf_len, "null arrow schema");
		return nullptr;
	}
	lhip::write_err(err_buf, err_buf_len,
	                "create_from_arrow failed: multi-column (Arrow) tables are not supported by the HIP backend yet");
	return nullptr;
}

void *lance_open_detached(const char *db_path, const char *table_name, const char *metric, char *err_buf,
                          int err_buf_len) {
	try {
		auto ix = new Index();
		try {
			ix->db_path = cstr(db_path);
			ix->table = cstr(table_name);
			if (ix->table.empty()) ix->table = "vectors";
			ix->metric_name = cstr(metric);
			ix->metric = lhip::metric_id(ix->metric_name);
			if (ix->db_path.empty()) throw Error("empty db_path");
			// read the dimension first so the device store can be laid out
			{
				FILE *f = fopen(ix->log_path().c_str(), "rb");
				if (!f) throw Error("table '" + ix->table + "' not found under " + ix->db_path);
				fclose(f);
			}
			ix->init_device(-1);
			lhip::replay_log(ix, ix->log_path());
			ix->log_open(false);
		} catch (...) {
			delete ix;
			throw;
		}
		return ix;
	}
	API_GUARD("open failed: ", nullptr)
}

void lance_free_detached(void *handle) {
	if (handle) delete as_index(handle);
}

int32_t lance_detached_has_extra_columns(void *handle) {
	return 0;  // vector-only tables (Arrow multi-column path not supported yet)
}

int32_t lance_detached_dimension(void *handle) {
	if (!handle) return 0;
	return as_index(handle)->dim;
}

int64_t lance_detached_add(void *handle, const float *vector, int32_t dimension, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (dimension != ix->dim)
			throw Error("expected dimension " + std::to_string(ix->dim) + ", got " + std::to_string(dimension));
		if (!vector) throw Error("null vector");
		ix->bind();
		int64_t first = ix->add_host(vector, 1);
		ix->log_add(first, vector, 1);
		return first;
	}
	API_GUARD("add failed: ", -1)
}

int32_t lance_detached_add_batch(void *handle, const float *vectors, int32_t num, int32_t dim, int64_t *out_labels,
                                 char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (dim != ix->dim) throw Error("vector data size mismatch");
		if (num < 0) throw Error("negative batch size");
		if (num == 0) return 0;
		if (!vectors || !out_labels) throw Error("null buffer");
		ix->bind();
		int64_t first = ix->add_host(vectors, num);
		ix->log_add(first, vectors, num);
		for (int32_t i = 0; i < num; ++i) out_labels[i] = first + i;
		return num;
	}
	API_GUARD("add_batch failed: ", -1)
}

int32_t lance_detached_add_batch_arrow(void *handle, void *arrow_schema, void *arrow_array, int64_t *out_labels,
                                       char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	if (!arrow_schema || !arrow_array) {
		lhip::write_err(err_buf, err_buf_len, "null arrow schema/array");
		return -1;
	}
	lhip::write_err(err_buf, err_buf_len,
	                "add_batch_arrow failed: multi-column (Arrow) ingest is not supported by the HIP backend yet");
	return -1;
}

int32_t lance_detached_merge(void *target_handle, void *source_handle, const int64_t *live_source_labels,
                             int32_t live_count, int64_t *out_old_labels, int64_t *out_new_labels, char *err_buf,
                             int err_buf_len) {
	if (!target_handle || !source_handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *tg = as_index(target_handle);
		Index *src = as_index(source_handle);
		if (live_count <= 0 || !live_source_labels) return 0;
		if (tg->dim != src->dim) throw Error("dimension mismatch between merged indexes");
		// rows of source selected by `label IN (...)`, in source (label) order
		std::vector<int64_t> want(live_source_labels, live_source_labels + live_count);
		std::sort(want.begin(), want.end());
		want.erase(std::unique(want.begin(), want.end()), want.end());
		std::vector<int64_t> olds;
		std::vector<float> vecs;
		{
			std::lock_guard<std::mutex> g(src->mu);
			src->bind();
			std::vector<float> row((size_t)src->dim);
			for (int64_t l : want) {
				int64_t s = src->slot_of(l);
				if (s < 0 || !src->live[(size_t)s]) continue;
				src->read_rows(s, 1, row.data());
				vecs.insert(vecs.end(), row.begin(), row.end());
				olds.push_back(l);
			}
		}
		if (olds.empty()) return 0;
		std::lock_guard<std::mutex> g(tg->mu);
		tg->bind();
		int64_t first = tg->add_host(vecs.data(), (int64_t)olds.size());
		tg->log_add(first, vecs.data(), (int64_t)olds.size());
		for (size_t i = 0; i < olds.size(); ++i) {
			out_old_labels[i] = olds[i];
			out_new_labels[i] = first + (int64_t)i;
		}
		return (int32_t)olds.size();
	}
	API_GUARD("merge failed: ", -1)
}

int32_t lance_detached_search_batch(void *handle, const float *queries, int32_t nq, int32_t dim, int32_t k,
                                    int32_t nprobes, int32_t refine_factor, const char *predicate,
                                    int64_t *out_labels, float *out_distances, int32_t *out_counts, char *err_buf,
                                    int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		if (predicate && predicate[0])
			throw Error("predicate pushdown needs metadata columns, which the HIP backend does not store yet");
		if (dim != ix->dim)
			throw Error("expected query dimension " + std::to_string(ix->dim) + ", got " + std::to_string(dim));
		if (nq < 0) throw Error("negative query count");
		if (nq == 0) return 0;
		if (!queries || !out_labels || !out_distances || !out_counts) throw Error("null buffer");
		std::lock_guard<std::mutex> g(ix->mu);
		if (k <= 0 || ix->n_live == 0) {
			for (int32_t i = 0; i < nq; ++i) out_counts[i] = 0;
			for (int64_t i = 0; i < (int64_t)nq * std::max(k, 0); ++i) {
				out_labels[i] = -1;
				out_distances[i] = NAN;
			}
			return nq;
		}
		ix->bind();
		auto &ws = ix->ws;
		ws.Qin.need((size_t)nq * dim);
		ws.out_l.need((size_t)nq * k);
		ws.out_d.need((size_t)nq * k);
		ws.out_c.need((size_t)nq);
		HIPCHK(hipMemcpyAsync(ws.Qin.p, queries, (size_t)nq * dim * sizeof(float), hipMemcpyHostToDevice, ix->stream));
		ix->search_device(ws.Qin.p, nq, k, refine_factor, ws.out_l.p, ws.out_d.p, ws.out_c.p);
		HIPCHK(hipMemcpyAsync(out_labels, ws.out_l.p, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost,
		                      ix->stream));
		HIPCHK(hipMemcpyAsync(out_distances, ws.out_d.p, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost,
		                      ix->stream));
		HIPCHK(hipMemcpyAsync(out_counts, ws.out_c.p, (size_t)nq * sizeof(int32_t), hipMemcpyDeviceToHost,
		                      ix->stream));
		HIPCHK(hipStreamSynchronize(ix->stream));
		return nq;
	}
	API_GUARD("search failed: ", -1)
}

int32_t lance_detached_search_with_predicate(void *handle, const float *query, int32_t dim, int32_t k,
                                             int32_t nprobes, int32_t refine_factor, const char *predicate,
                                             int64_t *out_labels, float *out_distances, char *err_buf,
                                             int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	if (k <= 0) return 0;
	std::vector<int64_t> l((size_t)k);
	std::vector<float> d((size_t)k);
	int32_t cnt = 0;
	int32_t r = lance_detached_search_batch(handle, query, 1, dim, k, nprobes, refine_factor, predicate, l.data(),
	                                        d.data(), &cnt, err_buf, err_buf_len);
	if (r < 0) return -1;
	for (int32_t i = 0; i < cnt; ++i) {
		out_labels[i] = l[(size_t)i];
		out_distances[i] = d[(size_t)i];
	}
	return cnt;
}

int32_t lance_detached_search(void *handle, const float *query, int32_t dim, int32_t k, int32_t nprobes,
                              int32_t refine_factor, int64_t *out_labels, float *out_distances, char *err_buf,
                              int err_buf_len) {
	return lance_detached_search_with_predicate(handle, query, dim, k, nprobes, refine_factor, nullptr, out_labels,
	                                            out_distances, err_buf, err_buf_len);
}

int64_t lance_detached_count(void *handle, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	return ix->n_live;
}

int32_t lance_detached_delete_batch(void *handle, const int64_t *labels, int32_t count, char *err_buf,
                                    int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		if (count <= 0) return 0;
		if (!labels) throw Error("null labels");
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();
		auto done = ix->remove(labels, count);
		ix->log_del(done);
		return 0;
	}
	API_GUARD("delete_batch failed: ", -1)
}

int32_t lance_detached_delete(void *handle, int64_t label, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	int32_t r = lance_detached_delete_batch(handle, &label, 1, err_buf, err_buf_len);
	if (r != 0 && err_buf && err_buf_len > 0) {
		std::string m(err_buf);
		const std::string pre = "delete_batch failed: ";
		if (m.compare(0, pre.size(), pre) == 0) lhip::write_err(err_buf, err_buf_len, "delete failed: " + m.substr(pre.size()));
	}
	return r;
}

int32_t lance_detached_create_index(void *handle, int32_t num_partitions, int32_t num_sub_vectors, char *err_buf,
                                    int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	ix->ivf_partitions = num_partitions;
	ix->ivf_sub_vectors = num_sub_vectors;
	return 0;
}

int32_t lance_detached_create_hnsw_index(void *handle, int32_t m, int32_t ef_construction, char *err_buf,
                                          int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	return 0;
}

int32_t lance_detached_compact(void *handle, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();
		ix->compact();
		return 0;
	}
	API_GUARD("compact failed: ", -1)
}

int32_t lance_detached_get_vector(void *handle, int64_t label, float *out_vec, int32_t capacity, char *err_buf,
                                  int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		int64_t s = ix->slot_of(label);
		if (s < 0 || !ix->live[(size_t)s]) throw Error("label " + std::to_string(label) + " not found");
		if (ix->dim > capacity) {
			lhip::write_err(err_buf, err_buf_len, "output buffer too small");
			return -1;
		}
		ix->bind();
		ix->read_rows(s, 1, out_vec);
		return ix->dim;
	}
	API_GUARD("get_vector failed: ", -1)
}

int32_t lance_detached_get_all_vectors(void *handle, int64_t *out_labels, float *out_vectors, int64_t *out_count,
                                       char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (out_count) *out_count = ix->n_live;
		if (out_labels && out_vectors && ix->n_live > 0) {
			ix->bind();
			std::vector<float> all((size_t)ix->n_slots * ix->dim);
			ix->read_rows(0, ix->n_slots, all.data());
			int64_t j = 0;
			for (int64_t s = 0; s < ix->n_slots; ++s) {
				if (!ix->live[(size_t)s]) continue;
				out_labels[j] = ix->slot_label[(size_t)s];
				memcpy(out_vectors + j * ix->dim, all.data() + s * ix->dim, (size_t)ix->dim * sizeof(float));
				++j;
			}
		}
		return (int32_t)ix->n_live;
	}
	API_GUARD("get_all_vectors failed: ", -1)
}

int32_t lance_hip_set_option(void *handle, const char *key, const char *value, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		std::string k = cstr(key), v = cstr(value);
		if (k == "metric_quirk") {
			bool on = (v == "1" || v == "true");
			if (on && ix->metric != lhip::METRIC_L2 && !ix->rowaux_l2) {
				// build L2 aux for the rows already stored
				ix->bind();
				HIPCHK(hipMalloc(&ix->rowaux_l2, (size_t)std::max<int64_t>(ix->cap, 1) * sizeof(float4)));
				if (ix->n_slots > 0) {
					lhip::launch_rowaux(ix->X, ix->xbf16, ix->ld, ix->dim, lhip::METRIC_L2, 0, ix->n_slots, ix->rowaux_l2,
					                    ix->stats.p + 2, ix->stream);
					// re-apply tombstones
					std::vector<int64_t> dead;
					for (int64_t s = 0; s < ix->n_slots; ++s)
						if (!ix->live[(size_t)s]) dead.push_back(s);
					if (!dead.empty()) {
						ix->ws.idx.need(dead.size());
						HIPCHK(hipMemcpyAsync(ix->ws.idx.p, dead.data(), dead.size() * sizeof(int64_t),
						                      hipMemcpyHostToDevice, ix->stream));
						lhip::launch_tombstone(ix->rowaux_l2, ix->ws.idx.p, (int)dead.size(), ix->stream);
					}
					HIPCHK(hipStreamSynchronize(ix->stream));
					ix->refresh_stats();
				}
			}
			ix->metric_quirk = on;
			return 0;
		}
		if (k == "time_kernels") {
			ix->bind();
			ix->time_kernels = (v == "1" || v == "true");
			for (auto &e : ix->ev)
				if (!e) HIPCHK(hipEventCreate(&e));
			ix->kt_append_ms = ix->kt_dense_ms = 0.0;
			ix->kt_append_n = ix->kt_dense_n = 0;
			return 0;
		}
		if (k == "storage") {
			if (v != "f32" && v != "bf16") throw Error("storage must be 'f32' or 'bf16'");
			ix->bind();
			const bool was = ix->xbf16;
			ix->set_storage(v == "bf16");
			if (was != ix->xbf16) ix->log_storage();
			return 0;
		}
		if (k == "scan_copy") {
			if (v != "on" && v != "off") throw Error("scan_copy must be 'on' or 'off'");
			ix->bind();
			ix->set_scan_copy(v == "on");
			return 0;
		}
		if (k == "sample_div") {
			const int d = std::stoi(v);
			if (d < 1) throw Error("sample_div must be >= 1");
			ix->sample_div = d;
			return 0;
		}
		if (k == "reserve_rows") {
			ix->bind();
			ix->reserve(std::stoll(v));
			return 0;
		}
		throw Error("unknown option '" + k + "'");
	}
	API_GUARD("set_option failed: ", -1)
}

int32_t lance_hip_last_search_stats(void *handle, int64_t *out, int32_t n) {
	if (!handle || !out) return -1;
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	for (int32_t i = 0; i < n && i < 4; ++i) out[i] = ix->last_stats[i];
	return 0;
}

// out[0] = total ms of threshold-scan launches, out[1] = their count,
// out[2] = rows scanned per launch, out[3] = padded queries per launch,
// out[4] = total ms of small-store dense scans, out[5] = their count,
// out[6] = bytes per element the scan streams (2: bf16 store or scan copy).
int32_t lance_hip_kernel_times(void *handle, double *out, int32_t n) {
	if (!handle || !out) return -1;
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	double v[7] = {ix->kt_append_ms, (double)ix->kt_append_n, (double)ix->kt_append_rows,
		               (double)ix->kt_append_qpad, ix->kt_dense_ms, (double)ix->kt_dense_n,
		               (ix->xbf16 || ix->Xs) ? 2.0 : 4.0};
		for (int32_t i = 0; i < n && i < 7; ++i) out[i] = v[i];
	return 0;
}

// ---- device-pointer entry points (benchmarks / multi-GPU ranks) -----------

int64_t lance_hip_add_batch_device(void *handle, const float *d_vectors, int64_t num, int32_t dim, char *err_buf,
                                   int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (dim != ix->dim) throw Error("vector data size mismatch");
		if (num <= 0) return ix->next_label;
		ix->bind();
		int64_t first = ix->add_device(d_vectors, num);
		if (ix->log) {
			std::vector<float> h((size_t)num * dim);
			HIPCHK(hipMemcpy(h.data(), d_vectors, h.size() * sizeof(float), hipMemcpyDeviceToHost));
			ix->log_add(first, h.data(), num);
		}
		return first;
	}
	API_GUARD("add_batch failed: ", -1)
}

int32_t lance_hip_search_batch_device(void *handle, const float *d_queries, int32_t nq, int32_t dim, int32_t k,
                                      int32_t nprobes, int32_t refine_factor, int64_t *d_out_labels,
                                      float *d_out_distances, int32_t *d_out_counts, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		if (dim != ix->dim)
			throw Error("expected query dimension " + std::to_string(ix->dim) + ", got " + std::to_string(dim));
		if (k <= 0) throw Error("k must be positive");
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();
		if (ix->n_live == 0) {
			HIPCHK(hipMemsetAsync(d_out_counts, 0, (size_t)nq * sizeof(int32_t), ix->stream));
			HIPCHK(hipStreamSynchronize(ix->stream));
			return nq;
		}
		ix->search_device(d_queries, nq, k, refine_factor, d_out_labels, d_out_distances, d_out_counts);
		return nq;
	}
	API_GUARD("search failed: ", -1)
}

int32_t lance_hip_merge_topk(int32_t nshard, int32_t nq, int32_t k, const int64_t *part_labels,
                             const float *part_dists, const int32_t *part_counts, int64_t *out_labels,
                             float *out_dists, int32_t *out_counts, char *err_buf, int err_buf_len) {
	try {
		if (nshard <= 0 || nq <= 0 || k <= 0) return 0;
		int dev = 0;
		HIPCHK(hipGetDevice(&dev));
		hipStream_t st;
		HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
		int64_t *pl = nullptr, *ol = nullptr;
		float *pd = nullptr, *od = nullptr;
		int *pc = nullptr, *oc = nullptr;
		const size_t P = (size_t)nshard * nq * k;
		HIPCHK(hipMalloc(&pl, P * sizeof(int64_t)));
		HIPCHK(hipMalloc(&pd, P * sizeof(float)));
		HIPCHK(hipMalloc(&pc, (size_t)nshard * nq * sizeof(int)));
		HIPCHK(hipMalloc(&ol, (size_t)nq * k * sizeof(int64_t)));
		HIPCHK(hipMalloc(&od, (size_t)nq * k * sizeof(float)));
		HIPCHK(hipMalloc(&oc, (size_t)nq * sizeof(int)));
		HIPCHK(hipMemcpyAsync(pl, part_labels, P * sizeof(int64_t), hipMemcpyHostToDevice, st));
		HIPCHK(hipMemcpyAsync(pd, part_dists, P * sizeof(float), hipMemcpyHostToDevice, st));
		HIPCHK(hipMemcpyAsync(pc, part_counts, (size_t)nshard * nq * sizeof(int), hipMemcpyHostToDevice, st));
		lhip::launch_merge_topk(nshard, nq, k, pl, pd, pc, ol, od, oc, st);
		HIPCHK(hipGetLastError());
		HIPCHK(hipMemcpyAsync(out_labels, ol, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost, st));
		HIPCHK(hipMemcpyAsync(out_dists, od, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, st));
		HIPCHK(hipMemcpyAsync(out_counts, oc, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st));
		HIPCHK(hipStreamSynchronize(st));
		(void)hipFree(pl);
		(void)hipFree(pd);
		(void)hipFree(pc);
		(void)hipFree(ol);
		(void)hipFree(od);
		(void)hipFree(oc);
		(void)hipStreamDestroy(st);
		return nq;
	}
	API_GUARD("merge_topk failed: ", -1)
}

// device-pointer merge (all arguments device pointers, stream = handle-free)
int32_t lance_hip_merge_topk_device(int32_t nshard, int32_t nq, int32_t k, const int64_t *d_part_labels,
                                    const float *d_part_dists, const int32_t *d_part_counts, int64_t *d_out_labels,
                                    float *d_out_dists, int32_t *d_out_counts, char *err_buf, int err_buf_len) {
	try {
		if (nshard <= 0 || nq <= 0 || k <= 0) return 0;
		lhip::launch_merge_topk(nshard, nq, k, d_part_labels, d_part_dists, d_part_counts, d_out_labels, d_out_dists,
		                        d_out_counts, nullptr);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(nullptr));
		return nq;
	}
	API_GUARD("merge_topk failed: ", -1)
}

}  // extern "C"
