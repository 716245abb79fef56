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
#include <unistd.h>
#include <vector>
#include "index.h"
#include "ivf.h"

namespace lhip {

void Index::search_device(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC) {
	for (auto &v : last_stats) v = 0;
	// one pipeline pass covers up to MAX_PASS_Q queries (several query tiles
	// per scan launch): the per-pass fixed cost is paid once per pass
	for (int s = 0; s < nq; s += MAX_PASS_Q) {
		int c = std::min(MAX_PASS_Q, nq - s);
		search_chunk(dQ + (int64_t)s * dim, c, k, refine, dL + (int64_t)s * k, dD + (int64_t)s * k, dC + s);
	}
}

void Index::search_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC) {
	PendingPass p;
	if (enqueue_chunk(dQ, nq, k, refine, dL, dD, dC, pb_free_slot(), false, p)) finish_chunk(p);
}

// the pass-buffer set no pending pass holds (at most one pass is pending when
// a new one is enqueued)
int Index::pb_free_slot() const {
	for (int i = 0; i < 2; ++i) {
		bool used = false;
		for (const auto &q : pending) used |= q.slot == i;
		if (!used) return i;
	}
	throw Error("internal: no free pass buffers");
}

// Everything of a search pass up to its completion wait: prep, sample pass,
// threshold scan, final refine (or the dense path of small stores), enqueued
// on the handle's stream.  Returns false when the pass already completed (the
// one-launch small exact search); otherwise `p` describes what finish_chunk
// checks once the stream reaches its end.  async: other passes may still be
// pending on the stream; any workspace the pending kernels read is kept
// (growth drains them first).
bool Index::enqueue_chunk(const float *dQ, int nq, int k, int refine, int64_t *dL, float *dD, int *dC, int slot,
                          bool async, PendingPass &p) {
	PassBufs &P = pb[slot];
	// an asynchronous pass runs on its pass-buffer set's own stream, after
	// everything already on the handle's stream: pass i+1's prep, sample pass and
	// tau refine overlap pass i's final refine (they share no buffer: queries,
	// status and segment pools are per set)
	hipStream_t st = stream;
	if (async) {
		st = pass_stream(slot);
		HIPCHK(hipEventRecord(ev_order, stream));
		HIPCHK(hipStreamWaitEvent(st, ev_order, 0));
	}
	const int eff_metric = metric_quirk ? METRIC_L2 : metric;
	const float4 *aux = search_aux((metric_quirk && metric != METRIC_L2) ? rowaux_l2 : rowaux);
	const float ma = (metric_quirk && metric != METRIC_L2) ? max_alpha_l2 : max_alpha;
	// int8 scan copy (option scan_i8): the scans st int8 rows with their own
	// row terms; refine, fallback and the outputs read X and rowaux as always.
	// Any k on the threshold path (pool_refine refines as far as its certificate
	// needs); k <= 32 on the dense path of small stores (a fixed candidate count:
	// past that the looser bounds leave more rows below the k-th distance than
	// it holds); otherwise bf16 rows
	const bool use8 = scan_uses_i8(nq, k);
	if (!use8) ensure_xs();
	const float mu = (metric_quirk && metric != METRIC_L2) ? max_ux_l2 : max_ux;
	StoreView sv{X, aux, dlabels, n_slots, ld, dim, eff_metric, xbf16 ? 1 : 0,
	             Xs ? static_cast<const void *>(Xs) : X, (xbf16 || Xs) ? 1 : 0};
	sv.pr_first = pr_first;
	sv.s8_variant = s8_variant;
	sv.tie_desc = tie_desc;
	if (s8_couple > 0) {
		if (!P.s8prog.p) {
			P.s8prog.need((size_t)scan8_prog_words());
			HIPCHK(hipMemsetAsync(P.s8prog.p, 0, (size_t)scan8_prog_words() * sizeof(unsigned long long), st));
		}
		sv.s8_prog = P.s8prog.p;
		sv.s8_couple = s8_couple;
	}
	last_scan_esz = use8 ? 1 : (xbf16 || Xs) ? 2 : 4;
	if (use8) {
		ensure_i8();
		sv.Xscan = Xq;
		sv.scan_aux = rowaux8;
		sv.scan_i8 = 1;
		sv.tstat = tstat8;
	}
	if (small_exact && small_exact_fits(n_slots, dim, nq, k)) {
		// a few queries over a small store (one query per lance_search call):
		// one launch of exact distances + merge, no bounds, no status readback
		last_stats[3] = 2;
		const size_t np = (size_t)nq * small_exact_grid(n_slots) * k;
		ws.spart.need(np);
		if (ws.scnt.n < (size_t)SMALL_MAX_Q) {
			ws.scnt.need(SMALL_MAX_Q);
			HIPCHK(hipMemsetAsync(ws.scnt.p, 0, ws.scnt.n * sizeof(unsigned), st));
		}
		tic(0);
		launch_small_exact(sv, dQ, nq, k, ws.spart.p, ws.scnt.p, dL, dD, dC, st);
		tic(1);
		HIPCHK(hipGetLastError());
		if (time_kernels) {
			kt_dense_ms += toc_ms(0, 1);  // reported with the dense-path launches
			kt_dense_n += 1;
		}
		if (!defer_sync) HIPCHK(hipStreamSynchronize(st));
		return false;
	}
	const int nq_pad = (int)round_up(nq, SCAN_BQ);
	P.Qf.need((size_t)nq_pad * ld);
	P.Qb.need((size_t)nq_pad * ld);
	P.qaux.need(nq_pad);
	P.tau.need(nq);
	ws.cut.need(nq);
	ws.cand_slot.need((size_t)nq * MAX_CAND);
	ws.cand_dist.need((size_t)nq * MAX_CAND);
	P.need_host_status((size_t)3 * nq);
	// [cert | cand_cnt | pool_cnt]: on the threshold path the kernels write it
	// straight into pinned host memory (only pool_refine / retry_scatter store
	// into it, no kernel reads it back), so the step ends with one st wait
	// and no readback copy; the dense path keeps it in HBM (its refine and
	// finalize read the candidate counts) and copies it back once
	const bool hmap = n_slots > 65536;
	int *dstat;
	if (hmap) {
		dstat = P.d_status_map;
	} else {
		P.status.need((size_t)3 * nq);
		dstat = P.status.p;
	}
	int *d_cert = dstat, *d_cand_cnt = dstat + nq, *d_pool_cnt = dstat + 2 * nq;
	if (use8) {
		P.qm.need(nq);
		launch_prep_queries_i8(dQ, nq, dim, ld, nq_pad, eff_metric, max_alpha8, max_x8, P.qm.p, P.Qf.p, P.Qb.p,
		                       P.qaux.p, dstat, st);
	}
	else
		launch_prep_queries(dQ, nq, dim, ld, nq_pad, eff_metric, ma, mu, P.Qf.p, P.Qb.p, P.qaux.p, dstat,
		                    st);
	QueryView qv{P.Qf.p, P.Qb.p, P.qaux.p, nq, nq_pad};

	// refined candidates: k + max(32, k) — past k the bound slack (bf16 query
	// rounding) spans more ranks as the neighbour distances crowd (C3: k = 100)
	// (int8 scan: looser bounds, more rows below the k-th distance, cand_extra_i8)
	const int Mfinal = std::min(MAX_CAND, std::max(k * std::max(refine, 1), k + std::max(use8 ? cand_extra_i8_eff() : cand_extra, k)));
	const int64_t n_tiles = (n_slots + SCAN_BR - 1) / SCAN_BR;
	const bool fast_ok = (k + 8 <= MAX_CAND) && live_rows() > 0;
	constexpr int64_t DENSE_MAX_ROWS = 65536;

	if (fast_ok && n_slots <= DENSE_MAX_ROWS) {
		// small store: dense lower bounds for every row, one selection
		last_stats[3] = 1;
		const int64_t cols = n_tiles * SCAN_BR;
		ws.dense.need((size_t)nq * cols);
		tic(0);
		launch_scan_dense(sv, qv, n_tiles, 1, ws.dense.p, cols, st);
		tic(1);
		launch_select_dense(ws.dense.p, cols, cols, 1, nq, Mfinal, ws.cand_slot.p, d_cand_cnt, ws.cut.p, st,
		                    tie_desc);
		launch_refine(sv, qv, ws.cand_slot.p, d_cand_cnt, Mfinal, ws.cand_dist.p, st);
		launch_finalize(sv, ws.cand_slot.p, d_cand_cnt, ws.cand_dist.p, ws.cut.p, nq, Mfinal, k, 1, 0, nullptr, dL,
		                dD, dC, d_cert, st, live_rows());
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
		const int sdiv = sample_div_eff(n_tiles);
		const int64_t n_sample = std::min<int64_t>(
		    n_tiles, std::max<int64_t>({(n_tiles + sdiv - 1) / sdiv, 32, (k + 9) / 2}));
		const int64_t stride = std::max<int64_t>(1, n_tiles / n_sample);
		const int Ms = k + 8;
		// (int8 copy: scan8_kernel's tilemin mode, one entry per 32-row unit; else
		// scan_kernel's, one per 64-row quarter)
		const bool s8s = scan8_fits(sv);
		const int n_seg_s = s8s ? scan8_segments(n_sample) : scan_grid(n_sample);
		const int cap_s = s8s ? scan8_tilemin_cap(n_sample) : (int)round_up(4 * ((n_sample + n_seg_s - 1) / n_seg_s), 4);
		// 2) threshold scan over every row into per-(workgroup, query) segments;
		//    a segment holds ~4x its expected share of the (k+8)*N/sample pool.
		//    int8 scan8 path, large stores: progressive threshold.  The first
		//    1/split_div of the tiles (A) with the sample's tau; A's pool refined
		//    in tau mode gives tau' = min(tau, k-th exact distance among A's
		//    smallest bounds) (~d_80 instead of ~d_320 of 10M rows at 1/8); the
		//    other tiles (B) with tau'.  Rows left out have LB > tau >= tau' (A)
		//    or LB > tau' (B): the final pass certifies against tau'.  About 2.5x
		//    fewer appended bounds at 10M x 768.
		const int64_t tA = (split_div > 1 && scan8_fits(sv) && n_tiles >= (int64_t)128 * split_div)
		                       ? n_tiles / split_div
		                       : 0;
		const int nA = tA ? scan8_segments(tA) : 0;
		const int n_seg = tA ? nA + scan8_segments(n_tiles - tA) : scan_append_segments(sv, n_tiles);
		const int n_seg1 = tA ? n_seg : scan_append_segments(sv, n_tiles);  // (segments one pass would write)
		// (32x headroom: the int8 bounds put several times more rows under tau
		// than (k+4)*N/sample, and pool_refine keeps the smallest of a pool past
		// its LDS capacity, but a segment past seg_cap fails the certificate)
		const int64_t expect = (int64_t)(k + 4) * ((n_tiles + n_sample - 1) / n_sample);
		const int seg_cap = (int)std::min<int64_t>(1024, round_up(std::max<int64_t>(64, 32 * expect / n_seg1), 32));
		const size_t pool_s = (size_t)n_seg_s * nq * cap_s + (size_t)n_seg_s * (nq_pad / SCAN_BQ);
		const size_t pool_a = (size_t)n_seg * nq * seg_cap + (size_t)n_seg * (nq_pad / SCAN_BQ);  // + per-workgroup sink
		const size_t cnt_n = (size_t)std::max(n_seg_s, n_seg) * nq;
		// (this pass's own segment pools: no pending pass reads them)
		P.seg_pool.need(std::max(pool_s, pool_a));
		P.seg_cnt.need(cnt_n);
		if (s8s)
			launch_scan8_tilemin(sv, qv, n_sample, stride, P.seg_pool.p, P.seg_cnt.p, cap_s, st);
		else
			launch_scan_tilemin(sv, qv, n_sample, stride, P.seg_pool.p, P.seg_cnt.p, cap_s, st);
		launch_pool_refine(sv, qv, P.seg_pool.p, P.seg_cnt.p, cap_s, n_seg_s, nullptr, k, 0, Ms, -1, P.tau.p,
		                   nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st);
		tic(2);
		last_stats[5] += tA ? 2 : 1;  // threshold append launches of the first pass
		if (tA) {
			launch_scan8_append(sv, qv, P.tau.p, P.seg_pool.p, P.seg_cnt.p, seg_cap, st, 0, tA, 0);
			tic(3);
			launch_pool_refine(sv, qv, P.seg_pool.p, P.seg_cnt.p, seg_cap, nA, P.tau.p, k, 0, Ms, -1, P.tau.p,
			                   nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, st);
			tic(4);
			launch_scan8_append(sv, qv, P.tau.p, P.seg_pool.p, P.seg_cnt.p, seg_cap, st, tA, n_tiles, nA);
			tic(5);
		} else {
			launch_scan_append(sv, qv, P.tau.p, P.seg_pool.p, P.seg_cnt.p, seg_cap, st);
			tic(3);
		}
		// 3) the pool in bound order, exact refine until certified
#ifdef LHIP_DEV_PR_IDLE  // (development build: the final refine starts on an idle GPU, DVFS probe)
		HIPCHK(hipStreamSynchronize(st));
		usleep(LHIP_DEV_PR_IDLE);
#endif
		launch_pool_refine(sv, qv, P.seg_pool.p, P.seg_cnt.p, seg_cap, n_seg, P.tau.p, k, 1, 0, live_rows(),
		                   nullptr, dL, dD, dC, d_cert, d_cand_cnt, d_pool_cnt, st);
		p.two_append = tA > 0;
	}
	HIPCHK(hipGetLastError());
	// [cert | cand_cnt | pool_cnt] on the host: written in place (threshold
	// path) or one pinned readback (dense path)
	if (!hmap)
		HIPCHK(hipMemcpyAsync(P.h_status, P.status.p, (size_t)3 * nq * sizeof(int), hipMemcpyDeviceToHost, st));
	p.slot = slot;
	p.nq = nq;
	p.k = k;
	p.dL = dL;
	p.dD = dD;
	p.dC = dC;
	p.sv = sv;
	p.qv = qv;
	p.hmap = hmap;
	p.fast_ok = fast_ok;
	p.dense = last_stats[3] == 1;
	p.n_tiles = n_tiles;
	if (async) {
		if (!P.done) HIPCHK(hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
		HIPCHK(hipEventRecord(P.done, st));
	}
	return true;
}

// The rest of a pass once its kernels completed: the certificate check, the
// reruns of uncertified queries and the exact fallback (synchronous).
void Index::finish_chunk(PendingPass &p) {
	PassBufs &P = pb[p.slot];
	// reruns and the exact fallback run on the pass's own stream (an
	// asynchronous pass's kernels and the later pass share no buffer)
	const hipStream_t st = p.async ? pass_stream(p.slot) : stream;
	const int nq = p.nq, k = p.k;
	int64_t *dL = p.dL;
	float *dD = p.dD;
	int *dC = p.dC;
	const StoreView &sv = p.sv;
	const QueryView &qv = p.qv;
	const bool hmap = p.hmap, fast_ok = p.fast_ok, all_fallback = !p.fast_ok;
	const int64_t n_tiles = p.n_tiles;
	constexpr int64_t DENSE_MAX_ROWS = 65536;
	int *dstat = hmap ? P.d_status_map : P.status.p;
	int *d_cert = dstat;
	// a pass enqueued asynchronously completes at its event (later passes may be
	// queued behind it); a synchronous one at the end of the st
	if (p.async) {
		for (auto &v : last_stats) v = 0;  // this pass's statistics alone
		last_stats[3] = p.st3;
		last_stats[5] = p.st5;
		hipError_t e;
		while ((e = hipEventQuery(P.done)) == hipErrorNotReady) {
		}
		if (e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e) + " at pass completion");
	} else {
		spin_sync(st);
	}
	if (time_kernels && !all_fallback && !p.dense) {
		// the append scan's own time (both launches of a progressive pass)
		kt_append_ms += toc_ms(2, 3) + (p.two_append ? toc_ms(4, 5) : 0.f);
		kt_append_n += 1;
		kt_append_rows = n_slots;
		kt_append_qpad = qv.nq_pad;
		kt_append_kernel = scan8_fits(sv) ? 2 : 0;
	}
	const int *h_cert = P.h_status;
	for (int q = 0; q < nq; ++q) {
		last_stats[1] += P.h_status[nq + q];
		last_stats[2] = std::max<int64_t>(last_stats[2], P.h_status[2 * nq + q]);
	}
	// (reruns / fallback below: a later pass still in flight on the other pass
	// stream reads none of the workspace they use — its queries, status, tau and
	// segment pools are its own set's)
	// threshold path: rerun the uncertified queries as a batch of their own,
	// tau = their previous pass's k-th exact distance, full-size segments (up
	// to two reruns: a pool over the selection's capacity still yields real
	// candidates, so each rerun's tau tightens)
	// A query that found no candidate at all (NaN bound: a zero cosine query)
	// goes straight to the exact fallback.
	std::vector<char> rerun(nq, 0);
	for (int q = 0; q < nq; ++q) rerun[q] = !h_cert[q] && P.h_status[nq + q] > 0;
	bool enqueued = false;
	for (int attempt = 0; attempt < 2 && fast_ok && n_slots > DENSE_MAX_ROWS && retry_pass; ++attempt) {
		std::vector<int> fq;
		for (int q = 0; q < nq; ++q)
			if (rerun[q] && !h_cert[q]) fq.push_back(q);
		const int nf = (int)fq.size();
		if (nf == 0) break;
		enqueued = true;
		{
			if (attempt == 0) last_stats[4] += nf;
			const int nf_pad = (int)round_up(nf, SCAN_BQ);
			ws.rfq.need(nf);
			ws.rQf.need((size_t)nf_pad * ld);
			ws.rQb.need((size_t)nf_pad * ld);
			ws.rqaux.need(nf_pad);
			ws.rtau.need(nf);
			ws.rstat.need((size_t)3 * nf);
			ws.rL.need((size_t)nf * k);
			ws.rD.need((size_t)nf * k);
			ws.rC.need(nf);
			HIPCHK(hipMemcpyAsync(ws.rfq.p, fq.data(), (size_t)nf * sizeof(int), hipMemcpyHostToDevice, st));
			// tau tightened to just above the first pass's k-th distance (a pool
			// that overflowed shrinks; pool_refine refines as far as it needs)
			launch_retry_gather(ws.rfq.p, nf, nf_pad, ld, k, qv, P.tau.p, dD, ws.rQf.p, ws.rQb.p, ws.rqaux.p,
			                    ws.rtau.p, ws.rstat.p, st);
			const QueryView qv2{ws.rQf.p, ws.rQb.p, ws.rqaux.p, nf, nf_pad};
			const int n_seg = scan_append_segments(sv, n_tiles);
			int cap2 = 1024;  // the scan's maximum, bounded to a 1 GiB pool
			while (cap2 > 64 && (size_t)n_seg * nf * cap2 * sizeof(uint2) > ((size_t)1 << 30)) cap2 /= 2;
			P.seg_pool.need((size_t)n_seg * nf * cap2 + (size_t)n_seg * (nf_pad / SCAN_BQ));
			P.seg_cnt.need((size_t)n_seg * nf);
			int *cert2 = ws.rstat.p, *cnt2 = ws.rstat.p + nf, *pool2 = ws.rstat.p + 2 * nf;
			launch_scan_append(sv, qv2, ws.rtau.p, P.seg_pool.p, P.seg_cnt.p, cap2, st);
			launch_pool_refine(sv, qv2, P.seg_pool.p, P.seg_cnt.p, cap2, n_seg, ws.rtau.p, k, 1, 0, live_rows(),
			                   nullptr, ws.rL.p, ws.rD.p, ws.rC.p, cert2, cnt2, pool2, st);
			launch_retry_scatter(ws.rfq.p, nf, k, ws.rL.p, ws.rD.p, ws.rC.p, cert2, ws.rtau.p, dL, dD, dC, d_cert, P.tau.p,
			                     st);
			HIPCHK(hipGetLastError());
			if (!hmap)
				HIPCHK(hipMemcpyAsync(P.h_status, d_cert, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st));
			spin_sync(st);
		}
	}
	// exact fallback for every query whose certificate failed: one batched
	// pass — exact distances of every slot for a group of such queries, then
	// the k smallest per query by (distance, slot) with the selection the scan
	// uses (slots ascend with labels, so that is the (distance, label) order),
	// refine + finalize for the outputs — instead of a full scan and an
	// N-key radix sort per query.  A query whose selection comes up short of
	// min(k, live rows) (NaN distances: a zero cosine query) and every query
	// when k is past the selection's capacity take the per-query sort below.
	// (a query with no candidate while live rows exist had NaN bounds — a zero
	// cosine query — which no threshold keeps: exact fallback too)
	std::vector<int> fbq;
	for (int q = 0; q < nq; ++q)
		if (all_fallback || !h_cert[q] || (P.h_status[nq + q] == 0 && live_rows() > 0)) fbq.push_back(q);
	last_stats[0] += (int64_t)fbq.size();
	std::vector<int> slow;
	if (!fbq.empty() && fast_ok) {
		enqueued = true;
		const int nf = (int)fbq.size();
		const int nf_pad = (int)round_up(nf, SCAN_BQ);
		ws.rfq.need(nf);
		ws.rQf.need((size_t)nf_pad * ld);
		ws.rQb.need((size_t)nf_pad * ld);
		ws.rqaux.need(nf_pad);
		ws.rtau.need(nf);
		ws.rstat.need((size_t)3 * nf);
		ws.rL.need((size_t)nf * k);
		ws.rD.need((size_t)nf * k);
		ws.rC.need(nf);
		HIPCHK(hipMemcpyAsync(ws.rfq.p, fbq.data(), (size_t)nf * sizeof(int), hipMemcpyHostToDevice, st));
		launch_retry_gather(ws.rfq.p, nf, nf_pad, ld, k, qv, P.tau.p, dD, ws.rQf.p, ws.rQb.p, ws.rqaux.p, ws.rtau.p,
		                    ws.rstat.p, st);
		// keys of up to FB_GROUP queries at a time, within 1 GiB
		constexpr int FB_GROUP = 16;
		const int64_t cols = round_up(n_slots, 4);
		const int G = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)FB_GROUP, (int64_t)nf,
		                                                             ((int64_t)1 << 28) / cols}));
		ws.fb_keys.need((size_t)G * cols);
		int *cert2 = ws.rstat.p, *cnt2 = ws.rstat.p + nf;
		for (int g0 = 0; g0 < nf; g0 += G) {
			const int gq = std::min(G, nf - g0);
			const QueryView qg{ws.rQf.p + (size_t)g0 * ld, ws.rQb.p + (size_t)g0 * ld, ws.rqaux.p + g0, gq,
			                   (int)round_up(gq, SCAN_BQ)};
			launch_exact_dense(sv, qg, ws.fb_keys.p, cols, st);
			launch_select_dense(ws.fb_keys.p, cols, n_slots, 1, gq, k, ws.cand_slot.p, cnt2 + g0, ws.cut.p, st,
			                    tie_desc);
			launch_refine(sv, qg, ws.cand_slot.p, cnt2 + g0, k, ws.cand_dist.p, st);
			launch_finalize(sv, ws.cand_slot.p, cnt2 + g0, ws.cand_dist.p, ws.cut.p, gq, k, k, 1, 0, nullptr,
			                ws.rL.p + (size_t)g0 * k, ws.rD.p + (size_t)g0 * k, ws.rC.p + g0, cert2 + g0, st);
		}
		// exact keys: the selection is the answer whatever the certificate
		// says about ties at the cut
		HIPCHK(hipMemsetAsync(cert2, 0x01, (size_t)nf * sizeof(int), st));
		launch_retry_scatter(ws.rfq.p, nf, k, ws.rL.p, ws.rD.p, ws.rC.p, cert2, ws.rtau.p, dL, dD, dC, d_cert,
		                     P.tau.p, st);
		HIPCHK(hipGetLastError());
		std::vector<int> hc((size_t)nf);
		HIPCHK(hipMemcpyAsync(hc.data(), ws.rC.p, (size_t)nf * sizeof(int), hipMemcpyDeviceToHost, st));
		HIPCHK(hipStreamSynchronize(st));
		const int64_t want = std::min<int64_t>(k, live_rows());
		for (int i = 0; i < nf; ++i)
			if (hc[(size_t)i] < want) slow.push_back(fbq[(size_t)i]);
	} else {
		slow = fbq;
	}
	for (int q : slow) {
		enqueued = true;
		ws.fb_keys.need((size_t)n_slots);
		ws.fb_keys2.need((size_t)n_slots);
		ws.fb_vals.need((size_t)n_slots);
		ws.fb_vals2.need((size_t)n_slots);
		launch_exact_all(sv, qv, q, ws.fb_keys.p, ws.fb_vals.p, st);
		size_t tb = 0;
		HIPCHK((hipError_t)sort_pairs(nullptr, tb, ws.fb_keys.p, ws.fb_keys2.p, ws.fb_vals.p, ws.fb_vals2.p, n_slots,
		                              st));
		ws.sort_tmp.need(tb);
		HIPCHK((hipError_t)sort_pairs(ws.sort_tmp.p, tb, ws.fb_keys.p, ws.fb_keys2.p, ws.fb_vals.p, ws.fb_vals2.p,
		                              n_slots, st));
		launch_copy_fallback(ws.fb_keys2.p, ws.fb_vals2.p, live_rows(), k, q, dL, dD, dC, st);
		HIPCHK(hipGetLastError());
	}
	if (enqueued) HIPCHK(hipStreamSynchronize(st));
}

// ---- asynchronous searches (lance_hip_search_batch_device_async) ----------
// A threshold-path pass (one pipeline pass, no filter / IVF / timing) is only
// enqueued; its certificate check and any reruns run at wait (or when a third
// search arrives, or before anything else touches the handle).  Two pass-buffer
// sets let pass i+1 be enqueued while pass i is still on the device.
int64_t Index::search_async(const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD,
                            int *dC) {
	const int64_t ticket = next_ticket++;
	if (ivf && !filter_on && !time_kernels && nq <= MAX_PASS_Q) {
		// IVF: the whole search enqueued on the handle's stream (its kernels run in
		// stream order behind the previous search's, which shares the workspace),
		// the end wait and the coarse flags' check at ivf_finish.  A search whose
		// shape differs from the pending ones' drains them first (its workspace
		// may grow: no buffer is reallocated under a search in flight).
		while (pending.size() >= 2) finish_oldest();
		if (!pending.empty()) {
			const PendingPass &b = pending.back();
			if (!b.ivf || b.nq != nq || b.k != k || b.nprobes != nprobes || b.refine != refine) drain();
		}
		for (auto &v : last_stats) v = 0;
		PendingPass p;
		p.slot = pb_free_slot();
		ivf_search(this, dQ, nq, k, nprobes, refine, dL, dD, dC, &p);
		if (!p.ivf) return ticket;  // (completed: more than one pass)
		PassBufs &P = pb[p.slot];
		if (!P.done) HIPCHK(hipEventCreateWithFlags(&P.done, hipEventDisableTiming));
		HIPCHK(hipEventRecord(P.done, stream));
		p.async = true;
		p.ticket = ticket;
		pending.push_back(p);
		return ticket;
	}
	const bool asyncable = !ivf && !filter_on && !time_kernels && nq <= MAX_PASS_Q && n_slots > 65536 &&
	                       !(small_exact && small_exact_fits(n_slots, dim, nq, k));
	if (!asyncable) {
		drain();
		search_any(dQ, nq, k, nprobes, refine, dL, dD, dC);
		return ticket;
	}
	while (pending.size() >= 2) finish_oldest();
	// a stale int8 copy / missing scan copy is rebuilt in place: not under pending
	// passes (only the copy this search will stream: enqueue_chunk's choice)
	if (!pending.empty()) {
		const bool use8 = scan_uses_i8(nq, k);
		if ((use8 && !(Xq && q8_ver == mut_ver && q8_cap == cap)) || (!use8 && has_scan_copy() && !Xs)) drain();
	}
	for (auto &v : last_stats) v = 0;
	PendingPass p;
	const int slot = pb_free_slot();
	if (!enqueue_chunk(dQ, nq, k, refine, dL, dD, dC, slot, true, p)) return ticket;  // (completed)
	p.async = true;
	p.st3 = last_stats[3];
	p.st5 = last_stats[5];
	p.ticket = ticket;
	pending.push_back(p);
	return ticket;
}

void Index::finish_oldest() {
	PendingPass p = pending.front();
	pending.pop_front();
	if (p.ivf)
		ivf_finish(this, p);
	else
		finish_chunk(p);
}

void Index::wait_ticket(int64_t ticket) {
	while (!spending.empty() && (ticket <= 0 || spending.front().ticket <= ticket)) shard_finish_oldest(this);
	while (!pending.empty() && (ticket <= 0 || pending.front().ticket <= ticket)) finish_oldest();
}

void Index::drain() {
	while (!spending.empty()) shard_finish_oldest(this);
	while (!pending.empty()) finish_oldest();
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
	if (ix->sharded() && ix->dim != d) {
		fclose(f);
		throw Error("table log dimension " + std::to_string(d) + " != handle dimension");
	}
	ix->dim = d;
	ix->ld = (int)round_up(d, DPAD);
	// the stores the records apply to: this handle, or (multi-device handle) its
	// shards, an ingest record going whole to the shard with the fewest slots as
	// at ingest time
	std::vector<Index *> all;
	if (ix->sharded())
		for (auto &sh : ix->shards) all.push_back(sh.get());
	else
		all.push_back(ix);
	Index *last_add = ix;
	std::vector<float> buf;
	for (;;) {
		uint8_t tag;
		if (fread(&tag, 1, 1, f) != 1) break;
		if (tag == 1) {
			int64_t first, num;
			if (fread(&first, 8, 1, f) != 1 || fread(&num, 8, 1, f) != 1) break;
			buf.resize((size_t)num * d);
			if (fread(buf.data(), sizeof(float), buf.size(), f) != buf.size()) break;  // torn tail: ignore
			Index *t = ix->sharded() ? shard_for_add(ix) : ix;
			// a label at or below an existing slot label can only follow a reopen
			// that reused labels of deleted rows: drop the tombstones first so the
			// slot -> label order stays strictly ascending
			if (t->n_slots > 0 && first <= t->slot_label.back()) t->compact();
			if (ix->sharded()) t->bind();
			t->next_label = first;
			t->add_host(buf.data(), num);
			ix->next_label = first + num;
			last_add = t;
		} else if (tag == 3) {
			uint8_t v;
			if (fread(&v, 1, 1, f) != 1) break;
			if (ix->sharded()) ix->xbf16 = v == 1;
			for (Index *t : all) t->set_storage(v == 1);
		} else if (tag == 2) {
			int64_t n;
			if (fread(&n, 8, 1, f) != 1) break;
			std::vector<int64_t> labs((size_t)n);
			if (fread(labs.data(), 8, (size_t)n, f) != (size_t)n) break;
			for (Index *t : all) {
				if (ix->sharded()) t->bind();
				t->remove(labs.data(), n);
			}
		} else if (tag == 4) {
			// IVF model (lance_detached_create_index): re-index the rows present
			// at that point of the log with the persisted centroids / codebook
			int32_t hdr[3];
			if (fread(hdr, 4, 3, f) != 3) break;
			const int type = hdr[0], nl = hdr[1], m = hdr[2];
			if (nl <= 0 || (type == IVF_PQ && (m <= 0 || d % m != 0))) break;
			std::vector<float> C((size_t)nl * d), cb;
			if (fread(C.data(), sizeof(float), C.size(), f) != C.size()) break;
			if (type == IVF_PQ) {
				cb.resize((size_t)m * PQ_K * (d / m));
				if (fread(cb.data(), sizeof(float), cb.size(), f) != cb.size()) break;
			}
			for (Index *t : all) {
				if (ix->sharded()) t->bind();
				ivf_set_model(t, type, nl, m, C.data(), type == IVF_PQ ? cb.data() : nullptr);
			}
		} else if (tag == 5) {
			for (Index *t : all) {
				if (ix->sharded()) t->bind();
				t->compact();
				ivf_optimize(t);
			}
		} else if (tag == 8) {
			// scalar index record: column, type (rebuilt over the rows present here)
			uint32_t a = 0, b = 0;
			if (fread(&a, 4, 1, f) != 1 || a > 4096) break;
			std::string col(a, '\0');
			if (fread(&col[0], 1, a, f) != a || fread(&b, 4, 1, f) != 1 || b > 64) break;
			std::string ty(b, '\0');
			if (fread(&ty[0], 1, b, f) != b) break;
			for (Index *t : all)
				if (t->meta)
					for (auto &c : t->meta->cols)
						if (c.name == col) c.build_index(ty);
		} else if (tag == 6 || tag == 7) {
			// multi-column table: metadata schema / the rows of the batch just replayed
			int64_t n;
			if (fread(&n, 8, 1, f) != 1 || n < 0) break;
			std::vector<uint8_t> b((size_t)n);
			if (fread(b.data(), 1, b.size(), f) != b.size()) break;
			if (tag == 6) {
				ix->meta = MetaStore::deserialize_schema(b.data(), b.size());
				if (ix->sharded())
					for (Index *t : all) t->meta = MetaStore::deserialize_schema(b.data(), b.size());
			} else if (last_add->meta) {
				// the tag-1 record before it filled these slots with NULLs
				MetaStore *mt = last_add->meta.get();
				const int64_t have = mt->cols.empty() ? 0 : (int64_t)mt->cols[0].size();
				int64_t nrec = 0;
				memcpy(&nrec, b.data(), std::min<size_t>(8, b.size()));
				mt->truncate((size_t)std::max<int64_t>(0, have - nrec));
				mt->deserialize_rows(b.data(), b.size());
			}
		} else {
			break;
		}
	}
	fclose(f);
	// rows added after the last create_index / optimize stay unindexed
	for (Index *t : all) {
		if (ix->sharded()) t->bind();
		t->compact();
	}
	// next_label = MAX(label)+1 over live rows, 0 when empty (lance_manager.rs:157-158, :662-696)
	int64_t mx = -1;
	for (Index *t : all)
		for (int64_t s = 0; s < t->n_slots; ++s)
			if (t->live[(size_t)s]) mx = std::max(mx, t->slot_label[(size_t)s]);
	ix->next_label = mx + 1;
	if (ix->sharded()) {
		shard_counts(ix);
		HIPCHK(hipSetDevice(ix->device));
	}
}

}  // namespace lhip

using lhip::Error;
using lhip::Index;

static Index *as_index(void *h) { return reinterpret_cast<Index *>(h); }

// the handle's device(s): LANCE_HIP_DEVICES lists two or more -> a multi-device
// handle (shards.cpp); one -> that device; unset -> the current device
static void init_devices(Index *ix) {
	ix->tie_desc = lhip::env_tie();
	const auto devs = lhip::env_devices();
	ix->init_device(devs.empty() ? -1 : devs[0]);
	if (devs.size() >= 2) lhip::shard_init(ix, devs);
}

// the device a device pointer lives on (-1 for host memory)
static int pointer_device(const void *p) {
	hipPointerAttribute_t a;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return -1;
	}
	return a.type == hipMemoryTypeDevice ? a.device : -1;
}
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
			init_devices(ix);
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
	try {
		// lance_manager.rs:62-126: dimension from the first FixedSizeList column,
		// every other field a metadata column; the schema stays caller-owned
		auto meta = lhip::MetaStore::from_schema(static_cast<const ArrowSchema *>(arrow_schema));
		auto ix = new Index();
		try {
			ix->db_path = cstr(db_path);
			ix->table = cstr(table_name);
			if (ix->table.empty()) ix->table = "vectors";
			ix->metric_name = cstr(metric);
			ix->metric = lhip::metric_id(ix->metric_name);
			ix->dim = meta->dim;
			ix->ld = (int)lhip::round_up(ix->dim, lhip::DPAD);
			ix->meta = std::move(meta);
			init_devices(ix);
			ix->log_open(true);
			ix->log_meta_schema();
		} catch (...) {
			delete ix;
			throw;
		}
		return ix;
	}
	API_GUARD("create_from_arrow failed: ", nullptr)
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
				char magic[8];
				int32_t d = 0;
				const bool ok = fread(magic, 1, 8, f) == 8 && fread(&d, 4, 1, f) == 1 && d > 0;
				fclose(f);
				if (!ok) throw Error("corrupt table log: " + ix->log_path());
				ix->dim = d;  // (a multi-device handle lays its shards out before the replay)
				ix->ld = (int)lhip::round_up(d, lhip::DPAD);
			}
			init_devices(ix);
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
	if (!handle) return 0;
	Index *ix = as_index(handle);
	return (ix->meta && !ix->meta->cols.empty()) ? 1 : 0;
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
		int64_t first = ix->sharded() ? lhip::shard_add(ix, vector, 1, -1, nullptr) : ix->add_host(vector, 1);
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
		int64_t first = ix->sharded() ? lhip::shard_add(ix, vectors, num, -1, nullptr) : ix->add_host(vectors, num);
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
	// lance_manager.rs:257: the callee takes the array over (its release runs
	// here, the caller's struct is left released); the schema stays borrowed
	ArrowArray *arr = static_cast<ArrowArray *>(arrow_array);
	struct Owned {
		ArrowArray a;
		~Owned() {
			if (a.release) a.release(&a);
		}
	} owned{*arr};
	arr->release = nullptr;
	try {
		Index *ix = as_index(handle);
		const ArrowSchema *sch = static_cast<const ArrowSchema *>(arrow_schema);
		std::lock_guard<std::mutex> g(ix->mu);
		std::unique_ptr<lhip::MetaStore> tmp;
		Index *tgt = ix->sharded() ? lhip::shard_for_add(ix) : ix;  // (the store that takes the batch)
		lhip::MetaStore *m = tgt->meta.get();
		if (!m) {  // a vector-only table: the batch may only carry the vector column
			tmp = lhip::MetaStore::from_schema(sch);
			if (!tmp->cols.empty()) throw Error("the table has no metadata columns");
			m = tmp.get();
		}
		if (m->dim != ix->dim)
			throw Error("expected dimension " + std::to_string(ix->dim) + ", got " + std::to_string(m->dim));
		std::vector<float> vecs;
		const int64_t n0 = tgt->n_slots;
		int64_t n;
		try {
			n = m->import_batch(sch, &owned.a, vecs);
		} catch (...) {
			m->truncate((size_t)n0);
			throw;
		}
		if (n == 0) return 0;
		if (!out_labels) {
			m->truncate((size_t)n0);
			throw Error("null buffer");
		}
		ix->bind();
		const int64_t first =
		    ix->sharded() ? lhip::shard_add(ix, vecs.data(), n, -1, nullptr, tgt) : ix->add_host(vecs.data(), n);
		ix->log_add(first, vecs.data(), n);
		ix->log_meta_rows(n0, n, tgt->meta.get());
		for (int64_t i = 0; i < n; ++i) out_labels[i] = first + i;
		return (int32_t)n;
	}
	API_GUARD("add_batch_arrow failed: ", -1)
}

// NEW — the predicate evaluator of filtered search on a host Arrow batch (no
// device, nothing taken over): mask[r] = live[r] && predicate TRUE for row r.
int64_t lance_hip_predicate_mask(void *arrow_schema, void *arrow_array, const int64_t *labels, const uint8_t *live,
                                 const char *predicate, const char *indexed_columns, uint8_t *out_mask, char *err_buf,
                                 int err_buf_len) {
	try {
		if (!arrow_schema || !arrow_array || !labels || !live || !out_mask) throw Error("null argument");
		const ArrowSchema *sch = static_cast<const ArrowSchema *>(arrow_schema);
		auto m = lhip::MetaStore::from_schema(sch);
		std::vector<float> vecs;
		const int64_t n = m->import_batch(sch, static_cast<const ArrowArray *>(arrow_array), vecs);
		// comma-separated columns to evaluate through a scalar index
		const std::string ic = cstr(indexed_columns);
		for (size_t a = 0; a < ic.size();) {
			size_t b = ic.find(',', a);
			if (b == std::string::npos) b = ic.size();
			const std::string name = ic.substr(a, b - a);
			bool found = false;
			for (auto &c : m->cols)
				if (c.name == name) {
					c.build_index("BTREE");
					found = true;
				}
			if (!found && !name.empty()) throw Error("no column named '" + name + "'");
			a = b + 1;
		}
		std::vector<int64_t> lab(labels, labels + n);
		std::vector<uint8_t> lv(live, live + n), mask;
		const int64_t c = lhip::eval_predicate(cstr(predicate), m.get(), lab, lv, mask);
		if (n > 0) memcpy(out_mask, mask.data(), (size_t)n);
		return c;
	}
	API_GUARD("predicate failed: ", -1)
}

// The call the reference's C++ already makes (lance_index.cpp:481-486) with no
// declaration or Rust export behind it: a scalar index on a
// metadata column, used by search predicates that compare the column with a
// literal.  index_type (case-insensitive): "BTREE" (default for NULL / "") or
// "BITMAP"; `label` is implicitly ordered (no-op).  0 or -1.
int32_t lance_detached_create_scalar_index(void *handle, const char *column, const char *index_type, char *err_buf,
                                           int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		std::string ty = cstr(index_type);
		for (auto &ch : ty) ch = (char)toupper((unsigned char)ch);
		if (ty.empty()) ty = "BTREE";
		if (ty != "BTREE" && ty != "BITMAP") throw Error("unsupported scalar index type '" + cstr(index_type) + "'");
		const std::string col = cstr(column);
		if (col == "label") return 0;
		std::vector<Index *> tg;
		if (ix->sharded())
			for (auto &sh : ix->shards) tg.push_back(sh.get());
		else
			tg.push_back(ix);
		for (Index *t : tg) {
			lhip::MetaColumn *mc = nullptr;
			if (t->meta)
				for (auto &c : t->meta->cols)
					if (c.name == col) mc = &c;
			if (!mc) throw Error("no column named '" + col + "'");
			mc->build_index(ty);
		}
		ix->log_scalar_index(col, ty);
		return 0;
	}
	API_GUARD("create_scalar_index failed: ", -1)
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
		if ((tg->sharded() || src->sharded()) && ((tg->meta && !tg->meta->cols.empty()) || (src->meta && !src->meta->cols.empty())))
			throw Error("merging multi-column tables of a multi-device handle is not supported");
		// rows of source selected by `label IN (...)`, in source (label) order
		std::vector<int64_t> want(live_source_labels, live_source_labels + live_count);
		std::sort(want.begin(), want.end());
		want.erase(std::unique(want.begin(), want.end()), want.end());
		std::vector<int64_t> olds, oslots;
		std::vector<float> vecs;
		{
			std::lock_guard<std::mutex> g(src->mu);
			src->bind();
			std::vector<float> row((size_t)src->dim);
			for (int64_t l : want) {
				int64_t s = -1;
				Index *from = src;
				if (src->sharded()) {
					from = lhip::shard_of_label(src, l, &s);
					if (!from) continue;
					from->bind();
				} else {
					s = src->slot_of(l);
					if (s < 0 || !src->live[(size_t)s]) continue;
				}
				from->read_rows(s, 1, row.data());
				vecs.insert(vecs.end(), row.begin(), row.end());
				olds.push_back(l);
				oslots.push_back(s);
			}
		}
		if (olds.empty()) return 0;
		std::lock_guard<std::mutex> g(tg->mu);
		tg->bind();
		const int64_t n0 = tg->n_slots;
		if (tg->meta && !tg->meta->cols.empty()) {  // the extra columns travel with the rows (lance_manager.rs:311-349)
			if (!src->meta) throw Error("merged indexes have different metadata columns");
			tg->meta->append_rows(*src->meta, oslots);
		}
		int64_t first = tg->sharded() ? lhip::shard_add(tg, vecs.data(), (int64_t)olds.size(), -1, nullptr)
		                              : tg->add_host(vecs.data(), (int64_t)olds.size());
		tg->log_add(first, vecs.data(), (int64_t)olds.size());
		tg->log_meta_rows(n0, (int64_t)olds.size());
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
		if (dim != ix->dim)
			throw Error("expected query dimension " + std::to_string(ix->dim) + ", got " + std::to_string(dim));
		if (nq < 0) throw Error("negative query count");
		if (nq == 0) return 0;
		if (!queries || !out_labels || !out_distances || !out_counts) throw Error("null buffer");
		std::lock_guard<std::mutex> g(ix->mu);
		if (ix->sharded()) {
			if (k <= 0) {
				for (int32_t i = 0; i < nq; ++i) out_counts[i] = 0;
				return nq;
			}
			lhip::shard_search(ix, queries, -1, nq, k, nprobes, refine_factor, predicate, out_labels, out_distances,
			                   out_counts, true);
			return nq;
		}
		// prefilter (lance_index.cpp:452-453 passes the optimizer's predicate,
		// lance_optimizer.cpp:555-584): slots whose predicate is TRUE
		lhip::FilterScope fs(ix, predicate);
		if (k <= 0 || ix->live_rows() == 0) {
			for (int32_t i = 0; i < nq; ++i) out_counts[i] = 0;
			for (int64_t i = 0; i < (int64_t)nq * std::max(k, 0); ++i) {
				out_labels[i] = -1;
				out_distances[i] = NAN;
			}
			return nq;
		}
		ix->bind();
		auto &ws = ix->ws;
		const size_t qb = (size_t)nq * dim * sizeof(float), lb = (size_t)nq * k * sizeof(int64_t);
		const size_t db = (size_t)nq * k * sizeof(float), cb = (size_t)nq * sizeof(int32_t);
		struct DeferSync {
			decltype(ix) p;
			~DeferSync() { p->defer_sync = false; }
		} defer{ix};
		if (nq <= 8) {
			// the lance_search() pattern (one query per call, lance_search.cpp:73-74):
			// no copies at all — the kernels read the query from, and write the
			// results into, pinned host memory (device-visible), one stream wait
			const size_t qb16 = (qb + 15) / 16 * 16;
			uint8_t *io = ws.need_host_io(qb16 + lb + db + cb);
			void *dio = nullptr;
			HIPCHK(hipHostGetDevicePointer(&dio, io, 0));
			uint8_t *d8 = static_cast<uint8_t *>(dio);
			memcpy(io, queries, qb);
			ix->defer_sync = true;
			ix->search_any(reinterpret_cast<const float *>(d8), nq, k, nprobes, refine_factor,
			               reinterpret_cast<int64_t *>(d8 + qb16), reinterpret_cast<float *>(d8 + qb16 + lb),
			               reinterpret_cast<int32_t *>(d8 + qb16 + lb + db));
			lhip::spin_sync(ix->stream);
			memcpy(out_labels, io + qb16, lb);
			memcpy(out_distances, io + qb16 + lb, db);
			memcpy(out_counts, io + qb16 + lb + db, cb);
			return nq;
		}
		ws.Qin.need((size_t)nq * dim);
		// pinned staging: true async copies on the handle's stream, one wait at
		// the end; the results [labels | distances | counts] are one device
		// block, read back by one copy
		ws.out_blk.need(lb + db + cb);
		int64_t *dL = reinterpret_cast<int64_t *>(ws.out_blk.p);
		float *dD = reinterpret_cast<float *>(ws.out_blk.p + lb);
		int32_t *dC = reinterpret_cast<int32_t *>(ws.out_blk.p + lb + db);
		uint8_t *io = ws.need_host_io(std::max(qb, lb + db + cb));
		memcpy(io, queries, qb);
		HIPCHK(hipMemcpyAsync(ws.Qin.p, io, qb, hipMemcpyHostToDevice, ix->stream));
		ix->defer_sync = true;  // the readback below waits for the search
		ix->search_any(ws.Qin.p, nq, k, nprobes, refine_factor, dL, dD, dC);
		HIPCHK(hipMemcpyAsync(io, ws.out_blk.p, lb + db + cb, hipMemcpyDeviceToHost, ix->stream));
		lhip::spin_sync(ix->stream);
		memcpy(out_labels, io, lb);
		memcpy(out_distances, io + lb, db);
		memcpy(out_counts, io + lb + db, cb);
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
	return ix->sharded() ? lhip::shard_live(ix) : ix->n_live;
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
		auto done = ix->sharded() ? lhip::shard_remove(ix, labels, count) : ix->remove(labels, count);
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
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();
		if (ix->sharded()) {
			lhip::shard_create_index(ix, ix->ivf_type_opt, num_partitions, num_sub_vectors);
			return 0;
		}
		lhip::ivf_build(ix, ix->ivf_type_opt, num_partitions, num_sub_vectors);
		ix->log_model();
		return 0;
	}
	API_GUARD("create_index failed: ", -1)
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
		if (ix->sharded()) {
			lhip::shard_compact(ix);
			if (ix->shards[0]->ivf) ix->log_optimize();
			return 0;
		}
		ix->compact();
		if (ix->ivf) {
			lhip::ivf_optimize(ix);  // optimize(All): unindexed rows join the partitions
			ix->log_optimize();
		}
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
		int64_t s = -1;
		Index *from = ix;
		if (ix->sharded()) {
			ix->bind();
			from = lhip::shard_of_label(ix, label, &s);
			if (!from) throw Error("label " + std::to_string(label) + " not found");
		} else {
			s = ix->slot_of(label);
			if (s < 0 || !ix->live[(size_t)s]) throw Error("label " + std::to_string(label) + " not found");
		}
		if (ix->dim > capacity) {
			lhip::write_err(err_buf, err_buf_len, "output buffer too small");
			return -1;
		}
		from->bind();
		from->read_rows(s, 1, out_vec);
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
		if (ix->sharded()) {
			const int64_t nl = lhip::shard_live(ix);
			if (out_count) *out_count = nl;
			if (out_labels && out_vectors && nl > 0) {
				std::vector<int64_t> labs;
				std::vector<float> vecs;
				lhip::shard_all_rows(ix, labs, vecs);
				memcpy(out_labels, labs.data(), labs.size() * sizeof(int64_t));
				memcpy(out_vectors, vecs.data(), vecs.size() * sizeof(float));
			}
			return (int32_t)nl;
		}
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

}  // extern "C"

// the options of one store (a single-device handle, or each shard of a
// multi-device one); throws on a bad key / value
static void set_option_store(Index *ix, const std::string &k, const std::string &v) {
	if (k == "s8_couple") {  // scan8 pair coupling lag in 32-row units (0 = off; results exact for any value)
		const int c = std::stoi(v);
		if (c < 0 || c > 4096) throw Error("s8_couple must be in [0, 4096]");
		ix->s8_couple = c;
		return;
	}
	if (k == "tie") {  // the final order's tie rule (label_desc reproduces the reference's tie golden)
		ix->tie_desc = lhip::parse_tie(v);
		return;
	}
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
		return;
	}
	if (k == "time_kernels") {
		ix->bind();
		ix->time_kernels = (v == "1" || v == "true");
		for (auto &e : ix->ev)
			if (!e) HIPCHK(hipEventCreate(&e));
		ix->kt_append_ms = ix->kt_dense_ms = 0.0;
		ix->kt_append_n = ix->kt_dense_n = 0;
		ix->kt_ivf_ms = ix->kt_ivf_bytes = ix->kt_ivf_pair_rows = ix->kt_ivf_coarse_ms = 0.0;
		ix->kt_ivf_n = 0;
		return;
	}
	if (k == "storage") {
		if (v != "f32" && v != "bf16") throw Error("storage must be 'f32' or 'bf16'");
		ix->bind();
		const bool was = ix->xbf16;
		ix->set_storage(v == "bf16");
		if (was != ix->xbf16) ix->log_storage();
		return;
	}
	if (k == "scan_copy") {
		if (v != "on" && v != "off") throw Error("scan_copy must be 'on' or 'off'");
		ix->bind();
		ix->set_scan_copy(v == "on");
		return;
	}
	if (k == "scan_i8") {
		if (v != "on" && v != "off") throw Error("scan_i8 must be 'on' or 'off'");
		ix->bind();
		ix->scan_i8 = v == "on";
		if (!ix->scan_i8) ix->drop_i8();
		return;
	}

	if (k == "prepare") {
		// build the derived scan structures now (the int8 scan copy) instead
		// of on the first search after a change
		ix->bind();
		if (ix->i8_usable()) ix->ensure_i8();
		return;
	}
	if (k == "pr_first") {  // this handle's first final-mode pool_refine chunk (results exact for any value)
		const int r = std::stoi(v);
		if (r != 0 && (r < 8 || r > lhip::pool_refine_max_first()))
			throw Error("pr_first must be 0 (default) or in [8, " + std::to_string(lhip::pool_refine_max_first()) + "]");
		ix->pr_first = r;
		return;
	}
	if (k == "scan8_variant") {  // this handle's ld = 768 scan8 geometry; release builds: 0 only
		const int r = std::stoi(v);
		if (!lhip::scan8_variant_ok(r))
			throw Error("scan8_variant " + v + " exists only in development (LHIP_ABLATION_BUILD) builds");
		ix->s8_variant = r;
		return;
	}
	if (k == "cand_extra_i8") {
		const int d = std::stoi(v);
		if (d != 0 && (d < 8 || d > 256)) throw Error("cand_extra_i8 must be 0 (auto) or in [8, 256]");
		ix->cand_extra_i8 = d;
		return;
	}
	if (k == "cand_extra") {
		const int d = std::stoi(v);
		if (d < 8 || d > 256) throw Error("cand_extra must be in [8, 256]");
		ix->cand_extra = d;
		return;
	}
	if (k == "small_exact") {
		ix->small_exact = (v == "1" || v == "on" || v == "true");
		return;
	}

	if (k == "retry_pass") {
		ix->retry_pass = (v == "1" || v == "on" || v == "true");
		return;
	}
	if (k == "split_div") {  // progressive threshold of the int8 append pass (0 or 1: one pass)
		const int d = std::stoi(v);
		if (d < 0 || d > 64) throw Error("split_div must be in [0, 64]");
		ix->split_div = d;
		return;
	}
	if (k == "sample_div") {
		const int d = std::stoi(v);
		if (d < 0) throw Error("sample_div must be >= 1, or 0 (auto)");
		ix->sample_div = d;
		return;
	}
	if (k == "index_type") {
		if (v == "ivf_pq" || v == "IVF_PQ")
			ix->ivf_type_opt = lhip::IVF_PQ;
		else if (v == "ivf_flat" || v == "IVF_FLAT")
			ix->ivf_type_opt = lhip::IVF_FLAT;
		else
			throw Error("index_type must be 'ivf_pq' or 'ivf_flat'");
		return;
	}
	if (k == "kmeans_iters") {
		const int it = std::stoi(v);
		if (it < 0) throw Error("kmeans_iters must be >= 0");
		ix->kmeans_iters = it;
		return;
	}
	if (k == "ivf_flat_scan") {
		bool b;
		if (v == "bound") b = true;
		else if (v == "exact") b = false;
		else throw Error("ivf_flat_scan must be 'bound' or 'exact'");
		ix->bind();
		// the bound scan's list-order rows are built with the layout
		if (b && !ix->ivf_flat_bound && ix->ivf) ix->ivf->dirty = true;
		ix->ivf_flat_bound = b;
		return;
	}
	if (k == "ivf_coarse") {  // (results identical either way)
		if (v == "fused") ix->ivf_coarse_fused = true;
		else if (v == "flat") ix->ivf_coarse_fused = false;
		else throw Error("ivf_coarse must be 'fused' or 'flat'");
		return;
	}
	if (k == "pq_lut") {  // (results identical either way; an A/B switch)
		if (v == "fused") ix->pq_lut_fused = true;
		else if (v == "split") ix->pq_lut_fused = false;
		else throw Error("pq_lut must be 'fused' or 'split'");
		return;
	}
	if (k == "pq_merge_bound") {  // (results identical either way; an A/B switch)
		if (v == "1") ix->pq_merge_bound = true;
		else if (v == "0") ix->pq_merge_bound = false;
		else throw Error("pq_merge_bound: 1 or 0");
		return;
	}
	if (k == "pq_seed") {
		if (v == "1") ix->pq_seed = true;
		else if (v == "0") ix->pq_seed = false;
		else throw Error("pq_seed: 1 or 0");
		return;
	}
	if (k == "pq_scan") {
		if (v == "fast") ix->pq_fast = true;
		else if (v == "exact_lut") ix->pq_fast = false;
		else throw Error("pq_scan must be 'fast' or 'exact_lut'");
		return;
	}
	if (k == "pq_query") {
		if (v == "fp8") ix->pq_fp8 = true;
		else if (v == "f32") ix->pq_fp8 = false;
		else throw Error("pq_query must be 'fp8' or 'f32'");
		return;
	}
	if (k == "ivf_seed") {
		ix->ivf_seed = std::stoull(v);
		return;
	}
	if (k == "reserve_rows") {
		ix->bind();
		ix->reserve(std::stoll(v));
		return;
	}
	throw Error("unknown option '" + k + "'");
}

extern "C" {

int32_t lance_hip_set_option(void *handle, const char *key, const char *value, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();  // every pending asynchronous search completes under the options it was enqueued with
		std::string k = cstr(key), v = cstr(value);
		if (k == "devices") {  // a multi-device handle over these devices (empty table only)
			lhip::shard_init(ix, lhip::parse_devices(v));
			return 0;
		}
		if (ix->sharded()) {
			// every shard takes the option; the handle keeps what its own log / new
			// shards need (storage), reserve_rows is split between the shards
			std::string fv = v;
			if (k == "reserve_rows")
				fv = std::to_string((std::stoll(v) + (int64_t)ix->shards.size() - 1) / (int64_t)ix->shards.size());
			for (auto &sh : ix->shards)
				if (lance_hip_set_option(sh.get(), key, fv.c_str(), err_buf, err_buf_len) != 0) return -1;
			if (k == "storage") {
				const bool was = ix->xbf16;
				ix->xbf16 = v == "bf16";
				if (was != ix->xbf16) ix->log_storage();
			}
			if (k == "index_type") ix->ivf_type_opt = ix->shards[0]->ivf_type_opt;
			return 0;
		}
		set_option_store(ix, k, v);
		// (replayed on each shard if the handle becomes multi-device later: shard_init)
		if (k != "prepare" && k != "time_kernels") ix->opt_log.emplace_back(k, v);
		return 0;
	}
	API_GUARD("set_option failed: ", -1)
}

int32_t lance_hip_last_search_stats(void *handle, int64_t *out, int32_t n) {
	if (!handle || !out) return -1;
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	for (int32_t i = 0; i < n && i < 6; ++i) out[i] = ix->last_stats[i];
	return 0;
}

// out[0] = total ms of threshold-scan launches, out[1] = their count,
// out[2] = rows scanned per launch, out[3] = padded queries per launch,
// out[4] = total ms of small-store dense scans, out[5] = their count,
// out[6] = bytes per element the scan streams (2: bf16 store or scan copy),
// out[7] = total ms of IVF list-scan launches, out[8] = their count,
// out[9] = their algorithmic bytes (summed), out[10] = (query, row) pairs
// they scored (summed), out[11] = total ms of the IVF coarse searches,
// out[12] = which kernel ran the last timed append pass: 0 scan_kernel, 2 scan8_kernel.
int32_t lance_hip_kernel_times(void *handle, double *out, int32_t n) {
	if (!handle || !out) return -1;
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	if (ix->sharded()) {  // times and counts summed over the shards, geometry of the first
		std::vector<double> acc(13, 0.0), one(13);
		for (size_t i = 0; i < ix->shards.size(); ++i) {
			lance_hip_kernel_times(ix->shards[i].get(), one.data(), 13);
			for (int j : {0, 1, 4, 5, 7, 8, 9, 10, 11}) acc[(size_t)j] += one[(size_t)j];
			if (i == 0)
				for (int j : {2, 3, 6, 12}) acc[(size_t)j] = one[(size_t)j];
		}
		for (int32_t i = 0; i < n && i < 13; ++i) out[i] = acc[(size_t)i];
		return 0;
	}
	double v[13] = {ix->kt_append_ms, (double)ix->kt_append_n, (double)ix->kt_append_rows,
		               (double)ix->kt_append_qpad, ix->kt_dense_ms, (double)ix->kt_dense_n,
		               ix->last_scan_esz ? (double)ix->last_scan_esz : (ix->xbf16 || ix->Xs) ? 2.0 : 4.0, ix->kt_ivf_ms,
		               (double)ix->kt_ivf_n,
		               ix->kt_ivf_bytes, ix->kt_ivf_pair_rows, ix->kt_ivf_coarse_ms,
		               (double)ix->kt_append_kernel};
	for (int32_t i = 0; i < n && i < 13; ++i) out[i] = v[i];
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
		int64_t first = ix->sharded() ? lhip::shard_add(ix, d_vectors, num, pointer_device(d_vectors), nullptr)
		                              : ix->add_device(d_vectors, num);
		if (ix->log) {
			std::vector<float> h((size_t)num * dim);
			HIPCHK(hipMemcpy(h.data(), d_vectors, h.size() * sizeof(float), hipMemcpyDefault));
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
		if (nq < 0) throw Error("negative query count");
		if (nq == 0) return 0;
		if (!d_queries || !d_out_labels || !d_out_distances || !d_out_counts) throw Error("null buffer");
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind();
		if (ix->sharded()) {  // queries and outputs on any device (the merge runs on the handle's first device)
			const int64_t t = lhip::shard_submit(ix, d_queries, pointer_device(d_queries), nq, k, nprobes,
			                                     refine_factor, d_out_labels, d_out_distances, d_out_counts, false,
			                                     pointer_device(d_out_labels));
			ix->wait_ticket(t);
			return nq;
		}
		if (ix->n_live == 0) {
			HIPCHK(hipMemsetAsync(d_out_counts, 0, (size_t)nq * sizeof(int32_t), ix->stream));
			HIPCHK(hipStreamSynchronize(ix->stream));
			return nq;
		}
		ix->search_any(d_queries, nq, k, nprobes, refine_factor, d_out_labels, d_out_distances, d_out_counts);
		return nq;
	}
	API_GUARD("search failed: ", -1)
}

int64_t lance_hip_search_batch_device_async(void *handle, const float *d_queries, int32_t nq, int32_t dim, int32_t k,
                                            int32_t nprobes, int32_t refine_factor, int64_t *d_out_labels,
                                            float *d_out_distances, int32_t *d_out_counts, char *err_buf,
                                            int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		if (dim != ix->dim)
			throw Error("expected query dimension " + std::to_string(ix->dim) + ", got " + std::to_string(dim));
		if (k <= 0) throw Error("k must be positive");
		if (nq < 0) throw Error("negative query count");
		if (nq > 0 && (!d_queries || !d_out_labels || !d_out_distances || !d_out_counts)) throw Error("null buffer");
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind_nodrain();
		if (nq == 0) return ix->next_ticket++;
		if (ix->sharded()) {
			// every shard's pass enqueued; certificates, peer copies and the merge at
			// the wait (two searches in flight: the shards scan the next batch
			// meanwhile).  Host queries complete here (their staging is reused).
			const int qdev = pointer_device(d_queries);
			const int64_t t = lhip::shard_submit(ix, d_queries, qdev, nq, k, nprobes, refine_factor, d_out_labels,
			                                     d_out_distances, d_out_counts, false, pointer_device(d_out_labels));
			if (qdev < 0) ix->wait_ticket(t);
			return t;
		}
		if (ix->n_live == 0) {
			ix->drain();
			HIPCHK(hipMemsetAsync(d_out_counts, 0, (size_t)nq * sizeof(int32_t), ix->stream));
			HIPCHK(hipStreamSynchronize(ix->stream));
			return ix->next_ticket++;
		}
		return ix->search_async(d_queries, nq, k, nprobes, refine_factor, d_out_labels, d_out_distances, d_out_counts);
	}
	API_GUARD("search failed: ", -1)
}

int32_t lance_hip_stream_after(void *handle, void *caller_stream, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		hipStream_t cs = static_cast<hipStream_t>(caller_stream);
		if (ix->sharded()) {  // (stores on several devices: a host wait on the caller's stream)
			HIPCHK(hipStreamSynchronize(cs));
			return 0;
		}
		ix->bind_nodrain();
		// an event on the caller's stream that the handle's stream waits on: every
		// later search of the handle (flat passes are ordered after the handle's
		// stream, IVF runs on it) starts after the caller's work so far, and the
		// host does not wait
		if (!ix->ev_caller) HIPCHK(hipEventCreateWithFlags(&ix->ev_caller, hipEventDisableTiming));
		HIPCHK(hipEventRecord(ix->ev_caller, cs));
		HIPCHK(hipStreamWaitEvent(ix->stream, ix->ev_caller, 0));
		return 0;
	}
	API_GUARD("stream_after failed: ", -1)
}

int32_t lance_hip_search_wait(void *handle, int64_t ticket, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		ix->bind_nodrain();
		ix->wait_ticket(ticket);
		return 0;
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
		lhip::launch_merge_topk(nshard, nq, k, pl, pd, pc, ol, od, oc, st, lhip::env_tie());
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
		// stream-ordered on the null stream, no host wait: a multi-rank pipeline's
		// exchange of batch i-1 must not hold the host until the scan of batch i
		// (which holds every CU) has finished (round 6: DESIGN section 7)
		lhip::launch_merge_topk(nshard, nq, k, d_part_labels, d_part_dists, d_part_counts, d_out_labels, d_out_dists,
		                        d_out_counts, nullptr, lhip::env_tie());
		HIPCHK(hipGetLastError());
		return nq;
	}
	API_GUARD("merge_topk failed: ", -1)
}

int64_t lance_hip_merge_packed_stride(int32_t nq, int32_t k) {
	if (nq <= 0 || k <= 0) return -1;
	const int64_t body = 3 * (int64_t)nq * k + nq;  // labels (2 words each), dists, counts
	return (body + 1) / 2 * 2 + 2;                  // even, then the label offset
}

int32_t lance_hip_merge_topk_packed(int32_t nshard, int32_t nq, int32_t k, const int32_t *d_gathered,
                                    int64_t row_stride, int64_t *d_out_labels, float *d_out_dists,
                                    int32_t *d_out_counts, char *err_buf, int err_buf_len) {
	try {
		if (nshard <= 0 || nq <= 0 || k <= 0) return 0;
		if (!d_gathered || !d_out_labels || !d_out_dists || !d_out_counts) throw std::invalid_argument("null buffer");
		if (row_stride < lance_hip_merge_packed_stride(nq, k) || (row_stride & 1) ||
		    (reinterpret_cast<uintptr_t>(d_gathered) & 7))
			throw std::invalid_argument("row_stride must be even and >= lance_hip_merge_packed_stride(nq, k), "
			                            "the gathered buffer 8-byte aligned");
		// stream-ordered on the null stream like lance_hip_merge_topk_device
		lhip::launch_merge_packed(nshard, nq, k, d_gathered, row_stride, d_out_labels, d_out_dists, d_out_counts,
		                          nullptr, lhip::env_tie());
		HIPCHK(hipGetLastError());
		return nq;
	}
	API_GUARD("merge_topk failed: ", -1)
}

// ---- IVF model / layout (multi-GPU model broadcast, parity tests) ----------

int32_t lance_hip_ivf_info(void *handle, int64_t *out, int32_t n) {
	if (!handle || !out) return -1;
	Index *ix = as_index(handle);
	std::lock_guard<std::mutex> g(ix->mu);
	int64_t v[6] = {-1, 0, 0, 0, 0, ix->n_slots};
	if (ix->sharded()) {  // the shards share one model; rows indexed and slots summed
		lance_hip_ivf_info(ix->shards[0].get(), v, 6);
		v[4] = v[5] = 0;
		for (auto &sh : ix->shards) {
			v[4] += sh->ivf ? sh->ivf->n_indexed : 0;
			v[5] += sh->n_slots;
		}
	} else if (ix->ivf) {
		v[0] = ix->ivf->type;
		v[1] = ix->ivf->nlist;
		v[2] = ix->ivf->m;
		v[3] = ix->ivf->dsub;
		v[4] = ix->ivf->n_indexed;
	}
	for (int32_t i = 0; i < n && i < 6; ++i) out[i] = v[i];
	return 0;
}

int32_t lance_hip_ivf_export(void *handle, float *centroids, float *codebook, int64_t *slot_labels,
                             uint8_t *slot_live, int32_t *slot_list, uint8_t *slot_codes, char *err_buf,
                             int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (ix->sharded()) throw Error("ivf_export: export a multi-device handle's shards one by one");
		if (!ix->ivf) throw Error("no IVF index");
		ix->bind();
		lhip::ivf_export_model(ix, centroids, codebook);
		lhip::ivf_export_slots(ix, slot_list, slot_codes);
		for (int64_t s = 0; s < ix->n_slots; ++s) {
			if (slot_labels) slot_labels[s] = ix->slot_label[(size_t)s];
			if (slot_live) slot_live[s] = ix->live[(size_t)s];
		}
		return 0;
	}
	API_GUARD("ivf_export failed: ", -1)
}

int32_t lance_hip_ivf_set_model(void *handle, int32_t index_type, int32_t num_partitions, int32_t num_sub_vectors,
                                const float *centroids, const float *codebook, char *err_buf, int err_buf_len) {
	if (!handle) {
		lhip::write_err(err_buf, err_buf_len, "null handle");
		return -1;
	}
	try {
		Index *ix = as_index(handle);
		std::lock_guard<std::mutex> g(ix->mu);
		if (index_type != lhip::IVF_FLAT && index_type != lhip::IVF_PQ) throw Error("index_type must be 0 or 1");
		if (!centroids) throw Error("null centroids");
		ix->bind();
		if (ix->sharded()) {
			for (auto &sh : ix->shards) {
				sh->bind();
				lhip::ivf_set_model(sh.get(), index_type, num_partitions, num_sub_vectors, centroids, codebook);
			}
			ix->log_model(ix->shards[0].get());
			return 0;
		}
		lhip::ivf_set_model(ix, index_type, num_partitions, num_sub_vectors, centroids, codebook);
		ix->log_model();
		return 0;
	}
	API_GUARD("ivf_set_model failed: ", -1)
}

}  // extern "C"
