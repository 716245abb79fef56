// Multi-device handles: one LANCE index row-sharded over several HIP devices
// inside ONE process (SURVEY.md §2 comm-backend row "one process + 8 HIP
// devices", §5 Config row "device-count/shard option in the new lib"), so a
// DuckDB process that calls lance_detached_search per query
// (lance_search.cpp:73-74 -> lance_index.cpp:452-453) uses every GPU of the
// node without any change on its side.
//
// The handle keeps what the reference's LanceIndex keeps host-side (dense
// labels from next_label, lance_manager.rs:227-242; the table log); each shard
// is an Index of its own (device store, streams, workspace) on one device.
// Ingest batches go whole to the shard with the fewest slots (DuckDB appends
// chunks of <= 2048 rows, so the shards stay balanced within a chunk) and keep
// their global labels, so a shard's search returns global labels directly.  A
// search runs on every shard (enqueued on all of them before the first wait:
// the shards scan concurrently), the per-shard top-k lists (nq * k * 12 bytes
// each) are copied to the first device (hipMemcpyPeerAsync over xGMI) and
// merged there by merge_topk_kernel under the (distance, label) order — the
// same lists a single-device search returns.
#include "index.h"
#include "ivf.h"
#include "../../include/lancedb_hip.h"

#include <cmath>
#include <cstdlib>

namespace lhip {

std::vector<int> parse_devices(const std::string &spec) {
	std::vector<int> d;
	size_t a = 0;
	while (a < spec.size()) {
		size_t b = spec.find(',', a);
		if (b == std::string::npos) b = spec.size();
		const std::string t = spec.substr(a, b - a);
		if (!t.empty()) {
			char *end = nullptr;
			const long v = std::strtol(t.c_str(), &end, 10);
			if (!end || *end != 0 || v < 0 || v > 1024) throw Error("devices: bad device id '" + t + "'");
			d.push_back((int)v);
		}
		a = b + 1;
	}
	return d;
}

// LANCE_HIP_DEVICES=0,1,... (a DuckDB process has no per-call option channel:
// CREATE INDEX options stop at metric / nprobes / refine_factor,
// lance_index.cpp:157-165); unset or a single device: a single-device handle
std::vector<int> env_devices() {
	const char *e = std::getenv("LANCE_HIP_DEVICES");
	if (!e || !*e) return {};
	return parse_devices(e);
}

int parse_tie(const std::string &v) {
	if (v == "label_desc" || v == "desc") return 1;
	if (v == "label_asc" || v == "asc") return 0;
	throw Error("tie must be 'label_desc' or 'label_asc', got '" + v + "'");
}

// LANCE_HIP_TIE=label_asc|label_desc (unset: label_desc), read when a handle
// is created (the same channel as LANCE_HIP_DEVICES)
int env_tie() {
	const char *e = std::getenv("LANCE_HIP_TIE");
	if (!e || !*e) return 1;
	return parse_tie(e);
}

void shard_init(Index *ix, const std::vector<int> &devs) {
	if (ix->sharded()) throw Error("the handle is already sharded");
	if (ix->n_slots > 0) throw Error("devices can only be set on an empty table");
	if (devs.size() < 2) throw Error("devices: list at least two devices");
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) throw Error("no HIP device available");
	for (int d : devs)
		if (d >= n) throw Error("HIP device " + std::to_string(d) + " out of range (" + std::to_string(n) + " visible)");
	std::vector<uint8_t> schema;
	if (ix->meta) ix->meta->serialize_schema(schema);
	for (int d : devs) {
		auto sh = std::make_unique<Index>();
		sh->table = ix->table;
		sh->metric_name = ix->metric_name;
		sh->metric = ix->metric;
		sh->dim = ix->dim;
		sh->ld = ix->ld;
		sh->xbf16 = ix->xbf16;
		sh->tie_desc = ix->tie_desc;
		if (ix->meta) sh->meta = MetaStore::deserialize_schema(schema.data(), schema.size());
		sh->init_device(d);
		ix->shards.push_back(std::move(sh));
	}
	// peer access between the distinct devices (the partial lists travel over
	// xGMI to the first device; without it hipMemcpyPeer stages through the host)
	for (int a : devs)
		for (int b : devs)
			if (a != b) {
				int can = 0;
				if (hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can) {
					HIPCHK(hipSetDevice(a));
					const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
					if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
					(void)hipGetLastError();
				}
			}
	// the handle's own stream (the merge stream) and stats on the first device
	if (ix->device != devs[0]) {
		HIPCHK(hipSetDevice(ix->device));
		if (ix->stream) {
			HIPCHK(hipStreamSynchronize(ix->stream));
			HIPCHK(hipStreamDestroy(ix->stream));
			ix->stream = nullptr;
		}
		ix->stats.release();
		ix->init_device(devs[0]);
	}
	HIPCHK(hipSetDevice(ix->device));
	// options set before `devices`: every shard takes them (reserve_rows split)
	for (const auto &kv : ix->opt_log) {
		std::string v = kv.second;
		if (kv.first == "reserve_rows")
			v = std::to_string((std::stoll(v) + (int64_t)devs.size() - 1) / (int64_t)devs.size());
		char err[512];
		for (auto &sh : ix->shards)
			if (lance_hip_set_option(sh.get(), kv.first.c_str(), v.c_str(), err, (int)sizeof(err)) != 0)
				throw Error(std::string("devices: replaying option ") + kv.first + ": " + err);
		if (kv.first == "index_type") ix->ivf_type_opt = ix->shards[0]->ivf_type_opt;
	}
}

Index *shard_for_add(Index *ix) {
	Index *best = nullptr;
	for (auto &s : ix->shards)
		if (!best || s->n_slots < best->n_slots) best = s.get();
	return best;
}

int64_t shard_live(const Index *ix) {
	int64_t n = 0;
	for (auto &s : ix->shards) n += s->n_live;
	return n;
}

// labels [next_label, next_label + num) to one shard; v on the host, or on
// device `vdev` (>= 0)
int64_t shard_add(Index *ix, const float *v, int64_t num, int vdev, Index **into, Index *force) {
	Index *t = force ? force : shard_for_add(ix);
	t->bind();
	t->next_label = ix->next_label;
	int64_t first;
	if (vdev < 0) {
		first = t->add_host(v, num);
	} else if (vdev == t->device) {
		first = t->add_device(v, num);
	} else {
		DevBuf<float> tmp;
		tmp.need((size_t)num * ix->dim);
		HIPCHK(hipMemcpyPeerAsync(tmp.p, t->device, v, vdev, (size_t)num * ix->dim * sizeof(float), t->stream));
		first = t->add_device(tmp.p, num);
	}
	ix->next_label = first + num;
	ix->n_live += num;
	ix->n_slots += num;
	if (into) *into = t;
	return first;
}

std::vector<int64_t> shard_remove(Index *ix, const int64_t *labels, int64_t n) {
	std::vector<int64_t> done;
	for (auto &s : ix->shards) {
		s->bind();
		auto d = s->remove(labels, n);
		done.insert(done.end(), d.begin(), d.end());
	}
	std::sort(done.begin(), done.end());
	ix->n_live -= (int64_t)done.size();
	return done;
}

// Sharded search, asynchronous: shard_submit enqueues every shard's pass (its
// own pass streams; nothing waits), shard_finish_oldest completes the oldest
// submitted search — per shard the certificate check / reruns / fallback
// (host, Index::wait_ticket), the B*k partial lists copied to the first device
// on the shard's stream and an event the merge stream waits on (no host wait
// per shard), then ONE merge on the first device.  Two searches may be in
// flight (per-slot query / list buffers on every shard): the shards scan batch
// i+1 while batch i's lists are checked, copied and merged.
// Q: nq x dim f32 on the host (qdev < 0) or on device qdev; outputs on the
// host (out_host), on device odev, or (odev < 0, not out_host) anywhere the
// first device can write through hipMemcpy.
int64_t shard_submit(Index *ix, const float *Q, int qdev, int nq, int k, int nprobes, int refine, int64_t *L,
                     float *D, int *C, bool out_host, int odev) {
	while (ix->spending.size() >= 2) shard_finish_oldest(ix);
	const int S = (int)ix->shards.size();
	const int dim = ix->dim;
	int slot = 0;
	for (const auto &p : ix->spending)
		if (p.slot == slot) slot = 1;
	ShardPending p;
	p.ticket = ix->next_ticket++;
	p.slot = slot;
	p.nq = nq;
	p.k = k;
	p.odev = odev;
	p.out_host = out_host;
	p.L = L;
	p.D = D;
	p.C = C;
	p.st.assign((size_t)S, 0);
	p.empty.assign((size_t)S, 0);
	const size_t qb = (size_t)nq * dim * sizeof(float), lb = (size_t)nq * k * sizeof(int64_t);
	const size_t db = (size_t)nq * k * sizeof(float), cb = (size_t)nq * sizeof(int);
	for (int s = 0; s < S; ++s) {
		Index *t = ix->shards[(size_t)s].get();
		t->bind_nodrain();
		if (t->live_rows() == 0) {
			p.empty[(size_t)s] = 1;
			continue;
		}
		t->sh_q[slot].need((size_t)nq * dim);
		t->sh_out[slot].need(lb + db + cb);
		if (qdev < 0) {
			// (host queries come from the synchronous wrappers only: the staging
			// buffer is not reused before this search completes)
			uint8_t *io = t->ws.need_host_io(qb);
			memcpy(io, Q, qb);
			HIPCHK(hipMemcpyAsync(t->sh_q[slot].p, io, qb, hipMemcpyHostToDevice, t->stream));
		} else {
			HIPCHK(hipMemcpyPeerAsync(t->sh_q[slot].p, t->device, Q, qdev, qb, t->stream));
		}
		uint8_t *o = t->sh_out[slot].p;
		p.st[(size_t)s] = t->search_async(t->sh_q[slot].p, nq, k, nprobes, refine, reinterpret_cast<int64_t *>(o),
		                                  reinterpret_cast<float *>(o + lb), reinterpret_cast<int *>(o + lb + db));
	}
	ix->spending.push_back(std::move(p));
	return ix->spending.back().ticket;
}

void shard_finish_oldest(Index *ix) {
	ShardPending p = std::move(ix->spending.front());
	ix->spending.pop_front();
	const int S = (int)ix->shards.size(), nq = p.nq, k = p.k, sl = p.slot;
	const size_t lb = (size_t)nq * k * sizeof(int64_t), db = (size_t)nq * k * sizeof(float), cb = (size_t)nq * sizeof(int);
	HIPCHK(hipSetDevice(ix->device));
	ix->m_pl[sl].need((size_t)S * nq * k);
	ix->m_pd[sl].need((size_t)S * nq * k);
	ix->m_pc[sl].need((size_t)S * nq);
	const hipStream_t ms = ix->stream;  // the merge stream (first device)
	for (auto &v : ix->last_stats) v = 0;
	for (int s = 0; s < S; ++s) {
		Index *t = ix->shards[(size_t)s].get();
		const size_t o = (size_t)s * nq * k;
		if (p.empty[(size_t)s]) {
			HIPCHK(hipSetDevice(ix->device));
			HIPCHK(hipMemsetAsync(ix->m_pc[sl].p + (size_t)s * nq, 0, cb, ms));
			continue;
		}
		t->bind_nodrain();
		t->wait_ticket(p.st[(size_t)s]);  // certificates, reruns, exact fallback of this shard's pass
		// statistics of the search: summed over the shards that searched (max pool: the largest)
		for (int i : {0, 1, 4, 5}) ix->last_stats[i] += t->last_stats[i];
		ix->last_stats[2] = std::max(ix->last_stats[2], t->last_stats[2]);
		ix->last_stats[3] = std::max(ix->last_stats[3], t->last_stats[3]);
		const uint8_t *src = t->sh_out[sl].p;
		HIPCHK(hipMemcpyPeerAsync(ix->m_pl[sl].p + o, ix->device, src, t->device, lb, t->stream));
		HIPCHK(hipMemcpyPeerAsync(ix->m_pd[sl].p + o, ix->device, src + lb, t->device, db, t->stream));
		HIPCHK(hipMemcpyPeerAsync(ix->m_pc[sl].p + (size_t)s * nq, ix->device, src + lb + db, t->device, cb,
		                          t->stream));
		if (!t->sh_ev[sl]) HIPCHK(hipEventCreateWithFlags(&t->sh_ev[sl], hipEventDisableTiming));
		HIPCHK(hipEventRecord(t->sh_ev[sl], t->stream));
		HIPCHK(hipSetDevice(ix->device));
		HIPCHK(hipStreamWaitEvent(ms, t->sh_ev[sl], 0));
	}
	// merge on the first device: straight into the outputs when they live there,
	// else into m_out and one copy to wherever they are (host, another device)
	HIPCHK(hipSetDevice(ix->device));
	const bool direct = !p.out_host && p.odev == ix->device;
	int64_t *oL = p.L;
	float *oD = p.D;
	int *oC = p.C;
	if (!direct) {
		ix->m_out[sl].need(lb + db + cb);
		oL = reinterpret_cast<int64_t *>(ix->m_out[sl].p);
		oD = reinterpret_cast<float *>(ix->m_out[sl].p + lb);
		oC = reinterpret_cast<int *>(ix->m_out[sl].p + lb + db);
	}
	launch_merge_topk(S, nq, k, ix->m_pl[sl].p, ix->m_pd[sl].p, ix->m_pc[sl].p, oL, oD, oC, ms, ix->tie_desc);
	HIPCHK(hipGetLastError());
	if (p.out_host) {
		uint8_t *io = ix->shards[0]->ws.need_host_io(lb + db + cb);
		HIPCHK(hipMemcpyAsync(io, ix->m_out[sl].p, lb + db + cb, hipMemcpyDeviceToHost, ms));
		spin_sync(ms);
		memcpy(p.L, io, lb);
		memcpy(p.D, io + lb, db);
		memcpy(p.C, io + lb + db, cb);
	} else {
		if (!direct) {
			HIPCHK(hipMemcpyAsync(p.L, oL, lb, hipMemcpyDefault, ms));
			HIPCHK(hipMemcpyAsync(p.D, oD, db, hipMemcpyDefault, ms));
			HIPCHK(hipMemcpyAsync(p.C, oC, cb, hipMemcpyDefault, ms));
		}
		spin_sync(ms);
	}
}

// Synchronous sharded search (the host-buffer entry points, predicates): the
// predicate's mask per shard (FilterScope) for the duration of the search.
void shard_search(Index *ix, const float *Q, int qdev, int nq, int k, int nprobes, int refine, const char *pred,
                  int64_t *L, float *D, int *C, bool out_host) {
	ix->drain();
	std::vector<std::unique_ptr<FilterScope>> fs;
	for (auto &sh : ix->shards) fs.emplace_back(new FilterScope(sh.get(), pred));
	const int64_t t = shard_submit(ix, Q, qdev, nq, k, nprobes, refine, L, D, C, out_host, out_host ? -1 : ix->device);
	ix->wait_ticket(t);
}

// this handle's live / slot counts from its shards (after compaction, replay)
void shard_counts(Index *ix) {
	ix->n_live = 0;
	ix->n_slots = 0;
	for (auto &s : ix->shards) {
		ix->n_live += s->n_live;
		ix->n_slots += s->n_slots;
	}
}

// the shard whose live rows hold `label` (or null)
Index *shard_of_label(Index *ix, int64_t label, int64_t *slot) {
	for (auto &s : ix->shards) {
		const int64_t sl = s->slot_of(label);
		if (sl >= 0 && s->live[(size_t)sl]) {
			if (slot) *slot = sl;
			return s.get();
		}
	}
	return nullptr;
}

// every live row in ascending label order
void shard_all_rows(Index *ix, std::vector<int64_t> &labels, std::vector<float> &vecs) {
	std::vector<std::pair<int64_t, std::pair<Index *, int64_t>>> at;
	for (auto &s : ix->shards)
		for (int64_t sl = 0; sl < s->n_slots; ++sl)
			if (s->live[(size_t)sl]) at.push_back({s->slot_label[(size_t)sl], {s.get(), sl}});
	std::sort(at.begin(), at.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
	labels.resize(at.size());
	vecs.resize(at.size() * (size_t)ix->dim);
	std::vector<std::vector<float>> rows(ix->shards.size());
	for (size_t i = 0; i < ix->shards.size(); ++i) {
		Index *s = ix->shards[i].get();
		s->bind();
		rows[i].resize((size_t)s->n_slots * ix->dim);
		s->read_rows(0, s->n_slots, rows[i].data());
	}
	for (size_t j = 0; j < at.size(); ++j) {
		labels[j] = at[j].first;
		size_t si = 0;
		while (ix->shards[si].get() != at[j].second.first) ++si;
		memcpy(vecs.data() + j * ix->dim, rows[si].data() + (size_t)at[j].second.second * ix->dim,
		       (size_t)ix->dim * sizeof(float));
	}
}

void shard_compact(Index *ix) {
	for (auto &s : ix->shards) {
		s->bind();
		s->compact();
		if (s->ivf) ivf_optimize(s.get());
	}
	shard_counts(ix);
}

// IVF: one model for the whole table, installed on every shard (each indexes
// its own rows with the same centroids / codebook, as the multi-process path
// does, lance_hip_ivf_set_model).  nlist / m defaults and the size checks come
// from the TABLE's live count, so a handle gets the model a single store of the
// same rows would (ivf_build's rules: sqrt(live) lists, dim / 16 sub-vectors).
// Training runs on the shard with the most live rows when it holds the sample
// ivf_build would draw (min(live, 256 nlist) rows: the shards hold whole
// ingest batches, so that is a sample of the table); otherwise on a temporary
// store on the first device holding that many live rows drawn evenly from
// every shard.
void shard_create_index(Index *ix, int type, int num_partitions, int num_sub_vectors) {
	const int64_t total = shard_live(ix);
	if (total <= 0) throw Error("cannot build an index on an empty table");
	const int dim = ix->dim;
	const int nlist = num_partitions > 0 ? num_partitions : std::max(1, (int)std::sqrt((double)total));
	const int m = num_sub_vectors > 0 ? num_sub_vectors : (dim % 16 == 0 ? dim / 16 : dim % 8 == 0 ? dim / 8 : 1);
	if (nlist > total)
		throw Error("KMeans: cannot train " + std::to_string(nlist) + " centroids with " + std::to_string(total) +
		            " vectors");
	if (type == IVF_PQ && total < PQ_K)
		throw Error("PQ training needs at least 256 rows, the table has " + std::to_string(total));
	Index *tr = nullptr;
	for (auto &s : ix->shards)
		if (!tr || s->n_live > tr->n_live) tr = s.get();
	const int64_t want = std::min<int64_t>(total, (int64_t)nlist * 256);
	std::unique_ptr<Index> tmp;
	if (tr->n_live < want) {
		tmp = std::make_unique<Index>();
		tmp->table = "ivf_train";
		tmp->metric_name = ix->metric_name;
		tmp->metric = ix->metric;
		tmp->dim = dim;
		tmp->ld = ix->ld;
		tmp->init_device(ix->device);
		tmp->reserve(want + (int64_t)ix->shards.size());
		for (auto &sp : ix->shards) {
			Index *s = sp.get();
			if (s->n_live == 0) continue;
			// this shard's share, every (n_live / quota)-th live slot
			const int64_t quota = std::min<int64_t>(s->n_live, (want * s->n_live + total - 1) / total);
			std::vector<float> rows((size_t)quota * dim), chunk;
			int64_t got = 0, c = 0;
			constexpr int64_t CH = 65536;
			s->bind();
			for (int64_t s0 = 0; s0 < s->n_slots && got < quota; s0 += CH) {
				const int64_t n = std::min<int64_t>(CH, s->n_slots - s0);
				chunk.resize((size_t)n * dim);
				s->read_rows(s0, n, chunk.data());
				for (int64_t i = 0; i < n && got < quota; ++i) {
					if (!s->live[(size_t)(s0 + i)]) continue;
					if ((c * quota) / s->n_live != ((c + 1) * quota) / s->n_live)
						memcpy(rows.data() + (size_t)got++ * dim, chunk.data() + (size_t)i * dim, (size_t)dim * sizeof(float));
					++c;
				}
			}
			tmp->bind();
			if (got > 0) tmp->add_host(rows.data(), got);
		}
		tr = tmp.get();
	}
	tr->bind();
	tr->ivf_type_opt = type;
	tr->kmeans_iters = ix->shards[0]->kmeans_iters;
	tr->ivf_seed = ix->shards[0]->ivf_seed;
	ivf_build(tr, type, nlist, m);
	const int nl = tr->ivf->nlist, mm = tr->ivf->m;
	std::vector<float> C((size_t)nl * dim), cb;
	if (type == IVF_PQ) cb.resize((size_t)mm * PQ_K * (dim / mm));
	ivf_export_model(tr, C.data(), cb.empty() ? nullptr : cb.data());
	for (auto &s : ix->shards) {
		if (s.get() == tr) continue;
		s->bind();
		ivf_set_model(s.get(), type, nl, mm, C.data(), cb.empty() ? nullptr : cb.data());
	}
	ix->log_model(tr);
}

}  // namespace lhip
