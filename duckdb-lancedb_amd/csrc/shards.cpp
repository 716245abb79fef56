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
	ix->device = devs[0];
	HIPCHK(hipSetDevice(ix->device));
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

// Sharded search.  Q: nq x dim f32 on the host (qdev < 0) or on device qdev;
// outputs on the host (out_host) or on the first shard's device.
void shard_search(Index *ix, const float *Q, int qdev, int nq, int k, int nprobes, int refine, const char *pred,
                  int64_t *L, float *D, int *C, bool out_host) {
	const int S = (int)ix->shards.size();
	const int dim = ix->dim;
	std::vector<std::unique_ptr<FilterScope>> fs;
	for (auto &sh : ix->shards) fs.emplace_back(new FilterScope(sh.get(), pred));
	Index *p0 = ix->shards[0].get();
	const size_t qb = (size_t)nq * dim * sizeof(float), lb = (size_t)nq * k * sizeof(int64_t);
	const size_t db = (size_t)nq * k * sizeof(float), cb = (size_t)nq * sizeof(int);
	HIPCHK(hipSetDevice(p0->device));
	ix->m_pl.need((size_t)S * nq * k);
	ix->m_pd.need((size_t)S * nq * k);
	ix->m_pc.need((size_t)S * nq);
	std::vector<int64_t> ticket((size_t)S, 0);
	std::vector<char> empty((size_t)S, 0);
	// 1) every shard's search enqueued (asynchronous passes) before any wait
	for (int s = 0; s < S; ++s) {
		Index *t = ix->shards[(size_t)s].get();
		t->bind();
		if (t->live_rows() == 0) {
			empty[(size_t)s] = 1;
			continue;
		}
		t->ws.Qin.need((size_t)nq * dim);
		t->ws.out_blk.need(lb + db + cb);
		if (qdev < 0) {
			uint8_t *io = t->ws.need_host_io(qb);
			memcpy(io, Q, qb);
			HIPCHK(hipMemcpyAsync(t->ws.Qin.p, io, qb, hipMemcpyHostToDevice, t->stream));
		} else {
			HIPCHK(hipMemcpyPeerAsync(t->ws.Qin.p, t->device, Q, qdev, qb, t->stream));
		}
		int64_t *dL = reinterpret_cast<int64_t *>(t->ws.out_blk.p);
		float *dD = reinterpret_cast<float *>(t->ws.out_blk.p + lb);
		int *dC = reinterpret_cast<int *>(t->ws.out_blk.p + lb + db);
		ticket[(size_t)s] = t->search_async(t->ws.Qin.p, nq, k, nprobes, refine, dL, dD, dC);
	}
	// 2) completions (certificates, reruns, fallbacks) and the partial lists to
	//    the first device
	for (int s = 0; s < S; ++s) {
		Index *t = ix->shards[(size_t)s].get();
		const size_t o = (size_t)s * nq * k;
		if (empty[(size_t)s]) {
			HIPCHK(hipSetDevice(p0->device));
			HIPCHK(hipMemsetAsync(ix->m_pc.p + (size_t)s * nq, 0, cb, p0->stream));
			continue;
		}
		t->bind_nodrain();
		t->wait_ticket(ticket[(size_t)s]);
		HIPCHK(hipMemcpyPeerAsync(ix->m_pl.p + o, p0->device, t->ws.out_blk.p, t->device, lb, t->stream));
		HIPCHK(hipMemcpyPeerAsync(ix->m_pd.p + o, p0->device, t->ws.out_blk.p + lb, t->device, db, t->stream));
		HIPCHK(hipMemcpyPeerAsync(ix->m_pc.p + (size_t)s * nq, p0->device, t->ws.out_blk.p + lb + db, t->device, cb,
		                          t->stream));
		HIPCHK(hipStreamSynchronize(t->stream));
	}
	// 3) merge on the first device
	HIPCHK(hipSetDevice(p0->device));
	int64_t *oL = L;
	float *oD = D;
	int *oC = C;
	if (out_host) {
		ix->m_out.need(lb + db + cb);
		oL = reinterpret_cast<int64_t *>(ix->m_out.p);
		oD = reinterpret_cast<float *>(ix->m_out.p + lb);
		oC = reinterpret_cast<int *>(ix->m_out.p + lb + db);
	}
	launch_merge_topk(S, nq, k, ix->m_pl.p, ix->m_pd.p, ix->m_pc.p, oL, oD, oC, p0->stream, ix->tie_desc);
	HIPCHK(hipGetLastError());
	if (out_host) {
		uint8_t *io = p0->ws.need_host_io(lb + db + cb);
		HIPCHK(hipMemcpyAsync(io, ix->m_out.p, lb + db + cb, hipMemcpyDeviceToHost, p0->stream));
		spin_sync(p0->stream);
		memcpy(L, io, lb);
		memcpy(D, io + lb, db);
		memcpy(C, io + lb + db, cb);
	} else {
		spin_sync(p0->stream);
	}
	// statistics of the search: summed over the shards (max pool: the largest)
	for (auto &v : ix->last_stats) v = 0;
	for (auto &sh : ix->shards) {
		for (int i : {0, 1, 4, 5}) ix->last_stats[i] += sh->last_stats[i];
		ix->last_stats[2] = std::max(ix->last_stats[2], sh->last_stats[2]);
		ix->last_stats[3] = std::max(ix->last_stats[3], sh->last_stats[3]);
	}
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

// IVF: trained on the shard with the most live rows (the shards hold whole
// ingest batches, so that is a sample of the table), installed on every other
// shard, each indexing its own rows with the same centroids / codebook (as the
// multi-process path does, lance_hip_ivf_set_model)
void shard_create_index(Index *ix, int type, int num_partitions, int num_sub_vectors) {
	Index *tr = nullptr;
	for (auto &s : ix->shards)
		if (!tr || s->n_live > tr->n_live) tr = s.get();
	tr->bind();
	tr->ivf_type_opt = type;
	ivf_build(tr, type, num_partitions, num_sub_vectors);
	const int nl = tr->ivf->nlist, m = tr->ivf->m;
	std::vector<float> C((size_t)nl * ix->dim), cb;
	if (type == IVF_PQ) cb.resize((size_t)m * PQ_K * (ix->dim / m));
	ivf_export_model(tr, C.data(), cb.empty() ? nullptr : cb.data());
	for (auto &s : ix->shards) {
		if (s.get() == tr) continue;
		s->bind();
		ivf_set_model(s.get(), type, nl, m, C.data(), cb.empty() ? nullptr : cb.data());
	}
	ix->log_model(tr);
}

}  // namespace lhip
