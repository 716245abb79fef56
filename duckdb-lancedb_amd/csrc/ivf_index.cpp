// IVF_FLAT / IVF_PQ host side: training, indexing, list layout and the search
// orchestration over the kernels of ivf_kernels.hip (contract in ivf.h).
//
// Reference behaviour restated (paths relative to /root/reference):
//   rust_lib/src/lance_manager.rs:483-515  create_ann_index: IVF_PQ with the
//       index metric (cosine / dot|ip / else L2), num_partitions and
//       num_sub_vectors only when > 0 (LanceDB defaults otherwise), replace(true)
//   rust_lib/src/lance_manager.rs:411-418  vector_search(q).limit(k)
//       .nprobes(n).refine_factor(r): probe the n nearest partitions, rank by
//       PQ distance, re-rank the top k*r exactly
//   rust_lib/src/lance_manager.rs:557-561  compact = optimize(All): rows added
//       after the build join the existing partitions
//   src/lance_index.hpp:91-92              nprobes 20 / refine_factor 1 defaults
// LanceDB-side defaults restated from lancedb 0.15 / lance-index 0.22 (not in
// the container): num_partitions = sqrt(rows), num_sub_vectors = dim/16 (or
// dim/8, else 1), k-means on a sample of 256 rows per centroid, <= 50
// iterations, PQ trained on <= 256*256 residual rows, 8-bit codes.
#include "ivf.h"

#include <chrono>

#include <memory>
#include <random>

namespace lhip {

IvfState::~IvfState() {
	delete coarse;
	if (h_cflag) (void)hipHostFree(h_cflag);
}
void ivf_free(IvfState *s) { delete s; }

static StoreView store_view(Index *ix) {
	// (the IVF_FLAT bound scan streams its own list-order bf16 rows, IvfState::lrows;
	// the exact list scans, re-ranks and PQ read X)
	StoreView sv{ix->X,  ix->rowaux, ix->dlabels, ix->n_slots, ix->ld, ix->dim, ix->metric, ix->xbf16 ? 1 : 0,
	             ix->Xs ? static_cast<const void *>(ix->Xs) : ix->X, (ix->xbf16 || ix->Xs) ? 1 : 0};
	sv.tie_desc = ix->tie_desc;
	return sv;
}

static int bits_for(int64_t n) {
	int b = 1;
	while (((int64_t)1 << b) < n) ++b;
	return b;
}

// grow a device buffer preserving its first `keep` elements
template <typename T>
static void grow_keep(DevBuf<T> &b, size_t want, size_t keep, hipStream_t st) {
	if (want <= b.n) return;
	T *p = nullptr;
	HIPCHK(hipMalloc(&p, want * sizeof(T)));
	if (keep > 0 && b.p) HIPCHK(hipMemcpyAsync(p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, st));
	HIPCHK(hipStreamSynchronize(st));
	b.release();
	b.p = p;
	b.n = want;
}

// f32 centroids padded with zero rows to nc_pad (the f32 assignment kernel's tiles)
static void pad_centroids(const float *C, int nc, int nc_pad, int ld, DevBuf<float> &Cf, hipStream_t st) {
	Cf.need((size_t)nc_pad * ld);
	HIPCHK(hipMemsetAsync(Cf.p, 0, (size_t)nc_pad * ld * sizeof(float), st));
	HIPCHK(hipMemcpyAsync(Cf.p, C, (size_t)nc * ld * sizeof(float), hipMemcpyDeviceToDevice, st));
}

// scratch for the sort-based k-means updates
struct SortBufs {
	DevBuf<uint32_t> k0, v0, k1, v1;
	DevBuf<int> seg;
	DevBuf<uint8_t> tmp;
	DevBuf<double> dsum;
	void sort(int64_t n, int end_bit, hipStream_t st) {
		size_t tb = 0;
		HIPCHK((hipError_t)sort_u32_pairs(nullptr, tb, k0.p, k1.p, v0.p, v1.p, n, end_bit, st));
		tmp.need(tb);
		HIPCHK((hipError_t)sort_u32_pairs(tmp.p, tb, k0.p, k1.p, v0.p, v1.p, n, end_bit, st));
	}
};

static double read_double(const double *d, hipStream_t st) {
	double h = 0.0;
	HIPCHK(hipMemcpyAsync(&h, d, sizeof(double), hipMemcpyDeviceToHost, st));
	HIPCHK(hipStreamSynchronize(st));
	return h;
}

// Lloyd k-means on n sample rows S (f32 + bf16 copies, stride ld): C[nc][ld]
// initialised with the first nc sample rows (the sample is a seeded random
// draw).  Stops after `iters` updates or when the total squared error moves by
// less than 1e-4 relative.  Leaves the final assignment of the sample in assign.
static void kmeans(const float *S, const uint16_t *Sb, int64_t n, int ld, int dim, int nc, int iters, float *C,
                   int *assign, SortBufs &sb, hipStream_t st) {
	const int nc_pad = (int)round_up(nc, 128);
	DevBuf<uint16_t> Cb;
	DevBuf<float> cnorm;
	DevBuf<uint64_t> best;
	Cb.need((size_t)nc_pad * ld);
	cnorm.need(nc_pad);
	best.need(n);
	sb.k0.need(n);
	sb.v0.need(n);
	sb.k1.need(n);
	sb.v1.need(n);
	sb.seg.need((size_t)nc + 1);
	sb.dsum.need(2);
	HIPCHK(hipMemcpyAsync(C, S, (size_t)nc * ld * sizeof(float), hipMemcpyDeviceToDevice, st));
	launch_sq_sum(S, n * ld, sb.dsum.p + 1, st);
	const double sumx2 = read_double(sb.dsum.p + 1, st);
	double prev = 0.0;
	for (int it = 0;; ++it) {
		launch_centroid_prep(C, nc, nc_pad, ld, Cb.p, cnorm.p, st);
		HIPCHK(hipMemsetAsync(best.p, 0xFF, (size_t)n * sizeof(uint64_t), st));
		launch_kmeans_assign(Sb, 1, ld, 0, n, nullptr, Cb.p, cnorm.p, nc_pad, best.p, st);
		HIPCHK(hipGetLastError());
		if (it >= iters) break;
		launch_score_sum(best.p, n, sb.dsum.p, st);
		const double loss = read_double(sb.dsum.p, st) + sumx2;  // sum |x - c|^2
		if (it > 0 && std::fabs(prev - loss) <= 1e-4 * std::fabs(loss)) break;
		prev = loss;
		launch_best_to_assign(best.p, n, nullptr, sb.k0.p, sb.v0.p, st);
		sb.sort(n, bits_for(nc), st);
		launch_segments(sb.k1.p, n, nc, sb.seg.p, st);
		launch_centroid_mean(S, ld, dim, sb.v1.p, sb.seg.p, nc, C, st);
		HIPCHK(hipGetLastError());
	}
	// the sample's final lists (PQ residuals) with exact-f32 scores
	DevBuf<float> Cf;
	pad_centroids(C, nc, nc_pad, ld, Cf, st);
	HIPCHK(hipMemsetAsync(best.p, 0xFF, (size_t)n * sizeof(uint64_t), st));
	launch_kmeans_assign_f32(S, 0, ld, 0, n, nullptr, Cf.p, cnorm.p, nc_pad, best.p, st);
	launch_best_to_assign(best.p, n, assign, nullptr, nullptr, st);
	HIPCHK(hipGetLastError());
	HIPCHK(hipStreamSynchronize(st));
}

// PQ codebook (m sub-spaces x 256 codes x dsub) by k-means on residual rows R
static void pq_train(const float *R, int64_t n, int ld, int m, int dsub, int iters, float *cb, SortBufs &sb,
                     hipStream_t st) {
	// init: code c of sub-space j = residual row c's slice j
	std::vector<float> h((size_t)PQ_K * ld), hc((size_t)m * PQ_K * dsub);
	HIPCHK(hipMemcpyAsync(h.data(), R, h.size() * sizeof(float), hipMemcpyDeviceToHost, st));
	HIPCHK(hipStreamSynchronize(st));
	for (int j = 0; j < m; ++j)
		for (int c = 0; c < PQ_K; ++c)
			for (int t = 0; t < dsub; ++t) hc[((size_t)j * PQ_K + c) * dsub + t] = h[(size_t)c * ld + j * dsub + t];
	HIPCHK(hipMemcpyAsync(cb, hc.data(), hc.size() * sizeof(float), hipMemcpyHostToDevice, st));
	const int64_t tot = n * m;
	sb.k0.need(tot);
	sb.v0.need(tot);
	sb.k1.need(tot);
	sb.v1.need(tot);
	sb.seg.need((size_t)m * PQ_K + 1);
	for (int it = 0; it < iters; ++it) {
		launch_pq_assign(R, ld, n, m, dsub, cb, sb.k0.p, sb.v0.p, st);
		sb.sort(tot, bits_for((int64_t)m * PQ_K), st);
		launch_segments(sb.k1.p, tot, m * PQ_K, sb.seg.p, st);
		launch_pq_mean(R, ld, sb.v1.p, sb.seg.p, m, dsub, cb, st);
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipStreamSynchronize(st));
}

// assign (and PQ-encode) slots [n_indexed, n_slots) with the installed model
static void index_tail(Index *ix) {
	IvfState *s = ix->ivf;
	const int64_t n0 = s->n_indexed, n1 = ix->n_slots;
	if (n1 <= n0) return;
	hipStream_t st = ix->stream;
	const int nc_pad = (int)round_up(s->nlist, 128);
	DevBuf<uint16_t> Cb;
	DevBuf<float> cnorm, Cf;
	Cb.need((size_t)nc_pad * ix->ld);
	cnorm.need(nc_pad);
	launch_centroid_prep(s->centroids.p, s->nlist, nc_pad, ix->ld, Cb.p, cnorm.p, st);
	pad_centroids(s->centroids.p, s->nlist, nc_pad, ix->ld, Cf, st);
	grow_keep(s->assign, (size_t)std::max<int64_t>(n1, 1), (size_t)n0, st);
	const bool cos = s->metric == METRIC_COSINE;
	const float *ra = reinterpret_cast<const float *>(ix->rowaux);
	// rows go to their nearest centroid by exact-f32 scores, read from the stored rows
	const void *Xa = ix->X;
	const int xab = ix->xbf16 ? 1 : 0;
	// bounded chunks of rows keep the arg-min scratch small
	const int64_t chunk = 1 << 22;
	s->best.need((size_t)std::min<int64_t>(chunk, n1 - n0));
	for (int64_t a = n0; a < n1; a += chunk) {
		const int64_t n = std::min<int64_t>(chunk, n1 - a);
		HIPCHK(hipMemsetAsync(s->best.p, 0xFF, (size_t)n * sizeof(uint64_t), st));
		launch_kmeans_assign_f32(Xa, xab, ix->ld, a, n, cos ? ra : nullptr, Cf.p, cnorm.p, nc_pad, s->best.p, st);
		launch_best_to_assign(s->best.p, n, s->assign.p + a, nullptr, nullptr, st);
		HIPCHK(hipGetLastError());
	}
	if (s->type == IVF_PQ) {
		grow_keep(s->codes, (size_t)std::max<int64_t>(n1, 1) * s->mp, (size_t)n0 * s->mp, st);
		HIPCHK(hipMemsetAsync(s->codes.p + (size_t)n0 * s->mp, 0, (size_t)(n1 - n0) * s->mp, st));
		launch_pq_encode(ix->X, ix->xbf16 ? 1 : 0, ix->ld, ix->dim, n0, n1 - n0, ra, cos ? 1 : 0, s->assign.p,
		                 s->centroids.p, s->codebook.p, s->m, s->dsub, s->mp, s->codes.p, st);
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipStreamSynchronize(st));
	s->n_indexed = n1;
	s->dirty = true;
}

// install a model given as device buffers (centroids [nlist][ld], codebook)
static void install_model(Index *ix, int type, int nlist, int m, const float *dC, const float *dcb) {
	hipStream_t st = ix->stream;
	auto s = std::make_unique<IvfState>();
	s->type = type;
	s->nlist = nlist;
	s->metric = ix->metric;
	if (type == IVF_PQ) {
		s->m = m;
		s->dsub = ix->dim / m;
		s->mp = (int)round_up(m, 16);
	}
	s->centroids.need((size_t)nlist * ix->ld);
	HIPCHK(hipMemcpyAsync(s->centroids.p, dC, (size_t)nlist * ix->ld * sizeof(float), hipMemcpyDeviceToDevice, st));
	if (type == IVF_PQ) {
		const size_t ncb = (size_t)m * PQ_K * s->dsub;
		s->codebook.need(ncb);
		HIPCHK(hipMemcpyAsync(s->codebook.p, dcb, ncb * sizeof(float), hipMemcpyDeviceToDevice, st));
		if (s->metric != METRIC_DOT) {
			s->T.need((size_t)nlist * m * PQ_K);
			launch_pq_tables_T(s->centroids.p, ix->ld, s->codebook.p, nlist, m, s->dsub, s->T.p, st);
			HIPCHK(hipGetLastError());
		}
	}
	// the centroid store: the exact flat path ranks the partitions (dot for a
	// dot index, L2 otherwise; cosine probes with normalised queries)
	auto co = std::make_unique<Index>();
	co->table = "ivf_centroids";
	co->tie_desc = 0;  // probes at a distance tie: the lower partition id (oracle/ivf.py, flat_knn.c)
	co->metric = s->metric == METRIC_DOT ? METRIC_DOT : METRIC_L2;
	co->dim = ix->dim;
	co->ld = ix->ld;
	co->init_device(ix->device);
	{
		DevBuf<float> packed;
		packed.need((size_t)nlist * ix->dim);
		HIPCHK(hipMemcpy2DAsync(packed.p, (size_t)ix->dim * sizeof(float), s->centroids.p, (size_t)ix->ld * sizeof(float),
		                        (size_t)ix->dim * sizeof(float), (size_t)nlist, hipMemcpyDeviceToDevice, st));
		HIPCHK(hipStreamSynchronize(st));
		co->add_device(packed.p, nlist);
	}
	ix->bind();
	s->coarse = co.release();
	ivf_free(ix->ivf);
	ix->ivf = s.release();
	index_tail(ix);
}

static void check_params(Index *ix, int type, int nlist, int m) {
	if (nlist <= 0) throw Error("num_partitions must be positive");
	if (type == IVF_PQ) {
		if (m <= 0 || ix->dim % m != 0)
			throw Error("num_sub_vectors (" + std::to_string(m) + ") must divide the dimension " +
			            std::to_string(ix->dim));
		if (m > PQ_MAX_M) throw Error("num_sub_vectors > " + std::to_string(PQ_MAX_M) + " is not supported");
		if (ix->dim / m > PQ_MAX_DSUB)
			throw Error("sub-vectors longer than " + std::to_string(PQ_MAX_DSUB) +
			            " dims are not supported; raise num_sub_vectors");
	}
}

void ivf_build(Index *ix, int type, int num_partitions, int num_sub_vectors) {
	if (ix->n_live <= 0) throw Error("cannot build an index on an empty table");
	const int dim = ix->dim, ld = ix->ld;
	const int nlist = num_partitions > 0 ? num_partitions : std::max(1, (int)std::sqrt((double)ix->n_live));
	const int m = num_sub_vectors > 0 ? num_sub_vectors : (dim % 16 == 0 ? dim / 16 : dim % 8 == 0 ? dim / 8 : 1);
	check_params(ix, type, nlist, m);
	if (nlist > ix->n_live)
		throw Error("KMeans: cannot train " + std::to_string(nlist) + " centroids with " +
		            std::to_string(ix->n_live) + " vectors");
	if (type == IVF_PQ && ix->n_live < PQ_K)
		throw Error("PQ training needs at least 256 rows, the table has " + std::to_string(ix->n_live));
	hipStream_t st = ix->stream;
	// seeded uniform sample of the live rows (partial Fisher-Yates)
	std::vector<int64_t> live_slots;
	live_slots.reserve((size_t)ix->n_live);
	for (int64_t s = 0; s < ix->n_slots; ++s)
		if (ix->live[(size_t)s]) live_slots.push_back(s);
	const int64_t nS = std::min<int64_t>((int64_t)live_slots.size(), (int64_t)nlist * 256);
	std::mt19937_64 rng(ix->ivf_seed);
	for (int64_t i = 0; i < nS; ++i) {
		std::uniform_int_distribution<int64_t> u(i, (int64_t)live_slots.size() - 1);
		std::swap(live_slots[(size_t)i], live_slots[(size_t)u(rng)]);
	}
	const bool cos = ix->metric == METRIC_COSINE;
	DevBuf<int64_t> dslots;
	DevBuf<float> S, C, R, cb;
	DevBuf<uint16_t> Sb;
	DevBuf<int> sassign;
	dslots.need((size_t)nS);
	S.need((size_t)nS * ld);
	Sb.need((size_t)nS * ld);
	C.need((size_t)nlist * ld);
	sassign.need((size_t)nS);
	HIPCHK(hipMemcpyAsync(dslots.p, live_slots.data(), (size_t)nS * sizeof(int64_t), hipMemcpyHostToDevice, st));
	launch_gather_sample(ix->X, ix->xbf16 ? 1 : 0, ld, dim, dslots.p, nS, cos ? 1 : 0, S.p, Sb.p, st);
	HIPCHK(hipGetLastError());
	SortBufs sb;
	kmeans(S.p, Sb.p, nS, ld, dim, nlist, ix->kmeans_iters, C.p, sassign.p, sb, st);
	if (type == IVF_PQ) {
		const int64_t nR = std::min<int64_t>(nS, (int64_t)PQ_K * PQ_K);
		R.need((size_t)nR * ld);
		launch_residuals(S.p, sassign.p, C.p, ld, nR, R.p, st);
		cb.need((size_t)m * PQ_K * (dim / m));
		pq_train(R.p, nR, ld, m, dim / m, ix->kmeans_iters, cb.p, sb, st);
	}
	HIPCHK(hipStreamSynchronize(st));
	install_model(ix, type, nlist, m, C.p, type == IVF_PQ ? cb.p : nullptr);
}

void ivf_set_model(Index *ix, int type, int nlist, int m, const float *centroids, const float *codebook) {
	check_params(ix, type, nlist, m);
	if (type == IVF_PQ && !codebook) throw Error("IVF_PQ model needs a codebook");
	hipStream_t st = ix->stream;
	DevBuf<float> C, cb;
	C.need((size_t)nlist * ix->ld);
	HIPCHK(hipMemsetAsync(C.p, 0, (size_t)nlist * ix->ld * sizeof(float), st));
	HIPCHK(hipMemcpy2DAsync(C.p, (size_t)ix->ld * sizeof(float), centroids, (size_t)ix->dim * sizeof(float),
	                        (size_t)ix->dim * sizeof(float), (size_t)nlist, hipMemcpyHostToDevice, st));
	if (type == IVF_PQ) {
		const size_t ncb = (size_t)m * PQ_K * (ix->dim / m);
		cb.need(ncb);
		HIPCHK(hipMemcpyAsync(cb.p, codebook, ncb * sizeof(float), hipMemcpyHostToDevice, st));
	}
	HIPCHK(hipStreamSynchronize(st));
	install_model(ix, type, nlist, m, C.p, type == IVF_PQ ? cb.p : nullptr);
}

void ivf_optimize(Index *ix) {
	if (ix->ivf) index_tail(ix);
}

void ivf_remap(Index *ix, const std::vector<int64_t> &keep) {
	IvfState *s = ix->ivf;
	hipStream_t st = ix->stream;
	const int64_t nk = std::lower_bound(keep.begin(), keep.end(), s->n_indexed) - keep.begin();
	DevBuf<int64_t> idx;
	idx.need((size_t)std::max<int64_t>(nk, 1));
	HIPCHK(hipMemcpyAsync(idx.p, keep.data(), (size_t)nk * sizeof(int64_t), hipMemcpyHostToDevice, st));
	{
		std::vector<int> h((size_t)s->n_indexed), o((size_t)nk);
		HIPCHK(hipMemcpyAsync(h.data(), s->assign.p, h.size() * sizeof(int), hipMemcpyDeviceToHost, st));
		HIPCHK(hipStreamSynchronize(st));
		for (int64_t i = 0; i < nk; ++i) o[(size_t)i] = h[(size_t)keep[(size_t)i]];
		DevBuf<int> na;
		na.need((size_t)std::max<int64_t>(nk, 1));
		HIPCHK(hipMemcpyAsync(na.p, o.data(), (size_t)nk * sizeof(int), hipMemcpyHostToDevice, st));
		HIPCHK(hipStreamSynchronize(st));
		std::swap(s->assign.p, na.p);
		std::swap(s->assign.n, na.n);
	}
	if (s->type == IVF_PQ) {
		DevBuf<uint8_t> nc;
		nc.need((size_t)std::max<int64_t>(nk, 1) * s->mp);
		launch_gather_bytes(s->codes.p, idx.p, nk, s->mp, nc.p, st);
		HIPCHK(hipGetLastError());
		HIPCHK(hipStreamSynchronize(st));
		std::swap(s->codes.p, nc.p);
		std::swap(s->codes.n, nc.n);
	}
	s->n_indexed = nk;
	s->dirty = true;
}

// list layout: positions grouped by list (ascending slot inside a list), each
// list padded to a multiple of 64 positions; IVF_FLAT work items of 256
// positions; IVF_PQ codes in the blocked order the list scan streams
static void layout(Index *ix) {
	IvfState *s = ix->ivf;
	hipStream_t st = ix->stream;
	const int nl = s->nlist;
	std::vector<int> a((size_t)s->n_indexed);
	if (s->n_indexed > 0)
		HIPCHK(hipMemcpyAsync(a.data(), s->assign.p, a.size() * sizeof(int), hipMemcpyDeviceToHost, st));
	HIPCHK(hipStreamSynchronize(st));
	std::vector<int64_t> cnt((size_t)nl, 0);
	for (int l : a) cnt[(size_t)l] += 1;
	s->h_lcnt = cnt;
	s->h_loff.assign((size_t)nl + 1, 0);
	for (int l = 0; l < nl; ++l) s->h_loff[(size_t)l + 1] = s->h_loff[(size_t)l] + round_up(cnt[(size_t)l], 64);
	const int64_t npos = s->h_loff[(size_t)nl];
	std::vector<uint32_t> ls((size_t)std::max<int64_t>(npos, 1), SLOT_NONE);
	std::vector<int64_t> cur(s->h_loff.begin(), s->h_loff.end() - 1);
	for (int64_t sl = 0; sl < s->n_indexed; ++sl) ls[(size_t)cur[(size_t)a[(size_t)sl]]++] = (uint32_t)sl;
	s->loff.need((size_t)nl + 1);
	s->lslot.need(ls.size());
	HIPCHK(hipMemcpyAsync(s->loff.p, s->h_loff.data(), ((size_t)nl + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
	HIPCHK(hipMemcpyAsync(s->lslot.p, ls.data(), ls.size() * sizeof(uint32_t), hipMemcpyHostToDevice, st));
	if (s->type == IVF_FLAT) {
		std::vector<int> bl, l0((size_t)nl + 1);
		std::vector<int64_t> bp;
		int maxb = 1;
		for (int l = 0; l < nl; ++l) {
			l0[(size_t)l] = (int)bl.size();
			const int64_t len = s->h_loff[(size_t)l + 1] - s->h_loff[(size_t)l];
			const int nb = (int)((len + FLAT_BLK - 1) / FLAT_BLK);
			maxb = std::max(maxb, nb);
			for (int b = 0; b < nb; ++b) {
				bl.push_back(l);
				bp.push_back(s->h_loff[(size_t)l] + (int64_t)b * FLAT_BLK);
			}
		}
		l0[(size_t)nl] = (int)bl.size();
		s->nblk = (int)bl.size();
		s->maxb = maxb;
		s->blk_list.need(std::max<size_t>(bl.size(), 1));
		s->blk_pos0.need(std::max<size_t>(bp.size(), 1));
		s->lblk0.need(l0.size());
		if (!bl.empty()) {
			HIPCHK(hipMemcpyAsync(s->blk_list.p, bl.data(), bl.size() * sizeof(int), hipMemcpyHostToDevice, st));
			HIPCHK(hipMemcpyAsync(s->blk_pos0.p, bp.data(), bp.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
		}
		HIPCHK(hipMemcpyAsync(s->lblk0.p, l0.data(), l0.size() * sizeof(int), hipMemcpyHostToDevice, st));
		// the bound scan's rows in list order (+ one item of zero rows past the
		// end: the last item reads 256 positions); rebuilt with the layout
		s->lrows_ok = false;
		if (ix->ivf_flat_bound && ix->ld % 64 == 0) {
			const size_t rows = (size_t)npos + FLAT_BLK;
			s->lrows.need(rows * ix->ld);
			HIPCHK(hipMemsetAsync(s->lrows.p + (size_t)npos * ix->ld, 0, (size_t)FLAT_BLK * ix->ld * sizeof(uint16_t), st));
			launch_list_rows_bf16(ix->X, ix->xbf16 ? 1 : 0, ix->ld, ix->dim, s->lslot.p, npos, s->lrows.p, st);
			s->lterms.need(rows);
			{  // padding positions past the last list: alpha = +inf
				const std::vector<float4> pad((size_t)FLAT_BLK, make_float4(INFINITY, 0.f, 0.f, 0.f));
				HIPCHK(hipMemcpyAsync(s->lterms.p + npos, pad.data(), pad.size() * sizeof(float4), hipMemcpyHostToDevice,
				                      st));
				HIPCHK(hipStreamSynchronize(st));  // (pad is a host temporary)
			}
			launch_list_terms(ix->rowaux, s->lslot.p, npos, s->lterms.p, st);
			HIPCHK(hipGetLastError());
			s->lrows_ok = true;
		} else {
			s->lrows.release();
			s->lterms.release();
		}
	} else {
		s->lcodes.need((size_t)std::max<int64_t>(npos, 64) * s->mp);
		launch_pq_layout(s->codes.p, s->lslot.p, npos, s->mp, s->lcodes.p, st);
		if (s->metric != METRIC_DOT) {
			s->ltau.need((size_t)std::max<int64_t>(npos, 1));
			launch_pq_tau(s->codes.p, s->lslot.p, s->loff.p, nl, npos, s->m, s->mp, s->T.p, s->ltau.p, st);
		}
		HIPCHK(hipGetLastError());
	}
	HIPCHK(hipStreamSynchronize(st));
	s->dirty = false;
}

// time_kernels: the list-scan launch (events 0/1 on the handle's stream) and
// its algorithmic work: every probed list's rows once (IVF_FLAT: dim x esz
// bytes; IVF_PQ: m code bytes + the 4-B row term tau for L2 / cosine) plus, for
// IVF_PQ, each query's LUT (m x 256 entries: f32 P[q], or the fast scan's
// 8-bit table) once; pair rows = sum over
// (query, list) pairs of the list's rows.
static void account_list_scan(Index *ix, int esz, int nq, int lut_bytes) {
	IvfState *s = ix->ivf;
	std::vector<int> ps((size_t)s->nlist + 1);
	HIPCHK(hipMemcpy(ps.data(), s->pstart.p, ps.size() * sizeof(int), hipMemcpyDeviceToHost));
	double bytes = esz ? 0.0 : (double)nq * s->m * PQ_K * lut_bytes, pair_rows = 0.0;
	const double row_pq = (double)s->m + (s->metric == METRIC_DOT ? 0.0 : 4.0);
	for (int l = 0; l < s->nlist; ++l) {
		const int np = ps[(size_t)l + 1] - ps[(size_t)l];
		if (np <= 0) continue;
		const double rows = (double)s->h_lcnt[(size_t)l];
		bytes += esz ? rows * ix->dim * esz : rows * row_pq;
		pair_rows += rows * np;
	}
	ix->kt_ivf_ms += ix->toc_ms(0, 1);
	ix->kt_ivf_n += 1;
	ix->kt_ivf_bytes += bytes;
	ix->kt_ivf_pair_rows += pair_rows;
}

void ivf_search(Index *ix, const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD, int *dC,
                PendingPass *defer) {
	IvfState *s = ix->ivf;
	hipStream_t st = ix->stream;
	if (s->dirty) layout(ix);
	if (k > IVF_MAX_K) throw Error("k > " + std::to_string(IVF_MAX_K) + " is not supported by the IVF path");
	const int nprobe = std::min(s->nlist, nprobes > 0 ? nprobes : 20);  // lance_index.hpp:91 default
	const int rf = std::max(refine, 1);
	const int kp = (int)std::min<int64_t>((int64_t)k * rf, IVF_MAX_K);
	const int kk = std::min(k, FLAT_BLK);
	const int64_t tail_n = ix->n_slots - s->n_indexed;
	const int tail_nb = (int)((tail_n + FLAT_BLK - 1) / FLAT_BLK);
	const bool cos = s->metric == METRIC_COSINE;
	const int ld = ix->ld, dim = ix->dim;
	StoreView sv = store_view(ix);
	sv.rowaux = ix->search_aux(ix->rowaux);  // filtered search: unselected slots read as tombstones
	// queries per pass: bounded by MAX_PASS_Q and ~1 GiB of list-scan keys
	const int64_t per_q = s->type == IVF_FLAT ? (int64_t)nprobe * s->maxb * kk + (int64_t)tail_nb * kk
	                                          : (int64_t)32 * kp + (int64_t)tail_nb * kk;
	const int pass = (int)std::max<int64_t>(1, std::min<int64_t>(MAX_PASS_Q, (int64_t)(1 << 27) / std::max<int64_t>(per_q, 1)));
	const bool fast_pq = s->type == IVF_PQ && ix->pq_fast && s->m <= FQ_MAX_M && kp <= FQ_MAX_KK;
	// IVF_FLAT bound scan: bf16 scan rows, k within an item's leaders
	const bool lb_flat = s->type == IVF_FLAT && ix->ivf_flat_bound && (s->lrows_ok || sv.scan_bf16) && ld % 64 == 0 &&
	                     k <= FL_KEYS - 1;
	for (int q0 = 0; q0 < nq; q0 += pass) {
		const int n = std::min(pass, nq - q0);
		bool fused = ix->ivf_coarse_fused && coarse_fused_fits(dim, s->nlist, nprobe) && s->coarse->n_slots == s->nlist &&
		             !s->coarse->xbf16;
		// one pass, asynchronous: the end wait and the flag check move to ivf_finish
		const bool deferred = defer && n == nq;
		for (;;) {  // (twice when the fused coarse search flagged a query: the second time on the flat path)
			s->Qf.need((size_t)n * ld);
			if (cos) s->Qn.need((size_t)n * dim);
			launch_ivf_prep(dQ + (int64_t)q0 * dim, n, dim, ld, cos ? 1 : 0, s->Qf.p, cos ? s->Qn.p : nullptr, st);
			// f64 queries for the exact f64 scans (tail, IVF_FLAT exact / fallback): made
			// only when one of them runs (the IVF_PQ fast path never reads them)
			bool qd_ready = false;
			auto need_qd = [&]() {
				if (qd_ready) return;
				s->Qd.need((size_t)n * ld);
				s->qn2.need((size_t)n);
				launch_ivf_qd(s->Qf.p, n, ld, dim, s->Qd.p, s->qn2.p, st);
				qd_ready = true;
			};
			HIPCHK(hipGetLastError());
			if (!fused) HIPCHK(hipStreamSynchronize(st));
			// coarse: exact top-nprobe partitions (fused: on this stream; else synchronous on the
			// centroid store's stream)
			s->probe_l.need((size_t)n * nprobe);
			s->probe_d.need((size_t)n * nprobe);
			s->probe_c.need((size_t)n);
			const auto tc0 = std::chrono::steady_clock::now();
			const float *Qc = cos ? s->Qn.p : dQ + (int64_t)q0 * dim;
			if (fused) {
				// two launches (f32 MFMA bounds, per-query select + exact refine); the flags'
				// copy is enqueued behind them and read once the pass has completed (no host
				// wait here): a flagged query has no probes, and the pass reruns on the flat
				// path below
				s->cbnd.need((size_t)n * s->nlist);
				s->cflag.need((size_t)n);
				launch_coarse_search(Qc, n, dim, static_cast<const float *>(s->coarse->X), s->coarse->ld, s->nlist,
				                     s->coarse->metric, nprobe, s->cbnd.p, s->probe_l.p, s->probe_d.p, s->probe_c.p,
				                     s->cflag.p, st);
				HIPCHK(hipGetLastError());
				if (!s->h_cflag) HIPCHK(hipHostMalloc(&s->h_cflag, (size_t)2 * MAX_PASS_Q * sizeof(int)));
				s->cflag_slot ^= 1;  // (the other slot may belong to a search still in flight)
				HIPCHK(hipMemcpyAsync(s->h_cflag + (size_t)s->cflag_slot * MAX_PASS_Q, s->cflag.p, (size_t)n * sizeof(int),
				                      hipMemcpyDeviceToHost, st));
				if (ix->time_kernels) spin_sync(st);  // (the coarse time below is host-measured)
			} else {
				s->coarse->search_device(Qc, n, nprobe, 1, s->probe_l.p, s->probe_d.p, s->probe_c.p);
			}
			if (ix->time_kernels)
				ix->kt_ivf_coarse_ms +=
				    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
			ix->bind_nodrain();  // (the coarse store's search may have switched the device; nothing to drain here)
			s->lcnt.need((size_t)s->nlist);
			s->pstart.need((size_t)s->nlist + 1);
			s->pairs.need((size_t)n * nprobe);
			// (fast PQ scan: the invert also lays out the scan's work items)
			const bool items_in_invert = fast_pq && invert_fused_fits(s->nlist);
			if (items_in_invert) {
				s->item_off.need((size_t)s->nlist + 1);
				s->xbeg.need(9);
			}
			launch_invert(s->probe_l.p, n, nprobe, s->nlist, s->lcnt.p, s->pstart.p, s->pairs.p, st,
			              items_in_invert ? s->loff.p : nullptr, items_in_invert ? s->item_off.p : nullptr,
			              items_in_invert ? s->xbeg.p : nullptr);
			int64_t *oL = dL + (int64_t)q0 * k;
			float *oD = dD + (int64_t)q0 * k;
			int *oC = dC + q0;
			if (tail_n > 0) {
				need_qd();
				s->tkeys.need((size_t)n * tail_nb * kk);
				launch_flat_list_scan(sv, nullptr, nullptr, nullptr, nullptr, nullptr, tail_nb, nullptr, nullptr, 1, 1,
				                      s->n_indexed, tail_n, n, s->Qd.p, s->qn2.p, kk, s->tkeys.p, st);
			}
			bool exact_flat = s->type == IVF_FLAT;
			if (s->type == IVF_FLAT && lb_flat) {
				// MFMA lower bounds per (query, item) -> top-M by bound -> exact
				// re-rank with a certificate; an uncertified pass reruns exactly
				const int nq_pad = (int)round_up(n, SCAN_BQ);
				s->lbQf.need((size_t)nq_pad * ld);
				s->lbQb.need((size_t)nq_pad * ld);
				s->lbqaux.need((size_t)nq_pad);
				launch_prep_queries(dQ + (int64_t)q0 * dim, n, dim, ld, nq_pad, s->metric, ix->max_alpha, ix->max_ux,
				                    s->lbQf.p, s->lbQb.p, s->lbqaux.p, nullptr, st);
				s->keys.need((size_t)n * nprobe * s->maxb * FL_KEYS);
				ix->tic(0);
				s->boff.need((size_t)s->nblk + 1);
				// items <= blocks x query groups of the pass (a block's list is probed by at most n queries)
				const int itb_cap = (int)std::min<int64_t>((int64_t)s->nblk * ((n + 15) / 16), (int64_t)1 << 28);
				s->itb.need((size_t)itb_cap);
				s->btot.need(1);
				s->live_bits.need((size_t)(ix->n_slots / 32 + 2));
				launch_flat_list_lb(sv, s->blk_list.p, s->blk_pos0.p, s->lblk0.p, s->loff.p, s->lslot.p, s->nblk,
				                    s->pstart.p, s->pairs.p, nprobe, s->maxb, s->lbQb.p, s->lbqaux.p, s->keys.p, st,
				                    s->lrows_ok ? s->lrows.p : nullptr, s->lrows_ok ? s->lterms.p : nullptr, s->live_bits.p,
				                    s->boff.p, s->btot.p, s->itb.p, itb_cap);
				ix->tic(1);
				const int M = std::min(IVF_TOPK_CAP - 1, k + 32);
				s->cand_a.need((size_t)n * M);
				s->cut.need((size_t)n);
				launch_flat_lb_merge(n, nprobe, s->probe_l.p, s->lblk0.p, s->maxb, s->keys.p, M, s->cand_a.p, s->cut.p, st);
				if (tail_n > 0) {
					s->cand_b.need((size_t)n * k);
					launch_ivf_merge(n, 0, nullptr, nullptr, 1, kk, nullptr, tail_nb, s->tkeys.p, k, s->cand_b.p, st);
				}
				s->cert.need((size_t)n);
				launch_flat_lb_refine(sv, s->Qf.p, s->cand_a.p, M, tail_n > 0 ? s->cand_b.p : nullptr, tail_n > 0 ? k : 0,
				                      s->cut.p, n, k, oL, oD, oC, s->cert.p, st);
				HIPCHK(hipGetLastError());
				s->h_cert.resize((size_t)n);
				HIPCHK(hipMemcpyAsync(s->h_cert.data(), s->cert.p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, st));
				spin_sync(st);
				exact_flat = false;
				for (int i = 0; i < n; ++i)
					if (!s->h_cert[(size_t)i]) exact_flat = true;
				if (exact_flat) ix->ivf_flat_fallbacks += 1;
				if (ix->time_kernels) account_list_scan(ix, 2, n, 0);
			}
			if (exact_flat) {
				need_qd();
				s->keys.need((size_t)n * nprobe * s->maxb * kk);
				ix->tic(0);
				launch_flat_list_scan(sv, s->blk_list.p, s->blk_pos0.p, s->lblk0.p, s->loff.p, s->lslot.p, s->nblk,
				                      s->pstart.p, s->pairs.p, nprobe, s->maxb, 0, 0, n, s->Qd.p, s->qn2.p, kk, s->keys.p, st);
				ix->tic(1);
				s->cand_a.need((size_t)n * k);
				launch_ivf_merge(n, nprobe, s->probe_l.p, s->lblk0.p, s->maxb, kk, s->keys.p, tail_nb,
				                 tail_n > 0 ? s->tkeys.p : nullptr, k, s->cand_a.p, st);
				launch_keys_to_output(s->cand_a.p, n, k, k, ix->dlabels, oL, oD, oC, st, ix->tie_desc);
			} else if (s->type == IVF_FLAT) {
				// bound scan certified every query of the pass
			} else if (ix->pq_fast && s->m <= FQ_MAX_M && kp <= FQ_MAX_KK) {
				// list-major 8-bit-LUT scan: FQ_G queries per LUT lookup, each probed
				// list's codes streamed once per query group
				const float *Qp = cos ? s->Qn.p : s->Qf.p;
				const int qld = cos ? dim : ld;
				const float sP = s->metric == METRIC_DOT ? -1.0f : -2.0f;
				s->lut8.need((size_t)n * s->m * PQ_K);
				s->qpar.need((size_t)2 * n);
				if (ix->pq_lut_fused && s->m * s->dsub == dim && pq_lut_fused_fits(s->m, dim)) {
					launch_pq_lut_fused(Qp, qld, n, dim, ix->pq_fp8 ? 1 : 0, s->codebook.p, s->m, s->dsub, sP, s->lut8.p,
					                    reinterpret_cast<float2 *>(s->qpar.p), st);
				} else {
					if (ix->pq_fp8) {
						s->Qq.need((size_t)n * qld);
						launch_pq_query_fp8(Qp, qld, n, dim, s->Qq.p, st);
						Qp = s->Qq.p;
					}
					s->P.need((size_t)n * s->m * PQ_K);
					launch_pq_P(Qp, qld, n, s->codebook.p, s->m, s->dsub, s->P.p, st);
					launch_pq_lut_u8(s->P.p, n, s->m, sP, s->lut8.p, reinterpret_cast<float2 *>(s->qpar.p), st);
				}
				s->item_off.need((size_t)s->nlist + 1);
				s->xbeg.need(9);
				int64_t maxpos = 0;
				for (int l = 0; l < s->nlist; ++l) maxpos = std::max(maxpos, s->h_loff[(size_t)l + 1] - s->h_loff[(size_t)l]);
				// items <= (query groups: n nprobe / FQ_G, + one partial group per list) x row chunks per list
				const int64_t maxnc = (maxpos + FQ_CHUNK - 1) / FQ_CHUNK;
				const int itab_cap = (int)std::min<int64_t>(((int64_t)n * nprobe / FQ_G + s->nlist) * std::max<int64_t>(maxnc, 1),
				                                            (int64_t)1 << 28);
				s->itab.need((size_t)2 * itab_cap);
				launch_pq_fast_items(s->pstart.p, s->loff.p, s->pairs.p, s->nlist, s->item_off.p, s->xbeg.p, s->itab.p,
				                     itab_cap, st, items_in_invert);
				const int ocap = (int)std::min<int64_t>((int64_t)1 << 30,
				                                        (int64_t)nprobe * ((maxpos + FQ_CHUNK - 1) / FQ_CHUNK) * FQ_CAP);
				s->okeys.need((size_t)n * ocap);
				s->ocnt.need((size_t)n);
				s->thrq.need((size_t)n);
				s->work.need(8);
				HIPCHK(hipMemsetAsync(s->ocnt.p, 0, (size_t)n * sizeof(int), st));
				HIPCHK(hipMemsetAsync(s->thrq.p, 0xFF, (size_t)n * sizeof(uint64_t), st));
				HIPCHK(hipMemsetAsync(s->work.p, 0, 8 * sizeof(int), st));
				if (ix->pq_seed)
					launch_pq_seed(s->lcodes.p, s->m, s->mp, s->loff.p, s->lslot.p, reinterpret_cast<const float *>(sv.rowaux),
					               n, nprobe, s->probe_l.p, s->probe_d.p, s->metric == METRIC_DOT ? nullptr : s->ltau.p,
					               s->lut8.p, reinterpret_cast<const float2 *>(s->qpar.p), kp, s->thrq.p, st);
				ix->tic(0);
				launch_pq_fast_scan(s->lcodes.p, s->m, s->mp, s->loff.p, s->lslot.p,
				                    reinterpret_cast<const float *>(sv.rowaux), s->nlist, nprobe, s->pstart.p, s->pairs.p,
				                    s->item_off.p, s->xbeg.p, s->probe_d.p, s->metric == METRIC_DOT ? nullptr : s->ltau.p, s->lut8.p,
				                    reinterpret_cast<const float2 *>(s->qpar.p), kp, s->work.p, s->thrq.p, s->ocnt.p,
				                    s->okeys.p, ocap, s->itab.p, scan_grid(1 << 20), st);
				ix->tic(1);
				s->cand_a.need((size_t)n * kp);
				launch_pq_run_merge(s->okeys.p, s->ocnt.p, n, ocap, kp, s->cand_a.p, st,
				                    ix->pq_merge_bound ? s->thrq.p : nullptr);
				if (tail_n > 0) {
					s->cand_b.need((size_t)n * k);
					launch_ivf_merge(n, 0, nullptr, nullptr, 1, kk, nullptr, tail_nb, s->tkeys.p, k, s->cand_b.p, st);
				}
				launch_ivf_refine_final(sv, s->Qf.p, s->cand_a.p, kp, tail_n > 0 ? s->cand_b.p : nullptr,
				                        tail_n > 0 ? k : 0, n, k, oL, oD, oC, st);
			} else {
				const float *Qp = cos ? s->Qn.p : s->Qf.p;
				const int qld = cos ? dim : ld;
				if (ix->pq_fp8) {
					s->Qq.need((size_t)n * qld);
					launch_pq_query_fp8(Qp, qld, n, dim, s->Qq.p, st);
					Qp = s->Qq.p;
				}
				s->P.need((size_t)n * s->m * PQ_K);
				launch_pq_P(Qp, qld, n, s->codebook.p, s->m, s->dsub, s->P.p, st);
				const int S = pq_segments(n);
				s->pref.need((size_t)n * (nprobe + 1));
				launch_probe_prefix(s->probe_l.p, n, nprobe, s->loff.p, s->pref.p, st);
				s->keys.need((size_t)n * S * kp);
				ix->tic(0);
				launch_pq_query_scan(s->lcodes.p, s->m, s->mp, s->loff.p, s->lslot.p,
				                     reinterpret_cast<const float *>(sv.rowaux), n, nprobe, s->probe_l.p, s->probe_d.p,
				                     s->metric == METRIC_DOT ? nullptr : s->ltau.p, s->P.p, s->pref.p, S, kp, s->keys.p, st);
				ix->tic(1);
				s->cand_a.need((size_t)n * kp);
				// the S segment lists of each query: the merge kernel's tail mode ([q][S][kp])
				launch_ivf_merge(n, 0, nullptr, nullptr, 1, kp, nullptr, S, s->keys.p, kp, s->cand_a.p, st);
				if (tail_n > 0) {
					s->cand_b.need((size_t)n * k);
					launch_ivf_merge(n, 0, nullptr, nullptr, 1, kk, nullptr, tail_nb, s->tkeys.p, k, s->cand_b.p, st);
				}
				launch_ivf_refine_final(sv, s->Qf.p, s->cand_a.p, kp, tail_n > 0 ? s->cand_b.p : nullptr,
				                        tail_n > 0 ? k : 0, n, k, oL, oD, oC, st);
			}
			HIPCHK(hipGetLastError());
			if (deferred) {
				defer->ivf = true;
				defer->ivf_fused = fused;
				defer->ivf_flag_slot = s->cflag_slot;
				defer->dQ = dQ;
				defer->nq = nq;
				defer->k = k;
				defer->nprobes = nprobes;
				defer->refine = refine;
				defer->dL = dL;
				defer->dD = dD;
				defer->dC = dC;
				return;
			}
			spin_sync(st);
			if (fused) {
				bool flagged = false;
				const int *fl = s->h_cflag + (size_t)s->cflag_slot * MAX_PASS_Q;
				for (int i = 0; i < n; ++i) flagged = flagged || fl[i] != 0;
				if (flagged) {
					ix->ivf_coarse_fallbacks += 1;
					fused = false;
					continue;
				}
			}
			if (ix->time_kernels && !(s->type == IVF_FLAT && lb_flat && !exact_flat))
				account_list_scan(ix, s->type == IVF_FLAT ? (ix->xbf16 ? 2 : 4) : 0, n, fast_pq ? 1 : 4);
			break;
		}
	}
}

}  // namespace lhip

namespace lhip {

// completion of an asynchronous IVF search: the stream has passed it (its
// event); a query the fused coarse search flagged reruns the whole search on
// the flat coarse path (synchronously, behind anything enqueued since)
void ivf_finish(Index *ix, PendingPass &p) {
	IvfState *s = ix->ivf;
	hipError_t e;
	while ((e = hipEventQuery(ix->pb[p.slot].done)) == hipErrorNotReady) {
	}
	if (e != hipSuccess) throw Error(std::string("HIP error: ") + hipGetErrorString(e) + " at search completion");
	if (!p.ivf_fused) return;
	const int *fl = s->h_cflag + (size_t)p.ivf_flag_slot * MAX_PASS_Q;
	bool flagged = false;
	for (int i = 0; i < p.nq; ++i) flagged = flagged || fl[i] != 0;
	if (!flagged) return;
	ix->ivf_coarse_fallbacks += 1;
	const bool f = ix->ivf_coarse_fused;
	ix->ivf_coarse_fused = false;
	try {
		ivf_search(ix, p.dQ, p.nq, p.k, p.nprobes, p.refine, p.dL, p.dD, p.dC);
	} catch (...) {
		ix->ivf_coarse_fused = f;
		throw;
	}
	ix->ivf_coarse_fused = f;
}

void Index::search_any(const float *dQ, int nq, int k, int nprobes, int refine, int64_t *dL, float *dD, int *dC) {
	if (ivf)
		ivf_search(this, dQ, nq, k, nprobes, refine, dL, dD, dC);
	else
		search_device(dQ, nq, k, refine, dL, dD, dC);
}

// model export as host arrays: centroids [nlist][dim], codebook [m][256][dsub]
static void model_host(Index *ix, std::vector<float> &C, std::vector<float> &cb) {
	IvfState *s = ix->ivf;
	C.resize((size_t)s->nlist * ix->dim);
	HIPCHK(hipMemcpy2D(C.data(), (size_t)ix->dim * sizeof(float), s->centroids.p, (size_t)ix->ld * sizeof(float),
	                   (size_t)ix->dim * sizeof(float), (size_t)s->nlist, hipMemcpyDeviceToHost));
	cb.clear();
	if (s->type == IVF_PQ) {
		cb.resize((size_t)s->m * PQ_K * s->dsub);
		HIPCHK(hipMemcpy(cb.data(), s->codebook.p, cb.size() * sizeof(float), hipMemcpyDeviceToHost));
	}
}

void ivf_export_model(Index *ix, float *centroids, float *codebook) {
	std::vector<float> C, cb;
	model_host(ix, C, cb);
	if (centroids) memcpy(centroids, C.data(), C.size() * sizeof(float));
	if (codebook && !cb.empty()) memcpy(codebook, cb.data(), cb.size() * sizeof(float));
}

void ivf_export_slots(Index *ix, int32_t *slot_list, uint8_t *slot_codes) {
	IvfState *s = ix->ivf;
	const int64_t n = ix->n_slots, ni = s->n_indexed;
	if (slot_list) {
		std::vector<int> a((size_t)ni);
		if (ni > 0) HIPCHK(hipMemcpy(a.data(), s->assign.p, (size_t)ni * sizeof(int), hipMemcpyDeviceToHost));
		for (int64_t i = 0; i < n; ++i) slot_list[i] = i < ni ? a[(size_t)i] : -1;
	}
	if (slot_codes) {
		memset(slot_codes, 0, (size_t)n * (s->type == IVF_PQ ? s->m : 0));
		if (s->type == IVF_PQ && ni > 0) {
			std::vector<uint8_t> c((size_t)ni * s->mp);
			HIPCHK(hipMemcpy(c.data(), s->codes.p, c.size(), hipMemcpyDeviceToHost));
			for (int64_t i = 0; i < ni; ++i) memcpy(slot_codes + i * s->m, c.data() + i * s->mp, (size_t)s->m);
		}
	}
}

void Index::log_model(Index *src) {
	if (!src) src = this;
	if (!log || !src->ivf) return;
	std::vector<float> C, cb;
	model_host(src, C, cb);
	uint8_t tag = 4;
	int32_t hdr[3] = {src->ivf->type, src->ivf->nlist, src->ivf->m};
	fwrite(&tag, 1, 1, log);
	fwrite(hdr, 4, 3, log);
	fwrite(C.data(), sizeof(float), C.size(), log);
	if (!cb.empty()) fwrite(cb.data(), sizeof(float), cb.size(), log);
	fflush(log);
}

void Index::log_optimize() {
	if (!log) return;
	uint8_t tag = 5;
	fwrite(&tag, 1, 1, log);
	fflush(log);
}

}  // namespace lhip
