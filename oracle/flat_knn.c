/*
 * CPU ORACLE / CPU BASELINE — test infrastructure only, never the product path.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load this
 * library (oracle/build/liboracle_knn.so).  The product search path is the HIP
 * library behind include/lancedb_hip.h; it never links or calls this file.
 *
 * Restates the reference's flat exact k-NN (paths relative to /root/reference):
 *   rust_lib/src/lance_manager.rs:393-451  LanceIndex::search -> lancedb 0.15
 *   Table::vector_search(q).limit(k) with no ANN index = lance 0.22 flat KNN:
 *   distance of every live row (lance-linalg 0.22: l2 = sum (x-q)^2, no sqrt;
 *   dot = 1 - x.q; cosine = 1 - x.q/(|x||q|)), ascending, at most k hits.
 * The reference itself cannot be built here (no cargo/rustc, crates offline,
 * duckdb submodule empty — SURVEY.md §0.3), so this file is the "port" CPU
 * baseline of BASELINE.md: OpenMP over host cores, per-thread top-k heaps,
 * merged at the end.
 *
 *   acc64 = 1 : float64 accumulation, rounded once to float32 (the checker:
 *               identical to oracle/flat_knn.py and to the HIP refine stage)
 *   acc64 = 0 : float32 accumulation in a SIMD-friendly loop (what
 *               lance-linalg does; used for the timed cpu_baseline)
 * Ties: (distance asc, label under the tie rule): label descending by default
 * (the reference's golden at test/sql/lance_optimizer_filter.test:36-44 keeps
 * the higher of two tied labels), ascending after oracle_set_tie(0) — the
 * library's option "tie" / LANCE_HIP_TIE.  Coarse probes and PQ (ADC)
 * candidates keep (value, id ascending), as the library does.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef struct {
	float d;
	int64_t l;
} hit_t;

static int g_tie_desc = 1; /* the final order's tie rule (oracle_set_tie) */

void oracle_set_tie(int32_t desc) { g_tie_desc = desc ? 1 : 0; }
int32_t oracle_get_tie(void) { return g_tie_desc; }

static inline int hit_less(hit_t a, hit_t b, int desc) {
	/* NaN sorts after everything */
	int an = isnan(a.d), bn = isnan(b.d);
	if (an != bn) return bn;
	if (a.d != b.d) return a.d < b.d;
	return desc ? a.l > b.l : a.l < b.l;
}

/* max-heap on hit_less (root = worst kept hit) */
static void heap_push(hit_t *h, int *n, int cap, hit_t x, int desc) {
	if (*n < cap) {
		int i = (*n)++;
		h[i] = x;
		while (i > 0) {
			int p = (i - 1) >> 1;
			if (hit_less(h[p], h[i], desc)) {
				hit_t t = h[p];
				h[p] = h[i];
				h[i] = t;
				i = p;
			} else {
				break;
			}
		}
		return;
	}
	if (!hit_less(x, h[0], desc)) return;
	h[0] = x;
	int i = 0;
	for (;;) {
		int l = 2 * i + 1, r = l + 1, m = i;
		if (l < cap && hit_less(h[m], h[l], desc)) m = l;
		if (r < cap && hit_less(h[m], h[r], desc)) m = r;
		if (m == i) break;
		hit_t t = h[m];
		h[m] = h[i];
		h[i] = t;
		i = m;
	}
}

static int cmp_hit_asc(const void *a, const void *b) {
	hit_t x = *(const hit_t *)a, y = *(const hit_t *)b;
	if (hit_less(x, y, 0)) return -1;
	if (hit_less(y, x, 0)) return 1;
	return 0;
}
static int cmp_hit_desc(const void *a, const void *b) {
	hit_t x = *(const hit_t *)a, y = *(const hit_t *)b;
	if (hit_less(x, y, 1)) return -1;
	if (hit_less(y, x, 1)) return 1;
	return 0;
}
#define CMP_HIT(desc) ((desc) ? cmp_hit_desc : cmp_hit_asc)

static inline float dist64(const float *x, const float *q, int32_t d, int metric, double qn2) {
	if (metric == 0) {
		double s = 0.0;
		for (int32_t i = 0; i < d; i++) {
			double t = (double)x[i] - (double)q[i];
			s += t * t;
		}
		return (float)s;
	}
	double dot = 0.0, xx = 0.0;
	for (int32_t i = 0; i < d; i++) {
		dot += (double)x[i] * (double)q[i];
		xx += (double)x[i] * (double)x[i];
	}
	if (metric == 1) return (float)(1.0 - dot);
	return (float)(1.0 - dot / (sqrt(xx) * sqrt(qn2)));
}

static inline float dist32(const float *restrict x, const float *restrict q, int32_t d, int metric, float qn2) {
	/* 8 independent f32 partial sums: vectorises to one AVX2 register */
	float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	float acc2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	int32_t i = 0;
	if (metric == 0) {
		for (; i + 8 <= d; i += 8)
			for (int j = 0; j < 8; j++) {
				float t = x[i + j] - q[i + j];
				acc[j] += t * t;
			}
		float s = 0.f;
		for (int j = 0; j < 8; j++) s += acc[j];
		for (; i < d; i++) {
			float t = x[i] - q[i];
			s += t * t;
		}
		return s;
	}
	for (; i + 8 <= d; i += 8)
		for (int j = 0; j < 8; j++) {
			acc[j] += x[i + j] * q[i + j];
			acc2[j] += x[i + j] * x[i + j];
		}
	float dot = 0.f, xx = 0.f;
	for (int j = 0; j < 8; j++) {
		dot += acc[j];
		xx += acc2[j];
	}
	for (; i < d; i++) {
		dot += x[i] * q[i];
		xx += x[i] * x[i];
	}
	if (metric == 1) return 1.f - dot;
	return 1.f - dot / (sqrtf(xx) * sqrtf(qn2));
}

/*
 * Batched exact top-k.  base [n][d] row-major f32; live (nullable) 1 = live;
 * labels (nullable) -> label = row index; Q [nq][d].
 * Rows are split over threads in blocks of ROWBLK so each block of base rows is
 * reused from cache for every query; per-(thread, query) heaps of size k are
 * merged at the end.  Returns 0, or -1 on allocation failure.
 */
#define ROWBLK 64
int oracle_flat_search_batch(const float *base, int64_t n, int32_t d, const uint8_t *live, const int64_t *labels,
                             const float *Q, int32_t nq, int32_t k, int32_t metric, int32_t acc64, int32_t nthreads,
                             int64_t *out_labels, float *out_dist, int32_t *out_counts) {
	if (k <= 0 || nq <= 0) return 0;
	if (nthreads <= 0) nthreads = omp_get_max_threads();
	const int tie = g_tie_desc;
	double *qn2 = (double *)calloc((size_t)nq, sizeof(double));
	hit_t *heaps = (hit_t *)malloc((size_t)nthreads * nq * k * sizeof(hit_t));
	int *hn = (int *)calloc((size_t)nthreads * nq, sizeof(int));
	if (!qn2 || !heaps || !hn) {
		free(qn2);
		free(heaps);
		free(hn);
		return -1;
	}
	for (int32_t j = 0; j < nq; j++) {
		double s = 0;
		for (int32_t i = 0; i < d; i++) s += (double)Q[(size_t)j * d + i] * Q[(size_t)j * d + i];
		qn2[j] = s;
	}
	int64_t nblk = (n + ROWBLK - 1) / ROWBLK;
#pragma omp parallel num_threads(nthreads)
	{
		int t = omp_get_thread_num();
		hit_t *my = heaps + (size_t)t * nq * k;
		int *myn = hn + (size_t)t * nq;
#pragma omp for schedule(dynamic, 16)
		for (int64_t b = 0; b < nblk; b++) {
			int64_t r0 = b * ROWBLK, r1 = r0 + ROWBLK < n ? r0 + ROWBLK : n;
			for (int32_t j = 0; j < nq; j++) {
				const float *q = Q + (size_t)j * d;
				for (int64_t r = r0; r < r1; r++) {
					if (live && !live[r]) continue;
					const float *x = base + (size_t)r * d;
					float dd = acc64 ? dist64(x, q, d, metric, qn2[j]) : dist32(x, q, d, metric, (float)qn2[j]);
					hit_t h = {dd, labels ? labels[r] : r};
					heap_push(my + (size_t)j * k, &myn[j], k, h, tie);
				}
			}
		}
	}
	/* merge per-thread heaps */
	hit_t *tmp = (hit_t *)malloc((size_t)nthreads * k * sizeof(hit_t));
	for (int32_t j = 0; j < nq; j++) {
		int m = 0;
		for (int t = 0; t < nthreads; t++) {
			memcpy(tmp + m, heaps + ((size_t)t * nq + j) * k, (size_t)hn[(size_t)t * nq + j] * sizeof(hit_t));
			m += hn[(size_t)t * nq + j];
		}
		qsort(tmp, (size_t)m, sizeof(hit_t), CMP_HIT(tie));
		int c = m < k ? m : k;
		out_counts[j] = c;
		for (int i = 0; i < k; i++) {
			out_labels[(size_t)j * k + i] = i < c ? tmp[i].l : -1;
			out_dist[(size_t)j * k + i] = i < c ? tmp[i].d : NAN;
		}
	}
	free(tmp);
	free(qn2);
	free(heaps);
	free(hn);
	return 0;
}

/* exact distances of all rows to one query (checker for size-independent tests) */
void oracle_distances(const float *base, int64_t n, int32_t d, const float *q, int32_t metric, float *out) {
	double qn2 = 0;
	for (int32_t i = 0; i < d; i++) qn2 += (double)q[i] * q[i];
#pragma omp parallel for schedule(static)
	for (int64_t r = 0; r < n; r++) out[r] = dist64(base + (size_t)r * d, q, d, metric, qn2);
}

/*
 * IVF_FLAT / IVF_PQ search over a given model and list layout (the CPU port of
 * the IVF path, oracle/ivf.py's numerics; timed as the cpu_baseline of the IVF
 * bench configs and cross-checked against oracle/ivf.py in tests/).
 * Reference: rust_lib/src/lance_manager.rs:411-418 (vector_search(q).limit(k)
 * .nprobes(n).refine_factor(r)) over the IVF_PQ index of :483-515.
 *
 *   base [n][d] f32 rows by slot, labels [n]; lists as CSR over LIVE indexed
 *   slots: loff [nlist+1], lrows [loff[nlist]] (ascending slots per list);
 *   tail [ntail] live slots not indexed (searched exactly);
 *   C [nlist][d] centroids; IVF_PQ when codes != NULL: codes [n][m] (by slot),
 *   codebook cb [m][256][d/m], T [nlist][m][256] (NULL for dot).
 *   ADC = (d0 + tau) + sum_j LUT[j][c_j] (f32, j order), tau = sum_j
 *   T[l][j][c_j] (f32 from 0), LUT = -2 P (l2) / -P and tau = 0 (dot).
 *   pq_flags bit 0: the fast scan's 8-bit LUT (oracle/ivf.py pq_lut_u8: ADC =
 *   ((d0 + tau) + L0) + D * sum_j u[j][c_j]); bit 1: P from the fp8 (e4m3)
 *   query (oracle/ivf.py fp8_queries).
 *   metric 0 l2, 1 dot (cosine: -2, not ported).  acc64: f64 exact distances
 *   (the checker) or f32 SIMD (the timed baseline) for the coarse / flat /
 *   re-rank distances; the ADC is f32 in j order in both.
 * Parallel over the probed lists of each query (per-thread heaps).
 */
/* OCP e4m3fn round-to-nearest-even, |v| <= 448 (oracle/ivf.py e4m3_round) */
static float e4m3_round(float v) {
	const float a = fabsf(v);
	if (!(a > 0.0f)) return v;
	int e;
	(void)frexpf(a, &e);
	const int E = e - 1 > -6 ? e - 1 : -6;
	const float ulp = ldexpf(1.0f, E - 3);
	const float r = fminf(rintf(a / ulp) * ulp, 448.0f);
	return copysignf(r, v);
}

static void topk_sel(const float *dv, int64_t n, int32_t np, int32_t *ids, float *ds) {
	hit_t *h = (hit_t *)malloc((size_t)np * sizeof(hit_t));
	int hn = 0;
	for (int64_t i = 0; i < n; i++) {
		hit_t x = {dv[i], i};
		heap_push(h, &hn, np, x, 0); /* probes: (distance, partition id ascending) */
	}
	qsort(h, (size_t)hn, sizeof(hit_t), cmp_hit_asc);
	for (int i = 0; i < hn; i++) {
		ids[i] = (int32_t)h[i].l;
		ds[i] = h[i].d;
	}
	free(h);
}

int oracle_ivf_search_batch(const float *base, int32_t d, const int64_t *labels, const int64_t *loff,
                            const int64_t *lrows, int32_t nlist, const int64_t *tail, int64_t ntail, const float *C,
                            const uint8_t *codes, int32_t m, const float *cb, const float *T, const float *Q,
                            int32_t nq, int32_t k, int32_t nprobe, int32_t refine, int32_t metric, int32_t acc64,
                            int32_t pq_flags, int32_t nthreads, int64_t *out_labels, float *out_dist,
                            int32_t *out_counts) {
	if (metric != 0 && metric != 1) return -2;
	const int lut8 = pq_flags & 1, qfp8 = (pq_flags >> 1) & 1;
	if (nthreads <= 0) nthreads = omp_get_max_threads();
	if (nprobe > nlist) nprobe = nlist;
	const int pq = codes != NULL;
	/* list candidates: PQ by (ADC, slot ascending); IVF_FLAT exact distances by
	   slot under the tie rule (slots ascend with labels); the final order too */
	const int tie = g_tie_desc, ltie = pq ? 0 : tie;
	const int dsub = pq ? d / m : 0;
	const int kp = pq ? k * (refine > 1 ? refine : 1) : k;
	float *cd = (float *)malloc((size_t)nlist * sizeof(float));
	int32_t *pid = (int32_t *)malloc((size_t)nprobe * sizeof(int32_t));
	float *pd = (float *)malloc((size_t)nprobe * sizeof(float));
	float *P = pq ? (float *)malloc((size_t)m * 256 * sizeof(float)) : NULL;
	uint8_t *U = pq ? (uint8_t *)malloc((size_t)m * 256) : NULL;
	float *qp = (float *)malloc((size_t)d * sizeof(float));
	float D8 = 1.0f, L08 = 0.0f;
	hit_t *heaps = (hit_t *)malloc((size_t)nthreads * kp * sizeof(hit_t));
	int *hn = (int *)malloc((size_t)nthreads * sizeof(int));
	hit_t *all = (hit_t *)malloc(((size_t)nthreads * kp + (size_t)k) * sizeof(hit_t));
	if (!cd || !pid || !pd || (pq && !P) || !heaps || !hn || !all) return -1;
	for (int32_t qi = 0; qi < nq; qi++) {
		const float *q = Q + (size_t)qi * d;
		double qn2 = 0.0;
		for (int32_t i = 0; i < d; i++) qn2 += (double)q[i] * q[i];
		/* coarse: dot for a dot index, l2 otherwise; top-nprobe by (dist, id) */
#pragma omp parallel for num_threads(nthreads) schedule(static)
		for (int32_t l = 0; l < nlist; l++)
			cd[l] = acc64 ? dist64(C + (size_t)l * d, q, d, metric, qn2) : dist32(C + (size_t)l * d, q, d, metric, (float)qn2);
		topk_sel(cd, nlist, nprobe, pid, pd);
		if (pq) {
			/* the ADC tables' query: f32, or e4m3(q / s) * s, s = absmax / 448 */
			float mx = 0.0f;
			for (int32_t i = 0; i < d; i++) mx = fmaxf(mx, fabsf(q[i]));
			const float sc = mx / 448.0f;
			for (int32_t i = 0; i < d; i++) qp[i] = (qfp8 && sc > 0.0f) ? e4m3_round(q[i] / sc) * sc : (qfp8 ? 0.0f : q[i]);
#pragma omp parallel for num_threads(nthreads) schedule(static)
			for (int32_t e = 0; e < m * 256; e++) {
				const int j = e / 256;
				const float *y = cb + (size_t)e * dsub;
				float acc = 0.0f;
				for (int t = 0; t < dsub; t++) acc = acc + qp[j * dsub + t] * y[t];
				P[e] = acc;
			}
			if (lut8) { /* 8-bit LUT, per oracle/ivf.py pq_lut_u8 */
				const float sP = T ? -2.0f : -1.0f;
				float mxs = 0.0f;
				L08 = 0.0f;
				float *lo = (float *)malloc((size_t)m * sizeof(float));
				for (int j = 0; j < m; j++) {
					float a = INFINITY, b = -INFINITY;
					for (int c = 0; c < 256; c++) {
						const float v = sP * P[j * 256 + c];
						a = fminf(a, v);
						b = fmaxf(b, v);
					}
					lo[j] = a;
					mxs = fmaxf(mxs, b - a);
				}
				for (int j = 0; j < m; j++) L08 = L08 + lo[j];
				D8 = mxs > 0.0f ? mxs / 255.0f : 1.0f;
				const float inv = 1.0f / D8;
				for (int e = 0; e < m * 256; e++)
					U[e] = (uint8_t)fminf(rintf((sP * P[e] - lo[e / 256]) * inv), 255.0f);
				free(lo);
			}
		}
		for (int t = 0; t < nthreads; t++) hn[t] = 0;
#pragma omp parallel num_threads(nthreads)
		{
			const int t = omp_get_thread_num();
			hit_t *my = heaps + (size_t)t * kp;
			float *lut = pq ? (float *)malloc((size_t)m * 256 * sizeof(float)) : NULL;
#pragma omp for schedule(dynamic, 1)
			for (int32_t p = 0; p < nprobe; p++) {
				const int32_t l = pid[p];
				if (pq) {
					for (int e = 0; e < m * 256; e++) lut[e] = T ? -2.0f * P[e] : -P[e];
				}
				for (int64_t i = loff[l]; i < loff[l + 1]; i++) {
					const int64_t s = lrows[i];
					float dd;
					if (pq) {
						const uint8_t *c = codes + (size_t)s * m;
						float acc = pd[p];
						if (T) { /* row term tau = sum_j T[l][j][c_j], then the query LUT */
							const float *Tl = T + (size_t)l * m * 256;
							float tau = 0.0f;
							for (int j = 0; j < m; j++) tau = tau + Tl[j * 256 + c[j]];
							acc = acc + tau;
						}
						if (lut8) {
							int32_t S = 0;
							for (int j = 0; j < m; j++) S += U[j * 256 + c[j]];
							acc = acc + L08;
							acc = acc + D8 * (float)S;
						} else {
							for (int j = 0; j < m; j++) acc = acc + lut[j * 256 + c[j]];
						}
						dd = acc;
					} else {
						dd = acc64 ? dist64(base + (size_t)s * d, q, d, metric, qn2)
						           : dist32(base + (size_t)s * d, q, d, metric, (float)qn2);
					}
					hit_t h = {dd, s}; /* by slot: slots ascend with labels, so ties go by label */
					heap_push(my, &hn[t], kp, h, ltie);
				}
			}
			free(lut);
		}
		int na = 0;
		for (int t = 0; t < nthreads; t++) {
			memcpy(all + na, heaps + (size_t)t * kp, (size_t)hn[t] * sizeof(hit_t));
			na += hn[t];
		}
		qsort(all, (size_t)na, sizeof(hit_t), CMP_HIT(ltie));
		if (na > kp) na = kp;
		/* re-rank (PQ) + the unindexed tail, exact */
		int nc = 0;
		hit_t *cand = (hit_t *)malloc(((size_t)na + (size_t)ntail + 1) * sizeof(hit_t));
		for (int i = 0; i < na; i++) {
			const int64_t s = all[i].l;
			float dd = all[i].d;
			if (pq) dd = acc64 ? dist64(base + (size_t)s * d, q, d, metric, qn2) : dist32(base + (size_t)s * d, q, d, metric, (float)qn2);
			hit_t h = {dd, labels[s]};
			cand[nc++] = h;
		}
		for (int64_t i = 0; i < ntail; i++) {
			const int64_t s = tail[i];
			hit_t h = {acc64 ? dist64(base + (size_t)s * d, q, d, metric, qn2) : dist32(base + (size_t)s * d, q, d, metric, (float)qn2), labels[s]};
			cand[nc++] = h;
		}
		qsort(cand, (size_t)nc, sizeof(hit_t), CMP_HIT(tie));
		const int c = nc < k ? nc : k;
		out_counts[qi] = c;
		for (int i = 0; i < k; i++) {
			out_labels[(size_t)qi * k + i] = i < c ? cand[i].l : -1;
			out_dist[(size_t)qi * k + i] = i < c ? cand[i].d : NAN;
		}
		free(cand);
	}
	free(cd);
	free(pid);
	free(pd);
	free(P);
	free(U);
	free(qp);
	free(heaps);
	free(hn);
	free(all);
	return 0;
}
