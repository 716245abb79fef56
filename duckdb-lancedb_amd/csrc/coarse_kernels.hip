// gfx950: the IVF coarse search (top-nprobe partitions per query) in two
// launches, exact.  Reference: rust_lib/src/lance_manager.rs:411-418
// (vector_search(q).nprobes(n)) over the IVF index of :483-515; the order is
// oracle/ivf.py coarse_probes: exact distances (f64 accumulation rounded once
// to f32, knn_kernels.hip's exact_distance), then (distance, partition id
// ascending), NaN last.
//
// Round 5 ran it as a flat search over the centroid store (its dense path:
// a bf16 bound scan over 16 row tiles = 16 workgroups, select, refine,
// finalize: five launches, ~81 us at C5's 256 x 4096 x 768).  Here:
//   coarse_bounds_kernel  f32 MFMA (v_mfma_f32_32x32x2_f32: exact products,
//                         f32 accumulation) over 64 x 64 (query, centroid)
//                         tiles through LDS — 256 workgroups at C5 — with the
//                         norms accumulated in f64 on the side; per pair a
//                         rigorous interval [LB, UB] of the f32 exact distance
//                         (|S~ - S| <= ld 2^-23 |q||c| for the f32 sum of a
//                         dot product, plus the roundings of the epilogue);
//   coarse_select_kernel  per query: T = the nprobe-th smallest UB (every one
//                         of those partitions lies within T, so the nprobe-th
//                         exact distance does), candidates = LB <= T (every
//                         partition at or below the nprobe-th exact distance,
//                         ties included), their exact distances, a
//                         (distance, id) sort, the top nprobe.
// A query whose bounds are not all finite (a NaN / inf query) or whose
// candidates overflow the buffer (many identical centroids) is flagged; the
// caller reruns the batch on the flat path (ivf_index.cpp).
#include "ivf.h"
#include "device_common.h"

#include <stdexcept>

namespace lhip {

namespace {
constexpr int CB_T = 64;       // queries x centroids per workgroup tile
constexpr int CB_KC = 64;      // k-chunk staged in LDS
constexpr int CB_PAD = 1;      // LDS row pad (floats)
constexpr int CS_THREADS = 1024;
constexpr int CS_CAP = 2048;   // candidates per query
}  // namespace

// LDS tiles: Qs[64][KC+1], Cs[64][KC+1]; wave w: queries 32 (w >> 1), centroids
// 32 (w & 1).  32x32x2 f32 MFMA: A (queries) lane l = row l % 32, k = l / 32;
// B (centroids) lane l = column l % 32, k = l / 32; accumulator register r of
// lane l = row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32.
template <int METRIC>
__global__ __launch_bounds__(256) void coarse_bounds_kernel(const float *__restrict__ Q, int nq, int dim,
                                                            const float *__restrict__ C, int ld, int nc,
                                                            float2 *__restrict__ out) {
	__shared__ float Qs[CB_T][CB_KC + CB_PAD], Cs[CB_T][CB_KC + CB_PAD];
	__shared__ double nrm[2][CB_T];  // |q|^2, |c|^2 (f64)
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	const int q0 = blockIdx.y * CB_T, c0 = blockIdx.x * CB_T;
	const int qa = (w >> 1) * 32, ca = (w & 1) * 32;
	f32x16 acc;
#pragma unroll
	for (int i = 0; i < 16; ++i) acc[i] = 0.f;
	double n2 = 0.0;  // threads 0..63: query q0 + t; 64..127: centroid c0 + t - 64
	for (int k0 = 0; k0 < dim; k0 += CB_KC) {
		__syncthreads();
		// stage: 64 rows x 64 floats of each operand, 16 floats per thread and operand
		for (int e = t; e < CB_T * CB_KC; e += 256) {
			const int r = e / CB_KC, c = e % CB_KC, k = k0 + c;
			const int q = q0 + r, cc = c0 + r;
			Qs[r][c] = (q < nq && k < dim) ? Q[(int64_t)q * dim + k] : 0.f;
			Cs[r][c] = (cc < nc && k < dim) ? C[(int64_t)cc * ld + k] : 0.f;
		}
		__syncthreads();
		if (t < 2 * CB_T) {
			const float *row = t < CB_T ? Qs[t] : Cs[t - CB_T];
			for (int c = 0; c < CB_KC; ++c) n2 = fma((double)row[c], (double)row[c], n2);
		}
#pragma unroll 8
		for (int kk = 0; kk < CB_KC; kk += 2) {
			const float a = Qs[qa + (lane & 31)][kk + (lane >> 5)];
			const float b = Cs[ca + (lane & 31)][kk + (lane >> 5)];
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
		}
	}
	mfma_operand_guard();
	if (t < 2 * CB_T) nrm[t < CB_T ? 0 : 1][t & (CB_T - 1)] = n2;
	__syncthreads();
	// |S~ - S| <= g |q||c|: an f32 sum of ld exact products, every addition rounded
	const double g = (double)ld * 0x1p-23;
	const int col = ca + (lane & 31), cc = c0 + col;
#pragma unroll
	for (int r = 0; r < 16; ++r) {
		const int row = qa + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3), q = q0 + row;
		if (q >= nq || cc >= nc) continue;
		const double qq = nrm[0][row], ccn = nrm[1][col], s = (double)acc[r];
		const double e_s = g * sqrt(qq) * sqrt(ccn) * (1.0 + 0x1p-40);
		double d, e;
		if (METRIC == METRIC_DOT) {
			d = 1.0 - s;
			e = e_s;
		} else {
			d = qq + ccn - 2.0 * s;
			e = 2.0 * e_s + 0x1p-50 * (qq + ccn + 2.0 * fabs(s));  // (the f64 norms and the sum)
		}
		// the exact distance is then rounded to f32: one more half ulp either side
		e += fabs(d) * 0x1p-23 + 1e-37;
		out[(int64_t)q * nc + cc] = make_float2(__double2float_rd(d - e), __double2float_ru(d + e));
	}
}

// per query: T = the nprobe-th smallest UB (radix select on ordered keys),
// candidates LB <= T, exact distances (exact_distance: the flat refine's
// value), (distance, id) bitonic sort, the first nprobe out
template <int METRIC>
__global__ __launch_bounds__(CS_THREADS) void coarse_select_kernel(const float2 *__restrict__ bnd, int nc,
                                                                   const float *__restrict__ Q, int dim,
                                                                   const float *__restrict__ C, int ld, int nprobe,
                                                                   int64_t *__restrict__ probe_l,
                                                                   float *__restrict__ probe_d,
                                                                   int *__restrict__ probe_c,
                                                                   int *__restrict__ flag) {
	__shared__ unsigned hist[256];
	__shared__ uint64_t keys[CS_CAP];
	__shared__ __attribute__((aligned(16))) float qs[4096];
	__shared__ unsigned s_prefix, s_rem, s_n, s_bad;
	const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
	const float2 *b = bnd + (int64_t)q * nc;
	if (t == 0) {
		s_prefix = 0;
		s_rem = (unsigned)min(nprobe, nc);
		s_n = 0;
		s_bad = 0;
	}
	for (int i = t; i < ((dim + 3) & ~3); i += CS_THREADS) qs[i] = i < dim ? Q[(int64_t)q * dim + i] : 0.f;
	__syncthreads();
	// radix select of the rem-th smallest UB key, 8 bits at a time
	unsigned mask = 0;
	for (int sh = 24; sh >= 0; sh -= 8) {
		for (int i = t; i < 256; i += CS_THREADS) hist[i] = 0;
		__syncthreads();
		const unsigned pre = s_prefix;
		for (int i = t; i < nc; i += CS_THREADS) {
			const float2 v = b[i];
			if (!(__builtin_isfinite(v.x) && __builtin_isfinite(v.y))) s_bad = 1;
			const uint32_t k = fkey(v.y);
			if ((k & mask) == pre) atomicAdd(&hist[(k >> sh) & 255], 1u);
		}
		__syncthreads();
		if (t == 0) {
			unsigned rem = s_rem, c = 0;
			int d = 0;
			for (; d < 256; ++d) {
				if (c + hist[d] >= rem) break;
				c += hist[d];
			}
			s_prefix = pre | ((unsigned)d << sh);
			s_rem = rem - c;
		}
		mask |= 255u << sh;
		__syncthreads();
	}
	if (s_bad) {
		if (t == 0) flag[q] = 1;
		return;
	}
	const float T = fkey_inv(s_prefix);
	// candidates: every partition whose LB <= T
	for (int i = t; i < nc; i += CS_THREADS) {
		if (b[i].x <= T) {
			const unsigned p = atomicAdd(&s_n, 1u);
			if (p < (unsigned)CS_CAP) keys[p] = (uint64_t)i;
		}
	}
	__syncthreads();
	const int n = (int)s_n;
	if (n > CS_CAP) {
		if (t == 0) flag[q] = 1;
		return;
	}
	// exact distances, one wave per candidate (the row from L2: the centroids are
	// read by every query)
	for (int i = w; i < n; i += CS_THREADS / 64) {
		const uint32_t id = (uint32_t)keys[i];
		const float d = exact_distance<METRIC, float>(C + (int64_t)id * ld, qs, dim, lane);
		if (lane == 0) keys[i] = ((uint64_t)fkey(d) << 32) | id;
	}
	int np2 = 64;
	while (np2 < n) np2 <<= 1;
	__syncthreads();
	for (int i = n + t; i < np2; i += CS_THREADS) keys[i] = ~0ull;
	// bitonic sort of the candidates' (distance, id) keys
	for (int size = 2; size <= np2; size <<= 1)
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			__syncthreads();
			for (int i = t; i < (np2 >> 1); i += CS_THREADS) {
				const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
				const bool asc = (lo & size) == 0;
				const uint64_t x = keys[lo], y = keys[hi];
				if ((x > y) == asc) {
					keys[lo] = y;
					keys[hi] = x;
				}
			}
		}
	__syncthreads();
	const int nout = min(nprobe, n);
	for (int i = t; i < nprobe; i += CS_THREADS) {
		probe_l[(int64_t)q * nprobe + i] = i < nout ? (int64_t)(uint32_t)keys[i] : -1;
		probe_d[(int64_t)q * nprobe + i] = i < nout ? fkey_inv((uint32_t)(keys[i] >> 32)) : __builtin_nanf("");
	}
	if (t == 0) {
		probe_c[q] = nout;
		flag[q] = 0;
	}
}

bool coarse_fused_fits(int dim, int nc, int nprobe) { return dim <= 4096 && nprobe <= nc && nc > 0 && nprobe > 0; }

void launch_coarse_search(const float *Q, int nq, int dim, const float *C, int ld, int nc, int metric, int nprobe,
                          float2 *bnd, int64_t *probe_l, float *probe_d, int *probe_c, int *flag, hipStream_t st) {
	if (nq <= 0) return;
	if (!coarse_fused_fits(dim, nc, nprobe)) throw std::runtime_error("coarse search: shape out of range");
	const dim3 g1((unsigned)((nc + CB_T - 1) / CB_T), (unsigned)((nq + CB_T - 1) / CB_T));
	if (metric == METRIC_DOT) {
		coarse_bounds_kernel<METRIC_DOT><<<g1, 256, 0, st>>>(Q, nq, dim, C, ld, nc, bnd);
		coarse_select_kernel<METRIC_DOT><<<dim3((unsigned)nq), CS_THREADS, 0, st>>>(bnd, nc, Q, dim, C, ld, nprobe,
		                                                                           probe_l, probe_d, probe_c, flag);
	} else {
		coarse_bounds_kernel<METRIC_L2><<<g1, 256, 0, st>>>(Q, nq, dim, C, ld, nc, bnd);
		coarse_select_kernel<METRIC_L2><<<dim3((unsigned)nq), CS_THREADS, 0, st>>>(bnd, nc, Q, dim, C, ld, nprobe,
		                                                                          probe_l, probe_d, probe_c, flag);
	}
}

}  // namespace lhip
