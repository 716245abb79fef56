// gfx950 (MI355X / CDNA4) kernels of the flat k-NN path.
//
// Replaces the arithmetic the reference delegates to lance 0.22 / lance-linalg
// 0.22 (flat KNN behind rust_lib/src/lance_manager.rs:411-419, paths relative
// to /root/reference).  Pipeline per search (DESIGN.md "Search pipeline"):
//
//   prep_queries   f32 queries -> zero-padded f32 + bf16 copies + LB constants
//   scan           bf16 MFMA (v_mfma_f32_32x32x16_bf16) query x base tiles with
//                  the base streamed once from HBM as f32, converted in
//                  registers, staged through XOR-swizzled LDS; the epilogue
//                  turns each dot product into a rigorous LOWER BOUND of the
//                  exact distance and either writes it (dense mode, small N /
//                  sample) or appends (LB, slot) when LB <= tau[q] (append mode)
//   select         per-query radix select of the M smallest lower bounds
//   refine         exact distance of the M candidates, f64 accumulation
//   finalize       sort by (distance, label), top-k, exactness certificate:
//                  every row left out has LB >= cut > k-th exact distance
//   exact_all/sort fallback for a query whose certificate failed
//
// No hipify, no CUDA shims: wave64, MFMA and LDS idioms written for CDNA4.
#include <atomic>
#include "knn_kernels.h"

#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <stdexcept>
#include <cfloat>
#include <cmath>

#include "device_common.h"

namespace lhip {



// ---------------------------------------------------------------------------
// ingest: per-row auxiliary data
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void rowaux_row(const T *__restrict__ X, int ld, int dim, int metric, int64_t s0, int64_t r,
                                           float4 *__restrict__ rowaux, unsigned &m0, unsigned &m1, int lane) {
	const T *x = X + (s0 + r) * (int64_t)ld;
	double s2 = 0.0, e2 = 0.0;
	for (int i = lane; i < dim; i += 64) {
		float v = xval(x, i);
		float e = v - bf16_round(v);
		s2 += (double)v * v;
		e2 += (double)e * e;
	}
	s2 = wave_sum_f64(s2);
	e2 = wave_sum_f64(e2);
	if (lane == 0) {
		double xn = sqrt(s2), ex = sqrt(e2);
		double ux = (xn + ex) * (1.0 + 4.0 * U_BOUND);
		float4 a;
		if (metric == METRIC_L2) {
			// alpha = +inf is the tombstone code: a live row whose |x|^2 overflows f32
			// keeps the largest finite alpha (below |x|^2: the bound stays a lower
			// bound; finalize's count check catches a bound that still overflows)
			a = make_float4(fminf((float)s2, F_MAX), (float)xn, (float)ux, 1.0f);
		} else if (metric == METRIC_DOT) {
			a = make_float4(0.0f, (float)xn, (float)ux, 1.0f);
		} else {
			if (xn > 0.0) {
				a = make_float4(0.0f, 0.0f, (float)(ux / xn * (1.0 + 4.0 * U_BOUND)), (float)(1.0 / xn));
			} else {
				a = make_float4(__builtin_nanf(""), 0.0f, 0.0f, 0.0f);  // cosine undefined: exact fallback
			}
		}
		float *ra = reinterpret_cast<float *>(rowaux);
		ra[raix(s0 + r, 0)] = a.x;
		ra[raix(s0 + r, 1)] = a.y;
		ra[raix(s0 + r, 2)] = a.z;
		ra[raix(s0 + r, 3)] = a.w;
		if (a.x == a.x) m0 = max(m0, __float_as_uint(fabsf(a.x)));
		m1 = max(m1, __float_as_uint(a.z));
	}
}

template <typename T>
__global__ __launch_bounds__(256) void rowaux_kernel(const T *__restrict__ X, int ld, int dim, int metric,
                                                     int64_t s0, int64_t n, float4 *__restrict__ rowaux,
                                                     unsigned *__restrict__ stats) {
	// grid-stride, one wave per row at a time; the maxima go out once per wave
	// (one atomicMax per row on the same two words serialised: 5.7 ms per 262k rows)
	const int lane = threadIdx.x & 63;
	unsigned m0 = 0u, m1 = 0u;
	for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < n; r += (int64_t)gridDim.x * 4)
		rowaux_row(X, ld, dim, metric, s0, r, rowaux, m0, m1, lane);
	if (lane == 0) {
		atomicMax(&stats[0], m0);
		atomicMax(&stats[1], m1);
	}
}

void launch_rowaux(const void *X, int xbf16, int ld, int dim, int metric, int64_t s0, int64_t n, float4 *rowaux,
                   unsigned *stats, hipStream_t st) {
	if (n <= 0) return;
	const int64_t blocks = std::min<int64_t>((n + 3) / 4, 4096);
	if (xbf16)
		rowaux_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>((const uint16_t *)X, ld, dim, metric, s0, n, rowaux,
		                                                            stats);
	else
		rowaux_kernel<<<dim3((unsigned)blocks), dim3(256), 0, st>>>((const float *)X, ld, dim, metric, s0, n, rowaux,
		                                                            stats);
}

__global__ __launch_bounds__(256) void rows_to_bf16_kernel(const float *__restrict__ src, int64_t src_ld, int64_t n,
                                                           int dim, int ld, uint16_t *__restrict__ dst) {
	const int64_t r = (int64_t)blockIdx.x;
	if (r >= n) return;
	for (int i = threadIdx.x; i < ld; i += blockDim.x)
		dst[r * ld + i] = i < dim ? bf16_bits(src[r * src_ld + i]) : (uint16_t)0;
}

void launch_rows_to_bf16(const float *src, int64_t src_ld, int64_t n, int dim, int ld, uint16_t *dst, hipStream_t st) {
	if (n <= 0) return;
	rows_to_bf16_kernel<<<dim3((unsigned)n), dim3(256), 0, st>>>(src, src_ld, n, dim, ld, dst);
}

// ---------------------------------------------------------------------------
// int8 scan copy (option scan_i8, an f32 store), one scale per 256-row tile:
//   v = x (l2, dot) or x/|x| (cosine), s_T = max over the tile's rows of
//   max|v_i| / 127 (an f32 value), x^ = rint(v / s_T) in [-127, 127], x~ = s_T x^.
// The int8 scans' rigorous bound:
//   |v.q - s_T s_Q (x^.q^)| <= |e_x||q| + |x~||e_q|,   e_x = v - x~  (f64)
// and x^.q^ is an exact integer (|x^.q^| <= ld * 127^2 < 2^24 for ld <= 1024:
// exact in f32 too).  Row terms (tile-blocked SoA like rowaux):
//   l2: (|x|^2, |e_x|, |x~|, s_T)   dot: (0, |e_x|, |x~|, s_T)
//   cosine: (0, |e_x|, |x~|, s_T) of the normalised row   (norms rounded up)
// Layout (k-major tiles): tile t is one block of 256 * ld bytes holding its rows'
// 64-byte k-chunks chunk-major, byte c of row r at
//   t * 256 * ld + (c / 64) * 16384 + (r % 256) * 64 + c % 64,
// so one k-step of 16 rows (an MFMA operand load) is 1 KiB contiguous.  The
// two workgroups that read a tile (scan8's query halves) then share it in L2;
// row-major rows (16 half-used lines per load) ran 1.5x longer at 10M x 768.
// Per tile: tstat = (s_T, max |e_x|, max |x~|, 0) over its rows.  A scale common
// to the tile (and one common to the query batch, prep_queries_i8) makes the
// product scale of a bound s_T s_Q the same for every (row, query) of a tile:
// scan8_kernel screens bounds in exact integers with it.  alpha copies the
// store's tombstones (+inf); a zero cosine row is NaN (exact fallback), as in
// rowaux.  stats[0] = max |alpha|, stats[1] = max(xn, ux).
// One 256-thread workgroup per tile: row maxima into LDS, the tile scale, then
// each wave quantises rows (rows past n_slots: zero, alpha = +inf).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void tiles_to_i8_kernel(const T *__restrict__ X, int ld, int dim, int metric,
                                                          int64_t n_slots, int64_t t0,
                                                          const float4 *__restrict__ rowaux, int8_t *__restrict__ Xq,
                                                          float4 *__restrict__ aux8, float4 *__restrict__ tstat,
                                                          unsigned *__restrict__ stats) {
	__shared__ float rmax[SCAN_BR];
	__shared__ double rnorm[SCAN_BR];
	__shared__ float red[3][4];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const int64_t tile = t0 + blockIdx.x;
	const bool cosine = metric == METRIC_COSINE;
	// pass 1: per row max|v_i| and |x|
	for (int rr = wv; rr < SCAN_BR; rr += 4) {
		const int64_t r = tile * SCAN_BR + rr;
		float m = 0.f;
		double s2 = 0.0;
		if (r < n_slots) {
			const T *x = X + r * (int64_t)ld;
			for (int i = lane; i < dim; i += 64) {
				const float v = xval(x, i);
				m = fmaxf(m, fabsf(v));
				s2 += (double)v * v;
			}
		}
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
		s2 = wave_sum_f64(s2);
		if (lane == 0) {
			const double xn = sqrt(s2);
			rnorm[rr] = xn;
			rmax[rr] = cosine ? (xn > 0.0 ? (float)((double)m / xn) : 0.f) : m;
		}
	}
	__syncthreads();
	float M = 0.f;
	for (int i = threadIdx.x; i < SCAN_BR; i += 256) M = fmaxf(M, rmax[i]);
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
	if (lane == 0) red[0][wv] = M;
	__syncthreads();
	M = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
	// (cosine: the rounded row maxima may sit a hair under the f64 quotients;
	// the clamp to +-127 keeps x^ in range and e_x stays exact either way)
	const float sT = M / 127.0f;
	const double inv = M > 0.f ? 127.0 / (double)M : 0.0;
	const double up = 1.0 + 4.0 * U_BOUND;
	unsigned m0 = 0u, m1 = 0u;
	float wxn = 0.f, wux = 0.f;  // this wave's row maxima of |e_x|, |x~|
	__syncthreads();             // red[0] read by every wave before it is reused
	// pass 2: quantise
	for (int rr = wv; rr < SCAN_BR; rr += 4) {
		const int64_t r = tile * SCAN_BR + rr;
		int8_t *xrow = Xq + tile * SCAN_BR * (int64_t)ld + rr * 64;  // k-chunk c at xrow + c * I8_CHUNK_STRIDE
		auto xq_at = [&](int i0) -> uint32_t * {
			return reinterpret_cast<uint32_t *>(xrow + (int64_t)(i0 >> 6) * I8_CHUNK_STRIDE + (i0 & 63));
		};
		float *o = reinterpret_cast<float *>(aux8);
		if (r >= n_slots) {
			for (int i0 = 4 * lane; i0 < ld; i0 += 256) *xq_at(i0) = 0u;
			if (lane == 0) {
				o[raix(r, 0)] = F_INF;
				o[raix(r, 1)] = 0.f;
				o[raix(r, 2)] = 0.f;
				o[raix(r, 3)] = sT;
			}
			continue;
		}
		const T *x = X + r * (int64_t)ld;
		const double xn = rnorm[rr];
		const double rs = (cosine && xn > 0.0) ? 1.0 / xn : 1.0;
		double e2 = 0.0, t2 = 0.0;
		// four elements per lane and step: one packed 4-byte store (ld is a multiple of 128)
		for (int i0 = 4 * lane; i0 < ld; i0 += 256) {
			uint32_t packed = 0u;
#pragma unroll
			for (int j = 0; j < 4; ++j) {
				const int i = i0 + j;
				int qv = 0;
				if (i < dim) {
					const double v = cosine ? (double)xval(x, i) * rs : (double)xval(x, i);
					qv = (int)fmin(127.0, fmax(-127.0, rint(v * inv)));
					const double xt = (double)sT * (double)qv;
					const double e = v - xt;
					e2 += e * e;
					t2 += xt * xt;
				}
				packed |= ((uint32_t)qv & 0xFFu) << (8 * j);
			}
			*xq_at(i0) = packed;
		}
		e2 = wave_sum_f64(e2);
		t2 = wave_sum_f64(t2);
		// cosine: v = x/|x| carries the f64 rounding of the quotient; 2^-40
		// covers it in |e_x| (the bound needs |v_true - x~|)
		const double ex = sqrt(e2) * up + (cosine ? 0x1p-40 : 0.0), xt = sqrt(t2) * up;
		float4 a;
		if (metric == METRIC_L2)
			a = make_float4((float)(xn * xn), (float)ex, (float)xt, sT);
		else if (!cosine || xn > 0.0)
			a = make_float4(0.0f, (float)ex, (float)xt, sT);
		else
			a = make_float4(__builtin_nanf(""), 0.0f, 0.0f, sT);  // cosine undefined: exact fallback
		const float *ra = reinterpret_cast<const float *>(rowaux);
		if (__builtin_isinf(ra[raix(r, 0)])) a.x = F_INF;  // tombstone
		// (|x|^2 as rowaux computes it: the f64 sum rounded once)
		if (metric == METRIC_L2 && a.x != F_INF) a.x = ra[raix(r, 0)];
		if (lane == 0) {
			o[raix(r, 0)] = a.x;
			o[raix(r, 1)] = a.y;
			o[raix(r, 2)] = a.z;
			o[raix(r, 3)] = a.w;
		}
		wxn = fmaxf(wxn, a.y);
		wux = fmaxf(wux, a.z);
		if (a.x == a.x && a.x != F_INF) m0 = max(m0, __float_as_uint(fabsf(a.x)));
		m1 = max(m1, __float_as_uint(fmaxf(a.y, a.z)));
	}
	if (lane == 0) {
		red[1][wv] = wxn;
		red[2][wv] = wux;
		atomicMax(&stats[0], m0);
		atomicMax(&stats[1], m1);
	}
	__syncthreads();
	if (threadIdx.x == 0)
		tstat[tile] = make_float4(sT, fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3])),
		                          fmaxf(fmaxf(red[2][0], red[2][1]), fmaxf(red[2][2], red[2][3])), 0.f);
}

void launch_tiles_to_i8(const void *X, int xbf16, int ld, int dim, int metric, int64_t n_slots, int64_t t0,
                        int64_t t1, const float4 *rowaux, int8_t *Xq, float4 *aux8, float4 *tstat, unsigned *stats,
                        hipStream_t st) {
	if (t1 <= t0) return;
	const dim3 grid((unsigned)(t1 - t0)), blk(256);
	if (xbf16)
		tiles_to_i8_kernel<uint16_t><<<grid, blk, 0, st>>>(static_cast<const uint16_t *>(X), ld, dim, metric, n_slots,
		                                                   t0, rowaux, Xq, aux8, tstat, stats);
	else
		tiles_to_i8_kernel<float><<<grid, blk, 0, st>>>(static_cast<const float *>(X), ld, dim, metric, n_slots, t0,
		                                                rowaux, Xq, aux8, tstat, stats);
}

__global__ void fill_rowaux_kernel(float4 *rowaux, int64_t from, int64_t to) {
	const int64_t i = from + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i < to) {
		float *ra = reinterpret_cast<float *>(rowaux);
		ra[raix(i, 0)] = F_INF;
		ra[raix(i, 1)] = 0.f;
		ra[raix(i, 2)] = 0.f;
		ra[raix(i, 3)] = 0.f;
	}
}

void launch_fill_rowaux(float4 *rowaux, int64_t from, int64_t to, hipStream_t st) {
	if (to <= from) return;
	fill_rowaux_kernel<<<dim3((unsigned)((to - from + 255) / 256)), dim3(256), 0, st>>>(rowaux, from, to);
}

__global__ void tombstone_kernel(float4 *rowaux, const int64_t *slots, int n) {
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < n) reinterpret_cast<float *>(rowaux)[raix(slots[i], 0)] = F_INF;
}

void launch_tombstone(float4 *rowaux, const int64_t *slots, int n, hipStream_t st) {
	if (n <= 0) return;
	tombstone_kernel<<<dim3((n + 255) / 256), dim3(256), 0, st>>>(rowaux, slots, n);
}

__global__ void filter_rowaux_kernel(const float *__restrict__ src, const uint8_t *__restrict__ mask, int64_t n_slots,
                                     int64_t cap, float *__restrict__ dst) {
	const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (r >= cap) return;
#pragma unroll
	for (int c = 0; c < 4; ++c) dst[raix(r, c)] = src[raix(r, c)];
	if (r < n_slots && !mask[r]) dst[raix(r, 0)] = F_INF;
}

void launch_filter_rowaux(const float4 *src, const uint8_t *mask, int64_t n_slots, int64_t cap, float4 *dst,
                          hipStream_t st) {
	if (cap <= 0) return;
	filter_rowaux_kernel<<<dim3((unsigned)((cap + 255) / 256)), 256, 0, st>>>(
	    reinterpret_cast<const float *>(src), mask, n_slots, cap, reinterpret_cast<float *>(dst));
}

// ---------------------------------------------------------------------------
// queries
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prep_queries_kernel(const float *__restrict__ Q, int nq, int dim, int ld,
                                                           int metric, float max_alpha, float max_ux,
                                                           float *__restrict__ Qf, uint16_t *__restrict__ Qb,
                                                           float4 *__restrict__ qaux, int *__restrict__ zero3) {
	__shared__ double red[2][4];
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	if (zero3 && t < 3 && q < nq) zero3[t * nq + q] = 0;  // the search's status words
	double s2 = 0.0, e2 = 0.0;
	for (int i = t; i < ld; i += 256) {
		float v = (q < nq && i < dim) ? Q[(int64_t)q * dim + i] : 0.0f;
		Qf[(int64_t)q * ld + i] = v;
		uint16_t b = bf16_bits(v);
		// L2 / dot: the scan accumulates S*s directly (S = -2 / -1, a power of
		// two: bf16(S*v) == S*bf16(v) exactly), see scan_kernel's bound fold
		Qb[(int64_t)q * ld + i] =
		    metric == METRIC_L2 ? bf16_bits(-2.0f * v) : metric == METRIC_DOT ? bf16_bits(-v) : b;
		float e = v - __uint_as_float((uint32_t)b << 16);
		s2 += (double)v * v;
		e2 += (double)e * e;
	}
	s2 = wave_sum_f64(s2);
	e2 = wave_sum_f64(e2);
	if ((t & 63) == 0) {
		red[0][t >> 6] = s2;
		red[1][t >> 6] = e2;
	}
	__syncthreads();
	if (t != 0) return;
	s2 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
	e2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
	if (q >= nq) {
		qaux[q] = make_float4(0.f, 0.f, 0.f, 0.f);
		return;
	}
	const double u = U_BOUND;
	const double gamma = 2.0 * ld * u;  // accumulation of ld exact bf16 products in f32
	const double qn = sqrt(s2), eq = sqrt(e2);
	const double uq = (qn + eq) * (1.0 + 4.0 * u);
	// L2 / dot fold the row/query terms into the accumulator before the k
	// loop (scan_kernel): the ld/16 MFMA k-steps then each round at the
	// magnitude of the whole bound, not of the partial dot product, and
	// the slack's evaluation budget grows from 16 to ld/16 + 16 unit roundoffs
	// of the same magnitudes.
	const double ev = (double)ld / 16.0 + 16.0;
	float4 a;
	if (metric == METRIC_L2) {
		double slack = ev * u * ((double)max_alpha + s2 + 7.0 * (double)max_ux * uq) + 1e-30;
		a = make_float4(-2.0f, (float)(-2.0 * (1.0 + gamma) * uq), (float)(2.0 * qn), (float)(s2 - slack));
	} else if (metric == METRIC_DOT) {
		double slack = ev * u * (1.0 + 7.0 * (double)max_ux * uq) + 1e-30;
		a = make_float4(-1.0f, (float)(-(1.0 + gamma) * uq), (float)qn, (float)(1.0 - slack));
	} else {
		if (qn > 0.0) {
			double ruq = uq / qn * (1.0 + 4.0 * u);
			double slack = 16.0 * u * (2.0 + 7.0 * (double)max_ux * ruq) + 1e-30;
			a = make_float4((float)(-1.0 / qn), (float)(-(1.0 + gamma) * ruq), 0.0f, (float)(2.0 - slack));
		} else {
			a = make_float4(0.f, 0.f, 0.f, __builtin_nanf(""));  // undefined: exact fallback
		}
	}
	qaux[q] = a;
}

void launch_prep_queries(const float *Q, int nq, int dim, int ld, int nq_pad, int metric, float max_alpha,
                         float max_ux, float *Qf, uint16_t *Qb, float4 *qaux, int *zero3, hipStream_t st) {
	prep_queries_kernel<<<dim3(nq_pad), dim3(256), 0, st>>>(Q, nq, dim, ld, metric, max_alpha, max_ux, Qf, Qb,
	                                                           qaux, zero3);
}

// int8 scan queries, one scale for the whole batch (tiles_to_i8_kernel keeps one
// per row tile): v = q (l2, dot) or q/|q| (cosine), s_Q = max over the batch of
// max|v_i| / 127, q^ = rint(v / s_Q).  Pass 1 (query_absmax_kernel): per query
// (max|v_i|, |q|); pass 2: Qf as prep_queries; Qi = q^ in the first ld bytes of
// each 2*ld-byte row of the Qb buffer (so the retry gather copies it like a bf16
// row); per-query constants of the int8 bound:
//   LB = alpha + xn*B + ux*A + (s*sc)*S + C      (sc = s_T of the row's tile)
//   l2: S = -2 s_Q, A = -2|e_q|, B = -2|q|, C = |q|^2 - slack
//   dot: S = -s_Q, A = -|e_q|, B = -|q|, C = 1 - slack
//   cosine: S = -s_Q, A = -|e_q|, B = -1, C = 1 - slack   (normalised rows and query)
// S is the same for every query of the batch (scan8_kernel relies on it).
// slack: f32 evaluation of the five-term sum, every intermediate bounded by
// max_alpha + |q|^2 + 4 max_x (|q| + |e_q|) (max_x = max over rows of xn, ux).
// (max|v_i|, |q|) of query q by the block (all threads call; every thread gets
// the result): one code path for query_absmax_kernel and the fused prep, so
// both give the same bits
__device__ __forceinline__ float2 query_absmax_block(const float *__restrict__ Q, int q, int dim, int metric,
                                                     float *redm, double *reds) {
	const int t = threadIdx.x;
	float m = 0.f;
	double s2 = 0.0;
	for (int i = t; i < dim; i += 256) {
		const float v = Q[(int64_t)q * dim + i];
		m = fmaxf(m, fabsf(v));
		s2 += (double)v * v;
	}
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
	s2 = wave_sum_f64(s2);
	if ((t & 63) == 0) {
		redm[t >> 6] = m;
		reds[t >> 6] = s2;
	}
	__syncthreads();
	m = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
	const double qn = sqrt(reds[0] + reds[1] + reds[2] + reds[3]);
	__syncthreads();  // (redm / reds are reused by the next call)
	const float mv = metric == METRIC_COSINE ? (qn > 0.0 ? (float)((double)m / qn) : 0.f) : m;
	return make_float2(mv, (float)qn);
}

__global__ __launch_bounds__(256) void query_absmax_kernel(const float *__restrict__ Q, int nq, int dim, int metric,
                                                           float2 *__restrict__ qm) {
	__shared__ float redm[4];
	__shared__ double reds[4];
	const float2 r = query_absmax_block(Q, blockIdx.x, dim, metric, redm, reds);
	if (threadIdx.x == 0) qm[blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void prep_queries_i8_kernel(const float *__restrict__ Q, int nq, int dim, int ld,
                                                              int metric, float max_alpha, float max_x,
                                                              const float2 *__restrict__ qm,
                                                              float *__restrict__ Qf, int8_t *__restrict__ Qi,
                                                              float4 *__restrict__ qaux, int *__restrict__ zero3) {
	__shared__ double red[2][4];
	__shared__ float redm[4];
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	if (zero3 && t < 3 && q < nq) zero3[t * nq + q] = 0;
	// the batch scale: max over every query's max|v_i|
	float m = 0.f;
	double qn0 = 0.0;  // (|q| rounded to f32: only scales v below)
	if (qm) {
		for (int i = t; i < nq; i += 256) m = fmaxf(m, qm[i].x);
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
		if ((t & 63) == 0) redm[t >> 6] = m;
		__syncthreads();
		m = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
		if (q < nq) qn0 = (double)qm[q].y;
	} else {
		// fused (a few queries: one launch instead of two): every block computes
		// every query's (max|v_i|, |q|) itself, with query_absmax_kernel's code
		__shared__ double reds[4];
		for (int j = 0; j < nq; ++j) {
			const float2 r = query_absmax_block(Q, j, dim, metric, redm, reds);
			m = fmaxf(m, r.x);
			if (j == q) qn0 = (double)r.y;
		}
	}
	const bool cosine = metric == METRIC_COSINE;
	const float sq = m / 127.0f;
	const double inv = m > 0.f ? 127.0 / (double)m : 0.0;
	double s2 = 0.0, e2 = 0.0;
	for (int i = t; i < ld; i += 256) {
		const float x = (q < nq && i < dim) ? Q[(int64_t)q * dim + i] : 0.0f;
		Qf[(int64_t)q * ld + i] = x;
		const double v = (cosine && qn0 > 0.0) ? (double)x / qn0 : (double)x;
		const int qv = (int)fmin(127.0, fmax(-127.0, rint(v * inv)));
		Qi[(int64_t)q * ld * 2 + i] = (int8_t)qv;
		const double e = v - (double)sq * (double)qv;
		s2 += (double)x * x;
		e2 += e * e;
	}
	s2 = wave_sum_f64(s2);
	e2 = wave_sum_f64(e2);
	if ((t & 63) == 0) {
		red[0][t >> 6] = s2;
		red[1][t >> 6] = e2;
	}
	__syncthreads();
	if (t != 0) return;
	s2 = red[0][0] + red[0][1] + red[0][2] + red[0][3];
	e2 = red[1][0] + red[1][1] + red[1][2] + red[1][3];
	if (q >= nq) {
		qaux[q] = make_float4(0.f, 0.f, 0.f, 0.f);
		return;
	}
	const double u = U_BOUND, up = 1.0 + 4.0 * u;
	const double qn = sqrt(s2), qnu = qn * up;
	// cosine: v = q/|q| in f64 from an f32-rounded |q|; |e_q| (taken against the
	// true q/|q|) and |v| <= 1 + 2^-20 cover both roundings
	const double equ = sqrt(e2) * up + (cosine ? 0x1p-20 * (1.0 + sqrt(e2)) : 0.0);
	float4 a;
	if (metric == METRIC_L2) {
		const double slack = 16.0 * u * ((double)max_alpha + s2 + 4.0 * (double)max_x * (qnu + equ)) + 1e-30;
		a = make_float4(-2.0f * sq, (float)(-2.0 * equ), (float)(-2.0 * qnu), (float)(s2 - slack));
	} else if (metric == METRIC_DOT) {
		const double slack = 16.0 * u * (1.0 + 4.0 * (double)max_x * (qnu + equ)) + 1e-30;
		a = make_float4(-sq, (float)(-equ), (float)(-qnu), (float)(1.0 - slack));
	} else if (qn > 0.0) {
		const double vn = 1.0 + 0x1p-20;  // |q/|q|| with the quotient's rounding
		const double slack = 16.0 * u * (2.0 + 4.0 * (double)max_x * (vn + equ)) + 1e-30;
		a = make_float4(-sq, (float)(-equ), (float)(-vn * up), (float)(1.0 - slack));
	} else {
		a = make_float4(0.f, 0.f, 0.f, __builtin_nanf(""));  // undefined: exact fallback
	}
	qaux[q] = a;
}

void launch_prep_queries_i8(const float *Q, int nq, int dim, int ld, int nq_pad, int metric, float max_alpha,
                            float max_x, float2 *qm, float *Qf, uint16_t *Qb, float4 *qaux, int *zero3,
                            hipStream_t st) {
	// up to PREP_FUSE_Q queries (DuckDB's one query per call): one launch, each
	// block reading the few query rows itself
	constexpr int PREP_FUSE_Q = 8;
	const bool fuse = nq <= PREP_FUSE_Q;
	if (nq > 0 && !fuse) query_absmax_kernel<<<dim3(nq), dim3(256), 0, st>>>(Q, nq, dim, metric, qm);
	prep_queries_i8_kernel<<<dim3(nq_pad), dim3(256), 0, st>>>(Q, nq, dim, ld, metric, max_alpha, max_x,
	                                                              fuse ? nullptr : qm, Qf,
	                                                              reinterpret_cast<int8_t *>(Qb), qaux, zero3);
}

constexpr int BR = SCAN_BR, BQ = SCAN_BQ;

// ---------------------------------------------------------------------------
// scan kernel (persistent, LDS-DMA ring)
//
// Tile = 256 base rows x 256 queries.  Workgroup = 512 threads = 8 waves, two
// per SIMD, laid out 4 (base rows) x 2 (queries): a wave owns 64 rows x 128
// queries = 2 x 4 v_mfma_f32_32x32x16_bf16 tiles (128 accumulator registers;
// A = base rows, B = queries: accumulator column = lane&31 = query, the 16
// registers walk base rows).  One workgroup per CU walks tiles blockIdx.x,
// +gridDim.x, ...; the k-stream never stops at a tile boundary.
//
// The k dimension streams in stages of SK = 32 through a ring of NST LDS
// slots, straight from HBM by global_load_lds_dwordx4 (no VGPR staging):
//   X stage: 256 rows x 32 base elements: f32 store 32 KiB (rows 128 B, chunk
//            c of row r at c ^ ((r>>1)&7), nt policy: read once), 3 slots;
//            bf16 store 16 KiB (rows 64 B, chunk c at c ^ ((r>>2)&3)), 4 slots;
//   Q stage: 256 queries x 32 bf16 (16 KiB, L2-resident), rows 64 B, chunk c at
//            c ^ ((r>>2)&3);
//   with stage 0 of a tile: the tile's row-aux block (4 KiB SoA, 2 slots).
// LDS-DMA writes lane-linearly, so the swizzle is applied on the per-lane
// SOURCE address and undone on the ds_read_b128 fragment reads (conflict-free
// per 16-lane group).  f32 A fragments are converted to bf16 after the read.
// Stage g is computed while stages g+1 .. g+NST-1 stream; one raw s_barrier
// per stage behind a counted s_waitcnt vmcnt.  The store is zero-padded (rows)
// and +inf-padded (row aux) to a multiple of BR rows, so no row is clamped.
//
// L2 / dot fold the bound: each tile's accumulators start at the row/query
// terms alpha + C + xn*B + ux*A (two exact f32 MFMAs) and the bf16 MFMAs add
// S*s (queries pre-scaled by S): at the tile end the accumulator IS the
// rigorous lower bound.  Dense mode stores it; append mode keeps (LB, row)
// when LB <= tau[q]: one ballot per bound, survivors appended to the wave's
// LDS list, written out at the next stage ahead of that stage's DMA.
// ---------------------------------------------------------------------------
// Development-only ablation switches (timing experiments; results are WRONG
// when set).  A release build refuses them: only tools/ablate.sh, which also
// defines LHIP_ABLATION_BUILD, may turn them on.
#if !defined(LHIP_ABLATION_BUILD) &&                                                                        \
    (defined(LHIP_ABL_NO_EPILOGUE) || defined(LHIP_ABL_NO_MFMA) || defined(LHIP_ABL_NO_READS) ||             \
     defined(LHIP_ABL_NO_QDMA) || defined(LHIP_ABL_NO_SLOW) || defined(LHIP_ABL_SLOW_NEVER) ||               \
     defined(LHIP_ABL_DRAIN_EPI) || defined(LHIP_ABL_NO_LISTWRITE) || defined(LHIP_ABL_NO_FLUSH) ||          \
     defined(LHIP_ABL_SMALL_NOWGSORT) || defined(LHIP_ABL_SMALL_NOMERGE) || defined(LHIP_ABL_SMALL_NOFENCE) || \
     defined(LHIP_ABL_PR_NOMERGE) || defined(LHIP_PROF))
#error "LHIP_ABL_* / LHIP_PROF are timing ablations that break results: build them through tools/ablate.sh"
#endif
#ifndef LHIP_ABL_NO_EPILOGUE
#define LHIP_ABL_NO_EPILOGUE 0
#endif
#ifndef LHIP_ABL_PR_NOMERGE
#define LHIP_ABL_PR_NOMERGE 0  // pool_refine: no top-k merge after a round (timing only)
#endif

#ifndef LHIP_ABL_NO_MFMA
#define LHIP_ABL_NO_MFMA 0  // fragments read, no MFMA
#endif
#ifndef LHIP_ABL_NO_READS
#define LHIP_ABL_NO_READS 0  // no fragment reads (MFMAs on stale registers)
#endif
#ifndef LHIP_ABL_NO_QDMA
#define LHIP_ABL_NO_QDMA 0  // query stages are not streamed (stale LDS)
#endif
#ifndef LHIP_ABL_NO_SLOW
#define LHIP_ABL_NO_SLOW 0  // survivors are tested but not written
#endif
#ifndef LHIP_ABL_SLOW_NEVER
#define LHIP_ABL_SLOW_NEVER 0  // survivor path compiled in, never taken (runtime-false guard)
#endif
#ifndef LHIP_SLOW_UNROLL
#define LHIP_SLOW_UNROLL 0  // survivor path: 16 unrolled uniform branches instead of mask loop + switch
#endif
#ifndef LHIP_ABL_DRAIN_EPI
#define LHIP_ABL_DRAIN_EPI 0  // drain the DMA in flight before each epilogue
#endif
#ifndef LHIP_ABL_NO_LISTWRITE
#define LHIP_ABL_NO_LISTWRITE 0  // survivor path runs, its LDS list writes do not
#endif
#ifndef LHIP_DEFER_LIST
#define LHIP_DEFER_LIST 0  // measured slower (C2 0.49-0.50 vs 0.47 ms): survivor list writes at the next wait point
#endif
#ifndef LHIP_SLOW_VALU
#define LHIP_SLOW_VALU 1  // survivor path: per-lane first hit by vector selects, one ballot + mbcnt
#endif
#ifndef LHIP_ABL_NO_FLUSH
#define LHIP_ABL_NO_FLUSH 0  // survivor lists are not written out
#endif
// development-only phase timer: per-wave s_memtime cycles in the DMA wait, the
// barrier, the stage's fragment reads + MFMA issue and the epilogue, summed over
// all waves into lhip_prof[MODE*8 + 0..3] ([4] waves, [5] stages, [6] tiles)
#ifndef LHIP_PROF
#define LHIP_PROF 0
#endif
#ifndef LHIP_NST_BF16_32
#define LHIP_NST_BF16_32 3  // ring slots of a 32-deep bf16 stage (3 or 4)
#endif
#ifndef LHIP_PRIO_HI_HALF
#define LHIP_PRIO_HI_HALF 0  // s_setprio 1 on waves 4..7 (the second-dispatched half) for the whole kernel
#endif
#if LHIP_PROF
__device__ unsigned long long lhip_prof[24];
extern "C" int lhip_prof_read(unsigned long long *out, int reset) {
	if (hipMemcpyFromSymbol(out, HIP_SYMBOL(lhip_prof), sizeof(unsigned long long) * 24) != hipSuccess) return -1;
	if (reset) {
		unsigned long long z[24] = {};
		if (hipMemcpyToSymbol(HIP_SYMBOL(lhip_prof), z, sizeof(z)) != hipSuccess) return -1;
	}
	return 0;
}
#define PROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#else
#define PROF_T(v)
#endif
#ifndef LHIP_X_NT
#define LHIP_X_NT 0  // nt on the base stream: measured slower (bf16 scan 0.59 vs 0.525 ms)
#endif
#ifndef LHIP_SK_BF16
#define LHIP_SK_BF16 64  // k per stage with a bf16 base: 64 (2 slots) or 32 (3 slots)
#endif
#ifndef LHIP_I8_TFOLD
#define LHIP_I8_TFOLD 1  // int8 append pass: fold the bound into the accumulators (convert + scale + two f32 MFMAs) before the screen
#endif
#ifndef LHIP_PF
#define LHIP_PF 0  // bf16 base: each stage issue also touches the rows of the stage this many ahead into L2 (0 = off)
#endif

constexpr int SCAN_THREADS = 512;
constexpr int SCAN_WAVES = SCAN_THREADS / 64;          // 8: 2 per SIMD, 256 registers each
constexpr int RA_SLOT = BR * 16;                       // 4 KiB
constexpr int RA_BYTES = 2 * RA_SLOT;
constexpr int CNT_BYTES = BQ * 4;
constexpr int QA_BYTES = BQ * 16 + BQ * 4;             // per-query bound constants + tau
static_assert(RA_SLOT / 1024 == 4 && SCAN_WAVES >= 4, "row aux: one DMA instruction on waves 0..3");
static_assert(SCAN_WAVES == 8, "8 waves: 4 row quarters x 2 query halves");

// per scanned element type XT: 0 = f32 store, 1 = bf16 store / scan copy,
// 2 = int8 scan copy (per-row scale; int8 queries, v_mfma_i32_32x32x32_i8)
template <int XT>
struct ScanCfg {
	static constexpr bool XB = XT != 0;                        // 16 B operand chunks straight from LDS
	static constexpr bool I8 = XT == 2;
	static constexpr int SK = I8 ? 128 : XB ? LHIP_SK_BF16 : 32;  // k per stage
	static constexpr int KQ = SK / (I8 ? 32 : 16);             // MFMA k-steps per stage: 4 / 4 / 2
	static constexpr int XE = I8 ? 1 : XB ? 2 : 4;             // bytes per base element
	static constexpr int XROW = SK * XE;                       // bytes per row and stage: 128
	static constexpr int XCH = XROW / 16;                      // 16 B chunks per row
	static constexpr int XST = BR * XROW;                      // 32 KiB
	static constexpr int QE = I8 ? 1 : 2;                      // bytes per query element
	static constexpr int QROW = SK * QE;                       // bytes per query and stage: 128 / 64
	static constexpr int QCH = QROW / 16;
	static constexpr int QST = BQ * QROW;                      // 32 / 16 KiB
	static constexpr int NST = XB ? (SK == 64 || I8 ? 2 : LHIP_NST_BF16_32) : 3;  // ring slots
	static constexpr int STAGE = XST + QST;
	static constexpr int RING = NST * STAGE;                   // 128 / 144 KiB
	static constexpr int XDMA = XST / 1024 / SCAN_WAVES;       // X DMA instructions per wave and stage
	static constexpr int QDMA = QST / 1024 / SCAN_WAVES;       // Q DMA instructions per wave and stage
	static constexpr int ROWS_PER_DMA = 1024 / XROW;
	static constexpr int QROWS_PER_DMA = 1024 / QROW;
	// L2 prefetch distance in stages (bf16 rows only): one touch instruction per
	// wave and stage issue, the youngest instruction of its issue group
	static constexpr int PF = XB ? LHIP_PF : 0;
	static constexpr int TCH = PF > 0 ? 1 : 0;
	static constexpr int PF_BYTES = TCH * 1024;  // the touches' scratch (16 B per lane, shared by the waves)
	static constexpr int DMA = XDMA + (LHIP_ABL_NO_QDMA ? 0 : QDMA) + TCH;  // + 1 row aux on waves 0..3 at a tile's stage 0
	// survivor list per wave (8 B entries): f32 32, flushed after every tile by
	// one counted store; bf16 256, kept across tiles and flushed (drained)
	// only past FLUSH_AT entries, or at the end
	static constexpr int WLIST = XB ? 256 : 32;
	static constexpr int FLUSH_AT = XB ? WLIST - 64 : 0;
	static constexpr int LIST_BYTES = SCAN_WAVES * WLIST * 8;
	static constexpr int LDS = RING + RA_BYTES + CNT_BYTES + QA_BYTES + LIST_BYTES + PF_BYTES;
	static_assert(LDS <= 160 * 1024, "LDS budget");
	static_assert(XDMA * SCAN_WAVES * 1024 == XST && QDMA * SCAN_WAVES * 1024 == QST, "stages = whole DMA instructions");
	static_assert((XROW == 128 || XROW == 64) && (QROW == 128 || QROW == 64), "swizzles below");
	static_assert(XB || SK == 32, "f32 fragments: 2 k-steps per stage");
	static_assert(KQ % 2 == 0, "k-step fragments alternate between two register sets");
	// 16 B chunk c of row r lives at physical chunk xswz(r, c) (an involution):
	// conflict-free ds_read_b128 fragment reads on 128 B (64 B) rows
	__device__ static __forceinline__ int xswz(int r, int c) { return XROW == 128 ? c ^ ((r >> 1) & 7) : c ^ ((r >> 2) & 3); }
	__device__ static __forceinline__ int qswz(int r, int c) { return QROW == 128 ? c ^ ((r >> 1) & 7) : c ^ ((r >> 2) & 3); }
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int METRIC, bool SC = false>
__device__ __forceinline__ float lower_bound(float s, float4 ra, float4 qa) {
	// LB = alpha + xn*B + ux*A + (s*sc)*S + C   (sc: cosine 1/|x|, int8 scan the row scale)
	float v = fmaf(ra.y, qa.z, ra.x);
	v = fmaf(ra.z, qa.y, v);
	float ss = (METRIC == METRIC_COSINE || SC) ? s * ra.w : s;
	v = fmaf(ss, qa.x, v);
	return v + qa.w;
}

// One global_load_lds_dwordx4: 64 lanes x 16 B land lane-linearly at the
// wave-uniform LDS byte address in M0.  Issued through inline asm so the
// compiler does not see an LDS write in flight: it would otherwise put a
// vmcnt(0) in front of every ds_read of the ring (any stage may alias) and
// serialise the pipeline.  Ordering is ours: counted vmcnt + s_barrier.
// M0 is written here and nowhere else in the kernel.  saddr form: wave-uniform
// 64-bit base in SGPRs + 32-bit per-lane byte offset.
template <bool NT = false>
__device__ __forceinline__ void dma16s(const void *sbase, uint32_t voff, uint32_t lds_addr) {
	// readfirstlane returns int: go through uint32_t so the low word is not
	// sign-extended into the high word of the address
	const uint64_t b = (uint64_t)(uintptr_t)sbase;
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
	const uint64_t ub = ((uint64_t)hi << 32) | (uint64_t)lo;
	// s_nop 4: the base may come straight from v_readfirstlane (a VALU write of
	// an SGPR that the VMEM below reads: the compiler cannot see through the asm);
	// s_nop 0: the M0 write -> LDS-DMA hazard
	if (NT)
		asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt" ::"s"(lds_addr),
		             "v"(voff), "s"(ub)
		             : "memory", "m0");
	else
		asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr),
		             "v"(voff), "s"(ub)
		             : "memory", "m0");
}

// L2 prefetch touch: one global_load_lds_dwordx4 (16 B per lane into scratch
// LDS nobody reads) pulls the 64 B sector of each lane's address into L2
// (and L1) without holding a VGPR: a dead VGPR destination would be written
// back whenever the load returned, after the compiler had reused the register.
// s_nop 4: the base may be fresh from v_readfirstlane (VALU SGPR write -> VMEM
// read); s_nop 0: the M0 write -> LDS-DMA hazard (else the load may take the
// previous M0, the last ring DMA's slot, and overwrite 1 KiB of it).  The same
// dwordx4 form as the ring DMA: a global_load_lds_dword touch in the same vmcnt
// stream gave wrong bounds (measured: counted waits no longer covered the ring).
__device__ __forceinline__ void touch4s(const void *sbase, uint32_t voff, uint32_t lds_addr) {
	const uint64_t b = (uint64_t)(uintptr_t)sbase;
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
	const uint64_t ub = ((uint64_t)hi << 32) | (uint64_t)lo;
	asm volatile("s_nop 4\n\ts_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr), "v"(voff), "s"(ub)
	             : "memory", "m0");
}

#define LHIP_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

template <int N>
__device__ __forceinline__ void wait_vm_c() {
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// s_waitcnt vmcnt takes an immediate: dispatch the counts that can occur
__device__ __forceinline__ void wait_vm(int n) {
	switch (n) {
	case 0: LHIP_WAIT_VM(0); break;
	case 1: LHIP_WAIT_VM(1); break;
	case 2: LHIP_WAIT_VM(2); break;
	case 3: LHIP_WAIT_VM(3); break;
	case 4: LHIP_WAIT_VM(4); break;
	case 5: LHIP_WAIT_VM(5); break;
	case 6: LHIP_WAIT_VM(6); break;
	case 7: LHIP_WAIT_VM(7); break;
	case 8: LHIP_WAIT_VM(8); break;
	case 9: LHIP_WAIT_VM(9); break;
	case 10: LHIP_WAIT_VM(10); break;
	case 11: LHIP_WAIT_VM(11); break;
	case 12: LHIP_WAIT_VM(12); break;
	case 13: LHIP_WAIT_VM(13); break;
	case 14: LHIP_WAIT_VM(14); break;
	case 15: LHIP_WAIT_VM(15); break;
	case 16: LHIP_WAIT_VM(16); break;
	default: LHIP_WAIT_VM(0); break;  // (not reached) conservative
	}
}

// Lane id that is not loop-invariant to the compiler, so values derived from
// it are recomputed where used instead of hoisted out of the tile loop and kept
// live across the MFMA loop.  The mbcnt instructions are the compiler's own
// (builtins): it pads their hazards.  They once sat inside the asm string,
// where nothing is padded: the v_mbcnt could overwrite a VGPR that the tile's
// last, still executing MFMA was reading as its A operand (register allocation
// put the lane id there in the cosine kernels), which corrupted one 32 x 32
// accumulator block now and then — wrong cosine bounds in ~1% of the queries.
// Only the all-ones mask goes through an (empty) asm statement, as an SGPR.
__device__ __forceinline__ int lane_id_fresh() {
	uint32_t m = 0xFFFFFFFFu;
	asm volatile("" : "+s"(m));
	return (int)__builtin_amdgcn_mbcnt_hi(m, __builtin_amdgcn_mbcnt_lo(m, 0u));
}

template <int METRIC, int MODE, int XT>
__global__ __launch_bounds__(SCAN_THREADS, 1) void scan_kernel(const void *__restrict__ Xv,
                                                               const float4 *__restrict__ rowaux, int ld,
                                                               const uint16_t *__restrict__ Qb,
                                                               const float4 *__restrict__ qaux, int nq,
                                                               int n_tiles, int tile_stride,
                                                               float *__restrict__ dense, int64_t ld_out,
                                                               const float *__restrict__ tau,
                                                               uint2 *__restrict__ seg_pool,
                                                               int *__restrict__ seg_cnt, int seg_cap) {
	using C = ScanCfg<XT>;
	constexpr bool XB = C::XB, I8 = C::I8;
	__shared__ __attribute__((aligned(16))) uint8_t smem[C::LDS];
	unsigned *CNT = reinterpret_cast<unsigned *>(smem + C::RING + RA_BYTES);
	float4 *QA = reinterpret_cast<float4 *>(smem + C::RING + RA_BYTES + CNT_BYTES);
	float *TAU = reinterpret_cast<float *>(smem + C::RING + RA_BYTES + CNT_BYTES + BQ * 16);
	uint2 *LIST = reinterpret_cast<uint2 *>(smem + C::RING + RA_BYTES + CNT_BYTES + QA_BYTES);
	const uint8_t *X = reinterpret_cast<const uint8_t *>(Xv);

	const int tid = threadIdx.x;
	[[maybe_unused]] const int lane = tid & 63;
	const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: SGPR math
	const int wr = w & 3, wq = w >> 2;                      // 64-row quarter, 128-query half
	if (LHIP_PRIO_HI_HALF && w >= 4) __builtin_amdgcn_s_setprio(1);
	const int q0 = blockIdx.y * BQ;
	const int S = ld / C::SK;  // >= 1 (ld is a multiple of 64)
	const int my_tiles = (n_tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
	const int G = my_tiles * S;

	// per-query constants of this query tile -> LDS (read in the epilogues)
	if (tid < BQ) {
		const int q = q0 + tid;
		QA[tid] = qaux[q];
		TAU[tid] = (MODE == 1 && q < nq) ? tau[q] : -F_INF;
		if (MODE >= 1) CNT[tid] = 0u;
	}
	LHIP_WAIT_VM(0);  // the ordinary loads above, before any counted DMA wait
	__syncthreads();

	// DMA sources.  X: wave instruction j covers rows (XDMA*w+j)*ROWS_PER_DMA +
	// lane/XCH, physical chunk lane%XCH.  Q: instruction j covers queries
	// (2w+j)*16 + lane/4, physical chunk lane%4.  Row aux (stage 0 only): waves
	// 0..3, rows w*64 + lane.  The per-lane source offsets are loop-invariant
	// (VGPRs, computed once); the wave-uniform parts — source pointers of the
	// next stage to issue and its LDS slot — run in SGPRs and advance by
	// constants, so a stage's issue costs a handful of scalar instructions.
	const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
	uint32_t xoff[C::XDMA], qoff[C::QDMA];
#pragma unroll
	for (int j = 0; j < C::XDMA; ++j) {
		const int xr = (C::XDMA * w + j) * C::ROWS_PER_DMA + lane / C::XCH;
		const int c = C::xswz(xr, lane % C::XCH);  // 16 B source chunk of the stage's SK bytes
		// int8: k-major tiles (tiles_to_i8_kernel): 64-B chunk c / 4 of the stage
		xoff[j] = I8 ? (uint32_t)((c >> 2) * I8_CHUNK_STRIDE + xr * 64 + ((c & 3) << 4))
		             : (uint32_t)(xr * ld * C::XE + (c << 4));
	}
#pragma unroll
	for (int j = 0; j < C::QDMA; ++j) {
		const int qr = (C::QDMA * w + j) * C::QROWS_PER_DMA + lane / C::QCH;
		qoff[j] = (uint32_t)(qr * ld * 2 + (C::qswz(qr, lane % C::QCH) << 4));  // query rows: 2*ld bytes apart
	}
	const uint32_t raoff = (uint32_t)lane * 16u;
	const int64_t tile_rows_step = (int64_t)gridDim.x * tile_stride * BR;  // rows between this workgroup's tiles
	const uint8_t *qbase = reinterpret_cast<const uint8_t *>(Qb + (int64_t)q0 * ld);
	const uint8_t *iss_xtile = X + (int64_t)blockIdx.x * tile_stride * BR * ld * C::XE;
	const uint8_t *iss_xt = iss_xtile;
	const float4 *iss_ra = rowaux + (int64_t)blockIdx.x * tile_stride * BR;
	const uint8_t *iss_q = qbase;
	uint32_t iss_lds = lds0;  // LDS slot of the next stage to issue
	int iss_g = 0, iss_s = 0, iss_t = 0;
	// Prefetch cursor: stage iss_g + PF (held at the last stage near the end,
	// so every issue group has the same instruction count).  Lane -> row
	// w*32 + lane%32, 64 B half lane/32 of the row's 128 B stage piece.
	const uint8_t *pf_xtile = iss_xtile, *pf_xt = iss_xt;
	int pf_g = 0, pf_s = 0;
	auto pf_adv = [&]() {
		if (pf_g + 1 >= G) return;
		++pf_g;
		if (++pf_s == S) {
			pf_s = 0;
			pf_xtile += tile_rows_step * ld * C::XE;
			pf_xt = pf_xtile;
		} else {
			pf_xt += C::SK * C::XE;
		}
	};
	for (int i = 0; i < C::PF; ++i) pf_adv();
	const uint32_t pfoff = (uint32_t)((w * 32 + (lane & 31)) * ld * C::XE + (lane >> 5) * 64);
	const uint32_t pf_lds = lds0 + (uint32_t)(C::LDS - C::PF_BYTES);
	auto issue_one = [&]() {
		if (iss_s == 0 && w < 4)
			dma16s(iss_ra + w * 64, raoff, lds0 + C::RING + (uint32_t)(iss_t & 1) * RA_SLOT + (uint32_t)w * 1024u);
#pragma unroll
		for (int j = 0; j < C::XDMA; ++j)
			dma16s<LHIP_X_NT>(iss_xt, xoff[j], iss_lds + (uint32_t)(C::XDMA * w + j) * 1024u);
#pragma unroll
		for (int j = 0; j < (LHIP_ABL_NO_QDMA ? 0 : C::QDMA); ++j)
			dma16s(iss_q, qoff[j], iss_lds + (uint32_t)C::XST + (uint32_t)(C::QDMA * w + j) * 1024u);
		if (C::TCH) {
			touch4s(pf_xt, pfoff, pf_lds);
			pf_adv();
		}
		++iss_g;
		iss_lds = iss_lds + C::STAGE == lds0 + C::RING ? lds0 : iss_lds + C::STAGE;
		if (++iss_s == S) {
			iss_s = 0;
			++iss_t;
			iss_xtile += tile_rows_step * ld * C::XE;
			iss_xt = iss_xtile;
			iss_ra += tile_rows_step;
			iss_q = qbase;
		} else {
			iss_xt += I8 ? (C::SK / 64) * I8_CHUNK_STRIDE : C::SK * C::XE;
			iss_q += C::SK * C::QE;
		}
	};

	// accumulators: acc[t][u] = rows wr*64 + 32t + (reg layout), queries wq*128 + 32u + lane&31.
	// Set at each tile's stage 0: L2 / dot start from the bound's row/query
	// terms (FOLD: alpha + C + xn*B + ux*A by two exact f32 MFMAs) and the
	// bf16 MFMAs add S*s (queries pre-scaled by S), so at the tile end the
	// accumulator IS the lower bound; cosine (per-row scale) starts at 0.
	// (int8: integer accumulators, scaled per row in the epilogue; kept as f32x16 bits)
	constexpr bool FOLD = METRIC != METRIC_COSINE && !I8;
	constexpr bool SCL = METRIC == METRIC_COSINE || I8;  // epilogue multiplies the dot product by the row's sc
	f32x16 acc[2][4];
	auto accf = [&](int t, int u, int r) -> float {
		return I8 ? (float)__float_as_int(acc[t][u][r]) : acc[t][u][r];
	};
	auto init_acc = [&](int ti) {
		if (!FOLD) {
#pragma unroll
			for (int t = 0; t < 2; ++t)
#pragma unroll
				for (int u = 0; u < 4; ++u)
#pragma unroll
					for (int r = 0; r < 16; ++r) acc[t][u][r] = 0.f;
			return;
		}
		const float *RAs = reinterpret_cast<const float *>(smem + C::RING + (ti & 1) * RA_SLOT);
		const int ln = lane_id_fresh();
		const int li = ln & 31, hk = ln >> 5;  // f32 32x32x2 operands: lane = (row or column, k)
		f32x16 zero;
#pragma unroll
		for (int r = 0; r < 16; ++r) zero[r] = 0.f;
		float bq[4], cq[4];
#pragma unroll
		for (int u = 0; u < 4; ++u) {
			const float4 qa = QA[wq * 128 + 32 * u + li];
			bq[u] = hk ? qa.y : qa.z;  // k0: B, k1: A
			cq[u] = hk ? qa.w : 1.0f;  // k0: 1, k1: C
		}
#pragma unroll
		for (int t = 0; t < 2; ++t) {
			const int r = wr * 64 + 32 * t + li;
			const float axu = RAs[(1 + hk) * BR + r];  // k0: xn, k1: ux
			const float aal = hk ? 1.0f : RAs[r];     // k0: alpha, k1: 1
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(axu, bq[u], zero, 0, 0, 0);
				acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(aal, cq[u], acc[t][u], 0, 0, 0);
			}
		}
	};

	// Stage h may be issued once every wave is done reading stage h-NST (its
	// slot), i.e. after the barrier of iteration h-NST; and a tile's stage 0
	// (which carries its row aux into RA slot tile&1) only once every wave is
	// past the epilogue of tile-2 (matters when S < NST; see the end of the loop).
	int tiles_done = 0;
	const bool ra_wave = w < 4;  // waves that issue a row-aux DMA with a tile's stage 0
	auto pump = [&](int limit) {
		while (iss_g < G && iss_g <= limit && !(iss_s == 0 && iss_t >= tiles_done + 2)) issue_one();
	};
	// s_waitcnt vmcnt for "stage h landed": this wave's DMA instructions of the
	// m = iss_g-1-h stages issued after it may stay in flight — DMA each, +1 on
	// waves 0..3 for each of them that is a tile's stage 0 (sh = in-tile index
	// of stage h).  The steady-state counts are immediates.
	// List flush stores: fpos1/fpos2 = iss_g when the latest two were issued
	// (a store is younger than stage h iff its fpos > h).
	int fpos1 = -1, fpos2 = -1;
	auto fl_younger = [&](int h) { return (fpos1 > h ? 1 : 0) + (fpos2 > h ? 1 : 0); };
	auto wait_stage = [&](int h, int sh) {
		// (+ TCH: stage h's own prefetch touch is issued after its DMA)
		const int m = iss_g - 1 - h;
		if (m <= 0) {
			wait_vm(C::TCH + fl_younger(h));
			return;
		}
		const int d0 = S - 1 - sh;  // stages after h up to the next tile start, exclusive
		const int n0 = ra_wave ? (d0 < m) + (d0 + S < m) : 0;
		wait_vm(m * C::DMA + C::TCH + n0 + fl_younger(h));
	};

	// This wave's survivor list: n_list entries (wave-uniform), possibly of
	// several tiles.  Entry = (raw LB bits, query << 24 | tile row << 16 |
	// tile iteration).  Written out with segment positions from the per-query
	// LDS counters.  A list of <= 64 entries goes out as exactly ONE
	// global_store_dwordx2 of all 64 lanes (lanes without an entry, or past
	// the segment capacity, write the workgroup's sink word past the
	// segments), which the DMA waits count (issued after the stage's DMA, it
	// never has to complete before a stage can be read); a longer list is
	// written by plain stores and drained.
	uint2 *wlist = LIST + w * C::WLIST;
	int n_list = 0;
	uint2 *const sink = seg_pool + (int64_t)gridDim.x * nq * seg_cap + (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
	auto entry_out = [&](uint2 e, uint2 *&dst, uint2 &val) {
		const int qloc = (int)(e.y >> 24), rloc = (int)((e.y >> 16) & 255u), ti = (int)(e.y & 0xFFFFu);
		const unsigned p = atomicAdd(&CNT[qloc], 1u);
		if (p < (unsigned)seg_cap) {
			const int64_t prow0 = ((int64_t)blockIdx.x + (int64_t)ti * gridDim.x) * tile_stride * BR;
			dst = seg_pool + ((int64_t)blockIdx.x * nq + q0 + qloc) * seg_cap + p;
			val = make_uint2(fkey(__uint_as_float(e.x)), (uint32_t)(prow0 + rloc));
		}
	};
	auto write_list_one = [&]() {  // n_list <= 64
		const int ln = lane_id_fresh();
		uint2 *dst = sink;
		uint2 val = make_uint2(0u, 0u);
		if (ln < n_list) entry_out(wlist[ln], dst, val);
		const uint64_t v64 = (uint64_t)val.x | ((uint64_t)val.y << 32);
		asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(dst), "v"(v64) : "memory");
		n_list = 0;
	};
	auto write_list_all = [&]() {
		const int ln = lane_id_fresh();
		for (int b = 0; b < n_list; b += 64) {
			if (b + ln < n_list) {
				uint2 *dst = nullptr;
				uint2 val;
				entry_out(wlist[b + ln], dst, val);
				if (dst) *dst = val;
			}
		}
		n_list = 0;
	};
	// a bound whose survivors do not fit the wave's list: straight to the
	// segment (position from the LDS counter); out of line, rare
	// per-lane form: each active lane its own (bound, query, row)
	auto overflow_lane = [&](bool act, float lb, int qv, int rr, int64_t row0) {
		if (act) {
			const unsigned p = atomicAdd(&CNT[qv], 1u);
			if (p < (unsigned)seg_cap)
				seg_pool[((int64_t)blockIdx.x * nq + q0 + qv) * seg_cap + p] = make_uint2(fkey(lb), (uint32_t)(row0 + rr));
		}
		LHIP_WAIT_VM(0);
	};
	// (its store is not counted by the DMA waits: drained right away)
	auto overflow = [&](uint64_t mm, float lb, int qv, int rr, int64_t row0) {
		if ((mm >> lane_id_fresh()) & 1ull) {
			const unsigned p = atomicAdd(&CNT[qv], 1u);
			if (p < (unsigned)seg_cap)
				seg_pool[((int64_t)blockIdx.x * nq + q0 + qv) * seg_cap + p] = make_uint2(fkey(lb), (uint32_t)(row0 + rr));
		}
		LHIP_WAIT_VM(0);
	};
	// Fragments of one 16-deep k-step of a stage: A raw (f32: two 16 B reads
	// per fragment, converted at use; bf16: one), B bf16.  Two sets alternate:
	// k-step j's MFMAs run while k-step j+1 loads.
	struct Frag {
		float4 a[2][2];  // [t][lo/hi] raw 16 B reads (bf16: [t][0] only)
		bf16x8 b[4];
	};
	// Per-lane fragment byte offsets inside a stage.  Row r's chunk c sits at
	// physical chunk c ^ f(r) and f is the same for r and r + 32, so every
	// fragment of k-step kq is one base XOR (kq << 5) (f32: two chunks per
	// fragment, kq << 6, the second chunk ^ 16) plus an immediate per 32-row
	// (32-query) block.
	uint32_t abase, bbase;
	{
		const int r = wr * 64 + (lane & 31), hh = lane >> 5;
		abase = (uint32_t)(r * C::XROW + (C::xswz(r, XB ? hh : 2 * hh) << 4));
		const int q = wq * 128 + (lane & 31);
		bbase = (uint32_t)(C::XST + q * C::QROW + (C::qswz(q, hh) << 4));
	}
	auto read_k = [&](Frag &f, const uint8_t *st_base, int kq) {
		if (LHIP_ABL_NO_READS) {
			float4 z;
			bf16x8 zb;
			asm volatile("" : "=v"(z));
			asm volatile("" : "=v"(zb));
#pragma unroll
			for (int t = 0; t < 2; ++t) f.a[t][0] = f.a[t][1] = z;
#pragma unroll
			for (int u = 0; u < 4; ++u) f.b[u] = zb;
			return;
		}
		const uint32_t ao = abase ^ ((uint32_t)kq << (XB ? 5 : 6));
#pragma unroll
		for (int t = 0; t < 2; ++t) {
			f.a[t][0] = *reinterpret_cast<const float4 *>(st_base + ao + t * 32 * C::XROW);
			if (!XB) f.a[t][1] = *reinterpret_cast<const float4 *>(st_base + (ao ^ 16u) + t * 32 * C::XROW);
		}
		const uint32_t bo = bbase ^ ((uint32_t)kq << 5);
#pragma unroll
		for (int u = 0; u < 4; ++u) f.b[u] = *reinterpret_cast<const bf16x8 *>(st_base + bo + u * 32 * C::QROW);
	};
	auto mfma_rows = [&](const Frag &f, int t_lo, int t_hi) {
#pragma unroll
		for (int t = t_lo; t < t_hi; ++t) {
			bf16x8 av;
			if (XB) {
				av = __builtin_bit_cast(bf16x8, f.a[t][0]);
			} else {
				const float4 lo = f.a[t][0], hi = f.a[t][1];
				av[0] = (__bf16)lo.x;
				av[1] = (__bf16)lo.y;
				av[2] = (__bf16)lo.z;
				av[3] = (__bf16)lo.w;
				av[4] = (__bf16)hi.x;
				av[5] = (__bf16)hi.y;
				av[6] = (__bf16)hi.z;
				av[7] = (__bf16)hi.w;
			}
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				if (LHIP_ABL_NO_MFMA)
					asm volatile("" ::"v"(av), "v"(f.b[u]));
				else if (I8)
					acc[t][u] = __builtin_bit_cast(
					    f32x16, __builtin_amdgcn_mfma_i32_32x32x32_i8(__builtin_bit_cast(i32x4, av),
					                                                  __builtin_bit_cast(i32x4, f.b[u]),
					                                                  __builtin_bit_cast(i32x16, acc[t][u]), 0, 0, 0));
				else
					acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, f.b[u], acc[t][u], 0, 0, 0);
			}
		}
	};
	auto mfma_k = [&](const Frag &f) { mfma_rows(f, 0, 2); };

	// prologue: stages 0 .. NST-1 in flight; (0, kk0) into registers
	pump(C::NST - 1);
	wait_stage(0, 0);
	__builtin_amdgcn_s_barrier();
	asm volatile("" ::: "memory");
	Frag F[2];
	read_k(F[0], smem, 0);

#if LHIP_PROF
	uint64_t pw = 0, pb = 0, pc = 0, pe = 0;
	uint64_t prof_surv = 0, prof_over = 0, prof_slow = 0, prof_slown = 0;
#endif
	// Survivor entries of the last epilogue, written into the list at the next
	// stage's wait point: an LDS write issued while this wave's own LDS-DMA is
	// in flight holds its later LDS accesses until that DMA lands (measured:
	// one stage of pipelining lost per tile), so the epilogue only reserves
	// the positions (ppos, -1 = none) and keeps the entries in registers.
	// (L2 / dot; cosine keeps its row terms live in the epilogue and writes at
	// once: the 24 registers would spill)
	constexpr bool DEFER = LHIP_DEFER_LIST && LHIP_SLOW_VALU && FOLD;
	int ppos[8];
	float psv[8];
	uint32_t ppl[8];
	bool pend = false;
	auto write_pending = [&]() {
#pragma unroll
		for (int gi = 0; gi < 8; ++gi)
			if (ppos[gi] >= 0) wlist[ppos[gi]] = make_uint2(__float_as_uint(psv[gi]), ppl[gi]);
		pend = false;
	};
	int cur_t = 0, cur_s = 0;
	const uint8_t *rd = smem;  // LDS slot of stage g
	for (int g = 0; g < G; ++g) {
		PROF_T(t0);
		const bool tile_end = cur_s + 1 == S;
		const uint8_t *rd_next = rd + C::STAGE == smem + C::RING ? smem : rd + C::STAGE;
		if (cur_s == 0) init_acc(cur_t);
		// (g, kq+1) loads while (g, kq) multiplies
#pragma unroll
		for (int kq = 0; kq + 1 < C::KQ; ++kq) {
			read_k(F[(kq + 1) & 1], rd, kq + 1);
			mfma_k(F[kq & 1]);
		}
		// stage g+1 must have landed (the stages issued after it may stay in
		// flight); this wave's reads of stage g are complete before the
		// barrier, so after it slot g % NST is free for stage g+NST
		if (iss_g == g + C::NST) {
			// steady state: stages g+2 .. g+NST-1 in flight after g+1; the one
			// extra DMA on waves 0..3 if one of them is a tile's stage 0
			static_assert(C::NST >= 2 && C::NST <= 4, "steady-state wait counts below");
			const bool st0 = C::NST >= 3 && (cur_s + 2 == S || (C::NST == 4 && (cur_s + 3 == S || (S == 2 && cur_s == 1))));
			switch ((ra_wave && st0 ? 1 : 0) + fl_younger(g + 1)) {
			case 0: wait_vm_c<(C::NST - 2) * C::DMA + C::TCH>(); break;
			case 1: wait_vm_c<(C::NST - 2) * C::DMA + C::TCH + 1>(); break;
			case 2: wait_vm_c<(C::NST - 2) * C::DMA + C::TCH + 2>(); break;
			default: wait_vm_c<(C::NST - 2) * C::DMA + C::TCH + 3>(); break;
			}
		} else if (g + 1 < G) {
			wait_stage(g + 1, tile_end ? 0 : cur_s + 1);  // the last stages, or a held-back issue
		}
		if (MODE == 1 && DEFER && pend) write_pending();
		asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
		PROF_T(t1);
		__builtin_amdgcn_s_barrier();
		asm volatile("" ::: "memory");
		PROF_T(t2);
		// stage g+NST into slot g % NST, then the survivor list of the tile
		// finished last iteration (its store younger than that DMA: counted)
		pump(g + C::NST);
		if (MODE == 1 && n_list > C::FLUSH_AT) {
			if (LHIP_ABL_NO_FLUSH) {
				n_list = 0;
			} else if (C::FLUSH_AT + 1 <= 64 && n_list <= 64) {
				write_list_one();
				fpos2 = fpos1;
				fpos1 = iss_g;
			} else {
				write_list_all();
				LHIP_WAIT_VM(0);  // rare: uncounted stores, drained here
			}
		}
		// (g+1, 0) loads while (g, KQ-1) multiplies (unconditional: on the
		// last stage it reads a stale, stable slot; the values are unused)
		read_k(F[0], rd_next, 0);
		mfma_k(F[1]);
		rd = rd_next;
		if (tile_end) mfma_operand_guard();  // the epilogue follows the tile's last MFMAs
		asm volatile("" ::: "memory");
		PROF_T(t3);
#if LHIP_PROF
		pw += t1 - t0;
		pb += t2 - t1;
		pc += t3 - t2;
#endif
		if (!tile_end) {
			++cur_s;
			continue;
		}
		cur_s = 0;
		const int ti = cur_t++;

		if (LHIP_ABL_DRAIN_EPI) LHIP_WAIT_VM(0);
		// ---- epilogue of tile ti (its row aux landed with its stage 0) ------
		const int64_t tile = (int64_t)blockIdx.x + (int64_t)ti * gridDim.x;
		const int64_t row0 = tile * tile_stride * BR;
		// row aux of the tile (SoA): alpha [0,256), xn [256,512), ux [512,768), sc [768,1024)
		const float *RAs = reinterpret_cast<const float *>(smem + C::RING + (ti & 1) * RA_SLOT);
		auto ra4 = [&](int r0, int c) { return *reinterpret_cast<const float4 *>(RAs + c * BR + r0); };
		const int eln = lane_id_fresh();
		const int qlb = wq * 128 + (eln & 31);  // tile-local query of acc[.][u]: qlb + 32u
		const int rb = wr * 64 + 4 * (eln >> 5); // tile-local row of acc[t][.] reg r: rb + 32t + (r&3) + 8(r>>2)
		// int8 (TFOLD): turn each integer accumulator block into the finished
		// lower bound in place, as the bf16 path's fold does at the tile start:
		// acc = f32(s) * sc * S (row scale, query scale), then + alpha + C +
		// xn*B + ux*A by the same two exact-f32 MFMAs (row terms from the
		// tile's RA slot, query terms from QA); the screen below then reads
		// the bounds straight from the accumulators
		constexpr bool FOLDE = FOLD || (I8 && LHIP_I8_TFOLD && MODE != 0);
		if (I8 && LHIP_I8_TFOLD && MODE != 0) {
			const int ln = lane_id_fresh();
			const int li = ln & 31, hk = ln >> 5;
			float bq[4], cq[4], sq[4];
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				const float4 qf = QA[wq * 128 + 32 * u + li];
				bq[u] = hk ? qf.y : qf.z;  // k0: B, k1: A
				cq[u] = hk ? qf.w : 1.0f;  // k0: 1, k1: C
				sq[u] = QA[qlb + 32 * u].x;  // S of this lane's accumulator column
			}
#pragma unroll
			for (int t = 0; t < 2; ++t) {
				const int r = wr * 64 + 32 * t + li;
				const float axu = RAs[(1 + hk) * BR + r];  // k0: xn, k1: ux
				const float aal = hk ? 1.0f : RAs[r];     // k0: alpha, k1: 1
				float4 scv[4];
#pragma unroll
				for (int gq = 0; gq < 4; ++gq) scv[gq] = ra4(rb + 32 * t + 8 * gq, 3);
#pragma unroll
				for (int u = 0; u < 4; ++u) {
#pragma unroll
					for (int gq = 0; gq < 4; ++gq) {
						acc[t][u][4 * gq + 0] = (float)__float_as_int(acc[t][u][4 * gq + 0]) * scv[gq].x * sq[u];
						acc[t][u][4 * gq + 1] = (float)__float_as_int(acc[t][u][4 * gq + 1]) * scv[gq].y * sq[u];
						acc[t][u][4 * gq + 2] = (float)__float_as_int(acc[t][u][4 * gq + 2]) * scv[gq].z * sq[u];
						acc[t][u][4 * gq + 3] = (float)__float_as_int(acc[t][u][4 * gq + 3]) * scv[gq].w * sq[u];
					}
					acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(axu, bq[u], acc[t][u], 0, 0, 0);
					acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(aal, cq[u], acc[t][u], 0, 0, 0);
				}
			}
			mfma_operand_guard();
		}
		if (LHIP_ABL_NO_EPILOGUE) {
			if (acc[0][0][0] == 12345.f && acc[1][3][3] == 54321.f && acc[0][1][1] == acc[1][2][2]) seg_cnt[0] = 1;
		} else if (MODE == 0) {
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				const int ql = qlb + 32 * u;
				if (q0 + ql >= nq) continue;
				const float4 qa = QA[ql];
				float *dst = dense + (int64_t)(q0 + ql) * ld_out + tile * BR;
#pragma unroll
				for (int t = 0; t < 2; ++t)
#pragma unroll
					for (int gq = 0; gq < 4; ++gq) {
						const int r0 = rb + 32 * t + 8 * gq;
						if (FOLD) {
							*reinterpret_cast<float4 *>(dst + r0) = make_float4(
							    acc[t][u][4 * gq + 0], acc[t][u][4 * gq + 1], acc[t][u][4 * gq + 2], acc[t][u][4 * gq + 3]);
							continue;
						}
						const float4 al = ra4(r0, 0), xn = ra4(r0, 1), ux = ra4(r0, 2), sc = ra4(r0, 3);
						*reinterpret_cast<float4 *>(dst + r0) = make_float4(
						    lower_bound<METRIC, I8>(accf(t, u, 4 * gq + 0), make_float4(al.x, xn.x, ux.x, sc.x), qa),
						    lower_bound<METRIC, I8>(accf(t, u, 4 * gq + 1), make_float4(al.y, xn.y, ux.y, sc.y), qa),
						    lower_bound<METRIC, I8>(accf(t, u, 4 * gq + 2), make_float4(al.z, xn.z, ux.z, sc.z), qa),
						    lower_bound<METRIC, I8>(accf(t, u, 4 * gq + 3), make_float4(al.w, xn.w, ux.w, sc.w), qa));
					}
			}
		} else if (MODE == 2) {
			// sample pass: per query, the smallest bound of this wave's 64 rows
			// (lanes l and l^32 hold 32 rows each) -> one segment entry
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				const float4 qa = QA[qlb + 32 * u];
				float mv = F_INF;
				int mr = 0;
#pragma unroll
				for (int t = 0; t < 2; ++t)
#pragma unroll
					for (int gq = 0; gq < 4; ++gq) {
						const int r0 = rb + 32 * t + 8 * gq;
						float4 al, xn, ux, sc;
						if (!FOLDE) al = ra4(r0, 0), xn = ra4(r0, 1), ux = ra4(r0, 2), sc = ra4(r0, 3);
#pragma unroll
						for (int j = 0; j < 4; ++j) {
							const float a = FOLDE ? acc[t][u][4 * gq + j] : accf(t, u, 4 * gq + j);
							const float lb =
							    FOLDE ? a
							         : lower_bound<METRIC, I8>(a,
							                               j == 0   ? make_float4(al.x, xn.x, ux.x, sc.x)
							                               : j == 1 ? make_float4(al.y, xn.y, ux.y, sc.y)
							                               : j == 2 ? make_float4(al.z, xn.z, ux.z, sc.z)
							                                        : make_float4(al.w, xn.w, ux.w, sc.w),
							                               qa);
							if (lb < mv) mv = lb, mr = r0 + j;
						}
					}
				const float ov = __shfl_xor(mv, 32, 64);
				const int orr = __shfl_xor(mr, 32, 64);
				if (ov < mv) mv = ov, mr = orr;
				const int ql = qlb + 32 * u;
				if (eln < 32 && q0 + ql < nq && mv < F_INF) {
					const unsigned p = atomicAdd(&CNT[ql], 1u);
					if (p < (unsigned)seg_cap)
						seg_pool[((int64_t)blockIdx.x * nq + q0 + ql) * seg_cap + p] =
						    make_uint2(fkey(mv), (uint32_t)(row0 + mr));
				}
			}
		} else {
			// tau = +inf (fewer live sample rows than needed) must still drop
			// dead rows (LB = +inf): compare against min(tau, FLT_MAX)
			float4 qa[4];
			float tq[4], tqs[4];
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				qa[u] = QA[qlb + 32 * u];
				tq[u] = fminf(TAU[qlb + 32 * u], F_MAX);
				tqs[u] = fmaxf(tq[u], -F_MAX);
			}
			// Per group of 4 rows x 4 queries (16 bounds per lane): the bounds
			// of two consecutive rows are one v_pk_fma_f32 chain (row terms are
			// SoA; per-lane results identical to the scalar formula), one
			// ballot per bound; positions in the wave's list from mbcnt.  A
			// list that fills (rare) sends further survivors straight to their
			// segment.
			[[maybe_unused]] const int nl0 = n_list;
#pragma unroll
			for (int gi = 0; gi < 8 && DEFER; ++gi) ppos[gi] = -1;
			int nl = n_list;  // list entries + survivors of this tile so far (wave-uniform)
			int nw = n_list;  // of which in the list: entries [0, nw) are written
#pragma unroll
			for (int t = 0; t < 2; ++t)
#pragma unroll
				for (int gq = 0; gq < 4; ++gq) {
					const int r0 = rb + 32 * t + 8 * gq;
					float l[4][4];
					if (FOLDE) {
#pragma unroll
						for (int j = 0; j < 4; ++j)
#pragma unroll
							for (int u = 0; u < 4; ++u) l[j][u] = acc[t][u][4 * gq + j];
					}
					const float4 al = FOLDE ? make_float4(0.f, 0.f, 0.f, 0.f) : ra4(r0, 0);
					const float4 xn = FOLDE ? al : ra4(r0, 1), ux = FOLDE ? al : ra4(r0, 2);
					const float4 sc = (SCL && !FOLDE) ? ra4(r0, 3) : make_float4(1.f, 1.f, 1.f, 1.f);
#pragma unroll
					for (int u = 0; u < 4 && !FOLDE; ++u) {
						const f32x2 Bq = {qa[u].z, qa[u].z}, Aq = {qa[u].y, qa[u].y}, Sq = {qa[u].x, qa[u].x};
						const f32x2 Cq = {qa[u].w, qa[u].w};
#pragma unroll
						for (int p = 0; p < 2; ++p) {
							const f32x2 a2 = p ? f32x2{al.z, al.w} : f32x2{al.x, al.y};
							const f32x2 x2 = p ? f32x2{xn.z, xn.w} : f32x2{xn.x, xn.y};
							const f32x2 u2 = p ? f32x2{ux.z, ux.w} : f32x2{ux.x, ux.y};
							f32x2 s2 = {accf(t, u, 4 * gq + 2 * p), accf(t, u, 4 * gq + 2 * p + 1)};
							if (SCL) s2 = s2 * (p ? f32x2{sc.z, sc.w} : f32x2{sc.x, sc.y});
							// = lower_bound(): alpha + xn*B + ux*A + (s*sc)*S + C
							f32x2 y = __builtin_elementwise_fma(x2, Bq, a2);
							y = __builtin_elementwise_fma(u2, Aq, y);
							y = __builtin_elementwise_fma(s2, Sq, y);
							y = y + Cq;
							l[2 * p][u] = y.x;
							l[2 * p + 1][u] = y.y;
						}
					}
					// Screen: one ballot per group.  min_j l[j][u] - tq[u] <= 0
					// iff some l[j][u] <= tq[u] (exact sign of the rounded
					// difference; a flushed denormal only adds a false
					// positive, rechecked below; NaN bounds never pass either
					// test; tq clamped to >= -FLT_MAX so -inf - -inf = NaN
					// cannot hide a -inf bound).
					float scr = F_MAX;
#pragma unroll
					for (int u = 0; u < 4; ++u)
						scr = fminf(scr, fminf(fminf(l[0][u], l[1][u]), fminf(l[2][u], l[3][u])) - tqs[u]);
					const uint64_t any = __builtin_amdgcn_ballot_w64(scr <= 0.f);
					if (LHIP_ABL_NO_SLOW) {
						asm volatile("" ::"s"(any));  // masks computed, nothing written
					} else if (any && (!LHIP_ABL_SLOW_NEVER || seg_cap == 0x7FFFFFF3)) {
#if LHIP_PROF
						const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
						// Rare: each bound with a survivor in the wave appends the
						// raw LB bits of its lanes at nl + (lanes below); the key
						// conversion happens at write-out.  A scalar loop over the
						// bounds that have survivors, with a uniform switch picking
						// the bound: compact code (the epilogue must stay resident
						// in the instruction cache; 16 unrolled copies per group
						// would not).
#if LHIP_SLOW_VALU
						// Vector side: each lane's first hit among its 16 bounds
						// (k = 4 * row j + query u) by selects; one ballot gives
						// the list positions.  Lanes with a second hit (rare)
						// take the per-bound path below for the others.
						int c = 0, sk = 0;
						float sv = 0.f;
#pragma unroll
						for (int k = 0; k < 16; ++k) {
							const bool hit = l[k >> 2][k & 3] <= tq[k & 3];
							const bool first = hit && c == 0;
							sv = first ? l[k >> 2][k & 3] : sv;
							sk = first ? k : sk;
							c += hit ? 1 : 0;
						}
						{
							const uint64_t b1 = __builtin_amdgcn_ballot_w64(c > 0);
							const int n1 = __builtin_popcountll(b1);
							const int qv = qlb + 32 * (sk & 3), rr = r0 + (sk >> 2);
							if (nl + n1 <= C::WLIST) {
								const int pos = nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
								                                               __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
								if (LHIP_ABL_NO_LISTWRITE) {
									asm volatile("" ::"v"(pos), "v"(sv), "v"(qv), "v"(rr));  // list stays as it was
								} else {
									const uint32_t pl = ((uint32_t)qv << 24) | ((uint32_t)rr << 16) | ((uint32_t)ti & 0xFFFFu);
									if (DEFER) {
										ppos[4 * t + gq] = c > 0 ? pos : -1;  // written at the next wait point
										psv[4 * t + gq] = sv;
										ppl[4 * t + gq] = pl;
										pend = true;
									} else if (c > 0) {
										wlist[pos] = make_uint2(__float_as_uint(sv), pl);
									}
									nw = nl + n1;
								}
							} else {
								overflow_lane(c > 0, sv, qv, rr, row0);
							}
							nl += n1;
						}
						if (!LHIP_ABL_NO_LISTWRITE && __builtin_amdgcn_ballot_w64(c > 1)) {
#pragma unroll
							for (int k = 0; k < 16; ++k) {
								const uint64_t mm =
								    __builtin_amdgcn_ballot_w64(l[k >> 2][k & 3] <= tq[k & 3] && k != sk);
								if (mm) {
									const float lv = l[k >> 2][k & 3];
									const int qv = qlb + 32 * (k & 3), rr = r0 + (k >> 2);
									const int cntm = __builtin_popcountll(mm);
									if (nl + cntm <= C::WLIST) {
										const int pos =
										    nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
										                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
										if ((mm >> eln) & 1ull)
											wlist[pos] = make_uint2(__float_as_uint(lv), ((uint32_t)qv << 24) |
											                                                 ((uint32_t)rr << 16) |
											                                                 ((uint32_t)ti & 0xFFFFu));
										nw = nl + cntm;
									} else {
										overflow(mm, lv, qv, rr, row0);
									}
									nl += cntm;
								}
							}
						}
#elif LHIP_SLOW_UNROLL
#pragma unroll
						for (int k = 0; k < 16; ++k) {
							const uint64_t mm = __builtin_amdgcn_ballot_w64(l[k >> 2][k & 3] <= tq[k & 3]);
							if (mm) {
								const float lv = l[k >> 2][k & 3];
								const int qv = qlb + 32 * (k & 3), rr = r0 + (k >> 2);
								const int cntm = __builtin_popcountll(mm);
								if (nl + cntm <= C::WLIST) {
									const int pos = nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
									                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
									if ((mm >> eln) & 1ull)
										wlist[pos] = make_uint2(__float_as_uint(lv), ((uint32_t)qv << 24) |
										                                                 ((uint32_t)rr << 16) |
										                                                 ((uint32_t)ti & 0xFFFFu));
									nw = nl + cntm;
								} else {
									overflow(mm, lv, qv, rr, row0);
								}
								nl += cntm;
							}
						}
#else
						uint64_t m[4][4];
						uint32_t kmask = 0;
#pragma unroll
						for (int k = 0; k < 16; ++k) {
							m[k >> 2][k & 3] = __builtin_amdgcn_ballot_w64(l[k >> 2][k & 3] <= tq[k & 3]);
							kmask |= (m[k >> 2][k & 3] != 0ull ? 1u : 0u) << k;
						}
						while (kmask) {
							const int k = __builtin_ctz(kmask);
							kmask &= kmask - 1;
							uint64_t mm = 0;
							float lv = 0.f;
							switch (k) {
#define LHIP_PICK(K)                         \
	case K:                                  \
		mm = m[(K) >> 2][(K)&3];             \
		lv = l[(K) >> 2][(K)&3];             \
		break;
								LHIP_PICK(0) LHIP_PICK(1) LHIP_PICK(2) LHIP_PICK(3) LHIP_PICK(4) LHIP_PICK(5)
								LHIP_PICK(6) LHIP_PICK(7) LHIP_PICK(8) LHIP_PICK(9) LHIP_PICK(10) LHIP_PICK(11)
								LHIP_PICK(12) LHIP_PICK(13) LHIP_PICK(14) LHIP_PICK(15)
#undef LHIP_PICK
							}
							const int qv = qlb + 32 * (k & 3), rr = r0 + (k >> 2);
							const int cntm = __builtin_popcountll(mm);
							if (nl + cntm <= C::WLIST) {
								const int pos = nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
								                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
								if ((mm >> eln) & 1ull)
									wlist[pos] = make_uint2(__float_as_uint(lv),
									                        ((uint32_t)qv << 24) | ((uint32_t)rr << 16) | ((uint32_t)ti & 0xFFFFu));
								nw = nl + cntm;
							} else {
								overflow(mm, lv, qv, rr, row0);
							}
							nl += cntm;
						}
#endif
#if LHIP_PROF
						prof_slow += __builtin_amdgcn_s_memtime() - ts0;
						++prof_slown;
#endif
					}
					__builtin_amdgcn_sched_barrier(0);
				}
			n_list = nw;
#if LHIP_PROF
			prof_surv += nl - nl0;
			prof_over += nl > C::WLIST ? nl - C::WLIST : 0;
#endif
		}
		// A tile's stage 0 carries its row aux into RA slot tile&1, the slot
		// tile-2's epilogue reads (cosine and the sample pass read the row terms
		// from LDS there).  When S < NST that stage falls inside the pump limit
		// before the epilogue of tile-2 is over, so pump holds it back (iss_t >=
		// tiles_done + 2).  It may only go out once EVERY wave has left that
		// epilogue: releasing it on this wave's own tiles_done let waves 0..3
		// overwrite the slot while slower waves still read it (wrong cosine
		// bounds in ~1% of the queries of small-dim stores).  So a stage held
		// back here is issued behind a workgroup barrier.  The condition only
		// depends on g, S, G and the tile count, so it is uniform over the
		// workgroup and every wave takes the barrier or none does.
		tiles_done = cur_t;
		if (iss_g < G && iss_g <= g + C::NST && iss_s == 0 && iss_t < tiles_done + 2) {
			asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
			__builtin_amdgcn_s_barrier();
			asm volatile("" ::: "memory");
			pump(g + C::NST);
		}
#if LHIP_PROF
		PROF_T(t4);
		pe += t4 - t3;
#endif
	}
#if LHIP_PROF
	if (lane == 0) {
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 0], (unsigned long long)pw);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 1], (unsigned long long)pb);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 2], (unsigned long long)pc);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 3], (unsigned long long)pe);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 4], 1ull);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 5], (unsigned long long)G);
		atomicAdd(&lhip_prof[(MODE == 1) * 8 + 6], (unsigned long long)cur_t);
		atomicAdd(&lhip_prof[16 + (MODE == 1) * 2 + 0], (unsigned long long)prof_surv);
		atomicAdd(&lhip_prof[16 + (MODE == 1) * 2 + 1], (unsigned long long)prof_over);
		atomicAdd(&lhip_prof[20 + (MODE == 1) * 2 + 0], (unsigned long long)prof_slow);
		atomicAdd(&lhip_prof[20 + (MODE == 1) * 2 + 1], (unsigned long long)prof_slown);
	}
#endif
	// the last prefetch touches write the workgroup's LDS: land them before it can be reallocated
	if (C::TCH) LHIP_WAIT_VM(0);
	if (MODE >= 1) {
		if (DEFER && pend) write_pending();
		if (n_list > 0) write_list_all();  // what is left in the list
		__syncthreads();                         // every wave's counter updates
		if (tid < BQ && q0 + tid < nq) seg_cnt[(int64_t)blockIdx.x * nq + q0 + tid] = (int)CNT[tid];
	}
}

static int num_cus() {
	// (a function-local static: initialised once, thread-safe, C++11)
	static const int n = [] {
		int dev = 0, v = 0;
		return (hipGetDevice(&dev) == hipSuccess &&
		        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
		           ? v
		           : 256;
	}();
	return n;
}

int scan_grid(int64_t n_tiles) { return (int)std::min<int64_t>(n_tiles, (int64_t)num_cus()); }

template <int MODE, int XT>
static void scan_dispatch_x(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, float *dense,
                            int64_t ld_out, const float *tau, uint2 *seg_pool, int *seg_cnt, int seg_cap,
                            hipStream_t st) {
	dim3 grid((unsigned)scan_grid(n_tiles), (unsigned)(q.nq_pad / BQ));
	dim3 block(SCAN_THREADS);
	const float4 *saux = s.scan_aux ? s.scan_aux : s.rowaux;
	switch (s.metric) {
	case METRIC_L2:
		scan_kernel<METRIC_L2, MODE, XT><<<grid, block, 0, st>>>(s.Xscan, saux, s.ld, q.Qb, q.qaux, q.nq, (int)n_tiles,
		                                                          (int)tile_stride, dense, ld_out, tau, seg_pool,
		                                                          seg_cnt, seg_cap);
		break;
	case METRIC_DOT:
		scan_kernel<METRIC_DOT, MODE, XT><<<grid, block, 0, st>>>(s.Xscan, saux, s.ld, q.Qb, q.qaux, q.nq, (int)n_tiles,
		                                                           (int)tile_stride, dense, ld_out, tau, seg_pool,
		                                                           seg_cnt, seg_cap);
		break;
	default:
		scan_kernel<METRIC_COSINE, MODE, XT><<<grid, block, 0, st>>>(s.Xscan, saux, s.ld, q.Qb, q.qaux, q.nq,
		                                                              (int)n_tiles, (int)tile_stride, dense, ld_out,
		                                                              tau, seg_pool, seg_cnt, seg_cap);
		break;
	}
}

template <int MODE>
static void scan_dispatch(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, float *dense,
                          int64_t ld_out, const float *tau, uint2 *seg_pool, int *seg_cnt, int seg_cap,
                          hipStream_t st) {
	if (s.scan_i8) {
		if (s.ld % 128) throw std::runtime_error("int8 scan: row stride must be a multiple of 128");
		scan_dispatch_x<MODE, 2>(s, q, n_tiles, tile_stride, dense, ld_out, tau, seg_pool, seg_cnt, seg_cap, st);
	} else if (s.scan_bf16) {
		scan_dispatch_x<MODE, 1>(s, q, n_tiles, tile_stride, dense, ld_out, tau, seg_pool, seg_cnt, seg_cap, st);
	} else {
		scan_dispatch_x<MODE, 0>(s, q, n_tiles, tile_stride, dense, ld_out, tau, seg_pool, seg_cnt, seg_cap, st);
	}
}

void launch_scan_dense(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, float *out,
                       int64_t ld_out, hipStream_t st) {
	if (n_tiles <= 0) return;
	scan_dispatch<0>(s, q, n_tiles, tile_stride, out, ld_out, nullptr, nullptr, nullptr, 0, st);
}

void launch_scan_tilemin(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, uint2 *seg_pool,
                         int *seg_cnt, int seg_cap, hipStream_t st) {
	if (n_tiles <= 0) return;
	if (seg_cap <= 0 || seg_cap > 1024) throw std::runtime_error("scan: segment capacity must be in [1, 1024]");
	scan_dispatch<2>(s, q, n_tiles, tile_stride, nullptr, 0, nullptr, seg_pool, seg_cnt, seg_cap, st);
}

int scan_append_segments(const StoreView &s, int64_t n_tiles) {
	return scan8_fits(s) ? scan8_segments(n_tiles) : scan_grid(n_tiles);
}

void launch_scan_append(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                        int seg_cap, hipStream_t st) {
	int64_t n_tiles = (s.n_slots + BR - 1) / BR;
	if (n_tiles <= 0) return;
	if (seg_cap <= 0 || seg_cap > 1024) throw std::runtime_error("scan: segment capacity must be in [1, 1024]");
	if (scan8_fits(s)) {
		launch_scan8_append(s, q, tau, seg_pool, seg_cnt, seg_cap, st);
		return;
	}
	if ((n_tiles + scan_grid(n_tiles) - 1) / scan_grid(n_tiles) >= 65536)
		throw std::runtime_error("scan: more than 65535 tiles per workgroup");  // 16-bit tile index in list entries
	scan_dispatch<1>(s, q, n_tiles, 1, nullptr, 0, tau, seg_pool, seg_cnt, seg_cap, st);
}

// ---------------------------------------------------------------------------
// select: per-query radix select of the M smallest lower bounds
// One 512-thread workgroup per query; 11/11/10-bit digits over ordered keys.
// Sources: a dense LB matrix (sample pass / small stores) or the append scan's
// per-(workgroup, query) segments.  Lists that fit are staged in LDS once and
// every pass reads LDS; larger dense lists stream from global memory with
// 8 loads in flight per thread.
// ---------------------------------------------------------------------------
constexpr int SEL_THREADS = 512;
constexpr int SEL_BINS = 2048;
constexpr int SEL_LDS_KEYS = 32768;   // dense lists (keys only)
constexpr int SEL_LDS_PAIRS = 16384;  // segment lists (key, slot)
constexpr int SEL_U = 8;

struct SelSrc {
	const float *dense;
	int64_t ld_dense, n_entries, tile_stride;
	const uint2 *seg_pool;
	const int *seg_cnt;
	int seg_cap, n_seg;
	int tie_desc;  // dense ties at the M-th place: by slot descending
};

// exclusive scan of one value per thread across the block
template <int NT = SEL_THREADS>
__device__ __forceinline__ unsigned block_excl_scan(unsigned v, unsigned *sh /*[NT/64]*/, unsigned &total) {
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	unsigned x = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		unsigned y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	if (lane == 63) sh[w] = x;
	__syncthreads();
	unsigned base = 0, tot = 0;
#pragma unroll
	for (int i = 0; i < NT / 64; ++i) {
		base += (i < w) ? sh[i] : 0u;
		tot += sh[i];
	}
	total = tot;
	__syncthreads();
	return base + x - v;
}

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor(v, o, 64));
	return v;
}

// calls f(i, key) for every entry of this query's list
template <typename F>
__device__ __forceinline__ void sel_for_each(bool in_lds, const uint32_t *s_keys, const float *row, int64_t n, F f) {
	const int t = threadIdx.x;
	if (in_lds) {
		for (int64_t i = t; i < n; i += SEL_THREADS) f(i, s_keys[i]);
		return;
	}
	for (int64_t i0 = 0; i0 < n; i0 += (int64_t)SEL_U * SEL_THREADS) {
		uint32_t k[SEL_U];
#pragma unroll
		for (int u = 0; u < SEL_U; ++u) {
			const int64_t i = i0 + u * SEL_THREADS + t;
			k[u] = i < n ? fkey(row[i]) : KEY_NAN;
		}
#pragma unroll
		for (int u = 0; u < SEL_U; ++u) {
			const int64_t i = i0 + u * SEL_THREADS + t;
			if (i < n) f(i, k[u]);
		}
	}
}

__global__ __launch_bounds__(SEL_THREADS) void select_kernel(SelSrc src, const float *__restrict__ tau, int nq, int M,
                                                             uint32_t *__restrict__ cand_slot,
                                                             int *__restrict__ cand_cnt, float *__restrict__ cut,
                                                             int *__restrict__ pool_total,
                                                             const int *__restrict__ big) {
	__shared__ __attribute__((aligned(16))) uint32_t s_keys[SEL_LDS_KEYS];
	__shared__ unsigned hist[SEL_BINS];
	__shared__ unsigned sh[SEL_THREADS / 64];
	__shared__ unsigned s_digit, s_rem, s_nlt, s_neq, s_minex, s_over, s_heq;
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	if (big && !big[q]) return;  // done by select_small_kernel
	const bool dense = src.dense != nullptr;
	uint32_t *s_slots = s_keys + SEL_LDS_PAIRS;  // segment mode: [keys 16K | slots 16K]
	const float *row = dense ? src.dense + (int64_t)q * src.ld_dense : nullptr;
	if (t == 0) {
		s_nlt = 0;
		s_neq = 0;
		s_minex = 0xFFFFFFFFu;
		s_over = 0;
	}
	__syncthreads();

	int64_t n;
	bool in_lds;
	if (dense) {
		n = src.n_entries;
		in_lds = n <= SEL_LDS_KEYS;
		if (in_lds) {
			const int n4 = (int)(n >> 2);
			for (int i0 = 0; i0 < n4; i0 += SEL_U * SEL_THREADS) {
				float4 v[SEL_U];
#pragma unroll
				for (int u = 0; u < SEL_U; ++u) {
					const int i = i0 + u * SEL_THREADS + t;
					v[u] = i < n4 ? reinterpret_cast<const float4 *>(row)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
				}
#pragma unroll
				for (int u = 0; u < SEL_U; ++u) {
					const int i = i0 + u * SEL_THREADS + t;
					if (i < n4)
						reinterpret_cast<uint4 *>(s_keys)[i] =
						    make_uint4(fkey(v[u].x), fkey(v[u].y), fkey(v[u].z), fkey(v[u].w));
				}
			}
			for (int64_t i = (int64_t)n4 * 4 + t; i < n; i += SEL_THREADS) s_keys[i] = fkey(row[i]);
		}
	} else {
		// segments: thread s < n_seg owns segment s of this query
		unsigned c = 0;
		if (t < src.n_seg) {
			const int cs = src.seg_cnt[(int64_t)t * nq + q];
			if (cs > src.seg_cap) s_over = 1u;
			c = (unsigned)min(cs, src.seg_cap);
		}
		unsigned total;
		const unsigned off = block_excl_scan(c, sh, total);
		// a pool over the LDS capacity keeps its first SEL_LDS_PAIRS entries:
		// the certificate fails (cut = -inf), but the candidates are still
		// real rows, so their k-th exact distance bounds the second pass's tau
		in_lds = true;
		if (total > (unsigned)SEL_LDS_PAIRS) s_over = 1u;
		n = total < (unsigned)SEL_LDS_PAIRS ? total : (unsigned)SEL_LDS_PAIRS;
		unsigned room = off < (unsigned)SEL_LDS_PAIRS ? (unsigned)SEL_LDS_PAIRS - off : 0u;
		c = c < room ? c : room;
		if (c) {
			const uint2 *seg = src.seg_pool + ((int64_t)t * nq + q) * src.seg_cap;
			unsigned i = 0;
			for (; i + 4 <= c; i += 4) {
				uint2 e0 = seg[i], e1 = seg[i + 1], e2 = seg[i + 2], e3 = seg[i + 3];
				s_keys[off + i] = e0.x;
				s_slots[off + i] = e0.y;
				s_keys[off + i + 1] = e1.x;
				s_slots[off + i + 1] = e1.y;
				s_keys[off + i + 2] = e2.x;
				s_slots[off + i + 2] = e2.y;
				s_keys[off + i + 3] = e3.x;
				s_slots[off + i + 3] = e3.y;
			}
			for (; i < c; ++i) {
				uint2 e = seg[i];
				s_keys[off + i] = e.x;
				s_slots[off + i] = e.y;
			}
		}
	}
	const float ftau = (dense || !tau) ? F_INF : tau[q];
	auto slot_at = [&](int64_t i) -> uint32_t {
		if (dense) return (uint32_t)((i / BR) * src.tile_stride * BR + (i % BR));
		return s_slots[i];
	};

	for (int i = t; i < SEL_BINS; i += SEL_THREADS) hist[i] = 0;
	__syncthreads();
	// pass 1: histogram of the top 11 bits (also counts +inf / NaN keys)
	sel_for_each(in_lds, s_keys, row, n, [&](int64_t, uint32_t k) { atomicAdd(&hist[k >> 21], 1u); });
	__syncthreads();
	const unsigned n_nan = hist[SEL_BINS - 1];
	const unsigned n_inf = hist[KEY_INF >> 21];  // bin 0x7FC holds +inf only
	const int64_t n_fin = n - n_nan - n_inf;
	float c_out;
	if (n_fin <= M) {
		sel_for_each(in_lds, s_keys, row, n, [&](int64_t i, uint32_t k) {
			if (k < KEY_INF) {
				unsigned p = atomicAdd(&s_nlt, 1u);
				cand_slot[(int64_t)q * M + p] = slot_at(i);
			}
		});
		__syncthreads();
		c_out = ftau;
	} else {
		unsigned prefix = 0, mask = 0, rem = (unsigned)M;
#pragma unroll 1
		for (int p = 0; p < 3; ++p) {
			const int sh_ = p == 0 ? 21 : (p == 1 ? 10 : 0);
			const unsigned dmask = p == 2 ? 0x3FFu : 0x7FFu;
			if (p > 0) {
				for (int i = t; i < SEL_BINS; i += SEL_THREADS) hist[i] = 0;
				__syncthreads();
				sel_for_each(in_lds, s_keys, row, n, [&](int64_t, uint32_t k) {
					if ((k & mask) == prefix) atomicAdd(&hist[(k >> sh_) & dmask], 1u);
				});
				__syncthreads();
			}
			constexpr int BPT = SEL_BINS / SEL_THREADS;
			unsigned local = 0;
#pragma unroll
			for (int j = 0; j < BPT; ++j) local += hist[t * BPT + j];
			unsigned total;
			unsigned excl = block_excl_scan(local, sh, total);
			if (excl < rem && rem <= excl + local) {
				unsigned c = excl;
				for (int j = 0; j < BPT; ++j) {
					unsigned h = hist[t * BPT + j];
					if (rem <= c + h) {
						s_digit = (unsigned)(t * BPT + j);
						s_rem = rem - c;
						s_heq = h;  // last pass: entries equal to the M-th smallest key
						break;
					}
					c += h;
				}
			}
			__syncthreads();
			prefix |= s_digit << sh_;
			mask |= dmask << sh_;
			rem = s_rem;
			__syncthreads();
		}
		const uint32_t T = prefix;                // key of the M-th smallest
		const unsigned n_lt = (unsigned)M - rem;  // entries strictly below T
		unsigned my_min = 0xFFFFFFFFu;            // smallest key left out
		if (dense && s_heq > rem) {
			// Dense source with ties straddling the M-th place: take the equal
			// keys in entry order = slot order (one block scan per chunk; the
			// label-descending tie rule walks the entries backwards), so the
			// selection is the M smallest by (key, slot) under the tie rule — the
			// order the batched exact fallback relies on (slots ascend with labels).
			unsigned base = 0;
			for (int64_t i0 = 0; i0 < n; i0 += SEL_THREADS) {
				const int64_t ii = i0 + t, i = src.tie_desc ? n - 1 - ii : ii;
				const uint32_t k = ii < n ? (in_lds ? s_keys[i] : fkey(row[i])) : KEY_NAN;
				if (k < T) {
					unsigned p = atomicAdd(&s_nlt, 1u);
					cand_slot[(int64_t)q * M + p] = slot_at(i);
				} else if (k > T && k < KEY_INF) {
					my_min = min(my_min, k);
				}
				unsigned tot;
				const unsigned ex = block_excl_scan(k == T ? 1u : 0u, sh, tot);
				if (k == T) {
					if (base + ex < rem)
						cand_slot[(int64_t)q * M + n_lt + base + ex] = slot_at(i);
					else
						my_min = min(my_min, k);
				}
				base += tot;
			}
		} else
		sel_for_each(in_lds, s_keys, row, n, [&](int64_t i, uint32_t k) {
			if (k < T) {
				unsigned p = atomicAdd(&s_nlt, 1u);
				cand_slot[(int64_t)q * M + p] = slot_at(i);
			} else if (k == T) {
				unsigned p = atomicAdd(&s_neq, 1u);
				if (p < rem)
					cand_slot[(int64_t)q * M + n_lt + p] = slot_at(i);
				else
					my_min = min(my_min, k);
			} else if (k < KEY_INF) {
				my_min = min(my_min, k);
			}
		});
		my_min = wave_min_u32(my_min);
		if ((t & 63) == 0 && my_min != 0xFFFFFFFFu) atomicMin(&s_minex, my_min);
		__syncthreads();
		c_out = (s_minex == 0xFFFFFFFFu) ? F_INF : fkey_inv(s_minex);
		if (ftau < c_out) c_out = ftau;
		if (t == 0) s_nlt = (unsigned)M;
		__syncthreads();
	}
	if (t == 0) {
		if (s_over || n_nan > 0) c_out = -F_INF;
		cand_cnt[q] = (int)s_nlt;
		cut[q] = c_out;
		if (pool_total) pool_total[q] = s_over ? -1 : (int)n;
	}
}

void launch_select_dense(const float *dense, int64_t ld_dense, int64_t n_entries, int64_t tile_stride, int nq, int M,
                         uint32_t *cand_slot, int *cand_cnt, float *cut, hipStream_t st, int tie_desc) {
	SelSrc s{dense, ld_dense, n_entries, tile_stride, nullptr, nullptr, 0, 0, tie_desc};
	select_kernel<<<dim3(nq), dim3(SEL_THREADS), 0, st>>>(s, nullptr, nq, M, cand_slot, cand_cnt, cut, nullptr,
	                                                        nullptr);
}

// Small pools (the common case: a few hundred survivors per query): one wave
// per query gathers its segments as (key << 32 | slot) into LDS and bitonic-
// sorts them — 8 KiB of LDS instead of the radix select's 136 KiB, so many
// queries run per CU.  Same outputs as select_kernel (candidates = the M
// smallest keys, ties by slot; cut = the smallest key left out, or tau; -inf
// after a segment overflow or a NaN bound).  A pool over SSEL_CAP entries sets
// big[q] and is left to select_kernel.
constexpr int SSEL_CAP = 1024;
__global__ __launch_bounds__(64) void select_small_kernel(const uint2 *__restrict__ seg_pool,
                                                          const int *__restrict__ seg_cnt, int seg_cap, int n_seg,
                                                          const float *__restrict__ tau, int nq, int M,
                                                          uint32_t *__restrict__ cand_slot,
                                                          int *__restrict__ cand_cnt, float *__restrict__ cut,
                                                          int *__restrict__ pool_total, int *__restrict__ big) {
	__shared__ uint64_t sk[SSEL_CAP];
	const int q = blockIdx.x, lane = threadIdx.x;
	unsigned mine = 0;
	bool over = false;
	for (int s = lane; s < n_seg; s += 64) {
		const int cs = seg_cnt[(int64_t)s * nq + q];
		over |= cs > seg_cap;
		mine += (unsigned)min(cs, seg_cap);
	}
	unsigned x = mine;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const unsigned y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	const unsigned total = __shfl(x, 63, 64);
	const bool any_over = __builtin_amdgcn_ballot_w64(over) != 0ull;
	if (total > (unsigned)SSEL_CAP) {
		if (lane == 0) big[q] = 1;
		return;
	}
	if (lane == 0) big[q] = 0;
	unsigned o = x - mine;
	for (int s = lane; s < n_seg; s += 64) {
		const int c = min(seg_cnt[(int64_t)s * nq + q], seg_cap);
		const uint2 *seg = seg_pool + ((int64_t)s * nq + q) * seg_cap;
		for (int i = 0; i < c; ++i) sk[o++] = ((uint64_t)seg[i].x << 32) | seg[i].y;
	}
	int P = 64;
	while (P < (int)total) P <<= 1;
	for (int i = (int)total + lane; i < P; i += 64) sk[i] = ~0ull;
	__syncthreads();
	for (int size = 2; size <= P; size <<= 1) {
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			for (int i = lane; i < (P >> 1); i += 64) {
				const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
				const bool asc = (lo & size) == 0;
				const uint64_t a = sk[lo], b = sk[hi];
				if ((a > b) == asc) {
					sk[lo] = b;
					sk[hi] = a;
				}
			}
			__syncthreads();
		}
	}
	// sorted: finite keys, then +inf, then NaN (KEY_INF < KEY_NAN), then padding
	unsigned nfin = 0, nnan = 0;
	for (int i = lane; i < (int)total; i += 64) {
		const uint32_t k = (uint32_t)(sk[i] >> 32);
		nfin += k < KEY_INF ? 1u : 0u;
		nnan += k == KEY_NAN ? 1u : 0u;
	}
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) {
		nfin += __shfl_xor(nfin, off, 64);
		nnan += __shfl_xor(nnan, off, 64);
	}
	const float ftau = tau ? tau[q] : F_INF;
	const int nc = (int)min(nfin, (unsigned)M);
	for (int i = lane; i < nc; i += 64) cand_slot[(int64_t)q * M + i] = (uint32_t)sk[i];
	if (lane == 0) {
		float c_out = ftau;
		if ((int)nfin > M) {
			const float kx = fkey_inv((uint32_t)(sk[M] >> 32));
			c_out = kx < ftau ? kx : ftau;
		}
		if (any_over || nnan > 0) c_out = -F_INF;
		cand_cnt[q] = nc;
		cut[q] = c_out;
		if (pool_total) pool_total[q] = any_over ? -1 : (int)total;
	}
}

void launch_select_segments(const uint2 *seg_pool, const int *seg_cnt, int seg_cap, int n_seg, const float *tau,
                            int nq, int M, uint32_t *cand_slot, int *cand_cnt, float *cut, int *pool_total,
                            int *big, hipStream_t st) {
	// one wave per query pays off once there are enough queries to fill the
	// chip (measured: 2048 queries 108 -> ~70 us; 256 queries 23 -> 93 us)
	const bool small = nq >= 1024;
	if (small)
		select_small_kernel<<<dim3(nq), dim3(64), 0, st>>>(seg_pool, seg_cnt, seg_cap, n_seg, tau, nq, M, cand_slot,
		                                                     cand_cnt, cut, pool_total, big);
	SelSrc s{nullptr, 0, 0, 1, seg_pool, seg_cnt, seg_cap, n_seg};
	select_kernel<<<dim3(nq), dim3(SEL_THREADS), 0, st>>>(s, tau, nq, M, cand_slot, cand_cnt, cut, pool_total,
	                                                        small ? big : nullptr);
}

// ---------------------------------------------------------------------------
// refine: one wave per (query, candidate), f64 accumulation
// ---------------------------------------------------------------------------

template <int METRIC, typename T>
__global__ __launch_bounds__(256) void refine_kernel(const T *__restrict__ X, int ld, int dim,
                                                     const float *__restrict__ Qf,
                                                     const uint32_t *__restrict__ cand_slot,
                                                     const int *__restrict__ cand_cnt, int nq, int M,
                                                     float *__restrict__ cand_dist) {
	const int lane = threadIdx.x & 63;
	const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	if (g >= (int64_t)nq * M) return;
	const int q = (int)(g / M), m = (int)(g % M);
	if (m >= cand_cnt[q]) return;
	const uint32_t slot = cand_slot[(int64_t)q * M + m];
	float d = exact_distance<METRIC, T>(X + (int64_t)slot * ld, Qf + (int64_t)q * ld, dim, lane);
	if (lane == 0) cand_dist[(int64_t)q * M + m] = d;
}

template <typename T>
static void refine_dispatch(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt,
                            int M, float *cand_dist, hipStream_t st) {
	int64_t waves = (int64_t)q.nq * M;
	dim3 grid((unsigned)((waves + 3) / 4));
	const T *X = static_cast<const T *>(s.X);
	switch (s.metric) {
	case METRIC_L2:
		refine_kernel<METRIC_L2, T><<<grid, 256, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, q.nq, M, cand_dist);
		break;
	case METRIC_DOT:
		refine_kernel<METRIC_DOT, T><<<grid, 256, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, q.nq, M, cand_dist);
		break;
	default:
		refine_kernel<METRIC_COSINE, T><<<grid, 256, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, q.nq, M,
		                                                       cand_dist);
		break;
	}
}

void launch_refine(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt, int M,
                   float *cand_dist, hipStream_t st) {
	if (s.xbf16)
		refine_dispatch<uint16_t>(s, q, cand_slot, cand_cnt, M, cand_dist, st);
	else
		refine_dispatch<float>(s, q, cand_slot, cand_cnt, M, cand_dist, st);
}

// ---------------------------------------------------------------------------
// refine + tau in one launch (the sample pass's candidates): one 8-wave
// workgroup per query computes the exact distances of its m candidates (the
// value refine_kernel computes) into LDS and writes tau = the need-th smallest
// of them (+inf when fewer, NaN when any is NaN): finalize_kernel's mode 0
// without the refine launch and the cand_dist round trip
// ---------------------------------------------------------------------------
template <int METRIC, typename T>
__global__ __launch_bounds__(512) void refine_tau_kernel(const T *__restrict__ X, int ld, int dim,
                                                         const float *__restrict__ Qf,
                                                         const uint32_t *__restrict__ cand_slot,
                                                         const int *__restrict__ cand_cnt, int M, int need,
                                                         float *__restrict__ tau) {
	__shared__ float sd[MAX_CAND];
	const int q = blockIdx.x;
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	const int m = min(cand_cnt[q], M);
	for (int i = w; i < m; i += 8) {
		const uint32_t slot = cand_slot[(int64_t)q * M + i];
		const float d = exact_distance<METRIC, T>(X + (int64_t)slot * ld, Qf + (int64_t)q * ld, dim, lane);
		if (lane == 0) sd[i] = d;
	}
	__syncthreads();
	bool nan = false;
	for (int i = 0; i < m; ++i) nan |= __builtin_isnan(sd[i]);
	if (m < need || m == 0 || nan) {
		if (t == 0) tau[q] = nan ? __builtin_nanf("") : F_INF;
		return;
	}
	for (int i = t; i < m; i += 512) {
		int rank = 0;
		const float d = sd[i];
		for (int j = 0; j < m; ++j) rank += (sd[j] < d || (sd[j] == d && j < i)) ? 1 : 0;
		if (rank == need - 1) tau[q] = d;
	}
}

template <typename T>
static void refine_tau_dispatch(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt,
                                int M, int need, float *tau, hipStream_t st) {
	const T *X = static_cast<const T *>(s.X);
	const dim3 grid((unsigned)q.nq);
	switch (s.metric) {
	case METRIC_L2:
		refine_tau_kernel<METRIC_L2, T><<<grid, 512, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, M, need, tau);
		break;
	case METRIC_DOT:
		refine_tau_kernel<METRIC_DOT, T><<<grid, 512, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, M, need, tau);
		break;
	default:
		refine_tau_kernel<METRIC_COSINE, T><<<grid, 512, 0, st>>>(X, s.ld, s.dim, q.Qf, cand_slot, cand_cnt, M, need,
		                                                          tau);
		break;
	}
}

void launch_refine_tau(const StoreView &s, const QueryView &q, const uint32_t *cand_slot, const int *cand_cnt, int M,
                       int need, float *tau, hipStream_t st) {
	if (M > MAX_CAND) throw std::runtime_error("refine_tau: M past MAX_CAND");
	if (s.xbf16)
		refine_tau_dispatch<uint16_t>(s, q, cand_slot, cand_cnt, M, need, tau, st);
	else
		refine_tau_dispatch<float>(s, q, cand_slot, cand_cnt, M, need, tau, st);
}

// ---------------------------------------------------------------------------
// finalize: rank candidates by (distance, label); top-k + certificate, or tau
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void finalize_kernel(const int64_t *__restrict__ labels,
                                                       const uint32_t *__restrict__ cand_slot,
                                                       const int *__restrict__ cand_cnt,
                                                       const float *__restrict__ cand_dist,
                                                       const float *__restrict__ cut, int M, int k, int mode,
                                                       int need_for_tau, float *__restrict__ tau,
                                                       int64_t *__restrict__ out_labels,
                                                       float *__restrict__ out_dists, int *__restrict__ out_counts,
                                                       int *__restrict__ cert_ok, int64_t live, int64_t tx) {
	__shared__ float sd[MAX_CAND];
	__shared__ int64_t sl[MAX_CAND];
	__shared__ float s_dk;
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	const int m = cand_cnt[q];
	for (int i = t; i < m; i += 256) {
		sd[i] = cand_dist[(int64_t)q * M + i];
		sl[i] = labels[cand_slot[(int64_t)q * M + i]];
	}
	if (t == 0) s_dk = F_INF;
	__syncthreads();
	if (mode == 0) {
		// tau = the need_for_tau-th smallest exact distance among the
		// candidates: they are real rows, so any need_for_tau (>= k) of them
		// bound the true k-th distance from above.  Fewer than that: +inf; a
		// NaN distance: NaN (nothing survives; the certificate sends the query
		// to the exact fallback).
		bool nan = false;
		for (int i = 0; i < m; ++i) nan |= __builtin_isnan(sd[i]);
		if (m < need_for_tau || m == 0 || nan) {
			if (t == 0) tau[q] = nan ? __builtin_nanf("") : F_INF;
			return;
		}
		for (int i = t; i < m; i += 256) {
			int rank = 0;
			const float d = sd[i];
			for (int j = 0; j < m; ++j) rank += (sd[j] < d || (sd[j] == d && j < i)) ? 1 : 0;
			if (rank == need_for_tau - 1) tau[q] = d;
		}
		return;
	}
	const int nout = m < k ? m : k;
	for (int i = t; i < m; i += 256) {
		int rank = 0;
		const float d = sd[i];
		const int64_t l = sl[i];
		for (int j = 0; j < m; ++j) rank += hit_less(sd[j], sl[j], d, l, tx) ? 1 : 0;
		if (rank < k) {
			out_labels[(int64_t)q * k + rank] = l;
			out_dists[(int64_t)q * k + rank] = d;
		}
		if (rank == k - 1) s_dk = d;
	}
	for (int i = nout + t; i < k; i += 256) {
		out_labels[(int64_t)q * k + i] = -1;
		out_dists[(int64_t)q * k + i] = __builtin_nanf("");
	}
	__syncthreads();
	if (t == 0) {
		out_counts[q] = nout;
		const float c = cut[q];
		bool ok;
		if (c == F_INF) {
			ok = true;  // nothing live was left out
		} else {
			const float dk = s_dk;  // +inf when fewer than k candidates
			ok = !__builtin_isnan(dk) && dk < F_INF && c > nextafterf(dk, F_INF);
		}
		// fewer hits than min(k, live rows): a live row is missing (one whose
		// bound overflowed to +inf, as a tombstone's does): never certified
		if (live >= 0 && (int64_t)nout < (live < (int64_t)k ? live : (int64_t)k)) ok = false;
		cert_ok[q] = ok ? 1 : 0;
	}
}

void launch_finalize(const StoreView &s, const uint32_t *cand_slot, const int *cand_cnt, const float *cand_dist,
                     const float *cut, int nq, int M, int k, int mode, int need_for_tau, float *tau,
                     int64_t *out_labels, float *out_dists, int *out_counts, int *cert_ok, hipStream_t st,
                     int64_t live) {
	finalize_kernel<<<dim3(nq), dim3(256), 0, st>>>(s.labels, cand_slot, cand_cnt, cand_dist, cut, M, k, mode,
	                                                 need_for_tau, tau, out_labels, out_dists, out_counts, cert_ok,
	                                                 live, tie_x64(s.tie_desc));
}

// ---------------------------------------------------------------------------
// pool_refine: select + refine + finalize of a threshold pass in ONE launch,
// refining only as far as the certificate needs.  One 512-thread workgroup
// per query gathers the query's segments (every row with LB <= tau, from the
// append or sample scan) into LDS as (orderedkey(LB), slot) and refines it in
// threshold chunks, no sort: a chunk is every unrefined bound up to a key
// picked from a histogram of the pool's keys, refined 128 per round (16 per
// wave, exact f64 distances as refine_kernel computes them) and merged into the
// running top-k by (distance, label):
//   final mode: the first chunk holds the ~PR_R smallest bounds; each later one
//   every unrefined bound <= nextafter(d_k) (d_k of the top so far: it only
//   falls, so each row a bound-order refine would take is taken), until none
//   is left; then every unrefined row, in the pool or not, has LB > d_k:
//   certified as finalize does, cut = min(smallest unrefined bound, tau) (the
//   int8 bounds put ~60-250 rows below d_k at 1M-10M rows x 768);
//   tau mode (the sample pass): refine at least the m_tau smallest bounds (a
//   whole chunk), tau = the k-th smallest exact distance among them (+inf when
//   fewer than k, NaN when any is NaN): an upper bound on the k-th nearest
//   distance, never above refine_tau_kernel's from the m_tau smallest alone;
//   given an input tau (the pool of a first threshold pass over part of the
//   tiles), tau = min(input, that) (the input when that is NaN).
// A segment that overflowed, a pool past PR_CAP or a NaN bound fails the
// certificate (cut = -inf), as select_kernel's does; the rows refined still
// give the rerun a tau.  Returns the refined count and the pool size.
// ---------------------------------------------------------------------------
#ifndef LHIP_PR_THREADS
#define LHIP_PR_THREADS 512
#endif
constexpr int PR_THREADS = LHIP_PR_THREADS;  // 256, 512 or 1024 (one workgroup per query)
static_assert(PR_THREADS == 256 || PR_THREADS == 512 || PR_THREADS == 1024, "pool_refine geometry");
#ifndef LHIP_PR_CAP
#define LHIP_PR_CAP 16384
#endif
// (256 threads with a 4096-entry pool: ~54 KB of LDS and one wave per SIMD, two
// workgroups per CU — a development geometry for A/B timing)
constexpr int PR_MIN_WAVES = PR_THREADS == 256 ? 2 : 1;  // waves per SIMD the register allocation must allow
#ifdef LHIP_PR_PROF
constexpr int PR_NSTAMP = 32, PR_PROF_Q = 4096;
__device__ uint64_t g_pr_stamps[PR_PROF_Q * (PR_NSTAMP + 3)];
#endif
constexpr int PR_CAP = LHIP_PR_CAP;  // pool entries held in LDS
constexpr int PR_PER_WAVE = 16;     // candidates per wave and round
constexpr int PR_MAXK = MAX_CAND;   // k of the fast path (k + 8 <= MAX_CAND)
#ifndef LHIP_PR_SPREAD
#define LHIP_PR_SPREAD 0  // 1: the pool gather spread over every thread (an A/B: within noise, r06w)
#endif

// exact distances of NC rows to one query by one wave (each the value
// exact_distance returns), every row's loads issued before any accumulates.
// NI > 0: rows of at most 256 NI elements (d4 <= 64 NI); a lane's NI x NC
// 16-B loads are ALL in flight together (one memory latency per round, not
// NI of them) and the query comes from LDS (qs: 256 NI floats, zero past
// dim).  NI = 0: any dimension, one 16-B column step at a time.
template <int METRIC, typename T, int NC, int NI>
__device__ __forceinline__ void exact_distance_multi(const T *__restrict__ X, int ld, const uint32_t *slots,
                                                     int nvalid, const float *__restrict__ q, const float *qs,
                                                     int dim, int lane, float *out) {
	double a[NC], b[NC], c[NC];
#pragma unroll
	for (int r = 0; r < NC; ++r) a[r] = b[r] = c[r] = 0.0;
	const int d4 = dim >> 2;
	if constexpr (NI > 0) {
		float4 xv[NI][NC];
#pragma unroll
		for (int it = 0; it < NI; ++it) {
			const int i4 = lane + 64 * it;
#pragma unroll
			for (int r = 0; r < NC; ++r)
				xv[it][r] = (r < nvalid && i4 < d4) ? xval4(X + (int64_t)slots[r] * ld, 4 * i4)
				                                    : make_float4(0.f, 0.f, 0.f, 0.f);
		}
#pragma unroll
		for (int it = 0; it < NI; ++it) {
			const float4 qv = *reinterpret_cast<const float4 *>(qs + 4 * (lane + 64 * it));  // zero past dim
#pragma unroll
			for (int r = 0; r < NC; ++r) {
				exact_acc<METRIC>(xv[it][r].x, qv.x, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[it][r].y, qv.y, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[it][r].z, qv.z, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[it][r].w, qv.w, a[r], b[r], c[r]);
			}
		}
	} else {
		for (int i4 = lane; i4 < d4; i4 += 64) {
			const float4 qv = *reinterpret_cast<const float4 *>(q + 4 * i4);
			float4 xv[NC];
#pragma unroll
			for (int r = 0; r < NC; ++r)
				xv[r] = r < nvalid ? xval4(X + (int64_t)slots[r] * ld, 4 * i4) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
			for (int r = 0; r < NC; ++r) {
				exact_acc<METRIC>(xv[r].x, qv.x, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[r].y, qv.y, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[r].z, qv.z, a[r], b[r], c[r]);
				exact_acc<METRIC>(xv[r].w, qv.w, a[r], b[r], c[r]);
			}
		}
	}
	for (int i = 4 * d4 + lane; i < dim; i += 64)
#pragma unroll
		for (int r = 0; r < NC; ++r)
			if (r < nvalid) exact_acc<METRIC>(xval(X + (int64_t)slots[r] * ld, i), q[i], a[r], b[r], c[r]);
#pragma unroll
	for (int r = 0; r < NC; ++r) {
		const double sa = wave_sum_f64(a[r]);
		double res;
		if (METRIC == METRIC_L2) {
			res = sa;
		} else if (METRIC == METRIC_DOT) {
			res = 1.0 - sa;
		} else {
			const double sb = wave_sum_f64(b[r]), sc = wave_sum_f64(c[r]);
			res = 1.0 - sa / (sqrt(sb) * sqrt(sc));
		}
		float f = (float)res + 0.0f;  // canonical +0
		if (__builtin_isnan(f)) f = __builtin_nanf("");
		out[r] = f;
	}
}

// Exact distances of NC rows (NC a power of two <= 16) to one query by one
// wave, NS = ceil(dim / 256) 16-B column steps per row, each the value
// exact_distance returns (f64 accumulation, one rounding to f32):
//   * loads: the rows' bases are wave-uniform (SGPR slots, recomputed per
//     use); the rows in two halves, one half's loads in flight while the other
//     half is summed (per-lane accumulation order unchanged: steps ascending,
//     x y z w);
//   * the per-row wave sums as a transpose-reduce: at each xor level a lane
//     keeps half of its rows' partial sums and adds the partner's copy of them
//     (NC-1 f64 shuffles for the halving levels + log2(64/NC) for the rest,
//     instead of 6 NC); row r ends up in lanes r * (64 / NC) .. (r + 1) * (64 / NC) - 1.
// Returns this lane's value (row lane / (64 / NC)); rows >= nvalid read nothing.
// The query comes from LDS (qs: NS * 256 floats, zero past dim).
template <int METRIC, typename T, int NC, int NS>
__device__ __forceinline__ float exact_rows_ring(const T *__restrict__ X, int ld, const uint32_t *slots, int nvalid,
                                                 const float *qs, int dim, int lane) {
	static_assert(NC == 1 || NC == 2 || NC == 4 || NC == 8 || NC == 16, "NC: a power of two <= 16");
	static_assert(NS >= 1 && NS <= 4, "NS: 256-element steps of a row");
	constexpr int NSUM = METRIC == METRIC_COSINE ? 3 : 1;
	const int d4 = dim >> 2;
	uint32_t svr[NC];  // the rows' slots (wave-uniform: SGPRs)
#pragma unroll
	for (int r = 0; r < NC; ++r) svr[r] = __builtin_amdgcn_readfirstlane(slots[r]);
	// a row's base, recomputed at each use (opaque to CSE: NC live 64-bit
	// pointers would not fit the SGPR budget and spill into VGPRs)
	auto xr = [&](int r) -> const T * {
		uint32_t sv = svr[r];
		asm volatile("" : "+s"(sv));
		return X + (int64_t)sv * ld;
	};
	double acc[NSUM][NC];
#pragma unroll
	for (int r = 0; r < NC; ++r)
#pragma unroll
		for (int u = 0; u < NSUM; ++u) acc[u][r] = 0.0;
	// loads: a rolled loop over the column steps in two halves of the rows: a
	// half's loads are issued before the other half is summed, so the memory
	// stays busy while the wave sums (a fully unrolled ring let the compiler
	// hoist every step's loads and the 256 VGPRs of two waves per SIMD spilled)
	constexpr int HR = NC > 1 ? NC / 2 : 1, NH = NC / HR;
	auto issue = [&](int s, int h, float4 (&b)[HR]) {
		const int i4 = lane + 64 * s;
#pragma unroll
		for (int r = 0; r < HR; ++r)
			b[r] = (h * HR + r < nvalid && i4 < d4) ? xval4(xr(h * HR + r), 4 * i4) : make_float4(0.f, 0.f, 0.f, 0.f);
	};
	auto consume = [&](int s, int h, const float4 (&b)[HR]) {
		const float4 qv = *reinterpret_cast<const float4 *>(qs + 4 * (lane + 64 * s));  // zero past dim
#pragma unroll
		for (int r = 0; r < HR; ++r) {
			const int rr = h * HR + r;
			double a = acc[0][rr], bb = NSUM > 1 ? acc[1][rr] : 0.0, cc = NSUM > 1 ? acc[2][rr] : 0.0;
			exact_acc<METRIC>(b[r].x, qv.x, a, bb, cc);
			exact_acc<METRIC>(b[r].y, qv.y, a, bb, cc);
			exact_acc<METRIC>(b[r].z, qv.z, a, bb, cc);
			exact_acc<METRIC>(b[r].w, qv.w, a, bb, cc);
			acc[0][rr] = a;
			if (NSUM > 1) {
				acc[1][rr] = bb;
				acc[2][rr] = cc;
			}
		}
	};
	float4 b0[HR], b1[HR];
	issue(0, 0, b0);
#pragma unroll 1
	for (int s = 0; s < NS; ++s) {
		if (NH > 1) issue(s, 1, b1);
		consume(s, 0, b0);
		if (s + 1 < NS) issue(s + 1, 0, b0);
		if (NH > 1) consume(s, 1, b1);
	}
	// dim % 4 tail elements (rows of any dim the path admits)
	for (int i = 4 * d4 + lane; i < dim; i += 64)
#pragma unroll
		for (int r = 0; r < NC; ++r)
			if (r < nvalid) {
				double a = acc[0][r], bb = NSUM > 1 ? acc[1][r] : 0.0, cc = NSUM > 1 ? acc[2][r] : 0.0;
				exact_acc<METRIC>(xval(xr(r), i), qs[i], a, bb, cc);
				acc[0][r] = a;
				if (NSUM > 1) {
					acc[1][r] = bb;
					acc[2][r] = cc;
				}
			}
	// transpose-reduce: level o (32, 16, ..) halves the rows a lane holds
	double v[NSUM];
	{
		double cur[NSUM][NC];
#pragma unroll
		for (int u = 0; u < NSUM; ++u)
#pragma unroll
			for (int r = 0; r < NC; ++r) cur[u][r] = acc[u][r];
		int o = 32;
#pragma unroll
		for (int h = NC / 2; h >= 1; h >>= 1, o >>= 1) {
			const bool hi = (lane & o) != 0;
#pragma unroll
			for (int u = 0; u < NSUM; ++u)
#pragma unroll
				for (int r = 0; r < h; ++r) {
					const double send = hi ? cur[u][r] : cur[u][r + h];
					const double keep = hi ? cur[u][r + h] : cur[u][r];
					cur[u][r] = keep + __shfl_xor(send, o, 64);
				}
		}
#pragma unroll
		for (int u = 0; u < NSUM; ++u) {
			double x = cur[u][0];
			for (int oo = o; oo > 0; oo >>= 1) x += __shfl_xor(x, oo, 64);
			v[u] = x;
		}
	}
	double res;
	if (METRIC == METRIC_L2) {
		res = v[0];
	} else if (METRIC == METRIC_DOT) {
		res = 1.0 - v[0];
	} else {
		res = 1.0 - v[0] / (sqrt(v[1]) * sqrt(v[NSUM - 1]));
	}
	float f = (float)res + 0.0f;  // canonical +0
	if (__builtin_isnan(f)) f = __builtin_nanf("");
	return f;
}

// rows per wave and refine round of pool_refine within the register budget of
// two waves per SIMD; cosine keeps three f64 sums per row (half the rows)
// NI: the refine path and row length of a pool_refine instantiation.
//   NI = 1..4: rows of <= 256 NI elements, every load of a wave's round in
//     flight at once (exact_distance_multi): small rounds (tau mode: k + 8
//     rows) pay one memory latency;
//   NI = 8 + (1..4): exact_rows_ring (SGPR row bases, half the rows' loads in
//     flight while the other half is summed, transpose-reduced sums): twice
//     the rows per wave, the final mode's large rounds;
//   NI = 0: rows past 1024 elements, one column step at a time.
template <int METRIC, int NI>
struct PrGeom {
	static constexpr int NS = NI & 7;  // 256-element steps (0: any length)
	static constexpr bool RING = NI >= 8;
	// rows per wave: the all-in-flight loads within the 256 VGPRs of two waves
	// per SIMD; cosine keeps three f64 sums per row (half the rows); 1024 threads
	// (four waves per SIMD, 128 VGPRs): half as many
	static constexpr int base = RING ? 16 : NS == 0 ? 16 : NS == 1 ? 16 : NS == 2 ? 12 : 8;
	static constexpr int PW0 = METRIC == METRIC_COSINE ? base / 2 : base;
	static constexpr int PW = PR_THREADS == 1024 ? PW0 / 2 : PW0;
};

// one refine round's exact distances of a wave's rows: lane r < nv gets row r's
// (PrGeom: the ring path, the all-in-flight path or the column-step path)
template <int METRIC, typename T, int PW, int NI>
__device__ __forceinline__ float pr_distances(const T *__restrict__ X, int ld, const uint32_t *sl, int nv,
                                              const float *__restrict__ qrow, const float *qs, int dim, int lane) {
	if (nv <= 0) return 0.f;
	constexpr int NS = PrGeom<METRIC, NI>::NS;
	if constexpr (PrGeom<METRIC, NI>::RING) {
		const float rv = exact_rows_ring<METRIC, T, PW, NS>(X, ld, sl, nv, qs, dim, lane);
		return __shfl(rv, (lane & (PW - 1)) * (64 / PW), 64);
	} else {
		float d[PW];
		exact_distance_multi<METRIC, T, PW, NS>(X, ld, sl, nv, qrow, qs, dim, lane, d);
		float dv = d[0];
#pragma unroll
		for (int r = 1; r < PW; ++r)
			if (lane == r) dv = d[r];
		return dv;
	}
}

// The k smallest of m entries (d[i], l[i]) by (distance, label) -> od/ol
// [0, min(m, k)), ascending (hit_less order; distances are canonical: +0, one
// NaN, so (fkey(d), label) is that order).  k <= PR_WMK, 48 < m <= 192: wave 0
// alone, entries in registers (3 per lane): a 32-step radix select of the
// min(m, k)-th smallest key by ballot counts, the entries at or below it
// compacted into od/ol, then each ranked against the others (a handful).
// Otherwise every thread ranks one entry against all m (O(m^2) LDS reads).
// The caller synchronises the block afterwards.
constexpr int PR_WMK = 32;
#ifndef LHIP_PR_WMK_MIN_M
#define LHIP_PR_WMK_MIN_M 48
#endif
constexpr int PR_WMK_MIN_M = LHIP_PR_WMK_MIN_M;  // (smaller merges, e.g. the tau mode's k + 8 rows: the rank form is cheaper)
template <int TH>
__device__ __forceinline__ void pr_merge(const float *d, const int64_t *l, float *od, int64_t *ol, int m, int k,
                                         int64_t tx) {
	const int t = threadIdx.x, lane = t & 63;
	if (k <= PR_WMK && m > PR_WMK_MIN_M && m <= 192) {
		if (t >= 64) return;
		constexpr int E = 3;
		uint32_t kk[E];
		bool vm[E];
#pragma unroll
		for (int e = 0; e < E; ++e) {
			const int i = lane + 64 * e;
			vm[e] = i < m;
			kk[e] = vm[e] ? fkey(d[i]) : 0xFFFFFFFFu;
		}
		const int want = min(m, k);
		// T = the want-th smallest key: bits from the top, below = keys < prefix
		uint32_t T = 0u;
		int below = 0;
		for (int b = 31; b >= 0; --b) {
			int c0 = 0;
#pragma unroll
			for (int e = 0; e < E; ++e)
				c0 += __builtin_popcountll(__builtin_amdgcn_ballot_w64(vm[e] && ((kk[e] ^ T) >> b) == 0u));
			if (below + c0 < want) {
				below += c0;
				T |= 1u << b;
			}
		}
		// every entry with key <= T (want of them, more on ties at T) -> od/ol [0, ns)
		float dv[E];
		int64_t lv[E];
		int base = 0;
#pragma unroll
		for (int e = 0; e < E; ++e) {
			const bool sel = vm[e] && kk[e] <= T;
			const uint64_t bm = __builtin_amdgcn_ballot_w64(sel);
			if (sel) {
				const int i = lane + 64 * e;
				dv[e] = d[i];
				lv[e] = l[i];
			}
			const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
			base += __builtin_popcountll(bm);
			kk[e] = sel ? (uint32_t)pos : 0xFFFFFFFFu;  // (now: the compacted position)
		}
		const int ns = base;
		// (d and od may alias nothing: the caller's buffers are the two halves)
#pragma unroll
		for (int e = 0; e < E; ++e)
			if (kk[e] != 0xFFFFFFFFu) {
				od[kk[e]] = dv[e];
				ol[kk[e]] = lv[e];
			}
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
		__builtin_amdgcn_wave_barrier();
		// rank each compacted entry (lane j < ns) among the ns: the smallest want go out
		float dj[E];
		int64_t lj[E];
		int rk[E];
#pragma unroll
		for (int e = 0; e < E; ++e) {
			const int j = lane + 64 * e;
			rk[e] = 0;
			if (j < ns) {
				dj[e] = od[j];
				lj[e] = ol[j];
			}
		}
		for (int i = 0; i < ns; ++i) {
			const float di = od[i];
			const int64_t li = ol[i];
#pragma unroll
			for (int e = 0; e < E; ++e)
				if (lane + 64 * e < ns) rk[e] += hit_less(di, li, dj[e], lj[e], tx) ? 1 : 0;
		}
		__builtin_amdgcn_wave_barrier();
#pragma unroll
		for (int e = 0; e < E; ++e)
			if (lane + 64 * e < ns && rk[e] < want) {
				od[rk[e]] = dj[e];
				ol[rk[e]] = lj[e];
			}
		return;
	}
	for (int i = t; i < m; i += TH) {
		const float di = d[i];
		const int64_t li = l[i];
		int rank = 0;
#pragma unroll 8
		for (int j = 0; j < m; ++j) rank += hit_less(d[j], l[j], di, li, tx) ? 1 : 0;
		if (rank < k) {
			od[rank] = di;
			ol[rank] = li;
		}
	}
}

// ascending bitonic sort of a[0, P) (P a power of two >= 64) by the block
template <int TH>
__device__ __forceinline__ void pr_bitonic(uint64_t *a, int P) {
	const int t = threadIdx.x;
	for (int size = 2; size <= P; size <<= 1) {
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			for (int i = t; i < (P >> 1); i += TH) {
				const int lo = 2 * i - (i & (stride - 1)), hi = lo + stride;
				const bool asc = (lo & size) == 0;
				const uint64_t x = a[lo], y = a[hi];
				if ((x > y) == asc) {
					a[lo] = y;
					a[hi] = x;
				}
			}
			__syncthreads();
		}
	}
}

constexpr int PR_SEL = 1024;  // chunk capacity
constexpr int PR_HB = 1024;   // histogram bins of a chunk selection
// Geometry of one pool_refine instantiation.  The tau-mode instantiations (NI
// = 1..4: the dispatch gives mode 0 the all-loads-in-flight path, mode 1 the
// ring) may take a smaller workgroup and pool (LHIP_PR_TAU_THREADS /
// LHIP_PR_TAU_CAP): they refine k + 8 rows, and a pool past the cap keeps its
// smallest bounds (any >= k real rows give a valid tau), so several of them
// can share a CU with the scans and the final refine.
#ifndef LHIP_PR_TAU_THREADS
#define LHIP_PR_TAU_THREADS LHIP_PR_THREADS
#endif
#ifndef LHIP_PR_TAU_CAP
#define LHIP_PR_TAU_CAP LHIP_PR_CAP
#endif
#ifndef LHIP_PR_TAU_MINW
#define LHIP_PR_TAU_MINW (LHIP_PR_TAU_THREADS == 256 ? 2 : 1)
#endif
template <int NI>
struct PrCfg {
	static constexpr bool TAU = NI >= 1 && NI <= 4;
	static constexpr int TH = TAU ? LHIP_PR_TAU_THREADS : PR_THREADS;
	static constexpr int CAP = TAU ? LHIP_PR_TAU_CAP : PR_CAP;
	static constexpr int MINW = TAU ? LHIP_PR_TAU_MINW : PR_MIN_WAVES;
	static constexpr int WAVES = TH / 64;
	static constexpr int BPT = PR_HB / TH;  // histogram bins per thread (4, 2 or 1)
	static_assert(TH == 256 || TH == 512 || TH == 1024, "pool_refine geometry");
	static_assert(BPT * TH == PR_HB && BPT >= 1 && BPT <= 4, "bins per thread");
};
constexpr int PR_R = 96;      // first chunk of the final pass (C2: ~80 rows lie below d_k; refined rows
                              // are the kernel's HBM traffic: 96 refined 18 % fewer than 128 at equal
                              // step time or better, r03s2)

template <int METRIC, typename T, int NI>
__global__ __launch_bounds__(PrCfg<NI>::TH, PrCfg<NI>::MINW) void pool_refine_kernel(
    const uint2 *__restrict__ seg_pool, const int *__restrict__ seg_cnt, int seg_cap, int n_seg, int nq,
    const float *__restrict__ tau, const T *__restrict__ X, int ld, int dim, const float *__restrict__ Qf,
    const int64_t *__restrict__ labels, int k, int mode, int m_tau, int64_t live, float *__restrict__ tau_out,
    int64_t *__restrict__ outL, float *__restrict__ outD, int *__restrict__ outC, int *__restrict__ cert,
    int *__restrict__ refined, int *__restrict__ pool_total, int prof_on, int r_first, int64_t tx) {
	constexpr int TH = PrCfg<NI>::TH, CAP = PrCfg<NI>::CAP, WAVES = PrCfg<NI>::WAVES, BPT = PrCfg<NI>::BPT;
	__shared__ uint64_t keys[CAP];
	__shared__ uint32_t sel[PR_SEL];  // slots of the chunk being refined
	__shared__ unsigned hist[PR_HB];
	__shared__ float cd[2][PR_MAXK + WAVES * PR_PER_WAVE];  // running top-k (double-buffered) + the round's distances
	__shared__ int64_t cl[2][PR_MAXK + WAVES * PR_PER_WAVE];
	__shared__ unsigned sh[WAVES];
	__shared__ int s_over, s_nnan, s_dnan;
	__shared__ unsigned s_nfin, s_knf, s_kmin, s_kmax, s_bstar, s_cum, s_below, s_ns, s_hi, s_pmin, s_pmax;
	__shared__ unsigned segc[TH];  // (big pools) segment counts
	constexpr int NS_ = PrGeom<METRIC, NI>::NS;
	__shared__ __attribute__((aligned(16))) float qs[NS_ > 0 ? 256 * NS_ : 4];  // the query row (NS_ > 0)
	const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
#ifdef LHIP_PR_PROF
	// phase stamps (diagnostic build, one designated launch): thread 0 keeps the
	// cycle counter at each phase boundary and stores them to g_pr_stamps at the
	// end (the host prints them after the launch: no printf inside the kernel,
	// whose host calls slowed the workgroups still running)
	uint64_t stamp[PR_NSTAMP];
	int nst = 0;
	auto mark = [&]() {
		if (nst < PR_NSTAMP) stamp[nst++] = __builtin_amdgcn_s_memtime();
	};
	mark();
#else
	auto mark = [&]() {};
#endif
	// candidates per wave and round (cosine: three f64 sums per row, half as many)
	constexpr int PW = PrGeom<METRIC, NI>::PW, CH = WAVES * PW;
	static_assert(CH <= WAVES * PR_PER_WAVE, "round buffer");
	if (t == 0) {
		s_over = 0;
		s_nnan = 0;
		s_dnan = 0;
		s_nfin = 0;
		s_knf = 0xFFFFFFFFu;
		s_pmin = 0xFFFFFFFFu;
		s_pmax = 0;
	}
	__syncthreads();
	// statistics of the keys as they are gathered (one reduction below, no pass
	// over the pool): finite count, NaN count, smallest non-finite key, the
	// finite keys' range (the first chunk's histogram range)
	unsigned g_nf = 0, g_nn = 0, g_knf = 0xFFFFFFFFu, g_kmn = 0xFFFFFFFFu, g_kmx = 0;
	auto gstat = [&](uint32_t kk) {
		if (kk < KEY_INF) {
			++g_nf;
			g_kmn = min(g_kmn, kk);
			g_kmx = max(g_kmx, kk);
		} else {
			g_knf = min(g_knf, kk);
		}
		g_nn += kk == KEY_NAN ? 1u : 0u;
	};
	// ---- gather the pool (thread s < n_seg: segment s) ----------------------
	unsigned c = 0;
	// the segment's first PR_SPEC entries (within its capacity) are loaded with
	// its count: one memory latency for the typical segment, not two (entries
	// past the count are never used)
	constexpr int PR_SPEC = 8;
	uint2 e0[PR_SPEC];
	if (t < n_seg) {
		const uint2 *seg = seg_pool + ((int64_t)t * nq + q) * seg_cap;
#pragma unroll
		for (int u = 0; u < PR_SPEC; ++u) e0[u] = u < seg_cap ? seg[u] : make_uint2(0u, 0u);
		const int cs = seg_cnt[(int64_t)t * nq + q];
		if (cs > seg_cap) s_over = 1;
		c = (unsigned)min(cs, seg_cap);
	}
	unsigned total;
	const unsigned off = block_excl_scan<TH>(c, sh, total);
	// a pool past CAP: keep its smallest bounds (whole histogram bins, at most
	// CAP) and treat the rest like rows outside the pool: cut <= the smallest
	// bound left out (excl_min), an exact certificate without a rerun.  Only when
	// one bin alone overflows do the first CAP entries stay (uncertified).
	unsigned excl_min = 0xFFFFFFFFu;
	bool big = false;
	if (total > (unsigned)CAP) {
		if (t < n_seg) segc[t] = c;
		if (t == 0) {
			s_kmin = 0xFFFFFFFFu;
			s_kmax = 0;
			s_bstar = 0xFFFFFFFFu;
			s_ns = 0;
			s_hi = 0xFFFFFFFFu;
		}
		for (int i = t; i < PR_HB; i += TH) hist[i] = 0;
		__syncthreads();
		const int m = max(1, TH / max(n_seg, 1));  // threads per segment
		const int sg = t / m, sub = t - sg * m;
		// every entry of this thread's segment share, 4 loads in flight
		auto each = [&](auto &&f) {
			if (sg >= n_seg) return;
			const uint2 *seg = seg_pool + ((int64_t)sg * nq + q) * seg_cap;
			const unsigned cs = segc[sg];
			for (unsigned i = sub; i < cs; i += 4u * m) {
				uint2 e[4];
#pragma unroll
				for (int u = 0; u < 4; ++u)
					if (i + u * m < cs) e[u] = seg[i + u * m];
#pragma unroll
				for (int u = 0; u < 4; ++u)
					if (i + u * m < cs) f(e[u]);
			}
		};
		unsigned kmn = 0xFFFFFFFFu, kmx = 0, nn = 0;
		each([&](uint2 e) {
			if (e.x < KEY_INF) {
				kmn = min(kmn, e.x);
				kmx = max(kmx, e.x);
			}
			nn += e.x == KEY_NAN ? 1u : 0u;
		});
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) {
			kmn = min(kmn, (unsigned)__shfl_xor(kmn, o, 64));
			kmx = max(kmx, (unsigned)__shfl_xor(kmx, o, 64));
			nn += __shfl_xor(nn, o, 64);
		}
		if (lane == 0) {
			atomicMin(&s_kmin, kmn);
			atomicMax(&s_kmax, kmx);
			if (nn) atomicAdd(&s_nnan, (int)nn);
		}
		__syncthreads();
		const unsigned kmin = s_kmin, kmax = s_kmax;
		const unsigned span = kmax - kmin;
		const int shift = kmin == 0xFFFFFFFFu ? 0 : (span >= (unsigned)PR_HB ? (32 - __builtin_clz(span)) - 10 : 0);
		if (kmin != 0xFFFFFFFFu) {
			each([&](uint2 e) {
				if (e.x < KEY_INF) atomicAdd(&hist[(e.x - kmin) >> shift], 1u);
			});
		}
		__syncthreads();
		{
			unsigned hb[BPT], hs = 0;
#pragma unroll
			for (int b = 0; b < BPT; ++b) {
				hb[b] = hist[BPT * t + b];
				hs += hb[b];
			}
			unsigned tot;
			const unsigned ex = block_excl_scan<TH>(hs, sh, tot);
			int cand = -1;  // the last bin whose inclusive count fits
			unsigned run = ex;
#pragma unroll
			for (int b = 0; b < BPT; ++b) {
				run += hb[b];
				if (run <= (unsigned)CAP) cand = BPT * t + b;
			}
			if (cand >= 0) atomicMax(reinterpret_cast<int *>(&s_bstar) + 0, cand);  // (s_bstar starts at -1)
		}
		__syncthreads();
		const int bstar = (int)s_bstar;
		if (kmin != 0xFFFFFFFFu && bstar >= 0) {
			big = true;
			unsigned xm = 0xFFFFFFFFu;
			each([&](uint2 e) {
				const bool keep = e.x < KEY_INF && (int)((e.x - kmin) >> shift) <= bstar;
				if (keep) {
					keys[atomicAdd(&s_ns, 1u)] = ((uint64_t)e.x << 32) | e.y;
					gstat(e.x);  // (finite: NaN bounds were counted over the whole pool above)
				} else
					xm = min(xm, e.x);
			});
#pragma unroll
			for (int o = 32; o > 0; o >>= 1) xm = min(xm, (unsigned)__shfl_xor(xm, o, 64));
			if (lane == 0) atomicMin(&s_hi, xm);
		}
		__syncthreads();
		excl_min = s_hi;
	}
	const int n = big ? (int)s_ns : (int)min(total, (unsigned)CAP);
#if LHIP_PR_SPREAD
	if (!big) {
		// each segment's first PR_SPEC entries came with its count (its owner thread
		// stores them); the rest are spread over every thread, 8 loads in flight,
		// each entry's segment found by a binary search of the segment offsets in
		// LDS: one or two memory latencies whatever the longest segment (the tau
		// mode's ~120 sample segments hold ~64 entries each: 7 rounds of 8 loads
		// for their owners before, round 6)
		if (t < n_seg && c && off < (unsigned)CAP) {
			const unsigned cm = min(min(c, (unsigned)CAP - off), (unsigned)PR_SPEC);
#pragma unroll
			for (int u = 0; u < PR_SPEC; ++u)
				if ((unsigned)u < cm) {
					keys[off + u] = ((uint64_t)e0[u].x << 32) | e0[u].y;
					gstat(e0[u].x);
				}
		}
		if (t < n_seg) segc[t] = off;  // segment start offsets (ascending; an empty one shares the next's)
		__syncthreads();
		for (int i0 = t; i0 < n; i0 += TH * 8) {
			uint2 e[8];
			int dst[8];
#pragma unroll
			for (int u = 0; u < 8; ++u) {
				const int i = i0 + u * TH;
				dst[u] = -1;
				if (i < n) {
					int lo = 0, hi = n_seg - 1;  // the last segment starting at or before i
					while (lo < hi) {
						const int mid = (lo + hi + 1) >> 1;
						if (segc[mid] <= (unsigned)i) lo = mid;
						else hi = mid - 1;
					}
					const unsigned j = (unsigned)i - segc[lo];
					if (j >= (unsigned)PR_SPEC) {
						e[u] = seg_pool[((int64_t)lo * nq + q) * seg_cap + j];
						dst[u] = i;
					}
				}
			}
#pragma unroll
			for (int u = 0; u < 8; ++u)
				if (dst[u] >= 0) {
					keys[dst[u]] = ((uint64_t)e[u].x << 32) | e[u].y;
					gstat(e[u].x);
				}
		}
	}
#else
	if (!big && t < n_seg && c && off < (unsigned)CAP) {
		const uint2 *seg = seg_pool + ((int64_t)t * nq + q) * seg_cap;
		const unsigned cm = min(c, (unsigned)CAP - off);
#pragma unroll
		for (int u = 0; u < PR_SPEC; ++u)
			if ((unsigned)u < cm) {
				keys[off + u] = ((uint64_t)e0[u].x << 32) | e0[u].y;
				gstat(e0[u].x);
			}
		for (unsigned i = PR_SPEC; i < cm; i += 8) {  // 8 loads in flight per thread
			uint2 e[8];
#pragma unroll
			for (int u = 0; u < 8; ++u)
				if (i + u < cm) e[u] = seg[i + u];
#pragma unroll
			for (int u = 0; u < 8; ++u)
				if (i + u < cm) {
					keys[off + i + u] = ((uint64_t)e[u].x << 32) | e[u].y;
					gstat(e[u].x);
				}
		}
	}
#endif
	// finite bounds (key < KEY_INF), NaN bounds, the smallest non-finite key and
	// the finite range, from the gather (big: NaN bounds were counted over the
	// whole pool above)
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) {
		g_nf += __shfl_xor(g_nf, o, 64);
		g_nn += __shfl_xor(g_nn, o, 64);
		g_knf = min(g_knf, (unsigned)__shfl_xor(g_knf, o, 64));
		g_kmn = min(g_kmn, (unsigned)__shfl_xor(g_kmn, o, 64));
		g_kmx = max(g_kmx, (unsigned)__shfl_xor(g_kmx, o, 64));
	}
	if (lane == 0) {
		if (g_nf) {
			atomicAdd(&s_nfin, g_nf);
			atomicMin(&s_pmin, g_kmn);
			atomicMax(&s_pmax, g_kmx);
		}
		if (g_nn) atomicAdd(&s_nnan, (int)g_nn);
		if (g_knf != 0xFFFFFFFFu) atomicMin(&s_knf, g_knf);
	}
	__syncthreads();
	mark();
	if (t == 0 && total > (unsigned)CAP && !big) s_over = 1;
	const int nfin = (int)s_nfin;
	const float ftau = tau ? tau[q] : F_INF;
	const float *qrow = Qf + (int64_t)q * ld;
	// the query row in LDS (NI > 0: every refine round reads it there, zero past dim)
	if (NS_ > 0)
		for (int i = t; i < 64 * 4 * (NS_ > 0 ? NS_ : 1); i += TH) qs[i] = i < dim ? qrow[i] : 0.f;

	// next chunk: the finite keys in [lo, hi_goal] up to a histogram bin holding
	// the R-th smallest of them (all of them when fewer), at most PR_SEL, slots
	// into sel.  Returns its size (0: none in the range) and its largest key in
	// s_hi (every key in [lo, s_hi] is in it); -1 when more than PR_SEL keys share
	// one value.
	auto next_chunk = [&](unsigned lo, unsigned hi_goal, int R) -> int {
		// every finite key (the first chunk): the range from the gather
		const bool whole_range = lo == 0u && hi_goal == KEY_INF - 1u;
		if (t == 0) {
			s_kmin = whole_range ? s_pmin : 0xFFFFFFFFu;
			s_kmax = whole_range ? s_pmax : 0u;
			s_ns = 0;
			s_hi = 0;
		}
		__syncthreads();
		if (!whole_range && R >= PR_SEL) {
			// a later chunk that takes every key in range (R = the capacity): one
			// appending pass, no histogram, unless the range holds more than a chunk
			for (int i = t; i < n; i += TH) {
				const uint64_t e = keys[i];
				const uint32_t kk = (uint32_t)(e >> 32);
				if (kk >= lo && kk <= hi_goal && kk < KEY_INF) {
					const unsigned p = atomicAdd(&s_ns, 1u);
					if (p < (unsigned)PR_SEL) sel[p] = (uint32_t)e;
					atomicMax(&s_hi, kk);
				}
			}
			__syncthreads();
			const unsigned cnt_in = s_ns;
			if (cnt_in <= (unsigned)PR_SEL) return (int)cnt_in;
			__syncthreads();
			if (t == 0) {
				s_ns = 0;
				s_hi = 0;
			}
			__syncthreads();
		}
		if (!whole_range) {
			unsigned kmn = 0xFFFFFFFFu, kmx = 0;
			for (int i = t; i < n; i += TH) {
				const uint32_t kk = (uint32_t)(keys[i] >> 32);
				if (kk >= lo && kk <= hi_goal && kk < KEY_INF) {
					kmn = min(kmn, kk);
					kmx = max(kmx, kk);
				}
			}
#pragma unroll
			for (int o = 32; o > 0; o >>= 1) {
				kmn = min(kmn, (unsigned)__shfl_xor(kmn, o, 64));
				kmx = max(kmx, (unsigned)__shfl_xor(kmx, o, 64));
			}
			if (lane == 0) {
				atomicMin(&s_kmin, kmn);
				atomicMax(&s_kmax, kmx);
			}
		}
		__syncthreads();
		unsigned kmin = s_kmin, kmax = s_kmax;
		if (kmin == 0xFFFFFFFFu) return 0;
		int shift;
		unsigned bstar;
		for (;;) {  // narrow until the chunk fits
			const unsigned span = kmax - kmin;
			shift = span >= (unsigned)PR_HB ? (32 - __builtin_clz(span)) - 10 : 0;  // (span >> shift) < PR_HB
			for (int i = t; i < PR_HB; i += TH) hist[i] = 0;
			if (t == 0) {
				s_bstar = PR_HB - 1;
				s_cum = 0xFFFFFFFFu;
				s_below = 0;
			}
			__syncthreads();
			for (int i = t; i < n; i += TH) {
				const uint32_t kk = (uint32_t)(keys[i] >> 32);
				if (kk >= kmin && kk <= kmax) atomicAdd(&hist[(kk - kmin) >> shift], 1u);
			}
			__syncthreads();
			unsigned hb[BPT], hs = 0;
#pragma unroll
			for (int b = 0; b < BPT; ++b) {
				hb[b] = hist[BPT * t + b];
				hs += hb[b];
			}
			unsigned tot;
			const unsigned ex = block_excl_scan<TH>(hs, sh, tot);
			if (ex < (unsigned)R && ex + hs >= (unsigned)R) {
				// this thread's first bin where the count reaches R
				unsigned run = ex;
				bool found = false;
#pragma unroll
				for (int b = 0; b < BPT; ++b) {
					if (!found && run + hb[b] >= (unsigned)R) {
						s_bstar = BPT * t + b;
						s_cum = run + hb[b];
						s_below = run;
						found = true;
					}
					run += hb[b];
				}
			}
			__syncthreads();
			bstar = s_bstar;
			const unsigned cum = s_cum == 0xFFFFFFFFu ? tot : s_cum, below = s_cum == 0xFFFFFFFFu ? tot : s_below;
			if (cum <= (unsigned)PR_SEL) break;
			if (below > 0) {  // the bins before b* alone
				unsigned b = bstar;
				while (b > 0 && hist[b - 1] == 0) --b;  // uniform: every thread reads the same bins
				bstar = b - 1;
				break;
			}
			if (shift == 0) return -1;  // > PR_SEL keys of one value
			// everything up to b* is inside b*: histogram that bin alone
			const unsigned nlo = kmin + (bstar << shift);
			kmin = nlo;
			kmax = min(kmax, nlo + ((1u << shift) - 1u));
			__syncthreads();
		}
		for (int i = t; i < n; i += TH) {
			const uint64_t e = keys[i];
			const uint32_t kk = (uint32_t)(e >> 32);
			if (kk >= kmin && kk <= kmax && ((kk - kmin) >> shift) <= bstar) {
				sel[atomicAdd(&s_ns, 1u)] = (uint32_t)e;
				atomicMax(&s_hi, kk);
			}
		}
		__syncthreads();
		return (int)s_ns;
	};

	// ---- refine in threshold chunks -------------------------------------------
	int cnt = 0, cur = 0, pos = 0;  // top entries held, buffer holding them, candidates refined
	float dk = F_INF;               // k-th distance of the top (+inf while fewer than k)
	unsigned lo = 0;                // the finite keys < lo are refined, those >= lo are not
	bool whole = false;             // > PR_SEL bounds of one value: the rest by the whole-pool sort
	const uint64_t *order = nullptr;  // (whole) the sorted pool
	for (;;) {
		int ns;
		const uint32_t *slots = sel;
		if (mode == 0) {
			if (pos >= min(nfin, m_tau)) break;
			ns = next_chunk(lo, KEY_INF - 1u, m_tau - pos);
		} else {
			// the bounds a bound-order refine could still take: <= nextafter(d_k)
			unsigned hi_goal = KEY_INF - 1u;
			if (cnt >= k && !__builtin_isnan(dk)) {
				const uint32_t kt = fkey(nextafterf(dk, F_INF));
				if (kt < lo) break;
				hi_goal = min(kt, KEY_INF - 1u);
			}
			ns = next_chunk(lo, hi_goal, cnt >= k ? PR_SEL : r_first);
		}
		mark();
		if (ns == 0) break;
		if (ns < 0) {
			whole = true;
			break;
		}
		lo = s_hi + 1u;  // (finite keys < KEY_INF: no wrap)
		for (int sp = 0; sp < ns; sp += CH) {
			const int nr = min(CH, ns - sp);
			// wave w refines candidates sp + w*PW .. (all its loads in flight together);
			// a small round of the ring instantiation (a later chunk: typically a
			// few dozen rows) spreads PR_SMALL rows per wave over every wave with all
			// its loads in flight (one memory latency, not one per column step)
			constexpr int PR_SMALL = 8;
			constexpr bool HAS_SMALL = PrGeom<METRIC, NI>::RING && PW > PR_SMALL && PrGeom<METRIC, NI>::NS <= 3;
			const bool small = HAS_SMALL && nr <= WAVES * PR_SMALL;
			{
				const int pw = small ? PR_SMALL : PW;
				uint32_t sl[PW];
				const int b0 = w * pw, nv = max(0, min(pw, nr - b0));
#pragma unroll
				for (int r = 0; r < PW; ++r) sl[r] = r < nv ? slots[sp + b0 + r] : 0u;
				// this lane's label load in flight with the row loads
				const int64_t lab = lane < nv ? labels[slots[sp + b0 + lane]] : 0;
				float dv;
				if constexpr (HAS_SMALL) {
					if (small)
						dv = pr_distances<METRIC, T, PR_SMALL, PrGeom<METRIC, NI>::NS>(X, ld, sl, nv, qrow, qs, dim, lane);
					else
						dv = pr_distances<METRIC, T, PW, NI>(X, ld, sl, nv, qrow, qs, dim, lane);
				} else {
					dv = pr_distances<METRIC, T, PW, NI>(X, ld, sl, nv, qrow, qs, dim, lane);
				}
				if (lane < nv) {
					cd[cur][cnt + b0 + lane] = dv;
					cl[cur][cnt + b0 + lane] = lab;
					if (__builtin_isnan(dv)) s_dnan = 1;
				}
			}
			mark();  // (thread 0 = wave 0: its own rows' distances done)
			__syncthreads();
			mark();
			// merge the top so far and this round by (distance, label)
			const int m = cnt + nr;
			if (!LHIP_ABL_PR_NOMERGE) pr_merge<TH>(cd[cur], cl[cur], cd[cur ^ 1], cl[cur ^ 1], m, k, tx);
			__syncthreads();
			cur ^= 1;
			cnt = min(m, k);
			dk = cnt >= k ? cd[cur][k - 1] : F_INF;
			pos += nr;
			mark();
		}
	}
	if (whole) {
		// > PR_SEL bounds of one value (duplicate rows): the rest in bound order
		// from the sorted pool, as a bound-order refine takes them
		int P = 64;
		while (P < n) P <<= 1;
		for (int i = n + t; i < P; i += TH) keys[i] = ~0ull;
		__syncthreads();
		pr_bitonic<TH>(keys, P);
		order = keys;
		int sp = pos;  // the first pos entries of the sorted pool are the keys < lo
		const int limit = mode == 0 ? min(nfin, m_tau) : nfin;
		while (sp < limit) {
			if (mode == 1 && cnt >= k && fkey_inv((uint32_t)(order[sp] >> 32)) > nextafterf(dk, F_INF)) break;
			const int nr = min(CH, limit - sp);
			{
				uint32_t sl[PW];
				const int b0 = w * PW, nv = max(0, min(PW, nr - b0));
#pragma unroll
				for (int r = 0; r < PW; ++r) sl[r] = r < nv ? (uint32_t)order[sp + b0 + r] : 0u;
				const float dv = pr_distances<METRIC, T, PW, NI>(X, ld, sl, nv, qrow, qs, dim, lane);
				if (lane < nv) {
					uint32_t sv = sl[0];
#pragma unroll
					for (int r = 1; r < PW; ++r)
						if (lane == r) sv = sl[r];
					cd[cur][cnt + b0 + lane] = dv;
					cl[cur][cnt + b0 + lane] = labels[sv];
					if (__builtin_isnan(dv)) s_dnan = 1;
				}
			}
			__syncthreads();
			const int m = cnt + nr;
			pr_merge<TH>(cd[cur], cl[cur], cd[cur ^ 1], cl[cur ^ 1], m, k, tx);
			__syncthreads();
			cur ^= 1;
			cnt = min(m, k);
			dk = cnt >= k ? cd[cur][k - 1] : F_INF;
			sp += nr;
			pos += nr;
		}
		lo = sp < nfin ? (uint32_t)(order[sp] >> 32) : KEY_INF;  // the next bound, as the smallest unrefined key
	}
	if (mode == 0) {
		if (t == 0) {
			const float tk = s_dnan ? __builtin_nanf("") : (cnt >= k ? cd[cur][k - 1] : F_INF);
			// with an input tau (a later threshold pass): the smaller of the two,
			// the input when this one is NaN
			tau_out[q] = !tau ? tk : (tk < ftau ? tk : ftau);
			if (refined) refined[q] = pos;
			if (pool_total) pool_total[q] = s_over ? -1 : (int)total;
		}
		return;
	}
	// ---- outputs and the certificate -----------------------------------------
	// the smallest unrefined finite bound (every finite key < lo is refined)
	if (t == 0) s_kmin = 0xFFFFFFFFu;
	__syncthreads();
	if (!whole) {
		unsigned kmn = 0xFFFFFFFFu;
		for (int i = t; i < n; i += TH) {
			const uint32_t kk = (uint32_t)(keys[i] >> 32);
			if (kk >= lo && kk < KEY_INF) kmn = min(kmn, kk);
		}
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) kmn = min(kmn, (unsigned)__shfl_xor(kmn, o, 64));
		if (lane == 0) atomicMin(&s_kmin, kmn);
	} else if (t == 0 && lo < KEY_INF) {
		s_kmin = lo;
	}
	for (int i = t; i < k; i += TH) {
		outL[(int64_t)q * k + i] = i < cnt ? cl[cur][i] : -1;
		outD[(int64_t)q * k + i] = i < cnt ? cd[cur][i] : __builtin_nanf("");
	}
	__syncthreads();
	if (t == 0) {
		// every row not refined has LB >= cut: the smallest unrefined bound (a
		// finite one, else the smallest non-finite), +inf when the pool is
		// exhausted; tau for the rows outside the pool
		float cutv;
		if (s_kmin != 0xFFFFFFFFu)
			cutv = fkey_inv(s_kmin);
		else if (n > nfin)
			cutv = fkey_inv(s_knf);
		else
			cutv = F_INF;
		// (big pool: the bounds left out of it)
		if (excl_min != 0xFFFFFFFFu && excl_min != KEY_NAN && fkey_inv(excl_min) < cutv) cutv = fkey_inv(excl_min);
		if (ftau < cutv) cutv = ftau;
		if (s_over || s_nnan > 0) cutv = -F_INF;
		bool ok;
		if (cutv == F_INF)
			ok = true;  // nothing live was left out
		else
			ok = !__builtin_isnan(dk) && dk < F_INF && cutv > nextafterf(dk, F_INF);
		if (live >= 0 && (int64_t)cnt < (live < (int64_t)k ? live : (int64_t)k)) ok = false;
		outC[q] = cnt;
		cert[q] = ok ? 1 : 0;
#ifdef LHIP_PR_PROF
		mark();
		if (prof_on && q < PR_PROF_Q) {
			uint64_t *o = g_pr_stamps + (size_t)q * (PR_NSTAMP + 3);
			o[0] = (uint64_t)nst;
			o[1] = (uint64_t)n;
			o[2] = (uint64_t)pos;
			for (int i = 0; i < nst; ++i) o[3 + i] = stamp[i];
		}
#endif
		if (refined) refined[q] = pos;
		if (pool_total) pool_total[q] = s_over ? -1 : (int)total;
	}
}

int pool_refine_max_first() { return PR_SEL; }

#ifdef LHIP_PR_PROF
// host side of the phase stamps: the designated launch's per-query stamps,
// printed as cycle deltas (PR q=.. pool=.. refined=.. | d0 d1 ...)
static void pr_prof_dump(hipStream_t st) {
	static uint64_t h[PR_PROF_Q * (PR_NSTAMP + 3)];
	if (hipStreamSynchronize(st) != hipSuccess) return;
	if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_pr_stamps), sizeof(h)) != hipSuccess) return;
	for (int q = 0; q < PR_PROF_Q; ++q) {
		const uint64_t *o = h + (size_t)q * (PR_NSTAMP + 3);
		const int nst = (int)o[0];
		if (nst < 2) continue;
		fprintf(stderr, "PR q=%d pool=%d refined=%d nst=%d total=%lld |", q, (int)o[1], (int)o[2], nst,
		        (long long)(o[3 + nst - 1] - o[3]));
		for (int i = 1; i < nst; ++i) fprintf(stderr, " %lld", (long long)(o[3 + i] - o[3 + i - 1]));
		fprintf(stderr, "\n");
	}
}
#endif

template <typename T>
static void pool_refine_dispatch(const StoreView &s, const QueryView &q, const uint2 *seg_pool, const int *seg_cnt,
                                 int seg_cap, int n_seg, const float *tau, int k, int mode, int m_tau,
                                 int64_t live, float *tau_out, int64_t *L, float *D, int *C, int *cert, int *refined,
                                 int *pool_total, hipStream_t st) {
	const T *X = static_cast<const T *>(s.X);
	const dim3 grid((unsigned)q.nq);
#ifdef LHIP_PR_PROF
	static std::atomic<int> calls{0};  // (diagnostic build: the 12th final-mode launch of the process prints its phases)
	const int prof_on = mode == 1 && ++calls == 12;
	struct Dump {  // prints after the designated launch (any return path)
		int on;
		hipStream_t st;
		~Dump() {
			if (on) pr_prof_dump(st);
		}
	} dump_{prof_on, st};
#else
	const int prof_on = 0;
#endif
	const int r_first = s.pr_first > 0 ? std::max(8, std::min(PR_SEL, s.pr_first)) : PR_R;
#define LHIP_PR(MET, NI)                                                                                              \
	pool_refine_kernel<MET, T, NI><<<grid, PrCfg<NI>::TH, 0, st>>>(seg_pool, seg_cnt, seg_cap, n_seg, q.nq, tau, X, s.ld,\
	                                                            s.dim, q.Qf, s.labels, k, mode, m_tau, live, tau_out,  \
	                                                            L, D, C, cert, refined, pool_total, prof_on, r_first,  \
	                                                            tie_x64(s.tie_desc))
#define LHIP_PR_NI(MET)                                                                                               \
	switch (ni) {                                                                                                      \
	case 1: LHIP_PR(MET, 1); break;                                                                                    \
	case 2: LHIP_PR(MET, 2); break;                                                                                    \
	case 3: LHIP_PR(MET, 3); break;                                                                                    \
	case 4: LHIP_PR(MET, 4); break;                                                                                    \
	case 9: LHIP_PR(MET, 9); break;                                                                                    \
	case 10: LHIP_PR(MET, 10); break;                                                                                  \
	case 11: LHIP_PR(MET, 11); break;                                                                                  \
	case 12: LHIP_PR(MET, 12); break;                                                                                  \
	default: LHIP_PR(MET, 0); break;                                                                                   \
	}
	// row length in 256-element steps (one 16-B load per lane each, PrGeom): <= 4
	// -> tau mode all loads of a round in flight, final mode exact_rows_ring;
	// longer rows one column step at a time
#ifdef LHIP_PR_FORCE_NI0  // (development builds: the one-column-step path everywhere)
	const int ni = 0;
#else
	const int ns = s.dim <= 256 ? 1 : s.dim <= 512 ? 2 : s.dim <= 768 ? 3 : s.dim <= 1024 ? 4 : 0;
	// tau mode (k + 8 rows: one small round) every load in flight; final mode the ring
	// (more segments than a tau-mode workgroup has threads: the column-step path,
	// which keeps the default geometry)
	const int ni = ns == 0 ? 0 : mode == 1 ? 8 + ns : n_seg > PrCfg<1>::TH ? 0 : ns;
#endif
	switch (s.metric) {
	case METRIC_L2: LHIP_PR_NI(METRIC_L2); break;
	case METRIC_DOT: LHIP_PR_NI(METRIC_DOT); break;
	default: LHIP_PR_NI(METRIC_COSINE); break;
	}
#undef LHIP_PR_NI
#undef LHIP_PR
}

void launch_pool_refine(const StoreView &s, const QueryView &q, const uint2 *seg_pool, const int *seg_cnt,
                        int seg_cap, int n_seg, const float *tau, int k, int mode, int m_tau, int64_t live,
                        float *tau_out, int64_t *L, float *D, int *C, int *cert, int *refined, int *pool_total,
                        hipStream_t st) {
	if (q.nq <= 0) return;
	if (n_seg > PR_THREADS) throw std::runtime_error("pool_refine: more segments than threads");
	if (k <= 0 || k > PR_MAXK) throw std::runtime_error("pool_refine: k past the selection capacity");
	if (mode == 0 && m_tau > PR_MAXK) throw std::runtime_error("pool_refine: m_tau past the selection capacity");
	if (s.xbf16)
		pool_refine_dispatch<uint16_t>(s, q, seg_pool, seg_cnt, seg_cap, n_seg, tau, k, mode, m_tau, live, tau_out, L,
		                               D, C, cert, refined, pool_total, st);
	else
		pool_refine_dispatch<float>(s, q, seg_pool, seg_cnt, seg_cap, n_seg, tau, k, mode, m_tau, live, tau_out, L, D,
		                            C, cert, refined, pool_total, st);
}

// ---------------------------------------------------------------------------
// exact fallback
// ---------------------------------------------------------------------------
template <int METRIC, typename T>
__global__ __launch_bounds__(256) void exact_all_kernel(const T *__restrict__ X, const float4 *__restrict__ rowaux,
                                                        const int64_t *__restrict__ labels, int64_t n, int ld,
                                                        int dim, const float *__restrict__ q,
                                                        float *__restrict__ keys, int64_t *__restrict__ vals,
                                                        int tie_desc) {
	const int lane = threadIdx.x & 63;
	const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	if (r >= n) return;
	float d = exact_distance<METRIC, T>(X + r * ld, q, dim, lane);
	if (lane == 0) {
		const float a = reinterpret_cast<const float *>(rowaux)[raix(r, 0)];
		const bool dead = (a == F_INF);
		// (label-descending ties: entry n-1-r, the stable sort then keeps equal
		// distances in reverse slot = label order)
		const int64_t e = tie_desc ? n - 1 - r : r;
		keys[e] = dead ? __uint_as_float(0x7FFFFFFFu) : d;
		vals[e] = labels[r];
	}
}

template <typename T>
static void exact_all_dispatch(const StoreView &s, const QueryView &q, int qi, float *keys, int64_t *vals,
                               hipStream_t st) {
	dim3 grid((unsigned)((s.n_slots + 3) / 4));
	const float *qq = q.Qf + (int64_t)qi * s.ld;
	const T *X = static_cast<const T *>(s.X);
	switch (s.metric) {
	case METRIC_L2:
		exact_all_kernel<METRIC_L2, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld, s.dim, qq, keys,
		                                                      vals, s.tie_desc);
		break;
	case METRIC_DOT:
		exact_all_kernel<METRIC_DOT, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld, s.dim, qq, keys,
		                                                       vals, s.tie_desc);
		break;
	default:
		exact_all_kernel<METRIC_COSINE, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld, s.dim, qq,
		                                                          keys, vals, s.tie_desc);
		break;
	}
}

// Batched exact fallback: one wave per row computes the row's exact distance
// to each of the nq queries with the same exact_distance() as refine (f64
// accumulation, identical order), so a key equals the distance refine will
// report; the row is read from HBM once and from L1/L2 for the other queries.
// Dead / filtered slots get +inf (select_kernel leaves them out).
template <int METRIC, typename T>
__global__ __launch_bounds__(256) void exact_dense_kernel(const T *__restrict__ X, const float4 *__restrict__ rowaux,
                                                          int64_t n, int ld, int dim, const float *__restrict__ Qf,
                                                          int nq, float *__restrict__ keys, int64_t ld_keys) {
	const int lane = threadIdx.x & 63;
	const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	if (r >= n) return;
	const bool dead = reinterpret_cast<const float *>(rowaux)[raix(r, 0)] == F_INF;
	for (int qi = 0; qi < nq; ++qi) {
		float d = F_INF;
		if (!dead) d = exact_distance<METRIC, T>(X + r * ld, Qf + (int64_t)qi * ld, dim, lane);
		if (lane == 0) keys[(int64_t)qi * ld_keys + r] = d;
	}
}

template <typename T>
static void exact_dense_dispatch(const StoreView &s, const QueryView &q, float *keys, int64_t ld_keys, hipStream_t st) {
	dim3 grid((unsigned)((s.n_slots + 3) / 4));
	const T *X = static_cast<const T *>(s.X);
	switch (s.metric) {
	case METRIC_L2:
		exact_dense_kernel<METRIC_L2, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.n_slots, s.ld, s.dim, q.Qf, q.nq, keys,
		                                                        ld_keys);
		break;
	case METRIC_DOT:
		exact_dense_kernel<METRIC_DOT, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.n_slots, s.ld, s.dim, q.Qf, q.nq, keys,
		                                                         ld_keys);
		break;
	default:
		exact_dense_kernel<METRIC_COSINE, T><<<grid, 256, 0, st>>>(X, s.rowaux, s.n_slots, s.ld, s.dim, q.Qf, q.nq,
		                                                            keys, ld_keys);
		break;
	}
}

void launch_exact_dense(const StoreView &s, const QueryView &q, float *keys, int64_t ld_keys, hipStream_t st) {
	if (s.n_slots <= 0 || q.nq <= 0) return;
	if (ld_keys < s.n_slots) throw std::runtime_error("exact_dense: key rows shorter than the store");
	if (s.xbf16)
		exact_dense_dispatch<uint16_t>(s, q, keys, ld_keys, st);
	else
		exact_dense_dispatch<float>(s, q, keys, ld_keys, st);
}

void launch_exact_all(const StoreView &s, const QueryView &q, int qi, float *keys, int64_t *vals, hipStream_t st) {
	if (s.n_slots <= 0) return;
	if (s.xbf16)
		exact_all_dispatch<uint16_t>(s, q, qi, keys, vals, st);
	else
		exact_all_dispatch<float>(s, q, qi, keys, vals, st);
}

int sort_pairs(void *temp, size_t &temp_bytes, const float *keys_in, float *keys_out, const int64_t *vals_in,
               int64_t *vals_out, int64_t n, hipStream_t st) {
	hipError_t e = rocprim::radix_sort_pairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (size_t)n, 0,
	                                         32, st);
	return (int)e;
}

__global__ void copy_fallback_kernel(const float *keys, const int64_t *vals, int64_t n_live, int k, int qi,
                                     int64_t *out_labels, float *out_dists, int *out_counts) {
	int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= k) return;
	if (i < n_live) {
		out_labels[(int64_t)qi * k + i] = vals[i];
		out_dists[(int64_t)qi * k + i] = keys[i];
	} else {
		out_labels[(int64_t)qi * k + i] = -1;
		out_dists[(int64_t)qi * k + i] = __builtin_nanf("");
	}
	if (i == 0) out_counts[qi] = (int)(n_live < k ? n_live : k);
}

void launch_copy_fallback(const float *keys, const int64_t *vals, int64_t n_live, int k, int qi, int64_t *out_labels,
                          float *out_dists, int *out_counts, hipStream_t st) {
	copy_fallback_kernel<<<dim3((k + 255) / 256), dim3(256), 0, st>>>(keys, vals, n_live, k, qi, out_labels,
	                                                                   out_dists, out_counts);
}

// ---------------------------------------------------------------------------
// small exact search: one launch for a few queries over a small store
// (the per-query lance_search call pattern, C1).  Thread = row: exact distance
// in f64 (sequential over the dimension, rounded once to f32: the oracle's
// definition); a bitonic sort of the workgroup's 256 rows by (distance,
// label) puts its top-k in a partial list; the last workgroup of the query to
// finish (device-scope counter) keeps the partial entries that can still
// place and sorts those.  No bounds, no certificate, no host round trip in between.
// ---------------------------------------------------------------------------
#ifndef LHIP_ABL_SMALL_NOWGSORT
#define LHIP_ABL_SMALL_NOWGSORT 0
#endif
#ifndef LHIP_ABL_SMALL_NOMERGE
#define LHIP_ABL_SMALL_NOMERGE 0
#endif
#ifndef LHIP_ABL_SMALL_NOFENCE
#define LHIP_ABL_SMALL_NOFENCE 0  // timing ablation (tools/ablate.sh): results wrong by design
#endif
struct SHit {
	float d;
	int v;  // 1 = live row
	int64_t l;
};

__device__ __forceinline__ bool shit_less(const SHit &a, const SHit &b, int64_t tx) {
	if (a.v != b.v) return a.v > b.v;
	return hit_less(a.d, a.l, b.d, b.l, tx);
}

// ascending bitonic sort of s[0..n) (n a power of two) by the whole block
__device__ __forceinline__ void shit_sort(SHit *s, int n, int64_t tx) {
	const int t = threadIdx.x;
	for (int size = 2; size <= n; size <<= 1) {
		for (int j = size >> 1, lj = __builtin_ctz(size >> 1); j > 0; j >>= 1, --lj) {
			for (int i = t; i < (n >> 1); i += SMALL_THREADS) {
				const int lo = ((i >> lj) << (lj + 1)) | (i & (j - 1)), hi = lo + j;
				const bool up = (lo & size) == 0;
				const SHit a = s[lo], b = s[hi];
				if (up ? shit_less(b, a, tx) : shit_less(a, b, tx)) {
					s[lo] = b;
					s[hi] = a;
				}
			}
			__syncthreads();
		}
	}
}

// ascending bitonic sort of one 64-bit key per lane across the wave (registers
// and cross-lane shuffles only: no LDS round trips, no barriers)
__device__ __forceinline__ uint64_t wave_sort_u64(uint64_t key, int lane) {
#pragma unroll
	for (int size = 2; size <= 64; size <<= 1)
#pragma unroll
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			const uint64_t other = __shfl_xor(key, stride, 64);
			const bool keep_min = ((lane & stride) == 0) == ((lane & size) == 0 || size == 64);
			key = keep_min ? (key < other ? key : other) : (key < other ? other : key);
		}
	return key;
}
// a and b ascending in lanes 0..31 (~0 past their valid entries): the 64
// smallest of both, ascending (a bitonic merge of a with b reversed)
__device__ __forceinline__ uint64_t wave_merge_u64(uint64_t a, uint64_t b, int lane) {
	const uint64_t br = __shfl(b, 63 - lane, 64);
	uint64_t key = lane < 32 ? a : br;
#pragma unroll
	for (int stride = 32; stride > 0; stride >>= 1) {
		const uint64_t other = __shfl_xor(key, stride, 64);
		key = (lane & stride) == 0 ? (key < other ? key : other) : (key < other ? other : key);
	}
	return key;
}

template <int METRIC, typename T>
__global__ __launch_bounds__(SMALL_THREADS) void small_exact_kernel(const T *__restrict__ X,
                                                                    const float4 *__restrict__ rowaux,
                                                                    const int64_t *__restrict__ labels, int64_t n,
                                                                    int ld, int dim, const float *__restrict__ Q, int k,
                                                                    SHit *__restrict__ part,
                                                                    unsigned *__restrict__ counter,
                                                                    int64_t *__restrict__ out_l,
                                                                    float *__restrict__ out_d, int *__restrict__ out_c,
                                                                    int se_prof, int tie_desc) {
	const int64_t tx = tie_x64(tie_desc);
	const uint32_t sx = tie_x32(tie_desc);  // (k <= 32 keys: slot ^ sx)
	__shared__ __attribute__((aligned(16))) float sq[SMALL_MAX_DIM];
	__shared__ SHit s_rows[SMALL_MAX_PART], s2[SMALL_MAX_PART], red[SMALL_THREADS];
	__shared__ unsigned s_ns;
	__shared__ int s_last;
	SHit *s = s_rows;
	const int q = blockIdx.y, G = gridDim.x, t = threadIdx.x;
	uint64_t mykey;  // (k <= 32 path) this lane's row key
	__shared__ uint64_t wkeys[SMALL_THREADS];
#ifdef LHIP_SE_PROF
	uint64_t st_[12];
	int nst_ = 0;
#define SE_T() \
	if (nst_ < 12) st_[nst_++] = __builtin_amdgcn_s_memtime()
	SE_T();
#else
#define SE_T()
#endif
	for (int i = t; i < dim; i += SMALL_THREADS) sq[i] = Q[(int64_t)q * dim + i];
	__syncthreads();
	// distances: each wave takes 64 of the workgroup's rows in 8 groups of 8;
	// a row is split over 8 lanes (float4 chunks sub, sub + 8, ...: coalesced
	// row reads), partial f64 sums reduced over the 8 lanes (the sum of the
	// same products as exact_distance).  Per chunk of SE_CH float4 per lane
	// the loads of all 8 groups are issued before any product (one memory
	// latency per chunk instead of one per group and chunk; each lane's
	// summation order is unchanged: chunk, then its float4 in order).
	{
		constexpr int SE_CH = 4;
		const int lane = t & 63, w = t >> 6, sub = lane & 7;
		const int d4 = dim >> 2;  // rows are padded to a multiple of 4 elements: aligned 16-B (8-B bf16) loads
		int64_t r[8];
		bool ok[8];
		double a[8], b[8], c[8];
		mykey = ~0ull;
#pragma unroll
		for (int g = 0; g < 8; ++g) {
			r[g] = (int64_t)blockIdx.x * SMALL_THREADS + w * 64 + g * 8 + (lane >> 3);
			ok[g] = r[g] < n && reinterpret_cast<const float *>(rowaux)[raix(r[g] < n ? r[g] : 0, 0)] != F_INF;
			a[g] = b[g] = c[g] = 0.0;
		}
		for (int c0 = sub; c0 < d4; c0 += 8 * SE_CH) {
			float4 qv[SE_CH], xv[8][SE_CH];
#pragma unroll
			for (int u = 0; u < SE_CH; ++u) {
				const int i4 = c0 + 8 * u;
				qv[u] = i4 < d4 ? *reinterpret_cast<const float4 *>(sq + 4 * i4) : make_float4(0.f, 0.f, 0.f, 0.f);
			}
#pragma unroll
			for (int g = 0; g < 8; ++g)
#pragma unroll
				for (int u = 0; u < SE_CH; ++u) {
					const int i4 = c0 + 8 * u;
					xv[g][u] = (ok[g] && i4 < d4) ? xval4(X + r[g] * ld, 4 * i4) : make_float4(0.f, 0.f, 0.f, 0.f);
				}
#pragma unroll
			for (int g = 0; g < 8; ++g)
#pragma unroll
				for (int u = 0; u < SE_CH; ++u)
					if (c0 + 8 * u < d4) {  // (only real chunks: a padded product would change cosine's sums)
						exact_acc<METRIC>(xv[g][u].x, qv[u].x, a[g], b[g], c[g]);
						exact_acc<METRIC>(xv[g][u].y, qv[u].y, a[g], b[g], c[g]);
						exact_acc<METRIC>(xv[g][u].z, qv[u].z, a[g], b[g], c[g]);
						exact_acc<METRIC>(xv[g][u].w, qv[u].w, a[g], b[g], c[g]);
					}
		}
#pragma unroll
		for (int g = 0; g < 8; ++g) {
			if (ok[g])
				for (int i = 4 * d4 + sub; i < dim; i += 8)
					exact_acc<METRIC>(xval(X + r[g] * ld, i), sq[i], a[g], b[g], c[g]);
#pragma unroll
			for (int o = 1; o < 8; o <<= 1) {
				a[g] += __shfl_xor(a[g], o, 64);
				if (METRIC == METRIC_COSINE) {
					b[g] += __shfl_xor(b[g], o, 64);
					c[g] += __shfl_xor(c[g], o, 64);
				}
			}
			if (sub == 0) {
				SHit h{F_INF, 0, INT64_MAX};
				if (ok[g]) {
					double v;
					if (METRIC == METRIC_L2)
						v = a[g];
					else if (METRIC == METRIC_DOT)
						v = 1.0 - a[g];
					else
						v = 1.0 - a[g] / (sqrt(b[g]) * sqrt(c[g]));
					float f = (float)v + 0.0f;
					if (__builtin_isnan(f)) f = __builtin_nanf("");
					h = SHit{f, 1, labels[r[g]]};
				}
				s[w * 64 + g * 8 + (lane >> 3)] = h;
			}
			// (every lane of the 8 holds the sums: lane sub keeps group sub's row,
			// one row per lane; key = (ordered distance, slot ^ sx): slots ascend
			// with labels, so key order is (distance, label) order under the tie
			// rule, NaN last, none last)
			if (sub == g && ok[g]) {
				double v;
				if (METRIC == METRIC_L2)
					v = a[g];
				else if (METRIC == METRIC_DOT)
					v = 1.0 - a[g];
				else
					v = 1.0 - a[g] / (sqrt(b[g]) * sqrt(c[g]));
				float f = (float)v + 0.0f;
				if (__builtin_isnan(f)) f = __builtin_nanf("");
				mykey = ((uint64_t)fkey(f) << 32) | ((uint32_t)r[g] ^ sx);
			}
		}
	}
	__syncthreads();
	SE_T();
	const int lane = t & 63, wv = t >> 6;
	constexpr int NWV = SMALL_THREADS / 64;
	if (k <= 32) {
		// ---- k <= 32: register sorts of 64-bit keys, no workgroup sort --------
		uint64_t key = wave_sort_u64(mykey, lane);
		wkeys[t] = lane < k ? key : ~0ull;
		__syncthreads();
		if (wv == 0) {
			uint64_t acc = wkeys[lane];
#pragma unroll
			for (int v = 1; v < NWV; ++v) {
				acc = wave_merge_u64(acc, wkeys[v * 64 + lane], lane);
				if (lane >= k) acc = ~0ull;
			}
			uint64_t *mine = reinterpret_cast<uint64_t *>(part) + ((int64_t)q * G + blockIdx.x) * k;
			if (lane < k) mine[lane] = acc;
			__threadfence();
		}
		__syncthreads();
		if (t == 0) s_last = atomicAdd(&counter[q], 1u) == (unsigned)(G - 1);
		__syncthreads();
		if (!s_last) return;
		__threadfence();
		// merge: only keys <= thr = the smallest of the lists' k-th keys can
		// place; each wave takes 64-key chunks of those, keeps a running top-k,
		// and wave 0 merges the waves' lists
		const uint64_t *all = reinterpret_cast<const uint64_t *>(part) + (int64_t)q * G * k;
		const int P = G * k;
		uint64_t tk = ~0ull;
		for (int g = t; g < G; g += SMALL_THREADS) tk = min(tk, all[(int64_t)g * k + k - 1]);
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) tk = min(tk, (uint64_t)__shfl_xor(tk, o, 64));
		if (lane == 0) wkeys[wv] = tk;
		if (t == 0) s_ns = 0;
		__syncthreads();
		uint64_t thr = wkeys[0];
#pragma unroll
		for (int v = 1; v < NWV; ++v) thr = min(thr, wkeys[v]);
		uint64_t *cand = reinterpret_cast<uint64_t *>(s2);
		for (int i = t; i < P; i += SMALL_THREADS) {
			const uint64_t e = all[i];
			if (e <= thr) cand[atomicAdd(&s_ns, 1u)] = e;
		}
		__syncthreads();
		const int ns = (int)s_ns;
		uint64_t best = ~0ull;
		for (int c0 = wv * 64; c0 < ns; c0 += NWV * 64) {
			uint64_t ck = c0 + lane < ns ? cand[c0 + lane] : ~0ull;
			ck = wave_sort_u64(ck, lane);
			if (lane >= k) ck = ~0ull;
			best = wave_merge_u64(best, ck, lane);
			if (lane >= k) best = ~0ull;
		}
		__syncthreads();  // (wkeys reused)
		wkeys[t] = best;
		__syncthreads();
		if (wv == 0) {
			uint64_t acc = wkeys[lane];
#pragma unroll
			for (int v = 1; v < NWV; ++v) {
				acc = wave_merge_u64(acc, wkeys[v * 64 + lane], lane);
				if (lane >= k) acc = ~0ull;
			}
			if (lane < k) {
				const bool valid = acc != ~0ull;
				out_l[(int64_t)q * k + lane] = valid ? labels[(uint32_t)acc ^ sx] : -1;
				out_d[(int64_t)q * k + lane] = valid ? fkey_inv((uint32_t)(acc >> 32)) : __builtin_nanf("");
			}
			const uint64_t vm = __builtin_amdgcn_ballot_w64(lane < k && acc != ~0ull);
			if (lane == 0) {
				out_c[q] = __builtin_popcountll(vm);
				counter[q] = 0u;  // ready for the next launch on this stream
			}
		}
		return;
	}
	// ---- k > 32: bitonic sorts of the workgroup's rows ------------------------
	// this workgroup's top-k: sorted by (distance, label)
	if (!LHIP_ABL_SMALL_NOWGSORT) shit_sort(s, SMALL_THREADS, tx);
	SE_T();
	SHit *mine = part + ((int64_t)q * G + blockIdx.x) * k;
	for (int i = t; i < k; i += SMALL_THREADS) mine[i] = s[i];
	if (!LHIP_ABL_SMALL_NOFENCE) __threadfence();
	__syncthreads();
	if (t == 0) s_last = atomicAdd(&counter[q], 1u) == (unsigned)(G - 1);
	__syncthreads();
	SE_T();
#ifdef LHIP_SE_PROF
	if (!s_last && t == 0 && blockIdx.x < 2 && se_prof)
		printf("SE wg=%d dist=%d sort=%d publish=%d\n", blockIdx.x, (int)(st_[1] - st_[0]), (int)(st_[2] - st_[1]),
		       (int)(st_[3] - st_[2]));
#endif
	if (!s_last) return;
	if (!LHIP_ABL_SMALL_NOFENCE) __threadfence();
	// merge: every list is sorted, so the k-th smallest overall is <= each
	// list's k-th entry; only entries <= thr = the smallest of those can place
	// (typically a few k of the G*k): they alone are sorted
	const int P = G * k;
	const SHit *all = part + (int64_t)q * G * k;
	for (int i = t; i < P; i += SMALL_THREADS) s[i] = all[i];
	if (t == 0) s_ns = 0;
	__syncthreads();
	if (t < G) red[t] = s[t * k + k - 1];
	__syncthreads();
	for (int w = 1; w < G; w <<= 1) {
		if ((t & (2 * w - 1)) == 0 && t + w < G && shit_less(red[t + w], red[t], tx)) red[t] = red[t + w];
		__syncthreads();
	}
	const SHit thr = red[0];
	SE_T();
	for (int i = t; i < P; i += SMALL_THREADS)
		if (!shit_less(thr, s[i], tx)) s2[atomicAdd(&s_ns, 1u)] = s[i];
	__syncthreads();
	const int ns = (int)s_ns;
	int n2 = 2;
	while (n2 < ns) n2 <<= 1;
	for (int i = ns + t; i < n2; i += SMALL_THREADS) s2[i] = SHit{F_INF, 0, INT64_MAX};
	__syncthreads();
	SE_T();
	if (!LHIP_ABL_SMALL_NOMERGE) shit_sort(s2, n2, tx);
	SE_T();
	s = s2;
	for (int i = t; i < k; i += SMALL_THREADS) {
		out_l[(int64_t)q * k + i] = s[i].v ? s[i].l : -1;
		out_d[(int64_t)q * k + i] = s[i].v ? s[i].d : __builtin_nanf("");
	}
	if (t == 0) {
		int cnt = 0;
		for (int i = 0; i < k; ++i) cnt += s[i].v;
		out_c[q] = cnt;
		counter[q] = 0u;  // ready for the next launch on this stream
	}
#ifdef LHIP_SE_PROF
	SE_T();
	if (t == 0 && se_prof)
		printf("SE last wg=%d dist=%d sort=%d publish=%d load+thr=%d compact=%d sort2=%d out=%d ns=%d\n", blockIdx.x,
		       (int)(st_[1] - st_[0]), (int)(st_[2] - st_[1]), (int)(st_[3] - st_[2]), (int)(st_[4] - st_[3]),
		       (int)(st_[5] - st_[4]), (int)(st_[6] - st_[5]), (int)(st_[7] - st_[6]), ns);
#endif
}

int small_exact_grid(int64_t n_slots) { return (int)((n_slots + SMALL_THREADS - 1) / SMALL_THREADS); }

bool small_exact_fits(int64_t n_slots, int dim, int nq, int k) {
	const int64_t G = (n_slots + SMALL_THREADS - 1) / SMALL_THREADS;
	return n_slots > 0 && n_slots <= SMALL_MAX_ROWS && dim <= SMALL_MAX_DIM && nq <= SMALL_MAX_Q && k <= SMALL_MAX_K &&
	       G * k <= SMALL_MAX_PART;
}

template <typename T>
static void small_exact_dispatch(const StoreView &s, const float *Q, int nq, int k, void *part, unsigned *counter,
                                 int64_t *L, float *D, int *C, hipStream_t st) {
	const dim3 grid((unsigned)small_exact_grid(s.n_slots), (unsigned)nq);
	const T *X = static_cast<const T *>(s.X);
	SHit *p = static_cast<SHit *>(part);
#ifdef LHIP_SE_PROF
	static std::atomic<int> calls{0};  // (diagnostic build: the 200th launch of the process prints its phases)
	const int se_prof = ++calls == 200;
#else
	const int se_prof = 0;
#endif
	switch (s.metric) {
	case METRIC_L2:
		small_exact_kernel<METRIC_L2, T><<<grid, SMALL_THREADS, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld, s.dim, Q,
		                                                                 k, p, counter, L, D, C, se_prof,
		                                                                 s.tie_desc);
		break;
	case METRIC_DOT:
		small_exact_kernel<METRIC_DOT, T><<<grid, SMALL_THREADS, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld, s.dim,
		                                                                  Q, k, p, counter, L, D, C, se_prof,
		                                                                 s.tie_desc);
		break;
	default:
		small_exact_kernel<METRIC_COSINE, T><<<grid, SMALL_THREADS, 0, st>>>(X, s.rowaux, s.labels, s.n_slots, s.ld,
		                                                                     s.dim, Q, k, p, counter, L, D, C, se_prof,
		                                                                 s.tie_desc);
		break;
	}
}

void launch_small_exact(const StoreView &s, const float *Q, int nq, int k, void *part, unsigned *counter, int64_t *L,
                        float *D, int *C, hipStream_t st) {
	if (!small_exact_fits(s.n_slots, s.dim, nq, k)) throw std::runtime_error("small exact search: shape out of range");
	if (s.xbf16)
		small_exact_dispatch<uint16_t>(s, Q, nq, k, part, counter, L, D, C, st);
	else
		small_exact_dispatch<float>(s, Q, nq, k, part, counter, L, D, C, st);
}

// ---------------------------------------------------------------------------
// second threshold pass for queries whose certificate failed (a segment
// overflowed, or the sampled tau was loose): the failed queries are packed
// into a batch of their own with tau = the k-th exact distance the first pass
// found (k real live rows lie within it) and rerun with full segments
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void retry_gather_kernel(const int *__restrict__ fq, int nf, int ld, int k,
                                                           const float *__restrict__ Qf,
                                                           const uint16_t *__restrict__ Qb,
                                                           const float4 *__restrict__ qaux,
                                                           const float *__restrict__ tau,
                                                           const float *__restrict__ dists, float *__restrict__ Qf2,
                                                           uint16_t *__restrict__ Qb2, float4 *__restrict__ qaux2,
                                                           float *__restrict__ tau2, int *__restrict__ status2,
                                                           int keep_tau) {
	const int i = blockIdx.x;
	const int t = threadIdx.x;
	const int src = i < nf ? fq[i] : -1;
	for (int j = t; j < ld; j += 256) {
		Qf2[(int64_t)i * ld + j] = src >= 0 ? Qf[(int64_t)src * ld + j] : 0.0f;
		Qb2[(int64_t)i * ld + j] = src >= 0 ? Qb[(int64_t)src * ld + j] : (uint16_t)0;
	}
	if (t != 0) return;
	qaux2[i] = src >= 0 ? qaux[src] : make_float4(0.f, 0.f, 0.f, 0.f);
	if (src < 0) return;
	const float t0 = tau[src];
	const float dk = dists[(int64_t)src * k + k - 1];  // NaN when fewer than k were found
	// two steps above d_k: a rerun's cut (<= tau2) can then still exceed
	// nextafter(d_k), which the certificate needs
	const float dk2 = nextafterf(nextafterf(dk, F_INF), F_INF);
	tau2[i] = (!keep_tau && dk2 < t0) ? dk2 : t0;
	status2[i] = status2[nf + i] = status2[2 * nf + i] = 0;
}

void launch_retry_gather(const int *fq, int nf, int nf_pad, int ld, int k, const QueryView &q, const float *tau,
                         const float *dists, float *Qf2, uint16_t *Qb2, float4 *qaux2, float *tau2, int *status2,
                         hipStream_t st, int keep_tau) {
	retry_gather_kernel<<<dim3(nf_pad), dim3(256), 0, st>>>(fq, nf, ld, k, q.Qf, q.Qb, q.qaux, tau, dists, Qf2, Qb2,
	                                                         qaux2, tau2, status2, keep_tau);
}

__global__ __launch_bounds__(64) void retry_scatter_kernel(const int *__restrict__ fq, int k,
                                                           const int64_t *__restrict__ L2,
                                                           const float *__restrict__ D2, const int *__restrict__ C2,
                                                           const int *__restrict__ cert2,
                                                           const float *__restrict__ tau2, int64_t *__restrict__ L,
                                                           float *__restrict__ D, int *__restrict__ C,
                                                           int *__restrict__ cert, float *__restrict__ tau) {
	const int i = blockIdx.x;
	const int dst = fq[i];
	if (!cert2[i]) {
		// still uncertified: keep the tighter bound for a further rerun (the
		// exact fallback writes the results)
		if (threadIdx.x == 0) {
			const float dk = D2[(int64_t)i * k + k - 1];
			const float t1 = tau2[i];
			tau[dst] = (dk < t1) ? dk : t1;
		}
		return;
	}
	for (int j = threadIdx.x; j < k; j += 64) {
		L[(int64_t)dst * k + j] = L2[(int64_t)i * k + j];
		D[(int64_t)dst * k + j] = D2[(int64_t)i * k + j];
	}
	if (threadIdx.x == 0) {
		C[dst] = C2[i];
		cert[dst] = 1;
	}
}

void launch_retry_scatter(const int *fq, int nf, int k, const int64_t *L2, const float *D2, const int *C2,
                          const int *cert2, const float *tau2, int64_t *L, float *D, int *C, int *cert, float *tau,
                          hipStream_t st) {
	retry_scatter_kernel<<<dim3(nf), dim3(64), 0, st>>>(fq, k, L2, D2, C2, cert2, tau2, L, D, C, cert, tau);
}

// ---------------------------------------------------------------------------
// multi-shard merge of partial top-k lists (one workgroup per query)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void merge_topk_kernel(int nshard, int nq, int k,
                                                         const int64_t *__restrict__ part_labels,
                                                         const float *__restrict__ part_dists,
                                                         const int *__restrict__ part_counts,
                                                         int64_t *__restrict__ out_labels,
                                                         float *__restrict__ out_dists, int *__restrict__ out_counts,
                                                         int64_t tx) {
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	const int total = nshard * k;
	int written = 0;
	for (int s = 0; s < nshard; ++s) {
		int c = part_counts[(int64_t)s * nq + q];
		written += c < k ? c : k;
	}
	for (int e = t; e < total; e += 256) {
		const int s = e / k, i = e % k;
		int c = part_counts[(int64_t)s * nq + q];
		if (i >= c) continue;
		const int64_t base = ((int64_t)s * nq + q) * k;
		const float d = part_dists[base + i];
		const int64_t l = part_labels[base + i];
		int rank = 0;
		for (int s2 = 0; s2 < nshard; ++s2) {
			int c2 = part_counts[(int64_t)s2 * nq + q];
			c2 = c2 < k ? c2 : k;
			const int64_t b2 = ((int64_t)s2 * nq + q) * k;
			for (int j = 0; j < c2; ++j) rank += hit_less(part_dists[b2 + j], part_labels[b2 + j], d, l, tx) ? 1 : 0;
			if (rank >= k) break;
		}
		if (rank < k) {
			out_labels[(int64_t)q * k + rank] = l;
			out_dists[(int64_t)q * k + rank] = d;
		}
	}
	const int nout = written < k ? written : k;
	for (int i = nout + t; i < k; i += 256) {
		out_labels[(int64_t)q * k + i] = -1;
		out_dists[(int64_t)q * k + i] = __builtin_nanf("");
	}
	if (t == 0) out_counts[q] = nout;
}

void launch_merge_topk(int nshard, int nq, int k, const int64_t *part_labels, const float *part_dists,
                       const int *part_counts, int64_t *out_labels, float *out_dists, int *out_counts,
                       hipStream_t st, int tie_desc) {
	merge_topk_kernel<<<dim3(nq), dim3(256), 0, st>>>(nshard, nq, k, part_labels, part_dists, part_counts,
	                                                   out_labels, out_dists, out_counts, tie_x64(tie_desc));
}

// Merge of packed shard rows as one all-gather delivers them (row s at
// g + s * stride, int32 units: labels int64[nq*k], dists f32[nq*k], counts
// i32[nq], and the shard's label offset int64 in the row's last two words).
// The local -> global label shift happens here, so the exchange is the
// all-gather and this one launch.  LDS: the query's live entries of every
// shard are staged compacted (nshard * k <= MP_LDS_CAP), then each entry's rank
// is its count of (distance, label)-smaller entries, as in merge_topk_kernel.
#define MP_LDS_CAP 4096

template <bool LDS>
__global__ __launch_bounds__(256) void merge_packed_kernel(int nshard, int nq, int k, const int32_t *__restrict__ g,
                                                           int64_t stride, int64_t *__restrict__ out_labels,
                                                           float *__restrict__ out_dists,
                                                           int *__restrict__ out_counts, int64_t tx) {
	extern __shared__ __align__(16) unsigned char mp_smem[];
	const int q = blockIdx.x;
	const int t = threadIdx.x;
	const int64_t nqk = (int64_t)nq * k;
	auto lab = [&](int s, int i) { return reinterpret_cast<const int64_t *>(g + s * stride)[(int64_t)q * k + i]; };
	auto dis = [&](int s, int i) { return reinterpret_cast<const float *>(g + s * stride + 2 * nqk)[(int64_t)q * k + i]; };
	auto cnt = [&](int s) {
		const int c = g[s * stride + 3 * nqk + q];
		return c < 0 ? 0 : (c < k ? c : k);
	};
	auto off = [&](int s) { return *reinterpret_cast<const int64_t *>(g + s * stride + stride - 2); };
	auto glob = [&](int64_t l, int s) { return l >= 0 ? l + off(s) : l; };
	int m = 0;
	if (LDS) {
		const int cap = nshard * k;
		int64_t *sl = reinterpret_cast<int64_t *>(mp_smem);
		float *sd = reinterpret_cast<float *>(sl + cap);
		int *sbase = reinterpret_cast<int *>(sd + cap);
		if (t == 0) {
			for (int s = 0; s < nshard; ++s) {
				sbase[s] = m;
				m += cnt(s);
			}
			sbase[nshard] = m;
		}
		__syncthreads();
		m = sbase[nshard];
		for (int e = t; e < cap; e += 256) {
			const int s = e / k, i = e - s * k;
			const int b = sbase[s];
			if (i < sbase[s + 1] - b) {
				sl[b + i] = glob(lab(s, i), s);
				sd[b + i] = dis(s, i);
			}
		}
		__syncthreads();
		for (int e = t; e < m; e += 256) {
			const float d = sd[e];
			const int64_t l = sl[e];
			int rank = 0;
			for (int j = 0; j < m && rank < k; ++j) rank += hit_less(sd[j], sl[j], d, l, tx) ? 1 : 0;
			if (rank < k) {
				out_labels[(int64_t)q * k + rank] = l;
				out_dists[(int64_t)q * k + rank] = d;
			}
		}
	} else {
		for (int s = 0; s < nshard; ++s) m += cnt(s);
		for (int64_t e = t; e < (int64_t)nshard * k; e += 256) {
			const int s = (int)(e / k), i = (int)(e - (int64_t)s * k);
			if (i >= cnt(s)) continue;
			const float d = dis(s, i);
			const int64_t l = glob(lab(s, i), s);
			int rank = 0;
			for (int s2 = 0; s2 < nshard && rank < k; ++s2) {
				const int c2 = cnt(s2);
				for (int j = 0; j < c2; ++j) rank += hit_less(dis(s2, j), glob(lab(s2, j), s2), d, l, tx) ? 1 : 0;
			}
			if (rank < k) {
				out_labels[(int64_t)q * k + rank] = l;
				out_dists[(int64_t)q * k + rank] = d;
			}
		}
	}
	const int nout = m < k ? m : k;
	for (int i = nout + t; i < k; i += 256) {
		out_labels[(int64_t)q * k + i] = -1;
		out_dists[(int64_t)q * k + i] = __builtin_nanf("");
	}
	if (t == 0) out_counts[q] = nout;
}

void launch_merge_packed(int nshard, int nq, int k, const int32_t *gathered, int64_t stride, int64_t *out_labels,
                         float *out_dists, int *out_counts, hipStream_t st, int tie_desc) {
	if ((int64_t)nshard * k <= MP_LDS_CAP && nshard <= 1024) {  // (<= 53 KB of LDS)
		const size_t lds = (size_t)nshard * k * (sizeof(int64_t) + sizeof(float)) + (size_t)(nshard + 1) * sizeof(int);
		merge_packed_kernel<true><<<dim3(nq), dim3(256), lds, st>>>(nshard, nq, k, gathered, stride, out_labels,
		                                                           out_dists, out_counts, tie_x64(tie_desc));
	} else {
		merge_packed_kernel<false><<<dim3(nq), dim3(256), 0, st>>>(nshard, nq, k, gathered, stride, out_labels,
		                                                          out_dists, out_counts, tie_x64(tie_desc));
	}
}

// ---------------------------------------------------------------------------
// compaction gather
// ---------------------------------------------------------------------------
// rows are moved as 16 B units: ld * element size is a multiple of 128 B
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4 *__restrict__ X, int row_u4,
                                                          const float4 *__restrict__ rowaux,
                                                          const int64_t *__restrict__ labels,
                                                          const int64_t *__restrict__ idx, int64_t n,
                                                          uint4 *__restrict__ Xo, float4 *__restrict__ rowaux_o,
                                                          int64_t *__restrict__ labels_o) {
	const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	if (r >= n) return;
	const int64_t s = idx[r];
	for (int i = lane; i < row_u4; i += 64) Xo[r * row_u4 + i] = X[s * row_u4 + i];
	if (lane == 0) {
		const float *ri = reinterpret_cast<const float *>(rowaux);
		float *ro = reinterpret_cast<float *>(rowaux_o);
#pragma unroll
		for (int c = 0; c < 4; ++c) ro[raix(r, c)] = ri[raix(s, c)];
		labels_o[r] = labels[s];
	}
}

void launch_gather_rows(const void *X, int xbf16, const float4 *rowaux, const int64_t *labels, const int64_t *idx,
                        int64_t n, int ld, void *Xo, float4 *rowaux_o, int64_t *labels_o, hipStream_t st) {
	if (n <= 0) return;
	const int row_u4 = ld * (xbf16 ? 2 : 4) / 16;
	gather_rows_kernel<<<dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st>>>(
	    static_cast<const uint4 *>(X), row_u4, rowaux, labels, idx, n, static_cast<uint4 *>(Xo), rowaux_o, labels_o);
}

}  // namespace lhip
