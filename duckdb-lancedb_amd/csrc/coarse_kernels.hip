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
	// staging: a 64 x 64 f32 tile of each operand = 1024 float4, 4 per thread and
	// operand, loaded for the NEXT chunk while this one multiplies (every load in
	// flight together: dim % 4 == 0, coarse_fused_fits)
	float4 rq[4], rc[4];
	auto fetch = [&](int k0) {
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const int e = t + 256 * j, r = e >> 4, c4 = (e & 15) * 4, k = k0 + c4;
			const int q = q0 + r, cc = c0 + r;
			rq[j] = (q < nq && k < dim) ? *reinterpret_cast<const float4 *>(Q + (int64_t)q * dim + k)
			                            : make_float4(0.f, 0.f, 0.f, 0.f);
			rc[j] = (cc < nc && k < dim) ? *reinterpret_cast<const float4 *>(C + (int64_t)cc * ld + k)
			                             : make_float4(0.f, 0.f, 0.f, 0.f);
		}
	};
	// norms: thread t sums row t >> 1 of the 128 staged rows (query rows, then
	// centroid rows), columns 32 (t & 1) .. + 32 of each chunk, in f64
	const int nr = t >> 1, nh = (t & 1) * 32;
	double n2 = 0.0;
	fetch(0);
	for (int k0 = 0; k0 < dim; k0 += CB_KC) {
		__syncthreads();  // the previous chunk consumed
#pragma unroll
		for (int j = 0; j < 4; ++j) {
			const int e = t + 256 * j, r = e >> 4, c4 = (e & 15) * 4;
			Qs[r][c4] = rq[j].x;
			Qs[r][c4 + 1] = rq[j].y;
			Qs[r][c4 + 2] = rq[j].z;
			Qs[r][c4 + 3] = rq[j].w;
			Cs[r][c4] = rc[j].x;
			Cs[r][c4 + 1] = rc[j].y;
			Cs[r][c4 + 2] = rc[j].z;
			Cs[r][c4 + 3] = rc[j].w;
		}
		__syncthreads();
		if (k0 + CB_KC < dim) fetch(k0 + CB_KC);  // in flight during the MFMAs
		{
			const float *row = nr < CB_T ? Qs[nr] : Cs[nr - CB_T];
#pragma unroll 8
			for (int c = 0; c < 32; ++c) n2 = fma((double)row[nh + c], (double)row[nh + c], n2);
		}
#pragma unroll 8
		for (int kk = 0; kk < CB_KC; kk += 2) {
			const float a = Qs[qa + (lane & 31)][kk + (lane >> 5)];
			const float b = Cs[ca + (lane & 31)][kk + (lane >> 5)];
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
		}
	}
	mfma_operand_guard();
	n2 += __shfl_xor(n2, 1, 64);
	if ((t & 1) == 0) nrm[nr < CB_T ? 0 : 1][nr & (CB_T - 1)] = n2;
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
	// this thread's bounds in registers (read once), then a radix select of the
	// rem-th smallest UB key, 8 bits at a time (wave 0 scans the 256 bins)
	constexpr int BPT = 8;  // (nc <= CS_THREADS * BPT, coarse_fused_fits)
	float lbv[BPT];
	uint32_t ubk[BPT];
	bool bad = false;
#pragma unroll
	for (int j = 0; j < BPT; ++j) {
		const int i = t + j * CS_THREADS;
		const float2 v = i < nc ? b[i] : make_float2(F_INF, F_INF);
		if (i < nc && !(__builtin_isfinite(v.x) && __builtin_isfinite(v.y))) bad = true;
		lbv[j] = v.x;
		ubk[j] = i < nc ? fkey(v.y) : 0xFFFFFFFFu;
	}
	if (bad) s_bad = 1;
	unsigned mask = 0;
	for (int sh = 24; sh >= 0; sh -= 8) {
		for (int i = t; i < 256; i += CS_THREADS) hist[i] = 0;
		__syncthreads();
		const unsigned pre = s_prefix;
#pragma unroll
		for (int j = 0; j < BPT; ++j)
			if (t + j * CS_THREADS < nc && (ubk[j] & mask) == pre) atomicAdd(&hist[(ubk[j] >> sh) & 255], 1u);
		__syncthreads();
		if (t < 64) {
			const unsigned rem = s_rem;
			unsigned h4[4], c = 0;
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				h4[u] = hist[4 * t + u];
				c += h4[u];
			}
			unsigned x = c;
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const unsigned y = __shfl_up(x, o, 64);
				if (t >= o) x += y;
			}
			unsigned ex = x - c;
			if (ex < rem && rem <= x) {
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					if (rem <= ex + h4[u]) {
						s_prefix = pre | ((unsigned)(4 * t + u) << sh);
						s_rem = rem - ex;
						break;
					}
					ex += h4[u];
				}
			}
		}
		mask |= 255u << sh;
		__syncthreads();
	}
	// a flagged query leaves no probes (every later kernel skips probe -1; the
	// host reruns the batch on the flat path once the pass has completed)
	auto flagged = [&]() {
		for (int i = t; i < nprobe; i += CS_THREADS) {
			probe_l[(int64_t)q * nprobe + i] = -1;
			probe_d[(int64_t)q * nprobe + i] = __builtin_nanf("");
		}
		if (t == 0) {
			probe_c[q] = 0;
			flag[q] = 1;
		}
	};
	if (s_bad) {
		flagged();
		return;
	}
	const float T = fkey_inv(s_prefix);
	// candidates: every partition whose LB <= T
#pragma unroll
	for (int j = 0; j < BPT; ++j) {
		const int i = t + j * CS_THREADS;
		if (i < nc && lbv[j] <= T) {
			const unsigned p = atomicAdd(&s_n, 1u);
			if (p < (unsigned)CS_CAP) keys[p] = (uint64_t)i;
		}
	}
	__syncthreads();
	const int n = (int)s_n;
	if (n > CS_CAP) {
		flagged();
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

bool coarse_fused_fits(int dim, int nc, int nprobe) {
	return dim <= 4096 && dim % 4 == 0 && nprobe <= nc && nc > 0 && nc <= CS_THREADS * 8 && nprobe > 0;
}

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
