// gfx950 kernels of the IVF_FLAT / IVF_PQ path (ivf.h has the numerics contract).
//
// Replaces lance-index 0.22's IVF_PQ training and search (behind
// rust_lib/src/lance_manager.rs:483-515 / :411-418, paths relative to
// /root/reference):
//   build   gather_sample -> kmeans_assign (bf16 MFMA |c|^2 - 2x.c, fused
//           arg-min) -> sort-based deterministic centroid means; residual PQ
//           k-means per sub-space (codebook slice in LDS); encode; T tables
//   search  prep -> coarse (the exact flat path over the centroid store) ->
//           invert probes into per-list query sets -> list scans:
//             IVF_FLAT  256-row work items, rows staged through LDS, f64
//                       exact distances for every query of the list, bitonic
//                       top-k per (query, item)
//             IVF_PQ    work items of (list chunk, 4 probing queries): the
//                       4 queries' 8-bit LUTs interleaved in LDS, codes
//                       streamed row-major in list order, LDS threshold
//                       candidates per (query, item); exact re-rank after
//           -> per-query merge -> exact re-rank (PQ) -> (distance, label) top-k
#include "ivf.h"
#include "device_common.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <atomic>
#include <vector>

// Development-only timing ablations of pq_fast_scan_kernel (results are wrong
// when set): only an ablation build (tools/pq_ablate.sh) may turn them on.
#if !defined(LHIP_ABLATION_BUILD) && (defined(LHIP_PQ_ABL_NO_LUT) || defined(LHIP_PQ_ABL_NO_LOOKUP) || \
                                      defined(LHIP_PQ_ABL_NO_CAND) || defined(LHIP_FB_ABL_LUTLOAD))
#error "PQ ablation switches are for ablation builds only"
#endif

namespace lhip {

static constexpr uint64_t KEY64_NONE = ~0ull;

#ifdef LHIP_PQ_PROF
// diagnostic build: per workgroup of pq_fast_scan_kernel, cycles in each phase
// (LUT build, row rounds, candidate sorts, flush), items and sorted items;
// thread 0 accumulates, the host prints after the launch (launch_pq_fast_scan)
constexpr int PQ_PROF_WG = 4096, PQ_PROF_N = 8;
__device__ uint64_t g_pq_prof[PQ_PROF_WG * PQ_PROF_N];
#define PQ_T(i)                                                   \
	{                                                             \
		const uint64_t now_ = __builtin_amdgcn_s_memtime();        \
		pq_acc[i] += now_ - pq_t;                                 \
		pq_t = now_;                                              \
	}
#else
#define PQ_T(i)
#endif

// f32 steps rounded one at a time, as the oracle's ISO C11 port does them: HIP
// compiles with fp-contract=fast-honor-pragmas, and __fmul_rn / __fadd_rn
// are plain operators in their headers, so a product feeding a sum became a
// v_fmac; operators created under contract(off) carry no contract flag
__device__ __forceinline__ float add_nc(float a, float b) {
#pragma clang fp contract(off)
	return a + b;
}
__device__ __forceinline__ float sub_nc(float a, float b) {
#pragma clang fp contract(off)
	return a - b;
}
__device__ __forceinline__ float mul_nc(float a, float b) {
#pragma clang fp contract(off)
	return a * b;
}

__device__ __forceinline__ uint64_t key64(float d, uint32_t slot) { return ((uint64_t)fkey(d) << 32) | slot; }
__device__ __forceinline__ float key64_dist(uint64_t k) { return fkey_inv((uint32_t)(k >> 32)); }
// tombstones and padding rows carry alpha = +inf in the row aux
__device__ __forceinline__ bool slot_alive(const float *rowaux_f, uint32_t slot) {
	return rowaux_f[raix(slot, 0)] != F_INF;
}

// ---------------------------------------------------------------------------
// workgroup-wide helpers (LDS)
// ---------------------------------------------------------------------------
// Bitonic sort of a[0..n), n a power of two, ascending.  All threads call it.
__device__ void wg_bitonic_sort(uint64_t *a, int n) {
	for (int size = 2; size <= n; size <<= 1) {
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			__syncthreads();
			for (int i = threadIdx.x; i < (n >> 1); i += blockDim.x) {
				const int lo = 2 * i - (i & (stride - 1));
				const int hi = lo + stride;
				const bool asc = (lo & size) == 0;
				const uint64_t x = a[lo], y = a[hi];
				if ((x > y) == asc) {
					a[lo] = y;
					a[hi] = x;
				}
			}
		}
	}
	__syncthreads();
}

// ascending bitonic sort of one 64-bit key per lane across the wave (no LDS, no barrier)
__device__ __forceinline__ uint64_t wave_sort64(uint64_t k) {
	const int lane = threadIdx.x & 63;
#pragma unroll
	for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
		for (int stride = size >> 1; stride > 0; stride >>= 1) {
			const uint64_t o = __shfl_xor(k, stride, 64);
			const bool asc = (lane & size) == 0, lower = (lane & stride) == 0;
			k = (lower == asc) ? (o < k ? o : k) : (o > k ? o : k);
		}
	}
	return k;
}

__device__ __forceinline__ int pow2_ceil(int v) {
	int p = 2;
	while (p < v) p <<= 1;
	return p;
}

// Sort one query's candidate buffer b[0..cnt_i) of a fast-scan item and cut it
// to kk.  The scan loops offer rows without reading their liveness (a global
// read in the loop makes the wave wait, vmcnt(0), for every load issued
// before it: the rows prefetched two rounds ahead), so dead rows are dropped
// here, before the kk-th key becomes the bound, and at the flush.  All
// threads call it; cnt_i, thr_i and nlive are LDS.
__device__ void fq_cut(uint64_t *b, int &cnt_i, uint64_t &thr_i, int q, int kk, const float *rowaux_f,
                       unsigned long long *thrq, int &nlive) {
	const int c = cnt_i, n2 = pow2_ceil(c);
	if (threadIdx.x == 0) nlive = 0;
	for (int e = threadIdx.x; e < n2; e += blockDim.x)
		if (e >= c || !slot_alive(rowaux_f, (uint32_t)b[e])) b[e] = KEY64_NONE;
	wg_bitonic_sort(b, n2);
	for (int e = threadIdx.x; e < n2; e += blockDim.x)
		if (b[e] != KEY64_NONE && (e + 1 == n2 || b[e + 1] == KEY64_NONE)) nlive = e + 1;
	__syncthreads();
	if (threadIdx.x == 0) {
		const int lv = nlive;
		if (lv >= kk) {
			thr_i = b[kk - 1];  // inclusive bound: the kk-th live key stays
			cnt_i = kk;
			atomicMin(thrq + q, (unsigned long long)b[kk - 1]);
		} else {
			cnt_i = lv;
		}
	}
	__syncthreads();
}

// Streaming top-K of 64-bit keys in LDS: every round each thread offers at
// most one key; keys below the threshold are appended; when the buffer could
// overflow in the next round it is sorted and cut to K (threshold = K-th key).
struct TopK {
	uint64_t *buf;
	int *cnt;
	uint64_t *thr;
	int K;
	__device__ void reset() {
		if (threadIdx.x == 0) {
			*cnt = 0;
			*thr = KEY64_NONE;
		}
		__syncthreads();
	}
	__device__ void compact() {
		__syncthreads();
		const int c = *cnt;
		const int n = pow2_ceil(c);
		for (int i = c + threadIdx.x; i < n; i += blockDim.x) buf[i] = KEY64_NONE;
		wg_bitonic_sort(buf, n);
		if (threadIdx.x == 0) {
			if (c >= K) {
				*thr = buf[K - 1];
				*cnt = K;
			}
		}
		__syncthreads();
	}
	// all threads call; valid per thread
	__device__ void offer(uint64_t key, bool valid) {
		if (valid && key < *thr) {
			const int p = atomicAdd(cnt, 1);
			buf[p] = key;
		}
		__syncthreads();
		if (*cnt > IVF_TOPK_CAP - (int)blockDim.x) compact();
	}
	// sorted result in buf[0 .. min(cnt, K))
	__device__ int finish() {
		compact();
		const int c = *cnt;
		return c < K ? c : K;
	}
};

__device__ __forceinline__ float4 load4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 load4(const uint16_t *p) {
	const uint2 u = *reinterpret_cast<const uint2 *>(p);
	return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
	                   __uint_as_float(u.y & 0xFFFF0000u));
}

// ---------------------------------------------------------------------------
// build: sample gather, centroid prep
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void gather_sample_kernel(const T *__restrict__ X, int ld, int dim,
                                                            const int64_t *__restrict__ slots, int64_t n,
                                                            int normalize, float *__restrict__ out,
                                                            uint16_t *__restrict__ outb) {
	const int lane = threadIdx.x & 63;
	const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	if (r >= n) return;
	const T *x = X + slots[r] * (int64_t)ld;
	float inv = 1.0f;
	if (normalize) {
		double ss = 0.0;
		for (int i = lane; i < dim; i += 64) {
			const double v = xval(x, i);
			ss += v * v;
		}
		ss = wave_sum_f64(ss);
		inv = ss > 0.0 ? (float)(1.0 / sqrt(ss)) : 0.0f;
	}
	for (int i = lane; i < ld; i += 64) {
		const float v = i < dim ? xval(x, i) * inv : 0.0f;
		out[r * ld + i] = v;
		outb[r * ld + i] = bf16_bits(v);
	}
}

void launch_gather_sample(const void *X, int xbf16, int ld, int dim, const int64_t *slots, int64_t n, int normalize,
                          float *out_f32, uint16_t *out_bf16, hipStream_t st) {
	dim3 grid((unsigned)((n + 3) / 4));
	if (xbf16)
		gather_sample_kernel<uint16_t><<<grid, 256, 0, st>>>(static_cast<const uint16_t *>(X), ld, dim, slots, n,
		                                                      normalize, out_f32, out_bf16);
	else
		gather_sample_kernel<float><<<grid, 256, 0, st>>>(static_cast<const float *>(X), ld, dim, slots, n, normalize,
		                                                   out_f32, out_bf16);
}

__global__ __launch_bounds__(256) void centroid_prep_kernel(const float *__restrict__ C, int nc, int nc_pad, int ld,
                                                            uint16_t *__restrict__ Cb, float *__restrict__ cnorm) {
	const int lane = threadIdx.x & 63;
	const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
	if (c >= nc_pad) return;
	double ss = 0.0;
	for (int i = lane; i < ld; i += 64) {
		const float v = c < nc ? C[(int64_t)c * ld + i] : 0.0f;
		Cb[(int64_t)c * ld + i] = bf16_bits(v);
		ss += (double)v * v;
	}
	ss = wave_sum_f64(ss);
	if (lane == 0) cnorm[c] = c < nc ? (float)ss : F_INF;
}

void launch_centroid_prep(const float *C, int nc, int nc_pad, int ld, uint16_t *Cb, float *cnorm, hipStream_t st) {
	centroid_prep_kernel<<<dim3((unsigned)((nc_pad + 3) / 4)), 256, 0, st>>>(C, nc, nc_pad, ld, Cb, cnorm);
}

// ---------------------------------------------------------------------------
// k-means assignment: bf16 MFMA (v_mfma_f32_32x32x16_bf16) centroid x row
// tiles of 128 x 128, K staged 32 at a time through padded LDS (80-B rows:
// the 16-lane groups of ds_read_b128 hit 16 distinct 16-B bank slots).
// A = centroids (MFMA rows), B = data rows (MFMA columns): a lane's 16
// accumulator registers are 16 centroids of ONE data row, so the arg-min is
// register-local plus one lane swap, then one 64-bit atomicMin per row.
// ---------------------------------------------------------------------------
constexpr int KM_T = 128;       // tile edge
constexpr int KM_K = 32;        // k per stage
constexpr int KM_ROWB = 80;     // LDS bytes per tile row (64 + 16 pad)

template <typename T>
__device__ __forceinline__ void km_load_rows(const T *__restrict__ X, int ld, int64_t r0, int64_t n, int k0,
                                             uint4 (&reg)[4]);
template <>
__device__ __forceinline__ void km_load_rows<uint16_t>(const uint16_t *__restrict__ X, int ld, int64_t r0, int64_t n,
                                                       int k0, uint4 (&reg)[4]) {
#pragma unroll
	for (int i = 0; i < 2; ++i) {
		const int e = threadIdx.x + i * 256, row = e >> 2, seg = e & 3;
		const int64_t r = r0 + row;
		reg[i] = r < n ? *reinterpret_cast<const uint4 *>(X + r * ld + k0 + seg * 8) : make_uint4(0, 0, 0, 0);
	}
}
template <>
__device__ __forceinline__ void km_load_rows<float>(const float *__restrict__ X, int ld, int64_t r0, int64_t n, int k0,
                                                    uint4 (&reg)[4]) {
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const int e = threadIdx.x + i * 256, row = e >> 3, seg = e & 7;
		const int64_t r = r0 + row;
		float4 v = r < n ? *reinterpret_cast<const float4 *>(X + r * ld + k0 + seg * 4) : make_float4(0, 0, 0, 0);
		reg[i] = make_uint4(pk_bf16(v.x, v.y), pk_bf16(v.z, v.w), 0, 0);
	}
}
template <typename T>
__device__ __forceinline__ void km_store_rows(uint8_t *Bs, const uint4 (&reg)[4]);
template <>
__device__ __forceinline__ void km_store_rows<uint16_t>(uint8_t *Bs, const uint4 (&reg)[4]) {
#pragma unroll
	for (int i = 0; i < 2; ++i) {
		const int e = threadIdx.x + i * 256, row = e >> 2, seg = e & 3;
		*reinterpret_cast<uint4 *>(Bs + row * KM_ROWB + seg * 16) = reg[i];
	}
}
template <>
__device__ __forceinline__ void km_store_rows<float>(uint8_t *Bs, const uint4 (&reg)[4]) {
#pragma unroll
	for (int i = 0; i < 4; ++i) {
		const int e = threadIdx.x + i * 256, row = e >> 3, seg = e & 7;
		*reinterpret_cast<uint2 *>(Bs + row * KM_ROWB + seg * 8) = make_uint2(reg[i].x, reg[i].y);
	}
}

template <typename T>
__global__ __launch_bounds__(256) void kmeans_assign_kernel(const T *__restrict__ X, int ld, int64_t r0, int64_t n,
                                                            const float *__restrict__ row_scale_aux,
                                                            const uint16_t *__restrict__ Cb,
                                                            const float *__restrict__ cnorm,
                                                            uint64_t *__restrict__ best) {
	__shared__ __attribute__((aligned(16))) uint8_t As[2][KM_T * KM_ROWB];
	__shared__ __attribute__((aligned(16))) uint8_t Bs[2][KM_T * KM_ROWB];
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	const int64_t rt0 = (int64_t)blockIdx.x * KM_T;  // first data row of the tile (relative)
	const int c0 = blockIdx.y * KM_T;
	const int cw = (w & 1) * 64, rw = (w >> 1) * 64;
	const T *Xb = X + r0 * (int64_t)ld;
	const int64_t nrel = n;
	const int nst = ld / KM_K;

	uint4 ra[2], rb[4];
	auto load_a = [&](int k0) {
#pragma unroll
		for (int i = 0; i < 2; ++i) {
			const int e = t + i * 256, row = e >> 2, seg = e & 3;
			ra[i] = *reinterpret_cast<const uint4 *>(Cb + (int64_t)(c0 + row) * ld + k0 + seg * 8);
		}
	};
	auto store_a = [&](uint8_t *A) {
#pragma unroll
		for (int i = 0; i < 2; ++i) {
			const int e = t + i * 256, row = e >> 2, seg = e & 3;
			*reinterpret_cast<uint4 *>(A + row * KM_ROWB + seg * 16) = ra[i];
		}
	};
	f32x16 acc[2][2];
#pragma unroll
	for (int a = 0; a < 2; ++a)
#pragma unroll
		for (int b = 0; b < 2; ++b)
#pragma unroll
			for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;

	load_a(0);
	km_load_rows<T>(Xb, ld, rt0, nrel, 0, rb);
	store_a(As[0]);
	km_store_rows<T>(Bs[0], rb);
	__syncthreads();
	const int fr = lane & 31, fh = lane >> 5;
	for (int s = 0; s < nst; ++s) {
		const int cur = s & 1;
		if (s + 1 < nst) {
			load_a((s + 1) * KM_K);
			km_load_rows<T>(Xb, ld, rt0, nrel, (s + 1) * KM_K, rb);
		}
#pragma unroll
		for (int kk = 0; kk < 2; ++kk) {
			bf16x8 av[2], bv[2];
#pragma unroll
			for (int mi = 0; mi < 2; ++mi)
				av[mi] = *reinterpret_cast<const bf16x8 *>(As[cur] + (cw + mi * 32 + fr) * KM_ROWB + kk * 32 + fh * 16);
#pragma unroll
			for (int ni = 0; ni < 2; ++ni)
				bv[ni] = *reinterpret_cast<const bf16x8 *>(Bs[cur] + (rw + ni * 32 + fr) * KM_ROWB + kk * 32 + fh * 16);
#pragma unroll
			for (int mi = 0; mi < 2; ++mi)
#pragma unroll
				for (int ni = 0; ni < 2; ++ni)
					acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
		}
		if (s + 1 < nst) {
			store_a(As[cur ^ 1]);
			km_store_rows<T>(Bs[cur ^ 1], rb);
		}
		__syncthreads();
	}
	mfma_operand_guard();
	// epilogue: this lane's data row = rw + ni*32 + fr; centroids in registers
#pragma unroll
	for (int ni = 0; ni < 2; ++ni) {
		const int64_t row = rt0 + rw + ni * 32 + fr;
		const float sc = (row_scale_aux && row < nrel) ? row_scale_aux[raix(r0 + row, 3)] : 1.0f;
		uint64_t bk = KEY64_NONE;
#pragma unroll
		for (int mi = 0; mi < 2; ++mi)
#pragma unroll
			for (int r = 0; r < 16; ++r) {
				const int c = c0 + cw + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
				const float score = cnorm[c] - 2.0f * sc * acc[mi][ni][r];
				const uint64_t kv = ((uint64_t)fkey(score) << 32) | (uint32_t)c;
				bk = kv < bk ? kv : bk;
			}
		const uint64_t o = __shfl_xor(bk, 32, 64);
		bk = o < bk ? o : bk;
		if (fh == 0 && row < nrel) atomicMin((unsigned long long *)(best + row), (unsigned long long)bk);
	}
}

void launch_kmeans_assign(const void *X, int xbf16, int ld, int64_t r0, int64_t n, const float *row_scale_aux,
                          const uint16_t *Cb, const float *cnorm, int nc_pad, uint64_t *best, hipStream_t st) {
	if (n <= 0) return;
	dim3 grid((unsigned)((n + KM_T - 1) / KM_T), (unsigned)(nc_pad / KM_T));
	if (xbf16)
		kmeans_assign_kernel<uint16_t><<<grid, 256, 0, st>>>(static_cast<const uint16_t *>(X), ld, r0, n,
		                                                      row_scale_aux, Cb, cnorm, best);
	else
		kmeans_assign_kernel<float><<<grid, 256, 0, st>>>(static_cast<const float *>(X), ld, r0, n, row_scale_aux, Cb,
		                                                   cnorm, best);
}

// Exact-f32 variant for placing rows into lists (v_mfma_f32_32x32x2_f32:
// f32 products and accumulation, ~1e-6 relative): the bf16 scores above are
// good enough to train on, but near-equidistant rows would land in a
// farther list.  Same tiling and epilogue; LDS rows of 33 floats (ds_read_b32
// banks are mod 32: the 32 lanes of a half read 32 consecutive rows).
constexpr int KF_ROW = KM_K + 1;

template <typename T>
__global__ __launch_bounds__(256) void kmeans_assign_f32_kernel(const T *__restrict__ X, int ld, int64_t r0, int64_t n,
                                                                const float *__restrict__ row_scale_aux,
                                                                const float *__restrict__ Cf,
                                                                const float *__restrict__ cnorm,
                                                                uint64_t *__restrict__ best) {
	__shared__ float As[2][KM_T * KF_ROW];
	__shared__ float Bs[2][KM_T * KF_ROW];
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	const int64_t rt0 = (int64_t)blockIdx.x * KM_T;
	const int c0 = blockIdx.y * KM_T;
	const int cw = (w & 1) * 64, rw = (w >> 1) * 64;
	const T *Xb = X + r0 * (int64_t)ld;
	const int nst = ld / KM_K;
	float4 ra[4], rb[4];
	auto load = [&](int k0) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const int e = t + i * 256, row = e >> 3, seg = e & 7;
			ra[i] = *reinterpret_cast<const float4 *>(Cf + (int64_t)(c0 + row) * ld + k0 + seg * 4);
			const int64_t r = rt0 + row;
			rb[i] = r < n ? load4(Xb + r * ld + k0 + seg * 4) : make_float4(0, 0, 0, 0);
		}
	};
	auto store = [&](float *A, float *B) {
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const int e = t + i * 256, row = e >> 3, seg = e & 7;
			float *a = A + row * KF_ROW + seg * 4, *b = B + row * KF_ROW + seg * 4;
			a[0] = ra[i].x, a[1] = ra[i].y, a[2] = ra[i].z, a[3] = ra[i].w;
			b[0] = rb[i].x, b[1] = rb[i].y, b[2] = rb[i].z, b[3] = rb[i].w;
		}
	};
	f32x16 acc[2][2];
#pragma unroll
	for (int a = 0; a < 2; ++a)
#pragma unroll
		for (int b = 0; b < 2; ++b)
#pragma unroll
			for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.0f;
	load(0);
	store(As[0], Bs[0]);
	__syncthreads();
	const int fr = lane & 31, fh = lane >> 5;
	for (int s = 0; s < nst; ++s) {
		const int cur = s & 1;
		if (s + 1 < nst) load((s + 1) * KM_K);
#pragma unroll
		for (int kk = 0; kk < KM_K / 2; ++kk) {
			float av[2], bv[2];
#pragma unroll
			for (int mi = 0; mi < 2; ++mi) av[mi] = As[cur][(cw + mi * 32 + fr) * KF_ROW + 2 * kk + fh];
#pragma unroll
			for (int ni = 0; ni < 2; ++ni) bv[ni] = Bs[cur][(rw + ni * 32 + fr) * KF_ROW + 2 * kk + fh];
#pragma unroll
			for (int mi = 0; mi < 2; ++mi)
#pragma unroll
				for (int ni = 0; ni < 2; ++ni)
					acc[mi][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[mi], bv[ni], acc[mi][ni], 0, 0, 0);
		}
		if (s + 1 < nst) store(As[cur ^ 1], Bs[cur ^ 1]);
		__syncthreads();
	}
	mfma_operand_guard();
#pragma unroll
	for (int ni = 0; ni < 2; ++ni) {
		const int64_t row = rt0 + rw + ni * 32 + fr;
		const float sc = (row_scale_aux && row < n) ? row_scale_aux[raix(r0 + row, 3)] : 1.0f;
		uint64_t bk = KEY64_NONE;
#pragma unroll
		for (int mi = 0; mi < 2; ++mi)
#pragma unroll
			for (int r = 0; r < 16; ++r) {
				const int c = c0 + cw + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
				const float score = cnorm[c] - 2.0f * sc * acc[mi][ni][r];
				const uint64_t kv = ((uint64_t)fkey(score) << 32) | (uint32_t)c;
				bk = kv < bk ? kv : bk;
			}
		const uint64_t o = __shfl_xor(bk, 32, 64);
		bk = o < bk ? o : bk;
		if (fh == 0 && row < n) atomicMin((unsigned long long *)(best + row), (unsigned long long)bk);
	}
}

void launch_kmeans_assign_f32(const void *X, int xbf16, int ld, int64_t r0, int64_t n, const float *row_scale_aux,
                              const float *Cf, const float *cnorm, int nc_pad, uint64_t *best, hipStream_t st) {
	if (n <= 0) return;
	dim3 grid((unsigned)((n + KM_T - 1) / KM_T), (unsigned)(nc_pad / KM_T));
	if (xbf16)
		kmeans_assign_f32_kernel<uint16_t><<<grid, 256, 0, st>>>(static_cast<const uint16_t *>(X), ld, r0, n,
		                                                          row_scale_aux, Cf, cnorm, best);
	else
		kmeans_assign_f32_kernel<float><<<grid, 256, 0, st>>>(static_cast<const float *>(X), ld, r0, n, row_scale_aux,
		                                                       Cf, cnorm, best);
}

// deterministic sum (fixed per-thread strides + fixed tree) of the winning scores
__global__ __launch_bounds__(1024) void score_sum_kernel(const uint64_t *__restrict__ best, int64_t n,
                                                         double *__restrict__ out) {
	__shared__ double sh[1024];
	double s = 0.0;
	for (int64_t i = threadIdx.x; i < n; i += 1024) s += (double)key64_dist(best[i]);
	sh[threadIdx.x] = s;
	__syncthreads();
	for (int o = 512; o > 0; o >>= 1) {
		if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
		__syncthreads();
	}
	if (threadIdx.x == 0) *out = sh[0];
}

void launch_score_sum(const uint64_t *best, int64_t n, double *out, hipStream_t st) {
	score_sum_kernel<<<1, 1024, 0, st>>>(best, n, out);
}

// sum of squares of n f32 values (deterministic order), for the k-means stopping rule
__global__ __launch_bounds__(1024) void sq_sum_kernel(const float *__restrict__ v, int64_t n, double *__restrict__ out) {
	__shared__ double sh[1024];
	double s = 0.0;
	for (int64_t i = threadIdx.x; i < n; i += 1024) s += (double)v[i] * v[i];
	sh[threadIdx.x] = s;
	__syncthreads();
	for (int o = 512; o > 0; o >>= 1) {
		if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
		__syncthreads();
	}
	if (threadIdx.x == 0) *out = sh[0];
}

void launch_sq_sum(const float *v, int64_t n, double *out, hipStream_t st) { sq_sum_kernel<<<1, 1024, 0, st>>>(v, n, out); }

// dst row i = src row idx[i] (rows of row_bytes, a multiple of 16)
__global__ void gather_bytes_kernel(const uint8_t *__restrict__ src, const int64_t *__restrict__ idx, int64_t n,
                                    int row_bytes, uint8_t *__restrict__ dst) {
	const int nch = row_bytes >> 4;
	const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (e >= n * nch) return;
	const int64_t r = e / nch;
	const int ch = (int)(e % nch);
	*reinterpret_cast<uint4 *>(dst + r * row_bytes + ch * 16) =
	    *reinterpret_cast<const uint4 *>(src + idx[r] * row_bytes + ch * 16);
}

void launch_gather_bytes(const uint8_t *src, const int64_t *idx, int64_t n, int row_bytes, uint8_t *dst,
                         hipStream_t st) {
	const int64_t tot = n * (row_bytes >> 4);
	if (tot <= 0) return;
	gather_bytes_kernel<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(src, idx, n, row_bytes, dst);
}

__global__ void best_to_assign_kernel(const uint64_t *__restrict__ best, int64_t n, int *__restrict__ assign,
                                      uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
	const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint32_t c = (uint32_t)best[i];
	if (assign) assign[i] = (int)c;
	if (keys) keys[i] = c;
	if (vals) vals[i] = (uint32_t)i;
}

void launch_best_to_assign(const uint64_t *best, int64_t n, int *assign, uint32_t *keys, uint32_t *vals,
                           hipStream_t st) {
	if (n <= 0) return;
	best_to_assign_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(best, n, assign, keys, vals);
}

int sort_u32_pairs(void *temp, size_t &temp_bytes, const uint32_t *kin, uint32_t *kout, const uint32_t *vin,
                   uint32_t *vout, int64_t n, int end_bit, hipStream_t st) {
	return (int)rocprim::radix_sort_pairs(temp, temp_bytes, kin, kout, vin, vout, (size_t)n, 0, end_bit, st);
}

__global__ void segments_kernel(const uint32_t *__restrict__ keys, int64_t n, int nseg, int *__restrict__ seg_start) {
	const int c = blockIdx.x * blockDim.x + threadIdx.x;
	if (c > nseg) return;
	int64_t lo = 0, hi = n;  // first index with key >= c
	while (lo < hi) {
		const int64_t mid = (lo + hi) >> 1;
		if (keys[mid] < (uint32_t)c)
			lo = mid + 1;
		else
			hi = mid;
	}
	seg_start[c] = (int)lo;
}

void launch_segments(const uint32_t *sorted_keys, int64_t n, int nseg, int *seg_start, hipStream_t st) {
	segments_kernel<<<dim3((unsigned)((nseg + 1 + 255) / 256)), 256, 0, st>>>(sorted_keys, n, nseg, seg_start);
}

// new centroid = mean of its members, summed in member order (f64); an empty
// cluster keeps its previous centroid
__global__ __launch_bounds__(256) void centroid_mean_kernel(const float *__restrict__ S, int ld, int dim,
                                                            const uint32_t *__restrict__ idx,
                                                            const int *__restrict__ seg_start, float *__restrict__ C) {
	const int c = blockIdx.x;
	const int a = seg_start[c], b = seg_start[c + 1];
	if (b <= a) return;
	const double inv = 1.0 / (double)(b - a);
	for (int i = threadIdx.x; i < dim; i += 256) {
		double s = 0.0;
		for (int m = a; m < b; ++m) s += S[(int64_t)idx[m] * ld + i];
		C[(int64_t)c * ld + i] = (float)(s * inv);
	}
}

void launch_centroid_mean(const float *S, int ld, int dim, const uint32_t *sorted_idx, const int *seg_start, int nc,
                          float *C, hipStream_t st) {
	centroid_mean_kernel<<<dim3((unsigned)nc), 256, 0, st>>>(S, ld, dim, sorted_idx, seg_start, C);
}

__global__ void residuals_kernel(const float *__restrict__ S, const int *__restrict__ assign,
                                 const float *__restrict__ C, int ld, int64_t n, float *__restrict__ R) {
	const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (e >= n * ld) return;
	const int64_t r = e / ld;
	const int i = (int)(e % ld);
	R[e] = S[e] - C[(int64_t)assign[r] * ld + i];
}

void launch_residuals(const float *S, const int *assign, const float *C, int ld, int64_t n, float *R,
                      hipStream_t st) {
	const int64_t tot = n * ld;
	residuals_kernel<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(S, assign, C, ld, n, R);
}

// ---------------------------------------------------------------------------
// PQ: per-sub-space assignment / means / encoding (codebook slice in LDS)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int pq_argmin(const float *cbs /*[256][dsub+1]*/, const float (&r)[PQ_MAX_DSUB],
                                         int dsub) {
	float bd = F_INF;
	int bc = 0;
	for (int c = 0; c < PQ_K; ++c) {
		const float *y = cbs + c * (dsub + 1);
		float d = 0.0f;
#pragma unroll
		for (int t = 0; t < PQ_MAX_DSUB; ++t) {
			if (t < dsub) {
				const float u = r[t] - y[t];
				d += u * u;
			}
		}
		if (d < bd) {  // strict: ties keep the lowest code
			bd = d;
			bc = c;
		}
	}
	return bc;
}

__device__ __forceinline__ void pq_load_cb(const float *__restrict__ cb, int j, int dsub, float *cbs) {
	for (int e = threadIdx.x; e < PQ_K * dsub; e += blockDim.x) {
		const int c = e / dsub, t = e % dsub;
		cbs[c * (dsub + 1) + t] = cb[((int64_t)j * PQ_K + c) * dsub + t];
	}
	__syncthreads();
}

__global__ __launch_bounds__(256) void pq_assign_kernel(const float *__restrict__ R, int ld, int64_t n, int m, int dsub,
                                                        const float *__restrict__ cb, uint32_t *__restrict__ keys,
                                                        uint32_t *__restrict__ vals) {
	__shared__ float cbs[PQ_K * (PQ_MAX_DSUB + 1)];
	const int j = blockIdx.y;
	pq_load_cb(cb, j, dsub, cbs);
	const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
	if (r >= n) return;
	float v[PQ_MAX_DSUB];
#pragma unroll
	for (int t = 0; t < PQ_MAX_DSUB; ++t) v[t] = t < dsub ? R[r * ld + j * dsub + t] : 0.0f;
	const int c = pq_argmin(cbs, v, dsub);
	keys[(int64_t)j * n + r] = (uint32_t)(j * PQ_K + c);
	vals[(int64_t)j * n + r] = (uint32_t)r;
}

void launch_pq_assign(const float *R, int ld, int64_t n, int m, int dsub, const float *cb, uint32_t *keys,
                      uint32_t *vals, hipStream_t st) {
	dim3 grid((unsigned)((n + 255) / 256), (unsigned)m);
	pq_assign_kernel<<<grid, 256, 0, st>>>(R, ld, n, m, dsub, cb, keys, vals);
}

// one thread per (sub-space j, code c, component t): mean over the members in order
__global__ void pq_mean_kernel(const float *__restrict__ R, int ld, const uint32_t *__restrict__ idx,
                               const int *__restrict__ seg_start, int m, int dsub, float *__restrict__ cb) {
	const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (e >= (int64_t)m * PQ_K * dsub) return;
	const int seg = (int)(e / dsub), t = (int)(e % dsub);
	const int j = seg / PQ_K;
	const int a = seg_start[seg], b = seg_start[seg + 1];
	if (b <= a) return;
	double s = 0.0;
	for (int i = a; i < b; ++i) s += R[(int64_t)idx[i] * ld + j * dsub + t];
	cb[e] = (float)(s / (double)(b - a));
}

void launch_pq_mean(const float *R, int ld, const uint32_t *sorted_idx, const int *seg_start, int m, int dsub,
                    float *cb, hipStream_t st) {
	const int64_t tot = (int64_t)m * PQ_K * dsub;
	pq_mean_kernel<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(R, ld, sorted_idx, seg_start, m, dsub, cb);
}

template <typename T>
__global__ __launch_bounds__(256) void pq_encode_kernel(const T *__restrict__ X, int ld, int64_t s0, int64_t n,
                                                        const float *__restrict__ rowaux_f, int normalize,
                                                        const int *__restrict__ assign, const float *__restrict__ C,
                                                        const float *__restrict__ cb, int dsub, int mp,
                                                        uint8_t *__restrict__ codes) {
	__shared__ float cbs[PQ_K * (PQ_MAX_DSUB + 1)];
	const int j = blockIdx.y;
	pq_load_cb(cb, j, dsub, cbs);
	const int64_t s = s0 + (int64_t)blockIdx.x * 256 + threadIdx.x;
	if (s >= s0 + n) return;
	const float sc = normalize ? rowaux_f[raix(s, 3)] : 1.0f;  // 1/|x| (cosine)
	const float *c = C + (int64_t)assign[s] * ld + j * dsub;
	const T *x = X + s * ld + j * dsub;
	float v[PQ_MAX_DSUB];
#pragma unroll
	for (int t = 0; t < PQ_MAX_DSUB; ++t) v[t] = t < dsub ? xval(x, t) * sc - c[t] : 0.0f;
	codes[s * mp + j] = (uint8_t)pq_argmin(cbs, v, dsub);
}

void launch_pq_encode(const void *X, int xbf16, int ld, int dim, int64_t s0, int64_t n, const float *rowaux_f,
                      int normalize, const int *assign, const float *C, const float *cb, int m, int dsub, int mp,
                      uint8_t *codes, hipStream_t st) {
	if (n <= 0) return;
	dim3 grid((unsigned)((n + 255) / 256), (unsigned)m);
	if (xbf16)
		pq_encode_kernel<uint16_t><<<grid, 256, 0, st>>>(static_cast<const uint16_t *>(X), ld, s0, n, rowaux_f,
		                                                  normalize, assign, C, cb, dsub, mp, codes);
	else
		pq_encode_kernel<float><<<grid, 256, 0, st>>>(static_cast<const float *>(X), ld, s0, n, rowaux_f, normalize,
		                                               assign, C, cb, dsub, mp, codes);
}

// T[l][j][c] = sum_t y (y + 2 c_l)  (f32, t in order, no contraction)
__global__ __launch_bounds__(256) void pq_T_kernel(const float *__restrict__ C, int ld, const float *__restrict__ cb,
                                                   int m, int dsub, float *__restrict__ T) {
	const int l = blockIdx.x, j = blockIdx.y, c = threadIdx.x;
	const float *y = cb + ((int64_t)j * PQ_K + c) * dsub;
	const float *cl = C + (int64_t)l * ld + j * dsub;
	float acc = 0.0f;
	for (int t = 0; t < dsub; ++t) acc = add_nc(acc, mul_nc(y[t], add_nc(y[t], 2.0f * cl[t])));
	T[((int64_t)l * m + j) * PQ_K + c] = acc;
}

void launch_pq_tables_T(const float *C, int ld, const float *cb, int nlist, int m, int dsub, float *T,
                        hipStream_t st) {
	pq_T_kernel<<<dim3((unsigned)nlist, (unsigned)m), PQ_K, 0, st>>>(C, ld, cb, m, dsub, T);
}

__global__ void pq_layout_kernel(const uint8_t *__restrict__ codes, const uint32_t *__restrict__ lslot, int64_t npos,
                                 int mp, uint8_t *__restrict__ lcodes) {
	const int nch = mp >> 4;
	const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (e >= npos * nch) return;
	const int64_t pos = e / nch;
	const int ch = (int)(e % nch);
	const uint32_t slot = lslot[pos];
	uint4 v = make_uint4(0, 0, 0, 0);
	if (slot != SLOT_NONE) v = *reinterpret_cast<const uint4 *>(codes + (int64_t)slot * mp + ch * 16);
	*reinterpret_cast<uint4 *>(lcodes + (pos * nch + ch) * 16) = v;
}

void launch_pq_layout(const uint8_t *codes, const uint32_t *lslot, int64_t npos, int mp, uint8_t *lcodes,
                      hipStream_t st) {
	const int64_t tot = npos * (mp >> 4);
	if (tot <= 0) return;
	pq_layout_kernel<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(codes, lslot, npos, mp, lcodes);
}

// list-ordered row term of the L2 / cosine ADC: tau[pos] = sum_j T[l][j][c_j]
// (f32, j ascending, from 0) of the row at pos in list l; 0 for padding
__global__ void pq_tau_kernel(const uint8_t *__restrict__ codes, const uint32_t *__restrict__ lslot,
                              const int64_t *__restrict__ loff, int nlist, int64_t npos, int m, int mp,
                              const float *__restrict__ T, float *__restrict__ ltau) {
	const int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (pos >= npos) return;
	const uint32_t slot = lslot[pos];
	float acc = 0.0f;
	if (slot != SLOT_NONE) {
		int lo = 0, hi = nlist - 1;  // list of pos: last l with loff[l] <= pos
		while (lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if (loff[mid] <= pos) lo = mid;
			else hi = mid - 1;
		}
		const float *Tl = T + (int64_t)lo * m * PQ_K;
		const uint8_t *c = codes + (int64_t)slot * mp;
		for (int j = 0; j < m; ++j) acc = acc + Tl[j * PQ_K + c[j]];
	}
	ltau[pos] = acc;
}

void launch_pq_tau(const uint8_t *codes, const uint32_t *lslot, const int64_t *loff, int nlist, int64_t npos, int m,
                   int mp, const float *T, float *ltau, hipStream_t st) {
	if (npos <= 0) return;
	pq_tau_kernel<<<dim3((unsigned)((npos + 255) / 256)), 256, 0, st>>>(codes, lslot, loff, nlist, npos, m, mp, T,
	                                                                      ltau);
}

// ---------------------------------------------------------------------------
// search: query prep, probe inversion
// ---------------------------------------------------------------------------
// Qf = zero-padded f32 queries; Qn = normalised queries (cosine):
// q^ = q / f32(sqrt(sum q^2)) with an IEEE f32 division (oracle/ivf.py)
__global__ __launch_bounds__(256) void ivf_prep_kernel(const float *__restrict__ Q, int dim, int ld, int normalize,
                                                       float *__restrict__ Qf, float *__restrict__ Qn) {
	__shared__ double sh[256];
	const int q = blockIdx.x, t = threadIdx.x;
	const float *x = Q + (int64_t)q * dim;
	double ss = 0.0;
	for (int i = t; i < ld; i += 256) {
		const float v = i < dim ? x[i] : 0.0f;
		Qf[(int64_t)q * ld + i] = v;
		ss += (double)v * v;
	}
	if (!normalize) return;
	sh[t] = ss;
	__syncthreads();
	for (int o = 128; o > 0; o >>= 1) {
		if (t < o) sh[t] += sh[t + o];
		__syncthreads();
	}
	const float nrm = (float)sqrt(sh[0]);
	for (int i = t; i < dim; i += 256) Qn[(int64_t)q * dim + i] = nrm > 0.0f ? __fdiv_rn(x[i], nrm) : x[i];
}

void launch_ivf_prep(const float *Q, int nq, int dim, int ld, int normalize, float *Qf, float *Qn, hipStream_t st) {
	ivf_prep_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(Q, dim, ld, normalize, Qf, Qn);
}

// f64 copies of the padded f32 queries and their |q|^2 summed in element
// order (the IVF_FLAT list scan reads them through scalar loads)
__global__ __launch_bounds__(256) void ivf_qd_kernel(const float *__restrict__ Qf, int ld, int dim,
                                                     double *__restrict__ Qd, double *__restrict__ qn2) {
	const int q = blockIdx.x, t = threadIdx.x;
	for (int i = t; i < ld; i += 256) Qd[(int64_t)q * ld + i] = (double)Qf[(int64_t)q * ld + i];
	if (t == 0) {
		double s = 0.0;
		for (int i = 0; i < dim; ++i) {
			const double v = (double)Qf[(int64_t)q * ld + i];
			s = fma(v, v, s);
		}
		qn2[q] = s;
	}
}

void launch_ivf_qd(const float *Qf, int nq, int ld, int dim, double *Qd, double *qn2, hipStream_t st) {
	ivf_qd_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(Qf, ld, dim, Qd, qn2);
}

__global__ void invert_count_kernel(const int64_t *__restrict__ probe_l, int n, int *__restrict__ lcnt) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const int64_t l = probe_l[i];
	if (l >= 0) atomicAdd(lcnt + l, 1);
}

// exclusive scan of lcnt into pstart[0..nlist], then lcnt = 0 (fill cursors)
__global__ __launch_bounds__(1024) void invert_scan_kernel(int *__restrict__ lcnt, int nlist, int *__restrict__ pstart) {
	__shared__ int sh[1024];
	const int t = threadIdx.x;
	const int per = (nlist + 1023) / 1024;
	const int a = t * per, b = min(nlist, a + per);
	int s = 0;
	for (int i = a; i < b; ++i) s += lcnt[i];
	sh[t] = s;
	__syncthreads();
	for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
		const int v = t >= o ? sh[t - o] : 0;
		__syncthreads();
		sh[t] += v;
		__syncthreads();
	}
	int run = sh[t] - s;
	for (int i = a; i < b; ++i) {
		pstart[i] = run;
		run += lcnt[i];
		lcnt[i] = 0;
	}
	if (t == 1023) pstart[nlist] = sh[1023];
}

__global__ void invert_fill_kernel(const int64_t *__restrict__ probe_l, int n, const int *__restrict__ pstart,
                                   int *__restrict__ cursor, int *__restrict__ pairs) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const int64_t l = probe_l[i];
	if (l < 0) return;
	const int p = atomicAdd(cursor + l, 1);
	pairs[pstart[l] + p] = i;
}

// Work items are laid out XCD-major: the lists l = x, x + 8, x + 16, ... first
// for XCD x, and a workgroup claims from its own XCD's counter (workgroups are
// dispatched round-robin over the 8 XCDs: XCD = blockIdx.x % 8) before it steals
// from the others.  The query groups of one list then run on one XCD, close in
// time, so a list's codes come from that XCD's L2 after its first group instead
// of from HBM once per group.
constexpr int NXCD = 8;
__device__ __forceinline__ int xcd_lists(int nlist, int x) { return x < nlist ? (nlist - x + NXCD - 1) / NXCD : 0; }
// the list at position p of the XCD-major order
__device__ __forceinline__ int lperm(int nlist, int p) {
	int x = 0;
	while (x < NXCD - 1 && p >= xcd_lists(nlist, x)) {
		p -= xcd_lists(nlist, x);
		++x;
	}
	return x + NXCD * p;
}

// the three launches above (and the cursor memset) as one workgroup when the
// per-list counters fit in LDS (round 6: ~17 -> a few us at C5): count with
// LDS atomics, exclusive scan (a thread per run of lists, wave scans), fill.
// With loff (the IVF_PQ fast scan), the same workgroup then lays out the scan's
// work items as pq_fast_items_kernel does (item_off over the XCD-major list
// order, xbeg), from the counts it already holds: one launch less.
constexpr int INV_THREADS = 1024, INV_MAX_LISTS = 16384;
__device__ __forceinline__ int block_excl_scan_i(int s, int *wsum, int &total) {
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	int x = s;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const int y = __shfl_up(x, o, 64);
		if (lane >= o) x += y;
	}
	if (lane == 63) wsum[w] = x;
	__syncthreads();
	int woff = 0, tot = 0;
	for (int j = 0; j < INV_THREADS / 64; ++j) {
		woff += j < w ? wsum[j] : 0;
		tot += wsum[j];
	}
	__syncthreads();  // (wsum is reused by the next scan)
	total = tot;
	return woff + x - s;
}
constexpr int INV_PT = 32;  // probes per thread kept in registers between the count and the fill
__global__ __launch_bounds__(INV_THREADS) void invert_fused_kernel(const int64_t *__restrict__ probe_l, int n,
                                                                   int nlist, int *__restrict__ pstart,
                                                                   int *__restrict__ pairs,
                                                                   const int64_t *__restrict__ loff,
                                                                   int *__restrict__ item_off,
                                                                   int *__restrict__ xbeg) {
	__shared__ int cnt[INV_MAX_LISTS];
	__shared__ int wsum[INV_THREADS / 64];
	const int t = threadIdx.x;
	const int per = (nlist + INV_THREADS - 1) / INV_THREADS;
	const int a = min(nlist, t * per), b = min(nlist, a + per);
	// every global read first, all in flight together: this thread's probes
	// (kept for the fill) and the row counts of its positions of the XCD-major
	// list order (the item layout)
	constexpr int IPT = 16;  // (per <= INV_MAX_LISTS / INV_THREADS)
	int pl[INV_PT];
#pragma unroll
	for (int u = 0; u < INV_PT; ++u) {
		const int i = t + u * INV_THREADS;
		pl[u] = i < n ? (int)probe_l[i] : -1;
	}
	int len[IPT], lst[IPT];
	if (loff) {
#pragma unroll
		for (int u = 0; u < IPT; ++u) {
			const int p = a + u;
			lst[u] = p < b ? lperm(nlist, p) : 0;
			len[u] = p < b ? (int)(loff[lst[u] + 1] - loff[lst[u]]) : 0;
		}
	}
	for (int i = t; i < nlist; i += INV_THREADS) cnt[i] = 0;
	__syncthreads();
#pragma unroll
	for (int u = 0; u < INV_PT; ++u)
		if (pl[u] >= 0) atomicAdd(&cnt[pl[u]], 1);
	for (int i = t + INV_PT * INV_THREADS; i < n; i += INV_THREADS) {  // (past the registers' share)
		const int64_t l = probe_l[i];
		if (l >= 0) atomicAdd(&cnt[l], 1);
	}
	__syncthreads();
	int is = 0, itm[IPT];
	if (loff) {
#pragma unroll
		for (int u = 0; u < IPT; ++u) {
			const int np = a + u < b ? cnt[lst[u]] : 0;
			itm[u] = np > 0 && len[u] > 0 ? ((np + FQ_G - 1) / FQ_G) * ((len[u] + FQ_CHUNK - 1) / FQ_CHUNK) : 0;
			is += itm[u];
		}
	}
	int s = 0;
	for (int i = a; i < b; ++i) s += cnt[i];
	int total;
	int run = block_excl_scan_i(s, wsum, total);
	for (int i = a; i < b; ++i) {  // (this thread's lists only: cnt becomes their fill cursor)
		const int c = cnt[i];
		pstart[i] = run;
		cnt[i] = run;
		run += c;
	}
	if (t == 0) pstart[nlist] = total;
	if (loff) {
		int itot;
		int ir = block_excl_scan_i(is, wsum, itot);
		// item_off over the positions; xbeg[x] = item_off at XCD x's first position
		// (written by the thread holding it; thread 0 writes those at nlist)
#pragma unroll
		for (int u = 0; u < IPT; ++u)
			if (a + u < b) {
				const int p = a + u;
				item_off[p] = ir;
				int p0 = 0;
				for (int x = 0; x < NXCD; ++x) {
					if (p == p0) xbeg[x] = ir;
					p0 += xcd_lists(nlist, x);
				}
				ir += itm[u];
			}
		if (t == 0) {
			item_off[nlist] = itot;
			int p0 = 0;
			for (int x = 0; x <= NXCD; ++x) {
				if (p0 >= nlist) xbeg[x] = itot;
				if (x < NXCD) p0 += xcd_lists(nlist, x);
			}
		}
	}
	__syncthreads();
#pragma unroll
	for (int u = 0; u < INV_PT; ++u)
		if (pl[u] >= 0) pairs[atomicAdd(&cnt[pl[u]], 1)] = t + u * INV_THREADS;
	for (int i = t + INV_PT * INV_THREADS; i < n; i += INV_THREADS) {
		const int64_t l = probe_l[i];
		if (l >= 0) pairs[atomicAdd(&cnt[l], 1)] = i;
	}
}

bool invert_fused_fits(int nlist) { return nlist <= INV_MAX_LISTS; }

void launch_invert(const int64_t *probe_l, int nq, int nprobe, int nlist, int *lcnt, int *pstart, int *pairs,
                   hipStream_t st, const int64_t *loff, int *item_off, int *xbeg) {
	const int n = nq * nprobe;
	if (invert_fused_fits(nlist)) {
		invert_fused_kernel<<<1, INV_THREADS, 0, st>>>(probe_l, n, nlist, pstart, pairs, loff, item_off, xbeg);
		return;
	}
	if (loff) throw std::runtime_error("launch_invert: the fused item layout needs nlist <= INV_MAX_LISTS");
	(void)hipMemsetAsync(lcnt, 0, (size_t)nlist * sizeof(int), st);
	invert_count_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(probe_l, n, lcnt);
	invert_scan_kernel<<<1, 1024, 0, st>>>(lcnt, nlist, pstart);
	invert_fill_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(probe_l, n, pstart, lcnt, pairs);
}

// ---------------------------------------------------------------------------
// IVF_FLAT list scan: work item = 256 positions of one list (or 256 rows of
// the unindexed tail) x every query probing the list, FS_G at a time (one
// pass for up to FS_G queries, so the rows stream from HBM once per item).
// Rows arrive FS_KC dims at a time in coalesced 128-B row segments, the next
// chunk prefetched into registers while the current one is consumed from LDS
// (rows padded to FS_KC + 1 floats: conflict-free column reads); each thread
// owns one row and accumulates (x - q)^2 (or x.q) in f64 for all FS_G queries.
// ---------------------------------------------------------------------------
constexpr int FS_G = 16;
#ifndef LHIP_FS_KC
#define LHIP_FS_KC 32
#endif
constexpr int FS_KC = LHIP_FS_KC;                       // dims per staged chunk (32 or 64)
constexpr int FS_NP = FS_KC / 4;                        // float4 pieces per row and chunk
constexpr int FS_PIECES = FLAT_BLK * FS_KC / 4 / 256;  // float4 pieces per thread and chunk

template <typename T>
__device__ __forceinline__ void fs_fetch(const T *__restrict__ X, int ld, int dim, const uint32_t *sslot, int d0,
                                         float4 (&v)[FS_PIECES]) {
#pragma unroll
	for (int i = 0; i < FS_PIECES; ++i) {
		const int e = threadIdx.x + i * 256, row = e / FS_NP, piece = e % FS_NP;
		const uint32_t s = sslot[row];
		v[i] = (s != SLOT_NONE && d0 < dim) ? load4(X + (int64_t)s * ld + d0 + piece * 4) : make_float4(0, 0, 0, 0);
	}
}

// chunk of FS_KC dims of 256 rows as float4 pieces, piece p of row r at
// p ^ (r % FS_NP): one ds_write_b128 per loaded piece, one ds_read_b128 per 4
// dims of a thread's row
__device__ __forceinline__ void fs_store(float4 (*xs)[FS_NP], const float4 (&v)[FS_PIECES]) {
#pragma unroll
	for (int i = 0; i < FS_PIECES; ++i) {
		const int e = threadIdx.x + i * 256, row = e / FS_NP, piece = e % FS_NP;
		xs[row][piece ^ (row % FS_NP)] = v[i];
	}
}

// one pass over the item's rows for G queries (sq / spair hold them).  The
// query values come through scalar loads of their f64 copies (wave-uniform
// addresses), the rows from LDS.  L2 as |x|^2 + |q|^2 - 2 x.q with every sum
// in f64 in element order (one FMA per element and query; x == q gives
// exactly 0): its f32 rounding equals the oracle's rounded sum of squared
// differences except within f64 noise of an f32 rounding boundary.
template <int METRIC, typename T, int G>
__device__ __forceinline__ void fs_group(const T *__restrict__ X, int ld, int dim, const double *__restrict__ Qd,
                                         const double *__restrict__ qn2, int ng, const uint32_t *sslot,
                                         const int *sq, const int *spair, float4 (*xs)[FS_NP], uint64_t *sk,
                                         uint64_t *o0, int64_t ostride, int kk, uint32_t sx) {
	const int t = threadIdx.x;
	const double *qp[G];
#pragma unroll
	for (int g = 0; g < G; ++g) qp[g] = Qd + (int64_t)__builtin_amdgcn_readfirstlane(sq[g < ng ? g : 0]) * ld;
	double acc[G], xx = 0.0;
#pragma unroll
	for (int g = 0; g < G; ++g) acc[g] = 0.0;
	float4 v[FS_PIECES];
	fs_fetch<T>(X, ld, dim, sslot, 0, v);
	for (int d0 = 0; d0 < dim; d0 += FS_KC) {
		__syncthreads();  // previous chunk consumed
		fs_store(xs, v);
		__syncthreads();
		if (d0 + FS_KC < dim) fs_fetch<T>(X, ld, dim, sslot, d0 + FS_KC, v);  // in flight during the FMAs
#pragma unroll 2
		for (int j = 0; j < FS_NP; ++j) {
			const float4 x4 = xs[t][j ^ (t % FS_NP)];
			const double xv[4] = {(double)x4.x, (double)x4.y, (double)x4.z, (double)x4.w};
#pragma unroll
			for (int c = 0; c < 4; ++c) {
				if (METRIC != METRIC_DOT) xx = fma(xv[c], xv[c], xx);
#pragma unroll
				for (int g = 0; g < G; ++g) acc[g] = fma(xv[c], qp[g][d0 + 4 * j + c], acc[g]);
			}
		}
	}
	const bool valid = sslot[t] != SLOT_NONE;
#pragma unroll
	for (int g = 0; g < G; ++g) {
		if (g >= ng) continue;  // ng is uniform: every thread skips together
		const double qq = METRIC == METRIC_DOT ? 0.0 : qn2[__builtin_amdgcn_readfirstlane(sq[g])];
		double r;
		if (METRIC == METRIC_L2)
			r = fmax(fma(-2.0, acc[g], xx + qq), 0.0);
		else if (METRIC == METRIC_DOT)
			r = 1.0 - acc[g];
		else
			r = 1.0 - acc[g] / (sqrt(xx) * sqrt(qq));
		float f = (float)r + 0.0f;
		if (__builtin_isnan(f)) f = __builtin_nanf("");
		// (exact keys: slot ^ sx, the tie rule of the final order; decoded by
		// whoever reads them: keys_to_output, the re-rank kernels' tail lists)
		const uint64_t key = valid ? key64(f, sslot[t] ^ sx) : KEY64_NONE;
		uint64_t *o = o0 + (int64_t)spair[g] * ostride;
		__syncthreads();  // sk reuse
		if (kk <= 16) {
			// each wave sorts its 64 keys in registers; the 4 x kk leaders are
			// sorted again by wave 0: two barriers instead of the 36 of a
			// workgroup bitonic sort of 256 keys
			const uint64_t ks = wave_sort64(key);
			const int lane = t & 63, w = t >> 6;
			if (lane < kk) sk[w * kk + lane] = ks;
			__syncthreads();
			if (w == 0) {
				const uint64_t k2 = wave_sort64(lane < 4 * kk ? sk[lane] : KEY64_NONE);
				if (lane < kk) o[lane] = k2;
			}
		} else {
			sk[t] = key;
			wg_bitonic_sort(sk, FLAT_BLK);
			for (int i = t; i < kk; i += 256) o[i] = i < FLAT_BLK ? sk[i] : KEY64_NONE;
		}
	}
}

template <int METRIC, typename T>
__global__ __launch_bounds__(256) void flat_list_scan_kernel(
    const T *__restrict__ X, int ld, int dim, const float *__restrict__ rowaux_f, const int *__restrict__ blk_list,
    const int64_t *__restrict__ blk_pos0, const int *__restrict__ lblk0, const int64_t *__restrict__ loff,
    const uint32_t *__restrict__ lslot, const int *__restrict__ pstart, const int *__restrict__ pairs, int nprobe,
    int maxb, int64_t tail_s0, int64_t tail_n, int nq, const double *__restrict__ Qd, const double *__restrict__ qn2,
    int kk, uint64_t *__restrict__ out, uint32_t sx) {
	__shared__ float4 xs[FLAT_BLK][FS_NP];
	__shared__ uint32_t sslot[FLAT_BLK];
	__shared__ uint64_t sk[FLAT_BLK];
	__shared__ int sq[FS_G], spair[FS_G];
	const int t = threadIdx.x;
	const int b = blockIdx.x;
	const bool tail = tail_n > 0;
	int pa, pb, bi = 0;
	int64_t p0, p1;
	if (tail) {
		p0 = (int64_t)b * FLAT_BLK;
		p1 = min<int64_t>(tail_n, p0 + FLAT_BLK);
		pa = 0;
		pb = nq;
	} else {
		const int l = blk_list[b];
		p0 = blk_pos0[b];
		p1 = min<int64_t>(loff[l + 1], p0 + FLAT_BLK);
		pa = pstart[l];
		pb = pstart[l + 1];
		bi = b - lblk0[l];
	}
	if (pa >= pb) return;
	{
		uint32_t s = SLOT_NONE;
		if (p0 + t < p1) {
			s = tail ? (uint32_t)(tail_s0 + p0 + t) : lslot[p0 + t];
			if (s != SLOT_NONE && !slot_alive(rowaux_f, s)) s = SLOT_NONE;
		}
		sslot[t] = s;
	}
	const int tail_nb = (int)((tail_n + FLAT_BLK - 1) / FLAT_BLK);
	// output of pair pid: out + pid * ostride + o_off
	uint64_t *o0 = tail ? out + (int64_t)b * kk : out + (int64_t)bi * kk;
	const int64_t ostride = tail ? (int64_t)tail_nb * kk : (int64_t)maxb * kk;
	for (int g0 = pa; g0 < pb; g0 += FS_G) {
		const int ng = min(FS_G, pb - g0);
		__syncthreads();
		if (t < FS_G) {
			const int pid = t < ng ? (tail ? g0 + t : pairs[g0 + t]) : -1;
			spair[t] = pid;
			sq[t] = pid < 0 ? 0 : (tail ? pid : pid / nprobe);
		}
		__syncthreads();
		// per-item query count decides the register block (f64 work scales with it)
#define FS_CALL(GG) fs_group<METRIC, T, GG>(X, ld, dim, Qd, qn2, ng, sslot, sq, spair, xs, sk, o0, ostride, kk, sx)
		if (ng <= 2) FS_CALL(2);
		else if (ng <= 4) FS_CALL(4);
		else if (ng <= 8) FS_CALL(8);
		else FS_CALL(FS_G);
#undef FS_CALL
	}
}

// ---------------------------------------------------------------------------
// IVF_FLAT bound scan (MFMA): the same work items, but each (query, row) pair
// gets the flat scan's rigorous bf16 lower bound LB <= exact distance
// (knn_kernels.hip prep_queries / scan_kernel numerics: bf16 rows of the scan
// copy or bf16 store, v_mfma_f32_16x16x32_bf16, the row / query bound terms)
// instead of an f64 distance; per (query, item) the FL_T smallest (LB, slot)
// keys go out.  The per-query merge keeps the FL_T - 1 leaders of every item
// and takes the top M by LB; cut = min(the (M+1)-th merged LB, every item's
// FL_T-th LB): every row left out has LB >= cut.  The exact f64 re-rank of the
// M then returns the top k, certified when cut > the k-th exact distance;
// an uncertified batch reruns on the exact list scan.
// Block: 4 waves x 64 rows (4 blocks of 16), one 16-query MFMA column block.
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
#ifndef LHIP_FL_V2
#define LHIP_FL_V2 1  // round 6: bound words in the query rows' LDS, 3 workgroups per CU (0: round 5's layout, an A/B)
#endif
constexpr int FL_G = 16;   // queries per MFMA column block
constexpr int FL_T = FL_KEYS;  // keys per (query, item)

template <int METRIC>
__global__ __launch_bounds__(256) void flat_list_lb_kernel(
    const uint16_t *__restrict__ Xb, int ld, const float *__restrict__ rowaux_f, const int *__restrict__ blk_list,
    const int64_t *__restrict__ blk_pos0, const int *__restrict__ lblk0, const int64_t *__restrict__ loff,
    const uint32_t *__restrict__ lslot, int nblk, const int *__restrict__ pstart, const int *__restrict__ pairs,
    int nprobe, int maxb, const uint16_t *__restrict__ Qb, const float4 *__restrict__ qaux,
    uint64_t *__restrict__ out, const uint16_t *__restrict__ Lrows, const float4 *__restrict__ Lterms,
    const uint32_t *__restrict__ live_bits, const int *__restrict__ boff, const int *__restrict__ tot,
    const int *__restrict__ itb, int itb_cap) {
	extern __shared__ __attribute__((aligned(16))) uint8_t fl_smem[];
	const int qrow = ld * 2 + 16;  // padded query row (bytes): 16 lanes reading 16 rows hit distinct banks
	uint8_t *qs = fl_smem;  // [FL_G][qrow]
#if LHIP_FL_V2
	// the bound words [FL_G][256] (u32: the row's slot is sslot[row]) share the
	// query rows' LDS, which the K loop has finished reading when they are
	// written: ~31 KB per workgroup, 3 resident per CU (was 57 KB, 2)
	uint32_t *sk = reinterpret_cast<uint32_t *>(fl_smem);
#else
	uint64_t *sk = reinterpret_cast<uint64_t *>(fl_smem + FL_G * qrow);            // [FL_G][256] keys
#endif
	__shared__ uint32_t sslot[FLAT_BLK];
	__shared__ float4 ras[FLAT_BLK];
	__shared__ float4 qas[FL_G];
	__shared__ int sq[FL_G], spair[FL_G];
	__shared__ int snan[FL_G];  // a live row of this item has a NaN bound for the query (zero cosine row / query)
	constexpr bool FOLD = METRIC != METRIC_COSINE;
	const int t = threadIdx.x, lane = t & 63, w = t >> 6;
	const int gq = lane >> 4, rr = lane & 15;
	// work items = (block b, query group g) for every block of a probed list
	// (boff: exclusive prefix of ceil(probing queries / FL_G) over the blocks, tot
	// = their sum), cut into 8 contiguous ranges, one per XCD (workgroups are
	// dispatched round-robin over the XCDs: XCD = blockIdx.x % 8).  The workgroups
	// of an XCD take consecutive items, so the query groups of one block run side
	// by side on ONE XCD and its rows come from that XCD's L2 after the first
	// group instead of from HBM once per group.
	const int T = *tot, Tx = (T + 7) >> 3, xc = blockIdx.x & 7, Wx = gridDim.x >> 3;
	for (int j = blockIdx.x >> 3; j < Tx; j += Wx) {
	const int it = xc * Tx + j;
	if (it >= T) break;
	int b;
	if (itb && it < itb_cap) {
		b = itb[it];  // (flat_lb_table_kernel: one read instead of a chain of dependent ones)
	} else {
		int lo = 0, hi = nblk - 1;  // the last block whose items start at or before it
		while (lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if (boff[mid] <= it) lo = mid;
			else hi = mid - 1;
		}
		b = lo;
	}
	const int l = blk_list[b];
	const int64_t p0 = blk_pos0[b];
	const int64_t p1 = min<int64_t>(loff[l + 1], p0 + FLAT_BLK);
	const int pa = pstart[l], pb = pstart[l + 1];
	const int bi = b - lblk0[l];
	__syncthreads();  // (the previous item's LDS reads done)
	{
		uint32_t s = SLOT_NONE;
		if (p0 + t < p1) s = lslot[p0 + t];
		sslot[t] = s;
		// row terms (alpha, xn, ux, sc); padding: alpha = +inf (LB = +inf).  With
		// list-order rows the terms come in list order too (one coalesced 16-B read
		// per position, fixed since the layout was built) and whether the row is live
		// (not deleted, selected by the predicate) from a bitmap of the slots built
		// per search (live_bits: 1 bit per slot, L2-resident) instead of four random
		// row-aux lines per row
		float4 r = make_float4(F_INF, 0.f, 0.f, 0.f);
		if (s != SLOT_NONE) {
			if (Lterms) {
				if ((live_bits[s >> 5] >> (s & 31)) & 1u) r = Lterms[p0 + t];
			} else {
				r = make_float4(rowaux_f[raix(s, 0)], rowaux_f[raix(s, 1)], rowaux_f[raix(s, 2)], rowaux_f[raix(s, 3)]);
			}
		}
		ras[t] = r;
	}
	const int nw = ld / 64;  // 64-deep k windows (ld is a multiple of 64)
	{
		const int g0 = pa + (it - boff[b]) * FL_G;
		const int ng = min(FL_G, pb - g0);
		__syncthreads();
		if (t < FL_G) {
			const int pid = t < ng ? pairs[g0 + t] : -1;
			spair[t] = pid;
			sq[t] = pid < 0 ? -1 : pid / nprobe;
			qas[t] = pid < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : qaux[pid / nprobe];
			snan[t] = 0;
		}
		__syncthreads();
		// the group's bf16 query rows into LDS (zero rows for unused columns)
		for (int e = t; e < FL_G * (ld / 8); e += 256) {
			const int c = e / (ld / 8), k8 = e % (ld / 8);
			uint4 v = make_uint4(0u, 0u, 0u, 0u);
			if (sq[c] >= 0) v = *reinterpret_cast<const uint4 *>(Qb + (int64_t)sq[c] * ld + 8 * k8);
			*reinterpret_cast<uint4 *>(qs + c * qrow + 16 * k8) = v;
		}
		__syncthreads();
		// accumulators: rows 64w + 16rb + (4 gq .. 4 gq + 3), query rr
		f32x4 acc[4];
		if (FOLD) {
			// alpha + C + xn*B + ux*A by one exact-f32 16x16x4 MFMA per block:
			// A[row][k] = (xn, ux, alpha, 1), B[k][query] = (B, A, 1, C)
			const float4 qa = qas[rr];
			const float bv = gq == 0 ? qa.z : gq == 1 ? qa.y : gq == 2 ? 1.0f : qa.w;
			const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
			for (int rb = 0; rb < 4; ++rb) {
				const float4 ra = ras[64 * w + 16 * rb + rr];
				const float av = gq == 0 ? ra.y : gq == 1 ? ra.z : gq == 2 ? ra.x : 1.0f;
				acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, z, 0, 0, 0);
			}
			mfma_operand_guard();  // VALU (row pointers) follows the fold MFMAs
		} else {
#pragma unroll
			for (int rb = 0; rb < 4; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
		}
		// row pointers of this lane's 4 rows: list-order rows (the item is one
		// contiguous 256 x ld block; positions past the list end read the next
		// list's or zero padding rows), else by slot (padding rows read slot 0);
		// either way a padding row's LB is +inf through alpha
		const uint16_t *xp[4];
#pragma unroll
		for (int rb = 0; rb < 4; ++rb) {
			const int r = 64 * w + 16 * rb + rr;
			const uint32_t s = sslot[r];
			xp[rb] = Lrows ? Lrows + (p0 + r) * (int64_t)ld + 8 * gq : Xb + (int64_t)(s == SLOT_NONE ? 0u : s) * ld + 8 * gq;
		}
		const uint8_t *qb = qs + rr * qrow + 16 * gq;
		// two windows of rows in flight
		uint4 xa[2][4][2];
		auto ldx = [&](uint4 (&d)[4][2], int kw) __attribute__((always_inline)) {
#pragma unroll
			for (int rb = 0; rb < 4; ++rb) {
				d[rb][0] = *reinterpret_cast<const uint4 *>(xp[rb] + 64 * kw);
				d[rb][1] = *reinterpret_cast<const uint4 *>(xp[rb] + 64 * kw + 32);
			}
		};
		ldx(xa[0], 0);
		if (nw > 1) ldx(xa[1], 1);
		for (int kw = 0; kw < nw; kw += 2) {
#pragma unroll
			for (int h = 0; h < 2; ++h) {
				const int k = kw + h;
				if (k < nw) {
					const bf16x8 b0 = *reinterpret_cast<const bf16x8 *>(qb + 128 * k);
					const bf16x8 b1 = *reinterpret_cast<const bf16x8 *>(qb + 128 * k + 64);
#pragma unroll
					for (int rb = 0; rb < 4; ++rb) {
						acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa[h][rb][0]), b0,
						                                                  acc[rb], 0, 0, 0);
						acc[rb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xa[h][rb][1]), b1,
						                                                  acc[rb], 0, 0, 0);
					}
					// refill the window's registers after the MFMAs that read them (no
					// register copy between the load and the MFMAs; the load lands late)
					if (k + 2 < nw) ldx(xa[h], k + 2);
				}
			}
		}
		mfma_operand_guard();
#if LHIP_FL_V2
		__syncthreads();  // (every wave's query-row reads done: the bound words overwrite them)
#endif
		// keys -> LDS [query][row]
		{
			const float4 qa = qas[rr];
#pragma unroll
			for (int rb = 0; rb < 4; ++rb)
#pragma unroll
				for (int i = 0; i < 4; ++i) {
					const int r = 64 * w + 16 * rb + 4 * gq + i;
					const uint32_t s = sslot[r];
					float lb;
					if (FOLD) {
						lb = acc[rb][i];
					} else {
						const float4 ra = ras[r];
						float v = fmaf(ra.y, qa.z, ra.x);
						v = fmaf(ra.z, qa.y, v);
						v = fmaf(acc[rb][i] * ra.w, qa.x, v);
						lb = v + qa.w;
					}
					const bool live = s != SLOT_NONE && ras[r].x != F_INF;
					const bool ok = live && !__builtin_isnan(lb);
					// a live row without a bound cannot be certified away: the
					// item's boundary becomes -inf (the query reruns exactly)
					if (live && __builtin_isnan(lb)) snan[rr] = 1;
#if LHIP_FL_V2
					sk[rr * FLAT_BLK + r] = ok ? fkey(lb) : 0xFFFFFFFFu;  // (fkey of a non-NaN float < 0xFFFFFFFF)
#else
					sk[rr * FLAT_BLK + r] = ok ? key64(lb, s) : KEY64_NONE;
#endif
				}
		}
		__syncthreads();
		// per query: each wave sorts its 64 rows' keys, the 4 x 16 leaders are
		// sorted again; wave w handles queries w, w + 4, ...
		for (int c = w; c < ng; c += 4) {
			uint64_t best = KEY64_NONE;
#pragma unroll
			for (int ww = 0; ww < 4; ++ww) {
#if LHIP_FL_V2
				const uint32_t hw = sk[c * FLAT_BLK + 64 * ww + lane];
				const uint64_t ks = wave_sort64(hw == 0xFFFFFFFFu ? KEY64_NONE
				                                                  : ((uint64_t)hw << 32) | sslot[64 * ww + lane]);
#else
				const uint64_t ks = wave_sort64(sk[c * FLAT_BLK + 64 * ww + lane]);
#endif
				// leader lanes 16 ww .. 16 ww + 15 of the final sort take ks[0..15]
				const uint64_t moved = __shfl(ks, lane & 15, 64);
				if ((lane >> 4) == ww) best = moved;
			}
			best = wave_sort64(best);
			if (lane == FL_T - 1 && snan[c]) best = key64(-F_INF, 0u);  // boundary -inf: never certified
			if (lane < FL_T) out[((int64_t)spair[c] * maxb + bi) * FL_T + lane] = best;
		}
	}
	}  // items
}

// boff [nblk + 1]: exclusive prefix over the blocks of ceil(probing queries of
// the block's list / FL_G) (the bound scan's work items); tot[0] = the total
__global__ __launch_bounds__(1024) void flat_lb_items_kernel(const int *__restrict__ blk_list,
                                                             const int *__restrict__ pstart, int nblk,
                                                             int *__restrict__ boff, int *__restrict__ tot) {
	__shared__ int sh[1024];
	const int t = threadIdx.x;
	const int per = (nblk + 1023) / 1024;
	const int a = t * per, e = min(nblk, a + per);
	auto items = [&](int b) {
		const int l = blk_list[b];
		return (pstart[l + 1] - pstart[l] + FL_G - 1) / FL_G;
	};
	int s = 0;
	for (int i = a; i < e; ++i) s += items(i);
	sh[t] = s;
	__syncthreads();
	for (int o = 1; o < 1024; o <<= 1) {
		const int v = t >= o ? sh[t - o] : 0;
		__syncthreads();
		sh[t] += v;
		__syncthreads();
	}
	int run = sh[t] - s;
	for (int i = a; i < e; ++i) {
		boff[i] = run;
		run += items(i);
	}
	if (t == 1023) {
		boff[nblk] = sh[1023];
		*tot = sh[1023];
	}
}

// itb[it] = the block of bound-scan item it (thread per block: its
// ceil(probing queries / FL_G) items), so the scan finds an item's block with
// one read
__global__ __launch_bounds__(256) void flat_lb_table_kernel(const int *__restrict__ boff, int nblk,
                                                            int *__restrict__ itb, int itb_cap) {
	const int b = blockIdx.x * 256 + threadIdx.x;
	if (b >= nblk) return;
	const int e = min(boff[b + 1], itb_cap);
	for (int it = boff[b]; it < e; ++it) itb[it] = b;
}

// per query: merge the items' leaders of its probed lists (FL_T - 1 per item
// into a top-M), cut = min(the item boundaries, the merged (M+1)-th LB)
__global__ __launch_bounds__(256) void flat_lb_merge_kernel(int nprobe, const int64_t *__restrict__ probe_l,
                                                            const int *__restrict__ lblk0, int maxb,
                                                            const uint64_t *__restrict__ keys, int M,
                                                            uint64_t *__restrict__ cand, float *__restrict__ cut) {
	__shared__ uint64_t buf[IVF_TOPK_CAP];
	__shared__ int cnt;
	__shared__ uint64_t thr;
	__shared__ uint32_t bmin;
	const int q = blockIdx.x, t = threadIdx.x;
	TopK tk{buf, &cnt, &thr, M + 1};
	if (t == 0) bmin = 0xFFFFFFFFu;
	tk.reset();
	uint32_t mymin = 0xFFFFFFFFu;
	for (int p = 0; p < nprobe; ++p) {
		const int64_t l = probe_l[(int64_t)q * nprobe + p];
		if (l < 0) continue;
		const int nb = lblk0[l + 1] - lblk0[l];
		const uint64_t *src = keys + ((int64_t)q * nprobe + p) * maxb * FL_T;
		const int tot = nb * FL_T;
		for (int e0 = 0; e0 < tot; e0 += 256) {
			const int e = e0 + t;
			uint64_t k = e < tot ? src[e] : KEY64_NONE;
			if (e < tot && (e % FL_T) == FL_T - 1) {  // an item's boundary
				if (k != KEY64_NONE) mymin = min(mymin, (uint32_t)(k >> 32));
				k = KEY64_NONE;
			}
			tk.offer(k, k != KEY64_NONE);
		}
	}
	atomicMin(&bmin, mymin);
	const int n = tk.finish();
	__syncthreads();
	uint32_t cm = bmin;
	if (n > M) cm = min(cm, (uint32_t)(buf[M] >> 32));
	for (int i = t; i < M; i += 256) cand[(int64_t)q * M + i] = i < n ? buf[i] : KEY64_NONE;
	if (t == 0) cut[q] = cm == 0xFFFFFFFFu ? F_INF : fkey_inv(cm);
}

// exact f64 re-rank of the M bound candidates (+ the tail's exact keys), top k,
// certificate: cut > the k-th exact distance of the result (or fewer than k
// rows exist and nothing was cut)
constexpr int RR_THREADS = 1024;  // re-rank workgroup: 16 waves, ~k r / 16 candidate rows each
template <int METRIC, typename T>
__global__ __launch_bounds__(RR_THREADS) void flat_lb_refine_kernel(const T *__restrict__ X, int ld, int dim,
                                                             const float *__restrict__ Qf,
                                                             const uint64_t *__restrict__ ca, int M,
                                                             const uint64_t *__restrict__ cbk, int kb,
                                                             const float *__restrict__ cut, int k,
                                                             const int64_t *__restrict__ labels,
                                                             int64_t *__restrict__ outL, float *__restrict__ outD,
                                                             int *__restrict__ outC, int *__restrict__ cert,
                                                             uint32_t sx) {
	__shared__ uint64_t sk[IVF_TOPK_CAP];
	__shared__ uint32_t ss[IVF_TOPK_CAP];
	__shared__ int n;
	const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
	if (t == 0) n = 0;
	__syncthreads();
	for (int i = t; i < M + kb; i += RR_THREADS) {
		// (bound keys carry the slot; the tail's exact keys slot ^ sx)
		const uint64_t key = i < M ? ca[(int64_t)q * M + i] : cbk[(int64_t)q * kb + (i - M)];
		if (key != KEY64_NONE) ss[atomicAdd(&n, 1)] = (uint32_t)key ^ (i < M ? 0u : sx);
	}
	__syncthreads();
	const int nc = n;
	for (int i = w; i < nc; i += RR_THREADS / 64) {
		const uint32_t slot = ss[i];
		const float d = exact_distance<METRIC, T>(X + (int64_t)slot * ld, Qf + (int64_t)q * ld, dim, lane);
		if (lane == 0) sk[i] = key64(d, slot ^ sx);
	}
	const int np = pow2_ceil(nc);
	__syncthreads();
	for (int i = nc + t; i < np; i += RR_THREADS) sk[i] = KEY64_NONE;
	wg_bitonic_sort(sk, np);
	const int nout = nc < k ? nc : k;
	for (int i = t; i < k; i += RR_THREADS) {
		if (i < nout) {
			outL[(int64_t)q * k + i] = labels[(uint32_t)sk[i] ^ sx];
			outD[(int64_t)q * k + i] = key64_dist(sk[i]);
		} else {
			outL[(int64_t)q * k + i] = -1;
			outD[(int64_t)q * k + i] = __builtin_nanf("");
		}
	}
	if (t == 0) {
		outC[q] = nout;
		const float cq = cut[q];
		bool ok;
		if (nout < k) ok = cq == F_INF;  // every row of the probed lists is a candidate
		else ok = cq > key64_dist(sk[k - 1]);  // NaN cut or distance: false
		cert[q] = ok ? 1 : 0;
	}
}

size_t flat_lb_lds_bytes(int ld) {
#if LHIP_FL_V2
	return std::max((size_t)FL_G * (ld * 2 + 16), (size_t)FL_G * FLAT_BLK * 4);
#else
	return (size_t)FL_G * (ld * 2 + 16) + (size_t)FL_G * FLAT_BLK * 8;
#endif
}

__global__ __launch_bounds__(256) void live_bits_kernel(const float *__restrict__ rowaux_f, int64_t n,
                                                        uint32_t *__restrict__ bits);

void launch_flat_list_lb(const StoreView &s, const int *blk_list, const int64_t *blk_pos0, const int *lblk0,
                         const int64_t *loff, const uint32_t *lslot, int nblk, const int *pstart, const int *pairs,
                         int nprobe, int maxb, const uint16_t *Qb, const float4 *qaux, uint64_t *out, hipStream_t st,
                         const uint16_t *lrows, const float4 *lterms, uint32_t *live_bits, int *boff, int *tot,
                         int *itb, int itb_cap) {
	if (nblk <= 0) return;
	if (lrows) {  // the live bitmap of the slots (deletes / the predicate of this search: alpha = +inf)
		const int64_t n = s.n_slots;
		if (n > 0)
			live_bits_kernel<<<dim3((unsigned)((n + 255) / 256)), 256, 0, st>>>(reinterpret_cast<const float *>(s.rowaux), n,
			                                                                    live_bits);
	}
	flat_lb_items_kernel<<<1, 1024, 0, st>>>(blk_list, pstart, nblk, boff, tot);
	if (itb) flat_lb_table_kernel<<<dim3((unsigned)((nblk + 255) / 256)), 256, 0, st>>>(boff, nblk, itb, itb_cap);
	if ((!lrows && !s.scan_bf16) || s.ld % 64) throw std::runtime_error("IVF_FLAT bound scan needs bf16 scan rows");
	const uint16_t *Xb = static_cast<const uint16_t *>(s.Xscan);
	const float *ra = reinterpret_cast<const float *>(s.rowaux);
	const size_t lds = flat_lb_lds_bytes(s.ld);
	auto go = [&](auto kern) {
		HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
		                           (int)lds));
		// persistent, a multiple of the 8 XCDs: LHIP_FL_V2 3 workgroups per CU (31 KB
		// of LDS, 148 VGPRs: 3 waves per SIMD), else 2 (57 KB)
		const int grid = std::max(8, ((LHIP_FL_V2 ? 3 : 2) * scan_grid(1 << 20) / 8) * 8);
		kern<<<dim3((unsigned)grid), 256, lds, st>>>(Xb, s.ld, ra, blk_list, blk_pos0, lblk0, loff, lslot, nblk, pstart,
		                                             pairs, nprobe, maxb, Qb, qaux, out, lrows, lrows ? lterms : nullptr,
		                                             live_bits, boff, tot, itb, itb_cap);
	};
	switch (s.metric) {
	case METRIC_L2: go(flat_list_lb_kernel<METRIC_L2>); break;
	case METRIC_DOT: go(flat_list_lb_kernel<METRIC_DOT>); break;
	default: go(flat_list_lb_kernel<METRIC_COSINE>); break;
	}
}

// one wave per list position: 8 elements per lane and step (two 16-B f32 loads
// or one 16-B bf16 load -> one 16-B store)
__global__ __launch_bounds__(256) void list_rows_bf16_kernel(const void *__restrict__ X, int xbf16, int ld, int dim,
                                                             const uint32_t *__restrict__ lslot, int64_t npos,
                                                             uint16_t *__restrict__ out) {
	const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
	const int lane = threadIdx.x & 63;
	if (p >= npos) return;
	const uint32_t s = lslot[p];
	for (int c = 8 * lane; c < ld; c += 512) {
		uint4 o = make_uint4(0u, 0u, 0u, 0u);
		if (s != SLOT_NONE) {
			if (xbf16) {
				o = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(X) + (int64_t)s * ld + c);
			} else {
				const float *x = static_cast<const float *>(X) + (int64_t)s * ld + c;
				const float4 a = *reinterpret_cast<const float4 *>(x), b = *reinterpret_cast<const float4 *>(x + 4);
				// (padding columns of the store are zero: bf16 zero)
				o = make_uint4(pk_bf16(a.x, a.y), pk_bf16(a.z, a.w), pk_bf16(b.x, b.y), pk_bf16(b.z, b.w));
			}
		}
		*reinterpret_cast<uint4 *>(out + p * ld + c) = o;
	}
}

// out [npos] = the row terms (alpha, xn, ux, sc) of the row at each list position (+inf alpha for padding);
// fixed for the rows of a layout (a deleted row is masked by live_bits, not here)
__global__ __launch_bounds__(256) void list_terms_kernel(const float *__restrict__ rowaux_f,
                                                         const uint32_t *__restrict__ lslot, int64_t npos,
                                                         float4 *__restrict__ out) {
	const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
	if (p >= npos) return;
	const uint32_t s = lslot[p];
	out[p] = s == SLOT_NONE ? make_float4(F_INF, 0.f, 0.f, 0.f)
	                        : make_float4(rowaux_f[raix(s, 0)], rowaux_f[raix(s, 1)], rowaux_f[raix(s, 2)],
	                                      rowaux_f[raix(s, 3)]);
}

// bits [ceil(n / 32)]: bit s = slot s is live for this search (its row aux alpha < +inf)
__global__ __launch_bounds__(256) void live_bits_kernel(const float *__restrict__ rowaux_f, int64_t n,
                                                        uint32_t *__restrict__ bits) {
	const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
	const bool live = s < n && rowaux_f[raix(s, 0)] != F_INF;
	const uint64_t m = __builtin_amdgcn_ballot_w64(live);
	const int lane = threadIdx.x & 63;
	if (lane == 0 && s < n) bits[s >> 5] = (uint32_t)m;
	if (lane == 32 && s < n) bits[s >> 5] = (uint32_t)(m >> 32);
}

void launch_list_terms(const float4 *rowaux, const uint32_t *lslot, int64_t npos, float4 *out, hipStream_t st) {
	if (npos > 0)
		list_terms_kernel<<<dim3((unsigned)((npos + 255) / 256)), 256, 0, st>>>(reinterpret_cast<const float *>(rowaux),
		                                                                        lslot, npos, out);
}

void launch_list_rows_bf16(const void *X, int xbf16, int ld, int dim, const uint32_t *lslot, int64_t npos,
                           uint16_t *out, hipStream_t st) {
	if (npos <= 0) return;
	if (ld % 8) throw std::runtime_error("list rows: row stride must be a multiple of 8");
	list_rows_bf16_kernel<<<dim3((unsigned)((npos + 3) / 4)), 256, 0, st>>>(X, xbf16, ld, dim, lslot, npos, out);
}

void launch_flat_lb_merge(int nq, int nprobe, const int64_t *probe_l, const int *lblk0, int maxb, const uint64_t *keys,
                          int M, uint64_t *cand, float *cut, hipStream_t st) {
	flat_lb_merge_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(nprobe, probe_l, lblk0, maxb, keys, M, cand, cut);
}

void launch_flat_lb_refine(const StoreView &s, const float *Qf, const uint64_t *ca, int M, const uint64_t *cb, int kb,
                           const float *cut, int nq, int k, int64_t *outL, float *outD, int *outC, int *cert,
                           hipStream_t st) {
	dim3 grid((unsigned)nq);
	auto go = [&](auto kern, auto X) {
		kern<<<grid, RR_THREADS, 0, st>>>(X, s.ld, s.dim, Qf, ca, M, cb, kb, cut, k, s.labels, outL, outD, outC, cert,
		                           tie_x32(s.tie_desc));
	};
	if (s.xbf16) {
		const uint16_t *X = static_cast<const uint16_t *>(s.X);
		if (s.metric == METRIC_L2) go(flat_lb_refine_kernel<METRIC_L2, uint16_t>, X);
		else if (s.metric == METRIC_DOT) go(flat_lb_refine_kernel<METRIC_DOT, uint16_t>, X);
		else go(flat_lb_refine_kernel<METRIC_COSINE, uint16_t>, X);
	} else {
		const float *X = static_cast<const float *>(s.X);
		if (s.metric == METRIC_L2) go(flat_lb_refine_kernel<METRIC_L2, float>, X);
		else if (s.metric == METRIC_DOT) go(flat_lb_refine_kernel<METRIC_DOT, float>, X);
		else go(flat_lb_refine_kernel<METRIC_COSINE, float>, X);
	}
}

template <typename T>
static void flat_scan_dispatch(const StoreView &s, const int *blk_list, const int64_t *blk_pos0, const int *lblk0,
                               const int64_t *loff, const uint32_t *lslot, int nblk, const int *pstart,
                               const int *pairs, int nprobe, int maxb, int64_t tail_s0, int64_t tail_n, int nq,
                               const double *Qd, const double *qn2, int kk, uint64_t *out, hipStream_t st) {
	const T *X = static_cast<const T *>(s.X);
	const float *ra = reinterpret_cast<const float *>(s.rowaux);
	dim3 grid((unsigned)nblk);
#define FS_ARGS X, s.ld, s.dim, ra, blk_list, blk_pos0, lblk0, loff, lslot, pstart, pairs, nprobe, maxb, tail_s0, tail_n, nq, Qd, qn2, kk, out, tie_x32(s.tie_desc)
	switch (s.metric) {
	case METRIC_L2: flat_list_scan_kernel<METRIC_L2, T><<<grid, 256, 0, st>>>(FS_ARGS); break;
	case METRIC_DOT: flat_list_scan_kernel<METRIC_DOT, T><<<grid, 256, 0, st>>>(FS_ARGS); break;
	default: flat_list_scan_kernel<METRIC_COSINE, T><<<grid, 256, 0, st>>>(FS_ARGS); break;
	}
#undef FS_ARGS
}

void launch_flat_list_scan(const StoreView &s, const int *blk_list, const int64_t *blk_pos0, const int *lblk0,
                           const int64_t *loff, const uint32_t *lslot, int nblk, const int *pstart, const int *pairs,
                           int nprobe, int maxb, int64_t tail_s0, int64_t tail_n, int nq, const double *Qd, const double *qn2, int kk,
                           uint64_t *out, hipStream_t st) {
	if (nblk <= 0) return;
	if (s.xbf16)
		flat_scan_dispatch<uint16_t>(s, blk_list, blk_pos0, lblk0, loff, lslot, nblk, pstart, pairs, nprobe, maxb,
		                             tail_s0, tail_n, nq, Qd, qn2, kk, out, st);
	else
		flat_scan_dispatch<float>(s, blk_list, blk_pos0, lblk0, loff, lslot, nblk, pstart, pairs, nprobe, maxb,
		                          tail_s0, tail_n, nq, Qd, qn2, kk, out, st);
}

// ---------------------------------------------------------------------------
// IVF_PQ
// ---------------------------------------------------------------------------
// P[q][j][c] = sum_t q_{j,t} y_{j,c,t}  (f32, t in order, no contraction)
// (a workgroup per (PQ_PQB queries, sub-space): the codebook slice is read once
// for the group; one query per workgroup was 24576 tiny workgroups for C5,
// ~90 us of workgroup dispatch)
constexpr int PQ_PQB = 8, PQ_PDS = 16;
__global__ __launch_bounds__(256) void pq_P_kernel(const float *__restrict__ Q, int qld, const float *__restrict__ cb,
                                                   int nq, int m, int dsub, float *__restrict__ P) {
	const int q0 = blockIdx.x * PQ_PQB, j = blockIdx.y, c = threadIdx.x;
	const float *y = cb + ((int64_t)j * PQ_K + c) * dsub;
	if (dsub <= PQ_PDS) {
		// every load in flight before the sums (a runtime-length loop waited on each)
		float yv[PQ_PDS];
#pragma unroll
		for (int t = 0; t < PQ_PDS; ++t) yv[t] = t < dsub ? y[t] : 0.0f;
		for (int qi = 0; qi < PQ_PQB && q0 + qi < nq; ++qi) {
			const int q = q0 + qi;
			const float *x = Q + (int64_t)q * qld + j * dsub;
			float xv[PQ_PDS];
#pragma unroll
			for (int t = 0; t < PQ_PDS; ++t) xv[t] = t < dsub ? x[t] : 0.0f;
			float acc = 0.0f;
#pragma unroll
			for (int t = 0; t < PQ_PDS; ++t)
				if (t < dsub) acc = add_nc(acc, mul_nc(xv[t], yv[t]));
			P[((int64_t)q * m + j) * PQ_K + c] = acc;
		}
		return;
	}
	for (int qi = 0; qi < PQ_PQB && q0 + qi < nq; ++qi) {
		const int q = q0 + qi;
		const float *x = Q + (int64_t)q * qld + j * dsub;
		float acc = 0.0f;
		for (int t = 0; t < dsub; ++t) acc = add_nc(acc, mul_nc(x[t], y[t]));
		P[((int64_t)q * m + j) * PQ_K + c] = acc;
	}
}

void launch_pq_P(const float *Q, int qld, int nq, const float *cb, int m, int dsub, float *P, hipStream_t st) {
	pq_P_kernel<<<dim3((unsigned)((nq + PQ_PQB - 1) / PQ_PQB), (unsigned)m), PQ_K, 0, st>>>(Q, qld, cb, nq, m, dsub, P);
}

constexpr int PQ_THREADS = 512;

// pref[q][p] = positions (padded list lengths) of probes 0..p-1 of query q,
// pref[q][nprobe] = the total: the concatenation the IVF_PQ scan splits.
__global__ __launch_bounds__(256) void probe_prefix_kernel(const int64_t *__restrict__ probe_l, int nprobe,
                                                           const int64_t *__restrict__ loff,
                                                           int64_t *__restrict__ pref) {
	__shared__ int64_t sc[256];
	__shared__ int64_t carry;
	const int q = blockIdx.x, t = threadIdx.x;
	if (t == 0) carry = 0;
	for (int p0 = 0; p0 < nprobe; p0 += 256) {
		const int p = p0 + t;
		int64_t len = 0;
		if (p < nprobe) {
			const int64_t l = probe_l[(int64_t)q * nprobe + p];
			if (l >= 0) len = loff[l + 1] - loff[l];
		}
		__syncthreads();
		sc[t] = len;
		__syncthreads();
		for (int off = 1; off < 256; off <<= 1) {
			const int64_t v = t >= off ? sc[t - off] : 0;
			__syncthreads();
			sc[t] += v;
			__syncthreads();
		}
		if (p < nprobe) pref[(int64_t)q * (nprobe + 1) + p] = carry + sc[t] - len;
		__syncthreads();
		if (t == 255) carry += sc[255];
	}
	__syncthreads();
	if (t == 0) pref[(int64_t)q * (nprobe + 1) + nprobe] = carry;
}

void launch_probe_prefix(const int64_t *probe_l, int nq, int nprobe, const int64_t *loff, int64_t *pref,
                         hipStream_t st) {
	probe_prefix_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(probe_l, nprobe, loff, pref);
}

// ADCs of PQ_R rows at list positions pos[i] (canonical f32 order: d0 + tau,
// then j = 0..m-1), the PQ_R chains interleaved so their LDS lookups overlap
constexpr int PQ_R = 4;
__device__ __forceinline__ void pq_adc_r(const uint8_t *__restrict__ lcodes, int nch, int m, const int64_t (&pos)[PQ_R],
                                         const float *lut, float d0, const float *__restrict__ ltau,
                                         float (&acc)[PQ_R]) {
	const uint8_t *cp[PQ_R];
#pragma unroll
	for (int i = 0; i < PQ_R; ++i) {
		cp[i] = lcodes + pos[i] * nch * 16;
		acc[i] = ltau ? d0 + ltau[pos[i]] : d0;
	}
	for (int ch = 0; ch < nch; ++ch) {
		uint32_t wd[PQ_R][4];
#pragma unroll
		for (int i = 0; i < PQ_R; ++i) {
			const uint4 w = *reinterpret_cast<const uint4 *>(cp[i] + ch * 16);
			wd[i][0] = w.x;
			wd[i][1] = w.y;
			wd[i][2] = w.z;
			wd[i][3] = w.w;
		}
#pragma unroll
		for (int u = 0; u < 16; ++u) {
			const int j = ch * 16 + u;
			if (j < m) {
#pragma unroll
				for (int i = 0; i < PQ_R; ++i) acc[i] = acc[i] + lut[j * PQ_K + ((wd[i][u >> 2] >> (8 * (u & 3))) & 255u)];
			}
		}
	}
}

// IVF_PQ scan, query-major: workgroup (s, q) takes segment s of S of the
// concatenation of query q's probed lists (balanced whatever the list sizes),
// builds the query's LUT -2 P[q] (L2 / cosine; -P[q] for dot) in LDS ONCE (the
// list term T[l][j][c_j] is folded into the per-row tau at index time), and
// keeps ONE streaming top-kk over its whole segment (the threshold tightens
// across lists).  Rows stream as 16-B code pieces of the row-major list
// layout, PQ_R rows per thread per round.
__global__ __launch_bounds__(PQ_THREADS) void pq_query_scan_kernel(
    const uint8_t *__restrict__ lcodes, int m, int mp, const int64_t *__restrict__ loff,
    const uint32_t *__restrict__ lslot, const float *__restrict__ rowaux_f, int nprobe,
    const int64_t *__restrict__ probe_l, const float *__restrict__ probe_d, const float *__restrict__ ltau,
    const float *__restrict__ P, const int64_t *__restrict__ pref, int S, int kk, uint64_t *__restrict__ out) {
	__shared__ float lut[PQ_MAX_M * PQ_K];
	__shared__ uint64_t buf[IVF_TOPK_CAP];
	__shared__ int cnt;
	__shared__ uint64_t thr;
	__shared__ int sp0;
	const int s = blockIdx.x, q = blockIdx.y, t = threadIdx.x;
	const int64_t *pr = pref + (int64_t)q * (nprobe + 1);
	const int64_t R = pr[nprobe];
	const int64_t a = R * s / S, b = R * (s + 1) / S;
	const int nch = mp >> 4;
	const int nlut = m * PQ_K;
	TopK tk{buf, &cnt, &thr, kk};
	tk.reset();
	if (a < b) {
		const float *Pq = P + (int64_t)q * nlut;
		const float sP = ltau ? -2.0f : -1.0f;  // exact scaling
		for (int e = t; e < nlut; e += PQ_THREADS) lut[e] = sP * Pq[e];
		if (t == 0) {  // last probe starting at or before a
			int lo = 0, hi = nprobe - 1;
			while (lo < hi) {
				const int mid = (lo + hi + 1) >> 1;
				if (pr[mid] <= a) lo = mid;
				else hi = mid - 1;
			}
			sp0 = lo;
		}
		__syncthreads();
		for (int p = sp0; p < nprobe && pr[p] < b; ++p) {
			const int64_t g0 = max(a, pr[p]), g1 = min(b, pr[p + 1]);
			if (g0 >= g1) continue;
			const int64_t l = probe_l[(int64_t)q * nprobe + p];
			const float d0 = probe_d[(int64_t)q * nprobe + p];
			const int64_t end = loff[l] + (g1 - pr[p]);
			for (int64_t r0 = loff[l] + (g0 - pr[p]); r0 < end; r0 += PQ_R * PQ_THREADS) {
				int64_t pos[PQ_R];
				uint32_t sl[PQ_R];
#pragma unroll
				for (int i = 0; i < PQ_R; ++i) {
					const int64_t ps = r0 + i * PQ_THREADS + t;
					sl[i] = ps < end ? lslot[ps] : SLOT_NONE;
					pos[i] = ps < end ? ps : end - 1;  // in bounds; the key is dropped
				}
				float da[PQ_R];
				pq_adc_r(lcodes, nch, m, pos, lut, d0, ltau, da);
				// liveness (a random 4-B read of the row aux) only for keys that
				// pass the current threshold: most rows stop at the compare
				const uint64_t th = *tk.thr;
#pragma unroll
				for (int i = 0; i < PQ_R; ++i) {
					const uint64_t key = sl[i] != SLOT_NONE ? key64(da[i], sl[i]) : KEY64_NONE;
					const bool ok = sl[i] != SLOT_NONE && key < th && slot_alive(rowaux_f, sl[i]);
					tk.offer(key, ok);
				}
			}
		}
	}
	const int nout = tk.finish();
	uint64_t *o = out + ((int64_t)q * S + s) * kk;
	for (int i = t; i < kk; i += PQ_THREADS) o[i] = i < nout ? buf[i] : KEY64_NONE;
}

int pq_segments(int nq) { return std::max(1, std::min(32, (4096 + nq - 1) / std::max(nq, 1))); }

void launch_pq_query_scan(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                          const float *rowaux_f, int nq, int nprobe, const int64_t *probe_l, const float *probe_d,
                          const float *ltau, const float *P, const int64_t *pref, int S, int kk, uint64_t *out,
                          hipStream_t st) {
	pq_query_scan_kernel<<<dim3((unsigned)S, (unsigned)nq), PQ_THREADS, 0, st>>>(
	    lcodes, m, mp, loff, lslot, rowaux_f, nprobe, probe_l, probe_d, ltau, P, pref, S, kk, out);
}

// ---------------------------------------------------------------------------
// IVF_PQ fast scan (list-major, 8-bit LUT, FQ_G queries per lookup)
// ---------------------------------------------------------------------------
// OCP e4m3fn round-to-nearest-even of v, |v| <= 448 (3 mantissa bits, minimum
// normal exponent -6, subnormal step 2^-9); the division by the power-of-two
// step and the rint are exact, so any IEEE implementation (oracle/ivf.py
// e4m3_round) gives the same value.
__device__ __forceinline__ float e4m3_round(float v) {
	const float a = fabsf(v);
	if (!(a > 0.0f)) return v;
	int e;
	(void)frexpf(a, &e);  // a = f 2^e, f in [0.5, 1): exponent e - 1
	const int E = e - 1 > -6 ? e - 1 : -6;
	const float ulp = ldexpf(1.0f, E - 3);
	const float r = fminf(mul_nc(rintf(__fdiv_rn(a, ulp)), ulp), 448.0f);
	return copysignf(r, v);
}

// fp8 queries: q' = e4m3(q / s) * s, s = absmax(q) / 448 (per query, f32)
__global__ __launch_bounds__(256) void pq_query_fp8_kernel(const float *__restrict__ Q, int qld, int dim,
                                                           float *__restrict__ Qo) {
	__shared__ float red[4];
	const int q = blockIdx.x, t = threadIdx.x;
	const float *x = Q + (int64_t)q * qld;
	float mx = 0.0f;
	for (int i = t; i < dim; i += 256) mx = fmaxf(mx, fabsf(x[i]));
	for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
	if ((t & 63) == 0) red[t >> 6] = mx;
	__syncthreads();
	mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
	const float sc = __fdiv_rn(mx, 448.0f);
	float *y = Qo + (int64_t)q * qld;
	for (int i = t; i < qld; i += 256)
		y[i] = (i < dim && sc > 0.0f) ? mul_nc(e4m3_round(__fdiv_rn(x[i], sc)), sc) : 0.0f;
}

void launch_pq_query_fp8(const float *Q, int qld, int nq, int dim, float *Qo, hipStream_t st) {
	pq_query_fp8_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(Q, qld, dim, Qo);
}

// 8-bit LUT of query q: L = sP P[q] (exact scaling), lo_j = min_c L[j][c],
// D = max_j (max_c L[j][c] - lo_j) / 255 (1 if 0), u[j][c] = min(255,
// rint((L[j][c] - lo_j) * (1 / D))), L0 = sum_j lo_j (j ascending).
// ADC(row) = ((d0 + tau) + L0) + D * sum_j u[j][c_j]  (oracle/ivf.py pq_lut_u8)
// Layout of lut8[q]: [j][c] (m x 256 bytes), or, for the bank-conflict-free
// fast scan (wb = m / 32 > 0), its LUT-build order [x][c >> 4][b][c & 15]
// with j = 4 wb (b >> 2) + 4 x + (b & 3): the 32 lanes that fill one LDS
// store group read 512 contiguous bytes
__host__ __device__ __forceinline__ int lut8_index(int wb, int j, int c) {
	if (wb == 0) return j * PQ_K + c;
	const int pp = j / (4 * wb), rem = j - pp * 4 * wb, x = rem >> 2, b = 4 * pp + (rem & 3);
	return ((x * 16 + (c >> 4)) * 32 + b) * 16 + (c & 15);
}
__global__ __launch_bounds__(256) void pq_lut_u8_kernel(const float *__restrict__ P, int m, float sP, int wb,
                                                        uint8_t *__restrict__ lut8, float2 *__restrict__ qpar) {
	__shared__ float lo[PQ_MAX_M], sp[PQ_MAX_M];
	__shared__ float dsh;
	const int q = blockIdx.x, t = threadIdx.x;
	const float *Pq = P + (int64_t)q * m * PQ_K;
	// per sub-space j (wave w takes j = w, w + 4, ...): min / max over its 256
	// entries, 4 per lane and a wave reduction (one serial 256-read loop per j was
	// ~29 us for C5)
	{
		const int w = t >> 6, lane = t & 63;
		for (int j = w; j < m; j += 4) {
			float a = F_INF, b = -F_INF;
#pragma unroll
			for (int i = 0; i < 4; ++i) {
				const float v = mul_nc(sP, Pq[j * PQ_K + lane + 64 * i]);
				a = fminf(a, v);
				b = fmaxf(b, v);
			}
#pragma unroll
			for (int o = 32; o > 0; o >>= 1) {
				a = fminf(a, __shfl_xor(a, o, 64));
				b = fmaxf(b, __shfl_xor(b, o, 64));
			}
			if (lane == 0) {
				lo[j] = a;
				sp[j] = sub_nc(b, a);
			}
		}
	}
	__syncthreads();
	if (t == 0) {
		float mxs = 0.0f, l0 = 0.0f;
		for (int j = 0; j < m; ++j) {
			mxs = fmaxf(mxs, sp[j]);
			l0 = add_nc(l0, lo[j]);
		}
		const float D = mxs > 0.0f ? __fdiv_rn(mxs, 255.0f) : 1.0f;
		dsh = D;
		qpar[q] = make_float2(D, l0);
	}
	__syncthreads();
	const float inv = __fdiv_rn(1.0f, dsh);
	uint8_t *o = lut8 + (int64_t)q * m * PQ_K;
	// 16-byte output chunks: chunk d holds codes c0 .. c0 + 15 of sub-space j
	// (lut8_index(wb, j, c0 + i) = 16 d + i), from four float4 reads of P
#pragma unroll 2
	for (int d = t; d < m * 16; d += 256) {
		int j, c0;
		if (wb) {
			const int b = d & 31, cp = (d >> 5) & 15, x = d >> 9;
			j = 4 * wb * (b >> 2) + 4 * x + (b & 3);
			c0 = cp * 16;
		} else {
			j = d >> 4;
			c0 = (d & 15) * 16;
		}
		const float4 *src = reinterpret_cast<const float4 *>(Pq + j * PQ_K + c0);
		const float l = lo[j];
		uint32_t w[4];
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const float4 f = src[i];
			const float fv[4] = {f.x, f.y, f.z, f.w};
			uint32_t word = 0u;
#pragma unroll
			for (int k2 = 0; k2 < 4; ++k2) {
				const float u = fminf(rintf(mul_nc(sub_nc(mul_nc(sP, fv[k2]), l), inv)), 255.0f);
				word |= (uint32_t)u << (8 * k2);
			}
			w[i] = word;
		}
		reinterpret_cast<uint4 *>(o)[d] = make_uint4(w[0], w[1], w[2], w[3]);
	}
}

static int pq_bank_w(int m);
void launch_pq_lut_u8(const float *P, int nq, int m, float sP, uint8_t *lut8, float2 *qpar, hipStream_t st) {
	pq_lut_u8_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(P, m, sP, pq_bank_w(m), lut8, qpar);
}

// The fast scan's per-query tables in one launch (round 6; was pq_query_fp8 +
// pq_P + pq_lut_u8, three launches and two 25-MB round trips of P through
// HBM at C5): one workgroup per query keeps its query row (fp8-rounded when
// asked, pq_query_fp8_kernel's arithmetic) and its m x 256 f32 table P in LDS,
// then takes the per-sub-space ranges, D, L0 and the 8-bit entries from LDS
// (pq_lut_u8_kernel's arithmetic).  The codebook comes from L2 (every query's
// workgroup reads the same m x 256 x dsub floats).  Bit-identical to the three
// launches.
constexpr int PQL_THREADS = 1024, PQL_W = PQL_THREADS / 64;
constexpr int PQL_PS = PQ_K + 1;  // P row stride in LDS: the quantize reads of 32 sub-spaces hit 32 banks
__global__ __launch_bounds__(PQL_THREADS) void pq_lut_fused_kernel(const float *__restrict__ Q, int qld, int dim,
                                                                   int fp8, const float *__restrict__ cb, int m,
                                                                   int dsub, float sP, int wb,
                                                                   uint8_t *__restrict__ lut8,
                                                                   float2 *__restrict__ qpar) {
	extern __shared__ __attribute__((aligned(16))) float pql_smem[];
	float *Ps = pql_smem;                  // [m][PQL_PS]
	float *xq = pql_smem + m * PQL_PS;     // [dim]
	__shared__ float lo[PQ_MAX_M], sp[PQ_MAX_M], red[PQL_W];
	__shared__ float dsh;
	const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
	const float *x = Q + (int64_t)q * qld;
	float sc = 0.0f;
	if (fp8) {
		float mx = 0.0f;
		for (int i = t; i < dim; i += PQL_THREADS) mx = fmaxf(mx, fabsf(x[i]));
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
		if (lane == 0) red[w] = mx;
		__syncthreads();
		mx = red[0];
#pragma unroll
		for (int i = 1; i < PQL_W; ++i) mx = fmaxf(mx, red[i]);
		sc = __fdiv_rn(mx, 448.0f);
	}
	for (int i = t; i < dim; i += PQL_THREADS)
		xq[i] = !fp8 ? x[i] : (sc > 0.0f ? mul_nc(e4m3_round(__fdiv_rn(x[i], sc)), sc) : 0.0f);
	__syncthreads();
	// P[j][c] = sum_t x_{j,t} y_{j,c,t} (t ascending, no contraction): thread
	// (c = t & 255, j = t >> 8, +4, ...); a codebook row is dsub / 4 16-B loads,
	// two sub-spaces' rows requested before their sums
	{
		const int c = t & (PQ_K - 1);
		constexpr int JS = PQL_THREADS / PQ_K;
		if (dsub == 8) {
			for (int j0 = t >> 8; j0 < m; j0 += 2 * JS) {
				const int j1 = j0 + JS;
				const float4 *p0 = reinterpret_cast<const float4 *>(cb + ((int64_t)j0 * PQ_K + c) * 8);
				const float4 *p1 = reinterpret_cast<const float4 *>(cb + ((int64_t)(j1 < m ? j1 : j0) * PQ_K + c) * 8);
				const float4 a0 = p0[0], a1 = p0[1], b0 = p1[0], b1 = p1[1];
				const float ya[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
				const float yb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
				float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
				for (int u = 0; u < 8; ++u) {
					s0 = add_nc(s0, mul_nc(xq[j0 * 8 + u], ya[u]));
					s1 = add_nc(s1, mul_nc(xq[(j1 < m ? j1 : j0) * 8 + u], yb[u]));
				}
				Ps[j0 * PQL_PS + c] = s0;
				if (j1 < m) Ps[j1 * PQL_PS + c] = s1;
			}
		} else {
			for (int j = t >> 8; j < m; j += JS) {
				const float *y = cb + ((int64_t)j * PQ_K + c) * dsub;
				float a = 0.0f;
				for (int u = 0; u < dsub; ++u) a = add_nc(a, mul_nc(xq[j * dsub + u], y[u]));
				Ps[j * PQL_PS + c] = a;
			}
		}
	}
	__syncthreads();
	// per sub-space: min / max of sP P over its 256 entries (wave w: j = w, w + 16, ...)
	for (int j = w; j < m; j += PQL_W) {
		float a = F_INF, b = -F_INF;
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			const float v = mul_nc(sP, Ps[j * PQL_PS + lane + 64 * i]);
			a = fminf(a, v);
			b = fmaxf(b, v);
		}
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) {
			a = fminf(a, __shfl_xor(a, o, 64));
			b = fmaxf(b, __shfl_xor(b, o, 64));
		}
		if (lane == 0) {
			lo[j] = a;
			sp[j] = sub_nc(b, a);
		}
	}
	__syncthreads();
	if (t == 0) {
		float mxs = 0.0f, l0 = 0.0f;
		for (int j = 0; j < m; ++j) {
			mxs = fmaxf(mxs, sp[j]);
			l0 = add_nc(l0, lo[j]);
		}
		const float D = mxs > 0.0f ? __fdiv_rn(mxs, 255.0f) : 1.0f;
		dsh = D;
		qpar[q] = make_float2(D, l0);
	}
	__syncthreads();
	const float inv = __fdiv_rn(1.0f, dsh);
	uint8_t *o = lut8 + (int64_t)q * m * PQ_K;
	for (int d = t; d < m * 16; d += PQL_THREADS) {
		int j, c0;
		if (wb) {
			const int b = d & 31, cp = (d >> 5) & 15, xx = d >> 9;
			j = 4 * wb * (b >> 2) + 4 * xx + (b & 3);
			c0 = cp * 16;
		} else {
			j = d >> 4;
			c0 = (d & 15) * 16;
		}
		const float *src = Ps + j * PQL_PS + c0;
		const float l = lo[j];
		uint32_t wd[4];
#pragma unroll
		for (int i = 0; i < 4; ++i) {
			uint32_t word = 0u;
#pragma unroll
			for (int k2 = 0; k2 < 4; ++k2) {
				const float u = fminf(rintf(mul_nc(sub_nc(mul_nc(sP, src[4 * i + k2]), l), inv)), 255.0f);
				word |= (uint32_t)u << (8 * k2);
			}
			wd[i] = word;
		}
		reinterpret_cast<uint4 *>(o)[d] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
	}
}

bool pq_lut_fused_fits(int m, int dim) { return m <= PQ_MAX_M && (size_t)(m * PQL_PS + dim) * 4 <= 150 * 1024; }

void launch_pq_lut_fused(const float *Q, int qld, int nq, int dim, int fp8, const float *cb, int m, int dsub, float sP,
                         uint8_t *lut8, float2 *qpar, hipStream_t st) {
	const size_t lds = (size_t)(m * PQL_PS + dim) * sizeof(float);
	HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(pq_lut_fused_kernel),
	                           hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));
	pq_lut_fused_kernel<<<dim3((unsigned)nq), PQL_THREADS, lds, st>>>(Q, qld, dim, fp8, cb, m, dsub, sP, pq_bank_w(m),
	                                                                   lut8, qpar);
}

// work items: list l with np_l probing queries -> ceil(np_l / FQ_G) query
// groups x ceil(positions_l / FQ_CHUNK) row chunks; item_off [nlist + 1] =
// exclusive prefix over the XCD-major list order, xbeg [NXCD + 1] = item_off
// at each XCD's first list
__global__ __launch_bounds__(1024) void pq_fast_items_kernel(const int *__restrict__ pstart,
                                                             const int64_t *__restrict__ loff, int nlist,
                                                             int *__restrict__ item_off, int *__restrict__ xbeg) {
	__shared__ int sh[1024];
	const int t = threadIdx.x;
	const int per = (nlist + 1023) / 1024;
	const int a = t * per, b = min(nlist, a + per);
	auto items = [&](int p) {
		const int l = lperm(nlist, p);
		const int np = pstart[l + 1] - pstart[l];
		const int64_t len = loff[l + 1] - loff[l];
		return np > 0 && len > 0 ? ((np + FQ_G - 1) / FQ_G) * (int)((len + FQ_CHUNK - 1) / FQ_CHUNK) : 0;
	};
	int s = 0;
	for (int i = a; i < b; ++i) s += items(i);
	sh[t] = s;
	__syncthreads();
	for (int o = 1; o < 1024; o <<= 1) {
		const int v = t >= o ? sh[t - o] : 0;
		__syncthreads();
		sh[t] += v;
		__syncthreads();
	}
	int run = sh[t] - s;
	for (int i = a; i < b; ++i) {
		item_off[i] = run;
		run += items(i);
	}
	if (t == 1023) item_off[nlist] = sh[1023];
	__syncthreads();
	if (t <= NXCD) {
		int p0 = 0;
		for (int x = 0; x < t; ++x) p0 += xcd_lists(nlist, x);
		xbeg[t] = item_off[min(p0, nlist)];
	}
}

// itab[2 it], itab[2 it + 1] = (list position of the item's first row (lo, hi),
// its rows, list), (the 4 pair ids of the
// item's query group, -1 past the group): an item's whole description in one
// 32-B read (pq_fast_scan_bank_kernel), instead of a binary search over
// item_off and the pair ids behind it (a chain of dependent global reads at
// every item).  One thread per list position.
__global__ __launch_bounds__(256) void pq_fast_table_kernel(const int *__restrict__ pstart,
                                                            const int64_t *__restrict__ loff,
                                                            const int *__restrict__ pairs, int nlist,
                                                            const int *__restrict__ item_off, int4 *__restrict__ itab,
                                                            int cap) {
	const int pos = blockIdx.x * blockDim.x + threadIdx.x;
	if (pos >= nlist) return;
	const int l = lperm(nlist, pos);
	const int np = pstart[l + 1] - pstart[l];
	const int64_t len = loff[l + 1] - loff[l];
	if (np <= 0 || len <= 0) return;
	const int nc = (int)((len + FQ_CHUNK - 1) / FQ_CHUNK), ngr = (np + FQ_G - 1) / FQ_G;
	int it = item_off[pos];
	for (int g = 0; g < ngr; ++g) {
		int id[FQ_G];
		for (int i = 0; i < FQ_G; ++i) id[i] = g * FQ_G + i < np ? pairs[pstart[l] + g * FQ_G + i] : -1;
		for (int ch = 0; ch < nc; ++ch, ++it) {
			if (it >= cap) return;
			const int64_t pos = loff[l] + (int64_t)ch * FQ_CHUNK;
			const int nrow = (int)min<int64_t>(FQ_CHUNK, len - (int64_t)ch * FQ_CHUNK);
			itab[2 * it] = make_int4((int)(uint32_t)pos, (int)(pos >> 32), nrow, l);
			itab[2 * it + 1] = make_int4(id[0], id[1], id[2], id[3]);
		}
	}
}

// Persistent: each workgroup takes work items (one atomic per item, XCD-major).  An item
// = one 8192-position chunk of list l x up to FQ_G queries probing l: their
// 8-bit LUTs interleaved in LDS as u32 [j][c] = (u_0, u_1, u_2, u_3)[j][c], so
// ONE ds_read_b32 per (row, j) serves all FQ_G queries; the four byte lanes
// are summed two at a time in packed 16-bit halves (max 128 x 255 < 2^16).
// Per query a threshold-filtered LDS candidate buffer, sorted and cut to kk
// when it could overflow; its kk-th key is a valid bound for every other item
// of the query (global atomicMin), and the candidates <= the bound go to the
// query's output run (atomic cursor; the final order is by key, so the
// arrival order does not matter).
template <int MT>  // m at compile time (0: runtime m)
__global__ __launch_bounds__(FQ_THREADS) void pq_fast_scan_kernel(
    const uint8_t *__restrict__ lcodes, int m, int mp, const int64_t *__restrict__ loff,
    const uint32_t *__restrict__ lslot, const float *__restrict__ rowaux_f, int nlist, int nprobe,
    const int *__restrict__ pstart, const int *__restrict__ pairs, const int *__restrict__ item_off,
    const int *__restrict__ xbeg, const float *__restrict__ probe_d, const float *__restrict__ ltau,
    const uint8_t *__restrict__ lut8, const float2 *__restrict__ qpar, int kk, int *__restrict__ work,
    unsigned long long *__restrict__ thrq, int *__restrict__ ocnt, uint64_t *__restrict__ out, int ocap) {
	extern __shared__ __attribute__((aligned(16))) uint8_t fq_smem[];
	uint32_t *L = reinterpret_cast<uint32_t *>(fq_smem);                  // [m][256]
	uint64_t *buf = reinterpret_cast<uint64_t *>(fq_smem + (size_t)m * PQ_K * 4);  // [FQ_G][FQ_CAP]
	__shared__ int cnt[FQ_G], qid[FQ_G], item, nlive;
	__shared__ uint64_t thr[FQ_G];
	__shared__ float d0s[FQ_G], dls[FQ_G], l0s[FQ_G];
	const int t = threadIdx.x;
	const int nch = mp >> 4;
	int xc = blockIdx.x & (NXCD - 1), tries = 0;  // (thread 0's claim state: XCD counter, counters exhausted)
#ifdef LHIP_PQ_PROF
	uint64_t pq_acc[PQ_PROF_N] = {0, 0, 0, 0, 0, 0, 0, 0};
	uint64_t pq_t = __builtin_amdgcn_s_memtime();
#endif
	for (;;) {
		PQ_T(0);  // (item claim + loop overhead)
		if (t == 0) {
			int itc = -1;
			while (tries < NXCD) {  // every workgroup ends once all 8 counters ran out
				const int c = atomicAdd(work + xc, 1);
				if (c < xbeg[xc + 1] - xbeg[xc]) {
					itc = xbeg[xc] + c;
					break;
				}
				xc = (xc + 1) & (NXCD - 1);
				++tries;
			}
			item = itc;
		}
		__syncthreads();
		const int it = item;
		if (it < 0) break;
#ifdef LHIP_PQ_PROF
		pq_acc[5] += 1;
#endif
		// list of the item: last position p with item_off[p] <= it (binary search)
		int lo = 0, hi = nlist - 1;
		while (lo < hi) {
			const int mid = (lo + hi + 1) >> 1;
			if (item_off[mid] <= it) lo = mid;
			else hi = mid - 1;
		}
		const int l = lperm(nlist, lo);
		const int64_t p0 = loff[l], len = loff[l + 1] - p0;
		const int nc = (int)((len + FQ_CHUNK - 1) / FQ_CHUNK);
		const int loc = it - item_off[lo], g = loc / nc, ch = loc % nc;
		const int np = pstart[l + 1] - pstart[l];
		const int ng = min(FQ_G, np - g * FQ_G);
		if (t < FQ_G) {
			int q = -1;
			if (t < ng) {
				const int id = pairs[pstart[l] + g * FQ_G + t];
				q = id / nprobe;
				d0s[t] = probe_d[id];
				const float2 qp = qpar[q];
				dls[t] = qp.x;
				l0s[t] = qp.y;
				thr[t] = thrq[q];
			} else {
				thr[t] = 0;
			}
			qid[t] = q;
			cnt[t] = 0;
		}
		__syncthreads();
		// interleaved LUT: u32 [j][c] = bytes (u_0, u_1, u_2, u_3)
#ifndef LHIP_PQ_ABL_NO_LUT
		if constexpr (MT > 0 && (MT * PQ_K / 16) % FQ_THREADS == 0) {
			// 16 codes per lane and query per step, every step's loads in flight at
			// once (the four tables are L2 / MALL reads: one latency per item, not
			// one per step), then 4 x 4 byte transposes into four 16-B LDS stores
			constexpr int NS = MT * PQ_K / 16 / FQ_THREADS;  // steps per thread (m = 96: 3)
			uint4 w[NS][FQ_G];
#pragma unroll
			for (int sI = 0; sI < NS; ++sI)
#pragma unroll
				for (int i = 0; i < FQ_G; ++i)
					w[sI][i] = qid[i] >= 0 ? reinterpret_cast<const uint4 *>(lut8 + (int64_t)qid[i] * MT * PQ_K)[t + sI * FQ_THREADS]
					                       : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
			for (int sI = 0; sI < NS; ++sI) {
				const int e16 = t + sI * FQ_THREADS;
#pragma unroll
				for (int sub = 0; sub < 4; ++sub) {
					const uint32_t w0 = sub == 0 ? w[sI][0].x : sub == 1 ? w[sI][0].y : sub == 2 ? w[sI][0].z : w[sI][0].w;
					const uint32_t w1 = sub == 0 ? w[sI][1].x : sub == 1 ? w[sI][1].y : sub == 2 ? w[sI][1].z : w[sI][1].w;
					const uint32_t w2 = sub == 0 ? w[sI][2].x : sub == 1 ? w[sI][2].y : sub == 2 ? w[sI][2].z : w[sI][2].w;
					const uint32_t w3 = sub == 0 ? w[sI][3].x : sub == 1 ? w[sI][3].y : sub == 2 ? w[sI][3].z : w[sI][3].w;
					const uint32_t a01 = __builtin_amdgcn_perm(w1, w0, 0x05010400u);
					const uint32_t a23 = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
					const uint32_t b01 = __builtin_amdgcn_perm(w1, w0, 0x07030602u);
					const uint32_t b23 = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
					uint4 o;
					o.x = __builtin_amdgcn_perm(a23, a01, 0x05040100u);
					o.y = __builtin_amdgcn_perm(a23, a01, 0x07060302u);
					o.z = __builtin_amdgcn_perm(b23, b01, 0x05040100u);
					o.w = __builtin_amdgcn_perm(b23, b01, 0x07060302u);
					reinterpret_cast<uint4 *>(L)[4 * e16 + sub] = o;
				}
			}
		} else {
			const int ne = m * PQ_K / 4;  // 4 codes per step
			for (int e = t; e < ne; e += FQ_THREADS) {
				uint32_t w[FQ_G];
#pragma unroll
				for (int i = 0; i < FQ_G; ++i)
					w[i] = qid[i] >= 0 ? reinterpret_cast<const uint32_t *>(lut8 + (int64_t)qid[i] * m * PQ_K)[e] : 0u;
				// transpose 4 x 4 bytes: out c = byte c of each w[i]
				const uint32_t a01 = __builtin_amdgcn_perm(w[1], w[0], 0x05010400u);  // w0.b0 w1.b0 w0.b1 w1.b1
				const uint32_t a23 = __builtin_amdgcn_perm(w[3], w[2], 0x05010400u);
				const uint32_t b01 = __builtin_amdgcn_perm(w[1], w[0], 0x07030602u);  // w0.b2 w1.b2 w0.b3 w1.b3
				const uint32_t b23 = __builtin_amdgcn_perm(w[3], w[2], 0x07030602u);
				uint4 o;
				o.x = __builtin_amdgcn_perm(a23, a01, 0x05040100u);  // c0: w0 w1 w2 w3
				o.y = __builtin_amdgcn_perm(a23, a01, 0x07060302u);  // c1
				o.z = __builtin_amdgcn_perm(b23, b01, 0x05040100u);  // c2
				o.w = __builtin_amdgcn_perm(b23, b01, 0x07060302u);  // c3
				reinterpret_cast<uint4 *>(L)[e] = o;
			}
		}
#endif
		__syncthreads();
		PQ_T(1);  // item setup + LUT build
		const int64_t c0 = (int64_t)ch * FQ_CHUNK, c1 = len < c0 + FQ_CHUNK ? len : c0 + FQ_CHUNK;
		// codes of the next round are loaded while the current round is summed
		constexpr int NCH = FQ_MAX_M / 16;
		uint4 cw[NCH];
		uint32_t cslot = SLOT_NONE;
		float ctau = 0.0f;
		auto load_row = [&](int64_t r, uint4 (&w)[NCH], uint32_t &sl, float &ta) __attribute__((always_inline)) {
			sl = SLOT_NONE;
			ta = 0.0f;
			if (r < c1) {
				const int64_t ps = p0 + r;
				sl = lslot[ps];
				if (ltau) ta = ltau[ps];
				const uint8_t *cp = lcodes + ps * mp;
#pragma unroll
				for (int c = 0; c < NCH; ++c)
					if (c < nch) w[c] = *reinterpret_cast<const uint4 *>(cp + c * 16);
			}
		};
		// two code buffers, the loop unrolled twice: round i sums one buffer while
		// round i + 1's codes land in the other (a copy of the prefetched registers
		// at the round's end made every round wait for its own prefetch)
		auto round = [&](const uint4 (&cw)[NCH], uint32_t cslot, float ctau, uint4 (&nw)[NCH], uint32_t &nslot,
		                 float &ntau, int64_t rpre, uint64_t &gprev) __attribute__((always_inline)) {
			// the query's bound from its other items, consumed at the NEXT round's end
			// (gprev): a whole round hides its latency (a global round trip under
			// load is about one round; waiting on it in the same round stalled every
			// round's barrier); a stale read is only a looser bound.  Issued before
			// the prefetch: its wait then leaves the prefetch in flight (vmcnt counts
			// in issue order)
			uint64_t gthr = KEY64_NONE;
			if (t < FQ_G && qid[t] >= 0) gthr = __builtin_nontemporal_load(thrq + qid[t]);
			load_row(rpre, nw, nslot, ntau);
			uint32_t s02 = 0u, s13 = 0u;
#ifdef LHIP_PQ_ABL_NO_LOOKUP
			s02 = cw[0].x ^ cw[1].y ^ cw[2].z ^ cw[3].w ^ cw[4].x ^ cw[5].y;
			s13 = cw[0].y ^ cw[1].z ^ cw[2].w ^ cw[3].x ^ cw[4].y ^ cw[5].z;
			if (false) {
#else
			{
#endif
				// rows past the chunk hold stale codes: summed, never offered
				if constexpr (MT > 0) {
					// m known at compile time: 16 independent LDS reads per code
					// piece, then the sums (no per-j branch, batched lgkm waits)
					// PQ_LB code pieces (16 lookups each) per LDS wait
#ifndef LHIP_PQ_LB
#define LHIP_PQ_LB 1
#endif
					constexpr int NCP = (MT + 15) / 16, LB = LHIP_PQ_LB;
#pragma unroll
					for (int c0 = 0; c0 < NCP; c0 += LB) {
						uint32_t v[LB][16];
#pragma unroll
						for (int cc = 0; cc < LB; ++cc) {
							const int c = c0 + cc;
							if (c < NCP) {
								const uint32_t wd[4] = {cw[c].x, cw[c].y, cw[c].z, cw[c].w};
#pragma unroll
								for (int u = 0; u < 16; ++u) {
									const int j = c * 16 + u;
									if (j < MT) v[cc][u] = L[j * PQ_K + ((wd[u >> 2] >> (8 * (u & 3))) & 255u)];
								}
							}
						}
#pragma unroll
						for (int cc = 0; cc < LB; ++cc)
#pragma unroll
							for (int u = 0; u < 16; ++u) {
								if (c0 + cc < NCP && (c0 + cc) * 16 + u < MT) {
									s02 += v[cc][u] & 0x00FF00FFu;
									s13 += __builtin_amdgcn_perm(0u, v[cc][u], 0x0c030c01u);  // bytes 1, 3 -> 0, 2
								}
							}
					}
				} else {
#pragma unroll
					for (int c = 0; c < NCH; ++c) {
						if (c < nch) {
							const uint32_t wd[4] = {cw[c].x, cw[c].y, cw[c].z, cw[c].w};
#pragma unroll
							for (int u = 0; u < 16; ++u) {
								const int j = c * 16 + u;
								if (j < m) {
									const uint32_t code = (wd[u >> 2] >> (8 * (u & 3))) & 255u;
									const uint32_t v = L[j * PQ_K + code];
									s02 += v & 0x00FF00FFu;
									s13 += (v >> 8) & 0x00FF00FFu;
								}
							}
						}
					}
				}
			}
			const uint32_t S[FQ_G] = {s02 & 0xFFFFu, s13 & 0xFFFFu, s02 >> 16, s13 >> 16};
			uint64_t key[FQ_G];
			bool pass[FQ_G], any = false;
#pragma unroll
			for (int i = 0; i < FQ_G; ++i) {
				float a = ltau ? add_nc(d0s[i], ctau) : d0s[i];
				a = add_nc(a, l0s[i]);
				a = add_nc(a, mul_nc(dls[i], (float)S[i]));
				key[i] = key64(a, cslot);
				pass[i] = cslot != SLOT_NONE && qid[i] >= 0 && key[i] <= thr[i];
#ifdef LHIP_PQ_ABL_NO_CAND
				pass[i] = pass[i] && key[i] == 0;
#endif
				any |= pass[i];
			}
			// (row liveness: checked at the cut and the flush, fq_cut)
			if (any) {
#pragma unroll
				for (int i = 0; i < FQ_G; ++i)
					if (pass[i]) {
						const int p = atomicAdd(&cnt[i], 1);
						buf[i * FQ_CAP + p] = key[i];
					}
			}
			__syncthreads();
			PQ_T(2);  // row round
			for (int i = 0; i < FQ_G; ++i) {
				if (cnt[i] > FQ_CAP - FQ_THREADS) {  // the next round could overflow: sort, keep kk
#ifdef LHIP_PQ_PROF
					pq_acc[6] += 1;
#endif
					fq_cut(buf + i * FQ_CAP, cnt[i], thr[i], qid[i], kk, rowaux_f, thrq, nlive);
				}
			}
			if (t < FQ_G && gprev < thr[t]) thr[t] = gprev;
			gprev = gthr;
			__syncthreads();
			PQ_T(3);  // candidate sorts
		};
		// three code buffers: round i sums one while rounds i + 1 and i + 2 land in the
		// others (two rounds of codes in flight per thread: ~96 KiB per CU)
		uint4 cwB[NCH], cwC[NCH];
		uint32_t cslotB = SLOT_NONE, cslotC = SLOT_NONE;
		float ctauB = 0.0f, ctauC = 0.0f;
		uint64_t gprev = KEY64_NONE;
		load_row(c0 + t, cw, cslot, ctau);
		load_row(c0 + FQ_THREADS + t, cwB, cslotB, ctauB);
		for (int64_t r0 = c0; r0 < c1; r0 += 3 * FQ_THREADS) {
			round(cw, cslot, ctau, cwC, cslotC, ctauC, r0 + 2 * FQ_THREADS + t, gprev);
			if (r0 + FQ_THREADS >= c1) break;
			round(cwB, cslotB, ctauB, cw, cslot, ctau, r0 + 3 * FQ_THREADS + t, gprev);
			if (r0 + 2 * FQ_THREADS >= c1) break;
			round(cwC, cslotC, ctauC, cwB, cslotB, ctauB, r0 + 4 * FQ_THREADS + t, gprev);
		}
		// flush: the item's keys within its final bound (entries appended before
		// the bound tightened may lie above it)
#ifdef LHIP_PQ_PROF
		for (int i = 0; i < FQ_G; ++i) pq_acc[7] += qid[i] >= 0 ? (uint64_t)cnt[i] : 0;
#endif
		for (int i = 0; i < FQ_G; ++i) {
			const int q = qid[i];
			if (q < 0) continue;
			const uint64_t th = thr[i];
			const uint64_t *b = buf + i * FQ_CAP;
			for (int e = t; e < cnt[i]; e += FQ_THREADS) {
				const uint64_t key = b[e];
				if (key <= th && slot_alive(rowaux_f, (uint32_t)key)) {
					const int p = atomicAdd(ocnt + q, 1);
					if (p < ocap) out[(int64_t)q * ocap + p] = key;
				}
			}
		}
		__syncthreads();
		PQ_T(4);  // flush
	}
#ifdef LHIP_PQ_PROF
	if (t == 0 && blockIdx.x < PQ_PROF_WG)
		for (int i = 0; i < PQ_PROF_N; ++i) g_pq_prof[blockIdx.x * PQ_PROF_N + i] = pq_acc[i];
#endif
}

// The fast scan for m = 32 W (W = 1..3; C5's m = 96 is W = 3), free of LDS
// bank conflicts.  pq_fast_scan_kernel gives each lane one row: the 32 lanes
// of a ds_read_b32 group look up 32 random codes of one table, and the bank
// of a [j][c] entry is c mod 32, so a lookup costs ~3.5 LDS cycles per group
// instead of 1.  Here 8 lanes share a row: lane p holds the 4W codes of
// subspaces [4W p, 4W p + 4W) as W words, and the table of subspace
// j = 4W p + 4x + y (word x, byte y) lives entirely in bank 4p + y.  At
// sub-step s the lane of row r (r = 0..3 of its 32-lane group) looks up byte
// y = (s + r) & 3 of word x, so the group's 32 lanes (4 rows x 8 parts) read
// 32 distinct banks.  The lane builds the entry address from its code byte in
// one v_perm (byte 1 = the code, byte 0 = its bank offset: 256-B code rows)
// for x < 2; the third word's tables sit in a compact region with 128-B code
// rows (bfe + shift-add).  A row's 8 partial sums meet by DPP (3 steps), and
// lane p < 4 keys the row for query p of the item.  Items, LUT values, keys,
// bounds and outputs are pq_fast_scan_kernel's (same integers summed: the
// order of the sums is free), so the results are identical.
// 1024 threads (16 waves: four per SIMD, for the VALU issue and the LDS / HBM
// latencies; one workgroup per CU holds the 128 KiB of LUT and buffers), four
// row steps per lane and round, the next round's rows in flight.  Codes, slots
// and row terms come by buffer loads from per-item resources: the whole
// per-lane part of an address is set once per item, the round and step parts
// are scalar offsets, and rows past the chunk read 0 (out of range).
constexpr int FB_THREADS = 1024;
constexpr int FB_META_BYTES = 192;
constexpr uint32_t FB_RSRC3 = 0x00020000u;  // gfx9 buffer descriptor word 3 (raw bytes, range checked)
// cache policy of the row streams (read once): nt (aux 2) keeps the L2 for the
// 4 x 24 KiB of LUT bytes every item re-reads
#ifndef LHIP_FB_AUX
#define LHIP_FB_AUX 2
#endif
constexpr int FB_AUX = LHIP_FB_AUX;
// LUT entries by absolute LDS address (the kernel has no static LDS, so its
// dynamic allocation starts at address 0): the constant part of an entry's
// address then folds into the ds immediate instead of a per-lookup add
__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) {
	return *(const __attribute__((address_space(3))) uint32_t *)(size_t)a;
}
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) {
	*(__attribute__((address_space(3))) uint32_t *)(size_t)a = v;
}
// store at base + a compile-time byte offset (the offset folds into the
// ds_write immediate: one address register for a thread's 16 LUT stores)
template <uint32_t OFF>
__device__ __forceinline__ void lds_st32o(uint32_t base, uint32_t v) {
	*(__attribute__((address_space(3))) uint32_t *)((__attribute__((address_space(3))) uint8_t *)(size_t)base + OFF) = v;
}
// threadIdx.x through an opaque copy: lane quantities derived from it inside
// the item loop are recomputed per item (a few VALU ops) instead of hoisted
// out of it, where their long live ranges spilled at m = 96 (21 VGPRs, 88 B of
// scratch reloaded at every item start, round 5)
__device__ __forceinline__ int opaque_tid() {
	int v = (int)threadIdx.x;
	asm volatile("" : "+v"(v));
	return v;
}
#ifndef LHIP_FB_ROWS_FIRST
#define LHIP_FB_ROWS_FIRST 0  // 1: round 0's rows requested before the LUT reads (round 5; 0 measured 1.6 % faster, r06o)
#endif
#ifndef LHIP_FB_L2PRE
#define LHIP_FB_L2PRE 0  // 1: an item's last round pulls the next item's first codes and LUTs into L2 (measured 2.6 % slower, r06u)
#endif
constexpr int FB_RS = 4;                            // row steps per lane and round
constexpr int FB_ROWS = FB_THREADS / 8 * FB_RS;     // rows per round (512)
template <int W>
__global__ __launch_bounds__(FB_THREADS) void pq_fast_scan_bank_kernel(
    const uint8_t *__restrict__ lcodes, const int64_t *__restrict__ loff, const uint32_t *__restrict__ lslot,
    const float *__restrict__ rowaux_f, int nlist, int nprobe, const int *__restrict__ pstart,
    const int *__restrict__ pairs, const int *__restrict__ item_off, const int *__restrict__ xbeg,
    const float *__restrict__ probe_d, const float *__restrict__ ltau, const uint8_t *__restrict__ lut8,
    const float2 *__restrict__ qpar, int kk, int *__restrict__ work, unsigned long long *__restrict__ thrq,
    int *__restrict__ ocnt, uint64_t *__restrict__ out, int ocap, const int4 *__restrict__ itab) {
	constexpr int MT = 32 * W;
	constexpr int NPERM = W >= 2 ? 2 : 0, NCOMP = W - NPERM;
	constexpr int PBASE = NCOMP * 32768;  // the v_perm region (words 0, 1) after the compact one
	// no static LDS (see lds_ld32); FB_META_BYTES of per-item state follow the candidate buffers
	extern __shared__ __attribute__((aligned(16))) uint8_t fq_smem[];
	uint64_t *buf = reinterpret_cast<uint64_t *>(fq_smem + MT * PQ_K * 4);  // [FQ_G][FQ_CAP]
	uint64_t *thr = buf + FQ_G * FQ_CAP;
	int *cnt = reinterpret_cast<int *>(thr + FQ_G), *qid = cnt + FQ_G;
	float *d0s = reinterpret_cast<float *>(qid + FQ_G), *dls = d0s + FQ_G, *l0s = dls + FQ_G;
	int &item = *reinterpret_cast<int *>(l0s + FQ_G), &nlive = (&item)[1];
	int4 *nent = reinterpret_cast<int4 *>(l0s + FQ_G + 4);  // the item's itab entry
#if LHIP_FB_L2PRE
	int4 *nnext = nent + 2;  // the next item's itab entry, published in round 1
	static_assert(FB_META_BYTES >= 192, "per-item LDS state");
#endif
	const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
	const int p = lane & 7, rw = lane >> 3, r = rw & 3, pq = p & 3;
	// per sub-step s (code byte y = (s + r) & 3, bank b = 4p + y): byte s of lb4 /
	// lb8 is 4b / 8b, and ysel[s] makes v_perm(lb, word, ysel[s]) = (code << 8) | byte s
	// of lb: the entry address 256 code + 4b in the v_perm region, and
	// (256 code + 8b) >> 1 = 128 code + 4b in the compact one
	uint32_t ysel[4], lb4 = 0u, lb8 = 0u;
#pragma unroll
	for (int s = 0; s < 4; ++s) {
		const uint32_t y = (uint32_t)((s + r) & 3), bk = 4u * (uint32_t)p + y;
		ysel[s] = 0x0c0c0000u | (y << 8) | (4u + (uint32_t)s);
		lb4 |= (4u * bk) << (8 * s);
		lb8 |= (8u * bk) << (8 * s);
	}
	// the lane's row within a round step, and its per-item buffer offsets
	const uint32_t lrow = (uint32_t)((wv << 3) + rw);
	const uint32_t vcode = lrow * MT + 4 * W * p, vrow = lrow * 4;
	int xc = blockIdx.x & (NXCD - 1), tries = 0;  // (thread 0's claim state, as pq_fast_scan_kernel)
#ifdef LHIP_PQ_PROF
	uint64_t pq_acc[PQ_PROF_N] = {0, 0, 0, 0, 0, 0, 0, 0};
	uint64_t pq_t = __builtin_amdgcn_s_memtime();
#endif
	// thread 0 issues the claim of the NEXT item when an item starts and resolves
	// it in the item's first round, where wave 0 also reads its itab entry (a
	// scalar read): an item starts with one global round trip (its LUT) instead
	// of three (claim, entry, LUT)
	auto claim = [&]() -> int {
		int itc = -1;
		while (tries < NXCD) {
			const int c = atomicAdd(work + xc, 1);
			if (c < xbeg[xc + 1] - xbeg[xc]) {
				itc = xbeg[xc] + c;
				break;
			}
			xc = (xc + 1) & (NXCD - 1);
			++tries;
		}
		return itc;
	};
	if (t == 0) {
		const int c = claim();
		item = c;
		if (c >= 0) {
			nent[0] = itab[2 * c];
			nent[1] = itab[2 * c + 1];
		}
	}
	__syncthreads();
	// (LHIP_FB_L2PRE) the L2 prefetch's dword, consumed one item later so that no
	// wait for it lands in the item that issued it
	uint32_t pf_v = 0u;
	for (;;) {
		PQ_T(0);
		const int it = item;
		if (it < 0) break;
#ifdef LHIP_PQ_PROF
		pq_acc[5] += 1;
#endif
		const int4 e0 = nent[0], e1 = nent[1];
		// the next item: thread 0 issues its claim in round 0 after the row
		// prefetch and resolves it at the round's end; wave 0 then reads its entry
		// (scalar) and stores it at this item's flush.  No wait on a global
		// atomic or entry sits between two items.
		int pend = 0;
		int4 ne0 = make_int4(0, 0, 0, 0), ne1 = ne0;
		const int64_t pos0 = (int64_t)(((uint64_t)(uint32_t)e0.y << 32) | (uint32_t)e0.x);
		const uint32_t nrow = (uint32_t)e0.z;  // rows of the item, from list position pos0
		const int ids[FQ_G] = {e1.x, e1.y, e1.z, e1.w};
		int qv[FQ_G];
#pragma unroll
		for (int i = 0; i < FQ_G; ++i) qv[i] = ids[i] >= 0 ? ids[i] / nprobe : -1;
		// the item's rows as buffer resources (rows past the end read 0); round 0's
		// rows are requested with the LUT build's reads, in the same round trip
		const __amdgpu_buffer_rsrc_t rcode =
		    __builtin_amdgcn_make_buffer_rsrc((void *)(lcodes + pos0 * MT), 0, (int)(nrow * MT), FB_RSRC3);
		const __amdgpu_buffer_rsrc_t rslot =
		    __builtin_amdgcn_make_buffer_rsrc((void *)(lslot + pos0), 0, (int)(nrow * 4), FB_RSRC3);
		const __amdgpu_buffer_rsrc_t rtau =
		    __builtin_amdgcn_make_buffer_rsrc((void *)(ltau ? ltau + pos0 : nullptr), 0, ltau ? (int)(nrow * 4) : 0,
		                                      FB_RSRC3);
		struct Rows {
			uint32_t cw[FB_RS][W];
			uint32_t sl[FB_RS];
			float ta[FB_RS];
		};
		// row step k of the round at item row rb: the wave's 8 consecutive rows
		auto load = [&](uint32_t rb, Rows &R) __attribute__((always_inline)) {
#pragma unroll
			for (int k = 0; k < FB_RS; ++k) {
				const uint32_t srow = rb + (uint32_t)(k * (FB_THREADS / 8));  // (scalar)
				if constexpr (W == 3) {
					const auto v = __builtin_amdgcn_raw_buffer_load_b96(rcode, vcode, (int)(srow * MT), FB_AUX);
					R.cw[k][0] = v[0];
					R.cw[k][1] = v[1];
					R.cw[k][2] = v[2];
				} else if constexpr (W == 2) {
					const auto v = __builtin_amdgcn_raw_buffer_load_b64(rcode, vcode, (int)(srow * MT), FB_AUX);
					R.cw[k][0] = v[0];
					R.cw[k][1] = v[1];
				} else {
					R.cw[k][0] = __builtin_amdgcn_raw_buffer_load_b32(rcode, vcode, (int)(srow * MT), FB_AUX);
				}
				const uint32_t sl = __builtin_amdgcn_raw_buffer_load_b32(rslot, vrow, (int)(srow * 4), FB_AUX);
				R.sl[k] = srow + lrow < nrow ? sl : SLOT_NONE;
				R.ta[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rtau, vrow, (int)(srow * 4), FB_AUX));
			}
		};
		Rows RA, RB;
#if LHIP_FB_ROWS_FIRST
		load(0, RA);
#endif
		const int tl = opaque_tid();  // (the item-start block's lane quantities: short live ranges)
		if (tl < FQ_G) {
			const int id = tl == 0 ? e1.x : tl == 1 ? e1.y : tl == 2 ? e1.z : e1.w;
			const int q = id >= 0 ? id / nprobe : -1;
			if (q >= 0) {
				d0s[tl] = probe_d[id];
				const float2 qp = qpar[q];
				dls[tl] = qp.x;
				l0s[tl] = qp.y;
				thr[tl] = thrq[q];
			} else {
				thr[tl] = 0;
			}
			qid[tl] = q;
			cnt[tl] = 0;
		}
		// LUT: thread (word set xs, piece cp of 16 codes, bank b = 4 pp + yy) writes
		// the 16 entries of subspaces 4W pp + 4x + yy for x = xs, xs + 2: the 32 lanes
		// of a store group write 32 distinct banks
		{
			constexpr int NX = (W + 1) / 2;
			const int b = tl & 31, cp = (tl >> 5) & 15, xs = tl >> 9;  // (xs: 0 or 1)
			uint4 w[NX][FQ_G];
#pragma unroll
			for (int xi = 0; xi < NX; ++xi) {
				const int x = xs + 2 * xi;
#pragma unroll
				for (int i = 0; i < FQ_G; ++i)
#ifdef LHIP_FB_ABL_LUTLOAD  // (timing ablation: no LUT reads)
					w[xi][i] = make_uint4((uint32_t)qv[i], (uint32_t)b, (uint32_t)cp, (uint32_t)x);
#else
					w[xi][i] = x < W && qv[i] >= 0 ? reinterpret_cast<const uint4 *>(
					                                      lut8 + (int64_t)qv[i] * MT * PQ_K)[(x * 16 + cp) * 32 + b]
					                                : make_uint4(0u, 0u, 0u, 0u);
#endif
			}
#if !LHIP_FB_ROWS_FIRST
			// round 0's rows behind the LUT reads: the LUT stores wait for the LUT
			// reads only (vmcnt counts in issue order), the rows land meanwhile
			load(0, RA);
#endif
			// x = xs + 2 xi with xs in {0, 1}: xi = 0 is word 0 / 1 (the v_perm region
			// when W >= 2, 256-B code rows), xi = 1 word 2 / 3 (the compact region,
			// 128-B rows): the row stride is a compile-time constant per xi, so a
			// thread's 16 stores of one xi are one base register + ds immediates
			auto store_x = [&](auto xic) __attribute__((always_inline)) {
				constexpr int xi = decltype(xic)::value;
				constexpr uint32_t CS = (xi == 0 && NPERM == 2) ? 256u : 128u;
				const int x = xs + 2 * xi;
				if (x >= W) return;
				const uint32_t dst = x < NPERM ? PBASE + 128 * x + 4 * b : (x - NPERM) * 32768 + 4 * b;
				const uint32_t base = dst + (uint32_t)cp * 16u * CS;
				const uint4 *wx = w[xi];
				auto sub4 = [&](auto subc) __attribute__((always_inline)) {
					constexpr int sub = decltype(subc)::value;
					const uint32_t w0 = sub == 0 ? wx[0].x : sub == 1 ? wx[0].y : sub == 2 ? wx[0].z : wx[0].w;
					const uint32_t w1 = sub == 0 ? wx[1].x : sub == 1 ? wx[1].y : sub == 2 ? wx[1].z : wx[1].w;
					const uint32_t w2 = sub == 0 ? wx[2].x : sub == 1 ? wx[2].y : sub == 2 ? wx[2].z : wx[2].w;
					const uint32_t w3 = sub == 0 ? wx[3].x : sub == 1 ? wx[3].y : sub == 2 ? wx[3].z : wx[3].w;
					const uint32_t a01 = __builtin_amdgcn_perm(w1, w0, 0x05010400u);
					const uint32_t a23 = __builtin_amdgcn_perm(w3, w2, 0x05010400u);
					const uint32_t b01 = __builtin_amdgcn_perm(w1, w0, 0x07030602u);
					const uint32_t b23 = __builtin_amdgcn_perm(w3, w2, 0x07030602u);
					lds_st32o<(sub * 4 + 0) * CS>(base, __builtin_amdgcn_perm(a23, a01, 0x05040100u));
					lds_st32o<(sub * 4 + 1) * CS>(base, __builtin_amdgcn_perm(a23, a01, 0x07060302u));
					lds_st32o<(sub * 4 + 2) * CS>(base, __builtin_amdgcn_perm(b23, b01, 0x05040100u));
					lds_st32o<(sub * 4 + 3) * CS>(base, __builtin_amdgcn_perm(b23, b01, 0x07060302u));
				};
				sub4(std::integral_constant<int, 0>{});
				sub4(std::integral_constant<int, 1>{});
				sub4(std::integral_constant<int, 2>{});
				sub4(std::integral_constant<int, 3>{});
			};
			store_x(std::integral_constant<int, 0>{});
			if constexpr (NX > 1) store_x(std::integral_constant<int, 1>{});
		}
		__syncthreads();
		PQ_T(1);
		const int pql = tl & 3;  // (= pq)
		const int myq = qid[pql];
		const float myd0 = d0s[pql], mydl = dls[pql], myl0 = l0s[pql];
		uint64_t mythr = thr[pql];
		auto round = [&](const Rows &R, Rows &N, uint32_t rpre, uint64_t &gprev, bool first) __attribute__((always_inline)) {
			uint64_t gthr = KEY64_NONE;  // (the query's bound from its other items: as pq_fast_scan_kernel)
			if (t < FQ_G && qid[t] >= 0) gthr = __builtin_nontemporal_load(thrq + qid[t]);
			load(rpre, N);  // (past the item's rows: reads 0, no memory traffic; N stays a fresh value)
#if LHIP_FB_L2PRE
			if (rpre >= nrow && rpre >= 3 * FB_ROWS) {
				// this item's last round (round 2 on; round 1 published the next entry):
				// the next item's first round of codes and its queries' LUTs pulled into
				// L2, one dword per 128-B line with the default cache policy, so that its
				// start reads them from L2 rather than from HBM / the fabric
				const int4 nx = nnext[0], np4 = nnext[1];
				const uint32_t nnr = (uint32_t)__builtin_amdgcn_readfirstlane(nx.z);
				if (nnr > 0) {
					constexpr int CL = FB_ROWS * MT / 128;  // code lines of a round (threads [0, CL))
					if (t < CL) {
						const uint32_t nlo = (uint32_t)__builtin_amdgcn_readfirstlane(nx.x);
						const uint32_t nhi = (uint32_t)__builtin_amdgcn_readfirstlane(nx.y);
						const int64_t p0 = (int64_t)(((uint64_t)nhi << 32) | nlo);
						if ((uint32_t)t * 128u < min(nnr, (uint32_t)FB_ROWS) * (uint32_t)MT)
							pf_v = *reinterpret_cast<const uint32_t *>(lcodes + p0 * MT + (int64_t)t * 128);
					} else {
						constexpr int QL = MT * PQ_K / 128;  // LUT lines of a query
						const int li = t - CL, qi = li / QL;
						const int pid = qi == 0 ? np4.x : qi == 1 ? np4.y : qi == 2 ? np4.z : qi == 3 ? np4.w : -1;
						if (pid >= 0)
							pf_v = *reinterpret_cast<const uint32_t *>(lut8 + (int64_t)(pid / nprobe) * MT * PQ_K +
							                                           (int64_t)(li - qi * QL) * 128);
					}
				}
			}
			if (rpre == 2 * FB_ROWS && t == 0) {  // round 1: wave 0 read the next entry in round 0
				nnext[0] = ne0;
				nnext[1] = ne1;
			}
#endif
			if (first && t == 0 && tries < NXCD) pend = atomicAdd(work + xc, 1);
			// two steps' totals are keyed together: lanes p < 4 key step k, lanes
			// p >= 4 step k + 1, for query p & 3
			uint32_t va[4 * W];
			auto lookups = [&](int k, uint32_t (&v)[4 * W]) __attribute__((always_inline)) {
#pragma unroll
				for (int x = 0; x < W; ++x)
#pragma unroll
					for (int s = 0; s < 4; ++s) {
						uint32_t a;
						if (x < NPERM)
							a = PBASE + 128 * x + __builtin_amdgcn_perm(lb4, R.cw[k][x], ysel[s]);
						else
							a = (x - NPERM) * 32768 + (__builtin_amdgcn_perm(lb8, R.cw[k][x], ysel[s]) >> 1);
						v[4 * x + s] = lds_ld32(a);
					}
			};
			uint64_t key[FB_RS / 2];
			uint32_t pass = 0u;
			uint32_t s02[2], s13[2];
#pragma unroll
			for (int k = 0; k < FB_RS; ++k) {
				lookups(k, va);
				const uint32_t(&v)[4 * W] = va;
				uint32_t e02 = 0u, e13 = 0u;
#pragma unroll
				for (int e = 0; e < 4 * W; ++e) {
					e02 += v[e] & 0x00FF00FFu;
					e13 += __builtin_amdgcn_perm(0u, v[e], 0x0c030c01u);  // bytes 1, 3 -> 0, 2
				}
				s02[k & 1] = e02;
				s13[k & 1] = e13;
				if (k & 1) {
					// the rows' 8 parts: xor 1, xor 2 (quad_perm), then 7 - i (row_half_mirror);
					// four chains interleaved
#pragma unroll
					for (int h = 0; h < 2; ++h) {
						s02[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s02[h], 0xB1, 0xF, 0xF, false);
						s13[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s13[h], 0xB1, 0xF, 0xF, false);
					}
#pragma unroll
					for (int h = 0; h < 2; ++h) {
						s02[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s02[h], 0x4E, 0xF, 0xF, false);
						s13[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s13[h], 0x4E, 0xF, 0xF, false);
					}
#pragma unroll
					for (int h = 0; h < 2; ++h) {
						s02[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s02[h], 0x141, 0xF, 0xF, false);
						s13[h] += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s13[h], 0x141, 0xF, 0xF, false);
					}
					const int h = p >> 2;  // which of the two steps this lane keys
					const int kh = k - 1 + h;
					const uint32_t sv = (p & 1) ? (h ? s13[1] : s13[0]) : (h ? s02[1] : s02[0]);
					const uint32_t S = (p & 2) ? (sv >> 16) : (sv & 0xFFFFu);
					const uint32_t sl = h ? R.sl[k] : R.sl[k - 1];
					const float ta = h ? R.ta[k] : R.ta[k - 1];
					float a = ltau ? add_nc(myd0, ta) : myd0;
					a = add_nc(a, myl0);
					a = add_nc(a, mul_nc(mydl, (float)S));
					key[k >> 1] = key64(a, sl);
					(void)kh;
					if (myq >= 0 && sl != SLOT_NONE && key[k >> 1] <= mythr) pass |= 1u << (k >> 1);  // (liveness: fq_cut, flush)
				}
			}
			// the offers after all row steps: no branch inside the lookup block
			if (pass) {
#pragma unroll
				for (int j = 0; j < FB_RS / 2; ++j)
					if (pass & (1u << j)) {
						const int e = atomicAdd(&cnt[pq], 1);
						buf[pq * FQ_CAP + e] = key[j];
					}
			}
			if (first) {
				int nxt = -1;
				if (t == 0) {
					if (tries < NXCD && pend < xbeg[xc + 1] - xbeg[xc]) {
						nxt = xbeg[xc] + pend;
					} else {
						if (tries < NXCD) {
							xc = (xc + 1) & (NXCD - 1);
							++tries;
						}
						nxt = claim();
					}
					item = nxt;  // (every thread read item before the LUT barrier)
				}
				const int nx = __builtin_amdgcn_readfirstlane(nxt);
				if (wv == 0 && nx >= 0) {
					ne0 = itab[2 * nx];
					ne1 = itab[2 * nx + 1];
				}
			}
			__syncthreads();
			PQ_T(2);
			if (LHIP_FB_L2PRE && first) asm volatile("" ::"v"(pf_v));  // (the previous item's prefetch: long complete)
			for (int i = 0; i < FQ_G; ++i) {
				if (cnt[i] > FQ_CAP - FB_ROWS) {  // the next round could overflow: sort, keep kk
#ifdef LHIP_PQ_PROF
					pq_acc[6] += 1;
#endif
					fq_cut(buf + i * FQ_CAP, cnt[i], thr[i], qid[i], kk, rowaux_f, thrq, nlive);
				}
			}
			if (t < FQ_G && gprev < thr[t]) thr[t] = gprev;
			gprev = gthr;
			__syncthreads();
			mythr = thr[pq];
			PQ_T(3);
		};
		// two row buffers: the next round's rows land while one is summed
		uint64_t gprev = KEY64_NONE;
		for (uint32_t r0 = 0; r0 < nrow; r0 += 2 * FB_ROWS) {
			round(RA, RB, r0 + FB_ROWS, gprev, r0 == 0);
			if (r0 + FB_ROWS >= nrow) break;
			round(RB, RA, r0 + 2 * FB_ROWS, gprev, false);
		}
#ifdef LHIP_PQ_PROF
		for (int i = 0; i < FQ_G; ++i) pq_acc[7] += qid[i] >= 0 ? (uint64_t)cnt[i] : 0;
#endif
		if (t == 0) {  // the next item's entry (read in round 0; nent was read before the LUT barrier)
			nent[0] = ne0;
			nent[1] = ne1;
		}
		for (int i = 0; i < FQ_G; ++i) {
			const int q = qid[i];
			if (q < 0) continue;
			const uint64_t th = thr[i];
			const uint64_t *b = buf + i * FQ_CAP;
			for (int e = t; e < cnt[i]; e += FB_THREADS) {
				const uint64_t key = b[e];
				if (key <= th && slot_alive(rowaux_f, (uint32_t)key)) {
					const int o = atomicAdd(ocnt + q, 1);
					if (o < ocap) out[(int64_t)q * ocap + o] = key;
				}
			}
		}
		__syncthreads();
		PQ_T(4);
	}
#ifdef LHIP_PQ_PROF
	if (t == 0 && blockIdx.x < PQ_PROF_WG)
		for (int i = 0; i < PQ_PROF_N; ++i) g_pq_prof[blockIdx.x * PQ_PROF_N + i] = pq_acc[i];
#endif
}

// Seed of the fast scan's per-query bound (thrq): one workgroup per query
// scores the first PQ_SEED_ROWS positions of its NEAREST probed list with its
// own 8-bit LUT, exactly as pq_fast_scan_kernel keys them (same ADC terms,
// same rounding, live rows only), and stores the kk-th smallest key: kk real
// keys of a probed list lie at or below it, so no key above it can be among
// the query's kk smallest (the bound is inclusive, as the scan's).  Without
// it every query's first items pass every row until a buffer sort sets one.
// (2048 positions: half the seed's cost of 4096 for the same scan time at C5,
// while 1024 loosened the bound enough to slow the scan; profiles/r05j_ab_*)
#ifndef LHIP_SEED_ROWS
#define LHIP_SEED_ROWS 2048
#endif
constexpr int PQ_SEED_ROWS = LHIP_SEED_ROWS, PQ_SEED_THREADS = 1024;  // (2 rows per thread: short per-thread chains)
template <int MT>
__global__ __launch_bounds__(PQ_SEED_THREADS) void pq_seed_kernel(const uint8_t *__restrict__ lcodes, int m, int mp,
                                                      const int64_t *__restrict__ loff,
                                                      const uint32_t *__restrict__ lslot,
                                                      const float *__restrict__ rowaux_f, int nprobe,
                                                      const int64_t *__restrict__ probe_l,
                                                      const float *__restrict__ probe_d,
                                                      const float *__restrict__ ltau, const uint8_t *__restrict__ lut8,
                                                      const float2 *__restrict__ qpar, int kk, int wb,
                                                      unsigned long long *__restrict__ thrq) {
	__shared__ __attribute__((aligned(16))) uint8_t L[FQ_MAX_M * PQ_K];
	__shared__ unsigned hist[256];
	__shared__ unsigned s_pre, s_rem;
	const int q = blockIdx.x, t = threadIdx.x;
	const int mm = MT > 0 ? MT : m;
	const int64_t l = probe_l[(int64_t)q * nprobe];
	if (l < 0) return;  // no probed list (a NaN query): no seed; the whole block leaves before any barrier
	const float d0 = probe_d[(int64_t)q * nprobe];
	const float2 qp = qpar[q];
	const uint8_t *lq = lut8 + (int64_t)q * mm * PQ_K;
	// the LUT in [j][c] order (lut8 may be in the bank scan's layout: lut8_index)
	const int wbc = MT > 0 ? (wb ? MT / 32 : 0) : wb;  // (a compile-time divisor for MT = 96)
	if (wbc == 0) {
		for (int i = t; i < mm * PQ_K / 16; i += PQ_SEED_THREADS) reinterpret_cast<uint4 *>(L)[i] = reinterpret_cast<const uint4 *>(lq)[i];
	} else {
		// the bank layout's 16-B chunk d holds codes c0 .. c0 + 15 of sub-space j
		// (pq_lut_u8_kernel): one 16-B read and one 16-B LDS store per chunk
		for (int d = t; d < mm * 16; d += PQ_SEED_THREADS) {
			const int b = d & 31, cp = (d >> 5) & 15, x = d >> 9;
			const int j = 4 * wbc * (b >> 2) + 4 * x + (b & 3);
			reinterpret_cast<uint4 *>(L + j * PQ_K)[cp] = reinterpret_cast<const uint4 *>(lq)[d];
		}
	}
	const int64_t p0 = loff[l], len = loff[l + 1] - p0;
	const int n = (int)(len < PQ_SEED_ROWS ? len : PQ_SEED_ROWS);
	const int nch = mp >> 4;
	if (t == 0) {
		s_pre = 0;
		s_rem = (unsigned)kk;
	}
	__syncthreads();
	// this thread's rows' ordered distance keys (the high word of the scan's key)
	constexpr int RPT = (PQ_SEED_ROWS + PQ_SEED_THREADS - 1) / PQ_SEED_THREADS;
	uint32_t hk[RPT];
#pragma unroll
	for (int i = 0; i < RPT; ++i) {
		const int r = t + i * PQ_SEED_THREADS;
		uint64_t key = KEY64_NONE;
		if (r < n) {
			const int64_t ps = p0 + r;
			const uint32_t slot = lslot[ps];
			if (slot != SLOT_NONE && slot_alive(rowaux_f, slot)) {
				const uint8_t *cp = lcodes + ps * mp;
				uint32_t S = 0;
				for (int c = 0; c < nch; ++c) {
					const uint4 w = *reinterpret_cast<const uint4 *>(cp + c * 16);
					const uint32_t wd[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
					for (int u = 0; u < 16; ++u) {
						const int j = c * 16 + u;
						if (j < mm) S += L[j * PQ_K + ((wd[u >> 2] >> (8 * (u & 3))) & 255u)];
					}
				}
				// the scan's key: ((d0 + tau) + L0) + D * S, each step rounded
				float a = ltau ? add_nc(d0, ltau[ps]) : d0;
				a = add_nc(a, qp.y);
				a = add_nc(a, mul_nc(qp.x, (float)S));
				key = key64(a, slot);
			}
		}
		hk[i] = (uint32_t)(key >> 32);
	}
	// the kk-th smallest high word T by a radix select (4 passes of 8 bits, no
	// sort); (T << 32) | 0xFFFFFFFF is then an inclusive bound with kk live keys
	// at or below it (as the kk-th full key was: looser only among equal high words)
	if (kk > n) return;  // (uniform: fewer rows than kk, no seed)
	uint32_t mask = 0;
	for (int sh = 24; sh >= 0; sh -= 8) {
		for (int i = t; i < 256; i += PQ_SEED_THREADS) hist[i] = 0;
		__syncthreads();
		const uint32_t pre = s_pre;
#pragma unroll
		for (int i = 0; i < RPT; ++i)
			if (t + i * PQ_SEED_THREADS < n && (hk[i] & mask) == pre) atomicAdd(&hist[(hk[i] >> sh) & 255u], 1u);
		__syncthreads();
		if (t < 64) {  // wave 0: prefix sums over the 256 bins (4 per lane), find the bin holding the rem-th
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
			unsigned ex = x - c;  // keys in bins before this lane's four
			if (ex < rem && rem <= x) {
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					if (rem <= ex + h4[u]) {
						s_pre = pre | ((uint32_t)(4 * t + u) << sh);
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
	if (t == 0 && s_pre != KEY_NAN) atomicMin(thrq + q, ((unsigned long long)s_pre << 32) | 0xFFFFFFFFull);
}

void launch_pq_seed(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                    const float *rowaux_f, int nq, int nprobe, const int64_t *probe_l, const float *probe_d,
                    const float *ltau, const uint8_t *lut8, const float2 *qpar, int kk, uint64_t *thrq, hipStream_t st) {
	if (nq <= 0 || kk > PQ_SEED_ROWS || m > FQ_MAX_M) return;
	auto thr = reinterpret_cast<unsigned long long *>(thrq);
	const int wb = pq_bank_w(m);
	if (m == 96)
		pq_seed_kernel<96><<<dim3((unsigned)nq), PQ_SEED_THREADS, 0, st>>>(lcodes, m, mp, loff, lslot, rowaux_f, nprobe, probe_l,
		                                                        probe_d, ltau, lut8, qpar, kk, wb, thr);
	else
		pq_seed_kernel<0><<<dim3((unsigned)nq), PQ_SEED_THREADS, 0, st>>>(lcodes, m, mp, loff, lslot, rowaux_f, nprobe, probe_l,
		                                                       probe_d, ltau, lut8, qpar, kk, wb, thr);
}

// LANCE_HIP_PQ_LANE_ROWS=1: the one-row-per-lane fast scan for every m (A/B of
// the two forms; the same results)
static bool pq_scan_lane_rows() {
	static const bool v = [] {
		const char *e = getenv("LANCE_HIP_PQ_LANE_ROWS");
		return e && e[0] == '1';
	}();
	return v;
}

// m / 32 when the fast scan takes the bank-conflict-free form (m = 32, 64, 96), else 0
static int pq_bank_w(int m) { return (m == 32 || m == 64 || m == 96) && !pq_scan_lane_rows() ? m / 32 : 0; }

int pq_fast_lds_bytes(int m) { return m * PQ_K * 4 + FQ_G * FQ_CAP * 8; }

void launch_pq_fast_items(const int *pstart, const int64_t *loff, const int *pairs, int nlist, int *item_off,
                          int *xbeg, int4 *itab, int itab_cap, hipStream_t st, bool offsets_done) {
	if (!offsets_done) pq_fast_items_kernel<<<1, 1024, 0, st>>>(pstart, loff, nlist, item_off, xbeg);
	if (itab) pq_fast_table_kernel<<<dim3((unsigned)((nlist + 255) / 256)), 256, 0, st>>>(pstart, loff, pairs, nlist,
	                                                                                       item_off, itab, itab_cap);
}

void launch_pq_fast_scan(const uint8_t *lcodes, int m, int mp, const int64_t *loff, const uint32_t *lslot,
                         const float *rowaux_f, int nlist, int nprobe, const int *pstart, const int *pairs,
                         const int *item_off, const int *xbeg, const float *probe_d, const float *ltau,
                         const uint8_t *lut8, const float2 *qpar, int kk, int *work, uint64_t *thrq, int *ocnt,
                         uint64_t *out, int ocap, const int4 *itab, int grid, hipStream_t st) {
	const int lds = pq_fast_lds_bytes(m);
	auto go = [&](auto kern) {
		HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
		                           160 * 1024 - 256));
		kern<<<dim3((unsigned)grid), FQ_THREADS, (size_t)lds, st>>>(
		    lcodes, m, mp, loff, lslot, rowaux_f, nlist, nprobe, pstart, pairs, item_off, xbeg, probe_d, ltau, lut8,
		    qpar, kk, work, reinterpret_cast<unsigned long long *>(thrq), ocnt, out, ocap);
	};
#ifdef LHIP_PQ_PROF
	{
		std::vector<uint64_t> z((size_t)PQ_PROF_WG * PQ_PROF_N, 0);
		HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_pq_prof), z.data(), z.size() * 8, 0, hipMemcpyHostToDevice, st));
		HIPCHK(hipStreamSynchronize(st));
	}
	struct Dump {
		hipStream_t st;
		int grid;
		~Dump() {
			static std::atomic<int> calls{0};
			if (++calls != 3 || hipStreamSynchronize(st) != hipSuccess) return;  // (the 3rd launch of the process)
			std::vector<uint64_t> h((size_t)PQ_PROF_WG * PQ_PROF_N);
			if (hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_pq_prof), h.size() * 8) != hipSuccess) return;
			double sum[PQ_PROF_N] = {0};
			uint64_t mx = 0;
			const int g = std::min(grid, PQ_PROF_WG);
			for (int b = 0; b < g; ++b) {
				uint64_t tot = 0;
				for (int i = 0; i < PQ_PROF_N; ++i) sum[i] += (double)h[(size_t)b * PQ_PROF_N + i];
				for (int i = 0; i < 5; ++i) tot += h[(size_t)b * PQ_PROF_N + i];
				mx = std::max(mx, tot);
			}
			fprintf(stderr, "PQPROF wgs=%d avg cycles: claim %.0f lut %.0f rows %.0f sort %.0f flush %.0f | items %.1f sorts %.1f cand %.0f | max wg total %llu\n",
			        g, sum[0] / g, sum[1] / g, sum[2] / g, sum[3] / g, sum[4] / g, sum[5] / g, sum[6] / g, sum[7] / g,
			        (unsigned long long)mx);
		}
	} dump_{st, grid};
#endif
	auto bank = [&](auto kern) {
		HIPCHK(hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
		                           160 * 1024 - 256));
		kern<<<dim3((unsigned)grid), FB_THREADS, (size_t)(lds + FB_META_BYTES), st>>>(
		    lcodes, loff, lslot, rowaux_f, nlist, nprobe, pstart, pairs, item_off, xbeg, probe_d, ltau, lut8, qpar,
		    kk, work, reinterpret_cast<unsigned long long *>(thrq), ocnt, out, ocap, itab);
	};
	if (pq_bank_w(m)) {  // m = 32, 64, 96: the bank-conflict-free form (lut8 in its layout)
		if (m == 96) return bank(pq_fast_scan_bank_kernel<3>);
		if (m == 64) return bank(pq_fast_scan_bank_kernel<2>);
		if (m == 32) return bank(pq_fast_scan_bank_kernel<1>);
	}
	switch (m) {
	case 96: go(pq_fast_scan_kernel<96>); break;
	case 64: go(pq_fast_scan_kernel<64>); break;
	case 48: go(pq_fast_scan_kernel<48>); break;
	case 32: go(pq_fast_scan_kernel<32>); break;
	case 16: go(pq_fast_scan_kernel<16>); break;
	case 8: go(pq_fast_scan_kernel<8>); break;
	default: go(pq_fast_scan_kernel<0>); break;
	}
}

// per query: top-K of its output run (count ocnt[q], capped at ocap).  thrq
// (the scan's final per-query bound, nullable): an inclusive upper bound on the
// run's K-th key — the cut that set it held K keys at or below it, and those
// went out at their item's flush — so keys above it are never offered (no
// buffer sorts for them)
__global__ __launch_bounds__(256) void pq_run_merge_kernel(const uint64_t *__restrict__ keys, const int *__restrict__ ocnt,
                                                           int ocap, int K, uint64_t *__restrict__ out,
                                                           const uint64_t *__restrict__ thrq) {
	__shared__ uint64_t buf[IVF_TOPK_CAP];
	__shared__ int cnt;
	__shared__ uint64_t thr;
	const int q = blockIdx.x, t = threadIdx.x;
	TopK tk{buf, &cnt, &thr, K};
	tk.reset();
	const int n = min(ocnt[q], ocap);
	const uint64_t *src = keys + (int64_t)q * ocap;
	if (thrq) {
		// one pass: only keys at or below the bound (typically ~K .. 2K of the
		// run) go to the buffer, 8 loads in flight per thread; then one sort
		const uint64_t bq = thrq[q];
		for (int e0 = t; e0 < n; e0 += 256 * 8) {
			uint64_t kv[8];
#pragma unroll
			for (int u = 0; u < 8; ++u) kv[u] = e0 + 256 * u < n ? src[e0 + 256 * u] : KEY64_NONE;
#pragma unroll
			for (int u = 0; u < 8; ++u)
				if (kv[u] != KEY64_NONE && kv[u] <= bq) {
					const int p = atomicAdd(&cnt, 1);
					if (p < IVF_TOPK_CAP) buf[p] = kv[u];
				}
		}
		__syncthreads();
		const int c = cnt;
		if (c <= IVF_TOPK_CAP) {
			const int np = pow2_ceil(c);
			for (int i = c + t; i < np; i += 256) buf[i] = KEY64_NONE;
			wg_bitonic_sort(buf, np);
			const int nout = c < K ? c : K;
			for (int i = t; i < K; i += 256) out[(int64_t)q * K + i] = i < nout ? buf[i] : KEY64_NONE;
			return;
		}
		// (more than the buffer at or below the bound: the streaming top-K below, from the bound)
		__syncthreads();
		if (t == 0) {
			cnt = 0;
			thr = bq == KEY64_NONE ? KEY64_NONE : bq + 1;  // (offer keeps key < thr)
		}
		__syncthreads();
	}
	for (int e0 = 0; e0 < n; e0 += 256) {
		const int e = e0 + t;
		const uint64_t k = e < n ? src[e] : KEY64_NONE;
		tk.offer(k, k != KEY64_NONE);
	}
	const int nout = tk.finish();
	for (int i = t; i < K; i += 256) out[(int64_t)q * K + i] = i < nout ? buf[i] : KEY64_NONE;
}

// The run merge with the scan's final bound (pq_merge_bound, the default), on
// 1024 threads: the run's keys at or below thrq[q] are gathered into LDS; up
// to RS_SORT of them are sorted directly, more (a bound that stayed loose: no
// item of the query ever cut its buffer, so thrq is the seed's) go through a
// radix select of the K-th smallest distance word (4 passes of 8 bits, wave 0
// scans the 256 bins) and only the keys at or below that word are sorted.  A
// gather past RS_CAP, or a tie group leaving more than RS_SORT keys at the
// selected word, takes the streaming top-K over the whole run.  The output is
// the same K keys as pq_run_merge_kernel's in every case.
constexpr int RS_THREADS = 1024, RS_CAP = 8192, RS_SORT = 2048, RS_PT = RS_CAP / RS_THREADS;
static_assert(IVF_TOPK_CAP <= RS_CAP && FQ_MAX_KK <= IVF_TOPK_CAP - RS_THREADS, "run select buffers");
__global__ __launch_bounds__(RS_THREADS) void pq_run_select_kernel(const uint64_t *__restrict__ keys,
                                                                   const int *__restrict__ ocnt, int ocap, int K,
                                                                   uint64_t *__restrict__ out,
                                                                   const uint64_t *__restrict__ thrq) {
	__shared__ uint64_t buf[RS_CAP];
	__shared__ unsigned hist[256];
	__shared__ int s_cnt, s_n2;
	__shared__ unsigned s_pre, s_rem;
	__shared__ uint64_t s_thr;
	const int q = blockIdx.x, t = threadIdx.x;
	const int n = min(ocnt[q], ocap);
	const uint64_t *src = keys + (int64_t)q * ocap;
	const uint64_t bq = thrq[q];
	if (t == 0) {
		s_cnt = 0;
		s_n2 = 0;
		s_pre = 0;
		s_rem = (unsigned)K;
	}
	__syncthreads();
	for (int e0 = t; e0 < n; e0 += RS_THREADS * 4) {
		uint64_t kv[4];
#pragma unroll
		for (int u = 0; u < 4; ++u) kv[u] = e0 + RS_THREADS * u < n ? src[e0 + RS_THREADS * u] : KEY64_NONE;
#pragma unroll
		for (int u = 0; u < 4; ++u)
			if (kv[u] != KEY64_NONE && kv[u] <= bq) {
				const int p = atomicAdd(&s_cnt, 1);
				if (p < RS_CAP) buf[p] = kv[u];
			}
	}
	__syncthreads();
	const int c = s_cnt;
	// buf[0, m) sorted, its first K out
	auto emit_sorted = [&](int m) {
		const int np = pow2_ceil(m);
		for (int i = m + t; i < np; i += RS_THREADS) buf[i] = KEY64_NONE;
		wg_bitonic_sort(buf, np);
		const int nout = m < K ? m : K;
		for (int i = t; i < K; i += RS_THREADS) out[(int64_t)q * K + i] = i < nout ? buf[i] : KEY64_NONE;
	};
	if (c <= RS_SORT) {
		emit_sorted(c);
		return;
	}
	if (c <= RS_CAP) {
		uint32_t hw[RS_PT];
		uint64_t kv[RS_PT];
#pragma unroll
		for (int j = 0; j < RS_PT; ++j) {
			const int i = t + j * RS_THREADS;
			kv[j] = i < c ? buf[i] : KEY64_NONE;
			hw[j] = (uint32_t)(kv[j] >> 32);
		}
		unsigned mask = 0;
		for (int sh = 24; sh >= 0; sh -= 8) {
			if (t < 256) hist[t] = 0;
			__syncthreads();
			const unsigned pre = s_pre;
#pragma unroll
			for (int j = 0; j < RS_PT; ++j)
				if (t + j * RS_THREADS < c && (hw[j] & mask) == pre) atomicAdd(&hist[(hw[j] >> sh) & 255], 1u);
			__syncthreads();
			if (t < 64) {
				const unsigned rem = s_rem;
				unsigned h4[4], cs = 0;
#pragma unroll
				for (int u = 0; u < 4; ++u) {
					h4[u] = hist[4 * t + u];
					cs += h4[u];
				}
				unsigned x = cs;
#pragma unroll
				for (int o = 1; o < 64; o <<= 1) {
					const unsigned y = __shfl_up(x, o, 64);
					if (t >= o) x += y;
				}
				unsigned ex = x - cs;
				if (ex < rem && rem <= x) {
#pragma unroll
					for (int u = 0; u < 4; ++u) {
						if (rem <= ex + h4[u]) {
							s_pre = pre | ((unsigned)(4 * t + u) << sh);
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
		// T: the K-th smallest distance word (K < c); at least K keys lie at or
		// below it and every key above it has K smaller ones
		const uint32_t T = s_pre;
#pragma unroll
		for (int j = 0; j < RS_PT; ++j)
			if (t + j * RS_THREADS < c && hw[j] <= T) {
				const int p = atomicAdd(&s_n2, 1);
				if (p < RS_SORT) buf[p] = kv[j];
			}
		__syncthreads();
		const int m2 = s_n2;
		if (m2 <= RS_SORT) {
			emit_sorted(m2);
			return;
		}
	}
	// streaming top-K over the whole run from the bound (buf as its buffer)
	__syncthreads();
	if (t == 0) {
		s_cnt = 0;
		s_thr = bq == KEY64_NONE ? KEY64_NONE : bq + 1;  // (offer keeps key < thr)
	}
	__syncthreads();
	TopK tk{buf, &s_cnt, &s_thr, K};
	for (int e0 = 0; e0 < n; e0 += RS_THREADS) {
		const int e = e0 + t;
		const uint64_t k = e < n ? src[e] : KEY64_NONE;
		tk.offer(k, k != KEY64_NONE);
	}
	const int nout = tk.finish();
	for (int i = t; i < K; i += RS_THREADS) out[(int64_t)q * K + i] = i < nout ? buf[i] : KEY64_NONE;
}

void launch_pq_run_merge(const uint64_t *keys, const int *ocnt, int nq, int ocap, int K, uint64_t *out,
                         hipStream_t st, const uint64_t *thrq) {
	if (thrq && K <= FQ_MAX_KK)
		pq_run_select_kernel<<<dim3((unsigned)nq), RS_THREADS, 0, st>>>(keys, ocnt, ocap, K, out, thrq);
	else
		pq_run_merge_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(keys, ocnt, ocap, K, out, thrq);
}

// ---------------------------------------------------------------------------
// merge / output
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ivf_merge_kernel(int nprobe, const int64_t *__restrict__ probe_l,
                                                        const int *__restrict__ lblk0, int maxb, int kk,
                                                        const uint64_t *__restrict__ keys, int tail_nb,
                                                        const uint64_t *__restrict__ tkeys, int K,
                                                        uint64_t *__restrict__ out) {
	__shared__ uint64_t buf[IVF_TOPK_CAP];
	__shared__ int cnt;
	__shared__ uint64_t thr;
	const int q = blockIdx.x, t = threadIdx.x;
	TopK tk{buf, &cnt, &thr, K};
	tk.reset();
	if (keys) {
		for (int p = 0; p < nprobe; ++p) {
			const int64_t l = probe_l[(int64_t)q * nprobe + p];
			if (l < 0) continue;
			const int nb = lblk0 ? lblk0[l + 1] - (int)lblk0[l] : 1;
			const uint64_t *src = keys + ((int64_t)q * nprobe + p) * maxb * kk;
			const int tot = nb * kk;
			for (int e0 = 0; e0 < tot; e0 += 256) {
				const int e = e0 + t;
				const uint64_t k = e < tot ? src[e] : KEY64_NONE;
				tk.offer(k, k != KEY64_NONE);
			}
		}
	}
	if (tkeys) {
		const uint64_t *src = tkeys + (int64_t)q * tail_nb * kk;
		const int tot = tail_nb * kk;
		for (int e0 = 0; e0 < tot; e0 += 256) {
			const int e = e0 + t;
			const uint64_t k = e < tot ? src[e] : KEY64_NONE;
			tk.offer(k, k != KEY64_NONE);
		}
	}
	const int nout = tk.finish();
	for (int i = t; i < K; i += 256) out[(int64_t)q * K + i] = i < nout ? buf[i] : KEY64_NONE;
}

void launch_ivf_merge(int nq, int nprobe, const int64_t *probe_l, const int *lblk0, int maxb, int kk,
                      const uint64_t *keys, int tail_nb, const uint64_t *tkeys, int K, uint64_t *out, hipStream_t st) {
	ivf_merge_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(nprobe, probe_l, lblk0, maxb, kk, keys, tail_nb, tkeys, K,
	                                                      out);
}

__global__ void keys_to_output_kernel(const uint64_t *__restrict__ keys, int K, int k,
                                      const int64_t *__restrict__ labels, int64_t *__restrict__ outL,
                                      float *__restrict__ outD, int *__restrict__ outC, uint32_t sx) {
	const int q = blockIdx.x;
	__shared__ int n;
	if (threadIdx.x == 0) n = 0;
	__syncthreads();
	for (int i = threadIdx.x; i < k; i += blockDim.x) {
		const uint64_t key = i < K ? keys[(int64_t)q * K + i] : KEY64_NONE;
		if (key != KEY64_NONE) {
			outL[(int64_t)q * k + i] = labels[(uint32_t)key ^ sx];
			outD[(int64_t)q * k + i] = key64_dist(key);
			atomicAdd(&n, 1);
		} else {
			outL[(int64_t)q * k + i] = -1;
			outD[(int64_t)q * k + i] = __builtin_nanf("");
		}
	}
	__syncthreads();
	if (threadIdx.x == 0) outC[q] = n;
}

void launch_keys_to_output(const uint64_t *keys, int nq, int K, int k, const int64_t *labels, int64_t *outL,
                           float *outD, int *outC, hipStream_t st, int tie_desc) {
	keys_to_output_kernel<<<dim3((unsigned)nq), 256, 0, st>>>(keys, K, k, labels, outL, outD, outC,
	                                                           tie_x32(tie_desc));
}

// exact re-rank of the ADC candidates (+ the tail's exact candidates): one
// wave per candidate (f64, the flat path's refine arithmetic), bitonic sort
template <int METRIC, typename T>
__global__ __launch_bounds__(RR_THREADS) void ivf_refine_final_kernel(const T *__restrict__ X, int ld, int dim,
                                                               const float *__restrict__ Qf,
                                                               const uint64_t *__restrict__ ca, int ka,
                                                               const uint64_t *__restrict__ cbk, int kb, int k,
                                                               const int64_t *__restrict__ labels,
                                                               int64_t *__restrict__ outL, float *__restrict__ outD,
                                                               int *__restrict__ outC, uint32_t sx) {
	__shared__ uint64_t sk[IVF_TOPK_CAP];
	__shared__ uint32_t ss[IVF_TOPK_CAP];
	__shared__ int n;
	const int q = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
	if (t == 0) n = 0;
	__syncthreads();
	for (int i = t; i < ka + kb; i += RR_THREADS) {
		// (ADC keys carry the slot; the tail's exact keys slot ^ sx)
		const uint64_t key = i < ka ? ca[(int64_t)q * ka + i] : cbk[(int64_t)q * kb + (i - ka)];
		if (key != KEY64_NONE) ss[atomicAdd(&n, 1)] = (uint32_t)key ^ (i < ka ? 0u : sx);
	}
	__syncthreads();
	const int nc = n;
	for (int i = w; i < nc; i += RR_THREADS / 64) {
		const uint32_t slot = ss[i];
		const float d = exact_distance<METRIC, T>(X + (int64_t)slot * ld, Qf + (int64_t)q * ld, dim, lane);
		if (lane == 0) sk[i] = key64(d, slot ^ sx);
	}
	const int np = pow2_ceil(nc);
	__syncthreads();
	for (int i = nc + t; i < np; i += RR_THREADS) sk[i] = KEY64_NONE;
	wg_bitonic_sort(sk, np);
	const int nout = nc < k ? nc : k;
	for (int i = t; i < k; i += RR_THREADS) {
		if (i < nout) {
			outL[(int64_t)q * k + i] = labels[(uint32_t)sk[i] ^ sx];
			outD[(int64_t)q * k + i] = key64_dist(sk[i]);
		} else {
			outL[(int64_t)q * k + i] = -1;
			outD[(int64_t)q * k + i] = __builtin_nanf("");
		}
	}
	if (t == 0) outC[q] = nout;
}

template <typename T>
static void refine_final_dispatch(const StoreView &s, const float *Qf, const uint64_t *ca, int ka, const uint64_t *cb,
                                  int kb, int nq, int k, int64_t *outL, float *outD, int *outC, hipStream_t st) {
	const T *X = static_cast<const T *>(s.X);
	dim3 grid((unsigned)nq);
#define RF_ARGS X, s.ld, s.dim, Qf, ca, ka, cb, kb, k, s.labels, outL, outD, outC, tie_x32(s.tie_desc)
	switch (s.metric) {
	case METRIC_L2: ivf_refine_final_kernel<METRIC_L2, T><<<grid, RR_THREADS, 0, st>>>(RF_ARGS); break;
	case METRIC_DOT: ivf_refine_final_kernel<METRIC_DOT, T><<<grid, RR_THREADS, 0, st>>>(RF_ARGS); break;
	default: ivf_refine_final_kernel<METRIC_COSINE, T><<<grid, RR_THREADS, 0, st>>>(RF_ARGS); break;
	}
#undef RF_ARGS
}

void launch_ivf_refine_final(const StoreView &s, const float *Qf, const uint64_t *ca, int ka, const uint64_t *cb,
                             int kb, int nq, int k, int64_t *outL, float *outD, int *outC, hipStream_t st) {
	if (s.xbf16)
		refine_final_dispatch<uint16_t>(s, Qf, ca, ka, cb, kb, nq, k, outL, outD, outC, st);
	else
		refine_final_dispatch<float>(s, Qf, ca, ka, cb, kb, nq, k, outL, outD, outC, st);
}

}  // namespace lhip
