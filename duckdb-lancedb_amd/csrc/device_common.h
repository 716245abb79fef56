// Device helpers shared by the gfx950 kernel files (knn_kernels.hip: flat
// path, ivf_kernels.hip: IVF_FLAT / IVF_PQ).  Canonical numerics of this build:
// ordered float keys, the (distance, label) order, exact distances with f64
// accumulation rounded once to f32 (DESIGN.md "Oracle and parity").
#pragma once
#include "knn_kernels.h"

namespace lhip {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(16))) int i32x16;

static constexpr float F_INF = __builtin_huge_valf();
static constexpr float F_MAX = 3.40282347e+38f;
static constexpr uint32_t KEY_INF = 0xFF800000u;  // ordered key of +inf
static constexpr uint32_t KEY_NAN = 0xFFFFFFFFu;  // every NaN is canonicalised to this

// ---------------------------------------------------------------------------
// MFMA operand guard (gfx950, ROCm 7.2).  hipcc lets a VALU instruction right
// after the last MFMAs of a tile overwrite one of their A / B operand VGPRs
// (the epilogue's first v_mbcnt was allocated onto the A register of the
// still-executing last MFMA, ~9 issue slots after it): the MFMA then read the
// new value and one accumulator column came out wrong (wrong cosine bounds in
// ~1 of 40 repeated searches; which kernel build shows it depends only on
// register allocation).  A scheduling fence with 64 wait states between the
// last MFMA and the first instruction after it closes the window: once per
// tile, not per k-step (within the k-loop the next writes of the operand
// registers are ds_reads, whose data lands much later than the MFMA reads).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void mfma_operand_guard() {
	__builtin_amdgcn_sched_barrier(0);
	asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
	__builtin_amdgcn_sched_barrier(0);
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fkey(float f) {
	uint32_t u = __float_as_uint(f);
	if ((u & 0x7FFFFFFFu) > 0x7F800000u) return KEY_NAN;
	return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
	uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
	return __uint_as_float(u);
}
__device__ __forceinline__ uint16_t bf16_bits(float f) {
	__bf16 h = (__bf16)f;  // RNE: v_cvt_pk_bf16_f32 on gfx950
	return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf16_round(float f) {
	return (float)(__bf16)f;
}
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
	return (uint32_t)bf16_bits(a) | ((uint32_t)bf16_bits(b) << 16);
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
	return v;
}
// Tie rule of the final (exact-distance) order, per handle (option "tie",
// LANCE_HIP_TIE): label ascending, or label descending — the order the
// reference's own golden shows at a tie (lance_optimizer_filter.test:36-44:
// ids 3 and 4 tie at d = 2.0 and LanceDB returns 4).  Applied as an XOR on the
// label (int64, labels >= 0) or on the slot of a (key << 32 | slot) word
// (slots < 2^31; slots ascend with labels): 0 keeps the order, the all-ones
// pattern below the sign bit reverses it and never forms the all-ones
// "no entry" word.
__host__ __device__ __forceinline__ int64_t tie_x64(int desc) { return desc ? INT64_MAX : 0; }
__host__ __device__ __forceinline__ uint32_t tie_x32(int desc) { return desc ? 0x7FFFFFFFu : 0u; }
// (distance, label) total order used everywhere: NaN after +inf, then the
// label under the tie rule tx = tie_x64(desc).
__device__ __forceinline__ bool hit_less(float da, int64_t la, float db, int64_t lb, int64_t tx) {
	bool an = __builtin_isnan(da), bn = __builtin_isnan(db);
	if (an != bn) return bn;
	if (!an && da != db) return da < db;
	return (la ^ tx) < (lb ^ tx);
}
// unit roundoff used by the bounds; 2^-23 (not 2^-24) leaves room for an
// accumulation that truncates instead of rounding.
static constexpr double U_BOUND = 1.1920928955078125e-07;

// a base element as f32: the store holds f32, or bf16 bits (uint16_t)
__device__ __forceinline__ float xval(const float *p, int64_t i) { return p[i]; }
__device__ __forceinline__ float xval(const uint16_t *p, int64_t i) { return __uint_as_float((uint32_t)p[i] << 16); }

// Row aux layout: tile-blocked SoA, 16 B per slot.  For slot r of tile
// T = r / 256 the four terms live at floats [T*1024 + c*256 + r%256],
// c = 0 alpha, 1 xn, 2 ux, 3 sc.  A tile's block is the 4 KiB the scan DMAs
// into LDS, and four consecutive rows' terms are one 16 B read.
__host__ __device__ __forceinline__ int64_t raix(int64_t r, int c) { return ((r >> 8) << 10) | ((int64_t)c << 8) | (r & 255); }

// four consecutive base elements as f32 (16-B / 8-B aligned: rows are ld-padded)
__device__ __forceinline__ float4 xval4(const float *p, int64_t i) { return *reinterpret_cast<const float4 *>(p + i); }
__device__ __forceinline__ float4 xval4(const uint16_t *p, int64_t i) {
	const uint2 u = *reinterpret_cast<const uint2 *>(p + i);
	return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
	                   __uint_as_float(u.y & 0xFFFF0000u));
}

template <int METRIC>
__device__ __forceinline__ void exact_acc(double xv, double qv, double &a, double &b, double &c) {
	if (METRIC == METRIC_L2) {
		const double d = xv - qv;
		a += d * d;
	} else {
		a += xv * qv;
		if (METRIC == METRIC_COSINE) {
			b += xv * xv;
			c += qv * qv;
		}
	}
}

// Exact distance of one row to one query by one wave: f64 accumulation, f32
// result.  Each lane takes 4 consecutive elements per step (one 16-B load of
// the row, one of the query; the steps of a lane are independent loads, so a
// row costs one memory latency, not dim/64 of them).
template <int METRIC, typename T>
__device__ __forceinline__ float exact_distance(const T *__restrict__ x, const float *__restrict__ q, int dim,
                                                int lane) {
	double a = 0.0, b = 0.0, c = 0.0;
	const int d4 = dim >> 2;
#pragma unroll 4
	for (int i4 = lane; i4 < d4; i4 += 64) {
		const float4 xv = xval4(x, 4 * i4);
		const float4 qv = *reinterpret_cast<const float4 *>(q + 4 * i4);
		exact_acc<METRIC>(xv.x, qv.x, a, b, c);
		exact_acc<METRIC>(xv.y, qv.y, a, b, c);
		exact_acc<METRIC>(xv.z, qv.z, a, b, c);
		exact_acc<METRIC>(xv.w, qv.w, a, b, c);
	}
	for (int i = 4 * d4 + lane; i < dim; i += 64) exact_acc<METRIC>(xval(x, i), q[i], a, b, c);
	a = wave_sum_f64(a);
	if (METRIC == METRIC_COSINE) {
		b = wave_sum_f64(b);
		c = wave_sum_f64(c);
	}
	double r;
	if (METRIC == METRIC_L2)
		r = a;
	else if (METRIC == METRIC_DOT)
		r = 1.0 - a;
	else
		r = 1.0 - a / (sqrt(b) * sqrt(c));
	float f = (float)r + 0.0f;  // canonical +0
	if (__builtin_isnan(f)) f = __builtin_nanf("");
	return f;
}

}  // namespace lhip
