// gfx950 (MI355X / CDNA4) register-streamed threshold scan: the append pass of
// the flat search (knn_kernels.h launch_scan_append) for large stores.
//
// Same contract and numerics as scan_kernel<.., MODE 1, ..> (knn_kernels.hip):
// per (row, query) a rigorous lower bound LB of the exact distance from a bf16
// MFMA dot product plus the row/query bound terms, and (LB, slot) appended to
// the workgroup's segment of the query when LB <= tau[q].  What differs is how
// the base reaches the matrix cores.  The LDS-staged scan_kernel holds one
// 32 KiB stage of rows in flight per CU (its ring shares LDS with the query
// stages).  Here the rows never touch LDS:
//
//   * a workgroup is 4 MFMA waves + 4 loader waves (two waves per SIMD, 256
//     registers each); an MFMA wave owns 32 rows x 256 queries of the 128 x 256
//     tile: 2 x 16 blocks of v_mfma_f32_16x16x32_bf16, 128 accumulators;
//   * each MFMA wave loads its own rows straight into a 4-window register ring
//     (global loads, windows of 128 B per row; 3 windows = 48 KiB per CU in
//     flight ahead of the one being multiplied); f32 rows are rounded to bf16
//     in registers;
//   * the loader waves stream the queries' windows (L2-resident, 16 / 32 KiB
//     each) into a 4-slot LDS image by LDS-DMA, three windows ahead, and the
//     next tile's row terms; one barrier per window.  vmcnt is per wave, so
//     the MFMA waves' row loads are never drained by a query load (the first
//     version loaded the queries in the MFMA waves, behind the row loads, and
//     every window waited for the whole ring: 3x slower, profiles/r02_g_*).
// Restricted to stores whose row stride is a multiple of 4 windows (ld % 128
// == 0 for f32, % 256 for bf16): the ring is unrolled by 4 and a tile ends on
// a ring boundary.
#include "device_common.h"

#include <stdexcept>

// Development-only timing ablations (results are wrong when set): only an
// ablation build (tools/rs_ablate.sh, -DLHIP_ABLATION_BUILD) may turn them on.
#if !defined(LHIP_ABLATION_BUILD) && (defined(LHIP_RS_ABL_NO_QDMA) || defined(LHIP_RS_ABL_NO_MFMA) || \
                                      defined(LHIP_RS_ABL_NO_EPI) || defined(LHIP_RS_ABL_NO_XLOAD))
#error "rscan ablation switches are for ablation builds only"
#endif
#include <type_traits>

namespace lhip {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int RS_MW = 8;                 // MFMA waves (two per SIMD)
constexpr int RS_NL = 4;                 // loader waves (one per SIMD)
constexpr int RS_THREADS = 64 * (RS_MW + RS_NL);
constexpr int RS_BR = 128;               // rows per tile
constexpr int RS_WR = RS_BR / RS_MW;     // rows per MFMA wave: 16
constexpr int RS_RB = RS_WR / 16;        // 16-row blocks per MFMA wave
constexpr int RS_WIN = 128;              // bytes of each row per window
constexpr int RS_NQS = 4;                // query image slots: window v+3 streams in while v is multiplied
constexpr int RS_WLIST = 256;            // survivor list entries per MFMA wave
constexpr int RS_FLUSH_AT = 192;

template <bool XB>
struct RsCfg {
	static constexpr int XE = XB ? 2 : 4;        // bytes per base element
	static constexpr int KW = RS_WIN / XE;       // k per window: 64 / 32
	static constexpr int KS = KW / 32;           // 16x16x32 k-steps per window: 2 / 1
	static constexpr int QW = KW * 2;            // bytes of one query per window (bf16): 128 / 64
	static constexpr int QSLOT = SCAN_BQ * QW;   // 32 / 16 KiB
	static constexpr int QNI = QSLOT / 1024 / RS_NL;  // 1-KiB DMA pieces per loader wave and window: 8 / 4
	static constexpr int RA_SLOT = RS_BR * 16;   // 2 KiB of row terms per tile
	static constexpr int OFF_RA = RS_NQS * QSLOT;
	static constexpr int OFF_QA = OFF_RA + 2 * RA_SLOT;
	static constexpr int OFF_TAU = OFF_QA + SCAN_BQ * 16;
	static constexpr int OFF_CNT = OFF_TAU + SCAN_BQ * 4;
	static constexpr int OFF_LIST = OFF_CNT + SCAN_BQ * 4;
	static constexpr int LDS = OFF_LIST + RS_MW * RS_WLIST * 8;
	static_assert(LDS <= 160 * 1024, "LDS budget");
	static_assert(QSLOT % (1024 * RS_NL) == 0, "query slot in whole DMA pieces");
	// physical 16-B chunk of chunk c of query row q (an involution): conflict-
	// free ds_read_b128 over each 16-lane group (16 queries, one chunk each)
	__device__ static __forceinline__ int qswz(int q, int c) {
		return QW == 128 ? c ^ ((q >> 1) & 7) : c ^ ((q >> 2) & 3);
	}
};

// compile-time loop: f(integral_constant<int, I>) for I in [B, E) — keeps every
// accumulator index a constant (a runtime index would put them in scratch)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F &&f) {
	if constexpr (B < E) {
		f(std::integral_constant<int, B>{});
		static_for<B + 1, E>(f);
	}
}

// Lane id the compiler cannot prove loop-invariant (the all-ones mask goes
// through an empty asm statement as an SGPR; the mbcnt instructions are the
// compiler's own), so the epilogue's 128 per-lane list payloads are computed
// where used instead of hoisted out of the tile loop and spilled.
__device__ __forceinline__ int rs_lane_fresh() {
	uint32_t m = 0xFFFFFFFFu;
	asm volatile("" : "+s"(m));
	return (int)__builtin_amdgcn_mbcnt_hi(m, __builtin_amdgcn_mbcnt_lo(m, 0u));
}

// One global_load_lds_dwordx4 (64 lanes x 16 B, lane-linear at the
// wave-uniform LDS byte address in M0), issued only by the loader waves.
// Inline asm: the compiler does not see the LDS write in flight, so it puts
// no vmcnt(0) in front of the MFMA waves' ds_reads or the barriers; ordering is
// the loader's counted vmcnt + the step barrier.
__device__ __forceinline__ void rs_dma16(const void *sbase, uint32_t voff, uint32_t lds_addr) {
	const uint64_t b = (uint64_t)(uintptr_t)sbase;
	const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
	const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
	const uint64_t ub = ((uint64_t)hi << 32) | (uint64_t)lo;
	asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds_addr), "v"(voff), "s"(ub) : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void rs_wait_vm() {
	asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int METRIC>
__device__ __forceinline__ float rs_lower_bound(float s, float4 ra, float4 qa) {
	// LB = alpha + xn*B + ux*A + (s*sc)*S + C  (scan_kernel's lower_bound)
	float v = fmaf(ra.y, qa.z, ra.x);
	v = fmaf(ra.z, qa.y, v);
	float ss = (METRIC == METRIC_COSINE) ? s * ra.w : s;
	v = fmaf(ss, qa.x, v);
	return v + qa.w;
}

// Workgroup = 4 MFMA waves + 4 loader waves (two waves per SIMD).  Step v of
// the workgroup = window v of its row stream (window v % S of tile v / S):
//   MFMA wave: [tile start: accumulators <- row/query bound terms]; issue the
//              global loads of its 32 rows' window v+R-1 into the register
//              ring; multiply window v (registers) x the queries' window v
//              (LDS slot v % NQS); barrier; [tile end: epilogue];
//   loader wave: LDS-DMA the queries' window v+NQS-1 into slot (v-1) % NQS
//              (read by the MFMA waves in step v-1, finished at its barrier)
//              and, at window 1 of a tile, the next tile's row terms; wait
//              (its own vmcnt) for window v+1's pieces; barrier.
// vmcnt is per wave, so the MFMA waves' row ring never waits for a query
// load: the row loads of a window are waited for only where it is multiplied.
template <int METRIC, bool XB, int R>
__global__ __launch_bounds__(RS_THREADS, 1) void rscan_kernel(const uint8_t *__restrict__ X,
                                                              const float4 *__restrict__ rowaux, int ld,
                                                              const uint16_t *__restrict__ Qb,
                                                              const float4 *__restrict__ qaux, int nq, int n_tiles,
                                                              const float *__restrict__ tau,
                                                              uint2 *__restrict__ seg_pool,
                                                              int *__restrict__ seg_cnt, int seg_cap) {
	using C = RsCfg<XB>;
	constexpr bool FOLD = METRIC != METRIC_COSINE;
	__shared__ __attribute__((aligned(16))) uint8_t smem[C::LDS];
	float4 *QA = reinterpret_cast<float4 *>(smem + C::OFF_QA);
	float *TAU = reinterpret_cast<float *>(smem + C::OFF_TAU);
	unsigned *CNT = reinterpret_cast<unsigned *>(smem + C::OFF_CNT);

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int q0 = blockIdx.y * SCAN_BQ;
	const int64_t rowb = (int64_t)ld * C::XE;      // bytes per row
	const int S = (int)(rowb / RS_WIN);            // windows per tile (multiple of R, >= 4)
	const int my_tiles = (n_tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
	const int G = my_tiles * S;                    // windows of this workgroup
	auto tile_row0 = [&](int t) __attribute__((always_inline)) {
		return ((int64_t)blockIdx.x + (int64_t)t * gridDim.x) * RS_BR;
	};
	const uint32_t smem_base = (uint32_t)(uintptr_t)smem;

	if (tid < SCAN_BQ) {
		QA[tid] = qaux[q0 + tid];
		TAU[tid] = (q0 + tid < nq) ? tau[q0 + tid] : -F_INF;
		CNT[tid] = 0u;
	}

	if (w >= RS_MW) {
		// ================= loader waves =================
		const int lw = w - RS_MW;
		const uint16_t *qbase = Qb + (int64_t)q0 * ld;
		// piece i of this wave: bytes [1024 (lw QNI + i), +1024) of the slot
		// image; lane l's 16 B = physical chunk of query (off / QW)
		uint32_t qoff[C::QNI];
#pragma unroll
		for (int i = 0; i < C::QNI; ++i) {
			const int off = 1024 * (lw * C::QNI + i) + 16 * lane;
			const int q = off / C::QW, pc = (off % C::QW) / 16;
			qoff[i] = (uint32_t)(q * ld * 2) + 16u * (uint32_t)C::qswz(q, pc);  // chunk qswz(q, pc) of row q
		}
		auto dma_q = [&](int v) __attribute__((always_inline)) {
#ifdef LHIP_RS_ABL_NO_QDMA
			return;
#endif
			const int s = v % S, slot = v % RS_NQS;
#pragma unroll
			for (int i = 0; i < C::QNI; ++i)
				rs_dma16(qbase, qoff[i] + (uint32_t)(s * C::QW),
				         smem_base + (uint32_t)(slot * C::QSLOT + 1024 * (lw * C::QNI + i)));
		};
		// row terms of tile t: term 2 lw + (lane >> 5), rows 4 (lane & 31) .. +3
		// (loader waves 0 and 1, one piece each)
		auto dma_ra = [&](int t) __attribute__((always_inline)) {
			const int64_t r0 = tile_row0(t);
			const uint32_t off = (uint32_t)(raix(r0, 2 * lw + (lane >> 5)) - raix(r0 & ~(int64_t)255, 0)) * 4u +
			                     16u * (uint32_t)(lane & 31);
			rs_dma16(reinterpret_cast<const float *>(rowaux) + raix(r0 & ~(int64_t)255, 0), off,
			         smem_base + (uint32_t)(C::OFF_RA + (t & 1) * C::RA_SLOT + 1024 * lw));
		};
		// prologue: windows 0 .. NQS-2 and tile 0's row terms, all landed
		for (int v = 0; v < RS_NQS - 1 && v < G; ++v) dma_q(v);
		if (lw < 2) dma_ra(0);
		rs_wait_vm<0>();
		__syncthreads();
		int cur_s = 0, cur_t = 0;
		for (int v = 0; v < G; ++v) {
			const bool ra_now = cur_s == 1 && cur_t + 1 < my_tiles && lw < 2;
			if (ra_now) dma_ra(cur_t + 1);
			const bool issued = v + RS_NQS - 1 < G;
			if (issued) dma_q(v + RS_NQS - 1);
			// window v+1's pieces were issued in step v+2-NQS; younger: the
			// pieces of steps v+3-NQS .. v (NQS-2 windows) and a row-term
			// piece issued in one of those steps (cur_s in 1 .. NQS-2)
			if (!issued || v + 1 >= G) {
				rs_wait_vm<0>();
			} else {
				static_assert(RS_NQS == 4, "vmcnt immediates below assume 4 slots");
				const bool ra_young = lw < 2 && (cur_s == 1 || cur_s == 2) && cur_t + 1 < my_tiles;
				if (ra_young) rs_wait_vm<2 * C::QNI + 1>();
				else rs_wait_vm<2 * C::QNI>();
			}
			__syncthreads();
			if (++cur_s == S) {
				cur_s = 0;
				++cur_t;
			}
		}
		__syncthreads();  // the MFMA waves' final counter barrier
		return;
	}

	// ================= MFMA waves =================
	// row stream: lane 16g + r of row block b holds row 32w + 16b + r: bf16
	// rows bytes [16g, +16) and [64 + 16g, +16) of the window (k 8g.. and
	// 32 + 8g.., one 16x16x32 k-step each); f32 rows bytes [32g, +32) (k 8g..
	// 8g+7, one k-step)
	const int gq = lane >> 4, rr = lane & 15;
	const uint32_t xlane = (uint32_t)((RS_WR * w + rr) * rowb + (XB ? 16 : 32) * gq);
	const int64_t tile_bytes = (int64_t)RS_BR * rowb;
	const int64_t tile_step = (int64_t)gridDim.x * tile_bytes;
	const uint8_t *x_tile = X + (int64_t)blockIdx.x * tile_bytes;  // tile of the next window to load
	int x_s = 0;                                                   // its window in the tile
	float4 xr[R][2 * RS_RB];
	auto load_x = [&](float4 (&dst)[2 * RS_RB], bool live) __attribute__((always_inline)) {
		// past the workgroup's last window: a dead load of the store's first
		// tile (x_tile may already point past the last tile)
		const uint8_t *p = live ? x_tile + x_s * RS_WIN + xlane : X + xlane;
#pragma unroll
		for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
			for (int j = 0; j < 2; ++j)
				dst[2 * rb + j] = *reinterpret_cast<const float4 *>(p + (int64_t)rb * 16 * rowb + j * (XB ? 64 : 16));
		if (live && ++x_s == S) {
			x_s = 0;
			x_tile += tile_step;
		}
	};

	static_for<0, R - 1>([&](auto I) __attribute__((always_inline)) {
		load_x(xr[decltype(I)::value], decltype(I)::value < G);
	});
	__syncthreads();  // prologue: query windows, row terms, QA / TAU / CNT

	f32x4 acc[RS_RB][16];
	auto init_acc = [&](int t) __attribute__((always_inline)) {
		if (!FOLD) {
#pragma unroll
			for (int rb = 0; rb < RS_RB; ++rb)
#pragma unroll
				for (int qb = 0; qb < 16; ++qb) acc[rb][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
			return;
		}
		// acc = alpha + C + xn*B + ux*A by one exact-f32 16x16x4 MFMA per block:
		// A[row][k] = (xn, ux, alpha, 1), B[k][query] = (B, A, 1, C)
		const float *RAs = reinterpret_cast<const float *>(smem + C::OFF_RA + (t & 1) * C::RA_SLOT);
		float av[RS_RB];
#pragma unroll
		for (int rb = 0; rb < RS_RB; ++rb) {
			const int r = RS_WR * w + 16 * rb + rr;
			av[rb] = gq == 0 ? RAs[RS_BR + r] : gq == 1 ? RAs[2 * RS_BR + r] : gq == 2 ? RAs[r] : 1.0f;
		}
		const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
		for (int qb = 0; qb < 16; ++qb) {
			const float4 qa = QA[16 * qb + rr];
			const float bv = gq == 0 ? qa.z : gq == 1 ? qa.y : gq == 2 ? 1.0f : qa.w;
#pragma unroll
			for (int rb = 0; rb < RS_RB; ++rb) acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rb], bv, z, 0, 0, 0);
		}
	};

	// ---- the tile's MFMAs over one window
	auto mma = [&](const float4 (&xs)[2 * RS_RB], int slot) __attribute__((always_inline)) {
		const uint8_t *qs = smem + slot * C::QSLOT;
#pragma unroll
		for (int ks = 0; ks < C::KS; ++ks) {
			bf16x8 a[RS_RB];
#pragma unroll
			for (int rb = 0; rb < RS_RB; ++rb) {
				if (XB) {
					a[rb] = __builtin_bit_cast(bf16x8, xs[2 * rb + ks]);
				} else {
					const float4 lo = xs[2 * rb], hi = xs[2 * rb + 1];
					a[rb][0] = (__bf16)lo.x;
					a[rb][1] = (__bf16)lo.y;
					a[rb][2] = (__bf16)lo.z;
					a[rb][3] = (__bf16)lo.w;
					a[rb][4] = (__bf16)hi.x;
					a[rb][5] = (__bf16)hi.y;
					a[rb][6] = (__bf16)hi.z;
					a[rb][7] = (__bf16)hi.w;
				}
			}
#pragma unroll
			for (int qb = 0; qb < 16; ++qb) {
				const int q = 16 * qb + rr;
				const int ch = 4 * ks + gq;
				const bf16x8 b = *reinterpret_cast<const bf16x8 *>(qs + q * C::QW + C::qswz(q, ch) * 16);
#pragma unroll
				for (int rb = 0; rb < RS_RB; ++rb)
					acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rb], b, acc[rb][qb], 0, 0, 0);
			}
		}
	};
	// ---- survivors: per-wave LDS list of (raw LB bits, q << 24 | row << 16 | tile)
	uint2 *wlist = reinterpret_cast<uint2 *>(smem + C::OFF_LIST) + w * RS_WLIST;
	int n_list = 0;
	auto seg_put = [&](int qloc, float lb, int64_t slot) __attribute__((always_inline)) {
		const unsigned p = atomicAdd(&CNT[qloc], 1u);
		if (p < (unsigned)seg_cap)
			seg_pool[((int64_t)blockIdx.x * nq + q0 + qloc) * seg_cap + p] = make_uint2(fkey(lb), (uint32_t)slot);
	};
	auto flush_list = [&]() __attribute__((always_inline)) {
		for (int b = 0; b < n_list; b += 64) {
			if (b + lane < n_list) {
				const uint2 e = wlist[b + lane];
				const int qloc = (int)(e.y >> 24), rloc = (int)((e.y >> 16) & 255u), ti = (int)(e.y & 0xFFFFu);
				seg_put(qloc, __uint_as_float(e.x), tile_row0(ti) + rloc);
			}
		}
		n_list = 0;
	};

	auto epilogue = [&](int ti) __attribute__((always_inline)) {
		mfma_operand_guard();
		const float *RAs = reinterpret_cast<const float *>(smem + C::OFF_RA + (ti & 1) * C::RA_SLOT);
		auto ra4 = [&](int r0, int c) __attribute__((always_inline)) {
			return *reinterpret_cast<const float4 *>(RAs + c * RS_BR + r0);
		};
		const int64_t row0 = tile_row0(ti);
		const int eln = rs_lane_fresh();
		const int rr = eln & 15, gq = eln >> 4;  // (shadow the kernel's: recomputed per tile)
		int nl = n_list;
		static_for<0, 4>([&](auto QG) __attribute__((always_inline)) {
			constexpr int qg = decltype(QG)::value;
			float4 qa[4];
			float tq[4], tqs[4];
#pragma unroll
			for (int u = 0; u < 4; ++u) {
				const int q = 16 * (4 * qg + u) + rr;
				qa[u] = QA[q];
				tq[u] = fminf(TAU[q], F_MAX);  // tau = +inf must still drop dead rows (LB = +inf)
				tqs[u] = fmaxf(tq[u], -F_MAX);
			}
			static_for<0, RS_RB>([&](auto RB) __attribute__((always_inline)) {
				constexpr int rb = decltype(RB)::value;
				const int r0 = RS_WR * w + 16 * rb + 4 * gq;  // tile rows r0 .. r0+3 of this lane
				float l[4][4];                           // [row][query]
				if (FOLD) {
#pragma unroll
					for (int i = 0; i < 4; ++i)
#pragma unroll
						for (int u = 0; u < 4; ++u) l[i][u] = acc[rb][4 * qg + u][i];
				} else {
					const float4 al = ra4(r0, 0), xn = ra4(r0, 1), ux = ra4(r0, 2), sc = ra4(r0, 3);
#pragma unroll
					for (int u = 0; u < 4; ++u) {
						l[0][u] = rs_lower_bound<METRIC>(acc[rb][4 * qg + u][0], make_float4(al.x, xn.x, ux.x, sc.x), qa[u]);
						l[1][u] = rs_lower_bound<METRIC>(acc[rb][4 * qg + u][1], make_float4(al.y, xn.y, ux.y, sc.y), qa[u]);
						l[2][u] = rs_lower_bound<METRIC>(acc[rb][4 * qg + u][2], make_float4(al.z, xn.z, ux.z, sc.z), qa[u]);
						l[3][u] = rs_lower_bound<METRIC>(acc[rb][4 * qg + u][3], make_float4(al.w, xn.w, ux.w, sc.w), qa[u]);
					}
				}
				// screen: some l[i][u] <= tq[u] (exact sign of the rounded
				// difference; NaN never passes; see scan_kernel)
				float scr = F_MAX;
#pragma unroll
				for (int u = 0; u < 4; ++u)
					scr = fminf(scr, fminf(fminf(l[0][u], l[1][u]), fminf(l[2][u], l[3][u])) - tqs[u]);
				if (!__builtin_amdgcn_ballot_w64(scr <= 0.f)) return;
				// rare: each lane's first hit by selects, one ballot for the list
				// positions; lanes with more hits take the per-bound loop
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
					const int qv = 16 * (4 * qg + (sk & 3)) + rr, rv = r0 + (sk >> 2);
					if (nl + n1 <= RS_WLIST) {
						const int pos = nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32),
						                                               __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0u));
						if (c > 0)
							wlist[pos] = make_uint2(__float_as_uint(sv), ((uint32_t)qv << 24) | ((uint32_t)rv << 16) |
							                                                 ((uint32_t)ti & 0xFFFFu));
						nl += n1;
					} else if (c > 0) {
						seg_put(qv, sv, row0 + rv);
					}
				}
				if (__builtin_amdgcn_ballot_w64(c > 1)) {
#pragma unroll
					for (int k = 0; k < 16; ++k) {
						const bool h = l[k >> 2][k & 3] <= tq[k & 3] && k != sk;
						const uint64_t mm = __builtin_amdgcn_ballot_w64(h);
						if (!mm) continue;
						const int qv = 16 * (4 * qg + (k & 3)) + rr, rv = r0 + (k >> 2);
						const int cm = __builtin_popcountll(mm);
						if (nl + cm <= RS_WLIST) {
							const int pos = nl + __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
							                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
							if (h)
								wlist[pos] = make_uint2(__float_as_uint(l[k >> 2][k & 3]),
								                        ((uint32_t)qv << 24) | ((uint32_t)rv << 16) | ((uint32_t)ti & 0xFFFFu));
							nl += cm;
						} else if (h) {
							seg_put(qv, l[k >> 2][k & 3], row0 + rv);
						}
					}
				}
			});
		});
		n_list = nl;
		if (n_list > RS_FLUSH_AT) flush_list();
	};

	// ---- main loop: window v multiplies ring slot v % R while windows v+1 ..
	// v+R-1 stream in; unrolled by the ring so every slot is a register set.
	// A tile is a whole number of ring rounds (S % R == 0): it starts at slot
	// 0 and ends at slot R-1, so init and epilogue appear once in the code.
	int cur_s = 0, cur_t = 0;
	auto step = [&](auto SLOT) __attribute__((always_inline)) {
		constexpr int SL = decltype(SLOT)::value;
		const int v = cur_t * S + cur_s;
		if (SL == 0 && cur_s == 0) init_acc(cur_t);
#ifndef LHIP_RS_ABL_NO_XLOAD
		load_x(xr[(SL + R - 1) % R], v + R - 1 < G);  // window v+R-1
#endif
#ifndef LHIP_RS_ABL_NO_MFMA
		mma(xr[SL], v % RS_NQS);
#else
#pragma unroll
		for (int j = 0; j < 2 * RS_RB; ++j) asm volatile("" ::"v"(xr[SL][j].x));
#endif
		__syncthreads();
		++cur_s;
		if (SL == R - 1 && cur_s == S) {
#ifndef LHIP_RS_ABL_NO_EPI
			epilogue(cur_t);
#else
#pragma unroll
			for (int j = 0; j < 16; ++j) asm volatile("" ::"v"(acc[0][j][0]));
#endif
			cur_s = 0;
			++cur_t;
		}
	};
	for (int v0 = 0; v0 < G; v0 += R)
		static_for<0, R>([&](auto I) __attribute__((always_inline)) { step(I); });
	if (n_list > 0) flush_list();
	__syncthreads();  // every wave's counter updates
	if (q0 + tid < nq) seg_cnt[(int64_t)blockIdx.x * nq + q0 + tid] = (int)CNT[tid];
}

// ring depth for a store (0: the register-streamed scan does not apply)
static int rscan_ring(const StoreView &s) {
	const int64_t rowb = (int64_t)s.ld * (s.scan_bf16 ? 2 : 4);
	if (rowb % RS_WIN != 0) return 0;
	const int64_t S = rowb / RS_WIN;
	// cosine keeps per-row scale terms live through the epilogue: deeper rings
	// spill at the 168-register budget of three waves per SIMD
	for (int r : {8, 6, 4})
		if (S % r == 0 && (r == 4 || s.metric != METRIC_COSINE)) return r;
	return 0;
}

bool rscan_fits(const StoreView &s) { return !s.scan_i8 && rscan_ring(s) != 0; }

template <int METRIC, bool XB>
static void rscan_launch_r(int R, dim3 grid, hipStream_t st, const uint8_t *X, const StoreView &s, const QueryView &q,
                           int n_tiles, const float *tau, uint2 *seg_pool, int *seg_cnt, int seg_cap) {
#define LHIP_RS(RR)                                                                                                  \
	rscan_kernel<METRIC, XB, RR><<<grid, RS_THREADS, 0, st>>>(X, s.rowaux, s.ld, q.Qb, q.qaux, q.nq, n_tiles, tau, \
	                                                          seg_pool, seg_cnt, seg_cap)
	if (R == 8) LHIP_RS(8);
	else if (R == 6) LHIP_RS(6);
	else LHIP_RS(4);
#undef LHIP_RS
}

void launch_rscan_append(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                         int seg_cap, hipStream_t st) {
	if (s.n_slots <= 0) return;
	const int R = rscan_ring(s);
	if (!R) throw std::runtime_error("rscan: row bytes must be a multiple of 512");
	if (seg_cap <= 0 || seg_cap > 1024) throw std::runtime_error("rscan: segment capacity must be in [1, 1024]");
	// the selection reads scan_grid(256-row tiles) segments per query: launch
	// exactly that many workgroups and spread the 128-row tiles over them
	const int grid_x = scan_grid((s.n_slots + SCAN_BR - 1) / SCAN_BR);
	const int64_t n_tiles = (s.n_slots + RS_BR - 1) / RS_BR;  // the store is zero / +inf padded to 256 rows
	if ((n_tiles + grid_x - 1) / grid_x >= 65536)
		throw std::runtime_error("rscan: more than 65535 tiles per workgroup");  // 16-bit tile index in list entries
	dim3 grid((unsigned)grid_x, (unsigned)(q.nq_pad / SCAN_BQ));
	const uint8_t *X = static_cast<const uint8_t *>(s.Xscan);
	if (s.scan_bf16) {
		if (s.metric == METRIC_L2) rscan_launch_r<METRIC_L2, true>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
		else if (s.metric == METRIC_DOT) rscan_launch_r<METRIC_DOT, true>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
		else rscan_launch_r<METRIC_COSINE, true>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
	} else {
		if (s.metric == METRIC_L2) rscan_launch_r<METRIC_L2, false>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
		else if (s.metric == METRIC_DOT) rscan_launch_r<METRIC_DOT, false>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
		else rscan_launch_r<METRIC_COSINE, false>(R, grid, st, X, s, q, (int)n_tiles, tau, seg_pool, seg_cnt, seg_cap);
	}
}

}  // namespace lhip
