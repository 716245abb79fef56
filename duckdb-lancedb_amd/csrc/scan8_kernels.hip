// gfx950 (MI355X / CDNA4): the int8 append pass of the flat scan ("scan8").
//
// Replaces, for the int8 scan copy, the threshold pass of knn_kernels.hip's
// scan_kernel (MODE 1): every row's rigorous lower bound LB(row, query) is
// screened against tau[query] and the rows with LB <= tau go to the query's
// segment as (orderedkey(LB), slot).  The search it serves is the reference's
// flat KNN (rust_lib/src/lance_manager.rs:393-451 -> lance 0.22 flat scan);
// DESIGN.md §3 "scan8" has the derivation.
//
// Layout (one workgroup per CU, two per pair of CUs):
//   * a PAIR of workgroups walks the same row tiles (pair p: tiles p, p + NP, ...),
//     each with one half of a 256-query tile: its 128 int8 queries stay RESIDENT
//     in LDS for the whole launch (128 x ld bytes; ld = 768: 96 KiB), so nothing
//     but rows streams.  The partner's copy of a row comes from L2 / the
//     Infinity Cache (workgroups b and b + 8 share an XCD under round-robin
//     placement: speed only, never correctness).
//   * 8 waves, two per SIMD, no barrier after the prologue: wave w owns rows
//     32w .. 32w + 31 of every tile of its pair and all 128 queries,
//     2 x 8 v_mfma_i32_16x16x64_i8 accumulators (64 VGPRs).  Its rows stream
//     HBM -> VGPRs (global_load_dwordx4, 16 rows x 64 B per instruction) through
//     a D-deep register ring of 64-deep k-steps; query fragments come from LDS
//     (XOR-swizzled 16 B chunks: conflict-free ds_read_b128).
//   * the bound is screened in EXACT INTEGERS.  With one scale s_T per row tile
//     and one s_Q per query batch (tiles_to_i8_kernel, prep_queries_i8_kernel),
//       LB = alpha + C + xn B + ux A + s s_T S      (s = x^.q^ exact, S < 0)
//     and LB <= tau  <=>  s >= (alpha + C + xn B + ux A - tau) W,  W = 1/(-S s_T);
//     with xn, ux replaced by the tile's maxima (B, A <= 0: the threshold only
//     drops) it splits into a row part Bi <= alpha W and a query part
//     Gi <= (C + max xn B + max ux A - tau) W, both rounded DOWN to integers.
//     The accumulators start at -Bi (the first MFMA's C operand) and a bound
//     passes iff acc >= Gi: per lane and query block one v_max3 chain and one
//     compare.  Every (row, query) with LB <= tau passes (a superset; the
//     passes that exceed tau only cost a segment entry).
//   * a passing bound is kept in the wave's LDS list as (s, slot, query); the
//     list becomes (orderedkey(LB), slot) segment entries at the end (or when it
//     fills): LB is evaluated there exactly as scan_kernel's lower_bound does,
//     from the row terms in global memory.
// ---------------------------------------------------------------------------
#include "knn_kernels.h"

#include <algorithm>
#include <atomic>
#include <stdexcept>

#include "device_common.h"

namespace lhip {

namespace {
constexpr int QH = 128;               // queries per workgroup (half a SCAN_BQ tile)
constexpr int LDS8 = 160 * 1024;      // one workgroup per CU
constexpr int BIG = 1 << 30;          // row part of a dead row / query part that passes nothing
constexpr int LIVE_MAX = 1 << 29;     // largest row part of a live row
constexpr int GLO = -(1 << 29) - (1 << 25);  // query part that passes every live row
static_assert(BIG - (1 << 24) > -GLO, "a dead row (acc <= 2^24 - BIG) never reaches GLO");
static_assert(-(1 << 24) - LIVE_MAX > GLO, "a live row (acc >= -2^24 - LIVE_MAX) always reaches GLO");
}  // namespace



// row part: an integer Bi <= alpha * W (exact), in [0, LIVE_MAX]; BIG for a dead
// row (+inf) or a NaN bound (never passes, as in scan_kernel).  Branch-free: the
// per-block terms are selects, not exec-masked blocks.
__device__ __forceinline__ int s8_row_part(float alpha, float W) {
	float b = alpha * W;                          // alpha >= 0, W >= 0 (NaN: 0 * inf -> 0 below)
	b = fmaf(-fabsf(b), 0x1p-20f, b) - 1.0f;      // below alpha W despite the two roundings
	b = fminf(fmaxf(b, 0.0f), (float)LIVE_MAX);   // (fmaxf drops a NaN)
	return alpha < F_INF ? (int)b : BIG;
}

// query terms, once per query: qp = (C - tau, A, B, |C| + |tau|) from the
// query's (S, A, B, C) and tau
__device__ __forceinline__ float4 s8_query_terms(float4 qa, float tq) {
	return make_float4(qa.w - tq, qa.y, qa.z, fabsf(qa.w) + fabsf(tq));
}

// query part: an integer Gi <= (C - tau + xnmax B + uxmax A) W (exact), in
// [GLO, BIG]; BIG (nothing passes) for a NaN query term or tau (a zero cosine
// query, a NaN distance in the sample: exact fallback) and for padding queries
// (tau = -inf); GLO (every live row passes) when it overflows or tau = +inf
__device__ __forceinline__ int s8_query_part(float4 qp, float4 ts, float W) {
	float g = fmaf(ts.y, qp.z, fmaf(ts.z, qp.y, qp.x)) * W;
	// f32 evaluation error of the four terms (a few units of 2^-24 of their magnitudes)
	const float E = (qp.w + ts.y * fabsf(qp.z) + ts.z * fabsf(qp.y)) * W * 0x1p-20f + 1.0f;
	g = g - E;
	const int r = fabsf(g) < F_INF ? (int)floorf(fminf(fmaxf(g, (float)GLO), (float)BIG)) : GLO;
	return qp.x < F_INF ? r : BIG;
}

// ABL (timing ablations, wrong results): bit 0 skips the screen, bit 1 the
// per-block bound terms (constants instead), bit 2 the appends, bit 6 the appends
// kept in the code but never taken; bit 3 (a speed option, results exact):
// s_setprio 2 over the k-loop, 0 over the rest
//
// TM = 1: the SAMPLE pass instead (tilemin: row tile t of the launch is tile
// tile0 + t * tstride): no threshold, the accumulators hold s; per work unit
// (32 rows) and query the row of smallest score alpha - s_T |S| s (the bound's
// row-dependent terms), (orderedkey(score), slot), goes to the workgroup's
// segment (dead rows skipped): 8 entries per tile and query from which
// pool_refine's tau mode refines the k + 8 smallest exactly.
// Pair coupling (couple > 0, speed only — results never depend on it): the two
// workgroups of a pair read the same rows, the second from L2 only while the
// first's copy is still there; left alone they drift apart (at 10M rows the
// partner's reads miss L2: FETCH 1.22x the algorithmic bytes).  Each workgroup
// publishes the highest unit it has claimed (prog[b], tagged with the launch's
// epoch in the high word, atomicMax at agent scope) and a wave does not start a
// unit more than `couple` units ahead of its partner's; the wait is bounded
// (S8_COUPLE_SPINS sleeps, then the wave stops waiting), so a partner that is
// not resident (another kernel on its CU) costs time, never progress.
constexpr int S8_COUPLE_SPINS = 2048;
template <int KS, int D, int RB, int ABL = 0, int TM = 0>
__global__ __launch_bounds__(64 * (16 / RB), 1) void scan8_kernel(const int8_t *__restrict__ Xq, const float4 *__restrict__ aux8,
                                                      const float4 *__restrict__ tstat, int ld,
                                                      const int8_t *__restrict__ Qi, const float4 *__restrict__ qaux,
                                                      int nq, int n_tiles, int tile0, int seg_base,
                                                      const float *__restrict__ tau,
                                                      uint2 *__restrict__ seg_pool, int *__restrict__ seg_cnt,
                                                      int seg_cap, int list_cap, int tstride,
                                                      unsigned long long *__restrict__ prog, unsigned epoch,
                                                      int couple) {
	static_assert(KS % D == 0 && KS % 2 == 0, "ring slot and fragment buffer of a k-step must be static");
	constexpr int NW = 16 / RB, T8 = 64 * NW;  // waves: each owns 16 RB rows of every tile
	constexpr int WR = 16 * RB;                // rows per wave and tile
	constexpr int P = (KS * 64 + 255) / 256 * 256;  // LDS bytes per query row (XOR groups of 16 chunks)
	__shared__ __attribute__((aligned(16))) uint8_t smem[LDS8];
	uint8_t *QL = smem;
	float4 *QA = reinterpret_cast<float4 *>(smem + QH * P);
	float4 *QP = QA + QH;  // s8_query_terms of each query
	unsigned *CNT = reinterpret_cast<unsigned *>(QP + QH);
	unsigned *UCNT = CNT + QH;                                          // next unclaimed unit (+3 pad words)
	uint2 *LIST = reinterpret_cast<uint2 *>(CNT + QH + 4);             // [NW][list_cap] (s, slot)
	uint8_t *LISTQ = reinterpret_cast<uint8_t *>(LIST + NW * list_cap);  // [NW][list_cap] local query

	// Row group and query half of this workgroup.  A query tile with more than
	// QH queries: pairs (workgroups b, b + 8 share an XCD under round-robin
	// placement), each pair one row group, each workgroup one half; otherwise
	// (a small batch, a rerun) every workgroup its own row group, all queries.
	const int nb = (int)gridDim.x, b_id = (int)blockIdx.x;
	const int q_tile = (int)blockIdx.y * SCAN_BQ;
	const bool halves = nq - q_tile > QH;
	int h = 0, pr = b_id, NP = nb;
	if (halves) {
		NP = nb >> 1;
		if ((nb & 15) == 0) {
			h = (b_id >> 3) & 1;
			pr = (b_id & 7) | ((b_id >> 4) << 3);
		} else {
			h = b_id & 1;
			pr = b_id >> 1;
		}
	}
	const int qb = q_tile + h * QH;  // first query of this workgroup
#ifdef LHIP_S8_PROF
	const uint64_t rt_start = __builtin_amdgcn_s_memrealtime();  // (100 MHz: comparable across workgroups)
#endif
	const int tid = threadIdx.x, lane = tid & 63;
	const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
	const int lr = lane & 15, lg = lane >> 4;

	// ---- prologue: the 128 queries into LDS (chunk c of query n at c ^ (n & 15)) --
	// every load of the prologue in flight together (a load-wait-store loop paid
	// one L2 round trip per 16 B chunk step: 12 of them at ld = 768, ~10 us)
	{
		constexpr int NCH = KS * 4;          // 16 B chunks per query row
		constexpr int PER = QH * NCH / T8;   // chunks per thread
		static_assert(QH * NCH % T8 == 0, "whole chunk steps per thread");
		float4 qa = make_float4(0.f, 0.f, 0.f, 0.f);
		float tq = -F_INF;
		if (tid < QH) {
			const int q = qb + tid;
			qa = qaux[q];
			if (TM == 0 && q < nq) tq = tau[q];
		}
		i32x4 v[PER];
#pragma unroll
		for (int j = 0; j < PER; ++j) {
			const int i = tid + j * T8, n = i / NCH, c = i - n * NCH;
			v[j] = *reinterpret_cast<const i32x4 *>(Qi + (int64_t)(qb + n) * 2 * ld + 16 * c);
		}
#pragma unroll
		for (int j = 0; j < PER; ++j) {
			const int i = tid + j * T8, n = i / NCH, c = i - n * NCH;
			*reinterpret_cast<i32x4 *>(QL + n * P + ((c ^ (n & 15)) << 4)) = v[j];
		}
		if (tid < QH) {
			QA[tid] = qa;
			QP[tid] = s8_query_terms(qa, tq);
			CNT[tid] = 0u;
		}
	}
	if (tid == 0) *UCNT = (unsigned)NW;  // units 0 .. NW-1: one per wave, the rest claimed
	__syncthreads();
	// -S: the same for every query with a usable bound (0 for padding / zero cosine queries)
	float Sabs = fmaxf(-QA[lane].x, -QA[lane + 64].x);
#pragma unroll
	for (int o = 32; o > 0; o >>= 1) Sabs = fmaxf(Sabs, __shfl_xor(Sabs, o, 64));

	const int my_tiles = pr < n_tiles ? (n_tiles - 1 - pr) / NP + 1 : 0;
	// Work units: a unit = WR rows of one of this workgroup's tiles (unit u: tile
	// u / NW, rows WR (u % NW) ..) against its QH queries.  Wave w starts on unit
	// w and claims later ones from an LDS counter, two ahead (the claim's result
	// is read a block later: no wait): the waves of a SIMD share its issue and
	// the older one wins arbitration, so a fixed split (wave w: rows WR w of every
	// tile) left the younger half ~40 % behind, running the end of every launch
	// alone, one wave per SIMD.
	const int NU = my_tiles * NW;
	int n_list = 0;
#ifdef LHIP_S8_PROF
	// diagnostic build: per-wave cycles in each phase of the block loop
	uint64_t pf_pro = 0, pf_k = 0, pf_scr = 0, pf_app = 0, pf_t = 0;
	int pf_hitb = 0;
#define S8_T(acc)                                            \
	{                                                        \
		const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
		acc += now_ - pf_t;                                  \
		pf_t = now_;                                         \
	}
#else
#define S8_T(acc)
#endif
	uint2 *wl = LIST + w * list_cap;
	uint8_t *wq = LISTQ + w * list_cap;
	// list -> segment entries: LB as scan_kernel's lower_bound<., SC> evaluates it
	auto flush = [&]() {
		const float *ra = reinterpret_cast<const float *>(aux8);
		for (int e = lane; e < n_list; e += 64) {
			const uint2 en = wl[e];
			const int ql = wq[e];
			const int64_t r = (int64_t)en.y;
			const float al = ra[raix(r, 0)], xn = ra[raix(r, 1)], ux = ra[raix(r, 2)], sc = ra[raix(r, 3)];
			const float4 qa = QA[ql];
			float v = fmaf(xn, qa.z, al);
			v = fmaf(ux, qa.y, v);
			v = fmaf((float)(int)en.x * sc, qa.x, v);
			v = v + qa.w;
			const unsigned p = atomicAdd(&CNT[ql], 1u);
			if (p < (unsigned)seg_cap)
				seg_pool[((int64_t)(seg_base + b_id) * nq + qb + ql) * seg_cap + p] = make_uint2(fkey(v), en.y);
		}
		n_list = 0;
	};

	if (w < NU) {
		// this lane's A rows: WR (u % NW) + 16 rb + lr of the unit's tile, k bytes
		// 64 j + 16 lg, in the k-major tile layout (tiles_to_i8_kernel): a k-step of
		// 16 rows is 1 KiB contiguous.  Address = uniform unit base + 16 KiB j
		// (SGPRs) + per-lane offset: no VALU in the k-loop (a VALU write right after
		// an MFMA may land on one of its A / B registers while it still reads them:
		// device_common.h)
		uint32_t xo[RB];
#pragma unroll
		for (int rb = 0; rb < RB; ++rb) xo[rb] = (uint32_t)((16 * rb + lr) * 64 + 16 * lg);
		auto utile = [&](int u) -> int64_t { return tile0 + (pr + (int64_t)(u / NW) * NP) * (TM ? tstride : 1); };
		auto xunit = [&](int u) -> const int8_t * {
			return Xq + utile(u) * SCAN_BR * (int64_t)ld + (int64_t)(WR * (u % NW)) * 64;
		};
		auto xload = [&](const int8_t *tb, int j, int rb) -> i32x4 {
			return *reinterpret_cast<const i32x4 *>(tb + (int64_t)j * I8_CHUNK_STRIDE + xo[rb]);
		};
		// row terms of a unit: the alpha of ONE of its WR rows per lane (row lane %
		// WR; its row part is handed to the accumulator lanes of that row by
		// ds_bpermute: 16 lanes share each accumulator row) and the tile's terms.
		// (the tile terms by a vector load: a scalar load in flight forces
		// lgkmcnt(0) (SMEM returns out of order) at the block's first LDS wait)
		uint32_t vz;
		asm volatile("v_mov_b32 %0, 0" : "=v"(vz));  // a zero the compiler cannot see is uniform
		auto aload = [&](int u, float &a, float4 &ts) {
			const int64_t tile = utile(u);
			a = reinterpret_cast<const float *>(aux8)[(tile << 10) + WR * (u % NW) + (lane & (WR - 1))];
			ts = tstat[tile + vz];
		};
		auto claim = [&]() -> int {  // (lane 0's LDS atomic; read by readfirstlane where used)
			unsigned v = 0;
			if (lane == 0) v = atomicAdd(UCNT, 1u);
			return (int)v;
		};
		// B fragment of query block u, k-step j: query 16u + lr, logical chunk 4j + lg
		// (two base registers per j & 3 keep every offset an immediate below 64 KiB)
		uint32_t qo[2][4];
#pragma unroll
		for (int m = 0; m < 4; ++m) {
			qo[0][m] = (uint32_t)(lr * P + ((((4 * m + lg) ^ lr)) << 4));
			qo[1][m] = qo[0][m] + 64u * P;
			asm volatile("" : "+v"(qo[1][m]));  // a register of its own (not re-folded into an add per read)
		}
		auto bload = [&](int j, int u) -> i32x4 {
			return *reinterpret_cast<const i32x4 *>(QL + qo[u >> 2][j & 3] + 16 * (u & 3) * P + 256 * (j >> 2));
		};

		// the query terms of queries lane and lane + 64 (this lane's query parts,
		// handed to the accumulator lanes of column 16 u + lr by ds_bpermute)
		const float4 qp0 = QP[lane], qp1 = QP[lane + 64];
		// pair coupling: only for pairs on one XCD (b, b ^ 8: the (nb & 15) == 0 layout),
		// and in the ld <= 768 geometries (KS <= 12): the deeper register rings of
		// ld 896 / 1024 have no room for its state (a 12-B spill)
		const bool cpl = KS <= 12 && couple > 0 && prog && halves && (nb & 15) == 0;
		const uint64_t etag = (uint64_t)epoch << 32;
		int pseen = -1, spins = cpl ? S8_COUPLE_SPINS : 0;  // partner's unit last seen; sleeps left
		auto publish = [&](int u) {
			if (cpl && lane == 0) __hip_atomic_fetch_max(prog + b_id, etag | (uint32_t)u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		};
		auto await_partner = [&](int u) {  // before this wave's loads of unit u
			while (spins > 0 && u - couple > pseen) {
				uint64_t v = 0;
				if (lane == 0) v = __hip_atomic_load(prog + (b_id ^ 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
				const int pv = (v >> 32) == (uint64_t)epoch ? (int)(uint32_t)v : -1;
				pseen = __builtin_amdgcn_readfirstlane(pv);
				if (u - couple <= pseen) break;
				__builtin_amdgcn_s_sleep(8);
				--spins;
			}
		};
		int unit = w;                                        // this block's unit
		publish(unit);
		await_partner(unit);
		int unext = __builtin_amdgcn_readfirstlane(claim()); // the next one (>= NU: none)
		publish(unext);
		float an;
		float4 tn;
		aload(unit, an, tn);
		// complete on the entry path: the block loop carries an[] as plain copies,
		// and a pending load merged into its header made the waitcnt pass drain
		// every in-flight ring load at each block start
		__builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding: expcnt 7, lgkmcnt 15 = no wait)
		i32x4 xa[D][RB];
		{
			// issued in ring order, as the block loop refills it: the waitcnt pass
			// merges this path into the loop header, and a reordered entry (slot 0
			// youngest) made it wait for every ring load at each block's first MFMA
			const int8_t *tb = xunit(unit);
#pragma unroll
			for (int j = 0; j < D; ++j) {
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) xa[j][rb] = xload(tb, j, rb);
				__builtin_amdgcn_sched_barrier(0);
			}
		}
		// query fragments, double-buffered: k-step j + 1's are read while k-step j multiplies
		i32x4 bq[2][8];
#pragma unroll
		for (int q8 = 0; q8 < 8; ++q8) bq[0][q8] = bload(0, q8);

#ifdef LHIP_S8_PROF
		pf_t = __builtin_amdgcn_s_memtime();
#endif
		for (;;) {
			const int unn_raw = claim();        // the unit after next (read at this block's end)
			const int ux = unext < NU ? unext : unit;  // past the end: this unit's rows again (unused)
			if (cpl) {
				publish(__builtin_amdgcn_readfirstlane(unn_raw));
				if (unext < NU) await_partner(unext);  // (its rows stream during this block)
			}
			const float al = an;
			const float4 ts = tn;
			aload(ux, an, tn);
			const float W = (Sabs > 0.f && ts.x > 0.f) ? 1.0f / (Sabs * ts.x) : 0.f;
			i32x4 bias[RB];
			int gi[8];
			if (TM) {  // the sample pass: plain s in the accumulators
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) bias[rb] = i32x4{0, 0, 0, 0};
#pragma unroll
				for (int u = 0; u < 8; ++u) gi[u] = BIG;
			} else if (ABL & 2) {
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) bias[rb] = i32x4{rb, 1, 2, 3};
#pragma unroll
				for (int u = 0; u < 8; ++u) gi[u] = BIG - u;
			} else {
				const int bl = -s8_row_part(al, W);  // row lane % WR
#pragma unroll
				for (int rb = 0; rb < RB; ++rb)
#pragma unroll
					for (int i = 0; i < 4; ++i) bias[rb][i] = __builtin_amdgcn_ds_bpermute(4 * (16 * rb + 4 * lg + i), bl);
				const int g0 = s8_query_part(qp0, ts, W), g1 = s8_query_part(qp1, ts, W);
#pragma unroll
				for (int u = 0; u < 8; ++u) gi[u] = __builtin_amdgcn_ds_bpermute(4 * ((16 * u + lr) & 63), u < 4 ? g0 : g1);
			}

			// accumulators start at -Bi (copies, then every MFMA accumulates in place:
			// a bias operand shared by 8 MFMAs made the compiler rename them per k-step)
			i32x4 acc[RB][8];
#pragma unroll
			for (int rb = 0; rb < RB; ++rb)
#pragma unroll
				for (int u = 0; u < 8; ++u) acc[rb][u] = bias[rb];
			const int8_t *tb_cur = xunit(unit), *tb_next = xunit(ux);
			S8_T(pf_pro);
			if (ABL & 8) __builtin_amdgcn_s_setprio(2);  // the k-loop: MFMA issue first on the SIMD
			__builtin_amdgcn_sched_barrier(0);
#pragma unroll
			for (int j = 0; j < KS; ++j) {
				const int sl = j % D, cur = j & 1;  // (KS even: k-step 0 of the next block reads buffer 0)
#pragma unroll
				for (int u = 0; u < 8; ++u) bq[cur ^ 1][u] = bload((j + 1) % KS, u);
#pragma unroll
				for (int u = 0; u < 8; ++u) {
#pragma unroll
					for (int rb = 0; rb < RB; ++rb)
						acc[rb][u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[sl][rb], bq[cur][u], acc[rb][u], 0, 0, 0);
				}
				// refill the slot with k-step j + D of this wave's stream
				const int jn = j + D;
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) xa[sl][rb] = xload(jn < KS ? tb_cur : tb_next, jn % KS, rb);
				__builtin_amdgcn_sched_barrier(0);
			}
			mfma_operand_guard();  // the screen's VALU follows the block's last MFMAs
			S8_T(pf_k);
			if (ABL & 8) __builtin_amdgcn_s_setprio(0);  // screen, appends, next terms: behind the partner's MFMAs

			if (TM) {
				// per query: the row of smallest SCORE among this unit's WR rows (this
				// lane: rows 16 rb + 4 lg + i, query 16 u + lr; then across the four
				// lane groups).  The sample only picks which rows the tau-mode refine
				// computes exactly (tau = the k-th exact distance among real rows is an
				// upper bound whichever rows they are), so the score keeps the two terms
				// that separate rows of one tile for one query: alpha - (s_T |S|) s
				// (|S| is common to the batch, s_T to the tile; the error terms and C
				// barely move within a tile): two instructions per bound, not six
				const float *ra = reinterpret_cast<const float *>(aux8);
				const int64_t rbase = utile(unit) * SCAN_BR + (int64_t)(WR * (unit % NW));
				float4 al4[RB];
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) al4[rb] = *reinterpret_cast<const float4 *>(ra + raix(rbase + 16 * rb + 4 * lg, 0));
				const float cs = -ts.x * Sabs;  // -(s_T |S|) (ts: this unit's tile terms)
#pragma unroll
				for (int u = 0; u < 8; ++u) {
					float bv = F_INF;
					int bi = 0;
#pragma unroll
					for (int rb = 0; rb < RB; ++rb)
#pragma unroll
						for (int i = 0; i < 4; ++i) {
							const float a_ = i == 0 ? al4[rb].x : i == 1 ? al4[rb].y : i == 2 ? al4[rb].z : al4[rb].w;
							const float v = fmaf(cs, (float)acc[rb][u][i], a_);
							const bool lt = v < bv;  // (+inf alpha: a dead row, never picked; NaN never less)
							bv = lt ? v : bv;
							bi = lt ? 16 * rb + i : bi;
						}
					uint64_t best = ((uint64_t)fkey(bv) << 32) | (uint32_t)(rbase + 4 * lg + bi);
#pragma unroll
					for (int o = 16; o < 64; o <<= 1) {
						const uint64_t ob = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), o, 64) << 32) |
						                    (uint32_t)__shfl_xor((int)(uint32_t)best, o, 64);
						best = ob < best ? ob : best;
					}
					if (lg == 0 && (uint32_t)(best >> 32) < KEY_INF && qb + 16 * u + lr < nq) {
						const unsigned p = atomicAdd(&CNT[16 * u + lr], 1u);
						if (p < (unsigned)seg_cap)
							seg_pool[((int64_t)(seg_base + b_id) * nq + qb + 16 * u + lr) * seg_cap + p] =
							    make_uint2((uint32_t)(best >> 32), (uint32_t)best);
					}
				}
				if (unext >= NU) break;
				unit = unext;
				unext = __builtin_amdgcn_readfirstlane(unn_raw);
				continue;
			}
			// ---- screen: lane bit u = some bound of query 16u + lr passes ----
			int hitm = 0;
			if (ABL & 1) {
				int m = 0;
#pragma unroll
				for (int u = 0; u < 8; ++u) m ^= acc[0][u][0];
				hitm = m == 0x7fffffff ? 1 : 0;  // (keeps the MFMAs alive)
			} else
#pragma unroll
			for (int u = 0; u < 8; ++u) {
				int m = max(max(acc[0][u][0], acc[0][u][1]), max(acc[0][u][2], acc[0][u][3]));
#pragma unroll
				for (int rb = 1; rb < RB; ++rb)
					m = max(m, max(max(acc[rb][u][0], acc[rb][u][1]), max(acc[rb][u][2], acc[rb][u][3])));
				hitm |= (m >= gi[u] ? 1 : 0) << u;
			}
			if (ABL & 64) {  // append code kept, never taken (hit mask through an opaque zero)
				int z = 0;
				asm volatile("v_mov_b32 %0, 0" : "=v"(z));
				hitm &= z;
			}
			S8_T(pf_scr);
#ifdef LHIP_S8_PROF
			pf_hitb += __builtin_amdgcn_ballot_w64(hitm != 0) ? 1 : 0;
#endif
			if (ABL & 4) {
				if (__builtin_amdgcn_ballot_w64(hitm != 0) == 0x123456789ull) n_list += 1;  // (keeps the screen)
			} else if (__builtin_amdgcn_ballot_w64(hitm != 0)) {
				// rare: append every passing (s, slot, query) to the wave's list
				const uint32_t row0 = (uint32_t)(utile(unit) * SCAN_BR) + (uint32_t)(WR * (unit % NW)) + 4u * lg;
#pragma unroll
				for (int u = 0; u < 8; ++u) {
					if (!__builtin_amdgcn_ballot_w64((hitm >> u) & 1)) continue;
					// this query block's passing bounds (one ballot per accumulator
					// register), then ONE list-room check: a flush site per u, not per
					// (rb, i) (64 inlined flushes made the kernel ~4x larger than its
					// loop).  (A per-lane mask + wave prefix scan instead of the ballots
					// measured slower: six dependent ds_bpermute per hit block.)
					uint64_t mk[RB][4];
					unsigned cu = 0;
#pragma unroll
					for (int rb = 0; rb < RB; ++rb)
#pragma unroll
						for (int i = 0; i < 4; ++i) {
							mk[rb][i] = __builtin_amdgcn_ballot_w64(acc[rb][u][i] >= gi[u]);
							cu += (unsigned)__builtin_popcountll(mk[rb][i]);
						}
					if (n_list + (int)cu > list_cap) flush();
					if ((int)cu > list_cap) {
						// more than the whole list: these queries fail their certificate
						// (a segment count past seg_cap), never a silent drop
						if ((hitm >> u) & 1) atomicOr(&CNT[16 * u + lr], 1u << 30);  // sticky: > any seg_cap
						continue;
					}
#pragma unroll
					for (int rb = 0; rb < RB; ++rb)
#pragma unroll
						for (int i = 0; i < 4; ++i) {
							const uint64_t m = mk[rb][i];
							if (!m) continue;
							if ((m >> lane) & 1) {
								const int pos = n_list + (int)__builtin_amdgcn_mbcnt_hi(
								                             (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
								wl[pos] = make_uint2((uint32_t)(acc[rb][u][i] - bias[rb][i]), row0 + 16u * rb + (uint32_t)i);
								wq[pos] = (uint8_t)(16 * u + lr);
							}
							n_list += __builtin_popcountll(m);
						}
				}
			}
			S8_T(pf_app);
			if (unext >= NU) break;
			unit = unext;
			unext = __builtin_amdgcn_readfirstlane(unn_raw);
		}
	}
#ifdef LHIP_S8_PROF
	const int nl_end = n_list;
#endif
	if (n_list > 0) flush();
#ifdef LHIP_S8_PROF
	uint64_t pf_fl = 0;
	S8_T(pf_fl);
	const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
	if (b_id < 3 && lane == 0)
		printf("S8 wg=%d w=%d blocks=%d pro=%d k=%d scr=%d app=%d flush=%d list_end=%d hitblocks=%d rt=%d\n", b_id, w,
		       my_tiles, (int)pf_pro, (int)pf_k, (int)pf_scr, (int)pf_app, (int)pf_fl, nl_end, pf_hitb,
		       (int)(rt_end - rt_start));
#endif
	__syncthreads();  // every wave's counter updates
	// segment b_id of every query of the tile: this workgroup's counts for its
	// half, zero for the other half (its partner fills its own segment)
	for (int i = tid; i < SCAN_BQ; i += T8) {
		const int q = q_tile + i;
		if (q >= nq) break;
		const int ql = q - qb;
		seg_cnt[(int64_t)(seg_base + b_id) * nq + q] = (ql >= 0 && ql < QH) ? (int)CNT[ql] : 0;
	}
}

// workgroups of a launch over n_tiles row tiles: one per CU, an even count
// (pairs), at most two per tile
static int s8_groups(int64_t n_tiles) {
	// (a function-local static: initialised once, thread-safe, C++11)
	static const int cus = [] {
		int dev = 0, v = 0;
		return (hipGetDevice(&dev) == hipSuccess &&
		        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v >= 2)
		           ? v
		           : 256;
	}();
	return (int)(2 * std::max<int64_t>(1, std::min<int64_t>(cus / 2, n_tiles)));
}

bool scan8_fits(const StoreView &s) {
	return s.scan_i8 && s.tstat && s.ld >= 512 && s.ld <= 1024 && s.ld % 128 == 0;
}

int scan8_segments(int64_t n_tiles) { return s8_groups(n_tiles); }

static int s8_list_cap(int ld, int nw) {
	const int P = (ld + 255) / 256 * 256;
	const int room = LDS8 - QH * P - QH * 36 - 16;  // QA, QP, CNT, the unit counter
	return std::min(1024, room / (nw * 9) / 64 * 64);
}

// progress words a launch's pair coupling needs (StoreView::s8_prog)
int scan8_prog_words() { return 2048; }

template <int KS, int D, int RB, int ABL = 0, int TM = 0>
static void s8_launch(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                      int seg_cap, int64_t t0, int64_t n_tiles, int seg_base, hipStream_t st, int tstride = 1) {
#ifndef LHIP_ABLATION_BUILD
	static_assert(ABL == 0, "scan8 ablations (wrong results) exist only in LHIP_ABLATION_BUILD builds");
#endif
	const dim3 grid((unsigned)s8_groups(n_tiles), (unsigned)(q.nq_pad / SCAN_BQ));
	constexpr int NW = 16 / RB;
	// a launch's coupling words are tagged with a process-unique epoch (launches
	// sharing the buffer run in order on one stream; a stale word never matches)
	static std::atomic<unsigned> epochs{1u};
	const bool cpl = s.s8_couple > 0 && s.s8_prog && grid.y == 1 && (int)grid.x <= scan8_prog_words();
	const unsigned ep = cpl ? epochs.fetch_add(1u) : 0u;
	scan8_kernel<KS, D, RB, ABL, TM><<<grid, dim3(64 * NW), 0, st>>>(
	    static_cast<const int8_t *>(s.Xscan), s.scan_aux, s.tstat, s.ld, reinterpret_cast<const int8_t *>(q.Qb), q.qaux,
	    q.nq, (int)n_tiles, (int)t0, seg_base, tau, seg_pool, seg_cnt, seg_cap, s8_list_cap(s.ld, NW), tstride,
	    cpl ? s.s8_prog : nullptr, ep, cpl ? s.s8_couple : 0);
}

int scan8_tilemin_cap(int64_t n_tiles) {
	const int groups = s8_groups(n_tiles);
	const int64_t per = (n_tiles + groups / 2 - 1) / (groups / 2);  // tiles per pair (or per workgroup)
	return (int)round_up(8 * per, 4);  // 8 units of 32 rows per tile, one entry per unit and query
}

void launch_scan8_tilemin(const StoreView &s, const QueryView &q, int64_t n_tiles, int64_t tile_stride, uint2 *seg_pool,
                          int *seg_cnt, int seg_cap, hipStream_t st) {
	if (n_tiles <= 0) return;
	if (!scan8_fits(s)) throw std::runtime_error("scan8: int8 scan copy with ld in [512, 1024] required");
	const int64_t all_tiles = (s.n_slots + SCAN_BR - 1) / SCAN_BR;
	if ((n_tiles - 1) * tile_stride >= all_tiles) throw std::runtime_error("scan8 tilemin: tile range");
	if (all_tiles * (int64_t)SCAN_BR > ((int64_t)1 << 32)) throw std::runtime_error("scan8: slots past 2^32");
	if (q.nq_pad % SCAN_BQ) throw std::runtime_error("scan8: query tile padding");
	if (seg_cap < scan8_tilemin_cap(n_tiles)) throw std::runtime_error("scan8 tilemin: segment capacity");
	const int ts = (int)tile_stride;
	switch (s.ld / 64) {
	case 8: s8_launch<8, 4, 2, 0, 1>(s, q, nullptr, seg_pool, seg_cnt, seg_cap, 0, n_tiles, 0, st, ts); break;
	case 10: s8_launch<10, 5, 2, 0, 1>(s, q, nullptr, seg_pool, seg_cnt, seg_cap, 0, n_tiles, 0, st, ts); break;
	case 12: s8_launch<12, 4, 2, 0, 1>(s, q, nullptr, seg_pool, seg_cnt, seg_cap, 0, n_tiles, 0, st, ts); break;
	case 14: s8_launch<14, 7, 2, 0, 1>(s, q, nullptr, seg_pool, seg_cnt, seg_cap, 0, n_tiles, 0, st, ts); break;
	default: s8_launch<16, 4, 2, 0, 1>(s, q, nullptr, seg_pool, seg_cnt, seg_cap, 0, n_tiles, 0, st, ts); break;
	}
}

bool scan8_variant_ok(int v) {
#ifdef LHIP_ABLATION_BUILD
	return v >= 0;
#else
	return v == 0;  // release builds carry the default geometry only
#endif
}

void launch_scan8_append(const StoreView &s, const QueryView &q, const float *tau, uint2 *seg_pool, int *seg_cnt,
                         int seg_cap, hipStream_t st, int64_t t0, int64_t t1, int seg_base) {
	const int64_t all_tiles = (s.n_slots + SCAN_BR - 1) / SCAN_BR;
	if (t1 < 0 || t1 > all_tiles) t1 = all_tiles;
	if (t0 < 0 || t0 > t1) throw std::runtime_error("scan8: tile range");
	const int64_t n_tiles = t1 - t0;
	if (n_tiles <= 0) return;
	if (!scan8_fits(s)) throw std::runtime_error("scan8: int8 scan copy with ld in [512, 1024] required");
	if (all_tiles * (int64_t)SCAN_BR > ((int64_t)1 << 32)) throw std::runtime_error("scan8: slots past 2^32");
	if (q.nq_pad % SCAN_BQ) throw std::runtime_error("scan8: query tile padding");
	if (!scan8_variant_ok(s.s8_variant)) throw std::runtime_error("scan8: geometry variant of a development build");
	switch (s.ld / 64) {
	case 8: s8_launch<8, 4, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
	case 10: s8_launch<10, 5, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
	case 12:
		switch (s.s8_variant) {
#ifdef LHIP_ABLATION_BUILD
		// development geometries (handle option "scan8_variant"): 16-row blocks per
		// wave (4: four waves, one per SIMD; 2: eight waves), register ring depth in
		// 64-deep k-steps; ABL != 0: timing ablations (wrong results, 8: setprio)
		case 1: s8_launch<12, 4, 4>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 2: s8_launch<12, 6, 4>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 3: s8_launch<12, 12, 4>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 4: s8_launch<12, 3, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 5: s8_launch<12, 6, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 6: s8_launch<12, 12, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 21: s8_launch<12, 4, 2, 1>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 22: s8_launch<12, 4, 2, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 23: s8_launch<12, 4, 2, 3>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 24: s8_launch<12, 4, 2, 4>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 28: s8_launch<12, 4, 2, 8>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 34: s8_launch<12, 4, 2, 64>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		case 29: s8_launch<12, 6, 2, 8>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
#endif
		default: s8_launch<12, 4, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
		}
		break;
	case 14: s8_launch<14, 7, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
	default: s8_launch<16, 4, 2>(s, q, tau, seg_pool, seg_cnt, seg_cap, t0, n_tiles, seg_base, st); break;
	}
}

}  // namespace lhip
