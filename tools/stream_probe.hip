// Probe: what bounds scan8's row stream?  Streams an int8 table in scan8's
// geometry (256 workgroups of 8 waves, 32 rows per wave and 256-row tile, a
// 4-deep register ring of 64-byte k-steps, 16 i8 MFMAs per k-step on register
// operands) and times variants:
//   layout 0: row-major rows (a k-step load = 16 rows x 64 B, scan8 today)
//   layout 1: k-major tiles (a k-step load = 1 KiB contiguous)
//   mfma 0/1: without / with the MFMA work of a 128-query half
//   pairs 0/1: every tile read by one workgroup / by two (the query halves)
// Results are meaningless (checksums keep the loads alive).
// build: hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o tools/_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                          \
	do {                                                                                \
		hipError_t e_ = (x);                                                            \
		if (e_ != hipSuccess) {                                                         \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                                    \
		}                                                                               \
	} while (0)

constexpr int KS = 12, D = 4, LD = 768, TR = 256, P = 768;

// LDSB: B fragments read from a 128-query LDS image (scan8's swizzle, double
// buffered one k-step ahead) instead of constant registers
template <int LAYOUT, int MFMA, int LDSB, int RB>
__global__ __launch_bounds__(64 * (16 / RB), 1) void probe(const int8_t *__restrict__ X, int n_tiles, int pairs, int *out) {
	__shared__ __attribute__((aligned(16))) uint8_t QL[128 * P];
	const int nb = gridDim.x, b_id = blockIdx.x;
	int pr = b_id, NP = nb;
	if (pairs) {
		NP = nb >> 1;
		pr = (b_id & 7) | ((b_id >> 4) << 3);
	}
	const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, lr = lane & 15, lg = lane >> 4;
	constexpr int WR = 16 * RB;
	for (int i = tid; i < 128 * P / 16; i += 64 * (16 / RB)) {
		const unsigned hsh = (unsigned)i * 2654435761u;
		reinterpret_cast<i32x4 *>(QL)[i] = i32x4{(int)hsh, (int)(hsh * 747796405u), (int)(hsh ^ 0x9E3779B9u), (int)(hsh * 277803737u)};
	}
	__syncthreads();
	uint32_t qo[2][4];
#pragma unroll
	for (int m = 0; m < 4; ++m) {
		qo[0][m] = (uint32_t)(lr * P + ((((4 * m + lg) ^ lr)) << 4));
		qo[1][m] = qo[0][m] + 64u * P;
		asm volatile("" : "+v"(qo[1][m]));
	}
	auto bload = [&](int j, int u) -> i32x4 {
		return *reinterpret_cast<const i32x4 *>(QL + qo[u >> 2][j & 3] + 16 * (u & 3) * P + 256 * (j >> 2));
	};
	const int my_tiles = pr < n_tiles ? (n_tiles - 1 - pr) / NP + 1 : 0;
	uint32_t xo[RB];
#pragma unroll
	for (int rb = 0; rb < RB; ++rb)
		xo[rb] = LAYOUT == 0 ? (uint32_t)((WR * w + 16 * rb + lr) * LD + 16 * lg)
		                     : (uint32_t)((WR * w + 16 * rb + lr) * 64 + 16 * lg);
	auto xtile = [&](int b) -> const int8_t * {
		const int bb = b < my_tiles ? b : my_tiles - 1;
		return X + (pr + (int64_t)bb * NP) * TR * (int64_t)LD;
	};
	auto xload = [&](const int8_t *tb, int j, int rb) -> i32x4 {
		const uint32_t off = LAYOUT == 0 ? 64u * j : 16384u * j;
		return *reinterpret_cast<const i32x4 *>(tb + xo[rb] + off);
	};
	if (my_tiles == 0) return;
	i32x4 xa[D][RB];
	{
		const int8_t *tb = xtile(0);
#pragma unroll
		for (int j = 0; j < D; ++j) {
#pragma unroll
			for (int rb = 0; rb < RB; ++rb) xa[j][rb] = xload(tb, j, rb);
			__builtin_amdgcn_sched_barrier(0);
		}
	}
	i32x4 bq[2][8];
#pragma unroll
	for (int u = 0; u < 8; ++u) {
		const unsigned hsh = (unsigned)(lane * 8 + u + 1) * 2654435761u;
		bq[0][u] = bq[1][u] = i32x4{(int)hsh, (int)(hsh * 747796405u), (int)(hsh ^ 0x9E3779B9u), (int)(hsh * 277803737u)};
	}
	if (LDSB)
#pragma unroll
		for (int u = 0; u < 8; ++u) bq[0][u] = bload(0, u);
	i32x4 sum = {0, 0, 0, 0};
	for (int b = 0; b < my_tiles; ++b) {
		i32x4 acc[RB][8];
#pragma unroll
		for (int rb = 0; rb < RB; ++rb)
#pragma unroll
			for (int u = 0; u < 8; ++u) acc[rb][u] = i32x4{b, 0, 0, 0};
		const int8_t *tb_cur = xtile(b), *tb_next = xtile(b + 1);
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int j = 0; j < KS; ++j) {
			const int sl = j % D, cur = LDSB ? (j & 1) : 0;
			if (LDSB)
#pragma unroll
				for (int u = 0; u < 8; ++u) bq[cur ^ 1][u] = bload((j + 1) % KS, u);
			if (MFMA) {
#pragma unroll
				for (int u = 0; u < 8; ++u)
#pragma unroll
					for (int rb = 0; rb < RB; ++rb)
						acc[rb][u] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xa[sl][rb], bq[cur][u], acc[rb][u], 0, 0, 0);
			} else {
#pragma unroll
				for (int rb = 0; rb < RB; ++rb) acc[rb][0] ^= xa[sl][rb];
			}
			const int jn = j + D;
#pragma unroll
			for (int rb = 0; rb < RB; ++rb) xa[sl][rb] = xload(jn < KS ? tb_cur : tb_next, jn % KS, rb);
			__builtin_amdgcn_sched_barrier(0);
		}
		__builtin_amdgcn_sched_barrier(0);
		asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
		__builtin_amdgcn_sched_barrier(0);
#pragma unroll
		for (int rb = 0; rb < RB; ++rb)
#pragma unroll
			for (int u = 0; u < 8; ++u) sum += acc[rb][u];
	}
	const int s = sum[0] ^ sum[1] ^ sum[2] ^ sum[3];
	if (s == 0x7fffffff) out[b_id] = s;  // keeps the work alive
}

__global__ void fill_random(uint32_t *p, size_t n) {
	for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
		uint32_t h = (uint32_t)i * 2654435761u ^ (uint32_t)(i >> 32);
		h ^= h >> 15;
		h *= 2246822519u;
		h ^= h >> 13;
		p[i] = h;
	}
}

int main(int argc, char **argv) {
	const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
	const int n_tiles = (int)((n + TR - 1) / TR);
	const size_t bytes = (size_t)n_tiles * TR * LD;
	int8_t *X;
	int *out;
	CHK(hipMalloc(&X, bytes));
	CHK(hipMalloc(&out, 1024 * sizeof(int)));
	fill_random<<<4096, 256>>>(reinterpret_cast<uint32_t *>(X), bytes / 4);  // random operands: the clock MFMA work really runs at
	CHK(hipDeviceSynchronize());
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	auto run = [&](int layout, int mfma, int pairs, int ldsb, int rb) {
		auto launch = [&]() {
			const dim3 g(256), t2(512), t4(256);
			if (layout == 0 && mfma == 1 && ldsb == 0 && rb == 2) probe<0, 1, 0, 2><<<g, t2>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 0 && ldsb == 0 && rb == 2) probe<1, 0, 0, 2><<<g, t2>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 1 && ldsb == 0 && rb == 2) probe<1, 1, 0, 2><<<g, t2>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 1 && ldsb == 1 && rb == 2) probe<1, 1, 1, 2><<<g, t2>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 1 && ldsb == 0 && rb == 4) probe<1, 1, 0, 4><<<g, t4>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 1 && ldsb == 1 && rb == 4) probe<1, 1, 1, 4><<<g, t4>>>(X, n_tiles, pairs, out);
			if (layout == 1 && mfma == 0 && ldsb == 1 && rb == 2) probe<1, 0, 1, 2><<<g, t2>>>(X, n_tiles, pairs, out);
		};
		for (int i = 0; i < 3; ++i) launch();
		CHK(hipDeviceSynchronize());
		const int reps = 10;
		CHK(hipEventRecord(e0));
		for (int i = 0; i < reps; ++i) launch();
		CHK(hipEventRecord(e1));
		CHK(hipEventSynchronize(e1));
		float ms = 0;
		CHK(hipEventElapsedTime(&ms, e0, e1));
		ms /= reps;
		const double unique = (double)bytes / 1e9;
		printf("layout=%d mfma=%d pairs=%d ldsb=%d rb=%d  %.3f ms  unique %.2f GB -> %.0f GB/s  (CU ingest %.0f GB/s)\n", layout, mfma,
		       pairs, ldsb, rb, ms, unique, unique / ms * 1e3, unique * (pairs ? 2 : 1) / ms * 1e3);
		fflush(stdout);
	};
	run(0, 1, 1, 0, 2);
	run(1, 0, 1, 0, 2);
	run(1, 1, 1, 0, 2);
	run(1, 1, 1, 1, 2);
	run(1, 0, 1, 1, 2);
	run(1, 1, 1, 0, 4);
	run(1, 1, 1, 1, 4);
	run(1, 1, 0, 1, 2);
	CHK(hipFree(X));
	CHK(hipFree(out));
	return 0;
}
