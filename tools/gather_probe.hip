// Probe: how fast can one workgroup per CU gather random f32 rows (pool_refine's
// refine rounds: 768-float rows of a 3 GB store, exact f64 distances)?
// Variants: waves per workgroup, rows in flight per wave (every 16-B load of a
// row issued before any use), f64 accumulate or a plain f32 sum, rows per
// workgroup (a one-round burst of 128 like pool_refine vs a long stream).
// build: hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/_gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <algorithm>

#define CHK(x)                                                                          \
	do {                                                                                \
		hipError_t e_ = (x);                                                            \
		if (e_ != hipSuccess) {                                                         \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                                    \
		}                                                                               \
	} while (0)

constexpr int LD = 768, NI = LD / 256;

template <int NT, int R, int F64>
__global__ __launch_bounds__(NT) void gather(const float *__restrict__ X, const uint32_t *__restrict__ idx,
                                             const float *__restrict__ q, int rows_per_wg, float *out) {
	constexpr int NW = NT / 64;
	const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
	float4 qv[NI];
#pragma unroll
	for (int it = 0; it < NI; ++it) qv[it] = reinterpret_cast<const float4 *>(q)[lane + 64 * it];
	double acc = 0.0;
	float facc = 0.f;
	const uint32_t *my = idx + (size_t)blockIdx.x * rows_per_wg;
	for (int r0 = w * R; r0 < rows_per_wg; r0 += NW * R) {
		uint32_t s[R];
#pragma unroll
		for (int j = 0; j < R; ++j) s[j] = my[r0 + j];
		float4 xv[NI][R];
#pragma unroll
		for (int it = 0; it < NI; ++it)
#pragma unroll
			for (int j = 0; j < R; ++j)
				xv[it][j] = reinterpret_cast<const float4 *>(X + (size_t)s[j] * LD)[lane + 64 * it];
#pragma unroll
		for (int j = 0; j < R; ++j) {
			if (F64) {
				double a = 0.0;
#pragma unroll
				for (int it = 0; it < NI; ++it) {
					double d;
					d = (double)xv[it][j].x - (double)qv[it].x; a += d * d;
					d = (double)xv[it][j].y - (double)qv[it].y; a += d * d;
					d = (double)xv[it][j].z - (double)qv[it].z; a += d * d;
					d = (double)xv[it][j].w - (double)qv[it].w; a += d * d;
				}
#pragma unroll
				for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
				acc += a;
			} else {
#pragma unroll
				for (int it = 0; it < NI; ++it) facc += xv[it][j].x + xv[it][j].y + xv[it][j].z + xv[it][j].w;
			}
		}
	}
	if (lane == 0) out[blockIdx.x * NW + w] = (float)acc + facc;
}

constexpr int NSETS = 20;
static void *g_flush = nullptr;
static size_t g_flush_bytes = 0;

template <int NT, int R, int F64>
static void run(const float *X, const uint32_t *idx, const float *q, float *out, int wgs, int rows_per_wg,
                const char *tag) {
	hipEvent_t a, b;
	CHK(hipEventCreate(&a));
	CHK(hipEventCreate(&b));
	for (int i = 0; i < 3; ++i) gather<NT, R, F64><<<wgs, NT>>>(X, idx, q, rows_per_wg, out);
	CHK(hipDeviceSynchronize());
	const int iters = 20;
	float best = 1e30f, tot = 0.f;
	for (int i = 0; i < iters; ++i) {
		// cold rows: a fresh index set each launch (sets are disjoint slices of a
		// larger random table, and a 1 GB flush write runs in between)
		const uint32_t *ix = idx + (size_t)(i % NSETS) * wgs * rows_per_wg * (rows_per_wg <= 128 ? 1 : 0);
		if (g_flush) CHK(hipMemsetAsync(g_flush, i, g_flush_bytes));
		CHK(hipEventRecord(a));
		gather<NT, R, F64><<<wgs, NT>>>(X, ix, q, rows_per_wg, out);
		CHK(hipEventRecord(b));
		CHK(hipEventSynchronize(b));
		float ms;
		CHK(hipEventElapsedTime(&ms, a, b));
		best = ms < best ? ms : best;
		tot += ms;
	}
	const double bytes = (double)wgs * rows_per_wg * LD * 4;
	printf("%-10s NT=%4d R=%2d f64=%d rows/wg=%5d: best %8.2f us avg %8.2f us  %6.2f TB/s (best)\n", tag, NT, R, F64,
	       rows_per_wg, best * 1e3, tot / iters * 1e3, bytes / (best * 1e-3) / 1e12);
	CHK(hipEventDestroy(a));
	CHK(hipEventDestroy(b));
}

int main(int argc, char **argv) {
	const size_t N = argc > 1 ? (size_t)atol(argv[1]) : 1000000;
	const int wgs = 256;
	float *X, *q, *out;
	uint32_t *idx;
	CHK(hipMalloc(&X, N * LD * sizeof(float)));
	if (argc > 2 && atoi(argv[2]) == 1) {  // random rows (N(0,1)-like), as a real store holds
		std::vector<float> hx((size_t)1 << 22);
		std::mt19937 g(3);
		std::normal_distribution<float> nd;
		for (auto &v : hx) v = nd(g);
		for (size_t off = 0; off < N * LD; off += hx.size())
			CHK(hipMemcpy(X + off, hx.data(), std::min(hx.size(), N * LD - off) * sizeof(float), hipMemcpyHostToDevice));
	} else {
		CHK(hipMemset(X, 0, N * LD * sizeof(float)));
	}
	CHK(hipMalloc(&q, LD * sizeof(float)));
	CHK(hipMemset(q, 0, LD * sizeof(float)));
	CHK(hipMalloc(&out, 65536 * sizeof(float)));
	const int maxr = 2048;
	std::vector<uint32_t> h((size_t)wgs * std::max(maxr, 128 * NSETS));
	std::mt19937 rng(7);
	for (auto &v : h) v = (uint32_t)(rng() % N);
	CHK(hipMalloc(&idx, h.size() * sizeof(uint32_t)));
	CHK(hipMemcpy(idx, h.data(), h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
	if (argc > 3 && atoi(argv[3]) == 1) {  // evict caches between launches
		g_flush_bytes = (size_t)1 << 30;
		CHK(hipMalloc(&g_flush, g_flush_bytes));
	}
	printf("table %zu rows x %d f32 (%.2f GB, %s%s), %d workgroups\n", N, LD, N * LD * 4 / 1e9,
	       g_flush ? "cold: 1 GB flush between launches, " : "",
	       argc > 2 && atoi(argv[2]) == 1 ? "random" : "zeros", wgs);
	for (int rpw : {128}) {
		run<512, 4, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<512, 8, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<512, 16, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<512, 8, 0>(X, idx, q, out, wgs, rpw, "gather");
		run<512, 16, 0>(X, idx, q, out, wgs, rpw, "gather");
		run<1024, 4, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<1024, 8, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<1024, 8, 0>(X, idx, q, out, wgs, rpw, "gather");
		run<256, 8, 1>(X, idx, q, out, wgs * 4, rpw / 4, "gather4x");
		run<256, 4, 1>(X, idx, q, out, wgs * 4, rpw / 4, "gather4x");
		run<1024, 2, 1>(X, idx, q, out, wgs, rpw, "gather");
		run<512, 2, 1>(X, idx, q, out, wgs, rpw, "gather");
	}
	return 0;
}
