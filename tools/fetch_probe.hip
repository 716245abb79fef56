// FETCH_SIZE calibration probe (MI355X_MICROARCH.md 'HBM': "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Streams a known byte count (1 GiB, past the 256 MiB Infinity
// Cache) three ways and prints the byte count per launch; run it under
//   rocprofv3 --pmc FETCH_SIZE -- tools/_fetch_probe
// and divide FETCH_SIZE (KiB) x 1024 by the bytes: the factor that turns this
// kernel's FETCH_SIZE into bytes read.
//   k16   16 B per lane, global_load_dwordx4, consecutive lanes consecutive
//         16-B pieces (the guide's calibrated case: FETCH = 1/2 of the bytes)
//   k12   pq_fast_scan_bank_kernel<3>'s row stream (ivf_kernels.hip load()):
//         96-B rows, 8 lanes per row, lane p reads bytes [12 p, 12 p + 12) by
//         buffer_load_dwordx3 with the non-temporal policy (aux 2); a wave step
//         = 8 consecutive rows = 768 contiguous bytes, 1024-thread workgroups,
//         4 row steps per lane and round, rows of a workgroup's chunk in order
//   k12c  the same loads with the default cache policy
// Build: hipcc -O3 --offload-arch=gfx950 tools/fetch_probe.hip -o tools/_fetch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x)                                                                              \
	do {                                                                                   \
		hipError_t e_ = (x);                                                               \
		if (e_ != hipSuccess) {                                                            \
			fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
			return 1;                                                                      \
		}                                                                                  \
	} while (0)

constexpr int THREADS = 1024;
constexpr uint32_t RSRC3 = 0x00020000u;

__global__ __launch_bounds__(256) void k16(const uint4 *__restrict__ p, int64_t n16, uint32_t *__restrict__ out) {
	uint32_t acc = 0;
	for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
		const uint4 v = p[i];
		acc ^= v.x ^ v.y ^ v.z ^ v.w;
	}
	if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // (never: keeps the loads)
}

template <int AUX>
__global__ __launch_bounds__(THREADS) void k12(const uint8_t *__restrict__ codes, int64_t rows, int64_t rows_per_wg,
                                               uint32_t *__restrict__ out) {
	constexpr int MT = 96, RS = 4, ROUND = THREADS / 8 * RS;  // 512 rows per round
	const int t = threadIdx.x, lane = t & 63, wv = t >> 6, p = lane & 7, rw = lane >> 3;
	const uint32_t lrow = (uint32_t)((wv << 3) + rw), vcode = lrow * MT + 12 * p;
	const int64_t r0 = (int64_t)blockIdx.x * rows_per_wg;
	const int64_t r1 = r0 + rows_per_wg < rows ? r0 + rows_per_wg : rows;
	if (r0 >= r1) return;
	const uint32_t nrow = (uint32_t)(r1 - r0);
	const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc((void *)(codes + r0 * MT), 0, (int)(nrow * MT), RSRC3);
	uint32_t acc = 0;
	for (uint32_t rb = 0; rb < nrow; rb += ROUND) {
#pragma unroll
		for (int k = 0; k < RS; ++k) {
			const uint32_t srow = rb + (uint32_t)(k * (THREADS / 8));
			const auto v = __builtin_amdgcn_raw_buffer_load_b96(rc, vcode, (int)(srow * MT), AUX);
			acc ^= v[0] ^ v[1] ^ v[2];
		}
	}
	if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;
}

int main() {
	const int64_t bytes = (int64_t)1 << 30;  // 1 GiB (a multiple of 96 * 512 rows is not needed: rows past the chunk read 0)
	uint8_t *buf;
	uint32_t *out;
	CK(hipMalloc(&buf, bytes));
	CK(hipMalloc(&out, 1 << 20));
	CK(hipMemset(buf, 1, bytes));
	const int64_t rows = bytes / 96;
	const int wgs = 2048;
	const int64_t per = (rows + wgs - 1) / wgs;
	for (int rep = 0; rep < 3; ++rep) {
		k16<<<4096, 256>>>(reinterpret_cast<const uint4 *>(buf), bytes / 16, out);
		k12<2><<<wgs, THREADS>>>(buf, rows, per, out);
		k12<0><<<wgs, THREADS>>>(buf, rows, per, out);
	}
	CK(hipGetLastError());
	CK(hipDeviceSynchronize());
	printf("k16 bytes %lld\nk12 bytes %lld\nk12c bytes %lld\n", (long long)bytes, (long long)(rows * 96),
	       (long long)(rows * 96));
	CK(hipFree(buf));
	CK(hipFree(out));
	return 0;
}
