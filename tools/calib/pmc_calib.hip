// tools/calib/pmc_calib.hip — calibration of rocprofv3's FETCH_SIZE on gfx950
// for the access patterns of the classify kernels (MI355X_MICROARCH.md: the
// counter reads half the bytes of a wide coalesced stream; other widths are
// uncalibrated).  Each kernel reads a KNOWN number of bytes from a 4 GiB
// buffer (beyond the 256 MiB Infinity Cache, so the lines come from HBM):
//
//   stream  1 GiB of 16-byte non-temporal loads, coalesced (the frames)
//   lines   2^24 random 64-byte lines, four lanes x 16 bytes per line by
//           LDS-DMA (global_load_lds_dwordx4), 1 GiB (the bucket lines)
//   words   2^26 random 4-byte loads, 256 MiB requested (the Bloom words)
//
// Run each under `rocprofv3 --pmc FETCH_SIZE` (tools/calib/run.sh); the
// ratio FETCH_SIZE x 1024 / bytes is the correction for that pattern.
// Diagnostics only: not part of the product.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

__global__ __launch_bounds__(256) void k_stream(const u32x4 *src, uint64_t n16, u32x4 *sink)
{
	u32x4 acc = { 0, 0, 0, 0 };
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull)
		acc ^= __builtin_nontemporal_load(src + i);
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		sink[threadIdx.x] = acc;
}

// one wave: 16 random lines per instruction, 4 lanes x 16 B each
__global__ __launch_bounds__(256) void k_lines(const uint8_t *src, uint64_t nlines_buf,
					       uint32_t nlines, u32x4 *sink)
{
	__shared__ u32x4 buf[4][64];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	u32x4 acc = { 0, 0, 0, 0 };
	const uint32_t per_wave = 16;
	for (uint32_t base = (blockIdx.x * 4 + wv) * per_wave; base < nlines;
	     base += gridDim.x * 4 * per_wave) {
		const uint32_t line = base + (lane >> 2);
		const uint64_t l = mix(line * 2654435761u + 7) % nlines_buf;
		__builtin_amdgcn_global_load_lds(
			(const __attribute__((address_space(1))) void *)(src + l * 64 + (lane & 3) * 16),
			(__attribute__((address_space(3))) void *)&buf[wv][0], 16, 0, 0);
		__builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
		asm volatile("" ::: "memory");
		acc ^= buf[wv][lane];
	}
	if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u)
		sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_words(const uint32_t *src, uint64_t nwords_buf,
					       uint64_t nreads, uint32_t *sink)
{
	uint32_t acc = 0;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nreads; i += gridDim.x * 256ull)
		acc ^= src[mix((uint32_t)i * 2246822519u + 3) % nwords_buf];
	if (acc == 0x12345678u)
		sink[threadIdx.x] = acc;
}

#define CHK(x)                                                                   \
	do {                                                                     \
		hipError_t e_ = (x);                                             \
		if (e_ != hipSuccess) {                                          \
			fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
			return 1;                                                \
		}                                                                \
	} while (0)

int main(int argc, char **argv)
{
	const char *which = argc > 1 ? argv[1] : "stream";
	const uint64_t buf_bytes = 4ull << 30;
	uint8_t *src;
	u32x4 *sink;
	CHK(hipMalloc((void **)&src, buf_bytes));
	CHK(hipMalloc((void **)&sink, 4096));
	CHK(hipMemset(src, 1, buf_bytes));
	CHK(hipDeviceSynchronize());
	uint64_t bytes = 0;
	for (int rep = 0; rep < 3; rep++) {
		if (!strcmp(which, "stream")) {
			bytes = 1ull << 30;
			k_stream<<<4096, 256>>>((const u32x4 *)src, bytes / 16, sink);
		} else if (!strcmp(which, "lines")) {
			const uint32_t nlines = 1u << 24;
			bytes = (uint64_t)nlines * 64;
			k_lines<<<4096, 256>>>(src, buf_bytes / 64, nlines, sink);
		} else if (!strcmp(which, "words")) {
			const uint64_t nreads = 1ull << 26;
			bytes = nreads * 4;
			k_words<<<4096, 256>>>((const uint32_t *)src, buf_bytes / 4, nreads, (uint32_t *)sink);
		} else {
			fprintf(stderr, "usage: pmc_calib stream|lines|words\n");
			return 2;
		}
		CHK(hipGetLastError());
		CHK(hipDeviceSynchronize());
	}
	printf("{\"pattern\": \"%s\", \"requested_bytes_per_launch\": %llu}\n", which,
	       (unsigned long long)bytes);
	CHK(hipFree(src));
	CHK(hipFree(sink));
	return 0;
}
