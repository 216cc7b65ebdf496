// tools/mb_ta.hip — what a divergent gather costs a CU (diagnostic; not part
// of the product).  Each wave walks tiles as the classify kernel does and,
// per tile, issues G dword gathers whose 64 lanes touch D distinct 128-byte
// lines of a table of T bytes, optionally beside the 64-byte-per-lane packet
// stream (4 coalesced dwordx4 per tile).  Time per gather instruction per CU
// separates a per-line cost (address/tag processing) from a per-instruction
// one and from memory latency.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_ta tools/mb_ta.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                          \
	do {                                                                            \
		hipError_t e_ = (x);                                                    \
		if (e_ != hipSuccess) {                                                 \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                        \
		}                                                                       \
	} while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int G, bool STREAM>
__global__ __launch_bounds__(256) void k_gather(const u32x4 *__restrict__ data, uint32_t nt,
						  const uint32_t *__restrict__ tab, uint32_t tmask_lines,
						  uint32_t dlines, unsigned *sink)
{
	const int lane = threadIdx.x & 63;
	const uint32_t first = blockIdx.x * 4 + (threadIdx.x >> 6), step = gridDim.x * 4;
	uint32_t acc = 0, h = (first * 0x9E3779B1u) ^ lane;
	for (uint32_t t = first; t < nt; t += step) {
		if constexpr (STREAM) {
			const u32x4 *p = data + (uint64_t)t * 256 + lane;
#pragma unroll
			for (int i = 0; i < 4; i++) {
				const u32x4 v = __builtin_nontemporal_load(p + i * 64);
				acc ^= v.x ^ v.w;
			}
		}
#pragma unroll
		for (int g = 0; g < G; g++) {
			h = h * 1664525u + 1013904223u;
			// lane group (lane % dlines) shares a line; lines random per tile
			const uint32_t grp = (uint32_t)lane % dlines;
			const uint32_t line = ((h >> 8) + grp * 0x2545F491u) & tmask_lines;
			acc ^= tab[line * 32 + (lane & 31)];
		}
	}
	if (acc == 0x9abcdef1u)
		sink[0] = acc;
}

template <int G, bool STREAM>
static void run(const char *name, const u32x4 *data, uint32_t nt, const uint32_t *tab, uint32_t tlines,
		uint32_t dl, unsigned *sink, int per_cu, int ncu)
{
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	float best = 1e9;
	for (int r = 0; r < 5; r++) {
		CHK(hipEventRecord(e0));
		k_gather<G, STREAM><<<ncu * per_cu, 256>>>(data, nt, tab, tlines - 1, dl, sink);
		CHK(hipEventRecord(e1));
		CHK(hipEventSynchronize(e1));
		float ms;
		CHK(hipEventElapsedTime(&ms, e0, e1));
		if (r && ms < best)
			best = ms;
	}
	const double per_instr_ns = G ? best * 1e6 / ((double)nt * G / ncu) : 0;
	printf("{\"test\": \"%s\", \"G\": %d, \"stream\": %d, \"distinct_lines\": %u, \"table_KB\": %u, "
	       "\"waves_per_cu\": %d, \"ms\": %.4f, \"ns_per_gather_per_cu\": %.2f}\n",
	       name, G, (int)STREAM, dl, tlines * 128 / 1024, per_cu * 4, best, per_instr_ns);
	fflush(stdout);
	CHK(hipEventDestroy(e0));
	CHK(hipEventDestroy(e1));
}

int main()
{
	int ncu = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	const uint64_t n = 1ull << 26, bytes = n * 64;
	const uint32_t nt = (uint32_t)(n / 64);
	u32x4 *data;
	uint32_t *tab;
	unsigned *sink;
	CHK(hipMalloc(&data, bytes));
	CHK(hipMemset(data, 1, bytes));
	CHK(hipMalloc(&tab, 16u << 20));
	CHK(hipMemset(tab, 2, 16u << 20));
	CHK(hipMalloc(&sink, 64));
	const uint32_t small = 128, l2 = 8192, big = 131072;   // 16 KB, 1 MB, 16 MB
	run<0, true>("stream_only", data, nt, tab, small, 1, sink, 2, ncu);
	for (uint32_t dl : { 1u, 4u, 16u, 32u, 64u }) {
		run<1, false>("gather_only", data, nt, tab, l2, dl, sink, 2, ncu);
		run<1, true>("stream+gather", data, nt, tab, l2, dl, sink, 2, ncu);
	}
	for (int pc : { 1, 2, 4, 8 }) {
		run<1, false>("gather_only_occ", data, nt, tab, l2, 64, sink, pc, ncu);
		run<1, true>("stream+gather_occ", data, nt, tab, l2, 64, sink, pc, ncu);
	}
	run<2, true>("stream+2gathers", data, nt, tab, l2, 64, sink, 2, ncu);
	run<1, true>("stream+gather_16KB", data, nt, tab, small, 64, sink, 2, ncu);
	run<1, true>("stream+gather_16MB", data, nt, tab, big, 64, sink, 2, ncu);
	run<1, false>("gather_only_16KB", data, nt, tab, small, 64, sink, 2, ncu);
	run<1, false>("gather_only_16MB", data, nt, tab, big, 64, sink, 2, ncu);
	return 0;
}
