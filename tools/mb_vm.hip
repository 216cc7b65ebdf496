// tools/mb_vm.hip — what each vector-memory instruction per tile costs a
// stream of 64-byte packets (diagnostic; not part of the product).
//
// Every wave walks tiles of 64 packets (4 coalesced non-temporal dwordx4
// loads per tile, as the classify kernels stream them) and adds, per tile,
// a mix of the other instructions a classify tile issues: coalesced 16-bit
// length loads, coalesced byte / dword stores, 16-byte gathers from a 4 MB
// table (into registers, or by LDS-DMA), or the same spread over groups of
// tiles ("every G tiles").  The time per extra instruction separates the
// costs that the tile's memory instructions add to the stream.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb_vm tools/mb_vm.hip
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

struct Mix {
	int len;      // 16-bit length loads per tile
	int st8;      // byte stores per tile
	int st32;     // dword stores per tile
	int g16;      // 16-byte gathers per tile into registers
	int d16;      // 16-byte gathers per tile by LDS-DMA
	int every;    // the extras only on every `every`-th tile (1 = each)
	int st128;    // dwordx4 stores per `every` tiles
};

struct Args {
	const u32x4 *data;
	const uint16_t *lens;
	const u32x4 *tab;       // 4 MB: 2^18 x 16 B
	uint8_t *v8;
	uint32_t *v32;
	u32x4 *v128;
	uint32_t nt;
	unsigned *sink;
	uint32_t tshift;        // g16 index = h >> tshift (2^(32-tshift) x 16 B)
	uint32_t lanes;         // g16: lanes with their own random bucket (others repeat lane % lanes)
};

template <int LEN, int ST8, int ST32, int G16, int D16, int EVERY, int ST128, int PAIR = 0>
__global__ __launch_bounds__(256) void k_mix(const Args a)
{
	__shared__ u32x4 lds[4 * 64 * (D16 ? D16 : 1)];
	const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
	const uint32_t first = blockIdx.x * 4 + wv, step = gridDim.x * 4;
	// PAIR: lanes L and L+32 read the two halves of one random 32-byte bucket
	uint32_t acc = 0, h = (first * 0x9E3779B1u) ^ ((PAIR ? (lane & 31) : (uint32_t)lane % a.lanes) * 0x85ebca6bu);
	uint32_t k = 0;
	for (uint32_t t = first; t < a.nt; t += step, k++) {
		const u32x4 *p = a.data + (uint64_t)t * 256 + lane;
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const u32x4 v = __builtin_nontemporal_load(p + i * 64);
			acc ^= v.x ^ v.w;
		}
		if (EVERY == 1 || (k % EVERY) == 0) {
#pragma unroll
			for (int i = 0; i < LEN; i++)
				acc += __builtin_nontemporal_load(a.lens + (uint64_t)t * 64 + lane + i);
#pragma unroll
			for (int i = 0; i < G16; i++) {
				h = h * 1664525u + 1013904223u;
				const u32x4 v = PAIR ? a.tab[((h >> 15) << 1) + (lane >> 5)] : a.tab[(h >> a.tshift) + i];
				acc ^= v.y;
			}
#pragma unroll
			for (int i = 0; i < D16; i++) {
				h = h * 1664525u + 1013904223u;
				__builtin_amdgcn_global_load_lds(
					(const __attribute__((address_space(1))) void *)(a.tab + (h >> 14) + i),
					(__attribute__((address_space(3))) void *)(lds + (wv * D16 + i) * 64), 16, 0, 0);
			}
			if (D16) {
				__builtin_amdgcn_s_waitcnt(0x0F70);
				acc ^= lds[(wv * D16) * 64 + lane].x;
			}
#pragma unroll
			for (int i = 0; i < ST8; i++)
				__builtin_nontemporal_store((uint8_t)acc, a.v8 + (uint64_t)t * 64 + lane + i);
#pragma unroll
			for (int i = 0; i < ST32; i++)
				__builtin_nontemporal_store(acc, a.v32 + (uint64_t)t * 64 + lane + i);
#pragma unroll
			for (int i = 0; i < ST128; i++)
				__builtin_nontemporal_store(u32x4{ acc, h, acc, h }, a.v128 + (uint64_t)(t >> 3) * 64 + lane + i);
		}
	}
	if (acc == 0x9abcdef1u)
		a.sink[0] = acc;
}

template <int LEN, int ST8, int ST32, int G16, int D16, int EVERY, int ST128, int PAIR = 0>
static void run(const char *name, const Args &a, int per_cu, int ncu, double base)
{
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	float best = 1e9;
	for (int r = 0; r < 6; r++) {
		CHK(hipEventRecord(e0));
		k_mix<LEN, ST8, ST32, G16, D16, EVERY, ST128, PAIR><<<ncu * per_cu, 256>>>(a);
		CHK(hipEventRecord(e1));
		CHK(hipEventSynchronize(e1));
		float ms;
		CHK(hipEventElapsedTime(&ms, e0, e1));
		if (r && ms < best)
			best = ms;
	}
	CHK(hipGetLastError());
	const double extra = (double)(LEN + ST8 + ST32 + G16 + D16 + ST128) / EVERY;
	printf("{\"test\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.4f, \"extra_instr_per_tile\": %.3f, "
	       "\"ms_per_extra_instr_per_tile\": %.4f}\n",
	       name, per_cu * 4, best, extra, extra > 0 && base > 0 ? (best - base) / extra : 0.0);
	fflush(stdout);
	CHK(hipEventDestroy(e0));
	CHK(hipEventDestroy(e1));
}

int main()
{
	int ncu = 0;
	CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
	const uint64_t n = 1ull << 26, bytes = n * 64;
	Args a{};
	a.nt = (uint32_t)(n / 64);
	CHK(hipMalloc((void **)&a.data, bytes));
	CHK(hipMemset((void *)a.data, 1, bytes));
	CHK(hipMalloc((void **)&a.lens, n * 2 + 64));
	CHK(hipMemset((void *)a.lens, 0, n * 2 + 64));
	CHK(hipMalloc((void **)&a.tab, (16u << 20) + 256));
	CHK(hipMemset((void *)a.tab, 2, (16u << 20) + 256));
	a.tshift = 14;
	a.lanes = 64;
	CHK(hipMalloc((void **)&a.v8, n + 64));
	CHK(hipMalloc((void **)&a.v32, n * 4 + 256));
	CHK(hipMalloc((void **)&a.v128, n * 16 / 4 + 1024));
	CHK(hipMalloc((void **)&a.sink, 64));
	for (int pc : { 4, 2 }) {
		float base = 0;
		{
			hipEvent_t e0, e1;
			CHK(hipEventCreate(&e0));
			CHK(hipEventCreate(&e1));
			base = 1e9;
			for (int r = 0; r < 6; r++) {
				CHK(hipEventRecord(e0));
				k_mix<0, 0, 0, 0, 0, 1, 0><<<ncu * pc, 256>>>(a);
				CHK(hipEventRecord(e1));
				CHK(hipEventSynchronize(e1));
				float ms;
				CHK(hipEventElapsedTime(&ms, e0, e1));
				if (r && ms < base)
					base = ms;
			}
			printf("{\"test\": \"stream\", \"waves_per_cu\": %d, \"ms\": %.4f}\n", pc * 4, base);
		}
		run<1, 0, 0, 0, 0, 1, 0>("+len", a, pc, ncu, base);
		run<2, 0, 0, 0, 0, 1, 0>("+2len", a, pc, ncu, base);
		run<0, 1, 0, 0, 0, 1, 0>("+st8", a, pc, ncu, base);
		run<0, 0, 1, 0, 0, 1, 0>("+st32", a, pc, ncu, base);
		run<0, 0, 0, 1, 0, 1, 0>("+g16", a, pc, ncu, base);
		run<0, 0, 0, 2, 0, 1, 0>("+2g16", a, pc, ncu, base);
		run<0, 0, 0, 0, 1, 1, 0>("+d16", a, pc, ncu, base);
		run<0, 0, 0, 0, 2, 1, 0>("+2d16", a, pc, ncu, base);
		run<2, 1, 1, 0, 2, 1, 0>("+pipeq_mix(2len,st8,st32,2d16)", a, pc, ncu, base);
		run<1, 1, 1, 0, 2, 1, 0>("+1len,st8,st32,2d16", a, pc, ncu, base);
		run<0, 0, 0, 1, 0, 1, 0>("+g16_only", a, pc, ncu, base);
		run<1, 0, 0, 1, 0, 1, 0>("+len,g16", a, pc, ncu, base);
		run<1, 1, 0, 0, 0, 4, 0>("+len,st8_every4", a, pc, ncu, base);
		run<0, 0, 1, 0, 0, 4, 0>("+st32_every4", a, pc, ncu, base);
		run<0, 0, 0, 0, 0, 8, 1>("+st128_every8", a, pc, ncu, base);
		run<0, 0, 0, 2, 0, 1, 0, 1>("+2g16pair(32B buckets, 32 lines/instr)", a, pc, ncu, base);
		for (uint32_t ts : { 17u, 16u, 15u, 14u, 13u, 12u }) {
			Args b = a;
			b.tshift = ts;
			char nm[96];
			snprintf(nm, sizeof nm, "+g16 table %u KB", (1u << (32 - ts)) * 16 / 1024);
			run<0, 0, 0, 1, 0, 1, 0>(nm, b, pc, ncu, base);
		}
		for (uint32_t ln : { 8u, 16u, 32u, 48u }) {
			Args b = a;
			b.lanes = ln;
			char nm[96];
			snprintf(nm, sizeof nm, "+g16 4MB, %u random lines per tile", ln);
			run<0, 0, 0, 1, 0, 1, 0>(nm, b, pc, ncu, base);
		}
		run<0, 0, 0, 1, 0, 1, 0, 1>("+g16pair(one half of 32 buckets)", a, pc, ncu, base);
	}
	return 0;
}
