// tools/microbench.hip — hardware probes that decide the classifier's table
// and counter design (diagnostic; not part of the product).
//
//   atomics : 8.4M increments at random indices over 1.5M counters
//             (the C3 hit pattern) as device-scope u64/u32 atomics, and as
//             workgroup-scope atomics into a per-XCD replica (XCC_ID)
//   probes  : 25M random 64-byte bucket reads from tables of 1..48 MB,
//             and 8-byte reads from 0.5..4 MB filters
//   overlap : a 1 GiB non-temporal stream alone vs together with probes
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHK(x)                                                                 \
	do {                                                                   \
		hipError_t e_ = (x);                                           \
		if (e_ != hipSuccess) {                                        \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,      \
				hipGetErrorString(e_));                        \
			exit(1);                                               \
		}                                                              \
	} while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t xcc_id()
{
	// s_getreg_b32 HW_REG_XCC_ID (id 20), bits [3:0]
	return __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xf;
}

__global__ void k_atomic_dev_u64(const uint32_t *idx, uint64_t n, unsigned long long *c)
{
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		atomicAdd(&c[idx[i]], 1ull);
}
__global__ void k_atomic_dev_u32(const uint32_t *idx, uint64_t n, unsigned *c)
{
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		atomicAdd(&c[idx[i]], 1u);
}
__global__ void k_atomic_wg_u64_rep(const uint32_t *idx, uint64_t n, unsigned long long *c,
				    uint32_t m)
{
	unsigned long long *rep = c + (uint64_t)xcc_id() * m;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		__hip_atomic_fetch_add(&rep[idx[i]], 1ull, __ATOMIC_RELAXED,
				       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__global__ void k_atomic_wg_u32_rep(const uint32_t *idx, uint64_t n, unsigned *c, uint32_t m)
{
	unsigned *rep = c + (uint64_t)xcc_id() * m;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		__hip_atomic_fetch_add(&rep[idx[i]], 1u, __ATOMIC_RELAXED,
				       __HIP_MEMORY_SCOPE_WORKGROUP);
}
__global__ void k_atomic_agent_u32_rep(const uint32_t *idx, uint64_t n, unsigned *c, uint32_t m)
{
	unsigned *rep = c + (uint64_t)xcc_id() * m;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		__hip_atomic_fetch_add(&rep[idx[i]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_plain_u32_rep(const uint32_t *idx, uint64_t n, unsigned *c, uint32_t m)
{
	unsigned *rep = c + (uint64_t)xcc_id() * m;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		rep[idx[i]] += 1u;   // racy on purpose: timing reference only
}
__global__ void k_xcc_hist(unsigned *h)
{
	if (threadIdx.x == 0)
		atomicAdd(&h[xcc_id() * 8 + (blockIdx.x & 7)], 1u);
}

// random bucket probes: each lane reads one 64-byte bucket
__global__ void k_probe64(const u32x4 *tab, uint64_t nbuckets, const uint32_t *idx, uint64_t n,
			  unsigned *sink)
{
	uint32_t acc = 0;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
		const u32x4 *b = tab + (uint64_t)(idx[i] % nbuckets) * 4;
		u32x4 q0 = b[0], q1 = b[1], q2 = b[2], q3 = b[3];
		acc ^= q0.x ^ q1.y ^ q2.z ^ q3.w;
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}
// random 8-byte filter probes
__global__ void k_probe8(const unsigned long long *tab, uint64_t nwords, const uint32_t *idx,
			 uint64_t n, unsigned *sink)
{
	unsigned long long acc = 0;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
		acc ^= tab[(idx[i] * 2654435761u) % nwords];
	if (acc == 0x12345678u)
		sink[0] = (unsigned)acc;
}
// idx computed in-kernel (no index stream) for probes: hash of i
__global__ void k_probe64_hash(const u32x4 *tab, uint32_t nbuckets, uint64_t n, unsigned *sink)
{
	uint32_t acc = 0;
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
		uint32_t h = (uint32_t)i * 0x9E3779B1u;
		h ^= h >> 15;
		h *= 0x85ebca6bu;
		h ^= h >> 13;
		const u32x4 *b = tab + (uint64_t)(((uint64_t)h * nbuckets) >> 32) * 4;
		u32x4 q0 = b[0], q1 = b[1], q2 = b[2], q3 = b[3];
		acc ^= q0.x ^ q1.y ^ q2.z ^ q3.w;
	}
	if (acc == 0x12345678u)
		sink[0] = acc;
}
__global__ void k_stream(const u32x4 *src, uint64_t n16, unsigned *sink)
{
	u32x4 acc = { 0, 0, 0, 0 };
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull)
		acc ^= __builtin_nontemporal_load(src + i);
	if ((acc.x | acc.y) == 0x12345678u)
		sink[0] = acc.x;
}
// stream + per-16-packets probes in the same kernel
__global__ void k_stream_probe(const u32x4 *src, uint64_t n16, const u32x4 *tab, uint32_t nbuckets,
			       int probes_per_64B, unsigned *sink)
{
	u32x4 acc = { 0, 0, 0, 0 };
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
		u32x4 v = __builtin_nontemporal_load(src + i);
		acc ^= v;
		for (int p = 0; p < probes_per_64B; p++) {
			if (((i + p) & 3) == 0) {
				uint32_t h = v.x * 0x9E3779B1u + p;
				h ^= h >> 15;
				h *= 0x85ebca6bu;
				const u32x4 *b = tab + (uint64_t)(((uint64_t)h * nbuckets) >> 32) * 4;
				acc ^= b[0] ^ b[1] ^ b[2] ^ b[3];
			}
		}
	}
	if ((acc.x | acc.y) == 0x12345678u)
		sink[0] = acc.x;
}

static float time_it(hipEvent_t a, hipEvent_t b)
{
	float ms;
	CHK(hipEventSynchronize(b));
	CHK(hipEventElapsedTime(&ms, a, b));
	return ms;
}

int main(int argc, char **argv)
{
	const uint64_t NOPS = 8400000, M = 1500000, GRID = 2048;
	hipEvent_t e0, e1;
	CHK(hipEventCreate(&e0));
	CHK(hipEventCreate(&e1));
	std::vector<uint32_t> hidx(32000000);
	uint64_t s = 88172645463325252ull;
	for (auto &x : hidx) {
		s ^= s << 13; s ^= s >> 7; s ^= s << 17;
		x = (uint32_t)(s >> 16);
	}
	std::vector<uint32_t> hidxm(NOPS);
	for (uint64_t i = 0; i < NOPS; i++)
		hidxm[i] = hidx[i] % M;
	uint32_t *didx, *didxm;
	CHK(hipMalloc(&didx, hidx.size() * 4));
	CHK(hipMalloc(&didxm, NOPS * 4));
	CHK(hipMemcpy(didx, hidx.data(), hidx.size() * 4, hipMemcpyHostToDevice));
	CHK(hipMemcpy(didxm, hidxm.data(), NOPS * 4, hipMemcpyHostToDevice));
	unsigned *sink;
	CHK(hipMalloc(&sink, 4096));
	void *cnt;
	CHK(hipMalloc(&cnt, 8 * M * 8));

	// XCC placement census
	{
		unsigned h[64] = { 0 };
		CHK(hipMemset(sink, 0, 4096));
		k_xcc_hist<<<4096, 64>>>(sink);
		CHK(hipMemcpy(h, sink, 256, hipMemcpyDeviceToHost));
		printf("{\"xcc_census\": [");
		for (int x = 0; x < 8; x++) {
			printf("%s[", x ? "," : "");
			for (int b = 0; b < 8; b++)
				printf("%s%u", b ? "," : "", h[x * 8 + b]);
			printf("]");
		}
		printf("]}\n");
	}

	auto run_atomic = [&](const char *name, int kind) {
		float best = 1e9;
		unsigned long long total = 0;
		for (int r = 0; r < 4; r++) {
			CHK(hipMemset(cnt, 0, 8 * M * 8));
			CHK(hipEventRecord(e0));
			switch (kind) {
			case 0: k_atomic_dev_u64<<<GRID, 256>>>(didxm, NOPS, (unsigned long long *)cnt); break;
			case 1: k_atomic_dev_u32<<<GRID, 256>>>(didxm, NOPS, (unsigned *)cnt); break;
			case 2: k_atomic_wg_u64_rep<<<GRID, 256>>>(didxm, NOPS, (unsigned long long *)cnt, M); break;
			case 3: k_atomic_wg_u32_rep<<<GRID, 256>>>(didxm, NOPS, (unsigned *)cnt, M); break;
			case 4: k_atomic_agent_u32_rep<<<GRID, 256>>>(didxm, NOPS, (unsigned *)cnt, M); break;
			case 5: k_plain_u32_rep<<<GRID, 256>>>(didxm, NOPS, (unsigned *)cnt, M); break;
			}
			CHK(hipEventRecord(e1));
			float ms = time_it(e0, e1);
			if (ms < best)
				best = ms;
		}
		// verify sum
		size_t words = (kind == 0 || kind == 2) ? (kind == 0 ? M : 8 * M) : (kind == 1 ? M : 8 * M);
		if (kind == 0 || kind == 2) {
			std::vector<unsigned long long> h(words);
			CHK(hipMemcpy(h.data(), cnt, words * 8, hipMemcpyDeviceToHost));
			for (auto v : h) total += v;
		} else {
			std::vector<unsigned> h(words);
			CHK(hipMemcpy(h.data(), cnt, words * 4, hipMemcpyDeviceToHost));
			for (auto v : h) total += v;
		}
		printf("{\"test\": \"atomic_%s\", \"ms\": %.4f, \"Gops\": %.2f, \"sum\": %llu, \"expect\": %llu}\n",
		       name, best, NOPS / (best * 1e-3) / 1e9, total, (unsigned long long)NOPS);
	};
	run_atomic("dev_u64", 0);
	run_atomic("dev_u32", 1);
	run_atomic("wg_u64_xcc_replica", 2);
	run_atomic("wg_u32_xcc_replica", 3);
	run_atomic("agent_u32_xcc_replica", 4);
	run_atomic("plain_u32_xcc_replica_racy", 5);

	// probes
	const uint64_t NPROBE = 25000000;
	void *tab;
	CHK(hipMalloc(&tab, 64ull << 20));
	CHK(hipMemset(tab, 1, 64ull << 20));
	for (double mb : { 0.5, 1.0, 2.0, 3.0, 4.0, 6.0, 8.0, 12.0, 24.0, 48.0 }) {
		uint64_t nb = (uint64_t)(mb * 1048576 / 64);
		float best = 1e9;
		for (int r = 0; r < 3; r++) {
			CHK(hipEventRecord(e0));
			k_probe64_hash<<<GRID * 2, 256>>>((const u32x4 *)tab, (uint32_t)nb, NPROBE, sink);
			CHK(hipEventRecord(e1));
			float ms = time_it(e0, e1);
			if (ms < best) best = ms;
		}
		printf("{\"test\": \"probe64\", \"table_MB\": %.1f, \"ms\": %.4f, \"Gprobes\": %.2f}\n", mb,
		       best, NPROBE / (best * 1e-3) / 1e9);
	}
	for (double mb : { 0.5, 1.0, 2.0, 4.0 }) {
		uint64_t nw = (uint64_t)(mb * 1048576 / 8);
		float best = 1e9;
		for (int r = 0; r < 3; r++) {
			CHK(hipEventRecord(e0));
			k_probe8<<<GRID * 2, 256>>>((const unsigned long long *)tab, nw, didx, NPROBE, sink);
			CHK(hipEventRecord(e1));
			float ms = time_it(e0, e1);
			if (ms < best) best = ms;
		}
		printf("{\"test\": \"probe8\", \"table_MB\": %.1f, \"ms\": %.4f, \"Gprobes\": %.2f}\n", mb,
		       best, NPROBE / (best * 1e-3) / 1e9);
	}
	// stream alone vs stream + probes
	void *big;
	const uint64_t BIG = 1ull << 30;
	CHK(hipMalloc(&big, BIG));
	CHK(hipMemset(big, 3, BIG));
	for (int pp : { 0, 1, 2, 4 }) {
		for (double mb : { 4.0, 6.0, 12.0 }) {
			if (pp == 0 && mb != 4.0) continue;
			uint64_t nb = (uint64_t)(mb * 1048576 / 64);
			float best = 1e9;
			for (int r = 0; r < 3; r++) {
				CHK(hipEventRecord(e0));
				k_stream_probe<<<GRID, 256>>>((const u32x4 *)big, BIG / 16, (const u32x4 *)tab,
							     (uint32_t)nb, pp, sink);
				CHK(hipEventRecord(e1));
				float ms = time_it(e0, e1);
				if (ms < best) best = ms;
			}
			printf("{\"test\": \"stream_plus_probes\", \"probes_per_64B_pkt\": %d, \"table_MB\": %.1f, "
			       "\"ms\": %.4f, \"GBps\": %.1f}\n", pp, mb, best, BIG / (best * 1e-3) / 1e9);
		}
	}
	return 0;
}
