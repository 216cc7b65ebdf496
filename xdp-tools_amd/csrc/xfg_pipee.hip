// SPDX-License-Identifier: GPL-2.0
//
// xfg_pipee.hip — the Ethernet-key kernel: the programs xdpfilt_alw_eth and
// xdpfilt_dny_eth over fixed-stride batches.  Included by xfg_kernels.hip.
//
// Those programs parse nothing past the Ethernet header: parse_ethhdr fails
// only for a frame shorter than its 14 bytes (ABORTED; a VLAN tag past the
// frame ends the tag walk, not the parse: headers/xdp/parsing_helpers.h:
// 100-134), lookup_verdict_ethernet then checks the destination MAC and the
// source MAC (xdp-filter/xdpfilt_prog.h:187-196 via CHECK_VERDICT_ETHERNET,
// :224-226), and nothing else is compiled in.  A packet needs its first 12
// bytes and its length, and each lookup is a hash-map probe.  With the map
// small (at most XFG_EK_MAX_KEYS keys, flags alike on every device) the host
// keeps it as an open-addressed table of 16-byte entries (xfg_kargs.ek,
// xfg_ctx.c ek_refresh) that every workgroup copies into LDS: a lookup is a
// hash and ek_disp + 1 LDS reads, with no memory access after the frame's
// own bytes and no deferred packet.  The generic pipelined kernel
// (xfg_pipeline.hip) spends ~380 vector instructions per 64-packet tile on
// its general parse and plan for the same programs (C1 at 2^24: 6.0 per
// packet, profiles/archive/r05_s20_session.log).
//
// A wave takes G tiles of 64 packets per iteration (one packet per lane per
// tile; tiles dealt over the grid's waves as in the other pipelined kernels,
// so a wave's share is the same), their first 16 bytes and lengths loaded
// D - 1 iterations ahead into a ring of D register buffers.
namespace {

// (C1, one box, profiles/archive/r05_s22_session.log and r05_s23_session.log: G 1
// and D 2 0.185 ms at 2^24; G 2 0.190-0.201, G 4 0.209, G 8 0.258; D 3 and
// 4 and 8 waves a SIMD slower -- the smaller loop body wins)
#ifndef XFG_EK_G   /* tiles per wave iteration */
#define XFG_EK_G 1
#endif
#ifndef XFG_EK_D   /* register buffers of G tiles each */
#define XFG_EK_D 2
#endif
#define EK_WAVES 8
#define EK_THREADS (64 * EK_WAVES)
#ifndef XFG_EK_MINW   /* waves per SIMD the register budget allows for */
#define XFG_EK_MINW 6
#endif

template <uint32_t FEAT, bool L16>
__global__ __launch_bounds__(EK_THREADS, XFG_EK_MINW) void xfg_pipee_kernel(const xfg_kargs a)
{
	static_assert((FEAT & F_ETH) != 0 && (FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0,
		      "the Ethernet-key kernel runs the Ethernet-only programs");
	constexpr int NW = EK_WAVES, NT = EK_THREADS, G = XFG_EK_G, D = XFG_EK_D;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	__shared__ uint32_t s_ecnt[XFG_EK_SLOTS_MAX];   // hits per key-table entry
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t es = rfl(a.ek_slots), edisp = rfl(a.ek_disp);
	u32x4 *const s_ek = ek_base(a, s_dyn);
	for (uint32_t i = tid; i < es; i += NT) {
		s_ek[i] = reinterpret_cast<const u32x4 *>(a.ek)[i];
		s_ecnt[i] = 0;
	}
	// live lookups (flag census): dst, then src (xdpfilt_prog.h:187-196)
	const bool dlive = a.te.count && can_hit(a.te.fmask, M_DST);
	const bool slive = a.te.count && can_hit(a.te.fmask, M_SRC);
	const uint32_t seed = rfl(a.te.seed), gbe = rfl(a.gbase[2]);
	__syncthreads();

	const uint32_t n = (uint32_t)a.n, nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv, step = gridDim.x * NW;
	const uint32_t mytiles = first < nt ? (nt - 1 - first) / step + 1 : 0u;
	const uint32_t ng = (mytiles + G - 1) / G;
	const uint64_t stride = a.stride;
	const uint8_t *const lens = static_cast<const uint8_t *>(a.lens);

	// per-action packets (wave totals) and bytes (per lane)
	uint32_t st_c0 = 0, st_c1 = 0, st_c2 = 0, st_b0 = 0, st_b1 = 0, st_b2 = 0;
	auto stat = [&](bool valid, uint32_t act, uint32_t len) {
		st_c0 += (uint32_t)__popcll(__ballot(valid & (act == A_ABORTED)));
		st_c1 += (uint32_t)__popcll(__ballot(valid & (act == A_DROP)));
		st_c2 += (uint32_t)__popcll(__ballot(valid & (act == A_PASS)));
		st_b0 += (valid & (act == A_ABORTED)) ? len : 0u;
		st_b1 += (valid & (act == A_DROP)) ? len : 0u;
		st_b2 += (valid & (act == A_PASS)) ? len : 0u;
	};
	// CHECK_MAP (xdpfilt_prog.h:56-64) against the LDS table: the key found
	// with every bit of mask set, the entry it sits in.  Every lane reads
	// edisp + 1 entries from its home (a key sits at most that far past it;
	// keys are unique, so at most one entry matches).  A hit counts on its
	// entry's LDS counter (one LDS atomic, whatever the keys' heat), added to
	// the key's counter once per workgroup.
	auto probe = [&](uint32_t lo, uint32_t hi, uint32_t mask, uint32_t &ent) {
		return ek_probe<true>(s_ek, es, edisp, seed, lo, hi, mask, ent);
	};

	// a group's first 16 bytes and lengths (tiles past the wave's share and
	// lanes past the batch read a valid address; process() ignores them)
	auto issue = [&](uint32_t g, u32x4 (&f)[G], uint32_t (&l)[G]) {
#pragma unroll
		for (int j = 0; j < G; j++) {
			uint32_t t = first + (g * G + j) * step;
			t = t < nt ? t : nt - 1;
			uint32_t gi = t * 64 + lane;
			gi = gi < n ? gi : n - 1;
			f[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.data + gi * stride));
			l[j] = L16 ? (uint32_t)gload16((uint64_t)(uintptr_t)(lens + 2ull * gi))
				   : gload32((uint64_t)(uintptr_t)(lens + 4ull * gi));
		}
	};
	auto process = [&](uint32_t g, const u32x4 (&f)[G], const uint32_t (&l)[G]) {
#pragma unroll
		for (int j = 0; j < G; j++) {
			const uint32_t t = first + (g * G + j) * step;
			const uint32_t gi = t * 64 + lane;
			const bool valid = (t < nt) & (gi < n);
			// (the slot is the frame's buffer: a longer length is capped)
			const uint32_t len = valid ? min(l[j], a.stride) : 0u;
			const bool look = valid & (len >= 14);   // parse_ethhdr
			// h_dest: bytes 0-5, h_source: bytes 6-11
			const uint32_t dlo = f[j].x, dhi = f[j].y & 0xffffu;
			const uint32_t slo = __builtin_amdgcn_alignbyte(f[j].z, f[j].y, 2), shi = f[j].z >> 16;
			uint32_t sd = 0, ss = 0;
			bool hd = false, hs = false;
			if (dlive)
				hd = look & probe(dlo, dhi, M_DST, sd);
			if (slive)
				hs = look & !hd & probe(slo, shi, M_SRC, ss);
			const uint32_t act = !look ? A_ABORTED : (hd | hs) ? HIT : MISS;
			if (valid)
				__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
			if (hd | hs)
				atomicAdd(&s_ecnt[hd ? sd : ss], 1u);
			stat(valid, act, len);
		}
	};

	// D register buffers: group g in buffer g % D, D - 1 groups in flight
	// while one is processed
	u32x4 fb[D][G];
	uint32_t lb[D][G];
	if (ng) {
#pragma unroll
		for (int d = 0; d < D; d++)
			issue(d, fb[d], lb[d]);
	}
	uint32_t g = 0;
	for (; g + D <= ng; g += D) {
#pragma unroll
		for (int d = 0; d < D; d++) {
			process(g + d, fb[d], lb[d]);
			issue(g + d + D, fb[d], lb[d]);
		}
	}
#pragma unroll
	for (int d = 0; d < D - 1; d++)
		if (g + d < ng)
			process(g + d, fb[d], lb[d]);

	const uint32_t vb[3] = { st_b0, st_b1, st_b2 }, vc[3] = { st_c0, st_c1, st_c2 };
#pragma unroll
	for (int k = 0; k < 3; k++) {
		unsigned long long x = vb[k];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			x += __shfl_xor(x, o);
		if (lane == 0 && vc[k]) {
			atomicAdd(&s_stats[2 * k], (unsigned long long)vc[k]);
			atomicAdd(&s_stats[2 * k + 1], x);
		}
	}
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	for (uint32_t i = tid; i < es; i += NT)
		if (const uint32_t c = s_ecnt[i])
			atomicAdd(global_counter(a, gbe + s_ek[i].z), (unsigned long long)c);
}

}  // namespace
