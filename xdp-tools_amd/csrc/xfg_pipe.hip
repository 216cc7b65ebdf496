// SPDX-License-Identifier: GPL-2.0
//
// xfg_pipe.hip — the pipelined classify kernel (included by xfg_kernels.hip
// inside its anonymous namespace; uses its parse/probe helpers).
//
// Layouts: fixed stride >= W (every window byte readable without a length),
// no offsets array, no descriptors, fewer than 2^32 packets.  Each wave works
// alone on tiles of 64 packets (one per lane) and keeps THREE tiles in
// flight, one stage apart:
//
//   iteration i:
//     S3 (tile i-2)  its bucket lines have arrived: match, verdict, counter,
//                    stats;
//     S2 (tile i-1)  its Bloom words have arrived: the first lookup in
//                    reference order whose filter passes has its key copied
//                    from the tile's LDS rows and its bucket line fetched;
//     S1 (tile i)    its windows have arrived: LDS rows, fast parse, port
//                    check, lookup slots; their Bloom words fetched;
//     then           tile i+1's windows fetched; tile i-2's verdicts stored
//                    and counters bumped.
//
// A wave's vector-memory counter completes in issue order.  The loads are
// issued in the order their results are consumed next iteration (lines,
// Bloom words, windows) and the stores and atomics last, so a wait never
// covers a younger load, and one memory latency is paid per iteration
// instead of the window -> Bloom -> bucket chain.
//
// Only the dominant well-formed shapes run in the loop: untagged IPv4 with
// ihl 5 and untagged IPv6/UDP (parse_fast, whose result equals the generic
// walk's for them), whose keys sit at fixed window offsets.  Every other
// packet, and the rare lookup the pipeline cannot finish (a displaced key,
// a second candidate whose filter passed after a miss), is appended to the
// wave's deferred list and classified serially after the loop, with every
// lane busy, by the reference-order code path of the classic kernel.  This
// keeps divergent generic-parse code out of the loop.
//
// Lookup slots of a fast-path packet, in the order of xdpfilt_prog.h:224-307:
//   0 eth dst (bytes 0..5), 1 eth src (6..11)   lookup_verdict_ethernet
//   2 IP daddr (v4 30..33 | v6 38..53)           lookup_verdict_ipv4/_ipv6
//   3 IP saddr (v4 26..29 | v6 22..37)
// A slot is live only if its map has keys and the flag census says its mask
// can match; if no live slot hits, the verdict is ABORTED (a UDP length or
// TCP data-offset check failed), the port verdict, or MISS.

constexpr int NSLOT = 4;
enum PMap : uint32_t { PM_NONE = 0, PM_ETH = 1, PM_V4 = 2, PM_V6 = 3 };

// slot meta: bits 0-1 map, 2-5 mask, 6 zero key
__device__ __forceinline__ uint32_t smeta_make(uint32_t map, uint32_t mask)
{
	return map | (mask << 2);
}

// Byte offset of slot j's key for map m (fast-path shapes only).
__device__ __forceinline__ uint32_t slot_off(uint32_t j, uint32_t map)
{
	return map == PM_ETH ? (j == 0 ? 0u : 6u)
	       : map == PM_V4 ? (j == 2 ? 30u : 26u) : (j == 2 ? 38u : 22u);
}

// Little-endian dword at byte o of an LDS row (o + 4 <= W).
__device__ __forceinline__ uint32_t row32(const uint32_t *row, uint32_t o)
{
	return __builtin_amdgcn_alignbyte(row[(o >> 2) + 1], row[o >> 2], o & 3);
}

template <uint32_t FEAT>
__device__ __forceinline__ void row_key(const uint32_t *row, uint32_t map, uint32_t off,
					uint32_t (&k)[4])
{
	constexpr bool ETH = (FEAT & F_ETH) != 0;
	constexpr bool V6 = (FEAT & F_IPV6) != 0 && (FEAT & X_NOV6) == 0;
	k[0] = row32(row, off);
	k[1] = k[2] = k[3] = 0;
	if (ETH && map == PM_ETH) {
		k[1] = row32(row, off + 4) & 0xffff;
	} else if (V6 && map == PM_V6) {
		k[1] = row32(row, off + 4);
		k[2] = row32(row, off + 8);
		k[3] = row32(row, off + 12);
	}
}

// Per-map descriptor fields selected per lane.
struct TSel {
	const uint8_t *buckets;
	uint32_t nbuckets, nslots, spb, gbase, max_disp;
};

template <uint32_t FEAT>
__device__ __forceinline__ TSel tsel(const xfg_kargs &a, uint32_t map)
{
	constexpr bool ETH = (FEAT & F_ETH) != 0;
	constexpr bool V6 = (FEAT & F_IPV6) != 0 && (FEAT & X_NOV6) == 0;
	TSel s;
	s.buckets = static_cast<const uint8_t *>(a.t4.buckets);
	s.nbuckets = a.t4.nbuckets;
	s.nslots = a.t4.nslots;
	s.spb = XFG_SLOTS_V4;
	s.gbase = a.gbase[0];
	s.max_disp = a.t4.max_disp;
	if (V6 && map == PM_V6) {
		s.buckets = static_cast<const uint8_t *>(a.t6.buckets);
		s.nbuckets = a.t6.nbuckets;
		s.nslots = a.t6.nslots;
		s.spb = XFG_SLOTS_V6;
		s.gbase = a.gbase[1];
		s.max_disp = a.t6.max_disp;
	}
	if (ETH && map == PM_ETH) {
		s.buckets = static_cast<const uint8_t *>(a.te.buckets);
		s.nbuckets = a.te.nbuckets;
		s.nslots = a.te.nslots;
		s.spb = XFG_SLOTS_ETH;
		s.gbase = a.gbase[2];
		s.max_disp = a.te.max_disp;
	}
	return s;
}

// Serial classification of one packet (the deferred cases): its window
// reloaded into the lane's LDS row, the full parse and the ordered lookups.
template <uint32_t FEAT, int W>
__device__ __forceinline__ uint32_t classify_serial(const xfg_kargs &a, uint32_t *row,
						    const uint32_t *s_pbits, uint32_t gi,
						    uint32_t len, uint32_t &tag)
{
	const uint8_t *g = a.data + (uint64_t)gi * a.stride;
#pragma unroll
	for (int it = 0; it < W / 16; it++) {
		const u32x4 v = *reinterpret_cast<const u32x4 *>(g + 16 * it);
		row[4 * it] = v.x;
		row[4 * it + 1] = v.y;
		row[4 * it + 2] = v.z;
		row[4 * it + 3] = v.w;
	}
	Pkt<W> p{ row, g, len };
	const Parsed r = parse<FEAT, W>(p);
	tag = CT_NONE;
	return lookups<FEAT, false>(a, LazyKeys<Pkt<W>>{ p }, r, s_pbits, tag);
}

// OCC: waves per SIMD the register allocator is asked to fit (W = 64)
template <uint32_t FEAT, int W, bool DENSE, int OCC = 4>
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_waves_per_eu(W == 64 ? OCC : 2))) void xfg_classify_pipe_kernel(const xfg_kargs a)
{
	constexpr int CPP = W / 16;
	constexpr int ROWDW = Pkt<W>::ROWDW;
	constexpr bool ETH = (FEAT & F_ETH) != 0;
	constexpr bool V4 = (FEAT & F_IPV4) != 0;
	constexpr bool V6 = (FEAT & F_IPV6) != 0 && (FEAT & X_NOV6) == 0;
	constexpr bool L3 = (FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) != 0;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr bool HASH = ETH || V4 || V6;
	constexpr bool HIT_PASS = (FEAT & F_DENY) != 0;
	constexpr uint32_t HIT = HIT_PASS ? A_PASS : A_DROP;   // VERDICT_HIT
	constexpr uint32_t MISS = HIT_PASS ? A_DROP : A_PASS;  // VERDICT_MISS
	__shared__ uint32_t win[TILE * ROWDW];
	__shared__ uint32_t s_pbits[PORTS ? 2048 : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_pcnt[];   // hit-log fill per partition (hlog_parts)

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	if (tid < 6)
		s_stats[tid] = 0;
	for (int i = tid; i < CC_ENTRIES; i += TILE) {
		s_ctag[i] = CT_NONE;
		s_ccnt[i] = 0;
	}
	if (a.hlog)
		for (uint32_t i = tid; i < a.hlog_parts; i += TILE)
			s_pcnt[i] = 0;
	if constexpr (PORTS) {
		if (a.port_count)
			for (int i = tid; i < 2048; i += TILE)
				s_pbits[i] = a.port_tab ? a.port_tab[i] : a.port_bits[i];
	}
	__syncthreads();   // the only workgroup barrier before the tail

	uint32_t *const wrows = win + (tid >> 6) * 64 * ROWDW;   // this wave's rows
	uint32_t *const myrow = wrows + lane * ROWDW;
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t nw = gridDim.x * (TILE / 64);
	const uint32_t gw = blockIdx.x * (TILE / 64) + (tid >> 6);
	const uint32_t my_nt = gw < nt ? (nt - gw + nw - 1) / nw : 0;
	// deferred packets of this wave: fix_list[gw * fix_cap ...]
	uint32_t *const fixl = a.fix_list + (uint64_t)gw * a.fix_cap;
	uint32_t nfix = 0;
	auto defer = [&](bool f, uint32_t gi) {
		const unsigned long long fm = __ballot(f);
		if (fm) {
			if (f)
				fixl[nfix + __popcll(fm & ((1ull << lane) - 1))] = gi;
			nfix += (uint32_t)__popcll(fm);
		}
	};
	// live lookups (uniform): table non-empty and the census allows the mask
	const bool e_d = ETH && a.te.count && can_hit(a.te.fmask, M_DST);
	const bool e_s = ETH && a.te.count && can_hit(a.te.fmask, M_SRC);
	const bool v4_d = V4 && a.t4.count && can_hit(a.t4.fmask, M_DST);
	const bool v4_s = V4 && a.t4.count && can_hit(a.t4.fmask, M_SRC);
	const bool v6_d = V6 && a.t6.count && can_hit(a.t6.fmask, M_DST);
	const bool v6_s = V6 && a.t6.count && can_hit(a.t6.fmask, M_SRC);

	// ---- stage state
	u32x4 pre[CPP];            // tile i+1's windows in flight
	uint32_t plen = 0;
	// S1 -> S2
	uint32_t m1[NSLOT], h1[NSLOT];
	unsigned long long bw1[NSLOT];
	uint32_t pt1 = CT_NONE, inf1 = 0, len1 = 0;
	// S2 -> S3
	Line ln2 = { { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, { 0, 0, 0, 0 } };
	uint32_t k2[4] = { 0, 0, 0, 0 };
	uint32_t cm2 = 0, cb2 = 0, pt2 = CT_NONE, inf2 = 0, len2 = 0;
#pragma unroll
	for (int j = 0; j < NSLOT; j++) {
		m1[j] = 0;
		h1[j] = 0;
		bw1[j] = 0;
	}
	uint32_t c_ab = 0, c_dr = 0, c_pa = 0;
	unsigned long long b_ab = 0, b_dr = 0, b_pa = 0;
	// (arithmetic, not branches: a branchy form through the lambda's
	// references was lowered to a pointer select into scratch)
	auto count_stats = [&](uint32_t act, uint32_t len) {
		const uint32_t ab = act == A_ABORTED, dr = act == A_DROP, pa = act == A_PASS;
		c_ab += ab;
		c_dr += dr;
		c_pa += pa;
		b_ab += ab ? len : 0u;
		b_dr += dr ? len : 0u;
		b_pa += pa ? len : 0u;
	};
	// one cold hit: appended to the workgroup's region of its hit-log
	// partition (a plain store; xfg_hlog_count_kernel adds it up), or, with
	// no log or a full region, a memory-side atomic
	auto cold = [&](uint32_t tag) {
		if (a.hlog) {
			const uint32_t p = tag >> XFG_HLOG_SHIFT;
			const uint32_t pos = atomicAdd(&s_pcnt[p], 1u);
			if (pos < a.hlog_cap) {
				a.hlog[((uint64_t)p * gridDim.x + blockIdx.x) * a.hlog_cap + pos] = tag;
				return;
			}
		}
		atomicAdd(global_counter(a, tag), 1ull);
	};
	// counter bump: lanes of the wave hitting the same rule are merged (one
	// leader round), then summed in the LDS counter cache (hot rules: a
	// ruled port, an attacked address); what the cache cannot take is a
	// cold hit
	auto bump = [&](uint32_t tag) {
		const unsigned long long pend = __ballot(tag != CT_NONE);
		if (pend) {
			const int leader = __ffsll((long long)pend) - 1;
			const uint32_t lt = __shfl(tag, leader);
			const bool mine = tag == lt;
			const unsigned long long same = __ballot(mine);
			if (lane == leader) {
				const uint32_t cnt = (uint32_t)__popcll(same);
				if (!cache_hit(s_ctag, s_ccnt, lt, cnt)) {
					if (cnt > 1)
						atomicAdd(global_counter(a, lt), (unsigned long long)cnt);
					else
						cold(lt);
				}
			}
			if (mine)
				tag = CT_NONE;
		}
		if (tag != CT_NONE && !cache_hit(s_ctag, s_ccnt, tag, 1))
			cold(tag);
	};

	auto tile_of = [&](uint32_t k) -> uint32_t { return gw + k * nw; };
	auto issue = [&](uint32_t t) {
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64u ? 64u : n - base;
		if constexpr (DENSE) {
			const u32x4 *src = reinterpret_cast<const u32x4 *>(a.data + (uint64_t)base * W) + lane;
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				pre[it] = u32x4{ 0, 0, 0, 0 };
				if ((uint32_t)(it * 64 + lane) / CPP < rem)
					pre[it] = __builtin_nontemporal_load(src + it * 64);
			}
		} else {
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const uint32_t pk = c / CPP, sub = c % CPP;
				pre[it] = u32x4{ 0, 0, 0, 0 };
				if (pk < rem)
					pre[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
						a.data + (uint64_t)(base + pk) * a.stride + sub * 16));
			}
		}
		plen = (uint32_t)lane < rem ? load_len(a, base + lane) : 0;
	};
	if (my_nt)
		issue(tile_of(0));

	for (uint32_t i = 0; i < my_nt + 2; i++) {
		const bool s1 = i < my_nt, s2 = i >= 1 && i <= my_nt, s3 = i >= 2;
		// inf: bit 0 in the pipeline, bits 1-3 abort stage (NST or ST_L4)
		// ------------------------------------------------ S2 (tile i-1)
		// Bloom words arrived: first live slot whose filter passes; its key
		// is copied from the tile's rows and its bucket line fetched.  The
		// line fetch is cooperative: load r serves packets 16r..16r+15, four
		// lanes per line, 16 bytes each, so one wave instruction touches 16
		// lines instead of 64 (the vector memory pipeline's address rate,
		// not bytes, bounds scattered 16-byte loads).
		uint32_t cm2n = 0, cb2n = 0;
		uint32_t k2n[4] = { 0, 0, 0, 0 };
		Line ln2n = ln2;
		if constexpr (HASH) {
			if (s2) {
				uint32_t maybe = 0;
#pragma unroll
				for (int j = 0; j < NSLOT; j++) {
					const uint32_t m = m1[j];
					if (!m)
						continue;
					const uint32_t map = m & 3;
					bool mb;
					if (m & 64) {
						mb = map == PM_ETH ? a.te.zero_present
						     : map == PM_V6 ? a.t6.zero_present : a.t4.zero_present;
					} else {
						const uint32_t nbw = map == PM_ETH ? a.te.bloom_words
								     : map == PM_V6 ? a.t6.bloom_words
								     : a.t4.bloom_words;
						const unsigned long long bm = xfg_bloom_mask(h1[j]);
						mb = !nbw || (bw1[j] & bm) == bm;
					}
					maybe |= (uint32_t)mb << j;
				}
				uint64_t lb = 0;   // this packet's bucket line (0: none)
				if (maybe) {
					const uint32_t c = __builtin_ctz(maybe);
					uint32_t m = 0, h = 0;
#pragma unroll
					for (int j = 0; j < NSLOT; j++)
						if (c == (uint32_t)j) {
							m = m1[j];
							h = h1[j];
						}
					const uint32_t map = m & 3;
					const TSel ts = tsel<FEAT>(a, map);
					row_key<FEAT>(myrow, map, slot_off(c, map), k2n);
					cb2n = (m & 64) ? ts.nbuckets : xfg_home(h, ts.nbuckets);
					cm2n = m | ((maybe & (maybe - 1)) ? 128u : 0u);
					lb = (uint64_t)(uintptr_t)ts.buckets + (uint64_t)cb2n * XFG_BUCKET_BYTES;
				}
				if (__ballot(lb != 0)) {
					const uint32_t part = (lane & 3) * 16;
					const uint64_t l0 = __shfl(lb, (lane >> 2));
					const uint64_t l1 = __shfl(lb, 16 + (lane >> 2));
					const uint64_t l2 = __shfl(lb, 32 + (lane >> 2));
					const uint64_t l3 = __shfl(lb, 48 + (lane >> 2));
					if (l0)
						ln2n.q0 = *reinterpret_cast<const u32x4 *>(l0 + part);
					if (l1)
						ln2n.q1 = *reinterpret_cast<const u32x4 *>(l1 + part);
					if (l2)
						ln2n.q2 = *reinterpret_cast<const u32x4 *>(l2 + part);
					if (l3)
						ln2n.q3 = *reinterpret_cast<const u32x4 *>(l3 + part);
				}
			}
		}
		// ------------------------------------------------ S3 (tile i-2)
		// bucket lines arrived: transposed through this wave's rows (tile
		// i-1 is done with them), then the verdict; a displaced key or a
		// later live candidate after a miss defers the packet
		uint32_t act = A_NONE, tag = CT_NONE;
		bool fb = false;
		if (s3) {
			Line ln;
			if constexpr (HASH) {
				__builtin_amdgcn_wave_barrier();   // S2's row reads are done
				u32x4 *const tb = reinterpret_cast<u32x4 *>(wrows);
				tb[lane] = ln2.q0;
				tb[64 + lane] = ln2.q1;
				tb[128 + lane] = ln2.q2;
				tb[192 + lane] = ln2.q3;
				__builtin_amdgcn_wave_barrier();
				ln.q0 = tb[4 * lane];
				ln.q1 = tb[4 * lane + 1];
				ln.q2 = tb[4 * lane + 2];
				ln.q3 = tb[4 * lane + 3];
			}
			if (inf2 & 1) {
				const uint32_t ab = (inf2 >> 1) & 7;
				bool hit = false;
				if constexpr (HASH) {
					if (cm2) {
						const uint32_t map = cm2 & 3, mask = (cm2 >> 2) & 15;
						const TSel ts = tsel<FEAT>(a, map);
						int si = 0;
						if (!(cm2 & 64)) {
							if (V4 && map == PM_V4)
								si = match_v4(ln, k2[0]);
							if (V6 && map == PM_V6)
								si = match_v6(ln, k2[0], k2[1], k2[2], k2[3]);
							if (ETH && map == PM_ETH)
								si = match_eth(ln, k2[0], k2[1]);
						}
						if (si >= 0) {
							if ((ln.flag(si) & mask) == mask) {
								hit = true;
								tag = ts.gbase + ((cm2 & 64) ? ts.nslots
									: cb2 * ts.spb + (uint32_t)si);
							}
						} else if (ln.overflow() && ts.max_disp) {
							fb = true;   // the key may sit further along the chain
						}
						if (!hit && (cm2 & 128))
							fb = true;   // a later live lookup's filter passed too
					}
				}
				if (hit)
					act = HIT;
				else if (ab != NST)
					act = A_ABORTED;
				else if (pt2 != CT_NONE) {
					act = HIT;
					tag = pt2;
				} else
					act = MISS;
				if (fb) {
					act = A_NONE;
					tag = CT_NONE;
				}
			}
		}
		// ------------------------------------------------ S1 (tile i)
		uint32_t m1n[NSLOT], h1n[NSLOT];
		unsigned long long bw1n[NSLOT];
#pragma unroll
		for (int j = 0; j < NSLOT; j++) {
			m1n[j] = 0;
			h1n[j] = 0;
			bw1n[j] = 0;
		}
		uint32_t pt1n = CT_NONE, inf1n = 0, len1n = 0;
		bool df = false;
		const uint32_t gi1 = tile_of(i) * 64 + lane;
		if (s1) {
			__builtin_amdgcn_wave_barrier();   // S2/S3 row reads are done
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const int pk = c / CPP, sub = c % CPP;
				uint32_t *dst = &wrows[pk * ROWDW + sub * 4];
				dst[0] = pre[it].x;
				dst[1] = pre[it].y;
				dst[2] = pre[it].z;
				dst[3] = pre[it].w;
			}
			len1n = plen;
			__builtin_amdgcn_wave_barrier();
			if (gi1 < n) {
				Pkt<W> p{ myrow, nullptr, len1n };
				Parsed r;
				r.abort_at = NST;
				r.l3 = 0;
				r.l4proto = 0;
				bool fast;
				if constexpr (L3)
					fast = parse_fast<FEAT, W>(p, r);
				else
					fast = len1n >= 14;   // ethernet-only program
				df = !fast;
				if (fast) {
					inf1n = 1 | (r.abort_at << 1);
					if constexpr (ETH) {
						if (e_d)
							m1n[0] = smeta_make(PM_ETH, M_DST);
						if (e_s)
							m1n[1] = smeta_make(PM_ETH, M_SRC);
					}
					if (V4 && r.l3 == 1) {
						if (v4_d)
							m1n[2] = smeta_make(PM_V4, M_DST);
						if (v4_s)
							m1n[3] = smeta_make(PM_V4, M_SRC);
					}
					if (V6 && r.l3 == 3) {
						if (v6_d)
							m1n[2] = smeta_make(PM_V6, M_DST);
						if (v6_s)
							m1n[3] = smeta_make(PM_V6, M_SRC);
					}
					if constexpr (PORTS) {
						if (r.abort_at == NST && a.port_count && r.l4proto) {
							const uint32_t pm = r.l4proto == 17 ? M_UDP : M_TCP;
							uint32_t t = CT_NONE;
							if (check_port(a, s_pbits, r.pdst, M_DST | pm, t) ||
							    check_port(a, s_pbits, r.psrc, M_SRC | pm, t))
								pt1n = t;
						}
					}
					if constexpr (HASH) {
						// hash every live slot and fetch its Bloom word now
#pragma unroll
						for (int j = 0; j < NSLOT; j++) {
							const uint32_t m = m1n[j];
							if (!m)
								continue;
							const uint32_t map = m & 3;
							uint32_t k[4];
							row_key<FEAT>(myrow, map, slot_off(j, map), k);
							if ((k[0] | k[1] | k[2] | k[3]) == 0) {
								m1n[j] = m | 64;   // the all-zero key's own slot
								continue;
							}
							uint32_t h;
							if (ETH && map == PM_ETH)
								h = xfg_hash_eth(k[0] | ((uint64_t)k[1] << 32), a.te.seed);
							else if (V6 && map == PM_V6)
								h = xfg_hash_v6(k[0], k[1], k[2], k[3], a.t6.seed);
							else
								h = xfg_hash_v4(k[0], a.t4.seed);
							h1n[j] = h;
							const xfg_tdesc &td = (ETH && map == PM_ETH) ? a.te
									      : (V6 && map == PM_V6) ? a.t6 : a.t4;
							if (td.bloom_words)
								bw1n[j] = td.bloom[xfg_bloom_word(h, td.bloom_words)];
						}
					}
				}
			}
		}
		// ------------------------------------------------ next windows
		if (i + 1 < my_nt)
			issue(tile_of(i + 1));
		// ------------------------------------------------ stores
		if (s1)
			defer(df, gi1);
		if (s3) {
			const uint32_t gi3 = tile_of(i - 2) * 64 + lane;
			defer(fb, gi3);
			if (act != A_NONE)
				a.verdicts[gi3] = (uint8_t)act;
			if (a.ablate & 2)
				tag = CT_NONE;
			bump(tag);
			count_stats(act, len2);
		}
		// ------------------------------------------------ rotate
		ln2 = ln2n;
		k2[0] = k2n[0];
		k2[1] = k2n[1];
		k2[2] = k2n[2];
		k2[3] = k2n[3];
		cm2 = cm2n;
		cb2 = cb2n;
		pt2 = pt1;
		inf2 = s2 ? inf1 : 0;
		len2 = len1;
#pragma unroll
		for (int j = 0; j < NSLOT; j++) {
			m1[j] = m1n[j];
			h1[j] = h1n[j];
			bw1[j] = bw1n[j];
		}
		pt1 = pt1n;
		inf1 = inf1n;
		len1 = len1n;
	}
	// ---- the deferred packets, serially (rows are free now)
#ifndef XFG_EXP_NO_SERIAL
	if (nfix) {
		__threadfence_block();   // this wave's list stores before its loads
		for (uint32_t f = 0; f < nfix; f += 64) {
			uint32_t act = A_NONE, tag = CT_NONE, len = 0;
			if (f + lane < nfix) {
				const uint32_t gi = fixl[f + lane];
				len = load_len(a, gi);
				act = classify_serial<FEAT, W>(a, myrow, s_pbits, gi, len, tag);
				a.verdicts[gi] = (uint8_t)act;
			}
			if (a.ablate & 2)
				tag = CT_NONE;
			bump(tag);
			count_stats(act, len);
		}
	}
#endif
	// per-action stats: lane sums -> wave sums -> workgroup (LDS) -> device
	{
		unsigned long long v[6] = { c_ab, b_ab, c_dr, b_dr, c_pa, b_pa };
#pragma unroll
		for (int k = 0; k < 6; k++) {
			unsigned long long x = v[k];
#pragma unroll
			for (int o = 32; o > 0; o >>= 1)
				x += __shfl_xor(x, o);
			if (lane == 0 && x)
				atomicAdd(&s_stats[k], x);
		}
	}
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	for (int i = tid; i < CC_ENTRIES; i += TILE)
		if (s_ctag[i] != CT_NONE && s_ccnt[i])
			atomicAdd(global_counter(a, s_ctag[i]), (unsigned long long)s_ccnt[i]);
	if (a.hlog)
		for (uint32_t p = tid; p < a.hlog_parts; p += TILE)
			a.hlog_cnt[(uint64_t)p * gridDim.x + blockIdx.x] =
				s_pcnt[p] < a.hlog_cap ? s_pcnt[p] : a.hlog_cap;
}

// ---------------------------------------------------------------- hit-log count
// One workgroup per partition p (16384 consecutive counter identities): the
// regions every classify workgroup left for p are added up in LDS, then each
// counter of the partition gets its sum with one plain read-modify-write (a
// partition's counters belong to this workgroup alone; the classify
// kernel's own atomics are complete, since it ran before on the stream).
constexpr int HC_THREADS = 1024;

__global__ __launch_bounds__(HC_THREADS) void xfg_hlog_count_kernel(const xfg_kargs a, uint32_t grid)
{
	constexpr uint32_t PW = 1u << XFG_HLOG_SHIFT;
	__shared__ uint32_t hist[PW];
	const uint32_t tid = threadIdx.x, p = blockIdx.x;
	for (uint32_t i = tid; i < PW; i += HC_THREADS)
		hist[i] = 0;
	__syncthreads();
	for (uint32_t w = tid; w < grid; w += HC_THREADS) {
		const uint64_t r = (uint64_t)p * grid + w;
		const uint32_t c = a.hlog_cnt[r];
		const uint32_t *e = a.hlog + r * a.hlog_cap;   // hlog_cap % 4 == 0
		uint32_t k = 0;
		for (; k + 4 <= c; k += 4) {
			const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(e + k));
			atomicAdd(&hist[v.x & (PW - 1)], 1u);
			atomicAdd(&hist[v.y & (PW - 1)], 1u);
			atomicAdd(&hist[v.z & (PW - 1)], 1u);
			atomicAdd(&hist[v.w & (PW - 1)], 1u);
		}
		for (; k < c; k++)
			atomicAdd(&hist[e[k] & (PW - 1)], 1u);
	}
	__syncthreads();
	const uint32_t total = a.gbase[3] + 65536u;   // + the port counters
	for (uint32_t i = tid; i < PW; i += HC_THREADS) {
		const uint32_t g = p * PW + i;
		if (hist[i] && g < total)
			*global_counter(a, g) += hist[i];
	}
}
