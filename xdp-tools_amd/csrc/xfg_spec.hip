// SPDX-License-Identifier: GPL-2.0
//
// xfg_spec.hip — speculative classification for the single-lookup rule set
// (included by xfg_kernels.hip after xfg_pipe.hip, inside its anonymous
// namespace).
//
// When every fast-path packet has at most ONE live hash lookup — IPv4 rules
// of one direction only (the flag census says no key carries the other
// direction's bit), no Ethernet or IPv6 keys — the packet's verdict depends
// on the bucket line only through "is the key there with the mask set".  The
// Bloom filter already answers "no" exactly; for "maybe" the kernel takes the
// HIT verdict speculatively and appends a record {packet, key, the verdict
// and port counter the packet gets if the key is absent} to the partition of
// its home bucket.  No bucket line is read in the streaming kernel, which
// then moves little more than the frames themselves (the random 128-byte
// bucket lines were half again the frame bytes through the fabric).
//
// xfg_spec_resolve_kernel then walks each partition with its 1024 bucket
// lines held in LDS: a record whose key is there with the mask bumps the
// rule's counter (an LDS histogram, added to the counters once); a Bloom
// false positive gets its verdict, port counter and stats patched back to
// what the reference program returns (xdpfilt_prog.h:121-134: the lookup
// missed, so the program continues to the port stage / MISS).  Results are
// identical to the non-speculative path; only the order of work differs.
//
// Pipeline per wave (tiles of 64 packets, one per lane), iteration i:
//   S1 (tile i)    windows (fetched two iterations earlier) -> LDS rows ->
//                  fast parse, port check, key, hash; its Bloom word fetched;
//   next           tile i+2's windows fetched;
//   S2 (tile i-1)  Bloom word arrived: verdict (speculative HIT + record, or
//                  the miss verdict), counters, stats.
// Non-fast packets and records that find their region full are deferred to
// the serial pass after the loop (as in the pipelined kernel).

constexpr uint32_t SLOG_LB = 1u << XFG_SLOG_SHIFT;   // buckets per partition

template <uint32_t FEAT, int W, bool DENSE>
__global__ __launch_bounds__(TILE) __attribute__((amdgpu_waves_per_eu(W == 64 ? 5 : 3))) void xfg_classify_spec_kernel(const xfg_kargs a)
{
	constexpr int CPP = W / 16;
	constexpr int ROWDW = Pkt<W>::ROWDW;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr bool HIT_PASS = (FEAT & F_DENY) != 0;
	constexpr uint32_t HIT = HIT_PASS ? A_PASS : A_DROP;   // VERDICT_HIT
	constexpr uint32_t MISS = HIT_PASS ? A_DROP : A_PASS;  // VERDICT_MISS
	__shared__ uint32_t win[TILE * ROWDW];
	__shared__ uint32_t s_pbits[PORTS ? 2048 : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];   // hit-log fills [hlog_parts], record fills [slog_parts]

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	uint32_t *const s_pcnt = s_dyn;
	uint32_t *const s_scnt = s_dyn + (a.hlog ? a.hlog_parts : 0);
	if (tid < 6)
		s_stats[tid] = 0;
	for (int i = tid; i < CC_ENTRIES; i += TILE) {
		s_ctag[i] = CT_NONE;
		s_ccnt[i] = 0;
	}
	if (a.hlog)
		for (uint32_t i = tid; i < a.hlog_parts; i += TILE)
			s_pcnt[i] = 0;
	for (uint32_t i = tid; i < a.slog_parts; i += TILE)
		s_scnt[i] = 0;
	if constexpr (PORTS) {
		if (a.port_count)
			for (int i = tid; i < 2048; i += TILE)
				s_pbits[i] = a.port_tab ? a.port_tab[i] : a.port_bits[i];
	}
	__syncthreads();

	uint32_t *const wrows = win + (tid >> 6) * 64 * ROWDW;
	uint32_t *const myrow = wrows + lane * ROWDW;
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t nw = gridDim.x * (TILE / 64);
	const uint32_t gw = blockIdx.x * (TILE / 64) + (tid >> 6);
	const uint32_t my_nt = gw < nt ? (nt - gw + nw - 1) / nw : 0;
	uint32_t *const fixl = a.fix_list + (uint64_t)gw * a.fix_cap;
	uint32_t nfix = 0;
	// the one live lookup: IPv4 daddr (DST) or saddr (SRC)
	const bool dst = can_hit(a.t4.fmask, M_DST);
	const uint32_t kmask = dst ? M_DST : M_SRC, koff = dst ? 30u : 26u;

	auto defer = [&](bool f, uint32_t gi) {
		const unsigned long long fm = __ballot(f);
		if (fm) {
			if (f)
				fixl[nfix + __popcll(fm & ((1ull << lane) - 1))] = gi;
			nfix += (uint32_t)__popcll(fm);
		}
	};
	uint32_t c_ab = 0, c_dr = 0, c_pa = 0;
	unsigned long long b_ab = 0, b_dr = 0, b_pa = 0;
	auto count_stats = [&](uint32_t act, uint32_t len) {
		const uint32_t ab = act == A_ABORTED, dr = act == A_DROP, pa = act == A_PASS;
		c_ab += ab;
		c_dr += dr;
		c_pa += pa;
		b_ab += ab ? len : 0u;
		b_dr += dr ? len : 0u;
		b_pa += pa ? len : 0u;
	};
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
	// Every lane loads unconditionally (addresses past the batch end are
	// clamped to its last packet): a fixed number of loads per iteration
	// lets the compiler's waits count exactly, instead of draining to
	// vmcnt(0) where a load may or may not have been issued.
	auto load_win = [&](uint32_t t, u32x4 (&w)[CPP], uint32_t &wl) {
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64u ? 64u : n - base;
		if constexpr (DENSE) {
			const u32x4 *src = reinterpret_cast<const u32x4 *>(a.data + (uint64_t)base * W);
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const uint32_t c = it * 64 + lane;
				w[it] = __builtin_nontemporal_load(src + (c < rem * CPP ? c : rem * CPP - 1));
			}
		} else {
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const uint32_t pk = c / CPP, sub = c % CPP;
				const uint32_t pc = pk < rem ? pk : rem - 1;
				w[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
					a.data + (uint64_t)(base + pc) * a.stride + sub * 16));
			}
		}
		wl = load_len(a, base + ((uint32_t)lane < rem ? (uint32_t)lane : rem - 1));
	};

	// Two window buffers and two S1 -> S2 state sets alternate roles: tile
	// i's windows live in buffer i % 2 and are refilled with tile i+2 once
	// staged; S1 of tile i fills state i % 2, S2 of tile i-1 reads the other.
	// The loop is unrolled by two so no register holding a load in flight is
	// ever copied (a copy would wait for the load, serialising the pipeline).
	struct Win {
		u32x4 w[CPP];
		uint32_t len;
	};
	// inf: bit 0 valid, 1-3 abort stage, 4 has the lookup, 5 zero key
	struct S12 {
		uint32_t inf, pt, len, key, h;
		unsigned long long bw;
	};
	Win W0, W1;
	W0.len = W1.len = 0;
	S12 X0 = { 0, CT_NONE, 0, 0, 0, 0 }, X1 = { 0, CT_NONE, 0, 0, 0, 0 };
	if (my_nt)
		load_win(tile_of(0), W0.w, W0.len);
	if (my_nt > 1)
		load_win(tile_of(1), W1.w, W1.len);

	const unsigned long long *const bloom_base =
		a.t4.bloom_words ? a.t4.bloom : reinterpret_cast<const unsigned long long *>(a.stats);
	auto body = [&](uint32_t i, Win &Wc, const S12 &Sp, S12 &Sn) {
		const bool s1 = i < my_nt, s2 = i >= 1;
		// ------------------------------------------------ S1 (tile i)
		// (Sn.bw is not cleared: it is read only where inf bit 4 says the
		// load was issued, and a clear would wait for the old load)
		Sn.inf = 0;
		Sn.pt = CT_NONE;
		Sn.len = 0;
		Sn.key = 0;
		Sn.h = 0;
		bool df = false;
		uint32_t bwi = 0;   // Bloom word of this lane's key (0: a word nobody needs)
		const uint32_t gi1 = tile_of(i) * 64 + lane;
		if (s1) {
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const int pk = c / CPP, sub = c % CPP;
				uint32_t *d = &wrows[pk * ROWDW + sub * 4];
				d[0] = Wc.w[it].x;
				d[1] = Wc.w[it].y;
				d[2] = Wc.w[it].z;
				d[3] = Wc.w[it].w;
			}
			Sn.len = Wc.len;
			__builtin_amdgcn_wave_barrier();
			if (gi1 < n) {
				Pkt<W> p{ myrow, nullptr, Sn.len };
				Parsed r;
				r.abort_at = NST;
				r.l3 = 0;
				r.l4proto = 0;
				const bool fast = parse_fast<FEAT, W>(p, r);
				df = !fast;
				if (fast) {
					Sn.inf = 1 | (r.abort_at << 1);
					if constexpr (PORTS) {
						if (r.abort_at == NST && a.port_count && r.l4proto) {
							const uint32_t pm = r.l4proto == 17 ? M_UDP : M_TCP;
							uint32_t t = CT_NONE;
							if (check_port(a, s_pbits, r.pdst, M_DST | pm, t) ||
							    check_port(a, s_pbits, r.psrc, M_SRC | pm, t))
								Sn.pt = t;
						}
					}
					if (r.l3 == 1) {
						Sn.key = row32(myrow, koff);
						if (Sn.key == 0) {
							Sn.inf |= 16 | 32;
						} else {
							Sn.inf |= 16;
							Sn.h = xfg_hash_v4(Sn.key, a.t4.seed);
							if (a.t4.bloom_words)
								bwi = xfg_bloom_word(Sn.h, a.t4.bloom_words);
						}
					}
				}
			}
		}
		// one Bloom load per lane, always issued (see load_win)
		Sn.bw = bloom_base[bwi];
		// ------------------------------------------------ windows of tile i+2
		// (clamped to the wave's last tile: a fixed load count per iteration)
		load_win(tile_of(i + 2 < my_nt ? i + 2 : (my_nt ? my_nt - 1 : 0)), Wc.w, Wc.len);
		// ------------------------------------------------ S2 (tile i-1)
		uint32_t act = A_NONE, tag = CT_NONE;
		bool fk = false;
		const uint32_t gi2 = s2 ? tile_of(i - 1) * 64 + lane : 0;
		if (s2 && (Sp.inf & 1)) {
			const uint32_t ab = (Sp.inf >> 1) & 7;
			const uint32_t alt_act = ab != NST ? A_ABORTED : Sp.pt != CT_NONE ? HIT : MISS;
			const uint32_t alt_tag = ab != NST ? CT_NONE : Sp.pt;
			bool maybe = false;
			if (Sp.inf & 16) {
				if (Sp.inf & 32) {
					maybe = a.t4.zero_present;
				} else {
					const unsigned long long bm = xfg_bloom_mask(Sp.h);
					maybe = !a.t4.bloom_words || (Sp.bw & bm) == bm;
				}
			}
			if (maybe) {
				act = HIT;
				if (!(a.ablate & 8)) {
					const uint32_t b = (Sp.inf & 32) ? a.t4.nbuckets : xfg_home(Sp.h, a.t4.nbuckets);
					const uint32_t p = b >> XFG_SLOG_SHIFT;
					const uint32_t pos = atomicAdd(&s_scnt[p], 1u);
					if (pos < a.slog_cap) {
						const u32x4 rec = { gi2, Sp.key, alt_tag,
								    alt_act | (kmask << 4) | (HIT << 8) |
								    ((Sp.inf & 32) ? 1u << 12 : 0u) };
						static_cast<u32x4 *>(a.slog)[((uint64_t)p * gridDim.x +
									      blockIdx.x) * a.slog_cap + pos] = rec;
					} else {
						fk = true;   // region full: the serial pass decides
						act = A_NONE;
					}
				}
			} else {
				act = alt_act;
				tag = alt_tag;
			}
		}
		// ------------------------------------------------ stores
		if (s1)
			defer(df, gi1);
		if (s2) {
			defer(fk, gi2);
			if (act != A_NONE)
				a.verdicts[gi2] = (uint8_t)act;
			if (a.ablate & 2)
				tag = CT_NONE;
			bump(tag);
			count_stats(act, Sp.len);
		}
	};
	// (a wave without tiles must not enter: its clamped loads would read
	// past the batch)
	for (uint32_t i = 0; my_nt && i < my_nt + 1; i += 2) {
		body(i, W0, X1, X0);
		if (i + 1 < my_nt + 1)
			body(i + 1, W1, X0, X1);
	}
	// ---- the deferred packets, serially
	if (nfix) {
		__threadfence_block();
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
	for (uint32_t p = tid; p < a.slog_parts; p += TILE)
		a.slog_cnt[(uint64_t)p * gridDim.x + blockIdx.x] =
			s_scnt[p] < a.slog_cap ? s_scnt[p] : a.slog_cap;
}

// ---------------------------------------------------------------- resolve
// One workgroup per partition of SLOG_LB buckets: the lines in LDS, a u32
// hit histogram per slot, every record of the partition checked against its
// home line exactly as CHECK_MAP does (xdpfilt_prog.h:56-64).
constexpr int SR_THREADS = 1024;

__global__ __launch_bounds__(SR_THREADS) void xfg_spec_resolve_kernel(const xfg_kargs a, uint32_t grid)
{
	__shared__ u32x4 lines[SLOG_LB * 4];
	__shared__ uint32_t cnt[SLOG_LB * XFG_SLOTS_V4];
	// false positives: stats deltas and the counters they fall through to
	// (a ruled port is hot) are summed here, not with contended atomics
	__shared__ unsigned long long s_fix[6];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	const uint32_t p = blockIdx.x, tid = threadIdx.x;
	const uint32_t b0 = p * SLOG_LB;
	const uint32_t nb = a.t4.nbuckets + 1 - b0 < SLOG_LB ? a.t4.nbuckets + 1 - b0 : SLOG_LB;
	const u32x4 *src = static_cast<const u32x4 *>(a.t4.buckets) + (uint64_t)b0 * 4;
	for (uint32_t i = tid; i < nb * 4; i += SR_THREADS)
		lines[i] = src[i];
	for (uint32_t i = tid; i < SLOG_LB * XFG_SLOTS_V4; i += SR_THREADS)
		cnt[i] = 0;
	if (tid < 6)
		s_fix[tid] = 0;
	for (uint32_t i = tid; i < CC_ENTRIES; i += SR_THREADS) {
		s_ctag[i] = CT_NONE;
		s_ccnt[i] = 0;
	}
	__syncthreads();
	for (uint32_t w = tid; w < grid; w += SR_THREADS) {
		const uint64_t r = (uint64_t)p * grid + w;
		const uint32_t c = a.slog_cnt[r];
		const u32x4 *e = static_cast<const u32x4 *>(a.slog) + r * a.slog_cap;
		for (uint32_t k0 = 0; k0 < c; k0 += 4) {
		// four records in flight per thread (they are independent)
		u32x4 rq[4];
#pragma unroll
		for (int q = 0; q < 4; q++)
			rq[q] = k0 + q < c ? __builtin_nontemporal_load(e + k0 + q) : u32x4{ 0, 0, 0, 0 };
#pragma unroll
		for (int q = 0; q < 4; q++) {
			if (k0 + q >= c)
				break;
			const u32x4 rec = rq[q];
			const uint32_t gi = rec.x, key = rec.y, alt_tag = rec.z, meta = rec.w;
			const uint32_t mask = (meta >> 4) & 15, hit_act = (meta >> 8) & 3,
				       alt_act = meta & 15;
			bool hit = false;
			if (meta & (1u << 12)) {   // the all-zero key: bucket nbuckets, slot 0
				const uint32_t lb = a.t4.nbuckets - b0;
				if (((lines[lb * 4 + 3].x & 0xff) & mask) == mask) {
					hit = true;
					atomicAdd(&cnt[lb * XFG_SLOTS_V4], 1u);
				}
			} else {
				const uint32_t b = xfg_home(xfg_hash_v4(key, a.t4.seed), a.t4.nbuckets);
				const uint32_t lb = b - b0;
				const Line l = { lines[lb * 4], lines[lb * 4 + 1], lines[lb * 4 + 2],
						 lines[lb * 4 + 3] };
				const int si = match_v4(l, key);
				if (si >= 0) {
					if ((l.flag(si) & mask) == mask) {
						hit = true;
						atomicAdd(&cnt[lb * XFG_SLOTS_V4 + si], 1u);
					}
				} else if (l.overflow() && a.t4.max_disp) {
					// displaced key: the rest of the chain from HBM
					const Hit h = probe_chain<4, false>(a.t4, b, key, 0, 0, 0);
					if (h.slot >= 0 && (h.flags & mask) == mask) {
						hit = true;
						atomicAdd(a.t4.hits + h.slot, 1ull);
					}
				}
			}
			if (!hit) {
				// Bloom false positive: the packet continues past the
				// lookup, as the reference program does
				a.verdicts[gi] = (uint8_t)alt_act;
				if (alt_tag != CT_NONE && !cache_hit(s_ctag, s_ccnt, alt_tag, 1))
					atomicAdd(global_counter(a, alt_tag), 1ull);
				const unsigned long long len = load_len(a, gi);
				atomicAdd(&s_fix[hit_act * 2], ~0ull);          // -1
				atomicAdd(&s_fix[hit_act * 2 + 1], 0ull - len);
				atomicAdd(&s_fix[alt_act * 2], 1ull);
				atomicAdd(&s_fix[alt_act * 2 + 1], len);
			}
		}
		}
	}
	__syncthreads();
	for (uint32_t i = tid; i < nb * XFG_SLOTS_V4; i += SR_THREADS)
		if (cnt[i])
			atomicAdd(a.t4.hits + (uint64_t)b0 * XFG_SLOTS_V4 + i, (unsigned long long)cnt[i]);
	if (tid < 6 && s_fix[tid])
		atomicAdd(&a.stats[tid], s_fix[tid]);
	for (uint32_t i = tid; i < CC_ENTRIES; i += SR_THREADS)
		if (s_ctag[i] != CT_NONE && s_ccnt[i])
			atomicAdd(global_counter(a, s_ctag[i]), (unsigned long long)s_ccnt[i]);
}
