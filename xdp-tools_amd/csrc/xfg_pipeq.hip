// SPDX-License-Identifier: GPL-2.0
//
// xfg_pipeq.hip — the IPv4-key pipelined classify over the quotient index
// (kargs.qt; layout: xfg_layout.h).  Included by xfg_kernels.hip after
// xfg_pipeline.hip, whose parse (parse_bf), port probe and packing it uses.
//
// Why: the reference program's map lookup (CHECK_MAP,
// xdp-filter/xdpfilt_prog.h:56-64) is a random access per packet, and on
// gfx950 what a tile's random reads cost beside the frame stream is set by
// the distinct LINES they touch: 64 random lines per 64-packet tile add
// ~0.25 ms per 2^26 packets, 32 lines 0.07, 16 lines 0.02, from a table of
// 0.5 to 4 MB alike (tools/mb_vm.hip, profiles/archive/r03_mb_vm*.log).  The
// quotient index is the IPv4 map reduced to one 32-byte bucket per lookup
// -- 2^bits buckets of 16 entries, a bijective key hash so that a bucket's
// 15-bit remainders identify their keys exactly, only keys that carry the
// one live direction's mask -- read as two 16-byte halves by two lanes of
// ONE load instruction (32 packets' buckets per instruction, so each line
// is looked up once) and moved to the packet's lane by v_permlane32_swap:
// no prefilter hop, no LDS.  Lanes without a lookup load bucket 0 (one
// shared line), so they add no lines.
//
// Used when only IPv4 keys can hit (flag census), every device carries the
// same flags, and the map is large (xfg_ctx.c fill_kargs); with both lookup
// directions live (BOTH) each packet reads its dst bucket and its src
// bucket (one image for src|dst rule sets, two otherwise).  Results are
// identical to xfg_pipe4_kernel's: a miss in a bucket that overflowed, and
// every shape the static parse does not cover, go to the deferred list and
// the canonical table (classify_staged).
//
// Per wave, iteration k works on three tiles of 64 packets:
//   R  tile k-1's buckets (loaded by L last iteration): match -> verdict
//   W  tile k-1's verdict stores, counters, stats, deferrals
//   S  tile k's windows (loaded two iterations ago) into the LDS rows
//   L  tile k's key hashed from the row's fixed dwords, its buckets: two
//      dwordx4 loads, 32 packets' buckets each (before the parse: the
//      loads gain its duration)
//   P  parse tile k, plan its fallback (ports from LDS)
//   I  tile k+2's windows and length issued
// One wait per iteration, at its top: everything but the newest tile's
// CPP + 1 loads.  Every iteration issues the same loads (a lane without a
// lookup loads bucket 0), so the count is fixed.
// The hit log is write-combined in LDS (below): ring sizes per window.
#ifndef XFG_QT_LAG       /* iterations between a tile's bucket loads and their match */
#define XFG_QT_LAG 1
#endif
#ifndef XFG_QT_DEPTH     /* tiles of windows in flight per wave (3: with XFG_QT_LAG 2 only) */
#define XFG_QT_DEPTH 2
#endif
#ifndef XFG_QT_SPEC      /* both directions: src buckets loaded with the dst ones (A/B) */
#define XFG_QT_SPEC 0
#endif
#ifndef XFG_QT_OWNC      /* a wave owns PPW consecutive log partitions (0: every NW-th) */
#define XFG_QT_OWNC 1
#endif
#ifndef XFG_QT_SWZ       /* (A/B) lanes 8g..8g+7 carry one 16-byte piece of 8 packets */
#define XFG_QT_SWZ 0
#endif
#ifndef XFG_QT_LANEW     /* (A/B) each lane loads its own frame's window: no LDS rows */
#define XFG_QT_LANEW 0
#endif
#ifndef XFG_QT_ROWQ      /* rows of 16-byte-aligned stride: b128 LDS writes and reads (0: b32) */
#define XFG_QT_ROWQ 1
#endif
#ifndef XFG_QT_NTLEN     /* lengths loaded non-temporal (A/B) */
#define XFG_QT_NTLEN 0
#endif
#ifndef XFG_QT_NTLOG     /* hit-log stores non-temporal (A/B) */
#define XFG_QT_NTLOG 0
#endif
#ifndef XFG_QT_WC_R      /* ring entries per partition, 64-byte windows */
#define XFG_QT_WC_R 128
#endif
#ifndef XFG_QT_WC_F      /* flush chunk, 64-byte windows: 64 entries, one 128-byte line */
#define XFG_QT_WC_F 64
#endif
#ifndef XFG_QT_WC_R128   /* ... 128-byte windows (4 waves: two workgroups a CU) */
#define XFG_QT_WC_R128 32
#endif
#ifndef XFG_QT_ORDER     /* 1: W after L -- the bucket loads issued before the verdict / log work */
#define XFG_QT_ORDER 0
#endif
#ifndef XFG_QT_VST       /* 1: a tile's verdict bytes stored at the top of the next iteration */
#define XFG_QT_VST 0
#endif
#ifndef XFG_QT_VGRP      /* 1: a wave's tiles in runs of 4 consecutive tiles, verdicts stored 256 B at once */
#define XFG_QT_VGRP 0
#endif
#ifndef XFG_QT_CNT2      /* 1: the hit's ring atomics without exec masks (a word per lane past the rings) */
#define XFG_QT_CNT2 1
#endif
#ifndef XFG_QT_PKM       /* 1: the bucket match by packed u16 min (no compare masks in SGPRs; A/B:
			    16 fewer SALU and 4 more VALU a tile, 0.5-0.7 % slower at 2^26, r06_s2) */
#define XFG_QT_PKM 0
#endif
#ifndef XFG_QT_PLIP      /* 1: the bucket halves swapped in place by inline asm */
#define XFG_QT_PLIP 0
#endif
#ifndef XFG_QT_DYN       /* 1: a workgroup's waves take its tiles from an LDS counter (0: a fixed share each) */
#define XFG_QT_DYN 1
#endif
#ifndef XFG_QT_PADV      /* (A/B only: extra VALU / SALU instructions per tile, to price one) */
#define XFG_QT_PADV 0
#endif
#ifndef XFG_QT_PADS
#define XFG_QT_PADS 0
#endif

namespace {

// Deferred packets [d0, d0 + 64) of a wave's list (ndef entries): the whole
// reference walk over the canonical tables (classify_staged), the verdict
// stored; returns the action, the counter identity and length for the
// caller's counting.  Whole wave.
template <uint32_t FEAT, int W>
__device__ __forceinline__ uint32_t qt_drain_one(const xfg_kargs &a, const uint32_t *s_ports, uint32_t *row,
						const uint32_t *dlist, uint32_t d0, uint32_t ndef, uint32_t &tag,
						uint32_t &len)
{
	const int lane = threadIdx.x & 63;
	tag = CT_NONE;
	len = 0;
	const bool ok = d0 + lane < ndef;
	const uint32_t gi = ok ? gld32(dlist + d0 + lane) : 0u;
	if (ok)
		len = min(load_len(a, gi), a.stride);
	const uint32_t act = classify_staged<FEAT, W>(a, s_ports, row, ok, gi, len, tag);
	if (ok)
		__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
	return act;
}

// The count wave (CW): the ninth wave of a quotient-index workgroup counts
// the PREVIOUS launch's hit log while the other eight classify -- what the
// count kernel does after a launch, hidden inside the next one.  For each
// partition p this workgroup owns (p = blockIdx.x, + gridDim.x ...): the
// cw_n slices from cw_s0 (u16 local indices, one pass: log_span ==
// log_hist) summed in an LDS histogram, then added to p's QT-order counts
// with plain read-modify-writes -- the partition's counts in qt_hits have no
// other writer during the launch (the kernel's atomics go to qt_hitx).  A
// load instruction covers 64 / G slices of G lanes, 8 entries a lane, G the
// fewest lanes whose 8 G entries hold the partition's fullest slice (the
// bench's 2^24 batch: ~115 entries a slice, four slices an instruction),
// U instructions in flight.
typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __noinline__ void qt_count_wave(const xfg_kargs &a, lds_u32 *hist)
{
	constexpr uint32_t U = 8;
	const uint32_t lane = threadIdx.x & 63;
	const uint32_t S = rfl(a.cw_n), s0 = rfl(a.cw_s0), PS = rfl(a.pslices), cap = rfl(a.pcap);
	const uint32_t hn = rfl(a.log_hist);
	for (uint32_t p = blockIdx.x; p < XFG_LOG_PARTS; p += gridDim.x) {
		for (uint32_t i = lane; i < hn; i += 64)
			hist[i] = 0;
		const uint32_t *pf = a.pfill + (uint64_t)p * PS + s0;
		uint32_t mx = 0;
		for (uint32_t s = lane; s < S; s += 64)
			mx = max(mx, min(gld32(pf + s), cap));
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
		mx = rfl(mx);
		const uint32_t lgG = mx <= 64 ? 3u : mx <= 128 ? 4u : mx <= 256 ? 5u : 6u;
		const uint32_t G = 1u << lgG, per = 64u >> lgG;
		const uint32_t lg = lane >> lgG, lr = lane & (G - 1);
		const uint32_t chunks = (mx + G * 8 - 1) / (G * 8);   // (more than one: G 64 only)
		const uint16_t *pb = a.pbuf + ((uint64_t)p * PS + s0) * cap;
		__builtin_amdgcn_wave_barrier();
		auto add8 = [&](const u32x4 &v, uint32_t i0, uint32_t f) {
#pragma unroll
			for (uint32_t c = 0; c < 4; c++) {
				const uint32_t l0 = v[c] & 0xffffu, l1 = v[c] >> 16;
				if (i0 + 2 * c < f && l0 < hn)
					__atomic_fetch_add(&hist[l0], 1u, __ATOMIC_RELAXED);
				if (i0 + 2 * c + 1 < f && l1 < hn)
					__atomic_fetch_add(&hist[l1], 1u, __ATOMIC_RELAXED);
			}
		};
		// work items: (slice group, chunk), U loads in flight
		const uint32_t ngrp = (S + per - 1) / per, nitem = ngrp * chunks;
		for (uint32_t it = 0; it < nitem; it += U) {
			u32x4 v[U];
			uint32_t fl[U], i0[U];
#pragma unroll
			for (uint32_t u = 0; u < U; u++) {
				const uint32_t w = it + u, g = w / chunks, c = w - g * chunks;
				const uint32_t sl = g * per + lg;
				fl[u] = w < nitem && sl < S ? min(gld32(pf + sl), cap) : 0u;
				i0[u] = c * G * 8 + lr * 8;
				v[u] = i0[u] < fl[u] ? *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(
								(uintptr_t)(pb + (uint64_t)sl * cap + i0[u]))
						     : u32x4{ 0, 0, 0, 0 };
			}
#pragma unroll
			for (uint32_t u = 0; u < U; u++)
				add8(v[u], i0[u], fl[u]);
		}
		__builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the histogram's atomics done
		__builtin_amdgcn_wave_barrier();
		// (R counts a lane loaded at once, then added and stored: the
		// loads' latency paid once per R, not once per count)
		constexpr uint32_t R = 16;
		for (uint32_t l0 = 0; l0 < hn; l0 += 64 * R) {
			uint32_t cur[R];
#pragma unroll
			for (uint32_t r = 0; r < R; r++) {
				const uint32_t l = l0 + r * 64 + lane;
				cur[r] = l < hn ? gld32(a.qt_hits + (((l >> 4) << 12) | (p << 4) | (l & 15))) : 0u;
			}
#pragma unroll
			for (uint32_t r = 0; r < R; r++) {
				const uint32_t l = l0 + r * 64 + lane;
				const uint32_t c = l < hn ? (uint32_t)hist[l] : 0u;
				if (c)
					gst32(a.qt_hits + (((l >> 4) << 12) | (p << 4) | (l & 15)), cur[r] + c);
			}
		}
		__builtin_amdgcn_wave_barrier();
	}
}

template <uint32_t FEAT, int W, bool DENSE, bool L16, bool BOTH, bool WIDE, uint32_t V6, bool CW = false>
__global__ __launch_bounds__(QT_THREADS(W) + (CW ? 64 : 0), QT_MINW(W)) void xfg_pipeq_kernel(const xfg_kargs a)
{
	static_assert((FEAT & F_IPV4) != 0, "IPv4-key mode needs the IPv4 feature");
	constexpr int NW = QT_WAVES(W);
	constexpr int NT = 64 * NW;
	constexpr int CPP = W / 16;
	// (ROWQ: a 16-byte-aligned row stride of 20 / 36 dwords -- b128 accesses
	// of 16 lanes at a time fall in disjoint banks -- written and read a
	// quarter-line at a time, the parse working from registers)
	constexpr bool ROWQ = XFG_QT_ROWQ != 0;
	constexpr int ROWDW = ROWQ ? W / 4 + 4 : W / 4 + 1;
	constexpr int NQ = W >= 68 ? 5 : 4;   // (ROWQ) the row's first 16-byte pieces the parse reads
	// (LANEW, 64-byte windows: lane L's four loads are its own frame's
	// window, parsed from registers -- no row staging, strided loads)
	constexpr bool LANEW = XFG_QT_LANEW != 0 && W == 64;
	// (SWZ, 64-byte windows: lane L of load it carries piece (L >> 3) & 3 of
	// packet 16 it + 8 (L >> 5) + (L & 7) -- the same kilobyte, so that each
	// group of 8 lanes of the row store writes one piece of 8 consecutive
	// rows, whose banks are disjoint at the 20-dword row stride)
	constexpr bool SWZ = XFG_QT_SWZ != 0 && W == 64 && !LANEW;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t LAG = XFG_QT_LAG;
	static_assert(LAG == 1 || LAG == 2, "bucket lag: one or two iterations");
	// (both directions: the src buckets loaded in R are matched the next
	// iteration, so a third tile of windows could not stay in flight)
	constexpr uint32_t D = BOTH ? 2u : XFG_QT_DEPTH;
	// (both directions: the src buckets loaded in R for the packets whose dst
	// lookup decided nothing, matched by R2 an iteration later -- or, SPEC,
	// loaded beside the dst buckets in L for every IPv4 packet and matched
	// in R with them)
	constexpr bool SPEC = BOTH && XFG_QT_SPEC;
	constexpr bool R2 = BOTH && !SPEC;
	// V6P (IPv6 keys live beside the index, one direction, kargs.v6p): the
	// IPv6 lookups in the loop -- up to 16 IPv6 frames of a tile, their home
	// bucket lines of the canonical IPv6 table loaded four lanes to a line
	// (ONE load instruction), moved to the frame's lane through LDS and
	// matched next iteration; a 17th frame, the zero key and a miss in an
	// overflowed bucket are deferred.  V6 2 (V6B): both IPv6 directions live
	// -- a second line per frame, its src key's home bucket, loaded by a
	// second instruction beside the first and matched after the dst line
	// only where the dst lookup decided nothing (lookup_verdict_ipv6,
	// xdpfilt_prog.h:152-165: dst first, the first hit's counter alone)
	constexpr bool V6P = V6 != 0, V6B = V6 == 2;
	// (with both IPv4 directions (BOTH) the IPv6 frames' results ride in
	// R2's state with every other frame's: their lookups are the R stage's,
	// an IPv6 frame has no IPv4 src lookup to wait for)
	static_assert(V6 <= 2 && (!V6P || ((FEAT & F_IPV6) != 0 && !WIDE) || !BOTH), "IPv6 lookups");
	static_assert(V6 <= 2 && (!V6P || (FEAT & F_IPV6) != 0), "IPv6 lookups need the IPv6 feature");
	// bucket loads per iteration issued before the windows (L, L6)
	constexpr uint32_t NL = 2 + (SPEC ? 2 : 0) + (V6P ? 1 : 0) + (V6B ? 1 : 0);
	static_assert(D == 2 || (D == 3 && LAG == 2), "window depth: 2, or 3 with a bucket lag of 2");
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	constexpr uint32_t QTAG = CT_QTAG;   // tag bit: a QT slot (hit log), not a counter identity
	// Write-combined hit log.  A QT hit of partition p = log_part(slot)
	// goes, as its 16-bit local index, into p's ring of WR entries in LDS
	// (reserve a place: s_res[p]; take a ticket: s_hd[2p]; write; count the
	// write done: s_hd[2p + 1]).  Wave p / PPW owns p: once an iteration it
	// moves completed chunks of WF entries (all tickets written: done ==
	// head) into the workgroup's slice of p's partition buffer -- the
	// layout log_partition writes and xfg_log_count_kernel reads -- and
	// gives their places back.  A hit that finds the ring full (a hot key)
	// is summed in the LDS counter cache instead (QT tag), as is a chunk
	// that would overrun the slice.  No per-wave log, no workgroup-end sort.
	// partitions a wave owns (ownp): wave wv the consecutive run
	// [wv * 256 / NW, (wv + 1) * 256 / NW) -- PPW of them, or one fewer when
	// NW does not divide 256
	constexpr uint32_t PPW = (XFG_LOG_PARTS + NW - 1) / NW;
	static_assert(PPW <= 64 && (XFG_QT_OWNC || PPW * NW == XFG_LOG_PARTS), "partition ownership");
	// (WIDE: an index past 2^20 buckets -- local indices past 16 bits -- logs
	// u32 entries, a ring of the same bytes: half the entries; with 64-byte
	// windows a flush chunk is still a line)
	typedef typename std::conditional<WIDE, uint32_t, uint16_t>::type ring_t;
	constexpr uint32_t WR = (W <= 64 ? XFG_QT_WC_R : XFG_QT_WC_R128) / (WIDE ? 2 : 1);
	constexpr uint32_t WF = W <= 64 ? XFG_QT_WC_F / (WIDE ? 2 : 1) : WR / 2;   // flush chunk
	static_assert((WR & (WR - 1)) == 0 && WF <= 64, "ring: a power of two");
	__shared__ __attribute__((aligned(16))) uint32_t win[NW * 64 * ROWDW];
	// (CNT2: 64 words past the partitions, one a lane, take the atomics of
	// the lanes without a logged hit -- or a port hit -- so that the whole
	// wave runs them with no exec mask)
	constexpr uint32_t XL = XFG_QT_CNT2 ? 64u : 0u;
	__shared__ ring_t s_ring[XFG_LOG_PARTS * WR + XL];
	__shared__ uint32_t s_res[XFG_LOG_PARTS + XL];
	__shared__ __attribute__((aligned(8))) uint32_t s_hd[2 * (XFG_LOG_PARTS + XL)];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	// (EKF: past the ports' counters and the lanes' words, one a key-table
	// entry -- a live Ethernet key's hits, flushed once per workgroup)
	constexpr bool EKF = (FEAT & F_ETH) != 0;
	constexpr uint32_t EKC = EKF ? XFG_EK_SLOTS_MAX : 0u;
	static_assert(!EKF || PORTS, "the Ethernet lookups count beside the ports");
	static_assert(XFG_PORT_TAB + XL + EKC <= 0x1000u, "a counter slot fits its 12 bits");
	__shared__ uint32_t s_pcnt[PORTS ? XFG_PORT_TAB + XL + EKC : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES], s_tn[NW];
	__shared__ uint32_t s_lh[XFG_LOG_PARTS];
	__shared__ unsigned long long s_stats[6];
	__shared__ uint32_t s6b[V6P ? NW * (V6B ? 32 : 16) : 1];   // (V6P) a tile's IPv6 home buckets, by rank (V6B: + src)
	// (their lines, four lanes each; an A/B build with more than 8 waves has
	// no room for them: its IPv6-lookup variants trap rather than launch)
	constexpr bool V6ROOM = NW <= 8;
	__shared__ u32x4 s6l[V6P && V6ROOM ? NW * 64 : 1];
	if constexpr (V6P && !V6ROOM)
		__builtin_trap();
	constexpr uint32_t G = XFG_QT_VGRP ? 4u : 1u;   // tiles per run (VGRP)
	__shared__ uint32_t s_vb[G > 1 ? NW * 64 : 1];   // (VGRP) a run's verdict bytes, per wave
	extern __shared__ uint32_t s_dyn[];

#ifdef XFG_DIAG
	// (diagnostics: 1 no counting, 2 no bucket loads, 8 no verdict stores,
	// 16 no workgroup-end partition, 32 no LDS row staging, 64 no parse, 128
	// no stats or deferral lists, 2048 no deferred packets, 4096 hits as
	// memory-side atomics into scratch instead of the hit log, 8192 no match,
	// 16384 no hit-log store -- results wrong)
	const uint32_t dg = a.diag;
#else
	constexpr uint32_t dg = 0;
#endif
	const int tid = threadIdx.x, lane = tid & 63;
	// (diagnostics: phase stamps, 32 a workgroup -- 0 entry, 1 set-up done,
	// 2 + w wave w's loop done (10: the count wave's), 11 + w its deferred
	// walk done, 22 + w wave w at the first end barrier, 30 past it, 20 the
	// partitions moved, 21 wave 0's end)
#ifdef XFG_DIAG
#define QT_STAMP(slot)                                                                        \
	do {                                                                                  \
		if (a.tstamp && lane == 0)                                                    \
			a.tstamp[(uint64_t)blockIdx.x * 32 + (slot)] = wall_clock64();        \
	} while (0)
#else
#define QT_STAMP(slot) do { } while (0)
#endif
	if (tid == 0)
		QT_STAMP(0);
	auto piece = [&](int it, uint32_t &pk, uint32_t &sub) {
		const uint32_t c = it * 64 + (uint32_t)lane;
		pk = SWZ ? it * 16 + ((uint32_t)lane >> 5) * 8 + ((uint32_t)lane & 7) : c / CPP;
		sub = SWZ ? ((uint32_t)lane >> 3) & 3 : c % CPP;
	};
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
	static_assert(!CW || (W == 64 && !WIDE && !V6), "the count wave: u16 logs, 64-byte windows");
	const bool cwv = CW && wv == NW;   // (the count wave: no classify work)
	// the index, in scalar registers
	const uint64_t qb = rfl64((uint64_t)(uintptr_t)a.qt);
	const uint32_t qbits = rfl(a.qt_bits), qseed = rfl(a.qt_seed);
	const uint32_t rsh = 32 - qbits, rmask = (1u << rsh) - 1;
	const bool dlive = BOTH || a.qt_live == M_DST;   // the one live key: dst (else src)
	// (both directions: the src lookup's image and its QT slots' offset)
	const uint64_t qb2 = BOTH ? rfl64((uint64_t)(uintptr_t)a.qt2) : 0;
	const uint32_t qbase2 = BOTH ? rfl(a.qt_base) : 0u;
	const bool klive = a.t4.count != 0;
	// (no hit log -- an index too large for the count kernel to pay, the
	// host's choice: every hit through the LDS counter cache or an atomic)
	const bool logon = a.pbuf != nullptr;
	// (IPv6 keys live, no Ethernet key: every IPv6 frame takes the deferred
	// path -- the whole reference walk over the canonical tables)
	const bool v6d = (FEAT & F_IPV6) != 0 && a.v6d != 0;
	// (V6P: the canonical IPv6 table, its one live direction)
	const uint64_t b6base = V6P ? rfl64((uint64_t)(uintptr_t)a.t6.buckets) : 0;
	const uint32_t nb6 = V6P ? rfl(a.t6.nbuckets) : 0u, seed6 = V6P ? rfl(a.t6.seed) : 0u;
	const bool md6 = V6P && a.t6.max_disp != 0, k6live = V6P && a.t6.count != 0;
	const bool d6 = V6B || (a.t6.fmask & M_DST) == M_DST;
	const uint32_t m6 = d6 ? M_DST : M_SRC, gb6 = rfl(a.gbase[1]);
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv;
	const uint32_t step = gridDim.x * NW;
	// iteration kk's tile: every step-th tile (G 1), or runs of G consecutive
	// tiles, every step-th run (G 4: a run's 256 verdict bytes contiguous)
	auto tileOf = [&](uint32_t kk) -> uint32_t {
		return G == 1 ? first + kk * step : (first + (kk / G) * step) * G + (kk % G);
	};
	// (DYN: the workgroup's tiles -- round r holds tiles blockIdx.x * NW + j
	// + r * step, j < NW -- taken by its waves from an LDS counter: each wave
	// its own tile of rounds 0..D, loaded before the set-up as in the fixed
	// share, then the next free one for every later iteration, taken an
	// iteration before its windows are loaded.  Waves that share a SIMD do
	// not progress alike: with a fixed share the workgroup's first wave
	// ended its loop ~90 us before its last at 2^26, tools/qt_phases.py.  A
	// wave takes at most defer_cap / 64 tiles, its deferred list's room.
	// Not with the Ethernet key table: its state beside the table's took
	// C3e from 0.320 to 0.355 ms at 2^24, dynamic or not -- scalar
	// registers spilled; r06_s8 / r06_s14_session.log)
	constexpr bool DYN = XFG_QT_DYN && G == 1 && !EKF;
	__shared__ uint32_t s_next;
	// windows + lengths of tile t (clamped to the last tile): CPP + 1 loads,
	// always issued
	// (the length width is a template parameter: one load of a fixed kind,
	// so the compiler's wait counts stay exact across the loop)
	constexpr uint32_t lsh = L16 ? 1u : 2u;
	typedef typename std::conditional<L16, uint16_t, uint32_t>::type len_t;
	const uint64_t lb = rfl64((uint64_t)(uintptr_t)a.lens);
	auto ld_len = [](uint64_t p) {
		const auto *q = reinterpret_cast<const __attribute__((address_space(1))) len_t *>(p);
#if XFG_QT_NTLEN   /* (A/B: the lengths streamed like the windows) */
		return __builtin_nontemporal_load(q);
#else
		return *q;
#endif
	};
	// (a whole tile -- every one but a ragged last -- takes a uniform branch
	// with no per-lane clamps: a scalar tile base and per-lane offsets that
	// do not change from tile to tile; the same loads either way)
	auto issue = [&](uint32_t t, u32x4 (&pre)[CPP], len_t &plen) {
		t = t < nt ? t : nt - 1;
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64 ? 64u : n - base;
		if (rem == 64) {
			const uint8_t *tb = a.data + (uint64_t)base * (DENSE ? W : a.stride);
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				uint32_t pk, sub;
				piece(it, pk, sub);
				const u32x4 *src = LANEW ? reinterpret_cast<const u32x4 *>(tb + (uint32_t)lane * (DENSE ? W : a.stride) + it * 16)
					: DENSE ? reinterpret_cast<const u32x4 *>(tb) + (pk * CPP + sub)
						: reinterpret_cast<const u32x4 *>(tb + pk * a.stride + sub * 16);
				pre[it] = __builtin_nontemporal_load(src);
			}
			plen = ld_len(lb + ((uint64_t)base << lsh) + ((uint32_t)lane << lsh));
		} else {
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				uint32_t pk, sub;
				piece(it, pk, sub);
				if (LANEW) {
					pk = (uint32_t)lane;
					sub = (uint32_t)it;
				}
				const uint32_t q = pk < rem ? pk : 0u;
				const u32x4 *src = DENSE ? reinterpret_cast<const u32x4 *>(a.data + (uint64_t)base * W) + (q * CPP + sub)
							 : reinterpret_cast<const u32x4 *>(a.data + (uint64_t)(base + q) * a.stride + sub * 16);
				pre[it] = __builtin_nontemporal_load(src);
			}
			const uint64_t la = lb + ((uint64_t)(base + ((uint32_t)lane < rem ? lane : 0u)) << lsh);
			plen = ld_len(la);
		}
	};
	// the first tiles' windows in flight before the workgroup's LDS set-up
	// (counters, port image, log rings) and its barrier
	u32x4 preA[CPP], preB[CPP], preC[D == 3 ? CPP : 1];
	len_t lenA = 0, lenB = 0, lenC = 0;
	if (nt && !cwv) {
		issue(tileOf(0), preA, lenA);
		__builtin_amdgcn_sched_barrier(0);
		issue(tileOf(1), preB, lenB);
		__builtin_amdgcn_sched_barrier(0);
		if constexpr (D == 3) {
			issue(tileOf(2), preC, lenC);
			__builtin_amdgcn_sched_barrier(0);
		}
	}
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, NT);
	if (tid < 6)
		s_stats[tid] = 0;
	if (DYN && tid == 0)
		s_next = (D + 1) * NW;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, NT);
	const bool ptab = PORTS && a.port_count && a.port_tab;
	const uint32_t pdisp = rfl(a.port_tab_disp), gb3 = rfl(a.gbase[3]);
	// (ekon: live Ethernet keys beside the index, the Ethernet map as its
	// LDS key table -- lookup_verdict_ethernet answered in LDS before the
	// IP lookups, xdpfilt_prog.h:187-196,224-227; a hit ends the program)
	const bool ekon = EKF && a.ek != nullptr;
	const uint32_t ek_es = EKF ? rfl(a.ek_slots) : 0u, ek_disp = EKF ? rfl(a.ek_disp) : 0u;
	const uint32_t ek_seed = EKF ? rfl(a.te.seed) : 0u, ek_gb = EKF ? rfl(a.gbase[2]) : 0u;
	const bool ek_dl = ekon && can_hit(a.te.fmask, M_DST), ek_sl = ekon && can_hit(a.te.fmask, M_SRC);
	u32x4 *const s_ek = ek_base(a, s_dyn);
	if constexpr (EKF)
		if (ekon)
			for (uint32_t i = tid; i < ek_es; i += NT)
				s_ek[i] = reinterpret_cast<const u32x4 *>(a.ek)[i];
	if constexpr (PORTS)
		for (int i = tid; i < (int)(XFG_PORT_TAB + XL + EKC); i += NT)
			s_pcnt[i] = 0;
	for (int i = tid; i < (int)XFG_LOG_PARTS; i += NT)
		s_lh[i] = 0;
	for (int i = tid; i < (int)(XFG_LOG_PARTS + XL); i += NT) {
		s_res[i] = 0;
		s_hd[2 * i] = 0;
		s_hd[2 * i + 1] = 0;
	}
	// this lane's partition (lanes below PPW), the entries it has moved out
	// (OWNC: wave wv owns partitions wv * PPW .. + PPW - 1, so its lanes' head /
	// done words are consecutive: one conflict-free 8-byte LDS read)
	const uint32_t pbase = (uint32_t)wv * XFG_LOG_PARTS / NW;
	const uint32_t pcnt = ((uint32_t)wv + 1) * XFG_LOG_PARTS / NW - pbase;   // (uniform: PPW or PPW - 1)
	auto ownp = [&](uint32_t j) { return XFG_QT_OWNC ? pbase + j : j * NW + (uint32_t)wv; };
	const uint32_t wc_p = ownp((uint32_t)lane);
	uint32_t wc_fl = 0;
	const uint64_t wc_slice0 = (uint64_t)(blockIdx.x + a.pslice0) * a.pcap;
	const uint64_t wc_pstep = (uint64_t)a.pslices * a.pcap;
	__syncthreads();

	uint32_t *const rows = win + wv * 64 * ROWDW;
	const uint32_t *const myrow = rows + lane * ROWDW;
	uint32_t *const dlist = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.defer + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t tn = 0;
	// a hit's counter: a QT slot to the hit log (without one, to the LDS
	// counter cache or an atomic on its QT-order count); a ruled port's to
	// its table slot's LDS counter; any other (the deferred packets')
	// through Counters::bump
	auto count = [&](uint32_t tag, uint32_t pslot) {
		const bool q = (tag != CT_NONE) & ((tag & QTAG) != 0);
		const bool ps = pslot != XFG_PORT_TAB;   // (a port's table slot, or EKF a key-table entry's)
		const bool dc = !q & (tag < a.dcnt);
		const uint32_t qs = tag & ~QTAG;
		if constexpr (XFG_QT_CNT2) {
			if (!(dg & 4096)) {
				// the ring's protocol (below) run by every lane: a lane
				// without a logged hit reserves, takes a ticket, writes and
				// counts done on its own words past the partitions
				const bool ql = q & logon;
				const uint32_t dm = XFG_LOG_PARTS + (uint32_t)lane;
				const uint32_t p = ql ? log_part(qs) : dm;
				const uint32_t r = atomicAdd(&s_res[p], 1u);
				const bool ok = ql & (r < WR);
				const uint32_t ph = ok ? p : dm;
				const uint32_t t = atomicAdd(&s_hd[2 * ph], 1u);
				s_ring[ok ? p * WR + (t & (WR - 1)) : XFG_LOG_PARTS * WR + (uint32_t)lane] =
					(ring_t)log_local(qs);
				atomicAdd(&s_hd[2 * ph + 1], 1u);
				if constexpr (PORTS)
					atomicAdd(&s_pcnt[ps ? pslot : XFG_PORT_TAB + (uint32_t)lane], 1u);
				// rare: a full ring (or no log), counter identities other
				// than QT slots and ports
				const bool slow = (q & !ok) | (!q & !ps & (tag != CT_NONE));
				if (__ballot(slow)) {
					if (ql & !ok)
						atomicSub(&s_res[p], 1u);
					if ((q & !ok) && !cache_hit(cn.ctag, cn.ccnt, QTAG | qs, 1))
						gatomic_add32(a.qt_hitx + qs, 1u);
					if (dc & !ps)
						atomicAdd(&cn.dcnt[tag], 1u);
					cn.bump(a, pick(q | dc | ps, CT_NONE, tag), lane);
				}
				return;
			}
		}
		if (dg & 4096) {   // (diagnostics: a memory-side atomic per hit into scratch)
			if (q)
				atomicAdd(reinterpret_cast<uint32_t *>(a.pbuf) + qs, 1u);
		} else {
			if (q) {
				bool ring = false;
				if (logon) {
					const uint32_t p = log_part(qs);
					const uint32_t r = atomicAdd(&s_res[p], 1u);
					ring = r < WR;
					if (ring) {
						const uint32_t t = atomicAdd(&s_hd[2 * p], 1u);
						s_ring[p * WR + (t & (WR - 1))] = (ring_t)log_local(qs);
						atomicAdd(&s_hd[2 * p + 1], 1u);
					} else {
						atomicSub(&s_res[p], 1u);
					}
				}
				// the ring full (or no log): the LDS counter cache
				if (!ring && !cache_hit(cn.ctag, cn.ccnt, QTAG | qs, 1))
					gatomic_add32(a.qt_hitx + qs, 1u);
			}
		}
		if constexpr (PORTS)
			if (ps)
				atomicAdd(&s_pcnt[pslot], 1u);
		if (dc & !ps)
			atomicAdd(&cn.dcnt[tag], 1u);
		cn.bump(a, pick(q | dc | ps, CT_NONE, tag), lane);
	};
	// move entries [fl, fl + cnt) of lane j's partition to its slice (cnt
	// <= WR; positions past pcap: the counter cache instead)
	auto wc_move = [&](uint32_t j, uint32_t fl, uint32_t cnt) {
		const uint32_t p = ownp(j);
		for (uint32_t o = lane; o < cnt; o += 64) {
			const uint32_t e = s_ring[p * WR + ((fl + o) & (WR - 1))];
			const uint32_t pos = fl + o;
			if (pos < a.pcap) {
				auto *d = reinterpret_cast<__attribute__((address_space(1))) ring_t *>(
					(uintptr_t)(reinterpret_cast<ring_t *>(a.pbuf) + p * wc_pstep + wc_slice0 + pos));
#if XFG_QT_NTLOG   /* (A/B: the hit log's lines stored non-temporal) */
				__builtin_nontemporal_store((ring_t)e, d);
#else
				*d = (ring_t)e;
#endif
			} else {
				const uint32_t g = ((e >> 4) << 12) | (p << 4) | (e & 15);
				if (!cache_hit(cn.ctag, cn.ccnt, QTAG | g, 1))
					gatomic_add32(a.qt_hitx + g, 1u);
			}
		}
	};
	// once an iteration: this wave's partitions' completed chunks
	auto wc_flush = [&]() {
		// head and done of the partition in ONE 8-byte read (a snapshot):
		// done == head means every ticket taken has been written
		uint32_t hd0 = 0, hd1 = 0;
		if ((uint32_t)lane < pcnt) {
			const uint64_t v = *reinterpret_cast<const uint64_t *>(&s_hd[2 * wc_p]);
			hd0 = (uint32_t)v;
			hd1 = (uint32_t)(v >> 32);
		}
		unsigned long long fm = __ballot(((uint32_t)lane < pcnt) & (hd0 == hd1) & (hd1 - wc_fl >= WF));
		while (fm) {
			const uint32_t j = (uint32_t)__ffsll((long long)fm) - 1;
			fm &= fm - 1;
			const uint32_t fl = __builtin_amdgcn_readlane(wc_fl, j);
			wc_move(j, fl, WF);
			if (lane == 0)   // (after the ring reads: LDS keeps a wave's order)
				atomicSub(&s_res[ownp(j)], WF);
			wc_fl += (uint32_t)lane == j ? WF : 0u;
		}
	};
	// xdp_stats_record_action (headers/xdp/xdp_stats_kern.h): per lane, the
	// packets of each action in 10-bit fields of one word and their bytes
	// in 21-bit fields of one double word -- a shift-add each per tile,
	// the field chosen by the action (ABORTED, DROP, PASS; any other --
	// a deferred or absent packet -- into the top bits, discarded) --
	// folded into per-lane totals before a field can overflow (every
	// st_cap tiles: 1023 packets, 2^21 - 1 bytes of the longest length)
	uint32_t st_pk = 0, st_n = 0, st_c[3] = { 0, 0, 0 }, st_b[3] = { 0, 0, 0 };
	uint64_t st_bpk = 0;
	const uint32_t st_cap = rfl(min(1023u, 0x1fffffu / max(min(a.stride ? a.stride : 65535u, 65535u), 1u)));
	auto st_fold = [&]() {
#pragma unroll
		for (int k = 0; k < 3; k++) {
			st_c[k] += (st_pk >> (10 * k)) & 1023u;
			st_b[k] += (uint32_t)(st_bpk >> (21 * k)) & 0x1fffffu;
		}
		st_pk = 0;
		st_bpk = 0;
		st_n = 0;
	};
	auto stat = [&](uint32_t act, uint32_t len) {
		const uint32_t f = min(act, 3u);
		st_pk += 1u << (f * 10);
		st_bpk += (uint64_t)len << (f * 21);
		if (++st_n == st_cap)
			st_fold();
	};
	uint32_t ndef = 0;
	uint32_t vs_act = A_NONE, vs_gi = 0;   // (XFG_QT_VST) verdicts waiting for the next iteration's store


	auto pk3 = [](uint32_t act, uint32_t ps, uint32_t len) { return act | ps << 3 | len << 15; };
	auto pk_act = [](uint32_t p) { return p & 7; };
	auto pk_ps = [](uint32_t p) { return (p >> 3) & 0xfff; };
	auto pk_len = [](uint32_t p) { return p >> 15; };
	// P -> R (tile k-1): entry to find (USED | remainder), bucket, its
	// 32 bytes (L -> R), fallback
	// (XFG_QT_LAG 2: a tile's buckets are matched two iterations after its
	// loads, in the state set of its iteration's parity)
	struct RSt {
		uint32_t key, b, pk, tag, key2, b2;
		bool sel;
		u32x4 bk0, bk1, cs0, cs1;
		// (V6P) the IPv6 key, home bucket, rank in the tile, whether it is
		// looked up here; this lane's quarter of a line
		uint32_t k6[4], b6, r6;
		bool s6;
		u32x4 c6;
		// (V6B) the src key, its home bucket, this lane's quarter of its line
		uint32_t k6s[V6B ? 4 : 1], b6s;
		u32x4 c6s;
	};
	RSt stA = { 0, 0, pk3(A_NONE, XFG_PORT_TAB, 0), CT_NONE, 0, 0, false, { 0, 0, 0, 0 }, { 0, 0, 0, 0 },
		    { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, { 0, 0, 0, 0 }, 0, 0, false, { 0, 0, 0, 0 }, {}, 0, { 0, 0, 0, 0 } };
	RSt stB = stA;
	// (both directions: the src key's entry and bucket from P; tile k-1's
	// state after its dst lookup, for R2 next iteration; its src bucket)
	bool q_need = false;
	uint32_t q_act = A_NONE, q_tag = CT_NONE, q_ps = XFG_PORT_TAB, q_len = 0, q_key2 = 0, q_b2 = 0;
	u32x4 bs0 = { 0, 0, 0, 0 }, bs1 = { 0, 0, 0, 0 };
	// one bucket's 16 entries (halves in lanes i and i + 32 of h0 / h1, see
	// L) searched for entry q: found, its index, the overflow marker
	auto match = [](u32x4 &h0, u32x4 &h1, uint32_t q, bool &found, uint32_t &ix) {
		uint32_t w[8];
#pragma unroll
		for (int c = 0; c < 4; c++) {
#if XFG_QT_PLIP   /* the swap in place: the halves are dead after the match (no copies) */
			uint32_t x = h0[c], y = h1[c];
			asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
			w[c] = x;
			w[4 + c] = y;
#else
			const auto sw = __builtin_amdgcn_permlane32_swap(h0[c], h1[c], false, false);
			w[c] = sw[0];
			w[4 + c] = sw[1];
#endif
		}
		if constexpr (XFG_QT_PKM) {
			// entry e's half of w[e / 2] xor q is zero where it matches;
			// min(half, 1) per half (v_pk_min_u16) is 0 there, 1 elsewhere
			// -- dword i's two results at bits 2i and 2i + 16 of N, the
			// matching entry the lowest clear even bit (bit b: entry
			// 2 (b & 14) / 2 + b / 16); keys are unique, at most one matches
			const uint32_t qq = q * 0x10001u;
			uint32_t nm = 0;
#pragma unroll
			for (int i = 0; i < 8; i++) {
				uint32_t m;
				asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(w[i] ^ qq), "s"(0x10001u));
				nm |= m << (2 * i);
			}
			const uint32_t hitm = ~nm & 0x55555555u;
			found = hitm != 0;
			const uint32_t b = (uint32_t)__builtin_ctz(hitm | 0x80000000u);
			ix = (b & 14u) | (b >> 4);
		} else {
			found = false;
			ix = 0;
#pragma unroll
			for (int i = 0; i < 8; i++) {
				const bool lo = (w[i] & 0xffffu) == q, hi = (w[i] >> 16) == q;
				found |= lo | hi;
				ix = pick(lo, 2u * i, ix);
				ix = pick(hi, 2u * i + 1, ix);
			}
		}
		return (w[7] >> 16) == XFG_QT_OVF_MARK;
	};
	// (wcf: this iteration moves completed hit-log chunks -- every other one:
	// a ring of WR entries takes two iterations' hits with room to spare)
	// (one more with both directions: the last tile's src lookup resolves
	// an iteration after its dst lookup)
	const uint32_t nrun = (nt + G - 1) / G;
	uint32_t iters = first < nrun ? ((nrun - 1 - first) / step + 1) * G + LAG + (R2 ? 1 : 0) : 0u;
	// (DYN) tiles k - LAG - 1 .. k + D of iteration k (past the ends: nt);
	// tiles this wave has taken, the most it may; whether more may follow
	constexpr uint32_t RN = DYN ? LAG + D + 2 : 1;
	uint32_t tr[RN];
	uint32_t tmine = 0, tmax = 0;
	bool more = false;
	// (the host's choice per launch, kargs.qt_dyn: large batches; a fixed
	// share otherwise -- tile k + D + 1 then follows from k)
	const bool dyn_on = DYN && a.qt_dyn != 0;
	if constexpr (DYN) {
		tmax = rfl(a.defer_cap) / 64;
#pragma unroll
		for (uint32_t i = 0; i < RN; i++)
			tr[i] = nt;
#pragma unroll
		for (uint32_t d = 0; d <= D; d++) {
			const uint32_t t = first + d * step;
			tr[LAG + 1 + d] = t < nt ? t : nt;
			tmine += t < nt ? 1u : 0u;
		}
		more = dyn_on && tmine == D + 1;
		if (dyn_on)
			iters = more ? 0xffffffffu : tmine ? tmine + LAG + (R2 ? 1u : 0u) : 0u;
	}
	auto iteration = [&](uint32_t k, u32x4 (&cur)[CPP], len_t &curlen, RSt &rs, bool wcf) __attribute__((always_inline)) {
		// (DYN) tile k + D + 1, taken now from the counter and read at the
		// iteration's end (the atomic's return waited for with the
		// iteration's own LDS work): its windows are loaded next iteration;
		// none left (or no room left in this wave's list): the loop ends once
		// the tiles taken have drained through W
		uint32_t graw = 0xffffffffu;
		const bool take = DYN && more && tmine < tmax;
		if constexpr (DYN)
			if (take && lane == 0)
				graw = atomicAdd(&s_next, 1u);
		const uint32_t tP = DYN ? tr[LAG + 1] : tileOf(k);
		const bool vP = tP < nt;
		const uint32_t tR = DYN ? tr[1] : k >= LAG ? tileOf(k - LAG) : nt;
		const bool vR = tR < nt;
		// everything but the newest iteration's loads (LAG 1: tile k+1's
		// windows; LAG 2: also the last iteration's bucket loads; depth 3:
		// also the windows issued the iteration before)
		constexpr uint32_t VW = CPP + 1 + (LAG - 1) * NL + (D - 2) * (CPP + 1);
		__builtin_amdgcn_s_waitcnt(0x0F70 | (VW & 15) | ((VW >> 4) << 14));
		if constexpr (D == 3)   // (nothing that uses a load above the wait)
			__builtin_amdgcn_sched_barrier(0);
		// (the length is used from here on: without this the compiler
		// rotates its zero-extension to the previous iteration's end, where
		// it waits for the load -- and every older one -- early)
		asm volatile("" : "+v"(curlen));
		if constexpr (XFG_QT_VST) {   // (the last W's verdicts, their store acknowledged by the next wait)
			if (vs_act <= A_PASS)
				__builtin_nontemporal_store((uint8_t)vs_act, a.verdicts + vs_gi);
			vs_act = A_NONE;
		}

		PMARK("R");
		// ---- R: tile k-1's bucket -> CHECK_MAP (xdpfilt_prog.h:56-64)
		const uint32_t r_act = pk_act(rs.pk), r_ps = pk_ps(rs.pk), r_len = pk_len(rs.pk);
		uint32_t w_act = A_NONE, w_tag = CT_NONE, w_ps = r_ps, w_len = r_len;
		// (both directions: W works on tile k-2, whose src lookup -- read
		// last iteration for the packets whose dst lookup decided nothing --
		// R2 resolves first; one directions: W works on tile k-1)
		const uint32_t tW = R2 ? (DYN ? tr[0] : k >= LAG + 1 ? tileOf(k - LAG - 1) : nt) : tR;
		const bool vW = tW < nt;
		if constexpr (R2) {
			PMARK("R2");
			// lookup_verdict_ipv4 (xdpfilt_prog.h:121-134): the src key
			// only when the dst key decided nothing -- the first matching
			// lookup's counter alone is bumped
			w_act = q_act;
			w_tag = q_tag;
			w_ps = q_ps;
			w_len = q_len;
			if (vW && !(dg & 8192)) {
				bool f2;
				uint32_t ix2;
				const bool ovf2 = match(bs0, bs1, q_key2, f2, ix2);
				f2 &= q_need;
				const bool d2 = q_need & !f2 & ovf2;
				w_act = pick(f2, HIT, pick(d2, A_DEFER, w_act));
				w_tag = pick(f2, QTAG | (qbase2 + q_b2 * XFG_QT_SLOTS + ix2), pick(d2, CT_NONE, w_tag));
				w_ps = pick(f2 | d2, XFG_PORT_TAB, w_ps);
			}
		}
		if (vR && !(dg & 8192)) {
			// 16 entries, filled in order; keys are unique, so at most one
			// matches.  A miss in a bucket marked overflowed may be a key
			// that did not fit: the canonical table decides it (deferred).
			// the halves to their packet's lane (see L): lane i < 32 holds
			// half 0 of packet i in rs.bk0 and half 1 of packet i in lane
			// i + 32 of rs.bk0; lanes i + 32 likewise in rs.bk1 for packet 32 + i
			bool found;
			uint32_t ix;
			const bool ovf = match(rs.bk0, rs.bk1, rs.key, found, ix);
			found &= rs.sel;
			const bool defer = rs.sel & !found & ovf;
			const uint32_t slot = rs.b * XFG_QT_SLOTS + ix;
			uint32_t x_act = pick(found, HIT, pick(defer, A_DEFER, r_act));
			uint32_t x_tag = pick(found, QTAG | slot, pick(defer, CT_NONE, rs.tag));
			uint32_t x_ps = pick(found | defer, XFG_PORT_TAB, r_ps);
			if constexpr (V6P) {
				// lookup_verdict_ipv6 (xdpfilt_prog.h:152-165): the frame's
				// home line from its four lanes, three 16-byte keys, a flag
				// byte each (CHECK_MAP, :56-64), the overflow bit
				__builtin_amdgcn_wave_barrier();
				s6l[wv * 64 + lane] = rs.c6;
				__builtin_amdgcn_wave_barrier();
				// this lane's frame's line (rank r6, lanes 4 r6 .. + 3) against
				// key k: the key found with the mask's flags, a miss the
				// overflow bit leaves undecided, the slot
				auto m6line = [&](const uint32_t (&k)[4], uint32_t m, bool &f, bool &o, uint32_t &ix) {
					const u32x4 *ln = &s6l[wv * 64 + rs.r6 * 4];
					const u32x4 q0 = ln[0], q1 = ln[1], q2 = ln[2], q3 = ln[3];
					const bool e0 = (q0.x == k[0]) & (q0.y == k[1]) & (q0.z == k[2]) & (q0.w == k[3]);
					const bool e1 = (q1.x == k[0]) & (q1.y == k[1]) & (q1.z == k[2]) & (q1.w == k[3]);
					const bool e2 = (q2.x == k[0]) & (q2.y == k[1]) & (q2.z == k[2]) & (q2.w == k[3]);
					ix = pick(e0, 0u, pick(e1, 1u, 2u));
					const uint32_t fl = (q3.x >> (8 * ix)) & 0xff;
					f = (e0 | e1 | e2) & ((fl & m) == m);
					o = !(e0 | e1 | e2) & ((q3.w & XFG_META_OVERFLOW) != 0) & md6;
				};
				bool f6 = false, o6 = false;
				uint32_t i6 = 0;
				if (rs.s6)
					m6line(rs.k6, m6, f6, o6, i6);
				x_act = pick(f6, HIT, pick(o6, A_DEFER, x_act));
				x_tag = pick(f6, gb6 + rs.b6 * XFG_SLOTS_V6 + i6, pick(o6, CT_NONE, x_tag));
				x_ps = pick(f6 | o6, XFG_PORT_TAB, x_ps);
				if constexpr (V6B) {
					// the src line where the dst key decided nothing (found
					// without the dst flag, or absent from a bucket that
					// never overflowed)
					__builtin_amdgcn_wave_barrier();
					s6l[wv * 64 + lane] = rs.c6s;
					__builtin_amdgcn_wave_barrier();
					bool fs = false, os = false;
					uint32_t is = 0;
					if (rs.s6 & !f6 & !o6)
						m6line(rs.k6s, M_SRC, fs, os, is);
					x_act = pick(fs, HIT, pick(os, A_DEFER, x_act));
					x_tag = pick(fs, gb6 + rs.b6s * XFG_SLOTS_V6 + is, pick(os, CT_NONE, x_tag));
					x_ps = pick(fs | os, XFG_PORT_TAB, x_ps);
				}
			}
			if constexpr (SPEC) {   // the src lookup, its bucket loaded beside the dst one
				const bool need = rs.sel & !found & !defer;
				bool f2;
				uint32_t ix2;
				const bool ovf2 = match(rs.cs0, rs.cs1, rs.key2, f2, ix2);
				f2 &= need;
				const bool d2 = need & !f2 & ovf2;
				w_act = pick(f2, HIT, pick(d2, A_DEFER, x_act));
				w_tag = pick(f2, QTAG | (qbase2 + rs.b2 * XFG_QT_SLOTS + ix2), pick(d2, CT_NONE, x_tag));
				w_ps = pick(f2 | d2, XFG_PORT_TAB, x_ps);
			} else if constexpr (R2) {   // to R2 next iteration
				q_need = rs.sel & !found & !defer;
				q_act = x_act;
				q_tag = x_tag;
				q_ps = x_ps;
				q_len = r_len;
				q_key2 = rs.key2;
				q_b2 = pick(q_need, rs.b2, 0u);
			} else {
				w_act = x_act;
				w_tag = x_tag;
				w_ps = x_ps;
			}
		} else if constexpr (R2) {
			q_need = false;
			q_act = A_NONE;
			q_tag = CT_NONE;
			q_ps = XFG_PORT_TAB;
			q_b2 = 0;
		}
		if constexpr (R2) {
			// tile k-1's src buckets (bucket 0 for a packet whose dst lookup
			// decided it: a shared line), as L loads (see there)
			if (!(dg & 2)) {
				const auto ab2 = __builtin_amdgcn_permlane32_swap(q_b2, q_b2, false, false);
				const uint64_t hb2 = qb2 + (uint64_t)(lane >> 5) * 16;
				bs0 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb2 + ((uint64_t)ab2[0] << 5));
				bs1 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb2 + ((uint64_t)ab2[1] << 5));
			}
		}

		PMARK("W");
		// ---- W: verdicts, counters, stats, deferrals of tile k-1 (k-2)
		auto stageW = [&]() __attribute__((always_inline)) {
		if (vW) {
			const uint32_t gi = tW * 64 + lane;
			// (VGRP: a whole run's bytes gathered in LDS, stored as one
			// dword a lane at its last tile; a deferred packet's byte is
			// rewritten by the drain after the loop; a run past the batch's
			// end: bytes as they come)
			const uint32_t vj = tW % G;
			const bool vrun = G > 1 && (tW - vj + G) * 64 <= n;
			if (vrun) {
				reinterpret_cast<uint8_t *>(s_vb)[wv * 256 + vj * 64 + lane] = (uint8_t)w_act;
				if (vj == G - 1) {
					__builtin_amdgcn_wave_barrier();
					__builtin_nontemporal_store(s_vb[wv * 64 + lane],
								    reinterpret_cast<uint32_t *>(a.verdicts + (tW - vj) * 64) + lane);
				}
			} else if constexpr (XFG_QT_VST) {
				vs_act = (w_act <= A_PASS && !(dg & 8)) ? w_act : A_NONE;
				vs_gi = gi;
			} else if (w_act <= A_PASS && !(dg & 8)) {
				__builtin_nontemporal_store((uint8_t)w_act, a.verdicts + gi);
			}
			count((dg & 1) ? CT_NONE : w_tag, (dg & 1) ? XFG_PORT_TAB : w_ps);
			if (!(dg & 128))
				stat(w_act, w_len);
			const unsigned long long dm = (dg & 128) ? 0ull : __ballot(w_act == A_DEFER);
			if (dm) {
				const uint32_t pos = ndef + lanes_below(dm);
				if (w_act == A_DEFER)
					gst32(dlist + pos, gi);
				ndef += (uint32_t)__popcll(dm);
			}
		}
		if (vW && logon && wcf)
			wc_flush();
		};
		if constexpr (!XFG_QT_ORDER)
			stageW();

#if XFG_QT_PADV || XFG_QT_PADS
		{   // (A/B: a fixed number of independent do-nothing instructions)
			uint32_t pv = (uint32_t)lane, ps = k;
#pragma unroll
			for (int i = 0; i < XFG_QT_PADV; i++)
				asm volatile("v_add_u32 %0, 1, %0" : "+v"(pv));
#pragma unroll
			for (int i = 0; i < XFG_QT_PADS; i++)
				asm volatile("s_add_u32 %0, 1, %0" : "+s"(ps) :: "scc");
			asm volatile("" ::"v"(pv), "s"(ps));
		}
#endif
		PMARK("S");
		// ---- S: tile k's windows into the rows, lengths clamped to the
		// stride (rows past the batch's end hold a copy of the tile's first
		// packet: those lanes are not valid, nothing of theirs is stored or
		// counted)
		uint32_t len = 0;
		if (vP) {
			const uint32_t rem = n - tP * 64 >= 64 ? 64u : n - tP * 64;
			__builtin_amdgcn_wave_barrier();
			if (LANEW) {
				;   // (the window stays in registers)
			} else if (!(dg & 32)) {
#pragma unroll
				for (int it = 0; it < CPP; it++) {
					const int c = it * 64 + lane;
					uint32_t pk, sub;
					piece(it, pk, sub);
					(void)c;
					uint32_t *dst = &rows[pk * ROWDW + sub * 4];
					if constexpr (ROWQ) {
						*reinterpret_cast<u32x4 *>(dst) = cur[it];
					} else {
						dst[0] = cur[it].x;
						dst[1] = cur[it].y;
						dst[2] = cur[it].z;
						dst[3] = cur[it].w;
					}
				}
			} else {   // (diagnostics: the data kept live, not staged)
#pragma unroll
				for (int it = 0; it < CPP; it++)
					asm volatile("" ::"v"(cur[it]));
			}
			len = (uint32_t)lane < rem ? min((uint32_t)curlen, a.stride) : 0u;
			__builtin_amdgcn_wave_barrier();
		}

		PMARK("L");
		// ---- K + L: the key's hash from the row's fixed dwords and tile
		// k's bucket loads first, the rest of the parse after them (the
		// loads gain its duration).  Load q carries packets 32q..32q+31,
		// lane L the 16-byte half L >> 5 of packet 32q + (L & 31)'s bucket,
		// so both halves of a bucket are in ONE instruction (a line is
		// looked up once); R moves them to the packet's lane.  Every lane
		// loads (a fixed count); one whose frame is not IPv4 loads bucket 0
		// (a shared line).
		uint32_t hk = 0, lbk = 0, hk2 = 0, lbk2 = 0;
		uint32_t dw[17] = {};   // (ROWQ) the row's dwords, read four at a time
		if constexpr (LANEW) {
#pragma unroll
			for (int q = 0; q < CPP; q++) {
				dw[4 * q] = cur[q].x;
				dw[4 * q + 1] = cur[q].y;
				dw[4 * q + 2] = cur[q].z;
				dw[4 * q + 3] = cur[q].w;
			}
		} else if constexpr (ROWQ) {
			if (vP) {
#pragma unroll
				for (int q = 0; q < NQ; q++) {
					const u32x4 v = reinterpret_cast<const u32x4 *>(myrow)[q];
					dw[4 * q] = v.x;
					if (4 * q + 1 < 17)
						dw[4 * q + 1] = v.y;
					if (4 * q + 2 < 17)
						dw[4 * q + 2] = v.z;
					if (4 * q + 3 < 17)
						dw[4 * q + 3] = v.w;
				}
			}
		}
		auto rowd = [&](int j) { return (ROWQ || LANEW) ? dw[j] : myrow[j]; };
		if (vP) {
			const uint32_t e3 = rowd(3), e6 = rowd(6), e7 = rowd(7), e8 = rowd(8);
			const uint32_t key = dlive ? __builtin_amdgcn_alignbyte(e8, e7, 2) : __builtin_amdgcn_alignbyte(e7, e6, 2);
			hk = xfg_qt_hash(key, qseed);
			const bool ip4 = (e3 & 0xffffu) == 0x0008u;
			lbk = pick(ip4, hk >> rsh, 0u);
			if constexpr (BOTH) {   // the src key (saddr, bytes 26..29)
				hk2 = xfg_qt_hash(__builtin_amdgcn_alignbyte(e7, e6, 2), qseed);
				lbk2 = pick(ip4, hk2 >> rsh, 0u);
			}
		}
		if (!(dg & 2)) {
			const auto ab = __builtin_amdgcn_permlane32_swap(lbk, lbk, false, false);
			const uint64_t hb = qb + (uint64_t)(lane >> 5) * 16;
			rs.bk0 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb + ((uint64_t)ab[0] << 5));
			rs.bk1 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb + ((uint64_t)ab[1] << 5));
			if constexpr (SPEC) {
				const auto ab2 = __builtin_amdgcn_permlane32_swap(lbk2, lbk2, false, false);
				const uint64_t hb2 = qb2 + (uint64_t)(lane >> 5) * 16;
				rs.cs0 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb2 + ((uint64_t)ab2[0] << 5));
				rs.cs1 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(hb2 + ((uint64_t)ab2[1] << 5));
			}
		}
		__builtin_amdgcn_sched_barrier(0);
		if constexpr (XFG_QT_ORDER) {
			stageW();
			__builtin_amdgcn_sched_barrier(0);
		}
		PMARK("P");
		// ---- P: parse tile k, hash its key, plan its fallback
		uint32_t n6 = 0;   // (V6P) the tile's IPv6 lookups, at most 16
		rs.s6 = false;
		if (vP && (dg & 64)) {   // (diagnostics: no parse)
			const uint32_t gi = tP * 64 + lane;
			rs.b = pick(gi < n, hk >> rsh, 0u);
			rs.key = XFG_QT_USED | (hk & rmask);
			rs.sel = gi < n;
			rs.pk = pk3(pick(gi < n, MISS, A_NONE), XFG_PORT_TAB, len);
			rs.tag = CT_NONE;
		} else if (vP) {
			const uint32_t gi = tP * 64 + lane;
			Parse4 r;
			if constexpr (ROWQ || LANEW)
				r = parse_bf_dw<FEAT, W>(dw, len);
			else
				r = parse_bf<FEAT, W>(myrow, len);
			const bool valid = gi < n;
			// (ekon) the Ethernet lookups: dst MAC then src MAC against the
			// LDS table, for a frame past parse_ethhdr (14 bytes); a frame
			// the parse defers is walked whole, its MACs with it
			bool ekh = false;
			uint32_t eke = 0;
			if constexpr (EKF) {
				if (ekon) {
					uint32_t sl = 0;
					bool h = false;
					if (ek_dl)
						h = ek_probe<true>(s_ek, ek_es, ek_disp, ek_seed, dw[0], dw[1] & 0xffffu, M_DST, sl);
					if (ek_sl) {
						uint32_t s2 = 0;
						const bool h2 = ek_probe<true>(s_ek, ek_es, ek_disp, ek_seed,
									       __builtin_amdgcn_alignbyte(dw[2], dw[1], 2),
									       dw[2] >> 16, M_SRC, s2);
						sl = h ? sl : s2;
						h |= h2;
					}
					ekh = valid & (len >= 14) & !r.defer & h;
					eke = XFG_PORT_TAB + XL + sl;   // (the entry's LDS counter)
				}
			}
			bool def6 = false;
			if constexpr (V6P) {
				// the IPv6 key (daddr at 38, saddr at 22: two bytes into a
				// row dword), its home bucket, its rank among the tile's
				// lookups; ranks below 16 post their bucket for L6
				const bool k6 = valid & !r.defer & r.v6ok & k6live & !ekh;
				uint32_t w6[4], ws[4];
#pragma unroll
				for (int i = 0; i < 4; i++) {
					w6[i] = d6 ? __builtin_amdgcn_alignbyte(rowd(10 + i), rowd(9 + i), 2)
						   : __builtin_amdgcn_alignbyte(rowd(6 + i), rowd(5 + i), 2);
					ws[i] = __builtin_amdgcn_alignbyte(rowd(6 + i), rowd(5 + i), 2);   // (V6B: saddr)
				}
				// (the zero key lives in slot nslots: deferred; V6B: either)
				const bool z6 = (w6[0] | w6[1] | w6[2] | w6[3]) == 0 ||
						(V6B && (ws[0] | ws[1] | ws[2] | ws[3]) == 0);
				const unsigned long long bm6 = __ballot(k6 & !z6);
				const uint32_t rk = lanes_below(bm6);
				const bool sel6 = k6 & !z6 & (rk < 16);
				def6 = k6 & !sel6;
				const uint32_t hb6 = xfg_home(xfg_hash_v6(w6[0], w6[1], w6[2], w6[3], seed6), nb6);
				if (sel6)
					s6b[wv * (V6B ? 32 : 16) + rk] = hb6;
				if constexpr (V6B) {
					const uint32_t hs = xfg_home(xfg_hash_v6(ws[0], ws[1], ws[2], ws[3], seed6), nb6);
					if (sel6)
						s6b[wv * 32 + 16 + rk] = hs;
#pragma unroll
					for (int i = 0; i < 4; i++)
						rs.k6s[i] = ws[i];
					rs.b6s = hs;
				}
				n6 = min((uint32_t)__popcll(bm6), 16u);
#pragma unroll
				for (int i = 0; i < 4; i++)
					rs.k6[i] = w6[i];
				rs.b6 = hb6;
				rs.r6 = rk;
				rs.s6 = sel6;
			}
			// (IPv6 keys live without V6P: every IPv6 frame deferred)
			const bool rdef = r.defer | (v6d & r.is6 & !V6P) | def6;
			const bool kok = valid & !rdef & r.v4ok & klive & !ekh;
			const uint32_t h = hk;
			rs.b = pick(kok, h >> rsh, 0u);   // (no lookup: bucket 0, a shared line)
			rs.key = XFG_QT_USED | (h & rmask);
			rs.sel = kok;
			if constexpr (BOTH) {
				rs.b2 = pick(kok, hk2 >> rsh, 0u);
				rs.key2 = XFG_QT_USED | (hk2 & rmask);
			}
			uint32_t fa = pick(r.abort_at != NST, A_ABORTED, MISS), ft = CT_NONE, fs = XFG_PORT_TAB;
			if constexpr (PORTS) {
				if (a.port_count) {
					const uint32_t pm = pick(r.l4proto == 17, M_UDP, M_TCP);
					const uint32_t pfm = a.port_fmask;
					bool ph = false;
					if (can_hit(pfm, M_DST)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, r.pdst, sl);
						const uint32_t mk = M_DST | pm;
						ph = (r.l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(ph, gb3 + r.pdst, ft);
						fs = pick(ph, sl, fs);
					}
					if (can_hit(pfm, M_SRC)) {
						uint32_t sl;
						const uint32_t f = port_probe(s_ports, ptab, pdisp, r.psrc, sl);
						const uint32_t mk = M_SRC | pm;
						const bool h2 = !ph & (r.l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(h2, gb3 + r.psrc, ft);
						fs = pick(h2, sl, fs);
						ph |= h2;
					}
					fa = pick(ph, HIT, fa);
				}
			}
			fa = pick(ekh, HIT, fa);
			fs = pick(ekh, eke, fs);
			ft = pick(ekh, CT_NONE, ft);
			rs.pk = pk3(pick(!valid, A_NONE, pick(rdef, A_DEFER, fa)),
				   pick(valid & !rdef, fs, XFG_PORT_TAB), len);
			rs.tag = pick(valid & !rdef, ft, CT_NONE);
		} else {
			rs.sel = false;
			rs.b = 0;
			rs.pk = pk3(A_NONE, XFG_PORT_TAB, 0);
			rs.tag = CT_NONE;
		}

		if constexpr (V6P) {
			// ---- L6: the tile's IPv6 home lines, lane L the 16-byte quarter
			// L & 3 of rank L >> 2's line (lanes past the tile's lookups: a
			// line of bucket 0)
			__builtin_amdgcn_wave_barrier();
			const uint32_t j = (uint32_t)lane >> 2;
			const uint32_t bb = j < n6 ? s6b[wv * (V6B ? 32 : 16) + j] : 0u;
			rs.c6 = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(
				b6base + (uint64_t)bb * XFG_BUCKET_BYTES + ((uint32_t)lane & 3) * 16);
			if constexpr (V6B) {   // (the src lines: a second instruction, the same shape)
				const uint32_t bs = j < n6 ? s6b[wv * 32 + 16 + j] : 0u;
				rs.c6s = *reinterpret_cast<const __attribute__((address_space(1))) u32x4 *>(
					b6base + (uint64_t)bs * XFG_BUCKET_BYTES + ((uint32_t)lane & 3) * 16);
			}
		}

		PMARK("I");
		// ---- tile k+D's windows, last: in flight for D iterations
		// (issued before the parse instead, the compiler's register
		// reuse puts waits into R: not kept)
		__builtin_amdgcn_sched_barrier(0);
		issue(DYN ? tr[LAG + 1 + D] : tileOf(k + D), cur, curlen);
		__builtin_amdgcn_sched_barrier(0);
		if constexpr (DYN) {
			uint32_t nx = nt;
			if (dyn_on) {
				if (more) {
					const uint32_t g = rfl(graw);
					const uint32_t t = take ? blockIdx.x * NW + g % NW + g / NW * step : nt;
					if (t < nt) {
						nx = t;
						tmine++;
					} else {
						more = false;
						iters = k + D + 1 + LAG + (R2 ? 1u : 0u);
					}
				}
			} else {
				const uint32_t t = first + (k + D + 1) * step;
				nx = t < nt ? t : nt;
			}
#pragma unroll
			for (uint32_t i = 0; i + 1 < RN; i++)
				tr[i] = tr[i + 1];
			tr[RN - 1] = nx;
		}
	};

	// iteration k uses window buffer k % D and state set k % LAG: the loop
	// body is U = lcm(D, LAG) iterations
	constexpr uint32_t U = D == 3 ? 3 * LAG : 2;
	auto one = [&](uint32_t k, auto uc) __attribute__((always_inline)) {
		constexpr uint32_t u = decltype(uc)::value;
		RSt &rs = (LAG == 2 && (u & 1)) ? stB : stA;
		if constexpr (u % D == 0)
			iteration(k, preA, lenA, rs, u % 2 == 0);
		else if constexpr (u % D == 1)
			iteration(k, preB, lenB, rs, u % 2 == 0);
		else if constexpr (D == 3)
			iteration(k, preC, lenC, rs, u % 2 == 0);
	};
	if (tid == 0)
		QT_STAMP(1);
	if (cwv) {
		if constexpr (CW)   // (past the direct counters: the histogram)
			qt_count_wave(a, (lds_u32 *)(dcnt_base(a, s_dyn) + ((a.dcnt + 3) & ~3u)));
	} else if constexpr (D == 2) {
		uint32_t k = 0;
		for (; k + 1 < iters; k += 2) {
			iteration(k, preA, lenA, stA, true);
			iteration(k + 1, preB, lenB, LAG == 2 ? stB : stA, false);
		}
		if (k < iters)
			iteration(k, preA, lenA, stA, true);
	} else {
		// whole bodies unguarded (exact wait counts), then the rest guarded
		uint32_t k = 0;
		for (; k + U <= iters; k += U) {
			one(k, std::integral_constant<uint32_t, 0>{});
			one(k + 1, std::integral_constant<uint32_t, 1>{});
			one(k + 2, std::integral_constant<uint32_t, 2>{});
			if constexpr (U > 3) {
				one(k + 3, std::integral_constant<uint32_t, 3 % U>{});
				one(k + 4, std::integral_constant<uint32_t, 4 % U>{});
				one(k + 5, std::integral_constant<uint32_t, 5 % U>{});
			}
		}
		for (uint32_t u = 0; k < iters; k++, u++) {   // (u < U)
			if (u == 0)
				one(k, std::integral_constant<uint32_t, 0>{});
			else if (u == 1)
				one(k, std::integral_constant<uint32_t, 1>{});
			else if (u == 2)
				one(k, std::integral_constant<uint32_t, 2>{});
			else if constexpr (U > 3) {
				if (u == 3)
					one(k, std::integral_constant<uint32_t, 3 % U>{});
				else if (u == 4)
					one(k, std::integral_constant<uint32_t, 4 % U>{});
			}
		}
	}

	QT_STAMP(2 + wv);
	if constexpr (XFG_QT_VST)
		if (vs_act <= A_PASS)
			__builtin_nontemporal_store((uint8_t)vs_act, a.verdicts + vs_gi);
	if constexpr (G > 1)   // (the runs' verdict dwords before the drain rewrites bytes in them)
		__builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
	if (dg & 2048)
		ndef = 0;
	// the deferred packets: the whole reference walk over the canonical
	// table (classify_staged), 64 at a time -- or listed for
	// xfg_defer_kernel, which takes every wave's list after this kernel
	if (a.defer_sep && !cwv) {
		if (lane == 0)
			a.defer_n[blockIdx.x * NW + wv] = ndef;
		ndef = 0;
	}
	for (uint32_t d0 = 0; d0 < ndef; d0 += 64) {
		uint32_t tag, len;
		const uint32_t act = qt_drain_one<FEAT, W>(a, s_ports, const_cast<uint32_t *>(myrow), dlist, d0, ndef,
							   tag, len);
		count(tag, XFG_PORT_TAB);
		stat(act, len);
	}

	QT_STAMP(11 + wv);
	st_fold();
#pragma unroll
	for (int kk = 0; kk < 3; kk++) {
		unsigned long long x = st_b[kk];
		uint32_t c = st_c[kk];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1) {
			x += __shfl_xor(x, o);
			c += __shfl_xor(c, o);
		}
		if (lane == 0 && c) {
			atomicAdd(&s_stats[2 * kk], (unsigned long long)c);
			atomicAdd(&s_stats[2 * kk + 1], x);
		}
	}
	if (lane == 0 && !cwv)
		s_tn[wv] = tn;
	if (!cwv)
		QT_STAMP(22 + wv);
	__syncthreads();
	if (tid == 0)
		QT_STAMP(30);
	// (every wave's appends are done: done == head) the rest of this
	// wave's partitions, and the slices' fills for the count kernel; a
	// position past a slice goes to the counter cache, flushed below
	if (a.pbuf && !(dg & 16) && !cwv) {
		const uint32_t hd = (uint32_t)lane < pcnt ? s_hd[2 * wc_p] : 0u;
		// (every position within its slice -- the usual case: two rings
		// per instruction, 8 bytes a lane, one LDS read and one store each
		// for the lanes whose entries are consecutive tickets; a ring holds
		// tickets [fl, h) at slots t & (WR - 1), so slot s carries ticket
		// fl + ((s - fl) & (WR - 1)), 8-byte aligned in the slice)
		constexpr uint32_t EPL = 8 / sizeof(ring_t);
		if (WR * sizeof(ring_t) == 256 && __ballot(((uint32_t)lane < pcnt) & (hd > a.pcap)) == 0) {
			const uint32_t half = (uint32_t)lane >> 5, s0 = ((uint32_t)lane & 31) * EPL;
#pragma unroll 4
			for (uint32_t j = 0; j < pcnt; j += 2) {
				const uint32_t fl = half ? __builtin_amdgcn_readlane(wc_fl, j + 1) : __builtin_amdgcn_readlane(wc_fl, j);
				const uint32_t h = half ? __builtin_amdgcn_readlane(hd, j + 1) : __builtin_amdgcn_readlane(hd, j);
				const uint32_t p = ownp(j + half);
				const uint64_t v = *reinterpret_cast<const uint64_t *>(&s_ring[p * WR + s0]);
				const uint32_t t0 = fl + ((s0 - fl) & (WR - 1));
				ring_t *sl = reinterpret_cast<ring_t *>(a.pbuf) + p * wc_pstep + wc_slice0;
				if (t0 + EPL - 1 == fl + ((s0 + EPL - 1 - fl) & (WR - 1)) && t0 + EPL <= h) {
					*reinterpret_cast<__attribute__((address_space(1))) uint64_t *>((uintptr_t)(sl + t0)) = v;
				} else {
#pragma unroll
					for (uint32_t i = 0; i < EPL; i++) {
						const uint32_t t = fl + ((s0 + i - fl) & (WR - 1));
						if (t < h)
							*reinterpret_cast<__attribute__((address_space(1))) ring_t *>((uintptr_t)(sl + t)) =
								(ring_t)(v >> (i * 8 * sizeof(ring_t)));
					}
				}
			}
		} else {
			for (uint32_t j = 0; j < pcnt; j++) {
				const uint32_t fl = __builtin_amdgcn_readlane(wc_fl, j);
				const uint32_t h = __builtin_amdgcn_readlane(hd, j);
				wc_move(j, fl, h - fl);
			}
		}
		if ((uint32_t)lane < pcnt)
			gst32(a.pfill + (uint64_t)wc_p * a.pslices + a.pslice0 + blockIdx.x, hd);
	}
	__syncthreads();
	if (tid == 0)
		QT_STAMP(20);
	if (cwv)
		return;
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	cn.flush(a, tid, NT);
	if constexpr (PORTS)
		if (ptab)
			for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
				if (s_pcnt[i])
					atomicAdd(a.port_hits + (s_tab[i] & 0xffff), (unsigned long long)s_pcnt[i]);
	if constexpr (EKF)
		if (ekon)
			for (uint32_t i = tid; i < ek_es; i += NT)
				if (const uint32_t c = s_pcnt[XFG_PORT_TAB + XL + i])
					atomicAdd(global_counter(a, ek_gb + s_ek[i].z), (unsigned long long)c);
	if (tid == 0)
		QT_STAMP(21);
	if (dg & 16)
		return;
}

}  // namespace
