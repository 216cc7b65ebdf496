// SPDX-License-Identifier: GPL-2.0
//
// xfg_pipeline.hip — the production classify kernel for fixed-stride batches
// (stride >= header window, 16-byte aligned: device-resident batches and the
// staging layout of xfg_classify_host).  Included by xfg_kernels.hip.
//
// The reference program (xdp-filter/xdpfilt_prog.h:214-310) is a chain of
// dependent memory hops per packet: header bytes -> map lookups (a Bloom word
// in L2, then a bucket line) -> counter.  A wave's vector-memory counter
// completes in issue order, so a wave that waits for a lookup also waits for
// every load it issued before it.  Here a wave waits once per iteration, at
// its top, for loads it issued during the previous iteration: every wave
// works alone on tiles of 64 packets (one per lane, its own LDS rows, no
// workgroup barrier in the loop) and keeps three tiles one hop apart.
// Iteration k of a wave:
//
//   R(k-2)  match tile k-2's bucket lines -> verdict + counter identity
//   W(k-2)  its verdicts stored, counters bumped, stats kept (the stores go
//           out early: their completion overlaps the rest of the iteration)
//   Q(k-1)  tile k-1's Bloom words -> the first key the filter passes, in
//           reference order
//   S       tile k's windows (loaded into registers in iteration k-1) into
//           the wave's LDS rows; tile k+1's windows and lengths issued
//   P(k)    parse tile k from LDS (the common shapes at static offsets),
//           plan its ordered lookups (its live hash keys, then the abort
//           point and the port stage, which LDS answers) and issue the Bloom
//           words of the live keys
//   L       tile k-1's candidate bucket lines issued
//
// Nothing loaded in an iteration is used before the next one: the one wait
// (an explicit vmcnt(0) at the top) is for loads in flight a whole
// iteration.
//
// Whatever would need a further dependent hop, or a byte walk, inside an
// iteration -- a shape the static-offset parse does not cover (VLAN tags,
// ARP, IPv6 extension headers, ICMPv6, IPv4 options), more than PK live keys,
// a probe chain past a full bucket, a second Bloom-positive key after a miss
// -- defers the packet to the wave's list (global memory); the list is
// classified after the loop by the general path (classify_one: the whole
// reference walk over HBM).  Results are identical whichever way a packet
// goes.
//
// KM (key mode, chosen by the host from the flag census): 1 = only IPv4 keys
// are live (the Ethernet and IPv6 maps cannot hit: C2-C4 and any ip-only
// rule set), two keys per packet at most; 0 = any map.
namespace {

constexpr uint32_t K_ETH = 1, K_V4 = 2, K_V6 = 3;
constexpr uint32_t A_DEFER = 6;

#define PIPE_WAVES(W) ((W) <= 64 ? 8 : 4)
#define PIPE_THREADS(W) (64 * PIPE_WAVES(W))
// the quotient-index kernel (xfg_pipeq.hip): waves per workgroup (two
// workgroups per CU).  10 (5 waves per SIMD, 96 VGPRs) sped the stream and
// parse up 4 % but the whole classify down 4 %: more requests in flight
// than the CU's vector memory path serves (profiles/archive/r03_qt_waves_ab.log)
#ifndef XFG_QT_NW
#define XFG_QT_NW 8
#endif
#ifndef XFG_QT_NW128   /* waves per workgroup, 128-byte windows */
#define XFG_QT_NW128 4
#endif
#define QT_WAVES(W) ((W) <= 64 ? XFG_QT_NW : XFG_QT_NW128)
#define QT_THREADS(W) (64 * QT_WAVES(W))
#ifndef XFG_QT_WGCU   /* workgroups per CU the register bound assumes */
#define XFG_QT_WGCU 1
#endif
#define QT_MINW(W) ((W) <= 64 ? (XFG_QT_WGCU * XFG_QT_NW + 3) / 4 : 2)   // (128: 8 waves a CU)

// Key descriptor: kind | mask << 2 | zero << 4 | byte offset << 5.
__device__ __forceinline__ uint32_t kd_kind(uint32_t d) { return d & 3; }
__device__ __forceinline__ uint32_t kd_mask(uint32_t d) { return (d >> 2) & 3; }
__device__ __forceinline__ bool kd_zero(uint32_t d) { return (d >> 4) & 1; }
__device__ __forceinline__ uint32_t kd_off(uint32_t d) { return d >> 5; }

// Packet view over the wave's LDS row (key bytes of the generic plan).
template <int W>
struct PktL {
	const uint32_t *row;
	uint32_t len;
	mutable bool beyond;

	__device__ __forceinline__ uint32_t u32(uint32_t o) const
	{
		if (o + 4 <= (uint32_t)W)
			return __builtin_amdgcn_alignbyte(row[(o >> 2) + 1], row[o >> 2], o & 3);
		beyond = true;
		return 0;
	}
	__device__ __forceinline__ uint32_t raw16(uint32_t o) const
	{
		if (o + 2 <= (uint32_t)W)
			return __builtin_amdgcn_alignbyte(row[(o >> 2) + 1], row[o >> 2], o & 3) & 0xffffu;
		beyond = true;
		return 0;
	}
};

// Loads through the global address space: a generic (flat) load would also
// count against the LDS counter and complete out of order, so every wait
// near it would degrade to vmcnt(0).
typedef const __attribute__((address_space(1))) uint32_t gu32;
typedef const __attribute__((address_space(1))) u32x4 gu32x4;

__device__ __forceinline__ uint32_t gload32(uint64_t addr)
{
	return *reinterpret_cast<gu32 *>(addr);
}

__device__ __forceinline__ uint32_t gload16(uint64_t addr)
{
	return *reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(addr);
}

__device__ __forceinline__ u32x4 gload128(uint64_t addr)
{
	return *reinterpret_cast<gu32x4 *>(addr);
}

// Per-kind table fields, read once into scalar registers.  A per-lane
// select between fields of the kernel-argument struct would otherwise be
// folded into one load through a select of field addresses, which moves the
// whole argument struct to scratch memory.
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ uint64_t rfl64(uint64_t x)
{
	return ((uint64_t)rfl((uint32_t)(x >> 32)) << 32) | rfl((uint32_t)x);
}

// The key table in LDS: 16-byte aligned, past the direct counters and the
// staged Bloom words (the generic pipelined kernel's; none here).
__device__ __forceinline__ u32x4 *ek_base(const xfg_kargs &a, uint32_t *s_dyn)
{
	return reinterpret_cast<u32x4 *>(dcnt_base(a, s_dyn) + ((a.dcnt + a.bl_lds + 3) & ~3u));
}

// CHECK_MAP (xdpfilt_prog.h:56-64) of one MAC against the LDS key table
// (es entries, keys at most edisp past their home): found with every bit of
// mask set; its canonical slot (ENTRY: the table entry it sits in).  Every
// lane reads edisp + 1 entries (keys are unique: at most one matches).
template <bool ENTRY = false>
__device__ __forceinline__ bool ek_probe(const u32x4 *s_ek, uint32_t es, uint32_t edisp, uint32_t seed,
					 uint32_t lo, uint32_t hi, uint32_t mask, uint32_t &slot)
{
	uint32_t e = xfg_ek_home(lo, hi, seed, __builtin_ctz(es));
	bool hit = false;
	for (uint32_t d = 0; d <= edisp; d++) {
		const u32x4 v = s_ek[e];
		const bool m = (v.x == lo) & (v.y == hi) & ((v.w & XFG_EK_VALID) != 0);
		hit |= m & ((v.w & mask) == mask);
		slot = m ? (ENTRY ? e : v.z) : slot;
		e = (e + 1) & (es - 1);
	}
	return hit;
}

template <int KM>
struct KTabs {
	static constexpr int NK = KM == 1 ? 1 : 3;   // tables held (KM 1: IPv4 only)
	uint32_t nb[NK], md[NK], ns[NK], zp[NK], bw[NK], gb[NK], blo[NK];
	uint64_t bk[NK], bl[NK];
	__device__ __forceinline__ void load(const xfg_kargs &a)
	{
		const xfg_tdesc *t[3] = { &a.t4, &a.te, &a.t6 };
		const uint32_t g[3] = { a.gbase[0], a.gbase[2], a.gbase[1] };
#pragma unroll
		for (int i = 0; i < NK; i++) {
			nb[i] = rfl(t[i]->nbuckets);
			md[i] = rfl(t[i]->max_disp);
			ns[i] = rfl(t[i]->nslots);
			zp[i] = rfl(t[i]->zero_present);
			bw[i] = rfl(t[i]->bloom_words);
			gb[i] = rfl(g[i]);
			blo[i] = rfl(a.bl_off[i]);
			bk[i] = rfl64((uint64_t)(uintptr_t)t[i]->buckets);
			bl[i] = rfl64((uint64_t)(uintptr_t)t[i]->bloom);
		}
	}
};
// field f of the table of `kind` (always the IPv4 table in key mode 1)
#define TSEL(T, kind, f)                                                                   \
	(KM == 1 ? (T).f[0]                                                                \
		 : (kind) == K_V4 ? (T).f[0] : (kind) == K_ETH ? (T).f[1 % KTabs<KM>::NK]  \
							: (T).f[2 % KTabs<KM>::NK])

__device__ __forceinline__ uint32_t slots_by_kind(uint32_t kind)
{
	return kind == K_V4 ? XFG_SLOTS_V4 : kind == K_V6 ? XFG_SLOTS_V6 : XFG_SLOTS_ETH;
}

// Key words of a key of `kind` at byte `off` of the row (v4: w0; eth: w0 =
// bytes 0-3, w1 = bytes 4-5; v6: w0..w3).
template <class P>
__device__ __forceinline__ void key_words(const P &p, uint32_t kind, uint32_t off, uint32_t &w0,
					  uint32_t &w1, uint32_t &w2, uint32_t &w3)
{
	w0 = p.u32(off);
	w1 = w2 = w3 = 0;
	if (kind == K_ETH) {
		w1 = p.raw16(off + 4);
	} else if (kind == K_V6) {
		w1 = p.u32(off + 4);
		w2 = p.u32(off + 8);
		w3 = p.u32(off + 12);
	}
}

// The static-offset parse of the common, untagged shapes, exactly as
// parse() walks them (headers/xdp/parsing_helpers.h: parse_ethhdr,
// parse_iphdr, parse_ip6hdr with its extension walk, parse_udphdr,
// parse_tcphdr): runts, IPv4 with ihl 5 (any length, any protocol; the
// version nibble is not checked, as in the reference), IPv6 whose next
// header is final and not ICMPv6, and other non-VLAN ethertypes.  Returns
// false for every other packet (the general path takes it).
template <uint32_t FEAT, int W>
__device__ __forceinline__ bool parse_static(const uint32_t *row, uint32_t len, Parsed &r)
{
	r.abort_at = NST;
	r.l3 = 0;
	r.nd = 0;
	r.l4proto = 0;
	r.arp_op = 0;
	r.k4a = r.k4b = 0;
	r.ka_off = r.kb_off = 0;
	r.o6 = r.ond = 0;
	r.pdst = r.psrc = 0;
	if (len < 14) {
		r.abort_at = ST_ETH;
		return true;
	}
	const uint32_t d3 = row[3];
	const uint32_t et = d3 & 0xffff;   // raw (network-order) ethertype
	if (et == 0x0081 || et == 0xa888)
		return false;                  // VLAN: the tag walk
	if constexpr ((FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
		return true;                   // eth-only program: nothing after the eth stage
	} else {
		if (et == 0x0008) {
			if (len < 34) {
				r.abort_at = ST_IP;    // off + 20 > len
				return true;
			}
			if (((d3 >> 16) & 0xf) != 5)
				return false;          // ihl != 5: the L4 offset moves
			const uint32_t d5 = row[5], d6 = row[6], d7 = row[7];
			const uint32_t proto = d5 >> 24;   // byte 23
			r.l3 = 1;
			r.k4a = __builtin_amdgcn_alignbyte(row[8], d7, 2);   // daddr 30..33
			r.k4b = __builtin_amdgcn_alignbyte(d7, d6, 2);       // saddr 26..29
			r.ka_off = 30;
			r.kb_off = 26;
			if ((FEAT & F_UDP) && proto == 17) {
				if (len < 42) {
					r.abort_at = ST_L4;
					return true;
				}
				const uint32_t d8 = row[8], d9 = row[9];
				const uint32_t ulen = ((d9 >> 8) & 0xff00) | (d9 >> 24);   // be16 38,39
				r.psrc = d8 >> 16;     // bytes 34,35
				r.pdst = d9 & 0xffff;  // bytes 36,37
				if (ulen < 8)
					r.abort_at = ST_L4;
				else
					r.l4proto = 17;
			} else if ((FEAT & F_TCP) && proto == 6) {
				if (len < 54) {
					r.abort_at = ST_L4;
					return true;
				}
				const uint32_t doff = (row[11] >> 20) & 0xf;   // byte 46 >> 4
				r.psrc = row[8] >> 16;
				r.pdst = row[9] & 0xffff;
				if (34 + doff * 4 > len)
					r.abort_at = ST_L4;
				else
					r.l4proto = 6;
			}
			return true;
		}
		if (et == 0xdd86) {
			if (len < 54) {
				r.abort_at = ST_IP;    // off + 40 > len
				return true;
			}
			const uint32_t nh = row[5] & 0xff;   // byte 20
			if (nh == 0 || nh == 60 || nh == 43 || nh == 135 || nh == 51 || nh == 44 ||
			    nh == 58)
				return false;          // extension walk / ICMPv6 (NDISC)
			if (len < 56) {
				r.abort_at = ST_IP;    // the walk's 2-byte read at 54
				return true;
			}
			r.l3 = 3;
			r.o6 = 14;
			if ((FEAT & F_UDP) && nh == 17) {
				if (len < 62) {
					r.abort_at = ST_L4;
					return true;
				}
				const uint32_t d13 = row[13], d14 = row[14];
				const uint32_t ulen = ((d14 >> 8) & 0xff00) | (d14 >> 24);   // 58,59
				r.psrc = d13 >> 16;    // 54,55
				r.pdst = d14 & 0xffff; // 56,57
				if (ulen < 8)
					r.abort_at = ST_L4;
				else
					r.l4proto = 17;
			} else if ((FEAT & F_TCP) && nh == 6) {
				if (len < 74) {
					r.abort_at = ST_L4;
					return true;
				}
				if constexpr (W < 68) {
					return false;      // doff (byte 66) past the window
				} else {
					const uint32_t doff = (row[16] >> 20) & 0xf;   // byte 66 >> 4
					r.psrc = row[13] >> 16;
					r.pdst = row[14] & 0xffff;
					if (54 + doff * 4 > len)
						r.abort_at = ST_L4;
					else
						r.l4proto = 6;
				}
			}
			return true;
		}
		if ((FEAT & F_IPV4) && et == 0x0608)
			return false;              // ARP: parse_arphdr + its keys
		return true;                   // any other ethertype: MISS after eth
	}
}

// The lookup plan of one parsed packet: its live hash keys in reference
// order (xdpfilt_prog.h:224-307; a lookup whose mask no key of the map
// carries, or of an empty map, cannot hit and is left out) and the result
// when every one of them misses: ABORTED at a failed header check, else the
// port stage (lookup_verdict_tcp/udp, :76-101, answered from LDS) or MISS.
// Key mode 1 keeps only the IPv4 stage.
// (ek.on: the Ethernet map as the LDS key table of a small map,
// xfg_kargs.ek -- both Ethernet lookups answered here, exactly, and a hit
// ends the program, :224-227; no Bloom word, no bucket line)
struct EkL {
	const u32x4 *tab;
	uint32_t es, disp, seed, gb;
	bool on;
};

template <uint32_t FEAT, int W, int KM, int PK>
__device__ __forceinline__ void plan_packet(const xfg_kargs &a, const PktL<W> &p, const Parsed &r,
					    const uint32_t *s_ports, const EkL &ek, uint32_t (&kd)[PK],
					    uint32_t (&kh)[PK], uint32_t (&kv)[PK], uint32_t &nk,
					    uint32_t &fb_act, uint32_t &fb_tag, bool &over)
{
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	nk = 0;
	fb_tag = CT_NONE;
	over = false;
	auto add = [&](uint32_t kind, uint32_t mask, uint32_t off, uint32_t v4key) {
		uint32_t w0, w1 = 0, w2 = 0, w3 = 0, h;
		if (KM == 1 || kind == K_V4)
			w0 = v4key;
		else
			key_words(p, kind, off, w0, w1, w2, w3);
		const bool zero = (w0 | w1 | w2 | w3) == 0;
		if (KM == 1 || kind == K_V4)
			h = xfg_hash_v4(w0, a.t4.seed);
		else if (kind == K_V6)
			h = xfg_hash_v6(w0, w1, w2, w3, a.t6.seed);
		else
			h = xfg_hash_eth(w0 | ((uint64_t)w1 << 32), a.te.seed);
		const uint32_t d = kind | (mask << 2) | (zero ? 16u : 0u) | (off << 5);
#pragma unroll
		for (int i = 0; i < PK; i++) {
			kd[i] = nk == (uint32_t)i ? d : kd[i];
			kh[i] = nk == (uint32_t)i ? h : kh[i];
			kv[i] = nk == (uint32_t)i ? w0 : kv[i];
		}
		over |= nk >= (uint32_t)PK;
		nk++;
	};
	if (r.abort_at == ST_ETH) {
		fb_act = A_ABORTED;
		return;
	}
	if constexpr ((FEAT & F_ETH) != 0 && KM == 0) {
		// lookup_verdict_ethernet: dst then src (xdpfilt_prog.h:187-196)
		if (a.te.count && ek.on) {
			uint32_t w0, w1, w2, w3, sl = 0;
			bool h = false;
			if (can_hit(a.te.fmask, M_DST)) {
				key_words(p, K_ETH, 0, w0, w1, w2, w3);
				h = ek_probe(ek.tab, ek.es, ek.disp, ek.seed, w0, w1, M_DST, sl);
			}
			if (!h && can_hit(a.te.fmask, M_SRC)) {
				key_words(p, K_ETH, 6, w0, w1, w2, w3);
				h = ek_probe(ek.tab, ek.es, ek.disp, ek.seed, w0, w1, M_SRC, sl);
			}
			if (h) {
				fb_act = (FEAT & F_DENY) ? A_PASS : A_DROP;
				fb_tag = ek.gb + sl;
				return;
			}
		} else if (a.te.count) {
			if (can_hit(a.te.fmask, M_DST))
				add(K_ETH, M_DST, 0, 0);
			if (can_hit(a.te.fmask, M_SRC))
				add(K_ETH, M_SRC, 6, 0);
		}
	}
	if (r.abort_at == ST_IP) {
		fb_act = A_ABORTED;
		return;
	}
	if constexpr ((FEAT & F_IPV4) != 0) {
		if (a.t4.count && r.l3 == 1) {
			// lookup_verdict_ipv4: dst then src (:121-134)
			if (can_hit(a.t4.fmask, M_DST))
				add(K_V4, M_DST, r.ka_off, r.k4a);
			if (can_hit(a.t4.fmask, M_SRC))
				add(K_V4, M_SRC, r.kb_off, r.k4b);
		}
	}
	if constexpr ((FEAT & F_IPV6) != 0 && KM == 0) {
		if (a.t6.count && r.l3 == 3) {
			// lookup_verdict_ipv6: dst then src (:152-165)
			if (can_hit(a.t6.fmask, M_DST))
				add(K_V6, M_DST, r.o6 + 24, 0);
			if (can_hit(a.t6.fmask, M_SRC))
				add(K_V6, M_SRC, r.o6 + 8, 0);
		}
	}
	if (r.abort_at != NST) {   // ST_L4 (ST_ND shapes take the general path)
		fb_act = A_ABORTED;
		return;
	}
	fb_act = MISS;
	if constexpr ((FEAT & (F_UDP | F_TCP)) != 0) {
		if (a.port_count && r.l4proto) {
			const uint32_t pm = r.l4proto == 17 ? M_UDP : M_TCP;
			uint32_t t = CT_NONE;
			if (check_port(a, s_ports, r.pdst, M_DST | pm, t) ||
			    check_port(a, s_ports, r.psrc, M_SRC | pm, t)) {
				fb_act = HIT;
				fb_tag = t;
			}
		}
	}
}

template <uint32_t FEAT, int W, bool DENSE, int KM>
__global__ __launch_bounds__(PIPE_THREADS(W), (W) <= 64 ? 4 : 2) void xfg_pipeline_kernel(const xfg_kargs a)
{
	constexpr int NW = PIPE_WAVES(W);
	constexpr int NT = 64 * NW;
	constexpr int PK = KM == 1 ? 2 : 4;     // live hash keys carried per packet
	constexpr int CPP = W / 16;             // 16-byte chunks per window
	constexpr int ROWDW = W / 4 + 1;        // odd dword stride per LDS row
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	// the wave rows; after the loop, the hit-log partition scratch
	__shared__ uint32_t win[NW * 64 * ROWDW > LOG_SCRATCH ? NW * 64 * ROWDW : LOG_SCRATCH];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES], s_tn[NW];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar control flow
	KTabs<KM> T;
	T.load(a);
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, NT);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, NT);
	// (bl_lds: the live maps' Bloom filters copied into LDS, past the direct
	// counters -- the probes of small rule sets then read no memory: C1's
	// filter, 15 KB of random words, cost a random line per probe)
	uint32_t *const s_bl = dcnt_base(a, s_dyn) + a.dcnt;
	const bool bll = a.bl_lds != 0;
	if (bll) {
#pragma unroll
		for (int i = 0; i < KTabs<KM>::NK; i++) {
			if (T.blo[i] == ~0u)
				continue;
			const uint32_t *src = reinterpret_cast<const uint32_t *>(T.bl[i]);
			for (uint32_t w = tid; w < T.bw[i]; w += NT)
				s_bl[T.blo[i] + w] = src[w];
		}
	}
	// (ek: a small Ethernet map as its LDS key table, past the Bloom words;
	// its hits count in the LDS counter cache, as the Ethernet-key kernel's)
	EkL ek{ ek_base(a, s_dyn), 0, 0, 0, 0, false };
	if constexpr ((FEAT & F_ETH) != 0 && KM == 0) {
		if (a.ek) {
			ek.es = rfl(a.ek_slots);
			ek.disp = rfl(a.ek_disp);
			ek.seed = rfl(a.te.seed);
			ek.gb = rfl(a.gbase[2]);
			ek.on = true;
			u32x4 *const s_ek = const_cast<u32x4 *>(ek.tab);
			for (uint32_t i = tid; i < ek.es; i += NT)
				s_ek[i] = reinterpret_cast<const u32x4 *>(a.ek)[i];
		}
	}
	__syncthreads();

	uint32_t *const rows = win + wv * 64 * ROWDW;
	const uint32_t *const myrow = rows + lane * ROWDW;
	// this wave's deferred list (global: room for every packet of its tiles)
	uint32_t *const dlist = a.defer + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap;
	// this wave's hit-log region (same bound) and its fill
	uint32_t *const tregion = a.tlog + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap;
	uint32_t tn = 0;
	// a hit goes to the hit log when there is one and its counter is a
	// hash-map slot without a direct LDS counter; else to the Counters
	const uint32_t lg_lo = a.dcnt, lg_hi = a.tlog ? a.gbase[3] : 0u;
	const uint32_t lg_eth = ek.on ? rfl(a.gbase[2]) : 0xffffffffu;   // (ek: Ethernet counters not logged)
	auto count = [&](uint32_t tag) {
		const bool lg = tag >= lg_lo && tag < lg_hi && tag < lg_eth;
		log_append(tregion, tn, lg ? tag : CT_NONE, lane);
		cn.bump(a, lg ? CT_NONE : tag, lane);
	};
	// (the host guarantees n < 2^32: 32-bit packet and tile indices)
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv;
	const uint32_t step = gridDim.x * NW;
	// per-lane stats (u32: the host bounds a lane's byte sum below 2^32)
	uint32_t st_c0 = 0, st_c1 = 0, st_c2 = 0, st_b0 = 0, st_b1 = 0, st_b2 = 0;
	auto stat = [&](uint32_t act, uint32_t len) {
		st_c0 += act == A_ABORTED;
		st_c1 += act == A_DROP;
		st_c2 += act == A_PASS;
		st_b0 += act == A_ABORTED ? len : 0u;
		st_b1 += act == A_DROP ? len : 0u;
		st_b2 += act == A_PASS ? len : 0u;
	};
	uint32_t ndef = 0;

	// S: windows + lengths of a tile into registers (lengths clamped to the
	// stride: the slot is the frame's buffer)
	u32x4 pre[CPP];
	uint32_t plen = 0;
	auto issue = [&](uint32_t t) {
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64 ? 64u : n - base;
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
				const uint32_t c = it * 64 + lane, pk = c / CPP, sub = c % CPP;
				pre[it] = u32x4{ 0, 0, 0, 0 };
				if (pk < rem)
					pre[it] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
						a.data + (uint64_t)(base + pk) * a.stride + sub * 16));
			}
		}
		plen = (uint32_t)lane < rem ? min(load_len_fixed(a, base + lane), a.stride) : 0;
	};

	// P -> Q: tile k-1's plan and Bloom words
	uint32_t q_kd[PK], q_kh[PK], q_kv[PK], q_w[PK];
#pragma unroll
	for (int i = 0; i < PK; i++)
		q_kd[i] = q_kh[i] = q_kv[i] = q_w[i] = 0;
	uint32_t q_nk = 0, q_act = A_NONE, q_tag = CT_NONE, q_len = 0;
	// Q -> R: tile k-2's candidate key and its bucket line
	Line r_line;
	r_line.q0 = r_line.q1 = r_line.q2 = r_line.q3 = u32x4{ 0, 0, 0, 0 };
	uint32_t r_kd = 0, r_b = 0, r_w0 = 0, r_w1 = 0, r_w2 = 0, r_w3 = 0;
	uint32_t r_act = A_NONE, r_tag = CT_NONE, r_len = 0;
	bool r_sel = false, r_more = false;

	if (first < nt)
		issue(first);
	for (uint32_t k = 0;; k++) {
		const uint32_t tP = first + k * step;
		const bool vP = tP < nt;
		const bool vQ = k >= 1 && tP - step < nt;
		const bool vR = k >= 2 && tP - 2 * step < nt;
		if (!vP && !vQ && !vR)
			break;
		// the iteration's one wait: everything issued in the previous one
		// (an explicit vmcnt(0) the compiler's wait placement sees, so
		// nothing after it waits again for those loads)
		__builtin_amdgcn_s_waitcnt(0x0F70);

		// ---- R: tile k-2's bucket lines -> verdict, counter identity
		uint32_t w_act = A_NONE, w_tag = CT_NONE;
		const uint32_t w_len = r_len;
		if (vR) {
			w_act = r_act;
			w_tag = r_tag;
			if (r_sel) {
				const uint32_t kind = KM == 1 ? K_V4 : kd_kind(r_kd), mask = kd_mask(r_kd);
				int i = -1;
				uint32_t slot = 0;
				if (kd_zero(r_kd)) {
					// the all-zero key: bucket nbuckets, slot nslots
					i = 0;
					slot = TSEL(T, kind, ns);
				} else {
					if constexpr ((FEAT & F_IPV4) != 0)
						if (kind == K_V4)
							i = match_v4(r_line, r_w0);
					if constexpr ((FEAT & F_IPV6) != 0 && KM == 0)
						if (kind == K_V6)
							i = match_v6(r_line, r_w0, r_w1, r_w2, r_w3);
					if constexpr ((FEAT & F_ETH) != 0 && KM == 0)
						if (kind == K_ETH)
							i = match_eth(r_line, r_w0, r_w1);
					slot = r_b * (KM == 1 ? XFG_SLOTS_V4 : slots_by_kind(kind)) + (uint32_t)i;
				}
				if (i >= 0 && (r_line.flag(i) & mask) == mask) {
					w_act = HIT;
					w_tag = TSEL(T, kind, gb) + slot;
				} else if (r_more || (i < 0 && r_line.overflow() && TSEL(T, kind, md))) {
					w_act = A_DEFER;   // a further probe: the general path
					w_tag = CT_NONE;
				}
			}
		}

		// ---- W: tile k-2's verdicts, counters, stats, deferrals
		if (vR) {
			const uint32_t gi = (tP - 2 * step) * 64 + lane;
			if (w_act <= A_PASS)
				__builtin_nontemporal_store((uint8_t)w_act, a.verdicts + gi);
			count(w_tag);
			stat(w_act, w_len);
			const unsigned long long dm = __ballot(w_act == A_DEFER);
			if (dm) {
				const uint32_t pos = ndef + lanes_below(dm);
				if (w_act == A_DEFER)
					gst32(dlist + pos, gi);
				ndef += (uint32_t)__popcll(dm);
			}
		}

		// ---- Q: tile k-1's Bloom words -> the first candidate key; its
		// key bytes (from the LDS rows, before tile k overwrites them)
		if (vQ) {
			r_act = q_act;
			r_tag = q_tag;
			r_len = q_len;
			r_sel = false;
			r_more = false;
			uint32_t sd = 0, sv = 0;
#pragma unroll
			for (int i = 0; i < PK; i++) {
				if ((uint32_t)i < q_nk) {
					const uint32_t kind = KM == 1 ? K_V4 : kd_kind(q_kd[i]);
					bool m;
					if (kd_zero(q_kd[i])) {
						m = TSEL(T, kind, zp) != 0;
					} else {
						const uint32_t bm = xfg_bloom_mask(q_kh[i]);
						m = (q_w[i] & bm) == bm;
					}
					if (m) {
						r_more |= r_sel;
						if (!r_sel) {
							sd = q_kd[i];
							sv = q_kv[i];
							r_b = kd_zero(sd) ? TSEL(T, kind, nb)
									  : xfg_home(q_kh[i], TSEL(T, kind, nb));
						}
						r_sel = true;
					}
				}
			}
			r_kd = sd;
			r_w0 = sv;
			if constexpr (KM == 0) {
				if (r_sel && kd_kind(sd) != K_V4) {
					PktL<W> p{ myrow, 0, false };
					key_words(p, kd_kind(sd), kd_off(sd), r_w0, r_w1, r_w2, r_w3);
				}
			}
		}

		// ---- S: tile k's windows into the wave's LDS rows
		uint32_t len = 0;
		if (vP) {
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const int pk = c / CPP, sub = c % CPP;
				uint32_t *dst = &rows[pk * ROWDW + sub * 4];
				dst[0] = pre[it].x;
				dst[1] = pre[it].y;
				dst[2] = pre[it].z;
				dst[3] = pre[it].w;
			}
			len = plen;
			__builtin_amdgcn_wave_barrier();
		}
		// tile k+1's windows: in flight until the next iteration's staging
		if (tP + step < nt)
			issue(tP + step);

		// ---- P: parse tile k, plan its lookups, issue the Bloom words
		if (vP) {
			const uint32_t gi = tP * 64 + lane;
			q_nk = 0;
			q_act = A_NONE;
			q_tag = CT_NONE;
			q_len = len;
			if (gi < n) {
				Parsed r;
				bool over = false;
				PktL<W> p{ myrow, len, false };
				if (parse_static<FEAT, W>(myrow, len, r))
					plan_packet<FEAT, W, KM, PK>(a, p, r, s_ports, ek, q_kd, q_kh, q_kv, q_nk,
								     q_act, q_tag, over);
				else
					over = true;
				if (p.beyond || over) {
					q_act = A_DEFER;
					q_tag = CT_NONE;
					q_nk = 0;
				}
			}
#pragma unroll
			for (int i = 0; i < PK; i++) {
				q_w[i] = ~0u;
				if ((uint32_t)i < q_nk && !kd_zero(q_kd[i])) {
					const uint32_t kind = KM == 1 ? K_V4 : kd_kind(q_kd[i]);
					const uint32_t bwi = xfg_bloom_word(q_kh[i], TSEL(T, kind, bw));
					q_w[i] = bll ? s_bl[TSEL(T, kind, blo) + bwi]
						     : gload32(TSEL(T, kind, bl) + 4ull * bwi);
				}
			}
		}

		// ---- L: tile k-1's candidate bucket lines
		if (vQ && r_sel) {
			const uint64_t lp = TSEL(T, (KM == 1 ? K_V4 : kd_kind(r_kd)), bk) +
					    (uint64_t)r_b * XFG_BUCKET_BYTES;
			r_line.q0 = gload128(lp);
			r_line.q1 = gload128(lp + 16);
			r_line.q2 = gload128(lp + 32);
			r_line.q3 = gload128(lp + 48);
		}
	}

	// the deferred packets, by the general path (the whole reference walk
	// over the frame in HBM), 64 at a time
	for (uint32_t d0 = 0; d0 < ndef; d0 += 64) {
		uint32_t act = A_NONE, tag = CT_NONE, len = 0;
		if (d0 + lane < ndef) {
			const uint32_t gi = gld32(dlist + d0 + lane);
			len = min(load_len(a, gi), a.stride);
			act = classify_one<FEAT>(a, s_ports, gi, len, tag);
			__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
		}
		count(tag);
		stat(act, len);
	}

	const unsigned long long v[6] = { st_c0, st_b0, st_c1, st_b1, st_c2, st_b2 };
#pragma unroll
	for (int k = 0; k < 6; k++) {
		unsigned long long x = v[k];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			x += __shfl_xor(x, o);
		if (lane == 0 && x)
			atomicAdd(&s_stats[k], x);
	}
	if (lane == 0)
		s_tn[wv] = tn;
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	cn.flush(a, tid, NT);
	if (a.tlog)   // (win is free now: the partition scratch)
		log_partition<NW>(a, s_tn, nullptr, win, tid);
}

}  // namespace

// ---------------------------------------------------------------- IPv4-key mode
// Key mode 1 (only IPv4 keys live: no Ethernet or IPv6 lookup can hit by the
// flag census) as its own kernel, written branch-free wherever a select will
// do: the parse of the common shapes reads nine fixed dwords of the row and
// derives every bounds check from them at once, a packet carries at most two
// keys (dst then src, :121-134), and the match and verdict are selects.  Same
// pipeline, same deferral rules, same results as xfg_pipeline_kernel.
namespace {

struct Parse4 {
	uint32_t abort_at, l4proto, psrc, pdst, k4a, k4b;
	bool v4ok, defer, is6, v6ok;
};

// Branch-free helpers: every operand evaluated, combined with bitwise
// operators (short-circuit && / || and ?: chains over one value get turned
// into switch trees of divergent branches).
__device__ __forceinline__ uint32_t pick(bool c, uint32_t x, uint32_t y)
{
	return y ^ ((x ^ y) & (0u - (uint32_t)c));
}

// (the window's dwords 3..16 as values: dw[j] = dword j of the frame; the
// row form below reads them from an LDS row one at a time)
template <uint32_t FEAT, int W>
__device__ __forceinline__ Parse4 parse_bf_dw(const uint32_t (&dw)[17], uint32_t len)
{
	const uint32_t d3 = dw[3], d5 = dw[5], d6 = dw[6], d7 = dw[7], d8 = dw[8], d9 = dw[9];
	const uint32_t d11 = dw[11], d13 = dw[13], d14 = dw[14];
	uint32_t d16 = 0;
	if constexpr (W >= 68)
		d16 = dw[16];
	const uint32_t et = d3 & 0xffff;   // raw (network-order) ethertype
	const bool runt = len < 14;        // parse_ethhdr
	const bool is4 = et == 0x0008, is6 = et == 0xdd86;
	const bool vlan = (et == 0x0081) | (et == 0xa888);
	const bool arp = et == 0x0608;
	// a VLAN tag past the frame: parse_ethhdr stops at it (parsing_helpers.h
	// :121-126) and returns the tag's ethertype -- no IP, no lookups
	const bool vshort = len < 18;
	// parse_arphdr (parsing_helpers.h:235-253; ARP is parsed only with the
	// IPv4 feature, xdpfilt_prog.h:240-261): a short or non-Ethernet/IPv4
	// ARP header is a parse failure, decided here
	constexpr bool ARPP = (FEAT & F_IPV4) != 0;
	bool arpbad = false;
	if constexpr (ARPP)
		arpbad = arp & ((len < 42) | ((d3 >> 16) != 0x0100u) | (dw[4] != 0x04060008u));
	// IPv4 (__parse_iphdr, frags ok, no version check): ihl 5 keeps L4 at 34
	const bool s4 = len < 34;
	const uint32_t ihl = (d3 >> 16) & 0xf;
	const bool ihl5 = ihl == 5;
	// (parsing_helpers.h:215: a header past the frame is a parse failure,
	// decided here; any other ihl but 5 moves L4: deferred)
	const bool ihlx = 14 + ihl * 4 > len;
	const uint32_t proto = d5 >> 24;
	const bool u4 = (FEAT & F_UDP) && proto == 17, t4 = (FEAT & F_TCP) && proto == 6;
	const uint32_t ulen4 = ((d9 >> 8) & 0xff00) | (d9 >> 24);
	const uint32_t doff4 = (d11 >> 20) & 0xf;
	const bool ab4 = (u4 & ((len < 42) | (ulen4 < 8))) | (t4 & ((len < 54) | (34 + doff4 * 4 > len)));
	// IPv6 (__parse_ip6hdr + skip_ip6hdrext): a final next header at 54;
	// extension headers 0, 43, 44, 51, 58 (as the walk treats it), 60, 135
	const uint32_t nh = d5 & 0xff;
	constexpr uint64_t EXT = (1ull << 0) | (1ull << 43) | (1ull << 44) | (1ull << 51) | (1ull << 58) |
				 (1ull << 60);
	const bool ext = ((nh < 64) & (uint32_t)(EXT >> (nh & 63))) | (nh == 135);
	const bool s6 = len < 56;          // len < 54 (header) or the walk's read at 54
	const bool u6 = (FEAT & F_UDP) && nh == 17, t6 = (FEAT & F_TCP) && nh == 6;
	const uint32_t ulen6 = ((d14 >> 8) & 0xff00) | (d14 >> 24);
	const uint32_t doff6 = (d16 >> 20) & 0xf;
	const bool t6far = (W < 68) & t6 & (len >= 74);   // doff at byte 66: past the window
	const bool ab6 = (u6 & ((len < 62) | (ulen6 < 8))) | (t6 & ((len < 74) | (54 + doff6 * 4 > len)));
	Parse4 r;
	r.defer = !runt & ((vlan & !vshort) | (ARPP & arp & !arpbad) | (is4 & !s4 & !ihl5 & !ihlx) |
			   (is6 & !s6 & (ext | t6far)));
	const bool sip = (is4 & (s4 | ihlx)) | (is6 & s6) | arpbad;   // IP / ARP header fails
	const bool sl4 = (is4 & !s4 & ab4) | (is6 & !s6 & ab6);
	r.abort_at = pick(runt, ST_ETH, pick(sip, ST_IP, pick(sl4, ST_L4, NST)));
	const uint32_t l4 = pick(is4, pick(u4, 17u, pick(t4, 6u, 0u)), pick(is6, pick(u6, 17u, pick(t6, 6u, 0u)), 0u));
	r.l4proto = pick(r.abort_at == NST, l4, 0u);
	r.psrc = pick(is4, d8 >> 16, d13 >> 16);
	r.pdst = pick(is4, d9 & 0xffff, d14 & 0xffff);
	r.k4a = __builtin_amdgcn_alignbyte(d8, d7, 2);   // daddr 30..33
	r.k4b = __builtin_amdgcn_alignbyte(d7, d6, 2);   // saddr 26..29
	r.v4ok = !runt & is4 & !s4 & !ihlx;
	r.is6 = !runt & is6;
	r.v6ok = !runt & is6 & !s6;   // an IPv6 lookup runs (before any L4 check)
	return r;
}

template <uint32_t FEAT, int W>
__device__ __forceinline__ Parse4 parse_bf(const uint32_t *row, uint32_t len)
{
	uint32_t dw[17] = {};
	dw[3] = row[3];
	dw[4] = ((FEAT & F_IPV4) != 0) ? row[4] : 0u;
#pragma unroll
	for (int j = 5; j <= 9; j++)
		dw[j] = row[j];
	dw[11] = row[11];
	dw[13] = row[13];
	dw[14] = row[14];
	if constexpr (W >= 68)
		dw[16] = row[16];
	return parse_bf_dw<FEAT, W>(dw, len);
}

// The port rule of `key` in the workgroup's LDS copy: its flags, and with
// the open-addressed table its slot (the workgroup's direct counter for
// it; XFG_PORT_TAB with the nibble map).  The probe runs the table's
// longest displacement for every lane (keys are unique, so at most one
// slot matches).
__device__ __forceinline__ uint32_t port_probe(const uint32_t *s_ports, bool tab, uint32_t disp,
					       uint32_t key, uint32_t &slot)
{
	slot = XFG_PORT_TAB;
	if (!tab)
		return (s_ports[key >> 3] >> ((key & 7) * 4)) & 15;
	uint32_t f = 0, sl = xfg_port_slot(key);
	for (uint32_t d = 0; d <= disp; d++) {
		const uint32_t e = s_ports[sl];
		const bool m = (e != 0) & ((e & 0xffff) == key);
		f = pick(m, e >> 16, f);
		slot = pick(m, sl, slot);
		sl = (sl + 1) & (XFG_PORT_TAB - 1);
	}
	return f;
}

// bits of the per-packet key flags
constexpr uint32_t KF_A = 1, KF_B = 2, KF_AZ = 4, KF_BZ = 8;

#ifdef XFG_MARK   // ISA study: stage markers in the assembly
#define PMARK(x) asm volatile("; MARK " x)
#else
#define PMARK(x)
#endif

template <uint32_t FEAT, int W, bool DENSE>
__global__ __launch_bounds__(PIPE_THREADS(W), (W) <= 64 ? 4 : 2) void xfg_pipe4_kernel(const xfg_kargs a)
{
	static_assert((FEAT & F_IPV4) != 0, "IPv4-key mode needs the IPv4 feature");
	constexpr int NW = PIPE_WAVES(W);
	constexpr int NT = 64 * NW;
	constexpr int CPP = W / 16;
	constexpr int ROWDW = W / 4 + 1;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;
	// the wave rows; after the loop, the hit-log partition scratch
	__shared__ uint32_t win[NW * 64 * ROWDW > LOG_SCRATCH ? NW * 64 * ROWDW : LOG_SCRATCH];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_pcnt[PORTS ? XFG_PORT_TAB : 1];   // per port-table slot
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES], s_tn[NW];
	__shared__ uint32_t s_lh[XFG_LOG_PARTS];   // hit-log entries per partition
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: scalar control flow
	// the IPv4 table, in scalar registers
	const uint32_t nb = rfl(a.t4.nbuckets), md = rfl(a.t4.max_disp), ns = rfl(a.t4.nslots);
	const uint32_t zp = rfl(a.t4.zero_present), bw = rfl(a.t4.bloom_words);
	const uint32_t seed = rfl(a.t4.seed), gb = rfl(a.gbase[0]), gb3 = rfl(a.gbase[3]);
	const uint64_t bk = rfl64((uint64_t)(uintptr_t)a.t4.buckets);
	const uint64_t bl = rfl64((uint64_t)(uintptr_t)a.t4.bloom);
	// live lookups (census): key a = dst if dst rules exist else src; key b
	// = src when both directions are live
	const bool dlive = a.t4.count && can_hit(a.t4.fmask, M_DST);
	const bool slive = a.t4.count && can_hit(a.t4.fmask, M_SRC);
	const uint32_t mask_a = dlive ? M_DST : M_SRC;
#ifdef XFG_DIAG
	// diagnostics build: drop one cost (results wrong): 1 counter bumps,
	// 2 bucket-line loads, 4 Bloom loads, 8 verdict stores
	const uint32_t dg = a.diag;
#else
	constexpr uint32_t dg = 0;
#endif
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, NT);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, NT);
	const bool ptab = PORTS && a.port_count && a.port_tab;
	const uint32_t pdisp = rfl(a.port_tab_disp);
	if constexpr (PORTS)
		for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
			s_pcnt[i] = 0;
	for (int i = tid; i < (int)XFG_LOG_PARTS; i += NT)
		s_lh[i] = 0;
	__syncthreads();

	uint32_t *const rows = win + wv * 64 * ROWDW;
	const uint32_t *const myrow = rows + lane * ROWDW;
	// (wave-uniform pointers, kept in scalar registers)
	uint32_t *const dlist = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.defer + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t *const tregion = reinterpret_cast<uint32_t *>(
		rfl64((uint64_t)(uintptr_t)(a.tlog + ((uint64_t)blockIdx.x * NW + wv) * a.defer_cap)));
	uint32_t tn = 0;
	const uint32_t lg_lo = rfl(a.dcnt), lg_hi = a.tlog ? rfl(a.gbase[3]) : 0u;
	// a hit's counter: a ruled port's goes to its table slot's LDS counter,
	// a direct counter's to LDS, a hash-map counter's to the hit log, any
	// other (the nibble map's ports, the log off) through Counters::bump
	auto count = [&](uint32_t tag, uint32_t pslot) {
		const bool ps = pslot < XFG_PORT_TAB;
		const bool dc = tag < lg_lo;
		const bool lg = (tag >= lg_lo) & (tag < lg_hi);
		log_append(tregion, tn, pick(lg, tag, CT_NONE), lane);
		if (lg)
			atomicAdd(&s_lh[log_part(tag)], 1u);
		if constexpr (PORTS)
			if (ps)
				atomicAdd(&s_pcnt[pslot], 1u);
		if (dc & !ps)
			atomicAdd(&cn.dcnt[tag], 1u);
		cn.bump(a, pick(lg | dc | ps, CT_NONE, tag), lane);
	};
	const uint32_t n = (uint32_t)a.n;
	const uint32_t nt = (n + 63) / 64;
	const uint32_t first = blockIdx.x * NW + wv;
	const uint32_t step = gridDim.x * NW;
	// per-action packets (wave totals, scalar) and bytes (per lane)
	uint32_t st_c0 = 0, st_c1 = 0, st_c2 = 0, st_b0 = 0, st_b1 = 0, st_b2 = 0;
	auto stat = [&](uint32_t act, uint32_t len) {
		st_c0 += (uint32_t)__popcll(__ballot(act == A_ABORTED));
		st_c1 += (uint32_t)__popcll(__ballot(act == A_DROP));
		st_c2 += (uint32_t)__popcll(__ballot(act == A_PASS));
		st_b0 += pick(act == A_ABORTED, len, 0u);
		st_b1 += pick(act == A_DROP, len, 0u);
		st_b2 += pick(act == A_PASS, len, 0u);
	};
	uint32_t ndef = 0;

	// S: windows + lengths of tile t (clamped to the last tile) into
	// registers: CPP + 2 loads, always issued and not consumed here (lanes
	// past the batch's end read a valid address; the staging zeroes them),
	// so an iteration ends with exactly that many outstanding.  A length is
	// two 16-bit loads (the same one twice for 16-bit lengths), so that one
	// instruction sequence serves both length widths.
	const bool l16 = a.lens_u16 != 0;
	const uint32_t lsh = l16 ? 1u : 2u;
	const uint64_t lb = rfl64((uint64_t)(uintptr_t)a.lens);
	auto issue = [&](uint32_t t, u32x4 (&pre)[CPP], uint16_t (&plen)[2]) {
		t = t < nt ? t : nt - 1;
		const uint32_t base = t * 64;
		const uint32_t rem = n - base >= 64 ? 64u : n - base;
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const uint32_t c = it * 64 + lane, pk = c / CPP, sub = c % CPP;
			const uint32_t q = pk < rem ? pk : 0u;
			const u32x4 *src = DENSE ? reinterpret_cast<const u32x4 *>(a.data + (uint64_t)base * W) + (q * CPP + sub)
						 : reinterpret_cast<const u32x4 *>(a.data + (uint64_t)(base + q) * a.stride + sub * 16);
			pre[it] = __builtin_nontemporal_load(src);
		}
		const uint64_t la = lb + ((uint64_t)(base + ((uint32_t)lane < rem ? lane : 0u)) << lsh);
		plen[0] = *reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(la);
		plen[1] = *reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(la + (lsh - 1) * 2);
	};

	// per-packet fallback state, packed: action (3 bits), port-table slot
	// (12), length (17; the pipelined path takes strides below 2^16)
	auto pk3 = [](uint32_t act, uint32_t ps, uint32_t len) { return act | ps << 3 | len << 15; };
	auto pk_act = [](uint32_t p) { return p & 7; };
	auto pk_ps = [](uint32_t p) { return (p >> 3) & 0xfff; };
	auto pk_len = [](uint32_t p) { return p >> 15; };
	// P -> Q (tile k-1)
	uint32_t q_ka = 0, q_kb = 0, q_wa = 0, q_wb = 0, q_f = 0;
	uint32_t q_pk = pk3(A_NONE, XFG_PORT_TAB, 0), q_tag = CT_NONE;
	// Q -> R (tile k-2)
	uint32_t r_key = 0, r_b = 0, r_mask = 0, r_pk = pk3(A_NONE, XFG_PORT_TAB, 0), r_tag = CT_NONE;
	bool r_sel = false, r_zero = false, r_more = false;

	// One iteration: `cur` holds tile k's windows (issued two iterations
	// ago), `nxt` tile k+1's (issued one iteration ago, still in flight);
	// tile k+2's go into `cur` last.  The wave runs its tiles + 2 iterations
	// (a fixed trip count: no early-out path for the wait placement to merge).
	auto iteration = [&](uint32_t k, u32x4 (&cur)[CPP], uint16_t (&curlen)[2]) {
		const uint32_t tP = first + k * step;
		const bool vP = tP < nt;
		const bool vQ = k >= 1 && tP - step < nt;
		const bool vR = k >= 2 && tP - 2 * step < nt;
		// the iteration's one wait: everything but the last tile's windows
		// (an explicit wait the compiler's own placement sees)
		__builtin_amdgcn_s_waitcnt(0x0F70 | ((CPP + 2) & 15) | (((CPP + 2) >> 4) << 14));
		asm volatile("" ::: "memory");   // (the LDS-DMA'd lines: read only after the wait)

		PMARK("R");
		// ---- R: match (CHECK_MAP, xdpfilt_prog.h:56-64) -> verdict, counter
		const uint32_t r_act = pk_act(r_pk), r_ps = pk_ps(r_pk), w_len = pk_len(r_pk);
		uint32_t w_act = A_NONE, w_tag = CT_NONE, w_ps = r_ps;
		if (vR) {
			// the candidate line, LDS-DMA'd by L into the wave's rows
			// (packet p's at byte 64p)
			Line r_line;
			{
				const u32x4 *lp4 = reinterpret_cast<const u32x4 *>(rows) + lane * 4;
				r_line.q0 = lp4[0];
				r_line.q1 = lp4[1];
				r_line.q2 = lp4[2];
				r_line.q3 = lp4[3];
			}
			const int m = match_v4(r_line, r_key);
			const bool found = r_zero | (m >= 0);
			const uint32_t i = pick(r_zero | (m < 0), 0u, (uint32_t)m);
			const uint32_t fl = r_line.flag((int)i);
			const bool hit = r_sel & found & ((fl & r_mask) == r_mask);
			const uint32_t slot = pick(r_zero, ns, r_b * XFG_SLOTS_V4 + i);
			const bool defer = r_sel & !hit & (r_more | (!found & r_line.overflow() & (md != 0)));
			w_act = pick(hit, HIT, pick(defer, A_DEFER, r_act));
			w_tag = pick(hit, gb + slot, pick(defer, CT_NONE, r_tag));
			w_ps = pick(hit | defer, XFG_PORT_TAB, r_ps);
		}

		PMARK("W");
		// ---- W: verdicts, counters, stats, deferrals of tile k-2
		if (vR) {
			const uint32_t gi = (tP - 2 * step) * 64 + lane;
			if (w_act <= A_PASS && !(dg & 8))
				__builtin_nontemporal_store((uint8_t)w_act, a.verdicts + gi);
			PMARK("C");
			count((dg & 1) ? CT_NONE : w_tag, (dg & 1) ? XFG_PORT_TAB : w_ps);
			PMARK("T");
			stat(w_act, w_len);
			const unsigned long long dm = __ballot(w_act == A_DEFER);
			if (dm) {
				const uint32_t pos = ndef + lanes_below(dm);
				if (w_act == A_DEFER)
					gst32(dlist + pos, gi);
				ndef += (uint32_t)__popcll(dm);
			}
		}

		PMARK("Q");
		// ---- Q: tile k-1's Bloom words -> first candidate key, its bucket
		bool lsel = false;
		if (vQ) {
			const uint32_t q_ha = xfg_hash_v4(q_ka, seed), q_hb = xfg_hash_v4(q_kb, seed);
			const uint32_t bma = xfg_bloom_mask(q_ha), bmb = xfg_bloom_mask(q_hb);
			const bool za = (q_f & KF_AZ) != 0, zb = (q_f & KF_BZ) != 0;
			const bool ma = ((q_f & KF_A) != 0) & (za ? zp != 0 : (q_wa & bma) == bma);
			const bool mb = ((q_f & KF_B) != 0) & (zb ? zp != 0 : (q_wb & bmb) == bmb);
			r_sel = ma | mb;
			r_more = ma & mb;
			r_key = pick(ma, q_ka, q_kb);
			r_zero = ma ? za : zb;
			r_mask = pick(ma, mask_a, M_SRC);
			r_b = pick(r_zero, nb, xfg_home(pick(ma, q_ha, q_hb), nb));
			r_pk = q_pk;
			r_tag = q_tag;
			lsel = r_sel;
		}

		PMARK("S");
		// ---- S: tile k's windows into the LDS rows (past the batch's
		// end: zeroes), its lengths clamped to the stride (the slot is the
		// frame's buffer)
		uint32_t len = 0;
		if (vP) {
			const uint32_t rem = n - tP * 64 >= 64 ? 64u : n - tP * 64;
			__builtin_amdgcn_wave_barrier();
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * 64 + lane;
				const int pk = c / CPP, sub = c % CPP;
				const bool ok = (uint32_t)pk < rem;
				uint32_t *dst = &rows[pk * ROWDW + sub * 4];
				dst[0] = ok ? cur[it].x : 0u;
				dst[1] = ok ? cur[it].y : 0u;
				dst[2] = ok ? cur[it].z : 0u;
				dst[3] = ok ? cur[it].w : 0u;
			}
			const uint32_t l = l16 ? (uint32_t)curlen[0] : (uint32_t)curlen[0] | (uint32_t)curlen[1] << 16;
			len = (uint32_t)lane < rem ? min(l, a.stride) : 0u;
			__builtin_amdgcn_wave_barrier();
		}

		PMARK("P");
		// ---- P: parse tile k, its keys, its fallback; Bloom words issued
		if (vP) {
			const uint32_t gi = tP * 64 + lane;
			const Parse4 r = parse_bf<FEAT, W>(myrow, len);
			const bool valid = gi < n;
			const bool kok = valid & !r.defer & r.v4ok;
			const bool ka = kok & (dlive | slive);
			const bool kb = kok & dlive & slive;
			q_ka = dlive ? r.k4a : r.k4b;
			q_kb = r.k4b;
			const uint32_t q_ha = xfg_hash_v4(q_ka, seed), q_hb = xfg_hash_v4(q_kb, seed);
			q_f = pick(ka, KF_A, 0u) | pick(kb, KF_B, 0u) | pick(q_ka == 0, KF_AZ, 0u) |
			      pick(q_kb == 0, KF_BZ, 0u);
			// fallback: ABORTED at a failed check, else the port stage
			// (dst then src, xdpfilt_prog.h:268-301; l4proto is 0 unless the
			// parse reached a UDP/TCP header)
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
						const bool h = !ph & (r.l4proto != 0) & ((f & mk) == mk) & can_hit(pfm, mk);
						ft = pick(h, gb3 + r.psrc, ft);
						fs = pick(h, sl, fs);
						ph |= h;
					}
					fa = pick(ph, HIT, fa);
				}
			}
			PMARK("B");
			q_pk = pk3(pick(!valid, A_NONE, pick(r.defer, A_DEFER, fa)),
				   pick(valid & !r.defer, fs, XFG_PORT_TAB), len);
			q_tag = pick(valid & !r.defer, ft, CT_NONE);
			q_wa = q_wb = ~0u;
			if ((q_f & (KF_A | KF_AZ)) == KF_A && !(dg & 4))
				q_wa = gload32(bl + 4ull * xfg_bloom_word(q_ha, bw));
			if ((q_f & (KF_B | KF_BZ)) == KF_B && !(dg & 4))
				q_wb = gload32(bl + 4ull * xfg_bloom_word(q_hb, bw));
		}

		PMARK("L");
		// ---- L: tile k-1's candidate bucket lines, LDS-DMA'd into the
		// wave's rows (free again once P has read them): instruction q
		// carries packets 16q..16q+15, four lanes a line, so every line is
		// one full 64-byte request
		{
			const unsigned long long need = __ballot(lsel && !(dg & 2));
			if (need) {
				__builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): P's row reads are done
				__builtin_amdgcn_sched_barrier(0);
#pragma unroll
				for (int q = 0; q < 4; q++) {
					const uint32_t p = q * 16 + (lane >> 2);
					const uint32_t pj = lane & 3;
					const uint32_t bp = __shfl(r_b, (int)p);
					if ((need >> p) & 1)
						__builtin_amdgcn_global_load_lds(
							(const __attribute__((address_space(1))) void *)(
								bk + (uint64_t)bp * XFG_BUCKET_BYTES + pj * 16),
							(__attribute__((address_space(3))) void *)(rows + q * 256), 16, 0, 0);
				}
			}
		}
		PMARK("I");
		// ---- tile k+2's windows, last: in flight for two iterations
		__builtin_amdgcn_sched_barrier(0);
		issue(tP + 2 * step, cur, curlen);
		__builtin_amdgcn_sched_barrier(0);
	};

	u32x4 preA[CPP], preB[CPP];
	uint16_t lenA[2] = { 0, 0 }, lenB[2] = { 0, 0 };
	// (scheduling barriers keep the issue order the waits count on)
	if (nt) {
		issue(first, preA, lenA);
		__builtin_amdgcn_sched_barrier(0);
		issue(first + step, preB, lenB);
		__builtin_amdgcn_sched_barrier(0);
	}
	const uint32_t iters = first < nt ? (nt - 1 - first) / step + 3 : 0u;
	uint32_t k = 0;
	for (; k + 1 < iters; k += 2) {
		iteration(k, preA, lenA);
		iteration(k + 1, preB, lenB);
	}
	if (k < iters)
		iteration(k, preA, lenA);

	// (diagnostics: 2048 skips the deferred packets, 4096 the counter
	// flushes -- results wrong; the tail's phases measured by subtraction)
	if (dg & 2048)
		ndef = 0;
	for (uint32_t d0 = 0; d0 < ndef; d0 += 64) {
		uint32_t act = A_NONE, tag = CT_NONE, len = 0;
		const bool ok = d0 + lane < ndef;
		const uint32_t gi = ok ? gld32(dlist + d0 + lane) : 0u;
		if (ok)
			len = min(load_len(a, gi), a.stride);
#ifdef XFG_DIAG
		if (dg & 32) {   // diagnostics: the byte-load path
			if (ok)
				act = classify_one<FEAT>(a, s_ports, gi, len, tag);
		} else
#endif
			act = classify_staged<FEAT, W>(a, s_ports, const_cast<uint32_t *>(myrow), ok, gi, len, tag);
		if (ok)
			__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
		count(tag, XFG_PORT_TAB);
		stat(act, len);
	}

	const uint32_t vb[3] = { st_b0, st_b1, st_b2 }, vc[3] = { st_c0, st_c1, st_c2 };
#pragma unroll
	for (int kk = 0; kk < 3; kk++) {
		unsigned long long x = vb[kk];
#pragma unroll
		for (int o = 32; o > 0; o >>= 1)
			x += __shfl_xor(x, o);
		if (lane == 0 && vc[kk]) {
			atomicAdd(&s_stats[2 * kk], (unsigned long long)vc[kk]);
			atomicAdd(&s_stats[2 * kk + 1], x);
		}
	}
	if (lane == 0)
		s_tn[wv] = tn;
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	if (!(dg & 4096)) {
		cn.flush(a, tid, NT);
		if constexpr (PORTS)
			if (ptab)
				for (int i = tid; i < (int)XFG_PORT_TAB; i += NT)
					if (s_pcnt[i])
						atomicAdd(a.port_hits + (s_tab[i] & 0xffff), (unsigned long long)s_pcnt[i]);
	}
	if (a.tlog && !(dg & 16))   // (win is free now: the partition scratch)
		log_partition<NW>(a, s_tn, s_lh, win, tid);
}

}  // namespace
