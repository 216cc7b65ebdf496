// SPDX-License-Identifier: GPL-2.0
//
// xfg_kernels.hip — the xdp-filter per-packet program as a batch kernel for
// CDNA4 (gfx950).
//
// One kernel template, specialised at compile time exactly like the ten
// reference programs xdp-filter/xdpfilt_{alw,dny}_{all,eth,ip,tcp,udp}.c
// specialise xdp-filter/xdpfilt_prog.h (FEAT = the program's _features word,
// xdpfilt_prog.h:313-315), and by the header window W staged in LDS.
//
// Per workgroup tile of 256 packets (one lane per packet):
//   1. stage: the first W bytes of every packet of the NEXT tile are loaded
//      with coalesced 16-byte non-temporal loads into registers while the
//      current tile is processed (the fixed-stride layout needs no length
//      before loading, so nothing serialises the stream), then written to
//      one LDS row of W+4 bytes per packet (odd dword stride: conflict-free
//      lane-per-packet reads);
//   2. parse: the reference control flow (xdpfilt_prog.h:214-310 over
//      headers/xdp/parsing_helpers.h) is split into its side-effect-free
//      part — header walk, bounds checks, key extraction — done first, and
//      the ordered lookups done after; a packet's lookups and its abort
//      point keep the reference order (eth dst, eth src, ip dst, ip src /
//      ARP / NDISC target, port dst, port src; an abort of a later header
//      only counts if every earlier lookup missed);
//   3. lookups: a Bloom word per key (L2-resident) rejects most misses; the
//      bucket lines of all surviving keys of a stage are loaded together
//      (one 64-byte line holds 12 IPv4 keys, their flag bytes and the
//      overflow bit), then evaluated in reference order;
//   4. the first hit's counter is bumped once the wave re-converges, with
//      same-slot lanes aggregated into one atomic (hot rules);
//   5. verdict bytes are stored coalesced; per-action {packets, bytes}
//      (headers/xdp/xdp_stats_kern.h:29-48) are reduced per wave, per
//      workgroup in LDS, and added to the device stats once per workgroup.
//
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "xfg_layout.h"

namespace {

constexpr uint32_t F_TCP = 1u << 0;
constexpr uint32_t F_UDP = 1u << 1;
constexpr uint32_t F_IPV6 = 1u << 2;
constexpr uint32_t F_IPV4 = 1u << 3;
constexpr uint32_t F_ETH = 1u << 4;
constexpr uint32_t F_DENY = 1u << 6;
// Diagnostics only (XFG_VARIANT >= 0x100 on the headline program): feature-
// word bits that remove a code path to measure its instruction cost.
// Results are wrong with any of them set.
constexpr uint32_t X_NOGEN = 1u << 8;    // no generic parse (fast path or abort)
constexpr uint32_t X_NOV6 = 1u << 9;     // no IPv6 / NDISC lookups
constexpr uint32_t X_NOPORT = 1u << 10;  // no port lookups
constexpr uint32_t X_NOCNT = 1u << 11;   // no counter bump code

constexpr uint32_t M_SRC = 1, M_DST = 2, M_TCP = 4, M_UDP = 8;
constexpr uint32_t A_ABORTED = 0, A_DROP = 1, A_PASS = 2, A_NONE = 7;

constexpr int TILE = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Packet bytes past the staged window, read from HBM through a global-
// address-space pointer: a generic (flat) load would also count against the
// LDS counter and complete out of order, so every wait near it degrades to
// vmcnt(0).
__device__ __forceinline__ uint32_t gbyte(const uint8_t *p, uint32_t o)
{
	return reinterpret_cast<const __attribute__((address_space(1))) uint8_t *>(
		reinterpret_cast<uintptr_t>(p))[o];
}

// ---------------------------------------------------------------- packet view
template <int W>
struct Pkt {
	static constexpr int ROWDW = W / 4 + 1;
	const uint32_t *row;    // LDS row: bytes [0, min(len, W)) valid
	const uint8_t *g;       // packet start in HBM
	uint32_t len;

	// Byte o (caller has checked o < len, as the reference does).
	__device__ __forceinline__ uint32_t u8(uint32_t o) const
	{
		if (o < (uint32_t)W)
			return reinterpret_cast<const uint8_t *>(row)[o];
		return gbyte(g, o);
	}
	// Little-endian 32-bit load of bytes o..o+3 (o+3 < len).
	__device__ __forceinline__ uint32_t u32(uint32_t o) const
	{
		if (o + 4 <= (uint32_t)W) {
			uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, o & 3);
		}
		return gbyte(g, o) | (gbyte(g, o + 1) << 8) | (gbyte(g, o + 2) << 16) |
		       (gbyte(g, o + 3) << 24);
	}
	// Raw (memory-order) 16-bit value of bytes o, o+1: the BPF u16 load.
	__device__ __forceinline__ uint32_t raw16(uint32_t o) const
	{
		if (o + 2 <= (uint32_t)W) {
			uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, o & 3) & 0xffffu;
		}
		return gbyte(g, o) | (gbyte(g, o + 1) << 8);
	}
	// Network-order 16-bit field as a host value (bpf_ntohs of the load).
	__device__ __forceinline__ uint32_t be16(uint32_t o) const
	{
		uint32_t r = raw16(o);
		return ((r & 0xff) << 8) | (r >> 8);
	}
	// Dword k of the window (k < W / 4).
	__device__ __forceinline__ uint32_t dw(int k) const { return row[k]; }
};

// Lookup keys read lazily from a packet view (header bytes still staged).
template <class P>
struct LazyKeys {
	const P &p;
	__device__ __forceinline__ void eth(uint32_t o, uint32_t &lo, uint32_t &hi) const
	{
		lo = p.u32(o);
		hi = p.raw16(o + 4);
	}
	__device__ __forceinline__ void v6(uint32_t o, uint32_t (&k)[4]) const
	{
		k[0] = p.u32(o);
		k[1] = p.u32(o + 4);
		k[2] = p.u32(o + 8);
		k[3] = p.u32(o + 12);
	}
	__device__ __forceinline__ void v6_dst(uint32_t o6, uint32_t (&k)[4]) const { v6(o6 + 24, k); }
	__device__ __forceinline__ void v6_src(uint32_t o6, uint32_t (&k)[4]) const { v6(o6 + 8, k); }
	__device__ __forceinline__ void nd_tgt(uint32_t ond, uint32_t (&k)[4]) const { v6(ond, k); }
};

// ---------------------------------------------------------------- parse result
// Stages of lookups in reference order; `abort_at` = the first stage that is
// not reached because a header check failed (the packet is ABORTED iff every
// lookup of the earlier stages missed), NST = no abort.
enum Stage : uint32_t { ST_ETH = 0, ST_IP = 1, ST_ND = 2, ST_L4 = 3, NST = 4 };

struct Parsed {
	uint32_t abort_at;     // Stage
	uint32_t l3;           // 0 none, 1 IPv4, 2 ARP, 3 IPv6
	uint32_t arp_op;
	uint32_t k4a, k4b;     // IPv4: dst, src | ARP: sip, tip
	uint32_t ka_off, kb_off;   // byte offsets of k4a, k4b in the frame
	uint32_t o6;           // IPv6 header offset (saddr o6+8, daddr o6+24)
	uint32_t nd;           // NDISC: 0 none, 135 NS, 136 NA
	uint32_t ond;          // target offset
	uint32_t l4proto;      // 17 / 6 when an L4 stage runs, else 0
	uint32_t pdst, psrc;   // raw be16 port keys
};

// Fast path for the dominant, well-formed shapes, read at static offsets
// from the LDS row: untagged IPv4 with ihl 5 (UDP, TCP or other protocol)
// and untagged IPv6/UDP without extension headers, each at least as long
// as every field read here.  It produces exactly what parse_generic()
// produces for such a packet (same bounds checks, same keys); every other
// packet takes the generic walk.
template <uint32_t FEAT, int W, class P>
__device__ __forceinline__ bool parse_fast(const P &p, Parsed &r)
{
	if constexpr (W < 64 || (FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
		return false;
	} else {
		const uint32_t len = p.len;
		const uint32_t d3 = p.dw(3);                 // bytes 12..15
		const uint32_t et = d3 & 0xffff;              // raw ethertype
		if (et == 0x0008 && ((d3 >> 16) & 0xff) == 0x45 && len >= 54) {
			// IPv4, ihl 5: l4 at 34; 54 bytes cover the UDP or TCP header
			const uint32_t d5 = p.dw(5), d6 = p.dw(6), d7 = p.dw(7), d8 = p.dw(8),
				       d9 = p.dw(9);
			const uint32_t proto = d5 >> 24;          // byte 23
			r.l3 = 1;
			r.k4a = __builtin_amdgcn_alignbyte(d8, d7, 2);   // daddr 30..33
			r.k4b = __builtin_amdgcn_alignbyte(d7, d6, 2);   // saddr 26..29
			r.ka_off = 30;
			r.kb_off = 26;
			r.psrc = d8 >> 16;                        // bytes 34,35
			r.pdst = d9 & 0xffff;                     // bytes 36,37
			if ((FEAT & F_UDP) && proto == 17) {
				const uint32_t ulen = ((d9 >> 8) & 0xff00) | (d9 >> 24);   // be16 38,39
				if (ulen < 8)
					r.abort_at = ST_L4;
				else
					r.l4proto = 17;
			} else if ((FEAT & F_TCP) && proto == 6) {
				const uint32_t doff = (p.dw(11) >> 20) & 0xf;   // byte 46 >> 4
				if (34 + doff * 4 > len)
					r.abort_at = ST_L4;
				else
					r.l4proto = 6;
			}
			return true;
		}
		if (et == 0xdd86 && len >= 62 && (p.dw(5) & 0xff) == 17) {
			// IPv6, next header UDP: l4 at 54 (the 2-byte extension-walk
			// read at 54 is covered by len >= 62)
			r.l3 = 3;
			r.o6 = 14;
			if constexpr ((FEAT & F_UDP) != 0) {
				const uint32_t d13 = p.dw(13), d14 = p.dw(14);
				const uint32_t ulen = ((d14 >> 8) & 0xff00) | (d14 >> 24);   // 58,59
				r.psrc = d13 >> 16;                   // 54,55
				r.pdst = d14 & 0xffff;                // 56,57
				if (ulen < 8)
					r.abort_at = ST_L4;
				else
					r.l4proto = 17;
			}
			return true;
		}
		return false;
	}
}

template <uint32_t FEAT, int W, class P>
__device__ __forceinline__ Parsed parse(const P &p)
{
	Parsed r;
	r.abort_at = NST;
	r.l3 = 0;
	r.nd = 0;
	r.l4proto = 0;
	r.arp_op = 0;
	r.k4a = r.k4b = 0;
	r.ka_off = r.kb_off = 0;
	r.o6 = r.ond = 0;
	r.pdst = r.psrc = 0;
	if (parse_fast<FEAT, W, P>(p, r))
		return r;
	if constexpr ((FEAT & X_NOGEN) != 0) {
		r.abort_at = ST_ETH;
		return r;
	}
	const uint32_t len = p.len;

	// parse_ethhdr (parsing_helpers.h:100-134), VLAN_MAX_DEPTH 4
	if (14 > len) {
		r.abort_at = ST_ETH;
		return r;
	}
	uint32_t proto = p.be16(12), off = 14;
#pragma unroll
	for (int i = 0; i < 4; i++) {
		if (proto != 0x8100 && proto != 0x88A8)
			break;
		if (off + 4 > len)
			break;
		proto = p.be16(off + 2);
		off += 4;
	}
	if constexpr ((FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
		return r;
	} else {
		uint32_t ip_type = 0, l4 = 0;
		if (proto == 0x0800) {
			// __parse_iphdr, frags_ok = 1 (parsing_helpers.h:201-227)
			if (off + 20 > len) {
				r.abort_at = ST_IP;
				return r;
			}
			const uint32_t hdrsize = (p.u8(off) & 0xF) * 4;
			if (off + hdrsize > len) {
				r.abort_at = ST_IP;
				return r;
			}
			ip_type = p.u8(off + 9);
			l4 = off + hdrsize;
			r.l3 = 1;
			if constexpr ((FEAT & F_IPV4) != 0) {
				r.k4a = p.u32(off + 16);   // daddr: checked first
				r.k4b = p.u32(off + 12);   // saddr
				r.ka_off = off + 16;
				r.kb_off = off + 12;
			}
		} else if ((FEAT & F_IPV4) && proto == 0x0806) {
			// parse_arphdr (parsing_helpers.h:235-253), xdpfilt_prog.h:241-261
			if (off + 28 > len || p.be16(off) != 1 || p.be16(off + 2) != 0x0800 ||
			    p.u8(off + 4) != 6 || p.u8(off + 5) != 4) {
				r.abort_at = ST_IP;
				return r;
			}
			r.l3 = 2;
			r.arp_op = p.be16(off + 6);
			r.k4a = p.u32(off + 14);   // sip
			r.k4b = p.u32(off + 24);   // tip
			r.ka_off = off + 14;
			r.kb_off = off + 24;
			return r;                  // ip_type stays 0: no L4 stage
		} else if (proto == 0x86DD) {
			// __parse_ip6hdr + skip_ip6hdrext (parsing_helpers.h:136-199)
			if (off + 40 > len) {
				r.abort_at = ST_IP;
				return r;
			}
			uint32_t nh = p.u8(off + 6), cur = off + 40;
			bool done = false;
			for (int i = 0; i < 6; i++) {   // IPV6_EXT_MAX_CHAIN
				if (cur + 2 > len)
					break;
				if (nh == 0 || nh == 60 || nh == 43 || nh == 135) {
					const uint32_t hl = p.u8(cur + 1);
					nh = p.u8(cur);
					cur += (hl + 1) * 8;
				} else if (nh == 51) {
					const uint32_t hl = p.u8(cur + 1);
					nh = p.u8(cur);
					cur += (hl + 2) * 4;
				} else if (nh == 44) {
					nh = p.u8(cur);
					cur += 8;
				} else {
					done = true;
					break;
				}
			}
			if (!done) {
				r.abort_at = ST_IP;
				return r;
			}
			ip_type = nh;
			l4 = cur;
			r.l3 = 3;
			r.o6 = off;
			if (ip_type == 58) {
				// parse_icmp6hdr + NDISC target (xdpfilt_prog.h:268-287):
				// checked after the IPv6 address lookups
				if (cur + 8 > len) {
					r.abort_at = ST_ND;
					return r;
				}
				const uint32_t t = p.u8(cur);
				if (t == 135 || t == 136) {
					if (cur + 24 > len) {
						r.abort_at = ST_ND;
						return r;
					}
					r.nd = t;
					r.ond = cur + 8;
				}
				return r;
			}
		} else {
			return r;   // not IP: MISS after the ethernet stage
		}

		if ((FEAT & F_UDP) && ip_type == 17) {
			// parse_udphdr (parsing_helpers.h:303-321)
			if (l4 + 8 > len || p.be16(l4 + 4) < 8) {
				r.abort_at = ST_L4;
				return r;
			}
			r.l4proto = 17;
		} else if ((FEAT & F_TCP) && ip_type == 6) {
			// parse_tcphdr (parsing_helpers.h:326-344)
			if (l4 + 20 > len || l4 + (p.u8(l4 + 12) >> 4) * 4 > len) {
				r.abort_at = ST_L4;
				return r;
			}
			r.l4proto = 6;
		} else {
			return r;
		}
		r.pdst = p.raw16(l4 + 2);
		r.psrc = p.raw16(l4);
		return r;
	}
}

// ---------------------------------------------------------------- table probes
__device__ __forceinline__ const uint8_t *bucket_ptr(const xfg_tdesc &t, uint32_t b)
{
	return static_cast<const uint8_t *>(t.buckets) + (uint64_t)b * XFG_BUCKET_BYTES;
}

__device__ __forceinline__ bool bloom_maybe(const xfg_tdesc &t, uint32_t h)
{
	const unsigned long long w = t.bloom[xfg_bloom_word(h, t.bloom_words)];
	const unsigned long long m = xfg_bloom_mask(h);
	return (w & m) == m;
}

// One 64-byte bucket line held in registers.
struct Line {
	u32x4 q0, q1, q2, q3;
	__device__ __forceinline__ uint32_t w(int i) const   // dword i of the line
	{
		return i < 4 ? q0[i] : i < 8 ? q1[i - 4] : i < 12 ? q2[i - 8] : q3[i - 12];
	}
	__device__ __forceinline__ uint32_t flag(int slot) const   // flag byte of slot
	{
		const uint32_t fw = slot < 4 ? q3.x : slot < 8 ? q3.y : q3.z;
		return (fw >> (8 * (slot & 3))) & 0xff;
	}
	__device__ __forceinline__ bool overflow() const { return q3.w & XFG_META_OVERFLOW; }
};

// NT: non-temporal loads, so random bucket lines do not push the Bloom
// filter out of L2.
template <bool NT>
__device__ __forceinline__ Line load_line(const xfg_tdesc &t, uint32_t b)
{
	const u32x4 *p = reinterpret_cast<const u32x4 *>(bucket_ptr(t, b));
	Line l;
	if constexpr (NT) {
		l.q0 = __builtin_nontemporal_load(p);
		l.q1 = __builtin_nontemporal_load(p + 1);
		l.q2 = __builtin_nontemporal_load(p + 2);
		l.q3 = __builtin_nontemporal_load(p + 3);
	} else {
		l.q0 = p[0];
		l.q1 = p[1];
		l.q2 = p[2];
		l.q3 = p[3];
	}
	return l;
}

// Match result: slot (-1 = absent) and its flag byte.
struct Hit {
	int64_t slot;
	uint32_t flags;
};

__device__ __forceinline__ int match_v4(const Line &l, uint32_t k)
{
	uint32_t m = 0;
#pragma unroll
	for (int i = 0; i < 12; i++)
		m |= (uint32_t)(l.w(i) == k) << i;
	return m ? __builtin_ctz(m) : -1;
}

__device__ __forceinline__ int match_v6(const Line &l, uint32_t w0, uint32_t w1, uint32_t w2,
					uint32_t w3)
{
#pragma unroll
	for (int i = 0; i < 3; i++)
		if (l.w(4 * i) == w0 && l.w(4 * i + 1) == w1 && l.w(4 * i + 2) == w2 &&
		    l.w(4 * i + 3) == w3)
			return i;
	return -1;
}

__device__ __forceinline__ int match_eth(const Line &l, uint32_t lo, uint32_t hi)
{
#pragma unroll
	for (int i = 0; i < 6; i++)
		if (l.w(2 * i) == lo && l.w(2 * i + 1) == hi)
			return i;
	return -1;
}

template <int KIND>
__device__ __forceinline__ int match(const Line &l, uint32_t k0, uint32_t k1, uint32_t k2,
				     uint32_t k3)
{
	if constexpr (KIND == 4)
		return match_v4(l, k0);
	else if constexpr (KIND == 6)
		return match_v6(l, k0, k1, k2, k3);
	else
		return match_eth(l, k0, k1);
}

template <int KIND>
constexpr uint32_t slots_of()
{
	return KIND == 4 ? XFG_SLOTS_V4 : KIND == 6 ? XFG_SLOTS_V6 : XFG_SLOTS_ETH;
}

// The zero key lives in bucket nbuckets, slot 0.
__device__ __forceinline__ Hit zero_hit(const xfg_tdesc &t)
{
	if (!t.zero_present)
		return { -1, 0 };
	return { (int64_t)t.nslots, bucket_ptr(t, t.nbuckets)[XFG_FLAGS_OFF] };
}

// Continue a probe past a full home bucket (rare): linear over buckets.
template <int KIND, bool NT>
__device__ __forceinline__ Hit probe_chain(const xfg_tdesc &t, uint32_t b, uint32_t k0, uint32_t k1,
					uint32_t k2, uint32_t k3)
{
	for (uint32_t d = 1; d <= t.max_disp; d++) {
		b = b + 1 == t.nbuckets ? 0 : b + 1;
		const Line l = load_line<NT>(t, b);
		const int i = match<KIND>(l, k0, k1, k2, k3);
		if (i >= 0)
			return { (int64_t)b * slots_of<KIND>() + i, l.flag(i) };
		if (!l.overflow())
			break;
	}
	return { -1, 0 };
}

// A pending lookup: hash computed and Bloom word tested.  The Bloom words of
// all keys of a stage are loaded together (8 bytes each, L2-resident); the
// bucket line is fetched only for a key the filter passes, one at a time,
// which keeps a single 64-byte line live per lane.
template <int KIND, bool NT = false>
struct Probe {
	uint32_t k0, k1, k2, k3;
	uint32_t b;
	bool zero, live;

	__device__ __forceinline__ void start(const xfg_tdesc &t, bool want, uint32_t a0,
					      uint32_t a1 = 0, uint32_t a2 = 0, uint32_t a3 = 0)
	{
		k0 = a0; k1 = a1; k2 = a2; k3 = a3;
		zero = want && (a0 | a1 | a2 | a3) == 0;
		live = false;
		b = 0;
		if (!want || zero)
			return;
		uint32_t h;
		if constexpr (KIND == 4)
			h = xfg_hash_v4(a0, t.seed);
		else if constexpr (KIND == 6)
			h = xfg_hash_v6(a0, a1, a2, a3, t.seed);
		else
			h = xfg_hash_eth(a0 | ((uint64_t)a1 << 32), t.seed);
		b = xfg_home(h, t.nbuckets);
		live = bloom_maybe(t, h);
	}
	__device__ __forceinline__ Hit result(const xfg_tdesc &t) const
	{
		if (zero)
			return zero_hit(t);
		if (!live)
			return { -1, 0 };
		const Line l = load_line<NT>(t, b);
		const int i = match<KIND>(l, k0, k1, k2, k3);
		if (i >= 0)
			return { (int64_t)b * slots_of<KIND>() + i, l.flag(i) };
		if (l.overflow() && t.max_disp)
			return probe_chain<KIND, NT>(t, b, k0, k1, k2, k3);
		return { -1, 0 };
	}
};

// Counter identity of a hit: its index in the global counter space (v4
// slots, v6 slots, eth slots, ports; xfg_kargs.gbase), CT_NONE for none.
constexpr uint32_t CT_NONE = 0xffffffffu;

// Counter of global index g (threshold compares: no dynamic index into the
// kernel-argument struct, which would put it in scratch).
__device__ __forceinline__ unsigned long long *global_counter(const xfg_kargs &a, uint32_t g)
{
	if (g >= a.gbase[3])
		return a.port_hits + (g - a.gbase[3]);
	if (g >= a.gbase[2])
		return a.te.hits + (g - a.gbase[2]);
	if (g >= a.gbase[1])
		return a.t6.hits + (g - a.gbase[1]);
	return a.t4.hits + g;
}

// One cold counter bump: appended to the workgroup's region of its hit-log
// partition (a plain store; xfg_hlog_count_kernel adds the regions up), or,
// with no log or a full region, a memory-side atomic.
__device__ __forceinline__ void cold_bump(const xfg_kargs &a, uint32_t *s_pcnt, uint32_t tag)
{
	if (a.hlog) {
		const uint32_t p = tag >> XFG_HLOG_SHIFT;
		const uint32_t pos = atomicAdd(&s_pcnt[p], 1u);
		if (pos < a.hlog_cap) {
			a.hlog[((uint64_t)p * gridDim.x + blockIdx.x) * a.hlog_cap + pos] = tag;
			return;
		}
	}
	atomicAdd(global_counter(a, tag), 1ull);
}

// CHECK_MAP (xdp-filter/xdpfilt_prog.h:56-64): hit iff the key exists and
// (value & mask) == mask; the counter bump is deferred to the caller.
__device__ __forceinline__ bool take(const Hit &h, uint32_t mask, uint32_t base, uint32_t &tag)
{
	if (h.slot >= 0 && (h.flags & mask) == mask) {
		tag = base + (uint32_t)h.slot;
		return true;
	}
	return false;
}

// A lookup with mask m can only hit if some key of the map carries every bit
// of m (the host keeps fmask = OR of all flag bytes): otherwise it is skipped.
__device__ __forceinline__ bool can_hit(uint32_t fmask, uint32_t m)
{
	return (fmask & m) == m;
}

// s_ports: the port table (kargs.port_tab) or, without one, the "any flag"
// bitmap in front of a port_flags read.
__device__ __forceinline__ bool check_port(const xfg_kargs &a, const uint32_t *s_ports,
					   uint32_t key, uint32_t mask, uint32_t &tag)
{
	if (!can_hit(a.port_fmask, mask))
		return false;
	uint32_t f = 0;
	if (a.port_tab) {
		uint32_t sl = xfg_port_slot(key);
		for (uint32_t d = 0; d <= a.port_tab_disp; d++) {
			const uint32_t e = s_ports[sl];
			if (e == 0)
				break;
			if ((e & 0xffff) == key) {
				f = e >> 16;
				break;
			}
			sl = (sl + 1) & (XFG_PORT_TAB - 1);
		}
	} else {
		if (!((s_ports[key >> 5] >> (key & 31)) & 1))
			return false;
		f = a.port_flags[key];
	}
	if ((f & mask) == mask) {
		tag = a.gbase[3] + key;
		return true;
	}
	return false;
}

// ---------------------------------------------------------------- the program
// Ordered lookups over a parsed packet; returns the xdp action and sets tag
// to the first matching rule's counter identity (CT_NONE if none).
template <uint32_t FEAT, bool NT, class KS>
__device__ __forceinline__ uint32_t lookups(const xfg_kargs &a, const KS &ks, const Parsed &r,
					    const uint32_t *s_pbits, uint32_t &tag)
{
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;   // VERDICT_HIT
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;  // VERDICT_MISS

	if (r.abort_at == ST_ETH)
		return A_ABORTED;

	// lookup_verdict_ethernet (xdpfilt_prog.h:187-196): dst then src
	if constexpr ((FEAT & F_ETH) != 0) {
		if (a.te.count) {
			Probe<2, NT> d, s;
			uint32_t dl, dh, sl, sh;
			ks.eth(0, dl, dh);
			ks.eth(6, sl, sh);
			d.start(a.te, can_hit(a.te.fmask, M_DST), dl, dh);
			s.start(a.te, can_hit(a.te.fmask, M_SRC), sl, sh);
			if (take(d.result(a.te), M_DST, a.gbase[2], tag) ||
			    take(s.result(a.te), M_SRC, a.gbase[2], tag))
				return HIT;
		}
	}
	if (r.abort_at == ST_IP)
		return A_ABORTED;

	if constexpr ((FEAT & F_IPV4) != 0) {
		if (a.t4.count && (r.l3 == 1 || r.l3 == 2)) {
			// IPv4: dst (k4a, DST) then src (k4b, SRC)  (xdpfilt_prog.h:121-134)
			// ARP:  sip (k4a, SRC); op 1: tip DST; op 2: tip SRC  (:241-261)
			const bool arp = r.l3 == 2;
			const bool want_b = !arp || r.arp_op == 1 || r.arp_op == 2;
			// The second key's Bloom word is read only when the first key
			// missed: random L2 requests, not latency, bound this stage.
			Probe<4, NT> x, y;
			const uint32_t mx = arp ? M_SRC : M_DST;
			const uint32_t my = arp ? (r.arp_op == 1 ? M_DST : M_SRC) : M_SRC;
			x.start(a.t4, can_hit(a.t4.fmask, mx), r.k4a);
			if (take(x.result(a.t4), mx, a.gbase[0], tag))
				return HIT;
			y.start(a.t4, want_b && can_hit(a.t4.fmask, my), r.k4b);
			if (want_b && take(y.result(a.t4), my, a.gbase[0], tag))
				return HIT;
		}
	}
	if constexpr ((FEAT & F_IPV6) != 0 && (FEAT & X_NOV6) == 0) {
		if (a.t6.count && r.l3 == 3) {
			// lookup_verdict_ipv6: dst then src (xdpfilt_prog.h:152-165)
			Probe<6, NT> d, s;
			uint32_t kd[4], kq[4];
			ks.v6_dst(r.o6, kd);
			ks.v6_src(r.o6, kq);
			d.start(a.t6, can_hit(a.t6.fmask, M_DST), kd[0], kd[1], kd[2], kd[3]);
			s.start(a.t6, can_hit(a.t6.fmask, M_SRC), kq[0], kq[1], kq[2], kq[3]);
			if (take(d.result(a.t6), M_DST, a.gbase[1], tag) ||
			    take(s.result(a.t6), M_SRC, a.gbase[1], tag))
				return HIT;
		}
	}
	if (r.abort_at == ST_ND)
		return A_ABORTED;
	if constexpr ((FEAT & F_IPV6) != 0 && (FEAT & X_NOV6) == 0) {
		if (a.t6.count && r.nd) {
			// NDISC target: NS => DST, NA => SRC (xdpfilt_prog.h:277-285)
			const uint32_t mt = r.nd == 135 ? M_DST : M_SRC;
			Probe<6, NT> t;
			uint32_t kt[4];
			ks.nd_tgt(r.ond, kt);
			t.start(a.t6, can_hit(a.t6.fmask, mt), kt[0], kt[1], kt[2], kt[3]);
			if (take(t.result(a.t6), mt, a.gbase[1], tag))
				return HIT;
		}
	}
	if (r.abort_at == ST_L4)
		return A_ABORTED;
	if constexpr ((FEAT & (F_UDP | F_TCP)) != 0 && (FEAT & X_NOPORT) == 0) {
		if (a.port_count && r.l4proto) {
			// lookup_verdict_udp / _tcp (xdpfilt_prog.h:92-101 / :76-85)
			const uint32_t pm = r.l4proto == 17 ? M_UDP : M_TCP;
			if (check_port(a, s_pbits, r.pdst, M_DST | pm, tag) ||
			    check_port(a, s_pbits, r.psrc, M_SRC | pm, tag))
				return HIT;
		}
	}
	return MISS;
}

// Per-workgroup counter cache in LDS: direct-mapped on the counter identity.
// A rule hit by many packets (a hot port, an attacked address) is summed
// here and reaches memory once per workgroup; a slot already owned by a
// different counter sends the bump straight to its global atomic.
constexpr int CC_ENTRIES = 512;

// Returns true when the LDS cache absorbed the n bumps of counter `tag`.
__device__ __forceinline__ bool cache_hit(uint32_t *s_ctag, uint32_t *s_ccnt, uint32_t tag,
					  uint32_t n)
{
	const uint32_t e = (tag * 0x9E3779B1u) >> 23;   // 9 bits
	uint32_t t = s_ctag[e];
	if (t == CT_NONE) {
		t = atomicCAS(&s_ctag[e], CT_NONE, tag);
		if (t == CT_NONE)
			t = tag;
	}
	if (t != tag)
		return false;
	atomicAdd(&s_ccnt[e], n);
	return true;
}


// Diagnostics (build variant V & 4): per-workgroup cycles spent in each
// phase of the tile loop, stamped by wave 0 and written to kargs.prof.
constexpr int NPHASE = 8;
struct Stamps {
	unsigned long long last;
	uint32_t *acc;   // LDS, NPHASE words
	__device__ __forceinline__ void init(uint32_t *lds)
	{
		acc = lds;
		if (threadIdx.x < NPHASE)
			acc[threadIdx.x] = 0;
		last = __builtin_amdgcn_s_memtime();
	}
	__device__ __forceinline__ void mark(int i)
	{
		const unsigned long long t = __builtin_amdgcn_s_memtime();
		if (threadIdx.x == 0)
			acc[i] += (uint32_t)(t - last);
		last = t;
	}
	__device__ __forceinline__ void store(unsigned long long *prof) const
	{
		if (prof && threadIdx.x == 0 && blockIdx.x < XFG_PROF_WG)
			for (int i = 0; i < NPHASE; i++)
				prof[(uint64_t)blockIdx.x * NPHASE + i] = acc[i];
	}
};

// Word w of packet i's AF_XDP descriptor (ring index wraps with desc_mask).
__device__ __forceinline__ uint64_t desc_word(const xfg_kargs &a, uint64_t i, int w)
{
	return a.descs[2ull * ((a.desc_first + (uint32_t)i) & a.desc_mask) + w];
}

__device__ __forceinline__ uint32_t load_len(const xfg_kargs &a, uint64_t i)
{
	if (a.descs)
		return (uint32_t)desc_word(a, i, 1);   // xdp_desc.len (low half, little-endian)
	return a.lens_u16 ? static_cast<const uint16_t *>(a.lens)[i]
			  : static_cast<const uint32_t *>(a.lens)[i];
}

__device__ __forceinline__ const uint8_t *pkt_ptr(const xfg_kargs &a, uint64_t i)
{
	if (a.descs) {
		// xsk_umem__add_offset_to_addr() (headers/xdp/xsk.h:173-186): the
		// unaligned-chunk mode keeps an offset in bits 48..63
		const uint64_t addr = desc_word(a, i, 0);
		return a.data + (addr & ((1ull << 48) - 1)) + (addr >> 48);
	}
	return a.data + (a.offsets ? a.offsets[i] : i * (uint64_t)a.stride);
}

// ---------------------------------------------------------------- the kernel
// V: build variant bits (production = 0 unless measured better):
//   1 = non-temporal bucket-line loads, 2 = ask the allocator for 5 waves/SIMD
// DENSE: the batch is known to be the dense fixed-stride layout (stride == W,
// no offsets/descriptors), so the stream loads need no per-packet address
// or length: a separate build, as the general load path costs registers.
template <uint32_t FEAT, int W, int V, bool DENSE = false>
__global__ __launch_bounds__(TILE, (V & 2) ? 5 : 1) void xfg_classify_kernel(const xfg_kargs a)
{
	constexpr int CPP = W / 16;            // 16-byte chunks per packet window
	constexpr int ROWDW = Pkt<W>::ROWDW;   // odd dword stride per LDS row
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
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
	for (uint32_t i = tid; i < a.dcnt; i += TILE)   // (s_pcnt holds the direct counters)
		s_pcnt[i] = 0;
	if constexpr (PORTS) {
		if (a.port_count)
			for (int i = tid; i < 2048; i += TILE)
				s_pbits[i] = a.port_tab ? a.port_tab[i] : a.port_bits[i];
	}
	// fixed-stride layout with stride >= W: every window byte is readable,
	// so loads need no length (no load->load dependency on the stream)
	const bool guarded = a.offsets != nullptr || a.stride < (uint32_t)W;

	// WT (V & 8): every wave walks its own tiles of 64 packets with its own
	// LDS rows, so no workgroup barrier sits in the loop; otherwise tiles of
	// TILE packets shared by the workgroup's four waves.
	constexpr bool WT = (V & 8) != 0;
	constexpr int U = WT ? 64 : TILE;          // packets per tile
	const int me = WT ? lane : tid;            // this lane's packet within the tile
	uint32_t *const wrows = WT ? win + (tid >> 6) * 64 * ROWDW : win;
	const uint64_t ntiles = (a.n + U - 1) / U;
	const uint64_t tstep = WT ? (uint64_t)gridDim.x * (TILE / 64) : gridDim.x;
	// dense layout (stride == W, no offsets): a tile is one contiguous block
	// of U * W bytes and chunk c of it sits at byte 16 * c
	const bool dense = !guarded && a.stride == (uint32_t)W;
	uint64_t tile = WT ? (uint64_t)blockIdx.x * (TILE / 64) + (tid >> 6) : blockIdx.x;
	u32x4 pre[CPP];
	uint32_t plen = 0;
	uint32_t c_ab = 0, c_dr = 0, c_pa = 0;
	unsigned long long b_ab = 0, b_dr = 0, b_pa = 0;
	auto issue = [&](uint64_t t) {
		const uint64_t base = t * U;
		if constexpr (DENSE) {
			const u32x4 *src = reinterpret_cast<const u32x4 *>(a.data + base * W) + me;
			const uint32_t rem = a.n - base >= (uint64_t)U ? U : (uint32_t)(a.n - base);
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				pre[it] = u32x4{ 0, 0, 0, 0 };
				if ((uint32_t)(it * U + me) / CPP < rem)
					pre[it] = __builtin_nontemporal_load(src + it * U);
			}
			plen = base + me < a.n ? load_len(a, base + me) : 0;
			return;
		}
		if (dense && base + U <= a.n) {
			const u32x4 *src = reinterpret_cast<const u32x4 *>(a.data + base * W) + me;
#pragma unroll
			for (int it = 0; it < CPP; it++)
				pre[it] = __builtin_nontemporal_load(src + it * U);
		} else {
#pragma unroll
			for (int it = 0; it < CPP; it++) {
				const int c = it * U + me;
				const int pk = c / CPP, sub = c % CPP;
				const uint64_t gi = base + pk;
				pre[it] = u32x4{ 0, 0, 0, 0 };
				if (gi < a.n && (!guarded || (uint32_t)sub * 16 < load_len(a, gi)))
					pre[it] = __builtin_nontemporal_load(
						reinterpret_cast<const u32x4 *>(pkt_ptr(a, gi) + sub * 16));
			}
		}
		plen = base + me < a.n ? load_len(a, base + me) : 0;
	};
	auto tile_sync = [&]() {
		if constexpr (WT)
			__builtin_amdgcn_wave_barrier();   // rows are this wave's own
		else
			__syncthreads();
	};
#ifndef XFG_EXP_NO_PREFETCH
	if (tile < ntiles)
		issue(tile);
#endif
	constexpr bool PROF = (V & 4) != 0;
	__shared__ uint32_t s_prof[PROF ? NPHASE : 1];
	Stamps st;
	if constexpr (PROF)
		st.init(s_prof);

	for (; tile < ntiles; tile += tstep) {
		const uint64_t base = tile * U;
#ifdef XFG_EXP_NO_PREFETCH
		issue(tile);
#endif
		if constexpr (PROF)
			st.mark(7);   // end-of-tile bookkeeping + loop
		// 1. stage the prefetched windows into LDS
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const int c = it * U + me;
			const int pk = c / CPP, sub = c % CPP;
			uint32_t *dst = &wrows[pk * ROWDW + sub * 4];
			dst[0] = pre[it].x;
			dst[1] = pre[it].y;
			dst[2] = pre[it].z;
			dst[3] = pre[it].w;
		}
		const uint32_t len = plen;
		if constexpr (PROF) {
			asm volatile("" ::"v"(len));
			st.mark(0);   // prefetched windows landed and written to LDS
		}
		tile_sync();
		if constexpr (PROF)
			st.mark(1);   // barrier
#ifndef XFG_EXP_NO_PREFETCH
		if (tile + tstep < ntiles)
			issue(tile + tstep);   // next tile's stream overlaps this tile's work
#endif
		if constexpr (PROF)
			st.mark(2);   // next tile issued

		// 2-4. parse, match, verdict
		const uint64_t gi = base + me;
		uint32_t act = A_NONE;
		uint32_t tag = CT_NONE;
		if (gi < a.n) {
			Pkt<W> p{ &wrows[me * ROWDW], pkt_ptr(a, gi), len };
			if (a.ablate & 4) {
				act = p.u8(0) & 1;
			} else {
				const Parsed r = parse<FEAT, W>(p);
				if constexpr (PROF) {
					asm volatile("" ::"v"(r.abort_at), "v"(r.k4a), "v"(r.l3));
					st.mark(3);   // parse
				}
				act = lookups<FEAT, (V & 1) != 0>(a, LazyKeys<Pkt<W>>{ p }, r, s_pbits, tag);
			}
			if constexpr (PROF) {
				asm volatile("" ::"v"(act), "v"(tag));
				st.mark(4);   // lookups
			}
			a.verdicts[gi] = (uint8_t)act;
		}
		if (a.ablate & 2)
			tag = CT_NONE;
		if constexpr ((FEAT & X_NOCNT) != 0)
			tag = CT_NONE;

		// counter bump: lanes of the wave hitting the same rule are merged
		// (one leader round), then summed in the LDS counter cache; a bump
		// the cache cannot take goes straight to a memory-side atomic
		{
			const unsigned long long pend = __ballot(tag != CT_NONE);
			if (pend) {
				const int leader = __ffsll((long long)pend) - 1;
				const uint32_t lt = __shfl(tag, leader);
				const bool mine = tag == lt;
				const unsigned long long same = __ballot(mine);
				if (lane == leader) {
					const uint32_t cnt = (uint32_t)__popcll(same);
					if (lt < a.dcnt)
						atomicAdd(&s_pcnt[lt], cnt);
					else if (!cache_hit(s_ctag, s_ccnt, lt, cnt)) {
						if (cnt > 1)
							atomicAdd(global_counter(a, lt), (unsigned long long)cnt);
						else
							cold_bump(a, s_pcnt, lt);
					}
				}
				if (mine)
					tag = CT_NONE;
			}
		}
		if (tag != CT_NONE && tag < a.dcnt)
			atomicAdd(&s_pcnt[tag], 1u);
		else if (tag != CT_NONE && !cache_hit(s_ctag, s_ccnt, tag, 1))
			cold_bump(a, s_pcnt, tag);

		// 5. per-action stats (xdp_stats_record_action), kept per lane
#ifdef XFG_EXP_NO_STATS
		if (0) {
#else
		if (act == A_ABORTED) {
#endif
			c_ab++;
			b_ab += len;
		} else if (act == A_DROP) {
			c_dr++;
			b_dr += len;
		} else if (act == A_PASS) {
			c_pa++;
			b_pa += len;
		}
		if constexpr (PROF)
			st.mark(5);   // counters, verdict, stats
		tile_sync();   // LDS window reuse
		if constexpr (PROF)
			st.mark(6);   // end barrier
	}
	if constexpr (PROF)
		st.store(a.prof);
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
	for (uint32_t i = tid; i < a.dcnt; i += TILE)
		if (s_pcnt[i])
			atomicAdd(global_counter(a, i), (unsigned long long)s_pcnt[i]);
}

// ---------------------------------------------------------------- streamed kernel
// The fixed-stride layout (stride >= 64, 16-byte aligned) with the header
// stream taken off the lookup waves.  A workgroup is four lookup waves (one
// packet per lane) plus one I/O wave:
//
//   I/O wave      global_load_lds (LDS-DMA, no VGPRs) of tile k+2's header
//                 windows and lengths into the buffer tile k has just
//                 released; then the counter atomics and the verdict store
//                 of tile k-1, read from LDS;
//   lookup waves  parse tile k from LDS, copy its keys to registers, release
//                 the buffer (barrier P), probe, and leave verdict bytes and
//                 cold counter bumps in LDS (barrier E).
//
// A wave's vector-memory counter completes in issue order, so a lookup wave
// that also streamed headers or issued atomics would wait for them at every
// probe; here its counter holds nothing but its own probes.
//
// Tile buffer: 256 windows of 64 bytes, 16-byte chunk c of packet p at chunk
// slot p*4 + (c ^ ((p >> 2) & 3)): every LDS-DMA instruction writes 1 KiB
// lane-linearly (the swizzle is applied to the source address), and a lane-
// per-packet read of any dword touches 16 distinct banks per 16 lanes.
constexpr int IO_THREADS = TILE + 64;
constexpr int SBUF_DW = TILE * 16;   // one tile buffer, dwords

__device__ __forceinline__ uint32_t lds_addr(const void *p)
{
	return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

// 16 bytes per lane from gsrc to LDS lds + 16 * lane (lds wave-uniform).  The
// compiler does not see this load: its completion is counted by hand.
__device__ __forceinline__ void glds16(const void *gsrc, uint32_t lds)
{
	unsigned keep;
	asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
		     "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
		     : "=&s"(keep)
		     : "v"(gsrc), "s"(lds)
		     : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm()
{
	asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// Wait until at most y (wave-uniform, <= 23) vector-memory operations of this
// wave are outstanding.
__device__ __forceinline__ void wait_vm_dyn(uint32_t y)
{
	switch (y) {
#define XFG_W(n) case n: wait_vm<n>(); break;
	XFG_W(1) XFG_W(2) XFG_W(3) XFG_W(4) XFG_W(5) XFG_W(6) XFG_W(7) XFG_W(8)
	XFG_W(9) XFG_W(10) XFG_W(11) XFG_W(12) XFG_W(13) XFG_W(14) XFG_W(15) XFG_W(16)
	XFG_W(17) XFG_W(18) XFG_W(19) XFG_W(20) XFG_W(21) XFG_W(22) XFG_W(23)
#undef XFG_W
	default: wait_vm<0>(); break;
	}
}

// Workgroup barrier that waits for this wave's LDS operations only (an LDS-
// DMA in flight stays in flight; __syncthreads() would drain it).
__device__ __forceinline__ void wg_barrier()
{
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Packet view over a swizzled tile buffer (same interface as Pkt<64>).
struct SPkt {
	const uint32_t *tb;   // tile buffer
	uint32_t base;        // 16 * p
	uint32_t xr;          // (p >> 2) & 3
	const uint8_t *g;
	uint32_t len;

	__device__ __forceinline__ uint32_t dw(uint32_t k) const
	{
		return tb[base + (((k >> 2) ^ xr) << 2) + (k & 3)];
	}
	__device__ __forceinline__ uint32_t u8(uint32_t o) const
	{
		if (o < 64)
			return (dw(o >> 2) >> (8 * (o & 3))) & 0xff;
		return gbyte(g, o);
	}
	__device__ __forceinline__ uint32_t u32(uint32_t o) const
	{
		if (o + 4 <= 64) {
			const uint32_t k = o >> 2;
			return __builtin_amdgcn_alignbyte(dw(k < 15 ? k + 1 : 15), dw(k), o & 3);
		}
		return gbyte(g, o) | (gbyte(g, o + 1) << 8) | (gbyte(g, o + 2) << 16) |
		       (gbyte(g, o + 3) << 24);
	}
	__device__ __forceinline__ uint32_t raw16(uint32_t o) const
	{
		if (o + 2 <= 64) {
			const uint32_t k = o >> 2;
			return __builtin_amdgcn_alignbyte(dw(k < 15 ? k + 1 : 15), dw(k), o & 3) & 0xffffu;
		}
		return gbyte(g, o) | (gbyte(g, o + 1) << 8);
	}
	__device__ __forceinline__ uint32_t be16(uint32_t o) const
	{
		uint32_t r = raw16(o);
		return ((r & 0xff) << 8) | (r >> 8);
	}
};

// Lookup keys copied to registers before the tile buffer is released; the
// NDISC target (rare) is read from the packet in HBM.
struct RegKeys {
	uint32_t e0, e1, e2;          // bytes 0..11: dst MAC, src MAC
	uint32_t d6[4], s6[4];        // IPv6 daddr, saddr
	const uint8_t *g;

	__device__ __forceinline__ void eth(uint32_t o, uint32_t &lo, uint32_t &hi) const
	{
		if (o == 0) {
			lo = e0;
			hi = e1 & 0xffff;
		} else {
			lo = __builtin_amdgcn_alignbyte(e2, e1, 2);
			hi = e2 >> 16;
		}
	}
	__device__ __forceinline__ void v6_dst(uint32_t, uint32_t (&k)[4]) const
	{
		k[0] = d6[0]; k[1] = d6[1]; k[2] = d6[2]; k[3] = d6[3];
	}
	__device__ __forceinline__ void v6_src(uint32_t, uint32_t (&k)[4]) const
	{
		k[0] = s6[0]; k[1] = s6[1]; k[2] = s6[2]; k[3] = s6[3];
	}
	__device__ __forceinline__ void nd_tgt(uint32_t o, uint32_t (&k)[4]) const
	{
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const uint8_t *q = g + o + 4 * i;
			k[i] = gbyte(q, 0) | (gbyte(q, 1) << 8) | (gbyte(q, 2) << 16) | (gbyte(q, 3) << 24);
		}
	}
};

template <uint32_t FEAT, int V>
__global__ __launch_bounds__(IO_THREADS) __attribute__((amdgpu_waves_per_eu(4))) void xfg_classify_stream_kernel(const xfg_kargs a)
{
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	__shared__ __attribute__((aligned(16))) uint32_t ring[2 * SBUF_DW];
	__shared__ __attribute__((aligned(16))) uint32_t s_lens[2][TILE];
	__shared__ uint32_t s_verd[2][TILE / 4];
	__shared__ uint32_t s_q[2][TILE];
	__shared__ uint32_t s_qn[2];
	__shared__ uint32_t s_pbits[PORTS ? 2048 : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ unsigned long long s_stats[6];

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	const bool io = tid >= TILE;
	if (tid < 6)
		s_stats[tid] = 0;
	if (tid < 2)
		s_qn[tid] = 0;
	for (int i = tid; i < CC_ENTRIES; i += IO_THREADS) {
		s_ctag[i] = CT_NONE;
		s_ccnt[i] = 0;
	}
	if constexpr (PORTS) {
		if (a.port_count)
			for (int i = tid; i < 2048; i += IO_THREADS)
				s_pbits[i] = a.port_tab ? a.port_tab[i] : a.port_bits[i];
	}

	const uint64_t ntiles = (a.n + TILE - 1) / TILE;
	const uint64_t G = gridDim.x;
	const uint64_t b = blockIdx.x;
	const uint64_t K = b < ntiles ? (ntiles - 1 - b) / G + 1 : 0;
	const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(lds_addr(ring));
	const uint32_t lens_lds = __builtin_amdgcn_readfirstlane(lds_addr(&s_lens[0][0]));
	const uint32_t esz = a.lens_u16 ? 2 : 4;

	// I/O wave: 17 LDS-DMA instructions per tile (16 window KiBs + lengths).
	// Instruction j, lane l loads packet 16j + l/4, chunk c(l) = (l & 3) ^
	// ((l >> 4) & 3) (the swizzle; independent of j), so a lane's source
	// address advances by 16 packets per instruction.
	const uint64_t io_off = (uint64_t)(lane >> 2) * a.stride + 16u * ((lane & 3) ^ ((lane >> 4) & 3));
	auto io_issue = [&](uint64_t k) {
		const uint64_t p0 = (b + k * G) * TILE;
		const uint32_t ldsb = ring_lds + (uint32_t)(k & 1) * (SBUF_DW * 4);
		const uint64_t step = 16ull * a.stride;
		const uint8_t *src = a.data + p0 * a.stride + io_off;
		if (p0 + TILE <= a.n) {
#pragma unroll
			for (int j = 0; j < 16; j++) {
				glds16(src, __builtin_amdgcn_readfirstlane(ldsb + j * 1024));
				src += step;
			}
		} else {
#pragma unroll
			for (int j = 0; j < 16; j++) {
				const uint64_t gi = p0 + 16 * j + (lane >> 2);
				glds16(gi < a.n ? src : a.data, __builtin_amdgcn_readfirstlane(ldsb + j * 1024));
				src += step;
			}
		}
		const uint64_t first = p0 + (uint64_t)lane * (16 / esz);
		const uint8_t *lsrc = static_cast<const uint8_t *>(a.lens);
		if (lane < (a.lens_u16 ? 32 : 64))
			glds16(first < a.n ? lsrc + first * esz : lsrc,
			       __builtin_amdgcn_readfirstlane(lens_lds + (uint32_t)(k & 1) * (TILE * 4)));
	};
	// I/O wave: counter atomics and verdict bytes of tile k (LDS parity
	// k & 1).  Returns a lower bound of the vector-memory instructions it
	// issued (exact on full tiles): one per 64 queued bumps, one store.
	auto io_flush = [&](uint64_t k) -> uint32_t {
		const uint32_t q = (uint32_t)(k & 1);
		const uint32_t nq = (a.ablate & 2) ? 0 : s_qn[q];
		uint32_t ops = 0;
#pragma unroll
		for (uint32_t i = 0; i < TILE / 64; i++) {
			if (i * 64 < nq) {   // wave-uniform: lane 0 is active below
				ops++;
				if (i * 64 + lane < nq)
					atomicAdd(global_counter(a, s_q[q][i * 64 + lane]), 1ull);
			}
		}
		const uint64_t p0 = (b + k * G) * TILE;
		const uint32_t v = s_verd[q][lane];
		if (p0 + TILE <= a.n && !((uintptr_t)a.verdicts & 3)) {
			reinterpret_cast<uint32_t *>(a.verdicts + p0)[lane] = v;
			ops++;
		} else {
#pragma unroll
			for (int i = 0; i < 4; i++)
				if (p0 + lane * 4 + i < a.n)
					a.verdicts[p0 + lane * 4 + i] = (uint8_t)(v >> (8 * i));
		}
		if (lane == 0)
			s_qn[q] = 0;
		return ops;
	};

	uint32_t c_ab = 0, c_dr = 0, c_pa = 0;
	unsigned long long b_ab = 0, b_dr = 0, b_pa = 0;

	if (io) {
		if (K > 0)
			io_issue(0);
		if (K > 1) {
			io_issue(1);
			wait_vm<17>();
		} else {
			wait_vm<0>();
		}
	}
	wg_barrier();   // S: LDS set up, tile 0 landed

	for (uint64_t k = 0; k < K; k++) {
		const uint32_t par = (uint32_t)(k & 1);
		if (io) {
			wg_barrier();   // P_k: tile k parsed, its buffer free
			// issue order F(k-1), I(k+2): wait for I(k+1) (issued a step
			// ago, older than both) and whatever preceded it
			uint32_t younger = k >= 1 ? io_flush(k - 1) : 0;
			if (k + 2 < K) {
				io_issue(k + 2);
				younger += 17;
			}
			if (k + 1 < K)
				wait_vm_dyn(younger);
			wg_barrier();   // E_k
			continue;
		}
		// lookup waves
		const uint64_t gi = (b + k * G) * TILE + tid;
		const bool valid = gi < a.n;
		const uint32_t len = a.lens_u16 ? reinterpret_cast<const uint16_t *>(s_lens[par])[tid]
						: s_lens[par][tid];
		const SPkt p{ ring + par * SBUF_DW, (uint32_t)tid * 16, ((uint32_t)tid >> 2) & 3,
			      a.data + gi * a.stride, len };
		Parsed r;
		RegKeys ks;
		ks.g = p.g;
		uint32_t act = A_NONE;
		if (valid) {
			if (a.ablate & 4) {
				act = p.u8(0) & 1;
			} else {
				r = parse<FEAT, 64>(p);
				if constexpr ((FEAT & F_ETH) != 0) {
					ks.e0 = p.dw(0);
					ks.e1 = p.dw(1);
					ks.e2 = p.dw(2);
				}
				if constexpr ((FEAT & F_IPV6) != 0) {
					if (r.l3 == 3) {
#pragma unroll
						for (int i = 0; i < 4; i++) {
							ks.s6[i] = p.u32(r.o6 + 8 + 4 * i);
							ks.d6[i] = p.u32(r.o6 + 24 + 4 * i);
						}
					}
				}
			}
		}
		wg_barrier();   // P_k
		uint32_t tag = CT_NONE;
		if (valid && !(a.ablate & 4))
			act = lookups<FEAT, (V & 1) != 0>(a, ks, r, s_pbits, tag);
		reinterpret_cast<uint8_t *>(s_verd[par])[tid] = (uint8_t)act;
		if (a.ablate & 2)
			tag = CT_NONE;

		// counter bump: wave leader merge, LDS counter cache, else queue the
		// bump for the I/O wave
		bool cold = false;
		{
			const unsigned long long pend = __ballot(tag != CT_NONE);
			if (pend) {
				const int leader = __ffsll((long long)pend) - 1;
				const uint32_t lt = __shfl(tag, leader);
				const bool mine = tag == lt;
				const unsigned long long same = __ballot(mine);
				const uint32_t cnt = (uint32_t)__popcll(same);
				if (lane == leader && !cache_hit(s_ctag, s_ccnt, lt, cnt)) {
					if (cnt == 1)
						cold = true;
					else
						atomicAdd(global_counter(a, lt), (unsigned long long)cnt);
				}
				if (mine && !cold)
					tag = CT_NONE;
			}
		}
		if (tag != CT_NONE && !cold) {
			if (cache_hit(s_ctag, s_ccnt, tag, 1))
				tag = CT_NONE;
			else
				cold = true;
		}
		{
			const unsigned long long m = __ballot(cold);
			if (m) {
				const int first = __ffsll((long long)m) - 1;
				uint32_t qb = 0;
				if (lane == first)
					qb = atomicAdd(&s_qn[par], (uint32_t)__popcll(m));
				qb = __shfl(qb, first);
				if (cold) {
					const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
						(uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
					s_q[par][qb + rank] = tag;
				}
			}
		}

		if (act == A_ABORTED) {
			c_ab++;
			b_ab += len;
		} else if (act == A_DROP) {
			c_dr++;
			b_dr += len;
		} else if (act == A_PASS) {
			c_pa++;
			b_pa += len;
		}
		wg_barrier();   // E_k
	}
	if (io && K > 0)
		io_flush(K - 1);

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
	for (int i = tid; i < CC_ENTRIES; i += IO_THREADS)
		if (s_ctag[i] != CT_NONE && s_ccnt[i])
			atomicAdd(global_counter(a, s_ctag[i]), (unsigned long long)s_ccnt[i]);
}

#include "xfg_pipe.hip"
#include "xfg_spec.hip"

template <uint32_t FEAT>
hipError_t launch_feat(const xfg_kargs &a, unsigned grid, hipStream_t s)
{
	if constexpr ((FEAT & F_IPV4) != 0) {
		if (a.pipe && a.spec) {
			const size_t dl = ((a.hlog ? a.hlog_parts : 0) + a.slog_parts) * 4;
			if (a.window <= 64) {
				if (a.dense)
					hipLaunchKernelGGL((xfg_classify_spec_kernel<FEAT, 64, true>), dim3(grid), dim3(TILE), dl, s, a);
				else
					hipLaunchKernelGGL((xfg_classify_spec_kernel<FEAT, 64, false>), dim3(grid), dim3(TILE), dl, s, a);
			} else {
				if (a.dense)
					hipLaunchKernelGGL((xfg_classify_spec_kernel<FEAT, 128, true>), dim3(grid), dim3(TILE), dl, s, a);
				else
					hipLaunchKernelGGL((xfg_classify_spec_kernel<FEAT, 128, false>), dim3(grid), dim3(TILE), dl, s, a);
			}
			hipError_t e = hipGetLastError();
			if (e != hipSuccess)
				return e;
			if (a.hlog) {
				hipLaunchKernelGGL(xfg_hlog_count_kernel, dim3(a.hlog_parts), dim3(HC_THREADS), 0, s, a, grid);
				if ((e = hipGetLastError()) != hipSuccess)
					return e;
			}
			if (!(a.ablate & 8))
				hipLaunchKernelGGL(xfg_spec_resolve_kernel, dim3(a.slog_parts), dim3(SR_THREADS), 0, s, a, grid);
			return hipGetLastError();
		}
	}
	if (a.pipe) {
		const size_t dl = a.hlog ? a.hlog_parts * 4 : 0;   // s_pcnt
		if (a.window <= 64) {
			if constexpr (FEAT == (F_TCP | F_UDP | F_IPV6 | F_IPV4 | F_ETH | F_DENY)) {
				if (a.dense && a.variant == 0x15) {   // diagnostics: 5 waves/SIMD
					hipLaunchKernelGGL((xfg_classify_pipe_kernel<FEAT, 64, true, 5>), dim3(grid), dim3(TILE), dl, s, a);
					return hipGetLastError();
				}
			}
			if (a.dense)
				hipLaunchKernelGGL((xfg_classify_pipe_kernel<FEAT, 64, true>), dim3(grid), dim3(TILE), dl, s, a);
			else
				hipLaunchKernelGGL((xfg_classify_pipe_kernel<FEAT, 64, false>), dim3(grid), dim3(TILE), dl, s, a);
		} else {
			if (a.dense)
				hipLaunchKernelGGL((xfg_classify_pipe_kernel<FEAT, 128, true>), dim3(grid), dim3(TILE), dl, s, a);
			else
				hipLaunchKernelGGL((xfg_classify_pipe_kernel<FEAT, 128, false>), dim3(grid), dim3(TILE), dl, s, a);
		}
		const hipError_t e = hipGetLastError();
		if (e != hipSuccess || !a.hlog)
			return e;
		hipLaunchKernelGGL(xfg_hlog_count_kernel, dim3(a.hlog_parts), dim3(HC_THREADS), 0, s, a, grid);
		return hipGetLastError();
	}
	const size_t dl = a.hlog ? a.hlog_parts * 4 : a.dcnt * 4;   // classic kernel's s_pcnt
	if (a.streamed) {
		hipLaunchKernelGGL((xfg_classify_stream_kernel<FEAT, 0>), dim3(grid), dim3(IO_THREADS), 0, s, a);
		return hipGetLastError();
	} else if (a.window <= 64) {
		// build variants of the headline program (diagnostics: XFG_VARIANT)
		if constexpr (FEAT == (F_TCP | F_UDP | F_IPV6 | F_IPV4 | F_ETH | F_DENY)) {
			switch (a.variant) {
			case 1:
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 1>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
			case 2:
				if (a.dense)
					hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 2, true>), dim3(grid), dim3(TILE), 0, s, a);
				else
					hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 2>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
			case 3:
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 3>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
			case 4:
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 4>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
			case 8:
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 8>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
			case 12:
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 12>), dim3(grid), dim3(TILE), 0, s, a);
				return hipGetLastError();
#define XFG_XV(x)                                                                              \
			case x:                                                                \
				hipLaunchKernelGGL((xfg_classify_kernel<FEAT | x, 64, 0>), dim3(grid), \
						   dim3(TILE), 0, s, a);                       \
				return hipGetLastError();
			XFG_XV(0x100) XFG_XV(0x200) XFG_XV(0x400) XFG_XV(0x800) XFG_XV(0xF00)
#undef XFG_XV
			default:
				break;
			}
		}
		if (a.dense)
			hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 0, true>), dim3(grid), dim3(TILE), dl, s, a);
		else
			hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64, 0>), dim3(grid), dim3(TILE), dl, s, a);
	} else {
		hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 128, 0>), dim3(grid), dim3(TILE), dl, s, a);
	}
	hipError_t e = hipGetLastError();
	if (e != hipSuccess || !a.hlog)
		return e;
	hipLaunchKernelGGL(xfg_hlog_count_kernel, dim3(a.hlog_parts), dim3(HC_THREADS), 0, s, a, grid);
	return hipGetLastError();
}

}  // namespace

// Feature words of the ten programs (xdp-filter/xdpfilt_*.c + :313-315).
#define XFG_ALL (F_TCP | F_UDP | F_IPV6 | F_IPV4 | F_ETH)
#define XFG_ALLOW (1u << 5)

extern "C" int xfg_launch_classify(uint32_t prog_features, const struct xfg_kargs *a,
				   unsigned grid, void *stream)
{
	hipStream_t s = static_cast<hipStream_t>(stream);
	hipError_t e;
	switch (prog_features) {
	case F_UDP | F_DENY:              e = launch_feat<F_UDP | F_DENY>(*a, grid, s); break;
	case F_TCP | F_DENY:              e = launch_feat<F_TCP | F_DENY>(*a, grid, s); break;
	case F_IPV4 | F_IPV6 | F_DENY:    e = launch_feat<F_IPV4 | F_IPV6 | F_DENY>(*a, grid, s); break;
	case F_ETH | F_DENY:              e = launch_feat<F_ETH | F_DENY>(*a, grid, s); break;
	case XFG_ALL | F_DENY:            e = launch_feat<XFG_ALL | F_DENY>(*a, grid, s); break;
	case F_UDP | XFG_ALLOW:           e = launch_feat<F_UDP | XFG_ALLOW>(*a, grid, s); break;
	case F_TCP | XFG_ALLOW:           e = launch_feat<F_TCP | XFG_ALLOW>(*a, grid, s); break;
	case F_IPV4 | F_IPV6 | XFG_ALLOW: e = launch_feat<F_IPV4 | F_IPV6 | XFG_ALLOW>(*a, grid, s); break;
	case F_ETH | XFG_ALLOW:           e = launch_feat<F_ETH | XFG_ALLOW>(*a, grid, s); break;
	case XFG_ALL | XFG_ALLOW:         e = launch_feat<XFG_ALL | XFG_ALLOW>(*a, grid, s); break;
	default:
		return -22; /* -EINVAL */
	}
	return e == hipSuccess ? 0 : -(int)e - 1000;
}

// Resident workgroups per CU of the classify kernel a launch would use
// (grid sizing: one persistent wave of workgroups); window 1 = the streamed
// kernel, 2 / 3 = the pipelined kernel with a 64 / 128-byte window.
template <uint32_t FEAT>
static int occupancy_feat(uint32_t window)
{
	int n = 0;
	if constexpr ((FEAT & F_IPV4) != 0) {
		if (window == 4) {
			hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
				&n, xfg_classify_spec_kernel<FEAT, 64, true>, TILE, 1024);
			return e == hipSuccess && n > 0 ? n : 4;
		}
	}
	hipError_t e = window == 2 || window == 4
		? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_pipe_kernel<FEAT, 64, true>, TILE, 0)
		: window == 3
		? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_pipe_kernel<FEAT, 128, false>, TILE, 0)
		: window == 1
		? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_stream_kernel<FEAT, 0>, IO_THREADS, 0)
		: window <= 64
		? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_kernel<FEAT, 64, 0, true>, TILE, 0)
		: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_kernel<FEAT, 128, 0>, TILE, 0);
	return e == hipSuccess && n > 0 ? n : 4;
}

extern "C" int xfg_classify_occupancy(uint32_t prog_features, uint32_t window)
{
	switch (prog_features) {
	case F_UDP | F_DENY:              return occupancy_feat<F_UDP | F_DENY>(window);
	case F_TCP | F_DENY:              return occupancy_feat<F_TCP | F_DENY>(window);
	case F_IPV4 | F_IPV6 | F_DENY:    return occupancy_feat<F_IPV4 | F_IPV6 | F_DENY>(window);
	case F_ETH | F_DENY:              return occupancy_feat<F_ETH | F_DENY>(window);
	case XFG_ALL | F_DENY:            return occupancy_feat<XFG_ALL | F_DENY>(window);
	case F_UDP | XFG_ALLOW:           return occupancy_feat<F_UDP | XFG_ALLOW>(window);
	case F_TCP | XFG_ALLOW:           return occupancy_feat<F_TCP | XFG_ALLOW>(window);
	case F_IPV4 | F_IPV6 | XFG_ALLOW: return occupancy_feat<F_IPV4 | F_IPV6 | XFG_ALLOW>(window);
	case F_ETH | XFG_ALLOW:           return occupancy_feat<F_ETH | XFG_ALLOW>(window);
	case XFG_ALL | XFG_ALLOW:         return occupancy_feat<XFG_ALL | XFG_ALLOW>(window);
	default:                          return 4;
	}
}

// Streaming-read probe: the achievable HBM read rate on this device, used by
// bench.py next to the 8 TB/s spec peak.  Reads n16 16-byte words, writes one
// word per workgroup so the loads cannot be elided.
__global__ __launch_bounds__(256) void xfg_stream_read_kernel(const u32x4 *__restrict__ src,
							      uint64_t n16, u32x4 *__restrict__ sink)
{
	u32x4 acc = { 0, 0, 0, 0 };
	for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull)
		acc ^= __builtin_nontemporal_load(src + i);
	if ((acc.x | acc.y | acc.z | acc.w) == 0x9e3779b9u)   // practically never
		sink[blockIdx.x] = acc;
}

extern "C" int xfg_launch_stream_read(const void *src, uint64_t bytes, void *sink,
				      unsigned grid, void *stream)
{
	hipLaunchKernelGGL(xfg_stream_read_kernel, dim3(grid), dim3(256), 0,
			   static_cast<hipStream_t>(stream), static_cast<const u32x4 *>(src),
			   bytes / 16, static_cast<u32x4 *>(sink));
	return hipGetLastError() == hipSuccess ? 0 : -5;
}

// ---------------------------------------------------------------- verdict compaction
// The indices of the packets whose verdict equals `action`, in packet order
// (the PASS list a forwarding stage walks: the reference chains only on
// XDP_PASS, xdp-filter/xdpfilt_prog.h:209-212).  One pass over the verdict
// bytes: a workgroup takes tiles of CT_TILE verdicts in ticket order; each
// lane counts its 16 bytes, wave prefix sums (shuffles) and an LDS step give
// the workgroup's offsets, and a decoupled look-back over the earlier tiles'
// published {flag, sum} words gives the tile's base.  A status word packs
// flag (bits 62-63: 1 = tile aggregate, 2 = inclusive prefix) and value, so
// one 8-byte agent-scope atomic carries both.
namespace {
constexpr int CT_LANES = 256;
constexpr int CT_TILE = CT_LANES * 16;
constexpr unsigned long long CT_AGG = 1ull << 62, CT_INC = 2ull << 62, CT_VAL = (1ull << 62) - 1;

__device__ __forceinline__ uint32_t count_eq(uint32_t w, uint32_t act4)
{
	const uint32_t x = w ^ act4;   // a zero byte where the verdict matches
	const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
	return __builtin_popcount(z);
}
}  // namespace

__global__ __launch_bounds__(CT_LANES) void xfg_compact_kernel(
	const uint8_t *__restrict__ verdicts, uint64_t n, uint32_t action,
	uint32_t *__restrict__ idx, unsigned long long *__restrict__ count,
	unsigned long long *status, uint32_t *ticket, uint64_t ntiles)
{
	__shared__ uint32_t s_wave[CT_LANES / 64];
	__shared__ uint64_t s_tile, s_base;
	const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
	const uint32_t act4 = action * 0x01010101u;
	for (;;) {
		if (tid == 0)
			s_tile = atomicAdd(ticket, 1u);
		__syncthreads();
		const uint64_t t = s_tile;
		if (t >= ntiles)
			break;
		const uint64_t first = t * CT_TILE + (uint64_t)tid * 16;
		uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
		uint32_t valid = 0;   // bytes of this lane inside the batch
		if (first + 16 <= n) {
			const u32x4 v = __builtin_nontemporal_load(
				reinterpret_cast<const u32x4 *>(verdicts + first));
			w0 = v.x;
			w1 = v.y;
			w2 = v.z;
			w3 = v.w;
			valid = 16;
		} else if (first < n) {
			valid = (uint32_t)(n - first);
		}
		auto byte_at = [&](uint32_t k) -> uint32_t {
			if (valid < 16)   // the batch's last lane: read the tail bytewise
				return verdicts[first + k];
			const uint32_t w = k < 4 ? w0 : k < 8 ? w1 : k < 12 ? w2 : w3;
			return (w >> (8 * (k & 3))) & 0xff;
		};
		uint32_t mine = 0;
		if (valid == 16) {
			mine = count_eq(w0, act4) + count_eq(w1, act4) + count_eq(w2, act4) +
			       count_eq(w3, act4);
		} else {
			for (uint32_t k = 0; k < valid; k++)
				mine += byte_at(k) == action;
		}
		// wave inclusive scan, then the workgroup's
		uint32_t x = mine;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t y = __shfl_up(x, o);
			if (lane >= o)
				x += y;
		}
		if (lane == 63)
			s_wave[wave] = x;
		__syncthreads();
		uint32_t before = x - mine, agg = 0;
#pragma unroll
		for (int k = 0; k < CT_LANES / 64; k++) {
			before += k < wave ? s_wave[k] : 0;
			agg += s_wave[k];
		}
		// decoupled look-back (one lane): publish the aggregate, walk back
		if (tid == 0) {
			unsigned long long base = 0;
			if (t == 0) {
				__hip_atomic_store(&status[0], CT_INC | agg, __ATOMIC_RELAXED,
						   __HIP_MEMORY_SCOPE_AGENT);
			} else {
				__hip_atomic_store(&status[t], CT_AGG | agg, __ATOMIC_RELAXED,
						   __HIP_MEMORY_SCOPE_AGENT);
				for (uint64_t p = t - 1;;) {
					const unsigned long long w = __hip_atomic_load(
						&status[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
					if (w & CT_INC) {
						base += w & CT_VAL;
						break;
					}
					if (w & CT_AGG) {
						base += w & CT_VAL;
						p--;   // tile 0 always publishes CT_INC
						continue;
					}
					__builtin_amdgcn_s_sleep(1);   // predecessor still counting
				}
				__hip_atomic_store(&status[t], CT_INC | (base + agg), __ATOMIC_RELAXED,
						   __HIP_MEMORY_SCOPE_AGENT);
			}
			s_base = base;
			if (t == ntiles - 1)
				*count = base + agg;
		}
		__syncthreads();
		uint64_t pos = s_base + before;
		if (mine) {
			for (uint32_t k = 0; k < valid; k++)
				if (byte_at(k) == action)
					idx[pos++] = (uint32_t)(first + k);
		}
		__syncthreads();   // s_tile / s_wave reuse
	}
}

extern "C" int xfg_launch_compact(const uint8_t *verdicts, uint64_t n, uint32_t action,
				  uint32_t *idx, unsigned long long *count,
				  unsigned long long *status, uint32_t *ticket, unsigned grid,
				  void *stream)
{
	hipStream_t s = static_cast<hipStream_t>(stream);
	const uint64_t ntiles = (n + CT_TILE - 1) / CT_TILE;
	if (hipMemsetAsync(status, 0, ntiles * 8, s) != hipSuccess ||
	    hipMemsetAsync(ticket, 0, 4, s) != hipSuccess)
		return -5;
	if (!n)
		return hipMemsetAsync(count, 0, 8, s) == hipSuccess ? 0 : -5;
	hipLaunchKernelGGL(xfg_compact_kernel, dim3(grid), dim3(CT_LANES), 0, s, verdicts, n, action,
			   idx, count, status, ticket, ntiles);
	return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" uint64_t xfg_compact_tiles(uint64_t n)
{
	return (n + CT_TILE - 1) / CT_TILE;
}
