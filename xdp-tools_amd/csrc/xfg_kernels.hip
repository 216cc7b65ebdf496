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
#include <type_traits>

#include "xfg_layout.h"

// Split build (xdp-tools_amd/Makefile): the same file compiled as several
// translation units in parallel, XFG_PART_MASK choosing the programs whose
// kernels one instantiates (bit i: program i of xfg_lc_<i> below) and
// XFG_PART_COMMON the unit with the shared kernels and the C ABI dispatch.
// Unset (tools/abbuild.sh, one unit): every program, the shared part too.
#ifndef XFG_PART_MASK
#define XFG_PART_MASK 0x3ffu
#define XFG_PART_COMMON 1
#endif
#ifndef XFG_PART_COMMON
#define XFG_PART_COMMON 0
#endif

namespace {

constexpr uint32_t F_TCP = 1u << 0;
constexpr uint32_t F_UDP = 1u << 1;
constexpr uint32_t F_IPV6 = 1u << 2;
constexpr uint32_t F_IPV4 = 1u << 3;
constexpr uint32_t F_ETH = 1u << 4;
constexpr uint32_t F_DENY = 1u << 6;

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
	// header-window batch (kargs.hwin): the slot holds only the window, so
	// a read past it is not made -- it flags the packet here (returns 0)
	uint32_t *oob = nullptr;

	// Byte o (caller has checked o < len, as the reference does).
	__device__ __forceinline__ uint32_t u8(uint32_t o) const
	{
		if (o < (uint32_t)W)
			return reinterpret_cast<const uint8_t *>(row)[o];
		if (oob) {
			*oob = 1;
			return 0;
		}
		return gbyte(g, o);
	}
	// Little-endian 32-bit load of bytes o..o+3 (o+3 < len).
	__device__ __forceinline__ uint32_t u32(uint32_t o) const
	{
		if (o + 4 <= (uint32_t)W) {
			uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, o & 3);
		}
		if (oob) {
			*oob = 1;
			return 0;
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
		if (oob) {
			*oob = 1;
			return 0;
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
	const uint32_t w = t.bloom[xfg_bloom_word(h, t.bloom_words)];
	const uint32_t m = xfg_bloom_mask(h);
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
// (tag bit of a QT slot in the quotient-index kernel: canonical counter
// identities stay below 2^30)
constexpr uint32_t CT_QTAG = 0x80000000u;

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

// Counter of hit-log entry g: a counter identity, or with the quotient index
// (kargs.qt) a QT slot, whose canonical identity qt_trans holds.
__device__ __forceinline__ unsigned long long *log_counter(const xfg_kargs &a, uint32_t g)
{
	return global_counter(a, a.qt ? a.qt_trans[g] : g);
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

// s_ports: the workgroup's LDS copy of the ruled ports -- the open-addressed
// table (kargs.port_tab, at most XFG_PORT_TAB_MAX ports) or, with more, the
// 65536-entry nibble map of every port's flags (kargs.port_nib).  Only the
// four flag bits CHECK_MAP can test (SRC|DST|TCP|UDP) are kept.
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
		f = (s_ports[key >> 3] >> ((key & 7) * 4)) & 15;
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
	if constexpr ((FEAT & F_IPV6) != 0) {
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
	if constexpr ((FEAT & F_IPV6) != 0) {
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
	if constexpr ((FEAT & (F_UDP | F_TCP)) != 0) {
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

// Per-workgroup counter cache in LDS: open addressing on the counter
// identity, CC_PROBES slots from its home.  A rule hit by many packets (a
// hot port, an attacked address, one of a handful of MAC rules) is summed
// here and reaches memory once per workgroup; when its probe run is owned by
// other counters the bump goes straight to its global atomic.
constexpr int CC_ENTRIES = 512, CC_PROBES = 4;

// Returns true when the LDS cache absorbed the n bumps of counter `tag`.
__device__ __forceinline__ bool cache_hit(uint32_t *s_ctag, uint32_t *s_ccnt, uint32_t tag,
					  uint32_t n)
{
	uint32_t e = (tag * 0x9E3779B1u) >> 23;   // 9 bits
	for (int q = 0; q < CC_PROBES; q++) {
		uint32_t t = s_ctag[e];
		if (t == CT_NONE) {
			t = atomicCAS(&s_ctag[e], CT_NONE, tag);
			if (t == CT_NONE)
				t = tag;
		}
		if (t == tag) {
			atomicAdd(&s_ccnt[e], n);
			return true;
		}
		e = (e + 1) & (CC_ENTRIES - 1);
	}
	return false;
}


// Word w of packet i's AF_XDP descriptor (ring index wraps with desc_mask).
__device__ __forceinline__ uint64_t desc_word(const xfg_kargs &a, uint64_t i, int w)
{
	return reinterpret_cast<const __attribute__((address_space(1))) uint64_t *>(
		reinterpret_cast<uintptr_t>(a.descs))[2ull * ((a.desc_first + (uint32_t)i) & a.desc_mask) + w];
}

// Length of packet i in the pipelined kernels' layout (no descriptors).
// (through the global address space: a FLAT load would also count against
// the LDS counter, and the loops' LDS waits would wait for it)
__device__ __forceinline__ uint32_t load_len_fixed(const xfg_kargs &a, uint32_t i)
{
	const uintptr_t p = reinterpret_cast<uintptr_t>(a.lens);
	return a.lens_u16 ? reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(p)[i]
			  : reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(p)[i];
}

__device__ __forceinline__ uint32_t load_len(const xfg_kargs &a, uint64_t i)
{
	if (a.descs)
		return (uint32_t)desc_word(a, i, 1);   // xdp_desc.len (low half, little-endian)
	const uintptr_t p = reinterpret_cast<uintptr_t>(a.lens);
	return a.lens_u16 ? reinterpret_cast<const __attribute__((address_space(1))) uint16_t *>(p)[i]
			  : reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>(p)[i];
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

// A 32-bit atomic add through the global address space (atomicAdd on a
// generic pointer may become a FLAT atomic, which counts against the LDS
// counter as well: the loop's LDS waits would wait for it)
__device__ __forceinline__ void gatomic_add32(uint32_t *p, uint32_t v)
{
	__hip_atomic_fetch_add(reinterpret_cast<__attribute__((address_space(1))) uint32_t *>((uintptr_t)p), v,
			       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- counters and stats
// Per-workgroup counter state.  A hit adds 1 << COUNTER_SHIFT to the first
// matching rule's value (xdp-filter/xdpfilt_prog.h:60-61), i.e. 1 to its
// `hits` word.  Per-CPU values made that a plain add in the reference; here
// many waves add to one table, so a bump goes, in order of preference, to
//   * a direct LDS counter (rule sets of at most XFG_DCNT_MAX counters),
//   * the LDS counter cache (lanes of a wave on the same rule are merged
//     first; a hot rule, e.g. a ruled port, is summed here and reaches
//     memory once per workgroup),
//   * a memory-side atomic.
// The pipelined kernels send their hash-map hits to the hit log instead
// (HitLog below): random memory-side atomics are what bounds a 1M-rule
// table's millions of cold hits per launch.
struct Counters {
	uint32_t *ctag, *ccnt;   // LDS counter cache, CC_ENTRIES each
	uint32_t *dcnt;          // LDS direct counters, a.dcnt of them

	__device__ __forceinline__ void init(const xfg_kargs &a, int tid, int nthr)
	{
		for (int i = tid; i < CC_ENTRIES; i += nthr) {
			ctag[i] = CT_NONE;
			ccnt[i] = 0;
		}
		for (uint32_t i = tid; i < a.dcnt; i += nthr)
			dcnt[i] = 0;
	}
	// Bump the counter of every lane's tag (CT_NONE: none).  Whole wave.
	__device__ __forceinline__ void bump(const xfg_kargs &a, uint32_t tag, int lane)
	{
		const unsigned long long pend = __ballot(tag != CT_NONE);
		if (!pend)
			return;
		const int leader = __ffsll((long long)pend) - 1;
		const uint32_t lt = __shfl(tag, leader);
		const bool mine = tag == lt;
		const unsigned long long same = __ballot(mine);
		if (lane == leader) {
			const uint32_t cnt = (uint32_t)__popcll(same);
			if (lt < a.dcnt)
				atomicAdd(&dcnt[lt], cnt);
			else if (!cache_hit(ctag, ccnt, lt, cnt))
				atomicAdd(global_counter(a, lt), (unsigned long long)cnt);
		}
		if (mine)
			tag = CT_NONE;
		if (tag != CT_NONE) {
			if (tag < a.dcnt)
				atomicAdd(&dcnt[tag], 1u);
			else if (!cache_hit(ctag, ccnt, tag, 1))
				atomicAdd(global_counter(a, tag), 1ull);
		}
	}
	// Workgroup end (after a barrier): LDS sums to memory (a tag with
	// CT_QTAG is a QT slot: its QT-order count, xfg_pipeq_kernel).
	__device__ __forceinline__ void flush(const xfg_kargs &a, int tid, int nthr)
	{
		for (int i = tid; i < CC_ENTRIES; i += nthr)
			if (ctag[i] != CT_NONE && ccnt[i]) {
				if (ctag[i] & CT_QTAG)
					gatomic_add32(a.qt_hitx + (ctag[i] & ~CT_QTAG), ccnt[i]);
				else
					atomicAdd(global_counter(a, ctag[i]), (unsigned long long)ccnt[i]);
			}
		for (uint32_t i = tid; i < a.dcnt; i += nthr)
			if (dcnt[i])
				atomicAdd(global_counter(a, i), (unsigned long long)dcnt[i]);
	}
};

// ---------------------------------------------------------------- hit log
// The pipelined kernels' counting of hash-map hits (kargs.tlog != NULL):
//   1. each wave appends its hits' counter identities to its own region,
//      one coalesced store per tile (log_append);
//   2. at its end each workgroup counting-sorts its entries by partition
//      (g >> 4) % XFG_LOG_PARTS -- 16 consecutive counters, one 128-byte
//      line of u64, per chunk; chunks dealt round-robin -- and writes them,
//      as 16-bit indices local to the partition (log_local), into its OWN
//      slice of every partition's buffer: slice (partition p, workgroup b)
//      at pbuf[(p * pslices + b) * pcap], its fill written (not reserved,
//      no atomics) to pfill[p * pslices + b] (log_partition);
//   3. xfg_log_count_kernel, one workgroup per partition, reads the
//      partition's slices one after another into an LDS histogram and adds
//      each count to its counter with a plain read-modify-write (it owns
//      those counters).
// Every hit costs a 4-byte coalesced store and two L2-resident passes
// instead of a random memory-side atomic.  Entries past a slice's pcap go
// straight to their counter with an atomic (log_counter; exact either way).
__device__ __forceinline__ uint32_t log_part(uint32_t g) { return (g >> 4) & (XFG_LOG_PARTS - 1); }
__device__ __forceinline__ uint32_t log_local(uint32_t g) { return ((g >> 12) << 4) | (g & 15); }

// Set bits of the wave mask m below this lane (mbcnt: no lane mask register).
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Global-address-space accesses to buffers the pipelined kernels use in
// their loops.  Through a generic pointer the compiler emits FLAT
// instructions, which also count against the LDS counter: every later
// lgkmcnt(0) of the iteration (each LDS read the parse waits for) then waits
// for the store's write acknowledgement as well -- a memory round trip per
// iteration.  A global store counts only against vmcnt, where the next
// iteration's one wait covers it.
__device__ __forceinline__ void gst32(uint32_t *p, uint32_t v)
{
	*reinterpret_cast<__attribute__((address_space(1))) uint32_t *>((uintptr_t)p) = v;
}
__device__ __forceinline__ uint32_t gld32(const uint32_t *p)
{
	return *reinterpret_cast<const __attribute__((address_space(1))) uint32_t *>((uintptr_t)p);
}

__device__ __forceinline__ void log_append(uint32_t *region, uint32_t &cnt, uint32_t tag, int lane)
{
	const unsigned long long m = __ballot(tag != CT_NONE);
	if (m) {
		if (tag != CT_NONE)
			gst32(region + cnt + lanes_below(m), tag);
		cnt += (uint32_t)__popcll(m);
	}
}

// Workgroup end: the NW wave regions (counts in s_n) into the partition
// buffers.  s_hist: the workgroup's per-partition entry counts (LDS; built
// during the loop by the appenders, or here when null).  One reservation
// per partition in its buffer (pfill), then chunks of LOG_CHUNK entries
// counting-sorted by partition in LDS and written out as per-partition runs
// (consecutive lanes, consecutive addresses).  s: LDS scratch of
// 4 * XFG_LOG_PARTS + LOG_CHUNK words.  Whole workgroup, after a barrier.
#ifndef XFG_LOG_CHUNK
#define XFG_LOG_CHUNK 8192
#endif
#ifndef XFG_PART_LDSBAR
#define XFG_PART_LDSBAR 1
#endif

// A workgroup barrier for LDS hand-offs only: the waves' LDS operations are
// complete (lgkmcnt(0)) but their global loads and stores stay in flight
// (__syncthreads() also drains vmcnt, which would serialise the partition's
// chunk prefetch and write-out on every barrier).  The memory clobber keeps
// the compiler from moving memory accesses across it.
__device__ __forceinline__ void lds_barrier()
{
#if XFG_PART_LDSBAR
	asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
	__syncthreads();
#endif
}
constexpr uint32_t LOG_CHUNK = XFG_LOG_CHUNK;
constexpr uint32_t LOG_SCRATCH = 4 * XFG_LOG_PARTS + LOG_CHUNK;   // words

template <int NW>
__device__ __forceinline__ void log_partition(const xfg_kargs &a, const uint32_t *s_n,
					      const uint32_t *s_hist, uint32_t *s, int tid)
{
	// (a chunk: whole entries per thread, at most LOG_CHUNK)
	constexpr int NTH = 64 * NW, K = LOG_CHUNK / NTH;
	constexpr uint32_t CH = K * NTH;
	static_assert(K >= 1, "chunk: at least one entry per thread");
	const int nthr = NTH;
	uint32_t *const s_h = s;                         // histogram, then the chunk's counts
	uint32_t *const s_cur = s + 2 * XFG_LOG_PARTS;   // entries written per partition
	uint32_t *const s_off = s + 3 * XFG_LOG_PARTS;   // the chunk's run starts
	uint32_t *const s_srt = s + 4 * XFG_LOG_PARTS;   // the chunk, sorted
	const uint64_t r0 = (uint64_t)blockIdx.x * NW * a.defer_cap;
	// this workgroup's slice of every partition: position 0, its count
	// stored for the count kernel (entries past pcap spill to atomics)
	const uint64_t slice0 = (uint64_t)(blockIdx.x + a.pslice0) * a.pcap;
	const uint64_t pstep = (uint64_t)a.pslices * a.pcap;
	for (int i = tid; i < (int)XFG_LOG_PARTS; i += nthr) {
		s_h[i] = 0;
		s_cur[i] = 0;
	}
	if (!s_hist) {
		__syncthreads();
		for (int w = 0; w < NW; w++) {
			const uint32_t *reg = a.tlog + r0 + (uint64_t)w * a.defer_cap;
			for (uint32_t e = tid; e < s_n[w]; e += nthr)
				atomicAdd(&s_h[log_part(reg[e])], 1u);
		}
	}
	__syncthreads();
	for (int p = tid; p < (int)XFG_LOG_PARTS; p += nthr) {
		gst32(a.pfill + (uint64_t)p * a.pslices + a.pslice0 + blockIdx.x, s_hist ? s_hist[p] : s_h[p]);
		s_h[p] = 0;
	}
	__syncthreads();
#ifdef XFG_DIAG
	if (a.diag & 1024)   // diagnostics: stop after the reservations (counts wrong)
		return;
#endif
	// the NW regions as one sequence (entry e of region w at pre[w] + e),
	// cut into chunks of CH: runs of about CH / 256 entries
	uint32_t pre[NW + 1];
	pre[0] = 0;
#pragma unroll
	for (int w = 0; w < NW; w++)
		pre[w + 1] = pre[w] + s_n[w];
	const uint32_t total = pre[NW];
	const int lane = tid & 63;
	// a chunk's entries; the next chunk's are in flight during the current
	// chunk's write-out
	uint32_t g[K], rk[K];
	auto fetch = [&](uint32_t c0) {
#pragma unroll
		for (int j = 0; j < K; j++) {
			const uint32_t e = c0 + tid + j * NTH;
			g[j] = CT_NONE;
			if (e < total) {
				int w = 0;
#pragma unroll
				for (int q = 1; q < NW; q++)
					w += e >= pre[q];
				g[j] = gld32(a.tlog + r0 + (uint64_t)w * a.defer_cap + (e - pre[w]));
			}
		}
	};
	if (total)
		fetch(0);
	for (uint32_t c0 = 0; c0 < total; c0 += CH) {
		const uint32_t cn = min(CH, total - c0);
		// rank each entry within its partition
#pragma unroll
		for (int j = 0; j < K; j++)
			rk[j] = g[j] != CT_NONE ? atomicAdd(&s_h[log_part(g[j])], 1u) : 0u;
		lds_barrier();
		// run starts: exclusive scan of the counts (one wave)
		if (tid < 64) {
			uint32_t v[XFG_LOG_PARTS / 64], sum = 0;
#pragma unroll
			for (int q = 0; q < (int)(XFG_LOG_PARTS / 64); q++) {
				v[q] = s_h[lane * (XFG_LOG_PARTS / 64) + q];
				sum += v[q];
			}
			uint32_t inc = sum;
#pragma unroll
			for (int o = 1; o < 64; o <<= 1) {
				const uint32_t y = __shfl_up(inc, o);
				if (lane >= o)
					inc += y;
			}
			uint32_t run = inc - sum;
#pragma unroll
			for (int q = 0; q < (int)(XFG_LOG_PARTS / 64); q++) {
				s_off[lane * (XFG_LOG_PARTS / 64) + q] = run;
				run += v[q];
			}
		}
		lds_barrier();
#pragma unroll
		for (int j = 0; j < K; j++)
			if (g[j] != CT_NONE)
				s_srt[s_off[log_part(g[j])] + rk[j]] = g[j];
		if (c0 + CH < total)
			fetch(c0 + CH);
		lds_barrier();
		for (uint32_t t = tid; t < cn; t += nthr) {
			const uint32_t x = s_srt[t], p = log_part(x);
			const uint32_t pos = s_cur[p] + (t - s_off[p]);
			if (a.diag & 256)   // diagnostics build only: no write-out
				continue;
			if (pos < a.pcap && a.pwide)   // (the partition is implied: the local index)
				*reinterpret_cast<__attribute__((address_space(1))) uint32_t *>(
					(uintptr_t)(reinterpret_cast<uint32_t *>(a.pbuf) + p * pstep + slice0 + pos)) = log_local(x);
			else if (pos < a.pcap)
				*reinterpret_cast<__attribute__((address_space(1))) uint16_t *>(
					(uintptr_t)(a.pbuf + p * pstep + slice0 + pos)) = (uint16_t)log_local(x);
			else
				atomicAdd(log_counter(a, x), 1ull);
		}
		lds_barrier();
		for (int p = tid; p < (int)XFG_LOG_PARTS; p += nthr) {
			s_cur[p] += s_h[p];
			s_h[p] = 0;
		}
		lds_barrier();
	}
}

// Per-action {packets, bytes} (xdp_stats_record_action,
// headers/xdp/xdp_stats_kern.h:29-48), summed per lane, then per wave, per
// workgroup (LDS) and once per workgroup into the device's stats.
struct LaneStats {
	uint32_t c0 = 0, c1 = 0, c2 = 0;
	unsigned long long b0 = 0, b1 = 0, b2 = 0;
	// (selects, not a branch on act: an indexed update would go to scratch)
	__device__ __forceinline__ void add(uint32_t act, uint32_t len)
	{
		c0 += act == A_ABORTED;
		c1 += act == A_DROP;
		c2 += act == A_PASS;
		b0 += act == A_ABORTED ? len : 0u;
		b1 += act == A_DROP ? len : 0u;
		b2 += act == A_PASS ? len : 0u;
	}
	// to s_stats[6] (LDS, zeroed before), by every wave
	__device__ __forceinline__ void reduce(unsigned long long *s_stats, int lane) const
	{
		unsigned long long v[6] = { c0, b0, c1, b1, c2, b2 };
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
};

// The whole reference program for one packet read from HBM (no staged
// window): the general path's and the deferred packets' classification.
template <uint32_t FEAT>
__device__ __forceinline__ uint32_t classify_one(const xfg_kargs &a, const uint32_t *s_ports,
					      uint64_t gi, uint32_t len, uint32_t &tag)
{
	Pkt<0> p{ nullptr, pkt_ptr(a, gi), len };
	const Parsed r = parse<FEAT, 0>(p);
	return lookups<FEAT, false>(a, LazyKeys<Pkt<0>>{ p }, r, s_ports, tag);
}

// A deferred packet of the pipelined kernels (fixed stride >= W, no
// offsets or descriptors): its first W bytes staged into the lane's LDS row
// with CPP independent 16-byte loads (one round trip), then the reference
// program over that window (bytes past it from HBM, rare) -- instead of a
// chain of dependent byte loads.  Whole wave; lanes with ok false idle.
template <uint32_t FEAT, int W>
__device__ __forceinline__ uint32_t classify_staged(const xfg_kargs &a, const uint32_t *s_ports,
						    uint32_t *row, bool ok, uint64_t gi, uint32_t len,
						    uint32_t &tag)
{
	constexpr int CPP = W / 16;
	const uint8_t *g = a.data + gi * (uint64_t)a.stride;
	u32x4 v[CPP];
#pragma unroll
	for (int it = 0; it < CPP; it++)
		v[it] = ok ? reinterpret_cast<const u32x4 *>(g)[it] : u32x4{ 0, 0, 0, 0 };
	__builtin_amdgcn_wave_barrier();
#pragma unroll
	for (int it = 0; it < CPP; it++) {
		row[4 * it] = v[it].x;
		row[4 * it + 1] = v[it].y;
		row[4 * it + 2] = v[it].z;
		row[4 * it + 3] = v[it].w;
	}
	__builtin_amdgcn_wave_barrier();
	tag = CT_NONE;
	if (!ok)
		return A_NONE;
	Pkt<W> p{ row, g, len };
	const Parsed r = parse<FEAT, W>(p);
	return lookups<FEAT, false>(a, LazyKeys<Pkt<W>>{ p }, r, s_ports, tag);
}

// Stage the ruled ports into LDS: the table into s_tab (static), or the
// nibble map into s_nib (the front of the dynamic LDS); returns the one the
// lookups read.
template <uint32_t FEAT>
__device__ __forceinline__ const uint32_t *stage_ports(const xfg_kargs &a, uint32_t *s_tab,
						       uint32_t *s_nib, int tid, int nthr)
{
	if constexpr ((FEAT & (F_UDP | F_TCP)) != 0) {
		if (a.port_count && a.port_tab) {
			for (int i = tid; i < (int)XFG_PORT_TAB; i += nthr)
				s_tab[i] = a.port_tab[i];
		} else if (a.port_count) {
			for (int i = tid; i < (int)XFG_PORT_NIB_WORDS; i += nthr)
				s_nib[i] = a.port_nib[i];
			return s_nib;
		}
	}
	return s_tab;
}

// Dynamic LDS of a classify kernel: the port nibble map (when used), then
// the direct counters.
__device__ __forceinline__ uint32_t *dcnt_base(const xfg_kargs &a, uint32_t *s_dyn)
{
	return s_dyn + (a.port_nib && !a.port_tab && a.port_count ? XFG_PORT_NIB_WORDS : 0);
}

// ---------------------------------------------------------------- general kernel
// Every batch layout (offsets, AF_XDP descriptors, strides below the window,
// lengths that must bound the window loads).  A workgroup of 256 lanes walks
// tiles of 256 packets (one per lane): the next tile's windows are loaded
// into registers while the current one is processed, staged into LDS rows
// of W + 4 bytes (odd dword stride: conflict-free lane-per-packet reads),
// parsed (xdpfilt_prog.h:224-307 over headers/xdp/parsing_helpers.h) and
// looked up in reference order (`lookups`).
template <uint32_t FEAT, int W>
__global__ __launch_bounds__(TILE) void xfg_classify_kernel(const xfg_kargs a)
{
	constexpr int CPP = W / 16;
	constexpr int ROWDW = Pkt<W>::ROWDW;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	__shared__ uint32_t win[TILE * ROWDW];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];

	const int tid = threadIdx.x, lane = tid & 63;
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, TILE);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, TILE);
	__syncthreads();

	const uint64_t ntiles = (a.n + TILE - 1) / TILE;
	uint64_t tile = blockIdx.x;
	u32x4 pre[CPP];
	uint32_t plen = 0;
	LaneStats st;
	auto issue = [&](uint64_t t) {
		const uint64_t base = t * TILE;
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const int c = it * TILE + tid;
			const int pk = c / CPP, sub = c % CPP;
			const uint64_t gi = base + pk;
			pre[it] = u32x4{ 0, 0, 0, 0 };
			if (gi < a.n && (uint32_t)sub * 16 < load_len(a, gi) &&
			    (a.offsets || a.descs || (uint32_t)sub * 16 < a.stride))
				pre[it] = __builtin_nontemporal_load(
					reinterpret_cast<const u32x4 *>(pkt_ptr(a, gi) + sub * 16));
		}
		plen = base + tid < a.n ? load_len(a, base + tid) : 0;
		// a fixed-stride slot bounds its frame (a longer length would read
		// the next slot or past the batch); header windows keep the true
		// length
		if (!a.offsets && !a.descs && !a.hwin)
			plen = min(plen, a.stride);
	};
	if (tile < ntiles)
		issue(tile);
	for (; tile < ntiles; tile += gridDim.x) {
		const uint64_t base = tile * TILE;
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const int c = it * TILE + tid;
			const int pk = c / CPP, sub = c % CPP;
			uint32_t *dst = &win[pk * ROWDW + sub * 4];
			dst[0] = pre[it].x;
			dst[1] = pre[it].y;
			dst[2] = pre[it].z;
			dst[3] = pre[it].w;
		}
		const uint32_t len = plen;
		__syncthreads();
		if (tile + gridDim.x < ntiles)
			issue(tile + gridDim.x);   // next tile's stream overlaps this tile's work
		const uint64_t gi = base + tid;
		uint32_t act = A_NONE, tag = CT_NONE;
		if (gi < a.n) {
			uint32_t oob = 0;
			Pkt<W> p{ &win[tid * ROWDW], pkt_ptr(a, gi), len, a.hwin ? &oob : nullptr };
			const Parsed r = parse<FEAT, W>(p);
			act = lookups<FEAT, false>(a, LazyKeys<Pkt<W>>{ p }, r, s_ports, tag);
			if (oob) {   // past the header window: the host's whole-frame pass
				act = A_NONE;
				tag = CT_NONE;
				const uint32_t k = atomicAdd(a.fb_cnt, 1u);
				if (k < a.fb_cap)
					a.fb[k] = (uint32_t)gi;
			} else {
				a.verdicts[gi] = (uint8_t)act;
			}
		}
		cn.bump(a, tag, lane);
		st.add(act, len);
		__syncthreads();   // LDS window reuse
	}
	st.reduce(s_stats, lane);
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	cn.flush(a, tid, TILE);
}

#include "xfg_pipeline.hip"
#include "xfg_pipee.hip"
#include "xfg_pipeq.hip"
#ifdef XFG_DIAG   // measured slower than xfg_pipe4_kernel: diagnostics only
#include "xfg_split.hip"
#endif

// ---------------------------------------------------------------- hit-log count
// One workgroup per log partition (see HitLog): sums the partition's
// slices (one per classify workgroup, 16-bit local indices) in an LDS
// histogram, then adds each non-zero count to its counter with a plain
// read-modify-write (the workgroup owns the partition's counters).  The
// counters' current values (and, for the quotient index, their identities)
// are read before the histogram is built, so the end is one round of
// stores.  A wave per slice, eight slices in flight per wave, one 8-byte
// load per lane (a wave load covers 256 entries: about a uniform slice, so
// few of the LDS atomics' lanes idle).
#if XFG_PART_COMMON
constexpr int LC_THREADS = 1024;
#ifndef XFG_LC_U   /* slices a wave has in flight (A/B) */
#define XFG_LC_U 8
#endif

__global__ __launch_bounds__(LC_THREADS) void xfg_log_count_kernel(const xfg_kargs a, uint32_t hist_n)
{
	extern __shared__ uint32_t hist[];
	__shared__ uint32_t s_fill[XFG_LOG_SLICES_MAX];
	// (partition p, pass j: local indices [j * hist_n, (j + 1) * hist_n))
	const uint32_t tid = threadIdx.x, p = blockIdx.x % XFG_LOG_PARTS, lane = tid & 63, w = tid >> 6;
	const uint32_t j0 = (blockIdx.x / XFG_LOG_PARTS) * hist_n;
	constexpr uint32_t NWV = LC_THREADS / 64, U = XFG_LC_U, J = XFG_LOG_HIST_MAX / LC_THREADS;
	// (S slices to read; PS between partitions: pending launches' logs side by side)
	const uint32_t S = a.pcount, PS = a.pslices, cap = a.pcap;
	// the identity span: hash-map + port counters, or the QT slots
	const uint32_t total = a.qt ? a.qt_n : a.gbase[3] + 65536u;
	// counters of histogram entries tid + j * LC_THREADS: identity, value
	// (the quotient index: the QT-order counts, 16 slots a line)
	uint32_t gid[J];
	unsigned long long val[J];
#pragma unroll
	for (uint32_t j = 0; j < J; j++) {
		const uint32_t k = tid + j * LC_THREADS, l = j0 + k;
		const uint32_t g = ((l >> 4) << 12) | (p << 4) | (l & 15);
		gid[j] = k < hist_n && l < a.log_span && g < total ? (a.qt_hits ? g : a.qt ? a.qt_trans[g] : g)
								   : CT_NONE;
	}
	const uint32_t fl = tid < S ? a.pfill[(uint64_t)p * PS + a.pfirst + tid] : 0u;
	for (uint32_t i = tid; i < hist_n; i += LC_THREADS)
		hist[i] = 0;
#ifdef XFG_DIAG
	const bool normw = (a.diag & 8192) != 0;   // (diagnostics: no counter read-modify-write)
	// (diagnostics: 65536 the slices loaded but not added, 131072 no slice read)
	const bool noadd = (a.diag & 65536) != 0, noslice = (a.diag & 131072) != 0;
#else
	constexpr bool normw = false, noadd = false, noslice = false;
#endif
#pragma unroll
	for (uint32_t j = 0; j < J; j++)
		val[j] = gid[j] == CT_NONE || normw ? 0ull
			 : a.qt_hits ? (unsigned long long)a.qt_hits[gid[j]] : *global_counter(a, gid[j]);
	if (tid < S)
		s_fill[tid] = min(fl, cap);
	__syncthreads();
	if (a.pwide) {   // (u32 local indices, a range beyond one pass)
		const uint32_t *wb = reinterpret_cast<const uint32_t *>(a.pbuf) + ((uint64_t)p * PS + a.pfirst) * cap;
		for (uint32_t sl = w; sl < S; sl += NWV) {
			const uint32_t np = s_fill[sl];
			for (uint32_t i = lane; i < np; i += 64) {
				const uint32_t l = __builtin_nontemporal_load(wb + (uint64_t)sl * cap + i) - j0;
				if (l < hist_n)
					atomicAdd(&hist[l], 1u);
			}
		}
	}
	const uint16_t *base = a.pbuf + ((uint64_t)p * PS + a.pfirst) * cap;
	// (a wave load covers 512 entries of a slice -- 16 bytes a lane: about a
	// uniform slice at the bench's batch; pcap is a multiple of 8, so every
	// slice starts 16-byte aligned; the buffer has 512 entries of slack)
	auto add8 = [&](u32x4 v, uint32_t i0, uint32_t np) {
		if (noadd) {
			asm volatile("" ::"v"(v));
			return;
		}
#pragma unroll
		for (uint32_t c = 0; c < 4; c++) {
			const uint32_t l0 = (v[c] & 0xffff) - j0, l1 = (v[c] >> 16) - j0;
			if (i0 + 2 * c < np && l0 < hist_n)
				atomicAdd(&hist[l0], 1u);
			if (i0 + 2 * c + 1 < np && l1 < hist_n)
				atomicAdd(&hist[l1], 1u);
		}
	};
	// (two rounds of U slices in flight: the next round's loads issued
	// before this round's LDS atomics -- with the logs of several launches
	// a wave takes dozens of slices; only the lanes whose 8 entries start
	// inside the slice's fill load: at a quarter of the bench's batch a
	// whole-wave load read four times the log, and the count kernel took
	// 62 us for four launches' logs against 47, profiles/archive/r05_s43_session.log)
	auto ld = [&](uint32_t s0, u32x4 (&d)[U]) {
#pragma unroll
		for (uint32_t u = 0; u < U; u++) {
			const uint32_t sl = s0 + u * NWV;
			const u32x4 *e = (const u32x4 *)(base + (uint64_t)sl * cap);
			d[u] = sl < S && lane * 8 < s_fill[sl] ? __builtin_nontemporal_load(e + lane)
							    : u32x4{ 0, 0, 0, 0 };
		}
	};
	u32x4 v[U], nx[U];
	if (!a.pwide && w < S && !noslice)
		ld(w, v);
	for (uint32_t s0 = a.pwide || noslice ? S : w; s0 < S; s0 += NWV * U) {
		if (s0 + NWV * U < S)
			ld(s0 + NWV * U, nx);
#pragma unroll
		for (uint32_t u = 0; u < U; u++) {
			const uint32_t sl = s0 + u * NWV;
			add8(v[u], lane * 8, sl < S ? s_fill[sl] : 0u);
		}
		// (a fuller slice: the rest)
#pragma unroll
		for (uint32_t u = 0; u < U; u++) {
			const uint32_t sl = s0 + u * NWV;
			const uint32_t np = sl < S ? s_fill[sl] : 0u;
			const u32x4 *e = (const u32x4 *)(base + (uint64_t)sl * cap);
			for (uint32_t i = 512 + lane * 8; i < np; i += 512)
				add8(__builtin_nontemporal_load(e + i / 8), i, np);
		}
#pragma unroll
		for (uint32_t u = 0; u < U; u++)
			v[u] = nx[u];
	}
	__syncthreads();
#pragma unroll
	for (uint32_t j = 0; j < J; j++) {
		const uint32_t k = tid + j * LC_THREADS;
		if (gid[j] != CT_NONE && hist[k] && !normw) {
			if (a.qt_hits)
				a.qt_hits[gid[j]] = (uint32_t)(val[j] + hist[k]);
			else
				*global_counter(a, gid[j]) = val[j] + hist[k];
		}
	}
}

#endif   // XFG_PART_COMMON

#ifdef XFG_DIAG   // (1-3 % slower than each wave's tail: DESIGN.md §5.3; diagnostics only)
// ---------------------------------------------------------------- deferred packets
// The quotient-index kernel's deferred packets (kargs.defer_sep): every
// wave's list (a.defer + w * defer_cap, a.defer_n[w] entries, defer_nsrc
// lists), classified by the whole reference walk (classify_staged), one
// packet per lane, the lists' concatenation dealt round-robin over the grid:
// the dependent loads of a few hundred thousand walks overlap across the chip
// instead of running as each classify wave's serial tail.
constexpr int DF_THREADS = 256;
constexpr uint32_t DF_SRC_MAX = XFG_DEFER_SRC_MAX;   // source lists (classify waves)

template <uint32_t FEAT, int W>
__global__ __launch_bounds__(DF_THREADS) void xfg_defer_kernel(const xfg_kargs a)
{
	constexpr int ROWDW = Pkt<W>::ROWDW;
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	constexpr uint32_t CH = DF_SRC_MAX / DF_THREADS;
	__shared__ uint32_t win[DF_THREADS * ROWDW];
	__shared__ uint32_t s_tab[PORTS ? XFG_PORT_TAB : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ uint32_t s_pre[DF_SRC_MAX + 1], s_part[DF_THREADS];
	__shared__ unsigned long long s_stats[6];
	extern __shared__ uint32_t s_dyn[];
	const int tid = threadIdx.x, lane = tid & 63;
	Counters cn{ s_ctag, s_ccnt, dcnt_base(a, s_dyn) };
	cn.init(a, tid, DF_THREADS);
	if (tid < 6)
		s_stats[tid] = 0;
	const uint32_t *s_ports = stage_ports<FEAT>(a, s_tab, s_dyn, tid, DF_THREADS);
	// exclusive prefix sums of the lists' fills: CH per thread, then the
	// DF_THREADS partial sums by one wave
	const uint32_t ns = a.defer_nsrc;
	uint32_t v[CH], sum = 0;
#pragma unroll
	for (uint32_t j = 0; j < CH; j++) {
		const uint32_t w = tid * CH + j;
		v[j] = w < ns ? a.defer_n[w] : 0u;
		sum += v[j];
	}
	s_part[tid] = sum;
	__syncthreads();
	if (tid < 64) {
		uint32_t p[DF_THREADS / 64], t = 0;
#pragma unroll
		for (int j = 0; j < DF_THREADS / 64; j++) {
			p[j] = s_part[tid * (DF_THREADS / 64) + j];
			t += p[j];
		}
		uint32_t x = t;   // inclusive scan over the wave
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint32_t y = __shfl_up(x, o);
			if (lane >= o)
				x += y;
		}
		x -= t;
#pragma unroll
		for (int j = 0; j < DF_THREADS / 64; j++) {
			s_part[tid * (DF_THREADS / 64) + j] = x;
			x += p[j];
		}
	}
	__syncthreads();
	uint32_t run = s_part[tid];
#pragma unroll
	for (uint32_t j = 0; j < CH; j++) {
		s_pre[tid * CH + j] = run;
		run += v[j];
	}
	if (tid == DF_THREADS - 1)
		s_pre[DF_SRC_MAX] = run;
	__syncthreads();
	const uint32_t total = s_pre[DF_SRC_MAX];
	LaneStats st;
	for (uint32_t base = blockIdx.x * DF_THREADS; base < total; base += gridDim.x * DF_THREADS) {
		const uint32_t q = base + tid;
		const bool ok = q < total;
		uint32_t gi = 0, len = 0, tag = CT_NONE;
		if (ok) {
			uint32_t lo = 0, hi = DF_SRC_MAX;   // the list: last w with s_pre[w] <= q
			while (hi - lo > 1) {
				const uint32_t mid = (lo + hi) >> 1;
				if (s_pre[mid] <= q)
					lo = mid;
				else
					hi = mid;
			}
			gi = a.defer[(uint64_t)lo * a.defer_cap + (q - s_pre[lo])];
			len = min(load_len(a, gi), a.stride);
		}
		const uint32_t act = classify_staged<FEAT, W>(a, s_ports, &win[tid * ROWDW], ok, gi, len, tag);
		if (ok)
			__builtin_nontemporal_store((uint8_t)act, a.verdicts + gi);
		cn.bump(a, tag, lane);
		st.add(act, len);
	}
	st.reduce(s_stats, lane);
	__syncthreads();
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	cn.flush(a, tid, DF_THREADS);
}
#endif

template <uint32_t FEAT, bool L16, bool BOTH, bool WIDE, uint32_t V6 = 0>
void launch_pipeq2(const xfg_kargs &a, unsigned grid, size_t dl, hipStream_t s)
{
	if (a.window <= 64 && a.dense)
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 64, true, L16, BOTH, WIDE, V6>), dim3(grid), dim3(QT_THREADS(64)), dl, s, a);
	else if (a.window <= 64)
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 64, false, L16, BOTH, WIDE, V6>), dim3(grid), dim3(QT_THREADS(64)), dl, s, a);
	else if (a.dense)
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 128, true, L16, BOTH, WIDE, V6>), dim3(grid), dim3(QT_THREADS(128)), dl, s, a);
	else
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 128, false, L16, BOTH, WIDE, V6>), dim3(grid), dim3(QT_THREADS(128)), dl, s, a);
#ifdef XFG_DIAG
	if (a.defer_sep) {
		if (a.window <= 64)
			hipLaunchKernelGGL((xfg_defer_kernel<FEAT, 64>), dim3(a.defer_grid), dim3(DF_THREADS), dl, s, a);
		else
			hipLaunchKernelGGL((xfg_defer_kernel<FEAT, 128>), dim3(a.defer_grid), dim3(DF_THREADS), dl, s, a);
	}
#endif
}

// (qt_live 3: both IPv4 lookups through the index; pwide: an index past
// 2^20 buckets, one lookup direction -- the host takes no other; v6p: the
// IPv6 lookups in the loop, 1 one direction, 2 both, beside one IPv4
// direction or both)
// (the count wave: a workgroup of nine waves, the histogram in dynamic LDS
// past the direct counters; 64-byte windows, u16 logs, no IPv6 lookups in
// the loop -- the host enables it for those launches only, xfg_ctx.c)
template <uint32_t FEAT, bool L16, bool BOTH>
void launch_pipeq_cw(const xfg_kargs &a, unsigned grid, size_t dl, hipStream_t s)
{
	const size_t dlc = (size_t)((a.dcnt + 3) & ~3u) * 4 +
			   (a.port_nib && !a.port_tab && a.port_count ? XFG_PORT_NIB_WORDS * 4 : 0) +
			   (size_t)a.log_hist * 4;
	(void)dl;
	if (a.dense)
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 64, true, L16, BOTH, false, 0, true>), dim3(grid),
				   dim3(QT_THREADS(64) + 64), dlc, s, a);
	else
		hipLaunchKernelGGL((xfg_pipeq_kernel<FEAT, 64, false, L16, BOTH, false, 0, true>), dim3(grid),
				   dim3(QT_THREADS(64) + 64), dlc, s, a);
}

template <uint32_t FEAT, bool L16>
void launch_pipeq(const xfg_kargs &a, unsigned grid, size_t dl, hipStream_t s)
{
	if constexpr ((FEAT & F_ETH) != 0) {
		// The Ethernet lookups are compiled in only where the Ethernet map
		// is live as the LDS key table (a.ek); otherwise every lookup would
		// miss, and the instantiation without them runs.  The host takes the
		// table beside IPv4 keys only: no count wave, no IPv6 in the loop.
		if (!a.ek)
			launch_pipeq<FEAT & ~F_ETH, L16>(a, grid, dl, s);
		else if (a.qt_live == 3)
			launch_pipeq2<FEAT, L16, true, false>(a, grid, dl, s);
		else if (a.pwide)
			launch_pipeq2<FEAT, L16, false, true>(a, grid, dl, s);
		else
			launch_pipeq2<FEAT, L16, false, false>(a, grid, dl, s);
	} else {
		if (a.cw_n) {
			if (a.qt_live == 3)
				launch_pipeq_cw<FEAT, L16, true>(a, grid, dl, s);
			else
				launch_pipeq_cw<FEAT, L16, false>(a, grid, dl, s);
			return;
		}
		if constexpr ((FEAT & F_IPV6) != 0)
			if (a.v6p) {
				if (a.qt_live == 3 && a.v6p == 2)
					launch_pipeq2<FEAT, L16, true, false, 2>(a, grid, dl, s);
				else if (a.qt_live == 3)
					launch_pipeq2<FEAT, L16, true, false, 1>(a, grid, dl, s);
				else if (a.v6p == 2 && a.pwide)
					launch_pipeq2<FEAT, L16, false, true, 2>(a, grid, dl, s);
				else if (a.v6p == 2)
					launch_pipeq2<FEAT, L16, false, false, 2>(a, grid, dl, s);
				else if (a.pwide)
					launch_pipeq2<FEAT, L16, false, true, 1>(a, grid, dl, s);
				else
					launch_pipeq2<FEAT, L16, false, false, 1>(a, grid, dl, s);
				return;
			}
		if (a.qt_live == 3)
			launch_pipeq2<FEAT, L16, true, false>(a, grid, dl, s);
		else if (a.pwide)
			launch_pipeq2<FEAT, L16, false, true>(a, grid, dl, s);
		else
			launch_pipeq2<FEAT, L16, false, false>(a, grid, dl, s);
	}
}

template <uint32_t FEAT>
hipError_t launch_feat(const xfg_kargs &a, unsigned grid, hipStream_t s)
{
	const size_t dl = (size_t)a.dcnt * 4 + (size_t)a.bl_lds * 4 +
			  (a.port_nib && !a.port_tab && a.port_count ? XFG_PORT_NIB_WORDS * 4 : 0) +
			  (a.ek ? 12 + (size_t)a.ek_slots * 16 : 0);   // (+ the table's alignment)
	if (a.pipe) {
		bool done = false;
		if constexpr ((FEAT & F_ETH) != 0 && (FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
			// the Ethernet-only programs with their map as an LDS key table
			if (a.ek) {
				done = true;
				if (a.lens_u16)
					hipLaunchKernelGGL((xfg_pipee_kernel<FEAT, true>), dim3(grid), dim3(EK_THREADS), dl, s, a);
				else
					hipLaunchKernelGGL((xfg_pipee_kernel<FEAT, false>), dim3(grid), dim3(EK_THREADS), dl, s, a);
			}
		}
		if constexpr ((FEAT & F_IPV4) != 0) {
			// key mode 1 (only IPv4 keys live): the branch-free kernel
			// (diagnostics build: or the split parse + lookup passes)
#ifdef XFG_DIAG
			if (a.km == 1 && a.split) {
				done = true;
				const dim3 gp(a.grid_parse), tp(64 * PARSE_WAVES);
				if (a.window <= 64 && a.dense)
					hipLaunchKernelGGL((xfg_parse4_kernel<FEAT, 64, true>), gp, tp, 0, s, a);
				else if (a.window <= 64)
					hipLaunchKernelGGL((xfg_parse4_kernel<FEAT, 64, false>), gp, tp, 0, s, a);
				else if (a.dense)
					hipLaunchKernelGGL((xfg_parse4_kernel<FEAT, 128, true>), gp, tp, 0, s, a);
				else
					hipLaunchKernelGGL((xfg_parse4_kernel<FEAT, 128, false>), gp, tp, 0, s, a);
				if (a.window <= 64)
					hipLaunchKernelGGL((xfg_look4_kernel<FEAT, 64>), dim3(grid), dim3(PIPE_THREADS(64)), dl, s, a);
				else
					hipLaunchKernelGGL((xfg_look4_kernel<FEAT, 128>), dim3(grid), dim3(PIPE_THREADS(128)), dl, s, a);
			} else
#endif
			if (a.km == 1 && a.qt) {
				// the quotient index: one bucket read per packet
				done = true;
				if (a.lens_u16)
					launch_pipeq<FEAT, true>(a, grid, dl, s);
				else
					launch_pipeq<FEAT, false>(a, grid, dl, s);
			} else if (a.km == 1) {
				done = true;
				if (a.window <= 64 && a.dense)
					hipLaunchKernelGGL((xfg_pipe4_kernel<FEAT, 64, true>), dim3(grid), dim3(PIPE_THREADS(64)), dl, s, a);
				else if (a.window <= 64)
					hipLaunchKernelGGL((xfg_pipe4_kernel<FEAT, 64, false>), dim3(grid), dim3(PIPE_THREADS(64)), dl, s, a);
				else if (a.dense)
					hipLaunchKernelGGL((xfg_pipe4_kernel<FEAT, 128, true>), dim3(grid), dim3(PIPE_THREADS(128)), dl, s, a);
				else
					hipLaunchKernelGGL((xfg_pipe4_kernel<FEAT, 128, false>), dim3(grid), dim3(PIPE_THREADS(128)), dl, s, a);
			}
		}
		if (!done) {
			if (a.window <= 64 && a.dense)
				hipLaunchKernelGGL((xfg_pipeline_kernel<FEAT, 64, true, 0>), dim3(grid), dim3(PIPE_THREADS(64)), dl, s, a);
			else if (a.window <= 64)
				hipLaunchKernelGGL((xfg_pipeline_kernel<FEAT, 64, false, 0>), dim3(grid), dim3(PIPE_THREADS(64)), dl, s, a);
			else if (a.dense)
				hipLaunchKernelGGL((xfg_pipeline_kernel<FEAT, 128, true, 0>), dim3(grid), dim3(PIPE_THREADS(128)), dl, s, a);
			else
				hipLaunchKernelGGL((xfg_pipeline_kernel<FEAT, 128, false, 0>), dim3(grid), dim3(PIPE_THREADS(128)), dl, s, a);
		}
	} else if (a.window <= 64) {
		hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64>), dim3(grid), dim3(TILE), dl, s, a);
	} else {
		hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 128>), dim3(grid), dim3(TILE), dl, s, a);
	}
	return hipGetLastError();
}

}  // namespace

// Feature words of the ten programs (xdp-filter/xdpfilt_*.c + :313-315).
#define XFG_ALL (F_TCP | F_UDP | F_IPV6 | F_IPV4 | F_ETH)
#define XFG_ALLOW (1u << 5)

#if XFG_PART_COMMON
// The hit log's count kernel (after a classify that filled a.pbuf / a.pfill,
// on the same stream: overlapping it with the next classify on a second
// stream slowed the classify)
extern "C" int xfg_launch_log_count(const struct xfg_kargs *a, void *stream)
{
	if (!a->pbuf)
		return 0;
	const uint32_t passes = (a->log_span + a->log_hist - 1) / a->log_hist;
	(void)hipGetLastError();   // (a stale error is not this launch's)
	hipLaunchKernelGGL(xfg_log_count_kernel, dim3(XFG_LOG_PARTS * passes), dim3(LC_THREADS),
			   (size_t)a->log_hist * 4, static_cast<hipStream_t>(stream), *a, a->log_hist);
	const hipError_t e = hipGetLastError();
	return e == hipSuccess ? 0 : -(int)e - 1000;
}
#endif

// The ten programs (xfg_lc_<i> / xfg_oc_<i>: launch and occupancy of
// program i, defined by the unit whose XFG_PART_MASK has bit i).  The A/B
// variant libraries instantiate C3's program (XFG_AB_C3) or the Ethernet
// programs (XFG_AB_ETH) only.
#if defined(XFG_AB_C3)
#define XFG_AB_OK(i) ((i) == 8)
#elif defined(XFG_AB_ETH)
#define XFG_AB_OK(i) ((i) == 6 || (i) == 7)
#else
#define XFG_AB_OK(i) 1
#endif
#define XFG_PROGS(X)                                     \
	X(0, F_UDP | F_DENY)                             \
	X(1, F_TCP | F_DENY)                             \
	X(2, F_IPV4 | F_IPV6 | F_DENY)                   \
	X(3, F_UDP | XFG_ALLOW)                          \
	X(4, F_TCP | XFG_ALLOW)                          \
	X(5, F_IPV4 | F_IPV6 | XFG_ALLOW)                \
	X(6, F_ETH | F_DENY)                             \
	X(7, F_ETH | XFG_ALLOW)                          \
	X(8, XFG_ALL | F_DENY)                           \
	X(9, XFG_ALL | XFG_ALLOW)
#define XFG_DECL(i, F)                                                                              \
	extern "C" hipError_t xfg_lc_##i(const xfg_kargs &a, unsigned grid, hipStream_t s);        \
	extern "C" int xfg_oc_##i(int kind, uint32_t window, size_t dyn);
XFG_PROGS(XFG_DECL)

#if XFG_PART_COMMON
extern "C" int xfg_launch_classify(uint32_t prog_features, const struct xfg_kargs *a,
				   unsigned grid, void *stream)
{
	hipStream_t s = static_cast<hipStream_t>(stream);
	hipError_t e;
	(void)hipGetLastError();   // (a stale error is not this launch's)
	switch (prog_features) {
#define XFG_CASE_L(i, F) \
	case F:                  \
		e = xfg_lc_##i(*a, grid, s); \
		break;
	XFG_PROGS(XFG_CASE_L)
	default:
		return -22; /* -EINVAL */
	}
	return e == hipSuccess ? 0 : -(int)e - 1000;
}
#endif

// Resident workgroups per CU of the quotient-index kernel with its count
// wave, `dyn` bytes of dynamic LDS (the direct counters, the port map, the
// histogram): 0 = it cannot launch (the host then counts with the count
// kernel).  The fewest over the variants a launch may take.
template <uint32_t FEAT>
static int occupancy_cw(size_t dyn)
{
	int m = 0;
	bool any = false;
	if constexpr ((FEAT & F_IPV4) != 0) {
		const void *k[4] = { (const void *)xfg_pipeq_kernel<FEAT, 64, true, true, false, false, 0, true>,
				     (const void *)xfg_pipeq_kernel<FEAT, 64, false, false, false, false, 0, true>,
				     (const void *)xfg_pipeq_kernel<FEAT, 64, true, true, true, false, 0, true>,
				     (const void *)xfg_pipeq_kernel<FEAT, 64, false, false, true, false, 0, true> };
		for (int i = 0; i < 4; i++) {
			int x = 0;
			if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&x, k[i], QT_THREADS(64) + 64, dyn) != hipSuccess)
				return 0;
			m = any ? (x < m ? x : m) : x;
			any = true;
		}
	}
	return m;
}

// Resident workgroups per CU of the quotient-index kernel (kind 5): the
// fewest over the variants a launch may take -- both directions, the u32
// log, the IPv6 lookups, the Ethernet key table: their LDS and registers
// differ -- so the persistent grid and the hit-log slices sized from it hold
// for whichever one runs.  (A program with Ethernet lookups runs the
// instantiations without them unless the key table is live, launch_pipeq.)
template <uint32_t FEAT>
static int occupancy_qt(uint32_t window, size_t dyn, hipError_t &e)
{
	constexpr uint32_t G = FEAT & ~F_ETH;
	int m = 0;
	auto q = [&](const void *k, int thr) {
		int x = 0;
		const hipError_t r = hipOccupancyMaxActiveBlocksPerMultiprocessor(&x, k, thr, dyn);
		if (r != hipSuccess)
			e = r;
		else if (x > 0 && (m == 0 || x < m))
			m = x;
	};
	if (window <= 64) {
		q((const void *)xfg_pipeq_kernel<G, 64, true, true, false, false, 0>, QT_THREADS(64));
		q((const void *)xfg_pipeq_kernel<G, 64, true, true, true, false, 0>, QT_THREADS(64));
		q((const void *)xfg_pipeq_kernel<G, 64, true, true, false, true, 0>, QT_THREADS(64));
		if constexpr ((FEAT & F_IPV6) != 0) {
			q((const void *)xfg_pipeq_kernel<G, 64, true, true, false, false, 1>, QT_THREADS(64));
			q((const void *)xfg_pipeq_kernel<G, 64, true, true, false, true, 2>, QT_THREADS(64));
			q((const void *)xfg_pipeq_kernel<G, 64, true, true, true, false, 2>, QT_THREADS(64));
		}
		if constexpr ((FEAT & F_ETH) != 0) {
			q((const void *)xfg_pipeq_kernel<FEAT, 64, true, true, false, false, 0>, QT_THREADS(64));
			q((const void *)xfg_pipeq_kernel<FEAT, 64, true, true, true, false, 0>, QT_THREADS(64));
			q((const void *)xfg_pipeq_kernel<FEAT, 64, true, true, false, true, 0>, QT_THREADS(64));
		}
	} else {
		q((const void *)xfg_pipeq_kernel<G, 128, false, true, false, false, 0>, QT_THREADS(128));
		q((const void *)xfg_pipeq_kernel<G, 128, false, true, true, false, 0>, QT_THREADS(128));
		q((const void *)xfg_pipeq_kernel<G, 128, false, true, false, true, 0>, QT_THREADS(128));
		if constexpr ((FEAT & F_IPV6) != 0) {
			q((const void *)xfg_pipeq_kernel<G, 128, false, true, false, false, 1>, QT_THREADS(128));
			q((const void *)xfg_pipeq_kernel<G, 128, false, true, false, true, 2>, QT_THREADS(128));
			q((const void *)xfg_pipeq_kernel<G, 128, false, true, true, false, 2>, QT_THREADS(128));
		}
		if constexpr ((FEAT & F_ETH) != 0) {
			q((const void *)xfg_pipeq_kernel<FEAT, 128, false, true, false, false, 0>, QT_THREADS(128));
			q((const void *)xfg_pipeq_kernel<FEAT, 128, false, true, true, false, 0>, QT_THREADS(128));
			q((const void *)xfg_pipeq_kernel<FEAT, 128, false, true, false, true, 0>, QT_THREADS(128));
		}
	}
	return m;
}

// Resident workgroups per CU of a classify kernel (persistent grid sizing)
// with `dyn` bytes of dynamic LDS: kind 0 = general, 1 = pipelined (key
// mode 0), 2 = pipelined (key mode 1), 5 = pipelined over the quotient
// index, 6 = the Ethernet-key kernel, 7 = kind 5 with its count wave (0:
// it cannot launch); window 64 or 128.
template <uint32_t FEAT>
static int occupancy_feat(int kind, uint32_t window, size_t dyn)
{
	int n = 0;
	hipError_t e = hipSuccess;
	bool done = false;
	if (kind == 7)   // (the quotient-index kernel with its count wave, 64-byte windows)
		return window <= 64 ? occupancy_cw<FEAT & ~F_ETH>(dyn) : 0;
	if constexpr ((FEAT & F_IPV4) != 0) {
#ifdef XFG_DIAG
		if (kind == 3) {        // split: the lookup pass
			done = true;
			e = window <= 64
				? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_look4_kernel<FEAT, 64>, PIPE_THREADS(64), dyn)
				: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_look4_kernel<FEAT, 128>, PIPE_THREADS(128), dyn);
		} else if (kind == 4) { // split: the parse pass (no dynamic LDS)
			done = true;
			e = window <= 64
				? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_parse4_kernel<FEAT, 64, true>, 64 * PARSE_WAVES, 0)
				: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_parse4_kernel<FEAT, 128, false>, 64 * PARSE_WAVES, 0);
		} else
#endif
		if (kind == 2) {
			done = true;
			e = window <= 64
				? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_pipe4_kernel<FEAT, 64, true>, PIPE_THREADS(64), dyn)
				: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_pipe4_kernel<FEAT, 128, false>, PIPE_THREADS(128), dyn);
		} else if (kind == 5) {
			done = true;
			n = occupancy_qt<FEAT>(window, dyn, e);
		}
	}
	if constexpr ((FEAT & F_ETH) != 0 && (FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
		if (kind == 6) {   // the Ethernet-key kernel (fewest of its two length widths)
			done = true;
			int x = 0, y = 0;
			e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&x, xfg_pipee_kernel<FEAT, true>, EK_THREADS, dyn + 12);
			if (e == hipSuccess)
				e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&y, xfg_pipee_kernel<FEAT, false>, EK_THREADS, dyn + 12);
			n = x < y ? x : y;
		}
	}
	if (done)
		;
	else if (kind == 6)
		n = 1;   // (no such kernel for this program: never launched)
	else if (kind >= 1)
		e = window <= 64
			? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_pipeline_kernel<FEAT, 64, true, 0>, PIPE_THREADS(64), dyn)
			: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_pipeline_kernel<FEAT, 128, false, 0>, PIPE_THREADS(128), dyn);
	else
		e = window <= 64
			? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_kernel<FEAT, 64>, TILE, dyn)
			: hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, xfg_classify_kernel<FEAT, 128>, TILE, dyn);
	return e == hipSuccess && n > 0 ? n : 1;
}

// Each program's entry points, in the unit that owns it (XFG_PART_MASK);
// a program the A/B macros leave out gets stubs.
#define XFG_DEF(i, F)                                                                               \
	extern "C" hipError_t xfg_lc_##i(const xfg_kargs &a, unsigned grid, hipStream_t s)          \
	{                                                                                           \
		return launch_feat<F>(a, grid, s);                                                  \
	}                                                                                           \
	extern "C" int xfg_oc_##i(int kind, uint32_t window, size_t dyn)                            \
	{                                                                                           \
		return occupancy_feat<F>(kind, window, dyn);                                        \
	}
#define XFG_STUB(i)                                                                                 \
	extern "C" hipError_t xfg_lc_##i(const xfg_kargs &, unsigned, hipStream_t)                  \
	{                                                                                           \
		return hipErrorInvalidValue;                                                        \
	}                                                                                           \
	extern "C" int xfg_oc_##i(int, uint32_t, size_t) { return 1; }
#if ((XFG_PART_MASK >> 0) & 1) && XFG_AB_OK(0)
XFG_DEF(0, F_UDP | F_DENY)
#elif ((XFG_PART_MASK >> 0) & 1)
XFG_STUB(0)
#endif
#if ((XFG_PART_MASK >> 1) & 1) && XFG_AB_OK(1)
XFG_DEF(1, F_TCP | F_DENY)
#elif ((XFG_PART_MASK >> 1) & 1)
XFG_STUB(1)
#endif
#if ((XFG_PART_MASK >> 2) & 1) && XFG_AB_OK(2)
XFG_DEF(2, F_IPV4 | F_IPV6 | F_DENY)
#elif ((XFG_PART_MASK >> 2) & 1)
XFG_STUB(2)
#endif
#if ((XFG_PART_MASK >> 3) & 1) && XFG_AB_OK(3)
XFG_DEF(3, F_UDP | XFG_ALLOW)
#elif ((XFG_PART_MASK >> 3) & 1)
XFG_STUB(3)
#endif
#if ((XFG_PART_MASK >> 4) & 1) && XFG_AB_OK(4)
XFG_DEF(4, F_TCP | XFG_ALLOW)
#elif ((XFG_PART_MASK >> 4) & 1)
XFG_STUB(4)
#endif
#if ((XFG_PART_MASK >> 5) & 1) && XFG_AB_OK(5)
XFG_DEF(5, F_IPV4 | F_IPV6 | XFG_ALLOW)
#elif ((XFG_PART_MASK >> 5) & 1)
XFG_STUB(5)
#endif
#if ((XFG_PART_MASK >> 6) & 1) && XFG_AB_OK(6)
XFG_DEF(6, F_ETH | F_DENY)
#elif ((XFG_PART_MASK >> 6) & 1)
XFG_STUB(6)
#endif
#if ((XFG_PART_MASK >> 7) & 1) && XFG_AB_OK(7)
XFG_DEF(7, F_ETH | XFG_ALLOW)
#elif ((XFG_PART_MASK >> 7) & 1)
XFG_STUB(7)
#endif
#if ((XFG_PART_MASK >> 8) & 1) && XFG_AB_OK(8)
XFG_DEF(8, XFG_ALL | F_DENY)
#elif ((XFG_PART_MASK >> 8) & 1)
XFG_STUB(8)
#endif
#if ((XFG_PART_MASK >> 9) & 1) && XFG_AB_OK(9)
XFG_DEF(9, XFG_ALL | XFG_ALLOW)
#elif ((XFG_PART_MASK >> 9) & 1)
XFG_STUB(9)
#endif

#if XFG_PART_COMMON
extern "C" int xfg_classify_occupancy(uint32_t prog_features, int kind, uint32_t window, size_t dyn)
{
	switch (prog_features) {
#define XFG_CASE_O(i, F) \
	case F:                  \
		return xfg_oc_##i(kind, window, dyn);
	XFG_PROGS(XFG_CASE_O)
	default:                          return 1;
	}
}

// Threads per workgroup of a classify kernel (host grid sizing).
extern "C" int xfg_classify_threads(int kind, uint32_t window)
{
	if (kind == 4)
		return 256;   // the split parse pass (diagnostics build)
	if (kind == 5)
		return window <= 64 ? QT_THREADS(64) : QT_THREADS(128);
	if (kind == 6)
		return EK_THREADS;
	return kind >= 1 ? (window <= 64 ? PIPE_THREADS(64) : PIPE_THREADS(128)) : TILE;
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
	(void)hipGetLastError();
	hipLaunchKernelGGL(xfg_stream_read_kernel, dim3(grid), dim3(256), 0,
			   static_cast<hipStream_t>(stream), static_cast<const u32x4 *>(src),
			   bytes / 16, static_cast<u32x4 *>(sink));
	return hipGetLastError() == hipSuccess ? 0 : -5;
}

// Fold the QT-order hit counts into the canonical IPv4 counters (qt_trans
// is injective: each canonical counter has at most one QT slot, so a plain
// read-modify-write) and zero them.  Runs at readout, not per batch.
__global__ __launch_bounds__(256) void xfg_qt_fold_kernel(uint32_t *__restrict__ qh,
							  const uint32_t *__restrict__ trans,
							  unsigned long long *__restrict__ hits, uint32_t n)
{
	for (uint32_t q = blockIdx.x * 256u + threadIdx.x; q < n; q += gridDim.x * 256u) {
		const uint32_t v = qh[q];
		if (v) {
			const uint32_t c = trans[q];
			if (c != CT_NONE)
				hits[c] += v;
			qh[q] = 0;
		}
	}
}

extern "C" int xfg_launch_qt_fold(uint32_t *qt_hits, const uint32_t *trans,
				  unsigned long long *hits, uint32_t n, void *stream)
{
	const uint32_t grid = n ? (n + 255) / 256 < 2048u ? (n + 255) / 256 : 2048u : 1u;
	(void)hipGetLastError();
	hipLaunchKernelGGL(xfg_qt_fold_kernel, dim3(grid), dim3(256), 0,
			   static_cast<hipStream_t>(stream), qt_hits, trans, hits, n);
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
	(void)hipGetLastError();
	hipLaunchKernelGGL(xfg_compact_kernel, dim3(grid), dim3(CT_LANES), 0, s, verdicts, n, action,
			   idx, count, status, ticket, ntiles);
	return hipGetLastError() == hipSuccess ? 0 : -5;
}

extern "C" uint64_t xfg_compact_tiles(uint64_t n)
{
	return (n + CT_TILE - 1) / CT_TILE;
}

#endif   // XFG_PART_COMMON
