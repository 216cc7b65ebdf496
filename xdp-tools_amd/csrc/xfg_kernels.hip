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

constexpr uint32_t M_SRC = 1, M_DST = 2, M_TCP = 4, M_UDP = 8;
constexpr uint32_t A_ABORTED = 0, A_DROP = 1, A_PASS = 2, A_NONE = 7;

constexpr int TILE = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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
		return g[o];
	}
	// Little-endian 32-bit load of bytes o..o+3 (o+3 < len).
	__device__ __forceinline__ uint32_t u32(uint32_t o) const
	{
		if (o + 4 <= (uint32_t)W) {
			uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, o & 3);
		}
		return g[o] | (g[o + 1] << 8) | (g[o + 2] << 16) | ((uint32_t)g[o + 3] << 24);
	}
	// Raw (memory-order) 16-bit value of bytes o, o+1: the BPF u16 load.
	__device__ __forceinline__ uint32_t raw16(uint32_t o) const
	{
		if (o + 2 <= (uint32_t)W) {
			uint32_t lo = row[o >> 2], hi = row[(o >> 2) + 1];
			return __builtin_amdgcn_alignbyte(hi, lo, o & 3) & 0xffffu;
		}
		return g[o] | ((uint32_t)g[o + 1] << 8);
	}
	// Network-order 16-bit field as a host value (bpf_ntohs of the load).
	__device__ __forceinline__ uint32_t be16(uint32_t o) const
	{
		uint32_t r = raw16(o);
		return ((r & 0xff) << 8) | (r >> 8);
	}
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
	uint32_t o6;           // IPv6 header offset (saddr o6+8, daddr o6+24)
	uint32_t nd;           // NDISC: 0 none, 135 NS, 136 NA
	uint32_t ond;          // target offset
	uint32_t l4proto;      // 17 / 6 when an L4 stage runs, else 0
	uint32_t pdst, psrc;   // raw be16 port keys
};

template <uint32_t FEAT, int W>
__device__ __forceinline__ Parsed parse(const Pkt<W> &p)
{
	Parsed r;
	r.abort_at = NST;
	r.l3 = 0;
	r.nd = 0;
	r.l4proto = 0;
	r.arp_op = 0;
	r.k4a = r.k4b = 0;
	r.o6 = r.ond = 0;
	r.pdst = r.psrc = 0;
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

__device__ __forceinline__ Line load_line(const xfg_tdesc &t, uint32_t b)
{
	const u32x4 *p = reinterpret_cast<const u32x4 *>(bucket_ptr(t, b));
	Line l;
	l.q0 = p[0];
	l.q1 = p[1];
	l.q2 = p[2];
	l.q3 = p[3];
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
template <int KIND>
__device__ __forceinline__ Hit probe_chain(const xfg_tdesc &t, uint32_t b, uint32_t k0, uint32_t k1,
					uint32_t k2, uint32_t k3)
{
	for (uint32_t d = 1; d <= t.max_disp; d++) {
		b = b + 1 == t.nbuckets ? 0 : b + 1;
		const Line l = load_line(t, b);
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
template <int KIND>
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
		const Line l = load_line(t, b);
		const int i = match<KIND>(l, k0, k1, k2, k3);
		if (i >= 0)
			return { (int64_t)b * slots_of<KIND>() + i, l.flag(i) };
		if (l.overflow() && t.max_disp)
			return probe_chain<KIND>(t, b, k0, k1, k2, k3);
		return { -1, 0 };
	}
};

// Counter identity of a hit: map id in the top two bits, slot below
// (slots < 2^30 for every capacity the host accepts).
constexpr uint32_t CT_NONE = 0xffffffffu;
constexpr uint32_t CT_V4 = 0u << 30, CT_V6 = 1u << 30, CT_ETH = 2u << 30, CT_PORT = 3u << 30;

__device__ __forceinline__ unsigned long long *counter_ptr(const xfg_kargs &a, uint32_t tag)
{
	const uint32_t slot = tag & 0x3fffffffu;
	switch (tag >> 30) {
	case 0: return a.t4.hits + slot;
	case 1: return a.t6.hits + slot;
	case 2: return a.te.hits + slot;
	default: return a.port_hits + slot;
	}
}

// CHECK_MAP (xdp-filter/xdpfilt_prog.h:56-64): hit iff the key exists and
// (value & mask) == mask; the counter bump is deferred to the caller.
__device__ __forceinline__ bool take(const Hit &h, uint32_t mask, uint32_t ct, uint32_t &tag)
{
	if (h.slot >= 0 && (h.flags & mask) == mask) {
		tag = ct | (uint32_t)h.slot;
		return true;
	}
	return false;
}

__device__ __forceinline__ bool check_port(const xfg_kargs &a, const uint32_t *s_pbits,
					   uint32_t key, uint32_t mask, uint32_t &tag)
{
	if (!((s_pbits[key >> 5] >> (key & 31)) & 1))
		return false;
	if ((a.port_flags[key] & mask) == mask) {
		tag = CT_PORT | key;
		return true;
	}
	return false;
}

// ---------------------------------------------------------------- the program
// Ordered lookups over a parsed packet; returns the xdp action and sets tag
// to the first matching rule's counter identity (CT_NONE if none).
template <uint32_t FEAT, int W>
__device__ __forceinline__ uint32_t lookups(const xfg_kargs &a, const Pkt<W> &p, const Parsed &r,
					    const uint32_t *s_pbits, uint32_t &tag)
{
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;   // VERDICT_HIT
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;  // VERDICT_MISS

	if (r.abort_at == ST_ETH)
		return A_ABORTED;

	// lookup_verdict_ethernet (xdpfilt_prog.h:187-196): dst then src
	if constexpr ((FEAT & F_ETH) != 0) {
		if (a.te.count) {
			Probe<2> d, s;
			d.start(a.te, true, p.u32(0), p.raw16(4));
			s.start(a.te, true, p.u32(6), p.raw16(10));
			if (take(d.result(a.te), M_DST, CT_ETH, tag) ||
			    take(s.result(a.te), M_SRC, CT_ETH, tag))
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
			Probe<4> x, y;
			x.start(a.t4, true, r.k4a);
			y.start(a.t4, want_b, r.k4b);
			const uint32_t mx = arp ? M_SRC : M_DST;
			const uint32_t my = arp ? (r.arp_op == 1 ? M_DST : M_SRC) : M_SRC;
			if (take(x.result(a.t4), mx, CT_V4, tag) ||
			    (want_b && take(y.result(a.t4), my, CT_V4, tag)))
				return HIT;
		}
	}
	if constexpr ((FEAT & F_IPV6) != 0) {
		if (a.t6.count && r.l3 == 3) {
			// lookup_verdict_ipv6: dst then src (xdpfilt_prog.h:152-165)
			const uint32_t o = r.o6;
			Probe<6> d, s;
			d.start(a.t6, true, p.u32(o + 24), p.u32(o + 28), p.u32(o + 32), p.u32(o + 36));
			s.start(a.t6, true, p.u32(o + 8), p.u32(o + 12), p.u32(o + 16), p.u32(o + 20));
			if (take(d.result(a.t6), M_DST, CT_V6, tag) ||
			    take(s.result(a.t6), M_SRC, CT_V6, tag))
				return HIT;
		}
	}
	if (r.abort_at == ST_ND)
		return A_ABORTED;
	if constexpr ((FEAT & F_IPV6) != 0) {
		if (a.t6.count && r.nd) {
			// NDISC target: NS => DST, NA => SRC (xdpfilt_prog.h:277-285)
			const uint32_t o = r.ond;
			Probe<6> t;
			t.start(a.t6, true, p.u32(o), p.u32(o + 4), p.u32(o + 8), p.u32(o + 12));
			if (take(t.result(a.t6), r.nd == 135 ? M_DST : M_SRC, CT_V6, tag))
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

// Per-workgroup counter cache in LDS: direct-mapped on the counter identity.
// A rule hit by many packets (a hot port, an attacked address) is summed
// here and reaches memory once per workgroup; a slot already owned by a
// different counter sends the bump straight to its global atomic.
constexpr int CC_ENTRIES = 1024;

__device__ __forceinline__ void count_hit(const xfg_kargs &a, uint32_t *s_ctag, uint32_t *s_ccnt,
					  uint32_t tag, uint32_t n)
{
	const uint32_t e = (tag * 0x9E3779B1u) >> 22;   // 10 bits
	uint32_t t = s_ctag[e];
	if (t == CT_NONE) {
		t = atomicCAS(&s_ctag[e], CT_NONE, tag);
		if (t == CT_NONE)
			t = tag;
	}
	if (t == tag)
		atomicAdd(&s_ccnt[e], n);
	else
		atomicAdd(counter_ptr(a, tag), (unsigned long long)n);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o);
	return v;
}

__device__ __forceinline__ uint32_t load_len(const xfg_kargs &a, uint64_t i)
{
	return a.lens_u16 ? static_cast<const uint16_t *>(a.lens)[i]
			  : static_cast<const uint32_t *>(a.lens)[i];
}

__device__ __forceinline__ const uint8_t *pkt_ptr(const xfg_kargs &a, uint64_t i)
{
	return a.data + (a.offsets ? a.offsets[i] : i * (uint64_t)a.stride);
}

// ---------------------------------------------------------------- the kernel
template <uint32_t FEAT, int W>
__global__ __launch_bounds__(TILE) void xfg_classify_kernel(const xfg_kargs a)
{
	constexpr int CPP = W / 16;            // 16-byte chunks per packet window
	constexpr int ROWDW = Pkt<W>::ROWDW;   // odd dword stride per LDS row
	constexpr bool PORTS = (FEAT & (F_UDP | F_TCP)) != 0;
	__shared__ uint32_t win[TILE * ROWDW];
	__shared__ uint32_t s_pbits[PORTS ? 2048 : 1];
	__shared__ uint32_t s_ctag[CC_ENTRIES], s_ccnt[CC_ENTRIES];
	__shared__ unsigned long long s_stats[6];

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	if (tid < 6)
		s_stats[tid] = 0;
	for (int i = tid; i < CC_ENTRIES; i += TILE) {
		s_ctag[i] = CT_NONE;
		s_ccnt[i] = 0;
	}
	if constexpr (PORTS) {
		if (a.port_count)
			for (int i = tid; i < 2048; i += TILE)
				s_pbits[i] = a.port_bits[i];
	}
	// fixed-stride layout with stride >= W: every window byte is readable,
	// so loads need no length (no load->load dependency on the stream)
	const bool guarded = a.offsets != nullptr || a.stride < (uint32_t)W;

	const uint64_t ntiles = (a.n + TILE - 1) / TILE;
	uint64_t tile = blockIdx.x;
	u32x4 pre[CPP];
	uint32_t plen = 0;
	auto issue = [&](uint64_t t) {
		const uint64_t base = t * TILE;
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const int c = it * TILE + tid;
			const int pk = c / CPP, sub = c % CPP;
			const uint64_t gi = base + pk;
			pre[it] = u32x4{ 0, 0, 0, 0 };
			if (gi < a.n && (!guarded || (uint32_t)sub * 16 < load_len(a, gi)))
				pre[it] = __builtin_nontemporal_load(
					reinterpret_cast<const u32x4 *>(pkt_ptr(a, gi) + sub * 16));
		}
		plen = base + tid < a.n ? load_len(a, base + tid) : 0;
	};
	if (tile < ntiles)
		issue(tile);

	for (; tile < ntiles; tile += gridDim.x) {
		const uint64_t base = tile * TILE;
		// 1. stage the prefetched windows into LDS
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

		// 2-4. parse, match, verdict
		const uint64_t gi = base + tid;
		uint32_t act = A_NONE;
		uint32_t tag = CT_NONE;
		if (gi < a.n) {
			Pkt<W> p{ &win[tid * ROWDW], pkt_ptr(a, gi), len };
			if (a.ablate & 4) {
				act = p.u8(0) & 1;
			} else {
				const Parsed r = parse<FEAT, W>(p);
				act = lookups<FEAT, W>(a, p, r, s_pbits, tag);
			}
			a.verdicts[gi] = (uint8_t)act;
		}
		if (a.ablate & 2)
			tag = CT_NONE;

		// counter bump: lanes of the wave hitting the same rule are merged
		// (two leader rounds), then summed in the LDS counter cache
#pragma unroll 1
		for (int rnd = 0; rnd < 2; rnd++) {
			const unsigned long long pend = __ballot(tag != CT_NONE);
			if (!pend)
				break;
			const int leader = __ffsll((long long)pend) - 1;
			const uint32_t lt = __shfl(tag, leader);
			const bool mine = tag == lt;
			const unsigned long long same = __ballot(mine);
			if (lane == leader)
				count_hit(a, s_ctag, s_ccnt, lt, (uint32_t)__popcll(same));
			if (mine)
				tag = CT_NONE;
		}
		if (tag != CT_NONE)
			count_hit(a, s_ctag, s_ccnt, tag, 1);

		// 5. per-action stats (xdp_stats_record_action)
#pragma unroll
		for (uint32_t k = 0; k < 3; k++) {
			const unsigned long long m = __ballot(act == k);
			const uint32_t bytes = wave_sum(act == k ? len : 0);
			if (lane == 0 && m) {
				atomicAdd(&s_stats[2 * k], (unsigned long long)__popcll(m));
				atomicAdd(&s_stats[2 * k + 1], (unsigned long long)bytes);
			}
		}
		__syncthreads();   // LDS window reuse
	}
	if (tid < 6 && s_stats[tid])
		atomicAdd(&a.stats[tid], s_stats[tid]);
	for (int i = tid; i < CC_ENTRIES; i += TILE)
		if (s_ctag[i] != CT_NONE && s_ccnt[i])
			atomicAdd(counter_ptr(a, s_ctag[i]), (unsigned long long)s_ccnt[i]);
}

template <uint32_t FEAT>
hipError_t launch_feat(const xfg_kargs &a, unsigned grid, hipStream_t s)
{
	if (a.window <= 64)
		hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 64>), dim3(grid), dim3(TILE), 0, s, a);
	else
		hipLaunchKernelGGL((xfg_classify_kernel<FEAT, 128>), dim3(grid), dim3(TILE), 0, s, a);
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
