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
// Per workgroup tile of 256 packets:
//   1. stage: the first min(len, W) bytes of each packet are copied from HBM
//      into LDS with coalesced 16-byte non-temporal loads (a wave reads 1 KiB
//      contiguous per instruction for the fixed-stride layout), one LDS row of
//      W+4 bytes per packet (odd dword stride: conflict-free lane-per-packet
//      reads);
//   2. parse + match: one lane per packet runs the reference control flow
//      (xdpfilt_prog.h:214-310 over headers/xdp/parsing_helpers.h) reading
//      header fields from its LDS row (bytes past W, only ever reached by
//      long IPv6 extension chains, are read from HBM);
//   3. rule lookups probe the device hash tables (xfg_layout.h) with 16-byte
//      loads of one 64-byte bucket line;
//   4. the first hit's counter is bumped after the wave re-converges, with
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

// ---------------------------------------------------------------- table probes
__device__ __forceinline__ uint32_t next_bucket(uint32_t b, uint32_t nb)
{
	return b + 1 == nb ? 0 : b + 1;
}

// filter_ipv4 lookup (BPF hash: exact match); returns slot or -1.
__device__ __forceinline__ int64_t find_v4(const xfg_tdesc &t, uint32_t k)
{
	if (k == 0)
		return t.zero_present ? (int64_t)t.nslots : -1;
	uint32_t b = xfg_home(xfg_hash_v4(k, t.seed), t.nbuckets);
	for (uint32_t d = 0; d <= t.max_disp; d++) {
		const uint4 *bk = reinterpret_cast<const uint4 *>(
			static_cast<const uint8_t *>(t.keys) + (uint64_t)b * XFG_BUCKET_BYTES);
		const uint4 q0 = bk[0], q1 = bk[1], q2 = bk[2], q3 = bk[3];
		const uint32_t m = (q0.x == k) | (q0.y == k) << 1 | (q0.z == k) << 2 | (q0.w == k) << 3 |
				   (q1.x == k) << 4 | (q1.y == k) << 5 | (q1.z == k) << 6 | (q1.w == k) << 7 |
				   (q2.x == k) << 8 | (q2.y == k) << 9 | (q2.z == k) << 10 | (q2.w == k) << 11 |
				   (q3.x == k) << 12 | (q3.y == k) << 13 | (q3.z == k) << 14 | (q3.w == k) << 15;
		if (m)
			return (int64_t)b * XFG_SLOTS_V4 + (__builtin_ctz(m));
		if (!(t.meta[b] & XFG_META_OVERFLOW))
			return -1;
		b = next_bucket(b, t.nbuckets);
	}
	return -1;
}

// filter_ipv6 lookup: 16-byte keys, 4 per bucket.
__device__ __forceinline__ int64_t find_v6(const xfg_tdesc &t, uint32_t w0, uint32_t w1,
					   uint32_t w2, uint32_t w3)
{
	if ((w0 | w1 | w2 | w3) == 0)
		return t.zero_present ? (int64_t)t.nslots : -1;
	uint32_t b = xfg_home(xfg_hash_v6(w0, w1, w2, w3, t.seed), t.nbuckets);
	for (uint32_t d = 0; d <= t.max_disp; d++) {
		const uint4 *bk = reinterpret_cast<const uint4 *>(
			static_cast<const uint8_t *>(t.keys) + (uint64_t)b * XFG_BUCKET_BYTES);
		const uint4 q[4] = { bk[0], bk[1], bk[2], bk[3] };
#pragma unroll
		for (int i = 0; i < 4; i++)
			if (q[i].x == w0 && q[i].y == w1 && q[i].z == w2 && q[i].w == w3)
				return (int64_t)b * XFG_SLOTS_V6 + i;
		if (!(t.meta[b] & XFG_META_OVERFLOW))
			return -1;
		b = next_bucket(b, t.nbuckets);
	}
	return -1;
}

// filter_ethernet lookup: MAC in the low 48 bits of a u64, 8 per bucket.
__device__ __forceinline__ int64_t find_eth(const xfg_tdesc &t, uint64_t mac)
{
	if (mac == 0)
		return t.zero_present ? (int64_t)t.nslots : -1;
	uint32_t b = xfg_home(xfg_hash_eth(mac, t.seed), t.nbuckets);
	for (uint32_t d = 0; d <= t.max_disp; d++) {
		const uint64_t *bk = reinterpret_cast<const uint64_t *>(
			static_cast<const uint8_t *>(t.keys) + (uint64_t)b * XFG_BUCKET_BYTES);
		uint64_t q[8];
#pragma unroll
		for (int i = 0; i < 8; i++)
			q[i] = bk[i];
#pragma unroll
		for (int i = 0; i < 8; i++)
			if (q[i] == mac)
				return (int64_t)b * XFG_SLOTS_ETH + i;
		if (!(t.meta[b] & XFG_META_OVERFLOW))
			return -1;
		b = next_bucket(b, t.nbuckets);
	}
	return -1;
}

// CHECK_MAP (xdp-filter/xdpfilt_prog.h:56-64): hit iff the key exists and
// (value & mask) == mask.  The counter bump is deferred to the caller.
__device__ __forceinline__ bool check_slot(const xfg_tdesc &t, int64_t slot, uint32_t mask,
					   unsigned long long *&hitp)
{
	if (slot >= 0 && (t.flags[slot] & mask) == mask) {
		hitp = t.hits + slot;
		return true;
	}
	return false;
}

__device__ __forceinline__ bool check_port(const xfg_kargs &a, uint32_t key, uint32_t mask,
					   unsigned long long *&hitp)
{
	if ((a.port_flags[key] & mask) == mask) {
		hitp = a.port_hits + key;
		return true;
	}
	return false;
}

// lookup_verdict_ipv4 (xdpfilt_prog.h:121-134): dst first, then src.
__device__ __forceinline__ bool v4_hit(const xfg_kargs &a, bool has_src, uint32_t src,
				       bool has_dst, uint32_t dst, unsigned long long *&hitp)
{
	if (!a.t4.count)
		return false;
	if (has_dst && check_slot(a.t4, find_v4(a.t4, dst), M_DST, hitp))
		return true;
	if (has_src && check_slot(a.t4, find_v4(a.t4, src), M_SRC, hitp))
		return true;
	return false;
}

template <int W>
__device__ __forceinline__ bool v6_check(const xfg_kargs &a, const Pkt<W> &p, uint32_t o,
					 uint32_t mask, unsigned long long *&hitp)
{
	return check_slot(a.t6, find_v6(a.t6, p.u32(o), p.u32(o + 4), p.u32(o + 8), p.u32(o + 12)),
			  mask, hitp);
}

// ---------------------------------------------------------------- the program
// xdpfilt_prog.h:214-310 for one packet; returns the xdp action and sets
// hitp to the counter of the first matching rule (or leaves it null).
template <uint32_t FEAT, int W>
__device__ uint32_t classify_one(const xfg_kargs &a, const Pkt<W> &p,
				 unsigned long long *&hitp)
{
	constexpr uint32_t HIT = (FEAT & F_DENY) ? A_PASS : A_DROP;   // VERDICT_HIT
	constexpr uint32_t MISS = (FEAT & F_DENY) ? A_DROP : A_PASS;  // VERDICT_MISS
	const uint32_t len = p.len;

	// parse_ethhdr (parsing_helpers.h:100-134), VLAN_MAX_DEPTH 4
	if (14 > len)
		return A_ABORTED;
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

	// lookup_verdict_ethernet (xdpfilt_prog.h:187-196)
	if constexpr ((FEAT & F_ETH) != 0) {
		if (a.te.count) {
			const uint64_t dmac = p.u32(0) | ((uint64_t)p.raw16(4) << 32);
			if (check_slot(a.te, find_eth(a.te, dmac), M_DST, hitp))
				return HIT;
			const uint64_t smac = p.u32(6) | ((uint64_t)p.raw16(10) << 32);
			if (check_slot(a.te, find_eth(a.te, smac), M_SRC, hitp))
				return HIT;
		}
	}

	if constexpr ((FEAT & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)) == 0) {
		return MISS;
	} else {
		uint32_t ip_type = 0, l4 = 0;
		if (proto == 0x0800) {
			// __parse_iphdr, frags_ok = 1 (parsing_helpers.h:201-227)
			if (off + 20 > len)
				return A_ABORTED;
			const uint32_t hdrsize = (p.u8(off) & 0xF) * 4;
			if (off + hdrsize > len)
				return A_ABORTED;
			ip_type = p.u8(off + 9);
			l4 = off + hdrsize;
			if constexpr ((FEAT & F_IPV4) != 0) {
				if (v4_hit(a, true, p.u32(off + 12), true, p.u32(off + 16), hitp))
					return HIT;
			}
		} else if ((FEAT & F_IPV4) && proto == 0x0806) {
			// parse_arphdr (parsing_helpers.h:235-253), xdpfilt_prog.h:241-261
			if (off + 28 > len)
				return A_ABORTED;
			if (p.be16(off) != 1 || p.be16(off + 2) != 0x0800 || p.u8(off + 4) != 6 ||
			    p.u8(off + 5) != 4)
				return A_ABORTED;
			const uint32_t op = p.be16(off + 6);
			const uint32_t sip = p.u32(off + 14), tip = p.u32(off + 24);
			if (v4_hit(a, true, sip, false, 0, hitp))
				return HIT;
			if (op == 1) {          // ARPOP_REQUEST: target is a DST
				if (v4_hit(a, false, 0, true, tip, hitp))
					return HIT;
			} else if (op == 2) {   // ARPOP_REPLY: target is a SRC
				if (v4_hit(a, true, tip, false, 0, hitp))
					return HIT;
			}
		} else if (proto == 0x86DD) {
			// __parse_ip6hdr + skip_ip6hdrext (parsing_helpers.h:136-199)
			if (off + 40 > len)
				return A_ABORTED;
			uint32_t nh = p.u8(off + 6), cur = off + 40;
			bool done = false;
			for (int i = 0; i < 6; i++) {   // IPV6_EXT_MAX_CHAIN
				if (cur + 2 > len)
					return A_ABORTED;
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
			if (!done)
				return A_ABORTED;
			ip_type = nh;
			l4 = cur;
			if constexpr ((FEAT & F_IPV6) != 0) {
				if (a.t6.count) {   // lookup_verdict_ipv6: dst, then src
					if (v6_check(a, p, off + 24, M_DST, hitp) ||
					    v6_check(a, p, off + 8, M_SRC, hitp))
						return HIT;
				}
			}
			if (ip_type == 58) {
				// parse_icmp6hdr + NDISC target (xdpfilt_prog.h:268-287)
				if (cur + 8 > len)
					return A_ABORTED;
				const uint32_t t = p.u8(cur);
				cur += 8;
				if (t == 135 || t == 136) {
					if (cur + 16 > len)
						return A_ABORTED;
					if constexpr ((FEAT & F_IPV6) != 0) {
						if (a.t6.count &&
						    v6_check(a, p, cur, t == 135 ? M_DST : M_SRC, hitp))
							return HIT;
					}
				}
			}
		} else {
			return MISS;
		}

		if constexpr ((FEAT & F_UDP) != 0) {
			if (ip_type == 17) {
				// parse_udphdr (parsing_helpers.h:303-321)
				if (l4 + 8 > len)
					return A_ABORTED;
				if (p.be16(l4 + 4) < 8)
					return A_ABORTED;
				// lookup_verdict_udp (xdpfilt_prog.h:92-101)
				if (a.port_count &&
				    (check_port(a, p.raw16(l4 + 2), M_DST | M_UDP, hitp) ||
				     check_port(a, p.raw16(l4), M_SRC | M_UDP, hitp)))
					return HIT;
			}
		}
		if constexpr ((FEAT & F_TCP) != 0) {
			if (ip_type == 6) {
				// parse_tcphdr (parsing_helpers.h:326-344)
				if (l4 + 20 > len)
					return A_ABORTED;
				if (l4 + (p.u8(l4 + 12) >> 4) * 4 > len)
					return A_ABORTED;
				// lookup_verdict_tcp (xdpfilt_prog.h:76-85)
				if (a.port_count &&
				    (check_port(a, p.raw16(l4 + 2), M_DST | M_TCP, hitp) ||
				     check_port(a, p.raw16(l4), M_SRC | M_TCP, hitp)))
					return HIT;
			}
		}
		return MISS;
	}
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
	__shared__ uint32_t win[TILE * ROWDW];
	__shared__ unsigned long long s_stats[6];

	const int tid = threadIdx.x;
	const int lane = tid & 63;
	if (tid < 6)
		s_stats[tid] = 0;

	const uint64_t ntiles = (a.n + TILE - 1) / TILE;
	for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
		const uint64_t base = tile * TILE;

		// 1. stage header windows into LDS
#pragma unroll
		for (int it = 0; it < CPP; it++) {
			const int c = it * TILE + tid;
			const int pk = c / CPP, sub = c % CPP;
			const uint64_t gi = base + pk;
			if (gi < a.n) {
				const uint32_t len = load_len(a, gi);
				if ((uint32_t)sub * 16 < len) {
					const u32x4 *src = reinterpret_cast<const u32x4 *>(pkt_ptr(a, gi) + sub * 16);
					const u32x4 v = __builtin_nontemporal_load(src);
					uint32_t *dst = &win[pk * ROWDW + sub * 4];
					dst[0] = v.x;
					dst[1] = v.y;
					dst[2] = v.z;
					dst[3] = v.w;
				}
			}
		}
		__syncthreads();

		// 2-4. parse, match, verdict
		const uint64_t gi = base + tid;
		uint32_t act = A_NONE, len = 0;
		unsigned long long *hitp = nullptr;
		if (gi < a.n) {
			len = load_len(a, gi);
			Pkt<W> p{ &win[tid * ROWDW], pkt_ptr(a, gi), len };
			if (a.ablate & 4)
				act = p.u8(0) & 1;
			else
				act = classify_one<FEAT, W>(a, p, hitp);
			a.verdicts[gi] = (uint8_t)act;
		}
		if (a.ablate & 2)
			hitp = nullptr;

		// counter bump, aggregated over same-slot lanes of the wave
#pragma unroll 1
		for (int r = 0; r < 4; r++) {
			const unsigned long long pend = __ballot(hitp != nullptr);
			if (!pend)
				break;
			const int leader = __ffsll((long long)pend) - 1;
			const unsigned long long lp = __shfl((unsigned long long)(uintptr_t)hitp, leader);
			const bool mine = (unsigned long long)(uintptr_t)hitp == lp;
			const unsigned long long same = __ballot(mine);
			if (lane == leader)
				atomicAdd(reinterpret_cast<unsigned long long *>(lp),
					  (unsigned long long)__popcll(same));
			if (mine)
				hitp = nullptr;
		}
		if (hitp)
			atomicAdd(hitp, 1ull);

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
