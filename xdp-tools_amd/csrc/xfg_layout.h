/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xfg_layout.h — device-resident table layout shared by the host runtime (C)
 * and the HIP kernels.  Nothing here is part of the public C ABI.
 *
 * The reference's BPF_MAP_TYPE_PERCPU_HASH maps (filter_ipv4/ipv6/ethernet,
 * xdp-filter/xdpfilt_prog.h:113-185) become bucketed open-addressed tables:
 *
 *   keys  [nbuckets][64 B]  one 64-byte line per bucket:
 *                             ipv4: 16 x u32, ipv6: 4 x 16 B, ethernet: 8 x u64
 *                             (MAC in the low 48 bits, little-endian byte copy)
 *                           an all-zero key marks an empty slot; the all-zero
 *                           KEY itself lives in the extra slot `nslots`.
 *   meta  [nbuckets] u8     bit0 = overflow: some key whose probe sequence
 *                           passed this bucket was placed further on.
 *   flags [nslots+1] u8     low 6 bits of the reference value (MAP_FLAGS..)
 *   hits  [nslots+1] u64    reference value >> COUNTER_SHIFT
 *
 * so the reference value is exactly (hits << 6) | flags, and a hit's
 * `*value += 1 << COUNTER_SHIFT` (xdp-filter/xdpfilt_prog.h:60-61) becomes
 * hits += 1.  Keeping hits apart from flags lets the multi-GPU reduction sum
 * counters directly (ncclUint64) without disturbing the flag bits.
 *
 * Probing: home bucket h(key) (multiplicative range reduction of a 32-bit
 * murmur3 finaliser chain), then linear over buckets; lookup stops at a
 * bucket whose overflow bit is clear or after max_disp+1 buckets.  Keys never
 * move once placed, so slot indices (and hence per-device counters) are
 * stable across inserts and deletes.
 *
 * filter_ports (PERCPU_ARRAY[65536], :67-73) is dense: flags[65536] u8 and
 * hits[65536] u64 indexed by the raw big-endian port value.
 */
#ifndef XFG_LAYOUT_H
#define XFG_LAYOUT_H

#include <stdint.h>

#define XFG_BUCKET_BYTES 64u
#define XFG_SLOTS_V4     16u
#define XFG_SLOTS_V6     4u
#define XFG_SLOTS_ETH    8u

#define XFG_META_OVERFLOW 1u

/* Per-hash-map descriptor passed to the kernel by value. */
struct xfg_tdesc {
	const void *keys;
	const uint8_t *meta;
	const uint8_t *flags;
	unsigned long long *hits;
	uint32_t nbuckets;
	uint32_t max_disp;
	uint32_t count;        /* keys present; 0 => lookups can never hit */
	uint32_t zero_present; /* the all-zero key is present (slot nslots) */
	uint32_t nslots;
	uint32_t seed;
};

/* Kernel arguments of one classify launch. */
struct xfg_kargs {
	struct xfg_tdesc t4, t6, te;
	const uint8_t *port_flags;
	unsigned long long *port_hits;
	uint32_t port_count;          /* ports with non-zero flags; 0 => skip */
	uint32_t window;              /* header window staged in LDS (64 or 128) */
	unsigned long long *stats;    /* [XFG_ACTION_MAX][2] {packets, bytes} */
	const uint8_t *data;
	const uint64_t *offsets;
	const void *lens;
	uint64_t n;
	uint32_t stride;
	uint32_t lens_u16;
	uint8_t *verdicts;
	uint32_t ablate;              /* diagnostics only (XFG_ABLATE env), 0 in production:
				       * 2 = no counter atomics, 4 = stage only (no parse) */
};

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
#define XFG_HD __host__ __device__ __forceinline__
#else
#define XFG_HD static inline
#endif

XFG_HD uint32_t xfg_fmix32(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

XFG_HD uint32_t xfg_hash_v4(uint32_t k, uint32_t seed)
{
	return xfg_fmix32(k ^ seed);
}

XFG_HD uint32_t xfg_hash_v6(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t seed)
{
	uint32_t h = xfg_fmix32(w0 ^ seed);
	h = xfg_fmix32(h ^ w1);
	h = xfg_fmix32(h ^ w2);
	return xfg_fmix32(h ^ w3);
}

XFG_HD uint32_t xfg_hash_eth(uint64_t mac, uint32_t seed)
{
	uint32_t h = xfg_fmix32((uint32_t)mac ^ seed);
	return xfg_fmix32(h ^ (uint32_t)(mac >> 32));
}

XFG_HD uint32_t xfg_home(uint32_t h, uint32_t nbuckets)
{
	return (uint32_t)(((uint64_t)h * nbuckets) >> 32);
}

#endif /* XFG_LAYOUT_H */
