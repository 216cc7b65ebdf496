/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xfg_layout.h — device-resident table layout shared by the host runtime (C)
 * and the HIP kernels.  Nothing here is part of the public C ABI.
 *
 * The reference's BPF_MAP_TYPE_PERCPU_HASH maps (filter_ipv4/ipv6/ethernet,
 * xdp-filter/xdpfilt_prog.h:113-185) become bucketed open-addressed tables,
 * one 64-byte line per bucket so that ONE random read answers a probe:
 *
 *   bytes  0..47  keys   ipv4: 12 x u32 | ipv6: 3 x 16 B | ethernet: 6 x u64
 *                        (MAC in the low 48 bits, little-endian byte copy)
 *   bytes 48..59  flags  one byte per slot: low 6 bits of the reference
 *                        value (MAP_FLAG_* and the two spare bits)
 *   bytes 60..63  meta   bit0 = overflow: a key whose probe sequence passed
 *                        this bucket was placed further on
 *
 * An all-zero key marks an empty slot; the all-zero KEY itself lives in the
 * extra bucket `nbuckets` (slot nslots = nbuckets * slots_per_bucket), which
 * hashing never reaches.  Key bytes are identical on every device (slot
 * indices agree across devices); flag bytes are per device, like the
 * reference's per-CPU values.
 *
 *   hits  [nslots+1] u64   reference value >> COUNTER_SHIFT, per device
 *
 * so the reference value is exactly (hits << 6) | flags, and a hit's
 * `*value += 1 << COUNTER_SHIFT` (xdp-filter/xdpfilt_prog.h:60-61) becomes
 * hits += 1.  Keeping hits apart from flags lets the multi-GPU reduction sum
 * counters directly (ncclUint64) without disturbing the flag bits.
 *
 * Probing: home bucket from a 32-bit murmur3-finaliser chain (multiplicative
 * range reduction), then linear over buckets; a lookup stops at a bucket
 * whose overflow bit is clear or after max_disp+1 buckets.  Keys never move
 * once placed, so slot indices (and the per-device counters) are stable
 * across inserts and deletes.
 *
 * Prefilter: a blocked Bloom filter of 32-bit words (one word per key, 4
 * bits from a second hash) answers most negative lookups from a table small
 * enough to stay in each XCD's L2.  Deleted keys leave their bits set
 * (false positives only; the bucket probe decides), and the host rebuilds
 * the filter when stale bits accumulate.
 *
 * Quotient index ("QT", xfg_table.h xfg_qt): a derived, read-only index of
 * the IPv4 map that answers a lookup with ONE random 32-byte read (two
 * 16-byte loads of one line by the packet's own lane) and no prefilter, for
 * the pipelined IPv4-key kernel when exactly one lookup direction can hit.
 * h = xfg_qt_hash(key) is a bijection of the 32-bit key, so (bucket = h >>
 * (32 - bits), remainder = h's low 32 - bits <= 15 bits) identifies the key
 * exactly.  A bucket is 16 u16 entries filled in order: 0 = empty, else
 * 0x8000 | remainder.  A bucket that more than 16 keys home in holds 15 of
 * them and, as entry 15, the overflow marker 0x0001 (no lookup's 0x8000 |
 * remainder equals it): a miss there is decided by the canonical table
 * instead (the kernel defers it); a miss in a bucket of exactly 16 is
 * final.  Only keys whose flags carry the one live mask are
 * indexed: any other key cannot hit this lookup, exactly as an absent one.
 * QT slot bucket * 16 + entry maps back to the canonical slot through
 * trans[] (the count kernel's job).  What a tile's lookups cost is set by
 * the random LINES they touch (tools/mb_vm.hip, profiles/archive/r03_mb_vm*.log:
 * 64 lines per 64-packet tile add ~0.25 ms per 2^26 packets to the frame
 * stream, 32 lines 0.07, 16 lines 0.02; a table of 0.5-4 MB the same), so
 * a bucket is one line's worth, and 16 entries at < 8 keys per bucket
 * keep the deferred share near 0.3 % of the misses.
 *
 * filter_ports (PERCPU_ARRAY[65536], :67-73) is dense: flags[65536] u8 and
 * hits[65536] u64 indexed by the raw big-endian port value, plus a 65536-bit
 * "any flag set" bitmap that each workgroup stages in LDS.
 */
#ifndef XFG_LAYOUT_H
#define XFG_LAYOUT_H

#include <stdint.h>

#define XFG_BUCKET_BYTES  64u
#define XFG_KEY_AREA      48u
#define XFG_FLAGS_OFF     48u
#define XFG_META_OFF      60u
#define XFG_SLOTS_V4      12u
#define XFG_SLOTS_V6      3u
#define XFG_SLOTS_ETH     6u

#define XFG_META_OVERFLOW 1u

#define XFG_PORT_TAB      2048u   /* LDS port table slots (8 KiB, the bitmap's size) */
#define XFG_PORT_TAB_MAX  1024u   /* at most this many ruled ports use the table */
#define XFG_PORT_NIB_WORDS 8192u  /* more: every port's 4 flag bits, 32 KiB of LDS */

#define XFG_BLOOM_K       4u
#define XFG_BLOOM_LDS_MAX 4096u   /* Bloom words a generic pipelined workgroup stages in LDS (16 KiB) */

#define XFG_QT_SLOTS      16u     /* entries per 32-byte QT bucket */
#define XFG_QT_BUCKET     32u
#ifndef XFG_QT_MIN_BITS   /* (A/B builds only: below 17 a remainder loses bits, timing-only) */
#define XFG_QT_MIN_BITS   17u     /* remainders of at most 15 bits */
#endif
#define XFG_QT_LOAD       8u      /* fewer keys per bucket than this on average */
#define XFG_QT_USED       0x8000u /* an occupied entry */
#define XFG_QT_OVF_MARK   0x0001u /* entry 15: the bucket overflowed */

#define XFG_DCNT_MAX      4096u   /* direct LDS counters (16 KiB) */
#define XFG_EK_SLOTS_MAX  1024u   /* Ethernet-key kernel: LDS key table entries (16 KiB) */
#define XFG_EK_MAX_KEYS   512u    /* ... at most this many keys (half the entries) */
#define XFG_EK_VALID      0x100u  /* an occupied entry (beside the flag byte) */
#define XFG_LOG_PARTS     256u    /* hit-log partitions (16-counter chunks dealt round-robin) */
#define XFG_LOG_HIST_MAX  16384u  /* count-kernel LDS histogram entries (64 KiB) */
#define XFG_CW_HIST_MAX   8192u   /* the QT kernel's count-wave histogram entries (32 KiB) */
#define XFG_CW_LOG_MIN    (1ull << 20)   /* packets from which the count wave's log runs */
#define XFG_CW_MAX_PACKETS (1ull << 25)   /* ... and below which it does */
#define XFG_QT_DYN_MIN    (1ull << 23)   /* packets from which the QT waves take tiles as they go */
#define XFG_LOG_PASSES_MAX 32u    /* histogram passes per partition (span 512K) */
#define XFG_LOG_SLICES_MAX 1024u  /* slices per partition: classify workgroups */
#define XFG_DEFER_SRC_MAX 4096u   /* deferred lists (classify waves) xfg_defer_kernel takes */
#define XFG_LOG_MIN_KEYS  256u    /* fewer hash-map keys: LDS counter cache, no log */


/* Per-hash-map descriptor passed to the kernel by value. */
struct xfg_tdesc {
	const void *buckets;         /* (nbuckets + 1) * 64 B */
	const uint32_t *bloom;       /* bloom_words x u32 */
	unsigned long long *hits;    /* nslots + 1 */
	uint32_t nbuckets;
	uint32_t max_disp;
	uint32_t count;              /* keys present; 0 => lookups can never hit */
	uint32_t zero_present;       /* the all-zero key is present (slot nslots) */
	uint32_t nslots;
	uint32_t seed;
	uint32_t bloom_words;        /* 0 => no prefilter */
	uint32_t fmask;              /* OR of every key's flag bits on any device: a
				      * lookup whose mask is not covered cannot hit */
};

/* Kernel arguments of one classify launch. */
struct xfg_kargs {
	struct xfg_tdesc t4, t6, te;
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
	uint32_t port_fmask;          /* OR of the port flag bytes (see tdesc.fmask) */
	/* The ruled ports, as each workgroup copies them to LDS: a small
	 * open-addressed table (at most XFG_PORT_TAB_MAX ports carry flags), or
	 * else (port_tab NULL) the nibble map of all 65536 ports' flags */
	const uint32_t *port_tab;     /* XFG_PORT_TAB entries: flags << 16 | key, 0 = empty */
	uint32_t port_tab_disp;       /* longest probe displacement in the table */
	const uint32_t *port_nib;     /* XFG_PORT_NIB_WORDS: port k's flags at bits 4(k%8) of word k/8 */
	/* Global counter index space (counter identities): v4 slots, v6 slots,
	 * eth slots (each with its zero-key slot), then the 65536 ports;
	 * gbase[i] = first index of each. */
	uint32_t gbase[4];
	/* AF_XDP descriptors (xfg_classify_descs): packet i is record
	 * (desc_first + i) & desc_mask of an array of struct xdp_desc {u64 addr;
	 * u32 len; u32 options} (headers/linux/if_xdp.h:110-114) over the UMEM at
	 * `data`; NULL for the other layouts */
	const uint64_t *descs;
	uint32_t desc_mask;
	uint32_t desc_first;
	uint32_t dense;               /* pipelined kernel: stride == window */
	uint32_t pipe;                /* the pipelined kernel (fixed stride >= window) */
	uint32_t km;                  /* pipelined key mode: 1 = only IPv4 keys are live */
	/* quotient-index kernel with IPv6 keys live (no Ethernet key): every IPv6
	 * frame goes to the deferred path, the IPv4 lookups through the index */
	uint32_t v6d;
	/* ... and (v6p) their lookups in the kernel's loop, with one IPv4
	 * lookup direction live: 1 = one IPv6 direction live, 2 = both */
	uint32_t v6p;
	/* Direct LDS counters: identities below dcnt (all hash maps, gbase[3],
	 * or the IPv4 map, gbase[1]) are summed per workgroup in LDS; 0 = off */
	uint32_t dcnt;
	/* The generic pipelined kernel's Bloom words in LDS, past the direct
	 * counters: bl_lds words in all, bl_off[i] the first of table i (t4,
	 * te, t6; ~0u: not staged) -- when every live map's filter fits in
	 * XFG_BLOOM_LDS_MAX words (C1's 10,000-entry Ethernet map: 3,750); 0 =
	 * the words read from memory */
	uint32_t bl_lds;
	uint32_t bl_off[3];
	/* The Ethernet map as an LDS key table (a map of at most
	 * XFG_EK_MAX_KEYS keys whose flags agree on every device; the
	 * Ethernet-key kernel, the generic pipelined kernel, the index kernel):
	 * an open-addressed table of ek_slots (a power of two) 16-byte entries
	 * {MAC bytes 0-3, bytes 4-5, slot, flags | XFG_EK_VALID}, copied to LDS
	 * by every workgroup; a key sits at most ek_disp entries past its home
	 * (xfg_ek_home with the map's seed).  NULL: no table. */
	const uint32_t *ek;
	uint32_t ek_slots;
	uint32_t ek_disp;
	/* Hit log of the pipelined kernels (tlog NULL = no log): per-wave
	 * regions of defer_cap counter identities; partition-major buffer of
	 * XFG_LOG_PARTS x pslices slices of pcap entries, slice (p, b) owned by
	 * classify workgroup b (pslices = the classify grid), its entry count in
	 * pfill[p * pslices + b] (written, not accumulated: no reservation
	 * atomics); the count kernel's LDS histogram has log_hist entries
	 * (xfg_kernels.hip, HitLog). */
	uint32_t *tlog;
	uint16_t *pbuf;               /* local indices (log_local: the partition implied) */
	uint32_t *pfill;
	uint32_t pcap;
	uint32_t pslices;
	/* this launch's first slice of each partition (slices pslice0 ..
	 * pslice0 + grid - 1: the quotient-index kernel's logs of up to
	 * pslices / grid launches share the buffers, counted together) and
	 * the count kernel's slices to read (pfirst .. pfirst + pcount - 1) */
	uint32_t pslice0;
	uint32_t pcount;
	uint32_t pfirst;
	uint32_t log_hist;
	/* a partition's local-index range (log_span) beyond one histogram: the
	 * count kernel takes it in passes of log_hist (one workgroup per
	 * partition and pass); past 65536 the slices hold u32 indices (pwide) */
	uint32_t log_span;
	uint32_t pwide;
	/* Pipelined kernel: deferred packets, defer_cap entries per wave.  With
	 * defer_sep the quotient-index kernel only lists them (its fill per wave
	 * in defer_n, defer_nsrc waves) and xfg_defer_kernel, defer_grid
	 * workgroups, classifies them after it, spread over the whole chip
	 * instead of each wave's serial tail */
	uint32_t *defer;
	uint32_t defer_cap;
	uint32_t *defer_n;
	uint32_t defer_nsrc;
	uint32_t defer_sep;
	uint32_t defer_grid;
	uint32_t diag;                /* diagnostics build only (XFG_DIAG_MASK); 0 */
	/* diagnostics build only (XFG_TSTAMP): the quotient-index kernel's phase
	 * times, 32 wall-clock stamps a workgroup (xfg_pipeq.hip QT_STAMP); NULL */
	unsigned long long *tstamp;
	/* quotient-index kernel: a workgroup's waves take its tiles from an LDS
	 * counter (XFG_QT_DYN) -- batches of at least XFG_QT_DYN_MIN packets */
	uint32_t qt_dyn;
	/* Header-window batches (xfg_classify_host): each slot holds only the
	 * first `stride` bytes of its frame, lens are the frames' true lengths.
	 * A packet whose program reads past the window is not classified here:
	 * its index goes to fb (fb_cnt entries, at most fb_cap) and it is
	 * counted nowhere; the host classifies it again from the whole frame. */
	uint32_t hwin;                /* 1 = header-window batch; 0 = whole frames */
	uint32_t fb_cap;
	uint32_t *fb;
	uint32_t *fb_cnt;
	/* Split IPv4-key classify (diagnostics build, xfg_split.hip): the parse
	 * pass (grid_parse workgroups) writes per-packet records -- a state byte
	 * in the verdict buffer, the first live key, the ports (dst | src << 16)
	 * and, with both directions live, the second key -- that the lookup pass
	 * reads.  bloom_off: the lookup pass goes to the bucket line without the
	 * prefilter (one live key per packet only). */
	uint32_t split;
	uint32_t grid_parse;
	uint32_t bloom_off;
	uint32_t *rec_ka, *rec_kb, *rec_port;
	/* Quotient index of the IPv4 map (NULL = none): 1 << qt_bits buckets
	 * per image; QT slot bucket * 16 + entry of image 0 (at qt), and
	 * qt_base + bucket * 16 + entry of the second lookup's image (at qt2),
	 * mapped to canonical slots by qt_trans.  qt_live: the live mask, 2
	 * (dst) or 1 (src) for one lookup, 3 for both (dst in image 0, src in
	 * qt2: image 1, or image 0 itself with qt_base 0 when every ruled key
	 * carries both directions) */
	const uint32_t *qt;
	const uint32_t *qt2;
	const uint32_t *qt_trans;
	/* hit counts of the QT slots (qt_n, QT-slot order): the count kernel
	 * adds there, the host folds them into the canonical counters through
	 * qt_trans before any counter read, write or re-index (the per-CPU
	 * counters of BPF are summed at readout the same way); 32-bit: the
	 * host folds them too before the packets classified since the last
	 * fold could reach 2^32 (a packet bumps at most one), which keeps the
	 * array half the size -- C5's 2^25 QT slots in 128 MB, inside the
	 * Infinity Cache -- for the kernels' atomics */
	uint32_t *qt_hits;
	uint32_t qt_bits;
	uint32_t qt_seed;
	uint32_t qt_base;
	uint32_t qt_n;
	uint32_t qt_live;
	/* where the QT kernel's counts that bypass the hit log go -- a full
	 * LDS ring, a chunk past its slice, the LDS counter cache's QT
	 * entries, no log at all -- by atomics: the second half of the
	 * allocation (qt_hits + qt_n), folded like the first, so that the
	 * counts the log brings (the count kernel's, the count wave's) are
	 * read-modify-writes no atomic races */
	uint32_t *qt_hitx;
	/* the count wave (the QT kernel's ninth wave, cw_n != 0): this
	 * launch's workgroups count the previous launch's log -- its cw_n
	 * slices from cw_s0 of every partition they own -- into qt_hits while
	 * their other waves classify, hiding the count kernel; this launch's
	 * own slices start at pslice0 (the other of two sets) */
	uint32_t cw_n;
	uint32_t cw_s0;
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

/* The LDS key table's home entry of a MAC (lo: bytes 0-3, hi: bytes 4-5)
 * in a table of 2^lg entries: multiply-shift over the MAC's two 24-bit
 * halves, the top lg bits of the sum.  Only 24-bit multiplies (full rate on
 * the vector ALU, where xfg_hash_eth's four 32-bit ones are quarter rate):
 * every frame probes both of its MACs, so this is on the per-packet path. */
XFG_HD uint32_t xfg_ek_home(uint32_t lo, uint32_t hi, uint32_t seed, uint32_t lg)
{
	const uint32_t a = (lo ^ seed) & 0xffffffu;
	const uint32_t b = ((lo >> 24) | (hi << 8)) ^ (seed >> 8);
	const uint32_t h = a * 0x9e3779u + (b & 0xffffffu) * 0x7f4a7bu;
	return h >> (32 - lg);
}

XFG_HD uint32_t xfg_home(uint32_t h, uint32_t nbuckets)
{
	return (uint32_t)(((uint64_t)h * nbuckets) >> 32);
}

/* Bloom filter: word index from the key hash h (a different range
 * reduction than the bucket's: the high-multiply of a re-mixed value), and
 * XFG_BLOOM_K bit positions from a second finaliser round. */
XFG_HD uint32_t xfg_bloom_word(uint32_t h, uint32_t nwords)
{
	return (uint32_t)(((uint64_t)(h * 0x9E3779B1u) * nwords) >> 32);
}

XFG_HD uint32_t xfg_bloom_mask(uint32_t h)
{
	uint32_t g = xfg_fmix32(h ^ 0x7f4a7c15u);
	return (1u << (g & 31)) | (1u << ((g >> 5) & 31)) | (1u << ((g >> 10) & 31)) |
	       (1u << ((g >> 15) & 31));
}

/* The QT index's key hash: a bijection of the 32-bit key (xor with the
 * seed, then the murmur3 finaliser: each step is invertible). */
XFG_HD uint32_t xfg_qt_hash(uint32_t k, uint32_t seed)
{
	return xfg_fmix32(k ^ seed);
}

/* Home slot of a port key in the LDS port table. */
XFG_HD uint32_t xfg_port_slot(uint32_t key)
{
	return (key * 0x9E3779B1u) >> 21;   /* 11 bits: XFG_PORT_TAB slots */
}

#endif /* XFG_LAYOUT_H */
