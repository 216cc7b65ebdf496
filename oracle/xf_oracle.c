/* oracle/xf_oracle.c — CPU restatement of xdp-filter's per-packet path.
 *
 * TEST INFRASTRUCTURE ONLY (see xf_oracle.h).  One function parameterised by
 * the program's feature word replaces the ten compile-time variants
 * xdp-filter/xdpfilt_{alw,dny}_{all,eth,ip,tcp,udp}.c.  Every step cites the
 * reference line it restates (reference v1.6.3 under /root/reference).
 * Bounds checks are written as "offset + size > len" on byte offsets, which
 * is exactly the verifier-style "ptr + 1 > data_end" checks of
 * headers/xdp/parsing_helpers.h.
 */
#include "xf_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define F_TCP   (1u << 0)
#define F_UDP   (1u << 1)
#define F_IPV6  (1u << 2)
#define F_IPV4  (1u << 3)
#define F_ETH   (1u << 4)
#define F_DENY  (1u << 6)

#define M_SRC 1u
#define M_DST 2u
#define M_TCP 4u
#define M_UDP 8u

enum { ABORTED = 0, DROP = 1, PASS = 2 };

/* ---------------- exact-match index (sorted keys + binary search) -------- */
struct xfo_map {
	uint32_t n, keylen;
	const uint8_t *keys;
	uint32_t *order; /* rule indices sorted by key bytes */
	/* Optional hash index (xfo_map_new_hashed): open addressing, linear
	 * probing, load <= 1/2; slot = fingerprint << 32 | flags << 26 |
	 * (index + 1), 0 = empty, where flags is the rule's flag byte (low 6
	 * bits of its value) when the index was built: one cache line answers
	 * a miss and a flag mismatch, as the reference's hash element holds its
	 * key and value together.  For 4-byte keys the fingerprint IS the key.
	 * It gives the restatement the reference's cost model -- one hash probe
	 * per CHECK_MAP (BPF_MAP_TYPE_PERCPU_HASH, xdp-filter/xdpfilt_prog.h:56-64)
	 * -- for the CPU baseline; the binary search stays the checker's index. */
	uint64_t *slots;
	uint64_t smask;
};

static inline uint32_t fmix32(uint32_t h)
{
	h ^= h >> 16;
	h *= 0x85ebca6bu;
	h ^= h >> 13;
	h *= 0xc2b2ae35u;
	h ^= h >> 16;
	return h;
}

static inline uint32_t key_hash(const uint8_t *k, uint32_t len)
{
	uint32_t h = 0x9747b28cu ^ len;
	uint32_t i = 0;
	for (; i + 4 <= len; i += 4) {
		uint32_t w;
		memcpy(&w, k + i, 4);
		h = fmix32(h ^ w);
	}
	if (i < len) {
		uint32_t w = 0;
		memcpy(&w, k + i, len - i);
		h = fmix32(h ^ w);
	}
	return h;
}

static inline uint32_t key_fp(const uint8_t *k, uint32_t len, uint32_t h)
{
	uint32_t w;
	if (len == 4) {
		memcpy(&w, k, 4);
		return w;
	}
	return h;
}

static const uint8_t *g_sort_keys;
static uint32_t g_sort_len;

static int cmp_idx(const void *a, const void *b)
{
	uint32_t i = *(const uint32_t *)a, j = *(const uint32_t *)b;
	int c = memcmp(g_sort_keys + (size_t)i * g_sort_len,
		       g_sort_keys + (size_t)j * g_sort_len, g_sort_len);
	if (c)
		return c;
	return i < j ? -1 : i > j; /* stable: first occurrence of a key wins */
}

xfo_map *xfo_map_new(uint32_t n, uint32_t keylen, const uint8_t *keys)
{
	static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
	xfo_map *m = calloc(1, sizeof(*m));
	if (!m)
		return NULL;
	m->n = n;
	m->keylen = keylen;
	m->keys = keys;
	m->order = malloc(sizeof(uint32_t) * (n ? n : 1));
	if (!m->order) {
		free(m);
		return NULL;
	}
	for (uint32_t i = 0; i < n; i++)
		m->order[i] = i;
	pthread_mutex_lock(&mu);
	g_sort_keys = keys;
	g_sort_len = keylen;
	qsort(m->order, n, sizeof(uint32_t), cmp_idx);
	pthread_mutex_unlock(&mu);
	return m;
}

#define SLOT_IDX(e) ((uint32_t)((e) & ((1u << 26) - 1)) - 1)
#define SLOT_FLAGS(e) ((uint32_t)((e) >> 26) & 63)

xfo_map *xfo_map_new_hashed(uint32_t n, uint32_t keylen, const uint8_t *keys,
			    const uint64_t *vals)
{
	if (n >= (1u << 26) - 1)
		return NULL;
	xfo_map *m = xfo_map_new(n, keylen, keys);
	if (!m)
		return NULL;
	uint64_t cap = 16;
	while (cap < 2ull * n)
		cap <<= 1;
	m->slots = calloc(cap, sizeof(uint64_t));
	if (!m->slots) {
		xfo_map_free(m);
		return NULL;
	}
	m->smask = cap - 1;
	for (uint32_t i = 0; i < n; i++) {   /* index order: the first occurrence wins */
		const uint8_t *k = keys + (size_t)i * keylen;
		const uint32_t h = key_hash(k, keylen), fp = key_fp(k, keylen, h);
		uint64_t j = h & m->smask;
		int dup = 0;
		while (m->slots[j]) {
			const uint64_t e = m->slots[j];
			if ((uint32_t)(e >> 32) == fp &&
			    !memcmp(keys + (size_t)SLOT_IDX(e) * keylen, k, keylen)) {
				dup = 1;
				break;
			}
			j = (j + 1) & m->smask;
		}
		if (!dup)
			m->slots[j] = ((uint64_t)fp << 32) | ((uint64_t)(vals[i] & 63) << 26) | (i + 1u);
	}
	return m;
}

void xfo_map_free(xfo_map *m)
{
	if (m) {
		free(m->order);
		free(m->slots);
		free(m);
	}
}

/* Returns the rule index holding @key, or -1 (BPF hash lookup -> NULL). */
static int64_t map_find(const xfo_map *m, const uint8_t *key)
{
	if (!m || !m->n)
		return -1;
	uint32_t lo = 0, hi = m->n;
	while (lo < hi) {
		uint32_t mid = lo + (hi - lo) / 2;
		int c = memcmp(m->keys + (size_t)m->order[mid] * m->keylen, key, m->keylen);
		if (c < 0)
			lo = mid + 1;
		else
			hi = mid;
	}
	if (lo < m->n && !memcmp(m->keys + (size_t)m->order[lo] * m->keylen, key, m->keylen))
		return m->order[lo];
	return -1;
}

/* ---------------- the per-packet program --------------------------------- */
static inline uint32_t be16(const uint8_t *p, uint32_t o) { return ((uint32_t)p[o] << 8) | p[o + 1]; }
static inline uint32_t raw16(const uint8_t *p, uint32_t o) { return p[o] | ((uint32_t)p[o + 1] << 8); }

struct run_state {
	uint32_t feat;
	uint64_t *ports;
	const xfo_map *m4, *m6, *me;
	uint64_t *v4, *v6, *ve;
};

/* CHECK_MAP, xdp-filter/xdpfilt_prog.h:56-64: hit iff the key exists and
 * (value & mask) == mask; a hit adds 1 << COUNTER_SHIFT to that value. */
/* The hashed index's probe: the slot of @key, or 0. */
static inline uint64_t hash_probe(const xfo_map *m, const uint8_t *key)
{
	const uint32_t h = key_hash(key, m->keylen), fp = key_fp(key, m->keylen, h);
	for (uint64_t j = h & m->smask;; j = (j + 1) & m->smask) {
		const uint64_t e = m->slots[j];
		if (!e || ((uint32_t)(e >> 32) == fp &&
			   (m->keylen == 4 || !memcmp(m->keys + (size_t)SLOT_IDX(e) * m->keylen, key, m->keylen))))
			return e;
	}
}

static inline int check_hash(const xfo_map *m, uint64_t *vals, const uint8_t *key, uint32_t mask)
{
	if (m && m->slots) {
		/* one probe; the rule's value is touched only when its flags
		 * (as indexed) carry the mask -- then it is the authority */
		if (!m->n)
			return 0;
		const uint64_t e = hash_probe(m, key);
		if (!e || (SLOT_FLAGS(e) & mask) != mask)
			return 0;
		const uint32_t i = SLOT_IDX(e);
		if ((vals[i] & mask) != mask)
			return 0;
		vals[i] += 1u << 6;
		return 1;
	}
	int64_t i = map_find(m, key);
	if (i >= 0 && (vals[i] & mask) == mask) {
		vals[i] += 1u << 6;
		return 1;
	}
	return 0;
}

static inline int check_port(uint64_t *ports, uint32_t key, uint32_t mask)
{
	if ((ports[key] & mask) == mask) {   /* PERCPU_ARRAY: every key exists */
		ports[key] += 1u << 6;
		return 1;
	}
	return 0;
}

/* lookup_verdict_ipv4/ipv6, xdp-filter/xdpfilt_prog.h:121-134 / :152-165:
 * dst first (mask DST), then src (mask SRC); NULL arguments skipped. */
static int v4_hit(const struct run_state *s, const uint8_t *src, const uint8_t *dst)
{
	if (dst && check_hash(s->m4, s->v4, dst, M_DST))
		return 1;
	if (src && check_hash(s->m4, s->v4, src, M_SRC))
		return 1;
	return 0;
}

static int v6_hit(const struct run_state *s, const uint8_t *src, const uint8_t *dst)
{
	if (dst && check_hash(s->m6, s->v6, dst, M_DST))
		return 1;
	if (src && check_hash(s->m6, s->v6, src, M_SRC))
		return 1;
	return 0;
}

/* One packet: xdp-filter/xdpfilt_prog.h:214-310. */
static uint32_t classify_one(const struct run_state *s, const uint8_t *p, uint32_t len)
{
	const uint32_t f = s->feat;
	const uint32_t hit = (f & F_DENY) ? PASS : DROP;   /* VERDICT_HIT, :26-34 */
	const uint32_t miss = (f & F_DENY) ? DROP : PASS;  /* VERDICT_MISS */
	uint32_t off, proto, ip_type = 0, l4 = 0;

	/* parse_ethhdr, headers/xdp/parsing_helpers.h:100-134 */
	if (14 > len)
		return ABORTED;
	proto = be16(p, 12);
	off = 14;
	for (int i = 0; i < 4; i++) {            /* VLAN_MAX_DEPTH = 4, :79-81 */
		if (proto != 0x8100 && proto != 0x88A8)
			break;
		if (off + 4 > len)
			break;
		proto = be16(p, off + 2);
		off += 4;
	}

	/* lookup_verdict_ethernet, xdp-filter/xdpfilt_prog.h:187-196 */
	if (f & F_ETH) {
		if (check_hash(s->me, s->ve, p + 0, M_DST) ||
		    check_hash(s->me, s->ve, p + 6, M_SRC))
			return hit;
	}

	if (!(f & (F_IPV4 | F_IPV6 | F_TCP | F_UDP)))    /* :229-230 */
		return miss;

	if (proto == 0x0800) {
		/* __parse_iphdr(frags_ok=1), parsing_helpers.h:201-227 */
		if (off + 20 > len)
			return ABORTED;
		uint32_t hdrsize = (p[off] & 0xF) * 4;
		if (off + hdrsize > len)
			return ABORTED;
		ip_type = p[off + 9];
		l4 = off + hdrsize;
		if ((f & F_IPV4) && v4_hit(s, p + off + 12, p + off + 16))   /* :239 */
			return hit;
	} else if (proto == 0x0806 && (f & F_IPV4)) {
		/* parse_arphdr, parsing_helpers.h:235-253; xdpfilt_prog.h:241-261 */
		if (off + 28 > len)
			return ABORTED;
		if (be16(p, off) != 1 || be16(p, off + 2) != 0x0800 ||
		    p[off + 4] != 6 || p[off + 5] != 4)
			return ABORTED;
		uint32_t op = be16(p, off + 6);
		const uint8_t *sip = p + off + 14, *tip = p + off + 24;
		if (v4_hit(s, sip, NULL))
			return hit;
		if (op == 1) {            /* ARPOP_REQUEST: target is a DST */
			if (v4_hit(s, NULL, tip))
				return hit;
		} else if (op == 2) {     /* ARPOP_REPLY: target is a SRC */
			if (v4_hit(s, tip, NULL))
				return hit;
		}
		/* ip_type stays 0: no L4 step */
	} else if (proto == 0x86DD) {
		/* __parse_ip6hdr + skip_ip6hdrext, parsing_helpers.h:136-199 */
		if (off + 40 > len)
			return ABORTED;
		uint32_t nh = p[off + 6];
		const uint8_t *saddr = p + off + 8, *daddr = p + off + 24;
		uint32_t cur = off + 40;
		int done = 0;
		for (int i = 0; i < 6 && !done; i++) {   /* IPV6_EXT_MAX_CHAIN = 6 */
			if (cur + 2 > len)
				return ABORTED;
			switch (nh) {
			case 0: case 60: case 43: case 135:   /* HOPOPTS DSTOPTS ROUTING MH */
				nh = p[cur];
				cur += (p[cur + 1] + 1u) * 8;
				break;
			case 51:                               /* AH */
				nh = p[cur];
				cur += (p[cur + 1] + 2u) * 4;
				break;
			case 44:                               /* FRAGMENT (frags_ok) */
				nh = p[cur];
				cur += 8;
				break;
			default:
				done = 1;
			}
		}
		if (!done)
			return ABORTED;
		ip_type = nh;
		l4 = cur;
		if ((f & F_IPV6) && v6_hit(s, saddr, daddr))        /* :266 */
			return hit;
		if (ip_type == 58) {
			/* parse_icmp6hdr, parsing_helpers.h:255-268; NDISC :268-287 */
			if (cur + 8 > len)
				return ABORTED;
			uint32_t t = p[cur];
			cur += 8;
			if (t == 135 || t == 136) {
				if (cur + 16 > len)
					return ABORTED;
				if (f & F_IPV6) {
					if (t == 135 ? v6_hit(s, NULL, p + cur)
						     : v6_hit(s, p + cur, NULL))
						return hit;
				}
			}
		}
	} else {
		return miss;                                         /* :288-290 */
	}

	if ((f & F_UDP) && ip_type == 17) {
		/* parse_udphdr, parsing_helpers.h:303-321 */
		if (l4 + 8 > len)
			return ABORTED;
		if (be16(p, l4 + 4) < 8)
			return ABORTED;
		/* lookup_verdict_udp, xdpfilt_prog.h:92-101 */
		if (check_port(s->ports, raw16(p, l4 + 2), M_DST | M_UDP) ||
		    check_port(s->ports, raw16(p, l4 + 0), M_SRC | M_UDP))
			return hit;
	}
	if ((f & F_TCP) && ip_type == 6) {
		/* parse_tcphdr, parsing_helpers.h:326-344 */
		if (l4 + 20 > len)
			return ABORTED;
		if (l4 + (p[l4 + 12] >> 4) * 4u > len)
			return ABORTED;
		/* lookup_verdict_tcp, xdpfilt_prog.h:76-85 */
		if (check_port(s->ports, raw16(p, l4 + 2), M_DST | M_TCP) ||
		    check_port(s->ports, raw16(p, l4 + 0), M_SRC | M_TCP))
			return hit;
	}
	return miss;
}

int xfo_run(uint32_t features, const uint8_t *data, const uint64_t *offsets,
	    uint32_t stride, const void *lens, int lens_u16, uint64_t n,
	    uint64_t *ports, const xfo_map *m4, uint64_t *v4,
	    const xfo_map *m6, uint64_t *v6, const xfo_map *me, uint64_t *ve,
	    uint8_t *verdicts, uint64_t *stats)
{
	struct run_state s = { features, ports, m4, m6, me, v4, v6, ve };
	for (uint64_t i = 0; i < n; i++) {
		const uint8_t *p = data + (offsets ? offsets[i] : i * (uint64_t)stride);
		uint32_t len = lens_u16 ? ((const uint16_t *)lens)[i] : ((const uint32_t *)lens)[i];
		uint32_t a = classify_one(&s, p, len);
		verdicts[i] = (uint8_t)a;
		/* xdp_stats_record_action, headers/xdp/xdp_stats_kern.h:29-48 */
		stats[2 * a] += 1;
		stats[2 * a + 1] += len;
	}
	return 0;
}

/* ---------------- per-CPU-style multithreaded run ------------------------ */
struct mt_arg {
	uint32_t features;
	const uint8_t *data;
	const uint64_t *offsets;
	uint32_t stride;
	const void *lens;
	int lens_u16;
	uint64_t begin, end;
	const xfo_map *m4, *m6, *me;
	uint64_t *ports, *v4, *v6, *ve, stats[10];
	uint8_t *verdicts;
	int err;
};

static void *mt_worker(void *p)
{
	struct mt_arg *a = p;
	const void *lens = a->lens_u16 ? (const void *)((const uint16_t *)a->lens + a->begin)
				       : (const void *)((const uint32_t *)a->lens + a->begin);
	a->err = xfo_run(a->features, a->data, a->offsets ? a->offsets + a->begin : NULL,
			 a->stride, lens, a->lens_u16, a->end - a->begin,
			 a->ports, a->m4, a->v4, a->m6, a->v6, a->me, a->ve,
			 a->verdicts + a->begin, a->stats);
	return NULL;
}

int xfo_run_mt(uint32_t features, const uint8_t *data, const uint64_t *offsets,
	       uint32_t stride, const void *lens, int lens_u16, uint64_t n,
	       uint64_t *ports, const xfo_map *m4, uint64_t *v4, uint32_t n4,
	       const xfo_map *m6, uint64_t *v6, uint32_t n6,
	       const xfo_map *me, uint64_t *ve, uint32_t ne,
	       uint8_t *verdicts, uint64_t *stats, int nthreads)
{
	if (nthreads < 1)
		nthreads = 1;
	struct mt_arg *args = calloc(nthreads, sizeof(*args));
	pthread_t *th = calloc(nthreads, sizeof(*th));
	int err = 0;
	if (!args || !th) {
		free(args);
		free(th);
		return -1;
	}
	for (int t = 0; t < nthreads; t++) {
		struct mt_arg *a = &args[t];
		a->features = features;
		a->data = offsets ? data : data + (n * t / nthreads) * (uint64_t)stride;
		a->offsets = offsets;
		a->stride = stride;
		a->lens = lens;
		a->lens_u16 = lens_u16;
		a->begin = n * t / nthreads;
		a->end = n * (t + 1) / nthreads;
		a->m4 = m4; a->m6 = m6; a->me = me;
		/* private "per-CPU" values: flags copied, counters start at 0 */
		a->ports = malloc(sizeof(uint64_t) * 65536);
		a->v4 = malloc(sizeof(uint64_t) * (n4 ? n4 : 1));
		a->v6 = malloc(sizeof(uint64_t) * (n6 ? n6 : 1));
		a->ve = malloc(sizeof(uint64_t) * (ne ? ne : 1));
		if (!a->ports || !a->v4 || !a->v6 || !a->ve) {
			err = -1;
			nthreads = t + 1;
			break;
		}
		for (uint32_t i = 0; i < 65536; i++) a->ports[i] = ports[i] & 63;
		for (uint32_t i = 0; i < n4; i++) a->v4[i] = v4[i] & 63;
		for (uint32_t i = 0; i < n6; i++) a->v6[i] = v6[i] & 63;
		for (uint32_t i = 0; i < ne; i++) a->ve[i] = ve[i] & 63;
		a->verdicts = verdicts;
	}
	/* The worker computes data+offsets for its slice itself; when no
	 * offsets are given data is pre-advanced to the slice start. */
	if (!err) {
		for (int t = 0; t < nthreads; t++)
			pthread_create(&th[t], NULL, mt_worker, &args[t]);
		for (int t = 0; t < nthreads; t++)
			pthread_join(th[t], NULL);
		for (int t = 0; t < nthreads; t++) {
			struct mt_arg *a = &args[t];
			err |= a->err;
			for (uint32_t i = 0; i < 65536; i++) ports[i] += a->ports[i] & ~63ull;
			for (uint32_t i = 0; i < n4; i++) v4[i] += a->v4[i] & ~63ull;
			for (uint32_t i = 0; i < n6; i++) v6[i] += a->v6[i] & ~63ull;
			for (uint32_t i = 0; i < ne; i++) ve[i] += a->ve[i] & ~63ull;
			for (int k = 0; k < 10; k++) stats[k] += a->stats[k];
		}
	}
	for (int t = 0; t < nthreads; t++) {
		free(args[t].ports); free(args[t].v4); free(args[t].v6); free(args[t].ve);
	}
	free(args);
	free(th);
	return err ? -1 : 0;
}
