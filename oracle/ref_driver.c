/* oracle/ref_driver.c — TEST INFRASTRUCTURE ONLY (never shipped, never the
 * thing measured as the product).
 *
 * Wraps ONE unmodified reference variant (xdp-filter/xdpfilt_<VARIANT>.c,
 * which expands xdp-filter/xdpfilt_prog.h:214-310) as a host C function so
 * its per-packet verdicts, per-rule counters and per-action stats can be
 * compared bit-for-bit with the HIP path.  Built by oracle/Makefile into
 * oracle/_ref/libxfref_<variant>.so, one shared object per variant because
 * the map symbols (filter_ipv4, xdp_stats_map, ...) collide across TUs.
 *
 * Map model (the only third-party behaviour on the path): the kernel's
 * PERCPU_HASH (kernel/bpf/hashtab.c) is exact-match on key bytes and returns
 * NULL when absent; PERCPU_ARRAY (kernel/bpf/arraymap.c) returns the slot for
 * any in-range index.  One "CPU" is modelled, so each rule has one u64 value.
 * Frames are copied into MAP_32BIT memory because struct xdp_md carries
 * 32-bit data/data_end (headers/linux/bpf.h, struct xdp_md).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#ifndef XFREF_VARIANT_FILE
#error "build with -DXFREF_VARIANT_FILE=\"/root/reference/xdp-filter/xdpfilt_xxx.c\""
#endif
#include XFREF_VARIANT_FILE

#define XSTR(x) #x
#define STR(x) XSTR(x)

/* ---- exact-match index over a caller-owned rule list ------------------- */
struct xidx {
	uint32_t n, keylen, mask;
	const uint8_t *keys;   /* n * keylen bytes */
	uint64_t *vals;        /* n values (in/out) */
	int64_t *slots;        /* open addressing, -1 = empty */
};

static uint64_t fnv(const uint8_t *k, uint32_t len)
{
	uint64_t h = 1469598103934665603ull;
	for (uint32_t i = 0; i < len; i++)
		h = (h ^ k[i]) * 1099511628211ull;
	return h ^ (h >> 29);
}

static int g_cache_index;   /* xfref_cache_index(1): timing loops over one rule list */

void xfref_cache_index(int on) { g_cache_index = on; }

static int xidx_build(struct xidx *x, uint32_t n, uint32_t keylen,
		      const uint8_t *keys, uint64_t *vals)
{
	uint32_t cap = 16;
	if (g_cache_index && x->slots && x->keys == keys && x->n == n && x->keylen == keylen) {
		x->vals = vals;   /* same rule list as the previous call: reuse the index */
		return 0;
	}
	free(x->slots);
	x->slots = NULL;
	while (cap < 2 * n + 16)
		cap <<= 1;
	x->n = n; x->keylen = keylen; x->mask = cap - 1;
	x->keys = keys; x->vals = vals;
	x->slots = malloc(sizeof(int64_t) * cap);
	if (!x->slots)
		return -1;
	for (uint32_t i = 0; i < cap; i++)
		x->slots[i] = -1;
	for (uint32_t i = 0; i < n; i++) {
		uint32_t s = (uint32_t)fnv(keys + (size_t)i * keylen, keylen) & x->mask;
		for (;; s = (s + 1) & x->mask) {
			int64_t j = x->slots[s];
			if (j < 0) { x->slots[s] = i; break; }
			if (!memcmp(keys + (size_t)j * keylen, keys + (size_t)i * keylen, keylen))
				break; /* duplicate key: first occurrence wins */
		}
	}
	return 0;
}

static uint64_t *xidx_find(const struct xidx *x, const void *key)
{
	if (!x->n)
		return NULL;
	uint32_t s = (uint32_t)fnv(key, x->keylen) & x->mask;
	for (;; s = (s + 1) & x->mask) {
		int64_t j = x->slots[s];
		if (j < 0)
			return NULL;
		if (!memcmp(x->keys + (size_t)j * x->keylen, key, x->keylen))
			return &x->vals[j];
	}
}

static struct xidx g_v4, g_v6, g_eth;
static uint64_t *g_ports;                   /* 65536 values */
static struct xdp_stats_record *g_stats;    /* XDP_ACTION_MAX records */

void *xfref_host_map_lookup(const void *map, const void *key)
{
	uint32_t k32;
	if (map == (const void *)&xdp_stats_map) {
		memcpy(&k32, key, 4);
		return k32 < XDP_ACTION_MAX ? (void *)&g_stats[k32] : NULL;
	}
#if defined(FILT_MODE_TCP) || defined(FILT_MODE_UDP)
	if (map == (const void *)&filter_ports) {
		memcpy(&k32, key, 4);
		return k32 < 65536 ? (void *)&g_ports[k32] : NULL;
	}
#endif
#ifdef FILT_MODE_IPV4
	if (map == (const void *)&filter_ipv4)
		return xidx_find(&g_v4, key);
#endif
#ifdef FILT_MODE_IPV6
	if (map == (const void *)&filter_ipv6)
		return xidx_find(&g_v6, key);
#endif
#ifdef FILT_MODE_ETHERNET
	if (map == (const void *)&filter_ethernet)
		return xidx_find(&g_eth, key);
#endif
	return NULL;
}

const char *xfref_name(void) { return STR(FUNCNAME); }
uint32_t xfref_features(void) { return _features; }

/* Run the reference program over a batch.
 *   data/offsets/lens: packet i = data[offsets ? offsets[i] : i*stride], lens[i] bytes
 *   ports: 65536 values (PERCPU_ARRAY filter_ports, key = raw be16 port)
 *   n4/k4/v4, n6/k6/v6, ne/ke/ve: hash-map rule lists (4/16/6-byte keys), values in/out
 *   verdicts: out, one byte per packet; stats: in/out, 5 x {packets, bytes}
 * Returns 0, or -1 on allocation failure. */
int xfref_run(const uint8_t *data, const uint64_t *offsets, uint32_t stride,
	      const uint32_t *lens, uint64_t n, uint64_t *ports,
	      uint32_t n4, const uint8_t *k4, uint64_t *v4,
	      uint32_t n6, const uint8_t *k6, uint64_t *v6,
	      uint32_t ne, const uint8_t *ke, uint64_t *ve,
	      uint8_t *verdicts, uint64_t *stats)
{
	static uint8_t *arena;
	const size_t arena_sz = 1 << 17;
	int ret = -1;

	if (!arena) {
		arena = mmap(NULL, arena_sz, PROT_READ | PROT_WRITE,
			     MAP_PRIVATE | MAP_ANONYMOUS | MAP_32BIT, -1, 0);
		if (arena == MAP_FAILED) {
			arena = NULL;
			return -1;
		}
	}
	if (xidx_build(&g_v4, n4, 4, k4, v4) || xidx_build(&g_v6, n6, 16, k6, v6) ||
	    xidx_build(&g_eth, ne, 6, ke, ve))
		goto out;
	g_ports = ports;
	g_stats = (struct xdp_stats_record *)stats;

	for (uint64_t i = 0; i < n; i++) {
		const uint8_t *p = data + (offsets ? offsets[i] : i * (uint64_t)stride);
		uint32_t len = lens[i];
		struct xdp_md ctx;

		if ((uintptr_t)p + len < (1ull << 32)) {
			/* caller's buffer already lies below 4 GiB: run in place */
			ctx.data = (uint32_t)(uintptr_t)p;
			ctx.data_end = (uint32_t)((uintptr_t)p + len);
		} else {
			if (len > arena_sz)
				goto out;
			memcpy(arena, p, len);
			ctx.data = (uint32_t)(uintptr_t)arena;
			ctx.data_end = (uint32_t)(uintptr_t)(arena + len);
		}
		verdicts[i] = (uint8_t)FUNCNAME(&ctx);
	}
	ret = 0;
out:
	return ret;
}
