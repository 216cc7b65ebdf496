/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xfg_io.c — host formats around the classifier (include/xdpfilter_io.h):
 * pcap/pcapng ingest, the pcapng verdict dump, and the persistent rule store
 * that stands in for the bpffs pin directory.  Plain C over the public C ABI
 * (include/xdpfilter_gpu.h); nothing here touches HIP.
 */
#define _GNU_SOURCE
#include "xdpfilter_io.h"

#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

/* ------------------------------------------------------------------ batch */
struct hb {
	struct xfg_host_batch b;
	uint64_t cap_pkts, cap_bytes;
};

static int hb_reserve(struct hb *h, uint64_t pkts, uint64_t bytes)
{
	if (pkts > h->cap_pkts) {
		uint64_t n = h->cap_pkts ? h->cap_pkts : 1024;
		while (n < pkts)
			n *= 2;
		uint64_t *o = realloc(h->b.offsets, n * 8);
		if (o)
			h->b.offsets = o;
		uint32_t *l = realloc(h->b.lens, n * 4);
		if (l)
			h->b.lens = l;
		uint32_t *ol = realloc(h->b.orig_lens, n * 4);
		if (ol)
			h->b.orig_lens = ol;
		uint64_t *t = realloc(h->b.ts_ns, n * 8);
		if (t)
			h->b.ts_ns = t;
		if (!o || !l || !ol || !t)
			return -ENOMEM;
		h->cap_pkts = n;
	}
	if (bytes > h->cap_bytes) {
		uint64_t n = h->cap_bytes ? h->cap_bytes : 1 << 20;
		while (n < bytes)
			n *= 2;
		uint8_t *d = realloc(h->b.data, n);
		if (!d)
			return -ENOMEM;
		h->b.data = d;
		h->cap_bytes = n;
	}
	return 0;
}

/* Append one frame at the next 16-byte boundary, zero-padded to it, and keep
 * 16 spare zero bytes at the end so every frame is readable to the next
 * boundary past its end (struct xfg_batch's rule). */
static int hb_add(struct hb *h, const uint8_t *p, uint32_t caplen, uint32_t origlen, uint64_t ts)
{
	uint64_t off = h->b.bytes;
	uint64_t span = ((uint64_t)caplen + 15) & ~15ull;
	int err = hb_reserve(h, h->b.count + 1, off + span + 16);
	if (err)
		return err;
	memcpy(h->b.data + off, p, caplen);
	memset(h->b.data + off + caplen, 0, span - caplen + 16);
	h->b.offsets[h->b.count] = off;
	h->b.lens[h->b.count] = caplen;
	h->b.orig_lens[h->b.count] = origlen;
	h->b.ts_ns[h->b.count] = ts;
	h->b.count++;
	h->b.bytes = off + span;
	return 0;
}

void xfg_host_batch_free(struct xfg_host_batch *b)
{
	if (!b)
		return;
	free(b->data);
	free(b->offsets);
	free(b->lens);
	free(b->orig_lens);
	free(b->ts_ns);
	memset(b, 0, sizeof(*b));
}

static int read_file(const char *path, uint8_t **buf, size_t *len)
{
	FILE *f = fopen(path, "rb");
	if (!f)
		return -errno;
	if (fseek(f, 0, SEEK_END) || ftell(f) < 0) {
		fclose(f);
		return -EIO;
	}
	size_t n = (size_t)ftell(f);
	rewind(f);
	uint8_t *p = malloc(n ? n : 1);
	if (!p) {
		fclose(f);
		return -ENOMEM;
	}
	if (n && fread(p, 1, n, f) != n) {
		free(p);
		fclose(f);
		return -EIO;
	}
	fclose(f);
	*buf = p;
	*len = n;
	return 0;
}

static uint32_t rd32(const uint8_t *p, int swap)
{
	uint32_t v;
	memcpy(&v, p, 4);
	return swap ? __builtin_bswap32(v) : v;
}

static uint16_t rd16(const uint8_t *p, int swap)
{
	uint16_t v;
	memcpy(&v, p, 2);
	return swap ? __builtin_bswap16(v) : v;
}

#define MAX_SNAP (256u * 1024u)
#define LINKTYPE_ETHERNET 1u

/* classic libpcap: 24-byte file header, 16-byte record headers */
static int parse_pcap(const uint8_t *f, size_t n, struct hb *h)
{
	uint32_t magic;
	memcpy(&magic, f, 4);
	int swap = magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u;
	int nsec = magic == 0xa1b23c4du || magic == 0x4d3cb2a1u;
	if (n < 24)
		return -EINVAL;
	uint32_t link = rd32(f + 20, swap) & 0x0fffffff;
	if (link != LINKTYPE_ETHERNET)
		return -EPROTONOSUPPORT;
	h->b.linktype = link;
	size_t o = 24;
	while (o < n) {
		if (n - o < 16)
			return -EINVAL;
		uint32_t sec = rd32(f + o, swap), frac = rd32(f + o + 4, swap);
		uint32_t cap = rd32(f + o + 8, swap), orig = rd32(f + o + 12, swap);
		o += 16;
		if (cap > MAX_SNAP || cap > n - o)
			return -EINVAL;
		uint64_t ts = (uint64_t)sec * 1000000000ull + (nsec ? frac : (uint64_t)frac * 1000ull);
		int err = hb_add(h, f + o, cap, orig, ts);
		if (err)
			return err;
		o += cap;
	}
	return 0;
}

/* pcapng: blocks {type, total_len, body, total_len}; per-section byte order */
#define NG_SHB 0x0A0D0D0Au
#define NG_IDB 1u
#define NG_OPB 2u
#define NG_SPB 3u
#define NG_EPB 6u
#define NG_MAX_IF 64

struct ng_if {
	uint32_t link, snap;
	uint64_t tsdiv_num, tsdiv_den;   /* ns = ts * num / den */
};

static void ng_tsresol(struct ng_if *i, uint8_t r)
{
	/* default 10^-6; bit 7 set: 2^-(r & 0x7f), else 10^-r */
	uint64_t per_sec;
	if (r & 0x80) {
		uint32_t e = r & 0x7f;
		per_sec = e < 63 ? 1ull << e : 1ull << 62;
	} else {
		per_sec = 1;
		for (uint32_t k = 0; k < r && k < 19; k++)
			per_sec *= 10;
	}
	i->tsdiv_num = 1000000000ull;
	i->tsdiv_den = per_sec;
}

static uint64_t ng_ns(const struct ng_if *i, uint64_t ts)
{
	if (i->tsdiv_den == i->tsdiv_num)
		return ts;
	if (i->tsdiv_den < i->tsdiv_num)
		return ts * (i->tsdiv_num / i->tsdiv_den);
	return ts / (i->tsdiv_den / i->tsdiv_num);
}

static int parse_pcapng(const uint8_t *f, size_t n, struct hb *h)
{
	struct ng_if ifs[NG_MAX_IF];
	uint32_t nif = 0;
	int swap = 0, seen_shb = 0;
	size_t o = 0;
	while (o < n) {
		if (n - o < 12)
			return -EINVAL;
		uint32_t type;
		memcpy(&type, f + o, 4);
		if (type == NG_SHB) {
			uint32_t bom;
			memcpy(&bom, f + o + 8, 4);
			if (bom == 0x1A2B3C4Du)
				swap = 0;
			else if (bom == 0x4D3C2B1Au)
				swap = 1;
			else
				return -EINVAL;
			nif = 0;   /* interface ids are per section */
			seen_shb = 1;
		} else if (!seen_shb) {
			return -EINVAL;
		}
		uint32_t blen = rd32(f + o + 4, swap);
		if (blen < 12 || (blen & 3) || blen > n - o)
			return -EINVAL;
		const uint8_t *body = f + o + 8;
		uint32_t bl = blen - 12;
		if (type != NG_SHB)
			type = rd32(f + o, swap);
		if (type == NG_IDB) {
			if (bl < 8 || nif >= NG_MAX_IF)
				return -EINVAL;
			struct ng_if *i = &ifs[nif++];
			i->link = rd16(body, swap);
			i->snap = rd32(body + 4, swap);
			ng_tsresol(i, 6);
			/* options: if_tsresol (9) */
			uint32_t p = 8;
			while (p + 4 <= bl) {
				uint16_t code = rd16(body + p, swap), ol = rd16(body + p + 2, swap);
				if (code == 0)
					break;
				if (p + 4 + ol > bl)
					return -EINVAL;
				if (code == 9 && ol >= 1)
					ng_tsresol(i, body[p + 4]);
				p += 4 + ((ol + 3u) & ~3u);
			}
		} else if (type == NG_EPB || type == NG_OPB) {
			uint32_t ifid, cap, orig;
			uint64_t ts;
			const uint8_t *pkt;
			if (type == NG_EPB) {
				if (bl < 20)
					return -EINVAL;
				ifid = rd32(body, swap);
				ts = ((uint64_t)rd32(body + 4, swap) << 32) | rd32(body + 8, swap);
				cap = rd32(body + 12, swap);
				orig = rd32(body + 16, swap);
				pkt = body + 20;
				if (cap > bl - 20)
					return -EINVAL;
			} else {
				if (bl < 20)
					return -EINVAL;
				ifid = rd16(body, swap);
				ts = ((uint64_t)rd32(body + 4, swap) << 32) | rd32(body + 8, swap);
				cap = rd32(body + 12, swap);
				orig = rd32(body + 16, swap);
				pkt = body + 20;
				if (cap > bl - 20)
					return -EINVAL;
			}
			if (ifid >= nif || cap > MAX_SNAP)
				return -EINVAL;
			if (ifs[ifid].link != LINKTYPE_ETHERNET)
				return -EPROTONOSUPPORT;
			int err = hb_add(h, pkt, cap, orig, ng_ns(&ifs[ifid], ts));
			if (err)
				return err;
		} else if (type == NG_SPB) {
			if (bl < 4 || nif < 1)
				return -EINVAL;
			if (ifs[0].link != LINKTYPE_ETHERNET)
				return -EPROTONOSUPPORT;
			uint32_t orig = rd32(body, swap);
			uint32_t cap = orig;
			if (ifs[0].snap && cap > ifs[0].snap)
				cap = ifs[0].snap;
			if (cap > bl - 4)
				cap = bl - 4;
			if (cap > MAX_SNAP)
				return -EINVAL;
			int err = hb_add(h, body + 4, cap, orig, 0);
			if (err)
				return err;
		}
		/* other block types (NRB, ISB, DSB, custom) carry no packets */
		o += blen;
	}
	h->b.linktype = LINKTYPE_ETHERNET;
	return 0;
}

int xfg_pcap_read(const char *path, struct xfg_host_batch *out)
{
	uint8_t *f = NULL;
	size_t n = 0;
	struct hb h;
	int err;

	if (!path || !out)
		return -EINVAL;
	memset(out, 0, sizeof(*out));
	memset(&h, 0, sizeof(h));
	if ((err = read_file(path, &f, &n)))
		return err;
	if (n < 4) {
		free(f);
		return -EINVAL;
	}
	uint32_t magic;
	memcpy(&magic, f, 4);
	if (magic == 0xa1b2c3d4u || magic == 0xd4c3b2a1u || magic == 0xa1b23c4du ||
	    magic == 0x4d3cb2a1u)
		err = parse_pcap(f, n, &h);
	else if (magic == NG_SHB)
		err = parse_pcapng(f, n, &h);
	else
		err = -EINVAL;
	free(f);
	if (!err && !h.b.data)   /* empty capture: still a valid batch */
		err = hb_reserve(&h, 1, 16);
	if (err) {
		xfg_host_batch_free(&h.b);
		return err;
	}
	*out = h.b;
	return 0;
}

/* ------------------------------------------------------------------ pcapng out */
struct wbuf {
	FILE *f;
	int err;
};

static void w_raw(struct wbuf *w, const void *p, size_t n)
{
	if (!w->err && n && fwrite(p, 1, n, w->f) != n)
		w->err = -EIO;
}

static void w32(struct wbuf *w, uint32_t v) { w_raw(w, &v, 4); }
static void w16(struct wbuf *w, uint16_t v) { w_raw(w, &v, 2); }

static void w_opt(struct wbuf *w, uint16_t code, const void *p, uint16_t len)
{
	static const uint8_t zero[4];
	w16(w, code);
	w16(w, len);
	w_raw(w, p, len);
	w_raw(w, zero, (4 - (len & 3)) & 3);
}

static uint32_t opt_len(size_t len) { return 4 + (((uint32_t)len + 3) & ~3u); }

int xfg_pcapng_write_verdicts(const char *path, const char *ifname,
			      const struct xfg_host_batch *b, const uint8_t *verdicts)
{
	static const uint8_t zero[4];
	static const char appl[] = "xdp-filter (MI355X classifier)";
	if (!path || !b || (!verdicts && b->count))
		return -EINVAL;
	struct wbuf w = { fopen(path, "wb"), 0 };
	if (!w.f)
		return -errno;
	setvbuf(w.f, NULL, _IOFBF, 1 << 20);
	const char *name = ifname ? ifname : "xdp";

	/* SHB: byte-order magic, version 1.0, section length unknown */
	uint32_t shb_len = 28 + opt_len(sizeof(appl) - 1) + 4;
	w32(&w, NG_SHB);
	w32(&w, shb_len);
	w32(&w, 0x1A2B3C4Du);
	w16(&w, 1);
	w16(&w, 0);
	uint64_t seclen = ~0ull;
	w_raw(&w, &seclen, 8);
	w_opt(&w, 4, appl, sizeof(appl) - 1);            /* shb_userappl */
	w32(&w, 0);                                     /* opt_endofopt */
	w32(&w, shb_len);

	/* IDB: Ethernet, if_name, if_tsresol = 9 (ns) */
	uint8_t tsres = 9;
	uint32_t idb_len = 20 + opt_len(strlen(name)) + opt_len(1) + 4;
	w32(&w, NG_IDB);
	w32(&w, idb_len);
	w16(&w, LINKTYPE_ETHERNET);
	w16(&w, 0);
	w32(&w, 0);                                     /* snaplen: none */
	w_opt(&w, 2, name, (uint16_t)strlen(name));     /* if_name */
	w_opt(&w, 9, &tsres, 1);                        /* if_tsresol */
	w32(&w, 0);
	w32(&w, idb_len);

	/* EPBs with epb_verdict (code 7): type 2 = eBPF XDP, then the u64
	 * verdict (lib/util/xpcapng.c:155-161, 400-404, 470-474) */
	for (uint64_t i = 0; i < b->count && !w.err; i++) {
		uint32_t cap = b->lens[i];
		uint32_t orig = b->orig_lens ? b->orig_lens[i] : cap;
		uint64_t ts = b->ts_ns ? b->ts_ns[i] : 0;
		uint8_t vopt[9];
		uint64_t v = verdicts[i];
		vopt[0] = 2;
		memcpy(vopt + 1, &v, 8);
		uint32_t pad = ((cap + 3) & ~3u) - cap;
		uint32_t len = 32 + cap + pad + opt_len(sizeof(vopt)) + 4;
		w32(&w, NG_EPB);
		w32(&w, len);
		w32(&w, 0);                             /* interface 0 */
		w32(&w, (uint32_t)(ts >> 32));
		w32(&w, (uint32_t)ts);
		w32(&w, cap);
		w32(&w, orig);
		w_raw(&w, b->data + (b->offsets ? b->offsets[i] : 0), cap);
		w_raw(&w, zero, pad);
		w_opt(&w, 7, vopt, sizeof(vopt));
		w32(&w, 0);
		w32(&w, len);
	}
	if (fclose(w.f) && !w.err)
		w.err = -EIO;
	return w.err;
}

/* ------------------------------------------------------------------ rule store */
/*
 * One file per map, named like the pinned BPF map:
 *   header { char magic[8] = "XFGMAP1"; u32 map; u32 keylen; u32 capacity;
 *            u32 reserved; u64 count }
 *   count records { key[keylen]; u64 value }   value = hits << 6 | flags
 * xdp_stats_map: { char magic[8] = "XFGSTA1"; 5 x {u64 packets, u64 bytes} }.
 */
#define STORE_MAGIC "XFGMAP1"
#define STATS_MAGIC "XFGSTA1"

struct store_hdr {
	char magic[8];
	uint32_t map;
	uint32_t keylen;
	uint32_t capacity;
	uint32_t reserved;
	uint64_t count;
};

static const char *map_names[XFG_MAP_NUM] = {
	XFG_STORE_MAP_PORTS, XFG_STORE_MAP_IPV4, XFG_STORE_MAP_IPV6, XFG_STORE_MAP_ETHERNET,
};
static const uint32_t map_keylen[XFG_MAP_NUM] = { 4, 4, 16, 6 };

const char *xfg_store_map_name(int map)
{
	return map >= 0 && map < XFG_MAP_NUM ? map_names[map] : NULL;
}

static int map_path(char *buf, size_t n, const char *dir, const char *name)
{
	int r = snprintf(buf, n, "%s/%s", dir, name);
	return r < 0 || (size_t)r >= n ? -ENAMETOOLONG : 0;
}

int xfg_store_has_map(const char *dir, int map)
{
	char p[4096];
	if (!dir || !xfg_store_map_name(map) || map_path(p, sizeof(p), dir, map_names[map]))
		return 0;
	return access(p, F_OK) == 0;
}

static int read_hdr(const char *dir, int map, struct store_hdr *h, FILE **fp)
{
	char p[4096];
	int err = map_path(p, sizeof(p), dir, map_names[map]);
	if (err)
		return err;
	FILE *f = fopen(p, "rb");
	if (!f)
		return -errno;
	if (fread(h, sizeof(*h), 1, f) != 1 || memcmp(h->magic, STORE_MAGIC, 8) ||
	    h->map != (uint32_t)map || h->keylen != map_keylen[map]) {
		fclose(f);
		return -EINVAL;
	}
	if (fp)
		*fp = f;
	else
		fclose(f);
	return 0;
}

/* Write @n records to <dir>/<name> through a temporary file + rename. */
static int write_map(const char *dir, int map, uint32_t capacity, const uint8_t *keys,
		     const uint64_t *vals, uint64_t n)
{
	char p[4096], tmp[4200];
	int err = map_path(p, sizeof(p), dir, map_names[map]);
	if (err)
		return err;
	snprintf(tmp, sizeof(tmp), "%s.tmp.%d", p, (int)getpid());
	FILE *f = fopen(tmp, "wb");
	if (!f)
		return -errno;
	setvbuf(f, NULL, _IOFBF, 1 << 20);
	struct store_hdr h;
	memset(&h, 0, sizeof(h));
	memcpy(h.magic, STORE_MAGIC, 8);
	h.map = (uint32_t)map;
	h.keylen = map_keylen[map];
	h.capacity = capacity;
	h.count = n;
	int ok = fwrite(&h, sizeof(h), 1, f) == 1;
	for (uint64_t i = 0; ok && i < n; i++)
		ok = fwrite(keys + (size_t)h.keylen * i, h.keylen, 1, f) == 1 &&
		     fwrite(&vals[i], 8, 1, f) == 1;
	if (fclose(f))
		ok = 0;
	if (!ok || rename(tmp, p)) {
		unlink(tmp);
		return -EIO;
	}
	return 0;
}

int xfg_store_create_map(const char *dir, int map, uint32_t capacity)
{
	if (!dir || !xfg_store_map_name(map))
		return -EINVAL;
	if (xfg_store_has_map(dir, map))
		return 0;
	if (map == XFG_MAP_PORTS)
		capacity = XFG_PORT_MAP_ENTRIES;
	return write_map(dir, map, capacity ? capacity : XFG_DEFAULT_MAP_CAPACITY, NULL, NULL, 0);
}

int xfg_store_remove_map(const char *dir, int map)
{
	char p[4096];
	if (!dir || !xfg_store_map_name(map))
		return -EINVAL;
	int err = map_path(p, sizeof(p), dir, map_names[map]);
	if (err)
		return err;
	if (unlink(p) && errno != ENOENT)
		return -errno;
	return 0;
}

int64_t xfg_store_map_capacity(const char *dir, int map)
{
	struct store_hdr h;
	if (!dir || !xfg_store_map_name(map))
		return -EINVAL;
	int err = read_hdr(dir, map, &h, NULL);
	return err ? err : (int64_t)h.capacity;
}

int xfg_store_load(xfg_ctx *ctx, const char *dir)
{
	if (!ctx || !dir)
		return -EINVAL;
	int nv = xfg_num_devices(ctx);
	if (nv < 1)
		nv = 1;
	for (int map = 0; map < XFG_MAP_NUM; map++) {
		struct store_hdr h;
		FILE *f = NULL;
		int err = read_hdr(dir, map, &h, &f);
		if (err == -ENOENT)
			continue;
		if (err)
			return err;
		if (h.count > (1ull << 32)) {
			fclose(f);
			return -EINVAL;
		}
		uint8_t *keys = malloc(h.count * h.keylen + 1);
		uint64_t *vals = malloc(h.count * 8 * nv + 8);
		int ok = keys && vals;
		for (uint64_t i = 0; ok && i < h.count; i++) {
			uint64_t v;
			ok = fread(keys + (size_t)h.keylen * i, h.keylen, 1, f) == 1 &&
			     fread(&v, 8, 1, f) == 1;
			/* device 0 carries the saved hits, the others the flags */
			vals[i * nv] = v;
			for (int d = 1; d < nv; d++)
				vals[i * nv + d] = v & (uint64_t)((1u << XFG_COUNTER_SHIFT) - 1);
		}
		fclose(f);
		err = ok ? 0 : (keys && vals ? -EINVAL : -ENOMEM);
		if (!err && h.count)
			err = xfg_map_update_batch_percpu(ctx, map, keys, vals, h.count);
		free(keys);
		free(vals);
		if (err)
			return err;
	}
	return 0;
}

/* Keys and summed values of one map of @ctx. */
static int collect(xfg_ctx *ctx, int map, uint8_t **keys_out, uint64_t **vals_out, uint64_t *n_out)
{
	int nv = xfg_num_devices(ctx);
	if (nv < 1)
		nv = 1;
	uint32_t kl = map_keylen[map];
	uint64_t cap = map == XFG_MAP_PORTS ? XFG_PORT_MAP_ENTRIES : 1024, n = 0;
	uint8_t *keys = NULL;
	uint64_t *all = NULL, *vals = NULL;
	int err = 0;

	if (map == XFG_MAP_PORTS) {
		keys = malloc((size_t)cap * kl);
		if (!keys)
			return -ENOMEM;
		for (uint32_t k = 0; k < XFG_PORT_MAP_ENTRIES; k++)
			memcpy(keys + 4ull * k, &k, 4);
		n = cap;
	} else {
		keys = malloc((size_t)cap * kl);
		if (!keys)
			return -ENOMEM;
		uint8_t prev[16], next[16];
		const void *pk = NULL;
		for (;;) {
			int r = xfg_map_get_next_key(ctx, map, pk, next);
			if (r == -ENOENT)
				break;
			if (r) {
				err = r;
				goto fail;
			}
			if (n == cap) {
				uint8_t *nk = realloc(keys, (size_t)cap * 2 * kl);
				if (!nk) {
					err = -ENOMEM;
					goto fail;
				}
				keys = nk;
				cap *= 2;
			}
			memcpy(keys + (size_t)n * kl, next, kl);
			memcpy(prev, next, kl);
			pk = prev;
			n++;
		}
	}
	all = malloc((n ? n : 1) * 8 * nv);
	vals = malloc((n ? n : 1) * 8);
	if (!all || !vals) {
		err = -ENOMEM;
		goto fail;
	}
	if (n) {
		int64_t r = xfg_map_lookup_batch(ctx, map, keys, n, all, NULL);
		if (r < 0) {
			err = (int)r;
			goto fail;
		}
	}
	/* sum hits over devices, flags from device 0 (map_get_counter_flags) */
	uint64_t m = 0;
	for (uint64_t i = 0; i < n; i++) {
		uint64_t hits = 0, v0 = all[i * nv];
		for (int d = 0; d < nv; d++)
			hits += all[i * nv + d] >> XFG_COUNTER_SHIFT;
		uint64_t v = (hits << XFG_COUNTER_SHIFT) | (v0 & ((1u << XFG_COUNTER_SHIFT) - 1));
		if (map == XFG_MAP_PORTS && !v)
			continue;   /* array slots that were never set */
		if (m != i)
			memmove(keys + (size_t)m * kl, keys + (size_t)i * kl, kl);
		vals[m++] = v;
	}
	free(all);
	*keys_out = keys;
	*vals_out = vals;
	*n_out = m;
	return 0;
fail:
	free(keys);
	free(all);
	free(vals);
	return err;
}

int xfg_store_save(xfg_ctx *ctx, const char *dir)
{
	if (!ctx || !dir)
		return -EINVAL;
	for (int map = 0; map < XFG_MAP_NUM; map++) {
		struct store_hdr h;
		int err = read_hdr(dir, map, &h, NULL);
		if (err == -ENOENT)
			continue;   /* not pinned: this program does not use the map */
		if (err)
			return err;
		uint8_t *keys = NULL;
		uint64_t *vals = NULL, n = 0;
		if ((err = collect(ctx, map, &keys, &vals, &n)))
			return err;
		err = write_map(dir, map, h.capacity, keys, vals, n);
		free(keys);
		free(vals);
		if (err)
			return err;
	}
	return 0;
}

int xfg_store_stats_read(const char *dir, struct xfg_stats_record out[XFG_ACTION_MAX])
{
	char p[4096], magic[8];
	if (!dir || !out)
		return -EINVAL;
	int err = map_path(p, sizeof(p), dir, XFG_STORE_MAP_STATS);
	if (err)
		return err;
	FILE *f = fopen(p, "rb");
	if (!f)
		return -errno;
	int ok = fread(magic, 8, 1, f) == 1 && !memcmp(magic, STATS_MAGIC, 8) &&
		 fread(out, sizeof(*out), XFG_ACTION_MAX, f) == XFG_ACTION_MAX;
	fclose(f);
	return ok ? 0 : -EINVAL;
}

int xfg_store_stats_write(const char *dir, const struct xfg_stats_record in[XFG_ACTION_MAX])
{
	char p[4096], tmp[4200];
	if (!dir || !in)
		return -EINVAL;
	int err = map_path(p, sizeof(p), dir, XFG_STORE_MAP_STATS);
	if (err)
		return err;
	snprintf(tmp, sizeof(tmp), "%s.tmp.%d", p, (int)getpid());
	FILE *f = fopen(tmp, "wb");
	if (!f)
		return -errno;
	int ok = fwrite(STATS_MAGIC, 8, 1, f) == 1 &&
		 fwrite(in, sizeof(*in), XFG_ACTION_MAX, f) == XFG_ACTION_MAX;
	if (fclose(f))
		ok = 0;
	if (!ok || rename(tmp, p)) {
		unlink(tmp);
		return -EIO;
	}
	return 0;
}

int xfg_store_stats_remove(const char *dir)
{
	char p[4096];
	if (!dir)
		return -EINVAL;
	int err = map_path(p, sizeof(p), dir, XFG_STORE_MAP_STATS);
	if (err)
		return err;
	if (unlink(p) && errno != ENOENT)
		return -errno;
	return 0;
}
