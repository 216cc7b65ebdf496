/* SPDX-License-Identifier: GPL-2.0 */
/* xfg_table.c — host side of the device hash tables (see xfg_layout.h). */
#include "xfg_table.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

/* Target load factors per key type (slots per bucket 12 / 3 / 6): with
 * 12-slot buckets at 0.6 about 3% of buckets overflow at full capacity. */
static uint32_t buckets_for(uint32_t capacity, uint32_t spb)
{
	double lf = spb >= 12 ? 0.6 : (spb >= 6 ? 0.55 : 0.45);
#ifdef XFG_DIAG
	const char *e = spb >= 12 ? getenv("XFG_LF4") : NULL;   /* diagnostics build only */
	if (e && atof(e) > 0.1 && atof(e) < 0.95)
		lf = atof(e);
#endif
	uint64_t nb = (uint64_t)((double)capacity / (spb * lf)) + 1;
	if (nb > 0x7fffffffull / spb - 1)
		nb = 0x7fffffffull / spb - 1;
	return (uint32_t)nb;
}

int xfg_table_init(struct xfg_table *t, uint32_t keylen, uint32_t capacity, uint32_t seed)
{
	memset(t, 0, sizeof(*t));
	switch (keylen) {
	case 4:  t->slot_bytes = 4;  t->slots_per_bucket = XFG_SLOTS_V4; break;
	case 16: t->slot_bytes = 16; t->slots_per_bucket = XFG_SLOTS_V6; break;
	case 6:  t->slot_bytes = 8;  t->slots_per_bucket = XFG_SLOTS_ETH; break;
	default: return -EINVAL;
	}
	if (!capacity)
		return -EINVAL;
	t->keylen = keylen;
	t->capacity = capacity;
	t->seed = seed;
	t->nbuckets = buckets_for(capacity, t->slots_per_bucket);
	t->nslots = t->nbuckets * t->slots_per_bucket;
	if (t->nslots >= (1u << 30))   /* kernel counter tags carry 30-bit slots */
		return -E2BIG;
	/* ~12 filter bits per key: a 1M-rule filter is 1.5 MB (L2-resident) */
	uint64_t words = ((uint64_t)capacity * 12 + 31) / 32;
	t->bloom_words = (uint32_t)(words < 32 ? 32 : words);
	t->img = calloc(xfg_table_img_bytes(t), 1);
	t->bloom = calloc(t->bloom_words, 4);
	if (!t->img || !t->bloom) {
		xfg_table_free(t);
		return -ENOMEM;
	}
	return 0;
}

void xfg_table_free(struct xfg_table *t)
{
	free(t->img);
	free(t->bloom);
	t->img = NULL;
	t->bloom = NULL;
}

static void stored_key(const struct xfg_table *t, const void *key, uint8_t *out)
{
	memset(out, 0, 16);
	memcpy(out, key, t->keylen);
}

static int is_zero(const uint8_t *k, uint32_t n)
{
	for (uint32_t i = 0; i < n; i++)
		if (k[i])
			return 0;
	return 1;
}

static uint32_t key_hash(const struct xfg_table *t, const uint8_t *sk)
{
	if (t->keylen == 4) {
		uint32_t k;
		memcpy(&k, sk, 4);
		return xfg_hash_v4(k, t->seed);
	} else if (t->keylen == 16) {
		uint32_t w[4];
		memcpy(w, sk, 16);
		return xfg_hash_v6(w[0], w[1], w[2], w[3], t->seed);
	}
	uint64_t m;
	memcpy(&m, sk, 8);
	return xfg_hash_eth(m, t->seed);
}

static inline uint32_t meta_of(const struct xfg_table *t, uint32_t b)
{
	uint32_t m;
	memcpy(&m, t->img + (uint64_t)b * XFG_BUCKET_BYTES + XFG_META_OFF, 4);
	return m;
}

int64_t xfg_table_find(const struct xfg_table *t, const void *key)
{
	uint8_t sk[16];
	stored_key(t, key, sk);
	if (is_zero(sk, t->slot_bytes))
		return t->zero_present ? (int64_t)t->nslots : -1;
	if (!t->count)
		return -1;
	uint32_t b = xfg_home(key_hash(t, sk), t->nbuckets);
	for (uint32_t d = 0; d <= t->max_disp; d++) {
		uint32_t bb = b + d;
		while (bb >= t->nbuckets)
			bb -= t->nbuckets;
		const uint8_t *bk = t->img + (uint64_t)bb * XFG_BUCKET_BYTES;
		for (uint32_t i = 0; i < t->slots_per_bucket; i++)
			if (!memcmp(bk + i * t->slot_bytes, sk, t->slot_bytes))
				return (int64_t)bb * t->slots_per_bucket + i;
		if (!(meta_of(t, bb) & XFG_META_OVERFLOW))
			return -1;
	}
	return -1;
}

static uint32_t bloom_add(struct xfg_table *t, uint32_t h)
{
	uint32_t w = xfg_bloom_word(h, t->bloom_words);
	t->bloom[w] |= xfg_bloom_mask(h);
	return w;
}

int64_t xfg_table_insert(struct xfg_table *t, const void *key,
			 void (*meta_changed)(void *arg, uint32_t bucket), void *arg,
			 int64_t *bloom_word)
{
	uint8_t sk[16];
	if (bloom_word)
		*bloom_word = -1;
	if (t->count >= t->capacity)
		return -E2BIG;
	stored_key(t, key, sk);
	if (is_zero(sk, t->slot_bytes)) {
		t->zero_present = 1;
		t->count++;
		return t->nslots;
	}
	uint32_t h = key_hash(t, sk);
	uint32_t b = xfg_home(h, t->nbuckets);
	for (uint32_t d = 0; d < t->nbuckets; d++) {
		uint32_t bb = b + d;
		while (bb >= t->nbuckets)
			bb -= t->nbuckets;
		uint8_t *bk = t->img + (uint64_t)bb * XFG_BUCKET_BYTES;
		for (uint32_t i = 0; i < t->slots_per_bucket; i++) {
			if (is_zero(bk + i * t->slot_bytes, t->slot_bytes)) {
				memcpy(bk + i * t->slot_bytes, sk, t->slot_bytes);
				if (d > t->max_disp)
					t->max_disp = d;
				t->count++;
				uint32_t w = bloom_add(t, h);
				if (bloom_word)
					*bloom_word = w;
				return (int64_t)bb * t->slots_per_bucket + i;
			}
		}
		uint32_t m = meta_of(t, bb);
		if (!(m & XFG_META_OVERFLOW)) {
			m |= XFG_META_OVERFLOW;
			memcpy(bk + XFG_META_OFF, &m, 4);
			if (meta_changed)
				meta_changed(arg, bb);
		}
	}
	return -E2BIG;
}

int64_t xfg_table_remove(struct xfg_table *t, const void *key)
{
	int64_t s = xfg_table_find(t, key);
	if (s < 0)
		return -ENOENT;
	if ((uint64_t)s == t->nslots)
		t->zero_present = 0;
	else {
		memset(t->img + xfg_table_key_off(t, s), 0, t->slot_bytes);
		t->bloom_stale++;
	}
	t->count--;
	return s;
}

int xfg_table_bloom_needs_rebuild(const struct xfg_table *t)
{
	return t->bloom_stale > 64 && t->bloom_stale * 4 > t->count;
}

void xfg_table_bloom_rebuild(struct xfg_table *t)
{
	memset(t->bloom, 0, (size_t)t->bloom_words * 4);
	for (uint64_t s = 0; s < t->nslots; s++) {
		const uint8_t *k = t->img + xfg_table_key_off(t, s);
		if (!is_zero(k, t->slot_bytes))
			bloom_add(t, key_hash(t, k));
	}
	t->bloom_stale = 0;
}

int xfg_table_slot_key(const struct xfg_table *t, uint64_t slot, void *out)
{
	if (slot == t->nslots) {
		if (!t->zero_present)
			return -ENOENT;
		memset(out, 0, t->keylen);
		return 0;
	}
	if (slot > t->nslots)
		return -ENOENT;
	const uint8_t *p = t->img + xfg_table_key_off(t, slot);
	if (is_zero(p, t->slot_bytes))
		return -ENOENT;
	memcpy(out, p, t->keylen);
	return 0;
}

int64_t xfg_table_next_slot(const struct xfg_table *t, int64_t after)
{
	for (uint64_t s = (uint64_t)(after + 1); s < t->nslots; s++)
		if (!is_zero(t->img + xfg_table_key_off(t, s), t->slot_bytes))
			return (int64_t)s;
	if ((uint64_t)(after + 1) <= t->nslots && t->zero_present)
		return t->nslots;
	return -1;
}

void xfg_table_desc(const struct xfg_table *t, struct xfg_tdesc *d)
{
	d->nbuckets = t->nbuckets;
	d->max_disp = t->max_disp;
	d->count = t->count;
	d->zero_present = t->zero_present;
	d->nslots = t->nslots;
	d->seed = t->seed;
	d->bloom_words = t->bloom_words;
}

/* ------------------------------------------------------------ quotient index */
uint32_t xfg_qt_bits_for(uint32_t count)
{
	uint32_t b = XFG_QT_MIN_BITS;
	while (b < 30 && ((uint64_t)count >> b) >= XFG_QT_LOAD)
		b++;
	return b;
}

void xfg_qt_free(struct xfg_qt *q)
{
	free(q->img);
	free(q->trans);
	q->img = NULL;
	q->trans = NULL;
}

/* Image @im of @q (mask @mask): keys homed per bucket first -- a bucket
 * that more than XFG_QT_SLOTS keys home in holds XFG_QT_SLOTS - 1 of them
 * and the overflow marker. */
static int qt_build_img(struct xfg_qt *q, uint32_t im, const struct xfg_table *t,
			const uint8_t *flags, uint32_t mask)
{
	const uint64_t nb = 1ull << q->bits;
	uint16_t *img = q->img + (uint64_t)im * q->nslots;
	uint32_t *trans = q->trans + (uint64_t)im * q->nslots;
	const uint32_t rbits = 32 - q->bits, rmask = (1u << rbits) - 1;
	uint8_t *homed = calloc(nb, 1);
	if (!homed)
		return -ENOMEM;
	for (int64_t s = xfg_table_next_slot(t, -1); s >= 0; s = xfg_table_next_slot(t, s)) {
		if ((flags[s] & mask) != mask)
			continue;
		uint32_t k;
		xfg_table_slot_key(t, (uint64_t)s, &k);
		const uint32_t b = xfg_qt_hash(k, q->seed) >> rbits;
		if (homed[b] < 255)
			homed[b]++;
	}
	for (int64_t s = xfg_table_next_slot(t, -1); s >= 0; s = xfg_table_next_slot(t, s)) {
		if ((flags[s] & mask) != mask)
			continue;   /* cannot hit this lookup: as absent */
		uint32_t k;
		xfg_table_slot_key(t, (uint64_t)s, &k);   /* the wire bytes, as the kernel loads them */
		const uint32_t h = xfg_qt_hash(k, q->seed), b = h >> rbits;
		uint16_t *e = img + (uint64_t)b * XFG_QT_SLOTS;
		const uint32_t room = homed[b] > XFG_QT_SLOTS ? XFG_QT_SLOTS - 1 : XFG_QT_SLOTS;
		uint32_t c = 0;
		while (c < room && (e[c] & XFG_QT_USED))
			c++;
		if (c == room) {   /* the canonical table answers this bucket's misses */
			e[XFG_QT_SLOTS - 1] = XFG_QT_OVF_MARK;
			q->spilled++;
			continue;
		}
		e[c] = (uint16_t)(XFG_QT_USED | (h & rmask));
		trans[(uint64_t)b * XFG_QT_SLOTS + c] = (uint32_t)s;
		q->placed++;
	}
	free(homed);
	return 0;
}

int xfg_qt_build(struct xfg_qt *q, const struct xfg_table *t, const uint8_t *flags,
		 uint32_t live, uint32_t seed)
{
	if (t->keylen != 4 || live < 1 || live > 3)
		return -EINVAL;
	const uint32_t bits = xfg_qt_bits_for(t->count);
	const uint64_t nb = 1ull << bits, ns = nb * XFG_QT_SLOTS;
	uint32_t nimg = 1;
	if (live == 3)   /* one image unless some key carries exactly one direction */
		for (int64_t s = xfg_table_next_slot(t, -1); s >= 0 && nimg == 1; s = xfg_table_next_slot(t, s))
			if ((flags[s] & 3) == 1 || (flags[s] & 3) == 2)
				nimg = 2;
	if (q->bits != bits || q->nimg != nimg || !q->img) {
		xfg_qt_free(q);
		q->img = malloc(nimg * ns * 2);
		q->trans = malloc(nimg * ns * 4);
		if (!q->img || !q->trans) {
			xfg_qt_free(q);
			return -ENOMEM;
		}
	}
	memset(q->img, 0, nimg * ns * 2);
	memset(q->trans, 0xff, nimg * ns * 4);
	q->bits = bits;
	q->seed = seed;
	q->live = live;
	q->nimg = nimg;
	q->nslots = (uint32_t)ns;
	q->placed = q->spilled = 0;
	for (uint32_t im = 0; im < nimg; im++) {
		int err = qt_build_img(q, im, t, flags, xfg_qt_img_mask(live, nimg, im));
		if (err)
			return err;
	}
	return 0;
}

uint32_t xfg_qt_patch(struct xfg_qt *q, uint32_t im, uint32_t key, uint32_t slot, int add)
{
	const uint32_t rbits = 32 - q->bits, rmask = (1u << rbits) - 1;
	const uint32_t h = xfg_qt_hash(key, q->seed), b = h >> rbits;
	const uint16_t r = (uint16_t)(XFG_QT_USED | (h & rmask));
	uint16_t *e = q->img + (uint64_t)im * q->nslots + (uint64_t)b * XFG_QT_SLOTS;
	uint32_t *tr = q->trans + (uint64_t)im * q->nslots + (uint64_t)b * XFG_QT_SLOTS;
	if (!add) {
		for (uint32_t c = 0; c < XFG_QT_SLOTS; c++)
			if (e[c] == r) {   /* (keys are unique: at most one entry) */
				e[c] = 0;
				tr[c] = 0xffffffffu;
				q->placed--;
				return b;
			}
		if (q->spilled)
			q->spilled--;
		return b;
	}
	const int marked = e[XFG_QT_SLOTS - 1] == XFG_QT_OVF_MARK;
	const uint32_t room = marked ? XFG_QT_SLOTS - 1 : XFG_QT_SLOTS;
	for (uint32_t c = 0; c < room; c++)
		if (!(e[c] & XFG_QT_USED)) {
			e[c] = r;
			tr[c] = slot;
			q->placed++;
			return b;
		}
	if (!marked) {   /* entry 15's key and this one go to the canonical table */
		e[XFG_QT_SLOTS - 1] = XFG_QT_OVF_MARK;
		tr[XFG_QT_SLOTS - 1] = 0xffffffffu;
		q->placed--;
		q->spilled++;
	}
	q->spilled++;
	return b;
}
