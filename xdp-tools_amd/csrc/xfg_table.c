/* SPDX-License-Identifier: GPL-2.0 */
/* xfg_table.c — host side of the device hash tables (see xfg_layout.h). */
#include "xfg_table.h"

#include <errno.h>
#include <stdlib.h>
#include <string.h>

/* Target load factors per key type (slots per 64-byte bucket 16 / 4 / 8):
 * with 16-slot buckets at 0.66 ~2% of buckets overflow at full capacity. */
static uint32_t buckets_for(uint32_t capacity, uint32_t spb)
{
	double lf = spb >= 16 ? 0.66 : (spb >= 8 ? 0.6 : 0.5);
	uint64_t nb = (uint64_t)((double)capacity / (spb * lf)) + 1;
	if (nb < 1)
		nb = 1;
	if (nb > 0x7fffffffull / spb)
		nb = 0x7fffffffull / spb;
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
	t->keys = calloc(t->nbuckets, XFG_BUCKET_BYTES);
	t->meta = calloc(t->nbuckets, 1);
	if (!t->keys || !t->meta) {
		xfg_table_free(t);
		return -ENOMEM;
	}
	return 0;
}

void xfg_table_free(struct xfg_table *t)
{
	free(t->keys);
	free(t->meta);
	t->keys = NULL;
	t->meta = NULL;
}

/* Stored form of a user key (zero-padded to slot_bytes). */
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

static uint32_t home_bucket(const struct xfg_table *t, const uint8_t *sk)
{
	uint32_t h;
	if (t->keylen == 4) {
		uint32_t k;
		memcpy(&k, sk, 4);
		h = xfg_hash_v4(k, t->seed);
	} else if (t->keylen == 16) {
		uint32_t w[4];
		memcpy(w, sk, 16);
		h = xfg_hash_v6(w[0], w[1], w[2], w[3], t->seed);
	} else {
		uint64_t m;
		memcpy(&m, sk, 8);
		h = xfg_hash_eth(m, t->seed);
	}
	return xfg_home(h, t->nbuckets);
}

static inline uint8_t *slot_ptr(const struct xfg_table *t, uint64_t slot)
{
	uint64_t b = slot / t->slots_per_bucket, i = slot % t->slots_per_bucket;
	return t->keys + b * XFG_BUCKET_BYTES + i * t->slot_bytes;
}

int64_t xfg_table_find(const struct xfg_table *t, const void *key)
{
	uint8_t sk[16];
	stored_key(t, key, sk);
	if (is_zero(sk, t->slot_bytes))
		return t->zero_present ? (int64_t)t->nslots : -1;
	if (!t->count)
		return -1;
	uint32_t b = home_bucket(t, sk);
	for (uint32_t d = 0; d <= t->max_disp; d++) {
		uint32_t bb = b + d;
		while (bb >= t->nbuckets)
			bb -= t->nbuckets;
		const uint8_t *bk = t->keys + (uint64_t)bb * XFG_BUCKET_BYTES;
		for (uint32_t i = 0; i < t->slots_per_bucket; i++)
			if (!memcmp(bk + i * t->slot_bytes, sk, t->slot_bytes))
				return (int64_t)bb * t->slots_per_bucket + i;
		if (!(t->meta[bb] & XFG_META_OVERFLOW))
			return -1;
	}
	return -1;
}

int64_t xfg_table_insert(struct xfg_table *t, const void *key,
			 void (*meta_changed)(void *arg, uint32_t bucket), void *arg)
{
	uint8_t sk[16];
	if (t->count >= t->capacity)
		return -E2BIG;
	stored_key(t, key, sk);
	if (is_zero(sk, t->slot_bytes)) {
		t->zero_present = 1;
		t->count++;
		return t->nslots;
	}
	uint32_t b = home_bucket(t, sk);
	for (uint32_t d = 0; d < t->nbuckets; d++) {
		uint32_t bb = b + d;
		while (bb >= t->nbuckets)
			bb -= t->nbuckets;
		uint8_t *bk = t->keys + (uint64_t)bb * XFG_BUCKET_BYTES;
		for (uint32_t i = 0; i < t->slots_per_bucket; i++) {
			if (is_zero(bk + i * t->slot_bytes, t->slot_bytes)) {
				memcpy(bk + i * t->slot_bytes, sk, t->slot_bytes);
				if (d > t->max_disp)
					t->max_disp = d;
				t->count++;
				return (int64_t)bb * t->slots_per_bucket + i;
			}
		}
		if (!(t->meta[bb] & XFG_META_OVERFLOW)) {
			t->meta[bb] |= XFG_META_OVERFLOW;
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
	else
		memset(slot_ptr(t, s), 0, t->slot_bytes);
	t->count--;
	return s;
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
	const uint8_t *p = slot_ptr(t, slot);
	if (is_zero(p, t->slot_bytes))
		return -ENOENT;
	memcpy(out, p, t->keylen);
	return 0;
}

int64_t xfg_table_next_slot(const struct xfg_table *t, int64_t after)
{
	for (uint64_t s = (uint64_t)(after + 1); s < t->nslots; s++)
		if (!is_zero(slot_ptr(t, s), t->slot_bytes))
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
}
