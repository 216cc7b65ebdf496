/* SPDX-License-Identifier: GPL-2.0 */
/* xfg_table.h — host image of one device hash table (layout: xfg_layout.h).
 *
 * The host owns the key bytes and overflow bits of every bucket (identical
 * on every device, so slot indices agree across devices and the counter
 * arrays can be reduced element-wise) and the Bloom prefilter; per-device
 * values (flag bytes inside the buckets, the hits array) live on the devices.
 */
#ifndef XFG_TABLE_H
#define XFG_TABLE_H

#include <stdint.h>
#include "xfg_layout.h"

struct xfg_table {
	uint32_t keylen;      /* user key bytes: 4, 16 or 6 */
	uint32_t slot_bytes;  /* stored key bytes: 4, 16 or 8 */
	uint32_t slots_per_bucket;
	uint32_t nbuckets;    /* hashed buckets; bucket nbuckets holds the zero key */
	uint32_t nslots;      /* nbuckets * slots_per_bucket (= slot of the zero key) */
	uint32_t capacity;    /* max keys (the reference's max_entries) */
	uint32_t count;
	uint32_t max_disp;
	uint32_t zero_present;
	uint32_t seed;
	uint32_t bloom_words;
	uint32_t bloom_stale; /* deletes since the filter was last rebuilt */
	uint8_t *img;         /* (nbuckets + 1) * 64 bytes: keys + meta, flags zero */
	uint32_t *bloom;
};

/* keylen 4 (ipv4), 16 (ipv6), 6 (ethernet). Returns 0 or -ENOMEM/-EINVAL. */
int xfg_table_init(struct xfg_table *t, uint32_t keylen, uint32_t capacity, uint32_t seed);
void xfg_table_free(struct xfg_table *t);

/* Slot of @key, or -1.  The all-zero key maps to slot nslots. */
int64_t xfg_table_find(const struct xfg_table *t, const void *key);

/* Insert @key (must be absent): returns its slot, or -E2BIG when count ==
 * capacity.  Buckets whose meta word changed are reported through the
 * optional callback; the Bloom word that changed is returned in *bloom_word
 * (or -1 for the zero key). */
int64_t xfg_table_insert(struct xfg_table *t, const void *key,
			 void (*meta_changed)(void *arg, uint32_t bucket), void *arg,
			 int64_t *bloom_word);

/* Remove @key: returns its former slot, or -ENOENT. */
int64_t xfg_table_remove(struct xfg_table *t, const void *key);

/* True when deletes have left enough stale Bloom bits that a rebuild pays. */
int xfg_table_bloom_needs_rebuild(const struct xfg_table *t);
/* Recompute the Bloom filter from the keys present. */
void xfg_table_bloom_rebuild(struct xfg_table *t);

/* Copy the user-visible key stored in @slot to @out; returns 0, or -ENOENT
 * if the slot is empty. */
int xfg_table_slot_key(const struct xfg_table *t, uint64_t slot, void *out);

/* Iteration in slot order (zero-key slot last): first slot > @after that
 * holds a key (after = -1 to start), or -1 when exhausted. */
int64_t xfg_table_next_slot(const struct xfg_table *t, int64_t after);

/* Byte offsets inside the bucket image of a slot's key and flag byte. */
static inline uint64_t xfg_table_key_off(const struct xfg_table *t, uint64_t slot)
{
	return (slot / t->slots_per_bucket) * XFG_BUCKET_BYTES +
	       (slot % t->slots_per_bucket) * t->slot_bytes;
}
static inline uint64_t xfg_table_flag_off(const struct xfg_table *t, uint64_t slot)
{
	return (slot / t->slots_per_bucket) * XFG_BUCKET_BYTES + XFG_FLAGS_OFF +
	       (slot % t->slots_per_bucket);
}
static inline uint64_t xfg_table_img_bytes(const struct xfg_table *t)
{
	return ((uint64_t)t->nbuckets + 1) * XFG_BUCKET_BYTES;
}

/* Quotient index of a table of 4-byte keys (layout: xfg_layout.h).  Built
 * from the table's keys and each slot's flag byte (@flags[slot], the same on
 * every device); only keys carrying the live mask of an image's lookup are
 * entered in it.  @live 2 (dst) or 1 (src): one image.  @live 3 (both
 * directions): image 0 answers the dst lookup, image 1 the src lookup --
 * unless every key with a direction bit has both (`xdp-filter ip -m
 * src,dst` rule sets), when one image serves both lookups (nimg 1).
 * Returns 0 or -ENOMEM / -EINVAL (not 4-byte keys). */
struct xfg_qt {
	uint32_t bits, seed, live;
	uint32_t nslots;      /* per image: (1 << bits) * XFG_QT_SLOTS */
	uint32_t nimg;        /* images: 1, or 2 (both directions, asymmetric) */
	uint16_t *img;        /* nimg * nslots entries, image after image */
	uint32_t *trans;      /* nimg * nslots: canonical slot, or ~0u */
	uint32_t placed, spilled;
};
int xfg_qt_build(struct xfg_qt *q, const struct xfg_table *t, const uint8_t *flags,
		 uint32_t live, uint32_t seed);
/* One key entering (@add) or leaving the index in place, for a single map
 * edit between rebuilds: @key at canonical @slot.  An entry goes into the
 * first free entry of its bucket; a full bucket without the overflow marker
 * gives up its entry 15 to the marker (that key and the new one are then
 * answered by the canonical table); a leaving key's entry is cleared (a
 * spilled one leaves nothing to clear).  The marker is never cleared here:
 * a marked bucket only sends its misses to the canonical table, which is
 * always exact.  Returns the bucket touched.  The caller has folded the
 * QT-order counts first: an entry given to another key must count from 0. */
uint32_t xfg_qt_patch(struct xfg_qt *q, uint32_t img, uint32_t key, uint32_t slot, int add);
/* The mask a key must carry to be entered in image @img of an index of
 * live mask @live (nimg images). */
static inline uint32_t xfg_qt_img_mask(uint32_t live, uint32_t nimg, uint32_t img)
{
	return live != 3 ? live : (nimg == 1 ? 3u : (img == 0 ? 2u : 1u));
}
void xfg_qt_free(struct xfg_qt *q);
/* Bucket bits for @count keys: fewer than XFG_QT_LOAD keys per 16-entry
 * bucket on average (a 1M-key map: 2^17 buckets, 4 MB). */
uint32_t xfg_qt_bits_for(uint32_t count);

/* Descriptor for the kernel (device pointers filled by the caller). */
void xfg_table_desc(const struct xfg_table *t, struct xfg_tdesc *d);

#endif
