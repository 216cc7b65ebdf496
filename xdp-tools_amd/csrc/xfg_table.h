/* SPDX-License-Identifier: GPL-2.0 */
/* xfg_table.h — host image of one device hash table (layout: xfg_layout.h).
 *
 * The host owns the key image (identical on every device, so slot indices
 * agree across devices and the counter arrays can be reduced element-wise);
 * per-device values (flags, hits) live on the devices only.
 */
#ifndef XFG_TABLE_H
#define XFG_TABLE_H

#include <stdint.h>
#include "xfg_layout.h"

struct xfg_table {
	uint32_t keylen;      /* user key bytes: 4, 16 or 6 */
	uint32_t slot_bytes;  /* stored key bytes: 4, 16 or 8 */
	uint32_t slots_per_bucket;
	uint32_t nbuckets;
	uint32_t nslots;      /* nbuckets * slots_per_bucket */
	uint32_t capacity;    /* max keys (the reference's max_entries) */
	uint32_t count;
	uint32_t max_disp;
	uint32_t zero_present;
	uint32_t seed;
	uint8_t *keys;        /* nbuckets * 64 bytes */
	uint8_t *meta;        /* nbuckets bytes */
};

/* keylen 4 (ipv4), 16 (ipv6), 6 (ethernet). Returns 0 or -ENOMEM/-EINVAL. */
int xfg_table_init(struct xfg_table *t, uint32_t keylen, uint32_t capacity, uint32_t seed);
void xfg_table_free(struct xfg_table *t);

/* Slot of @key, or -1.  The all-zero key maps to slot nslots. */
int64_t xfg_table_find(const struct xfg_table *t, const void *key);

/* Insert @key (must be absent): returns its slot, or -E2BIG when count ==
 * capacity.  *touched_bucket (if not NULL) receives the bucket whose key
 * bytes changed (-1 for the zero key); every bucket whose meta changed is
 * reported through the optional callback. */
int64_t xfg_table_insert(struct xfg_table *t, const void *key,
			 void (*meta_changed)(void *arg, uint32_t bucket), void *arg);

/* Remove @key: returns its former slot, or -ENOENT. */
int64_t xfg_table_remove(struct xfg_table *t, const void *key);

/* Copy the user-visible key stored in @slot to @out; returns 0, or -ENOENT
 * if the slot is empty. */
int xfg_table_slot_key(const struct xfg_table *t, uint64_t slot, void *out);

/* Iteration in slot order (zero-key slot last): first slot > @after that
 * holds a key (after = -1 to start), or -1 when exhausted. */
int64_t xfg_table_next_slot(const struct xfg_table *t, int64_t after);

/* Descriptor for the kernel (device pointers filled by the caller). */
void xfg_table_desc(const struct xfg_table *t, struct xfg_tdesc *d);

#endif
