/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xfg_ctx.c — host runtime behind include/xdpfilter_gpu.h (plain C over the
 * HIP runtime C API; the kernels live in xfg_kernels.hip).
 *
 * What replaces what in the reference:
 *   program selection     find_prog_file()          xdp-filter/xdp-filter.c:48-60
 *   BPF map CRUD          bpf_map_*_elem() on pinned per-CPU maps
 *                         (xdp-filter/xdp-filter.c:73-157; lib/util/util.h:29-33)
 *   per-CPU value copies  one value per device (flag bytes + hits in HBM)
 *   stats readout         map_get_value_percpu_array  lib/util/stats.c:140-172
 *   prog_lock_acquire     a context mutex           lib/util/util.c:727-767
 */
#define _GNU_SOURCE
#include "xdpfilter_gpu.h"

#include <errno.h>
#include <stddef.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "xfg_layout.h"
#include "xfg_table.h"

/* from xfg_kernels.hip */
int xfg_launch_log_count(const struct xfg_kargs *a, void *stream);
int xfg_launch_classify(uint32_t prog_features, const struct xfg_kargs *a, unsigned grid,
			void *stream);
int xfg_launch_stream_read(const void *src, uint64_t bytes, void *sink, unsigned grid,
			   void *stream);
int xfg_classify_occupancy(uint32_t prog_features, int kind, uint32_t window, size_t dyn);
int xfg_classify_threads(int kind, uint32_t window);
int xfg_launch_compact(const uint8_t *verdicts, uint64_t n, uint32_t action, uint32_t *idx,
		       unsigned long long *count, unsigned long long *status, uint32_t *ticket,
		       unsigned grid, void *stream);
uint64_t xfg_compact_tiles(uint64_t n);
int xfg_launch_qt_fold(uint32_t *qt_hits, const uint32_t *trans,
		       unsigned long long *hits, uint32_t n, void *stream);

#define NMAPS_HASH 3 /* ipv4, ipv6, ethernet */
#define XFG_HOST_REG_MAX 16 /* registered host buffers per context */
/* host-resident classify: staging slots in flight (each: a chunk's copies,
 * kernel and verdicts on its own stream; the host prepares the next chunk
 * while the others move) */
#ifndef HOST_SLOTS
#define HOST_SLOTS 4
#endif

struct dev_map {           /* device arrays of one hash map */
	uint8_t *buckets;      /* (nbuckets + 1) * 64 B: keys, per-device flags, meta */
	uint32_t *bloom;
	unsigned long long *hits;
	unsigned long long *red_hits; /* reduction copy (multi-process) */
};

struct xfg_dev {
	int ordinal;
	int ncu;
	hipStream_t stream;
	hipEvent_t ev0, ev1;
	struct dev_map m[NMAPS_HASH];
	uint8_t *port_flags;
	unsigned long long *port_hits;
	unsigned long long *red_port_hits;
	unsigned long long *stats;      /* 10 */
	unsigned long long *red_stats;  /* 10 */
	void *sink;                     /* stream-read probe sink */
	/* port table (xfg_layout.h): host mirror of this device's port flag
	 * bytes, rebuilt into port_tab before a launch when dirty */
	uint8_t *port_flags_h;
	uint32_t *port_tab;             /* XFG_PORT_TAB entries (ruled ports <= XFG_PORT_TAB_MAX) */
	uint32_t *port_nib;             /* XFG_PORT_NIB_WORDS (more ruled ports) */
	uint32_t port_tab_disp;
	int port_tab_ok, port_tab_dirty;
	/* resident classify workgroups per CU: [kernel: 0 general, 1 pipelined,
	 * 2 pipelined IPv4-key mode, 3 split lookup pass, 4 split parse pass,
	 * 5 pipelined IPv4-key mode over the quotient index, 6 Ethernet-key]
	 * [window 64, 128][dynamic LDS: none, direct counters, port nibble map,
	 * both] */
	int occ[8][2][16];  /* [..][dynamic LDS: + bit 2, the Bloom words (bl_lds);
			     * + bit 3, the LDS Ethernet key table (xfg_kargs.ek)]; kind 7:
			     * kind 5 with its count wave (0: cannot launch) */
	/* the Ethernet-key kernel's key table (kind 6), uploaded from ctx->ek
	 * when ek_gen falls behind ctx->ek_gen; params read at launch under
	 * d->lock */
	uint32_t *ek_img;
	uint64_t ek_img_bytes;
	uint32_t ek_gen, ek_slots, ek_disp;
	/* quotient index of the IPv4 map (kind 5 kernel), uploaded from
	 * ctx->qt when qt_gen falls behind ctx->qt_gen; params read at launch
	 * under d->lock */
	uint32_t *qt_img, *qt_trans;
	uint64_t qt_img_bytes, qt_trans_bytes;
	uint32_t qt_gen, qt_bits, qt_seed, qt_live, qt_n, qt_nimg;
	/* the count kernel's QT-order hit counts (xfg_kargs.qt_hits) and
	 * whether a launch may have added to them since the last fold */
	uint32_t *qt_hits;
	uint64_t qt_hits_bytes;
	uint64_t qt_pk;                /* packets classified through the index since the last fold */
	int qt_pending;
	int last_kind;                 /* kernel kind of the last launch (-1: none) */
	/* host-resident classify (xfg_classify_host / xfg_classify_xsk_host),
	 * under host_lock: a gather pool, two fixed-size staging slots of
	 * HOST_CH packets x HOST_WIN bytes (header windows, or whole slots of
	 * a batch with a stride <= HOST_WIN) with their fallback lists, and the
	 * whole-frame fallback staging (FB_BYTES) */
	pthread_mutex_t host_lock;
	struct hpool *pool;
	uint8_t *hs_hbuf[HOST_SLOTS], *hs_dbuf[HOST_SLOTS], *hs_dv[HOST_SLOTS];
	uint32_t *hs_hl[HOST_SLOTS], *hs_dl[HOST_SLOTS];
	uint32_t *hs_fb[HOST_SLOTS], *hs_fbc[HOST_SLOTS], *hs_hfbc[HOST_SLOTS];
	hipStream_t hs_st[HOST_SLOTS];
	hipEvent_t hs_done[HOST_SLOTS];
	uint8_t *fb_h, *fb_d, *fb_dv;   /* fallback frames (pinned / device), verdicts */
	uint64_t *fb_ho, *fb_do;        /* their offsets */
	uint32_t *fb_hl, *fb_dl, *fb_idx;
	pthread_mutex_t lock;           /* launch scratch below + compaction scratch */
	int lock_ok;
	uint32_t *defer;                /* pipelined kernel: deferred-packet lists */
	uint64_t defer_bytes;
	uint32_t *defer_n;              /* ... their fills (xfg_defer_kernel) */
	uint64_t defer_n_bytes;
	uint32_t *tlog, *pfill;         /* hit log: wave regions, slice fills */
	uint16_t *pbuf;                 /* hit log: partition slices */
	uint64_t tlog_bytes, pbuf_bytes, pfill_bytes;
	/* quotient-index logs not yet counted: log_pend launches of log_grid
	 * workgroups, side by side in the partition buffers, counted by one
	 * count kernel with log_args (their shape) -- when the buffers are
	 * full, before any read of the counts (qt_fold_locked) and before a
	 * launch of another shape */
	uint32_t log_pend, log_grid;
	struct xfg_kargs log_args;
	/* (log_cw: the pending log was written in the count wave's mode --
	 * one launch's slices, set log_first of two -- for the next launch's
	 * count wave to take; log_first: the first pending slice) */
	uint32_t log_cw, log_first;
	uint32_t *rec;                  /* split classify: parse-pass records */
	uint64_t rec_bytes;
	unsigned long long *cstatus;    /* verdict compaction: tile status words */
	uint64_t cstatus_cap;
	uint32_t *cticket;
	hipEvent_t ev_user, ev_done;    /* ordering against a caller's stream */
};

struct xfg_ctx {
	pthread_mutex_t lock;
	uint32_t prog_features;
	const char *prog_name;
	int ndev;
	struct xfg_dev *dev;
	struct xfg_table t[NMAPS_HASH];  /* index = map id - 1 */
	/* host-only context: value store for ndev == 0 */
	uint64_t *host_vals[NMAPS_HASH];
	uint64_t *host_port_vals;
	uint8_t *port_flags_host;        /* OR over devices of the port flags */
	uint32_t port_count;
	/* flag-bit census: flag_or[map][slot] = OR over devices of the slot's
	 * flag byte; flag_cnt[map][bit] = slots with that bit (likewise for the
	 * ports).  The kernel skips a lookup whose mask no key carries. */
	uint8_t *flag_or[NMAPS_HASH];
	uint32_t flag_cnt[NMAPS_HASH][8];   /* bit 7: slots whose flags differ between devices */
	/* quotient index of the IPv4 map (xfg_table.h): rebuilt before a
	 * classify that uses it when the map changed (qt_dirty); generation
	 * qt_gen (0 = never built) */
	struct xfg_qt qt;
	int qt_dirty;
	uint32_t qt_gen;
	/* the Ethernet map as the Ethernet-key kernel's LDS key table
	 * (xfg_kargs.ek): rebuilt when an Ethernet flag byte or key changed
	 * (ek_edits moved past ek_built); ek_ok: it can serve (few keys, the
	 * same flags on every device) */
	uint32_t ek_host[XFG_EK_SLOTS_MAX * 4];
	uint32_t ek_slots, ek_disp;
	uint32_t ek_edits, ek_seen;   /* Ethernet map edits; those the table holds */
	uint32_t ek_gen;              /* tables built (0: none yet) */
	int ek_ok;
	uint32_t qt_min_keys;
	uint32_t window;                /* header window above a 64-byte stride: 64 or 128 */
	uint32_t port_flag_cnt[8];
	/* multi-process reduction */
	ncclComm_t comm;
	int comm_ready;
	int reduced;
	/* host buffers registered for direct DMA (xfg_host_register) */
	pthread_mutex_t reg_lock;
	struct { const uint8_t *p; size_t bytes; } reg[XFG_HOST_REG_MAX];
	int nreg;
};

/* Default smallest IPv4 map that takes the quotient index (its 2^17 buckets
 * are 4 MiB: below this the canonical table and its prefilter stay in L2). */
#define XFG_QT_MIN_KEYS (1u << 18)
#define XFG_LOG_PEND_MAX 4u   /* quotient-index launches per count kernel */

/* ------------------------------------------------------------------ misc */
static const struct { const char *name; uint32_t feat; } prog_table[] = {
	/* xdp-filter/Makefile:3-6 order; features = each program's _features */
	{ "xdpfilt_dny_udp", XFG_FEAT_UDP | XFG_FEAT_DENY },
	{ "xdpfilt_dny_tcp", XFG_FEAT_TCP | XFG_FEAT_DENY },
	{ "xdpfilt_dny_ip", XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_DENY },
	{ "xdpfilt_dny_eth", XFG_FEAT_ETHERNET | XFG_FEAT_DENY },
	{ "xdpfilt_dny_all", XFG_FEAT_ALL | XFG_FEAT_DENY },
	{ "xdpfilt_alw_udp", XFG_FEAT_UDP | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_tcp", XFG_FEAT_TCP | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_ip", XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_eth", XFG_FEAT_ETHERNET | XFG_FEAT_ALLOW },
	{ "xdpfilt_alw_all", XFG_FEAT_ALL | XFG_FEAT_ALLOW },
};

int xfg_select_program(uint32_t features, const char **prog_name, uint32_t *prog_features)
{
	if (!features)
		return -EINVAL;
	for (size_t i = 0; i < sizeof(prog_table) / sizeof(prog_table[0]); i++) {
		if ((prog_table[i].feat & features) == features) {
			if (prog_name)
				*prog_name = prog_table[i].name;
			if (prog_features)
				*prog_features = prog_table[i].feat;
			return 0;
		}
	}
	return -ENOENT;
}

const char *xfg_strerror(int err)
{
	if (err <= -1000)
		return "HIP runtime error";
	return strerror(err < 0 ? -err : err);
}

static int hip_err(hipError_t e)
{
	if (e == hipSuccess)
		return 0;
	if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation)
		return -ENOMEM;
	if (e == hipErrorNoDevice || e == hipErrorInvalidDevice)
		return -ENODEV;
	return -1000 - (int)e;
}

#define HIPCHK(call)                                  \
	do {                                          \
		int _e = hip_err(call);               \
		if (_e) {                             \
			err = _e;                     \
			goto fail;                    \
		}                                     \
	} while (0)

static int keylen_of(int map)
{
	switch (map) {
	case XFG_MAP_PORTS: return 4;
	case XFG_MAP_IPV4: return 4;
	case XFG_MAP_IPV6: return 16;
	case XFG_MAP_ETHERNET: return 6;
	default: return -EINVAL;
	}
}

/* ------------------------------------------------------------------ gather pool */
/* Persistent worker threads of one device's host path: hpool_run(fn, arg)
 * runs fn(arg, slice, nslices) for every slice, slice 0 on the caller.  As
 * many as the process's CPU set allows, capped by HOST_THREADS; the
 * caller's share of a shared box (whose CPU set shows the whole machine) is
 * XFG_HOST_THREADS, else OMP_NUM_THREADS when it is above 1 -- a value of 1
 * is what torch.distributed.run exports to every rank by default, and taken
 * at its word it would leave each rank's gather one thread.  Performance
 * only: the slices' results do not depend on their count.  xfg_host_threads()
 * reports the size. */
#define HOST_THREADS 16

static int hpool_size(void)
{
	int n = HOST_THREADS;
	cpu_set_t cs;
	if (!sched_getaffinity(0, sizeof(cs), &cs) && CPU_COUNT(&cs) > 0 && CPU_COUNT(&cs) < n)
		n = CPU_COUNT(&cs);
	const char *ht = getenv("XFG_HOST_THREADS");
	const char *omp = getenv("OMP_NUM_THREADS");
	if (ht && atoi(ht) > 0)
		n = atoi(ht) < HOST_THREADS ? atoi(ht) : HOST_THREADS;
	else if (omp && atoi(omp) > 1 && atoi(omp) < n)
		n = atoi(omp);
	return n;
}

int xfg_host_threads(void)
{
	return hpool_size();
}

struct hpool {
	pthread_t th[HOST_THREADS];
	struct hpool_arg {
		struct hpool *p;
		int id;
	} args[HOST_THREADS];
	int nth;                   /* workers (slices 1..nth) */
	pthread_mutex_t mu;
	pthread_cond_t go, done;
	void (*fn)(void *, int, int);
	void *arg;
	unsigned gen;
	int pending, stop;
};

static void *hpool_main(void *v)
{
	struct hpool_arg *w = v;
	struct hpool *p = w->p;
	unsigned seen = 0;
	pthread_mutex_lock(&p->mu);
	for (;;) {
		while (p->gen == seen && !p->stop)
			pthread_cond_wait(&p->go, &p->mu);
		if (p->stop)
			break;
		seen = p->gen;
		void (*fn)(void *, int, int) = p->fn;
		void *arg = p->arg;
		const int n = p->nth + 1;
		pthread_mutex_unlock(&p->mu);
		fn(arg, w->id, n);
		pthread_mutex_lock(&p->mu);
		if (--p->pending == 0)
			pthread_cond_signal(&p->done);
	}
	pthread_mutex_unlock(&p->mu);
	return NULL;
}

static struct hpool *hpool_start(void)
{
	struct hpool *p = calloc(1, sizeof(*p));
	if (!p)
		return NULL;
	pthread_mutex_init(&p->mu, NULL);
	pthread_cond_init(&p->go, NULL);
	pthread_cond_init(&p->done, NULL);
	/* (workers are told their count under the lock, before any run) */
	const int nt = hpool_size();
	pthread_mutex_lock(&p->mu);
	for (int t = 1; t < nt; t++) {
		p->args[t] = (struct hpool_arg){ p, t };
		if (pthread_create(&p->th[t], NULL, hpool_main, &p->args[t]))
			break;
		p->nth = t;
	}
	pthread_mutex_unlock(&p->mu);
	return p;
}

static void hpool_run(struct hpool *p, void (*fn)(void *, int, int), void *arg)
{
	pthread_mutex_lock(&p->mu);
	p->fn = fn;
	p->arg = arg;
	p->pending = p->nth;
	p->gen++;
	pthread_cond_broadcast(&p->go);
	pthread_mutex_unlock(&p->mu);
	fn(arg, 0, p->nth + 1);
	pthread_mutex_lock(&p->mu);
	while (p->pending)
		pthread_cond_wait(&p->done, &p->mu);
	pthread_mutex_unlock(&p->mu);
}

static void hpool_stop(struct hpool *p)
{
	if (!p)
		return;
	pthread_mutex_lock(&p->mu);
	p->stop = 1;
	pthread_cond_broadcast(&p->go);
	pthread_mutex_unlock(&p->mu);
	for (int t = 1; t <= p->nth; t++)
		pthread_join(p->th[t], NULL);
	pthread_cond_destroy(&p->go);
	pthread_cond_destroy(&p->done);
	pthread_mutex_destroy(&p->mu);
	free(p);
}

/* ------------------------------------------------------------------ open */
static void dev_free(struct xfg_dev *d)
{
	hpool_stop(d->pool);
	d->pool = NULL;
	if (d->lock_ok) {
		pthread_mutex_destroy(&d->lock);
		pthread_mutex_destroy(&d->host_lock);
		d->lock_ok = 0;
	}
	if (hipSetDevice(d->ordinal) != hipSuccess)
		return;
	for (int i = 0; i < NMAPS_HASH; i++) {
		hipFree(d->m[i].buckets);
		hipFree(d->m[i].bloom);
		hipFree(d->m[i].hits);
		hipFree(d->m[i].red_hits);
	}
	hipFree(d->port_flags);
	hipFree(d->port_nib);
	hipFree(d->port_hits);
	hipFree(d->red_port_hits);
	hipFree(d->stats);
	hipFree(d->red_stats);
	hipFree(d->sink);
	hipFree(d->port_tab);
	hipFree(d->qt_img);
	hipFree(d->ek_img);
	hipFree(d->qt_trans);
	hipFree(d->qt_hits);
	free(d->port_flags_h);
	hipFree(d->cstatus);
	for (int k = 0; k < HOST_SLOTS; k++) {
		if (d->hs_st[k])
			hipStreamSynchronize(d->hs_st[k]);
		hipHostFree(d->hs_hbuf[k]);
		hipHostFree(d->hs_hl[k]);
		hipHostFree(d->hs_hfbc[k]);
		hipFree(d->hs_dbuf[k]);
		hipFree(d->hs_dl[k]);
		hipFree(d->hs_dv[k]);
		hipFree(d->hs_fb[k]);
		hipFree(d->hs_fbc[k]);
		if (d->hs_done[k])
			hipEventDestroy(d->hs_done[k]);
		if (d->hs_st[k])
			hipStreamDestroy(d->hs_st[k]);
	}
	hipHostFree(d->fb_h);
	hipHostFree(d->fb_ho);
	hipHostFree(d->fb_hl);
	hipHostFree(d->fb_idx);
	hipFree(d->fb_d);
	hipFree(d->fb_do);
	hipFree(d->fb_dl);
	hipFree(d->fb_dv);
	hipFree(d->defer);
	hipFree(d->defer_n);
	hipFree(d->tlog);
	hipFree(d->pbuf);
	hipFree(d->rec);
	hipFree(d->pfill);
	hipFree(d->cticket);
	if (d->ev_user)
		hipEventDestroy(d->ev_user);
	if (d->ev_done)
		hipEventDestroy(d->ev_done);
	if (d->ev0)
		hipEventDestroy(d->ev0);
	if (d->ev1)
		hipEventDestroy(d->ev1);
	if (d->stream)
		hipStreamDestroy(d->stream);
}

static int dev_init(xfg_ctx *ctx, struct xfg_dev *d)
{
	int err = 0;
	hipDeviceProp_t prop;

	pthread_mutex_init(&d->lock, NULL);
	pthread_mutex_init(&d->host_lock, NULL);
	d->lock_ok = 1;
	HIPCHK(hipSetDevice(d->ordinal));
	HIPCHK(hipGetDeviceProperties(&prop, d->ordinal));
	d->ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
	HIPCHK(hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking));
	HIPCHK(hipEventCreate(&d->ev0));
	HIPCHK(hipEventCreate(&d->ev1));
	for (int i = 0; i < NMAPS_HASH; i++) {
		const struct xfg_table *t = &ctx->t[i];
		size_t ns = (size_t)t->nslots + 1;
		HIPCHK(hipMalloc((void **)&d->m[i].buckets, xfg_table_img_bytes(t)));
		HIPCHK(hipMalloc((void **)&d->m[i].bloom, (size_t)t->bloom_words * 4));
		HIPCHK(hipMalloc((void **)&d->m[i].hits, ns * 8));
		HIPCHK(hipMemset(d->m[i].buckets, 0, xfg_table_img_bytes(t)));
		HIPCHK(hipMemset(d->m[i].bloom, 0, (size_t)t->bloom_words * 4));
		HIPCHK(hipMemset(d->m[i].hits, 0, ns * 8));
	}
	HIPCHK(hipMalloc((void **)&d->port_flags, XFG_PORT_MAP_ENTRIES));
	HIPCHK(hipMalloc((void **)&d->port_nib, XFG_PORT_NIB_WORDS * 4));
	HIPCHK(hipMalloc((void **)&d->port_hits, XFG_PORT_MAP_ENTRIES * 8));
	HIPCHK(hipMemset(d->port_flags, 0, XFG_PORT_MAP_ENTRIES));
	HIPCHK(hipMemset(d->port_hits, 0, XFG_PORT_MAP_ENTRIES * 8));
	HIPCHK(hipMalloc((void **)&d->stats, 10 * 8));
	HIPCHK(hipMemset(d->stats, 0, 10 * 8));
	HIPCHK(hipMalloc(&d->sink, 16 * 65536));
	HIPCHK(hipMalloc((void **)&d->port_tab, XFG_PORT_TAB * 4));
	d->port_flags_h = calloc(XFG_PORT_MAP_ENTRIES, 1);
	if (!d->port_flags_h) {
		err = -ENOMEM;
		goto fail;
	}
	d->port_tab_dirty = 1;
	d->last_kind = -1;
	HIPCHK(hipEventCreateWithFlags(&d->ev_user, hipEventDisableTiming));
	HIPCHK(hipEventCreateWithFlags(&d->ev_done, hipEventDisableTiming));

	for (int k = 0; k < 8; k++)
		for (int w = 0; w < 2; w++)
			for (int c = 0; c < 16; c++)
				d->occ[k][w][c] = xfg_classify_occupancy(
					ctx->prog_features, k, w ? 128 : 64,
					(c & 1 ? XFG_DCNT_MAX * 4 : 0) + (c & 2 ? XFG_PORT_NIB_WORDS * 4 : 0) +
					(c & 4 ? XFG_BLOOM_LDS_MAX * 4 : 0) + (c & 8 ? 12 + XFG_EK_SLOTS_MAX * 16 : 0) +
					(k == 7 ? 16 + XFG_CW_HIST_MAX * 4 : 0));
	/* (a query past the LDS a workgroup can have may leave an error behind:
	 * not a launch's) */
	(void)hipGetLastError();
	HIPCHK(hipDeviceSynchronize());
	return 0;
fail:
	return err;
}

int xfg_open(xfg_ctx **out, const struct xfg_open_opts *opts)
{
	int err;
	xfg_ctx *ctx;

	if (!out || !opts)
		return -EINVAL;
	*out = NULL;
	ctx = calloc(1, sizeof(*ctx));
	if (!ctx)
		return -ENOMEM;
	pthread_mutex_init(&ctx->lock, NULL);
	pthread_mutex_init(&ctx->reg_lock, NULL);
	err = xfg_select_program(opts->features, &ctx->prog_name, &ctx->prog_features);
	if (err)
		goto fail;

	uint32_t seed = opts->hash_seed ? opts->hash_seed : 0x5eed1234u;
	ctx->qt_min_keys = XFG_QT_MIN_KEYS;
	if (opts->sz >= offsetof(struct xfg_open_opts, qt_min_keys) + sizeof(uint32_t) && opts->qt_min_keys)
		ctx->qt_min_keys = opts->qt_min_keys;
	ctx->window = 64;
	if (opts->sz >= offsetof(struct xfg_open_opts, window) + sizeof(uint32_t) && opts->window) {
		if (opts->window != 64 && opts->window != 128) {
			err = -EINVAL;
			goto fail;
		}
		ctx->window = opts->window;
	}
	uint32_t cap4 = opts->ipv4_capacity ? opts->ipv4_capacity : XFG_DEFAULT_MAP_CAPACITY;
	uint32_t cap6 = opts->ipv6_capacity ? opts->ipv6_capacity : XFG_DEFAULT_MAP_CAPACITY;
	uint32_t cape = opts->eth_capacity ? opts->eth_capacity : XFG_DEFAULT_MAP_CAPACITY;
	if ((err = xfg_table_init(&ctx->t[0], 4, cap4, seed)) ||
	    (err = xfg_table_init(&ctx->t[1], 16, cap6, seed ^ 0x6a09e667u)) ||
	    (err = xfg_table_init(&ctx->t[2], 6, cape, seed ^ 0xbb67ae85u)))
		goto fail;
	for (int i = 0; i < NMAPS_HASH; i++) {
		ctx->flag_or[i] = calloc((size_t)ctx->t[i].nslots + 1, 1);
		if (!ctx->flag_or[i]) {
			err = -ENOMEM;
			goto fail;
		}
	}
	ctx->port_flags_host = calloc(XFG_PORT_MAP_ENTRIES, 1);
	if (!ctx->port_flags_host) {
		err = -ENOMEM;
		goto fail;
	}

	ctx->ndev = opts->ndev > 0 ? opts->ndev : 0;
	if (!ctx->ndev) {
		for (int i = 0; i < NMAPS_HASH; i++) {
			ctx->host_vals[i] = calloc((size_t)ctx->t[i].nslots + 1, 8);
			if (!ctx->host_vals[i]) {
				err = -ENOMEM;
				goto fail;
			}
		}
		ctx->host_port_vals = calloc(XFG_PORT_MAP_ENTRIES, 8);
		if (!ctx->host_port_vals) {
			err = -ENOMEM;
			goto fail;
		}
	} else {
		int count = 0;
		if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
			err = -ENODEV;
			goto fail;
		}
		ctx->dev = calloc(ctx->ndev, sizeof(*ctx->dev));
		if (!ctx->dev) {
			err = -ENOMEM;
			goto fail;
		}
		for (int i = 0; i < ctx->ndev; i++) {
			ctx->dev[i].ordinal = opts->devices ? opts->devices[i] : i;
			if (ctx->dev[i].ordinal < 0 || ctx->dev[i].ordinal >= count) {
				err = -ENODEV;
				goto fail;
			}
			if ((err = dev_init(ctx, &ctx->dev[i])))
				goto fail;
		}
	}
	*out = ctx;
	return 0;
fail:
	xfg_close(ctx);
	return err;
}

void xfg_close(xfg_ctx *ctx)
{
	if (!ctx)
		return;
	if (ctx->comm_ready)
		ncclCommDestroy(ctx->comm);
	for (int i = 0; i < ctx->ndev && ctx->dev; i++)
		dev_free(&ctx->dev[i]);
	for (int i = 0; i < ctx->nreg; i++)
		hipHostUnregister((void *)ctx->reg[i].p);
	pthread_mutex_destroy(&ctx->reg_lock);
	free(ctx->dev);
	for (int i = 0; i < NMAPS_HASH; i++) {
		xfg_table_free(&ctx->t[i]);
		free(ctx->host_vals[i]);
		free(ctx->flag_or[i]);
	}
	xfg_qt_free(&ctx->qt);
	free(ctx->host_port_vals);
	free(ctx->port_flags_host);
	pthread_mutex_destroy(&ctx->lock);
	free(ctx);
}

const char *xfg_prog_name(const xfg_ctx *ctx) { return ctx ? ctx->prog_name : NULL; }

int xfg_last_path(const xfg_ctx *ctx, int dev)
{
	if (!ctx || dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	return ctx->dev[dev].last_kind < 0 ? -ENOENT : ctx->dev[dev].last_kind;
}
uint32_t xfg_prog_features(const xfg_ctx *ctx) { return ctx ? ctx->prog_features : 0; }
int xfg_num_devices(const xfg_ctx *ctx) { return ctx ? ctx->ndev : -EINVAL; }

/* ------------------------------------------------------------------ maps */
static int dev_read(struct xfg_dev *d, void *dst, const void *src, size_t n)
{
	int err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = hip_err(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, d->stream));
	if (!err)
		err = hip_err(hipStreamSynchronize(d->stream));
	return err;
}

static int dev_write(struct xfg_dev *d, void *dst, const void *src, size_t n)
{
	int err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = hip_err(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, d->stream));
	if (!err)
		err = hip_err(hipStreamSynchronize(d->stream));
	return err;
}

static unsigned long long *hits_view(xfg_ctx *ctx, struct xfg_dev *d, int mi)
{
	return ctx->reduced ? d->m[mi].red_hits : d->m[mi].hits;
}

/* Count the pending quotient-index logs into the QT-order counts (d->lock
 * held): one count kernel over every pending launch's slices. */
static int log_flush_locked(struct xfg_dev *d)
{
	if (!d->log_pend)
		return 0;
	struct xfg_kargs c = d->log_args;
	c.pcount = d->log_pend * d->log_grid;
	c.pfirst = d->log_first;   /* (the count wave's mode: the set of the last launch) */
	c.cw_n = 0;
	d->log_pend = 0;
	int err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = xfg_launch_log_count(&c, d->stream);
	return err;
}

/* Both halves of the QT-order counts (the log's and the atomics',
 * xfg_kargs.qt_hitx) into the canonical counters, one fold each. */
static int qt_fold_launch(struct xfg_dev *d)
{
	int err = xfg_launch_qt_fold(d->qt_hits, d->qt_trans, d->m[0].hits, d->qt_n, d->stream);
	if (!err)
		err = xfg_launch_qt_fold(d->qt_hits + d->qt_n, d->qt_trans, d->m[0].hits, d->qt_n, d->stream);
	return err;
}

/* Add @d's QT-order hit counts into its canonical IPv4 counters, through the
 * index's current qt_trans (d->lock held): in stream order after every
 * classify that counted into them (and after the count kernel of every
 * log still pending). */
static int qt_fold_locked(struct xfg_dev *d)
{
	int err = log_flush_locked(d);
	if (err || !d->qt_pending)
		return err;
	err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = qt_fold_launch(d);
	if (!err)
		err = hip_err(hipStreamSynchronize(d->stream));
	if (!err) {
		d->qt_pending = 0;
		d->qt_pk = 0;
	}
	return err;
}

/* The same fold queued on the device stream with no wait (d->lock held):
 * before a launch whose packets could take a 32-bit QT-order count past
 * 2^32 - 1 (xfg_kargs.qt_hits). */
static int qt_fold_queued(struct xfg_dev *d)
{
	int err = log_flush_locked(d);
	if (!err)
		err = qt_fold_launch(d);
	if (!err)
		d->qt_pk = 0;
	return err;
}

/* Before the IPv4 map's counters are read, written or reduced (ctx->lock
 * held): fold every device's QT-order counts. */
static int qt_fold(xfg_ctx *ctx, int mi)
{
	int err = 0;
	for (int i = 0; mi == 0 && i < ctx->ndev && !err; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		pthread_mutex_lock(&d->lock);
		err = qt_fold_locked(d);
		pthread_mutex_unlock(&d->lock);
	}
	return err;
}

/* Read the per-device values of @slot of hash map @mi (0..2). */
static int slot_values(xfg_ctx *ctx, int mi, uint64_t slot, uint64_t *vals)
{
	if (!ctx->ndev) {
		vals[0] = ctx->host_vals[mi][slot];
		return 0;
	}
	const struct xfg_table *t = &ctx->t[mi];
	int e0 = qt_fold(ctx, mi);
	if (e0)
		return e0;
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		uint8_t f;
		unsigned long long h;
		int err = dev_read(d, &f, d->m[mi].buckets + xfg_table_flag_off(t, slot), 1);
		if (!err)
			err = dev_read(d, &h, hits_view(ctx, d, mi) + slot, 8);
		if (err)
			return err;
		vals[i] = (h << XFG_COUNTER_SHIFT) | f;
	}
	return 0;
}

static void census(uint32_t *cnt, uint8_t old, uint8_t f)
{
	for (int b = 0; b < 8; b++) {
		cnt[b] -= (old >> b) & 1;
		cnt[b] += (f >> b) & 1;
	}
}

static uint32_t census_mask(const uint32_t *cnt)
{
	uint32_t m = 0;
	for (int b = 0; b < 6; b++)
		if (cnt[b])
			m |= 1u << b;
	return m;
}

/* @any / @all: the OR / AND over devices of the slot's flag byte (bit 7 of
 * the census byte records that they differ).  A changed IPv4 flag byte
 * marks the quotient index for a rebuild unless @patch (a single edit, which
 * slot_store applies to the index in place); returns the old byte. */
static uint8_t flags_note(xfg_ctx *ctx, int mi, uint64_t slot, uint8_t any, uint8_t all, int patch)
{
	const uint8_t f = any | (any != all ? 0x80 : 0), old = ctx->flag_or[mi][slot];
	census(ctx->flag_cnt[mi], old, f);
	if (mi == 2)   /* (every key insert and delete passes here) */
		ctx->ek_edits++;
	ctx->flag_or[mi][slot] = f;
	if (mi == 0 && old != f && !patch)
		ctx->qt_dirty = 1;
	return old;
}

/* One IPv4 key's flag byte went from @old to @nw (ctx->lock held, every
 * device's QT-order counts folded): enter it into or take it out of the
 * quotient index in place (xfg_qt_patch) and send the one bucket and its
 * trans[] entries to every device whose copy was current; a change of the
 * index's size (bits follow the key count) leaves a full rebuild to the
 * next classify, as before.  @key: the key bytes (NULL: read from the
 * table, where the key still is). */
static int qt_edit(xfg_ctx *ctx, uint64_t slot, const void *key, uint8_t old, uint8_t nw)
{
	struct xfg_qt *q = &ctx->qt;
	if (ctx->qt_dirty || !ctx->qt_gen || !q->img)
		return 0;   /* (rebuilt before its next use anyway) */
#ifdef XFG_DIAG
	const char *po = getenv("XFG_QT_PATCH");   /* "off": every edit rebuilds (round 3) */
	if (po && !strcmp(po, "off")) {
		ctx->qt_dirty = 1;
		return 0;
	}
#endif
	/* per image: does the key enter or leave it */
	int chg[2] = { 0, 0 }, any = 0;
	for (uint32_t im = 0; im < q->nimg; im++) {
		const uint32_t mk = xfg_qt_img_mask(q->live, q->nimg, im);
		const int was = (old & mk) == mk, is = (nw & mk) == mk;
		chg[im] = was == is ? 0 : (is ? 1 : -1);
		any |= chg[im];
	}
	/* one image for both directions holds only keys with both or neither:
	 * a key with exactly one direction needs the second image (rebuild) */
	if (q->live == 3 && q->nimg == 1 && ((nw & 3) == 1 || (nw & 3) == 2)) {
		ctx->qt_dirty = 1;
		return 0;
	}
	if (!any)
		return 0;
	if (xfg_qt_bits_for(ctx->t[0].count) != q->bits) {
		ctx->qt_dirty = 1;
		return 0;
	}
	uint32_t k;
	if (key)
		memcpy(&k, key, 4);
	else if (xfg_table_slot_key(&ctx->t[0], slot, &k)) {
		ctx->qt_dirty = 1;
		return 0;
	}
	uint32_t bk[2] = { 0, 0 };
	for (uint32_t im = 0; im < q->nimg; im++)
		if (chg[im])
			bk[im] = xfg_qt_patch(q, im, k, (uint32_t)slot, chg[im] > 0);
	uint32_t gen = ctx->qt_gen + 1;
	if (!gen)
		gen = 1;
	int err = 0;
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		pthread_mutex_lock(&d->lock);
		/* (a classify launched since slot_store's fold counted through the
		 * old bucket: fold it in the same lock section as the bucket write,
		 * as qt_refresh does, so no count is read through the new trans[]) */
		int e = qt_fold_locked(d);
		if (e) {
			if (!err)
				err = e;
		} else if (d->qt_gen == ctx->qt_gen) {
			for (uint32_t im = 0; im < q->nimg && !e; im++) {
				if (!chg[im])
					continue;
				const uint64_t o = (uint64_t)im * q->nslots + (uint64_t)bk[im] * XFG_QT_SLOTS;
				e = dev_write(d, (uint8_t *)d->qt_img + o * 2, q->img + o, XFG_QT_BUCKET);
				if (!e)
					e = dev_write(d, d->qt_trans + o, q->trans + o, XFG_QT_SLOTS * 4);
			}
			if (!e)
				d->qt_gen = gen;
			else if (!err)
				err = e;
		}
		pthread_mutex_unlock(&d->lock);
	}
	ctx->qt_gen = gen;
	if (err)   /* (a device whose copy may not match the map: rebuild before the next use) */
		ctx->qt_dirty = 1;
	return err;
}

static int slot_store(xfg_ctx *ctx, int mi, uint64_t slot, const uint64_t *vals, const void *key)
{
	uint8_t any = 0, all = 63;
	for (int i = 0; i < (ctx->ndev ? ctx->ndev : 1); i++) {
		any |= vals[i] & 63;
		all &= vals[i] & 63;
	}
	const uint8_t old = flags_note(ctx, mi, slot, any, all, ctx->ndev != 0);
	if (!ctx->ndev) {
		ctx->host_vals[mi][slot] = vals[0];
		return 0;
	}
	const struct xfg_table *t = &ctx->t[mi];
	int e0 = qt_fold(ctx, mi);
	if (!e0 && mi == 0 && old != ctx->flag_or[0][slot])
		e0 = qt_edit(ctx, slot, key, old, ctx->flag_or[0][slot]);
	if (e0) {
		if (mi == 0)   /* (flags_note skipped the rebuild mark for the patch that failed) */
			ctx->qt_dirty = 1;
		return e0;
	}
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		uint8_t f = vals[i] & 63;
		unsigned long long h = vals[i] >> XFG_COUNTER_SHIFT;
		int err = dev_write(d, d->m[mi].buckets + xfg_table_flag_off(t, slot), &f, 1);
		if (!err)
			err = dev_write(d, d->m[mi].hits + slot, &h, 8);
		if (err)
			return err;
	}
	return 0;
}

/* Push the key bytes of @slot (host image) to every device. */
static int push_key(xfg_ctx *ctx, int mi, uint64_t slot)
{
	const struct xfg_table *t = &ctx->t[mi];
	uint64_t off = xfg_table_key_off(t, slot);
	for (int i = 0; i < ctx->ndev; i++) {
		int err = dev_write(&ctx->dev[i], ctx->dev[i].m[mi].buckets + off, t->img + off,
				    t->slot_bytes);
		if (err)
			return err;
	}
	return 0;
}

static int push_bloom(xfg_ctx *ctx, int mi, int64_t word)
{
	const struct xfg_table *t = &ctx->t[mi];
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		int err = word < 0 ? dev_write(d, d->m[mi].bloom, t->bloom, (size_t)t->bloom_words * 4)
				   : dev_write(d, d->m[mi].bloom + word, t->bloom + word, 4);
		if (err)
			return err;
	}
	return 0;
}

struct meta_push { xfg_ctx *ctx; int mi; int err; };

static void meta_changed(void *arg, uint32_t b)
{
	struct meta_push *mp = arg;
	xfg_ctx *ctx = mp->ctx;
	uint64_t off = (uint64_t)b * XFG_BUCKET_BYTES + XFG_META_OFF;
	for (int i = 0; i < ctx->ndev && !mp->err; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		mp->err = dev_write(d, d->m[mp->mi].buckets + off, ctx->t[mp->mi].img + off, 4);
	}
}

static int port_key(const void *key, uint32_t *k)
{
	memcpy(k, key, 4);
	return *k < XFG_PORT_MAP_ENTRIES ? 0 : -ENOENT;
}

/* Track which ports have any flag on any device: port_count (the empty-map
 * skip) and the flag census. */
static int port_flags_note(xfg_ctx *ctx, uint32_t k, uint8_t f)
{
	census(ctx->port_flag_cnt, ctx->port_flags_host[k], f);
	if (!ctx->port_flags_host[k] && f)
		ctx->port_count++;
	else if (ctx->port_flags_host[k] && !f)
		ctx->port_count--;
	ctx->port_flags_host[k] = f;
	return 0;
}

int xfg_map_lookup(xfg_ctx *ctx, int map, const void *key, uint64_t *vals)
{
	int err = 0;
	if (!ctx || !key || !vals || keylen_of(map) < 0)
		return -EINVAL;
	pthread_mutex_lock(&ctx->lock);
	if (map == XFG_MAP_PORTS) {
		uint32_t k;
		if ((err = port_key(key, &k)))
			goto out;
		if (!ctx->ndev) {
			vals[0] = ctx->host_port_vals[k];
			goto out;
		}
		for (int i = 0; i < ctx->ndev && !err; i++) {
			struct xfg_dev *d = &ctx->dev[i];
			uint8_t f;
			unsigned long long h = 0;
			err = dev_read(d, &f, d->port_flags + k, 1);
			if (!err)
				err = dev_read(d, &h, (ctx->reduced ? d->red_port_hits : d->port_hits) + k, 8);
			vals[i] = (h << XFG_COUNTER_SHIFT) | f;
		}
		goto out;
	}
	int mi = map - 1;
	int64_t s = xfg_table_find(&ctx->t[mi], key);
	if (s < 0) {
		err = -ENOENT;
		goto out;
	}
	err = slot_values(ctx, mi, (uint64_t)s, vals);
out:
	pthread_mutex_unlock(&ctx->lock);
	return err;
}

static int port_store(xfg_ctx *ctx, uint32_t k, const uint64_t *vals)
{
	int err = 0;
	uint8_t any = 0;
	if (!ctx->ndev) {
		ctx->host_port_vals[k] = vals[0];
		any = vals[0] & 63;
	}
	for (int i = 0; i < ctx->ndev && !err; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		uint8_t f = vals[i] & 63;
		unsigned long long h = vals[i] >> XFG_COUNTER_SHIFT;
		any |= f;
		d->port_flags_h[k] = f;
		d->port_tab_dirty = 1;
		err = dev_write(d, d->port_flags + k, &f, 1);
		if (!err)
			err = dev_write(d, d->port_hits + k, &h, 8);
	}
	if (!err)
		err = port_flags_note(ctx, k, any);
	return err;
}

int xfg_map_update(xfg_ctx *ctx, int map, const void *key, const uint64_t *vals)
{
	int err = 0;
	if (!ctx || !key || !vals || keylen_of(map) < 0)
		return -EINVAL;
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	if (map == XFG_MAP_PORTS) {
		uint32_t k;
		if (port_key(key, &k))
			err = -E2BIG; /* array map: index out of range */
		else
			err = port_store(ctx, k, vals);
		goto out;
	}
	int mi = map - 1;
	struct xfg_table *t = &ctx->t[mi];
	int64_t s = xfg_table_find(t, key);
	if (s < 0) {
		struct meta_push mp = { ctx, mi, 0 };
		int64_t bw = -1;
		s = xfg_table_insert(t, key, ctx->ndev ? meta_changed : NULL, &mp, &bw);
		if (s < 0) {
			err = (int)s;
			goto out;
		}
		if ((err = mp.err))
			goto out;
		if (ctx->ndev && (uint64_t)s != t->nslots) {
			err = push_key(ctx, mi, (uint64_t)s);
			if (!err && bw >= 0)
				err = push_bloom(ctx, mi, bw);
		}
		if (err)
			goto out;
	}
	err = slot_store(ctx, mi, (uint64_t)s, vals, key);
out:
	pthread_mutex_unlock(&ctx->lock);
	return err;
}

int xfg_map_delete(xfg_ctx *ctx, int map, const void *key)
{
	int err = 0;
	if (!ctx || !key || keylen_of(map) < 0)
		return -EINVAL;
	if (map == XFG_MAP_PORTS)
		return -EINVAL; /* BPF array maps do not support delete */
	pthread_mutex_lock(&ctx->lock);
	int mi = map - 1;
	struct xfg_table *t = &ctx->t[mi];
	int64_t s = xfg_table_remove(t, key);
	if (s < 0) {
		err = (int)s;
		goto out;
	}
	{
		uint64_t zero[64] = { 0 };
		uint64_t *z = ctx->ndev > 64 ? calloc(ctx->ndev, 8) : zero;
		if (!z) {
			err = -ENOMEM;
			goto out;
		}
		err = slot_store(ctx, mi, (uint64_t)s, z, key);
		if (z != zero)
			free(z);
	}
	if (!err && (uint64_t)s != t->nslots && ctx->ndev)
		err = push_key(ctx, mi, (uint64_t)s);
	if (!err && xfg_table_bloom_needs_rebuild(t)) {
		xfg_table_bloom_rebuild(t);
		if (ctx->ndev)
			err = push_bloom(ctx, mi, -1);
	}
out:
	pthread_mutex_unlock(&ctx->lock);
	return err;
}

int xfg_map_get_next_key(xfg_ctx *ctx, int map, const void *key, void *next_key)
{
	int err = 0;
	if (!ctx || !next_key || keylen_of(map) < 0)
		return -EINVAL;
	if (map == XFG_MAP_PORTS) {
		/* BPF array semantics: next index; a missing/invalid key restarts at 0 */
		uint32_t k = 0;
		if (key) {
			memcpy(&k, key, 4);
			if (k >= XFG_PORT_MAP_ENTRIES)
				k = 0;
			else if (k + 1 >= XFG_PORT_MAP_ENTRIES)
				return -ENOENT;
			else
				k++;
		}
		memcpy(next_key, &k, 4);
		return 0;
	}
	pthread_mutex_lock(&ctx->lock);
	const struct xfg_table *t = &ctx->t[map - 1];
	int64_t after = -1;
	if (key)
		after = xfg_table_find(t, key); /* BPF htab: a missing key restarts at the first */
	int64_t s = xfg_table_next_slot(t, after);
	if (s < 0)
		err = -ENOENT;
	else
		err = xfg_table_slot_key(t, (uint64_t)s, next_key);
	pthread_mutex_unlock(&ctx->lock);
	return err;
}

int64_t xfg_map_count(xfg_ctx *ctx, int map)
{
	if (!ctx || keylen_of(map) < 0)
		return -EINVAL;
	if (map == XFG_MAP_PORTS)
		return ctx->port_count;
	return ctx->t[map - 1].count;
}

int64_t xfg_map_lookup_batch(xfg_ctx *ctx, int map, const void *keys, uint64_t n,
			     uint64_t *vals, uint8_t *present)
{
	int err = 0, kl = keylen_of(map);
	int64_t found = 0;
	if (!ctx || (!keys && n) || (!vals && n) || kl < 0)
		return -EINVAL;
	int nd = ctx->ndev ? ctx->ndev : 1;
	const struct xfg_table *t = map == XFG_MAP_PORTS ? NULL : &ctx->t[map - 1];
	size_t ns = t ? (size_t)t->nslots + 1 : XFG_PORT_MAP_ENTRIES;
	size_t fbytes = t ? xfg_table_img_bytes(t) : XFG_PORT_MAP_ENTRIES;
	uint8_t *flags = NULL;
	unsigned long long *hits = NULL;
	pthread_mutex_lock(&ctx->lock);
	if (ctx->ndev) {
		flags = malloc(fbytes * nd);
		hits = malloc(ns * 8 * nd);
		if (!flags || !hits) {
			err = -ENOMEM;
			goto out;
		}
		if (t && (err = qt_fold(ctx, map - 1)))
			goto out;
		for (int i = 0; i < ctx->ndev && !err; i++) {
			struct xfg_dev *d = &ctx->dev[i];
			const void *fsrc = t ? (const void *)d->m[map - 1].buckets : (const void *)d->port_flags;
			const unsigned long long *hsrc =
				t ? hits_view(ctx, d, map - 1)
				  : (ctx->reduced ? d->red_port_hits : d->port_hits);
			err = dev_read(d, flags + fbytes * i, fsrc, fbytes);
			if (!err)
				err = dev_read(d, hits + ns * i, hsrc, ns * 8);
		}
		if (err)
			goto out;
	}
	for (uint64_t i = 0; i < n; i++) {
		const uint8_t *k = (const uint8_t *)keys + (size_t)kl * i;
		int64_t s;
		if (!t) {
			uint32_t pk;
			s = port_key(k, &pk) ? -1 : (int64_t)pk;
		} else {
			s = xfg_table_find(t, k);
		}
		if (present)
			present[i] = s >= 0;
		for (int d = 0; d < nd; d++) {
			uint64_t v = 0;
			if (s >= 0) {
				if (!ctx->ndev) {
					v = t ? ctx->host_vals[map - 1][s] : ctx->host_port_vals[s];
				} else {
					uint8_t f = t ? flags[fbytes * d + xfg_table_flag_off(t, s)]
						      : flags[fbytes * d + s];
					v = (hits[ns * d + s] << XFG_COUNTER_SHIFT) | f;
				}
			}
			vals[i * nd + d] = v;
		}
		found += s >= 0;
	}
out:
	free(flags);
	free(hits);
	pthread_mutex_unlock(&ctx->lock);
	return err ? err : found;
}

/* vals[i] on every device (percpu = 0) or vals[i * nvals + d] (percpu = 1). */
static int update_batch(xfg_ctx *ctx, int map, const void *keys, const uint64_t *vals,
			uint64_t n, int percpu)
{
	int err = 0, kl = keylen_of(map);
	if (!ctx || (!keys && n) || (!vals && n) || kl < 0)
		return -EINVAL;
	const int nv = ctx->ndev ? ctx->ndev : 1;
#define VAL(i, d) (percpu ? vals[(i) * (uint64_t)nv + (d)] : vals[i])
	if (map == XFG_MAP_PORTS) {
		uint64_t v[64];
		uint64_t *vv = ctx->ndev > 64 ? calloc(ctx->ndev, 8) : v;
		if (!vv)
			return -ENOMEM;
		for (uint64_t i = 0; i < n && !err; i++) {
			for (int d = 0; d < nv; d++)
				vv[d] = VAL(i, d);
			err = xfg_map_update(ctx, map, (const uint8_t *)keys + 4 * i, vv);
		}
		if (vv != v)
			free(vv);
		return err;
	}
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	int mi = map - 1;
	struct xfg_table *t = &ctx->t[mi];
	size_t ns = (size_t)t->nslots + 1, ib = xfg_table_img_bytes(t);
	uint8_t *img = NULL;           /* per-device bucket images */
	unsigned long long *hits = NULL;
	int nd = ctx->ndev;
	int fresh = t->count == 0;     /* nothing on the devices worth preserving */

	if (nd) {
		img = malloc(ib * nd);
		hits = malloc(ns * 8 * nd);
		if (!img || !hits) {
			err = -ENOMEM;
			goto out;
		}
		if ((err = qt_fold(ctx, mi)))
			goto out;
		for (int i = 0; i < nd && !err; i++) {
			struct xfg_dev *d = &ctx->dev[i];
			if (!fresh) {
				err = dev_read(d, img + ib * i, d->m[mi].buckets, ib);
				if (!err)
					err = dev_read(d, hits + ns * i, d->m[mi].hits, ns * 8);
			} else {
				memset(img + ib * i, 0, ib);
				memset(hits + ns * i, 0, ns * 8);
			}
		}
		if (err)
			goto out;
	}
	for (uint64_t i = 0; i < n; i++) {
		const uint8_t *k = (const uint8_t *)keys + (size_t)kl * i;
		int64_t s = xfg_table_find(t, k);
		if (s < 0)
			s = xfg_table_insert(t, k, NULL, NULL, NULL);
		if (s < 0) {
			err = (int)s;
			break;
		}
		uint8_t any = 0, all = 63;
		for (int d = 0; d < nv; d++) {
			any |= VAL(i, d) & 63;
			all &= VAL(i, d) & 63;
		}
		flags_note(ctx, mi, (uint64_t)s, any, all, 0);
		if (nd) {
			for (int d = 0; d < nd; d++) {
				img[ib * d + xfg_table_flag_off(t, s)] = VAL(i, d) & 63;
				hits[ns * d + s] = VAL(i, d) >> XFG_COUNTER_SHIFT;
			}
		} else {
			ctx->host_vals[mi][s] = VAL(i, 0);
		}
	}
#undef VAL
	/* merge host keys + meta into each device image (flags stay per device)
	 * and upload; also on partial failure: keys inserted so far stay */
	for (int i = 0; i < nd; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		uint8_t *di = img + ib * i;
		for (uint64_t b = 0; b <= t->nbuckets; b++) {
			memcpy(di + b * XFG_BUCKET_BYTES, t->img + b * XFG_BUCKET_BYTES, XFG_KEY_AREA);
			memcpy(di + b * XFG_BUCKET_BYTES + XFG_META_OFF,
			       t->img + b * XFG_BUCKET_BYTES + XFG_META_OFF, 4);
		}
		int e2 = dev_write(d, d->m[mi].buckets, di, ib);
		if (!e2)
			e2 = dev_write(d, d->m[mi].hits, hits + ns * i, ns * 8);
		if (!e2)
			e2 = dev_write(d, d->m[mi].bloom, t->bloom, (size_t)t->bloom_words * 4);
		if (e2 && !err)
			err = e2;
	}
out:
	free(img);
	free(hits);
	pthread_mutex_unlock(&ctx->lock);
	return err;
}

int xfg_map_update_batch(xfg_ctx *ctx, int map, const void *keys, const uint64_t *vals,
			 uint64_t n)
{
	return update_batch(ctx, map, keys, vals, n, 0);
}

int xfg_map_update_batch_percpu(xfg_ctx *ctx, int map, const void *keys, const uint64_t *vals,
				uint64_t n)
{
	return update_batch(ctx, map, keys, vals, n, 1);
}

/* ------------------------------------------------------------------ classify */
/* Rebuild a device's LDS port image from its flag bytes: the open-addressed
 * table (linear probing from xfg_port_slot()) when at most XFG_PORT_TAB_MAX
 * ports carry flags, else the nibble map of every port's low 4 flag bits
 * (the only ones CHECK_MAP can test). */
static int port_tab_refresh_locked(struct xfg_dev *d);


/* A partition's local-index range of a hit log over @span QT slots. */
static uint64_t qt_log_hist(uint64_t span)
{
	return ((span + 16 * XFG_LOG_PARTS - 1) / (16 * XFG_LOG_PARTS)) * 16;
}

/* Whether the count kernel covers the hit log of a QT of @span slots: in
 * passes of its LDS histogram (u32 local indices past 65536), or with both
 * lookup directions in one pass (that kernel logs u16 indices only). */
static int qt_log_fits(uint64_t span, int both)
{
	const uint64_t h = qt_log_hist(span);
	return both ? h <= XFG_LOG_HIST_MAX : h <= (uint64_t)XFG_LOG_HIST_MAX * XFG_LOG_PASSES_MAX;
}

static int port_tab_refresh(struct xfg_dev *d)
{
	/* (under the device lock: launch_batch reads the image's kind and
	 * displacement there; lock order ctx->lock, then d->lock) */
	pthread_mutex_lock(&d->lock);
	int err = port_tab_refresh_locked(d);
	pthread_mutex_unlock(&d->lock);
	return err;
}

static int port_tab_refresh_locked(struct xfg_dev *d)
{
	uint32_t tab[XFG_PORT_TAB];
	uint32_t n = 0, disp = 0;
	if (!d->port_tab_dirty)
		return 0;
	memset(tab, 0, sizeof(tab));
	for (uint32_t k = 0; k < XFG_PORT_MAP_ENTRIES; k++) {
		if (!d->port_flags_h[k])
			continue;
		if (++n > XFG_PORT_TAB_MAX)
			break;
		uint32_t sl = xfg_port_slot(k), dd = 0;
		while (tab[sl]) {
			sl = (sl + 1) & (XFG_PORT_TAB - 1);
			dd++;
		}
		tab[sl] = ((uint32_t)d->port_flags_h[k] << 16) | k;
		if (dd > disp)
			disp = dd;
	}
	d->port_tab_ok = n <= XFG_PORT_TAB_MAX;
	d->port_tab_disp = disp;
	d->port_tab_dirty = 0;
	if (d->port_tab_ok)
		return dev_write(d, d->port_tab, tab, sizeof(tab));
	uint32_t *nib = calloc(XFG_PORT_NIB_WORDS, 4);
	if (!nib)
		return -ENOMEM;
	for (uint32_t k = 0; k < XFG_PORT_MAP_ENTRIES; k++)
		nib[k >> 3] |= (uint32_t)(d->port_flags_h[k] & 15) << ((k & 7) * 4);
	int err = dev_write(d, d->port_nib, nib, XFG_PORT_NIB_WORDS * 4);
	free(nib);
	return err;
}

static int scratch(struct xfg_dev *d, void **p, uint64_t *have, uint64_t bytes);

/* Bring the quotient index of the IPv4 map up to date for lookups of mask
 * @live (ctx->lock held): rebuild the host image when the map changed, then
 * upload it to @d when its copy is older (under d->lock: launch_batch reads
 * the index's parameters there). */
static int qt_refresh(xfg_ctx *ctx, struct xfg_dev *d, uint32_t live)
{
	int err = 0;
	if (ctx->qt_dirty || !ctx->qt_gen || ctx->qt.live != live) {
		if ((err = xfg_qt_build(&ctx->qt, &ctx->t[0], ctx->flag_or[0], live,
					ctx->t[0].seed ^ 0x51ed2701u)))
			return err;
		ctx->qt_dirty = 0;
		if (!++ctx->qt_gen)
			ctx->qt_gen = 1;
	}
	if (d->qt_gen == ctx->qt_gen)
		return 0;
	const uint64_t ib = (uint64_t)ctx->qt.nimg * (1ull << ctx->qt.bits) * XFG_QT_BUCKET;
	const uint64_t tb = (uint64_t)ctx->qt.nimg * ctx->qt.nslots * 4;
	pthread_mutex_lock(&d->lock);
	if (!(err = qt_fold_locked(d)) &&   /* (through the index being replaced) */
	    !(err = scratch(d, (void **)&d->qt_img, &d->qt_img_bytes, ib)) &&
	    !(err = scratch(d, (void **)&d->qt_trans, &d->qt_trans_bytes, tb)) &&
	    !(err = dev_write(d, d->qt_img, ctx->qt.img, ib)) &&
	    !(err = dev_write(d, d->qt_trans, ctx->qt.trans, tb))) {
		d->qt_gen = ctx->qt_gen;
		d->qt_bits = ctx->qt.bits;
		d->qt_seed = ctx->qt.seed;
		d->qt_live = ctx->qt.live;
		d->qt_nimg = ctx->qt.nimg;
		d->qt_n = ctx->qt.nimg * ctx->qt.nslots;
	}
	pthread_mutex_unlock(&d->lock);
	return err;
}

/* The Ethernet map as the Ethernet-key kernel's key table (ctx->lock held):
 * rebuilt on the host after an edit, then uploaded to @d when its copy is
 * older.  A key at home xfg_ek_home, linear probing; slots
 * at least twice the keys.  ek_ok 0 (the generic kernel instead): more than
 * XFG_EK_MAX_KEYS keys, or a flag byte that differs between devices. */
static int ek_refresh(xfg_ctx *ctx, struct xfg_dev *d)
{
	int err = 0;
	const struct xfg_table *t = &ctx->t[2];
	if (!ctx->ek_gen || ctx->ek_seen != ctx->ek_edits) {
		ctx->ek_seen = ctx->ek_edits;
		if (!++ctx->ek_gen)
			ctx->ek_gen = 1;
		ctx->ek_ok = t->count <= XFG_EK_MAX_KEYS && !ctx->flag_cnt[2][7];
		if (!ctx->ek_ok)
			return 0;
		uint32_t sl = 64;
		while (sl < 2 * t->count)
			sl *= 2;
		memset(ctx->ek_host, 0, (size_t)sl * 16);
		ctx->ek_slots = sl;
		ctx->ek_disp = 0;
		for (int64_t s = xfg_table_next_slot(t, -1); s >= 0; s = xfg_table_next_slot(t, s)) {
			uint8_t k[8] = { 0 };
			if (xfg_table_slot_key(t, (uint64_t)s, k))
				continue;
			uint32_t lo, hi = k[4] | (uint32_t)k[5] << 8;
			memcpy(&lo, k, 4);
			uint32_t e = xfg_ek_home(lo, hi, t->seed, (uint32_t)__builtin_ctz(sl)), dsp = 0;
			while (ctx->ek_host[4 * e + 3] & XFG_EK_VALID) {
				e = (e + 1) & (sl - 1);
				dsp++;
			}
			ctx->ek_host[4 * e] = lo;
			ctx->ek_host[4 * e + 1] = hi;
			ctx->ek_host[4 * e + 2] = (uint32_t)s;
			ctx->ek_host[4 * e + 3] = XFG_EK_VALID | (ctx->flag_or[2][s] & 63);
			if (dsp > ctx->ek_disp)
				ctx->ek_disp = dsp;
		}
	}
	if (!ctx->ek_ok || d->ek_gen == ctx->ek_gen)
		return 0;
	pthread_mutex_lock(&d->lock);
	if (!(err = scratch(d, (void **)&d->ek_img, &d->ek_img_bytes, (uint64_t)XFG_EK_SLOTS_MAX * 16)) &&
	    !(err = dev_write(d, d->ek_img, ctx->ek_host, (size_t)ctx->ek_slots * 16))) {
		d->ek_gen = ctx->ek_gen;
		d->ek_slots = ctx->ek_slots;
		d->ek_disp = ctx->ek_disp;
	}
	pthread_mutex_unlock(&d->lock);
	return err;
}

static int fill_kargs(xfg_ctx *ctx, struct xfg_dev *d, const struct xfg_batch *b,
		      uint8_t *verdicts, struct xfg_kargs *a)
{
	memset(a, 0, sizeof(*a));
	int err = port_tab_refresh(d);
	if (err)
		return err;
	struct xfg_tdesc *td[NMAPS_HASH] = { &a->t4, &a->t6, &a->te };
	for (int i = 0; i < NMAPS_HASH; i++) {
		xfg_table_desc(&ctx->t[i], td[i]);
		td[i]->buckets = d->m[i].buckets;
		td[i]->bloom = d->m[i].bloom;
		td[i]->hits = d->m[i].hits;
		td[i]->fmask = census_mask(ctx->flag_cnt[i]);
	}
	a->port_fmask = census_mask(ctx->port_flag_cnt);
	uint64_t gb = 0;
	for (int i = 0; i < NMAPS_HASH; i++) {
		a->gbase[i] = (uint32_t)gb;
		gb += (uint64_t)ctx->t[i].nslots + 1;
	}
	a->gbase[3] = (uint32_t)gb;
	a->port_hits = d->port_hits;
	a->port_count = ctx->port_count;
	a->port_tab = d->port_tab_ok ? d->port_tab : NULL;
	a->port_nib = d->port_nib;
	a->port_tab_disp = d->port_tab_disp;
	a->stats = d->stats;
	a->data = b->data;
	a->offsets = b->offsets;
	a->lens = b->lens;
	a->n = b->count;
	a->stride = b->stride;
	a->lens_u16 = b->lens_u16;
	a->verdicts = verdicts;
	/* Header window: 64 bytes for fixed strides (a parse that reaches past
	 * it -- IPv6/TCP's doff at byte 66, long IPv6 extension chains -- is a
	 * deferred walk over the frame in HBM), unless the context asked for
	 * 128 (xfg_open_opts.window: such frames then stay on the fast path);
	 * frames at offsets stage 128 bytes in the general kernel.  On C4/C5's
	 * 1536-byte slots the 64-byte window was 14 % faster (r04 session 16). */
	a->window = (!b->offsets && b->stride && (b->stride <= 64 || ctx->window == 64)) ? 64 : 128;
#ifdef XFG_DIAG
	const char *wn = getenv("XFG_WINDOW");   /* "64" / "128" above a 64-byte stride */
	if (wn && !strcmp(wn, "64") && !b->offsets && b->stride)
		a->window = 64;
	else if (wn && !strcmp(wn, "128") && b->stride > 64)
		a->window = 128;
#endif
	/* The pipelined kernel takes every fixed-stride batch whose windows can
	 * be loaded without a length (stride >= window, 16-byte aligned; packet
	 * indices fit its 32-bit deferred lists); the general kernel the rest. */
	a->pipe = !b->offsets && b->stride >= a->window && !(b->stride & 15) &&
		  !((uintptr_t)b->data & 15) && b->count < (1ull << 32) && b->stride < 65536;
#ifdef XFG_DIAG
	const char *ks = getenv("XFG_KERNEL");   /* diagnostics build only */
	if (ks && !strcmp(ks, "general"))
		a->pipe = 0;
#endif
	a->dense = a->pipe && a->stride == a->window;
	/* key mode 1: no Ethernet or IPv6 lookup can hit (flag census), so the
	 * pipelined kernel carries IPv4 keys only */
	int eth_live = (ctx->prog_features & XFG_FEAT_ETHERNET) && a->te.count && (a->te.fmask & 3);
	int v6_live = (ctx->prog_features & XFG_FEAT_IPV6) && a->t6.count && (a->t6.fmask & 3);
	a->km = (ctx->prog_features & XFG_FEAT_IPV4) && !eth_live && !v6_live;
	/* (IPv6 keys live, Ethernet keys not: the quotient-index kernel may still
	 * take the batch, sending every IPv6 frame to its deferred path) */
	const int km6 = (ctx->prog_features & XFG_FEAT_IPV4) && !eth_live && v6_live;
	a->v6d = 0;
	/* per-lane u32 byte sums in the pipelined kernel: bound them */
	if (a->pipe && (uint64_t)a->stride * (((b->count + 63) / 64 + 1023) / 1024 + 1) >= (1ull << 32))
		a->pipe = 0;
#ifdef XFG_DIAG
	const char *dm = getenv("XFG_DIAG_MASK");   /* pipelined IPv4-key kernel: drop a cost */
	if (dm && *dm)
		a->diag = (uint32_t)strtoul(dm, NULL, 0);
	const char *tsp = getenv("XFG_TSTAMP");   /* device buffer for the QT kernel's phase stamps */
	if (tsp && *tsp)
		a->tstamp = (unsigned long long *)(uintptr_t)strtoull(tsp, NULL, 0);
	const char *kk = getenv("XFG_KERNEL");   /* "split": parse + lookup passes */
	if (kk && !strcmp(kk, "split"))
		a->split = a->pipe && a->km;
	const char *bo = getenv("XFG_BLOOM");    /* "off": lookup pass without the prefilter */
	if (bo && !strcmp(bo, "off") && !(a->t4.count && (a->t4.fmask & 3) == 3))
		a->bloom_off = 1;
	const char *em = getenv("XFG_EMPTY");   /* every table empty: stream + parse only */
	if (em && !strcmp(em, "1")) {
		a->t4.count = a->t6.count = a->te.count = 0;
		a->port_count = 0;
	}
#endif
	/* the Ethernet-key kernel (kind 6): the Ethernet-only programs, their
	 * map as an LDS key table -- every lookup answered in LDS, no frame
	 * byte past the two addresses read */
	/* (and, since round 6, for the generic pipelined kernel -- live
	 * Ethernet keys beside IP keys: dny_all / alw_all with a few MAC rules --
	 * which answers both Ethernet lookups from the same table in LDS) */
	const int ek_only = !(ctx->prog_features & (XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_TCP | XFG_FEAT_UDP));
	int ek = a->pipe && (ctx->prog_features & XFG_FEAT_ETHERNET) && (ek_only || eth_live);
#ifdef XFG_DIAG
	const char *eo = getenv("XFG_EK");   /* "off": the generic pipelined kernel */
	if (eo && !strcmp(eo, "off"))
		ek = 0;
#endif
	if (ek) {
		if ((err = ek_refresh(ctx, d)))
			return err;
		if (ctx->ek_ok)
			a->ek = d->ek_img;   /* (parameters: launch_batch, under d->lock) */
	}
	/* (live Ethernet keys, no IPv6 key, the Ethernet map as the LDS key
	 * table: the quotient-index kernel answers the Ethernet lookups from
	 * the table ahead of its IPv4 lookups -- since round 6; else the
	 * generic pipelined kernel takes the batch) */
	const int kme = (ctx->prog_features & XFG_FEAT_IPV4) && eth_live && !v6_live && a->ek && !ek_only;
	/* the quotient index (kind 5 kernel): the IPv4-key kernel with one or
	 * both IPv4 lookup directions live, the same flags on every device, and
	 * a map large enough that the prefilter + bucket-line chain leaves L2;
	 * its hit log must fit the count kernel's histogram */
	if (a->pipe && (a->km || km6 || kme) && !a->split) {
		/* (both directions live: up to two images, twice the QT slots) */
		const int dl = a->t4.count && (a->t4.fmask & 2), sl = a->t4.count && (a->t4.fmask & 1);
		const int ok = (dl | sl) && !ctx->flag_cnt[0][7] &&
			       qt_log_fits(((uint64_t)XFG_QT_SLOTS << xfg_qt_bits_for(a->t4.count)) << (dl & sl),
					   dl & sl);
		int use = ok && a->t4.count >= ctx->qt_min_keys;
#ifdef XFG_DIAG
		const char *qo = getenv("XFG_QT");   /* "off" / "on" (any size) */
		if (qo && !strcmp(qo, "off"))
			use = 0;
		else if (qo && !strcmp(qo, "on"))
			use = ok;
#endif
		if (use) {
			int err2 = qt_refresh(ctx, d, (dl ? 2u : 0u) | (sl ? 1u : 0u));
			if (err2)
				return err2;
			a->qt = d->qt_img;   /* (parameters: launch_batch, under d->lock) */
			if (!a->km) {
				a->km = 1;
				a->v6d = !kme;
			}
		}
	}
	return 0;
}

/* Device scratch buffer of at least @bytes (grown on demand; the old one may
 * still be in use by a launch queued on the device stream: wait for it). */
static int scratch(struct xfg_dev *d, void **p, uint64_t *have, uint64_t bytes)
{
	if (bytes <= *have)
		return 0;
	int err = hip_err(hipStreamSynchronize(d->stream));
	if (err)
		return err;
	hipFree(*p);
	*p = NULL;
	*have = 0;
	err = hip_err(hipMalloc(p, bytes));
	if (!err)
		*have = bytes;
	return err;
}

/* classify launches on the device's own stream (every classify of a device
 * is serialised there), ordered after and before @user (a caller's stream,
 * or NULL).  The per-launch scratch (hit log, deferred lists) is sized and
 * used under the device lock, so concurrent callers never see a buffer
 * being replaced. */
static int launch_batch(xfg_ctx *ctx, struct xfg_dev *d, const struct xfg_kargs *a0,
			void *user, int iters)
{
	int err = 0;
	struct xfg_kargs a = *a0;
	const char *cm = NULL;
	int nolog = 0;   /* (diagnostics: every kernel without the hit log) */
#ifdef XFG_DIAG
	cm = getenv("XFG_COUNT");   /* diagnostics build only: "atomic" */
	if (cm && !strcmp(cm, "atomic"))
		a.qt = NULL;             /* (the QT kernel's counting is the log, or no log) */
	const char *lg = getenv("XFG_LOG");   /* "off": counters by LDS cache + atomics */
	nolog = lg && !strcmp(lg, "off");
#endif
	/* small rule sets: a direct LDS counter per hash-map slot (their few
	 * counters are hot: more than the LDS counter cache holds) */
	if (a.gbase[3] <= XFG_DCNT_MAX)
		a.dcnt = a.gbase[3];       /* every hash-map counter */
	else if (a.gbase[1] <= XFG_DCNT_MAX)
		a.dcnt = a.gbase[1];       /* the IPv4 map's counters */
	pthread_mutex_lock(&d->lock);
	/* the port image in stream order at this launch (another caller's
	 * port_tab_refresh may have rewritten it since fill_kargs; both hold
	 * d->lock for that): its kind and its longest displacement */
	a.port_tab = d->port_tab_ok ? d->port_tab : NULL;
	a.port_tab_disp = d->port_tab_disp;
	/* the hit log (below) decides whether the quotient-index kernel can run:
	 * it counts through the log only.  Where the log cannot be set up (every
	 * counter has a direct LDS counter, or the grid has more workgroups than
	 * the log has slices) the IPv4-key kernel takes the batch instead. */
	/* (a few keys in all -- C1's 8 MAC rules -- are hot: the LDS counter
	 * cache holds every one of them, where the log would send their hits
	 * through a handful of overfull partitions to contended atomics) */
	const uint64_t nkeys = (uint64_t)a.t4.count + a.t6.count + a.te.count;
	const int logged = nkeys > XFG_LOG_MIN_KEYS;
	/* (the Ethernet-key kernel -- the Ethernet-only programs -- counts in LDS;
	 * the generic kernel with the LDS key table logs its IP hits as usual) */
	const int ek_only = a.pipe && a.ek && !(ctx->prog_features & (XFG_FEAT_IPV4 | XFG_FEAT_IPV6 | XFG_FEAT_TCP | XFG_FEAT_UDP));
	const int log_no = !a.pipe || !logged || a.dcnt >= a.gbase[3] || ek_only || (cm && !strcmp(cm, "atomic"));
	/* (a batch of fewer packets than counters: the count kernel's pass over
	 * every counter costs more than the atomics it saves -- C5's 15M + 1M
	 * rules at 2^23 packets: 0.45 ms with atomics, 0.65-0.71 with the log;
	 * C4's 1M at 2^23 and C3's at 2^24 and 2^26 keep the log, r04 sessions
	 * 16 and 18) */
	int qt_nolog = 0;
	if (a.qt) {
		const int k5 = 5, wi5 = a.window > 64;
		const int pc = d->occ[k5][wi5][(a.dcnt > 0) | (!a.port_tab && a.port_count ? 2 : 0) | (a.bl_lds ? 4 : 0) |
					      (a.ek ? 8 : 0)];
		const uint64_t pw = (uint64_t)xfg_classify_threads(k5, a.window);
		uint64_t g5 = (uint64_t)d->ncu * (pc > 0 ? pc : 1), need5 = (a.n + pw - 1) / pw;
		if (g5 > need5)
			g5 = need5 ? need5 : 1;
		/* (a log the count kernel cannot take: the index kernel counts
		 * through its LDS counter cache and atomics instead) */
		if (log_no)
			a.qt = NULL;
		/* (with the count wave the log's count costs the launch nothing:
		 * then the log from XFG_CW_LOG_MIN packets instead of twice the
		 * QT slots -- the atomics it saves are the slow part at C4's
		 * per-GPU shard of 2^21 packets) */
		const int occ_c5 = (a.dcnt > 0) | (!a.port_tab && a.port_count ? 2 : 0);
		const int cw_cap = qt_log_hist(d->qt_n) <= XFG_CW_HIST_MAX && a.window <= 64 && !a.v6d && !a.ek &&
				   2 * g5 <= XFG_LOG_SLICES_MAX && d->occ[7][0][occ_c5] > 0;
		uint64_t cw_min = XFG_CW_LOG_MIN;
#ifdef XFG_DIAG
		const char *cm2 = getenv("XFG_CW_LOG_MIN");   /* packets from which the count wave's log runs */
		if (cm2 && *cm2)
			cw_min = strtoull(cm2, NULL, 0);
		const char *cwo = getenv("XFG_CW");
		if (cwo && !strcmp(cwo, "off"))
			cw_min = ~0ull;
#endif
		if (nolog || g5 > XFG_LOG_SLICES_MAX || !qt_log_fits(d->qt_n, d->qt_live == 3) ||
		    (2 * (uint64_t)d->qt_n > a.n && !(cw_cap && a.n >= cw_min)))
			qt_nolog = 1;
		/* (the log from twice as many packets as QT slots: at as many, C3's
		 * and C4's 1M rules at 2^21 packets ran 0.068 / 0.088 ms with it and
		 * 0.060 / 0.080 without; at twice, the same; at four times, the log
		 * 10 % faster -- profiles/archive/r05_s39_session.log) */
	}
	const int log_off = log_no || nolog ||
			    (!a.qt && (uint64_t)a.gbase[3] + XFG_PORT_MAP_ENTRIES > a.n);
	if (!a.qt && a.v6d) {   /* (the IPv6 keys need the general kernel then) */
		a.km = 0;
		a.v6d = 0;
	}
	/* the generic pipelined kernel: small maps' Bloom filters staged in LDS */
	a.bl_lds = 0;
	if (!a.pipe)   /* (header windows of the host path: the general kernel) */
		a.ek = NULL;
	if (a.ek) {   /* the key table in stream order at this launch */
		a.ek = d->ek_img;
		a.ek_slots = d->ek_slots;
		a.ek_disp = d->ek_disp;
	}
	if (a.pipe && !a.km && !ek_only) {
		const struct xfg_tdesc *tt[3] = { &a.t4, &a.te, &a.t6 };
		uint32_t tot = 0;
		for (int i = 0; i < 3; i++) {
			a.bl_off[i] = ~0u;
			/* (the LDS key table answers the Ethernet lookups) */
			if (tt[i]->count && tt[i]->bloom_words && !(i == 1 && a.ek)) {
				a.bl_off[i] = tot;
				tot += tt[i]->bloom_words;
			}
		}
		if (tot <= XFG_BLOOM_LDS_MAX)
			a.bl_lds = tot;
#ifdef XFG_DIAG
		const char *bl = getenv("XFG_BLOOM_LDS");   /* "off": the words from memory */
		if (bl && !strcmp(bl, "off"))
			a.bl_lds = 0;
#endif
	}
	const int kind = ek_only ? 6 : a.pipe ? (a.km ? (a.split ? 3 : (a.qt ? 5 : 2)) : 1) : 0, wi = a.window > 64;
	if (a.qt) {   /* the index in stream order at this launch */
		a.qt = d->qt_img;
		a.qt_trans = d->qt_trans;
		a.qt_bits = d->qt_bits;
		a.qt_seed = d->qt_seed;
		a.qt_live = d->qt_live;
		a.qt_n = d->qt_n;
		/* the second (src) lookup's image and its slots' offset: the same
		 * image at offset 0 when one serves both directions */
		a.qt_base = d->qt_nimg == 2 ? d->qt_n / 2 : 0;
		a.qt2 = d->qt_img + (uint64_t)a.qt_base * 2 / 4;
		/* its QT-order counts (zeroed when (re)allocated; a resize only
		 * follows a fold: qt_refresh) */
		/* (two halves: the log's counts, the atomics' -- xfg_kargs.qt_hitx) */
		const uint64_t qb = (uint64_t)d->qt_n * 8, had = d->qt_hits_bytes;
		if ((err = scratch(d, (void **)&d->qt_hits, &d->qt_hits_bytes, qb)))
			goto out;
		if (d->qt_hits_bytes != had &&
		    (err = hip_err(hipMemsetAsync(d->qt_hits, 0, d->qt_hits_bytes, d->stream))))
			goto out;
		a.qt_hits = d->qt_hits;
		a.qt_hitx = d->qt_hits + d->qt_n;
	}
	int per_cu = d->occ[kind][wi][(a.dcnt > 0) | (!a.port_tab && a.port_count ? 2 : 0) |
				     (a.bl_lds ? 4 : 0) | (a.ek ? 8 : 0)];
#ifdef XFG_DIAG
	const char *g = getenv("XFG_GRID_PER_CU");
	if (g && *g)
		per_cu = (int)strtol(g, NULL, 0);
#endif
	const uint64_t per_wg = (uint64_t)xfg_classify_threads(kind, a.window);
	uint64_t grid = (uint64_t)d->ncu * (per_cu > 0 ? per_cu : 1);
	uint64_t need = (a.n + per_wg - 1) / per_wg;
	if (grid > need)
		grid = need ? need : 1;

	if (a.split) {
		/* the parse pass: its own persistent grid */
		uint64_t gp = (uint64_t)d->ncu * (d->occ[4][wi][0] > 0 ? d->occ[4][wi][0] : 1);
		uint64_t tpw = (uint64_t)xfg_classify_threads(4, a.window);   /* packets per round */
		uint64_t np = (a.n + tpw - 1) / tpw;
		a.grid_parse = (uint32_t)(gp < np ? gp : (np ? np : 1));
	}

	if (a.split) {
		/* parse-pass records: key a, ports, key b (both directions live) */
		int both = a.t4.count && (a.t4.fmask & 3) == 3;
		uint64_t per = (uint64_t)a.n * 4;
		if ((err = scratch(d, (void **)&d->rec, &d->rec_bytes, per * (both ? 3 : 2))))
			goto out;
		a.rec_ka = d->rec;
		a.rec_port = d->rec + a.n;
		a.rec_kb = both ? d->rec + 2 * a.n : NULL;
	}
	if (a.pipe && !ek_only) {   /* (the Ethernet-key kernel defers nothing) */
		/* one deferred list per wave, room for every packet of its tiles --
		 * a quarter more than a fixed share: the quotient-index kernel's
		 * waves take their workgroup's tiles as they go (XFG_QT_DYN), at
		 * most defer_cap / 64 each */
		uint64_t nw = grid * (per_wg / 64), nt = (a.n + 63) / 64;
		uint64_t per = (nt + nw - 1) / nw;
		uint64_t cap = (per + per / 4 + 2) * 64;
		if ((err = scratch(d, (void **)&d->defer, &d->defer_bytes, nw * cap * 4)))
			goto out;
		a.defer = d->defer;
		a.defer_cap = (uint32_t)cap;
		/* (diagnostics: the quotient-index kernel lists its deferred
		 * packets for xfg_defer_kernel, two workgroups a CU over every
		 * list -- 1-3 % slower than each wave's own tail on C3 and C5,
		 * r04 session 19) */
		int sep = 0;
#ifdef XFG_DIAG
		const char *dfe = getenv("XFG_DEFER");   /* "kernel" */
		sep = dfe && !strcmp(dfe, "kernel") && kind == 5 && nw <= XFG_DEFER_SRC_MAX;
#endif
		if (sep) {
			if ((err = scratch(d, (void **)&d->defer_n, &d->defer_n_bytes, nw * 4)))
				goto out;
			a.defer_n = d->defer_n;
			a.defer_nsrc = (uint32_t)nw;
			a.defer_sep = 1;
			a.defer_grid = (uint32_t)d->ncu * 2;
		}
	}
	/* IPv6 rules beside the index: their lookups in the kernel's loop (1:
	 * one IPv6 direction can hit, one line a frame; 2: both, the src line
	 * beside the dst one), beside one live IPv4 direction or both (the
	 * index never takes both directions with the u32 log: qt_log_fits) */
	a.v6p = !(a.qt && a.v6d) ? 0u
		: (a.t6.fmask & 3) == 3u ? 2u : (a.t6.fmask & 3) != 0 ? 1u : 0u;
#ifdef XFG_DIAG
	const char *v6e = getenv("XFG_V6P");   /* "off": every IPv6 frame deferred */
	if (v6e && !strcmp(v6e, "off"))
		a.v6p = 0;
#endif
	/* hit log (pipelined kernels): the hash-map counters without a direct
	 * LDS counter, when the count kernel's histogram covers them; the wave
	 * regions share the deferred lists' bound, the partition buffers hold
	 * twice a uniform share (a fuller one spills to atomics) */
	/* (with the quotient index the log holds QT slots only: its span) */
	uint64_t total = a.qt ? (uint64_t)a.qt_n : (uint64_t)a.gbase[3] + XFG_PORT_MAP_ENTRIES;
	uint64_t hist = ((total + 16 * XFG_LOG_PARTS - 1) / (16 * XFG_LOG_PARTS)) * 16;
	/* (a range past one histogram: the count kernel takes it in passes; past
	 * 65536 local indices the slices hold u32) */
	const int pwide = hist > 65536;
	const int logs = !log_off && !qt_nolog && hist <= (uint64_t)XFG_LOG_HIST_MAX * XFG_LOG_PASSES_MAX &&
			 grid <= XFG_LOG_SLICES_MAX;
	/* slice (partition, workgroup): twice a uniform share of the most the
	 * workgroup's waves can log (a fuller one spills) */
	/* (a workgroup's tiles are a fixed share whichever of its waves takes
	 * them: the share, not the deferred lists' room) */
	const uint64_t wg_nw = per_wg / 64, wg_all = grid * wg_nw;
	const uint64_t wg_max = wg_nw * (((a.n + 63) / 64 + wg_all - 1) / wg_all) * 64;
	const uint64_t pcap = (2 * ((wg_max + XFG_LOG_PARTS - 1) / XFG_LOG_PARTS) + 64 + 7) & ~7ull;
	/* the quotient-index kernel's logs of up to K launches side by side in
	 * the partition buffers, counted by one count kernel (its fixed cost
	 * -- a pass over every QT-order count -- paid once per K launches);
	 * every other log is counted after its own launch */
	uint64_t K = 1;
	if (logs && a.qt) {
		K = XFG_LOG_PEND_MAX;
#ifdef XFG_DIAG
		const char *lp = getenv("XFG_LOG_PEND");   /* launches per count kernel (1: round 4) */
		if (lp && *lp)
			K = strtoul(lp, NULL, 0) ? strtoul(lp, NULL, 0) : 1;
#endif
		while (K > 1 && K * grid > XFG_LOG_SLICES_MAX)
			K--;
	}
	/* the count wave (since round 6): the quotient-index kernel's ninth wave
	 * counts the previous launch's log while the others classify, so no
	 * count kernel runs between launches -- two sets of slices used in
	 * turn; for a 64-byte window, a u16 log in one histogram of at most
	 * XFG_CW_HIST_MAX (C3's 1M rules: 8192), no IPv6 lookups in the loop,
	 * and the kernel launchable with its histogram */
	const int occ_c = (a.dcnt > 0) | (!a.port_tab && a.port_count ? 2 : 0);
	/* (measured, profiles/r06_s2_session.log: C3 at 2^24 0.294 against
	 * 0.299 ms a launch; at 2^26 no better -- there the count kernel's
	 * cost is its proportional part, which the count wave pays inside the
	 * launch: it runs below XFG_CW_MAX_PACKETS) */
	/* (the LDS Ethernet table and the histogram do not fit beside each other) */
	int cw = logs && a.qt && !pwide && hist <= XFG_CW_HIST_MAX && a.window <= 64 && !a.v6p && !a.ek &&
		 2 * grid <= XFG_LOG_SLICES_MAX && d->occ[7][0][occ_c] > 0 && a.n < XFG_CW_MAX_PACKETS;
#ifdef XFG_DIAG
	const char *cwe = getenv("XFG_CW");   /* "off": the count kernel every XFG_LOG_PEND launches */
	if (cwe && !strcmp(cwe, "off"))
		cw = 0;
#endif
	if (cw)
		K = 2;
	/* (the QT kernel's waves taking their workgroup's tiles as they go,
	 * C3 on one box: 2^26 1.059-1.061 against 1.089-1.092 ms, 2^24
	 * 0.294-0.296 against 0.304-0.306, 2^21 equal; C4 at 2^21 1.5 % slower
	 * -- profiles/r06_s13_session.log) */
	uint64_t dyn_min = XFG_QT_DYN_MIN;
#ifdef XFG_DIAG
	const char *dme = getenv("XFG_QT_DYN_MIN");   /* packets from which they do */
	if (dme && *dme)
		dyn_min = strtoull(dme, NULL, 0);
#endif
	a.qt_dyn = a.qt && a.n >= dyn_min;
	/* logs pending from earlier launches: counted first unless this one
	 * appends to them -- or, in the count wave's mode, counts them (the
	 * same shape, the same counts) */
	const int append = logs && K > 1 && d->log_pend && d->log_grid == grid &&
			   d->log_args.pcap == pcap && d->log_args.pslices == K * grid &&
			   d->log_args.log_span == hist && d->log_args.pwide == (uint32_t)pwide &&
			   d->log_args.qt_hits == a.qt_hits && d->log_args.qt_n == a.qt_n &&
			   d->log_cw == (uint32_t)cw;
	if (d->log_pend && !append && (err = log_flush_locked(d)))
		goto out;
	if (logs) {
		/* (the quotient-index kernel combines its log in LDS and writes
		 * the partition buffers itself: no per-wave regions) */
		if ((!a.qt && (err = scratch(d, (void **)&d->tlog, &d->tlog_bytes,
					     grid * (per_wg / 64) * (uint64_t)a.defer_cap * 4))) ||
		    (err = scratch(d, (void **)&d->pbuf, &d->pbuf_bytes,
				   ((uint64_t)XFG_LOG_PARTS * K * grid * pcap + 1024) * (pwide ? 4 : 2))) ||   /* (+ the count kernel's overread) */
		    (err = scratch(d, (void **)&d->pfill, &d->pfill_bytes,
				   (uint64_t)XFG_LOG_PARTS * K * grid * 4)))
			goto out;
		a.tlog = a.qt ? NULL : d->tlog;
		a.pbuf = d->pbuf;
		a.pfill = d->pfill;
		a.pcap = (uint32_t)pcap;
		a.pslices = (uint32_t)(K * grid);
		a.pslice0 = 0;
		a.pcount = (uint32_t)grid;
		a.log_hist = (uint32_t)(hist < XFG_LOG_HIST_MAX ? hist : XFG_LOG_HIST_MAX);
		a.log_span = (uint32_t)hist;
		a.pwide = (uint32_t)pwide;
	}
	if (a.qt && !a.pbuf && !qt_nolog) {   /* (decided above: cannot happen) */
		err = -EIO;
		goto out;
	}
	if (user && user != (void *)d->stream) {
		if ((err = hip_err(hipEventRecord(d->ev_user, (hipStream_t)user))) ||
		    (err = hip_err(hipStreamWaitEvent(d->stream, d->ev_user, 0))))
			goto out;
	}
	if (a.qt_hits && iters > 0)
		d->qt_pending = 1;
	/* classify, then its hit log's count kernel, on the device stream (a
	 * count kernel on a second stream, overlapped with the next classify,
	 * shares the CUs and slowed the classify more than it hid:
	 * profiles/archive/r04_s11_count_overlap.log) */
	uint64_t fold_at = 0xffffffffull;   /* (a 32-bit QT-order count's room) */
#ifdef XFG_DIAG
	const char *fa = getenv("XFG_QT_FOLD_AT");   /* tests: fold after this many packets */
	if (fa && strtoull(fa, NULL, 0))
		fold_at = strtoull(fa, NULL, 0);
#endif
	for (int i = 0; i < iters && !err; i++) {
		if (a.qt_hits) {
			if (d->qt_pk + a.n > fold_at && (err = qt_fold_queued(d)))
				break;
			d->qt_pk += a.n;
		}
		a.cw_n = 0;
		a.pfirst = 0;
		if (a.pbuf && cw) {
			/* the pending launch's set, counted by this launch's count
			 * wave (or, with none pending, none); this launch's log
			 * into the other set */
			if (d->log_pend) {
				a.cw_n = (uint32_t)grid;
				a.cw_s0 = d->log_first;
			}
			a.pslice0 = d->log_pend && !d->log_first ? (uint32_t)grid : 0u;
		} else if (a.pbuf && K > 1) {
			a.pslice0 = d->log_pend * (uint32_t)grid;
		}
		err = xfg_launch_classify(ctx->prog_features, &a, (unsigned)grid, d->stream);
		if (!err && a.pbuf && cw) {
			d->log_args = a;
			d->log_grid = (uint32_t)grid;
			d->log_pend = 1;
			d->log_first = a.pslice0;
			d->log_cw = 1;
		} else if (!err && a.pbuf && K > 1) {
			if (!d->log_pend)
				d->log_first = 0;
			d->log_args = a;
			d->log_grid = (uint32_t)grid;
			d->log_cw = 0;
			if (++d->log_pend == K)
				err = log_flush_locked(d);
		} else if (!err) {
			err = xfg_launch_log_count(&a, d->stream);
		}
	}
	if (!err)
		d->last_kind = kind;
	if (!err && user && user != (void *)d->stream) {
		if (!(err = hip_err(hipEventRecord(d->ev_done, d->stream))))
			err = hip_err(hipStreamWaitEvent((hipStream_t)user, d->ev_done, 0));
	}
out:
	pthread_mutex_unlock(&d->lock);
	return err;
}

static int check_batch(xfg_ctx *ctx, int dev, const struct xfg_batch *b, const void *verdicts)
{
	if (!ctx || !b || (!verdicts && b->count))
		return -EINVAL;
	if (!ctx->ndev)
		return -ENODEV;
	if (dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	if (b->count && (!b->data || !b->lens))
		return -EINVAL;
	if (!b->offsets && b->count && (b->stride == 0 || (b->stride & 15)))
		return -EINVAL;
	if (((uintptr_t)b->data & 15))
		return -EINVAL;
	return 0;
}

int xfg_classify(xfg_ctx *ctx, int dev, const struct xfg_batch *b, uint8_t *verdicts,
		 void *stream)
{
	int err = check_batch(ctx, dev, b, verdicts);
	if (err)
		return err;
	if (!b->count)
		return 0;
	struct xfg_dev *d = &ctx->dev[dev];
	struct xfg_kargs a;
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	err = fill_kargs(ctx, d, b, verdicts, &a);
	pthread_mutex_unlock(&ctx->lock);
	if (!err)
		err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = launch_batch(ctx, d, &a, stream, 1);
	return err;
}

int xfg_classify_descs(xfg_ctx *ctx, int dev, const struct xfg_desc_batch *db,
		       uint8_t *verdicts, void *stream)
{
	if (!ctx || !db || (!verdicts && db->count))
		return -EINVAL;
	if (!ctx->ndev)
		return -ENODEV;
	if (dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	if (!db->count)
		return 0;
	if (!db->umem || !db->descs || ((uintptr_t)db->descs & 7) || (db->mask & (db->mask + 1u)))
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[dev];
	struct xfg_batch b = { db->umem, NULL, NULL, db->count, 0, 0 };
	struct xfg_kargs a;
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	int err = fill_kargs(ctx, d, &b, verdicts, &a);
	pthread_mutex_unlock(&ctx->lock);
	if (err)
		return err;
	a.descs = db->descs;
	a.desc_mask = db->mask;
	a.desc_first = db->first;
	a.window = 128;
	a.pipe = 0;
	a.dense = 0;
	err = hip_err(hipSetDevice(d->ordinal));
	if (!err)
		err = launch_batch(ctx, d, &a, stream, 1);
	return err;
}

int xfg_classify_timed(xfg_ctx *ctx, int dev, const struct xfg_batch *b, uint8_t *verdicts,
		       int iters, double *avg_ms)
{
	int err = check_batch(ctx, dev, b, verdicts);
	if (err)
		return err;
	if (iters < 1 || !avg_ms)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[dev];
	struct xfg_kargs a;
	float ms = 0;
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	err = fill_kargs(ctx, d, b, verdicts, &a);
	pthread_mutex_unlock(&ctx->lock);
	if (err)
		return err;
	HIPCHK(hipSetDevice(d->ordinal));
	HIPCHK(hipEventRecord(d->ev0, d->stream));
	if ((err = launch_batch(ctx, d, &a, NULL, iters)))
		goto fail;
	/* (the logs still pending are counted inside the timed region: the
	 * iterations' work is complete when ev1 fires) */
	pthread_mutex_lock(&d->lock);
	err = log_flush_locked(d);
	pthread_mutex_unlock(&d->lock);
	if (err)
		goto fail;
	HIPCHK(hipEventRecord(d->ev1, d->stream));
	HIPCHK(hipEventSynchronize(d->ev1));
	HIPCHK(hipEventElapsedTime(&ms, d->ev0, d->ev1));
	*avg_ms = ms / iters;
	return 0;
fail:
	return err;
}

/* Verdict compaction (include/xdpfilter_gpu.h).  The kernel uses per-device
 * scratch (tile status words, ticket), so it runs on the device's own stream,
 * ordered after and before the caller's stream: two compactions never
 * overlap on one device, whatever streams their callers pass. */
int xfg_compact(xfg_ctx *ctx, int dev, const uint8_t *verdicts, uint64_t n, uint32_t action,
		uint32_t *idx, uint64_t *count, void *stream)
{
	int err = 0;
	if (!ctx || !count || (n && (!verdicts || !idx)) || action > 255 || n > 0xffffffffull)
		return -EINVAL;
	if (!ctx->ndev)
		return -ENODEV;
	if (dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[dev];
	uint64_t tiles = xfg_compact_tiles(n);
	pthread_mutex_lock(&d->lock);
	HIPCHK(hipSetDevice(d->ordinal));
	if (!d->cticket)
		HIPCHK(hipMalloc((void **)&d->cticket, 4));
	if (tiles > d->cstatus_cap) {
		HIPCHK(hipStreamSynchronize(d->stream));   /* the old buffer may be in use */
		hipFree(d->cstatus);
		d->cstatus = NULL;
		d->cstatus_cap = 0;
		HIPCHK(hipMalloc((void **)&d->cstatus, tiles * 8));
		d->cstatus_cap = tiles;
	}
	hipStream_t user = (hipStream_t)stream;
	if (user && user != d->stream) {
		HIPCHK(hipEventRecord(d->ev_user, user));
		HIPCHK(hipStreamWaitEvent(d->stream, d->ev_user, 0));
	}
	err = xfg_launch_compact(verdicts, n, action, idx, (unsigned long long *)count,
				 d->cstatus, d->cticket, (unsigned)d->ncu * 4, d->stream);
	if (!err && user && user != d->stream) {
		HIPCHK(hipEventRecord(d->ev_done, d->stream));
		HIPCHK(hipStreamWaitEvent(user, d->ev_done, 0));
	}
fail:
	pthread_mutex_unlock(&d->lock);
	return err;
}

/* Achievable streaming-read rate of the device (bench.py roofline leg). */
int xfg_stream_read_timed(xfg_ctx *ctx, int dev, const void *src, uint64_t bytes, int iters,
			  double *avg_ms)
{
	int err = 0;
	float ms = 0;
	if (!ctx || dev < 0 || dev >= ctx->ndev || !avg_ms || iters < 1)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[dev];
	unsigned grid = (unsigned)d->ncu * 8;
	HIPCHK(hipSetDevice(d->ordinal));
	HIPCHK(hipEventRecord(d->ev0, d->stream));
	for (int i = 0; i < iters; i++)
		if ((err = xfg_launch_stream_read(src, bytes, d->sink, grid, d->stream)))
			goto fail;
	HIPCHK(hipEventRecord(d->ev1, d->stream));
	HIPCHK(hipEventSynchronize(d->ev1));
	HIPCHK(hipEventElapsedTime(&ms, d->ev0, d->ev1));
	*avg_ms = ms / iters;
	return 0;
fail:
	return err;
}

/* Host-resident batches (xfg_classify_host, xfg_classify_xsk_host).
 *
 * Only header windows cross PCIe: each packet's first HOST_WIN bytes go to
 * a pinned staging slot (gathered by the device's thread pool) with its
 * true length, H2D, and the general kernel classifies them in header-window
 * mode (kargs.hwin).  A packet whose program would read past its window
 * (long IPv6 extension chains and the like) is not classified or counted
 * there: the kernel lists it, and the host sends its whole frame through
 * the ordinary device path afterwards -- the verdicts, counters and stats
 * are exactly those of a whole-frame run.  A fixed-stride batch whose
 * stride is at most HOST_WIN is staged slot for slot instead (one memcpy
 * per slice; nothing can fall back).  HOST_SLOTS staging slots of HOST_CH
 * packets rotate (gather / H2D / kernel / D2H, each slot on its own
 * stream); their size is fixed (HOST_CH x HOST_WIN bytes each), whatever
 * the frames' lengths.
 * One lock per device: the devices' host paths run concurrently. */
#define HOST_CH (1u << 18)     /* packets per staging slot */
#define HOST_WIN 128u          /* header window (bytes) */
#define FB_BYTES (64u << 20)   /* whole-frame fallback staging */
#define FB_PKTS (1u << 16)     /* ... and its packets per pass */

/* where packet i of a host batch lies */
struct hsrc {
	const uint8_t *data;       /* batch data, or the UMEM */
	const uint64_t *offsets;
	uint32_t stride;
	const void *lens;
	int lens_u16;
	const uint64_t *descs;     /* AF_XDP RX ring (xdp_desc records), or NULL */
	uint32_t first, mask;
	uint64_t span;             /* descs: the bytes from the UMEM's start the
				    * kernels' 16-byte loads may touch */
};

static inline const uint8_t *hsrc_ptr(const struct hsrc *s, uint64_t i)
{
	if (s->descs) {
		/* xsk_umem__add_offset_to_addr(): unaligned-chunk offset in
		 * bits 48..63 (headers/xdp/xsk.h:173-186) */
		const uint64_t a = s->descs[2ull * ((s->first + (uint32_t)i) & s->mask)];
		return s->data + (a & ((1ull << 48) - 1)) + (a >> 48);
	}
	return s->data + (s->offsets ? s->offsets[i] : i * (uint64_t)s->stride);
}

static inline uint32_t hsrc_len(const struct hsrc *s, uint64_t i)
{
	if (s->descs)   /* xdp_desc.len: the low half of the record's second word */
		return (uint32_t)s->descs[2ull * ((s->first + (uint32_t)i) & s->mask) + 1];
	const uint32_t l = s->lens_u16 ? ((const uint16_t *)s->lens)[i] : ((const uint32_t *)s->lens)[i];
	/* a fixed-stride frame lies in its slot: a longer length is capped at the
	 * slot, as the device path caps it (the gather, the kernel and the
	 * whole-frame fallback then all see the same length, and no copy reads
	 * past the slot) */
	return (!s->offsets && s->stride && l > s->stride) ? s->stride : l;
}

struct gather_job {
	const struct hsrc *src;
	uint64_t first, m;         /* packets [first, first + m) */
	uint8_t *dst;
	uint32_t *dl;
	uint32_t stride;           /* staging stride: HOST_WIN, or the batch's */
	int whole;                 /* 1 whole slots copied (stride <= HOST_WIN, no
				    * offsets), 2 whole slots left where they lie
				    * (registered memory: lengths only), 3 frames
				    * left where they lie in a registered UMEM
				    * (offsets into dst, lengths), 4 the caller's
				    * lengths as they are (dl: u16 or u32; the
				    * kernels cap them at the stride), 0 windows */
};

static void gather_slice(void *arg, int t, int nt)
{
	const struct gather_job *j = arg;
	const uint64_t per = (j->m + nt - 1) / nt;
	const uint64_t s0 = t * per, s1 = s0 + per < j->m ? s0 + per : j->m;
	if (s0 >= s1)
		return;
	if (j->whole == 4) {
		const size_t ls = j->src->lens_u16 ? 2 : 4;
		memcpy((uint8_t *)j->dl + s0 * ls, (const uint8_t *)j->src->lens + (j->first + s0) * ls,
		       (s1 - s0) * ls);
		return;
	}
	if (j->whole == 1)
		memcpy(j->dst + s0 * j->stride, j->src->data + (j->first + s0) * j->stride,
		       (s1 - s0) * j->stride);
	for (uint64_t i = s0; i < s1; i++) {
		const uint32_t l = hsrc_len(j->src, j->first + i);
		if (j->whole == 3)
			((uint64_t *)j->dst)[i] = (uint64_t)(hsrc_ptr(j->src, j->first + i) - j->src->data);
		else if (!j->whole)
			memcpy(j->dst + i * HOST_WIN, hsrc_ptr(j->src, j->first + i),
			       l < HOST_WIN ? l : HOST_WIN);
		j->dl[i] = l;
	}
}

static int host_staging(struct xfg_dev *d)
{
	int err = 0;
	if (!d->pool && !(d->pool = hpool_start()))
		return -ENOMEM;
	if (d->hs_st[0])
		return 0;
	for (int k = 0; k < HOST_SLOTS; k++) {
		HIPCHK(hipStreamCreateWithFlags(&d->hs_st[k], hipStreamNonBlocking));
		HIPCHK(hipEventCreate(&d->hs_done[k]));
		HIPCHK(hipHostMalloc((void **)&d->hs_hbuf[k], (size_t)HOST_CH * HOST_WIN,
				     hipHostMallocDefault));
		HIPCHK(hipHostMalloc((void **)&d->hs_hl[k], HOST_CH * 4, hipHostMallocDefault));
		HIPCHK(hipHostMalloc((void **)&d->hs_hfbc[k], 4, hipHostMallocDefault));
		HIPCHK(hipMalloc((void **)&d->hs_dbuf[k], (size_t)HOST_CH * HOST_WIN));
		HIPCHK(hipMalloc((void **)&d->hs_dl[k], HOST_CH * 4));
		HIPCHK(hipMalloc((void **)&d->hs_dv[k], HOST_CH));
		HIPCHK(hipMalloc((void **)&d->hs_fb[k], HOST_CH * 4));
		HIPCHK(hipMalloc((void **)&d->hs_fbc[k], 4));
	}
	return 0;
fail:
	for (int k = 0; k < HOST_SLOTS; k++) {   /* all or nothing: a later call starts over */
		if (d->hs_st[k])
			hipStreamDestroy(d->hs_st[k]);
		if (d->hs_done[k])
			hipEventDestroy(d->hs_done[k]);
		hipHostFree(d->hs_hbuf[k]);
		hipHostFree(d->hs_hl[k]);
		hipHostFree(d->hs_hfbc[k]);
		hipFree(d->hs_dbuf[k]);
		hipFree(d->hs_dl[k]);
		hipFree(d->hs_dv[k]);
		hipFree(d->hs_fb[k]);
		hipFree(d->hs_fbc[k]);
		d->hs_st[k] = NULL;
		d->hs_done[k] = NULL;
		d->hs_hbuf[k] = d->hs_dbuf[k] = d->hs_dv[k] = NULL;
		d->hs_hl[k] = d->hs_dl[k] = d->hs_fb[k] = d->hs_fbc[k] = d->hs_hfbc[k] = NULL;
	}
	return err;
}

static int fb_staging(struct xfg_dev *d)
{
	int err = 0;
	if (d->fb_h)
		return 0;
	HIPCHK(hipHostMalloc((void **)&d->fb_ho, FB_PKTS * 8, hipHostMallocDefault));
	HIPCHK(hipHostMalloc((void **)&d->fb_hl, FB_PKTS * 4, hipHostMallocDefault));
	HIPCHK(hipHostMalloc((void **)&d->fb_idx, (size_t)HOST_CH * 4, hipHostMallocDefault));
	HIPCHK(hipMalloc((void **)&d->fb_d, FB_BYTES + 64));
	HIPCHK(hipMalloc((void **)&d->fb_do, FB_PKTS * 8));
	HIPCHK(hipMalloc((void **)&d->fb_dl, FB_PKTS * 4));
	HIPCHK(hipMalloc((void **)&d->fb_dv, FB_PKTS));
	HIPCHK(hipHostMalloc((void **)&d->fb_h, FB_BYTES + 64, hipHostMallocDefault));
	return 0;
fail:
	hipHostFree(d->fb_ho);
	hipHostFree(d->fb_hl);
	hipHostFree(d->fb_idx);
	hipFree(d->fb_d);
	hipFree(d->fb_do);
	hipFree(d->fb_dl);
	hipFree(d->fb_dv);
	d->fb_ho = NULL;
	d->fb_hl = d->fb_idx = d->fb_dl = NULL;
	d->fb_d = d->fb_dv = NULL;
	d->fb_do = NULL;
	return err;
}

/* Classify a device-resident sub-batch on stream st (kernels on the device
 * stream, ordered after st's uploads; st after the kernels). */
static int host_launch(xfg_ctx *ctx, struct xfg_dev *d, const struct xfg_batch *sub,
		       uint8_t *dv, int hwin, uint32_t *fb, uint32_t *fbc, hipStream_t st)
{
	struct xfg_kargs a;
	pthread_mutex_lock(&ctx->lock);
	ctx->reduced = 0;
	int err = fill_kargs(ctx, d, sub, dv, &a);
	pthread_mutex_unlock(&ctx->lock);
	if (err)
		return err;
	if (hwin) {   /* header windows: the general kernel, listing what leaves them */
		a.pipe = 0;
		a.hwin = 1;
		a.fb = fb;
		a.fb_cnt = fbc;
		a.fb_cap = HOST_CH;
	}
	return launch_batch(ctx, d, &a, st, 1);
}

/* The packets of the chunk at `c` whose programs left their windows (count
 * in *d->hs_hfbc[k], list in d->hs_fb[k]): their whole frames through the
 * ordinary path, FB_BYTES / FB_PKTS at a time; verdicts scattered back. */
static int host_fallback(xfg_ctx *ctx, struct xfg_dev *d, const struct hsrc *src, uint64_t c,
			 int k, uint8_t *verdicts)
{
	int err = 0;
	const uint32_t nf = *d->hs_hfbc[k];
	if (!nf)
		return 0;
	if (nf > HOST_CH)
		return -EIO;
	if ((err = fb_staging(d)))
		return err;
	HIPCHK(hipMemcpyAsync(d->fb_idx, d->hs_fb[k], (size_t)nf * 4, hipMemcpyDeviceToHost,
			      d->hs_st[k]));
	HIPCHK(hipStreamSynchronize(d->hs_st[k]));
	for (uint32_t j0 = 0; j0 < nf;) {
		uint64_t pos = 0;
		uint32_t m = 0;
		while (j0 + m < nf && m < FB_PKTS) {
			const uint64_t gi = c + d->fb_idx[j0 + m];
			const uint32_t l = hsrc_len(src, gi);
			if (l > FB_BYTES)
				return -E2BIG;
			if (pos + l > FB_BYTES)
				break;
			memcpy(d->fb_h + pos, hsrc_ptr(src, gi), l);
			d->fb_ho[m] = pos;
			d->fb_hl[m] = l;
			pos = (pos + l + 15) & ~15ull;   /* 16-byte aligned starts */
			m++;
		}
		HIPCHK(hipMemcpyAsync(d->fb_d, d->fb_h, pos, hipMemcpyHostToDevice, d->hs_st[k]));
		HIPCHK(hipMemcpyAsync(d->fb_do, d->fb_ho, (size_t)m * 8, hipMemcpyHostToDevice,
				      d->hs_st[k]));
		HIPCHK(hipMemcpyAsync(d->fb_dl, d->fb_hl, (size_t)m * 4, hipMemcpyHostToDevice,
				      d->hs_st[k]));
		struct xfg_batch sub = { d->fb_d, d->fb_do, d->fb_dl, m, 0, 0 };
		if ((err = host_launch(ctx, d, &sub, d->fb_dv, 0, NULL, NULL, d->hs_st[k])))
			return err;
		/* (the pinned frame buffer doubles as the verdicts' landing place) */
		HIPCHK(hipMemcpyAsync(d->fb_h, d->fb_dv, m, hipMemcpyDeviceToHost, d->hs_st[k]));
		HIPCHK(hipStreamSynchronize(d->hs_st[k]));
		for (uint32_t q = 0; q < m; q++)
			verdicts[c + d->fb_idx[j0 + q]] = d->fb_h[q];
		j0 += m;
	}
	*d->hs_hfbc[k] = 0;
	return 0;
fail:
	return err;
}

/* ---- registered host buffers: DMA straight from the caller's memory */
int xfg_host_register(xfg_ctx *ctx, void *p, size_t bytes)
{
	int err = 0;
	if (!ctx || !p || !bytes)
		return -EINVAL;
	pthread_mutex_lock(&ctx->reg_lock);
	for (int i = 0; i < ctx->nreg; i++) {
		const uint8_t *a = ctx->reg[i].p, *b = (const uint8_t *)p;
		if (b < a + ctx->reg[i].bytes && a < b + bytes) {
			err = -EEXIST;   /* overlaps a registered buffer */
			goto out;
		}
	}
	if (ctx->nreg == XFG_HOST_REG_MAX) {
		err = -ENOSPC;
		goto out;
	}
	/* mapped as well: whole slots are read by the kernels where they lie
	 * (host_run's zero-copy path) */
	if ((err = hip_err(hipHostRegister(p, bytes, hipHostRegisterPortable | hipHostRegisterMapped))))
		goto out;
	ctx->reg[ctx->nreg].p = p;
	ctx->reg[ctx->nreg].bytes = bytes;
	ctx->nreg++;
out:
	pthread_mutex_unlock(&ctx->reg_lock);
	return err;
}

int xfg_host_unregister(xfg_ctx *ctx, void *p)
{
	int err = -ENOENT;
	if (!ctx || !p)
		return -EINVAL;
	/* (no host-path call may be using it: the caller's contract, as for
	 * freeing any buffer it passed) */
	pthread_mutex_lock(&ctx->reg_lock);
	for (int i = 0; i < ctx->nreg; i++) {
		if (ctx->reg[i].p != p)
			continue;
		err = hip_err(hipHostUnregister(p));
		ctx->reg[i] = ctx->reg[--ctx->nreg];
		break;
	}
	pthread_mutex_unlock(&ctx->reg_lock);
	return err;
}

/* Whether [p, p + bytes) lies inside one registered buffer (*base: that
 * buffer's start). */
static int host_registered(xfg_ctx *ctx, const void *p, uint64_t bytes, const uint8_t **base)
{
	int r = 0;
	pthread_mutex_lock(&ctx->reg_lock);
	for (int i = 0; i < ctx->nreg && !r; i++)
		if ((r = (const uint8_t *)p >= ctx->reg[i].p &&
			 (const uint8_t *)p + bytes <= ctx->reg[i].p + ctx->reg[i].bytes) && base)
			*base = ctx->reg[i].p;
	pthread_mutex_unlock(&ctx->reg_lock);
	return r;
}

/* Zero copy: the batch's frames read by the kernels through the registered
 * buffer's device mapping; per chunk the pool copies the lengths (for
 * AF_XDP: gathers the frames' UMEM offsets and lengths) into the slot's
 * pinned buffer, one H2D copy takes them to the slot's device buffer, the
 * kernels run, the verdicts come back.  Chunks of 2^22 packets (AF_XDP:
 * 2^21), far larger than the staged path's: the kernels' reads cross PCIe
 * at its latency, and a short launch ramps up and drains for a larger share
 * of its time (C3, u32 lengths: 2^18-packet chunks 430 Mpps, 2^21 630, one
 * launch from device-resident lengths 790). */
#define ZC_CH (1u << 21)   /* AF_XDP (13 bytes a packet); fixed stride: twice (5 bytes) */
#ifndef HYB_ZC_CH   /* host_run_hyb: packets of a round's zero-copy chunk, ... */
#define HYB_ZC_CH (1ull << 20)
#endif
#ifndef HYB_ST_N    /* ... and its staged chunks of HOST_CH (0: no hybrid) */
/* (off: on C5 from a registered buffer, 2^23 frames of 1514 B, zero copy
 * alone ran 270 Mpps and every hybrid setting tried 175-220 -- the staged
 * gather's reads of the same host memory slow the kernels' PCIe reads more
 * than its chunks add, profiles/r06_s6_hyb_c5.log; the diagnostics build
 * still takes XFG_HYB_ZLOG2 / XFG_HYB_ST) */
#define HYB_ST_N 0u
#endif
_Static_assert((size_t)ZC_CH * 13 + 256 <= (size_t)HOST_CH * HOST_WIN, "slot buffers hold a chunk");
_Static_assert((size_t)ZC_CH * 2 * 5 + 256 <= (size_t)HOST_CH * HOST_WIN, "slot buffers hold a chunk");

static int host_run_zc(xfg_ctx *ctx, struct xfg_dev *d, const struct hsrc *src, uint64_t n,
		       const uint8_t *rbase, uint8_t *verdicts)
{
	int err = 0;
	void *dp = NULL;
	HIPCHK(hipHostGetDevicePointer(&dp, (void *)rbase, 0));
	const uint8_t *zdev = (const uint8_t *)dp + (src->data - rbase);   /* the batch, device side */
	/* (chunks growing from 2^17, so that the first kernel starts after a
	 * short copy, measured slower: 607 Mpps against 670 for C3) */
	uint64_t ch = src->descs ? ZC_CH : 2 * ZC_CH;
#ifdef XFG_DIAG
	const char *zl = getenv("XFG_ZC_LOG2");   /* chunk size (log2, at most the default) */
	if (zl && atoi(zl) >= 12 && (1ull << atoi(zl)) <= ch)
		ch = 1ull << atoi(zl);
#endif
	/* fixed-stride lengths go as the caller holds them (u16 or u32) */
	const size_t ls = src->descs ? 4 : src->lens_u16 ? 2 : 4;
	for (uint64_t c = 0, k = 0; c < n; c += ch, k = (k + 1) % HOST_SLOTS) {
		const uint64_t m = n - c < ch ? n - c : ch;
		/* slot layout (pinned and device alike): [offsets u64 x m] lens x m;
		 * verdicts after them, device side */
		const size_t ob = src->descs ? m * 8 : 0, lb = ob + m * ls, vb = (lb + 255) & ~(size_t)255;
		HIPCHK(hipEventSynchronize(d->hs_done[k]));   /* slot k free again */
		struct gather_job job = { src, c, m, d->hs_hbuf[k], (uint32_t *)(d->hs_hbuf[k] + ob),
					  HOST_WIN, src->descs ? 3 : 4 };
		hpool_run(d->pool, gather_slice, &job);
		HIPCHK(hipMemcpyAsync(d->hs_dbuf[k], d->hs_hbuf[k], lb, hipMemcpyHostToDevice, d->hs_st[k]));
		struct xfg_batch sub = { zdev + (src->descs ? 0 : c * src->stride),
					 src->descs ? (const uint64_t *)d->hs_dbuf[k] : NULL,
					 d->hs_dbuf[k] + ob, m, src->descs ? 0 : src->stride, ls == 2 };
		if ((err = host_launch(ctx, d, &sub, d->hs_dbuf[k] + vb, 0, NULL, NULL, d->hs_st[k])))
			goto fail;
		HIPCHK(hipMemcpyAsync(verdicts + c, d->hs_dbuf[k] + vb, m, hipMemcpyDeviceToHost,
				      d->hs_st[k]));
		HIPCHK(hipEventRecord(d->hs_done[k], d->hs_st[k]));
	}
	for (int k = 0; k < HOST_SLOTS; k++)
		HIPCHK(hipStreamSynchronize(d->hs_st[k]));
fail:
	return err;
}

/* Registered large slots (C5's 1514-byte frames at a 1536-byte stride): the
 * zero-copy kernels are bound by the rate of PCIe read requests (one 64-byte
 * window a frame, ~0.3 Gpps) and the staged path by the pool's gather (~0.13
 * Gpps), different resources -- so each round takes one zero-copy chunk of
 * zc_ch packets (its kernel reading mapped host memory while the pool works)
 * and then st_n staged chunks of header windows (gathered meanwhile, their
 * kernels queued behind it): slots 0-1 for the zero-copy chunks, 2-3 for the
 * staged ones.  Verdicts, counters and stats are those of either path: the
 * same kernels over the same frames, the staged windows' leavers walked
 * whole (host_fallback). */
static int host_run_hyb(xfg_ctx *ctx, struct xfg_dev *d, const struct hsrc *src, uint64_t n,
			const uint8_t *rbase, uint8_t *verdicts, uint64_t zc_ch, uint32_t st_n)
{
	int err = 0;
	void *dp = NULL;
	HIPCHK(hipHostGetDevicePointer(&dp, (void *)rbase, 0));
	const uint8_t *zdev = (const uint8_t *)dp + (src->data - rbase);
	const size_t ls = src->lens_u16 ? 2 : 4;
	uint64_t pend[HOST_SLOTS];
	for (int k = 0; k < HOST_SLOTS; k++)
		pend[k] = UINT64_MAX;
	uint32_t zk = 0, sk = 0;
	for (uint64_t c = 0; c < n;) {
		/* the zero-copy chunk: the pool copies its lengths, the kernel
		 * reads the frames where they lie */
		{
			const int k = (int)(zk++ & 1);
			const uint64_t m = n - c < zc_ch ? n - c : zc_ch;
			const size_t lb = m * ls, vb = (lb + 255) & ~(size_t)255;
			HIPCHK(hipEventSynchronize(d->hs_done[k]));
			struct gather_job job = { src, c, m, d->hs_hbuf[k], (uint32_t *)d->hs_hbuf[k], HOST_WIN, 4 };
			hpool_run(d->pool, gather_slice, &job);
			HIPCHK(hipMemcpyAsync(d->hs_dbuf[k], d->hs_hbuf[k], lb, hipMemcpyHostToDevice, d->hs_st[k]));
			struct xfg_batch sub = { zdev + c * src->stride, NULL, d->hs_dbuf[k], m, src->stride, ls == 2 };
			if ((err = host_launch(ctx, d, &sub, d->hs_dbuf[k] + vb, 0, NULL, NULL, d->hs_st[k])))
				goto fail;
			HIPCHK(hipMemcpyAsync(verdicts + c, d->hs_dbuf[k] + vb, m, hipMemcpyDeviceToHost,
					      d->hs_st[k]));
			HIPCHK(hipEventRecord(d->hs_done[k], d->hs_st[k]));
			c += m;
		}
		/* the staged chunks: 128-byte header windows gathered by the pool
		 * while the zero-copy kernel runs */
		for (uint32_t j = 0; j < st_n && c < n; j++) {
			const int k = 2 + (int)(sk++ & 1);
			const uint64_t m = n - c < HOST_CH ? n - c : HOST_CH;
			HIPCHK(hipEventSynchronize(d->hs_done[k]));
			if (pend[k] != UINT64_MAX && (err = host_fallback(ctx, d, src, pend[k], k, verdicts)))
				goto fail;
			struct gather_job job = { src, c, m, d->hs_hbuf[k], d->hs_hl[k], HOST_WIN, 0 };
			hpool_run(d->pool, gather_slice, &job);
			HIPCHK(hipMemcpyAsync(d->hs_dbuf[k], d->hs_hbuf[k], m * HOST_WIN, hipMemcpyHostToDevice,
					      d->hs_st[k]));
			HIPCHK(hipMemcpyAsync(d->hs_dl[k], d->hs_hl[k], m * 4, hipMemcpyHostToDevice, d->hs_st[k]));
			HIPCHK(hipMemsetAsync(d->hs_fbc[k], 0, 4, d->hs_st[k]));
			struct xfg_batch sub = { d->hs_dbuf[k], NULL, d->hs_dl[k], m, HOST_WIN, 0 };
			if ((err = host_launch(ctx, d, &sub, d->hs_dv[k], 1, d->hs_fb[k], d->hs_fbc[k],
					       d->hs_st[k])))
				goto fail;
			HIPCHK(hipMemcpyAsync(verdicts + c, d->hs_dv[k], m, hipMemcpyDeviceToHost, d->hs_st[k]));
			HIPCHK(hipMemcpyAsync(d->hs_hfbc[k], d->hs_fbc[k], 4, hipMemcpyDeviceToHost, d->hs_st[k]));
			HIPCHK(hipEventRecord(d->hs_done[k], d->hs_st[k]));
			pend[k] = c;
			c += m;
		}
	}
	for (int k = 0; k < HOST_SLOTS; k++) {
		HIPCHK(hipStreamSynchronize(d->hs_st[k]));
		if (pend[k] != UINT64_MAX && (err = host_fallback(ctx, d, src, pend[k], k, verdicts)))
			goto fail;
	}
fail:
	return err;
}

static int host_run(xfg_ctx *ctx, int dev, const struct hsrc *src, uint64_t n, uint8_t *verdicts)
{
	int err = 0;
	struct xfg_dev *d = &ctx->dev[dev];
	/* whole slots: a fixed stride within the window (16-byte aligned, or
	 * the kernel's 16-byte loads would straddle slots) */
	const int whole = !src->descs && !src->offsets && src->stride && src->stride <= HOST_WIN &&
			  !(src->stride & 15);
	const uint32_t stride = whole ? src->stride : HOST_WIN;
	/* fixed-stride slots (16-byte aligned) in a registered buffer: read by
	 * the kernels where they lie, through the buffer's device mapping (zero
	 * copy: the kernel's loads cross PCIe, the window and whatever a
	 * program walks past it, nothing else; whole frames in view, so no
	 * fallback) -- the pool gathers the lengths only.  Measured on MI355X
	 * against one DMA of the whole slots per chunk (C3, 64-byte frames,
	 * bench.py's host_path): 41-46 GB/s of frames against 34-36 on this
	 * round's boxes (profiles/archive/r05_s16..s19, s36, s47).  The
	 * slots must start 16-byte aligned, as the device path's batches do
	 * (check_batch): an unaligned registered batch takes the staged path. */
	const uint8_t *rbase = NULL;
	int zc = (!src->descs && !src->offsets && src->stride && !(src->stride & 15) &&
		  !((uintptr_t)src->data & 15) &&
		  host_registered(ctx, src->data, n * (uint64_t)src->stride, &rbase)) ||
		 /* AF_XDP frames in a registered UMEM: the descriptors' offsets
		  * and lengths gathered, the frames read in place */
		 (src->descs && host_registered(ctx, src->data, src->span, &rbase));
#ifdef XFG_DIAG
	const char *zs = getenv("XFG_HOST_ZC");   /* "off": round 4's DMA paths */
	if (zs && !strcmp(zs, "off"))
		zc = 0;
#endif
	/* whole slots in a registered buffer: copied by DMA where they lie */
	const int direct = !zc && whole && host_registered(ctx, src->data, n * (uint64_t)stride, NULL);
	/* windows of larger slots in a registered buffer: one strided DMA per
	 * chunk (rows of HOST_WIN bytes at the batch's stride; a window never
	 * leaves its slot) instead of the pool's gather -- the pool then
	 * gathers the lengths only */
	const int direct2d = !zc && !whole && !src->descs && !src->offsets && src->stride > HOST_WIN &&
			     !(src->stride & 15) &&
			     host_registered(ctx, src->data, n * (uint64_t)src->stride, NULL);
	uint64_t pend[HOST_SLOTS];   /* each slot's last chunk */
	for (int k = 0; k < HOST_SLOTS; k++)
		pend[k] = UINT64_MAX;

	pthread_mutex_lock(&d->host_lock);
	HIPCHK(hipSetDevice(d->ordinal));
	if ((err = host_staging(d)))
		goto fail;
	/* (registered large slots, a batch of several rounds: zero copy and the
	 * staged gather side by side, host_run_hyb -- off by default, HYB_ST_N) */
	uint64_t hyb_zc = HYB_ZC_CH;
	uint32_t hyb_st = HYB_ST_N;
#ifdef XFG_DIAG
	const char *hz = getenv("XFG_HYB_ZLOG2");   /* zero-copy chunk (log2); 0: no hybrid */
	if (hz && *hz)
		hyb_zc = atoi(hz) ? 1ull << atoi(hz) : 0;
	const char *hn = getenv("XFG_HYB_ST");      /* staged chunks a round */
	if (hn && *hn)
		hyb_st = (uint32_t)atoi(hn);
#endif
	if (zc && hyb_zc && hyb_st && !src->descs && src->stride > HOST_WIN && n >= 2 * hyb_zc &&
	    hyb_zc <= 2 * ZC_CH) {
		err = host_run_hyb(ctx, d, src, n, rbase, verdicts, hyb_zc, hyb_st);
		goto fail;
	}
	if (zc) {
		err = host_run_zc(ctx, d, src, n, rbase, verdicts);
		goto fail;
	}
	for (uint64_t c = 0, k = 0; c < n; c += HOST_CH, k = (k + 1) % HOST_SLOTS) {
		const uint64_t m = n - c < HOST_CH ? n - c : HOST_CH;
		HIPCHK(hipEventSynchronize(d->hs_done[k]));   /* slot k free again */
		if (pend[k] != UINT64_MAX && (err = host_fallback(ctx, d, src, pend[k], k, verdicts)))
			goto fail;
		struct gather_job job = { src, c, m, d->hs_hbuf[k], d->hs_hl[k], stride, whole && !direct };
		if (direct || direct2d)   /* (the slots go by DMA: only the lengths are gathered) */
			job.whole = 2;
		hpool_run(d->pool, gather_slice, &job);
		if (direct2d)
			HIPCHK(hipMemcpy2DAsync(d->hs_dbuf[k], HOST_WIN, src->data + c * src->stride,
						src->stride, HOST_WIN, m, hipMemcpyHostToDevice, d->hs_st[k]));
		else
			HIPCHK(hipMemcpyAsync(d->hs_dbuf[k], direct ? src->data + c * stride : d->hs_hbuf[k],
					      m * stride, hipMemcpyHostToDevice, d->hs_st[k]));
		HIPCHK(hipMemcpyAsync(d->hs_dl[k], d->hs_hl[k], m * 4, hipMemcpyHostToDevice, d->hs_st[k]));
		HIPCHK(hipMemsetAsync(d->hs_fbc[k], 0, 4, d->hs_st[k]));
		struct xfg_batch sub = { d->hs_dbuf[k], NULL, d->hs_dl[k], m, stride, 0 };
		if ((err = host_launch(ctx, d, &sub, d->hs_dv[k], !whole, d->hs_fb[k], d->hs_fbc[k],
				       d->hs_st[k])))
			goto fail;
		HIPCHK(hipMemcpyAsync(verdicts + c, d->hs_dv[k], m, hipMemcpyDeviceToHost, d->hs_st[k]));
		HIPCHK(hipMemcpyAsync(d->hs_hfbc[k], d->hs_fbc[k], 4, hipMemcpyDeviceToHost, d->hs_st[k]));
		HIPCHK(hipEventRecord(d->hs_done[k], d->hs_st[k]));
		pend[k] = whole ? UINT64_MAX : c;
	}
	for (int k = 0; k < HOST_SLOTS; k++) {
		HIPCHK(hipStreamSynchronize(d->hs_st[k]));
		if (pend[k] != UINT64_MAX && (err = host_fallback(ctx, d, src, pend[k], k, verdicts)))
			goto fail;
	}
fail:
	for (int k = 0; k < HOST_SLOTS; k++)   /* (after an error: nothing may still use them) */
		if (d->hs_st[k])
			hipStreamSynchronize(d->hs_st[k]);
	pthread_mutex_unlock(&d->host_lock);
	return err;
}

int xfg_classify_host(xfg_ctx *ctx, int dev, const struct xfg_batch *b, uint8_t *verdicts)
{
	if (!ctx || !b || (!verdicts && b->count) || (b->count && (!b->data || !b->lens)))
		return -EINVAL;
	if (!ctx->ndev)
		return -ENODEV;
	if (dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	if (!b->offsets && !b->stride && b->count)
		return -EINVAL;
	if (!b->count)
		return 0;
	const struct hsrc src = { b->data, b->offsets, b->stride, b->lens, b->lens_u16, NULL, 0, 0, 0 };
	return host_run(ctx, dev, &src, b->count, verdicts);
}

int xfg_classify_xsk_host(xfg_ctx *ctx, int dev, const struct xfg_desc_batch *b,
			  uint64_t umem_bytes, uint8_t *verdicts)
{
	if (!ctx || !b || (!verdicts && b->count) || (b->count && (!b->umem || !b->descs)))
		return -EINVAL;
	if (!ctx->ndev)
		return -ENODEV;
	if (dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	if (b->mask != 0xffffffffu && (b->mask & (b->mask + 1)))
		return -EINVAL;   /* a ring mask is 2^k - 1 */
	if (b->count > (uint64_t)b->mask + 1)
		return -EINVAL;
	if (!b->count)
		return 0;
	struct hsrc src = { b->umem, NULL, 0, NULL, 0, b->descs, b->first, b->mask, 0 };
	/* every frame inside the UMEM (the kernel ring would have refused it);
	 * span: the end of the last 16-byte load a kernel makes of a frame */
	for (uint64_t i = 0; i < b->count; i++) {
		const uint64_t a = ((const uint64_t *)b->descs)[2ull * ((b->first + (uint32_t)i) & b->mask)];
		const uint64_t off = (a & ((1ull << 48) - 1)) + (a >> 48);
		const uint32_t l = hsrc_len(&src, i);
		if (off + l > umem_bytes)
			return -EINVAL;
		if (off + ((l + 15ull) & ~15ull) > src.span)
			src.span = off + ((l + 15ull) & ~15ull);
	}
	return host_run(ctx, dev, &src, b->count, verdicts);
}

/* ------------------------------------------------------------------ stats */
int xfg_stats_read_dev(xfg_ctx *ctx, int dev, struct xfg_stats_record out[XFG_ACTION_MAX])
{
	if (!ctx || !out || dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[dev];
	unsigned long long s[10];
	int err = dev_read(d, s, ctx->reduced ? d->red_stats : d->stats, sizeof(s));
	if (err)
		return err;
	for (int a = 0; a < XFG_ACTION_MAX; a++) {
		out[a].packets = s[2 * a];
		out[a].bytes = s[2 * a + 1];
	}
	return 0;
}

int xfg_stats_read(xfg_ctx *ctx, struct xfg_stats_record out[XFG_ACTION_MAX])
{
	if (!ctx || !out)
		return -EINVAL;
	memset(out, 0, sizeof(*out) * XFG_ACTION_MAX);
	if (ctx->reduced)   /* every rank holds the job-wide sum already */
		return ctx->ndev ? xfg_stats_read_dev(ctx, 0, out) : 0;
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_stats_record r[XFG_ACTION_MAX];
		int err = xfg_stats_read_dev(ctx, i, r);
		if (err)
			return err;
		for (int a = 0; a < XFG_ACTION_MAX; a++) {
			out[a].packets += r[a].packets;
			out[a].bytes += r[a].bytes;
		}
	}
	return 0;
}

int xfg_stats_reset(xfg_ctx *ctx)
{
	if (!ctx)
		return -EINVAL;
	for (int i = 0; i < ctx->ndev; i++) {
		struct xfg_dev *d = &ctx->dev[i];
		unsigned long long z[10] = { 0 };
		int err = dev_write(d, d->stats, z, sizeof(z));
		if (err)
			return err;
	}
	ctx->reduced = 0;
	return 0;
}

int xfg_sync(xfg_ctx *ctx)
{
	if (!ctx)
		return -EINVAL;
	for (int i = 0; i < ctx->ndev; i++) {
		int err = hip_err(hipSetDevice(ctx->dev[i].ordinal));
		if (!err)
			err = hip_err(hipDeviceSynchronize());
		if (err)
			return err;
	}
	return 0;
}

/* ------------------------------------------------------------------ memory */
void *xfg_dev_alloc(xfg_ctx *ctx, int dev, size_t bytes)
{
	void *p = NULL;
	if (!ctx || dev < 0 || dev >= ctx->ndev)
		return NULL;
	if (hipSetDevice(ctx->dev[dev].ordinal) != hipSuccess)
		return NULL;
	if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess)
		return NULL;
	return p;
}

void xfg_dev_free(xfg_ctx *ctx, int dev, void *p)
{
	if (!ctx || dev < 0 || dev >= ctx->ndev || !p)
		return;
	hipSetDevice(ctx->dev[dev].ordinal);
	hipFree(p);
}

int xfg_memcpy_h2d(xfg_ctx *ctx, int dev, void *dst, const void *src, size_t bytes)
{
	if (!ctx || dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	int err = hip_err(hipSetDevice(ctx->dev[dev].ordinal));
	return err ? err : hip_err(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
}

int xfg_memcpy_d2h(xfg_ctx *ctx, int dev, void *dst, const void *src, size_t bytes)
{
	if (!ctx || dev < 0 || dev >= ctx->ndev)
		return -EINVAL;
	int err = hip_err(hipSetDevice(ctx->dev[dev].ordinal));
	if (!err)
		err = hip_err(hipDeviceSynchronize());
	return err ? err : hip_err(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
}

void *xfg_host_alloc_pinned(size_t bytes)
{
	void *p = NULL;
	if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess)
		return NULL;
	return p;
}

void xfg_host_free_pinned(void *p)
{
	if (p)
		hipHostFree(p);
}

/* ------------------------------------------------------------------ RCCL */
int xfg_comm_unique_id(uint8_t id[XFG_COMM_ID_BYTES])
{
	ncclUniqueId u;
	if (sizeof(u) != XFG_COMM_ID_BYTES)
		return -EINVAL;
	if (ncclGetUniqueId(&u) != ncclSuccess)
		return -EIO;
	memcpy(id, &u, sizeof(u));
	return 0;
}

/* The reduction copies (red_*) and the communicator.  A second init
 * replaces both; a failed init leaves the context without either. */
static void comm_release(xfg_ctx *ctx)
{
	struct xfg_dev *d = &ctx->dev[0];
	if (ctx->comm_ready) {
		ncclCommDestroy(ctx->comm);
		ctx->comm_ready = 0;
	}
	ctx->reduced = 0;
	hipSetDevice(d->ordinal);
	for (int i = 0; i < NMAPS_HASH; i++) {
		hipFree(d->m[i].red_hits);
		d->m[i].red_hits = NULL;
	}
	hipFree(d->red_port_hits);
	d->red_port_hits = NULL;
	hipFree(d->red_stats);
	d->red_stats = NULL;
}

int xfg_comm_init(xfg_ctx *ctx, int nranks, int rank, const uint8_t id[XFG_COMM_ID_BYTES])
{
	int err = 0;
	ncclUniqueId u;
	if (!ctx || !id || ctx->ndev != 1 || nranks < 1 || rank < 0 || rank >= nranks)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[0];
	memcpy(&u, id, sizeof(u));
	comm_release(ctx);
	HIPCHK(hipSetDevice(d->ordinal));
	for (int i = 0; i < NMAPS_HASH; i++)
		HIPCHK(hipMalloc((void **)&d->m[i].red_hits, ((size_t)ctx->t[i].nslots + 1) * 8));
	HIPCHK(hipMalloc((void **)&d->red_port_hits, XFG_PORT_MAP_ENTRIES * 8));
	HIPCHK(hipMalloc((void **)&d->red_stats, 10 * 8));
	if (ncclCommInitRank(&ctx->comm, nranks, u, rank) != ncclSuccess) {
		err = -EIO;
		goto fail;
	}
	ctx->comm_ready = 1;
	return 0;
fail:
	comm_release(ctx);
	return err;
}

int xfg_comm_allreduce(xfg_ctx *ctx)
{
	int err = 0;
	if (!ctx || !ctx->comm_ready)
		return -EINVAL;
	struct xfg_dev *d = &ctx->dev[0];
	HIPCHK(hipSetDevice(d->ordinal));
	pthread_mutex_lock(&d->lock);
	err = qt_fold_locked(d);   /* (the QT-order counts into the counters reduced) */
	pthread_mutex_unlock(&d->lock);
	if (err)
		return err;
	HIPCHK(hipStreamSynchronize(d->stream));
	ctx->reduced = 0;
	if (ncclGroupStart() != ncclSuccess)
		return -EIO;
	ncclResult_t r = ncclSuccess;
	for (int i = 0; i < NMAPS_HASH && r == ncclSuccess; i++)
		r = ncclAllReduce(d->m[i].hits, d->m[i].red_hits, (size_t)ctx->t[i].nslots + 1,
				  ncclUint64, ncclSum, ctx->comm, d->stream);
	if (r == ncclSuccess)
		r = ncclAllReduce(d->port_hits, d->red_port_hits, XFG_PORT_MAP_ENTRIES, ncclUint64,
				  ncclSum, ctx->comm, d->stream);
	if (r == ncclSuccess)
		r = ncclAllReduce(d->stats, d->red_stats, 10, ncclUint64, ncclSum, ctx->comm, d->stream);
	/* the group is closed whatever happened inside it */
	const ncclResult_t e = ncclGroupEnd();
	if (r != ncclSuccess || e != ncclSuccess)
		return -EIO;
	HIPCHK(hipStreamSynchronize(d->stream));
	ctx->reduced = 1;
	return 0;
fail:
	return err;
}
