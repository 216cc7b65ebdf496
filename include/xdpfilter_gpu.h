/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xdpfilter_gpu.h — C ABI of the MI355X-native xdp-filter classifier.
 *
 * This is the drop-in boundary for xdp-filter's per-packet hot path: the ten
 * eBPF programs xdpfilt_{alw,dny}_{all,eth,ip,tcp,udp} built from
 * xdp-filter/xdpfilt_prog.h:214-310 (reference v1.6.3), their BPF maps
 * (xdp-filter/xdpfilt_prog.h:67-185, headers/xdp/xdp_stats_kern.h:20-26) and
 * the userspace operations the xdp-filter CLI performs on them
 * (xdp-filter/xdp-filter.c:48-157).  The per-packet program becomes a batch
 * HIP kernel over packets resident in HBM; the per-CPU BPF maps become
 * per-device tables whose values keep the reference encoding
 * (hits << COUNTER_SHIFT) | flags.
 *
 * Plain C types only (no HIP/torch types): streams are passed as void*
 * (a hipStream_t, or NULL for the device's default stream of this library).
 * Errors are negative errno values, as in libxdp/libbpf
 * (headers/xdp/libxdp.h:51-53).
 */
#ifndef XDPFILTER_GPU_H
#define XDPFILTER_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants: identical values to xdp-filter/common_kern_user.h:4-19 ---- */
#define XFG_FEAT_TCP      (1u << 0)
#define XFG_FEAT_UDP      (1u << 1)
#define XFG_FEAT_IPV6     (1u << 2)
#define XFG_FEAT_IPV4     (1u << 3)
#define XFG_FEAT_ETHERNET (1u << 4)
#define XFG_FEAT_ALL      (XFG_FEAT_TCP | XFG_FEAT_UDP | XFG_FEAT_IPV6 | \
			   XFG_FEAT_IPV4 | XFG_FEAT_ETHERNET)
#define XFG_FEAT_ALLOW    (1u << 5)
#define XFG_FEAT_DENY     (1u << 6)

#define XFG_MAP_FLAG_SRC  (1u << 0)
#define XFG_MAP_FLAG_DST  (1u << 1)
#define XFG_MAP_FLAG_TCP  (1u << 2)
#define XFG_MAP_FLAG_UDP  (1u << 3)
#define XFG_MAP_FLAGS     (XFG_MAP_FLAG_SRC | XFG_MAP_FLAG_DST | \
			   XFG_MAP_FLAG_TCP | XFG_MAP_FLAG_UDP)
#define XFG_COUNTER_SHIFT 6

/* enum xdp_action values (headers/linux/bpf.h:6130-6136) */
#define XFG_XDP_ABORTED   0
#define XFG_XDP_DROP      1
#define XFG_XDP_PASS      2
#define XFG_ACTION_MAX    5   /* XDP_REDIRECT + 1, headers/xdp/xdp_stats_kern_user.h:21 */

/* Default hash-map capacity = the reference's max_entries
 * (xdp-filter/xdpfilt_prog.h:115,146,181). */
#define XFG_DEFAULT_MAP_CAPACITY 10000u
#define XFG_PORT_MAP_ENTRIES     65536u   /* xdp-filter/xdpfilt_prog.h:69 */

/* Maps, named as the reference pins them (xdp-filter/common_kern_user.h:21-24). */
enum xfg_map_id {
	XFG_MAP_PORTS    = 0, /* "filter_ports":    key u32 = raw be16 port (htons(port)), PERCPU_ARRAY */
	XFG_MAP_IPV4     = 1, /* "filter_ipv4":     key 4 bytes, network order */
	XFG_MAP_IPV6     = 2, /* "filter_ipv6":     key 16 bytes (struct in6_addr) */
	XFG_MAP_ETHERNET = 3, /* "filter_ethernet": key 6 bytes (struct ethaddr) */
	XFG_MAP_NUM      = 4,
};

/* struct xdp_stats_record, headers/xdp/xdp_stats_kern_user.h:10-19 */
struct xfg_stats_record {
	uint64_t packets;
	uint64_t bytes;
};

typedef struct xfg_ctx xfg_ctx;

struct xfg_open_opts {
	size_t sz;               /* sizeof(struct xfg_open_opts), for extension */
	uint32_t features;       /* XFG_FEAT_* requested | XFG_FEAT_ALLOW or _DENY */
	const int *devices;      /* HIP device ordinals; NULL with ndev>0 => 0..ndev-1 */
	int ndev;                /* 0 => host-only context: map CRUD works, classify -ENODEV */
	uint32_t ipv4_capacity;  /* 0 => XFG_DEFAULT_MAP_CAPACITY */
	uint32_t ipv6_capacity;
	uint32_t eth_capacity;
	uint32_t hash_seed;      /* 0 => fixed default seed */
	/* IPv4 maps with at least this many keys are looked up through the
	 * one-read quotient index when it applies (fixed-stride batches, no
	 * live Ethernet key, one or both IPv4 lookup directions live, the same
	 * flags on every device): 0 =>
	 * default (2^18), UINT32_MAX => never.  Results never depend on it. */
	uint32_t qt_min_keys;
	/* Header window of the pipelined kernels for fixed-stride batches
	 * whose stride exceeds 64 bytes: 0 => 64 (default: half the bytes of
	 * a 128-byte window per frame; a frame whose parse reaches past byte
	 * 64 -- IPv6/TCP, long IPv6 extension chains, IPv4 options -- takes the
	 * deferred walk over the whole frame), 128 => 128-byte windows.
	 * Results never depend on it. */
	uint32_t window;
};

/*
 * Program selection, same rule as find_prog_file() (xdp-filter/xdp-filter.c:48-60):
 * the first program in xdp-filter/Makefile:3-6 order whose feature bits are a
 * superset of @features.  Returns 0 and the program's name/features, or
 * -ENOENT (no program matches, e.g. ALLOW|DENY both set) / -EINVAL (0).
 */
int xfg_select_program(uint32_t features, const char **prog_name,
		       uint32_t *prog_features);

/* Open a context: selects the program, allocates the tables on every device. */
int xfg_open(xfg_ctx **out, const struct xfg_open_opts *opts);
void xfg_close(xfg_ctx *ctx);

const char *xfg_prog_name(const xfg_ctx *ctx);      /* e.g. "xdpfilt_dny_all" */
uint32_t xfg_prog_features(const xfg_ctx *ctx);     /* the program's _features word */
int xfg_num_devices(const xfg_ctx *ctx);            /* analogue of libbpf_num_possible_cpus() */
const char *xfg_strerror(int err);

/* The classify kernel the last launch on device @dev ran (introspection for
 * tests and tools): XFG_PATH_GENERAL (offsets, descriptors, header
 * windows), _PIPELINE (fixed stride, any live key), _IPV4 (IPv4 keys only:
 * prefilter + bucket line), _QT (IPv4 keys only: the quotient index),
 * _ETH (the Ethernet-only programs, their map as an LDS key table); or
 * -EINVAL / -ENOENT (no launch yet). */
#define XFG_PATH_GENERAL  0
#define XFG_PATH_PIPELINE 1
#define XFG_PATH_IPV4     2
#define XFG_PATH_QT       5
#define XFG_PATH_ETH      6
int xfg_last_path(const xfg_ctx *ctx, int dev);

/*
 * Map operations.  As with a BPF per-CPU map, a value is one u64 per device
 * (vals[xfg_num_devices()]), or exactly one u64 on a host-only context.
 *   lookup:  -ENOENT if the key is absent (hash maps); ports always exist.
 *   update:  insert or overwrite; -E2BIG when a hash map is full.
 *   delete:  -ENOENT if absent; ports: -EINVAL (array maps cannot delete).
 *   get_next_key: key==NULL => first key; -ENOENT after the last one.
 * Key sizes: ports 4 (u32, < 65536), ipv4 4, ipv6 16, ethernet 6.
 * A value read after a classify includes every hit of the classifies queued
 * before it on that device (the quotient-index path keeps its counts per
 * index slot on the device; the first IPv4-map read, write or all-reduce
 * after it folds them in, one kernel on the device's stream).
 */
int xfg_map_lookup(xfg_ctx *ctx, int map, const void *key, uint64_t *vals);
int xfg_map_update(xfg_ctx *ctx, int map, const void *key, const uint64_t *vals);
int xfg_map_delete(xfg_ctx *ctx, int map, const void *key);
int xfg_map_get_next_key(xfg_ctx *ctx, int map, const void *key, void *next_key);
/* Bulk insert/overwrite with per-device values, as bpf_map_update_elem()
 * takes one value per possible CPU: vals[i * nvals + d] is device d's value
 * of key i (nvals = max(xfg_num_devices(), 1)).  The rule store reloads
 * saved hit counts onto one device with it (xdpfilter_io.h). */
int xfg_map_update_batch_percpu(xfg_ctx *ctx, int map, const void *keys,
				const uint64_t *vals, uint64_t n);
/* Number of keys present (ports: number of non-zero entries). */
int64_t xfg_map_count(xfg_ctx *ctx, int map);
/* Bulk lookup of @n keys (status readout, parity checks): vals[i*ndev + d]
 * receives device d's value of key i, present[i] (if not NULL) 1/0; absent
 * keys read as 0.  Returns the number of keys found or a negative errno. */
int64_t xfg_map_lookup_batch(xfg_ctx *ctx, int map, const void *keys, uint64_t n,
			     uint64_t *vals, uint8_t *present);
/* Bulk insert/overwrite of @n keys with the same value on every device
 * (rule-set loading).  Returns 0 or the first error (-E2BIG, ...). */
int xfg_map_update_batch(xfg_ctx *ctx, int map, const void *keys, const uint64_t *vals,
			 uint64_t n);

/*
 * A packet batch resident on ONE device.  Packet i starts at
 *   data + (offsets ? offsets[i] : i * stride)
 * and is lens[i] bytes long (u16 lens if lens_u16, else u32).  Every packet
 * start must be 16-byte aligned and the buffer readable up to the next
 * 16-byte boundary past its end (AF_XDP UMEM chunks and the pcap/synthetic
 * ingest paths of this library satisfy this).  Packet length is not limited
 * by stride when offsets are given.
 */
struct xfg_batch {
	const void *data;
	const uint64_t *offsets;
	const void *lens;
	uint64_t count;
	uint32_t stride;
	uint32_t lens_u16;
};

/*
 * Classify a device-resident batch on device @dev (index into the context's
 * devices): writes one enum xdp_action byte per packet to @verdicts (device
 * memory), bumps the matched rule's counter on that device and records
 * per-action stats, exactly as xdpfilt_<mode>() + xdp_stats_record_action()
 * do per packet.  Stream-ordered on @stream (hipStream_t or NULL).
 */
int xfg_classify(xfg_ctx *ctx, int dev, const struct xfg_batch *batch,
		 uint8_t *verdicts, void *stream);

/*
 * AF_XDP descriptors in device memory: packet i is RX ring
 * record descs[(first + i) & mask], a struct xdp_desc {u64 addr; u32 len;
 * u32 options} (headers/linux/if_xdp.h:110-114, read with
 * xsk_ring_cons__rx_desc(), headers/xdp/xsk.h:79-85), over the UMEM at
 * @umem: its bytes start at umem + (addr & ((1 << 48) - 1)) + (addr >> 48)
 * (xsk_umem__add_offset_to_addr(), headers/xdp/xsk.h:173-186) and it is len
 * bytes long.  mask = ring entries - 1 (a power of two), or 0xffffffff for
 * a plain array.  Frame starts must be 16-byte aligned (default UMEM frame
 * sizes and headroom are) and readable up to the next 16-byte boundary past
 * their end.  Single-buffer descriptors only (XDP_PKT_CONTD clear).
 */
struct xfg_desc_batch {
	const void *umem;
	const void *descs;
	uint32_t first;
	uint32_t mask;
	uint64_t count;
};

int xfg_classify_descs(xfg_ctx *ctx, int dev, const struct xfg_desc_batch *batch,
		       uint8_t *verdicts, void *stream);

/*
 * Host-resident batch (struct xfg_batch in host memory): classifies it on
 * device @dev and writes the verdicts to host memory.  Only each frame's
 * first 128 bytes (its header window) and its length cross PCIe -- gathered
 * into pinned staging by a per-device thread pool and pipelined H2D / kernel
 * / D2H over chunks; a frame whose program reads past its window is sent
 * again whole and classified from it, so verdicts, counters and stats are
 * exactly those of a whole-frame run.  A fixed stride of at most 128 bytes
 * is staged slot for slot; a batch in a registered buffer
 * (xfg_host_register) is read in place instead.  Concurrent calls on different devices run in
 * parallel; staging memory per device is fixed (about 70 MB pinned).
 * Replaces the per-packet program run of the attach path
 * (xdp-filter/xdpfilt_prog.h:214-310 over frames the kernel hands it).
 */
int xfg_classify_host(xfg_ctx *ctx, int dev, const struct xfg_batch *batch,
		      uint8_t *verdicts);

/*
 * Register a long-lived host buffer (a capture ring, an AF_XDP UMEM) for
 * zero-copy reads: a host batch whose fixed-stride slots (stride a multiple
 * of 16) lie inside a registered buffer, or an AF_XDP batch
 * (xfg_classify_xsk_host) whose UMEM does, is read by the kernels where it
 * lies through the buffer's device mapping -- only the bytes the programs
 * load cross PCIe, and no frame is staged.  Pins and maps the pages
 * (hipHostRegister, portable + mapped) until xfg_host_unregister() or
 * xfg_close().  At most 16 buffers per context; -EEXIST if it overlaps a
 * registered one.
 */
int xfg_host_register(xfg_ctx *ctx, void *p, size_t bytes);
int xfg_host_unregister(xfg_ctx *ctx, void *p);

/* Threads of a device's host-path gather pool (1-16): the process's CPU set,
 * or XFG_HOST_THREADS, or OMP_NUM_THREADS when above 1 (torchrun's default
 * of 1 is not taken as the process's share).  Performance only. */
int xfg_host_threads(void);

/*
 * AF_XDP RX in host memory: the consumer side of an XDP socket's RX ring
 * (xsk_ring_cons__peek() / xsk_ring_cons__rx_desc() / xsk_ring_cons__release(),
 * headers/xdp/xsk.h:80-86,143-165).  Packet i is ring record
 * descs[(first + i) & mask], a struct xdp_desc {u64 addr; u32 len; u32
 * options} (headers/linux/if_xdp.h:110-114), over the host UMEM @umem of
 * @umem_bytes: its bytes start at umem + (addr & ((1 << 48) - 1)) +
 * (addr >> 48) (xsk_umem__add_offset_to_addr(), headers/xdp/xsk.h:173-186;
 * unaligned-chunk mode).  mask = ring entries - 1 (a power of two), or
 * 0xffffffff for a plain array; count <= entries.  Classified as
 * xfg_classify_host does (header windows, exact whole-frame fallback; a
 * registered UMEM read in place); -EINVAL if a frame lies outside the UMEM.  The caller releases the ring
 * entries after the call returns.
 */
int xfg_classify_xsk_host(xfg_ctx *ctx, int dev, const struct xfg_desc_batch *batch,
			  uint64_t umem_bytes, uint8_t *verdicts);

/*
 * Verdict compaction: writes the indices i (ascending) with verdicts[i] ==
 * @action to @idx and their number to *@count — the list a forwarding stage
 * walks (the reference passes XDP_PASS frames on up the chain,
 * xdp-filter/xdpfilt_prog.h:209-212).  Device memory: @verdicts (n bytes),
 * @idx (room for n u32), @count (one u64).  One pass (wave ballots and
 * prefix sums, decoupled look-back between tiles), stream-ordered on @stream
 * (NULL: the library's stream of the device).  n < 2^32.
 */
int xfg_compact(xfg_ctx *ctx, int dev, const uint8_t *verdicts, uint64_t n, uint32_t action,
		uint32_t *idx, uint64_t *count, void *stream);

/* Per-action stats summed over devices (the userspace per-CPU sum of
 * lib/util/stats.c:140-172), or for one device. */
int xfg_stats_read(xfg_ctx *ctx, struct xfg_stats_record out[XFG_ACTION_MAX]);
int xfg_stats_read_dev(xfg_ctx *ctx, int dev, struct xfg_stats_record out[XFG_ACTION_MAX]);
int xfg_stats_reset(xfg_ctx *ctx);

/* Wait for all work queued by this library on every device. */
int xfg_sync(xfg_ctx *ctx);

/* ---- device memory helpers (so a C host needs no HIP headers) ---- */
void *xfg_dev_alloc(xfg_ctx *ctx, int dev, size_t bytes);
void xfg_dev_free(xfg_ctx *ctx, int dev, void *p);
int xfg_memcpy_h2d(xfg_ctx *ctx, int dev, void *dst, const void *src, size_t bytes);
int xfg_memcpy_d2h(xfg_ctx *ctx, int dev, void *dst, const void *src, size_t bytes);
void *xfg_host_alloc_pinned(size_t bytes);
void xfg_host_free_pinned(void *p);

/* ---- timing: HIP events on the library's stream for device @dev ---- */
/* Launch classify @iters times back-to-back on the device's stream and
 * return the average kernel duration in ms measured with HIP events recorded
 * on that same stream (used by bench.py for the roofline figure). */
int xfg_classify_timed(xfg_ctx *ctx, int dev, const struct xfg_batch *batch,
		       uint8_t *verdicts, int iters, double *avg_ms);

/* Streaming-read probe: average duration of a kernel that reads @bytes of
 * device memory at @src with 16-byte non-temporal loads (the achievable HBM
 * read rate next to the spec peak, for the roofline report). */
int xfg_stream_read_timed(xfg_ctx *ctx, int dev, const void *src, uint64_t bytes, int iters,
			  double *avg_ms);

/*
 * Multi-process reduction over RCCL (one process per GPU, one device per
 * context).  Rank 0 calls xfg_comm_unique_id() and distributes the 128-byte
 * id out of band; every rank then calls xfg_comm_init().  xfg_comm_allreduce()
 * sums per-rule hit counters and per-action stats across ranks (ncclUint64,
 * ncclSum, in place on a reduction copy); afterwards xfg_map_lookup() /
 * xfg_stats_read() on every rank return the job-wide totals until the next
 * classify call.  This is the GPU analogue of summing per-CPU values
 * (xdp-filter/xdp-filter.c:93-103).
 */
#define XFG_COMM_ID_BYTES 128
int xfg_comm_unique_id(uint8_t id[XFG_COMM_ID_BYTES]);
int xfg_comm_init(xfg_ctx *ctx, int nranks, int rank, const uint8_t id[XFG_COMM_ID_BYTES]);
int xfg_comm_allreduce(xfg_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* XDPFILTER_GPU_H */
