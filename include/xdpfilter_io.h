/* SPDX-License-Identifier: GPL-2.0 */
/*
 * xdpfilter_io.h — the host-side formats on either side of the classifier
 * (SURVEY.md §8(f)): where packets come from, where verdicts go, and where
 * the rule maps live between runs.  Plain C, part of libxdpfilter_gpu.so;
 * nothing here touches the GPU.
 *
 *   f1  ingest     pcap / pcapng files -> a host batch of 16-byte aligned
 *                  frames (the layout xfg_classify_host() and the device
 *                  batch want); AF_XDP descriptor records (struct xdp_desc,
 *                  headers/linux/if_xdp.h:110-114) are classified in place
 *                  by xfg_classify_descs() in xdpfilter_gpu.h.
 *   f2  rule store the bpffs pin directory /sys/fs/bpf/xdp-filter/<map>
 *                  (LIBBPF_PIN_BY_NAME, xdp-filter/xdpfilt_prog.h:72,118,149,
 *                  184; lib/util/util.c:625-640) becomes a state directory
 *                  holding one file per map under the same names, plus one
 *                  program record per interface (programs/<ifname>).
 *   f3  readout    xdp_stats_map is a file of per-action {packets, bytes};
 *                  the CLI prints it like lib/util/stats.c:48-125.
 *   f4  dump       pcapng with the EPB verdict option (type eBPF-XDP), the
 *                  record xdpdump writes (lib/util/xpcapng.c:392-479).
 *
 * Errors are negative errno values.
 */
#ifndef XDPFILTER_IO_H
#define XDPFILTER_IO_H

#include <stddef.h>
#include <stdint.h>

#include "xdpfilter_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- f1: host batches ---------------------------------------------------- */
/* Frames packed at 16-byte aligned offsets in one buffer, so that the batch
 * satisfies struct xfg_batch's alignment rule as it stands.  lens[] is the
 * captured length: the bytes the program sees (data_end - data). */
struct xfg_host_batch {
	uint8_t *data;
	uint64_t *offsets;
	uint32_t *lens;
	uint32_t *orig_lens;    /* on-the-wire length from the capture record */
	uint64_t *ts_ns;        /* capture timestamp, ns since the epoch */
	uint64_t count;
	uint64_t bytes;         /* bytes used in data (16-byte multiple) */
	uint32_t linktype;      /* 1 = Ethernet (the only type the program parses) */
	uint32_t pad;
};

/* Read a classic pcap (µs or ns, either byte order) or pcapng file (SHB /
 * IDB / EPB / SPB / OPB).  -EINVAL for a malformed file, -EPROTONOSUPPORT for
 * a non-Ethernet link type. */
int xfg_pcap_read(const char *path, struct xfg_host_batch *out);
void xfg_host_batch_free(struct xfg_host_batch *b);

/* ---- f4: verdict dump ------------------------------------------------------ */
/* Write every frame of @b as a pcapng EPB on one interface named @ifname,
 * carrying option epb_verdict = {type 2 (eBPF XDP), u64 verdicts[i]} as
 * xpcapng_dump_enhanced_pkt() does (lib/util/xpcapng.c:392-479). */
int xfg_pcapng_write_verdicts(const char *path, const char *ifname,
			      const struct xfg_host_batch *b, const uint8_t *verdicts);

/* ---- f2: rule store -------------------------------------------------------- */
/* Map file names, as pinned by the reference (xdp-filter/common_kern_user.h:
 * 21-26, headers/xdp/xdp_stats_kern_user.h:8). */
#define XFG_STORE_MAP_PORTS    "filter_ports"
#define XFG_STORE_MAP_IPV4     "filter_ipv4"
#define XFG_STORE_MAP_IPV6     "filter_ipv6"
#define XFG_STORE_MAP_ETHERNET "filter_ethernet"
#define XFG_STORE_MAP_STATS    "xdp_stats_map"

const char *xfg_store_map_name(int map);   /* XFG_MAP_* -> file name */

/* Does the store hold map @map (i.e. was it "pinned" by a load)? 1 / 0 */
int xfg_store_has_map(const char *dir, int map);
/* Create an empty map file if none exists (load pins a program's maps). */
int xfg_store_create_map(const char *dir, int map, uint32_t capacity);
/* Remove a map file (unload's remove_unused_maps, xdp-filter.c:357-431). */
int xfg_store_remove_map(const char *dir, int map);
/* Capacity recorded for @map (hash maps; ports 65536); -ENOENT if absent. */
int64_t xfg_store_map_capacity(const char *dir, int map);

/* Copy every key of every map present in @dir into @ctx.  The store keeps
 * one value per key: flags | (hits summed over devices << 6), the readout
 * of map_get_counter_flags() (xdp-filter/xdp-filter.c:73-109).  Device 0
 * receives the value, the other devices the flags with zero hits, so sums
 * over devices are preserved whatever the device count. */
int xfg_store_load(xfg_ctx *ctx, const char *dir);
/* Write every map of @ctx that the store holds back to @dir (hits summed
 * over devices), atomically per file (write + rename). */
int xfg_store_save(xfg_ctx *ctx, const char *dir);

/* Per-action stats file: five {packets, bytes} records (created zeroed by
 * xfg_store_stats_write; reading an absent file gives -ENOENT). */
int xfg_store_stats_read(const char *dir, struct xfg_stats_record out[XFG_ACTION_MAX]);
int xfg_store_stats_write(const char *dir, const struct xfg_stats_record in[XFG_ACTION_MAX]);
int xfg_store_stats_remove(const char *dir);

#ifdef __cplusplus
}
#endif
#endif /* XDPFILTER_IO_H */
