/* Test-infrastructure shim (NOT product code).
 *
 * Lets the reference's eBPF-C hot path (xdp-filter/xdpfilt_prog.h and the
 * ten xdpfilt_*.c variants) compile unmodified as ordinary host C, so it can
 * serve as the parity oracle.  Only the handful of libbpf macros the path
 * touches are provided; bpf_map_lookup_elem() becomes a host hook that the
 * driver (oracle/ref_driver.c) implements with plain exact-match tables.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#define SEC(x)
#define __uint(name, val) int (*name)[val]
#define __type(name, val) __typeof__(val) *name
#define LIBBPF_PIN_BY_NAME 1
#ifndef __always_inline
#define __always_inline inline __attribute__((always_inline))
#endif

void *xfref_host_map_lookup(const void *map, const void *key);
#define bpf_map_lookup_elem(m, k) xfref_host_map_lookup((m), (k))
