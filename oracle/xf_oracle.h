/* oracle/xf_oracle.h — CPU restatement of xdp-filter's per-packet path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this; the product (libxdpfilter_gpu)
 * never links or calls it.  The reference itself cannot be built here
 * (xdpfilt_prog.h needs libbpf and the kernel's BPF map runtime; DESIGN.md
 * §2): parity of this restatement is pinned by the known-answer rows of
 * tests/kat.py, each restating a check of the reference's own tests
 * (under xdp-filter/tests/) with its file:line, and by tests/test_oracle.py.
 */
#ifndef XF_ORACLE_H
#define XF_ORACLE_H
#include <stdint.h>

typedef struct xfo_map xfo_map;

/* Exact-match index over a caller-owned rule list of @n keys of @keylen bytes
 * (the semantics of a BPF_MAP_TYPE_PERCPU_HASH lookup). */
xfo_map *xfo_map_new(uint32_t n, uint32_t keylen, const uint8_t *keys);
void xfo_map_free(xfo_map *m);

/* The same index plus a hash table probed once per lookup (the reference's
 * BPF hash-map cost model; bench.py's CPU baseline), whose slots carry each
 * rule's flag byte from @vals as it is now: runs must use values with the
 * same flags (counters may differ).  Same results as xfo_map_new. */
xfo_map *xfo_map_new_hashed(uint32_t n, uint32_t keylen, const uint8_t *keys,
			    const uint64_t *vals);

/* Run program @features (an XFG_FEAT_* word, e.g. _features of
 * xdpfilt_dny_all = ALL|DENY) over a batch: frames at data + offsets[i] (or
 * data + i * stride), u16 or u32 lengths; values and stats are accumulated
 * in place, one verdict byte per frame. */
int xfo_run(uint32_t features, const uint8_t *data, const uint64_t *offsets,
	    uint32_t stride, const void *lens, int lens_u16, uint64_t n,
	    uint64_t *ports, const xfo_map *m4, uint64_t *v4,
	    const xfo_map *m6, uint64_t *v6, const xfo_map *me, uint64_t *ve,
	    uint8_t *verdicts, uint64_t *stats);

/* Same, split over @nthreads threads with private value/stats copies that
 * are summed at the end — the per-CPU map model of the reference. */
int xfo_run_mt(uint32_t features, const uint8_t *data, const uint64_t *offsets,
	       uint32_t stride, const void *lens, int lens_u16, uint64_t n,
	       uint64_t *ports, const xfo_map *m4, uint64_t *v4, uint32_t n4,
	       const xfo_map *m6, uint64_t *v6, uint32_t n6,
	       const xfo_map *me, uint64_t *ve, uint32_t ne,
	       uint8_t *verdicts, uint64_t *stats, int nthreads);
#endif
