"""GPU parity at the bench's own batch size (SURVEY.md §8d's C3, as bench.py
runs it): everything sized by the batch -- the hit-log partition slices
(one per partition and classify workgroup, 2 * ceil(wg_max / 256) + 64
entries, wg_max = the most packets a workgroup's waves can log; a fuller
slice spills to the canonical counters, xfg_ctx.c launch_batch), the
per-wave deferred lists and hit-log regions, the count kernel -- is checked
against the CPU restatement (oracle/) on
every host thread, bit-exact: verdicts, all 1M rule values, per-action
stats.  Contract: xdp-filter/xdpfilt_prog.h:56-64,214-310.

  * C3 at 2^26 packets, 16-bit lengths: bench.py's rank-0 shard exactly;
  * a skewed C3 at 2^25: every hit on one of 8 hot rules, so each hot
    rule's hits in one workgroup (~1.9M over the grid) overfill that
    workgroup's slice of the rule's partition several times over: the
    spill paths (a full LDS ring or a chunk past the slice: the LDS counter
    cache, then an atomic on the QT-order count, beside the logged entries
    the count kernel adds) run at scale;
  * 9M IPv4 rules at 2^25 packets: an index of 2^21 buckets whose hit log
    holds u32 local indices (past 65536 per partition) and takes the count
    kernel eight passes -- the log runs only for batches of at least as many
    packets as the index has slots (xfg_ctx.c launch_batch).
"""
import os

import numpy as np
import pytest

import xftools as X
from test_gpu import assert_same, gpu_values, make_filter

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def _threads():
    t = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        t = min(t, int(omp))
    return max(1, min(t, 16))


def _c3_rules():
    # bench.py setup(): 1M IPv4 dst rules (seed 3) + 16 dst|tcp|udp ports
    v4 = X.rand_keys(3, int(1_000_000 * 1.02) + 16, 4)[:1_000_000]
    ports = (np.arange(16, dtype=np.uint16) * 1031 + 53).astype(np.uint16)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    return rules, v4, ports


def _check(G, rules, data, lens, cap=1_000_000, **kw):
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_dny_all"], data, lens, rules,
                                   stride=64, nthreads=_threads())
    f = make_filter(G, "xdpfilt_dny_all", ipv4_capacity=cap, **kw)
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert f.last_path() == f.PATH_QT   # the quotient index (1M dst rules)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()
    return ov, orules


@pytest.mark.timeout(900)
def test_c3_at_bench_batch_2p26(G):
    rules, v4, ports = _c3_rules()
    n = 1 << 26
    data, lens = X.gen_workload(3, 3, n, 64, v4=v4, ports=ports, dst_permille=500,
                                port_permille=250, bad_permille=10)
    ov, _ = _check(G, rules, data, lens.astype(np.uint16))
    assert (ov == 2).sum() > n // 3          # the hits PASS under deny
    assert (ov == 0).sum() > n // 1000       # malformed frames ABORT


@pytest.mark.timeout(900)
def test_c3_skewed_hits_overfill_log_partitions_2p25(G):
    rules, v4, ports = _c3_rules()
    n = 1 << 25
    hot = v4[:8]
    data, lens = X.gen_workload(33, 3, n, 64, v4=hot, ports=ports, dst_permille=500,
                                port_permille=250, bad_permille=10)
    _, orules = _check(G, rules, data, lens.astype(np.uint16))
    hits = orules.v4_vals[:8] >> 6
    # launch_batch's slice capacity for the QT kernel's grid (2 workgroups of
    # 8 waves per CU, 256 CUs on MI355X; any grid of 128-1024 workgroups
    # gives the same verdict): a hot rule's hits per workgroup exceed it
    for grid in (128, 256, 512, 1024):
        nw, nt = grid * 8, (n + 63) // 64
        wg_max = 8 * ((nt + nw - 1) // nw * 64)
        pcap = (2 * ((wg_max + 255) // 256) + 64 + 7) & ~7
        assert (hits // grid > 2 * pcap).all(), (grid, hits, pcap)
    # (the other rules only see random addresses that happen to be ruled)
    assert int((orules.v4_vals[8:] >> 6).sum()) < n // 1000


@pytest.mark.timeout(900)
@pytest.mark.parametrize("v6", ["none", "both"])
def test_wide_hit_log_9m_rules_2p25(G, v6):
    """... and (v6 "both") 200k IPv6 rules, dst, src and src|dst, beside
    them: the IPv6 lookups in the index kernel's loop with the u32 log
    (VERDICT r4 item 3), a third of the IPv6 frames from a ruled source."""
    n4 = 9_000_000
    v4 = X.rand_keys(41, int(n4 * 1.02) + 16, 4)[:n4]
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    n = 1 << 25
    kw = {}
    v6k = None
    if v6 == "both":
        rng = np.random.default_rng(43)
        v6k = X.rand_keys(44, 200_000, 16)
        rules.v6_keys = v6k
        rules.v6_vals = rng.choice(np.array([1, 2, 3], np.uint64), len(v6k))
        kw = {"ipv6_capacity": 200_000}
    data, lens = X.gen_workload(42, 3, n, 64, v4=v4, v6=v6k, dst_permille=600, bad_permille=10)
    if v6k is not None:
        fr = data.reshape(-1, 64)
        six = np.nonzero((fr[:, 12] == 0x86) & (fr[:, 13] == 0xdd))[0][::3]
        fr[six, 22:38] = v6k[np.arange(len(six)) * 7919 % len(v6k)]
    ov, _ = _check(G, rules, data, lens.astype(np.uint16), cap=n4, **kw)
    assert (ov == 2).sum() > n // 3


@pytest.mark.timeout(600)
def test_qt_counts_cross_2p32_packets_product(G):
    """More than 2^32 packets through the quotient index on one device, on
    the product library: a 2^26-packet batch whose every frame hits ONE
    rule, classified 65 times back to back (4.36e9 packets, all on that
    rule's 32-bit QT-order count, xfg_kargs.qt_hits).  The runtime must fold
    the counts into the 64-bit canonical counters before they could wrap
    (xfg_ctx.c qt_fold_queued, at the real 2^32 threshold): the rule's value
    is its pre-existing hits plus 65 * 2^26 (CHECK_MAP adds 1 << 6 a hit,
    xdpfilt_prog.h:60-61), the stats 65 passes.  The batch is a 2^16-frame
    pattern repeated, so the oracle runs on the pattern."""
    rng = np.random.default_rng(201)
    v4 = X.rand_keys(202, 20000, 4)
    hot = v4[17]
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64) | (rng.integers(0, 50, len(v4)).astype(np.uint64) << 6)
    ports = np.array([53, 80], np.uint16)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    m, reps_tile, launches = 1 << 16, 1 << 10, 65
    pd, pl = X.gen_workload(203, 3, m, 64, v4=hot.reshape(1, 4), ports=ports, dst_permille=1000,
                            bad_permille=0)
    fr = pd.reshape(m, 64)
    ip4 = (fr[:, 12] == 8) & (fr[:, 13] == 0)
    first = int(np.nonzero(ip4)[0][0])
    fr[~ip4] = fr[first]                       # every frame IPv4, dst = the hot rule
    pl[~ip4] = pl[first]
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, pd, pl, rules, stride=64, nthreads=_threads())
    assert (ov == 2).all()                     # every frame hits (PASS under deny)
    n = m * reps_tile
    total = n * launches
    assert total > 1 << 32
    data = np.tile(pd, reps_tile)
    lens = np.tile(pl.astype(np.uint16), reps_tile)
    f = make_filter(G, "xdpfilt_dny_all", ipv4_capacity=1 << 16, qt_min_keys=1)
    f.load_rules(rules)
    d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(lens)
    del data
    f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_v.ptr, launches, lens_u16=True)
    assert f.last_path() == f.PATH_QT
    v = d_v.download(np.zeros(n, np.uint8))
    assert (v == 2).all()
    six = np.uint64(6)
    pre = rules.v4_vals >> six
    per_pass = (orules.v4_vals >> six) - pre            # the pattern's hits per rule
    want = ((pre + per_pass * np.uint64(reps_tile * launches)) << six) | (rules.v4_vals & np.uint64(63))
    got = f.values_of(G.MAP_IPV4, rules.prepared().v4_keys)
    np.testing.assert_array_equal(got, want)
    hot_i = int(np.nonzero((rules.prepared().v4_keys == hot).all(axis=1))[0][0])
    assert int(got[hot_i] >> six) - int(pre[hot_i]) == total
    np.testing.assert_array_equal(f.stats(), ost * (reps_tile * launches))
    f.close()
