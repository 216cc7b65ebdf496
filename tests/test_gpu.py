"""GPU parity tests: the HIP path (libxdpfilter_gpu.so on an MI355X) against
the regression fixture (tests/golden/, restatement-derived: make_golden.py
runs oracle/xf_oracle.c; it pins regressions, the reference-held
expectations are tests/kat.py's rows, checked by test_kat_counters.py) and
against the CPU restatement (oracle/) on seeded batches.  Bit-exact:
verdicts, every rule's value (hits << 6 | flags) and the per-action stats.
"""
import errno

import numpy as np
import pytest

import xftools as X
from conftest import golden_expected_ports, golden_rules

pytestmark = pytest.mark.gpu

VARIANTS = [v for v, _ in X.VARIANTS]


@pytest.fixture(scope="module")
def G():
    import xfgpu
    return xfgpu


def make_filter(G, variant, **kw):
    f = G.Filter(X.VARIANT_FEATURES[variant], ndev=1, **kw)
    assert f.prog_name == variant
    return f


def gpu_values(f, G, rules):
    """Rule values read back through the C ABI, in rule-list order."""
    r = rules.prepared()
    out = X.RuleSet(ports=np.zeros(65536, np.uint64))
    out.ports = f.values_of(G.MAP_PORTS, np.arange(65536, dtype=np.uint32))
    out.v4_keys, out.v6_keys, out.eth_keys = r.v4_keys, r.v6_keys, r.eth_keys
    out.v4_vals = f.values_of(G.MAP_IPV4, r.v4_keys) if len(r.v4_keys) else r.v4_vals.copy()
    out.v6_vals = f.values_of(G.MAP_IPV6, r.v6_keys) if len(r.v6_keys) else r.v6_vals.copy()
    out.eth_vals = f.values_of(G.MAP_ETHERNET, r.eth_keys) if len(r.eth_keys) else r.eth_vals.copy()
    return out


def assert_same(a_verd, a_rules, a_stats, b_verd, b_rules, b_stats):
    np.testing.assert_array_equal(a_verd, b_verd)
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        np.testing.assert_array_equal(getattr(a_rules, fld), getattr(b_rules, fld), err_msg=fld)
    np.testing.assert_array_equal(a_stats, b_stats)


@pytest.mark.parametrize("tag", ["kat", "fuzz"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_restatement_fixture_on_gpu(G, golden, tag, variant):
    g = golden
    rules = golden_rules(g, f"{tag}_rules_")
    data, lens, stride = g[f"{tag}_data"], g[f"{tag}_lens"], int(g["stride"])
    f = make_filter(G, variant)
    f.load_rules(rules)
    verd = f.run(np.ascontiguousarray(data), lens, stride=stride)
    got = gpu_values(f, G, rules)
    p = f"{tag}_{variant}_"
    np.testing.assert_array_equal(verd, g[p + "verdicts"])
    np.testing.assert_array_equal(got.ports, golden_expected_ports(g, p, rules))
    np.testing.assert_array_equal(got.v4_vals, g[p + "v4_vals"])
    np.testing.assert_array_equal(got.v6_vals, g[p + "v6_vals"])
    np.testing.assert_array_equal(got.eth_vals, g[p + "eth_vals"])
    np.testing.assert_array_equal(f.stats()[:, :], g[p + "stats"])
    f.close()


@pytest.mark.parametrize("variant", VARIANTS)
def test_fuzz_vs_oracle_layouts(G, variant):
    """200k structured-fuzz frames: fixed stride (W=128 window), offsets
    layout with shuffled placement, and u16 lengths."""
    rules, pool = X.random_rules(hash(variant) & 0xffff, n4=200, n6=100, ne=40, nports=40)
    data, lens = X.gen_fuzz(17, 200000, 160, rules, pool)
    feats = X.VARIANT_FEATURES[variant]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=160)
    f = make_filter(G, variant)
    f.load_rules(rules)
    v = f.run(data, lens, stride=160)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()
    # offsets + u16 lens: same verdicts
    perm = np.random.default_rng(3).permutation(len(lens))
    data2 = np.zeros_like(data)
    data2.reshape(-1, 160)[np.arange(len(lens))] = data.reshape(-1, 160)[perm]
    offs = np.empty(len(lens), np.uint64)
    offs[perm] = np.arange(len(lens), dtype=np.uint64) * 160
    f = make_filter(G, variant)
    f.load_rules(rules)
    v2 = f.run(data2, lens.astype(np.uint16), offsets=offs)
    np.testing.assert_array_equal(v2, ov)
    np.testing.assert_array_equal(f.stats(), ost)
    f.close()


@pytest.mark.parametrize("kind,variant", [(2, "xdpfilt_dny_ip"), (3, "xdpfilt_dny_all"),
                                          (3, "xdpfilt_alw_all")])
def test_workload_64b_window(G, kind, variant):
    """The bench layout: 64-byte stride, W=64 header window in LDS, 100k IPv4
    rules, 16 dst-port rules, 1% malformed frames."""
    n = 1 << 20
    v4 = X.rand_keys(kind, 100000, 4)
    ports = np.arange(16, dtype=np.uint16) * 7 + 20
    data, lens = X.gen_workload(kind, kind, n, 64, v4=v4, ports=ports)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=64,
                                   nthreads=8)
    f = make_filter(G, variant, ipv4_capacity=len(v4))
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


def test_hot_rule_counter_aggregation(G):
    """Every packet hits one port rule: the wave/same-slot aggregation must
    still count each packet exactly once."""
    n = 1 << 20
    data, lens = X.gen_workload(1, 2, n, 64, dst_permille=0, port_permille=0, bad_permille=0)
    d = data.reshape(n, 64)
    d[:, 36:38] = [0, 53]                   # every UDP dport = 53
    rules = X.RuleSet()
    rules.ports[X.port_key(53)] = 2 | 8
    f = make_filter(G, "xdpfilt_dny_udp")
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert (v == 2).all()
    assert f.lookup(G.MAP_PORTS, X.port_key(53)) == [(n << 6) | 10]
    st = f.stats()
    assert st[2, 0] == n and st[2, 1] == lens.astype(np.uint64).sum()
    # a second batch accumulates like repeated packets in the kernel
    f.run(data, lens, stride=64)
    assert f.lookup(G.MAP_PORTS, X.port_key(53)) == [(2 * n << 6) | 10]
    f.close()


def test_rule_updates_between_batches(G):
    """CRUD between classify calls (the CLI editing live maps): flags change,
    deleted rules stop matching, counters survive flag edits
    (map_set_flags, xdp-filter/xdp-filter.c:111-157)."""
    rules, pool = X.random_rules(77, n4=100, n6=50, ne=20, nports=30)
    data, lens = X.gen_fuzz(5, 50000, 160, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    f = make_filter(G, "xdpfilt_dny_all")
    f.load_rules(rules)
    f.run(data, lens, stride=160)
    _, cur, _ = X.run_oracle(feats, data, lens, rules, stride=160)
    # edit: delete 10 v4 rules, flip flags of 10 v6 rules (counters kept), add a port rule
    keep = np.ones(len(cur.v4_keys), bool)
    keep[:10] = False
    for k in cur.v4_keys[:10]:
        f.delete(G.MAP_IPV4, bytes(k))
    cur.v4_keys, cur.v4_vals = cur.v4_keys[keep], cur.v4_vals[keep]
    for i in range(10):
        nv = (int(cur.v6_vals[i]) & ~0xF) | (3 - (int(cur.v6_vals[i]) & 3) or 1)
        f.update(G.MAP_IPV6, bytes(cur.v6_keys[i]), nv)
        cur.v6_vals[i] = nv
    f.update(G.MAP_PORTS, X.port_key(int(pool[0])), 15)
    cur.ports[X.port_key(int(pool[0]))] = 15
    ov, orules, _ = X.run_oracle(feats, data, lens, cur, stride=160)
    v = f.run(data, lens, stride=160)
    np.testing.assert_array_equal(v, ov)
    got = gpu_values(f, G, cur)
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        np.testing.assert_array_equal(getattr(got, fld), getattr(orules, fld), err_msg=fld)
    f.close()


def test_classify_host_matches_device_path(G):
    rules, pool = X.random_rules(12)
    data, lens = X.gen_fuzz(8, 300000, 160, rules, pool)
    ov, orules, ost = X.run_oracle(X.VARIANT_FEATURES["xdpfilt_alw_all"], data, lens, rules,
                                   stride=160)
    f = make_filter(G, "xdpfilt_alw_all")
    f.load_rules(rules)
    v = f.classify_host(data, lens, stride=160)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


def test_empty_and_tiny_batches(G):
    f = make_filter(G, "xdpfilt_dny_all")
    assert len(f.run(np.zeros(16, np.uint8), np.zeros(0, np.uint32), stride=64)) == 0
    v = f.run(np.zeros(64, np.uint8), np.array([13], np.uint32), stride=64)
    assert v.tolist() == [0]
    assert f.stats()[0].tolist() == [1, 13]
    f.close()


def test_bad_batch_rejected(G):
    f = make_filter(G, "xdpfilt_dny_all")
    with pytest.raises(OSError) as e:
        f.classify(0x1008, 0x1000, 4, 64, 0x1000)    # misaligned data
    assert e.value.errno == errno.EINVAL
    with pytest.raises(OSError):
        f.classify(0x1000, 0x1000, 4, 60, 0x1000)    # stride not a multiple of 16
    f.close()


def test_flag_census_skips_lookups(G):
    """The host keeps the OR of every key's flag bits per map and the kernel
    skips a lookup whose mask no key carries.  Walk the census through
    src-only -> dst-only -> zeroed flags -> deleted keys and check each step
    against the oracle."""
    rules, pool = X.random_rules(31, n4=150, n6=60, ne=30, nports=30)
    data, lens = X.gen_fuzz(9, 60000, 160, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    f = make_filter(G, "xdpfilt_dny_all")
    cur = rules

    def step(mutate):
        nonlocal cur
        mutate()
        f.stats_reset()
        ov, orules, ost = X.run_oracle(feats, data, lens, cur, stride=160)
        v = f.run(data, lens, stride=160)
        assert_same(v, gpu_values(f, G, cur), f.stats(), ov, orules, ost)
        cur = orules

    def set_all(bits):
        for m, kf in ((G.MAP_IPV4, "v4"), (G.MAP_IPV6, "v6"), (G.MAP_ETHERNET, "eth")):
            keys, vals = getattr(cur, kf + "_keys"), getattr(cur, kf + "_vals")
            for i in range(len(keys)):
                vals[i] = (int(vals[i]) & ~63) | bits
                f.update(m, bytes(keys[i]), int(vals[i]))
        for p in pool:
            k = X.port_key(int(p))
            cur.ports[k] = (int(cur.ports[k]) & ~63) | (bits | 8 if bits else 0)
            f.update(G.MAP_PORTS, k, int(cur.ports[k]))

    def first_load():
        for fld in ("v4_vals", "v6_vals", "eth_vals"):
            v = getattr(cur, fld)
            v[:] = (v & ~np.uint64(63)) | np.uint64(1)          # src only
        f.load_rules(cur)

    step(first_load)
    step(lambda: set_all(2))                                    # dst only
    step(lambda: set_all(0))                                    # no flags left
    step(lambda: set_all(3))                                    # both again

    def drop_half():
        keep = np.arange(len(cur.v4_keys)) % 2 == 0
        for k in cur.v4_keys[~keep]:
            f.delete(G.MAP_IPV4, bytes(k))
        cur.v4_keys, cur.v4_vals = cur.v4_keys[keep], cur.v4_vals[keep]
    step(drop_half)
    f.close()


@pytest.mark.parametrize("nports", [1000, 1500])
def test_many_port_rules(G, nports):
    """Up to XFG_PORT_TAB_MAX ruled ports live in the LDS port table (with
    probe displacement at this load); beyond it the kernel falls back to the
    bitmap + port_flags read.  Both against the oracle."""
    rules, pool = X.random_rules(41 + nports, n4=50, n6=20, ne=10, nports=nports)
    data, lens = X.gen_fuzz(13, 80000, 160, rules, pool)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=160)
    f = make_filter(G, "xdpfilt_dny_all")
    f.load_rules(rules)
    v = f.run(data, lens, stride=160)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


@pytest.mark.parametrize("direction", [1, 2])
@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_ip"])
def test_single_direction_rules_vs_oracle(G, direction, variant):
    """The pipelined kernel with IPv4 rules of one direction only (src or
    dst: one live key per packet by the flag census), hot ports, 1%
    malformed frames, the all-zero key among the rules (its own bucket)."""
    n = 1 << 20
    v4 = X.rand_keys(5 + direction, 60000, 4)
    v4 = v4[(v4 != 0).any(axis=1)]
    v4[0] = 0                                       # the zero key (0.0.0.0)
    ports = np.arange(16, dtype=np.uint16) * 7 + 20
    data, lens = X.gen_workload(11 + direction, 3, n, 64, v4=v4, ports=ports)
    d = data.reshape(n, 64)
    if direction == 1:                              # src rules: put rule keys in saddr
        d[:, 26:30] = d[:, 30:34]
    d[::97, 26:34] = 0                              # some 0.0.0.0 addresses
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), direction, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    feats = X.VARIANT_FEATURES[variant]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64, nthreads=8)
    f = make_filter(G, variant, ipv4_capacity=len(v4))
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


def test_hot_key_single_counter(G):
    """Every IPv4 packet hits ONE rule: the wave merge and the LDS counter
    cache must count each packet exactly once."""
    n = 1 << 20
    data, lens = X.gen_workload(2, 2, n, 64, dst_permille=0, port_permille=0, bad_permille=0)
    d = data.reshape(n, 64)
    is_v4 = (d[:, 12] == 8) & (d[:, 13] == 0)
    d[is_v4, 30:34] = [10, 1, 2, 3]
    rules = X.RuleSet()
    rules.v4_keys = np.array([[10, 1, 2, 3]], np.uint8)
    rules.v4_vals = np.array([2], np.uint64)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_ip"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64, nthreads=8)
    f = make_filter(G, "xdpfilt_dny_ip")
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_all", "xdpfilt_dny_eth"])
def test_pipelined_kernel_fuzz_vs_oracle(G, variant):
    """The pipelined kernel (all maps live) on structured fuzz at 128- and
    160-byte strides (W=128; the dense and the strided window loads):
    extension chains past the window, ND targets and multi-key packets go
    through the deferred general path."""
    rules, pool = X.random_rules(hash(variant) & 0xfff, n4=200, n6=100, ne=40, nports=40)
    feats = X.VARIANT_FEATURES[variant]
    for stride in (128, 160):
        data, lens = X.gen_fuzz(23, 100000, stride, rules, pool)
        ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=stride)
        f = make_filter(G, variant)
        f.load_rules(rules)
        v = f.run(data, lens, stride=stride)
        assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
        f.close()


@pytest.mark.parametrize("variant", ["xdpfilt_dny_all", "xdpfilt_alw_ip"])
def test_pipelined_kernel_64b_both_directions(G, variant):
    """W=64 pipelined kernel with IPv4 rules of both directions (two live
    lookups per packet; a Bloom-positive miss of the first key with a second
    candidate goes to the deferred general path)."""
    n = 1 << 20
    v4 = X.rand_keys(44, 80000, 4)
    ports = np.arange(16, dtype=np.uint16) * 7 + 20
    data, lens = X.gen_workload(9, 3, n, 64, v4=v4, ports=ports)
    d = data.reshape(n, 64)
    d[1::3, 26:30] = d[1::3, 30:34]                 # a third of the packets: key as saddr too
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = (np.arange(len(v4)) % 3 + 1).astype(np.uint64)   # src, dst, both
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    feats = X.VARIANT_FEATURES[variant]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64, nthreads=8)
    f = make_filter(G, variant, ipv4_capacity=len(v4))
    f.load_rules(rules)
    v = f.run(data, lens, stride=64)
    assert_same(v, gpu_values(f, G, rules), f.stats(), ov, orules, ost)
    f.close()


def test_rccl_single_rank_reduce(G):
    """The per-CPU-sum readout (xdp-filter/xdp-filter.c:93-103) through RCCL
    at one rank: xfg_comm_unique_id -> xfg_comm_init(nranks=1) -> classify ->
    xfg_comm_allreduce; lookups and stats then read the reduced copies, which
    at one rank equal the local counters.  A later classify invalidates the
    reduced view; a second init replaces the communicator."""
    import os
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    variant = "xdpfilt_dny_all"
    feats = X.VARIANT_FEATURES[variant]
    rules, pool = X.random_rules(91, n4=80, n6=40, ne=10, nports=20)
    data, lens = X.gen_fuzz(5, 20000, 160, rules, pool)
    _, once, st1 = X.run_oracle(feats, data, lens, rules, stride=160)
    _, twice, _ = X.run_oracle(feats, data, lens, once, stride=160)
    f = make_filter(G, variant)
    f.load_rules(rules)
    f.comm_init(1, 0, G.Filter.comm_unique_id())
    f.run(data, lens, stride=160)
    local = gpu_values(f, G, rules)
    local_stats = f.stats()
    assert_same(np.zeros(0), local, local_stats, np.zeros(0), once, st1)
    f.comm_allreduce()
    assert_same(np.zeros(0), gpu_values(f, G, rules), f.stats(), np.zeros(0), once, st1)
    # a later classify: the view is local again, and counts the new packets
    f.run(data, lens, stride=160)
    after = gpu_values(f, G, rules)
    np.testing.assert_array_equal(after.v4_vals, twice.v4_vals)
    np.testing.assert_array_equal(after.ports, twice.ports)
    np.testing.assert_array_equal(f.stats(), 2 * st1)
    f.comm_allreduce()
    np.testing.assert_array_equal(gpu_values(f, G, rules).v6_vals, twice.v6_vals)
    # re-init (replaces the communicator and the reduction copies)
    f.comm_init(1, 0, G.Filter.comm_unique_id())
    f.comm_allreduce()
    np.testing.assert_array_equal(f.stats(), 2 * st1)
    f.close()
