"""The known-answer corpus (tests/kat.py) as complete expectations: for every
program and every row that states a verdict for it, the verdict, the counter
the verdict bumps (kat.HIT; CHECK_MAP, xdp-filter/xdpfilt_prog.h:56-64) and
the per-action stats (xdp_stats_record_action,
headers/xdp/xdp_stats_kern.h:29-48) -- derived from the rows alone, not from
any implementation.  Checked against the CPU restatement here and against
the HIP path on the GPU (-m gpu).

Also the capacity boundary of xdp-filter/tests/test_slow.py:55-103: at the
reference's map size (10,000 entries), the address whose insert fails must
not match.  (The reference's own run inserts 257 addresses and so never
reaches the boundary; here it is reached.)
"""
import errno

import numpy as np
import pytest

import kat
import pktbuild as P
import xftools as X

VARIANTS = [v for v, _ in X.VARIANTS]
HIT_VERDICT = {"dny": 2, "alw": 1}   # VERDICT_HIT: PASS under deny, DROP under allow
STRIDE = 256


def corpus(variant):
    """(data, lens, rules, expected verdicts, expected rules after, stats)."""
    rows = [(n, fr, exp[variant]) for n, fr, exp in kat.kat_frames() if variant in exp]
    rules = kat.kat_rules()
    after = rules.prepared().copy()
    n = len(rows)
    data = np.zeros(n * STRIDE, np.uint8)
    lens = np.zeros(n, np.uint32)
    verd = np.zeros(n, np.uint8)
    stats = np.zeros((5, 2), np.uint64)
    hitv = HIT_VERDICT[variant.split("_")[1]]
    for i, (name, fr, want) in enumerate(rows):
        assert len(fr) <= STRIDE
        data[i * STRIDE:i * STRIDE + len(fr)] = np.frombuffer(fr, np.uint8)
        lens[i] = len(fr)
        verd[i] = want
        stats[want, 0] += 1
        stats[want, 1] += len(fr)
        if want != hitv:
            continue
        kind, key = kat.HIT[name]   # every HIT verdict names its rule
        if kind == "port":
            after.ports[X.port_key(key)] += 1 << 6
        else:
            keys, vals, kb = {"v4": (after.v4_keys, after.v4_vals, P.ip4),
                              "v6": (after.v6_keys, after.v6_vals, P.ip6),
                              "eth": (after.eth_keys, after.eth_vals, P.mac)}[kind]
            idx = np.nonzero((keys == np.frombuffer(kb(key), np.uint8)).all(axis=1))[0]
            assert len(idx) == 1, (name, key)
            vals[idx[0]] += 1 << 6
    return data, lens, rules, verd, after, stats


def test_every_hit_names_its_rule_and_source():
    frames = kat.kat_frames()
    assert len(kat.SOURCE) == len(frames)
    cited = [n for n in kat.SOURCE if kat.SOURCE[n].startswith("xdp-filter/tests/")]
    assert len(cited) >= 35
    for name, _, exp in frames:
        for v, want in exp.items():
            if want == HIT_VERDICT[v.split("_")[1]]:
                assert name in kat.HIT, name


@pytest.mark.parametrize("variant", VARIANTS)
def test_kat_counters_on_restatement(variant):
    data, lens, rules, verd, after, stats = corpus(variant)
    v, got, st = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=STRIDE)
    np.testing.assert_array_equal(v, verd)
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        np.testing.assert_array_equal(getattr(got, fld), getattr(after, fld), err_msg=fld)
    np.testing.assert_array_equal(st, stats)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
def test_kat_counters_on_gpu(variant):
    import xfgpu as G
    from test_gpu import gpu_values, make_filter
    data, lens, rules, verd, after, stats = corpus(variant)
    f = make_filter(G, variant)
    f.load_rules(rules)
    v = f.run(data, lens, stride=STRIDE)
    np.testing.assert_array_equal(v, verd)
    got = gpu_values(f, G, rules)
    for fld in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        np.testing.assert_array_equal(getattr(got, fld), getattr(after, fld), err_msg=fld)
    np.testing.assert_array_equal(f.stats(), stats)
    f.close()


def _capacity_boundary(G, make):
    """Fill a 10,000-entry IPv4 map with dst rules spread over the address
    space (test_slow.py:35-41's generator, carried to the boundary); return
    (filter, an inserted address, the address whose insert failed)."""
    f = make()
    step = (1 << 32) // 10007
    addrs = [(i * step).to_bytes(4, "big") for i in range(10001)]
    for a in addrs[:10000]:
        f.update(G.MAP_IPV4, a, 2)
    with pytest.raises(OSError) as e:
        f.update(G.MAP_IPV4, addrs[10000], 2)
    assert e.value.errno == errno.E2BIG
    return f, addrs[5000], addrs[10000]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["xdpfilt_alw_ip", "xdpfilt_dny_ip"])
def test_capacity_boundary_address_does_not_match(variant):
    import ipaddress
    import xfgpu as G
    from test_gpu import make_filter
    f, inside, missing = _capacity_boundary(G, lambda: make_filter(G, variant))
    frames = [P.eth() + P.ipv4("192.0.2.1", str(ipaddress.IPv4Address(a)), 1,
                               payload=P.icmp4_echo()) for a in (inside, missing)]
    data = np.zeros(2 * 128, np.uint8)
    lens = np.array([len(x) for x in frames], np.uint32)
    for i, fr in enumerate(frames):
        data[i * 128:i * 128 + len(fr)] = np.frombuffer(fr, np.uint8)
    v = f.run(data, lens, stride=128)
    hit, miss = (1, 2) if "alw" in variant else (2, 1)
    assert list(v) == [hit, miss]
    vals, present = f.lookup_batch(G.MAP_IPV4, np.frombuffer(inside + missing, np.uint8))
    assert list(present) == [1, 0]
    assert int(vals[0].sum()) == 2 | (1 << 6)   # the inserted rule counted its packet
    f.close()
