"""The CPU baseline's restatement (bench.py cpu_baseline): the same
program with a hash index probed once per CHECK_MAP -- the cost model of the
reference's BPF_MAP_TYPE_PERCPU_HASH lookups (xdp-filter/xdpfilt_prog.h:
56-64) -- and per-thread counters summed at the end, as per-CPU maps are
(xdp-filter/xdp-filter.c:93-103).  It must give exactly what the checker's
binary-search index gives, on one thread and on several.  Also the C3
workload generator's mix, which every GPU config test and
the bench rely on."""
import numpy as np
import pytest

import xftools as X
from conftest import golden_rules

VARIANTS = [v for v, _ in X.VARIANTS]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("threads", [1, 3])
def test_hashed_index_equals_checker(golden, variant, threads):
    g = golden
    rules = golden_rules(g, "fuzz_rules_")
    data, lens, stride = g["fuzz_data"], g["fuzz_lens"], int(g["stride"])
    feats = X.VARIANT_FEATURES[variant]
    v0, a0, s0 = X.run_oracle(feats, data, lens, rules, stride=stride)
    v1, a1, s1 = X.run_oracle(feats, data, lens, rules, stride=stride, nthreads=threads,
                              maps=X.OracleMaps(rules, hashed=True))
    np.testing.assert_array_equal(v1, v0)
    np.testing.assert_array_equal(s1, s0)
    for f in ("ports", "v4_vals", "v6_vals", "eth_vals"):
        np.testing.assert_array_equal(getattr(a1, f), getattr(a0, f), err_msg=f)


def test_hashed_index_duplicate_keys_first_wins():
    rules = X.RuleSet()
    k = np.array([[10, 0, 0, 1], [10, 0, 0, 2], [10, 0, 0, 1]], np.uint8)
    rules.v4_keys = k
    rules.v4_vals = np.array([2, 2, 2], np.uint64)
    data, lens = X.gen_workload(5, 3, 2000, 64, v4=k, dst_permille=900)
    feats = X.VARIANT_FEATURES["xdpfilt_dny_ip"]
    v0, a0, _ = X.run_oracle(feats, data, lens, rules, stride=64)
    v1, a1, _ = X.run_oracle(feats, data, lens, rules, stride=64,
                             maps=X.OracleMaps(rules, hashed=True))
    np.testing.assert_array_equal(v1, v0)
    np.testing.assert_array_equal(a1.v4_vals, a0.v4_vals)
    assert a0.v4_vals[2] == 2          # the duplicate never matches


def test_workload_generator_mix():
    """C3's traffic: 80 % IPv4/UDP, 10 % IPv4/TCP, 10 % IPv6/UDP,
    ~1 % malformed, 50 % of IPv4 destinations drawn from the rule set;
    deterministic in its seed."""
    n = 100000
    v4 = X.rand_keys(1, 1000, 4)
    data, lens = X.gen_workload(3, 3, n, 64, v4=v4, bad_permille=10)
    d = data.reshape(n, 64)
    et = (d[:, 12].astype(int) << 8) | d[:, 13]
    good = lens >= 62
    assert 0.78 < ((et == 0x0800) & (d[:, 23] == 17) & good).mean() < 0.81
    assert 0.08 < ((et == 0x0800) & (d[:, 23] == 6) & good).mean() < 0.11
    assert 0.08 < ((et == 0x86DD) & good).mean() < 0.11
    assert 0.003 < (lens < 62).mean() < 0.02
    dst = np.ascontiguousarray(d[:, 30:34]).view("<u4").reshape(-1)
    ip4 = (et == 0x0800) & good
    assert 0.47 < np.isin(dst[ip4], v4.view("<u4").reshape(-1)).mean() < 0.53
    data2, lens2 = X.gen_workload(3, 3, 1000, 64, v4=v4)
    np.testing.assert_array_equal(data2, data[:1000 * 64])
    np.testing.assert_array_equal(lens2, lens[:1000])
