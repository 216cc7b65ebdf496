"""CPU tests of the parity oracle (tools/xftools.py + oracle/).

* the CPU restatement (oracle/xf_oracle.c) reproduces the committed golden
  regression fixture (tests/golden/make_golden.py; provenance there) —
  verdicts, every rule value, stats;
* the golden fixture agrees with the stated known answers (SURVEY.md
  Appendix A, xdp-filter/tests/test-xdp-filter.sh, test_basic.py);
  tests/test_kat_counters.py carries those rows' counters and stats too.
"""
import numpy as np
import pytest

import kat
import xftools as X
from conftest import golden_expected_ports, golden_rules

VARIANTS = [v for v, _ in X.VARIANTS]


def _check_against_golden(g, tag, variant, verdicts, after, stats):
    p = f"{tag}_{variant}_"
    base = golden_rules(g, f"{tag}_rules_")
    np.testing.assert_array_equal(verdicts, g[p + "verdicts"])
    np.testing.assert_array_equal(after.ports, golden_expected_ports(g, p, base))
    np.testing.assert_array_equal(after.v4_vals, g[p + "v4_vals"])
    np.testing.assert_array_equal(after.v6_vals, g[p + "v6_vals"])
    np.testing.assert_array_equal(after.eth_vals, g[p + "eth_vals"])
    np.testing.assert_array_equal(stats, g[p + "stats"])


@pytest.mark.parametrize("tag", ["kat", "fuzz"])
@pytest.mark.parametrize("variant", VARIANTS)
def test_restatement_reproduces_own_regression_fixture(golden, tag, variant):
    g = golden
    rules = golden_rules(g, f"{tag}_rules_")
    data, lens, stride = g[f"{tag}_data"], g[f"{tag}_lens"], int(g["stride"])
    v, after, st = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=stride)
    _check_against_golden(g, tag, variant, v, after, st)


def test_golden_meets_known_answers(golden):
    frames = kat.kat_frames()
    assert list(golden["kat_names"]) == [n for n, _, _ in frames]
    checked = 0
    for i, (name, _, exp) in enumerate(frames):
        for variant, want in exp.items():
            got = int(golden[f"kat_{variant}_verdicts"][i])
            assert got == want, f"{name} / {variant}: expected {want}, got {got}"
            checked += 1
    assert checked > 100


def test_golden_exercises_every_outcome(golden):
    """The fixture is only useful if it covers aborts, hits and misses of
    every map in every program family."""
    for variant in VARIANTS:
        v = golden[f"fuzz_{variant}_verdicts"]
        assert set(np.unique(v)) == {0, 1, 2}, variant
    base = golden_rules(golden, "fuzz_rules_")
    p = "fuzz_xdpfilt_dny_all_"
    assert (golden[p + "v4_vals"] != base.v4_vals).any()
    assert (golden[p + "v6_vals"] != base.v6_vals).any()
    assert (golden[p + "eth_vals"] != base.eth_vals).any()
    assert (golden_expected_ports(golden, p, base) != base.ports).any()


def test_oracle_stats_count_every_packet(golden):
    for variant in VARIANTS:
        st = golden[f"fuzz_{variant}_stats"]
        assert st[:, 0].sum() == len(golden["fuzz_lens"])
        assert st[:, 1].sum() == golden["fuzz_lens"].astype(np.uint64).sum()


def test_oracle_layouts_and_threads():
    """offsets layout, u16 lens and the per-CPU-style threaded run all give
    the same result as the plain run."""
    rules, pool = X.random_rules(9)
    data, lens = X.gen_fuzz(31, 40000, 160, rules, pool)
    f = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    v0, r0, s0 = X.run_oracle(f, data, lens, rules, stride=160)
    # shuffled placement through an offsets array
    perm = np.random.default_rng(1).permutation(len(lens))
    data2 = np.zeros_like(data)
    for j, i in enumerate(perm):
        data2[j * 160:(j + 1) * 160] = data[i * 160:(i + 1) * 160]
    offs = np.empty(len(lens), np.uint64)
    offs[perm] = np.arange(len(lens), dtype=np.uint64) * 160
    v1, r1, s1 = X.run_oracle(f, data2, lens, rules, offsets=offs)
    v2, r2, s2 = X.run_oracle(f, data, lens.astype(np.uint16), rules, stride=160)
    v3, r3, s3 = X.run_oracle(f, data, lens, rules, stride=160, nthreads=4)
    for v, r, s in ((v1, r1, s1), (v2, r2, s2), (v3, r3, s3)):
        np.testing.assert_array_equal(v, v0)
        np.testing.assert_array_equal(r.v4_vals, r0.v4_vals)
        np.testing.assert_array_equal(r.v6_vals, r0.v6_vals)
        np.testing.assert_array_equal(r.eth_vals, r0.eth_vals)
        np.testing.assert_array_equal(r.ports, r0.ports)
        np.testing.assert_array_equal(s, s0)
