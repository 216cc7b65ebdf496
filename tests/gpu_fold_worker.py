"""Worker of tests/test_gpu_qt.py::test_qt_counts_folded_before_32_bits
(a fresh process: the diagnostics library, XFG_LIB=diag, with
XFG_QT_FOLD_AT in the environment so that the 32-bit QT-order counts are
folded every few launches instead of every 2^32 packets): the same batch
classified `reps` times through the quotient index, with and without the
hit log (as C3 and C5 count), the folds queued between launches; every
rule's value and the stats must be the oracle's one-pass figures `reps`
times over (xdp-filter/xdpfilt_prog.h:56-64: each hit adds 1 << 6).
Usage: python gpu_fold_worker.py REPS; prints OK or raises."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402


def main():
    reps = int(sys.argv[1])
    import xftools as X
    import xfgpu as G
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    rng = np.random.default_rng(5)
    v4 = X.rand_keys(5, 30000, 4)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64) | (rng.integers(0, 50, len(v4)).astype(np.uint64) << 6)
    ports = np.array([53, 80], np.uint16)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    for n in (1 << 16, 1 << 22):   # (2^21 QT slots: below twice them no log, atomics; at twice: the log)
        data, lens = X.gen_workload(7, 3, n, 64, v4=v4, ports=ports)
        ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64)
        f = G.Filter(feats, devices=[0], ipv4_capacity=1 << 16, qt_min_keys=1)
        f.load_rules(rules)
        d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
        d_data.upload(data)
        d_lens.upload(lens)
        f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_v.ptr, reps)
        assert f.last_path() == G.Filter.PATH_QT, f.last_path()
        np.testing.assert_array_equal(d_v.download(np.zeros(n, np.uint8)), ov)
        six = np.uint64(6)
        pre = rules.v4_vals >> six
        want = ((pre + ((orules.v4_vals >> six) - pre) * np.uint64(reps)) << six) | (rules.v4_vals & np.uint64(63))
        got = f.values_of(G.MAP_IPV4, rules.prepared().v4_keys)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(f.stats(), ost * reps)
        f.close()
    print("OK")


if __name__ == "__main__":
    main()
