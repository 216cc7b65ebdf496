"""Worker of tests/test_gpu_qt.py::test_qt_both_ipv4_directions_ipv6_in_loop
(a fresh process on the diagnostics library, XFG_LIB=diag): IPv4 rules on
both lookup directions (`xdp-filter ip -m src,dst`) beside IPv6 rules, C3
traffic without malformed frames.  With XFG_DIAG_MASK=2048 the quotient-index
kernel leaves its deferred packets unclassified (their verdict bytes are not
written), so a frame whose byte still holds the sentinel was deferred: every
IPv6 frame (but a 17th of a tile) must carry the oracle's verdict -- looked up in the kernel's loop
(xdpfilt_prog.h:152-165), not by the deferred whole-frame walk.  Without the
mask every verdict, rule value and stat equals the oracle's.
Usage: python gpu_defer_worker.py DIRS6 (dst|src|both); prints OK or raises."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402

SENTINEL = 0xEE


def main():
    dirs6 = sys.argv[1]
    import xftools as X
    import xfgpu as G
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    rng = np.random.default_rng(77)
    v4 = X.rand_keys(78, 20000, 4)
    v6 = X.rand_keys(79, 3000, 16)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 3, np.uint64)
    rules.v6_keys = v6
    f6 = {"dst": 2, "src": 1, "both": 3}[dirs6]
    rules.v6_vals = np.full(len(v6), f6, np.uint64) | (rng.integers(0, 50, len(v6)).astype(np.uint64) << 6)
    ports = np.array([53, 80], np.uint16)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    n, stride = 1 << 20, 64
    data, lens = X.gen_workload(80, 3, n, stride, v4=v4, v6=v6, ports=ports, bad_permille=0)
    fr = data.reshape(-1, stride)
    six = np.nonzero((fr[:, 12] == 0x86) & (fr[:, 13] == 0xdd))[0]
    assert len(six) > n // 20
    ip4 = np.nonzero((fr[:, 12] == 8) & (fr[:, 13] == 0))[0][::4]
    fr[ip4, 26:30] = v4[(np.arange(len(ip4)) * 7919) % len(v4)]       # ruled IPv4 sources
    srcs = six[::3]
    fr[srcs, 22:38] = v6[rng.integers(0, len(v6), len(srcs))]           # ruled IPv6 sources
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=stride, nthreads=8)
    assert len(np.unique(ov[six])) >= 2
    for mask in ("2048", "0"):
        os.environ["XFG_DIAG_MASK"] = mask
        # (an IPv6 table far from full: no bucket overflows, so no IPv6
        # miss is left to the canonical walk either)
        f = G.Filter(feats, devices=[0], ipv4_capacity=1 << 16, ipv6_capacity=1 << 17, qt_min_keys=1)
        f.load_rules(rules)
        d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
        d_data.upload(data)
        d_lens.upload(lens)
        d_v.upload(np.full(n, SENTINEL, np.uint8))
        f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_v.ptr, 1)
        assert f.last_path() == G.Filter.PATH_QT, f.last_path()
        v = d_v.download(np.zeros(n, np.uint8))
        if mask == "2048":
            # (by design a tile looks up at most 16 IPv6 frames in the loop:
            # a 17th IPv6 frame of a 64-frame tile is deferred -- with 10 %
            # IPv6 a tile or two in a million frames)
            tile = six // 64
            first = np.searchsorted(tile, tile)
            rank = np.arange(len(six)) - first
            six = six[rank < 16]
            bad = six[v[six] != ov[six]]
            print(f"IPv6 frames {len(six)}, deferred or wrong {len(bad)}; all frames left "
                  f"unclassified {int((v == SENTINEL).sum())}", flush=True)
            assert len(bad) == 0, f"{len(bad)} of {len(six)} IPv6 frames deferred or wrong: {bad[:8]}"
        else:
            np.testing.assert_array_equal(v, ov)
            r = rules.prepared()
            np.testing.assert_array_equal(f.values_of(G.MAP_IPV4, r.v4_keys), orules.v4_vals)
            np.testing.assert_array_equal(f.values_of(G.MAP_IPV6, r.v6_keys), orules.v6_vals)
            np.testing.assert_array_equal(f.stats(), ost)
        f.close()
    os.environ.pop("XFG_DIAG_MASK", None)
    print("OK")


if __name__ == "__main__":
    main()
