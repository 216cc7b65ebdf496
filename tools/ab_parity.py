#!/usr/bin/env python3
"""tools/ab_parity.py — bit-exact check of an A/B variant library (XFG_LIB)
against the CPU restatement on a C3-shaped batch (diagnostic: the variants
of tools/abbuild.sh are not what pytest loads).  Usage:
XFG_LIB=tools/abl/NAME.so python3 tools/ab_parity.py [--log2-packets 22] [--src-dst]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import xftools as X  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2-packets", type=int, default=22)
    ap.add_argument("--src-dst", action="store_true", help="every rule src|dst")
    ap.add_argument("--hot", type=int, default=0, help="every dst hit on one of N rules")
    ap.add_argument("--reps", type=int, default=1,
                    help="classify the batch N times back to back (the count wave counts each "
                         "launch's log in the next): counters and stats N times the oracle's")
    a = ap.parse_args()
    import xfgpu as G
    n = 1 << a.log2_packets
    v4 = X.rand_keys(3, int(1_000_000 * 1.02) + 16, 4)[:1_000_000]
    ports = (np.arange(16, dtype=np.uint16) * 1031 + 53).astype(np.uint16)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 3 if a.src_dst else 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    data, lens = X.gen_workload(3, 3, n, 64, v4=v4[:a.hot] if a.hot else v4, ports=ports)
    if a.src_dst:   # a quarter of the IPv4 frames get a ruled source too
        d = data.reshape(-1, 64)
        ip4 = np.nonzero((d[:, 12] == 8) & (d[:, 13] == 0))[0][::4]
        d[ip4, 26:30] = v4[np.arange(len(ip4)) * 7919 % len(v4)]
    feats = X.VARIANT_FEATURES["xdpfilt_dny_all"]
    ov, orules, ost = X.run_oracle(feats, data, lens, rules, stride=64, nthreads=16)
    f = G.Filter(feats, ndev=1, ipv4_capacity=1_000_000)
    f.load_rules(rules)
    if a.reps == 1:
        v = f.run(data, lens.astype(np.uint16), stride=64)
    else:
        l16 = lens.astype(np.uint16)
        d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(l16.nbytes), f.alloc(n)
        d_data.upload(data)
        d_lens.upload(l16)
        f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_v.ptr, a.reps, lens_u16=True)
        v = d_v.download(np.zeros(n, np.uint8))
        six, r = np.uint64(6), np.uint64(a.reps)
        pre = rules.v4_vals >> six
        orules.v4_vals = ((pre + ((orules.v4_vals >> six) - pre) * r) << six) | (rules.v4_vals & np.uint64(63))
        pp = rules.ports >> six
        orules.ports = ((pp + ((orules.ports >> six) - pp) * r) << six) | (rules.ports & np.uint64(63))
        ost = ost * a.reps
    path = f.last_path()
    from test_gpu import gpu_values
    got = gpu_values(f, G, rules)
    st = f.stats()
    ok = (np.array_equal(v, ov) and np.array_equal(got.v4_vals, orules.v4_vals)
          and np.array_equal(got.ports, orules.ports) and np.array_equal(st, ost))
    print(f"ab_parity lib={os.environ.get('XFG_LIB')} path={path} n={n} hot={a.hot} reps={a.reps} "
          f"verdicts={'ok' if np.array_equal(v, ov) else 'DIFF'} "
          f"v4={'ok' if np.array_equal(got.v4_vals, orules.v4_vals) else 'DIFF'} "
          f"stats={'ok' if np.array_equal(st, ost) else 'DIFF'} -> {'PASS' if ok else 'FAIL'}",
          flush=True)
    f.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
