#!/usr/bin/env python3
"""tools/split_debug.py — diagnostics: the split IPv4-key classify
(xfg_parse4 + xfg_look4) against the one-kernel pipeline (XFG_KERNEL=pipe4)
and the CPU restatement on one workload; prints where verdicts differ
(packet index, tile, lane, ethertype, length) to locate a divergence."""
import os
import sys

os.environ["XFG_LIB"] = "diag"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402
import xftools as X  # noqa: E402
import xfgpu as G  # noqa: E402


def main():
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    log2n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    variant = "xdpfilt_dny_ip" if kind == 2 else "xdpfilt_dny_all"
    n = 1 << log2n
    v4 = X.rand_keys(kind, 100000, 4)
    ports = np.arange(16, dtype=np.uint16) * 7 + 20
    data, lens = X.gen_workload(kind, kind, n, 64, v4=v4, ports=ports)
    rules = X.RuleSet()
    rules.v4_keys = v4
    rules.v4_vals = np.full(len(v4), 2, np.uint64)
    for p in ports:
        rules.ports[X.port_key(int(p))] = 2 | 4 | 8
    ov, _, ost = X.run_oracle(X.VARIANT_FEATURES[variant], data, lens, rules, stride=64, nthreads=8)
    res = {}
    for mode in ("split", "pipe4"):
        os.environ.pop("XFG_KERNEL", None)
        if mode == "pipe4":
            os.environ["XFG_KERNEL"] = "pipe4"
        f = G.Filter(X.VARIANT_FEATURES[variant], ndev=1, ipv4_capacity=len(v4))
        f.load_rules(rules)
        res[mode] = (f.run(data, lens, stride=64), f.stats())
        f.close()
    os.environ.pop("XFG_KERNEL", None)
    for mode, (v, st) in res.items():
        bad = np.nonzero(v != ov)[0]
        print(f"{mode}: {len(bad)} verdict mismatches; stats equal: {np.array_equal(st, ost)}")
        for i in bad[:40]:
            p = data[i * 64:(i + 1) * 64]
            et = (int(p[12]) << 8) | int(p[13])
            print(f"  i={i} tile={i // 64} lane={i % 64} et={et:#06x} len={int(lens[i])} "
                  f"b14={int(p[14]):#04x} proto={int(p[23])} dst={bytes(p[30:34]).hex()} "
                  f"got={int(v[i])} want={int(ov[i])}")
        if len(bad):
            t = bad // 64
            print(f"  tiles hit: {len(np.unique(t))}, lanes: {np.bincount(bad % 64, minlength=64).tolist()}")
            print(f"  first/last tile {t.min()} {t.max()}; got values {np.bincount(v[bad]).tolist()}")


if __name__ == "__main__":
    main()
