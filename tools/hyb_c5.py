#!/usr/bin/env python3
"""tools/hyb_c5.py — C5 end to end from a registered buffer under several
host-path settings in one process (diagnostic; the diagnostics library reads
XFG_HYB_ZLOG2 / XFG_HYB_ST at each call): zero copy alone (Z 0) against the
hybrid rounds of host_run_hyb (a zero-copy chunk of 2^Z packets, then S
staged chunks of 2^18 header windows).  C5 as tools/bench_configs.py builds
it (15M IPv4 + 1M IPv6 dst rules, 1024 dst ports, 2^23 frames of 1514 B at
a 1536 B stride).  Usage: XFG_LIB=diag python3 tools/hyb_c5.py Z:S ..."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))
os.environ.setdefault("XFG_LIB", "diag")

import numpy as np  # noqa: E402


def main():
    import xftools as X
    import xfgpu as G
    n, stride, n4, n6, nports = 1 << 23, 1536, 15_000_000, 1_000_000, 1024
    v4 = X.rand_keys(5, int(n4 * 1.02) + 16, 4)[:n4]
    v6 = X.rand_keys(105, int(n6 * 1.02) + 16, 16)[:n6]
    ports = (np.arange(nports, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    t0 = time.perf_counter()
    data, lens = X.gen_workload(5, 5, n, stride, v4=v4, v6=v6, ports=ports)
    print(f"workload {time.perf_counter() - t0:.1f} s", flush=True)
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[0], ipv4_capacity=n4, ipv6_capacity=n6)
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), 2, np.uint64))
    f.update_batch(G.MAP_IPV6, v6, np.full(len(v6), 2, np.uint64))
    pk = np.array([X.port_key(int(p)) for p in ports], "<u4").view(np.uint8)
    f.update_batch(G.MAP_PORTS, pk, np.full(len(ports), 2 | 4 | 8, np.uint64))
    f.host_register(data)
    print(f"rules and registration {time.perf_counter() - t0:.1f} s", flush=True)
    ref = None
    for rnd in range(2):
        for zs in sys.argv[1:]:
            z, s = zs.split(":")
            os.environ["XFG_HYB_ZLOG2"], os.environ["XFG_HYB_ST"] = z, s
            v = f.classify_host(data, lens, stride=stride)   # (warm)
            if ref is None:
                ref = v
            assert np.array_equal(v, ref), zs
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                f.classify_host(data, lens, stride=stride)
            el = (time.perf_counter() - t0) / reps
            print(json.dumps({"round": rnd, "Z": int(z), "S": int(s), "ms": round(el * 1e3, 2),
                              "Mpps": round(n / el / 1e6, 1), "host_threads": int(G.lib.xfg_host_threads())}),
                  flush=True)
    f.host_unregister(data)
    f.close()


if __name__ == "__main__":
    main()
