#!/usr/bin/env python3
"""tools/explore.py — classify time across workload shapes and measurement
knobs (diagnostic; loads the diagnostics build of the library).

Each scenario is 'rules:dst_permille:port_permille[:K=V,...]'; the workload is
bench.py's C3 generator with those parameters.  Knobs (read by the
diagnostics build only): XFG_KERNEL=general (the general kernel instead of
the pipelined one), XFG_COUNT=atomic (no hit log), XFG_EMPTY=1 (tables
treated as empty: stream + parse only), XFG_GRID_PER_CU=n, XFG_DIAG_MASK=m
(IPv4-key kernel: 1 no counter bumps, 2 no bucket lines, 4 no Bloom loads, 8 no
verdict stores; results wrong).
Prints one JSON line per scenario (median/min ms over rounds).
"""
import argparse
import json
import os
import sys

os.environ.setdefault("XFG_LIB", "diag")   # or a library file (A/B runs)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import bench  # noqa: E402

KNOBS = ("XFG_KERNEL", "XFG_COUNT", "XFG_EMPTY", "XFG_GRID_PER_CU", "XFG_DIAG_MASK", "XFG_QT", "XFG_LOG_PEND",
         "XFG_BLOOM_LDS", "XFG_CW", "XFG_CW_LOG_MIN", "XFG_QT_DYN_MIN")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--log2-packets", type=int, default=24)
    ap.add_argument("scenarios", nargs="+")
    a = ap.parse_args()
    a.cpu_seconds, a.no_cpu = 0, True
    groups = {}
    for sc in a.scenarios:
        parts = sc.split(":")
        key = (int(parts[0]), int(parts[1]), int(parts[2]))
        env = dict(x.split("=") for x in parts[3].split(",")) if len(parts) > 3 and parts[3] else {}
        groups.setdefault(key, []).append((sc, env))
    for (rules, dst, port), items in groups.items():
        a.rules, a.dst_permille, a.port_permille = rules, dst, port
        f, (d_data, d_lens, d_verd), n, stride, lens, alg, _, _, _ = bench.setup(a, 0, 0)
        res = {sc: [] for sc, _ in items}
        for _ in range(a.rounds):
            for sc, env in items:
                for k in KNOBS:
                    os.environ.pop(k, None)
                os.environ.update(env)
                res[sc].append(f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr,
                                                a.iters, lens_u16=True))
        for k in KNOBS:
            os.environ.pop(k, None)
        for sc, ts in res.items():
            ts = sorted(ts)
            print(json.dumps({"scenario": sc, "median_ms": round(ts[len(ts) // 2], 4),
                              "min_ms": round(ts[0], 4),
                              "GBps_alg": round(alg / (ts[len(ts) // 2] * 1e-3) / 1e9, 1)}),
                  flush=True)
        f.close()


if __name__ == "__main__":
    main()
