#!/usr/bin/env python3
"""tools/qt_phases.py — where a quotient-index launch spends its time, per
workgroup (diagnostic; diagnostics library, XFG_TSTAMP): the kernel writes
32 wall-clock stamps a workgroup (xfg_pipeq.hip QT_STAMP: entry, set-up
done, each wave's loop done, each wave's deferred walk done, the partitions
moved, the end) into a device buffer whose address the library reads from
XFG_TSTAMP; this prints, over the workgroups, how long each phase took.
Workloads as tools/bench_configs.py builds them (C3: 1M IPv4 dst rules + 16
ports, 64 B frames; C4: the same rules, IMIX at a 1536 B stride).
Usage: XFG_LIB=diag python3 tools/qt_phases.py c3|c4 LOG2 [XFG_ENV=VALUE ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))
os.environ.setdefault("XFG_LIB", "diag")

import numpy as np  # noqa: E402

TICK_US = 0.01   # the wall clock: 100 MHz


def main():
    import xftools as X
    import xfgpu as G
    name, lg = sys.argv[1], int(sys.argv[2])
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    kind = {"c3": 3, "c4": 4}[name]
    n, stride, n4 = 1 << lg, 64 if kind == 3 else 1536, 1_000_000
    v4 = X.rand_keys(kind, int(n4 * 1.02) + 16, 4)[:n4]
    ports = (np.arange(16, dtype=np.uint32) * 61 + 53).astype(np.uint16)
    data, lens = X.gen_workload(kind, kind, n, stride, v4=v4, ports=ports)
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[0], ipv4_capacity=n4, ipv6_capacity=1024)
    f.update_batch(G.MAP_IPV4, v4, np.full(len(v4), 2, np.uint64))
    pk = np.array([X.port_key(int(p)) for p in ports], "<u4").view(np.uint8)
    f.update_batch(G.MAP_PORTS, pk, np.full(len(ports), 2 | 4 | 8, np.uint64))
    d_data, d_lens, d_v = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(lens)
    NWG, SL = 2048, 32
    d_ts = f.alloc(NWG * SL * 8)
    ms = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_v.ptr, 20)
    rows = []
    for rep in range(3):
        d_ts.upload(np.zeros(NWG * SL, np.uint64))
        os.environ["XFG_TSTAMP"] = hex(d_ts.ptr)
        f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_v.ptr, 1)
        os.environ.pop("XFG_TSTAMP")
        ts = d_ts.download(np.zeros(NWG * SL, np.uint64)).reshape(NWG, SL).astype(np.int64)
        ts = ts[:int(np.nonzero(ts[:, 0])[0].max()) + 1]
        t0 = ts[:, 0].min()
        rel = (ts - t0) * TICK_US
        rel[ts == 0] = np.nan
        loop = rel[:, 2:10]
        dfr = rel[:, 11:19]
        ph = {
            "entry": rel[:, 0],
            "setup": rel[:, 1] - rel[:, 0],
            "loop_first_wave": np.nanmin(loop, 1) - rel[:, 1],
            "loop_last_wave": np.nanmax(loop, 1) - rel[:, 1],
            "count_wave": rel[:, 10] - rel[:, 1],
            "defer_walk": np.nanmax(dfr - loop, 1),
            "to_barrier": rel[:, 20] - np.nanmax(dfr, 1),
            "fold": np.nanmax(rel[:, 22:30] - dfr, 1),
            "barrier1_wait": rel[:, 30] - np.nanmax(rel[:, 22:30], 1),
            "partition_flush": rel[:, 20] - rel[:, 30],
            "flush": rel[:, 21] - rel[:, 20],
            "end": rel[:, 21],
        }
        out = {"config": name, "packets": n, "rep": rep, "workgroups": int(len(ts)),
               "kernel_ms_events_avg20": round(ms, 4), "path": f.last_path(),
               "span_us": round(float(np.nanmax(rel[:, 21])), 1)}
        # (workgroup i on XCD i % 8: the loop's last wave and the end, by XCD)
        wg = np.arange(len(ts))
        out["loop_last_by_xcd"] = [round(float(np.nanmedian(ph["loop_last_wave"][wg % 8 == x])), 1) for x in range(8)]
        out["end_by_xcd"] = [round(float(np.nanmedian(ph["end"][wg % 8 == x])), 1) for x in range(8)]
        out["end_slowest16_wg"] = [int(i) for i in np.argsort(-ph["end"])[:16]]
        for k, v in ph.items():
            v = v[~np.isnan(v)]
            if len(v):
                out[k] = [round(float(np.min(v)), 1), round(float(np.median(v)), 1), round(float(np.max(v)), 1)]
        print(json.dumps(out), flush=True)
        rows.append(out)
    f.close()


if __name__ == "__main__":
    main()
