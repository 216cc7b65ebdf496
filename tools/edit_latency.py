#!/usr/bin/env python3
"""tools/edit_latency.py — the cost of one rule edit on the quotient-index
path, C3's 1M IPv4 dst rules on one GPU: the wall time of
one `xdp-filter ip`-style edit (xfg_map_update of one key, or its delete)
plus the next classify of a small batch, against the same classify with no
edit; and the same edit made through xfg_map_update_batch, which marks the
index for a full rebuild at the next classify (the round-3 behaviour of
every edit).  One JSON line.  Reference: map_set_flags,
xdp-filter/xdp-filter.c:111-157 (one element per CPU)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import numpy as np  # noqa: E402
import xftools as X  # noqa: E402


def main():
    import xfgpu as G
    v4 = X.rand_keys(3, int(1_000_000 * 1.02) + 16, 4)
    keys, spare = v4[:1_000_000], v4[1_000_000:1_000_000 + 16]
    f = G.Filter(G.FEAT_ALL | G.FEAT_DENY, devices=[0], ipv4_capacity=1_100_000)
    f.update_batch(G.MAP_IPV4, keys, np.full(len(keys), 2, np.uint64))
    n = 1 << 16
    data, lens = X.gen_workload(5, 3, n, 64, v4=keys)
    d_data, d_lens, d_verd = f.alloc(data.nbytes), f.alloc(lens.nbytes), f.alloc(n)
    d_data.upload(data)
    d_lens.upload(lens)

    def classify():
        f.classify_timed(d_data.ptr, d_lens.ptr, n, 64, d_verd.ptr, 1)

    classify()
    assert f.last_path() == f.PATH_QT
    reps = 8

    def timed(edit):
        ts = []
        for i in range(reps):
            t0 = time.perf_counter()
            edit(i)
            classify()
            ts.append((time.perf_counter() - t0) * 1e3)
        return round(sorted(ts)[len(ts) // 2], 3)

    base = timed(lambda i: None)
    ins = timed(lambda i: f.update(G.MAP_IPV4, bytes(spare[i]), 2))
    dele = timed(lambda i: f.delete(G.MAP_IPV4, bytes(spare[i])))
    flg = timed(lambda i: f.update(G.MAP_IPV4, bytes(keys[i]), 4))   # live bit off: leaves the index
    reb = timed(lambda i: f.update_batch(G.MAP_IPV4, spare[i:i + 1], np.full(1, 2, np.uint64)))
    assert f.last_path() == f.PATH_QT
    print(json.dumps({"tool": "edit_latency", "rules_ipv4": len(keys), "batch": n,
                      "classify_only_ms": base, "insert_then_classify_ms": ins,
                      "delete_then_classify_ms": dele, "flag_change_then_classify_ms": flg,
                      "batch_edit_full_rebuild_then_classify_ms": reb,
                      "note": "median of 8; wall time of the edit call(s) and the next classify "
                              "(xfg_classify_timed, synchronous)"}), flush=True)
    f.close()


if __name__ == "__main__":
    main()
