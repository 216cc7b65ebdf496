#!/usr/bin/env python3
"""tools/phases.py — where a classify tile step spends its cycles (diagnostic).

Runs the headline setup once under build variant 4 (XFG_VARIANT=4: wave 0 of
every workgroup stamps s_memtime at the phase boundaries of the tile loop) and
prints the mean cycles per tile of each phase, next to the plain kernel time.
Optional scenario args as in tools/explore.py (rules:dst:port).
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import bench  # noqa: E402

PHASES = ["prefetch_wait+lds_write", "barrier1", "issue_next", "parse", "lookups",
          "counters+verdict+stats", "barrier2", "loop"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2-packets", type=int, default=24)
    ap.add_argument("--grid-per-cu", default="")
    ap.add_argument("scenarios", nargs="*", default=["1000000:500:250"])
    a = ap.parse_args()
    a.cpu_seconds, a.no_cpu = 0, True
    import xfgpu as G
    G.lib.xfg_diag_prof.restype = C.c_int
    G.lib.xfg_diag_prof.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_uint64), C.c_uint64]
    for sc in a.scenarios:
        r, d, p = (int(x) for x in sc.split(":")[:3])
        a.rules, a.dst_permille, a.port_permille = r, d, p
        f, (d_data, d_lens, d_verd), n, stride, lens, alg, _, _, _ = bench.setup(a, 0, 0)
        if a.grid_per_cu:
            os.environ["XFG_GRID_PER_CU"] = a.grid_per_cu
        plain = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, 5, lens_u16=True)
        os.environ["XFG_VARIANT"] = os.environ.get("PHASES_VARIANT", "4")
        buf = (C.c_uint64 * (8192 * 8))()
        G.lib.xfg_diag_prof(f.ctx, 0, buf, 8192 * 8)      # clear
        prof_ms = f.classify_timed(d_data.ptr, d_lens.ptr, n, stride, d_verd.ptr, 1, lens_u16=True)
        G.lib.xfg_diag_prof(f.ctx, 0, buf, 8192 * 8)
        os.environ.pop("XFG_VARIANT")
        os.environ.pop("XFG_GRID_PER_CU", None)
        v = np.frombuffer(buf, np.uint64).reshape(8192, 8).astype(np.float64)
        used = v.sum(1) > 0
        wg = int(used.sum())
        tiles_per_wg = (n / 256) / max(wg, 1)
        mean = v[used].mean(0) / tiles_per_wg
        tot = mean.sum()
        print(json.dumps({"scenario": sc, "kernel_ms": round(plain, 4), "profiled_ms": round(prof_ms, 4),
                          "workgroups": wg, "tiles_per_wg": round(tiles_per_wg, 2),
                          "cycles_per_tile": round(tot, 1),
                          "phases": {k: [round(x, 1), round(x / tot, 3)] for k, x in zip(PHASES, mean)}}),
              flush=True)
        f.close()


if __name__ == "__main__":
    main()
