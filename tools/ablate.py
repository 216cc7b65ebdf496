#!/usr/bin/env python3
"""tools/ablate.py — where does the classify kernel's time go?  (diagnostic)

Builds the bench.py C3 setup once, then times the kernel under the
XFG_ABLATE masks (see xfg_ctx.c:fill_kargs) in interleaved rounds in ONE
process (methodology rule: A/B in one process, report median and min):
  0  full kernel (production)
  2  no counter atomics
  1  every table treated as empty (parse only, no probes, no atomics)
  4  stage header windows + verdict store only
Outputs are wrong under any non-zero mask; only times matter.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "xdp-tools_amd", "python"))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--log2-packets", type=int, default=24)
    ap.add_argument("--rules", type=int, default=1_000_000)
    ap.add_argument("--masks", default="0,2,1,4")
    ap.add_argument("--envs", default="",
                    help="';'-separated variants, each 'K=V,K=V' (diagnostic env knobs), "
                         "timed with mask 0; e.g. 'XFG_MINW=5;XFG_GRID_PER_CU=4'")
    a = ap.parse_args()
    a.cpu_seconds, a.no_cpu = 0, True
    f, (d_data, d_lens, d_verd), n, stride, lens, alg, _, _, _ = bench.setup(a, 0, 0)
    variants = [("mask", int(m), {}) for m in a.masks.split(",") if m != ""]
    for v in a.envs.split(";"):
        if v.strip():
            kv = dict(x.split("=") for x in v.split(","))
            variants.append(("env", v, kv))
    res = {str(v[1]): [] for v in variants}
    knobs = {"XFG_ABLATE", "XFG_VARIANT", "XFG_GRID_PER_CU", "XFG_KERNEL"}
    base_env = {k: os.environ[k] for k in knobs if k in os.environ}   # e.g. XFG_VARIANT under rocprof
    for _ in range(a.rounds):
        for kind, key, kv in variants:
            for k in knobs:
                os.environ.pop(k, None)
            os.environ.update(base_env)
            if kind == "mask":
                os.environ["XFG_ABLATE"] = str(key)
            else:
                os.environ.update(kv)
            res[str(key)].append(f.classify_timed(d_data.ptr, d_lens.ptr, n, stride,
                                                  d_verd.ptr, a.iters, lens_u16=True))
    for k in knobs:
        os.environ.pop(k, None)
    masks = list(res)
    out = {}
    for m in masks:
        ts = sorted(res[m])
        out[str(m)] = {"median_ms": round(ts[len(ts) // 2], 4), "min_ms": round(ts[0], 4),
                       "GBps_alg": round(alg / (ts[len(ts) // 2] * 1e-3) / 1e9, 1)}
    print(json.dumps({"ablation": out, "packets": n, "alg_bytes": alg}))
    f.close()


if __name__ == "__main__":
    main()
