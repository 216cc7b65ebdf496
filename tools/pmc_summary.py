#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs of the classify kernel (per dispatch).

Usage: pmc_summary.py [--kernel SUBSTR] gpurun_out/pmc_<tag>_*  -> one line per counter with
the per-dispatch value, plus derived HBM bytes per launch (corrected as
MI355X_MICROARCH.md prescribes: FETCH_SIZE is KB and reads exactly half the
bytes of a wide coalesced stream on gfx950; TCC_EA0_RDREQ_128B x 128 B is
the request-count view of the same traffic)."""
import collections
import csv
import glob
import json
import sys


def main(dirs, kname="pipeline"):
    vals = collections.defaultdict(list)
    dur = []
    for d in dirs:
        for f in glob.glob(f"{d}/run_counter_collection.csv"):
            per = collections.defaultdict(float)
            for r in csv.DictReader(open(f)):
                if kname not in r["Kernel_Name"]:
                    continue
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (_, c), v in per.items():
                vals[c].append(v)
        for f in glob.glob(f"{d}/run_kernel_trace.csv"):
            for r in csv.DictReader(open(f)):
                if kname in r["Kernel_Name"]:
                    dur.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {c: sorted(v)[len(v) // 2] for c, v in vals.items()}
    if dur:
        out["kernel_ns_median_profiled"] = sorted(dur)[len(dur) // 2]
    if "TCC_EA0_RDREQ_128B_sum" in out:
        out["hbm_read_bytes_rdreq"] = out["TCC_EA0_RDREQ_128B_sum"] * 128 + \
            out.get("TCC_EA0_RDREQ_64B_sum", 0) * 64
    if "FETCH_SIZE" in out:
        out["fetch_bytes_x2"] = out["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in out:
        out["write_bytes"] = out["WRITE_SIZE"] * 1024
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    args = sys.argv[1:]
    k = "pipeline"
    if args and args[0] == "--kernel":
        k, args = args[1], args[2:]
    main(args, k)
