#!/bin/bash
# FETCH_SIZE calibration on the GPU box (see pmc_calib.hip): one rocprofv3
# --pmc pass per pattern; prints {pattern, requested bytes, FETCH_SIZE bytes,
# ratio}.  Build first (here): hipcc -O3 --offload-arch=gfx950 -o
# tools/calib/pmc_calib tools/calib/pmc_calib.hip
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out/calib"; mkdir -p "$OUT"
BIN="$GRAFT_REPO_ROOT/tools/calib/pmc_calib"
cd /tmp && export TMPDIR=/tmp
for p in stream lines words; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
     -d "$OUT/$p" -o run -- "$BIN" $p > "$OUT/$p.log" 2>&1 || { echo "$p failed"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, statistics
out = sys.argv[1]
for p in ("stream", "lines", "words"):
    req = json.loads([l for l in open(f"{out}/{p}.log") if l.startswith("{")][-1])["requested_bytes_per_launch"]
    vals = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/{p}/**/run_counter_collection.csv", recursive=True)
            for r in csv.DictReader(open(f)) if r["Counter_Name"] == "FETCH_SIZE"]
    kb = statistics.median(vals)
    print(json.dumps({"pattern": p, "requested_bytes": req, "fetch_size_bytes": kb * 1024,
                      "fetch_over_requested": round(kb * 1024 / req, 3)}))
PY
