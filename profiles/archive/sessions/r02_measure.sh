#!/bin/bash
# Round-2 measurement session on the GPU box: the bench line, a rocprofv3
# kernel-trace summary of the bench's full-batch launches only (no host-path
# or CPU legs), and the PMC traffic passes of the classify kernels, all at
# the bench's batch size (2^26 frames).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py > "$OUT/bench_r02.json" 2> "$OUT/bench_r02.err" || exit $?
cat "$OUT/bench_r02.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o run -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --host-log2-packets 0 > "$OUT/prof_bench.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
KNAME=pipe4 bash tools/pmc.sh c3p4 "--log2-packets 26 1000000:500:250" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum,TCC_EA0_WRREQ_sum" || exit $?
python3 tools/pmc_summary.py --kernel log_count "$OUT"/pmc_c3p4_* > "$OUT/pmc_c3lc.json"; cat "$OUT/pmc_c3lc.json"
