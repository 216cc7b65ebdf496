#!/bin/bash
# Round 2, session 3: the GPU suite, smoke, the bench line and a rocprofv3
# kernel-trace summary of the bench's full-batch launches, on the final tree.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/s3_pytest_gpu.log" 2>&1 || exit $?
tail -1 "$OUT/s3_pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > "$OUT/s3_smoke.log" 2>&1 || exit $?
tail -1 "$OUT/s3_smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/s3_bench.json" 2> "$OUT/s3_bench.err" || exit $?
cat "$OUT/s3_bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/s3_prof" -o run -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --host-log2-packets 0 > "$OUT/s3_prof.log" 2>&1 || exit $?
find "$OUT/s3_prof" -name "*kernel_stats.csv" | head -1 | xargs cat
