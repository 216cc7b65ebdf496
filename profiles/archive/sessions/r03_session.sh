#!/bin/bash
# Round-3 GPU session: selected GPU tests (or all), then the bench (and an
# optional rocprofv3 kernel-trace summary of it).  Each GPU step has its own
# time limit; the first failure ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-s}
export PYTHONUNBUFFERED=1
if [ -n "$MB" ]; then
  for m in $MB; do
    timeout -k 10 300 ./tools/$m > "$OUT/${m}_$TAG.log" 2>&1
    rc=$?; echo "$m rc=$rc"; cat "$OUT/${m}_$TAG.log" | cut -c1-200
    [ $rc -eq 0 ] || exit $rc
  done
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu $TESTS \
    > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" "$OUT/pytest_$TAG.log" | tail -3
  [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" "$OUT/pytest_$TAG.log" | head -30; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py $BENCH > "$OUT/bench_$TAG.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      -d "$OUT/prof_$TAG" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --host-log2-packets 0) > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "prof rc=$rc"
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -8
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
