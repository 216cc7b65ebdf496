#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (rc >= 2 for pytest,
# non-zero otherwise) ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
TAG=${1:-r01}
STEPS=${STEPS:-all}
rc=0
if [[ $STEPS == all || $STEPS == *test* ]]; then
  timeout -k 10 1200 python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > "$OUT/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu_$TAG.log"
  [ $rc -le 1 ] || exit $rc
fi
if [[ $STEPS == all || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == all || $STEPS == *bench* ]]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench_$TAG.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == all || $STEPS == *prof* ]]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
      -d "$OUT/prof_$TAG" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu) > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "prof rc=$rc"; tail -3 "$OUT/prof_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
