#!/bin/bash
# Round-4 same-box A/B session: optional bench line, then explore.py timings of
# each variant library in tools/abl/ (names in $VARIANTS), interleaved over
# $ROUNDS rounds.  Each GPU step has its own time limit; the first failure
# ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${TAG:-ab}
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > "$OUT/pytest_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" "$OUT/pytest_$TAG.log" | tail -3
  [ $rc -eq 0 ] || { grep -E "^E |Error|FAILED" "$OUT/pytest_$TAG.log" | head -30; exit $rc; }
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py $BENCH > "$OUT/bench_$TAG.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 2500 "$OUT/bench_$TAG.log"; echo
  [ $rc -eq 0 ] || exit $rc
fi
SC=${SC:-"1000000:500:250"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets ${LOG2:-26} \
        --rounds 3 --iters 5 $SC > "$OUT/ab_${TAG}_${v}_$r.log" 2>&1
    rc=$?
    sed "s/^/$v r$r /" "$OUT/ab_${TAG}_${v}_$r.log" | grep scenario
    [ $rc -eq 0 ] || { tail -20 "$OUT/ab_${TAG}_${v}_$r.log"; exit $rc; }
  done
done
exit 0
