#!/bin/bash
# tools/ab_session.sh LIB... — on the GPU box: parity subset, then C3 timing,
# for each variant library (tools/abbuild.sh), twice in alternation.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
LOG2=${LOG2:-24}
for v in "$@"; do
  XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_configs.py tests/test_gpu.py -m gpu -k "c2 or c3 or c4 or pipelined or workload_64b or fuzz or golden or hot or census or single_direction or many_port" \
    > "$OUT/ab_pytest_$v.log" 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 $OUT/ab_pytest_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in "$@"; do
    XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 200 python -u tools/explore.py --log2-packets $LOG2 --rounds 5 1000000:500:250 \
      > "$OUT/ab_t_${v}_$r.log" 2>&1 || exit $?
    echo "$v r$r $(tail -1 $OUT/ab_t_${v}_$r.log)"
  done
done
