#!/bin/bash
# Diagnostics session on the GPU box: explore.py scenarios, then a rocprofv3
# kernel-trace summary of the default C3 scenario.  Each GPU step has its own
# time limit; a timeout or crash ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-x}
fatal() { [ "$1" -ne 0 ]; }
SC=${SCENARIOS:-"1000000:500:250 1000000:500:250:XFG_COUNT=atomic 1000000:500:250:XFG_EMPTY=1 1000000:500:250:XFG_KERNEL=general"}
timeout -k 10 300 python -u tools/explore.py $SC > "$OUT/explore_$TAG.log" 2>&1
rc=$?; echo "explore rc=$rc"; cat "$OUT/explore_$TAG.log" | grep scenario; fatal $rc && exit $rc
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- \
     python3 "$GRAFT_REPO_ROOT/tools/explore.py" --rounds 1 --iters 10 ${PROF_SC:-1000000:500:250} > "$OUT/prof_$TAG.log" 2>&1
  rc=$?; echo "prof rc=$rc"; fatal $rc && exit $rc
  find "$OUT/prof_$TAG" -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -12
fi
exit 0
