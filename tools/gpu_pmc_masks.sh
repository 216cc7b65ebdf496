#!/bin/bash
# PMC passes over the headline classify kernel under several XFG_ABLATE masks
# (diagnostics).  PMC_SETS = ';'-separated counter sets, MASKS = ','-separated
# masks; one rocprofv3 pass per (mask, set), each under its own time limit.
# Other XFG_* knobs (XFG_KERNEL, ...) pass through the environment.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-r01}
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra PM <<< "${PMC_SETS:?}"
IFS=',' read -ra MK <<< "${MASKS:-0}"
for m in "${MK[@]}"; do
  i=0
  for pmc in "${PM[@]}"; do
    i=$((i+1))
    timeout -s KILL ${PASS_TIMEOUT:-90} rocprofv3 --pmc $pmc --kernel-trace --output-format csv \
       -d "$OUT/pmc_${TAG}_m${m}_$i" -o run -- \
       python3 "$GRAFT_REPO_ROOT/tools/ablate.py" --masks "$m" --rounds 1 --iters 2 \
       > "$OUT/pmc_${TAG}_m${m}_$i.log" 2>&1
    rc=$?; echo "mask $m pmc[$pmc] rc=$rc"; fatal $rc && exit $rc
  done
  python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT"/pmc_${TAG}_m${m}_* > "$OUT/pmc_${TAG}_m${m}.json"
  echo "== mask $m"; cat "$OUT/pmc_${TAG}_m${m}.json"
done
exit 0
