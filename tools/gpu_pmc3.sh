#!/bin/bash
# PMC passes over the headline classify kernel: PMC_SETS = ';'-separated
# counter sets (one rocprofv3 pass each).  Diagnostics.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-r01}
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra PM <<< "${PMC_SETS:?}"
i=0
for pmc in "${PM[@]}"; do
  i=$((i+1))
  timeout -k 10 ${PASS_TIMEOUT:-150} rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_$i" -o run -- \
     python3 "$GRAFT_REPO_ROOT/tools/ablate.py" --masks 0 --rounds 1 --iters 2 > "$OUT/pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pmc[$pmc] rc=$rc"; fatal $rc && exit $rc
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT"/pmc_${TAG}_* > "$OUT/pmc_${TAG}.json"
cat "$OUT/pmc_${TAG}.json"
exit 0
