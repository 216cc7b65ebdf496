#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group) over one explore.py
# scenario (diagnostics).  Usage: bash tools/pmc.sh TAG "scenario" "grp1" "grp2" ...
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=$1; SC=$2; shift 2
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_$i" -o run -- \
     python3 "$GRAFT_REPO_ROOT/tools/explore.py" --rounds 1 --iters 3 $SC > "$OUT/pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pmc[$pmc] rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" --kernel "${KNAME:-pipeline}" "$OUT"/pmc_${TAG}_* > "$OUT/pmc_${TAG}.json" 2>&1; cat "$OUT/pmc_${TAG}.json"
exit 0
