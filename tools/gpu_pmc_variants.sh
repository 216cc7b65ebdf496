#!/bin/bash
# Instruction counts of diagnostic build variants of the headline kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-r01}
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python tools/ablate.py --masks 0 --envs "${VARIANT_ENVS:-XFG_VARIANT=0x100;XFG_VARIANT=0x200;XFG_VARIANT=0x400;XFG_VARIANT=0x800;XFG_VARIANT=0xF00}" > "$OUT/ablate_$TAG.log" 2>&1
rc=$?; echo "ablate rc=$rc"; tail -1 "$OUT/ablate_$TAG.log"; fatal $rc && exit $rc
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-0 0x100 0x200 0x400 0x800 0xF00}; do
  XFG_VARIANT=$v timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS \
     --kernel-trace --output-format csv -d "$OUT/pmcv_${TAG}_$v" -o run -- \
     python3 "$GRAFT_REPO_ROOT/tools/ablate.py" --masks 0 --rounds 1 --iters 2 > "$OUT/pmcv_${TAG}_$v.log" 2>&1
  rc=$?; echo "pmc[$v] rc=$rc"; fatal $rc && exit $rc
  python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$OUT/pmcv_${TAG}_$v" | tr -d '\n '; echo
done
exit 0
