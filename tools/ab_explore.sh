#!/bin/bash
# tools/ab_explore.sh LIB... — on the GPU box: explore.py scenarios ($SC) at
# 2^$LOG2 packets for each diagnostics library variant (tools/abbuild.sh),
# twice in alternation (same box, so variants compare).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
LOG2=${LOG2:-26}
SC=${SC:-1000000:500:250}
for r in 1 2; do
  for v in "$@"; do
    lib=$PWD/tools/abl/$v.so
    [ "$v" = product ] && lib=product
    [ "$v" = diag ] && lib=diag
    XFG_LIB=$lib timeout -k 10 300 python -u tools/explore.py --log2-packets $LOG2 --rounds 3 --iters 5 $SC \
      > "$OUT/abx_${v}_$r.log" 2>&1 || exit $?
    sed "s/^/$v r$r /" "$OUT/abx_${v}_$r.log" | grep scenario
  done
done
