#!/bin/bash
# PMC + ablation session (diagnostics).  Each GPU step has its own limit; a
# timeout (124/137) or crash (134/139) ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-r01}
fatal() { [ "$1" -eq 124 ] || [ "$1" -eq 137 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 300 python tools/ablate.py ${ABLATE_ARGS:-} > "$OUT/ablate_$TAG.log" 2>&1
rc=$?; echo "ablate rc=$rc"; tail -2 "$OUT/ablate_$TAG.log"; fatal $rc && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/counters_$TAG.txt" 2>&1; echo "list rc=$?"
i=0
PM=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum"
    "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum"
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
    "GRBM_GUI_ACTIVE")
[ -n "$PMC_ONLY" ] && PM=("$PMC_ONLY")
for pmc in "${PM[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d "$OUT/pmc_${TAG}_$i" -o run -- \
     python3 "$GRAFT_REPO_ROOT/tools/ablate.py" --masks 0 --rounds 1 --iters 2 > "$OUT/pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pmc[$pmc] rc=$rc"; fatal $rc && exit $rc
done
exit 0
