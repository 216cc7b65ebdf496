#!/bin/bash
# Round-3 measurement session on the GPU box (product library): the C3
# bench line, a rocprofv3 kernel-trace summary of it, PMC passes of the QT
# classify kernel and the count kernel at the bench's batch, and the other
# BASELINE configurations (tools/bench_configs.py, incl. C3 src|dst).  Each
# step has its own time limit; the first failure ends the session.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"; mkdir -p "$OUT"
TAG=${1:-m}
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench_$TAG.log" 2>&1 || { tail -20 "$OUT/bench_$TAG.log"; exit 1; }
tail -1 "$OUT/bench_$TAG.log" | cut -c1-400
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats \
    -d "$OUT/prof_$TAG" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --host-log2-packets 0) > "$OUT/prof_$TAG.log" 2>&1 || { tail -20 "$OUT/prof_$TAG.log"; exit 2; }
find "$OUT/prof_$TAG" -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -5
export XFG_LIB=product
KNAME=pipeq bash tools/pmc.sh c3q_$TAG "--log2-packets 26 1000000:500:250" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum,TCC_MISS_sum" \
  "GRBM_GUI_ACTIVE,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY" \
  "SQ_INSTS_VMEM_RD,SQ_INSTS_VMEM_WR,TA_TA_BUSY_sum,TD_TD_BUSY_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum,TCP_PENDING_STALL_CYCLES_sum,TCP_TCC_READ_REQ_sum" > /dev/null || exit 3
python3 tools/pmc_summary.py --kernel log_count "$OUT"/pmc_c3q_${TAG}_* > "$OUT/pmc_c3lc_$TAG.json"
head -c 600 "$OUT/pmc_c3q_$TAG.json"
unset XFG_LIB
timeout -k 10 600 python -u tools/bench_configs.py c2 c3 c4 c5 c3sd > "$OUT/configs_$TAG.log" 2>&1 || { tail -20 "$OUT/configs_$TAG.log"; exit 4; }
cut -c1-300 "$OUT/configs_$TAG.log"
exit 0
