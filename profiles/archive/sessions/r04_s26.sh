# GPU session 26 (round 4): rows at a 16-byte-aligned stride, written and
# read a quarter-line at a time (rowq), a wave's log partitions
# consecutive (ownc), both (both2), against the product kernel (base).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
for vo in "rowq:" "rowq:--hot 8" "rowq:--src-dst" "ownc:" "ownc:--hot 8" "both2:--src-dst"; do v=${vo%%:*}; o=${vo#*:}
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/ab_parity.py $o > gpurun_out/par_$v.log 2>&1; tail -1 gpurun_out/par_$v.log
done
for r in 1 2; do for v in base rowq ownc both2; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c3 c3sd > gpurun_out/s26_${v}_$r.log 2>&1
grep config gpurun_out/s26_${v}_$r.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v r$r', d['config'], d['kernel_ms'], d['roofline']['frac'])"
done; done
for v in base rowq; do XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c5 > gpurun_out/s26_c5_$v.log 2>&1; grep config gpurun_out/s26_c5_$v.log | cut -c1-200 | sed "s/^/$v /"; done
TAG=s26 VARIANTS="base rowq ownc both2" ROUNDS=2 step 800 bash tools/r04_ab.sh
echo s26 done
