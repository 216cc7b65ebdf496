# GPU session 23 (round 4): deferred packets walked inside the loop, 64 at a
# time (drain) against each wave's tail after it (base): parity, then C3.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
for o in "" "--hot 8" "--src-dst"; do
XFG_LIB=$PWD/tools/abl/drain.so step 200 python -u tools/ab_parity.py $o > gpurun_out/par_drain.log 2>&1; tail -1 gpurun_out/par_drain.log
done
for r in 1 2; do for v in base drain; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c3 c5 > gpurun_out/s23_${v}_$r.log 2>&1
grep config gpurun_out/s23_${v}_$r.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v r$r', d['config'], d['kernel_ms'], d['roofline']['frac'])"
done; done
TAG=s23 VARIANTS="base drain" ROUNDS=2 step 600 bash tools/r04_ab.sh
echo s23 done
