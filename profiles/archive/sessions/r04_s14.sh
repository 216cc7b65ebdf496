# GPU session 14 (round 4): parity of the IPv6-deferral / wide-log QT paths,
# bench, C3 A/B of the bucket lag and window depth, PMC, configs.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_configs.py tests/test_a0_gpu_multirank.py tests/test_gpu_io.py > gpurun_out/pytest_s14.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s14.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s14.log | head -30; exit $rc; }
step 400 python -u bench.py --steps 20 --no-cpu > gpurun_out/bench_s14.log 2>&1 || exit 3
python3 -c "
import json;d=json.loads(open('gpurun_out/bench_s14.log').read().strip().split(chr(10))[-1]);print('bench',d['ms_per_step'],d['roofline']['frac'],d.get('host_path'))"
for v in lag2 d3l2; do for o in "" "--hot 8" "--src-dst"; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/ab_parity.py $o > gpurun_out/par_$v.log 2>&1; tail -1 gpurun_out/par_$v.log
done; done
TAG=s14 VARIANTS="lag1 lag2 d3l2" ROUNDS=2 step 700 bash tools/r04_ab.sh
step 600 python -u tools/bench_configs.py c5 c4 c3sd c3 > gpurun_out/cfg_s14.log 2>&1; grep config gpurun_out/cfg_s14.log | cut -c1-420
echo s14 done
