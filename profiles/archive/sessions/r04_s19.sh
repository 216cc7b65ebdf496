# GPU session 19 (round 4): the deferred-packet kernel, 64-byte windows by
# default and the hit-log bound: QT tests, then A/B of the deferred packets'
# kernel against each wave's tail (diagnostics library), then the whole GPU
# suite and the bench.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py > gpurun_out/pytest_s19_qt.log 2>&1
rc=$?; echo pytest-qt rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s19_qt.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s19_qt.log | head -30; exit $rc; }
cfg() {   # label, env..., command
	local lab=$1; shift
	env XFG_LIB=diag "$@" > gpurun_out/s19_$lab.log 2>&1; local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
	grep config gpurun_out/s19_$lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lab', d['config'], d['kernel_ms'], d['roofline']['frac'])"
}
for r in 1 2; do
cfg c3sep_$r timeout -k 10 200 python -u tools/bench_configs.py c3
cfg c3inl_$r XFG_DEFER=inline timeout -k 10 200 python -u tools/bench_configs.py c3
cfg c5sep_$r timeout -k 10 200 python -u tools/bench_configs.py c5
cfg c5inl_$r XFG_DEFER=inline timeout -k 10 200 python -u tools/bench_configs.py c5
done
for r in 1 2; do for m in "" "XFG_DEFER=inline"; do
env XFG_LIB=diag $m timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 1000000:500:250 > gpurun_out/s19_c3_2p26_$r.log 2>&1; rc=$?
if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
grep scenario gpurun_out/s19_c3_2p26_$r.log | sed "s/^/2^26 [$m] r$r /"
done; done
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s19.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s19.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s19.log | head -30; exit $rc; }
echo s19 done
