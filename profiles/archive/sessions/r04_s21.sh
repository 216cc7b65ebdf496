# GPU session 21 (round 4): IPv6 lookups in the index kernel's loop (V6P):
# QT + config parity tests, then C5 with them against every IPv6 frame
# deferred (diagnostics library, XFG_V6P=off), then C5 on the product.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_configs.py > gpurun_out/pytest_s21.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s21.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s21.log | head -30; exit $rc; }
cfg() {   # label, env..., command
	local lab=$1; shift
	env XFG_LIB=diag "$@" > gpurun_out/s21_$lab.log 2>&1; local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
	grep config gpurun_out/s21_$lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lab', d['config'], d['kernel_ms'], d['roofline']['frac'])"
}
for r in 1 2; do
cfg c5v6p_$r timeout -k 10 200 python -u tools/bench_configs.py c5
cfg c5defer_$r XFG_V6P=off timeout -k 10 200 python -u tools/bench_configs.py c5
done
step 300 python -u tools/bench_configs.py c5 > gpurun_out/s21_c5_product.log 2>&1; grep config gpurun_out/s21_c5_product.log | cut -c1-700
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s21_all.log 2>&1
rc=$?; echo pytest-all rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s21_all.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s21_all.log | head -30; exit $rc; }
echo s21 done
