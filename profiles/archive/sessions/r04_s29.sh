# GPU session 29 (round 4): the whole GPU suite again on another box, and the
# two-rank launcher rehearsal on one device (RCCL refuses the shared device,
# which the line reports).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s29.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s29.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s29.log | head -30; exit $rc; }
step 600 python -u bench.py --gpus 2 --one-device --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_w2_s29.log 2>&1; echo w2 rc=$?
tail -1 gpurun_out/bench_w2_s29.log | cut -c1-600
echo s29 done
