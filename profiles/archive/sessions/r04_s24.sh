# GPU session 24 (round 4): the committed tree as the driver runs it at round
# end -- smoke(), the whole GPU suite, bench.py.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s24.log 2>&1; tail -2 gpurun_out/smoke_s24.log
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s24.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s24.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s24.log | head -30; exit $rc; }
step 500 python -u bench.py > gpurun_out/bench_s24.log 2>&1 || exit 3
tail -1 gpurun_out/bench_s24.log | cut -c1-300
echo s24 done
