# GPU session 27 (round 4): the final tree as the driver runs it at round end
# -- smoke(), the whole GPU suite, bench.py -- then the rocprofv3 kernel
# summary of the bench and the PMC passes of C3 at 2^26.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_s27.log 2>&1; tail -2 gpurun_out/smoke_s27.log
step 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s27.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s27.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s27.log | head -30; exit $rc; }
step 500 python -u bench.py > gpurun_out/bench_s27.log 2>&1 || exit 3
tail -1 gpurun_out/bench_s27.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s27 -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/prof_s27.log 2>&1
echo prof rc=$?
TAG=r04f step 300 bash tools/r04_pmc.sh
echo s27 done
