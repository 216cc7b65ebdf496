# GPU session 22 (round 4): the status table's measurements on one box and
# one tree -- bench.py as the driver runs it, every configuration, rule-edit
# latency with and without the in-place index patch.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 500 python -u bench.py > gpurun_out/bench_s22.log 2>&1 || exit 3
tail -1 gpurun_out/bench_s22.log | cut -c1-400
step 900 python -u tools/bench_configs.py c2 c3 c3sd c4 c5 c1 > gpurun_out/cfg_s22.log 2>&1; grep config gpurun_out/cfg_s22.log | cut -c1-500
step 300 python -u tools/edit_latency.py > gpurun_out/edit_latency_s22.log 2>&1; tail -1 gpurun_out/edit_latency_s22.log
XFG_LIB=diag XFG_QT_PATCH=off step 300 python -u tools/edit_latency.py > gpurun_out/edit_latency_rebuild_s22.log 2>&1; tail -1 gpurun_out/edit_latency_rebuild_s22.log
echo s22 done
