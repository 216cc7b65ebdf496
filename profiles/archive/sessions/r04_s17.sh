# GPU session 17 (round 4): 64-byte windows on large strides (diagnostics
# knob), rule-edit latency, PMC of C3 at 2^26, C1/C2.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
XFG_LIB=diag step 400 python -u tools/bench_configs.py c4 c5 > gpurun_out/cfg_s17_diag_w128.log 2>&1; grep config gpurun_out/cfg_s17_diag_w128.log | cut -c1-300 | sed "s/^/w128 /"
XFG_LIB=diag XFG_WINDOW=64 step 400 python -u tools/bench_configs.py c4 c5 > gpurun_out/cfg_s17_diag_w64.log 2>&1; grep config gpurun_out/cfg_s17_diag_w64.log | cut -c1-300 | sed "s/^/w64 /"
step 300 python -u tools/edit_latency.py > gpurun_out/edit_latency.log 2>&1; tail -1 gpurun_out/edit_latency.log
XFG_LIB=diag XFG_QT_PATCH=off step 300 python -u tools/edit_latency.py > gpurun_out/edit_latency_rebuild.log 2>&1; tail -1 gpurun_out/edit_latency_rebuild.log
step 300 bash tools/r04_pmc.sh
step 300 python -u tools/bench_configs.py c2 c1 > gpurun_out/cfg_s17.log 2>&1; grep config gpurun_out/cfg_s17.log | cut -c1-420
echo s17 done
