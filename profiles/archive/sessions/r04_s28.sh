# GPU session 28 (round 4): rocprofv3 kernel summaries of the final tree on
# the other configurations (C5, C4, C3 src|dst, C2, C1).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s28 -o run -- python3 tools/bench_configs.py c5 c4 c3sd c2 c1 > gpurun_out/prof_s28.log 2>&1
echo prof rc=$?
grep config gpurun_out/prof_s28.log | cut -c1-200
echo s28 done
