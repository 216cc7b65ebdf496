# GPU session 25 (round 4): box-to-box spread of the committed tree -- bench.py
# (no CPU baseline) and C5 on whatever box the pool gives.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 400 python -u bench.py --no-cpu > gpurun_out/bench_s25.log 2>&1 || exit 3
tail -1 gpurun_out/bench_s25.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('C3 2^26', d['ms_per_step'], d['roofline']['frac'], d['roofline']['peak_measured_stream_read'])"
step 300 python -u tools/bench_configs.py c5 c3 > gpurun_out/cfg_s25.log 2>&1; grep config gpurun_out/cfg_s25.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config'], d['kernel_ms'], d['roofline']['frac'])"
echo s25 done
