# GPU session 18 (round 4): where the hit log pays (C3 at 2^26 and 2^24, C3
# src|dst, C4 at 64-byte windows) against LDS cache + atomics; one box.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cfg() {   # label, env..., config
	local lab=$1; shift
	env XFG_LIB=diag "$@" > gpurun_out/s18_$lab.log 2>&1; local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
	grep config gpurun_out/s18_$lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lab', d['config'], d['kernel_ms'], d['roofline']['frac'])"
}
for r in 1 2; do
cfg c3log_$r timeout -k 10 200 python -u tools/bench_configs.py c3
cfg c3nolog_$r XFG_LOG=off timeout -k 10 200 python -u tools/bench_configs.py c3
cfg c3sdlog_$r timeout -k 10 200 python -u tools/bench_configs.py c3sd
cfg c3sdnolog_$r XFG_LOG=off timeout -k 10 200 python -u tools/bench_configs.py c3sd
cfg c4w64log_$r XFG_WINDOW=64 timeout -k 10 200 python -u tools/bench_configs.py c4
cfg c4w64nolog_$r XFG_WINDOW=64 XFG_LOG=off timeout -k 10 200 python -u tools/bench_configs.py c4
done
for r in 1 2; do for m in "" "XFG_LOG=off"; do
env XFG_LIB=diag $m timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 1000000:500:250 > gpurun_out/s18_c3_2p26_$r.log 2>&1; rc=$?
if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
grep scenario gpurun_out/s18_c3_2p26_$r.log | sed "s/^/2^26 [$m] r$r /"
done; done
echo s18 done
