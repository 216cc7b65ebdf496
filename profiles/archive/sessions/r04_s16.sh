# GPU session 16 (round 4): C5 and C4 counting and window matrix on one box
# (diagnostics library): hit log vs LDS cache + atomics, QT vs general kernel,
# 128- vs 64-byte windows; a GPU test of the index without its log.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qt.py -k "ipv6 or past_one or falls_back or concentrated" > gpurun_out/pytest_s16.log 2>&1
rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s16.log | tail -2
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s16.log | head -30; exit $rc; }
XFG_LIB=diag XFG_LOG=off XFG_QT=on step 200 python -u tools/ab_parity.py > gpurun_out/par_nolog.log 2>&1; tail -1 gpurun_out/par_nolog.log
for m in "XFG_QT=on" "XFG_LOG=off" "XFG_QT=off XFG_LOG=off" "XFG_QT=off" "XFG_WINDOW=64" "XFG_WINDOW=64 XFG_LOG=off" "XFG_WINDOW=64 XFG_QT=off XFG_LOG=off"; do
t=$(echo $m | tr ' =' '__')
env XFG_LIB=diag $m timeout -k 10 300 python -u tools/bench_configs.py c5 > gpurun_out/c5m_$t.log 2>&1; rc=$?
if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
grep config gpurun_out/c5m_$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c5 $m', d['kernel_ms'], d['roofline']['frac'])"
done
for m in "XFG_QT=on" "XFG_WINDOW=64" "XFG_LOG=off"; do
t=$(echo $m | tr ' =' '__')
env XFG_LIB=diag $m timeout -k 10 300 python -u tools/bench_configs.py c4 > gpurun_out/c4m_$t.log 2>&1; rc=$?
if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP rc=$rc"; exit $rc; fi
grep config gpurun_out/c4m_$t.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('c4 $m', d['kernel_ms'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
XFG_LIB=diag step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 tools/bench_configs.py c5 > gpurun_out/prof_c5.log 2>&1; echo prof rc=$?
find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -3
echo s16 done
