# GPU session 31 (round 5): the host path's gather pool sized from the CPU
# share (16 threads on this box) against round 4's 8 -- host-path parity,
# then the staged (unregistered) legs of C3 (bench.py host_path) and C5
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "nproc $(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
echo "== host-path parity"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_io.py > $OUT/s31_pytest.log 2>&1
rc=$?; tail -1 $OUT/s31_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s31_pytest.log | head -30; exit $rc; }
show() { python3 -c "import json,sys; h=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])['host_path']; print(sys.argv[1], 'staged', h['Mpps'], h['GBps_h2d'], 'registered', h['registered_Mpps'])" "$@"; }
echo "== C3 host legs"
for r in 1 2; do
	step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s31_bench_16_$r.log 2>&1 || exit 3
	show "16" $OUT/s31_bench_16_$r.log
	XFG_LIB=diag XFG_HOST_THREADS=8 step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s31_bench_8_$r.log 2>&1 || exit 3
	show " 8" $OUT/s31_bench_8_$r.log
done
echo "== C5 staged"
step 400 python3 tools/bench_configs.py c5 > $OUT/s31_c5_16.log 2>&1 || exit 4
echo "16: $(grep '"config"' $OUT/s31_c5_16.log | grep -o '"host_path": {"Mpps": [0-9.]*')"
XFG_LIB=diag XFG_HOST_THREADS=8 step 400 python3 tools/bench_configs.py c5 > $OUT/s31_c5_8.log 2>&1 || exit 4
echo " 8: $(grep '"config"' $OUT/s31_c5_8.log | grep -o '"host_path": {"Mpps": [0-9.]*')"
echo s31 done
