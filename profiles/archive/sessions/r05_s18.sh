# GPU session 18 (round 5): zero-copy host path, chunks ramping 2^17 -> 2^21, raw u16 lengths --
# host-path parity, then bench.py's host leg (zero copy at chunk sizes
# 2^18..2^21 against round 4's DMA path) and C5's registered leg
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
show() { python3 -c "import json,sys; h=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])['host_path']; print(sys.argv[1], h['Mpps'], h['registered_Mpps'], h['registered_GBps_h2d'])" "$@"; }
cd $R
echo "== host-path parity"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_io.py > $OUT/s18_pytest.log 2>&1
rc=$?; tail -2 $OUT/s18_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s18_pytest.log | head -30; exit $rc; }
echo "== bench host leg: staged Mpps, registered Mpps, registered GB/s"
for r in 1 2; do
	step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s18_bench_zc_$r.log 2>&1 || exit 3
	show "zc21" $OUT/s18_bench_zc_$r.log
	XFG_LIB=diag XFG_ZC_RAMP=off step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s18_bench_noramp_$r.log 2>&1 || exit 3
	show "flat" $OUT/s18_bench_noramp_$r.log
	XFG_LIB=diag XFG_HOST_ZC=off step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s18_bench_dma_$r.log 2>&1 || exit 3
	show "dma " $OUT/s18_bench_dma_$r.log
done
echo "== C5 registered"
step 300 python3 tools/bench_configs.py c5 > $OUT/s18_c5_zc.log 2>&1 || exit 4
echo "zc : $(grep '"config"' $OUT/s18_c5_zc.log | grep -o '"registered_Mpps.*')"
echo s18 done
