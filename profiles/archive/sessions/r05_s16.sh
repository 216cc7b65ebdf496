# GPU session 16 (round 5): registered host buffers read in place (zero
# copy) by the kernels -- the host-path parity tests (test_gpu_io.py), then
# bench.py's host leg and C5's registered leg against round 4's DMA paths
# (diagnostics library, XFG_HOST_ZC=off)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== host-path parity"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_io.py > $OUT/s16_pytest.log 2>&1
rc=$?; tail -2 $OUT/s16_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s16_pytest.log | head -30; exit $rc; }
echo "== bench host leg"
for r in 1 2; do
	step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s16_bench_zc_$r.log 2>&1 || exit 3
	XFG_LIB=diag XFG_HOST_ZC=off step 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/s16_bench_dma_$r.log 2>&1 || exit 3
	python3 -c "import json,sys; [print(t, json.loads([l for l in open(f) if l.startswith('{')][-1])['host_path']) for t,f in (('zc ', '$OUT/s16_bench_zc_$r.log'), ('dma', '$OUT/s16_bench_dma_$r.log'))]"
done
echo "== C5 registered"
step 300 python3 tools/bench_configs.py c5 > $OUT/s16_c5_zc.log 2>&1 || exit 4
XFG_LIB=diag XFG_HOST_ZC=off step 300 python3 tools/bench_configs.py c5 > $OUT/s16_c5_dma.log 2>&1 || exit 4
echo "zc : $(grep '"config"' $OUT/s16_c5_zc.log | grep -o '"host_path.*')"
echo "dma: $(grep '"config"' $OUT/s16_c5_dma.log | grep -o '"host_path.*')"
echo s16 done
