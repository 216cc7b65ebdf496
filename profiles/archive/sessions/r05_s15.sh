# GPU session 15 (round 5): the generic pipelined kernel with small maps'
# Bloom filters staged in LDS (C1) -- parity (configs, fixture, KAT), C1
# A/B (diagnostics library, XFG_BLOOM_LDS=off against on), then the
# zero-copy probe (frames read from mapped host memory, tools/zerocopy_probe.py)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py tests/test_gpu.py tests/test_kat_counters.py > $OUT/s15_pytest.log 2>&1
rc=$?; tail -2 $OUT/s15_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s15_pytest.log | head -30; exit $rc; }
echo "== C1 A/B"
for r in 1 2; do
	XFG_LIB=diag step 300 python3 tools/bench_configs.py c1 > $OUT/s15_c1_on_$r.log 2>&1 || exit 3
	XFG_LIB=diag XFG_BLOOM_LDS=off step 300 python3 tools/bench_configs.py c1 > $OUT/s15_c1_off_$r.log 2>&1 || exit 3
	echo "on : $(grep '"config"' $OUT/s15_c1_on_$r.log | cut -c1-260)"
	echo "off: $(grep '"config"' $OUT/s15_c1_off_$r.log | cut -c1-260)"
done
echo "== zero-copy probe"
step 300 python3 tools/zerocopy_probe.py > $OUT/s15_zerocopy.log 2>&1 || { tail -5 $OUT/s15_zerocopy.log; exit 4; }
cat $OUT/s15_zerocopy.log | grep case
echo s15 done
