# GPU session 28 (round 5): registered large slots through zero-copy chunks
# alternating with DMA'd 64-byte windows -- host-path parity (test_gpu_io.py),
# then C5's registered leg: mixed (product), zero copy alone and DMA alone
# (diagnostics library, XFG_HOST_MIX=off / dma)
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
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_io.py > $OUT/s28_pytest.log 2>&1
rc=$?; tail -1 $OUT/s28_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s28_pytest.log | head -30; exit $rc; }
echo "== C5 registered"
for r in 1 2; do
	step 400 python3 tools/bench_configs.py c5 > $OUT/s28_c5_mix_$r.log 2>&1 || exit 4
	echo "mix: $(grep '"config"' $OUT/s28_c5_mix_$r.log | grep -o '"registered_Mpps[^,]*, "registered_ms[^,]*')"
	for md in off dma; do
		XFG_LIB=diag XFG_HOST_MIX=$md step 400 python3 tools/bench_configs.py c5 > $OUT/s28_c5_${md}_$r.log 2>&1 || exit 4
		echo "$md: $(grep '"config"' $OUT/s28_c5_${md}_$r.log | grep -o '"registered_Mpps[^,]*, "registered_ms[^,]*')"
	done
done
echo s28 done
