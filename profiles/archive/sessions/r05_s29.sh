# GPU session 29 (round 5): registered large slots through zero-copy chunks
# alternating with DMA'd 64-byte windows -- host-path parity (test_gpu_io.py),
# then C5's registered leg: mixed with 3 DMA'd chunks a zero-copy chunk
# (product), zero copy alone, 1 or 2 DMA'd chunks (diagnostics library)
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
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_io.py > $OUT/s29_pytest.log 2>&1
rc=$?; tail -1 $OUT/s29_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s29_pytest.log | head -30; exit $rc; }
echo "== C5 registered"
for r in 1 2; do
	step 400 python3 tools/bench_configs.py c5 > $OUT/s29_c5_mix_$r.log 2>&1 || exit 4
	echo "mix: $(grep '"config"' $OUT/s29_c5_mix_$r.log | grep -o '"registered_Mpps[^,]*, "registered_ms[^,]*')"
	for md in off nd1 nd2; do
		case $md in off) E="XFG_HOST_MIX=off";; nd1) E="XFG_HOST_MIX_ND=1";; nd2) E="XFG_HOST_MIX_ND=2";; esac
		env XFG_LIB=diag $E timeout -k 10 400 python3 tools/bench_configs.py c5 > $OUT/s29_c5_${md}_$r.log 2>&1 || exit 4
		echo "$md: $(grep '"config"' $OUT/s29_c5_${md}_$r.log | grep -o '"registered_Mpps[^,]*, "registered_ms[^,]*')"
	done
done
echo s29 done
