# GPU session 33 (round 5): 32-bit QT-order counts (folded before 2^32
# packets) -- the QT, scale and configuration tests and the fold test, then
# C5 / C4 / C3 kernel times against the previous commit's 64-bit counts
# (tools/abbuild.sh -DXFG_AB_C3, SRC= the previous tree), same box
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
step 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_scale.py tests/test_gpu_configs.py > $OUT/s33_pytest.log 2>&1
rc=$?; tail -1 $OUT/s33_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s33_pytest.log | head -30; exit $rc; }
echo "== A/B (kernel ms, frac)"
for r in 1 2; do
	for c in c5 c4 c3; do
		for v in u64 u32; do
			extra=""; [ $c = c5 ] && extra="--no-host"
			XFG_LIB=$R/tools/abl/$v.so step 400 python3 tools/bench_configs.py $c $extra > $OUT/s33_${c}_${v}_$r.log 2>&1 || { tail -3 $OUT/s33_${c}_${v}_$r.log; exit 3; }
			echo "$c $v $(grep -o '"kernel_ms": [0-9.]*' $OUT/s33_${c}_${v}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s33_${c}_${v}_$r.log)"
		done
	done
done
echo s33 done
