# GPU session 13 (round 5): the quotient index in 16-byte buckets (nine
# 14-bit remainders + an overflow flag; one load instruction a tile) -- A/B
# parity and timing (q9 against cnt2, the 32-byte-bucket kernel), then the
# product library's QT and scale GPU tests
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
for args in "" "--hot 8" "--src-dst" "--log2-packets 24"; do
	XFG_LIB=$R/tools/abl/q9.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cnt2 q9; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s13_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s13_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo "== QT + scale GPU tests (product library)"
step 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_scale.py tests/test_gpu_configs.py > $OUT/s13_pytest.log 2>&1
rc=$?; tail -3 $OUT/s13_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s13_pytest.log | head -30; exit $rc; }
echo s13 done
