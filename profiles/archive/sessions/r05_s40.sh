# GPU session 40 (round 5): the hit log from twice the QT slots -- the QT
# and configuration tests (the fold test and the concentrated-partitions test
# now at 2^22 packets), then C4 and C3 at 2^21 / 2^22 / 2^23 / 2^24
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
step 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_configs.py tests/test_gpu_scale.py > $OUT/s40_pytest.log 2>&1
rc=$?; tail -1 $OUT/s40_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s40_pytest.log | head -30; exit $rc; }
for c in c4 c3; do
	for l in 21 22 23 24; do
		step 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/s40_${c}_$l.log 2>&1 || exit 3
		echo "$c 2^$l $(grep -o '"kernel_ms": [0-9.]*' $OUT/s40_${c}_$l.log) $(grep -o '"frac": [0-9.]*' $OUT/s40_${c}_$l.log)"
	done
done
echo s40 done
