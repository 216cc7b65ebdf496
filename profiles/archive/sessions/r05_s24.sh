# GPU session 24 (round 5): the QT kernel with each lane loading its own
# frame's 64-byte window (no LDS row staging, XFG_QT_LANEW) against the
# current kernel, A/B on one box (tools/abbuild.sh -DXFG_AB_C3); then the
# product library (Ethernet kernel G 1, D 2) through C1 and the eth tests
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (qtlane)"
for args in "" "--src-dst" "--hot 8" "--log2-packets 24"; do
	XFG_LIB=$R/tools/abl/qtlane.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== A/B timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in qtcur qtlane; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 1000000:500:250 > $OUT/s24_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s24_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo "== product: eth tests + C1"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_eth.py tests/test_gpu_configs.py -k "eth or c1" > $OUT/s24_pytest.log 2>&1
rc=$?; tail -1 $OUT/s24_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s24_pytest.log | head -30; exit $rc; }
for l in 24 26; do
	step 300 python3 tools/bench_configs.py c1 --no-cpu --log2-packets $l > $OUT/s24_c1_$l.log 2>&1 || exit 4
	grep '"config"' $OUT/s24_c1_$l.log
done
echo s24 done
