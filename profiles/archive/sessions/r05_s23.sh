# GPU session 23 (round 5): the Ethernet-key kernel's shape, A/B on one box
# (tools/abbuild.sh -DXFG_AB_ETH variants): tiles per wave iteration (G) and register buffers (D),
# and the register budget (6 or 8 waves a SIMD); C1 at 2^24 and 2^26
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (each variant, C1 rules)"
for v in ekg2 ekg2d2 ekg2d3 ekg1d2 ekg1d3 ekg1d4 ekg1d3w8; do
	XFG_LIB=$R/tools/abl/$v.so step 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_eth.py -k "c1_rules or parity" > $OUT/s23_pytest_$v.log 2>&1
	rc=$?; echo "$v: $(tail -1 $OUT/s23_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
echo "== C1 A/B"
for r in 1 2; do
	for l in 24 26; do
		for v in ekg2 ekg2d2 ekg2d3 ekg1d2 ekg1d3 ekg1d4 ekg1d3w8; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/bench_configs.py c1 --no-cpu --log2-packets $l > $OUT/s23_${v}_${l}_$r.log 2>&1 || { tail -3 $OUT/s23_${v}_${l}_$r.log; exit 3; }
			echo "$v 2^$l $(grep -o '"kernel_ms": [0-9.]*' $OUT/s23_${v}_${l}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s23_${v}_${l}_$r.log)"
		done
	done
done
echo s23 done
