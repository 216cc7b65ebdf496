# GPU session 35 (round 5): 32-bit QT-order counts with the atomics through
# the global address space (session 34: atomicAdd on the u32 generic
# pointer became four FLAT atomics, whose LDS-counter waits cost the QT
# kernel 13 %) -- parity of the A/B library, then C3 / C5 / C4 against the
# 64-bit counts, same box
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (u32g)"
for args in "" "--src-dst" "--hot 8" "--log2-packets 24"; do
	XFG_LIB=$R/tools/abl/u32g.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== A/B"
for r in 1 2; do
	for v in u64 u32g; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets 26 --rounds 3 --iters 10 1000000:500:250 > $OUT/s35_c3_${v}_26_$r.log 2>&1 || exit 3
		echo "c3 2^26 $v $(grep scenario $OUT/s35_c3_${v}_26_$r.log | tail -1)"
	done
	for c in c3 c5 c4; do
		for v in u64 u32g; do
			extra=""; [ $c = c5 ] && extra="--no-host"
			XFG_LIB=$R/tools/abl/$v.so step 400 python3 tools/bench_configs.py $c $extra > $OUT/s35_${c}_${v}_$r.log 2>&1 || { tail -3 $OUT/s35_${c}_${v}_$r.log; exit 3; }
			echo "$c $v $(grep -o '"kernel_ms": [0-9.]*' $OUT/s35_${c}_${v}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s35_${c}_${v}_$r.log)"
		done
	done
done
echo s35 done
