# GPU session 12 (round 6): a workgroup's waves taking its tiles from an
# LDS counter (XFG_QT_DYN, dyn1) against a fixed share each (dyn0), A/B
# libraries with C3's program only: parity first, then C3 at 2^26 / 2^24 /
# 2^21 and C4 at 2^21, alternated, and the per-workgroup phases of dyn1.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (dyn1)"
for args in "" "--reps 5" "--reps 4 --src-dst" "--reps 3 --hot 8" "--reps 3 --log2-packets 21" "--reps 3 --log2-packets 24"; do
	XFG_LIB=$R/tools/abl/dyn1.so step 300 python3 tools/ab_parity.py $args > $OUT/s12_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s12_par.log | tail -2; [ $rc -eq 0 ] || exit 2
done
echo "== A/B timing"
for r in 1 2; do
	for lg in 26 24 21; do
		for v in dyn0 dyn1; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 \
				1000000:500:250 > $OUT/s12_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s12_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
	for v in dyn0 dyn1; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/bench_configs.py c4 --log2-packets 21 > $OUT/s12_c4_${v}_$r.log 2>&1 || exit 4
		echo "$v c4 2^21 $(grep -o '"kernel_ms": [0-9.]*' $OUT/s12_c4_${v}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s12_c4_${v}_$r.log)"
	done
done
echo "== phases (dyn1)"
for a in "c3 26" "c3 21"; do
	XFG_LIB=$R/tools/abl/dyn1.so step 400 python3 tools/qt_phases.py $a > $OUT/s12_ph.log 2>&1 || { tail -5 $OUT/s12_ph.log; exit 5; }
	grep '"config"' $OUT/s12_ph.log | tee -a $OUT/s12_phases.log | cut -c1-700
done
echo s12 done
