# GPU session 13 (round 6; run twice, the first on a stale library): the QT waves taking their workgroup's tiles as
# they go, the atomic's return now read at the iteration's end -- one
# diagnostics library, XFG_QT_DYN_MIN=0 (always) against 2^40 (never):
# parity with it always on, then C3 at 2^26 / 2^24 / 2^21, C4 at 2^21.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
export XFG_LIB=diag
echo "== parity (always on)"
for args in "--reps 5" "--reps 4 --src-dst" "--reps 3 --hot 8" "--reps 3 --log2-packets 21" "--reps 3 --log2-packets 24"; do
	XFG_QT_DYN_MIN=0 step 300 python3 tools/ab_parity.py $args > $OUT/s13_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s13_par.log | tail -1; [ $rc -eq 0 ] || exit 2
done
echo "== A/B timing"
for r in 1 2; do
	for lg in 26 24 21; do
		step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 \
			1000000:500:250:XFG_QT_DYN_MIN=1099511627776 1000000:500:250:XFG_QT_DYN_MIN=0 > $OUT/s13_ab_${lg}_$r.log 2>&1 || exit 3
		sed "s/^/2^$lg /" $OUT/s13_ab_${lg}_$r.log | grep scenario
	done
	for m in 1099511627776 0; do
		XFG_QT_DYN_MIN=$m step 300 python3 tools/bench_configs.py c4 --log2-packets 21 > $OUT/s13_c4_$r.log 2>&1 || exit 4
		echo "dyn_min $m c4 2^21 $(grep -o '"kernel_ms": [0-9.]*' $OUT/s13_c4_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s13_c4_$r.log)"
	done
done
echo s13 done
