# GPU session 2 (round 6, second form): the product library's parity over
# one and several launches (the count wave counts each launch's log inside
# the next), then the QT kernel A/B -- base (SDWA compares, masks in SGPRs) /
# pkm (packed u16 min) / plip (pkm + the halves swapped in place), each with
# the count wave off (XFG_CW=off: a count kernel every four launches) and on.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (product library; HIP errors logged)"
for args in "" "--reps 5" "--reps 5 --src-dst" "--reps 4 --hot 8" "--reps 3 --log2-packets 24" "--reps 3 --log2-packets 21"; do
	AMD_LOG_LEVEL=1 XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so step 300 python3 tools/ab_parity.py $args > $OUT/s2_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s2_par.log | tail -4; [ $rc -eq 0 ] || exit 2
done
echo "== parity (A/B libraries)"
for v in pkm plip; do
	for args in "" "--reps 4 --src-dst" "--reps 3 --hot 8"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== A/B timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in base pkm plip; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 \
				1000000:500:250:XFG_CW=off 1000000:500:250 > $OUT/s2_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s2_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s2 done
