# GPU session 7 (round 5): fewer waves a CU (6, 4)
#  cur3 : this tree (8 waves, one workgroup a CU)
#  nw6  : 6 waves (SIMDs with 2, 2, 1, 1), partitions owned 42 or 43 a wave
#  nw4  : 4 waves, one a SIMD
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
for v in nw6 nw4; do
	for args in "" "--hot 8"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cur3 nw6 nw4; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s7_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s7_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s7 done
