# GPU session 9 (round 5): the hit ring protocol without exec masks (cnt2) against the masked one (cnt0)
#  cur3 : this tree (8 waves, one workgroup a CU)
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
for v in cnt2 cnt0; do
	for args in "" "--hot 8" "--src-dst"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cnt0 cnt2; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s9_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s9_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s9 done
