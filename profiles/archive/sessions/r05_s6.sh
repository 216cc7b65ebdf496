# GPU session 6 (round 5): more waves a CU (12, or 16 with 68-byte rows)
#  cur3 : this tree (8 waves, one workgroup a CU)
#  nw12 : 12 waves (3 a SIMD), partitions owned 21 or 22 a wave
#  nw16 : 16 waves with 68-byte (unpadded-to-16) rows, b32 row access
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
for v in nw12 nw16; do
	for args in "" "--hot 8"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cur3 nw12 nw16; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s6_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s6_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s6 done
