# GPU session 12 (round 5): one 16-byte bucket load a lane (h1, timing only:
# results wrong) against two 32-packet instructions (cnt2), both with the
# diagnostics mask 1 (no counting) so that the hits they find do not differ in cost
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
for lg in 26 24; do
	for r in 1 2 3; do
		for v in cnt2 h1; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250:XFG_DIAG_MASK=1 1000000:500:250:XFG_DIAG_MASK=8193 > $OUT/s12_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s12_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s12 done
