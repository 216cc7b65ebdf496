# GPU session 5 (round 5): run-of-4 verdict stores and the early first loads
#  cur2 : the tree at session 4
#  vgrp : a wave's tiles in runs of 4, verdicts stored 256 B (a dword a lane) per run
#  early: the first tiles' window loads issued before the LDS set-up
#  ev   : both
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
for v in vgrp early ev; do
	for args in "" "--hot 8"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cur2 vgrp early ev; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s5_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s5_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s5 done
