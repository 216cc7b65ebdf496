# GPU session 4 (round 5): ordering A/Bs of the QT kernel's iteration
#  cur  : the tree at session 3 (count kernel one round of slices in flight)
#  cur2 : + the count kernel's next round of slices issued before this round's atomics
#  ord1 : W after L (bucket loads before the verdict / log work)
#  vst1 : a tile's verdict bytes stored at the top of the next iteration
#  ov   : cur2 + ord1 + vst1
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
for v in cur2 ord1 vst1 ov; do
	for args in "" "--hot 8"; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/ab_parity.py $args || exit 2
	done
done
echo "== timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in cur cur2 ord1 vst1 ov; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/s4_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s4_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo s4 done
