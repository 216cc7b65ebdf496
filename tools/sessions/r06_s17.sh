# GPU session 17 (round 6): the grid's tile pool (the last sixth of the
# rounds taken by any workgroup, XFG_QT_POOL): parity with it forced on at
# several sizes (diagnostics library, XFG_QT_DYN_MIN=0) and on the product
# library, then C3 at 2^26 / 2^24 against the previous commit's kernel
# (A/B libraries with C3's program only: prev, pool) and pool on/off in one
# library, C4 / C5 at 2^23 on/off, and the per-workgroup phases with it.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (pool forced: diagnostics library, dynamic from any size)"
for args in "--reps 3 --log2-packets 22" "--reps 4 --log2-packets 23 --src-dst" "--reps 3 --log2-packets 24 --hot 8" "--reps 3 --log2-packets 24"; do
	XFG_LIB=diag XFG_QT_DYN_MIN=0 step 120 python3 tools/ab_parity.py $args > $OUT/s17_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s17_par.log | tail -1; [ $rc -eq 0 ] || exit 2
done
echo "== parity (product library, 2^24 and 2^26)"
for args in "--reps 3 --log2-packets 24" "--reps 2 --log2-packets 26"; do
	XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so step 300 python3 tools/ab_parity.py $args > $OUT/s17_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s17_par.log | tail -1; [ $rc -eq 0 ] || exit 2
done
echo "== A/B timing"
for r in 1 2; do
	for lg in 26 24; do
		for v in prev pool; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 \
				1000000:500:250 1000000:500:250:XFG_QT_POOL=off > $OUT/s17_ab.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s17_ab.log | grep scenario
		done
	done
done
for c in c4 "c5 --no-host"; do
	for p in on off; do
		XFG_LIB=diag XFG_QT_POOL=$p step 300 python3 tools/bench_configs.py $c > $OUT/s17_c.log 2>&1 || exit 4
		echo "$c pool $p $(grep -o '"kernel_ms": [0-9.]*' $OUT/s17_c.log)"
	done
done
echo "== phases"
XFG_LIB=diag step 400 python3 tools/qt_phases.py c3 26 > $OUT/s17_ph.log 2>&1 || { tail -5 $OUT/s17_ph.log; exit 5; }
grep '"config"' $OUT/s17_ph.log | tee $OUT/s17_phases.log | cut -c1-600
echo s17 done
