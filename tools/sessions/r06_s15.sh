# GPU session 15 (round 6): C3e with the dynamic tiles on and off (same box),
# then the bench command under rocprofv3 --kernel-trace --stats (the
# summary the bench line's kernel time is checked against), then the PMC
# passes of the product QT kernel on C3 at 2^26 (tools/pmc_c3.sh, TAG r06).
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== c3e A/B"
for r in 1 2; do
	for m in 1099511627776 0; do
		XFG_LIB=diag XFG_QT_DYN_MIN=$m step 300 python3 tools/bench_configs.py c3e c3 > $OUT/s15_dyn.log 2>&1 || exit 8
		echo "dyn_min $m $(grep -o '"config": "[a-z0-9]*"\|"kernel_ms": [0-9.]*' $OUT/s15_dyn.log | tr '\n' ' ')"
	done
done
echo "== bench under rocprofv3"
cd /tmp && export TMPDIR=/tmp
step 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s15_prof -o run -- python3 $R/bench.py > $OUT/s15_bench_prof.log 2>&1 || { tail -5 $OUT/s15_bench_prof.log; exit 5; }
tail -1 $OUT/s15_bench_prof.log > $OUT/s15_bench_c3.json
find $OUT/s15_prof -name '*stats*'
echo "== PMC"
cd $R
TAG=r06 step 900 bash tools/pmc_c3.sh > $OUT/s15_pmc.log 2>&1 || { tail -5 $OUT/s15_pmc.log; exit 6; }
tail -30 $OUT/s15_pmc.log
echo s15 done
