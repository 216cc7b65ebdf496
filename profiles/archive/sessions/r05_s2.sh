# GPU session 2 (round 5): the fixed-cost and instruction cuts against round 4
#  (base: HEAD of round 4; cur: this tree -- hit logs of 4 launches per count
#  kernel, packed per-lane stats, hit-log chunks moved every other iteration,
#  the workgroup-end partition flush as 8-byte copies), parity first, then
#  same-box A/B at 2^26 and 2^24, a kernel-trace summary, then the GPU suite
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
ksum() {
	f=$(find "$1" -name "*kernel_stats.csv" | head -1)
	python3 - "$f" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(xfg_\w+|__amd\w+)(<[^>]*>)?", r["Name"])
    nm = m.group(0) if m else r["Name"][:60]
    print(f'   {nm[:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
}
cd $R
echo "== parity (A/B library cur)"
for args in "" "--src-dst" "--hot 8" "--log2-packets 24"; do
	XFG_LIB=$R/tools/abl/cur.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== A/B timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in base cur; do
			SC="1000000:500:250"; [ $v = cur ] && SC="$SC 1000000:500:250:XFG_LOG_PEND=1"
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 $SC > $OUT/s2_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s2_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo "== kernel trace (cur, 2^26 and 2^24)"
cd /tmp && export TMPDIR=/tmp
for lg in 26 24; do
	XFG_LIB=$R/tools/abl/cur.so step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s2_prof_$lg -o run -- \
		python3 $R/tools/explore.py --log2-packets $lg --rounds 2 --iters 12 1000000:500:250 > $OUT/s2_prof_$lg.log 2>&1 || exit 4
	echo "2^$lg: $(grep scenario $OUT/s2_prof_$lg.log)"; ksum $OUT/s2_prof_$lg
done
cd $R
echo "== GPU suite (product library)"
step 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/s2_pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/s2_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s2_pytest_gpu.log | head -30; exit $rc; }
echo "== bench"
step 400 python bench.py > $OUT/s2_bench.log 2>&1 || { tail -20 $OUT/s2_bench.log; exit 5; }
tail -1 $OUT/s2_bench.log | cut -c1-600
echo s2 done
