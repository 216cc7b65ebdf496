# GPU session 44 (round 5): the count kernel loads each hit-log slice 2, 4 or 8
#  entries a lane by its fill (fewer LDS atomics for short slices) -- parity,
#  same-box A/B at 2^24 and 2^26, kernel traces at 2^24, stage costs at
#  2^24 (diagnostics masks), and the hit-log tests
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s44
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
for args in "" "--src-dst" "--hot 8" "--log2-packets 24" "--log2-packets 24 --src-dst" "--log2-packets 22" "--log2-packets 23 --hot 8"; do
	XFG_LIB=$R/tools/abl/cur.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== A/B timing"
for lg in 24 26; do
	for r in 1 2; do
		for v in base cur; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 1000000:500:250 > $OUT/${T}_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/${T}_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo "== kernel trace (2^24)"
cd /tmp && export TMPDIR=/tmp
for v in base cur; do
	XFG_LIB=$R/tools/abl/$v.so step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${T}_prof_$v -o run -- \
		python3 $R/tools/explore.py --log2-packets 24 --rounds 2 --iters 12 1000000:500:250 > $OUT/${T}_prof_$v.log 2>&1 || exit 4
	echo "$v: $(grep scenario $OUT/${T}_prof_$v.log)"; ksum $OUT/${T}_prof_$v
done
cd $R
echo "== stage costs at 2^24 (diagnostics library; results wrong with a mask)"
XFG_LIB=diag step 300 python3 tools/explore.py --log2-packets 24 --rounds 3 --iters 10 1000000:500:250 1000000:500:250:XFG_DIAG_MASK=16 1000000:500:250:XFG_DIAG_MASK=2048 1000000:500:250:XFG_DIAG_MASK=1 1000000:500:250:XFG_DIAG_MASK=2 > $OUT/${T}_masks.log 2>&1 || exit 5
grep scenario $OUT/${T}_masks.log
echo "== hit-log tests (product library)"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py > $OUT/${T}_pytest_qt.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest_qt.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest_qt.log | head -30; exit $rc; }
echo ${T} done
