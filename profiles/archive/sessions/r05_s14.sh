# GPU session 14 (round 5): where the 16-byte-bucket index (q9) loses to the
# 32-byte one (cnt2) at 2^26: diagnostics masks (1 no counting, 2048 no
# deferred pass) and per-kernel times under rocprofv3
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
for r in 1 2; do
	for v in cnt2 q9; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets 26 --rounds 3 --iters 8 1000000:500:250 1000000:500:250:XFG_DIAG_MASK=1 1000000:500:250:XFG_DIAG_MASK=2048 1000000:500:250:XFG_DIAG_MASK=2049 > $OUT/s14_${v}_$r.log 2>&1 || exit 3
		sed "s/^/$v /" $OUT/s14_${v}_$r.log | grep scenario
	done
done
cd /tmp && export TMPDIR=/tmp
for v in cnt2 q9; do
	XFG_LIB=$R/tools/abl/$v.so step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s14_prof_$v -o run -- \
		python3 $R/tools/explore.py --log2-packets 26 --rounds 2 --iters 12 1000000:500:250 > $OUT/s14_prof_$v.log 2>&1 || exit 4
	echo "$v: $(grep scenario $OUT/s14_prof_$v.log)"; ksum $OUT/s14_prof_$v
done
echo s14 done
