# GPU session 34 (round 5): which kernel the 32-bit QT-order counts slowed on
# C3 (2^24): rocprofv3 kernel summaries of both A/B libraries
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
for v in u64 u32; do
	XFG_LIB=$R/tools/abl/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s34_prof_$v -o run -- \
		python3 $R/tools/explore.py --log2-packets 24 --rounds 2 --iters 12 1000000:500:250 > $OUT/s34_prof_$v.log 2>&1 || exit 4
	echo "$v: $(grep scenario $OUT/s34_prof_$v.log | tail -1)"
	f=$(find $OUT/s34_prof_$v -name "*kernel_stats.csv" | head -1)
	python3 - "$f" <<'PY'
import csv, sys, re
for r in csv.DictReader(open(sys.argv[1])):
    nm = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:70]
    print(f'   {nm:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
PY
done
echo s34 done
