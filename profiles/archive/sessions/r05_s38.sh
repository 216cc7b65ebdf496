# GPU session 38 (round 5): the QT kernel's fixed cost per launch -- C3's
# and C4's rule sets on tiny batches (2^10, 2^14 packets) and mid ones, under
# rocprofv3 so that the kernel's own duration is seen apart from the count
# kernel and launch gaps
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
for c in c3 c4; do
	for l in 10 14 18 21; do
		timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s38_${c}_$l -o run -- \
			python3 $R/tools/bench_configs.py $c --log2-packets $l > $OUT/s38_${c}_$l.log 2>&1 || { tail -3 $OUT/s38_${c}_$l.log; exit 3; }
		f=$(find $OUT/s38_${c}_$l -name "*kernel_stats.csv" | head -1)
		echo "$c 2^$l events $(grep -o '"kernel_ms": [0-9.]*' $OUT/s38_${c}_$l.log): $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'pipeq' in r['Name'] or 'count' in r['Name'] or 'pipe4' in r['Name']: print(r['Name'].split('(')[0][-28:], r['Calls'], round(float(r['AverageNs'])/1e3,2), end='; ')
")"
	done
done
echo s38 done
