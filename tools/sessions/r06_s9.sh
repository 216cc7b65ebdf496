# GPU session 9 (round 6): where a small launch's fixed cost goes -- the
# kernel trace (every dispatch, its start and end) of C3 and C4 at the
# per-GPU shard size 2^21, product library.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp
for c in c3 c4; do
	timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/s9_$c -o run -- python3 $R/tools/bench_configs.py $c --log2-packets 21 > $OUT/s9_$c.log 2>&1 || { tail -5 $OUT/s9_$c.log; exit 3; }
	grep '"config"' $OUT/s9_$c.log | cut -c1-250
done
find $OUT/s9_c3 $OUT/s9_c4 -name '*.csv' | head
echo s9 done
