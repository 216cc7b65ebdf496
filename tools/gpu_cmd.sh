cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
SC="1000000:500:250"
for r in 1 2; do
for v in lc8 lc16; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC > gpurun_out/explore_${v}_s17_$r.log 2>&1 || exit 2
sed "s/^/$v /" gpurun_out/explore_${v}_s17_$r.log | grep scenario
done; done
cd /tmp && export TMPDIR=/tmp
for v in lc8 lc16; do
XFG_LIB=$GRAFT_REPO_ROOT/tools/abl/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/explore.py --log2-packets 26 --rounds 1 --iters 5 $SC > /dev/null 2>&1 || exit 3
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_$v -name "*kernel_stats.csv" | head -1); echo "$v"; cut -d, -f1-4 $f | grep -E "pipeq|count"
done
