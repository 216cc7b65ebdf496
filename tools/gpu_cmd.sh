cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
SC="1000000:500:250"
cd /tmp && export TMPDIR=/tmp
for m in 0 8192; do
XFG_LIB=$GRAFT_REPO_ROOT/tools/abl/rmw.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rmw$m -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/explore.py --log2-packets 26 --rounds 2 --iters 5 $SC:XFG_DIAG_MASK=$m > /dev/null 2>&1 || exit 3
f=$(find $GRAFT_REPO_ROOT/gpurun_out/prof_rmw$m -name "*kernel_stats.csv" | head -1); echo "mask $m"; cut -d, -f1-4 $f | grep -E "count"
done
