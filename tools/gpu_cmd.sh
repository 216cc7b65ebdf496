cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
SC="1000000:500:250"
for r in 1 2 3; do
for v in nw8 nw4; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC $SC:XFG_DIAG_MASK=16 > gpurun_out/explore_${v}_s29_$r.log 2>&1 || exit 2
sed "s/^/$v /" gpurun_out/explore_${v}_s29_$r.log | grep scenario
done; done
