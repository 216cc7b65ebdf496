cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
XFG_LIB=$PWD/tools/abl/wc64n16.so timeout -k 10 200 python -u tools/ab_parity.py --hot 8 > gpurun_out/par_wc64n16.log 2>&1; tail -1 gpurun_out/par_wc64n16.log
SC="1000000:500:250 1000000:500:250:XFG_GRID_PER_CU=1"
for r in 1 2; do for v in base wc wc64 wc64n16 wc128; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC > gpurun_out/ab_s8_${v}_$r.log 2>&1 || exit 2
sed "s/^/$v r$r /" gpurun_out/ab_s8_${v}_$r.log | grep scenario
done; done
