cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
for v in wc; do for h in 0 8; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 200 python -u tools/ab_parity.py --hot $h > gpurun_out/par_${v}_$h.log 2>&1; tail -1 gpurun_out/par_${v}_$h.log
done; done
XFG_LIB=$PWD/tools/abl/wc.so timeout -k 10 200 python -u tools/ab_parity.py --src-dst > gpurun_out/par_wc_sd.log 2>&1; tail -1 gpurun_out/par_wc_sd.log
TAG=s7 VARIANTS="base wc wc64" ROUNDS=2 bash tools/r04_ab.sh
