cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
bash tools/r03_measure.sh m2 || exit $?
SC="1000000:500:250"
XFG_LIB=$PWD/tools/abl/final.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC $SC:XFG_DIAG_MASK=2048 $SC:XFG_DIAG_MASK=16 $SC:XFG_DIAG_MASK=1 $SC:XFG_DIAG_MASK=2051 $SC:XFG_DIAG_MASK=1024 > gpurun_out/explore_final_m2.log 2>&1 || exit 5
grep scenario gpurun_out/explore_final_m2.log
