cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_s15.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_s15.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s15.log | head -20; exit $rc; }
SC="1000000:500:250"
for r in 1 2; do
for v in q32p3 q32m; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC $SC:XFG_DIAG_MASK=2048 > gpurun_out/explore_${v}_s15_$r.log 2>&1 || exit 2
sed "s/^/$v /" gpurun_out/explore_${v}_s15_$r.log | grep scenario
done; done
