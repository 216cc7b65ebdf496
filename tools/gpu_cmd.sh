cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_scale.py tests/test_gpu_configs.py tests/test_gpu.py > gpurun_out/pytest_s25.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_s25.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s25.log | head -20; exit $rc; }
SC="1000000:500:250"
for r in 1 2 3; do
for v in wo0 wo1; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC $SC:XFG_DIAG_MASK=16 > gpurun_out/explore_${v}_s25_$r.log 2>&1 || exit 2
sed "s/^/$v /" gpurun_out/explore_${v}_s25_$r.log | grep scenario
done; done
