cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qt.py > gpurun_out/pytest_s5.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s5.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s5.log | head -20; exit $rc; }
XFG_LIB=$PWD/tools/abl/late.so timeout -k 10 200 python -u tools/ab_parity.py > gpurun_out/par_late.log 2>&1; tail -1 gpurun_out/par_late.log
timeout -k 10 300 python -u tools/bench_configs.py c3sd c3 > gpurun_out/cfg_s5.log 2>&1 || exit 3; grep config gpurun_out/cfg_s5.log
TAG=s5 VARIANTS="base late" ROUNDS=3 bash tools/r04_ab.sh
