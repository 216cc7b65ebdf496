cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/pytest_s22.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_s22.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s22.log | head -20; exit $rc; }
timeout -k 10 600 python -u tools/bench_configs.py c4 c5 c3sd c2 > gpurun_out/configs_s22.log 2>&1 || { tail -20 gpurun_out/configs_s22.log; exit 1; }
grep "^{" gpurun_out/configs_s22.log | cut -c1-330
