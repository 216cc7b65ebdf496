cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s9.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s9.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s9.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu --host-log2-packets 0 > gpurun_out/bench_s9.log 2>&1 || exit 3; tail -1 gpurun_out/bench_s9.log | cut -c1-700
timeout -k 10 400 python -u tools/bench_configs.py c3 c3sd c2 c4 c1 > gpurun_out/cfg_s9.log 2>&1 || exit 4; grep config gpurun_out/cfg_s9.log | cut -c1-300
TAG=s9 VARIANTS="wcm4 wcm2" ROUNDS=2 bash tools/r04_ab.sh
