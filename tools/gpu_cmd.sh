cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/bench_configs.py c5 > gpurun_out/configs_c5_s19.log 2>&1 || { tail -20 gpurun_out/configs_c5_s19.log; exit 1; }
grep "^{" gpurun_out/configs_c5_s19.log
