cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s18.log 2>&1 || { tail gpurun_out/smoke_s18.log; exit 1; }
tail -1 gpurun_out/smoke_s18.log
timeout -k 10 400 python -u bench.py --gpus 2 --one-device --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_w2_s18.log 2>&1; echo "rc=$?"
tail -3 gpurun_out/bench_w2_s18.log | cut -c1-600
