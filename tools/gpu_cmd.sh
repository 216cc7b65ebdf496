cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s30_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/s30_pytest_gpu.log; exit 2; }
tail -2 gpurun_out/s30_pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s30_smoke.log 2>&1 || { tail -20 gpurun_out/s30_smoke.log; exit 3; }
tail -1 gpurun_out/s30_smoke.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py > gpurun_out/s30_bench_$r.json 2> gpurun_out/s30_bench_$r.err || exit 4
cat gpurun_out/s30_bench_$r.json
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/s30_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py > $GRAFT_REPO_ROOT/gpurun_out/s30_prof.log 2>&1 || exit 5
find $GRAFT_REPO_ROOT/gpurun_out/s30_prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200
