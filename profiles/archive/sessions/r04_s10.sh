cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s10 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu --host-log2-packets 0) > gpurun_out/prof_s10.log 2>&1; echo prof rc=$?
find gpurun_out/prof_s10 -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -6
TAG=s10 VARIANTS="wf64 wf32 r256" ROUNDS=2 bash tools/r04_ab.sh
