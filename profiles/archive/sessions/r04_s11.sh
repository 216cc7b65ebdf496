cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > gpurun_out/pytest_s11.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s11.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_s11.log | head -20; exit $rc; }
for r in 1 2; do
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu --host-log2-packets 0 > gpurun_out/bench_s11_$r.log 2>&1 || exit 3; python3 -c "
import json;d=json.loads(open('gpurun_out/bench_s11_$r.log').read().strip().split(chr(10))[-1]);print('bench',d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline']['frac'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s11 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu --host-log2-packets 0) > gpurun_out/prof_s11.log 2>&1; echo prof rc=$?
find gpurun_out/prof_s11 -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -4
