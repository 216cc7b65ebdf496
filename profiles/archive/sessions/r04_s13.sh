cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_a0_gpu_multirank.py tests/test_gpu_io.py tests/test_gpu_configs.py tests/test_gpu_qt.py > gpurun_out/pytest_s13.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "passed|failed" gpurun_out/pytest_s13.log | tail -2; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" gpurun_out/pytest_s13.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 20 --no-cpu > gpurun_out/bench_s13.log 2>&1 || exit 3; python3 -c "
import json;d=json.loads(open('gpurun_out/bench_s13.log').read().strip().split(chr(10))[-1]);print('bench',d['ms_per_step'],d['roofline']['frac'],d['host_path'])"
for o in "" "--hot 8" "--src-dst"; do
XFG_LIB=$PWD/tools/abl/lag2.so timeout -k 10 200 python -u tools/ab_parity.py $o > gpurun_out/par_lag2.log 2>&1; tail -1 gpurun_out/par_lag2.log
done
TAG=s13 VARIANTS="lag1 lag2" ROUNDS=3 bash tools/r04_ab.sh
bash tools/r04_pmc.sh
for r in 1 2; do for v in c4base c4nw8; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/bench_configs.py c4 > gpurun_out/c4_${v}_$r.log 2>&1; grep config gpurun_out/c4_${v}_$r.log | cut -c1-200 | sed "s/^/$v r$r /"
done; done
timeout -k 10 300 python -u tools/edit_latency.py > gpurun_out/edit_latency.log 2>&1; tail -1 gpurun_out/edit_latency.log
XFG_LIB=diag XFG_QT_PATCH=off timeout -k 10 300 python -u tools/edit_latency.py > gpurun_out/edit_latency_rebuild.log 2>&1; tail -1 gpurun_out/edit_latency_rebuild.log
timeout -k 10 400 python -u tools/bench_configs.py c5 c3sd c3 > gpurun_out/cfg_s13.log 2>&1; grep config gpurun_out/cfg_s13.log | cut -c1-400
