# GPU session 46 (round 5): the tree with the masked count-kernel loads -- GPU suite, smoke, bench line
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s46
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== GPU suite"
step 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/${T}_pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
echo "== smoke"
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -5 $OUT/${T}_smoke.log; exit 4; }
tail -1 $OUT/${T}_smoke.log
echo "== bench"
step 400 python bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 5; }
tail -1 $OUT/${T}_bench.log > $OUT/${T}_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/${T}_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'],d['roofline']['peak_measured_stream_read'],d['host_path']['registered_GBps_h2d'],d['host_path']['Mpps'])"
echo ${T} done
