# GPU session 7 (round 6): the index kernel instantiated without its
# Ethernet lookups unless the LDS key table is live, and the key table's
# cheaper home function (24-bit multiplies): Ethernet and index-kernel
# tests, C1 / C3e / C3 / C2, the bench line.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=${T:-s7}
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== Ethernet + index-kernel tests"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_eth.py tests/test_gpu_qt.py > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest.log | head -30; exit $rc; }
echo "== configs"
step 500 python3 tools/bench_configs.py c1 c3e c3 c2 > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-300
echo "== bench"
step 400 python bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 5; }
tail -1 $OUT/${T}_bench.log > $OUT/${T}_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/${T}_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('host_path',{}))"
echo ${T} done
