# GPU session 14 (round 6): the tree after the dynamic tiles -- the whole GPU
# suite, smoke(), the bench line, every configuration, and the dynamic
# tiles' A/B (diagnostics library, XFG_QT_DYN_MIN 0 against 2^40) on C4 and
# C5 at 2^23 and C3 src|dst at 2^24.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=${T:-s14}
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
rc=$?; tail -3 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
echo "== smoke"
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -5 $OUT/${T}_smoke.log; exit 4; }
tail -2 $OUT/${T}_smoke.log
echo "== bench"
step 400 python bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 5; }
tail -1 $OUT/${T}_bench.log > $OUT/${T}_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/${T}_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('host_path',{}).get('registered_Mpps'))"
echo "== configs"
step 600 python3 tools/bench_configs.py c2 c3 c4 c5 c3sd c1 c3e > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-300
echo "== dynamic tiles A/B"
for r in 1 2; do
	for c in "c4" "c5 --no-host" "c3sd"; do
		for m in 1099511627776 0; do
			XFG_LIB=diag XFG_QT_DYN_MIN=$m step 300 python3 tools/bench_configs.py $c > $OUT/${T}_dyn.log 2>&1 || exit 8
			echo "$c dyn_min $m $(grep -o '"kernel_ms": [0-9.]*' $OUT/${T}_dyn.log) $(grep -o '"frac": [0-9.]*' $OUT/${T}_dyn.log)"
		done
	done
done
echo ${T} done
