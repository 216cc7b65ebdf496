# GPU session 3 (round 6): the product library after this round's changes
# (IPv6 lookups beside both IPv4 directions, the LDS Ethernet table in the
# generic kernel, the packed bucket match, the count wave, the QT-order
# counts' second half for atomics): the whole GPU suite (with the new tests:
# the 2^32 fold on the product library, unaligned registered batches, the
# Ethernet table's long chains and 513th key), smoke, the bench line.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=${T:-s3}
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== GPU suite"
step 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/${T}_pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
echo "== smoke"
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -5 $OUT/${T}_smoke.log; exit 4; }
tail -2 $OUT/${T}_smoke.log
echo "== bench"
step 400 python bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 5; }
tail -1 $OUT/${T}_bench.log > $OUT/${T}_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/${T}_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'],d['roofline']['peak_measured_stream_read'],d.get('host_path',{}))"
T=s4
echo "== configs"
step 900 python3 tools/bench_configs.py c2 c3 c4 c5 c3sd c1 c3e > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-330
echo "== per-GPU shard sizes"
for c in c3 c4; do
	for l in 21 22; do
		step 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/${T}_${c}_$l.log 2>&1 || exit 3
		echo "$c 2^$l cw $(grep -o '"kernel_path": [0-9]*, \|"kernel_ms": [0-9.]*' $OUT/${T}_${c}_$l.log | tr '\n' ' ') $(grep -o '"frac": [0-9.]*' $OUT/${T}_${c}_$l.log)"
		XFG_LIB=diag XFG_CW=off step 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/${T}_${c}_${l}_off.log 2>&1 || exit 3
		echo "$c 2^$l off $(grep -o '"kernel_ms": [0-9.]*' $OUT/${T}_${c}_${l}_off.log) $(grep -o '"frac": [0-9.]*' $OUT/${T}_${c}_${l}_off.log)"
	done
done
echo ${T} done
