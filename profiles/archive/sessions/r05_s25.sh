# GPU session 25 (round 5): checkpoint of the product library -- GPU suite,
# smoke, the bench line, its kernel-trace summary, the other configurations,
# PMC passes of C3 at the bench's batch (traffic) and of C1, C4, C5, C3 src|dst (two passes each)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=${T:-s25}
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== GPU suite"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/${T}_pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest_gpu.log | head -30; exit $rc; }
echo "== smoke"
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -5 $OUT/${T}_smoke.log; exit 4; }
tail -2 $OUT/${T}_smoke.log
echo "== bench"
step 400 python bench.py > $OUT/${T}_bench.log 2>&1 || { tail -20 $OUT/${T}_bench.log; exit 5; }
tail -1 $OUT/${T}_bench.log > $OUT/${T}_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/${T}_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'],d['roofline']['peak_measured_stream_read'],d.get('host_path',{}).get('registered_GBps_h2d'))"
echo "== kernel trace of the bench"
( cd /tmp && export TMPDIR=/tmp && step 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${T}_prof -o run -- \
	python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --host-log2-packets 0 ) > $OUT/${T}_prof.log 2>&1 || exit 6
f=$(find $OUT/${T}_prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/${T}_c3_bench_2p26_kernel_stats.csv; cut -d, -f1-4 $f | head -6 | cut -c1-160
echo "== configs"
step 900 python3 tools/bench_configs.py c2 c4 c5 c3sd c1 c3 > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-300
echo "== PMC C3 2^26"
TAG=${T}c3 bash tools/pmc_c3.sh > $OUT/${T}_pmc_c3.log 2>&1 || { tail -5 $OUT/${T}_pmc_c3.log; exit 8; }
cat $OUT/pmc_${T}c3.json
echo "== PMC configs"
cd /tmp && export TMPDIR=/tmp
for c in c1 c4 c5 c3sd; do
	extra=""; [ $c = c1 ] && extra="--no-cpu"
	step 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TD_TD_BUSY_sum TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
		--kernel-trace --output-format csv -d $OUT/pmc_${T}${c}_1 -o run -- python3 $R/tools/bench_configs.py $c $extra --iters 3 > $OUT/pmc_${T}${c}_1.log 2>&1 || { echo "pmc $c failed"; tail -3 $OUT/pmc_${T}${c}_1.log; exit 9; }
	step 300 rocprofv3 --pmc FETCH_SIZE \
		--kernel-trace --output-format csv -d $OUT/pmc_${T}${c}_2 -o run -- python3 $R/tools/bench_configs.py $c $extra --iters 3 > $OUT/pmc_${T}${c}_2.log 2>&1 || { echo "pmc $c failed"; tail -3 $OUT/pmc_${T}${c}_2.log; exit 9; }
	python3 $R/tools/pmc_summary.py --kernel pipe $OUT/pmc_${T}${c}_1 $OUT/pmc_${T}${c}_2 > $OUT/pmc_${T}${c}.json; echo "$c: $(tr -d '\n ' < $OUT/pmc_${T}${c}.json)"
done
echo ${T} done
