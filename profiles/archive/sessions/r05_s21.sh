# GPU session 21 (round 5): the Ethernet-key kernel (xfg_pipee.hip, path 6)
# -- its parity tests and the configuration tests, then C1 at 2^22/2^24/2^26
# against the generic pipelined kernel (diagnostics library, XFG_EK=off)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_eth.py tests/test_gpu_configs.py tests/test_gpu.py > $OUT/s21_pytest.log 2>&1
rc=$?; tail -2 $OUT/s21_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/s21_pytest.log | head -30; exit $rc; }
echo "== C1"
for l in 22 24 26; do
	for r in 1 2; do
		step 300 python3 tools/bench_configs.py c1 --no-cpu --log2-packets $l > $OUT/s21_c1_${l}_$r.log 2>&1 || { tail -3 $OUT/s21_c1_${l}_$r.log; exit 3; }
		echo "ek  $(grep '"config"' $OUT/s21_c1_${l}_$r.log)"
		XFG_LIB=diag XFG_EK=off step 300 python3 tools/bench_configs.py c1 --no-cpu --log2-packets $l > $OUT/s21_c1off_${l}_$r.log 2>&1 || { tail -3 $OUT/s21_c1off_${l}_$r.log; exit 3; }
		echo "gen $(grep '"config"' $OUT/s21_c1off_${l}_$r.log)"
	done
done
echo "== C1 PMC (2^24)"
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
	 "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
	 "FETCH_SIZE"; do
	i=$((i+1))
	timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/pmc_s21c1_$i -o run -- \
		python3 $R/tools/bench_configs.py c1 --no-cpu --iters 3 > $OUT/pmc_s21c1_$i.log 2>&1
	rc=$?; echo "pmc[$g] rc=$rc"; [ $rc -ne 0 ] && exit 9
done
python3 $R/tools/pmc_summary.py --kernel pipee $OUT/pmc_s21c1_* > $OUT/pmc_s21c1.json; cat $OUT/pmc_s21c1.json
echo s21 done
