# GPU session 26 (round 5): C5's device-resident leg alone under PMC (the
# checkpoint's pass also caught its host leg), and what C2's lookups cost on
# the IPv4-key kernel (diagnostics masks: 4 no Bloom loads, 2 no bucket
# lines, 6 neither; results wrong, timing only)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s26
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== C2 lookup cost (diagnostics library)"
for r in 1 2; do
	for m in 0 4 2 6; do
		XFG_LIB=diag XFG_DIAG_MASK=$m step 300 python3 tools/bench_configs.py c2 > $OUT/${T}_c2_m${m}_$r.log 2>&1 || { tail -3 $OUT/${T}_c2_m${m}_$r.log; exit 3; }
		echo "mask $m: $(grep -o '"kernel_ms": [0-9.]*' $OUT/${T}_c2_m${m}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/${T}_c2_m${m}_$r.log)"
	done
done
echo "== PMC C5 (device leg)"
cd /tmp && export TMPDIR=/tmp
step 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TD_TD_BUSY_sum TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
	--kernel-trace --output-format csv -d $OUT/pmc_${T}c5_1 -o run -- python3 $R/tools/bench_configs.py c5 --no-host --iters 3 > $OUT/pmc_${T}c5_1.log 2>&1 || { tail -3 $OUT/pmc_${T}c5_1.log; exit 9; }
step 300 rocprofv3 --pmc FETCH_SIZE \
	--kernel-trace --output-format csv -d $OUT/pmc_${T}c5_2 -o run -- python3 $R/tools/bench_configs.py c5 --no-host --iters 3 > $OUT/pmc_${T}c5_2.log 2>&1 || { tail -3 $OUT/pmc_${T}c5_2.log; exit 9; }
python3 $R/tools/pmc_summary.py --kernel pipe $OUT/pmc_${T}c5_1 $OUT/pmc_${T}c5_2 > $OUT/pmc_${T}c5.json; cat $OUT/pmc_${T}c5.json
echo ${T} done
