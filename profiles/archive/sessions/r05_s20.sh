# GPU session 20 (round 5): what bounds C1 (the Ethernet-key program on the
# generic pipelined kernel) -- kernel time at 2^22/2^24/2^26 packets (fixed
# cost vs per-packet), then PMC passes of the kernel at 2^24 (issue, waits,
# memory path, fetched bytes)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== C1 sizes"
for l in 22 24 26; do
	step 300 python3 tools/bench_configs.py c1 --no-cpu --log2-packets $l > $OUT/s20_c1_$l.log 2>&1 || { tail -3 $OUT/s20_c1_$l.log; exit 3; }
	grep '"config"' $OUT/s20_c1_$l.log
done
echo "== C1 PMC"
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
	 "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" \
	 "TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
	 "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
	i=$((i+1))
	timeout -s KILL 120 rocprofv3 --pmc $g --kernel-trace --output-format csv -d $OUT/pmc_s20c1_$i -o run -- \
		python3 $R/tools/bench_configs.py c1 --no-cpu --iters 3 > $OUT/pmc_s20c1_$i.log 2>&1
	rc=$?; echo "pmc[$g] rc=$rc"; [ $rc -ne 0 ] && exit 9
done
python3 $R/tools/pmc_summary.py --kernel pipeline $OUT/pmc_s20c1_* > $OUT/pmc_s20c1.json; cat $OUT/pmc_s20c1.json
echo s20 done
