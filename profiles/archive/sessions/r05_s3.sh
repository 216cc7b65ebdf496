# GPU session 3 (round 5): what one instruction per tile costs (A/B: 24
# extra VALU or SALU per tile), and the dynamic instruction mix per
# diagnostics mask (PMC, C3 at 2^24)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== instruction price (2^26)"
for r in 1 2; do
	for v in cur pv24 ps24; do
		XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets 26 --rounds 3 --iters 10 1000000:500:250 > $OUT/s3_pad_${v}_$r.log 2>&1 || exit 3
		sed "s/^/$v /" $OUT/s3_pad_${v}_$r.log | grep scenario
	done
done
echo "== PMC per mask (diagnostics library, 2^24)"
export XFG_LIB=diag KNAME=pipeq
for m in 0 1 2 8 16 128 8192 2051 10491; do
	bash $R/tools/pmc.sh s3m$m "--log2-packets 24 1000000:500:250:XFG_DIAG_MASK=$m" \
		"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" > $OUT/s3_pmc_$m.log 2>&1 || { echo "pmc $m failed"; tail -5 $OUT/s3_pmc_$m.log; exit 6; }
	echo "mask $m: $(python3 -c "import json;d=json.load(open('$OUT/pmc_s3m$m.json'));t=2**18;print({k.replace('SQ_',''):round(v/t,1) for k,v in d.items() if k.startswith('SQ_')}, d.get('kernel_ns_median_profiled'))")"
done
echo s3 done
