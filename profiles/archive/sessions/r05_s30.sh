# GPU session 30 (round 5): the QT kernel with the row-store lane swizzle
# (XFG_QT_SWZ: 8 lanes write one piece of 8 consecutive rows, no bank
# conflict) against the current one -- parity, timing at 2^26 and 2^24,
# and the LDS / TA counters of each
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== parity (qtswz)"
for args in "" "--src-dst" "--hot 8" "--log2-packets 24"; do
	XFG_LIB=$R/tools/abl/qtswz.so step 300 python3 tools/ab_parity.py $args || exit 2
done
echo "== A/B timing"
for lg in 26 24; do
	for r in 1 2; do
		for v in qtcur qtswz; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 1000000:500:250 > $OUT/s30_ab_${v}_${lg}_$r.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s30_ab_${v}_${lg}_$r.log | grep scenario
		done
	done
done
echo "== PMC"
cd /tmp && export TMPDIR=/tmp
for v in qtcur qtswz; do
	XFG_LIB=$R/tools/abl/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
		--kernel-trace --output-format csv -d $OUT/pmc_s30$v -o run -- python3 $R/tools/explore.py --rounds 1 --iters 3 --log2-packets 26 1000000:500:250 > $OUT/pmc_s30$v.log 2>&1 || exit 9
	python3 $R/tools/pmc_summary.py --kernel pipeq $OUT/pmc_s30$v > $OUT/pmc_s30$v.json; echo "$v: $(tr -d '\n ' < $OUT/pmc_s30$v.json)"
done
echo s30 done
