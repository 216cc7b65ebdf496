# GPU session 1 (round 5): where C3's time goes on the round-4 kernel.
#  1. index footprint: the same kernel over a 4 MB and a 2 MB quotient index
#     (A/B libraries ab17 / ab16: XFG_QT_MIN_BITS 17 / 16; 500k keys at 16 bits
#     keep the round-4 bucket density), kernel-trace summary per run
#  2. fixed costs: the product library at 2^20 .. 2^26 packets
#  3. stage isolation (diagnostics masks) at 2^26 and 2^24
#  4. PMC per mask: TCC hit/miss, LDS bank conflicts, TA/TD/TCP
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
ksum() {   # kernel name, avg us, calls from a kernel_stats.csv
	f=$(find "$1" -name "*kernel_stats.csv" | head -1)
	python3 - "$f" <<'EOF'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(xfg_\w+|__amd\w+)(<[^>]*>)?", r["Name"])
    nm = m.group(0) if m else r["Name"][:60]
    print(f'   {nm[:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
EOF
}
cd /tmp && export TMPDIR=/tmp
echo "== 1. index footprint (2^26, rocprof kernel trace)"
for v in ab17:1000000 ab16:500000 ab17:500000 ab16:1000000 ab17:1000000 ab16:500000; do
	lib=${v%%:*}; rules=${v##*:}; tag=s1_${lib}_${rules}_$RANDOM
	export XFG_LIB=$R/tools/abl/$lib.so
	step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
		python3 $R/tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $rules:500:250 > $OUT/$tag.log 2>&1 || exit 3
	echo "$lib $rules: $(grep scenario $OUT/$tag.log)"; ksum $OUT/$tag
done
echo "== 2. fixed costs (product library)"
export XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so
for lg in 20 22 24 26; do
	tag=s1_size_$lg
	step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
		python3 $R/tools/explore.py --log2-packets $lg --rounds 3 --iters 10 1000000:500:250 > $OUT/$tag.log 2>&1 || exit 4
	echo "2^$lg: $(grep scenario $OUT/$tag.log)"; ksum $OUT/$tag
done
echo "== 3. stage isolation (diagnostics library)"
export XFG_LIB=diag
M="0 1 2 8 16 128 2048 16384 2051 2059 10491 16402"
for lg in 26 24; do
	SC=""; for m in $M; do SC="$SC 1000000:500:250:XFG_DIAG_MASK=$m"; done
	step 300 python3 $R/tools/explore.py --log2-packets $lg --rounds 3 --iters 5 $SC > $OUT/s1_iso_$lg.log 2>&1 || exit 5
	echo "2^$lg"; grep scenario $OUT/s1_iso_$lg.log
done
echo "== 4. PMC per mask (2^26)"
export KNAME=pipeq
for m in 0 2 16384; do
	TAG=s1m$m bash $R/tools/pmc.sh s1m$m "--log2-packets 26 1000000:500:250:XFG_DIAG_MASK=$m" \
		"TCC_HIT_sum TCC_MISS_sum" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES" \
		"TD_TD_BUSY_sum TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" > $OUT/s1_pmc_$m.log 2>&1 || { echo "pmc $m failed"; tail -5 $OUT/s1_pmc_$m.log; exit 6; }
	echo "mask $m"; cat $OUT/pmc_s1m$m.json
done
echo s1 done
