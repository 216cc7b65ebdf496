# GPU session 1 (round 6): where C3's fixed cost per launch goes.
#  1. the product library at 2^21 .. 2^26 packets under a kernel trace: the
#     QT kernel's and the count kernel's duration per size (the intercept)
#  2. the count kernel with its stages removed (diagnostics library; results
#     wrong): 65536 slices loaded but not added, 131072 no slice read,
#     8192 no counter read-modify-write -- at 2^24 and 2^26
#  3. SQ counters of the count kernel at 2^24
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
    if nm.startswith("__amd"):
        continue
    print(f'   {nm[:70]:70s} calls={r["Calls"]:>5s} avg_us={float(r["AverageNs"])/1e3:9.2f}')
EOF
}
cd /tmp && export TMPDIR=/tmp
echo "== 1. batch sweep (product library)"
export XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so
for lg in 21 22 23 24 25 26; do
	tag=s1_size_$lg
	step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
		python3 $R/tools/explore.py --log2-packets $lg --rounds 3 --iters 8 1000000:500:250 > $OUT/$tag.log 2>&1 || exit 4
	echo "2^$lg: $(grep scenario $OUT/$tag.log)"; ksum $OUT/$tag
done
echo "== 2. count-kernel stages (diagnostics library)"
export XFG_LIB=diag
for lg in 24 26; do
	for m in 0 65536 131072 139264; do
		tag=s1_cnt_${lg}_$m
		step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- \
			python3 $R/tools/explore.py --log2-packets $lg --rounds 2 --iters 8 1000000:500:250:XFG_DIAG_MASK=$m > $OUT/$tag.log 2>&1 || exit 5
		echo "2^$lg mask $m: $(grep scenario $OUT/$tag.log)"; ksum $OUT/$tag
	done
done
echo "== 3. count-kernel SQ counters (2^24)"
export XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so
step 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
	--kernel-trace --output-format csv -d $OUT/pmc_s1cnt -o run -- python3 $R/tools/explore.py --rounds 1 --iters 8 --log2-packets 24 1000000:500:250 > $OUT/pmc_s1cnt.log 2>&1 || exit 9
python3 $R/tools/pmc_summary.py --kernel count $OUT/pmc_s1cnt > $OUT/pmc_s1cnt.json; echo "count: $(tr -d '\n ' < $OUT/pmc_s1cnt.json)"
echo s1 done
