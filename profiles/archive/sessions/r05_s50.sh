# GPU session 50 (round 5): instruction counts of C3 and C3 src|dst (2^24,
#  product library, one rocprofv3 --pmc pass of 8 SQ counters each) -- what
#  the second IPv4 direction adds per tile
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s50
cd /tmp && export TMPDIR=/tmp
for c in c3 c3sd; do
	timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
		--kernel-trace --output-format csv -d $OUT/pmc_${T}${c} -o run -- python3 $R/tools/bench_configs.py $c --iters 3 > $OUT/pmc_${T}${c}.log 2>&1 || { echo "pmc $c failed"; tail -3 $OUT/pmc_${T}${c}.log; exit 9; }
	python3 $R/tools/pmc_summary.py --kernel pipeq $OUT/pmc_${T}${c} > $OUT/pmc_${T}${c}.json; echo "$c: $(tr -d '\n ' < $OUT/pmc_${T}${c}.json)"
done
echo ${T} done
