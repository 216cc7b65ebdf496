# GPU session 18 (round 6): the rebuilt final libraries (smoke, the
# index-kernel tests, the bench line), then PMC passes of this round's
# kernels on C1, C4, C5 (device leg) and C3 src|dst, one rocprofv3 --pmc
# run per counter group (tools/pmc_summary.py: per launch).
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== smoke + index-kernel tests + bench"
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/s18_smoke.log 2>&1 || { tail -5 $OUT/s18_smoke.log; exit 4; }
tail -1 $OUT/s18_smoke.log
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_eth.py > $OUT/s18_pytest.log 2>&1 || { grep -E "^E |FAILED" $OUT/s18_pytest.log | head; exit 2; }
tail -1 $OUT/s18_pytest.log
step 400 python bench.py > $OUT/s18_bench.log 2>&1 || { tail -20 $OUT/s18_bench.log; exit 5; }
tail -1 $OUT/s18_bench.log > $OUT/s18_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/s18_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
echo "== PMC"
cd /tmp && export TMPDIR=/tmp
for cfg in "c1:pipee" "c4:pipeq" "c5 --no-host:pipeq" "c3sd:pipeq"; do
	c=${cfg%%:*}; k=${cfg##*:}; tag=$(echo $c | cut -d' ' -f1)
	i=0
	for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES"; do
		i=$((i+1))
		timeout -s KILL 150 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d $OUT/pmc_s18_${tag}_$i -o run -- \
			python3 $R/tools/bench_configs.py $c --iters 3 > $OUT/pmc_s18_${tag}_$i.log 2>&1
		rc=$?; echo "$tag pmc[$pmc] rc=$rc"; [ $rc -ne 0 ] && exit $rc
	done
	python3 $R/tools/pmc_summary.py --kernel $k $OUT/pmc_s18_${tag}_* > $OUT/r06_s18_${tag}_pmc.json 2>&1
	python3 -c "import json;d=json.load(open('$OUT/r06_s18_${tag}_pmc.json'));print('$tag',{k:d.get(k) for k in ('FETCH_SIZE','WRITE_SIZE','TCC_HIT_sum','TCC_MISS_sum','SQ_INSTS_VALU','kernel_ns_median_profiled')})"
done
echo s18 done
