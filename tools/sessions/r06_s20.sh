# GPU session 20 (round 6): the last workgroup barrier of the QT kernel
# waiting for LDS work only (XFG_QT_LBAR): parity (product library, several
# sizes and shapes), the index-kernel tests, same-box A/B (lbar1 / lbar0,
# C3's program only) at 2^26 / 2^24 / 2^21, the phases, the bench line.
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
for args in "--reps 3" "--reps 4 --src-dst" "--reps 3 --hot 8" "--reps 3 --log2-packets 24" "--reps 2 --log2-packets 26"; do
	XFG_LIB=$R/xdp-tools_amd/lib/libxdpfilter_gpu.so step 300 python3 tools/ab_parity.py $args > $OUT/s20_par.log 2>&1
	rc=$?; grep -v amdgpu.ids $OUT/s20_par.log | tail -1; [ $rc -eq 0 ] || exit 2
done
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_eth.py > $OUT/s20_pytest.log 2>&1 || { grep -E "^E |FAILED" $OUT/s20_pytest.log | head; exit 2; }
tail -1 $OUT/s20_pytest.log
echo "== A/B timing"
for r in 1 2; do
	for lg in 26 24 21; do
		for v in lbar0 lbar1; do
			XFG_LIB=$R/tools/abl/$v.so step 300 python3 tools/explore.py --log2-packets $lg --rounds 3 --iters 10 \
				1000000:500:250 > $OUT/s20_ab.log 2>&1 || exit 3
			sed "s/^/$v 2^$lg /" $OUT/s20_ab.log | grep scenario
		done
	done
done
echo "== phases"
XFG_LIB=diag step 400 python3 tools/qt_phases.py c3 24 > $OUT/s20_ph.log 2>&1 || { tail -5 $OUT/s20_ph.log; exit 5; }
grep '"config"' $OUT/s20_ph.log | tee $OUT/s20_phases.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k:d[k] for k in ('span_us','loop_last_wave','defer_walk','fold','partition_flush','flush','end') if k in d})"
echo "== bench"
step 400 python bench.py > $OUT/s20_bench.log 2>&1 || { tail -20 $OUT/s20_bench.log; exit 5; }
tail -1 $OUT/s20_bench.log > $OUT/s20_bench_c3.json; python3 -c "import json;d=json.load(open('$OUT/s20_bench_c3.json'));print(d['ms_per_step'],d['roofline']['frac'],d['roofline']['kernel_ms'])"
echo s20 done
