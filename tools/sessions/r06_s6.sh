# GPU session 6 (round 6): the LDS Ethernet key table inside the index
# kernel (Ethernet rules beside IPv4 rules keep path 5): the Ethernet and
# index-kernel GPU tests, C3e timing (C3 with a MAC map live), then the
# C5 host-path settings (zero copy alone against the hybrid rounds).
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s6
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== Ethernet + index-kernel tests"
step 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_eth.py tests/test_gpu_qt.py > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -3 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest.log | head -30; exit $rc; }
echo "== C3e / C3"
step 400 python3 tools/bench_configs.py c3e c3 > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-330
echo "== C5 host path"
XFG_LIB=diag step 900 python3 tools/hyb_c5.py 0:0 20:2 20:3 21:4 19:1 20:1 22:8 > $OUT/${T}_hyb.log 2>&1
rc=$?; cat $OUT/${T}_hyb.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
echo ${T} done
