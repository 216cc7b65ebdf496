# GPU session 48 (round 5): after the library-selection check in xfgpu.py --
#  the quotient-index tests (one runs the diagnostics library in a worker),
#  the Ethernet-key tests and smoke()
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s48
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_qt.py tests/test_gpu_eth.py > $OUT/${T}_pytest.log 2>&1
rc=$?; tail -2 $OUT/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $OUT/${T}_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${T}_smoke.log 2>&1 || { tail -5 $OUT/${T}_smoke.log; exit 4; }
tail -1 $OUT/${T}_smoke.log
echo ${T} done
