# GPU session 21 (round 6): the final tree once more -- the whole GPU suite
# and smoke() (the diagnostics library gained phase stamps since r06_s16).
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/s21_pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/s21_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "^E |FAILED" $OUT/s21_pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/s21_smoke.log 2>&1 || { tail -5 $OUT/s21_smoke.log; exit 4; }
tail -1 $OUT/s21_smoke.log
echo s21 done
