# GPU session 32 (round 5): where C5's kernel time goes (diagnostics masks
# on the QT kernel, results wrong, timing only): 1 no counting (its hits are
# 64-bit atomics on the QT-order counts: no log at 2^23 packets), 2 no
# bucket loads, 2048 no deferred walk, 4096 counting by a scratch atomic
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
for r in 1 2; do
	for m in 0 1 2 2048; do
		XFG_LIB=diag XFG_DIAG_MASK=$m timeout -k 10 400 python3 tools/bench_configs.py c5 --no-host > $OUT/s32_c5_m${m}_$r.log 2>&1 || { tail -3 $OUT/s32_c5_m${m}_$r.log; exit 3; }
		echo "mask $m: $(grep -o '"kernel_ms": [0-9.]*' $OUT/s32_c5_m${m}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s32_c5_m${m}_$r.log)"
	done
done
echo s32 done
