# GPU session 39 (round 5): the hit log against LDS cache + atomics near the
# log's threshold (batch = the QT slots, 2^21 for 1M rules): C3 and C4 at
# 2^21 and 2^22 with the diagnostics library, XFG_LOG=off against on
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
for r in 1 2; do
	for c in c3 c4; do
		for l in 21 22 23; do
			for lg in on off; do
				E=""; [ $lg = off ] && E="XFG_LOG=off"
				env XFG_LIB=diag $E timeout -k 10 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/s39_${c}_${l}_$lg.log 2>&1 || { tail -3 $OUT/s39_${c}_${l}_$lg.log; exit 3; }
				echo "$c 2^$l log=$lg $(grep -o '"kernel_ms": [0-9.]*' $OUT/s39_${c}_${l}_$lg.log)"
			done
		done
	done
done
echo s39 done
