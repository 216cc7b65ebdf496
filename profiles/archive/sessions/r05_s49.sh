# GPU session 49 (round 5): where C3 src|dst's time goes -- the diagnostics
#  library with stage masks (results wrong with a mask): none, 1 no counting,
#  2 no bucket loads, 16 no workgroup-end flush, 2048 no deferred walk; C3
#  (dst only) beside it for the same masks
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=s49
cd $R
for m in 0 1 2 16 2048; do
	for c in c3sd c3; do
		XFG_LIB=diag XFG_DIAG_MASK=$m timeout -k 10 300 python3 tools/bench_configs.py $c > $OUT/${T}_${c}_$m.log 2>&1 || { tail -5 $OUT/${T}_${c}_$m.log; exit 3; }
		echo "mask $m $c: $(grep '"config"' $OUT/${T}_${c}_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["kernel_ms"], d["roofline"]["frac"])')"
	done
done
echo ${T} done
