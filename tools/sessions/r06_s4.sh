# GPU session 4 (round 6): the configurations on the product library
# (bench_configs: C2, C3 at 2^24, C4, C5 with its host paths, C3 src|dst,
# C1, and C3 beside 8 MAC rules -- the generic kernel's LDS Ethernet table),
# then C3 and C4 at the 8-way per-GPU shard sizes 2^21 / 2^22 with the
# count wave's log (product) and without it (diagnostics, XFG_CW=off: the
# LDS cache and atomics below twice the QT slots).
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
T=${T:-s4}
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
cd $R
echo "== configs"
step 900 python3 tools/bench_configs.py c2 c3 c4 c5 c3sd c1 c3e > $OUT/${T}_configs.log 2>&1 || { tail -5 $OUT/${T}_configs.log; exit 7; }
grep '"config"' $OUT/${T}_configs.log | cut -c1-330
echo "== per-GPU shard sizes"
for c in c3 c4; do
	for l in 21 22; do
		step 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/${T}_${c}_$l.log 2>&1 || exit 3
		echo "$c 2^$l cw $(grep -o '"kernel_path": [0-9]*, \|"kernel_ms": [0-9.]*' $OUT/${T}_${c}_$l.log | tr '\n' ' ') $(grep -o '"frac": [0-9.]*' $OUT/${T}_${c}_$l.log)"
		XFG_LIB=diag XFG_CW=off step 300 python3 tools/bench_configs.py $c --log2-packets $l > $OUT/${T}_${c}_${l}_off.log 2>&1 || exit 3
		echo "$c 2^$l off $(grep -o '"kernel_ms": [0-9.]*' $OUT/${T}_${c}_${l}_off.log) $(grep -o '"frac": [0-9.]*' $OUT/${T}_${c}_${l}_off.log)"
	done
done
echo ${T} done
