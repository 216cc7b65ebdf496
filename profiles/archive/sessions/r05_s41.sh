# GPU session 41 (round 5): C2 (1k IPv4 rules) on the IPv4-key kernel (its
# default) against the quotient-index kernel forced on (XFG_QT=on), and the
# IPv4-key kernel without counting / Bloom loads (masks 1, 4; timing only)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
for r in 1 2; do
	for sc in default qt m1; do
		case $sc in default) E="";; qt) E="XFG_QT=on";; m1) E="XFG_DIAG_MASK=1";; esac
		env XFG_LIB=diag $E timeout -k 10 300 python3 tools/bench_configs.py c2 > $OUT/s41_c2_${sc}_$r.log 2>&1 || { tail -3 $OUT/s41_c2_${sc}_$r.log; exit 3; }
		echo "$sc $(grep -o '"kernel_ms": [0-9.]*' $OUT/s41_c2_${sc}_$r.log) $(grep -o '"frac": [0-9.]*' $OUT/s41_c2_${sc}_$r.log)"
	done
done
echo s41 done
