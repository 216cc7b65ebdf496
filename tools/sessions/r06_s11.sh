# GPU session 11 (round 6): the index kernel's per-workgroup phases by XCD
# (is the spread of the workgroups' ends systematic?) -- C3 at 2^24, 2^26.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
export XFG_LIB=diag
for a in "c3 24" "c3 26"; do
	timeout -k 10 400 python3 tools/qt_phases.py $a > $OUT/s11_tmp.log 2>&1 || { tail -5 $OUT/s11_tmp.log; exit 3; }
	echo "== $a"; grep '"config"' $OUT/s11_tmp.log | tee -a $OUT/s11_phases.log
done
echo s11 done
