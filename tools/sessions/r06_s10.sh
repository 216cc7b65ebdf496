# GPU session 10 (round 6): the index kernel's phases per workgroup
# (diagnostics library, wall-clock stamps, tools/qt_phases.py): C3 and C4 at
# the per-GPU shard 2^21, C3 at 2^24, and C3 2^21 without the count wave.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
export XFG_LIB=diag
for a in "c3 21" "c4 21" "c3 24" "c3 21 XFG_CW=off" "c4 21 XFG_CW=off"; do
	timeout -k 10 300 python3 tools/qt_phases.py $a > $OUT/s10_tmp.log 2>&1 || { tail -5 $OUT/s10_tmp.log; exit 3; }
	echo "== $a"; grep '"config"' $OUT/s10_tmp.log | tee -a $OUT/s10_phases.log
done
echo s10 done
