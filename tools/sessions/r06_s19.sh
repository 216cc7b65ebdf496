# GPU session 19 (round 6): the end of a QT workgroup split further -- each
# wave at the first end barrier, wave 0 past it, the partitions moved
# (tools/qt_phases.py fold / barrier1_wait / partition_flush): C3 at 2^21,
# 2^24, 2^26.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
export XFG_LIB=diag
for a in "c3 21" "c3 24" "c3 26"; do
	timeout -k 10 400 python3 tools/qt_phases.py $a > $OUT/s19_tmp.log 2>&1 || { tail -5 $OUT/s19_tmp.log; exit 3; }
	echo "== $a"; grep '"config"' $OUT/s19_tmp.log | tee -a $OUT/s19_phases.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print({k:d[k] for k in ('span_us','setup','loop_last_wave','defer_walk','fold','barrier1_wait','partition_flush','flush','end') if k in d})"
done
echo s19 done
