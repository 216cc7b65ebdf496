# GPU session 5 (round 6): C5 end to end from a registered buffer -- zero
# copy alone (Z 0) against the hybrid rounds (a zero-copy chunk of 2^Z
# packets, then S staged chunks of 2^18 header windows gathered by the
# pool meanwhile), diagnostics library, one process, two rounds.
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
XFG_LIB=diag timeout -k 10 900 python3 tools/hyb_c5.py 0:0 20:2 20:3 21:4 19:1 20:1 22:8 > $OUT/s5_hyb.log 2>&1
rc=$?; grep '"Z"' $OUT/s5_hyb.log; [ $rc -eq 0 ] || { tail -5 $OUT/s5_hyb.log; exit $rc; }
echo s5 done
