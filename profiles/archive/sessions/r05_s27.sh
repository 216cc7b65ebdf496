# GPU session 27 (round 5): do the kernel's zero-copy reads and the DMA
# engines' strided window copies add up on C5's 1536-byte slots?
# (tools/zerocopy_probe.py mix: each alone, then both at once)
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 600 python3 tools/zerocopy_probe.py mix > $OUT/s27_mix.log 2>&1; rc=$?
grep case $OUT/s27_mix.log; [ $rc -eq 0 ] || tail -5 $OUT/s27_mix.log
echo s27 done rc=$rc
