# GPU session 37 (round 5): C4 at SURVEY §8d's per-GPU shard (2^24 packets
# over 8 GPUs: 2^21 a GPU) and at 2^22, beside the 2^23 the status table uses
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; export PYTHONUNBUFFERED=1
cd $R
for l in 21 22 23; do
	timeout -k 10 400 python3 tools/bench_configs.py c4 --log2-packets $l > $OUT/s37_c4_$l.log 2>&1 || { tail -3 $OUT/s37_c4_$l.log; exit 3; }
	echo "2^$l $(grep -o '"kernel_ms": [0-9.]*' $OUT/s37_c4_$l.log) $(grep -o '"Mpps": [0-9.]*' $OUT/s37_c4_$l.log | head -1) $(grep -o '"frac": [0-9.]*' $OUT/s37_c4_$l.log)"
done
echo s37 done
