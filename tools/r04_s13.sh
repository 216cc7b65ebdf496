cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
for o in "" "--hot 8" "--src-dst"; do
XFG_LIB=$PWD/tools/abl/lag2.so timeout -k 10 200 python -u tools/ab_parity.py $o > gpurun_out/par_lag2.log 2>&1; tail -1 gpurun_out/par_lag2.log
done
TAG=s13 VARIANTS="lag1 lag2" ROUNDS=3 bash tools/r04_ab.sh
SC="1000000:500:250" LOG2=24 TAG=s13sd VARIANTS="lag1 lag2" ROUNDS=1 bash tools/r04_ab.sh
bash tools/r04_pmc.sh
