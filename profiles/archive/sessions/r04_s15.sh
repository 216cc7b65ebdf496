# GPU session 15 (round 4): same-box A/B of the round's QT kernel against the
# previous commit's (old), the bucket lag / window depth / non-temporal
# variants on C3; C4 old/new; C5 through the QT path vs the general kernel.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
for v in lag2 d3l2; do for o in "" "--hot 8" "--src-dst"; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/ab_parity.py $o > gpurun_out/par_$v.log 2>&1; tail -1 gpurun_out/par_$v.log
done; done
for v in ntlen ntboth; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/ab_parity.py > gpurun_out/par_$v.log 2>&1; tail -1 gpurun_out/par_$v.log
done
for r in 1 2; do for v in old lag1; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c4 > gpurun_out/c4_${v}_$r.log 2>&1; grep config gpurun_out/c4_${v}_$r.log | cut -c1-230 | sed "s/^/$v r$r /"
done; done
for m in "XFG_QT=on" "XFG_QT=off" "XFG_DIAG_MASK=2048" "XFG_WINDOW=64"; do
env XFG_LIB=diag $m timeout -k 10 300 python -u tools/bench_configs.py c5 > gpurun_out/c5_diag_${m%%=*}.log 2>&1; rc=$?
case $rc in 124|134|137|139) echo "STOP rc=$rc"; exit $rc ;; esac
grep config gpurun_out/c5_diag_${m%%=*}.log | cut -c1-260 | sed "s/^/$m /"
done
TAG=s15 VARIANTS="old lag1 lag2 d3l2 ntlen ntboth" ROUNDS=2 step 800 bash tools/r04_ab.sh
echo s15 done
