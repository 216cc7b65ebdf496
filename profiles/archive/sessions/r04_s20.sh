# GPU session 20 (round 4): both-direction src loads beside the dst loads
# (spec) against R2 (base) on C3 src|dst; the product bench with its rocprofv3
# kernel summary; PMC passes of C3 at 2^26.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
# a step that crashed, aborted or timed out ends the session (no GPU step after it)
step() {
	local t=$1; shift
	timeout -k 10 "$t" "$@"
	local rc=$?
	if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then echo "STOP: rc=$rc from: $*"; exit $rc; fi
	return $rc
}
for o in "--src-dst" "" "--hot 8"; do
XFG_LIB=$PWD/tools/abl/spec.so step 200 python -u tools/ab_parity.py $o > gpurun_out/par_spec.log 2>&1; tail -1 gpurun_out/par_spec.log
done
for r in 1 2; do for v in base spec; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c3sd > gpurun_out/s20_c3sd_${v}_$r.log 2>&1
grep config gpurun_out/s20_c3sd_${v}_$r.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v r$r', d['config'], d['kernel_ms'], d['roofline']['frac'])"
done; done
for r in 1 2; do for v in base lag2; do
XFG_LIB=$PWD/tools/abl/$v.so step 200 python -u tools/bench_configs.py c5 > gpurun_out/s20_c5_${v}_$r.log 2>&1
grep config gpurun_out/s20_c5_${v}_$r.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v r$r', d['config'], d['kernel_ms'], d['roofline']['frac'])"
done; done
step 400 python -u bench.py --steps 20 > gpurun_out/bench_s20.log 2>&1 || exit 3
tail -1 gpurun_out/bench_s20.log | cut -c1-900
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s20 -o run -- python3 bench.py --steps 20 --no-cpu > gpurun_out/prof_s20.log 2>&1
echo prof rc=$?
step 300 bash tools/r04_pmc.sh
echo s20 done
