# Partition chunk-size A/B (C3, 2^26). Build the libraries first, on the CPU:
#   tools/abbuild.sh base -DXFG_AB_C3; tools/abbuild.sh c4k -DXFG_AB_C3 -DXFG_LOG_CHUNK=4096
#   tools/abbuild.sh c16k -DXFG_AB_C3 -DXFG_LOG_CHUNK=16384
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
SC="1000000:500:250"
for r in 1 2 3; do
for v in base c4k c16k; do
XFG_LIB=$PWD/tools/abl/$v.so timeout -k 10 300 python -u tools/explore.py --log2-packets 26 --rounds 3 --iters 5 $SC > gpurun_out/explore_${v}_s33_$r.log 2>&1 || exit 2
sed "s/^/$v /" gpurun_out/explore_${v}_s33_$r.log | grep scenario
done; done
