#!/bin/bash
# tools/abbuild.sh NAME [-DMACRO ...] — a diagnostics library variant for
# same-box A/B timing (tools/explore.py with XFG_LIB=tools/abl/NAME.so):
# the kernels compiled with extra macros, the diagnostics host runtime.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/abl
P=xdp-tools_amd
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -DXFG_DIAG "$@" \
  -Iinclude -I$P/csrc -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
  -c $P/csrc/xfg_kernels.hip -o tools/abl/$name.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/abl/$name.so \
  $P/build/xfg_ctx_diag.o $P/build/xfg_table_diag.o $P/build/xfg_io.o tools/abl/$name.o \
  -L/opt/rocm/lib -lamdhip64 -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
rm -f tools/abl/$name.o
