#!/bin/bash
# tools/abbuild.sh NAME [-DMACRO ...] — a diagnostics library variant for
# same-box A/B timing (tools/explore.py with XFG_LIB=tools/abl/NAME.so):
# the kernels compiled with extra macros, the diagnostics host runtime.
# SRC=dir takes every source (kernels and host runtime, which must agree on
# the kernel-argument layout) from another tree's csrc/ (e.g. a git
# worktree of an older commit) for a before/after pair.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/abl
P=xdp-tools_amd
S=${SRC:-$P/csrc}
T=$(mktemp -d)
for c in xfg_ctx xfg_table xfg_io; do
  cc $(printf "%s\n" "$@" | grep -E "^-DXFG_QT_MIN_BITS" || true) -O2 -g -fPIC -Wall -Wno-unused-parameter -std=gnu11 -DXFG_DIAG -Iinclude -I$S -I/opt/rocm/include \
    -D__HIP_PLATFORM_AMD__ -c $S/$c.c -o $T/$c.o
done
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -DXFG_DIAG "$@" \
  -Iinclude -I$S -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
  -c $S/xfg_kernels.hip -o $T/k.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o tools/abl/$name.so \
  $T/xfg_ctx.o $T/xfg_table.o $T/xfg_io.o $T/k.o \
  -L/opt/rocm/lib -lamdhip64 -lrccl -lpthread -Wl,-rpath,/opt/rocm/lib
rm -rf $T
