#!/bin/bash
# The CPU suite (pytest -m "not gpu") against the ASAN + UBSAN builds of the
# host C: the restatement (oracle/), the runtime / pcap I/O / rule store
# (xdp-tools_amd/csrc/*.c), the CLI and the traffic synthesiser.  Python is
# not instrumented, so the ASAN runtime is preloaded; leak checking is off
# (the interpreter's own allocations), any ASAN or UBSAN report fails the run.
set -e
cd "$(dirname "$0")/.."
make asan
export XFG_LIB=asan
export LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
exec python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
