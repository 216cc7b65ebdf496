#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy / LDS of xfg_kernels.hip (gfx950).
Usage: python3 tools/kres.py [substring-filter]"""
import re, subprocess, sys
flt = sys.argv[1] if len(sys.argv) > 1 else ""
out = subprocess.run(
    "hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I xdp-tools_amd/csrc "
    "$KFLAGS -c xdp-tools_amd/csrc/xfg_kernels.hip -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage",
    shell=True, capture_output=True, text=True).stderr
cur, d = None, {}
for l in out.splitlines():
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur, d = m.group(1), {}
        continue
    for k, pat in (("VGPR", r"\bVGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                   ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("LDS", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, l)
        if m:
            d[k] = int(m.group(1))
    if "LDS Size" in l and cur and flt in cur:
        print(re.sub(r"_ZN12_GLOBAL__N_1\d+", "", cur)[:60], d)
