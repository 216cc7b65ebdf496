#!/bin/bash
# Print per-kernel VGPR / scratch / occupancy / LDS for the classify kernels.
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I include -I xdp-tools_amd/csrc -c xdp-tools_amd/csrc/xfg_kernels.hip -o /tmp/k.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c "
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1); d={}; continue
    for k in ('VGPRs','ScratchSize \[bytes/lane\]','Occupancy \[waves/SIMD\]','LDS Size \[bytes/block\]'):
        m=re.search(k+r': (\d+)',l)
        if m: d[k.split()[0]]=m.group(1)
    if 'LDS Size' in l and cur:
        mm=re.search(r'ILj(\d+)ELi(\d+)',cur); print(mm.groups() if mm else cur[:40], d)
"
