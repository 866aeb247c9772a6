#!/bin/bash
# register usage per kernel of one .hip file: name VGPRs spills occupancy
cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Rpass-analysis=kernel-resource-usage -c "$1" -o /tmp/regs_$$.o 2>&1 | \
python3 -c "
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r'Function Name: (\S+)',l)
    if m: cur=m.group(1).replace('_ZN12_GLOBAL__N_1',''); d={}
    for k in ('VGPRs','VGPRs Spill','Occupancy \[waves/SIMD\]','LDS Size \[bytes/block\]'):
        m=re.search(r'remark:\s+'+k+r': (\d+)',l)
        if m: d[k.split()[0]+('S' if 'Spill' in k else '')]=m.group(1)
    if cur and 'Occupancy' in d and 'VGPRsS' in d and 'VGPRs' in d:
        print(cur[:60], 'vgpr',d['VGPRs'],'spill',d['VGPRsS'],'occ',d['Occupancy']); cur=None
"
rm -f /tmp/regs_$$.o
