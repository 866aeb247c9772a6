"""Register / spill table from a hipcc -Rpass-analysis=kernel-resource-usage
log: python tools/kernel_regs.py remarks.txt [name regex]
columns: kernel, VGPRs, VGPR spills, SGPRs, SGPR spills, scratch bytes/lane"""
import re
import sys

rows, cur, d = [], None, {}
for line in open(sys.argv[1]):
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        if cur:
            rows.append((cur, d))
        cur, d = m.group(1), {}
        continue
    m = re.search(r'remark:\s+(?:\S+:\d+:\d+:\s+)?([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+) \[', line)
    if m:
        d[m.group(1).strip()] = int(m.group(2))
if cur:
    rows.append((cur, d))
pat = sys.argv[2] if len(sys.argv) > 2 else ''
for n, d in rows:
    if re.search(pat, n):
        print(n.replace('_ZN12_GLOBAL__N_1', '')[:80], d.get('VGPRs'), d.get('VGPRs Spill'), d.get('TotalSGPRs'),
              d.get('SGPRs Spill'), d.get('ScratchSize'))
