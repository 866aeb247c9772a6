"""Scan hipcc --save-temps device assembly for the 16-byte store data hazard:
a buffer/global store of 3-4 dwords whose data VGPRs a VALU instruction
overwrites within 2 wait states (cdna_hip_programming.md §5.7 item 1).
usage: python tools/store_hazard_check.py '/tmp/isa/*-gfx950.s'"""
import re,sys,glob
def regs(tok):
    m=re.match(r'v\[(\d+):(\d+)\]',tok)
    if m: return set(range(int(m[1]),int(m[2])+1))
    m=re.match(r'v(\d+)$',tok)
    if m: return {int(m[1])}
    return set()
for fn in sorted(glob.glob(sys.argv[1])):
    lines=[l.split(';')[0].strip() for l in open(fn)]
    lines=[l for l in lines if l and not l.endswith(':') and not l.startswith('.')]
    tot=bad=0
    for k,l in enumerate(lines):
        op=l.split()[0]
        if re.match(r'(buffer|global|flat|scratch)_store_dword(x3|x4)',op):
            tot+=1
            parts=[p.strip() for p in l[len(op):].split(',')]
            data=regs(parts[1]) if op.startswith('global') or op.startswith('flat') else regs(parts[0])
            ws=0
            for x in lines[k+1:k+6]:
                o=x.split()[0]
                if o.startswith('s_nop'): ws+=int(x.split()[1])+1
                elif o.startswith('v_'):
                    dst=regs(x.split()[1].rstrip(','))
                    if dst & data and ws<2:
                        bad+=1
                        if bad<=3: print('  HAZ',l,'|',x)
                        break
                    ws+=1
                else: ws+=1
                if ws>=2: break
    print(fn.split('/')[-1],tot,'wide stores',bad,'hazards')
