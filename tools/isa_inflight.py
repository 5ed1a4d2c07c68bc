"""In-flight register check of a device assembly file (hipcc --offload-device-only -S): the
hand-pipelined score kernels issue LDS fragment reads as inline asm, which the compiler believes
complete at issue.  For every ds_read this walks forward (straight-line code, counting younger
LDS / scalar-load ops against each s_waitcnt lgkmcnt(N)) and reports any instruction that reads
or writes the destination registers before the read is known to have landed: a compiler copy or
reuse of a pending register (QW1P r03: the drain reused a register whose read was still in
flight).  Usage: python tools/isa_inflight.py file.s"""
import re,sys
L=open(sys.argv[1]).read().split('\n')
def regs(tok):
    m=re.match(r'[va]\[(\d+):(\d+)\]',tok)
    if m: return {(tok[0],r) for r in range(int(m.group(1)),int(m.group(2))+1)}
    m=re.match(r'([va])(\d+)$',tok)
    return {(m.group(1),int(m.group(2)))} if m else set()
def toks(line):
    return [t.strip(' ,') for t in re.split(r'[ ,]+',line.strip())]
n=0
for i,l in enumerate(L):
    if re.search(r'^\s*ds_read',l):
        R=regs(toks(l)[1]); after=0
        for j in range(i+1,min(i+600,len(L))):
            s=L[j].strip()
            if not s or s.startswith(';'): continue
            t=toks(s)
            m=re.search(r'lgkmcnt\((\d+)\)',s)
            if t[0]=='s_waitcnt' and m:
                if after>=0 and int(m.group(1))<=after: break   # ours completed
                continue
            if t[0].startswith('ds_') or t[0].startswith('s_load') or t[0].startswith('s_buffer_load'): after+=1
            if t[0].startswith('v_mfma'):
                # mfma reading it before completion = real bug
                used=set()
                for tk in t[2:]: used|=regs(tk)
                if used&R: print('MFMA-EARLY',i+1,l.strip(),'->',j+1,s); n+=1; break
                continue
            used=set()
            for tk in t[1:]: used|=regs(tk)
            if used & R:
                print(i+1,l.strip(),'->',j+1,s); n+=1; break
            if t[0].startswith('s_cbranch') or t[0].startswith('s_branch') or t[0]=='s_endpgm': break
print('hits',n)
