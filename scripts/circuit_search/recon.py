import itertools
N=64
def bit(t,r): return (t>>r)&1
IN=[sum(1<<r for r in range(64) if (r>>i)&1) for i in range(6)]
CARE=0; TGT=0
for r in range(64):
    P=r&7; X=(r>>3)&3; c=(r>>5)&1
    if P<=6 and not (c and P==0): CARE|=1<<r
    S=P+X
    if S==3 or (S==4 and c): TGT|=1<<r
M=(1<<64)-1
def gate(a,b,c,f):
    r=0
    for m in range(8):
        if f>>m&1:
            r|=(a if m&4 else ~a&M)&(b if m&2 else ~b&M)&(c if m&1 else ~c&M)
    return r
names=['p0','p1','p2','x0','x1','c']
def find_gate(t, sigs):
    out=[]
    for i,j,k in itertools.combinations(range(len(sigs)),3):
        for f in range(256):
            if gate(sigs[i],sigs[j],sigs[k],f)&CARE==t&CARE: out.append((i,j,k,f))
    return out
def lut(inputs, target, care):
    # function table of target over inputs on care rows, None if inconsistent; dont care -> 0
    tab={}
    for r in range(64):
        if not care>>r&1: continue
        key=tuple(bit(s,r) for s in inputs)
        v=bit(target,r)
        if tab.setdefault(key,v)!=v: return None
    f=0
    for m in range(8):
        key=((m>>2)&1,(m>>1)&1,m&1)
        if tab.get(key,0): f|=1<<m
    return f
sols=[("00550055aa55aa55",(1,2,6,0x18),(2,4,5,6),0x7,0),]
import sys
g1=int(sys.argv[1],16); i,j,k,f=[int(x,0) for x in sys.argv[2].split(',')]
print("g1 =", [(names[a],names[b],names[c],hex(ff)) for a,b,c,ff in find_gate(g1, IN)][:4])
sig=IN+[g1]; names.append('g1')
g2=gate(sig[i],sig[j],sig[k],f); sig.append(g2); names.append('g2')
print("g2 = bitop3(%s,%s,%s,%#x)"%(names[i],names[j],names[k],f))
# find g3 over any triple, final over triple incl g3
best=[]
for a,b,c in itertools.combinations(range(8),3):
    for f3 in range(256):
        g3=gate(sig[a],sig[b],sig[c],f3)
        for x,y in itertools.combinations(range(8),2):
            F=lut([g3,sig[x],sig[y]],TGT,CARE)
            if F is not None:
                best.append((names[a],names[b],names[c],hex(f3),'final(g3,%s,%s)=%#x'%(names[x],names[y],F)))
print(len(best)); print(*best[:10],sep='\n')
