#!/usr/bin/env python3
"""LDS bank model of fused4's gather reads and element-vector writes (Q3, 4x4 tile):
prints the LDS cycles of the current pitches and searches (RP, P1, PC).
Model as scripts/lds_bank_sim.py: b64 accesses in 2 x 32 lanes, 64 4-byte banks,
identical addresses broadcast."""
from collections import defaultdict
def cyc(addrs, group=32, nbank=64):
    # addrs: list of (lane, double index) ; b64 access: 2 dwords
    tot=0
    for g0 in range(0,64,group):
        banks=defaultdict(set)
        act=False
        for ln in range(g0,g0+group):
            a=addrs.get(ln)
            if a is None: continue
            act=True
            for d in range(2): banks[(2*a+d)%nbank].add(a)
        if act: tot+=max(len(v) for v in banks.values())
    return tot
P=3; TY=TZ=4; DY=DZ=13; DZP=13; PLP=DY*DZP; PL=DY*DZ; RP,P1,PC=5,21,85; NT=256; ND=4
# gather reads: for k in NOUT, element e = tid + k*NT -> (pl, ly, lz), 4 sources
NOUT=(ND*PL+NT-1)//NT
def srcs(e):
    pl=e//PL; rem=e%PL; ly=rem//DZ; lz=rem%DZ
    cyh=min(ly//P,TY-1); cyl= ly//P-1 if (ly%P==0 and ly>0 and ly//P-1<cyh) else cyh
    czh=min(lz//P,TZ-1); czl= lz//P-1 if (lz%P==0 and lz>0 and lz//P-1<czh) else czh
    s=[]
    for ccy in range(cyl,cyh+1):
        for ccz in range(czl,czh+1):
            s.append((ccy*TZ+ccz)*PC+(ly-ccy*P)*P1+(lz-ccz*P)*RP+pl)
    return s
tot=ideal=0
for k in range(NOUT):
    for w in range(4):
        for si in range(4):
            addrs={}
            for ln in range(64):
                e=w*64+ln+k*NT
                if e>=ND*PL: continue
                s=srcs(e)
                if si<len(s): addrs[ln]=s[si]
            if addrs:
                c=cyc(addrs); tot+=c; ideal+=2
print('gather reads: cycles',tot,'ideal',ideal)
# e-vector writes: lane (g,n): c=4w+cs, eo = c*PC + g*RP + xi + r*P1
tot=ideal=0
for w in range(4):
    for r in range(4):
        addrs={}
        for ln in range(64):
            g=ln>>4; n=ln&15; xi=n&3; cs=n>>2; c=4*w+cs
            addrs[ln]=c*PC+g*RP+xi+r*P1
        tot+=cyc(addrs); ideal+=2
print('evec writes: cycles',tot,'ideal',ideal)
# staging writes: un[pl*PLP + ly*DZP + lz] for e=tid+k*NT, pl 1..P
NPF=(P*PL+NT-1)//NT
tot=ideal=0
for k in range(NPF):
    for w in range(4):
        addrs={}
        for ln in range(64):
            e=w*64+ln+k*NT
            if e>=P*PL: continue
            pl=1+e//PL; rem=e%PL; ly=rem//DZ; lz=rem%DZ
            addrs[ln]=pl*PLP+ly*DZP+lz
        if addrs: tot+=cyc(addrs); ideal+=2
print('staging writes: cycles',tot,'ideal',ideal)
# uu reads
tot=ideal=0
for w in range(4):
    for l in range(4):
        for j in range(4):
            addrs={}
            for ln in range(64):
                g=ln>>4; n=ln&15; cs=n>>2; c=4*w+cs; cy=c//TZ; cz=c%TZ
                addrs[ln]=(cy*P)*DZP+cz*P+g+l*PLP+j*DZP
            tot+=cyc(addrs); ideal+=2
print('uu reads: cycles',tot,'ideal',ideal)

def cost(RP_,P1_,PC_):
    global RP,P1,PC
    RP,P1,PC=RP_,P1_,PC_
    t=0
    for k in range(NOUT):
        for w in range(4):
            for si in range(4):
                addrs={}
                for ln in range(64):
                    e=w*64+ln+k*NT
                    if e>=ND*PL: continue
                    s=srcs(e)
                    if si<len(s): addrs[ln]=s[si]
                if addrs: t+=cyc(addrs)
    for w in range(4):
        for r in range(4):
            addrs={}
            for ln in range(64):
                g=ln>>4; n=ln&15; xi=n&3; cs=n>>2; c=4*w+cs
                addrs[ln]=c*PC+g*RP+xi+r*P1
            t+=cyc(addrs)
    return t
best=[]
for RP_ in range(4,10):
    for P1_ in range(4*RP_, 4*RP_+12):
        for PC_ in range(4*P1_, 4*P1_+24):
            best.append((cost(RP_,P1_,PC_), 16*PC_, RP_,P1_,PC_))
best.sort()
print(best[:10]); print('current', cost(5,21,85))
