"""Bank-conflict model of the resident kernel's tap gathers under different thread->quad
mappings of a C2 part (offline design tool; tools/lds_bank_sim.py models the pitch).  For the
bench's synthetic N(0, 2^2) offsets: LDS cycles of every ds_read_b64 footprint read (two
32-lane groups per wave-instruction, bank = dword mod 64) relative to conflict-free.
Round 5: row-major 3.26x, the ring-first order 3.63x (measured: C2 +3 %, C3 +5 % per section
without wave priorities, profiles/r05/ab_ring_noprio_r5h.json), column-major 7.4x.
usage: python tools/lds_map_sim.py row ring col blk2 blk4 str16 str8"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nlspn_eccv20_amd.synthetic import synth
K,REF,KW=8,4,3
H,W=228,304; W4=W//4
d=synth(1,H,W,K,seed=7240); off=d["off_aff"][0,:2*K]; offy,offx=off[0::2],off[1::2]
gy,gx=8,4
def cycles(addr):
    tot=0
    for g in (slice(0,32),slice(32,64)):
        a=addr[g]; a=a[a>=0]
        if a.size==0: continue
        dd=np.unique(np.concatenate([a,a+1])); tot+=np.bincount(dd%64,minlength=64).max()
    return tot
def part_quads(py,px,order):
    r0,r1=py*H//gy,(py+1)*H//gy; c0,c1=px*W4//gx,(px+1)*W4//gx
    nr,nq=r1-r0,c1-c0
    rr,cc=np.meshgrid(np.arange(nr),np.arange(nq),indexing='ij'); rr=rr.ravel(); cc=cc.ravel()
    if order=='row': idx=np.arange(nr*nq)
    elif order=='ring':
        Rb,Cb=min(9,nr//2),min(3,nq//2)
        key=np.where((rr<Rb),0,np.where(rr>=nr-Rb,1,np.where((cc<Cb)|(cc>=nq-Cb),2,3)))
        idx=np.lexsort((cc,rr,key))
    elif order=='col':  # column-major
        idx=np.lexsort((rr,cc))
    elif order.startswith('blk'):  # blocks of B rows x nq: within block column-major
        B=int(order[3:]); idx=np.lexsort((rr%B, cc, rr//B))
    elif order.startswith('str'):  # strips of S quads wide, row-major within strip
        S=int(order[3:]); idx=np.lexsort((cc%S, rr, cc//S))
    return r0+rr[idx], 4*(c0+cc[idx])
def sim(order, parts=6, pitch=128):
    tot=ideal=0
    rng=np.random.default_rng(1)
    for j in rng.choice(gy*gx,size=parts,replace=False):
        py,px=divmod(int(j),gx)
        y,x0=part_quads(py,px,order)
        n=len(y); nt=(n+63)//64*64
        hs=[];ws=[]
        for k in range(K):
            t=k if k<REF else k+1; i,jj=t//KW,t%KW
            for e in range(4):
                hs.append((y-1+i).astype(np.float32)+offy[k,y,x0+e]); ws.append((x0+e-1+jj).astype(np.float32)+offx[k,y,x0+e])
        h=np.stack(hs,1); w=np.stack(ws,1)
        valid=(h>-1)&(w>-1)&(h<H)&(w<W)
        hl=np.floor(h).astype(np.int64); wl=np.floor(w).astype(np.int64)
        rlo=hl[valid].min(); cmn=wl[valid].min()
        hl=np.where(valid,hl,rlo); wl=np.where(valid,wl,cmn-4)
        li=(hl-rlo)*pitch+wl-cmn+4
        idx=np.where(li&1, li+7804-1, li)+8
        A=np.full((nt,32),-1,np.int64); A[:n]=idx
        for wv in range(nt//64):
            sl=slice(64*wv,64*wv+64)
            for s in range(32):
                for row in (0,1):
                    a=A[sl,s].copy(); m=a>=0; a[m]+=row*pitch
                    tot+=cycles(a); ideal+=2
    return tot/ideal
for o in sys.argv[1:]:
    print(o, round(sim(o),3))
