#!/usr/bin/env python3
"""Wave-scheduling model of the lean traversal (pt_device.h trav_step_lean) on a scene's reference
BVH: per ray, the reference walk's node steps and leaf-pair test counts (f64 restatement of the
ray/box and ray/triangle tests, random rays inside the scene box), then a 64-lane wave with refill
running lean<K> turns under a node-bias policy; prints the modelled cost (VALU instructions) and
lane use, with and without dealing a leaf turn's tests over all lanes, and with
runs of 8 entries dealt one per lane (lean_leaf_pool, round 4).
usage: wave_model.py SCENE NRAYS"""
import math
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import SCENES, pack_with_node  # noqa: E402

name, NR = sys.argv[1], int(sys.argv[2])
d = tempfile.mkdtemp()
p = pack_with_node(os.path.join(SCENES, "scene_assets", name + ".xml"), d)
B = np.asarray(p.bvh_data, np.float64).tolist()
T = np.asarray(p.triangle_data, np.float64)
vs = int(T[2])
V = T
def vert(i): return np.array(V[vs+i:vs+i+3])
def tri_t(o,dv,rec):
    i0,i1,i2=[(int(x)-1)*3 for x in rec[:3]]
    v0,v1,v2=vert(i0),vert(i1),vert(i2)
    e1=v1-v0; e2=v2-v0; r=np.cross(dv,e2); det=e1@r
    if -1e-8<det<1e-8: return None
    inv=1/det; s=o-v0; u=inv*(s@r)
    if u<0 or u>1: return None
    q=np.cross(s,e1); v=inv*(dv@q)
    if v<0 or u+v>1: return None
    t=inv*(e2@q)
    return t if t>1e-8 else None
def bbox(o,inv,mn,mx):
    t1=(np.array(mn)-o)*inv; t2=(np.array(mx)-o)*inv
    tmin=max(-3e38,*np.minimum(t1,t2)); tmax=min(3e38,*np.maximum(t1,t2))
    if tmax>max(tmin,0): return tmin if tmin>0 else tmax
    return -1
lo=np.array(B[0:3]); hi=np.array(B[3:6])
rng=np.random.default_rng(1)
seqs=[]
for k in range(NR):
    o=lo+(hi-lo)*(0.1+0.8*rng.random(3)); dv=rng.normal(size=3); dv/=np.linalg.norm(dv); inv=1/dv
    st=[6]; best=-1.0; seq=[]
    while st:
        ptr=st.pop()
        ld=bbox(o,inv,B[ptr+5:ptr+8],B[ptr+8:ptr+11]); rd=bbox(o,inv,B[ptr+11:ptr+14],B[ptr+14:ptr+17])
        lp=int(B[ptr+2]); rp=int(B[ptr+3]); nt=0
        for hit,cp in ((ld>0,lp),(rd>0,rp)):
            if hit and B[cp]==1:
                n=int(B[cp+4]); nt+=n//4
                for i in range(cp+17,cp+17+n,4):
                    t=tri_t(o,dv,tuple(B[i:i+4]))
                    if t is not None and (best<0 or t<best): best=t
        seq.append(('N',)); 
        if nt: seq.append(('L',nt))
        ll = ld>0 and B[lp]==1; rl = rd>0 and B[rp]==1
        tl = ld>0 and not ll and not (best>0 and ld>best)
        tr = rd>0 and not rl and not (best>0 and rd>best)
        if tl: st.append(lp)
        if tr: st.append(rp)
    seqs.append(seq)
CN, CT, OV = 50.0, 35.0, 16.0
OVR = 40.0  # per run of 8 (lean_leaf_pool): owner fetches, gather, key atomic
def simulate(K, bias, redistribute):
    pool=list(range(len(seqs))); lanes=[None]*64; cost=0.0; useful=0.0
    def refill():
        for i in range(64):
            if lanes[i] is None and pool:
                r=pool.pop(); lanes[i]=[r,0,0]  # ray, unit idx, tests done in current leaf unit
    refill()
    while any(l is not None for l in lanes):
        st=[]
        for l in lanes:
            if l is None: st.append(None); continue
            u=seqs[l[0]][l[1]]; st.append(u[0])
        nL=st.count('L'); nN=st.count('N')
        if nL and nL >= bias*nN:
            rem=[seqs[l[0]][l[1]][1]-l[2] if s=='L' else 0 for l,s in zip(lanes,st)]
            if redistribute == 'runs':  # lean_leaf_pool: runs of 8 entries dealt one per lane
                tot=sum(rem); items=sum(math.ceil(x/8) for x in rem); steps=math.ceil(items/64)
                cost+=steps*(8*CT+OVR); useful+=tot*CT
                for i,s in enumerate(st):
                    if s=='L': lanes[i][2]=seqs[lanes[i][0]][lanes[i][1]][1]
            elif redistribute:
                tot=sum(rem); steps=math.ceil(tot/64); cost+=steps*(CT+OV); useful+=tot*CT
                for i,s in enumerate(st):
                    if s=='L': lanes[i][2]=seqs[lanes[i][0]][lanes[i][1]][1]
            else:
                turn=max(min(K,r) for r in rem); cost+=turn*CT
                for i,s in enumerate(st):
                    if s=='L': d=min(K,rem[i]); lanes[i][2]+=d; useful+=d*CT
        else:
            cost+=CN
            for i,s in enumerate(st):
                if s=='N': lanes[i][1]+=1; lanes[i][2]=0; useful+=CN
        for i,l in enumerate(lanes):
            if l is None: continue
            u=seqs[l[0]]
            if l[1]<len(u) and u[l[1]][0]=='L' and l[2]>=u[l[1]][1]: l[1]+=1; l[2]=0
            if l[1]>=len(u): lanes[i]=None
        refill()
    return cost, useful/(64*cost)
for K,bias,red in [(16,4,False),(16,8,False),(16,2,False),(16,1,False),(8,8,False),(16,8,True),(16,2,True),(16,1,True),
                   (16,4,'runs'),(16,2,'runs'),(16,1,'runs')]:
    c,u=simulate(K,bias,red); print(name,'K',K,'bias',bias,'redist',red,'cost',round(c),'util',round(u,3))
