"""Walk-length simulation (numpy): how many 1024-node rounds of the K(n)-sorted 1M-node inventory
a cfg3 group request walks before the exact stop rule holds (K + 1 = 65 keys below the next
round's lower bound), at the initial state.  Motivated the sorted walk.
  PYTHONPATH=training-operator_amd python tools/walk_sim.py
"""
import numpy as np, sys
from placement import synth
N=1_000_000
inv=synth.make_inventory(N, synth.SEED["cfg5"], gpu_frac=0.2)
r=inv.residual().astype(np.int64); lab=inv.labels
S=r[0]+(r[1]>>20)+(r[2]<<20)+(r[3]>>24)
K=(S.astype(np.uint64)<<np.uint64(24))|np.arange(N,dtype=np.uint64)
o=np.argsort(K); Ks=K[o]; rs=r[:,o]; ls=lab[o]
b=synth.make_jobs(10000, synth.SEED["cfg3"], "mixed")
KK=65; R=1024
nr=(N+R-1)//R
rmin=Ks[::R]
mx=np.stack([np.maximum.reduceat(rs[d],np.arange(0,N,R)) for d in range(4)])
orl=np.bitwise_or.reduceat(ls,np.arange(0,N,R))
res=[]
for g in range(0,len(b.group_req),37):
    q=b.group_req[g]; need=b.group_need[g]
    sq=q[0]+(q[1]>>20)+(q[2]<<20)+(q[3]>>24)
    start=np.searchsorted(Ks,np.uint64(sq)<<np.uint64(24))
    r0=start//R
    cand=(mx[0]>=q[0])&(mx[1]>=q[1])&(mx[2]>=q[2])&(mx[3]>=q[3])&((orl&need)==need)
    keys=[]; walked=0; rounds=0
    for rr in range(r0,nr):
        if not cand[rr]: continue
        X=int(rmin[rr])-((sq+2)<<24)
        if len(keys)>=KK and np.sum(np.array(keys)<X)>=KK: break
        lo,hi=rr*R,min(N,rr*R+R)
        fit=((ls[lo:hi]&need)==need)&np.all(rs[:,lo:hi]>=q[:,None],axis=0)
        left=rs[:,lo:hi]-q[:,None]
        sc=left[0]+(left[1]>>20)+(left[2]<<20)+(left[3]>>24)
        kk=(sc[fit].astype(np.uint64)<<np.uint64(24))|(Ks[lo:hi][fit]&np.uint64(0xFFFFFF))
        keys.extend(int(x) for x in kk); walked+=hi-lo; rounds+=1
    res.append(rounds)
    if len(res)<15: print(q, need, 'rounds',rounds, 'fits',len(keys))
res=np.array(res); print('groups',len(res),'rounds mean',res.mean(),'p50',np.median(res),'p90',np.percentile(res,90),'max',res.max())
