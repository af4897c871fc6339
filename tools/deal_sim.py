"""Bank conflicts of the index build's LDS bank dealing (build_index pass 3), simulated:
extra LDS cycles per 32-lane set of the scorer's 16-byte-load rounds for per-wave runs of
i.i.d. docs and impacts, dealt in impact-class order (deal), largest-remaining-first
(deal2), flat (one class) and unsorted.  CPU only:  python tools/deal_sim.py"""
import numpy as np
rng=np.random.default_rng(0)
def cls_of(v): return 7-int(np.floor(np.log2(v)))
def deal(docs, vals):
    n=len(docs); cls=np.array([cls_of(v) for v in vals])
    order=np.argsort(cls, kind='stable'); docs=docs[order]; cls=cls[order]
    out=[]; usedq=[0,0,0,0]; cursor=0; o=0
    for c in range(8):
        idx=np.where(cls==c)[0]
        if len(idx)==0: continue
        buckets={}
        for i in idx: buckets.setdefault(int(docs[i])&31,[]).append(int(docs[i]))
        avail=0
        for b in buckets: avail|=1<<b
        for _ in range(len(idx)):
            rp=o
            if rp%128==0: usedq=[0,0,0,0]
            used=usedq[rp&3]
            cand=avail & ~used
            if not cand: cand=avail
            rot=((cand>>cursor)|(cand<<(32-cursor))) & 0xFFFFFFFF if cursor else cand
            k=((rot & -rot).bit_length()-1 + cursor)&31
            out.append(buckets[k].pop())
            if not buckets[k]: avail&=~(1<<k)
            usedq[rp&3]|=1<<k; cursor=(k+1)&31; o+=1
    return np.array(out)
def conflicts(seq):
    # 16B loads: set for (block of 128, k) = positions 128*b + 4L + k, L<32
    extra=0; sets=0
    n=len(seq)
    for b0 in range(0,n,128):
        for k in range(4):
            pos=[b0+4*L+k for L in range(32) if b0+4*L+k<n]
            if not pos: continue
            banks=np.bincount(seq[pos]&31, minlength=32)
            extra+=banks.max()-1; sets+=1
    return extra, sets
# impacts: softplus(N(-.5,1.5)) quantized 255/7.9
def sample_vals(n):
    x=np.log1p(np.exp(rng.normal(-0.5,1.5,n)))
    v=np.trunc(x*255/7.9).astype(int); v=v[v>0]
    return v
for n in (64, 300, 1200):
    tot_e=tot_s=0
    for rep in range(30):
        v=sample_vals(n*2)[:n]
        d=rng.choice(1600, size=len(v), replace=False)
        seq=deal(d, v)
        e,s=conflicts(seq); tot_e+=e; tot_s+=s
    print(n, 'avg extra cycles per set (ideal 0; a set = 1 ds_read group):', round(tot_e/tot_s,3))

def deal2(docs, vals):
    # largest-remaining-first among banks unused in the position's set (ties: cursor order)
    cls=np.array([cls_of(v) for v in vals])
    order=np.argsort(cls, kind='stable'); docs=docs[order]; cls=cls[order]
    out=[]; usedq=[0,0,0,0]; o=0; cursor=0
    for c in range(8):
        idx=np.where(cls==c)[0]
        if len(idx)==0: continue
        buckets={}
        for i in idx: buckets.setdefault(int(docs[i])&31,[]).append(int(docs[i]))
        for _ in range(len(idx)):
            if o%128==0: usedq=[0,0,0,0]
            used=usedq[o&3]
            best=None; bc=-1
            for j in range(32):
                b=(cursor+j)&31
                if b in buckets and buckets[b] and not (used>>b)&1 and len(buckets[b])>bc:
                    best=b; bc=len(buckets[b])
            if best is None:
                for j in range(32):
                    b=(cursor+j)&31
                    if b in buckets and buckets[b] and len(buckets[b])>bc: best=b; bc=len(buckets[b])
            out.append(buckets[best].pop()); usedq[o&3]|=1<<best; cursor=(best+1)&31; o+=1
    return np.array(out)
for n in (64, 300, 1200):
    tot_e=tot_s=0
    for rep in range(30):
        v=sample_vals(n*2)[:n]
        d=rng.choice(1600, size=len(v), replace=False)
        seq=deal2(d, v)
        e,s=conflicts(seq); tot_e+=e; tot_s+=s
    print('LRF', n, round(tot_e/tot_s,3))
# random order baseline
for n in (300,):
    tot_e=tot_s=0
    for rep in range(30):
        d=rng.choice(1600, size=n, replace=False)
        e,s=conflicts(d); tot_e+=e; tot_s+=s
    print('random', n, round(tot_e/tot_s,3))
for n in (64, 300, 1200):
    tot_e=tot_s=0
    for rep in range(30):
        d=rng.choice(1600, size=n, replace=False)
        seq=deal(d, np.full(n, 200))
        e,s=conflicts(seq); tot_e+=e; tot_s+=s
    print('flat', n, round(tot_e/tot_s,3))
# class histogram
v=sample_vals(100000); print('class shares', np.bincount([cls_of(x) for x in v], minlength=8)/len(v))
