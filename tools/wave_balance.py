import sys, numpy as np, time
sys.path.insert(0, '/root/repo')
from improving_learned_index_amd import synthetic as S, _lib
n_docs = int(sys.argv[1]); skew = sys.argv[2] == 'skew'
t0=time.time()
term_off, pdoc, pval, _ = S.synth_postings(n_docs, 2*n_docs, seed=4321, skew=S.SKEW_CONFIG4 if skew else None)
print('gen', time.time()-t0, len(pval), flush=True)
nq=6980
qs = S.msmarco_like_queries(nq, 2*n_docs, seed=1234)
nb = (n_docs + 32767)//32768
bd = min(32768, ((n_docs + nb - 1)//nb + 63)//64*64)
S_ = (bd + 15)//16
terms = sorted({t for q in qs for t in q})
cnt = {}
for t in terms:
    d = pdoc[term_off[t]:term_off[t+1]]
    b = d // bd; w = np.minimum((d % bd)//S_, 15)
    c = np.zeros((nb, 16), np.int32)
    np.add.at(c, (b, w), 1)
    cnt[t] = c
print('terms', len(terms), time.time()-t0, flush=True)
nt_hist = np.bincount([len(q) for q in qs]); print('nt hist', nt_hist)
# per item per wave: max run, total
allfit = 0; tot = 0; wave_tot = []; item_max = []; item_sum=[]
for q in qs:
    C = np.stack([cnt[t] for t in q])  # nt x nb x 16
    blk = C.sum(2)                     # nt x nb
    long_ = blk >= 128
    run = np.where(long_[:, :, None], C, blk[:, :, None])  # nt x nb x 16
    mx = run.max(0)  # nb x 16
    allfit += (mx <= 256).sum(); tot += mx.size
    wt = run.sum(0)  # nb x 16 postings each wave reads
    wave_tot.append(wt.ravel())
    item_max.append(wt.max(1)); item_sum.append(blk.sum(0))
wave_tot = np.concatenate(wave_tot); item_max=np.concatenate(item_max); item_sum=np.concatenate(item_sum)
print('waves with all runs <=256: %.3f' % (allfit/tot))
print('per-wave postings read: mean %.1f p50 %d p90 %d p99 %d' % (wave_tot.mean(), *np.percentile(wave_tot,[50,90,99])))
print('item postings: mean %.1f; slowest wave/mean wave %.2f' % (item_sum.mean(), (item_max.mean()/ (wave_tot.mean()))))
# balanced segments: per block, boundaries at equal quantiles of all postings
pc = np.bincount(pdoc, minlength=nb*bd)[:nb*bd].reshape(nb, bd).astype(np.int64)
cum = np.cumsum(pc, 1)
bnd = np.zeros((nb, 17), np.int64); bnd[:, 16] = bd
for b in range(nb):
    tot_b = cum[b, -1]
    for w in range(1, 16):
        bnd[b, w] = np.searchsorted(cum[b], tot_b * w / 16.0)
print('balanced seg sizes: min %d max %d' % ((bnd[:,1:]-bnd[:,:-1]).min(), (bnd[:,1:]-bnd[:,:-1]).max()))
cnt2 = {}
for t in terms:
    d = pdoc[term_off[t]:term_off[t+1]]
    b = d // bd; r = d % bd
    w = np.empty(len(d), np.int64)
    for bb in np.unique(b):
        m = b == bb
        w[m] = np.minimum(np.searchsorted(bnd[bb], r[m], side='right') - 1, 15)
    c = np.zeros((nb, 16), np.int32)
    np.add.at(c, (b, w), 1)
    cnt2[t] = c
wave_tot = []; item_max = []
for q in qs:
    C = np.stack([cnt2[t] for t in q]); blk = C.sum(2); long_ = blk >= 128
    run = np.where(long_[:, :, None], C, blk[:, :, None])
    wt = run.sum(0); wave_tot.append(wt.ravel()); item_max.append(wt.max(1))
wave_tot = np.concatenate(wave_tot); item_max=np.concatenate(item_max)
print('balanced: per-wave mean %.1f; slowest/mean %.2f' % (wave_tot.mean(), item_max.mean()/wave_tot.mean()))
# all-wave form for comparison: slowest = ceil(item postings/16) + short-term reads
