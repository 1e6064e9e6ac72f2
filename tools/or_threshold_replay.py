"""Numpy replay of k_disj's MaxScore on a 1M-doc corpus (CPU):
thresholds a 2-5-term OR query could start from (the per-term K-th score the
planner uses, a seeded exact k-th over every clause's top-k docs, the final
k-th score), and at each fixed threshold the essential postings streamed and
the postings past bound 1 with 4096-doc tile maxima vs 512-doc sub-tile maxima.

  python tools/or_threshold_replay.py        (~2 min, 8 CPUs)
"""
import os
import sys, numpy as np, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fugu_amd import synth
N = 1_000_000
t0 = time.time()
c = synth.corpus(N, threads=8)
off = c.off.astype(np.int64); tok = c.tok
L = np.diff(off)
doc = np.repeat(np.arange(N, dtype=np.int64), L)
key = tok.astype(np.int64) * N + doc
key.sort()
u, tf = np.unique(key, return_counts=True)
pt = (u // N).astype(np.int64); pd = (u % N).astype(np.int64)
V = synth.VOCAB
toff = np.searchsorted(pt, np.arange(V + 1))
df = np.diff(toff)
tot = int(L.sum())
avgdl = np.float32(np.float32(tot) / np.float32(N))
# BM25 (K1 = 1.2, B = 0.75) in f32; docs are < 128 tokens here, so the fieldnorm
# code is the length itself up to 40 and a close value above (a model, not a checker)
K1, B = np.float32(1.2), np.float32(0.75)
cache_len = (K1 * ((np.float32(1) - B) + B * L.astype(np.float32) / avgdl)).astype(np.float32)
dff = df.astype(np.float64)
w = np.where(df > 0, np.log1p((N - dff + 0.5) / (dff + 0.5)) * 2.2, 0.0).astype(np.float32)
tff = tf.astype(np.float32)
sc = (w[pt] * (tff / (tff + cache_len[pd]))).astype(np.float32)
print('built', time.time() - t0, file=sys.stderr)
q_off, terms = synth.queries(256, 2, 5)
KS = [1, 10, 100, 1000]
def kth(a, k):
    if len(a) < k: return 0.0
    return float(np.partition(a, len(a) - k)[len(a) - k])
res = {20: [], 1000: []}
for qi in range(256):
    ts = terms[q_off[qi]:q_off[qi + 1]]
    acc = np.zeros(N, np.float32); hit = np.zeros(N, bool)
    for t in ts:
        a, b = toff[t], toff[t + 1]
        acc[pd[a:b]] += sc[a:b]; hit[pd[a:b]] = True
    tot_s = acc[hit]
    for k in (20, 1000):
        final = kth(tot_s, k)
        kp = min(x for x in KS if x >= k)
        thr0 = max(kth(sc[toff[t]:toff[t + 1]], kp) for t in ts)
        # seed: union of each clause's top-k docs, exact sums
        seed_docs = []
        for t in ts:
            a, b = toff[t], toff[t + 1]
            s = sc[a:b]
            if len(s) > k:
                idx = np.argpartition(s, len(s) - k)[len(s) - k:]
            else:
                idx = np.arange(len(s))
            seed_docs.append(pd[a:b][idx])
        sd = np.unique(np.concatenate(seed_docs))
        seed = kth(acc[sd], k)
        res[k].append((final, thr0, seed, len(ts)))
for k in (20, 1000):
    r = np.array(res[k])
    ok = r[:, 0] > 0
    print(k, 'n', ok.sum(), 'thr0/final median', np.median(r[ok, 1] / r[ok, 0]), 'seed/final median', np.median(r[ok, 2] / r[ok, 0]),
          'seed==final frac', np.mean(r[ok, 2] >= r[ok, 0] * 0.9999), 'p10 seed/final', np.percentile(r[ok, 2] / r[ok, 0], 10), 'p10 thr0/final', np.percentile(r[ok,1]/r[ok,0], 10))


# ---- bound-1 survivors under different fixed thresholds
TS = 12
ntile = (N + (1 << TS) - 1) >> TS
def work(ts, thr):
    m = len(ts)
    tub = np.zeros((m, ntile), np.float32)
    for i, t in enumerate(ts):
        a, b = toff[t], toff[t + 1]
        np.maximum.at(tub[i], pd[a:b] >> TS, sc[a:b])
    # MaxScore split per tile
    order = np.argsort(tub, axis=0, kind='stable')
    srt = np.take_along_axis(tub, order, axis=0)
    cs = np.cumsum(srt, axis=0)
    P = (cs < thr).sum(axis=0)   # non-essential prefix length
    ess = np.zeros((m, ntile), bool)
    for j in range(m):
        ess[order[j], np.arange(ntile)] |= (j >= P)
    tot_ub = tub.sum(axis=0)
    n_ess = 0; n_b1 = 0
    for i, t in enumerate(ts):
        a, b = toff[t], toff[t + 1]
        tl = pd[a:b] >> TS
        e = ess[i, tl]
        n_ess += int(e.sum())
        bnd = sc[a:b] + (tot_ub[tl] - tub[i, tl])
        n_b1 += int((e & (bnd >= thr)).sum())
    return n_ess, n_b1
agg = {k: np.zeros((3, 2)) for k in (20, 1000)}
for qi in range(64):
    ts = terms[q_off[qi]:q_off[qi + 1]]
    for k in (20, 1000):
        final, thr0, seed, _ = res[k][qi]
        for j, thr in enumerate((thr0, seed, final)):
            agg[k][j] += work(ts, thr)
for k in (20, 1000):
    print(k, 'thr0 (ess, b1)', agg[k][0], 'seed', agg[k][1], 'final', agg[k][2])

# ---- sub-tile maxima at the final threshold
def work2(ts, thr, TS=12, SS=9):
    m = len(ts)
    nt = (N + (1 << TS) - 1) >> TS
    ns = (N + (1 << SS) - 1) >> SS
    tub = np.zeros((m, nt), np.float32); sub = np.zeros((m, ns), np.float32)
    for i, t in enumerate(ts):
        a, b = toff[t], toff[t + 1]
        np.maximum.at(tub[i], pd[a:b] >> TS, sc[a:b])
        np.maximum.at(sub[i], pd[a:b] >> SS, sc[a:b])
    def split(ub):
        order = np.argsort(ub, axis=0, kind='stable')
        cs = np.cumsum(np.take_along_axis(ub, order, axis=0), axis=0)
        P = (cs < thr).sum(axis=0)
        ess = np.zeros(ub.shape, bool)
        for j in range(m):
            ess[order[j], np.arange(ub.shape[1])] |= (j >= P)
        return ess
    ess_t = split(tub); ess_s = split(sub)
    tt = tub.sum(0); ss = sub.sum(0)
    out = np.zeros(5)
    for i, t in enumerate(ts):
        a, b = toff[t], toff[t + 1]
        d = pd[a:b]; s = sc[a:b]; tl = d >> TS; sl = d >> SS
        e = ess_t[i, tl]
        b1 = s + (tt[tl] - tub[i, tl]) >= thr
        b1s = s + (ss[sl] - sub[i, sl]) >= thr
        es = ess_s[i, sl]
        out += [e.sum(), (e & b1).sum(), (e & b1s).sum(), es.sum(), (es & b1s).sum()]
    return out
for k in (20, 1000):
    agg = np.zeros(5)
    for qi in range(64):
        ts = terms[q_off[qi]:q_off[qi + 1]]
        final, thr0, seed, _ = res[k][qi]
        agg += work2(ts, final)
    print(k, 'at final thr: ess(tile) %d b1(tile) %d b1(sub512) %d | ess(sub512) %d b1(sub512, sub-split) %d' % tuple(agg))
