"""The K-th score bound a rescore without new deletions reuses (fugu.cpp
kth_reuse_bound), checked on the CPU: for random old
and new BM25 statistics and random postings (tf, fieldnorm id, one or two
fields), every term's K-th best score under the new statistics, computed in
tantivy's f32 order as k_score does, is at least r(t) times the K-th best under
the old ones, where r(t) = (1 - 2^-18) x min over the term's fields of
(new weight / old weight) x min over the 256 fieldnorm ids of (1 + c_old) /
(1 + c_new).  A lower bound of the K-th best score is a valid starting
threshold, so the searches' hits cannot change.
"""
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
from gen_golden import F, K1, TABLE, cache, weight  # noqa: E402


def score(tf, fn, w, c):
    """k_score's f32 order for one field: w * (tf / (tf + c[fn])), 0 where tf == 0."""
    tf32 = tf.astype(np.float32)
    s = w * (tf32 / (tf32 + c[fn]))
    return np.where(tf > 0, s, F(0.0)).astype(np.float32)


def bound_ratio(w_old, w_new, c_old, c_new, fields):
    cmin = []
    for f in range(2):
        q = (1.0 + c_old[f].astype(np.float64)) / (1.0 + c_new[f].astype(np.float64))
        q = q[np.isfinite(q)]
        cmin.append(min(1.0, float(q.min())) if len(q) else 1.0)
    r = math.inf
    for f in range(fields):
        if w_old[f] > 0:
            r = min(r, float(w_new[f]) / float(w_old[f]) * cmin[f])
    return (max(0.0, r) if math.isfinite(r) else 1.0) * (1.0 - 2.0 ** -18)


def test_reuse_bound_never_exceeds_the_new_kth():
    rng = np.random.default_rng(12)
    checked = 0
    for trial in range(300):
        fields = 1 + (trial % 2)
        n_old = int(rng.integers(1000, 2_000_000))
        n_new = n_old + int(rng.integers(0, n_old // 5 + 1))
        P = int(rng.integers(10, 3000))
        df_old = [int(rng.integers(1, min(P, n_old) + 1)) for _ in range(2)]
        df_new = [d + int(rng.integers(0, n_new - n_old + 1)) for d in df_old]
        df_new = [min(d, n_new) for d in df_new]
        w_old = [weight(df_old[f], n_old) for f in range(2)]
        w_new = [weight(df_new[f], n_new) for f in range(2)]
        avg_old = [F(rng.uniform(5, 200)) for _ in range(2)]
        avg_new = [F(a * F(rng.uniform(0.8, 1.25))) for a in avg_old]
        c_old = [cache(a) for a in avg_old]
        c_new = [cache(a) for a in avg_new]
        tf = [rng.integers(0 if fields == 2 else 1, 60, P) for _ in range(2)]
        if fields == 1:
            tf[1] = np.zeros(P, np.int64)
        else:
            tf[0] = np.where((tf[0] == 0) & (tf[1] == 0), 1, tf[0])
        fn = [rng.integers(0, 256, P) for _ in range(2)]
        s_old = (F(0.0) + score(tf[0], fn[0], w_old[0], c_old[0])) + score(tf[1], fn[1], w_old[1], c_old[1])
        s_new = (F(0.0) + score(tf[0], fn[0], w_new[0], c_new[0])) + score(tf[1], fn[1], w_new[1], c_new[1])
        r = bound_ratio(w_old, w_new, c_old, c_new, fields)
        o = np.sort(s_old)[::-1]
        n = np.sort(s_new)[::-1]
        for K in (1, 10, 20, 100, 1000):
            if K > P:
                continue
            b = np.float32(float(o[K - 1]) * r)
            if float(b) > float(o[K - 1]) * r:
                b = np.nextafter(b, np.float32(0))
            assert b <= n[K - 1], (trial, K, float(b), float(n[K - 1]), r)
            checked += 1
    assert checked > 800


def test_reuse_bound_is_tight_for_small_statistics_changes():
    """A commit of 1% more docs: the bound stays within 0.5% of the new K-th."""
    rng = np.random.default_rng(4)
    worst = 1.0
    for trial in range(100):
        n_old = 10_000_000
        n_new = n_old + 100_000
        df = int(rng.integers(100, 1_000_000))
        w_old, w_new = weight(df, n_old), weight(df + df // 100, n_new)
        avg = F(64.0)
        c_old, c_new = cache(avg), cache(F(avg * F(1.001)))
        tf = rng.integers(1, 20, 5000)
        fn = rng.integers(0, 120, 5000)
        s_old = np.sort(F(0.0) + score(tf, fn, w_old, c_old))[::-1]
        s_new = np.sort(F(0.0) + score(tf, fn, w_new, c_new))[::-1]
        r = bound_ratio([w_old, F(0)], [w_new, F(0)], [c_old, c_old], [c_new, c_new], 1)
        worst = min(worst, float(s_old[999]) * r / float(s_new[999]))
    assert 0.995 < worst <= 1.0, worst
    assert int(TABLE[255]) == 2013265944 and K1 == F(1.2)
