"""The ratio bounds a rescore uses instead of re-scoring on the device (round 6:
query-time BM25, fugu.cpp relate_stats / term_ratio / term_kth_now), checked on
the CPU.  For random old (build) and new BM25 statistics and random postings
(tf, fieldnorm id, one or two fields), every posting's score under the new
statistics, in tantivy's f32 order as the kernels form it at query time, lies
between rdn and rup times its build-time score, where per term
  rup = (1 + 2^-19) x max over its fields of (w_new / w_old) x max(1, max_fn (1 + c_old) / (1 + c_new)),
  rdn = (1 - 2^-19) x min over its fields of (w_new / w_old) x min(1, min_fn (1 + c_old) / (1 + c_new)).
So the build-time bounds scaled by rup -- in the kernels' f32 arithmetic: the
tile / bucket maxima times rup, and the u8 sub-tile bounds quantized against
the unscaled tile maximum then read against the scaled one -- still bound every
current score, and the build-time K-th scores times rdn stay below the current
K-th: valid starting thresholds, so the searches' hits cannot change.
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


def ratios(w_old, w_new, c_old, c_new, fields):
    """(rdn, rup) as f32, as fugu.cpp term_ratio rounds them (down / up)."""
    lo, hi = math.inf, 0.0
    for f in range(fields):
        q = (1.0 + c_old[f].astype(np.float64)) / (1.0 + c_new[f].astype(np.float64))
        q = q[np.isfinite(q)]
        cup = max(1.0, float(q.max())) if len(q) else 1.0
        cdn = min(1.0, float(q.min())) if len(q) else 1.0
        if w_old[f] > 0:
            r = float(w_new[f]) / float(w_old[f])
            hi, lo = max(hi, r * cup), min(lo, r * cdn)
    m = 2.0 ** -19
    u, d = hi * (1 + m), lo * (1 - m)
    fu, fd = np.float32(u), np.float32(d)
    if float(fu) < u:
        fu = np.nextafter(fu, np.float32(np.inf))
    if float(fd) > d:
        fd = np.nextafter(fd, np.float32(0))
    return fd, fu


def q8_step(M):
    return np.float32(M * np.float32(1.0 / 255.0))


def q8_bound(q, M):
    return M if q >= 255 else np.float32(np.float32(q) * q8_step(M))


def quant8(s, M):
    """fg_internal.h quant8: the least q with q8_bound(q, M) >= s."""
    st = q8_step(M)
    if not (st > 0) or not (s < M):
        return 255
    q = int(min(254.0, math.ceil(float(np.float32(s / st)))))
    while q < 255 and q8_bound(q, M) < s:
        q += 1
    return q


def _trial(rng, trial):
    fields = 1 + (trial % 2)
    n_old = int(rng.integers(1000, 2_000_000))
    n_new = n_old + int(rng.integers(0, 3 * n_old))
    P = int(rng.integers(10, 3000))
    df_old = [int(rng.integers(1, min(P, n_old) + 1)) for _ in range(2)]
    df_new = [min(d + int(rng.integers(0, n_new - n_old + 1)), n_new) for d in df_old]
    w_old = [weight(df_old[f], n_old) for f in range(2)]
    w_new = [weight(df_new[f], n_new) for f in range(2)]
    avg_old = [F(rng.uniform(5, 200)) for _ in range(2)]
    avg_new = [F(a * F(rng.uniform(0.25, 4.0))) for a in avg_old]
    c_old = [cache(a) for a in avg_old]
    c_new = [cache(a) for a in avg_new]
    tf = [rng.integers(0 if fields == 2 else 1, 400, P) for _ in range(2)]
    if fields == 1:
        tf[1] = np.zeros(P, np.int64)
    else:
        tf[0] = np.where((tf[0] == 0) & (tf[1] == 0), 1, tf[0])
    fn = [rng.integers(0, 256, P) for _ in range(2)]
    s_old = (F(0.0) + score(tf[0], fn[0], w_old[0], c_old[0])) + score(tf[1], fn[1], w_old[1], c_old[1])
    s_new = (F(0.0) + score(tf[0], fn[0], w_new[0], c_new[0])) + score(tf[1], fn[1], w_new[1], c_new[1])
    return P, s_old.astype(np.float32), s_new.astype(np.float32), ratios(w_old, w_new, c_old, c_new, fields)


def test_scaled_bounds_hold_every_current_score():
    rng = np.random.default_rng(12)
    checked = 0
    for trial in range(300):
        P, s_old, s_new, (rdn, rup) = _trial(rng, trial)
        # the tile / bucket maximum times rup, as k_disj's R phase (f32 product)
        M = np.float32(s_old.max())
        Ms = np.float32(M * rup)
        assert (s_new <= Ms).all(), (trial, float(Ms), float(s_new.max()))
        # a u8 sub-tile bound quantized at build against M, read against M * rup
        for blk in np.array_split(np.arange(P), 8):
            if len(blk) == 0:
                continue
            q = quant8(np.float32(s_old[blk].max()), M)
            assert (s_new[blk] <= q8_bound(q, Ms)).all(), (trial, q)
        # the K-th seeds times rdn (rounded down), as term_kth_now
        o = np.sort(s_old)[::-1]
        n = np.sort(s_new)[::-1]
        for K in (1, 10, 20, 100, 1000):
            if K > P:
                continue
            b = np.float32(float(o[K - 1]) * float(rdn))
            if float(b) > float(o[K - 1]) * float(rdn):
                b = np.nextafter(b, np.float32(0))
            assert b <= n[K - 1], (trial, K, float(b), float(n[K - 1]))
            checked += 1
    assert checked > 800


def test_ratio_bounds_are_tight_for_small_statistics_changes():
    """A commit of 1% more docs: the scaled K-th stays within 0.5% of the new
    K-th, the scaled maximum within 0.5% above the new maximum."""
    rng = np.random.default_rng(4)
    worst_lo, worst_hi = 1.0, 1.0
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
        rdn, rup = ratios([w_old, F(0)], [w_new, F(0)], [c_old, c_old], [c_new, c_new], 1)
        worst_lo = min(worst_lo, float(s_old[999]) * float(rdn) / float(s_new[999]))
        worst_hi = max(worst_hi, float(s_old[0]) * float(rup) / float(s_new[0]))
    assert 0.995 < worst_lo <= 1.0, worst_lo
    assert 1.0 <= worst_hi < 1.005, worst_hi
    assert int(TABLE[255]) == 2013265944 and K1 == F(1.2)
