"""numpy reference of the cross-shard top-k merge (test infrastructure)."""
import numpy as np


def merge_topk_numpy(sc, dc, nn, k):
    """sc/dc: [S, nq, k] per-shard lists in (score desc, doc asc) order; nn: [S, nq].
    Returns merged (score, doc, shard, n) by (score desc, shard asc, doc asc)."""
    S, nq, _ = sc.shape
    out_s = np.zeros((nq, k), np.float32)
    out_d = np.zeros((nq, k), np.uint32)
    out_sh = np.zeros((nq, k), np.int32)
    out_n = np.zeros(nq, np.int32)
    for q in range(nq):
        rows = [(float(sc[s, q, i]), s, int(dc[s, q, i])) for s in range(S) for i in range(int(nn[s, q]))]
        rows.sort(key=lambda r: (-r[0], r[1], r[2]))
        rows = rows[:k]
        out_n[q] = len(rows)
        for i, (a, s, d) in enumerate(rows):
            out_s[q, i], out_sh[q, i], out_d[q, i] = a, s, d
    return out_s, out_d, out_sh, out_n
