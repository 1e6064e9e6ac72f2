"""numpy mirror of fugu_amd/csrc/synth.cpp (test infrastructure).

Used to prove the C generator is bit-exact against its written spec
 and by tests/golden/gen_golden.py.  Also generates the
`name` field and deletion masks of the golden corpora, which only tests use.
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def h2(s, a):
    a = np.asarray(a, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(np.uint64(s) + GOLDEN * (a + np.uint64(1)))


def h3(s, a, b):
    b = np.asarray(b, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return mix64(h2(s, a) + GOLDEN * (b + np.uint64(1)))


class Zipf:
    def __init__(self, v: int, s: float):
        r = np.arange(1, v + 1, dtype=np.float64)
        w = 1.0 / r if s == 1.0 else np.power(r, -s)
        self.cum = np.cumsum(w)  # sequential accumulate == the C loop
        self.total = self.cum[-1]
        self.v = v

    def rank(self, h):
        h = np.asarray(h, dtype=np.uint64)
        u = (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        x = u * self.total
        return np.searchsorted(self.cum[:-1], x, side="right").astype(np.int64) + 1


def doc_lengths(n_docs: int, seed_l: int, len_min: int = 8, len_span: int = 113, doc_begin: int = 0):
    d = np.arange(doc_begin, doc_begin + n_docs, dtype=np.uint64)
    return (np.uint64(len_min) + h2(seed_l, d) % np.uint64(len_span)).astype(np.int64)


def corpus(n_docs: int, vocab: int, s: float, seed_l: int, seed_t: int, len_min: int = 8, len_span: int = 113):
    lens = doc_lengths(n_docs, seed_l, len_min, len_span)
    off = np.zeros(n_docs + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    doc = np.repeat(np.arange(n_docs, dtype=np.uint64), lens)
    j = np.arange(int(off[-1]), dtype=np.uint64) - np.repeat(off[:-1], lens)
    z = Zipf(vocab, s)
    tok = (z.rank(h3(seed_t, doc, j)) - 1).astype(np.uint32)
    return off, tok


def queries(n_queries: int, m_min: int, m_max: int, max_rank: int, s: float, seed_q: int):
    z = Zipf(max_rank, s)
    q_off = [0]
    terms = []
    for q in range(n_queries):
        m = m_min + int(h2(seed_q + 1, q) % np.uint64(m_max - m_min + 1))
        got = []
        i = 0
        while len(got) < m:
            t = int(z.rank(h3(seed_q, q, i))) - 1
            if t not in got:
                got.append(t)
            i += 1
        terms += got
        q_off.append(len(terms))
    return np.array(q_off, np.uint32), np.array(terms, np.uint32)


def names(n_docs: int, vocab: int, seed: int, max_len: int = 3, s: float = 1.0, present_every: int = 3):
    """`name` field of golden corpora: every `present_every`-th doc (by hash)
    gets 1..max_len tokens drawn from Zipf(s) over the first `vocab` ranks."""
    d = np.arange(n_docs, dtype=np.uint64)
    hd = h2(seed, d)
    has = (hd % np.uint64(present_every)) == 0
    lens = np.where(has, 1 + (hd >> np.uint64(8)) % np.uint64(max_len), 0).astype(np.int64)
    off = np.zeros(n_docs + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    doc = np.repeat(d, lens)
    j = np.arange(int(off[-1]), dtype=np.uint64) - np.repeat(off[:-1], lens)
    z = Zipf(vocab, s)
    tok = (z.rank(h3(seed ^ 0xA5A5, doc, j)) - 1).astype(np.uint32)
    return off, tok


def deleted_mask(n_docs: int, seed: int, every: int = 7):
    d = np.arange(n_docs, dtype=np.uint64)
    return ((h2(seed, d) % np.uint64(every)) == 0).astype(np.uint8)


def facet_paths(n_docs: int, seed: int):
    """Explicit `facets` of golden corpora (ObjectRecord.facets, src/object.rs:14-16):
    a namespace facet, data-type / org hierarchy facets, a repeated metadata
    tag (duplicate tokens), an escaped slash, the root facet, and docs with none."""
    out = []
    types = ["doc", "email", "chat", "page"]
    for d in range(n_docs):
        h = int(h2(seed, d))
        if h % 8 == 0:
            out.append([])
            continue
        ns = f"ns{(h >> 3) % 3}"
        f = [f"/namespace/{ns}"]
        if (h >> 5) % 10 < 7:
            f.append(f"/namespace/{ns}/data/{types[(h >> 9) % 4]}")
        if (h >> 12) % 10 < 4:
            f.append("/metadata/tags")
            if (h >> 16) % 2:
                f.append("/metadata/tags")
        if (h >> 20) % 10 < 3:
            f.append(f"org/acme/team{(h >> 24) % 5}/proj{(h >> 28) % 7}")  # no leading '/': normalized
        if (h >> 32) % 50 == 0:
            f.append("/a\\/b/c")
        if (h >> 40) % 100 == 0:
            f.append("/")
        out.append(f)
    return out


def facet_vocab():
    """Facet dictionary of facet_tokens(): encoded facet terms (U+0000 separators)."""
    v = ["", "namespace"]
    v += [f"namespace\x00ns{x}" for x in range(3)]
    v += [f"namespace\x00ns{x}\x00data" for x in range(3)]
    v += [f"namespace\x00ns{x}\x00data\x00{t}" for x in range(3) for t in ("doc", "email", "chat", "page")]
    v += ["metadata", "metadata\x00tags", "org", "org\x00acme"]
    v += [f"org\x00acme\x00team{a}" for a in range(5)]
    v += [f"org\x00acme\x00team{a}\x00proj{b}" for a in range(5) for b in range(7)]
    return v


def facet_tokens(n_docs: int, seed: int):
    """Vectorised FacetTokenizer output of facet_paths()-like facets at any scale
    (ids into facet_vocab()): (facet_off, facet_tok, n_facet_terms)."""
    d = np.arange(n_docs, dtype=np.uint64)
    h = h2(seed, d)
    u = lambda sh, m: ((h >> np.uint64(sh)) % np.uint64(m)).astype(np.int64)  # noqa: E731
    none = u(0, 8) == 0
    ns = u(3, 3)
    has_type = u(5, 10) < 7
    typ = u(9, 4)
    tags = u(12, 10) < 4
    tags2 = tags & (u(16, 2) == 1)
    org = u(20, 10) < 3
    team, proj = u(24, 5), u(28, 7)
    slots = []  # (valid mask, token id) in FacetTokenizer order per facet
    live = ~none
    slots += [(live, 0), (live, 1), (live, 2 + ns)]                                 # /namespace/nsX
    ht = live & has_type
    slots += [(ht, 0), (ht, 1), (ht, 2 + ns), (ht, 5 + ns), (ht, 8 + 4 * ns + typ)]  # .../data/type
    for m in (live & tags, live & tags2):
        slots += [(m, 0), (m, 20), (m, 21)]                                          # /metadata/tags
    og = live & org
    slots += [(og, 0), (og, 22), (og, 23), (og, 24 + team), (og, 29 + 7 * team + proj)]
    valid = np.stack([np.broadcast_to(np.asarray(m), (n_docs,)) for m, _ in slots], axis=1)
    ids = np.stack([np.broadcast_to(np.asarray(t, np.int64), (n_docs,)) for _, t in slots], axis=1)
    cnt = valid.sum(axis=1)
    off = np.zeros(n_docs + 1, np.uint64)
    off[1:] = np.cumsum(cnt)
    tok = ids[valid].astype(np.uint32)
    return off, tok, len(facet_vocab())
