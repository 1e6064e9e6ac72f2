"""Golden-vector generator: an INDEPENDENT numpy restatement of tantivy 0.24.1's
scoring as fugu uses it, brute force (no skip lists,
no leapfrog, no TopN pruning).  It writes the committed fixtures under
tests/golden/ that pin the C oracle (oracle/fugu_oracle.c) and, through it, the
gfx950 path.

Parity status: "parity unpinned" by the reference (fugu ships no search test
or golden vector and cannot be compiled or imported here).
These vectors are pinned to (1) the hand-derived Appendix C KAT, reproduced
here bit for bit, and (2) the published tantivy formulas.

Run:  python tests/golden/gen_golden.py      (writes tests/golden/*.json)
"""
from __future__ import annotations

import ctypes
import ctypes.util
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import facet_ref as fr  # noqa: E402
import synth_ref as sr  # noqa: E402

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.logf.restype = ctypes.c_float
_libm.logf.argtypes = [ctypes.c_float]

F = np.float32
K1 = F(1.2)
B = F(0.75)


def fieldnorm_table():
    t = list(range(41))
    v, step = 40, 2
    while len(t) < 256:
        for _ in range(8):
            if len(t) == 256:
                break
            v += step
            t.append(v)
        step *= 2
    return np.array(t, np.uint64)


TABLE = fieldnorm_table()
assert int(TABLE[255]) == 2013265944


def fieldnorm_id(n):
    return (np.searchsorted(TABLE, np.asarray(n, np.uint64), side="right") - 1).astype(np.int64)


def idf(df, n):
    x = (F(n - df) + F(0.5)) / (F(df) + F(0.5))
    return F(_libm.logf(ctypes.c_float(F(1.0) + x)))


_WCACHE = {}


def weight(df, n):
    key = (df, n)
    if key not in _WCACHE:
        _WCACHE[key] = idf(df, n) * (F(1.0) + K1)
    return _WCACHE[key]


def cache(avgdl):
    return np.array([K1 * ((F(1.0) - B) + (B * F(TABLE[i])) / avgdl) for i in range(256)], np.float32)


class Field:
    def __init__(self, n_docs, off, tok):
        self.post = {}  # term -> {doc: tf}
        lens = np.zeros(n_docs, np.int64)
        if off is not None:
            lens = (off[1:] - off[:-1]).astype(np.int64)
            for d in range(n_docs):
                toks, cnts = np.unique(tok[int(off[d]):int(off[d + 1])], return_counts=True)
                for t, c in zip(toks.tolist(), cnts.tolist()):
                    self.post.setdefault(t, {})[d] = c
        self.fn = fieldnorm_id(lens)
        self.total = int(lens.sum())
        self.avgdl = F(self.total) / F(n_docs)
        self.cache = cache(self.avgdl)

    def df(self, t):
        return len(self.post.get(t, {}))


class Index:
    def __init__(self, n_docs, text, name=None, deleted=None, facets=None):
        self.n = n_docs
        self.f = [Field(n_docs, *text), Field(n_docs, *(name if name else (None, None)))]
        self.deleted = deleted
        # facet field (schemas.rs:20, Basic record option, no fieldnorms): facets[d] =
        # FacetTokenizer token ids of doc d, duplicates included (total_num_tokens)
        self.fpost = {}
        ftot = 0
        for d, toks in enumerate(facets or []):
            ftot += len(toks)
            for t in toks:
                self.fpost.setdefault(t, set()).add(d)
        self.fc1 = cache(F(ftot) / F(n_docs))[1]  # FieldNormReader::constant(max_doc, 1) -> id 1

    def facet_clause(self, t, d):
        docs = self.fpost.get(t, set())
        if d not in docs:
            return None
        return weight(len(docs), self.n) * (F(1.0) / (F(1.0) + self.fc1))  # tf = 1

    def term_score(self, t, d):
        s = F(0.0)
        for fld in self.f:
            tf = fld.post.get(t, {}).get(d)
            if tf:
                w = weight(fld.df(t), self.n)
                tff = F(tf)
                s = s + w * (tff / (tff + fld.cache[fld.fn[d]]))
        return s

    def docs(self, t):
        return set(self.f[0].post.get(t, {})) | set(self.f[1].post.get(t, {}))

    def cost(self, t):
        return self.f[0].df(t) + self.f[1].df(t)

    def search(self, terms, k, mode, fterms=None):
        if fterms or not terms:
            return self.search_filtered(terms, k, mode, fterms or [])
        if mode == "and":
            order = sorted(range(len(terms)), key=lambda i: (self.cost(terms[i]), i))
            ts = [terms[i] for i in order]
            cand = set.intersection(*[self.docs(t) for t in ts])
            hits = []
            for d in cand:
                if len(ts) == 1:
                    s = self.term_score(ts[0], d)
                else:
                    others = F(0.0)
                    for t in ts[2:]:
                        others = others + self.term_score(t, d)
                    s = (self.term_score(ts[0], d) + self.term_score(ts[1], d)) + others
                hits.append((s, d))
        else:
            cand = set().union(*[self.docs(t) for t in terms])
            hits = []
            for d in cand:
                s = F(0.0)
                for t in terms:
                    if d in self.docs(t):
                        s = s + self.term_score(t, d)
                hits.append((s, d))
        if self.deleted is not None:
            hits = [h for h in hits if not self.deleted[h[1]]]
        hits.sort(key=lambda h: (-float(h[0]), h[1]))
        return [[int(d), int(np.float32(s).view(np.uint32))] for s, d in hits[:k]]


    def search_occ(self, terms, occur, k):
        """BooleanQuery with per-clause occurs (query/boolean_query/boolean_weight.rs
        complex_scorer): Must -> the clause / Intersection (cost order, left + right
        + others); Should with Must -> RequiredOptionalScorer: (0.0 + req) + the
        Should union when it is on the doc; Should alone -> the union from 0.0 in
        clause order; MustNot -> Exclude; neither Must nor Should -> no hits."""
        M = [t for t, o in zip(terms, occur) if o == "must"]
        S = [t for t, o in zip(terms, occur) if o == "should"]
        X = [t for t, o in zip(terms, occur) if o == "must_not"]
        if not M and not S:
            return []
        excl = set().union(*[self.docs(t) for t in X]) if X else set()
        if M:
            order = sorted(range(len(M)), key=lambda i: (self.cost(M[i]), i))
            ts = [M[i] for i in order]
            cand = set.intersection(*[self.docs(t) for t in ts])
        else:
            cand = set().union(*[self.docs(t) for t in S])
        hits = []
        for d in cand - excl:
            opt, any_s = F(0.0), False
            for t in S:
                if d in self.docs(t):
                    opt = opt + self.term_score(t, d)
                    any_s = True
            if M:
                if len(ts) == 1:
                    req = self.term_score(ts[0], d)
                else:
                    others = F(0.0)
                    for t in ts[2:]:
                        others = others + self.term_score(t, d)
                    req = (self.term_score(ts[0], d) + self.term_score(ts[1], d)) + others
                sc = F(0.0) + req
                if any_s:
                    sc = sc + opt
            else:
                sc = opt
            hits.append((sc, d))
        if self.deleted is not None:
            hits = [h for h in hits if not self.deleted[h[1]]]
        hits.sort(key=lambda h: (-float(h[0]), h[1]))
        return [[int(d), int(np.float32(s).view(np.uint32))] for s, d in hits[:k]]

    def search_filtered(self, terms, k, mode, fterms):
        """Bool[Must(text), Must(facet union)], the facet union alone, or AllQuery
        (src/db/search.rs:129-150); a union sums its matching clauses from 0.0
        in clause order, an Intersection of two children is left + right."""
        text = None
        if terms:
            text = dict(self._all_hits(terms, mode))
        hits = []
        cand = range(self.n) if text is None else sorted(text)
        for d in cand:
            if fterms:
                fs = F(0.0)
                any_ = False
                for t in fterms:
                    v = self.facet_clause(t, d)
                    if v is not None:
                        fs = fs + v
                        any_ = True
                if not any_:
                    continue
                s = fs if text is None else text[d] + fs
            else:
                s = F(1.0)  # AllQuery (text is None here)
            hits.append((s, d))
        if self.deleted is not None:
            hits = [h for h in hits if not self.deleted[h[1]]]
        hits.sort(key=lambda h: (-float(h[0]), h[1]))
        return [[int(d), int(np.float32(s).view(np.uint32))] for s, d in hits[:k]]

    def _all_hits(self, terms, mode):
        # every text match with its score, deletions not applied
        keep, self.deleted = self.deleted, None
        try:
            out = []
            for d, b in Index.search(self, terms, 1 << 40, mode):
                out.append((d, F(np.uint32(b).view(np.float32))))
            return out
        finally:
            self.deleted = keep


def write(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, separators=(",", ":"))
        f.write("\n")


def kat():
    # SURVEY.md Appendix C
    vocab = {"a": 0, "b": 1, "c": 2, "d": 3, "e": 4}
    docs = ["a b c", "a a b", "b c d e"]
    toks = [[vocab[w] for w in d.split()] for d in docs]
    off = np.cumsum([0] + [len(t) for t in toks]).astype(np.uint64)
    tok = np.array(sum(toks, []), np.uint32)
    ix = Index(3, (off, tok))
    hits = ix.search([0, 1], 10, "and")
    assert hits == [[1, int(np.float32(0.80418402).view(np.uint32))], [0, int(np.float32(0.62927824).view(np.uint32))]], hits
    assert abs(float(idf(2, 3)) - 0.47000366) < 1e-7 and abs(float(idf(3, 3)) - 0.13353144) < 1e-7
    assert abs(float(ix.f[0].cache[3]) - 1.11) < 1e-6
    assert fieldnorm_id(41) == 40 and fieldnorm_id(100) == 57 and TABLE[57] == 96 and fieldnorm_id(1000) == 87
    write("kat_appendix_c.json", {
        "corpus": {"kind": "tokens", "n_terms": 5, "text": [t for t in toks]},
        "queries": [{"terms": [0, 1], "mode": "and", "k": 10, "hits": hits},
                    {"terms": [0], "mode": "and", "k": 10, "hits": ix.search([0], 10, "and")},
                    {"terms": [0, 1], "mode": "or", "k": 10, "hits": ix.search([0, 1], 10, "or")},
                    {"terms": [0, 3], "mode": "and", "k": 10, "hits": ix.search([0, 3], 10, "and")}],
    })


def synth_set(fname, n_docs, vocab, s, seeds, qspecs, name_cfg=None, del_cfg=None):
    off, tok = sr.corpus(n_docs, vocab, s, seeds[0], seeds[1])
    name = sr.names(n_docs, **name_cfg) if name_cfg else None
    deleted = sr.deleted_mask(n_docs, **del_cfg) if del_cfg else None
    ix = Index(n_docs, (off, tok), name, deleted)
    queries = []
    for (nq, mmin, mmax, max_rank, qseed, mode, k) in qspecs:
        q_off, q_terms = sr.queries(nq, mmin, mmax, max_rank, 1.0, qseed)
        for i in range(nq):
            terms = q_terms[q_off[i]:q_off[i + 1]].tolist()
            queries.append({"terms": terms, "mode": mode, "k": k, "hits": ix.search(terms, k, mode)})
    write(fname, {
        "corpus": {"kind": "synth", "n_docs": n_docs, "vocab": vocab, "s": s, "seed_l": seeds[0], "seed_t": seeds[1],
                   "name": name_cfg, "deleted": del_cfg},
        "queries": queries,
    })
    return ix


def edge():
    # hand-made corpora for the edge cases the reference path has
    # term ids: 0 in every doc (df = N), ties via identical docs, long docs
    toks = [
        [0, 1, 2], [0, 1, 2], [0, 1, 2],          # three identical docs -> score ties, doc asc
        [0, 3] + [4] * 50,                        # long doc: fieldnorm 52 -> id 46 (quantized)
        [0, 3, 3, 3] + [5] * 200,                 # fieldnorm 204 -> id 66
        [0, 1],
        [0, 6, 7],
        [0] * 120,
    ]
    off = np.cumsum([0] + [len(t) for t in toks]).astype(np.uint64)
    tok = np.array(sum(toks, []), np.uint32)
    name_toks = [[1], [], [3, 3], [], [6], [], [], [1, 2]]
    noff = np.cumsum([0] + [len(t) for t in name_toks]).astype(np.uint64)
    ntok = np.array(sum(name_toks, []), np.uint32)
    deleted = np.array([0, 1, 0, 0, 0, 0, 0, 0], np.uint8)
    n_terms = 10
    qs = [([0], "and", 3), ([0], "and", 20), ([0, 1], "and", 10), ([1, 2], "and", 10), ([1, 2], "and", 1),
          ([0, 3], "and", 10), ([3], "and", 10), ([6, 7], "and", 10), ([8], "and", 10), ([0, 9], "and", 10),
          ([2, 1, 0], "and", 10), ([0, 0], "and", 10), ([1, 3, 6], "or", 10), ([4], "and", 5)]
    sets = []
    for (with_name, with_del) in [(False, False), (True, False), (True, True)]:
        ix = Index(len(toks), (off, tok), (noff, ntok) if with_name else None, deleted if with_del else None)
        sets.append({
            "name": with_name, "deleted": with_del,
            "queries": [{"terms": t, "mode": m, "k": k, "hits": ix.search(t, k, m)} for (t, m, k) in qs],
        })
    write("edge_cases.json", {
        "corpus": {"kind": "tokens", "n_terms": n_terms, "text": toks, "name_tokens": name_toks,
                   "deleted": deleted.tolist()},
        "sets": sets,
    })


MISSING = 0xFFFFFFFF


def facets_set(fname, n_docs, vocab, seeds, facet_seed):
    """Facet filters: text AND / OR + facet clauses, facet-only
    queries (empty text) and AllQuery, on a corpus with names and deletions."""
    off, tok = sr.corpus(n_docs, vocab, 1.0, seeds[0], seeds[1])
    name_cfg = {"vocab": 1 << 9, "seed": 4243}
    del_cfg = {"seed": 78}
    name = sr.names(n_docs, **name_cfg)
    deleted = sr.deleted_mask(n_docs, **del_cfg)
    paths = sr.facet_paths(n_docs, facet_seed)
    fvocab, ftoks = {}, []
    for plist in paths:
        ids = []
        for p in plist:
            enc = fr.from_text(fr.normalize(p))
            for t in fr.tokens(enc):
                ids.append(fvocab.setdefault(t, len(fvocab)))
        ftoks.append(ids)
    ix = Index(n_docs, (off, tok), name, deleted, ftoks)
    nfv = len(fvocab)
    queries = []
    qo, qt = sr.queries(160, 1, 3, 1 << 9, 1.0, 31)
    for i in range(160):
        terms = qt[qo[i]:qo[i + 1]].tolist()
        h = int(sr.h2(97, i))
        nfc = 1 + h % 3
        fterms = [int(sr.h3(98, i, j) % np.uint64(nfv)) for j in range(nfc)]
        if h % 17 == 0:
            fterms.append(MISSING)
        if h % 23 == 0:
            fterms.append(fterms[0])  # the same facet twice: two clauses
        kind = (h >> 8) % 8
        if kind < 4:
            mode = "and"
        elif kind < 6:
            mode = "or" if len(terms) > 1 else "and"
        else:
            mode, terms = "and", []  # facet-only (empty text query)
        k = [10, 10, 100, 1][(h >> 12) % 4]
        queries.append({"terms": terms, "fterms": fterms, "mode": mode, "k": k,
                        "hits": ix.search(terms, k, mode, fterms)})
    for k in (1, 10, 300):
        queries.append({"terms": [], "fterms": [], "mode": "and", "k": k, "hits": ix.search([], k, "and", [])})
    write(fname, {
        "corpus": {"kind": "synth", "n_docs": n_docs, "vocab": vocab, "s": 1.0, "seed_l": seeds[0],
                   "seed_t": seeds[1], "name": name_cfg, "deleted": del_cfg, "facet_seed": facet_seed},
        "facet_vocab": list(fvocab),
        "facet_tokens": ftoks,
        "queries": queries,
    })


OCCURS = ("must", "should", "must_not")


def occur_set(fname, n_docs, vocab, seeds):
    """Must / Should / MustNot mixes (`+a b -c`, `a OR b`): 2-5 terms with
    per-clause occurs drawn from the query hash, on a corpus with names and
    deletions; plus hand-picked edges (a term both Must and MustNot, missing
    terms in each role, only MustNot, duplicate Should terms)."""
    off, tok = sr.corpus(n_docs, vocab, 1.0, seeds[0], seeds[1])
    name_cfg = {"vocab": 1 << 9, "seed": 4244}
    del_cfg = {"seed": 79}
    ix = Index(n_docs, (off, tok), sr.names(n_docs, **name_cfg), sr.deleted_mask(n_docs, **del_cfg))
    queries = []
    qo, qt = sr.queries(192, 2, 5, 1 << 9, 1.0, 37)
    for i in range(192):
        terms = qt[qo[i]:qo[i + 1]].tolist()
        h = int(sr.h2(41, i))
        occ = [OCCURS[(h >> (2 * j)) % 3] for j in range(len(terms))]
        if i % 4 == 0:  # at least one Must
            occ[0] = "must"
        k = [10, 100, 1, 37][(h >> 20) % 4]
        queries.append({"terms": terms, "occur": occ, "k": k, "hits": ix.search_occ(terms, occ, k)})
    edges = [([1, 2, 1], ["must", "should", "must_not"]), ([MISSING, 3], ["must", "should"]),
             ([3, MISSING], ["must", "should"]), ([3, MISSING], ["should", "must_not"]),
             ([4, 5], ["must_not", "must_not"]), ([6, 6, 7], ["should", "should", "must_not"]),
             ([8, 9, 10], ["must", "must", "should"]), ([11], ["should"]), ([12, 13], ["must", "must_not"])]
    for terms, occ in edges:
        for k in (10, 1000):
            queries.append({"terms": terms, "occur": occ, "k": k, "hits": ix.search_occ(terms, occ, k)})
    write(fname, {
        "corpus": {"kind": "synth", "n_docs": n_docs, "vocab": vocab, "s": 1.0, "seed_l": seeds[0],
                   "seed_t": seeds[1], "name": name_cfg, "deleted": del_cfg},
        "queries": queries,
    })


def main():
    occur_set("occur_2k.json", 2_000, 1 << 11, (0x5EED4, 103))
    kat()
    edge()
    facets_set("facets_2k.json", 2_000, 1 << 12, (0x5EED3, 101), 555)
    seeds = (0x5EED1, 20250808)
    # config-1 scale (10k docs): 2-term AND (C1), 3-term AND (C2/C3 shape), mixed 1-5, OR
    synth_set("synth_10k.json", 10_000, 1 << 20, 1.0, seeds,
              [(48, 2, 2, 1 << 14, 7, "and", 10), (48, 3, 3, 1 << 14, 11, "and", 10),
               (48, 1, 5, 1 << 14, 13, "and", 10), (8, 3, 3, 1 << 14, 17, "and", 100),
               (16, 2, 4, 1 << 14, 19, "or", 10)])
    # `name` field present + deletions, smaller vocabulary so names collide with text
    synth_set("synth_names_2k.json", 2_000, 1 << 12, 1.0, (0x5EED2, 99),
              [(48, 1, 4, 1 << 9, 23, "and", 10), (16, 2, 3, 1 << 9, 29, "or", 10)],
              name_cfg={"vocab": 1 << 9, "seed": 4242}, del_cfg={"seed": 77})


if __name__ == "__main__":
    main()
