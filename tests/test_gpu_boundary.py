"""The drop-in boundary the Rust host calls, on the MI355X box.

* fg_index_build: postings inverted by the HOST (what a tantivy-segment reader
  would hand over: merged text U name postings, tf per field, fieldnorm ids,
  token totals, deletions, facet postings) must give exactly the snapshot
  fg_index_build_from_docs gives, and the oracle's results.
* Thread safety: tokio workers share one Arc<Dataset>
  (reference src/db/config.rs:93) and call search concurrently while a writer
  commits under its own lock (src/db/core.rs:211).  Eight threads search one
  index while another thread upserts and commits; every result is checked.
"""
import threading
from collections import Counter

import numpy as np
import pytest

from conftest import golden_corpus, golden_facets, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def native():
    from fugu_amd import native as nat
    if nat.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    return nat


@pytest.fixture(scope="module")
def ctx(native):
    return native.Context((0,))


def invert(n_docs, n_terms, off, tok, noff=None, ntok=None, foff=None, ftok=None, n_fterms=0):
    """Host inversion into fg_index_input: merged text U name postings per term
    (docs ascending), tf per field, fieldnorm ids, token totals, facet postings."""
    from oracle import oracle as orc
    per_term = [[] for _ in range(n_terms)]
    fn_text = np.zeros(n_docs, np.uint8)
    fn_name = np.zeros(n_docs, np.uint8)
    tot = [0, 0]
    for d in range(n_docs):
        t = tok[off[d]:off[d + 1]].tolist()
        n = ntok[noff[d]:noff[d + 1]].tolist() if noff is not None else []
        fn_text[d] = orc.fieldnorm_to_id(len(t))
        fn_name[d] = orc.fieldnorm_to_id(len(n))
        tot[0] += len(t)
        tot[1] += len(n)
        ct, cn = Counter(t), Counter(n)
        for term in sorted(set(ct) | set(cn)):
            per_term[term].append((d, ct.get(term, 0), cn.get(term, 0)))
    term_off = np.cumsum([0] + [len(p) for p in per_term]).astype(np.uint64)
    flat = [x for p in per_term for x in p]
    doc = np.array([x[0] for x in flat], np.uint32)
    tf_t = np.array([x[1] for x in flat], np.uint16)
    tf_n = np.array([x[2] for x in flat], np.uint16)
    facets = None
    if foff is not None:
        fl = [[] for _ in range(n_fterms)]
        for d in range(n_docs):
            for f in sorted(set(ftok[foff[d]:foff[d + 1]].tolist())):
                fl[f].append(d)
        facets = (np.cumsum([0] + [len(x) for x in fl]).astype(np.uint64),
                  np.array([d for x in fl for d in x], np.uint32), n_fterms, int(foff[-1]))
    return term_off, doc, tf_t, tf_n, fn_text, fn_name if noff is not None else None, tot, facets


def same_results(a, b):
    sa, da, na = a
    sb, db_, nb = b
    assert np.array_equal(na, nb)
    for i in range(len(na)):
        m = int(na[i])
        assert np.array_equal(da[i, :m], db_[i, :m]), i
        assert np.array_equal(sa[i, :m].view(np.uint32), sb[i, :m].view(np.uint32)), i


@pytest.mark.parametrize("fixture", ["synth_names_2k.json", "facets_2k.json", "synth_10k.json"])
def test_index_build_from_postings_equals_from_docs(native, ctx, fixture):
    from fugu_amd import synth
    fx = load_golden(fixture)
    n, nt, off, tok, no, ntk, dl = golden_corpus(fx)
    fo, ft, nf = golden_facets(fx)
    facets_docs = (fo, ft, nf) if fo is not None else None
    a = native.Index.from_docs(ctx, off, tok, nt, no, ntk, dl, facets=facets_docs)
    term_off, doc, tf_t, tf_n, fn_t, fn_n, tot, facets = invert(n, nt, off, tok, no, ntk, fo, ft, nf)
    b = native.Index.from_postings(ctx, n, term_off, doc, tf_t, tf_n if no is not None else None, fn_t, fn_n, tot,
                                   deleted=dl, facets=facets)
    sa, sb = a.stats(), b.stats()
    assert (sa.n_docs, sa.n_postings, sa.tot_tokens, sa.has_name, sa.n_facet_terms, sa.tot_facet_tokens) == \
        (sb.n_docs, sb.n_postings, sb.tot_tokens, sb.has_name, sb.n_facet_terms, sb.tot_facet_tokens)
    assert sa.avgdl == sb.avgdl
    for t in range(0, nt, max(1, nt // 200)):
        for field in (native.FIELD_TEXT, native.FIELD_NAME, -1):
            assert a.df(t, field) == b.df(t, field)
        assert a.bm25(t)[:2] == b.bm25(t)[:2]
    for (m0, m1, k, mode) in [(1, 3, 10, native.MODE_AND), (2, 4, 100, native.MODE_AND), (2, 5, 50, native.MODE_OR)]:
        q_off, terms = synth.queries(64, m0, m1, max_rank=min(nt, 1 << 14), seed_q=31)
        kw = {}
        if facets is not None:
            fl = [[int(i % nf)] if i % 2 else [] for i in range(64)]  # every other query filtered
            f_off = np.cumsum([0] + [len(x) for x in fl]).astype(np.uint32)
            kw = dict(f_off=f_off, f_terms=np.array([x for f in fl for x in f], np.uint32))
        same_results(a.search_batch(q_off, terms, k, mode=mode, **kw), b.search_batch(q_off, terms, k, mode=mode, **kw))
    # and both equal the fixture's golden hits (numpy restatement)
    from test_gpu_parity import check_fixture_queries
    if "facet_tokens" not in fx:
        check_fixture_queries(native, b, fx["queries"] if "queries" in fx else [])


def test_index_build_rejects_bad_postings(native, ctx):
    n = 4
    good = dict(term_off=np.array([0, 2, 3], np.uint64), doc=np.array([0, 2, 1], np.uint32),
                tf_text=np.array([1, 2, 1], np.uint16), tf_name=None, fn_text=np.ones(n, np.uint8), fn_name=None,
                tot_tokens=(5, 0))
    ix = native.Index.from_postings(ctx, n, **good)
    assert ix.stats().n_postings == 3 and ix.df(0, native.FIELD_TEXT) == 2 and not ix.stats().has_name
    bad = [
        dict(good, term_off=np.array([1, 2, 3], np.uint64)),             # term_off[0] != 0
        dict(good, term_off=np.array([0, 3, 2], np.uint64)),             # not monotone
        dict(good, doc=np.array([2, 0, 1], np.uint32)),                  # not ascending
        dict(good, doc=np.array([0, 9, 1], np.uint32)),                  # doc >= n_docs
        dict(good, tf_text=np.array([1, 0, 1], np.uint16)),              # tf 0 in both fields
    ]
    for kw in bad:
        with pytest.raises(native.FuguError) as e:
            native.Index.from_postings(ctx, n, **kw)
        assert e.value.code == native.FG_EINVAL, kw


def test_concurrent_searches_and_commit(native, ctx):
    """8 threads x fg_search_batch on one snapshot (each on its own HIP stream)
    while a writer thread upserts + commits a namespace of the host mirror."""
    from fugu_amd import db as fdb
    from fugu_amd import synth
    from oracle import oracle as orc
    corp = synth.corpus(200_000)
    ix = native.Index.from_docs(ctx, corp.off, corp.tok, synth.VOCAB, threads=16)
    ref = orc.OracleIndex(synth.VOCAB, corp.off, corp.tok, threads=16)
    work = []
    for t in range(8):
        mode = native.MODE_OR if t % 3 == 2 else native.MODE_AND
        q_off, terms = synth.queries(48, 1 if mode == native.MODE_AND else 2, 4, seed_q=100 + t)
        k = 100 if mode == native.MODE_AND else 200
        work.append((q_off, terms, k, mode, ref.search_batch(q_off, terms, k, mode=mode, threads=4)[:3]))
    errors = []

    def searcher(t):
        try:
            q_off, terms, k, mode, (rs, rd, rn) = work[t]
            for _ in range(6):
                s, d, n = ix.search_batch(q_off, terms, k, mode=mode)
                assert np.array_equal(n, rn), t
                for i in range(len(n)):
                    m = int(n[i])
                    assert np.array_equal(d[i, :m], rd[i, :m]), (t, i)
                    assert np.allclose(s[i, :m], rs[i, :m], rtol=1e-5, atol=0), (t, i)
        except Exception as e:  # noqa: BLE001
            errors.append(("search", t, repr(e)))

    # the writer: docs "w<a> w<b> ..." in batches, a commit after each batch
    rng = np.random.default_rng(3)
    docs = [[f"w{x}" for x in rng.zipf(1.3, rng.integers(3, 12)) % 300] for _ in range(3000)]
    d_ = fdb.Database(ctx)
    d_.create_namespace("conc")

    def writer():
        try:
            for b in range(0, len(docs), 600):
                for i in range(b, b + 600):
                    d_.upsert(fdb.ObjectRecord(id=f"d{i}", text=" ".join(docs[i])), namespace="conc")
                d_.commit("conc")
                assert d_.doc_count("conc") == (b + 600, b + 600)
        except Exception as e:  # noqa: BLE001
            errors.append(("commit", repr(e)))

    th = [threading.Thread(target=searcher, args=(t,)) for t in range(8)] + [threading.Thread(target=writer)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=300)
    assert not any(x.is_alive() for x in th), "a thread did not finish"
    assert not errors, errors
    # the committed namespace answers like the oracle over the same tokens
    vocab = {}
    for dd in docs:
        for w in dd:
            vocab.setdefault(w, len(vocab))
    toks = [[vocab[w] for w in dd] for dd in docs]
    off = np.cumsum([0] + [len(t) for t in toks]).astype(np.uint64)
    ref2 = orc.OracleIndex(len(vocab), off, np.array([x for t in toks for x in t], np.uint32), threads=4)
    for a, b in [("w1", "w2"), ("w3", "w5"), ("w7", "w1")]:
        got = d_.search("conc", f"{a} AND {b}", 0, 20)
        rs, rd = ref2.search([vocab[a], vocab[b]], 20)
        assert [g[1] for g in got] == rd.tolist()
        assert np.allclose([g[0] for g in got], rs, rtol=1e-5, atol=0)


def test_index_build_global_postings_segment(native, ctx):
    """fg_index_build_global: one segment's host-inverted postings scored with
    the namespace's statistics equal fg_index_build_from_docs_global's snapshot
    of the same docs (the per-segment build of a tantivy host)."""
    from fugu_amd import synth
    fx = load_golden("synth_names_2k.json")
    n, nt, off, tok, no, ntk, dl = golden_corpus(fx)
    cut = 1200  # segment = docs [cut, n); the namespace = all n docs
    so, st = off[cut:] - off[cut], tok[off[cut]:]
    sno, snt = no[cut:] - no[cut], ntk[no[cut]:]
    g = native.docs_stats(off, tok, nt, no, ntk)
    a = native.Index.from_docs(ctx, so, st, nt, sno, snt, dl[cut:], global_stats=g)
    term_off, doc, tf_t, tf_n, fn_t, fn_n, tot, _ = invert(n - cut, nt, so, st, sno, snt)
    b = native.Index.from_postings(ctx, n - cut, term_off, doc, tf_t, tf_n, fn_t, fn_n, tot, deleted=dl[cut:],
                                   global_stats=g)
    assert a.stats().avgdl == b.stats().avgdl
    for (m0, m1, k, mode) in [(1, 3, 10, native.MODE_AND), (2, 5, 50, native.MODE_OR)]:
        q_off, terms = synth.queries(64, m0, m1, max_rank=min(nt, 1 << 14), seed_q=33)
        same_results(a.search_batch(q_off, terms, k, mode=mode), b.search_batch(q_off, terms, k, mode=mode))
