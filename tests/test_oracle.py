"""The CPU oracle (oracle/fugu_oracle.c) against every committed golden vector.

Pins the restatement before it is trusted as the GPU checker: the Appendix C
hand KAT, the edge-case corpora (df = N, ties, quantized fieldnorms, `name`
unions, deletions, empty and missing-term intersections, k > |I|, k = 1) and
the independent numpy restatement on 10k / 2k-doc synthetic corpora.
Bit-exact: doc ids and f32 score bits.
"""
import numpy as np
import pytest

from conftest import golden_corpus, golden_facets, hits_of, load_golden, tokens_to_csr
from oracle import oracle as orc


def test_fieldnorm_table_and_kat_constants():
    t = orc.fieldnorm_table()
    assert t[255] == 2013265944 and t[40] == 40 and t[41] == 42 and t[57] == 96
    assert orc.fieldnorm_to_id(41) == 40
    assert orc.fieldnorm_to_id(100) == 57
    assert orc.fieldnorm_to_id(1000) == 87
    assert orc.fieldnorm_to_id(0) == 0
    assert orc.fieldnorm_to_id(2**32 - 1) == 255
    assert abs(orc.idf(2, 3) - 0.47000366) < 1e-7
    assert abs(orc.idf(3, 3) - 0.13353144) < 1e-7
    # df = N: idf -> ln(1 + 0.5 / (N + 0.5))
    assert abs(orc.idf(1000, 1000) - np.log1p(0.5 / 1000.5)) < 1e-6
    assert abs(orc.bm25_cache(np.float32(10 / 3))[3] - 1.11) < 1e-6


def _mode(m):
    return orc.AND if m == "and" else orc.OR


def test_kat_appendix_c():
    fx = load_golden("kat_appendix_c.json")
    n, nt, off, tok, *_ = golden_corpus(fx)
    ix = orc.OracleIndex(nt, off, tok)
    assert ix.avgdl() == np.float32(10) / np.float32(3)
    for q in fx["queries"]:
        s, d = ix.search(q["terms"], q["k"], _mode(q["mode"]))
        assert hits_of(s, d) == q["hits"], q
    s, d = ix.search([0, 1], 10)
    assert d.tolist() == [1, 0]
    assert abs(s[0] - 0.80418402) < 1e-7 and abs(s[1] - 0.62927824) < 1e-7


def test_edge_cases():
    fx = load_golden("edge_cases.json")
    c = fx["corpus"]
    off, tok = tokens_to_csr(c["text"])
    noff, ntok = tokens_to_csr(c["name_tokens"])
    dl = np.array(c["deleted"], np.uint8)
    for st in fx["sets"]:
        ix = orc.OracleIndex(c["n_terms"], off, tok, noff if st["name"] else None, ntok if st["name"] else None,
                             dl if st["deleted"] else None)
        for q in st["queries"]:
            s, d = ix.search(q["terms"], q["k"], _mode(q["mode"]))
            assert hits_of(s, d) == q["hits"], (st["name"], st["deleted"], q)


@pytest.mark.parametrize("name", ["synth_10k.json", "synth_names_2k.json"])
def test_synth_golden(name):
    fx = load_golden(name)
    n, nt, off, tok, no, ntk, dl = golden_corpus(fx)
    ix = orc.OracleIndex(nt, off, tok, no, ntk, dl, threads=4)
    bad = []
    for q in fx["queries"]:
        s, d = ix.search(q["terms"], q["k"], _mode(q["mode"]))
        if hits_of(s, d) != q["hits"]:
            bad.append(q["terms"])
    assert not bad, bad


def test_batch_matches_single_and_latencies():
    fx = load_golden("synth_10k.json")
    n, nt, off, tok, *_ = golden_corpus(fx)
    ix = orc.OracleIndex(nt, off, tok, threads=4)
    qs = [q for q in fx["queries"] if q["mode"] == "and" and q["k"] == 10]
    q_off = np.cumsum([0] + [len(q["terms"]) for q in qs]).astype(np.uint32)
    q_terms = np.array([t for q in qs for t in q["terms"]], np.uint32)
    sc, dc, cnt, wall, lat = ix.search_batch(q_off, q_terms, 10, threads=3, latencies=True)
    assert wall > 0 and (lat > 0).all()
    for i, q in enumerate(qs):
        assert hits_of(sc[i, :cnt[i]], dc[i, :cnt[i]]) == q["hits"]


def test_bytes_model_definition():
    # 3 docs KAT corpus: 'a AND b' -> lead a (df 2): B_merge = 8*(2+3), B_skip = 8*2 + 1024*1 + 4*1
    fx = load_golden("kat_appendix_c.json")
    n, nt, off, tok, *_ = golden_corpus(fx)
    ix = orc.OracleIndex(nt, off, tok)
    bm, bs, b, isz = ix.bytes_model([0, 1], 100)
    assert bm == 40 and bs == 16 + 1024 + 4 and isz == 2
    assert b == min(bm, bs) + 1 * 2 + 8 * 2
    bm, bs, b, isz = ix.bytes_model([1], 100)
    assert b == 8 * 3 + 8 * 3 and isz == 3


def test_facets_golden():
    """Facet filters, facet-only queries and AllQuery vs the numpy restatement."""
    fx = load_golden("facets_2k.json")
    n, nt, off, tok, no, ntk, dl = golden_corpus(fx)
    fo, ft, nf = golden_facets(fx)
    ix = orc.OracleIndex(nt, off, tok, no, ntk, dl, threads=4, facet_off=fo, facet_tok=ft, n_fterms=nf)
    assert ix.total_tokens(orc.FACET) == len(ft)
    bad = []
    for q in fx["queries"]:
        s, d = ix.search(q["terms"], q["k"], _mode(q["mode"]), q["fterms"])
        if hits_of(s, d) != q["hits"]:
            bad.append((q["terms"], q["fterms"]))
    assert not bad, bad
    # the batch entry point agrees with single queries
    qs = [q for q in fx["queries"] if q["mode"] == "and" and q["k"] == 10]
    q_off = np.cumsum([0] + [len(q["terms"]) for q in qs]).astype(np.uint32)
    q_terms = np.array([t for q in qs for t in q["terms"]], np.uint32)
    f_off = np.cumsum([0] + [len(q["fterms"]) for q in qs]).astype(np.uint32)
    f_terms = np.array([t for q in qs for t in q["fterms"]], np.uint32)
    sc, dc, cnt, _, _ = ix.search_batch(q_off, q_terms, 10, threads=3, f_off=f_off, f_terms=f_terms)
    for i, q in enumerate(qs):
        assert hits_of(sc[i, :cnt[i]], dc[i, :cnt[i]]) == q["hits"]


OCC = {"must": orc.MUST, "should": orc.SHOULD, "must_not": orc.MUST_NOT}


def test_occur_golden():
    """Must / Should / MustNot mixes (RequiredOptionalScorer, Exclude) vs the numpy
    restatement; the generic path also reproduces the all-Must / all-Should
    fixtures and the segmented search."""
    fx = load_golden("occur_2k.json")
    n, nt, off, tok, no, ntk, dl = golden_corpus(fx)
    ix = orc.OracleIndex(nt, off, tok, no, ntk, dl, threads=4)
    bad = []
    for q in fx["queries"]:
        s, d = ix.search(q["terms"], q["k"], occur=[OCC[o] for o in q["occur"]])
        if hits_of(s, d) != q["hits"]:
            bad.append((q["terms"], q["occur"]))
    assert not bad, bad
    assert sum(len(q["hits"]) for q in fx["queries"]) > 2000
    # batch entry point with per-term occurs
    qs = [q for q in fx["queries"] if q["k"] == 10]
    q_off = np.cumsum([0] + [len(q["terms"]) for q in qs]).astype(np.uint32)
    q_terms = np.array([t for q in qs for t in q["terms"]], np.uint32)
    occ = np.array([OCC[o] for q in qs for o in q["occur"]], np.uint8)
    sc, dc, cnt, _, _ = ix.search_batch(q_off, q_terms, 10, threads=3, occur=occ)
    for i, q in enumerate(qs):
        assert hits_of(sc[i, :cnt[i]], dc[i, :cnt[i]]) == q["hits"], q
    # all-Must / all-Should through the generic path = the mode fixtures
    fx2 = load_golden("synth_names_2k.json")
    n2, nt2, off2, tok2, no2, ntk2, dl2 = golden_corpus(fx2)
    ix2 = orc.OracleIndex(nt2, off2, tok2, no2, ntk2, dl2, threads=4)
    for q in fx2["queries"]:
        o = [orc.MUST if q["mode"] == "and" else orc.SHOULD] * len(q["terms"])
        s, d = ix2.search(q["terms"], q["k"], occur=o)
        assert hits_of(s, d) == q["hits"], q
        # segmented: the same as or_search_seg for AND / OR
        sb = [0, 700, 701, 1500, n2]
        s1, d1 = ix2.search(q["terms"], q["k"], occur=o, seg_bounds=sb)
        s2, d2 = ix2.search_segments(q["terms"], q["k"], sb, mode=_mode(q["mode"]))
        assert hits_of(s1, d1) == hits_of(s2, d2), q
