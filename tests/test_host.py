"""Host mirror (include/fugu_host.h): analyzer, query-parser subset, namespace
registry, upsert semantics and response shapes.  CPU tests use a db without a
device context (fg_db_create(ctx=NULL)); the end-to-end tests against the
oracle are marked gpu.

Reference behaviour followed:
  analyzer      src/db/schemas.rs:10,14 (SimpleTokenizer, RemoveLongFilter(40), LowerCaser)
  parser        src/db/search.rs:108-127 (QueryParser over [text, name])
  validation    src/object.rs:31-78, src/db/config.rs:302-315
  upsert        src/db/document.rs:23-67 (delete_term on the RAW id, then add_document)
  responses     src/server/handlers/search.rs:56-65,184-195,350-402
"""
import json
import random
import unicodedata

import numpy as np
import pytest

from conftest import hits_of


@pytest.fixture(scope="module")
def db():
    from fugu_amd import db as fdb
    return fdb


def py_analyze(s):
    """Restatement: runs of alphanumeric chars, drop >= 40 UTF-8 bytes, per-char lowercase."""
    out, cur = [], []
    for ch in s + " ":
        if ch.isalnum():
            cur.append(ch)
            continue
        if cur:
            t = "".join(cur)
            if len(t.encode()) < 40:
                out.append("".join(c.lower() for c in t))
            cur = []
    return out


# ------------------------------------------------------------------ analyzer
def test_analyzer_known_answers(db):
    assert db.analyze("Hello, World!") == ["hello", "world"]
    assert db.analyze("") == []
    assert db.analyze("  ...  ") == []
    assert db.analyze("foo_bar-baz") == ["foo", "bar", "baz"]  # '_' is not alphanumeric
    assert db.analyze("x" * 39 + " " + "y" * 40) == ["x" * 39]  # RemoveLongFilter limit 40
    # the limit is in UTF-8 bytes of the original token: 20 x 'é' = 40 bytes -> dropped
    assert db.analyze("é" * 19 + " " + "é" * 20) == ["é" * 19]
    assert db.analyze("İstanbul ΣΑΣ Straße") == ["i̇stanbul", "σασ", "straße"]  # per char, no final sigma
    assert db.analyze("１２３ⅫⅣ") == ["１２３ⅻⅳ"]  # Nd fullwidth digits, Nl roman numerals
    # Rust char::is_alphabetic includes Other_Alphabetic marks and circled letters
    assert db.analyze("नःि Ⓐb") == ["नःि", "ⓐb"]
    assert db.analyze("àb") == ["a", "b"]  # U+0300 is Mn without Other_Alphabetic
    assert db.analyze("日本語 テキスト") == ["日本語", "テキスト"]
    assert db.analyze("emoji😀split") == ["emoji", "split"]


def test_analyzer_matches_restatement_randomized(db):
    pools = [
        [chr(c) for c in range(0x20, 0x7F)],
        [chr(c) for c in range(0xA0, 0x180)],
        [chr(c) for c in range(0x370, 0x400) if unicodedata.category(chr(c)) != "Cn"],
        [chr(c) for c in range(0x400, 0x460)],
        [chr(c) for c in range(0x4E00, 0x4E40)],
        ["😀", "→", "—", "\t", "\n", "  "],
    ]
    rng = random.Random(1234)
    for _ in range(300):
        n = rng.randint(0, 120)
        s = "".join(rng.choice(rng.choice(pools)) for _ in range(n))
        assert db.analyze(s) == py_analyze(s), repr(s)


def test_alnum_table_extends_python_isalnum_only_with_marks():
    """kAlnumRanges = Python isalnum (L*, N*) + Other_Alphabetic (Mn/Mc/So marks)."""
    import os
    import re
    from conftest import ROOT
    src = open(os.path.join(ROOT, "fugu_amd", "csrc", "unicode_tables.inc")).read()
    body = src[src.index("kAlnumRanges"):src.index("kLower")]
    ranges = [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9A-F]+), 0x([0-9A-F]+)\}", body)]
    table = np.zeros(0x110000, bool)
    for a, b in ranges:
        table[a:b + 1] = True
    py = np.array([chr(c).isalnum() if not 0xD800 <= c <= 0xDFFF else False for c in range(0x110000)])
    py[:0x80] = False  # ASCII handled inline in host.cpp
    assert not (py & ~table).any()
    extra = np.nonzero(table & ~py)[0]
    cats = {unicodedata.category(chr(c)) for c in extra}
    assert cats <= {"Mn", "Mc", "So"}, cats


# ------------------------------------------------------------------ parser
def test_parser_device_subset(db):
    AND, OR = 0, 1
    assert db.parse_query("rust") == (AND, ["rust"])
    assert db.parse_query("Rust") == (AND, ["rust"])
    assert db.parse_query("  rust  ") == (AND, ["rust"])
    assert db.parse_query("foo AND Bar AND baz") == (AND, ["foo", "bar", "baz"])
    assert db.parse_query("+foo +bar") == (AND, ["foo", "bar"])
    assert db.parse_query("foo bar") == (OR, ["foo", "bar"])
    assert db.parse_query("straße ÜBER") == (OR, ["straße", "über"])
    # binary OR = the default Should conjunction; prefixes give per-clause occurs
    assert db.parse_query("foo OR Bar OR baz") == (OR, ["foo", "bar", "baz"])
    M, S, X = 0, 1, 2
    assert db.parse_query("+a b") == (db.MODE_MIXED, ["a", "b"])
    assert db.parse_query_occur("+a b") == [(M, "a"), (S, "b")]
    assert db.parse_query_occur("a -b") == [(S, "a"), (X, "b")]
    assert db.parse_query_occur("+Alpha beta -Gamma +delta") == [(M, "alpha"), (S, "beta"), (X, "gamma"), (M, "delta")]
    assert db.parse_query_occur("a OR b") == [(S, "a"), (S, "b")]
    assert db.parse_query_occur("a AND b") == [(M, "a"), (M, "b")]
    assert db.parse_query_occur("rust") == [(S, "rust")]
    assert db.parse_query("-a b") == (db.MODE_MIXED, ["a", "b"])


@pytest.mark.parametrize("q", ["", "   ", "name:x", '"a b"', "foo-bar", "a AND", "AND a", "a OR", "-a", "-a -b",
                               "a AND b OR c", "(a b)", "a^2", "a~1", "fo*", "a AND AND b", "+a AND b", "a OR -b",
                               "--a b", "..."])
def test_parser_rejects_outside_subset(db, q):
    from fugu_amd import native
    with pytest.raises(native.Unsupported):
        db.parse_query(q)


# ------------------------------------------------------------------ registry / ingest
def test_namespace_registry(db):
    d = db.Database(default_namespace="fugu_db")
    assert d.namespaces() == ["fugu_db"]
    d.create_namespace("docs")
    d.create_namespace("a.b-c_d")
    assert json.loads(d.namespaces_json()) == {"status": "success", "namespaces": ["a.b-c_d", "docs", "fugu_db"]}
    for bad in ["", "a/b", "a\\b", "a:b", "a*b", "a?b", 'a"b', "a<b", "a>b", "a|b"]:
        with pytest.raises(db.native.FuguError) as e:
            d.create_namespace(bad)
        assert e.value.code == db.native.FG_EINVAL
    with pytest.raises(db.Exists):
        d.create_namespace("docs")
    d.delete_namespace("docs")
    with pytest.raises(db.NotFound):
        d.delete_namespace("docs")
    with pytest.raises(db.NotFound):
        d.upsert(db.ObjectRecord("x", "y"), "docs")
    assert d.namespaces() == ["a.b-c_d", "fugu_db"]


def test_object_record_validation(db):
    d = db.Database()
    ok = dict(text="hello")
    cases = [
        (db.ObjectRecord("", "t"), "Object ID cannot be empty"),
        (db.ObjectRecord("x" * 257, "t"), "Object ID too long"),
        (db.ObjectRecord("x", ""), "Object text cannot be empty"),
        (db.ObjectRecord("x", "t" * 10001), "Text too long"),
    ]
    for rec, msg in cases:
        with pytest.raises(db.native.FuguError) as e:
            d.upsert(rec)
        assert msg in str(e.value)
    d.upsert(db.ObjectRecord("x" * 256, "t" * 10000))
    d.create_namespace("has space")
    with pytest.raises(db.native.FuguError) as e:
        d.upsert(db.ObjectRecord("x", **ok), "has space")
    assert "Invalid namespace format" in str(e.value)
    assert d.doc_count() == (1, 1)


def test_upsert_deletes_by_raw_id_term(db):
    """delete_term(id_field, raw id) matches the TOKENIZED id field: lowercase
    single-token ids replace, ids with capitals/punctuation accumulate."""
    d = db.Database()
    d.upsert(db.ObjectRecord("doc1", "a"))
    d.upsert(db.ObjectRecord("doc1", "b"))
    assert d.doc_count() == (2, 1)
    d.upsert(db.ObjectRecord("Doc2", "a"))
    d.upsert(db.ObjectRecord("Doc2", "b"))
    assert d.doc_count() == (4, 3)
    d.upsert(db.ObjectRecord("my-doc", "a"))     # tokens: my, doc
    d.upsert(db.ObjectRecord("my-doc", "b"))     # raw "my-doc" matches no token
    assert d.doc_count() == (6, 5)
    d.upsert(db.ObjectRecord("doc", "c"))        # raw "doc" matches the "doc" token of both my-doc docs
    assert d.doc_count() == (7, 4)


def test_commit_needs_a_device_and_search_before_commit_is_empty(db):
    d = db.Database()
    d.upsert(db.ObjectRecord("a", "hello world"))
    with pytest.raises(db.native.FuguError) as e:
        d.commit()
    assert e.value.code == db.native.FG_ENODEV
    assert d.search(None, "hello") == []
    r = json.loads(d.search_json(None, "hello", page=0, per_page=0))
    assert r == {"results": [], "total": 0, "page": 0, "per_page": 20, "query": "hello"}  # per_page clamp
    r = json.loads(d.search_json(None, "hello", page=2, per_page=5, shape=db.SHAPE_POST_SEARCH))
    assert r == {"status": "success", "query": "hello", "filters": [], "page": 2, "per_page": 5, "total": 0,
                 "results": []}
    with pytest.raises(db.NotFound) as e:
        d.search_json("nope", "hello")
    assert "Namespace 'nope' not found" in str(e.value)
    with pytest.raises(db.native.Unsupported):
        d.search(None, "-a -b")
    with pytest.raises(db.native.Unsupported):
        d.search(None, "hello", page=1000, per_page=100)  # offset + per_page > FG_MAX_K


def test_response_shapes_byte_exact(db):
    """The handlers build serde_json Values (json!, to_value): serde_json without
    preserve_order (reference Cargo.lock:4313-4322) keeps object keys in byte
    order, so the bytes below are what the reference server writes."""
    d = db.Database()
    d.create_namespace("ns1")
    assert d.search_json(None, "hello", 0, 0) == '{"page":0,"per_page":20,"query":"hello","results":[],"total":0}'
    assert d.search_json(None, "hello", 2, 5, shape=db.SHAPE_POST_SEARCH, filters=["/a/b"]) == \
        '{"filters":["/a/b"],"page":2,"per_page":5,"query":"hello","results":[],"status":"success","total":0}'
    assert d.namespaces_json() == '{"namespaces":["fugu_db","ns1"],"status":"success"}'
    # GET /search/{query}: URL-decoded path component, page 0, per_page 20 whatever is passed
    assert d.search_json("ns1", "hello%20w%C3%B6rld", 3, 7, shape=db.SHAPE_GET_SEARCH_PATH) == \
        '{"page":0,"per_page":20,"query":"hello w\u00f6rld","results":[],"total":0}'
    with pytest.raises(db.native.FuguError) as e:
        d.search_json("ns1", "bad%ffutf8", shape=db.SHAPE_GET_SEARCH_PATH)
    assert e.value.code == db.native.FG_EINVAL and e.value.body == '{"error":"Invalid URL encoding in query"}'
    # errors
    with pytest.raises(db.NotFound) as e:
        d.search_json("nope", "x")
    assert e.value.body == '{"error":"Search failed: Namespace \'nope\' not found"}'
    with pytest.raises(db.NotFound) as e:
        d.search_json("nope", "x", shape=db.SHAPE_POST_SEARCH)
    assert e.value.body == '{"error":"Namespace \'nope\' not found","status":"error"}'
    with pytest.raises(db.native.Unsupported) as e:
        d.search_json("ns1", "(a b)")
    assert e.value.body.startswith('{"error":"Search failed: Search failed: query outside the device subset')


def test_post_search_json_flags(db):
    """query_json_post (handlers/search.rs:210-301): text flag resolution,
    developer_message, includes_data_objects, targeting_conversations_or_organizations."""
    d = db.Database()
    r = d.search_json_post(None, "hello")
    assert r == ('{"includes_data_objects":true,"page":0,"per_page":20,"query":"hello","results":[],'
                 '"targeting_conversations_or_organizations":false,"total":0}')
    r = json.loads(d.search_json_post(None, "hello", url_text=True, body_text=False, page=(1, 500)))
    assert r["developer_message"] == "url and request body are set to different values; using url:true/false"
    assert (r["page"], r["per_page"]) == (1, 20)  # perform_search clamp
    assert "developer_message" not in json.loads(d.search_json_post(None, "h", url_text=True, body_text=True))
    assert "developer_message" not in json.loads(d.search_json_post(None, "h", body_text=False))
    r = json.loads(d.search_json_post(None, "h", filters=["organization/acme"]))
    assert r["targeting_conversations_or_organizations"] is True and r["includes_data_objects"] is False
    r = json.loads(d.search_json_post(None, "h", filters=["/x/conversation/1"], url_include_data=True))
    assert r["targeting_conversations_or_organizations"] is True and r["includes_data_objects"] is True
    r = json.loads(d.search_json_post(None, "h", filters=["/x"], url_include_data=True, body_include_data=False))
    assert r["targeting_conversations_or_organizations"] is False and r["includes_data_objects"] is False


# ------------------------------------------------------------------ facets
def string_leaves(v):
    if isinstance(v, dict):
        return sum(string_leaves(x) for x in v.values())
    if isinstance(v, list):
        return sum(string_leaves(x) for x in v)
    return 1 if isinstance(v, str) and v else 0


def py_facet_paths(meta, namespace=None, facets=None, org=None, conv=None, dtype=None):
    """get_all_facet_paths (src/db/document.rs:277-309) restated, as Facet Display strings."""
    import facet_ref as fr
    if facets is not None:
        paths = [fr.normalize(f) for f in facets]
    else:
        paths = []
        if namespace is not None:
            paths.append(f"/namespace/{namespace}")
            if org is not None:
                paths.append(f"/namespace/{namespace}/organization/{org}")
            if conv is not None:
                paths.append(f"/namespace/{namespace}/conversation/{conv}")
            if dtype is not None:
                paths.append(f"/namespace/{namespace}/data/{dtype}")
        for k, v in (meta or {}).items():
            p = k if k.startswith("/") else f"/metadata/{k}"
            paths += [p] * string_leaves(v)
    return [fr.display(fr.from_text(p)) for p in paths]


FACET_PATHS = ["/a/b", "/", "/a//b", "//b", "/a\\/b/c", "/a/", "/namespace/x/data/email", "/x\\\\y", "/é/日本"]


def test_facet_tokenizer_matches_restatement(db):
    import facet_ref as fr
    for p in FACET_PATHS:
        assert db.facet_tokens(p) == fr.tokens(fr.from_text(p)), p
    with pytest.raises(db.native.FuguError):
        db.facet_tokens("a/b")  # Facet::from_text needs a leading '/'
    # the golden facet corpus: every doc's tokens through the C++ tokenizer
    import synth_ref as sr
    from conftest import load_golden
    fx = load_golden("facets_2k.json")
    vocab = fx["facet_vocab"]
    for d, paths in enumerate(sr.facet_paths(200, fx["corpus"]["facet_seed"])):
        toks = [t for p in paths for t in db.facet_tokens(fr.normalize(p))]
        assert toks == [vocab[i] for i in fx["facet_tokens"][d]], d


def test_facet_filter_clauses(db):
    """parse_filters + build_facet_query (src/db/search.rs:221-324) and the
    wildcard split of Dataset::search (:89-103)."""
    fc = db.facet_clauses
    assert fc([]) == (False, False, [])
    assert fc(["a/b"]) == (True, False, ["a\x00b"])
    assert fc(["/a/b/*"]) == (True, False, ["a\x00b"])          # Prefix: the path itself (ancestors are indexed)
    assert fc(["ns=foo"]) == (True, False, ["ns"])               # key=value: Equals on the key, value dropped
    assert fc(["/a/*", "b", "c=d"]) == (True, False, ["b", "c", "a"])  # exact terms first, then prefixes
    assert fc(["*x*"]) == (False, False, [])                      # wildcard: dropped (never post-filtered)
    assert fc(["*", "*a*", "k"]) == (True, False, ["k"])
    assert fc(["/*"]) == (True, True, [])                         # prefix "" fails Facet::from_text -> AllQuery
    assert fc(["=x"]) == (True, False, [""])                      # "/=x" -> key "/" -> the root facet
    assert fc(["a\\/b"]) == (True, False, ["a/b"])


def test_upsert_facets(db):
    d = db.Database()
    d.create_namespace("n1")
    d.upsert(db.ObjectRecord("e1", "x", facets=["a/b", "/c//d", "/e\\/f"]), "n1")
    d.upsert(db.ObjectRecord("e2", "x", facets=[]), "n1")       # Some([]): no fallback facets
    d.upsert(db.ObjectRecord("e3", "x", namespace="n1", organization="acme", conversation_id="c7",
                             data_type="chat", metadata={"name": "N", "tags": ["t1", "", "t2", 5],
                                                         "nested": {"a": {"b": "v"}, "c": 1}, "/raw": "v",
                                                         "empty": "", "flag": True}))
    d.upsert(db.ObjectRecord("e4", "x", metadata={"n": None}))  # into the default namespace: no namespace facet
    assert d.doc_facets("n1", 0) == ["/a/b", "/c//d", "/e\\/f"]
    assert d.doc_facets("n1", 1) == []
    assert d.doc_facets("n1", 2) == ["/namespace/n1", "/namespace/n1/organization/acme",
                                     "/namespace/n1/conversation/c7", "/namespace/n1/data/chat", "/metadata/name",
                                     "/metadata/tags", "/metadata/tags", "/metadata/nested", "/raw"]
    assert d.doc_facets(None, 0) == []
    meta = {"name": "N", "tags": ["t1", "", "t2", 5], "nested": {"a": {"b": "v"}, "c": 1}, "/raw": "v", "empty": "",
            "flag": True}
    assert d.doc_facets("n1", 2) == py_facet_paths(meta, "n1", org="acme", conv="c7", dtype="chat")
    bad = [(db.ObjectRecord("x", "t", facets=["f"] * 101), "Too many facets (max 100 per object)"),
           (db.ObjectRecord("x", "t", facets=["a", ""]), "Facet at index 1 cannot be empty"),
           (db.ObjectRecord("x", "t", facets=["a" * 513]), "Facet at index 0 too long (max 512 characters)"),
           (db.ObjectRecord("x", "t", namespace="a b"), "Invalid namespace format"),
           (db.ObjectRecord("x", "t", namespace="n" * 129), "Namespace too long (max 128 characters)")]
    for rec, msg in bad:
        with pytest.raises(db.native.FuguError) as e:
            d.upsert(rec, "n1")
        assert msg in str(e.value)
    d.upsert(db.ObjectRecord("x", "t", facets=["f"] * 100), "n1")
    d.upsert(db.ObjectRecord("x", "t", facets=["a" * 512]), "n1")


# ------------------------------------------------------------------ end to end on the device
WORDS = ["Alpha", "beta", "Gamma", "delta", "épsilon", "ZETA", "eta", "théta", "iota", "kappa", "lambda", "mu",
         "nu", "xi", "omicron", "pi", "rho", "sigma", "tau", "upsilon", "phi", "chi", "psi", "omega", "日本",
         "straße", "1999", "x86"]


def build_corpus(seed, n):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        words = [rng.choice(WORDS[:rng.randint(3, len(WORDS))]) for _ in range(rng.randint(1, 30))]
        seps = [rng.choice([" ", ", ", ". ", "\n", " - "]) for _ in words]
        text = "".join(w + s for w, s in zip(words, seps))
        rid = rng.choice([f"doc{i}", f"doc{rng.randint(0, max(0, i - 1))}", f"Doc{i}", f"d-{i % 50}"])
        meta = {"name": " ".join(rng.choice(WORDS) for _ in range(rng.randint(1, 3)))} if rng.random() < 0.5 \
            else ({"tag": i} if rng.random() < 0.3 else None)
        recs.append((rid, text, meta))
    return recs


def deleted_of(recs):
    """Upsert semantics (src/db/document.rs:38-42): a record deletes every earlier
    doc whose tokenized id holds the RAW new id as a token."""
    ids, deleted = [], []
    for rid, _, _ in recs:
        for j, toks in enumerate(ids):
            if rid in toks:
                deleted[j] = 1
        ids.append(py_analyze(rid))
        deleted.append(0)
    return deleted


def oracle_of(recs, keep=None):
    """Token-id CSR + deleted mask restated in Python from the reference semantics.
    keep: the global ids of the docs the index holds (a merge dropped the rest),
    in order; None = all of them."""
    from oracle import oracle as orc
    deleted = deleted_of(recs)
    keep = list(range(len(recs))) if keep is None else keep
    dic, text, name = {}, [], []

    def intern(s):
        return [dic.setdefault(t, len(dic)) for t in py_analyze(s)]
    for g in keep:
        _, t, meta = recs[g]
        text.append(intern(t))
        nm = meta.get("name") if meta else None
        name.append(intern(nm) if isinstance(nm, str) else [])
    from conftest import tokens_to_csr
    to, tt = tokens_to_csr(text)
    no, nt = tokens_to_csr(name)
    ix = orc.OracleIndex(max(1, len(dic)), to, tt, no, nt, np.array([deleted[g] for g in keep], np.uint8))
    return ix, dic


@pytest.mark.gpu
def test_db_end_to_end_vs_oracle(db):
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("docs")
    recs = build_corpus(7, 3000)
    for rid, t, meta in recs:
        d.upsert(db.ObjectRecord(rid, t, metadata=meta), "docs")
    d.commit("docs")
    ix, dic = oracle_of(recs)
    assert d.doc_count("docs")[0] == len(recs)
    rng = random.Random(99)
    checked = 0
    for _ in range(60):
        m = rng.randint(1, 4)
        ws = [rng.choice(WORDS) for _ in range(m)]
        q = ws[0] if m == 1 else (" AND ".join(ws) if rng.random() < 0.5 else " ".join("+" + w for w in ws))
        page, per_page = rng.randint(0, 3), rng.choice([1, 5, 10, 20])
        got = d.search("docs", q, page, per_page)
        terms = [dic.get(t, native.FG_TERM_MISSING) for t in (py_analyze(w)[0] for w in ws)]
        s, dd = ix.search(np.array(terms, np.uint32), (page + 1) * per_page)
        want = hits_of(s, dd)[page * per_page:]
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == want, q
        checked += len(want)
        # the JSON shape carries the same hits: ids of the docs, shortest-f32 scores
        r = json.loads(d.search_json("docs", q, page, per_page, include_text=True))
        assert r["total"] == len(want) and r["page"] == page and r["per_page"] == per_page and r["query"] == q
        for h, (doc, bits) in zip(r["results"], want):
            assert h["id"] == recs[doc][0] and h["text"] == recs[doc][1]
            assert np.float32(h["score"]).view(np.uint32) == bits
            assert h["metadata"] == recs[doc][2]
            assert h["facets"] == (py_facet_paths(recs[doc][2], "docs") or None)
    assert checked > 100
    r = json.loads(d.search_json("docs", WORDS[1], 0, 3))
    assert all("text" not in h for h in r["results"])
    # bare terms = Should clauses (k_disj), scored in clause order
    for q in ["alpha beta", "Gamma straße 1999 x86", "omega omega psi"]:
        ws = q.split()
        terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
        s, dd = ix.search(np.array(terms, np.uint32), 40, mode=1)
        got = d.search("docs", q, 1, 20)
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == hits_of(s, dd)[20:], q
    # a second batch of upserts is invisible until commit, then visible
    before = d.search("docs", "brandnewword")
    d.add_file("docs", "notes.txt", "brandnewword appears here")
    assert before == []
    got = d.search("docs", "brandnewword")
    assert len(got) == 1 and got[0][1] == len(recs)
    r = json.loads(d.search_json("docs", "brandnewword", shape=db.SHAPE_POST_SEARCH))
    assert r["results"][0]["id"] == "notes.txt" and r["results"][0]["metadata"] == {"name": "notes.txt"}
    assert r["results"][0]["facets"] == ["/namespace/docs", "/metadata/name"]


@pytest.mark.gpu
def test_db_occur_queries_vs_oracle(db):
    """`+a b`, `a -b`, `a OR b`, `+a +b -c d`: the parser's occurs through
    Dataset::search on the device, against the oracle's BooleanQuery."""
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("oc")
    recs = build_corpus(23, 2500)
    for rid, t, meta in recs:
        d.upsert(db.ObjectRecord(rid, t, metadata=meta), "oc")
    d.commit("oc")
    ix, dic = oracle_of(recs)
    rng = random.Random(31)
    checked = 0
    for _ in range(80):
        m = rng.randint(1, 4)
        ws = [rng.choice(WORDS) for _ in range(m)]
        shape = rng.randint(0, 2)
        if shape == 0 and m > 1:
            q, occ = " OR ".join(ws), [1] * m
        else:
            pre = [rng.choice(["+", "", "-"]) for _ in ws]
            if all(p == "-" for p in pre):
                pre[0] = ""
            q = " ".join(p + w for p, w in zip(pre, ws))
            occ = [0 if p == "+" else 2 if p == "-" else 1 for p in pre]
        assert [o for o, _ in db.parse_query_occur(q)] == occ
        page, per_page = rng.randint(0, 2), rng.choice([5, 10, 20])
        got = d.search("oc", q, page, per_page)
        terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
        s, dd = ix.search(np.array(terms, np.uint32), (page + 1) * per_page, occur=occ)
        want = hits_of(s, dd)[page * per_page:]
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == want, q
        checked += len(want)
    assert checked > 200


def facet_corpus(seed, n):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        words = [rng.choice(WORDS[:rng.randint(3, len(WORDS))]) for _ in range(rng.randint(1, 30))]
        text = " ".join(words)
        kind = rng.random()
        rec = dict(id=f"doc{i}", text=text)
        if kind < 0.3:
            rec["facets"] = [rng.choice(["/lang/en", "/lang/de", "lang/fr", "/topic/a/b", "/topic/a/c", "/x\\/y"])
                             for _ in range(rng.randint(0, 3))]
        elif kind < 0.8:
            rec["organization"] = rng.choice(["acme", "initech", None])
            rec["data_type"] = rng.choice(["email", "chat", None])
            rec["metadata"] = {"tags": [rng.choice(["t1", "t2", ""]) for _ in range(rng.randint(0, 3))]} \
                if rng.random() < 0.5 else None
        recs.append(rec)
    return recs


@pytest.mark.gpu
def test_db_facet_filters_end_to_end_vs_oracle(db):
    """Upserts with explicit / namespace / metadata facets, then filtered,
    facet-only and empty-query searches through Dataset::search on the device,
    against the oracle on facet tokens restated in Python."""
    import facet_ref as fr
    from conftest import tokens_to_csr
    from fugu_amd import native
    from oracle import oracle as orc
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("fx")
    recs = facet_corpus(5, 1500)
    for r in recs:
        d.upsert(db.ObjectRecord(r["id"], r["text"], metadata=r.get("metadata"), facets=r.get("facets"),
                                 organization=r.get("organization"), data_type=r.get("data_type")), "fx")
    d.commit("fx")
    dic, fdic, text, ftoks = {}, {}, [], []
    for r in recs:
        text.append([dic.setdefault(t, len(dic)) for t in py_analyze(r["text"])])
        paths = py_facet_paths(r.get("metadata"), "fx", r.get("facets"), r.get("organization"), None,
                               r.get("data_type"))
        ftoks.append([fdic.setdefault(t, len(fdic)) for p in paths for t in fr.tokens(fr.from_text(p))])
    to, tt = tokens_to_csr(text)
    fo, ft = tokens_to_csr(ftoks)
    ix = orc.OracleIndex(len(dic), to, tt, facet_off=fo, facet_tok=ft, n_fterms=len(fdic))
    filters_pool = [["lang/en"], ["/lang/*"], ["/topic/a/*", "lang/de"], ["namespace/fx/organization/acme"],
                    ["/namespace/fx/data/*", "*chat*"], ["metadata=tags"], ["/nope"], ["/x\\/y", "/lang/fr"],
                    ["/"], ["*w*"]]
    rng = random.Random(3)
    checked = 0
    for qi in range(80):
        filters = rng.choice(filters_pool)
        if qi % 4 == 0:
            q, terms, mode = "", [], 0
        else:
            ws = [rng.choice(WORDS) for _ in range(rng.randint(1, 3))]
            q = " AND ".join(ws) if rng.random() < 0.6 else " ".join(ws)
            mode = 0 if (len(ws) == 1 or " AND " in q) else 1
            terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
        page, per_page = rng.randint(0, 2), rng.choice([5, 10, 20])
        applies, all_q, cl = db.facet_clauses(filters)
        fterms = [fdic.get(c, native.FG_TERM_MISSING) for c in cl] if applies and not all_q else None
        got = d.search("fx", q, page, per_page, filters=filters)
        s, dd = ix.search(np.array(terms, np.uint32), (page + 1) * per_page, mode=mode, fterms=fterms)
        want = hits_of(s, dd)[page * per_page:]
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == want, (q, filters)
        checked += len(want)
        r = json.loads(d.search_json("fx", q, page, per_page, shape=db.SHAPE_POST_SEARCH, filters=filters))
        assert r["filters"] == filters and r["total"] == len(want)
        for h, (doc, bits) in zip(r["results"], want):
            rc = recs[doc]
            assert h["id"] == rc["id"] and np.float32(h["score"]).view(np.uint32) == bits
            assert h["facets"] == (py_facet_paths(rc.get("metadata"), "fx", rc.get("facets"), rc.get("organization"),
                                                  None, rc.get("data_type")) or None)
    assert checked > 300
    with pytest.raises(native.Unsupported):  # text AND an AllQuery facet filter
        d.search("fx", "alpha", filters=["/*"])


@pytest.mark.gpu
def test_json_shapes_with_hits_and_canonical_metadata(db):
    """Hits through every handler shape, byte-exact: serde_json re-serializes the
    stored metadata (from_str -> Value: sorted keys, serde number forms) and
    every response object has its keys in byte order."""
    from fugu_amd import native
    ctx = native.Context((0,))
    d = db.Database(ctx)
    raw = ('{"z": 1, "a": {"y": 2.50, "b": 1e16, "c": -0, "d": 1.0E-5, "g": 1e-6, "e": 18446744073709551616, '
           '"f": [true, null, "s\\u00e9"]}, "m": -12, "name": "N1"}')
    assert db._lib.fg_db_upsert(d._h, None, b"d1", b"alpha beta", None, raw.encode()) == 0
    d.upsert(db.ObjectRecord("d2", "alpha gamma", facets=["/t/x"]))
    d.commit()
    canon = ('{"a":{"b":1e16,"c":-0.0,"d":0.00001,"e":1.8446744073709552e19,"f":[true,null,"sé"],'
             '"g":1e-6,"y":2.5},"m":-12,"name":"N1","z":1}')
    hits = d.search(None, "alpha", 0, 10)
    assert [h[1] for h in hits] == [0, 1] or [h[1] for h in hits] == [1, 0]
    out = d.search_json(None, "alpha", 0, 10, include_text=True)
    r = json.loads(out)
    by = {x["id"]: x for x in r["results"]}
    assert canon in out
    assert list(by["d1"].keys()) == ["facets", "id", "metadata", "score", "text"]
    assert by["d2"]["facets"] == ["/t/x"] and by["d2"]["metadata"] is None
    assert list(r.keys()) == ["page", "per_page", "query", "results", "total"]
    assert "text" not in json.loads(d.search_json(None, "alpha", 0, 10))["results"][0]
    p = json.loads(d.search_json_post(None, "alpha", filters=["/t/x"], url_text=True))
    assert list(p.keys()) == ["includes_data_objects", "page", "per_page", "query", "results",
                              "targeting_conversations_or_organizations", "total"]
    assert [x["id"] for x in p["results"]] == ["d2"] and "text" in p["results"][0]
    s = json.loads(d.search_json(None, "alpha", 0, 10, shape=db.SHAPE_POST_SEARCH))
    assert list(s.keys()) == ["filters", "page", "per_page", "query", "results", "status", "total"]
    assert all("text" in x for x in s["results"])
    g = json.loads(d.search_json(None, "alpha%20gamma", 5, 5, shape=db.SHAPE_GET_SEARCH_PATH))
    assert g["query"] == "alpha gamma" and (g["page"], g["per_page"]) == (0, 20) and g["results"][0]["id"] == "d2"


def pick_merge(n, max_docs=10_000_000):
    """host.cpp pick_merge, restated: tantivy 0.24.1's LogMergePolicy defaults
    (min_num_segments 8, min_layer_size 10000, level_log_size 0.75,
    max_docs_before_merge 10M) with levels merged as contiguous runs of >= 8
    (newest first); past 24 segments the 8 contiguous mergeable ones with the
    fewest docs; from 48 on the two newest.  Returns (j0, j1) or None."""
    import math
    c = len(n)
    by = sorted([i for i in range(c) if n[i] <= max_docs], key=lambda i: -n[i])  # stable
    lev = [-1] * c
    cur, lv = float("inf"), -1
    for i in by:
        ls = math.log2(max(n[i], 10000))
        if ls < cur - 0.75:
            cur, lv = ls, lv + 1
        lev[i] = lv
    j1 = c
    while j1 > 0:
        j0 = j1 - 1
        while j0 > 0 and lev[j0 - 1] == lev[j1 - 1]:
            j0 -= 1
        if lev[j1 - 1] >= 0 and j1 - j0 >= 8:
            return j0, j1
        j1 = j0
    if c > 24:
        wins = [(sum(n[j:j + 8]), j) for j in range(c - 7) if all(lev[i] >= 0 for i in range(j, j + 8))]
        if wins:
            j = min(wins)[1]
            return j, j + 8
    return (c - 2, c) if c >= 48 else None


def test_merge_policy_matches_restatement(db):
    rng = random.Random(3)
    for _ in range(400):
        c = rng.randint(0, 60)
        n = [rng.choice([1, 2, 5, 100, 9999, 10000, 20000, 30000, 1 << 20, 1_250_000, 9_999_999, 10_000_001])
             if rng.random() < 0.5 else rng.randint(1, 3_000_000) for _ in range(c)]
        assert db.merge_policy_pick(n) == pick_merge(n), n


def test_merge_policy_levels(db):
    assert db.merge_policy_pick([1_250_000] * 8) == (0, 8)  # one level: tantivy merges the 8
    assert db.merge_policy_pick([1_250_000] * 7 + [100]) is None  # 100 is the min-layer level, alone
    assert db.merge_policy_pick([10_000_001] * 8) is None  # past max_docs_before_merge
    assert db.merge_policy_pick([500_000] + [7] * 8) == (1, 9)  # the newest run of the small level
    # 2 and 5 docs share the clipped level (the round-4 policy kept them apart: log4 levels)
    assert db.merge_policy_pick([2, 5] * 4) == (0, 8)


def test_merge_policy_bounds_alternating_commits(db):
    """Commits of mixed small sizes keep the segment count bounded (each commit
    adds a segment, the merger then applies the policy until it picks nothing)."""
    for sizes in ([2, 5], [5000, 50000], [3, 40000, 700], [9000, 20000, 45000, 200000]):
        segs, most = [], 0
        for i in range(300):
            segs.append(sizes[i % len(sizes)])
            while (run := db.merge_policy_pick(segs)) is not None:
                j0, j1 = run
                segs[j0:j1] = [sum(segs[j0:j1])]
            most = max(most, len(segs))
        assert most <= 25, (sizes, most)


def test_merge_policy_max_docs_knob(db, monkeypatch):
    monkeypatch.setenv("FUGU_MERGE_MAX_DOCS", str(1 << 20))
    assert db.merge_policy_pick([1_250_000] * 8) is None  # bench.py keeps its 8 segments this way
    assert db.merge_policy_pick([1_000_000] * 8) == (0, 8)


def quantized(n):
    """FIELD_NORMS_TABLE[fieldnorm_id(n)]."""
    from oracle import oracle as orc
    return int(orc.fieldnorm_table()[orc.fieldnorm_to_id(n)])


@pytest.mark.gpu
def test_db_incremental_commits_segments_vs_oracle(db):
    """A commit per 100 upserts: each commit adds a segment and rescores the
    older ones with the new statistics (fg_index_rescore); past 8 segments the
    background merger replaces a run of small segments by one that, like a
    tantivy merge, drops the deleted docs (N and df count the alive docs) and
    takes its total_num_tokens per source segment: the source's own total
    without deletes, else its alive docs' quantized lengths (merger.rs
    compute_total_num_tokens).  The model below restates the policy and the
    statistics; after every commit (and its merges) the host's segments and
    statistics equal it, and the paged AND / OR results equal the oracle run
    over the same segments with those totals, bit for bit."""
    from fugu_amd import native
    from oracle import oracle as orc
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("inc")
    recs = build_corpus(11, 2400)
    length = [len(py_analyze(t)) for _, t, _ in recs]
    nlen = [len(py_analyze(m["name"])) if m and isinstance(m.get("name"), str) else 0 for _, _, m in recs]
    segs = []  # the model: {"ids": global ids (deleted included), "tot": [text, name]}
    rng = random.Random(5)
    checked = merges = dropped = 0
    for c in range(0, len(recs), 100):
        for rid, t, meta in recs[c:c + 100]:
            d.upsert(db.ObjectRecord(rid, t, metadata=meta), "inc")
        d.commit("inc")
        d.merge_wait("inc")
        n = c + 100
        dele = deleted_of(recs[:n])
        segs.append({"ids": list(range(c, n)), "tot": [sum(length[c:n]), sum(nlen[c:n])]})
        while (run := pick_merge([len(sg["ids"]) for sg in segs])) is not None:
            j0, j1 = run
            ids, tot = [], [0, 0]
            for sg in segs[j0:j1]:
                alive = [g for g in sg["ids"] if not dele[g]]
                ids += alive
                if len(alive) == len(sg["ids"]):
                    tot = [tot[0] + sg["tot"][0], tot[1] + sg["tot"][1]]
                else:
                    tot = [tot[0] + sum(quantized(length[g]) for g in alive),
                           tot[1] + sum(quantized(nlen[g]) for g in alive)]
                    dropped += len(sg["ids"]) - len(alive)
            segs[j0:j1] = [{"ids": ids, "tot": tot}]
            merges += 1
        assert d.segments("inc") == [sg["ids"] for sg in segs], n
        info = d.merge_info("inc")
        keep = [g for sg in segs for g in sg["ids"]]
        tot = [sum(sg["tot"][f] for sg in segs) for f in (0, 1)]
        assert info["n_docs_stats"] == len(keep) and info["tot_tokens"] == tot, (n, info, tot)
        assert info["merges"] == merges
        bounds = list(np.cumsum([0] + [len(sg["ids"]) for sg in segs]))
        ix, dic = oracle_of(recs[:n], keep)
        for f in (0, 1):
            ix.set_total_tokens(f, tot[f])
        for _ in range(8):
            m = rng.randint(1, 4)
            ws = [rng.choice(WORDS) for _ in range(m)]
            q = ws[0] if m == 1 else (" AND ".join(ws) if rng.random() < 0.6 else " ".join(ws))
            mode = 1 if (m > 1 and " AND " not in q) else 0
            page, per_page = rng.randint(0, 2), rng.choice([5, 10, 20])
            got = d.search("inc", q, page, per_page)
            terms = [dic.get(t, native.FG_TERM_MISSING) for t in (py_analyze(w)[0] for w in ws)]
            s, dd = ix.search_segments(np.array(terms, np.uint32), (page + 1) * per_page, bounds, mode=mode)
            want = [[keep[doc], bits] for doc, bits in hits_of(s, dd)[page * per_page:]]
            assert hits_of([g[0] for g in got], [g[1] for g in got]) == want, (n, q, bounds)
            checked += len(want)
        assert d.doc_count("inc")[0] == n
    assert checked > 300 and merges >= 3 and dropped > 0
    assert orc.fieldnorm_to_id(41) == 40


@pytest.mark.gpu
def test_db_alternating_small_commits_stay_bounded(db):
    """Commits of 2 and 5 docs in turn (under log4 levels they never
    formed a run, so the namespace grew to 48 segments and merged on the commit
    path): every small segment shares tantivy's min-layer level, so each run of
    8 merges in the background and the namespace stays at <= 8 segments, the
    segments' docs always those of the restated policy."""
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("alt")
    recs = build_corpus(31, 350)
    segs, i, c, most, merges = [], 0, 0, 0, 0
    while i < len(recs):
        b = i
        i = min(len(recs), b + (2, 5)[c % 2])
        for rid, t, meta in recs[b:i]:
            d.upsert(db.ObjectRecord(rid, t, metadata=meta), "alt")
        d.commit("alt")
        d.merge_wait("alt")
        c += 1
        dele = deleted_of(recs[:i])
        segs.append(list(range(b, i)))
        while (run := pick_merge([len(sg) for sg in segs])) is not None:
            j0, j1 = run
            segs[j0:j1] = [[g for sg in segs[j0:j1] for g in sg if not dele[g]]]
            merges += 1
        got = d.segments("alt")
        assert got == segs, c
        most = max(most, len(got))
    assert most <= 8 and merges >= 10 and d.merge_info("alt")["merges"] == merges
    assert d.search("alt", "alpha beta", 0, 10)


@pytest.mark.gpu
def test_db_search_during_background_merge(db, monkeypatch):
    """Searches while a merge is in flight (FUGU_MERGE_DELAY_MS holds the merge
    between its build and its swap) see the snapshot before the merge, bit-exact
    vs the oracle over those segments; after fg_db_merge_wait, the merged one."""
    import threading
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    monkeypatch.setenv("FUGU_MERGE_DELAY_MS", "1500")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("bg")
    recs = build_corpus(23, 800)
    for c in range(0, 800, 100):
        for rid, t, meta in recs[c:c + 100]:
            d.upsert(db.ObjectRecord(rid, t, metadata=meta), "bg")
        d.commit("bg")  # the eighth commit queues a merge of the eight segments (one size level)
    assert d.merge_info("bg")["pending"] == 1
    before = d.segments("bg")
    assert len(before) == 8
    rng = random.Random(3)
    qs = []
    for _ in range(24):
        ws = [rng.choice(WORDS) for _ in range(rng.randint(1, 3))]
        qs.append((ws, " AND ".join(ws) if rng.random() < 0.5 else " ".join(ws)))

    def check(segments):
        keep = [g for sg in segments for g in sg]
        bounds = list(np.cumsum([0] + [len(sg) for sg in segments]))
        ix, dic = oracle_of(recs, keep)
        if len(segments) == 1:  # merged: per source segment its own total, or its alive docs' quantized lengths
            dele = deleted_of(recs)
            length = [len(py_analyze(t)) for _, t, _ in recs]
            nlen = [len(py_analyze(m["name"])) if m and isinstance(m.get("name"), str) else 0 for _, _, m in recs]
            for f, ln in ((0, length), (1, nlen)):
                tot = 0
                for sg in before:
                    alive = [g for g in sg if not dele[g]]
                    tot += sum(ln[g] for g in sg) if len(alive) == len(sg) else sum(quantized(ln[g]) for g in alive)
                ix.set_total_tokens(f, tot)
        n = 0
        for ws, q in qs:
            mode = 1 if (len(ws) > 1 and " AND " not in q) else 0
            got = d.search("bg", q, 0, 20)
            terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
            s, dd = ix.search_segments(np.array(terms, np.uint32), 20, bounds, mode=mode)
            assert hits_of([g[0] for g in got], [g[1] for g in got]) == [[keep[x], b] for x, b in hits_of(s, dd)], q
            n += 1
        return n
    assert d.merge_info("bg")["pending"] == 1  # still in flight: the old segments answer
    assert check(before) == len(qs)
    t = threading.Thread(target=d.merge_wait, args=("bg",))
    t.start()
    t.join(60)
    after = d.segments("bg")
    assert len(after) == 1 and d.merge_info("bg")["merges"] == 1
    assert check(after) == len(qs)


@pytest.mark.gpu
def test_db_commits_during_background_merge(db, monkeypatch):
    """Commits that land while a merge is in flight (FUGU_MERGE_DELAY_MS holds it
    between its build and its swap) change the statistics and delete docs of the
    merge's sources: the merger rescores the merged segment with them outside the
    committer lock (again if another commit slips in) and swaps it in.  The
    namespace then answers like the oracle over [merged, the new segments], the
    merged segment keeping the docs alive at its gather (later deletions are
    flags, as in a tantivy segment)."""
    import threading
    import time
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    monkeypatch.setenv("FUGU_MERGE_DELAY_MS", "1500")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("bgc")
    recs = build_corpus(29, 1000)
    for c in range(0, 1000, 100):
        for rid, t, meta in recs[c:c + 100]:
            d.upsert(db.ObjectRecord(rid, t, metadata=meta), "bgc")
        d.commit("bgc")  # commits 9 and 10 land while the merge of the first eight sleeps
        if c == 700:
            assert d.merge_info("bgc")["pending"] == 1
            time.sleep(0.3)  # the merger has gathered its run (its build then sleeps 1.5 s)
    assert d.merge_info("bgc")["merges"] == 0  # commits 9 and 10 came before the swap
    t = threading.Thread(target=d.merge_wait, args=("bgc",))
    t.start()
    t.join(60)
    length = [len(py_analyze(x)) for _, x, _ in recs]
    nlen = [len(py_analyze(m["name"])) if m and isinstance(m.get("name"), str) else 0 for _, _, m in recs]
    dele0 = deleted_of(recs[:800])  # the deletions the merge's gather saw
    merged, tot = [], [0, 0]
    for c in range(0, 800, 100):
        alive = [g for g in range(c, c + 100) if not dele0[g]]
        merged += alive
        for f, ln in ((0, length), (1, nlen)):
            tot[f] += sum(ln[c:c + 100]) if len(alive) == 100 else sum(quantized(ln[g]) for g in alive)
    for f, ln in ((0, length), (1, nlen)):
        tot[f] += sum(ln[800:1000])
    assert len(merged) < 800 and any(deleted_of(recs)[g] for g in merged)  # later commits deleted merged docs
    assert d.segments("bgc") == [merged, list(range(800, 900)), list(range(900, 1000))]
    info = d.merge_info("bgc")
    assert info["merges"] == 1 and info["n_docs_stats"] == len(merged) + 200 and info["tot_tokens"] == tot, info
    keep = merged + list(range(800, 1000))
    bounds = [0, len(merged), len(merged) + 100, len(merged) + 200]
    ix, dic = oracle_of(recs, keep)
    for f in (0, 1):
        ix.set_total_tokens(f, tot[f])
    rng = random.Random(8)
    for _ in range(32):
        ws = [rng.choice(WORDS) for _ in range(rng.randint(1, 3))]
        q = " AND ".join(ws) if rng.random() < 0.5 else " ".join(ws)
        mode = 1 if (len(ws) > 1 and " AND " not in q) else 0
        got = d.search("bgc", q, 0, 20)
        terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
        s, dd = ix.search_segments(np.array(terms, np.uint32), 20, bounds, mode=mode)
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == [[keep[x], b] for x, b in hits_of(s, dd)], q


@pytest.mark.gpu
def test_db_uncommitted_delete_survives_a_merge(db, monkeypatch):
    """An upsert's delete takes effect at the next commit (IndexWriter::delete_term
    + commit, src/db/document.rs:38-65): a merge that swaps in between neither
    drops nor flags the doc, so searches keep finding it until the commit."""
    import threading
    import time
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    monkeypatch.setenv("FUGU_MERGE_DELAY_MS", "800")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("ud")
    recs = build_corpus(41, 800)
    for c in range(0, 800, 100):
        for rid, t, meta in recs[c:c + 100]:
            d.upsert(db.ObjectRecord(rid, t, metadata=meta), "ud")
        d.commit("ud")
    assert d.merge_info("ud")["pending"] == 1
    time.sleep(0.3)  # the merger has gathered its run
    dele = deleted_of(recs)
    # an alive doc whose id is its own token (lowercase alphanumeric): re-upserting that id deletes it
    x = next(g for g in range(100, 800) if not dele[g] and recs[g][0].isalnum() and recs[g][0].islower()
             and py_analyze(recs[g][0]) == [recs[g][0]])
    word = py_analyze(recs[x][1])[0]
    d.upsert(db.ObjectRecord(recs[x][0], "qqqzz"), "ud")  # deletes doc x -- not committed
    t = threading.Thread(target=d.merge_wait, args=("ud",))
    t.start()
    t.join(60)
    assert d.merge_info("ud")["merges"] == 1 and len(d.segments("ud")) == 1
    assert x in d.segments("ud")[0]

    def found(q):
        hits = []
        for page in range(0, 400):
            got = d.search("ud", q, page, 20)
            if not got:
                return hits
            hits += [int(g[1]) for g in got]
        return hits
    # the merged snapshot still holds doc x alive; the oracle over the committed docs agrees
    keep = d.segments("ud")[0]
    ix, dic = oracle_of(recs, keep)
    length = [len(py_analyze(r[1])) for r in recs]
    nlen = [len(py_analyze(m["name"])) if m and isinstance(m.get("name"), str) else 0 for _, _, m in recs]
    for f, ln in ((0, length), (1, nlen)):
        tot = 0
        for c in range(0, 800, 100):
            alive = [g for g in range(c, c + 100) if not dele[g]]
            tot += sum(ln[c:c + 100]) if len(alive) == 100 else sum(quantized(ln[g]) for g in alive)
        ix.set_total_tokens(f, tot)
    got = d.search("ud", word, 0, 20)
    s, dd = ix.search_segments(np.array([dic[word]], np.uint32), 20, [0, len(keep)], mode=0)
    assert hits_of([g[0] for g in got], [g[1] for g in got]) == [[keep[i], b] for i, b in hits_of(s, dd)]
    assert x in found(word)
    d.commit("ud")  # now the delete takes effect
    assert x not in found(word)


@pytest.mark.gpu
def test_db_failed_commit_leaves_statistics_unchanged(db, monkeypatch):
    """A commit whose device build fails (injected) changes nothing: the next
    commit counts the same docs once, so scores equal the oracle's."""
    from fugu_amd import native
    if native.device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    ctx = native.Context((0,))
    d = db.Database(ctx)
    d.create_namespace("ft")
    recs = build_corpus(17, 900)
    for rid, t, meta in recs[:300]:
        d.upsert(db.ObjectRecord(rid, t, metadata=meta), "ft")
    d.commit("ft")
    for rid, t, meta in recs[300:600]:
        d.upsert(db.ObjectRecord(rid, t, metadata=meta), "ft")
    monkeypatch.setenv("FUGU_FAULT_INJECT", "commit_build")
    with pytest.raises(native.FuguError):
        d.commit("ft")
    with pytest.raises(native.FuguError):
        d.commit("ft")
    monkeypatch.delenv("FUGU_FAULT_INJECT")
    d.commit("ft")
    ix, dic = oracle_of(recs[:600])
    rng = random.Random(8)
    checked = 0
    for _ in range(30):
        ws = [rng.choice(WORDS) for _ in range(rng.randint(1, 3))]
        q = " AND ".join(ws) if rng.random() < 0.5 else " ".join(ws)
        mode = 1 if (len(ws) > 1 and " AND " not in q) else 0
        got = d.search("ft", q, 0, 20)
        terms = [dic.get(py_analyze(w)[0], native.FG_TERM_MISSING) for w in ws]
        s, dd = ix.search_segments(np.array(terms, np.uint32), 20, [0, 300, 600], mode=mode)
        assert hits_of([g[0] for g in got], [g[1] for g in got]) == hits_of(s, dd), q
        checked += len(got)
    assert checked > 50


def test_upsert_batch_validates_first_and_upserts_in_order(db):
    """POST /batch/upsert: a bad record rejects the whole batch with its index;
    otherwise every record is upserted in order (raw-id deletes included) and
    one commit runs (no device here: FG_ENODEV after the upserts)."""
    from fugu_amd import synth
    d = db.Database()
    with pytest.raises(db.native.FuguError) as e:
        d.upsert_batch(None, ["a", "", "c"], ["x", "y", "z"])
    assert "Validation failed for object at index 1: Object ID cannot be empty" in str(e.value)
    assert d.doc_count() == (0, 0)
    with pytest.raises(db.native.FuguError) as e:
        d.upsert_batch(None, ["a", "b", "a"], ["x y", "z", "w"])
    assert e.value.code == db.native.FG_ENODEV
    assert d.doc_count() == (3, 2)  # the second "a" deleted the first
    c = synth.corpus(50)
    buf, off = synth.render_text(c)
    first = bytes(buf[int(off[0]):int(off[1])]).decode()
    assert first.split() == [f"t{t}" for t in c.tok[c.off[0]:c.off[1]]]
    with pytest.raises(db.native.FuguError):
        d.upsert_batch(None, [f"d{i}" for i in range(50)], text_buf=buf, text_off=off)
    assert d.doc_count() == (53, 52)
