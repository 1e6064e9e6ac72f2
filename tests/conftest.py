import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def tokens_to_csr(docs):
    off = np.cumsum([0] + [len(t) for t in docs]).astype(np.uint64)
    tok = np.array([x for t in docs for x in t], np.uint32)
    return off, tok


def golden_corpus(fx, use_c_synth=True):
    """(n_docs, n_terms, text_off, text_tok, name_off, name_tok, deleted) of a fixture."""
    c = fx["corpus"]
    if c["kind"] == "tokens":
        off, tok = tokens_to_csr(c["text"])
        return len(c["text"]), c["n_terms"], off, tok, None, None, None
    import synth_ref as sr
    if use_c_synth:
        from fugu_amd import synth
        cp = synth.corpus(c["n_docs"], c["vocab"], c["s"], c["seed_l"], c["seed_t"])
        off, tok = cp.off, cp.tok
    else:
        off, tok = sr.corpus(c["n_docs"], c["vocab"], c["s"], c["seed_l"], c["seed_t"])
    no = nt = dl = None
    if c.get("name"):
        no, nt = sr.names(c["n_docs"], **c["name"])
    if c.get("deleted"):
        dl = sr.deleted_mask(c["n_docs"], **c["deleted"])
    return c["n_docs"], c["vocab"], off, tok, no, nt, dl


def golden_facets(fx):
    """(facet_off, facet_tok, n_fterms) of a fixture with facets, else Nones."""
    if "facet_tokens" not in fx:
        return None, None, 0
    off, tok = tokens_to_csr(fx["facet_tokens"])
    return off, tok, len(fx["facet_vocab"])


def hits_of(scores, docs):
    return [[int(d), int(np.float32(s).view(np.uint32))] for s, d in zip(scores, docs)]


@pytest.fixture(scope="session")
def root():
    return ROOT
