"""ctypes loader of the CPU oracle (fugu_oracle.c) -- TEST INFRASTRUCTURE.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Parity status: "parity unpinned" (see fugu_oracle.c header
and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# FUGU_ORACLE_LIB: the -march=native build bench.py compiles on the box for the
# CPU baseline (oracle/Makefile `native`); default: the portable test build
LIB_PATH = os.environ.get("FUGU_ORACLE_LIB") or os.path.join(_HERE, "libfugu_oracle.so")
NATIVE_FLAGS = "-O3 -std=c11 -fPIC -ffp-contract=off -D_GNU_SOURCE -march=native"
if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} missing: run `make -C oracle`")
_lib = C.CDLL(LIB_PATH)

_p = C.c_void_p
_lib.or_index_build.restype = _p
_lib.or_index_build.argtypes = [C.c_uint32, C.c_uint32, _p, _p, _p, _p, _p, C.c_int]
_lib.or_index_free.restype = None
_lib.or_index_free.argtypes = [_p]
_lib.or_df.restype = C.c_uint32
_lib.or_df.argtypes = [_p, C.c_int, C.c_uint32]
_lib.or_total_tokens.restype = C.c_uint64
_lib.or_total_tokens.argtypes = [_p, C.c_int]
_lib.or_avgdl.restype = C.c_float
_lib.or_avgdl.argtypes = [_p, C.c_int]
_lib.or_cache.restype = None
_lib.or_cache.argtypes = [_p, C.c_int, _p]
_lib.or_fieldnorm_table.restype = None
_lib.or_fieldnorm_table.argtypes = [_p]
_lib.or_fieldnorm_to_id.restype = C.c_uint8
_lib.or_fieldnorm_to_id.argtypes = [C.c_uint32]
_lib.or_fieldnorm_id_of.restype = C.c_uint8
_lib.or_fieldnorm_id_of.argtypes = [_p, C.c_int, C.c_uint32]
_lib.or_idf.restype = C.c_float
_lib.or_idf.argtypes = [C.c_uint64, C.c_uint64]
_lib.or_term_weight.restype = C.c_float
_lib.or_term_weight.argtypes = [C.c_uint64, C.c_uint64]
_lib.or_bm25_cache.restype = None
_lib.or_bm25_cache.argtypes = [C.c_float, _p]
_lib.or_search.restype = C.c_int
_lib.or_search.argtypes = [_p, _p, C.c_uint32, C.c_int, C.c_uint32, _p, _p]
_lib.or_search_batch.restype = C.c_double
_lib.or_search_batch.argtypes = [_p, _p, _p, C.c_uint32, C.c_int, C.c_uint32, _p, _p, _p, _p, C.c_int]
_lib.or_index_set_facets.restype = C.c_int
_lib.or_index_set_facets.argtypes = [_p, C.c_uint32, _p, _p, C.c_int]
_lib.or_search_ex.restype = C.c_int
_lib.or_search_ex.argtypes = [_p, _p, C.c_uint32, C.c_int, _p, C.c_uint32, C.c_uint32, _p, _p]
_lib.or_search_batch_ex.restype = C.c_double
_lib.or_search_batch_ex.argtypes = [_p, _p, _p, _p, _p, C.c_uint32, C.c_int, C.c_uint32, _p, _p, _p, _p, C.c_int]
_lib.or_search_seg.restype = C.c_int
_lib.or_search_seg.argtypes = [_p, _p, C.c_uint32, C.c_int, C.c_uint32, _p, C.c_uint32, _p, _p]
_lib.or_search_q.restype = C.c_int
_lib.or_search_q.argtypes = [_p, _p, _p, C.c_uint32, _p, C.c_uint32, C.c_int, _p, C.c_uint32, C.c_uint32, _p, _p]
_lib.or_search_batch_q.restype = C.c_double
_lib.or_search_batch_q.argtypes = [_p, _p, _p, _p, _p, _p, C.c_uint32, C.c_int, C.c_uint32, _p, _p, _p, _p, C.c_int]
_lib.or_index_set_total_tokens.restype = C.c_int
_lib.or_index_set_total_tokens.argtypes = [_p, C.c_int, C.c_uint64]
_lib.or_bytes_model.restype = C.c_int
_lib.or_bytes_model.argtypes = [_p, _p, C.c_uint32, C.c_uint32, _p]

AND = 0
OR = 1
FACET = 2
# clause occurs (tantivy Occur; query/boolean_query): per term of a query
MUST = 0
SHOULD = 1
MUST_NOT = 2  # field slot of the facet field (or_df / or_total_tokens / or_avgdl)


def fieldnorm_table():
    t = np.zeros(256, np.uint32)
    _lib.or_fieldnorm_table(t.ctypes.data)
    return t


def fieldnorm_to_id(n: int) -> int:
    return int(_lib.or_fieldnorm_to_id(n))


def idf(df: int, n: int) -> float:
    return float(_lib.or_idf(df, n))


def term_weight(df: int, n: int) -> float:
    return float(_lib.or_term_weight(df, n))


def bm25_cache(avgdl: float):
    out = np.zeros(256, np.float32)
    _lib.or_bm25_cache(C.c_float(avgdl), out.ctypes.data)
    return out


class OracleIndex:
    def __init__(self, n_terms: int, text_off, text_tok, name_off=None, name_tok=None, deleted=None,
                 threads: int = 1, facet_off=None, facet_tok=None, n_fterms: int = 0):
        self._keep = [np.ascontiguousarray(text_off, np.uint64), np.ascontiguousarray(text_tok, np.uint32)]
        n_docs = len(self._keep[0]) - 1
        no = nt = dl = None
        if name_off is not None:
            no = np.ascontiguousarray(name_off, np.uint64)
            nt = np.ascontiguousarray(name_tok, np.uint32)
            self._keep += [no, nt]
        if deleted is not None:
            dl = np.ascontiguousarray(deleted, np.uint8)
            self._keep.append(dl)
        self._h = _lib.or_index_build(n_docs, n_terms, self._keep[0].ctypes.data, self._keep[1].ctypes.data,
                                      None if no is None else no.ctypes.data, None if nt is None else nt.ctypes.data,
                                      None if dl is None else dl.ctypes.data, threads)
        if not self._h:
            raise MemoryError("oracle index build failed")
        if facet_off is not None:
            fo = np.ascontiguousarray(facet_off, np.uint64)
            ft = np.ascontiguousarray(facet_tok, np.uint32)
            self._keep += [fo, ft]
            if _lib.or_index_set_facets(self._h, n_fterms, fo.ctypes.data, ft.ctypes.data, threads) != 0:
                raise ValueError("oracle facet build failed")
        self.n_docs = n_docs
        self.n_terms = n_terms

    def df(self, term: int, field: int = 0) -> int:
        return int(_lib.or_df(self._h, field, term))

    def total_tokens(self, field: int = 0) -> int:
        return int(_lib.or_total_tokens(self._h, field))

    def avgdl(self, field: int = 0) -> float:
        return float(_lib.or_avgdl(self._h, field))

    def cache(self, field: int = 0):
        out = np.zeros(256, np.float32)
        _lib.or_cache(self._h, field, out.ctypes.data)
        return out

    def fieldnorm_id(self, doc: int, field: int = 0) -> int:
        return int(_lib.or_fieldnorm_id_of(self._h, field, doc))

    def search(self, terms, k: int, mode: int = AND, fterms=None, occur=None, seg_bounds=None):
        """fterms: facet clauses (None: no filter); empty `terms` = empty text query.
        occur: per-term MUST / SHOULD / MUST_NOT (None: every term is `mode`'s);
        seg_bounds: segment doc-id bounds (None: one segment)."""
        t = np.ascontiguousarray(terms, np.uint32)
        if occur is not None or seg_bounds is not None:
            oc = np.ascontiguousarray(occur if occur is not None else [MUST if mode == AND else SHOULD] * len(t),
                                      np.uint8)
            f = np.ascontiguousarray(fterms if fterms is not None else [], np.uint32)
            sb = None if seg_bounds is None else np.ascontiguousarray(seg_bounds, np.uint32)
            score = np.zeros(k, np.float32)
            doc = np.zeros(k, np.uint32)
            n = _lib.or_search_q(self._h, t.ctypes.data, oc.ctypes.data, len(t), f.ctypes.data, len(f),
                                 1 if fterms is not None else 0, None if sb is None else sb.ctypes.data,
                                 0 if sb is None else len(sb) - 1, k, score.ctypes.data, doc.ctypes.data)
            if n < 0:
                raise ValueError("oracle rejected the query")
            return score[:n].copy(), doc[:n].copy()
        score = np.zeros(k, np.float32)
        doc = np.zeros(k, np.uint32)
        if fterms is None and len(t) > 0:
            n = _lib.or_search(self._h, t.ctypes.data, len(t), mode, k, score.ctypes.data, doc.ctypes.data)
        else:
            f = np.ascontiguousarray(fterms if fterms is not None else [], np.uint32)
            n = _lib.or_search_ex(self._h, t.ctypes.data, len(t), mode, f.ctypes.data, len(f), k,
                                  score.ctypes.data, doc.ctypes.data)
        if n < 0:
            raise ValueError("oracle rejected the query")
        return score[:n].copy(), doc[:n].copy()

    def search_segments(self, terms, k: int, seg_bounds, mode: int = AND):
        """or_search_seg: the index as segments [seg_bounds[i], seg_bounds[i+1]) (one per commit)."""
        t = np.ascontiguousarray(terms, np.uint32)
        sb = np.ascontiguousarray(seg_bounds, np.uint32)
        score = np.zeros(k, np.float32)
        doc = np.zeros(k, np.uint32)
        n = _lib.or_search_seg(self._h, t.ctypes.data, len(t), mode, k, sb.ctypes.data, len(sb) - 1,
                               score.ctypes.data, doc.ctypes.data)
        if n < 0:
            raise ValueError("oracle rejected the query")
        return score[:n].copy(), doc[:n].copy()

    def search_batch(self, q_off, q_terms, k: int, mode: int = AND, threads: int = 1, latencies: bool = False,
                     f_off=None, f_terms=None, occur=None):
        """occur: per-term MUST / SHOULD / MUST_NOT parallel to q_terms (None: `mode`)."""
        q_off = np.ascontiguousarray(q_off, np.uint32)
        q_terms = np.ascontiguousarray(q_terms, np.uint32)
        oc = None if occur is None else np.ascontiguousarray(occur, np.uint8)
        if f_off is not None:
            f_off = np.ascontiguousarray(f_off, np.uint32)
            f_terms = np.ascontiguousarray(f_terms, np.uint32)
        nq = len(q_off) - 1
        score = np.zeros(nq * k, np.float32)
        doc = np.zeros(nq * k, np.uint32)
        n = np.zeros(nq, np.uint32)
        lat = np.zeros(nq, np.float64) if latencies else None
        wall = _lib.or_search_batch_q(self._h, q_off.ctypes.data, q_terms.ctypes.data,
                                       None if oc is None else oc.ctypes.data,
                                       None if f_off is None else f_off.ctypes.data,
                                       None if f_off is None else f_terms.ctypes.data, nq, mode, k, score.ctypes.data,
                                       doc.ctypes.data, n.ctypes.data, None if lat is None else lat.ctypes.data, threads)
        return score.reshape(nq, k), doc.reshape(nq, k), n, wall, lat

    def set_total_tokens(self, field: int, tot: int):
        """total_num_tokens of a field from outside (a merged segment's, tantivy's rule); avgdl follows."""
        if _lib.or_index_set_total_tokens(self._h, field, tot) != 0:
            raise ValueError("bad field")

    def bytes_model(self, terms, k: int):
        t = np.ascontiguousarray(terms, np.uint32)
        out = np.zeros(4, np.float64)
        rc = _lib.or_bytes_model(self._h, t.ctypes.data, len(t), k, out.ctypes.data)
        if rc != 0:
            raise ValueError("bad query")
        return out

    def close(self):
        if self._h:
            _lib.or_index_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
