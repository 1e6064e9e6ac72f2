"""Deterministic synthetic Zipf corpora and query streams.

Bench/test input generation (libfugu_synth.so, spec in csrc/synth.cpp and
DESIGN.md §Corpus).  Not part of the search path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libfugu_synth.so")
if not os.path.exists(_LIB_PATH):
    raise ImportError(f"{_LIB_PATH} missing: run __graft_entry__.build()")
_lib = C.CDLL(_LIB_PATH)
_lib.fgs_mix64.restype = C.c_uint64
_lib.fgs_mix64.argtypes = [C.c_uint64]
_lib.fgs_h2.restype = C.c_uint64
_lib.fgs_h2.argtypes = [C.c_uint64, C.c_uint64]
_lib.fgs_h3.restype = C.c_uint64
_lib.fgs_h3.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
_lib.fgs_doc_lengths.restype = C.c_uint64
_lib.fgs_doc_lengths.argtypes = [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_void_p]
_lib.fgs_fill_tokens.restype = C.c_int
_lib.fgs_fill_tokens.argtypes = [C.c_uint64, C.c_uint32, C.c_void_p, C.c_uint32, C.c_double, C.c_uint64,
                                 C.c_void_p, C.c_int]
_lib.fgs_render_text.restype = C.c_uint64
_lib.fgs_render_text.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int]
_lib.fgs_render_ids.restype = C.c_uint64
_lib.fgs_render_ids.argtypes = [C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
_lib.fgs_queries.restype = C.c_int
_lib.fgs_queries.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_double, C.c_uint64, C.c_void_p,
                             C.c_void_p]

SEED_L = 0x5EED1
SEED_T = 20250808
SEED_Q = 7
VOCAB = 1 << 20
LEN_MIN = 8
LEN_SPAN = 113
QUERY_MAX_RANK = 1 << 14


@dataclass
class Corpus:
    n_docs: int
    vocab: int
    off: np.ndarray  # uint64 [n_docs+1]
    tok: np.ndarray  # uint32 term ids


def corpus(n_docs: int, vocab: int = VOCAB, s: float = 1.0, seed_l: int = SEED_L, seed_t: int = SEED_T,
           doc_begin: int = 0, len_min: int = LEN_MIN, len_span: int = LEN_SPAN, threads: int = 0) -> Corpus:
    off = np.zeros(n_docs + 1, np.uint64)
    total = _lib.fgs_doc_lengths(doc_begin, n_docs, seed_l, len_min, len_span, off.ctypes.data)
    tok = np.empty(int(total), np.uint32)
    th = threads if threads > 0 else min(os.cpu_count() or 1, 32)
    rc = _lib.fgs_fill_tokens(doc_begin, n_docs, off.ctypes.data, vocab, s, seed_t, tok.ctypes.data, th)
    assert rc == 0
    return Corpus(n_docs, vocab, off, tok)


def queries(n_queries: int, m_min: int, m_max: int, max_rank: int = QUERY_MAX_RANK, s: float = 1.0,
            seed_q: int = SEED_Q):
    q_off = np.zeros(n_queries + 1, np.uint32)
    q_terms = np.zeros(n_queries * m_max, np.uint32)
    rc = _lib.fgs_queries(n_queries, m_min, m_max, max_rank, s, seed_q, q_off.ctypes.data, q_terms.ctypes.data)
    if rc != 0:
        raise ValueError("bad query parameters")
    return q_off, q_terms[: q_off[-1]].copy()


def render_text(c: "Corpus", threads: int = 0):
    """The docs as text ("t<id>" words): (uint8 buffer, uint64 offsets [n+1]) for the
    host mirror's ingest path (fg_db_upsert_batch)."""
    th = threads if threads > 0 else min(os.cpu_count() or 1, 32)
    off = np.zeros(c.n_docs + 1, np.uint64)
    total = _lib.fgs_render_text(c.off.ctypes.data, c.tok.ctypes.data, c.n_docs, None, off.ctypes.data, th)
    buf = np.empty(max(int(total), 1), np.uint8)
    _lib.fgs_render_text(c.off.ctypes.data, c.tok.ctypes.data, c.n_docs, buf.ctypes.data, off.ctypes.data, th)
    return buf[: int(total)], off


def render_ids(n: int, doc_begin: int = 0):
    """Doc ids "d<i>" for i in [doc_begin, doc_begin + n): (uint8 buffer, uint64 offsets)."""
    total = _lib.fgs_render_ids(doc_begin, n, None, None)
    buf = np.empty(max(int(total), 1), np.uint8)
    off = np.zeros(n + 1, np.uint64)
    _lib.fgs_render_ids(doc_begin, n, buf.ctypes.data, off.ctypes.data)
    return buf[: int(total)], off


def mix64(z: int) -> int:
    return int(_lib.fgs_mix64(z))


def h2(s: int, a: int) -> int:
    return int(_lib.fgs_h2(s, a))


def h3(s: int, a: int, b: int) -> int:
    return int(_lib.fgs_h3(s, a, b))
