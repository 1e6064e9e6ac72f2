"""ctypes binding of libfugu (include/fugu.h).

Plumbing only: every search runs in libfugu.so's gfx950 kernels.  There is no
Python or CPU fallback in this package -- if the library is missing the import
fails, and if no gfx950 device is visible :class:`Context` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

# torch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1.  Only one HIP
# runtime can own the device in a process, and libfugu's NEEDED
# libamdhip64.so.7 binds by soname to whichever is loaded first: load torch's
# first so torch (streams, RCCL) and libfugu share it (tools/diag_runtime.py).
import torch  # noqa: F401,E402

_HERE = os.path.dirname(os.path.abspath(__file__))
# FUGU_LIB selects an alternative build of the same ABI (the -DFG_DIAG
# diagnostic build used by tools/diag_phases.py); default: the product build.
LIB_PATH = os.environ.get("FUGU_LIB") or os.path.join(_HERE, "libfugu.so")

FG_OK = 0
FG_EINVAL = -1
FG_ENODEV = -2
FG_EOOM = -3
FG_EHIP = -4
FG_EUNSUPPORTED = -5
FG_MAX_TERMS = 16
FG_MAX_FACET_CLAUSES = 8
FG_MAX_K = 1024
FG_TERM_MISSING = 0xFFFFFFFF
MODE_AND = 0
MODE_OR = 1
OCCUR_MUST = 0
OCCUR_SHOULD = 1
OCCUR_MUST_NOT = 2
FIELD_TEXT = 0
FIELD_NAME = 1
FIELD_FACET = 2
DIAG_PER_WG = 16  # fg_internal.h kDiagPerWg

# every symbol include/fugu.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "fg_device_count", "fg_ctx_create", "fg_ctx_destroy", "fg_last_error", "fg_version",
    "fg_index_build_from_docs", "fg_index_build", "fg_index_retain", "fg_index_release",
    "fg_thread_background",
    "fg_index_stats_get", "fg_index_df", "fg_index_bm25",
    "fg_plan_create", "fg_plan_execute", "fg_plan_results", "fg_plan_info_get",
    "fg_plan_execute_part", "fg_plan_hist_span", "fg_plan_set_hist_span", "fg_plan_hist_copy",
    "fg_plan_profile", "fg_plan_kernel_ms", "fg_plan_diag", "fg_plan_destroy",
    "fg_search_batch", "fg_search_sharded", "fg_merge_shards", "fg_bytes_model", "fg_bytes_model_gpu",
    "fg_docs_stats", "fg_index_build_from_docs_global", "fg_docs_facet_stats", "fg_index_rescore",
    "fg_index_rescore_many", "fg_index_build_global",
    "fg_ctx_peer_access", "fg_plan_link", "fg_bytes_model_or", "fg_plan_create_multi", "fg_plan_execute_merged", "fg_index_term_kth",
    "fg_model_batch", "fg_abi_version", "fg_index_term_ladder", "fg_kth_floor_combine", "fg_index_set_kth_floor",
    "fg_plan_set_peers", "fg_plan_ipc_export", "fg_plan_set_ipc_peers", "fg_plan_reset",
)
LADDER_KS = (1, 2, 3, 5, 10, 13, 20, 25, 50, 100, 125, 250, 500, 1000)  # FG_LADDER_LEVELS ranks
KTH_KS = (1, 10, 20, 100, 1000)  # fg_index_term_kth / fg_index_set_kth_floor ranks
HIST_BINS = 512  # fugu.h FG_HIST_BINS: score-histogram bins per query
MAX_PEERS = 15  # fugu.h FG_MAX_PEERS
ABI_VERSION = 5  # include/fugu.h FG_ABI_VERSION this binding's structs follow

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libfugu.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "(there is no CPU fallback for the device path)")

_lib = C.CDLL(LIB_PATH)

_p = C.c_void_p
_u32p = C.POINTER(C.c_uint32)
_u64p = C.POINTER(C.c_uint64)
_u16p = C.POINTER(C.c_uint16)
_u8p = C.POINTER(C.c_uint8)
_f32p = C.POINTER(C.c_float)
_f64p = C.POINTER(C.c_double)


class DocsInput(C.Structure):
    _fields_ = [("n_docs", C.c_uint32), ("n_terms", C.c_uint32), ("text_off", _u64p), ("text_tok", _u32p),
                ("name_off", _u64p), ("name_tok", _u32p), ("deleted", _u8p), ("threads", C.c_int),
                ("keep_host_postings", C.c_int), ("n_facet_terms", C.c_uint32), ("facet_off", _u64p),
                ("facet_tok", _u32p)]


class IndexInput(C.Structure):
    _fields_ = [("n_docs", C.c_uint32), ("n_terms", C.c_uint32), ("term_off", _u64p), ("doc", _u32p),
                ("tf_text", _u16p), ("tf_name", _u16p), ("fn_text", _u8p), ("fn_name", _u8p),
                ("tot_tokens", C.c_uint64 * 2), ("deleted", _u8p), ("n_facet_terms", C.c_uint32),
                ("facet_term_off", _u64p), ("facet_doc", _u32p), ("tot_facet_tokens", C.c_uint64)]


class GlobalStats(C.Structure):
    _fields_ = [("n_docs", C.c_uint64), ("tot_tokens", C.c_uint64 * 2), ("df_text", _u32p), ("df_name", _u32p),
                ("df_facet", _u32p), ("tot_facet_tokens", C.c_uint64)]


class QueryBatch(C.Structure):
    _fields_ = [("n_queries", C.c_uint32), ("q_off", _u32p), ("terms", _u32p), ("mode", C.c_int),
                ("f_off", _u32p), ("f_terms", _u32p), ("occur", _u8p)]


class IndexStats(C.Structure):
    _fields_ = [("n_docs", C.c_uint32), ("n_terms", C.c_uint32), ("n_postings", C.c_uint64),
                ("device_bytes", C.c_uint64), ("tot_tokens", C.c_uint64 * 2), ("avgdl", C.c_float * 2),
                ("has_name", C.c_int), ("device", C.c_int), ("n_facet_terms", C.c_uint32),
                ("tot_facet_tokens", C.c_uint64), ("n_dense_f32", C.c_uint32), ("n_rank_terms", C.c_uint32),
                ("n_sparse_rank_terms", C.c_uint32), ("reserved0", C.c_uint32), ("rank_bytes", C.c_uint64)]


class ModelOut(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("stream_bytes", "probe_bytes", "output_bytes", "alg_bytes", "line_bytes",
                                          "query_line_bytes", "loads", "candidates")]


class PlanIpc(C.Structure):
    """fugu.h fg_plan_ipc: a plan's threshold / histogram words as another process maps them."""
    _fields_ = [("handle", C.c_uint8 * 64), ("thresh_off", C.c_uint64), ("hist_off", C.c_uint64),
                ("n_queries", C.c_uint32), ("k", C.c_uint32), ("device", C.c_int), ("reserved", C.c_uint32)]


class PlanInfo(C.Structure):
    _fields_ = [("n_queries", C.c_uint32), ("k", C.c_uint32), ("total_chunks", C.c_uint32),
                ("workspace_bytes", C.c_uint64)]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


_sig("fg_device_count", C.c_int, C.POINTER(C.c_int))
_sig("fg_ctx_create", C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(_p))
_sig("fg_ctx_destroy", C.c_int, _p)
_sig("fg_ctx_peer_access", C.c_int, _p, C.c_int, C.c_int, C.POINTER(C.c_int))
_sig("fg_plan_link", C.c_int, C.POINTER(_p), C.c_uint32)
_sig("fg_bytes_model_or", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, _f32p, _f64p)
_sig("fg_last_error", C.c_char_p)
_sig("fg_version", C.c_char_p)
_sig("fg_index_build_from_docs", C.c_int, _p, C.c_int, C.POINTER(DocsInput), C.POINTER(_p))
_sig("fg_index_build", C.c_int, _p, C.c_int, C.POINTER(IndexInput), C.POINTER(_p))
_sig("fg_index_build_global", C.c_int, _p, C.c_int, C.POINTER(IndexInput), C.POINTER(GlobalStats), C.POINTER(_p))
_sig("fg_docs_stats", C.c_int, C.POINTER(DocsInput), _u32p, _u32p, _u64p)
_sig("fg_docs_facet_stats", C.c_int, C.POINTER(DocsInput), _u32p, _u64p)
_sig("fg_index_build_from_docs_global", C.c_int, _p, C.c_int, C.POINTER(DocsInput), C.POINTER(GlobalStats),
     C.POINTER(_p))
_sig("fg_index_rescore", C.c_int, _p, C.POINTER(GlobalStats), _u8p, C.POINTER(_p))
_sig("fg_index_rescore_many", C.c_int, C.POINTER(_p), C.c_uint32, C.POINTER(GlobalStats), C.POINTER(_u8p),
     C.POINTER(_p))
_sig("fg_index_retain", C.c_int, _p)
_sig("fg_thread_background", C.c_int, C.c_int)
_sig("fg_index_release", C.c_int, _p)
_sig("fg_index_stats_get", C.c_int, _p, C.POINTER(IndexStats))
_sig("fg_index_df", C.c_uint64, _p, C.c_int, C.c_uint32)
_sig("fg_index_bm25", C.c_int, _p, C.c_uint32, _f32p, _f32p, _f32p)
_sig("fg_plan_create", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, C.POINTER(_p))
_sig("fg_plan_create_multi", C.c_int, C.POINTER(_p), C.c_uint32, C.POINTER(QueryBatch), C.c_uint32, C.POINTER(_p))
_sig("fg_plan_execute_merged", C.c_int, _p, _p, _p, _p, _p, _p)
_sig("fg_index_term_kth", C.c_int, _p, C.c_uint32, _f32p)
_sig("fg_index_term_ladder", C.c_int, _p, _f32p)
_sig("fg_kth_floor_combine", C.c_int, C.c_uint32, C.c_uint32, C.POINTER(_f32p), _f32p)
_sig("fg_index_set_kth_floor", C.c_int, _p, _f32p, C.c_uint32)
_sig("fg_plan_execute", C.c_int, _p, _p, _p, _p, _p)
_sig("fg_plan_results", C.c_int, _p, _f32p, _u32p, _u32p)
_sig("fg_plan_hist_span", C.c_int, _p, _u32p, _u32p)
_sig("fg_plan_set_hist_span", C.c_int, _p, _u32p, _u32p)
_sig("fg_plan_execute_part", C.c_int, _p, _p, C.c_double, C.c_double, _p, _p, _p, _p)
_sig("fg_plan_hist_copy", C.c_int, _p, _p, _p, C.c_int)
_sig("fg_plan_set_peers", C.c_int, _p, C.POINTER(_p), C.c_uint32)
_sig("fg_plan_ipc_export", C.c_int, _p, C.POINTER(PlanIpc))
_sig("fg_plan_set_ipc_peers", C.c_int, _p, C.POINTER(PlanIpc), C.c_uint32)
_sig("fg_plan_reset", C.c_int, _p, _p)
_sig("fg_plan_info_get", C.c_int, _p, C.POINTER(PlanInfo))
_sig("fg_plan_profile", C.c_int, _p, C.c_int)
_sig("fg_plan_kernel_ms", C.c_int, _p, _f64p, _u32p)
_sig("fg_plan_diag", C.c_int, _p, _u64p, C.c_size_t, _u32p)
_sig("fg_plan_destroy", C.c_int, _p)
_sig("fg_search_batch", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, _f32p, _u32p, _u32p)
_sig("fg_search_sharded", C.c_int, _p, C.POINTER(_p), C.c_uint32, C.POINTER(QueryBatch), C.c_uint32, _f32p, _u32p,
     _u32p, _u32p)
_sig("fg_merge_shards", C.c_int, C.c_uint32, C.c_uint32, C.c_uint32, _p, _p, _p, _p, _p, _p, _p, _p)
_sig("fg_bytes_model", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, _f64p)
_sig("fg_bytes_model_gpu", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, _f64p)
_sig("fg_model_batch", C.c_int, _p, C.POINTER(QueryBatch), C.c_uint32, _f32p, _f64p, C.POINTER(ModelOut))
_sig("fg_abi_version", C.c_int)
if _lib.fg_abi_version() != ABI_VERSION:
    raise ImportError(f"{LIB_PATH} has ABI {_lib.fg_abi_version()}, this binding follows {ABI_VERSION}: rebuild")


class FuguError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libfugu error {code}: {msg}")
        self.code = code


class Unsupported(FuguError):
    """FG_EUNSUPPORTED: the query is outside the device subset (host CPU path)."""


def _check(rc: int):
    if rc != FG_OK:
        msg = (_lib.fg_last_error() or b"").decode(errors="replace")
        if rc == FG_EUNSUPPORTED:
            raise Unsupported(rc, msg)
        raise FuguError(rc, msg)


def _ptr(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def lib():
    return _lib


def version() -> str:
    return _lib.fg_version().decode()


def device_count() -> int:
    n = C.c_int(0)
    _check(_lib.fg_device_count(C.byref(n)))
    return n.value


class Context:
    def __init__(self, devices=(0,)):
        devs = (C.c_int * len(devices))(*devices)
        h = _p()
        _check(_lib.fg_ctx_create(len(devices), devs, C.byref(h)))
        self._h = h
        self.devices = tuple(devices)

    @property
    def handle(self):
        return self._h

    def peer_access(self, a: int, b: int) -> bool:
        """fg_ctx_peer_access: direct access from device a to device b enabled."""
        e = C.c_int(0)
        _check(_lib.fg_ctx_peer_access(self._h, a, b, C.byref(e)))
        return bool(e.value)

    def close(self):
        if self._h:
            _lib.fg_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Stats:
    n_docs: int
    n_terms: int
    n_postings: int
    device_bytes: int
    tot_tokens: tuple
    avgdl: tuple
    has_name: bool
    device: int
    n_facet_terms: int = 0
    tot_facet_tokens: int = 0
    n_dense_f32: int = 0
    n_rank_terms: int = 0
    n_sparse_rank_terms: int = 0
    rank_bytes: int = 0


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def _batch(q_off, terms, mode, f_off=None, f_terms=None, occur=None):
    """(QueryBatch, arrays it points into); occur: per-term OCCUR_* or None."""
    q_off = _u32(q_off)
    terms = _u32(terms)
    f_off = None if f_off is None else _u32(f_off)
    f_terms = None if f_off is None else _u32(f_terms)
    occur = None if occur is None else np.ascontiguousarray(occur, np.uint8)
    if occur is not None and len(occur) != len(terms):
        raise ValueError("occur must parallel terms")
    qb = QueryBatch(len(q_off) - 1, _ptr(q_off, _u32p), _ptr(terms, _u32p), mode, _ptr(f_off, _u32p),
                    _ptr(f_terms, _u32p), _ptr(occur, _u8p))
    return qb, (q_off, terms, f_off, f_terms, occur)


def _docs_input(text_off, text_tok, n_terms, name_off=None, name_tok=None, deleted=None, threads=0,
                keep_host=True, facets=None):
    """facets: (facet_off, facet_tok, n_facet_terms) or None."""
    text_off = _u64(text_off)
    text_tok = _u32(text_tok)
    name_off = None if name_off is None else _u64(name_off)
    name_tok = None if name_tok is None else _u32(name_tok)
    deleted = None if deleted is None else np.ascontiguousarray(deleted, dtype=np.uint8)
    fo = ft = None
    nft = 0
    if facets is not None:
        fo, ft, nft = _u64(facets[0]), _u32(facets[1]), int(facets[2])
    n_docs = len(text_off) - 1
    inp = DocsInput(n_docs, n_terms, _ptr(text_off, _u64p), _ptr(text_tok, _u32p), _ptr(name_off, _u64p),
                    _ptr(name_tok, _u32p), _ptr(deleted, _u8p), threads, 1 if keep_host else 0, nft,
                    _ptr(fo, _u64p), _ptr(ft, _u32p))
    return (text_off, text_tok, name_off, name_tok, deleted, fo, ft), inp


@dataclass
class ShardStats:
    """BM25 statistics of a (shard of a) namespace: summed across shards by one all-reduce."""
    n_docs: int
    tot_tokens: tuple
    df_text: np.ndarray
    df_name: np.ndarray
    df_facet: "np.ndarray | None" = None
    tot_facet_tokens: int = 0

    def __add__(self, o: "ShardStats") -> "ShardStats":
        dff = None
        if self.df_facet is not None or o.df_facet is not None:
            dff = (self.df_facet if self.df_facet is not None else 0) + (o.df_facet if o.df_facet is not None else 0)
        return ShardStats(self.n_docs + o.n_docs, tuple(a + b for a, b in zip(self.tot_tokens, o.tot_tokens)),
                          self.df_text + o.df_text, self.df_name + o.df_name, dff,
                          self.tot_facet_tokens + o.tot_facet_tokens)


def _global_stats(g: "ShardStats"):
    """(GlobalStats struct, arrays it points into) of summed ShardStats."""
    dft, dfn = _u32(g.df_text), _u32(g.df_name)
    dff = None if g.df_facet is None else _u32(g.df_facet)
    gs = GlobalStats(int(g.n_docs), (C.c_uint64 * 2)(*[int(x) for x in g.tot_tokens]), _ptr(dft, _u32p),
                     _ptr(dfn, _u32p), _ptr(dff, _u32p), int(g.tot_facet_tokens))
    return gs, (dft, dfn, dff)


def docs_stats(text_off, text_tok, n_terms: int, name_off=None, name_tok=None, threads: int = 0,
               facets=None) -> ShardStats:
    """fg_docs_stats (+ fg_docs_facet_stats): a shard's local statistics (host only, no device)."""
    keep, inp = _docs_input(text_off, text_tok, n_terms, name_off, name_tok, None, threads, False, facets)
    dft = np.zeros(n_terms, np.uint32)
    dfn = np.zeros(n_terms, np.uint32)
    tot = np.zeros(2, np.uint64)
    _check(_lib.fg_docs_stats(C.byref(inp), _ptr(dft, _u32p), _ptr(dfn, _u32p), _ptr(tot, _u64p)))
    dff = None
    totf = C.c_uint64(0)
    if facets is not None:
        dff = np.zeros(max(int(facets[2]), 1), np.uint32)[: int(facets[2])]
        _check(_lib.fg_docs_facet_stats(C.byref(inp), _ptr(dff, _u32p), C.byref(totf)))
    del keep
    return ShardStats(int(inp.n_docs), (int(tot[0]), int(tot[1])), dft, dfn, dff, int(totf.value))


class Index:
    """An immutable device snapshot of one namespace's docs index."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def from_docs(cls, ctx: Context, text_off, text_tok, n_terms: int, name_off=None, name_tok=None,
                  deleted=None, device: int | None = None, threads: int = 0, keep_host: bool = True,
                  global_stats: "ShardStats | None" = None, facets=None):
        """Build a snapshot; `global_stats` (a doc-sharded namespace's summed
        ShardStats) makes the BM25 statistics global while the postings stay local.
        `facets` = (facet_off, facet_tok, n_facet_terms): FacetTokenizer tokens per doc."""
        keep, inp = _docs_input(text_off, text_tok, n_terms, name_off, name_tok, deleted, threads, keep_host,
                                facets)
        h = _p()
        dev = ctx.devices[0] if device is None else device
        if global_stats is None:
            _check(_lib.fg_index_build_from_docs(ctx.handle, dev, C.byref(inp), C.byref(h)))
        else:
            g = global_stats
            dft, dfn = _u32(g.df_text), _u32(g.df_name)
            dff = None if g.df_facet is None else _u32(g.df_facet)
            gs = GlobalStats(int(g.n_docs), (C.c_uint64 * 2)(*[int(x) for x in g.tot_tokens]), _ptr(dft, _u32p),
                             _ptr(dfn, _u32p), _ptr(dff, _u32p), int(g.tot_facet_tokens))
            _check(_lib.fg_index_build_from_docs_global(ctx.handle, dev, C.byref(inp), C.byref(gs), C.byref(h)))
        del keep
        return cls(h)

    @classmethod
    def from_postings(cls, ctx: Context, n_docs: int, term_off, doc, tf_text, tf_name, fn_text, fn_name,
                      tot_tokens, deleted=None, facets=None, device: int | None = None,
                      global_stats: "ShardStats | None" = None):
        """fg_index_build: postings already inverted by the host (the entry the Rust
        binding feeds from tantivy's segment readers).  `facets` =
        (facet_term_off, facet_doc, n_facet_terms, tot_facet_tokens) or None."""
        term_off = _u64(term_off)
        doc = _u32(doc)
        tf_text = None if tf_text is None else np.ascontiguousarray(tf_text, np.uint16)
        tf_name = None if tf_name is None else np.ascontiguousarray(tf_name, np.uint16)
        fn_text = np.ascontiguousarray(fn_text, np.uint8)
        fn_name = None if fn_name is None else np.ascontiguousarray(fn_name, np.uint8)
        deleted = None if deleted is None else np.ascontiguousarray(deleted, np.uint8)
        fo = fd = None
        nft, totf = 0, 0
        if facets is not None:
            fo, fd, nft, totf = _u64(facets[0]), _u32(facets[1]), int(facets[2]), int(facets[3])
        inp = IndexInput(n_docs, len(term_off) - 1, _ptr(term_off, _u64p), _ptr(doc, _u32p), _ptr(tf_text, _u16p),
                         _ptr(tf_name, _u16p), _ptr(fn_text, _u8p), _ptr(fn_name, _u8p),
                         (C.c_uint64 * 2)(*[int(x) for x in tot_tokens]), _ptr(deleted, _u8p), nft,
                         _ptr(fo, _u64p), _ptr(fd, _u32p), totf)
        h = _p()
        dev = ctx.devices[0] if device is None else device
        if global_stats is None:
            _check(_lib.fg_index_build(ctx.handle, dev, C.byref(inp), C.byref(h)))
        else:
            gs, keep = _global_stats(global_stats)
            _check(_lib.fg_index_build_global(ctx.handle, dev, C.byref(inp), C.byref(gs), C.byref(h)))
            del keep
        return cls(h)

    @staticmethod
    def rescore_many(indexes, global_stats: "ShardStats", deleted=None) -> list:
        """fg_index_rescore_many: several snapshots scored with one set of
        statistics side by side (the weights once); deleted: None or a list of
        per-snapshot flag arrays (entries may be None)."""
        g = global_stats
        dft, dfn = _u32(g.df_text), _u32(g.df_name)
        dff = None if g.df_facet is None else _u32(g.df_facet)
        gs = GlobalStats(int(g.n_docs), (C.c_uint64 * 2)(*[int(x) for x in g.tot_tokens]), _ptr(dft, _u32p),
                         _ptr(dfn, _u32p), _ptr(dff, _u32p), int(g.tot_facet_tokens))
        n = len(indexes)
        bases = (_p * n)(*[ix._h for ix in indexes])
        dls = [None if deleted is None or deleted[i] is None else np.ascontiguousarray(deleted[i], np.uint8)
               for i in range(n)]
        dp = (_u8p * n)(*[_ptr(d, _u8p) for d in dls])
        outs = (_p * n)()
        _check(_lib.fg_index_rescore_many(bases, n, C.byref(gs), dp, outs))
        return [Index(outs[i]) for i in range(n)]

    def rescore(self, global_stats: "ShardStats", deleted=None) -> "Index":
        """fg_index_rescore: this snapshot's structure scored with other statistics."""
        g = global_stats
        dft, dfn = _u32(g.df_text), _u32(g.df_name)
        dff = None if g.df_facet is None else _u32(g.df_facet)
        gs = GlobalStats(int(g.n_docs), (C.c_uint64 * 2)(*[int(x) for x in g.tot_tokens]), _ptr(dft, _u32p),
                         _ptr(dfn, _u32p), _ptr(dff, _u32p), int(g.tot_facet_tokens))
        dl = None if deleted is None else np.ascontiguousarray(deleted, np.uint8)
        h = _p()
        _check(_lib.fg_index_rescore(self._h, C.byref(gs), _ptr(dl, _u8p), C.byref(h)))
        return Index(h)

    @property
    def handle(self):
        return self._h

    def stats(self) -> Stats:
        s = IndexStats()
        _check(_lib.fg_index_stats_get(self._h, C.byref(s)))
        return Stats(s.n_docs, s.n_terms, s.n_postings, s.device_bytes, tuple(s.tot_tokens), tuple(s.avgdl),
                     bool(s.has_name), s.device, s.n_facet_terms, s.tot_facet_tokens, s.n_dense_f32, s.n_rank_terms,
                     s.n_sparse_rank_terms, s.rank_bytes)

    def df(self, term: int, field: int = -1) -> int:
        return int(_lib.fg_index_df(self._h, field, term))

    def term_kth(self, term: int):
        """The per-term K-th best alive scores for K = 1, 10, 20, 100, 1000 (0: fewer postings)."""
        out = np.zeros(5, np.float32)
        _check(_lib.fg_index_term_kth(self._h, term, _ptr(out, _f32p)))
        return out

    def term_ladder(self) -> np.ndarray:
        """fg_index_term_ladder: [n_terms, len(LADDER_KS)] K-th best alive scores (one k_ktop pass)."""
        V = self.stats().n_terms
        out = np.zeros((V, len(LADDER_KS)), np.float32)
        _check(_lib.fg_index_term_ladder(self._h, _ptr(out, _f32p)))
        return out

    def set_kth_floor(self, floor):
        """fg_index_set_kth_floor: [n_terms, 5] namespace-wide floor of the starting thresholds (None clears)."""
        if floor is None:
            _check(_lib.fg_index_set_kth_floor(self._h, None, 0))
            return
        f = np.ascontiguousarray(floor, np.float32)
        if f.ndim != 2 or f.shape[1] != len(KTH_KS):
            raise ValueError(f"floor must be [n_terms, {len(KTH_KS)}]")
        _check(_lib.fg_index_set_kth_floor(self._h, _ptr(f, _f32p), f.shape[0]))

    def bm25(self, term: int):
        wt, wn = C.c_float(), C.c_float()
        cache = np.zeros(512, np.float32)
        _check(_lib.fg_index_bm25(self._h, term, C.byref(wt), C.byref(wn), _ptr(cache, _f32p)))
        return wt.value, wn.value, cache

    def plan(self, q_off, terms, k: int, mode: int = MODE_AND, f_off=None, f_terms=None, occur=None) -> "Plan":
        return Plan(self, q_off, terms, k, mode, f_off, f_terms, occur)

    def search_batch(self, q_off, terms, k: int, mode: int = MODE_AND, f_off=None, f_terms=None, occur=None):
        """f_off / f_terms: per-query facet clauses (facet term ids), or None;
        occur: per-term OCCUR_MUST / SHOULD / MUST_NOT (None: `mode`)."""
        qb, keep = _batch(q_off, terms, mode, f_off, f_terms, occur)
        nq = qb.n_queries
        score = np.zeros(nq * k, np.float32)
        doc = np.zeros(nq * k, np.uint32)
        n = np.zeros(nq, np.uint32)
        _check(_lib.fg_search_batch(self._h, C.byref(qb), k, _ptr(score, _f32p), _ptr(doc, _u32p), _ptr(n, _u32p)))
        return score.reshape(nq, k), doc.reshape(nq, k), n

    def bytes_model(self, q_off, terms, k: int, mode: int = MODE_AND):
        q_off = _u32(q_off)
        terms = _u32(terms)
        nq = len(q_off) - 1
        qb = QueryBatch(nq, _ptr(q_off, _u32p), _ptr(terms, _u32p), mode)
        out = np.zeros(4 * nq, np.float64)
        _check(_lib.fg_bytes_model(self._h, C.byref(qb), k, _ptr(out, _f64p)))
        return out.reshape(nq, 4)

    def bytes_model_or(self, q_off, terms, k: int, thr, occur=None):
        """fg_bytes_model_or: per query {stream, probe, output, total} bytes of k_disj's
        MaxScore at the device layout with the pruning threshold fixed at `thr` (the
        query's final k-th best score: the least any exact MaxScore reads)."""
        qb, keep = _batch(q_off, terms, MODE_OR, occur=occur)
        t = np.ascontiguousarray(thr, np.float32)
        out = np.zeros(4 * qb.n_queries, np.float64)
        _check(_lib.fg_bytes_model_or(self._h, C.byref(qb), k, _ptr(t, _f32p), _ptr(out, _f64p)))
        return out.reshape(qb.n_queries, 4)

    def model(self, q_off, terms, k: int, thr=None, mode: int = MODE_AND):
        """fg_model_batch: the loads k_conj / k_disj issue for the batch replayed on the
        host (thr: each query's final k-th best score, or None = k_conj's exhaustive
        cascade).  Returns (dict of the launch's bytes: algorithmic, 128-B line floor,
        per-query line sum, ...; per-query {stream, probe, output, total} array)."""
        qb, keep = _batch(q_off, terms, mode)
        t = None if thr is None else np.ascontiguousarray(thr, np.float32)
        per = np.zeros(4 * qb.n_queries, np.float64)
        o = ModelOut()
        _check(_lib.fg_model_batch(self._h, C.byref(qb), k, None if t is None else _ptr(t, _f32p), _ptr(per, _f64p),
                                   C.byref(o)))
        return {n: getattr(o, n) for n, _ in ModelOut._fields_}, per.reshape(qb.n_queries, 4)

    def bytes_model_gpu(self, q_off, terms, k: int, mode: int = MODE_AND):
        """fg_bytes_model_gpu: per query {lead, probe, output, total} bytes at the HBM layout."""
        q_off = _u32(q_off)
        terms = _u32(terms)
        nq = len(q_off) - 1
        qb = QueryBatch(nq, _ptr(q_off, _u32p), _ptr(terms, _u32p), mode)
        out = np.zeros(4 * nq, np.float64)
        _check(_lib.fg_bytes_model_gpu(self._h, C.byref(qb), k, _ptr(out, _f64p)))
        return out.reshape(nq, 4)

    def close(self):
        if self._h:
            _lib.fg_index_release(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    """A batch planned on the host and resident in HBM (fg_plan_create).  Given a
    list of indexes of one device: a multi-snapshot plan (fg_plan_create_multi),
    one launch per kernel over all of them; its results are per query slot
    s * nq + q ([n_segs * nq, k]), the input layout of merge_shards."""

    def __init__(self, index, q_off, terms, k: int, mode: int = MODE_AND, f_off=None, f_terms=None,
                 occur=None):
        qb, self._keep = _batch(q_off, terms, mode, f_off, f_terms, occur)
        self.k = k
        h = _p()
        if isinstance(index, (list, tuple)):
            self.n_segs = len(index)
            hs = (_p * len(index))(*[ix.handle for ix in index])
            _check(_lib.fg_plan_create_multi(hs, len(index), C.byref(qb), k, C.byref(h)))
        else:
            self.n_segs = 1
            _check(_lib.fg_plan_create(index.handle, C.byref(qb), k, C.byref(h)))
        self.n_batch = qb.n_queries
        self.n_queries = qb.n_queries * self.n_segs  # query slots
        self._h = h
        self.index = index

    def info(self) -> PlanInfo:
        i = PlanInfo()
        _check(_lib.fg_plan_info_get(self._h, C.byref(i)))
        return i

    def execute(self, stream: int | None = None, out_score: int | None = None, out_doc: int | None = None,
                out_n: int | None = None):
        """Asynchronous launch; `stream` and outputs are raw device addresses (ints)."""
        _check(_lib.fg_plan_execute(self._h, stream, out_score, out_doc, out_n))

    def execute_merged(self, stream: int | None, out_score: int, out_doc: int, out_shard: int, out_n: int):
        """A multi-snapshot plan straight to the merged top-k per batch query
        (device outputs [n_batch*k] x 3, [n_batch]; raw device addresses)."""
        _check(_lib.fg_plan_execute_merged(self._h, stream, out_score, out_doc, out_shard, out_n))

    def execute_part(self, stream: int | None, frm: float, to: float, out_score: int | None = None,
                     out_doc: int | None = None, out_shard: int | None = None, out_n: int | None = None):
        """fg_plan_execute_part: the k_disj items [frm, to) of the sweep (to = 1:
        the final select too, merged when out_shard is given)."""
        _check(_lib.fg_plan_execute_part(self._h, stream, frm, to, out_score, out_doc, out_shard, out_n))

    def hist_span(self):
        """(lo, hi) u32 [n_batch]: the f32 bits each query's histogram spans (0, 0: no work)."""
        lo = np.zeros(self.n_batch, np.uint32)
        hi = np.zeros(self.n_batch, np.uint32)
        _check(_lib.fg_plan_hist_span(self._h, _ptr(lo, _u32p), _ptr(hi, _u32p)))
        return lo, hi

    def set_hist_span(self, lo, hi):
        lo = np.ascontiguousarray(lo, np.uint32)
        hi = np.ascontiguousarray(hi, np.uint32)
        if lo.shape != (self.n_batch,) or hi.shape != (self.n_batch,):
            raise ValueError(f"spans of {lo.shape} / {hi.shape}, expected ({self.n_batch},)")
        _check(_lib.fg_plan_set_hist_span(self._h, _ptr(lo, _u32p), _ptr(hi, _u32p)))

    def hist_copy(self, stream: int | None, d_buf: int, into_plan: bool):
        """Copy the histograms [n_batch, HIST_BINS] u32 to / from device memory d_buf."""
        _check(_lib.fg_plan_hist_copy(self._h, stream, d_buf, 1 if into_plan else 0))

    def set_peers(self, peers):
        """fg_plan_set_peers: publish thresholds / hit counts into these plans too
        (same process; [] clears).  Executes then need reset() first."""
        hs = (_p * max(len(peers), 1))(*[x._h for x in peers])
        self._peers = list(peers)  # (kept alive while this plan can publish into them)
        _check(_lib.fg_plan_set_peers(self._h, hs, len(peers)))

    def ipc_export(self) -> bytes:
        """fg_plan_ipc_export: the plan's words for another process (set_ipc_peers)."""
        x = PlanIpc()
        _check(_lib.fg_plan_ipc_export(self._h, C.byref(x)))
        return bytes(x)

    def set_ipc_peers(self, blobs):
        """fg_plan_set_ipc_peers: peers in other processes, from their ipc_export() bytes."""
        arr = (PlanIpc * max(len(blobs), 1))()
        for i, b in enumerate(blobs):
            if len(b) != C.sizeof(PlanIpc):
                raise ValueError(f"peer {i}: {len(b)} bytes, expected {C.sizeof(PlanIpc)}")
            C.memmove(C.byref(arr, i * C.sizeof(PlanIpc)), b, len(b))
        _check(_lib.fg_plan_set_ipc_peers(self._h, arr, len(blobs)))

    def reset(self, stream: int | None = None):
        """fg_plan_reset: zero thresholds, histograms and candidate counts (peers: before every round)."""
        _check(_lib.fg_plan_reset(self._h, stream))

    def results(self):
        nq, k = self.n_queries, self.k
        score = np.zeros(nq * k, np.float32)
        doc = np.zeros(nq * k, np.uint32)
        n = np.zeros(nq, np.uint32)
        _check(_lib.fg_plan_results(self._h, _ptr(score, _f32p), _ptr(doc, _u32p), _ptr(n, _u32p)))
        return score.reshape(nq, k), doc.reshape(nq, k), n

    def profile(self, enable: bool = True):
        _check(_lib.fg_plan_profile(self._h, 1 if enable else 0))

    def kernel_ms(self):
        """(summed ms of (k_fmask + k_conj/k_disj + k_scan, k_final) over the profiled executes, executes)."""
        ms = np.zeros(2, np.float64)
        n = C.c_uint32(0)
        _check(_lib.fg_plan_kernel_ms(self._h, _ptr(ms, _f64p), C.byref(n)))
        return ms, n.value

    def candidate_counts(self):
        cnt = np.zeros(self.n_queries, np.uint32)
        _check(_lib.fg_plan_diag(self._h, None, 0, _ptr(cnt, _u32p)))
        return cnt

    def diag(self):
        """Per-workgroup phase stamps of the last execute (FG_DIAG builds only)."""
        info = self.info()
        n = DIAG_PER_WG * (info.total_chunks + self.n_queries)
        out = np.zeros(n, np.uint64)
        _check(_lib.fg_plan_diag(self._h, _ptr(out, _u64p), n, None))
        w = out.reshape(-1, DIAG_PER_WG)
        return w[: info.total_chunks], w[info.total_chunks:]

    def close(self):
        if self._h:
            _lib.fg_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def kth_floor_combine(ladders) -> np.ndarray:
    """fg_kth_floor_combine (host only): shard ladders [n_shards][n_terms, len(LADDER_KS)]
    -> [n_terms, 5] lower bounds of the namespace-wide K-th scores (K = KTH_KS)."""
    ls = [np.ascontiguousarray(x, np.float32) for x in ladders]
    if not ls:
        raise ValueError("no ladders")
    V = ls[0].shape[0]
    for x in ls:
        if x.shape != (V, len(LADDER_KS)):
            raise ValueError(f"ladder shape {x.shape}, expected ({V}, {len(LADDER_KS)})")
    arr = (_f32p * len(ls))(*[_ptr(x, _f32p) for x in ls])
    out = np.zeros((V, len(KTH_KS)), np.float32)
    _check(_lib.fg_kth_floor_combine(len(ls), V, arr, _ptr(out, _f32p)))
    return out


def link_plans(plans):
    """fg_plan_link: plans of one batch on one device share per-query pruning
    thresholds; execute plans[0] first in every round, destroy it last."""
    hs = (_p * len(plans))(*[p._h for p in plans])
    _check(_lib.fg_plan_link(hs, len(plans)))


def search_sharded(indexes, q_off, terms, k: int, mode: int = MODE_AND, f_off=None, f_terms=None, ctx=None,
                   occur=None):
    """fg_search_sharded: one batch over several shard / segment / namespace
    indexes, merged on the first one's device by (score desc, shard asc, doc
    asc).  Returns (score [nq,k], doc [nq,k], shard [nq,k], n [nq])."""
    qb, keep = _batch(q_off, terms, mode, f_off, f_terms, occur)
    nq = qb.n_queries
    hs = (_p * len(indexes))(*[ix._h for ix in indexes])
    score = np.zeros(nq * k, np.float32)
    doc = np.zeros(nq * k, np.uint32)
    shard = np.zeros(nq * k, np.uint32)
    n = np.zeros(nq, np.uint32)
    _check(_lib.fg_search_sharded(ctx._h if ctx is not None else None, hs, len(indexes), C.byref(qb), k,
                                  _ptr(score, _f32p), _ptr(doc, _u32p), _ptr(shard, _u32p), _ptr(n, _u32p)))
    return score.reshape(nq, k), doc.reshape(nq, k), shard.reshape(nq, k), n


def merge_shards(n_shards: int, n_queries: int, k: int, d_score: int, d_doc: int, d_n: int, d_out_score: int,
                 d_out_doc: int, d_out_shard: int | None, d_out_n: int, stream: int | None = None):
    _check(_lib.fg_merge_shards(n_shards, n_queries, k, d_score, d_doc, d_n, d_out_score, d_out_doc, d_out_shard,
                                d_out_n, stream))
