"""ctypes binding of the host mirror (include/fugu_host.h, csrc/host.cpp).

Same names and error behaviour as the reference's DatasetManager / Dataset
(src/db/config.rs, src/db/document.rs, src/db/search.rs) for the search path:
namespaces, upsert + commit, paged search, and the perform_search JSON shapes.
Every search runs on the gfx950 device path; queries outside the device subset
raise :class:`native.Unsupported` -- nothing here answers them on the CPU.
"""
from __future__ import annotations

import ctypes as C
import json
from dataclasses import dataclass
from typing import Optional

from . import native

FG_ENOTFOUND = -6
FG_EEXIST = -7
SHAPE_GET_SEARCH = 0
SHAPE_POST_SEARCH = 1
SHAPE_GET_SEARCH_PATH = 2

# every symbol include/fugu_host.h declares (checked by tests/test_abi.py)
HOST_EXPORTS = (
    "fg_db_create", "fg_db_destroy", "fg_db_namespace_create", "fg_db_namespace_delete",
    "fg_db_namespaces_json", "fg_db_upsert", "fg_db_commit", "fg_db_add_file", "fg_db_doc_count",
    "fg_db_search", "fg_db_search_json", "fg_analyze", "fg_parse_query", "fg_parse_query_occur",
    "fg_db_upsert_record", "fg_db_upsert_batch", "fg_db_search_ex", "fg_db_search_json_ex", "fg_db_doc_facets", "fg_facet_tokens",
    "fg_facet_clauses", "fg_db_search_json_post", "fg_db_merge_wait", "fg_db_merge_info_get", "fg_db_segment_docs",
    "fg_search_trace", "fg_merge_policy_pick",
)
SEARCH_PHASES = ("parse_dict", "plan", "launch", "wait_kernels_d2h", "json_fetch", "total")  # FG_SEARCH_PHASES

_lib = native.lib()
_p = C.c_void_p
_s = C.c_char_p
_sz = C.c_size_t


class Hit(C.Structure):
    _fields_ = [("score", C.c_float), ("doc", C.c_uint32)]


class _Record(C.Structure):
    _fields_ = [("id", _s), ("text", _s), ("metadata_json", _s), ("namespace_", _s), ("organization", _s),
                ("conversation_id", _s), ("data_type", _s), ("facets", C.POINTER(_s)), ("n_facets", C.c_uint32),
                ("has_facets", C.c_int)]


class MergeInfo(C.Structure):
    _fields_ = [("merges", C.c_uint64), ("merged_docs", C.c_uint64), ("merge_ms_total", C.c_double),
                ("merge_ms_last", C.c_double), ("merge_ms_max", C.c_double), ("segments", C.c_uint32),
                ("pending", C.c_int), ("n_docs_stats", C.c_uint64), ("tot_tokens", C.c_uint64 * 2),
                ("tot_facet_tokens", C.c_uint64)]


def _sig(name, *args):
    f = getattr(_lib, name)
    f.restype = C.c_int
    f.argtypes = list(args)


_sig("fg_db_create", _p, C.c_int, _s, C.POINTER(_p))
_sig("fg_db_destroy", _p)
_sig("fg_db_namespace_create", _p, _s)
_sig("fg_db_namespace_delete", _p, _s)
_sig("fg_db_namespaces_json", _p, _s, _sz, C.POINTER(_sz))
_sig("fg_db_upsert", _p, _s, _s, _s, _s, _s)
_sig("fg_db_commit", _p, _s)
_sig("fg_db_merge_wait", _p, _s)
_sig("fg_db_merge_info_get", _p, _s, C.POINTER(MergeInfo))
_sig("fg_db_segment_docs", _p, _s, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(C.c_uint32))
_sig("fg_db_add_file", _p, _s, _s, _s)
_sig("fg_db_doc_count", _p, _s, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
_sig("fg_db_search", _p, _s, _s, C.c_uint32, C.c_uint32, C.POINTER(Hit), C.c_uint32, C.POINTER(C.c_uint32))
_sig("fg_db_search_json", _p, _s, _s, C.c_uint32, C.c_uint32, C.c_int, C.c_int, _s, _sz, C.POINTER(_sz))
_sig("fg_db_upsert_record", _p, _s, C.POINTER(_Record))
_sig("fg_db_upsert_batch", _p, _s, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p)
_sig("fg_db_search_ex", _p, _s, _s, C.POINTER(_s), C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(Hit), C.c_uint32,
     C.POINTER(C.c_uint32))
_sig("fg_db_search_json_ex", _p, _s, _s, C.POINTER(_s), C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int, _s,
     _sz, C.POINTER(_sz))
_sig("fg_db_search_json_post", _p, _s, _s, C.POINTER(_s), C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
     C.c_int, C.c_int, C.c_int, _s, _sz, C.POINTER(_sz))
_sig("fg_db_doc_facets", _p, _s, C.c_uint32, _s, _sz, C.POINTER(_sz))
_sig("fg_facet_tokens", _s, _s, _sz, C.POINTER(_sz))
_sig("fg_facet_clauses", C.POINTER(_s), C.c_uint32, C.POINTER(C.c_int), C.POINTER(C.c_int), _s, _sz, C.POINTER(_sz))
_sig("fg_analyze", _s, _s, _sz, C.POINTER(_sz))
_sig("fg_search_trace", C.c_int, C.POINTER(C.c_double), C.c_uint32, C.POINTER(C.c_uint64))
_sig("fg_merge_policy_pick", C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32))
_sig("fg_parse_query", _s, C.POINTER(C.c_int), _s, _sz, C.POINTER(_sz))
_sig("fg_parse_query_occur", _s, _s, _sz, C.POINTER(_sz))


class NotFound(native.FuguError):
    """FG_ENOTFOUND: "Namespace '...' not found"."""


class Exists(native.FuguError):
    """FG_EEXIST: the namespace already exists."""


def _check(rc: int):
    if rc == FG_ENOTFOUND:
        raise NotFound(rc, (_lib.fg_last_error() or b"").decode(errors="replace"))
    if rc == FG_EEXIST:
        raise Exists(rc, (_lib.fg_last_error() or b"").decode(errors="replace"))
    native._check(rc)


def _b(s: Optional[str]):
    return None if s is None else s.encode()


def _string_call(fn, *args, cap: int = 1 << 16) -> str:
    """Fill a buffer; on "too small" (*len >= cap) call again with the reported size."""
    while True:
        buf = C.create_string_buffer(cap)
        n = _sz(0)
        rc = fn(*args, buf, cap, C.byref(n))
        if rc == native.FG_EINVAL and n.value + 1 > cap:
            cap = n.value + 1
            continue
        try:
            _check(rc)
        except native.FuguError as e:
            e.body = buf.raw[:n.value].decode(errors="replace")  # the handler's error JSON, when one was written
            raise
        return buf.raw[:n.value].decode()


def _strs(items):
    """(char** array, keep-alive) for a list of str."""
    items = list(items or [])
    arr = (_s * max(1, len(items)))(*[x.encode() for x in items])
    return arr, len(items)


def facet_tokens(path: str) -> list:
    """FacetTokenizer tokens of Facet::from_text(path) (encoded, U+0000 separators)."""
    out = _string_call(_lib.fg_facet_tokens, path.encode())
    return out.split("\n")


def facet_clauses(filters):
    """(applies, all_query, clauses) of build_facet_query for `filters`."""
    arr, n = _strs(filters)
    a, al = C.c_int(0), C.c_int(0)
    out = _string_call(_lib.fg_facet_clauses, arr, n, C.byref(a), C.byref(al))
    return bool(a.value), bool(al.value), (out.split("\n") if (a.value and not al.value) else [])


def merge_policy_pick(seg_docs):
    """fg_merge_policy_pick: the run [j0, j1) of segments (doc counts, doc order) the
    merger merges next, or None."""
    n = (C.c_uint64 * max(len(seg_docs), 1))(*[int(x) for x in seg_docs])
    j0, j1 = C.c_uint32(0), C.c_uint32(0)
    _check(_lib.fg_merge_policy_pick(n, len(seg_docs), C.byref(j0), C.byref(j1)))
    return (j0.value, j1.value) if j0.value < j1.value else None


def search_trace(enable: int = -1) -> dict:
    """fg_search_trace: the summed phase ms of every search since the last read
    (reset), the number of fg_db_search* calls; enable 1 / 0 switches tracing."""
    ms = (C.c_double * len(SEARCH_PHASES))()
    n = C.c_uint64(0)
    _check(_lib.fg_search_trace(enable, ms, len(SEARCH_PHASES), C.byref(n)))
    return {"calls": n.value, **{k: ms[i] for i, k in enumerate(SEARCH_PHASES)}}


def analyze(text: str) -> list:
    """The "default" analyzer: SimpleTokenizer -> RemoveLongFilter(40) -> LowerCaser."""
    out = _string_call(_lib.fg_analyze, text.encode())
    return out.split("\n") if out else []


MODE_MIXED = 2


def parse_query(query: str):
    """(mode, terms) for the QueryParser subset the device runs; Unsupported otherwise.
    mode: native.MODE_AND / MODE_OR when every clause is Must / Should, else MODE_MIXED."""
    mode = C.c_int(0)
    out = _string_call(_lib.fg_parse_query, query.encode(), C.byref(mode))
    return mode.value, out.split("\n")


def parse_query_occur(query: str):
    """[(occur, term)] with occur native.OCCUR_MUST / OCCUR_SHOULD / OCCUR_MUST_NOT."""
    out = _string_call(_lib.fg_parse_query_occur, query.encode())
    return [(int(x[0]), x[2:]) for x in out.split("\n")]


@dataclass
class ObjectRecord:
    """src/object.rs:8-27: id, text, metadata (JSON object), namespace, explicit
    facets, and the organization / conversation / data-type namespace facets."""
    id: str
    text: str
    namespace: Optional[str] = None
    metadata: Optional[dict] = None
    facets: Optional[list] = None
    organization: Optional[str] = None
    conversation_id: Optional[str] = None
    data_type: Optional[str] = None


class Database:
    """DatasetManager + the docs index of each namespace (host mirror)."""

    def __init__(self, ctx: Optional[native.Context] = None, device: int = 0, default_namespace: str = "fugu_db"):
        h = _p()
        _check(_lib.fg_db_create(ctx.handle if ctx is not None else None, device, _b(default_namespace),
                                 C.byref(h)))
        self._h = h
        self._ctx = ctx  # keep the device context alive as long as the db

    def close(self):
        if self._h:
            _lib.fg_db_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- registry (DatasetManager, src/db/config.rs) --
    def create_namespace(self, name: str):
        _check(_lib.fg_db_namespace_create(self._h, _b(name)))

    def delete_namespace(self, name: str):
        _check(_lib.fg_db_namespace_delete(self._h, _b(name)))

    def namespaces_json(self) -> str:
        return _string_call(_lib.fg_db_namespaces_json, self._h)

    def namespaces(self) -> list:
        return json.loads(self.namespaces_json())["namespaces"]

    # -- ingest (NamedIndex::upsert, src/db/document.rs) --
    def upsert(self, obj: ObjectRecord, namespace: Optional[str] = None):
        """Into `namespace` (default: obj.namespace, else the default namespace).  A record
        without its own namespace carries the target one, as POST /add/{namespace} does
        (ObjectRecord.namespace = namespace, cli.rs:392-397)."""
        ns = namespace if namespace is not None else obj.namespace
        rec_ns = obj.namespace if obj.namespace is not None else namespace
        meta = json.dumps(obj.metadata, separators=(",", ":"), ensure_ascii=False) if obj.metadata is not None \
            else None
        farr, nf = _strs(obj.facets)
        r = _Record(_b(obj.id), _b(obj.text), _b(meta), _b(rec_ns), _b(obj.organization),
                    _b(obj.conversation_id), _b(obj.data_type), farr, nf, 1 if obj.facets is not None else 0)
        _check(_lib.fg_db_upsert_record(self._h, _b(ns), C.byref(r)))

    def upsert_batch(self, namespace: Optional[str], ids=None, texts=None, text_buf=None, text_off=None,
                     id_buf=None, id_off=None):
        """POST /batch/upsert: records {id, text}, validated first, upserted in
        order, one commit.  ids / texts: lists of str, or each as one UTF-8
        buffer (bytes / uint8 array) with offsets [n+1]."""
        import numpy as np
        if ids is not None:
            ib = b"".join(x.encode() for x in ids)
            io = np.cumsum([0] + [len(x.encode()) for x in ids]).astype(np.uint64)
        else:
            ib, io = bytes(np.ascontiguousarray(id_buf, np.uint8)), np.ascontiguousarray(id_off, np.uint64)
        n = len(io) - 1
        if texts is not None:
            enc = [x.encode() for x in texts]
            text_buf = np.frombuffer(b"".join(enc), np.uint8)
            text_off = np.cumsum([0] + [len(x) for x in enc]).astype(np.uint64)
        tb = np.ascontiguousarray(np.frombuffer(text_buf, np.uint8) if isinstance(text_buf, bytes) else text_buf,
                                  np.uint8)
        to = np.ascontiguousarray(text_off, np.uint64)
        ibuf = np.frombuffer(ib, np.uint8) if ib else np.zeros(1, np.uint8)
        _check(_lib.fg_db_upsert_batch(self._h, _b(namespace), n, ibuf.ctypes.data, io.ctypes.data,
                                       tb.ctypes.data if tb.size else np.zeros(1, np.uint8).ctypes.data,
                                       to.ctypes.data))

    def doc_facets(self, namespace: Optional[str], doc: int) -> list:
        out = _string_call(_lib.fg_db_doc_facets, self._h, _b(namespace), doc)
        return out.split("\n") if out else []

    def commit(self, namespace: Optional[str] = None):
        _check(_lib.fg_db_commit(self._h, _b(namespace)))

    def merge_wait(self, namespace: Optional[str] = None):
        """Block until the namespace's background merges are done (fg_db_merge_wait)."""
        _check(_lib.fg_db_merge_wait(self._h, _b(namespace)))

    def merge_info(self, namespace: Optional[str] = None) -> dict:
        m = MergeInfo()
        _check(_lib.fg_db_merge_info_get(self._h, _b(namespace), C.byref(m)))
        d = {n: getattr(m, n) for n, _ in MergeInfo._fields_}
        d["tot_tokens"] = list(m.tot_tokens)
        return d

    def segments(self, namespace: Optional[str] = None) -> list:
        """Global doc ids of every segment of the current snapshot, in order."""
        out, seg = [], 0
        n = C.c_uint32(0)
        for seg in range(self.merge_info(namespace)["segments"]):
            _check(_lib.fg_db_segment_docs(self._h, _b(namespace), seg, None, 0, C.byref(n)))
            buf = (C.c_uint32 * max(n.value, 1))()
            _check(_lib.fg_db_segment_docs(self._h, _b(namespace), seg, buf, n.value, C.byref(n)))
            out.append(list(buf[:n.value]))
        return out

    def add_file(self, namespace: str, name: str, body: str):
        _check(_lib.fg_db_add_file(self._h, _b(namespace), _b(name), _b(body)))

    def doc_count(self, namespace: Optional[str] = None):
        t, a = C.c_uint64(0), C.c_uint64(0)
        _check(_lib.fg_db_doc_count(self._h, _b(namespace), C.byref(t), C.byref(a)))
        return t.value, a.value

    # -- search (Dataset::search / perform_search) --
    def search(self, namespace: Optional[str], query: str, page: int = 0, per_page: int = 20, filters=None):
        """[(score, doc)] of one page; doc = global insertion-order id."""
        out = (Hit * max(1, per_page))()
        n = C.c_uint32(0)
        farr, nf = _strs(filters)
        _check(_lib.fg_db_search_ex(self._h, _b(namespace), query.encode(), farr, nf, page, per_page, out,
                                    max(1, per_page), C.byref(n)))
        return [(out[i].score, out[i].doc) for i in range(n.value)]

    def search_json_post(self, namespace: Optional[str], query: str, filters=None, page: Optional[tuple] = None,
                         url_text: Optional[bool] = None, body_text: Optional[bool] = None,
                         url_include_data: Optional[bool] = None, body_include_data: Optional[bool] = None) -> str:
        """POST /search/json: page = (page, per_page) or None (no `page` object)."""
        tri = lambda b: -1 if b is None else int(bool(b))  # noqa: E731
        farr, nf = _strs(filters)
        pg, pp = page if page is not None else (0, 20)
        return _string_call(_lib.fg_db_search_json_post, self._h, _b(namespace), query.encode(), farr, nf,
                            int(page is not None), pg, pp, tri(url_text), tri(body_text), tri(url_include_data),
                            tri(body_include_data))

    def search_json(self, namespace: Optional[str], query: str, page: int = 0, per_page: int = 20,
                    include_text: bool = False, shape: int = SHAPE_GET_SEARCH, filters=None) -> str:
        farr, nf = _strs(filters)
        return _string_call(_lib.fg_db_search_json_ex, self._h, _b(namespace), query.encode(), farr, nf, page,
                            per_page, int(include_text), shape)
