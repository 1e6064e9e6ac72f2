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

# every symbol include/fugu_host.h declares (checked by tests/test_abi.py)
HOST_EXPORTS = (
    "fg_db_create", "fg_db_destroy", "fg_db_namespace_create", "fg_db_namespace_delete",
    "fg_db_namespaces_json", "fg_db_upsert", "fg_db_commit", "fg_db_add_file", "fg_db_doc_count",
    "fg_db_search", "fg_db_search_json", "fg_analyze", "fg_parse_query",
)

_lib = native.lib()
_p = C.c_void_p
_s = C.c_char_p
_sz = C.c_size_t


class Hit(C.Structure):
    _fields_ = [("score", C.c_float), ("doc", C.c_uint32)]


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
_sig("fg_db_add_file", _p, _s, _s, _s)
_sig("fg_db_doc_count", _p, _s, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64))
_sig("fg_db_search", _p, _s, _s, C.c_uint32, C.c_uint32, C.POINTER(Hit), C.c_uint32, C.POINTER(C.c_uint32))
_sig("fg_db_search_json", _p, _s, _s, C.c_uint32, C.c_uint32, C.c_int, C.c_int, _s, _sz, C.POINTER(_sz))
_sig("fg_analyze", _s, _s, _sz, C.POINTER(_sz))
_sig("fg_parse_query", _s, C.POINTER(C.c_int), _s, _sz, C.POINTER(_sz))


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
        _check(rc)
        return buf.raw[:n.value].decode()


def analyze(text: str) -> list:
    """The "default" analyzer: SimpleTokenizer -> RemoveLongFilter(40) -> LowerCaser."""
    out = _string_call(_lib.fg_analyze, text.encode())
    return out.split("\n") if out else []


def parse_query(query: str):
    """(mode, terms) for the QueryParser subset the device runs; Unsupported otherwise."""
    mode = C.c_int(0)
    out = _string_call(_lib.fg_parse_query, query.encode(), C.byref(mode))
    return mode.value, out.split("\n")


@dataclass
class ObjectRecord:
    """src/object.rs: id, text, optional namespace, optional metadata (JSON object)."""
    id: str
    text: str
    namespace: Optional[str] = None
    metadata: Optional[dict] = None


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
        ns = namespace if namespace is not None else obj.namespace
        name = None
        if obj.metadata is not None and isinstance(obj.metadata.get("name"), str):
            name = obj.metadata["name"]
        meta = json.dumps(obj.metadata, separators=(",", ":"), ensure_ascii=False) if obj.metadata is not None \
            else None
        _check(_lib.fg_db_upsert(self._h, _b(ns), _b(obj.id), _b(obj.text), _b(name), _b(meta)))

    def commit(self, namespace: Optional[str] = None):
        _check(_lib.fg_db_commit(self._h, _b(namespace)))

    def add_file(self, namespace: str, name: str, body: str):
        _check(_lib.fg_db_add_file(self._h, _b(namespace), _b(name), _b(body)))

    def doc_count(self, namespace: Optional[str] = None):
        t, a = C.c_uint64(0), C.c_uint64(0)
        _check(_lib.fg_db_doc_count(self._h, _b(namespace), C.byref(t), C.byref(a)))
        return t.value, a.value

    # -- search (Dataset::search / perform_search) --
    def search(self, namespace: Optional[str], query: str, page: int = 0, per_page: int = 20):
        """[(score, doc)] of one page; doc = global insertion-order id."""
        out = (Hit * max(1, per_page))()
        n = C.c_uint32(0)
        _check(_lib.fg_db_search(self._h, _b(namespace), query.encode(), page, per_page, out, max(1, per_page),
                                 C.byref(n)))
        return [(out[i].score, out[i].doc) for i in range(n.value)]

    def search_json(self, namespace: Optional[str], query: str, page: int = 0, per_page: int = 20,
                    include_text: bool = False, shape: int = SHAPE_GET_SEARCH) -> str:
        return _string_call(_lib.fg_db_search_json, self._h, _b(namespace), query.encode(), page, per_page,
                            int(include_text), shape)
