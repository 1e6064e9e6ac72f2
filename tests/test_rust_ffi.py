"""rust/ffi.rs (the Rust binding fugu would add) against the
C headers: every function the headers declare is bound with the same name,
arity, argument types in order and return type, and every struct of the
headers is a #[repr(C)] struct with the same fields in the same order.  No
Rust toolchain exists here, so this parse is what keeps the binding honest:
it fails on any header drift."""
import os
import re

import pytest

from conftest import ROOT

HEADERS = ("fugu.h", "fugu_host.h")
SCALARS = {"int": "c_int", "uint32_t": "u32", "uint64_t": "u64", "uint16_t": "u16", "uint8_t": "u8",
           "float": "f32", "double": "f64", "size_t": "usize", "char": "c_char", "void": "c_void"}


def c_source(name):
    return re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", name)).read(), flags=re.S)


def c_type_to_rust(t):
    """`const uint32_t*` -> `*const u32`, `fg_index* const*` -> `*const *mut fg_index`, ..."""
    t = " ".join(t.replace("*", " * ").split())
    toks = t.split()
    # base: [const] NAME, then a sequence of '*' each optionally followed by 'const'
    i, const_base = 0, False
    if toks[i] == "const":
        const_base, i = True, i + 1
    base = SCALARS.get(toks[i], toks[i])
    i += 1
    levels = []  # constness of the pointee at each pointer level, innermost first
    pointee_const = const_base
    while i < len(toks):
        assert toks[i] == "*", t
        i += 1
        levels.append(pointee_const)
        pointee_const = False
        if i < len(toks) and toks[i] == "const":
            pointee_const = True  # `T* const*`: the next level points to a const pointer
            i += 1
    r = base
    for c in levels:
        r = ("*const " if c else "*mut ") + r
    return r


def c_functions():
    out = {}
    for h in HEADERS:
        for m in re.finditer(r"\n([a-z][\w\s\*]*?)\b(fg_\w+)\s*\(([^;{]*?)\)\s*;", c_source(h)):
            ret, name, params = " ".join(m.group(1).split()), m.group(2), " ".join(m.group(3).split())
            args = []
            if params != "void":
                for p in params.split(","):
                    p = p.strip()
                    mm = re.match(r"(.*?)(\w+)$", p)
                    args.append(c_type_to_rust(mm.group(1).strip()))
            out[name] = (c_type_to_rust(ret), args)
    return out


def c_structs():
    out = {}
    for h in HEADERS:
        for m in re.finditer(r"(?:typedef )?struct (fg_\w+) \{(.*?)\}(?: \1)?;", c_source(h), flags=re.S):
            fields = []
            for decl in m.group(2).split(";"):
                decl = " ".join(decl.split())
                if not decl:
                    continue
                mm = re.match(r"(const )?([\w]+)((?:\s*\*\s*(?:const)?)*)\s*(.*)$", decl)
                base = (mm.group(1) or "") + mm.group(2) + mm.group(3)
                for name in mm.group(4).split(","):
                    name = name.strip()
                    ptr = ""
                    while name.startswith("*"):
                        ptr += "*"
                        name = name[1:].strip()
                    arr = re.match(r"(\w+)\[(\d+)\]$", name)
                    ty = c_type_to_rust(base + ptr)
                    if arr:
                        fields.append((arr.group(1), f"[{ty}; {arr.group(2)}]"))
                    else:
                        fields.append((name, ty))
            out[m.group(1)] = fields
    return out


def rust_source():
    src = open(os.path.join(ROOT, "rust", "ffi.rs")).read()
    return re.sub(r"//[^\n]*", "", src)


def norm(t):
    return " ".join(t.replace("*", " *").split()).replace("* ", "*")


def rust_functions():
    src = rust_source()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (fg_\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, flags=re.S):
        args = [a.split(":", 1)[1].strip() for a in m.group(2).replace("\n", " ").split(",") if a.strip()]
        out[m.group(1)] = (norm(m.group(3) or "()"), [norm(a) for a in args])
    return out


def rust_structs():
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*pub struct (fg_\w+)\s*\{([^{}]*)\}", rust_source()):
        fields = []
        for line in m.group(2).split(","):
            line = line.strip()
            if line.startswith("pub "):
                name, ty = line[4:].split(":", 1)
                fields.append((name.strip(), norm(ty.strip())))
        out[m.group(1)] = fields
    return out


def test_every_header_function_is_bound_in_order():
    cf, rf = c_functions(), rust_functions()
    assert len(cf) >= 60
    missing = sorted(set(cf) - set(rf))
    extra = sorted(set(rf) - set(cf))
    assert not missing and not extra, (missing, extra)
    for name, (ret, args) in cf.items():
        rret, rargs = rf[name]
        assert len(rargs) == len(args), (name, args, rargs)
        assert [norm(a) for a in args] == rargs, (name, args, rargs)
        assert norm(ret) == rret, (name, ret, rret)


def test_every_header_struct_is_repr_c_in_order():
    cs, rs = c_structs(), rust_structs()
    assert {"fg_query_batch", "fg_docs_input", "fg_index_input", "fg_global_stats", "fg_model_out",
            "fg_object_record", "fg_merge_info", "fg_hit"} <= set(cs)
    for name, fields in cs.items():
        assert name in rs, name
        assert [(n, norm(t)) for n, t in fields] == rs[name], name


def test_abi_version_constant_matches():
    h = c_source("fugu.h")
    v = re.search(r"#define FG_ABI_VERSION (\d+)", h).group(1)
    assert re.search(rf"pub const FG_ABI_VERSION: c_int = {v};", rust_source())
    from fugu_amd import native
    assert native.ABI_VERSION == int(v)


def test_parser_catches_drift():
    """The checks above would fail on a reordered argument or field."""
    assert c_type_to_rust("fg_index* const*") == "*const *mut fg_index"
    assert c_type_to_rust("const char* const*") == "*const *const c_char"
    assert c_type_to_rust("const uint32_t*") == "*const u32"
    cf = c_functions()
    args = cf["fg_search_batch"][1]
    with pytest.raises(AssertionError):
        assert list(reversed(args)) == rust_functions()["fg_search_batch"][1]


def test_integration_doc_declares_nothing_itself():
    """rust/ffi.rs is the one FFI source: INTEGRATION.md names its items and
    declares none (a second hand-written copy would drift unchecked)."""
    import os
    from conftest import ROOT
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert not re.search(r"pub fn fg_\w+\s*\(", doc)
    assert not re.search(r"#\[repr\(C\)\]\s*pub struct fg_", doc)
    for name in re.findall(r"`(fg_\w+)`", doc):
        if name.startswith("fg_") and not name.endswith("_"):
            assert name in rust_source() or name in c_source("fugu.h") or name in c_source("fugu_host.h"), name
