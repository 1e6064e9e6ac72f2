"""The C-ABI library loads and exports every symbol include/fugu.h declares.

No compute calls here (CPU-only container): only load/export checks and the
argument/error paths that never touch a device.
"""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT


def header_functions(header="fugu.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fg_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_abi():
    fns = header_functions()
    for f in ["fg_ctx_create", "fg_index_build_from_docs", "fg_index_build", "fg_plan_create", "fg_plan_execute",
              "fg_search_batch", "fg_search_sharded", "fg_merge_shards", "fg_last_error", "fg_bytes_model"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib_path = os.path.join(ROOT, "fugu_amd", "libfugu.so")
    assert os.path.exists(lib_path), "libfugu.so not built"
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (fg_[a-z0-9_]+)$", out, flags=re.M))
    declared = header_functions() + header_functions("fugu_host.h")
    missing = [f for f in declared if f not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(lib_path)
    for f in declared:
        getattr(lib, f)


def test_python_binding_matches_header():
    from fugu_amd import native
    assert sorted(native.EXPORTS) == header_functions()
    from fugu_amd import db
    assert sorted(db.HOST_EXPORTS) == header_functions("fugu_host.h")


def test_version_and_errors_without_device():
    from fugu_amd import native
    assert "gfx950" in native.version()
    n = native.device_count()
    assert n >= 0
    if n == 0:
        with pytest.raises(native.FuguError) as e:
            native.Context((0,))
        assert e.value.code == native.FG_ENODEV
        assert "device" in str(e.value).lower()


def test_null_arguments_are_rejected():
    from fugu_amd import native
    lib = native.lib()
    assert lib.fg_ctx_create(1, None, None) == native.FG_EINVAL
    assert lib.fg_plan_create(None, None, 10, None) == native.FG_EINVAL
    assert lib.fg_index_stats_get(None, None) == native.FG_EINVAL
    assert lib.fg_merge_shards(0, 1, 1, None, None, None, None, None, None, None, None) == native.FG_EINVAL
    assert lib.fg_search_sharded(None, None, 0, None, 10, None, None, None, None) == native.FG_EINVAL
    assert native.lib().fg_last_error()


def test_kernels_are_gfx950_code_objects():
    lib_path = os.path.join(ROOT, "fugu_amd", "libfugu.so")
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", lib_path], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout
