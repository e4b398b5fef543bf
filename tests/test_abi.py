"""CPU: the C-ABI library builds, loads and exports every symbol include/wcb.h declares
(no compute calls: there is no GPU here). Plus host-side logic that needs no device."""
import os
import re
import subprocess

import pytest

from whisper_context_biasing_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wcb.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wcb_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    _lib.build()
    return _lib.load()


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("wcb_create", "wcb_set_weight", "wcb_finalize_weights", "wcb_log_mel", "wcb_encode",
              "wcb_generate", "wcb_forward", "wcb_bias_create", "wcb_last_error", "wcb_destroy"):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (wcb_[a-z_0-9]+)$", out, flags=re.M))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    # and the ctypes signature table covers them all
    assert set(declared_symbols()) == set(_lib.SIGNATURES), set(declared_symbols()) ^ set(_lib.SIGNATURES)


def test_code_object_targets_gfx950(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True,
                         text=True).stdout
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "no gfx950 code object in libwcb.so"


def test_errors_do_not_cross_the_abi(lib):
    # a null descriptor is rejected with a status code and a message, not an exception/abort
    import ctypes as C
    h = C.c_void_p()
    rc = lib.wcb_create(None, 0, C.byref(h))
    assert rc == -1
    assert b"null" in lib.wcb_last_error(None)


def test_product_has_no_oracle_import():
    pkg = os.path.join(ROOT, "whisper_context_biasing_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in re.findall(r"^\s*(?:from|import)\s+(\w+)", src, flags=re.M), f
