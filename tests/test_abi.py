"""The C ABI: libnqk.so loads without a GPU and exports every symbol declared in
include/nqk.h, and the ctypes table binds exactly those symbols."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from numpy_quant import _lib

HEADER = os.path.join(ROOT, "include", "nqk.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nqk_[a-z0-9_]+)\s*\(", text)))


def test_library_built_for_gfx950():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", _lib.LIB_PATH], capture_output=True, text=True)
    # the offload bundle carries gfx950 code objects
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_exports_every_header_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    funcs = header_functions()
    assert len(funcs) >= 35
    for name in funcs:
        assert hasattr(lib, name), f"{name} declared in nqk.h but not exported"


def test_ctypes_table_matches_header():
    funcs = set(header_functions())
    bound = set(_lib.SIGNATURES) | {"nqk_last_error"}
    assert funcs == bound, (funcs - bound, bound - funcs)


def test_load_declares_signatures():
    lib = _lib.load()
    assert lib.nqk_quantize.restype is ctypes.c_int
    assert lib.nqk_last_error.restype is ctypes.c_char_p
