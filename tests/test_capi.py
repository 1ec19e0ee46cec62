"""The C-ABI library loads and exports every symbol include/k3m_hip.h declares (no GPU calls)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(REPO, "include", "k3m_hip.h")).read()
    return sorted(set(re.findall(r"^int (k3m_[a-z0-9_]+)\(", src, re.M)))


def test_header_matches_binding_table():
    from k3m_amd import _lib
    assert declared() == sorted(_lib.SIGNATURES), "include/k3m_hip.h and k3m_amd/_lib.py disagree"


def test_library_exports_every_symbol():
    from k3m_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from k3m_amd.build_lib import build
        build()
    got = _lib.exported_symbols()
    assert sorted(got) == declared()
    lib = _lib.load()
    assert lib is not None


def dynamic_k3m_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if re.search(r" T k3m_", ln)})


def test_library_exports_nothing_undeclared():
    """Every exported k3m_* function is declared in include/k3m_hip.h (no hidden entry points)."""
    from k3m_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from k3m_amd.build_lib import build
        build()
    assert dynamic_k3m_symbols(_lib.LIB_PATH) == declared()


def declared_data():
    src = open(os.path.join(REPO, "include", "k3m_data.h")).read()
    return sorted(set(re.findall(r"^(?:int|void|uint32_t|double|int64_t) (k3m_[a-z0-9_]+)\(", src, re.M)))


def test_data_header_matches_library():
    from k3m_amd import data
    if not os.path.exists(data.DATA_LIB_PATH):
        from k3m_amd.build_lib import build_data
        build_data()
    assert declared_data() == sorted(data.DATA_SIGNATURES)
    assert sorted(data.data_exported_symbols()) == declared_data()
