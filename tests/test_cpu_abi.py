"""The C-ABI library loads and exports every symbol include/ddt_hip.h declares."""
from __future__ import annotations

import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    text = open(os.path.join(ROOT, "include", "ddt_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ddt_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    import ompi_amd
    lib = ctypes.CDLL(ompi_amd.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) > 40
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from ompi_amd._lib import SIGNATURES
    missing = [s for s in declared_symbols() if s not in SIGNATURES]
    assert not missing, missing


def test_selftest_and_version():
    import ompi_amd
    assert ompi_amd.lib().ddt_selftest() == 0
    assert b"gfx950" in ompi_amd.lib().ddt_version()


def test_library_is_gfx950_code_object():
    import ompi_amd
    data = open(ompi_amd.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_errors_are_negative_codes():
    import pytest
    import ompi_amd
    from ompi_amd import datatype as D
    t = D.create_vector(3, 1, 2, D.MPI.MPI_INT)   # not committed
    with pytest.raises(ompi_amd.DDTError) as ei:
        ompi_amd.Convertor().prepare_for_send(t, 1, 0x1000)
    assert ei.value.code == -6
