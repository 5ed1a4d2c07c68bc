"""CPU: the C-ABI library loads and exports every symbol include/hcrag.h declares."""
import os
import re

import pytest

from hcrag_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_in_header():
    txt = open(os.path.join(ROOT, "include", "hcrag.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hcr_[a-z0-9_]+)\s*\(", txt)))


def test_library_loads_and_exports_all_symbols():
    L = _lib.lib()
    missing = [s for s in declared_in_header() if not hasattr(L, s)]
    assert not missing, f"symbols declared in hcrag.h but not exported: {missing}"


def test_every_header_symbol_has_a_ctypes_signature():
    assert set(declared_in_header()) <= set(_lib.declared_symbols())


def test_version_and_device_count_do_not_need_a_gpu():
    L = _lib.lib()
    assert b"gfx950" in L.hcr_version()
    assert _lib.device_count() >= 0


def test_create_rejects_bad_arguments():
    import ctypes
    h = ctypes.c_void_p()
    with pytest.raises(ValueError):
        _lib.check(_lib.lib().hcr_index_create(0, 0, 0, 0, ctypes.byref(h)))
    with pytest.raises(ValueError):
        _lib.check(_lib.lib().hcr_index_create(0, 16, 7, 0, ctypes.byref(h)))


def test_no_gpu_means_loud_failure():
    if _lib.device_count() > 0:
        pytest.skip("GPU present")
    from hcrag_amd import VectorIndex
    with pytest.raises(ValueError, match="not available"):
        VectorIndex(16)
