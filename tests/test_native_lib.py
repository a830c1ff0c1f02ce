"""The C-ABI library loads on a GPU-less host and exports exactly what
include/hipcycles.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

from raytracingproject_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "hipcycles.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hipcy_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = _declared()
    for need in ("hipcy_create", "hipcy_const_copy_to", "hipcy_bind_global", "hipcy_mem_alloc",
                 "hipcy_load_kernels", "hipcy_path_trace", "hipcy_error", "hipcy_synchronize"):
        assert need in names


def test_library_exports_every_declared_symbol():
    path = native.device_lib_path()
    if not os.path.exists(path):
        pytest.fail("libhipcycles.so missing: run python -m raytracingproject_amd.build")
    lib = ctypes.CDLL(path)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(native.DEVICE_SYMBOLS) == set(_declared())


def test_abi_version():
    lib = native.device_lib()
    assert lib.hipcy_abi_version() == native.ABI_VERSION


def test_library_is_gfx950_code_object():
    data = open(native.device_lib_path(), "rb").read()
    assert b"gfx950" in data


def test_host_builder_exports():
    lib = native.host_lib()
    for n in ("hcb_build", "hcb_pack", "hcb_free"):
        assert hasattr(lib, n)
