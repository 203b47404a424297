"""CPU: the C-ABI library loads and exports every symbol include/csm_amd.h
declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

from conftest import ROOT, ensure_built


def declared_functions():
    text = open(os.path.join(ROOT, "include", "csm_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(csm_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    for required in ["csm_fast2d_create", "csm_fast2d_match", "csm_fast2d_match_full_submap",
                     "csm_fast2d_match_batch", "csm_rt2d_match", "csm_scan_set_create"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    ensure_built()
    lib = ctypes.CDLL(os.path.join(ROOT, "cartographer-1_amd", "libcsm_amd.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_mirror_binds_every_symbol(csm):
    assert set(csm._SIGNATURES) == set(declared_functions())
    csm.load_library()


def test_strerror_without_gpu(csm):
    lib = csm.load_library()
    assert lib.csm_strerror(csm.CSM_ERANGE).decode().startswith("input exceeds")


def test_context_create_fails_loudly_without_gpu(csm):
    import pytest
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(csm.CsmError):
        csm.Context(0)
