"""CPU-side checks of the C ABI: the library loads, exports every symbol the
header declares, and refuses to run without a device (no CPU fallback)."""
import ctypes
import subprocess

import pytest

from cycloneml_amd import _native as N


def test_library_exports_every_declared_symbol():
    lib = N.load()
    syms = N.header_symbols()
    assert len(syms) >= 10
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    nm = subprocess.run(["nm", "-D", "--defined-only", N.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    exported = {line.split()[-1] for line in nm.splitlines() if line.strip()}
    assert set(syms) <= exported


def test_python_signatures_cover_header():
    assert set(N.header_symbols()) == set(N.SIGNATURES)


def test_version_and_error_plumbing():
    lib = N.load()
    assert lib.cyc_version() >= 100
    rc = lib.cyc_kmeans_plan_create(0, 2, 1, ctypes.byref(ctypes.c_void_p()))
    assert rc == N.CYC_ERR_INVALID_ARG
    assert b"requirement failed" in lib.cyc_last_error()
    with pytest.raises(N.IllegalArgumentException):
        N.check(rc)


def test_no_device_no_fallback():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    lib = N.load()
    rc = lib.cyc_kmeans_plan_create(8, 2, 1, ctypes.byref(ctypes.c_void_p()))
    assert rc == N.CYC_ERR_NO_DEVICE


def test_tiles_row_block_matches_python():
    """SparseTiles.ROW_BLOCK (the append granularity callers use) is the
    library's row block (a constant getter: no device call)."""
    from cycloneml_amd.optim import SparseTiles
    assert N.load().cyc_tiles_row_block() == SparseTiles.ROW_BLOCK == 2048
