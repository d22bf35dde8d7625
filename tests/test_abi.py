"""The C-ABI library: built for gfx950, loadable, and exporting every entry
point include/pa_hip.h declares (no compute calls: CPU only)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pa_hip.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(pa_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ["pa_ctx_create", "pa_index_create", "pa_xchg_create", "pa_vec_create", "pa_mat_from_csc",
                 "pa_spmv_all", "pa_exchange_all", "pa_dot_all", "pa_norm2_all", "pa_comm_init_rank"]:
        assert must in names


def test_library_exports_every_declared_symbol(pamd):
    L = pamd._lib.lib()
    for name in declared():
        assert hasattr(L, name), name
    assert set(declared()) == set(pamd._lib.EXPORTED)


def test_library_is_gfx950_code_object(pamd):
    # the HIP fat binary embeds the offload target id (amdgcn-amd-amdhsa--gfx950)
    data = open(pamd.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    # and only that target: no code objects for other GPUs
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx\w+)", data))
    assert targets == {b"gfx950"}, targets
    # the library links RCCL (the MPIBackend-role transport) and exports C symbols
    out = subprocess.run(["nm", "-D", "--defined-only", pamd.LIB_PATH], capture_output=True, text=True).stdout
    assert " T pa_spmv_all" in out and " T pa_comm_init_all" in out
    deps = subprocess.run(["ldd", pamd.LIB_PATH], capture_output=True, text=True).stdout
    assert "librccl" in deps


def test_error_reporting_without_gpu(pamd):
    L = pamd._lib.lib()
    assert L.pa_version() == 1
    n = ctypes.c_int(-1)
    assert L.pa_device_count(ctypes.byref(n)) == 0
    if n.value == 0:
        h = ctypes.c_void_p()
        rc = L.pa_ctx_create(0, 1, 1, ctypes.byref(h))
        assert rc != 0 and len(L.pa_last_error()) > 0
        # the product fails loudly: no CPU fallback
        import pytest
        with pytest.raises(pamd.PAError):
            pamd.HIPBackend()
