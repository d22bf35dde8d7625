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


def test_tune_knobs_round_trip_and_reject_bad_values(pamd):
    """pa_tune (no device needed): every knob returns its previous value and
    refuses out-of-range values with a PAError; spmv_flags keeps bit 8 (the
    per-matrix CSR flag) out of the user's reach."""
    knobs = {"spmv_merge": 0, "spmv_merge_max": 1024, "spmv_group": 0, "spmv_delta16": 0,
             "long_rows_exact": 0, "halo_direct": 0, "cg_fuse": 1, "halo_pull": 0, "spmv_format": 0,
             "issue_threads": 0, "pattern_min_regular": 90, "fault_inject": 1, "spmv_tri16": 0,
             "halo_barrier": 0, "spmv_xcd_chunk": 8,
             "spmv_tri_order": 0, "spmv_side_tail": 0, "f32_rows": 2, "spmv_tri_pack": 0, "spmv_uniform": 0}
    for k, v in knobs.items():
        prev = pamd._lib.tune(k, v)
        assert pamd._lib.tune(k, prev) == v, k
    prev = pamd._lib.tune("spmv_flags", 0)
    try:
        assert pamd._lib.tune("spmv_flags", prev | 32) == 0
        for bad in (256, 512, 1024, -1):
            try:
                pamd._lib.tune("spmv_flags", bad)
                raise AssertionError(f"spmv_flags accepted {bad}")
            except pamd.PAError:
                pass
    finally:
        pamd._lib.tune("spmv_flags", prev)
    for k, bad in (("spmv_merge", 2), ("spmv_merge_max", -1), ("cg_fuse", 3), ("pattern_min_regular", -1),
                   ("pattern_min_regular", 101), ("f32_rows", 1), ("f32_rows", 3), ("f32_rows", 8),
                   ("spmv_tri_pack", 8), ("spmv_uniform", 2)):
        try:
            pamd._lib.tune(k, bad)
            raise AssertionError(f"{k} accepted {bad}")
        except pamd.PAError:
            pass
    # the knobs of rounds 1-3's negative A/Bs are gone
    for k in ("spmv_quadsort", "spmv_patterns", "spmv_pattern_rule", "spmv_lds", "comm_cus", "spmv_short_occ",
              "alloc_contiguous", "spmv_unroll"):
        try:
            pamd._lib.tune(k, 0)
            raise AssertionError(f"{k} still accepted")
        except pamd.PAError:
            pass


def test_knobs_of_concurrent_calls_are_independent(pamd):
    """Each call resolves its knobs (process defaults under its context's
    overrides) into its own Knobs instead of swapping process globals
    (ADVICE r04): 4 and 8 host threads with different
    context values, read on the caller and on the IssuePool's threads while
    another thread moves the process default, never see another call's
    value."""
    for nthreads in (4, 8):
        assert pamd._lib.knob_selftest(nthreads, 3000) == 0
    assert pamd._lib.tune("spmv_merge_max", 65536) == 65536  # the selftest restored the default
