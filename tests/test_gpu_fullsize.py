"""Parity at BASELINE.json's full sizes, against the C
restatement of the reference's CSC column loop (oracle/build/spmv_ref,
SparseUtils.jl:157-187; test infrastructure only):

* C4 per GPU / the bench's headline operator: FE27, 256³ nodes, one part,
  442,840,880 nonzeros — bit-exact in both column encodings;
* C3 with 8 parts: FE27, 256³ nodes on Cartesian parts (2,2,2) of one
  device, halo included — rows whose stencil stays inside their part sum the
  same entries in the same order as the one-part oracle and are bit-exact;
  rows reading ghosts add their ghost columns last (the reference's own
  owned-then-ghost order, Interfaces.jl:2259-2272), so they are checked
  against the one-part sum within the reordering bound 27·ε·Σ|a_ij x_j|.
  The 8-part ordering itself is pinned bit-exactly against the Python oracle
  at smaller sizes (test_gpu_parity.py)."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "build", "spmv_ref")
N1 = 256
SEED = 20250114


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


@pytest.fixture(scope="module")
def ref256(tmp_path_factory):
    """(x, y = A·x) of the 256³ FE27 operator from the C oracle (~15 s)."""
    if not os.path.exists(REF):
        pytest.fail("oracle/build/spmv_ref missing: run __graft_entry__.build() first")
    d = tmp_path_factory.mktemp("ref256")
    x = np.random.default_rng(SEED + 11).uniform(-1, 1, N1 ** 3)
    x.tofile(d / "x.bin")
    subprocess.run([REF, "--kind", "27", "--n", str(N1), "--reps", "1", "--xin", str(d / "x.bin"),
                    "--yout", str(d / "y.bin")], check=True, capture_output=True, timeout=300)
    return x, np.fromfile(d / "y.bin")


@pytest.mark.parametrize("fmt", [1, 0], ids=["pattern", "int32"])
def test_fe27_256_one_part_bitexact(be, pamd, ref256, fmt):
    x_, yref = ref256
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids((1, 1, 1))
        A = pamd.drivers.stencil_operator(parts, (N1,) * 3, 27)
        assert A.values.local(1).info()["nnz"] == 442840880
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: x_, A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, x)
        got = y.to_host().local(1)
        bad = np.flatnonzero(got != yref)
        assert bad.size == 0, f"{bad.size} rows differ, first at gid {bad[0] + 1}"
    finally:
        pamd._lib.tune("spmv_format", prev)


def test_fe27_256_eight_parts(be, pamd, ref256):
    x_, yref = ref256
    N = (N1,) * 3
    parts = be.get_part_ids((2, 2, 2))
    A = pamd.drivers.stencil_operator(parts, N, 27)
    cp = A.cols.partition
    # ghost entries of x get garbage: mul!'s exchange! must replace them
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: _with_garbage_ghosts(s, x_), cp), A.cols)
    y = pamd.PVector.undef(A.rows)
    pamd.mul_(y, A, x)
    got = y.to_host()
    ke = np.abs(pamd.drivers.stencil_coeffs(27, N)).max()
    bound = 27 * np.finfo(np.float64).eps * 27 * 8 * ke  # Σ|a_ij x_j| <= 27 · 8·max|Ke| · max|x|
    n_exact = n_ghost_rows = 0
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        own = s.oid_to_lid - 1
        gid = s.lid_to_gid[own] - 1
        g = got.local(p)[own]
        gx, gy, gz = gid % N[0], (gid // N[0]) % N[1], gid // (N[0] * N[1])
        lo = [c.min() for c in (gx, gy, gz)]
        hi = [c.max() for c in (gx, gy, gz)]
        inner = np.ones(len(gid), bool)
        for c, l, h, n in zip((gx, gy, gz), lo, hi, N):  # box faces next to another part read ghosts
            if l > 0:
                inner &= c > l
            if h < n - 1:
                inner &= c < h
        assert np.array_equal(g[inner], yref[gid[inner]]), f"part {p}: rows without ghost columns differ"
        diff = np.abs(g[~inner] - yref[gid[~inner]])
        assert diff.max(initial=0.0) <= bound, f"part {p}: ghost rows off by {diff.max()} > {bound}"
        n_exact += int(inner.sum())
        n_ghost_rows += int((~inner).sum())
        # the halo: ghost values of x after mul! are their owners' values
        xs = x.to_host().local(p)
        sc = cp.local(p)
        hl = sc.hid_to_lid - 1
        assert np.array_equal(xs[hl], x_[sc.lid_to_gid[hl] - 1]), f"part {p}: ghost values of x differ"
    assert n_exact + n_ghost_rows == N1 ** 3 and n_ghost_rows > 0


def _with_garbage_ghosts(s, x_):
    v = x_[s.lid_to_gid - 1].copy()
    v[s.hid_to_lid - 1] = 1.0e300
    return v
