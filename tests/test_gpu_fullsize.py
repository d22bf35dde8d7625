"""Parity at BASELINE.json's full sizes, against the C
restatement of the reference (oracle/build/spmv_ref, test infrastructure,
pinned to the Python oracle by tests/test_oracle_c.py):

* C2 — FD7 128³ F64 and F32, one part: bit-exact against the literal CSC
  column loop (SparseUtils.jl:157-187), both column encodings; FE27 128³ in
  ComplexF64 and 256³ in Float32 likewise (the oracle's typed loops);
* the bench's headline operator / C4 per GPU — FE27 256³, one part,
  442,840,880 nonzeros: bit-exact, both encodings;
* C3 — FE27 256³ on Cartesian parts (2,1,1), (2,2,1), (2,2,2) of one device,
  halo included: every owned row bit-exact against the C oracle's
  partitioned mul! (owned columns by oid, then ghost columns by hid, the
  reference's own order, Interfaces.jl:2259-2272); ghost values of x equal
  their owners' after mul!;
* C4 — cg! (IterativeSolvers 0.9 recurrence, device-side scalars) on the
  one-part 256³ operator for 20 iterations, and on the (2,2,2) 512³ weak-
  scaling problem (8 parts of 256³ on one device) for 5 iterations, against
  the C oracle's cg!, and the first mul! of the 512³ problem bit-exact.

  The CG tolerance is derived, not chosen: the reference's local dot/nrm2
  are BLAS, whose summation order is unpinned, and this
  operator (test_fem_sa.jl's Dirichlet rows keep only their diagonal while
  interior rows keep the Dirichlet columns: non-symmetric) amplifies a
  last-bit change of α or β quickly — at 128³ the two orders below differ
  by 5e-14 relative at iteration 1 and by 7e-7 at iteration 10.  The C oracle runs cg! twice, with sequential and with
  pairwise local sums; the device's residual history must stay within 10×
  the spread of those two reference orders (running maximum up to each
  iteration) + 1e-12, the first two iterations within 1e-12, and the same
  iteration count; x likewise."""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "build", "spmv_ref")
N1 = 256
SEED = 20250114


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 4


def _oracle(*args, timeout=600):
    if not os.path.exists(REF):
        pytest.fail("oracle/build/spmv_ref missing: run __graft_entry__.build() first")
    return subprocess.run([REF, *map(str, args)], check=True, capture_output=True, text=True,
                          timeout=timeout).stdout


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


@pytest.fixture(scope="module")
def ref256(tmp_path_factory):
    """(x, y = A·x) of the 256³ FE27 operator, one part, literal column loop."""
    d = tmp_path_factory.mktemp("ref256")
    x = np.random.default_rng(SEED + 11).uniform(-1, 1, N1 ** 3)
    x.tofile(d / "x.bin")
    _oracle("--kind", 27, "--n", N1, "--reps", 1, "--xin", d / "x.bin", "--yout", d / "y.bin")
    return x, np.fromfile(d / "y.bin"), d


def _one_part_check(be, pamd, kind, n, x_, yref, fmt):
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids((1, 1, 1))
        A = pamd.drivers.stencil_operator(parts, (n,) * 3, kind)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: x_, A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, x)
        got = y.to_host().local(1)
        bad = np.flatnonzero(got != yref)
        assert bad.size == 0, f"{bad.size} rows differ, first at gid {bad[0] + 1}"
        return A.values.local(1).info()
    finally:
        pamd._lib.tune("spmv_format", prev)


@pytest.mark.parametrize("fmt", [1, 0], ids=["pattern", "int32"])
def test_c2_fd7_128_one_part_bitexact(be, pamd, tmp_path, fmt):
    n = 128
    x_ = np.random.default_rng(SEED + 2).uniform(-1, 1, n ** 3)
    x_.tofile(tmp_path / "x.bin")
    _oracle("--kind", 7, "--n", n, "--reps", 1, "--xin", tmp_path / "x.bin", "--yout", tmp_path / "y.bin")
    info = _one_part_check(be, pamd, 7, n, x_, np.fromfile(tmp_path / "y.bin"), fmt)
    assert info["nnz"] == 14099408  # SURVEY.md §8 size table


def _typed_one_part(be, pamd, tmp_path, kind, n, dtype, seed):
    """y = A·x of the n³ operator in Float32 / ComplexF64 (one part), device
    (both encodings) and the C oracle's literal column loop in that type."""
    rng = np.random.default_rng(seed)
    if np.dtype(dtype).kind == "c":
        x_ = (rng.uniform(-1, 1, n ** 3) + 1j * rng.uniform(-1, 1, n ** 3)).astype(dtype)
    else:
        x_ = rng.uniform(-1, 1, n ** 3).astype(dtype)
    x_.tofile(tmp_path / "x.bin")
    tname = {np.dtype(np.float32): "f32", np.dtype(np.complex128): "c128"}[np.dtype(dtype)]
    _oracle("--kind", kind, "--n", n, "--dtype", tname, "--xin", tmp_path / "x.bin", "--yout", tmp_path / "y.bin")
    yref = np.fromfile(tmp_path / "y.bin", dtype=dtype)
    parts = be.get_part_ids((1, 1, 1))
    infos = {}
    for fmt in (1, 0):
        prev = pamd._lib.tune("spmv_format", fmt)
        try:
            A = pamd.drivers.stencil_operator(parts, (n,) * 3, kind, dtype)
            x = pamd.PVector.from_host(pamd.map_parts(lambda s: x_, A.cols.partition), A.cols)
            y = pamd.PVector.undef(A.rows, dtype)
            pamd.mul_(y, A, x)
            got = y.to_host().local(1)
            w = np.int32 if np.dtype(dtype).itemsize == 4 else np.int64
            bad = np.flatnonzero((got.view(w).reshape(len(got), -1) != yref.view(w).reshape(len(got), -1)).any(axis=1))
            assert bad.size == 0, f"fmt {fmt}: {bad.size} rows differ from the oracle, first at gid {bad[0] + 1}"
            infos[fmt] = A.values.local(1).info()
            del A, x, y
        finally:
            pamd._lib.tune("spmv_format", prev)
    return infos


def test_c2_fd7_128_f32_bitexact(be, pamd, tmp_path):
    """C2 in Float32 against the C oracle's Float32 column loop
    (Float32.(A): each value rounded once; SparseUtils.jl:157-187), both
    encodings.  F32 slices are 256 rows (two x-lines of 128): the middle row
    of a slice is an x = 0 boundary row, so the pattern candidate must come
    from another row (1/4 or 3/4): every slice is a pattern slice."""
    infos = _typed_one_part(be, pamd, tmp_path, 7, 128, np.float32, SEED + 3)
    assert infos[1]["pattern_slices"] == infos[1]["nslices"] == 8192


def test_fe27_128_c128_one_part_bitexact(be, pamd, tmp_path):
    """ComplexF64 (A .* (1+0.5im), complex x; Julia's complex product) one part of
    the 128³ FE27 operator against the C oracle, both encodings."""
    _typed_one_part(be, pamd, tmp_path, 27, 128, np.complex128, SEED + 4)


def test_fe27_256_f32_one_part_bitexact(be, pamd, tmp_path):
    """the headline operator (FE27 256³, one part) in Float32 against the C
    oracle, both encodings."""
    _typed_one_part(be, pamd, tmp_path, 27, 256, np.float32, SEED + 5)


@pytest.mark.parametrize("fmt", [1, 0], ids=["pattern", "int32"])
def test_fe27_256_one_part_bitexact(be, pamd, ref256, fmt):
    x_, yref, _ = ref256
    info = _one_part_check(be, pamd, 27, N1, x_, yref, fmt)
    assert info["nnz"] == 442840880


def _with_garbage_ghosts(s, x_):
    v = x_[s.lid_to_gid - 1].copy()
    v[s.hid_to_lid - 1] = 1.0e300
    return v


def _split_check(be, pamd, N, shape, x_, yref):
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    cp = A.cols.partition
    # ghost entries of x get garbage: mul!'s exchange! must replace them
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: _with_garbage_ghosts(s, x_), cp), A.cols)
    y = pamd.PVector.undef(A.rows)
    pamd.mul_(y, A, x)
    got = y.to_host()
    xs = x.to_host()
    nrows = 0
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        own = s.oid_to_lid - 1
        gid = s.lid_to_gid[own] - 1
        g = got.local(p)[own]
        bad = np.flatnonzero(g != yref[gid])
        assert bad.size == 0, f"part {p}: {bad.size} rows differ from the C oracle, first gid {gid[bad[0]] + 1}"
        nrows += len(own)
        sc = cp.local(p)
        hl = sc.hid_to_lid - 1
        assert sc.num_hids > 0
        assert np.array_equal(xs.local(p)[hl], x_[sc.lid_to_gid[hl] - 1]), f"part {p}: ghost values of x differ"
    assert nrows == int(np.prod(N))


@pytest.mark.parametrize("shape", [(2, 1, 1), (2, 2, 1), (2, 2, 2)])
def test_c3_fe27_256_split_bitexact(be, pamd, ref256, shape):
    x_, _, d = ref256
    _oracle("--kind", 27, "--n", N1, "--parts", *shape, "--xin", d / "x.bin", "--yout", d / "yp.bin",
            "--threads", _threads())
    _split_check(be, pamd, (N1,) * 3, shape, x_, np.fromfile(d / "yp.bin"))


def _cg_check(be, pamd, tmp_path, n, shape, iters):
    N = (n,) * 3
    b_ = np.random.default_rng(SEED + 4).uniform(-1, 1, n ** 3)
    b_.tofile(tmp_path / "b.bin")
    ref = {}
    for order in ("seq", "pairwise"):
        out = _oracle("--kind", 27, "--n", n, "--parts", *shape, "--cg", iters, "--bin", tmp_path / "b.bin",
                      "--hist", tmp_path / f"h_{order}.bin", "--xout", tmp_path / f"x_{order}.bin",
                      "--dot", order, "--threads", _threads(), timeout=900)
        ref[order] = np.fromfile(tmp_path / f"h_{order}.bin")
        assert len(ref[order]) == iters, out
    href = ref["seq"]
    spread = np.maximum.accumulate(np.abs(ref["pairwise"] - href) / np.abs(href))
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    cols = A.cols
    b = pamd.PVector.from_host(pamd.map_parts(lambda s: b_[s.lid_to_gid - 1], cols.partition), cols)
    if shape != (1, 1, 1):  # the first mul! of the split problem, bit-exact
        _oracle("--kind", 27, "--n", n, "--parts", *shape, "--xin", tmp_path / "b.bin", "--yout",
                tmp_path / "yb.bin", "--threads", _threads())
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, b)
        yref = np.fromfile(tmp_path / "yb.bin")
        yh = y.to_host()
        for p, s in zip(parts.part_ids, A.rows.partition.parts):
            own = s.oid_to_lid - 1
            assert np.array_equal(yh.local(p)[own], yref[s.lid_to_gid[own] - 1]), f"part {p}: mul! differs"
        del y, yh, yref
    x = pamd.PVector.undef(cols).fill_(0.0)
    hist = []
    pamd.cg_(x, A, b, reltol=0.0, maxiter=iters, history=hist, device=True, batch=8)
    assert len(hist) == iters
    rel = np.abs(np.array(hist) - href) / np.abs(href)
    assert rel[:2].max() <= 1e-12, f"first iterations off by {rel[:2].max():.3e}"
    bound = 10 * spread + 1e-12
    bad = np.flatnonzero(rel > bound)
    assert bad.size == 0, (f"residual history off by {rel[bad[0]]:.3e} at iteration {bad[0] + 1}, beyond 10x the "
                           f"spread of the two reference summation orders ({spread[bad[0]]:.3e})")
    xs, xp = np.fromfile(tmp_path / "x_seq.bin"), np.fromfile(tmp_path / "x_pairwise.bin")
    xspread = np.abs(xp - xs).max()
    xh = x.to_host()
    for p, s in zip(parts.part_ids, cols.partition.parts):
        own = s.oid_to_lid - 1
        err = np.abs(xh.local(p)[own] - xs[s.lid_to_gid[own] - 1]).max()
        assert err <= 10 * xspread + 1e-12 * np.abs(xs).max(), f"part {p}: x off by {err:.3e} (spread {xspread:.3e})"


def test_c4_cg_256_one_part(be, pamd, tmp_path):
    _cg_check(be, pamd, tmp_path, N1, (1, 1, 1), 20)


@pytest.mark.timeout(1200)
def test_c4_cg_512_eight_parts_one_device(be, pamd, tmp_path):
    """the (2,2,2) weak-scaling problem of BASELINE config 4 (8 × 256³ DOFs,
    ≈45 GB of operator) on one MI355X, halo between its parts"""
    _cg_check(be, pamd, tmp_path, 2 * N1, (2, 2, 2), 5)
