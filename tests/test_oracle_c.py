"""The C restatement (oracle/build/spmv_ref, test infrastructure) against the
Python oracle, which the reference's own KATs pin (test_oracle_kats.py).

The C oracle is the checker of the BASELINE-size GPU tests (C2, C3, C4,
tests/test_gpu_fullsize.py), where the Python oracle is too slow:
* its partitioned mul! (Cartesian parts, ghosts in add_gids! first-touch
  order, owned-then-ghost summation) equals the Python oracle's mul! bit for
  bit, and its row-wise form equals its literal column loop over each part's
  local CSC (SparseUtils.jl:176-185) bit for bit;
* its cg! (IterativeSolvers 0.9 recurrence) follows the Python oracle's
  residual history (the two sum the owned partials of dot/norm in different
  orders: 1e-12 relative)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "build", "spmv_ref")


@pytest.fixture(scope="module")
def ref():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return REF


def _global_from_parts(O, pv, n):
    out = np.zeros(n)
    for s, v in zip(pv.rows.partition.parts, pv.values.parts):
        own = np.asarray(s.oid_to_lid) - 1
        out[np.asarray(s.lid_to_gid)[own] - 1] = v[own]
    return out


def _run(ref, *args):
    return subprocess.run([ref, *map(str, args)], check=True, capture_output=True, text=True).stdout


@pytest.mark.parametrize("kind", [7, 27])
@pytest.mark.parametrize("shape", [(1, 1, 1), (2, 1, 1), (2, 2, 1), (2, 2, 2), (3, 2, 1)])
def test_partitioned_spmv_equals_python_oracle(O, ref, tmp_path, kind, shape):
    N = 9
    n = N ** 3
    x = np.random.default_rng(5 + kind).uniform(-1, 1, n)
    x.tofile(tmp_path / "x.bin")
    _run(ref, "--kind", kind, "--n", N, "--parts", *shape, "--xin", tmp_path / "x.bin", "--yout",
         tmp_path / "y.bin", "--threads", 3)
    _run(ref, "--kind", kind, "--n", N, "--parts", *shape, "--xin", tmp_path / "x.bin", "--yout",
         tmp_path / "yl.bin", "--literal")
    y, yl = np.fromfile(tmp_path / "y.bin"), np.fromfile(tmp_path / "yl.bin")
    assert np.array_equal(y, yl), "row-wise form differs from the literal column loop"
    parts = O.get_part_ids(shape)
    A = O.stencil_problem(parts, (N,) * 3, kind)
    ox = O.PVector(O.map_parts(lambda s: x[np.asarray(s.lid_to_gid) - 1].copy(), A.cols.partition), A.cols)
    oy = O.pvector_undef(A.rows)
    O.mul_(oy, A, ox)
    got = _global_from_parts(O, oy, n)
    bad = np.flatnonzero(got != y)
    assert bad.size == 0, f"{bad.size} rows differ from the Python oracle (first gid {bad[:1] + 1})"


def test_one_part_literal_equals_partitioned(ref, tmp_path):
    """the one-part literal CSC mode (the headline checker) == --parts 1 1 1"""
    N = 12
    x = np.random.default_rng(3).uniform(-1, 1, N ** 3)
    x.tofile(tmp_path / "x.bin")
    _run(ref, "--kind", 27, "--n", N, "--reps", 1, "--xin", tmp_path / "x.bin", "--yout", tmp_path / "a.bin")
    _run(ref, "--kind", 27, "--n", N, "--parts", 1, 1, 1, "--xin", tmp_path / "x.bin", "--yout", tmp_path / "b.bin")
    assert np.array_equal(np.fromfile(tmp_path / "a.bin"), np.fromfile(tmp_path / "b.bin"))


@pytest.mark.parametrize("kind,shape", [(7, (2, 2, 2)), (27, (2, 2, 1)), (27, (1, 1, 1))])
def test_cg_history_equals_python_oracle(O, ref, tmp_path, kind, shape):
    N, K = 9, 12
    n = N ** 3
    b = np.random.default_rng(11).uniform(-1, 1, n)
    b.tofile(tmp_path / "b.bin")
    out = _run(ref, "--kind", kind, "--n", N, "--parts", *shape, "--cg", K, "--bin", tmp_path / "b.bin",
               "--hist", tmp_path / "h.bin", "--xout", tmp_path / "x.bin", "--threads", 2)
    h = np.fromfile(tmp_path / "h.bin")
    assert len(h) == K, out
    parts = O.get_part_ids(shape)
    A = O.stencil_problem(parts, (N,) * 3, kind)
    ob = O.PVector(O.map_parts(lambda s: b[np.asarray(s.lid_to_gid) - 1].copy(), A.cols.partition), A.cols)
    ox = O.pvector_undef(A.cols)
    hist = []
    O.cg_(ox, A, ob, reltol=0.0, maxiter=K, log=hist)
    assert len(hist) == K
    np.testing.assert_allclose(h, hist, rtol=1e-12, atol=0)
    np.testing.assert_allclose(np.fromfile(tmp_path / "x.bin"), _global_from_parts(O, ox, n), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("kind", [7, 27])
def test_f32_one_part_equals_python_oracle(O, ref, tmp_path, kind):
    """--dtype f32 (the Float32 checker of the full-size GPU tests): the
    literal column loop over Float32.(A) equals the Python oracle's mul! in
    Float32 bit for bit."""
    N = 10
    n = N ** 3
    x = np.random.default_rng(21 + kind).uniform(-1, 1, n).astype(np.float32)
    x.tofile(tmp_path / "x.bin")
    _run(ref, "--kind", kind, "--n", N, "--dtype", "f32", "--xin", tmp_path / "x.bin", "--yout", tmp_path / "y.bin")
    y = np.fromfile(tmp_path / "y.bin", dtype=np.float32)
    parts = O.get_part_ids((1, 1, 1))
    A = O.stencil_problem(parts, (N,) * 3, kind, np.float32)
    ox = O.PVector(O.map_parts(lambda s: x[np.asarray(s.lid_to_gid) - 1].copy(), A.cols.partition), A.cols)
    oy = O.pvector_undef(A.rows, np.float32)
    O.mul_(oy, A, ox)
    got = np.asarray(oy.values.parts[0])[np.asarray(A.rows.partition.parts[0].oid_to_lid) - 1]
    order = np.asarray(A.rows.partition.parts[0].lid_to_gid)[np.asarray(A.rows.partition.parts[0].oid_to_lid) - 1] - 1
    yy = np.empty(n, np.float32)
    yy[order] = got
    assert yy.dtype == np.float32 and np.array_equal(yy.view(np.int32), y.view(np.int32))


def test_c128_one_part_equals_python_oracle(O, ref, tmp_path):
    """--dtype c128 over A .* (1+0.5im) (BASELINE config 5's complex operator,
    the device stencil's too) with Julia's complex product equals the Python
    oracle's ComplexF64 mul! bit for bit."""
    N = 9
    n = N ** 3
    rng = np.random.default_rng(4)
    xr, xi = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    (xr + 1j * xi).astype(np.complex128).tofile(tmp_path / "xc.bin")
    _run(ref, "--kind", 27, "--n", N, "--dtype", "c128", "--xin", tmp_path / "xc.bin", "--yout", tmp_path / "yc.bin")
    yc = np.fromfile(tmp_path / "yc.bin", dtype=np.complex128)
    parts = O.get_part_ids((1, 1, 1))
    A = O.stencil_problem(parts, (N,) * 3, 27, np.complex128)
    s = A.cols.partition.parts[0]
    g = np.asarray(s.lid_to_gid) - 1
    ox = O.PVector(O.map_parts(lambda t: O.Cx(xr[g].copy(), xi[g].copy()), A.cols.partition), A.cols)
    oy = O.pvector_undef(A.rows, np.complex128)
    O.mul_(oy, A, ox)
    own = np.asarray(A.rows.partition.parts[0].oid_to_lid) - 1
    order = np.asarray(A.rows.partition.parts[0].lid_to_gid)[own] - 1
    v = oy.values.parts[0]
    assert np.array_equal(yc.real[order], v.re[own]) and np.array_equal(yc.imag[order], v.im[own])


@pytest.mark.parametrize("kind,dims,shape", [(27, (12, 10, 9), (2, 2, 1)), (7, (11, 13, 10), (2, 1, 2)),
                                             (27, (16, 16, 16), (2, 2, 2)), (27, (18, 9, 9), (2, 1, 1))])
def test_mpi_baseline_equals_partitioned_and_python(O, ref, tmp_path, kind, dims, shape):
    """--mpi (bench.py's CPU baseline beside the multi-GPU lines: one rank per
    part, its own CSC, a halo exchange of x in every mul!) computes exactly
    the partitioned mul! of the checker, on non-cubic global grids too, and
    that equals the Python oracle."""
    n = int(np.prod(dims))
    x = np.random.default_rng(8).uniform(-1, 1, n)
    x.tofile(tmp_path / "x.bin")
    _run(ref, "--kind", kind, "--dims", *dims, "--parts", *shape, "--xin", tmp_path / "x.bin", "--yout",
         tmp_path / "y1.bin")
    out = _run(ref, "--kind", kind, "--dims", *dims, "--parts", *shape, "--mpi", "--reps", 3, "--xin",
               tmp_path / "x.bin", "--yout", tmp_path / "y2.bin")
    y1, y2 = np.fromfile(tmp_path / "y1.bin"), np.fromfile(tmp_path / "y2.bin")
    assert np.array_equal(y1, y2), out
    parts = O.get_part_ids(shape)
    A = O.stencil_problem(parts, dims, kind)
    ox = O.PVector(O.map_parts(lambda s: x[np.asarray(s.lid_to_gid) - 1].copy(), A.cols.partition), A.cols)
    oy = O.pvector_undef(A.rows)
    O.mul_(oy, A, ox)
    assert np.array_equal(_global_from_parts(O, oy, n), y1)


@pytest.mark.parametrize("dims,shape", [((16, 16, 16), (2, 2, 2)), ((24, 12, 12), (2, 1, 1))])
def test_bench_cpu_baseline_mpi_leg(ref, dims, shape):
    """bench.py's CPU baseline beside the N > 1 lines and the halo leg: one
    rank per part, halo values counted, a positive rate, cores = ranks."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    r = bench.cpu_baseline_mpi(27, dims, shape, seconds=0.2)
    P = int(np.prod(shape))
    assert r["cores"] == r["ranks"] == P and r["kind"] == "port"
    assert r["value"] > 0 and r["ms_per_spmv"] > 0 and r["halo_values_per_spmv"] > 0
