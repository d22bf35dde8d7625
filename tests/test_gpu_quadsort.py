"""The quad-sorted layout (pa_tune "spmv_quadsort"): on
irregular partitions (BASELINE config 5) the lanes of the SELL layout —
quads of R consecutive owned rows — are reordered by class so that whole
slices become pattern slices or quad-run slices (kind 4: one column per lane
and entry, the x values as one 16 B run).  Only the slice-lane holding a row
changes, never the order of its entries: mul! stays bit-exact against the
oracle (SparseUtils.jl:176-185), and the CSC nz → slot map follows the rows
(set/get values, exchange!(A) / assemble!(A) on test_fem_sa's matrix)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250114
BIG = (128, 128, 128)


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


class _knob:
    def __init__(self, pamd, key, value):
        self.pamd, self.key, self.value = pamd, key, value

    def __enter__(self):
        self.prev = self.pamd._lib.tune(self.key, self.value)

    def __exit__(self, *a):
        self.pamd._lib.tune(self.key, self.prev)


_ORACLE = {}


def _oracle(O, N, nparts, dtype):
    if (N, nparts) not in _ORACLE:
        _ORACLE[(N, nparts)] = O.irregular_problem(O.get_part_ids(nparts), N, 27)
    A = _ORACLE[(N, nparts)]
    if np.dtype(dtype) == np.float64:
        return A
    vals = O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, O._convert_values(M.nzval, dtype)), A.values)
    return O.PSparseMatrix(vals, A.rows, A.cols)


def _rand(rng, n, dtype):
    if np.dtype(dtype).kind == "c":
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(dtype)
    return rng.uniform(-1, 1, n).astype(dtype)


def _eq(O, got, ref):
    if isinstance(ref, O.Cx):
        return np.array_equal(got.real, ref.re) and np.array_equal(got.imag, ref.im)
    return np.array_equal(got, ref)


@pytest.mark.parametrize("N,nparts,dtype,alpha,beta", [
    (BIG, 8, np.float64, 1.0, 0.0), (BIG, 8, np.float32, 1.0, 0.0), (BIG, 8, np.complex64, 1.0, 0.0),
    (BIG, 8, np.float64, 2.0, 0.5), ((24, 22, 20), 12, np.float64, 1.0, 0.0),
    ((40, 36, 32), 8, np.float32, -1.5, 1.0)])
def test_quadsort_spmv_bitexact(be, pamd, O, N, nparts, dtype, alpha, beta):
    with _knob(pamd, "spmv_quadsort", 1):
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
    info = A.info()
    assert any(i["quad_sorted"] for i in info.parts)
    if N == BIG:
        assert sum(i["quadrun_slices"] for i in info.parts) > 0
    OA = _oracle(O, N, nparts, dtype)
    rng = np.random.default_rng(SEED + 17)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    ys = {p: _rand(rng, A.rows.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], A.rows.partition), A.rows)
    pamd.mul_(y, A, x, alpha, beta)
    cx = lambda a: O.Cx(a.real.copy(), a.imag.copy()) if np.iscomplexobj(a) else a.copy()
    ox = O.PVector(O.map_parts(lambda s: cx(xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.PVector(O.map_parts(lambda s: cx(ys[s.part]), OA.rows.partition), OA.rows)
    O.mul_(oy, OA, ox, alpha, beta)
    got = y.to_host()
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        own = s.oid_to_lid - 1
        g = got.local(p)[own]
        r = oy.values[p]
        r = O.Cx(r.re[own], r.im[own]) if isinstance(r, O.Cx) else r[own]
        assert _eq(O, g, r), f"part {p}: SpMV differs on the quad-sorted layout"


def test_quadsort_c128_keeps_identity_layout(be, pamd):
    """R = 1 (ComplexF64: one row per lane): nothing to sort."""
    with _knob(pamd, "spmv_quadsort", 1):
        parts = be.get_part_ids(8)
        A = pamd.drivers.irregular_problem(parts, (24, 22, 20), 27, np.complex128)
    assert not any(i["quad_sorted"] for i in A.info().parts)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_quadsort_equals_identity_and_paths(be, pamd, dtype):
    """The same C5 matrix in the identity and the quad-sorted layout: mul!
    bit-identical, through the grouped merged launch and the per-part
    launches; the fused dot within 1e-12 (its per-slice partials follow the
    slices)."""
    N, nparts = (48, 44, 40), 8
    parts = be.get_part_ids(nparts)
    rng = np.random.default_rng(SEED + 19)
    out = {}
    for qs in (0, 1):
        with _knob(pamd, "spmv_quadsort", qs):
            A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids).astype(dtype) for p in parts.part_ids} \
            if qs == 0 else xs
        for grp in (1, 0):
            with _knob(pamd, "spmv_group", grp):
                x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
                y = pamd.PVector.undef(A.rows, dtype)
                d = pamd.mul_dot_(y, A, x)
                out[(qs, grp)] = ([v.copy() for v in y.to_host().parts], d)
    ref = out[(0, 1)]
    for key, (ys, d) in out.items():
        for p, (a, b) in enumerate(zip(ys, ref[0])):
            own = parts.part_ids[p]
            assert np.array_equal(a[:len(b)], b), f"{key}: part {own} differs"
        tol = 1e-12 if np.dtype(dtype) == np.float64 else 1e-5
        assert abs(d - ref[1]) <= tol * abs(ref[1])


def test_quadsort_values_and_matrix_exchange(be, pamd, O):
    """spmv_quadsort = 2 sorts every matrix: test_fem_sa's COO-assembled
    matrix (ghost rows stored after the slots) keeps nonzeros(A) in CSC
    order (the nz → slot map followed the lanes), and exchange!(A) /
    assemble!(A) and mul! stay bit-exact against the oracle."""
    with _knob(pamd, "spmv_quadsort", 2):
        parts = be.get_part_ids((2, 2))
        A, b, x0, _ = pamd.drivers.fem_sa_problem(parts, 10)
    assert all(i["quad_sorted"] for i in A.info().parts)
    OA, _, _, _ = O.fem_sa_problem(O.get_part_ids((2, 2)), 10)
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)
    rng = np.random.default_rng(13)
    for M, OM in zip(A.values.parts, OA.values.parts):
        v = rng.uniform(-1, 1, len(OM.nzval))
        M.set_values(v)
        OM.nzval[:] = v
    pamd.assemble_(A)
    O.assemble_matrix_(OA)
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    ox = O.PVector(O.PData([v.copy() for v in x.to_host().parts], OA.cols.partition.shape), OA.cols)
    y = pamd.PVector.undef(A.rows)
    oy = O.pvector_undef(OA.rows)
    pamd.mul_(y, A, x)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        assert np.array_equal(y.to_host().local(p)[s.oid_to_lid - 1], oy.values[p][s.oid_to_lid - 1])
    pamd.exchange_(A)
    O.exchange_matrix_(OA)
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_quadsort_device_cg_equals_host_cg(be, pamd, dtype):
    """The device CG (u update inside the SpMV) on a quad-sorted matrix
    equals the host-driven fused loop bit for bit (x incl. ghosts, history)."""
    parts = be.get_part_ids(8)
    with _knob(pamd, "spmv_quadsort", 1):
        A = pamd.drivers.irregular_problem(parts, (28, 26, 24), 27, dtype)
    assert any(i["quad_sorted"] for i in A.info().parts)
    b = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(31 + s.part).uniform(-1, 1, s.num_lids).astype(dtype), A.cols.partition),
        A.cols)
    xs, hs = [], []
    for device in (False, True):
        x = pamd.PVector.undef(A.cols, dtype).fill_(0)
        h = []
        pamd.cg_(x, A, b, reltol=0.0, maxiter=15, history=h, fused=True, device=device, batch=6)
        xs.append(x.to_host())
        hs.append(h)
    assert hs[0] == hs[1] and len(hs[0]) == 15
    for p in parts.part_ids:
        assert np.array_equal(xs[0].local(p), xs[1].local(p))
