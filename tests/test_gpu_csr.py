"""SparseMatrixCSR{Bi} local matrices on the device (SparseUtils.jl:189-300;
PSparseMatrix(sparsecsr, I, J, V, rows, cols; ids), Interfaces.jl:2194-2215):
pa_mat_from_csr, bit-exact against the oracle's CSR restatement — per row
the owned columns in storage order, then the ghost columns (the
owned_owned / owned_ghost passes of SparseUtils.jl:242-250), and α scaling
each product, (v*x)*α (:247), where a CSC parent scales x."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250114


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


def _rand(rng, n, dtype):
    if np.dtype(dtype).kind == "c":
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(dtype)
    return rng.uniform(-1, 1, n).astype(dtype)


def _ox(O, a):
    return O.Cx(a.real.copy(), a.imag.copy()) if np.iscomplexobj(a) else a.copy()


def _eq(O, got, ref):
    if isinstance(ref, O.Cx):
        return np.array_equal(got.real, ref.re) and np.array_equal(got.imag, ref.im)
    return np.array_equal(got, ref)


def _sel(O, ref, idx):
    return O.Cx(ref.re[idx], ref.im[idx]) if isinstance(ref, O.Cx) else ref[idx]


def _host_csr(pamd, O, M):
    nz = M.nzval
    if isinstance(nz, O.Cx):
        nz = (nz.re + 1j * nz.im).astype(np.complex64 if nz.re.dtype == np.float32 else np.complex128)
    return pamd.CSR(M.Bi, M.m, M.n, M.rowptr, M.colval, nz)


def _csr_init(O, Bi):
    return lambda i, j, v, m, n: O.sparse_csr(Bi, i, j, v, m, n)


@pytest.mark.parametrize("fmt", [1, 0], ids=["pattern", "int32"])
@pytest.mark.parametrize("Bi", [0, 1])
@pytest.mark.parametrize("shape,N,kind,dtype", [
    ((2, 2, 1), (12, 10, 9), 27, np.float64), ((2, 1, 2), (9, 7, 10), 7, np.float64),
    ((2, 2, 1), (10, 9, 8), 27, np.float32), ((2, 1, 1), (10, 9, 8), 27, np.complex128),
    ((1, 2, 2), (8, 10, 9), 27, np.complex64)])
def test_csr_stencil_spmv_bitexact(be, pamd, O, fmt, Bi, shape, N, kind, dtype):
    """pa_mat_from_csr of the oracle's CSR parts: mul! with (α, β) = (1, 0),
    (0.7, 0), (-1.3, 0.5) (complex: α = 0.3-0.8im) bit-exact against the
    oracle's CSR mul!; α = 1 equals the CSC parent's result."""
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids(shape)
        S = pamd.drivers.stencil_operator(parts, N, kind, dtype)  # the partition (and the CSC result at α = 1)
        OA = O.stencil_problem(O.get_part_ids(shape), N, kind, dtype, init=_csr_init(O, Bi))
        csr = pamd.PData(parts.backend, parts.part_ids, [_host_csr(pamd, O, M) for M in OA.values.parts], parts.shape)
        A = pamd.PSparseMatrix.from_csr(csr, S.rows, S.cols)
        rng = np.random.default_rng(SEED)
        xs = {p: _rand(rng, S.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        ys = {p: _rand(rng, S.rows.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        cx = np.dtype(dtype).kind == "c"
        ab = [(1.0, 0.0), (0.7, 0.0), (-1.3, 0.5)] + ([(0.3 - 0.8j, 0.25 + 0.5j)] if cx else [])
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], S.cols.partition), S.cols)
        for alpha, beta in ab:
            y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], S.rows.partition), S.rows)
            pamd.mul_(y, A, x, alpha, beta)
            ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
            oy = O.PVector(O.map_parts(lambda s: _ox(O, ys[s.part]), OA.rows.partition), OA.rows)
            oa = O.Cx(np.float64(alpha.real), np.float64(alpha.imag)) if isinstance(alpha, complex) else alpha
            ob = O.Cx(np.float64(beta.real), np.float64(beta.imag)) if isinstance(beta, complex) else beta
            if cx and np.dtype(dtype) == np.complex64:
                oa = O.Cx(np.float32(alpha.real), np.float32(alpha.imag)) if isinstance(alpha, complex) else np.float32(alpha)
                ob = O.Cx(np.float32(beta.real), np.float32(beta.imag)) if isinstance(beta, complex) else np.float32(beta)
            elif np.dtype(dtype) == np.float32:
                oa, ob = np.float32(alpha), np.float32(beta)
            O.mul_(oy, OA, ox, oa, ob)
            got = y.to_host()
            for p in parts.part_ids:
                own = S.rows.partition.local(p).oid_to_lid - 1
                assert _eq(O, got.local(p)[own], _sel(O, oy.values[p], own)), (alpha, beta, p)
            if alpha == 1.0 and beta == 0.0:
                yc = pamd.PVector.undef(S.rows, dtype)
                pamd.mul_(yc, S, x)
                for p in parts.part_ids:
                    own = S.rows.partition.local(p).oid_to_lid - 1
                    assert np.array_equal(yc.to_host().local(p)[own], got.local(p)[own])
    finally:
        pamd._lib.tune("spmv_format", prev)


def test_csr_literal_alpha_order(be, pamd, O):
    """α != 1 on a CSR parent follows the literal SparseUtils.jl:222-252 loop
    ((v*x)*α), not the CSC twin's v*(x*α): the device equals the literal
    oracle bit for bit, and differs from the CSC parent in some last bit."""
    shape, N = (2, 1, 1), (9, 8, 7)
    parts = be.get_part_ids(shape)
    S = pamd.drivers.stencil_operator(parts, N, 27)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27, init=_csr_init(O, 1))
    csr = pamd.PData(parts.backend, parts.part_ids, [_host_csr(pamd, O, M) for M in OA.values.parts], parts.shape)
    A = pamd.PSparseMatrix.from_csr(csr, S.rows, S.cols)
    rng = np.random.default_rng(3)
    xs = {p: rng.uniform(-1, 1, S.cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], S.cols.partition), S.cols)
    y, yc = pamd.PVector.undef(S.rows), pamd.PVector.undef(S.rows)
    alpha = 0.1
    pamd.mul_(y, A, x, alpha, 0.0)
    pamd.mul_(yc, S, x, alpha, 0.0)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows)
    O.mul_(oy, OA, ox, alpha, 0.0, literal=True)
    differs = False
    for p in parts.part_ids:
        own = S.rows.partition.local(p).oid_to_lid - 1
        a = y.to_host().local(p)[own]
        assert np.array_equal(a, oy.values[p][own])
        differs |= not np.array_equal(a, yc.to_host().local(p)[own])
    assert differs


@pytest.mark.parametrize("Bi", [0, 1])
@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_csr_fem_sa_from_coo_exchange_assemble(be, pamd, O, nparts, Bi):
    """PSparseMatrix(sparsecsr, I, J, V, rows, cols; ids=:global) of
    test_fem_sa's assembled triplets (ghost rows stored, duplicates summed):
    nonzeros(A) in CSR order == the oracle's after the build, assemble!(A),
    exchange!(A); mul! bit-exact."""
    parts = be.get_part_ids(nparts)
    rows, cols, I, J, V, _, _, _ = pamd.drivers.fem_sa_host(parts, 10)
    A = pamd.PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global", init=pamd.csr_init(Bi))
    OA, _, _, _ = O.fem_sa_problem(O.get_part_ids(nparts), 10, init=_csr_init(O, Bi))
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)
    rng = np.random.default_rng(11)
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
    pamd.mul_(y, A, x, 0.6, 0.0)
    O.mul_(oy, OA, ox, 0.6, 0.0)
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        assert np.array_equal(y.to_host().local(p)[s.oid_to_lid - 1], oy.values[p][s.oid_to_lid - 1])
    pamd.exchange_(A)
    O.exchange_matrix_(OA)
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)


@pytest.mark.parametrize("Bi,dtype,alpha", [(1, np.float64, 1.0), (0, np.float64, -0.35),
                                             (1, np.complex128, 0.5 + 0.25j), (0, np.float32, 1.0)])
def test_csr_irregular_bitexact(be, pamd, O, Bi, dtype, alpha):
    """C5-style Voronoi parts (non-box owned sets, first-touch ghosts,
    delta16 / int32 slices) with CSR parents: mul! and the ghost values of
    x bit-exact against the oracle."""
    N, nparts = (24, 22, 20), 8
    parts = be.get_part_ids(nparts)
    rows, cols, I, J, V = pamd.drivers.irregular_partition(parts, N, 27)
    V = pamd.map_parts(lambda v: pamd.drivers.convert_values(v, dtype), V)
    A = pamd.PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global", init=pamd.csr_init(Bi))
    OA = O.irregular_problem(O.get_part_ids(nparts), N, 27, dtype, init=_csr_init(O, Bi))
    rng = np.random.default_rng(SEED + 5)
    xs = {p: _rand(rng, cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], cols.partition), cols)
    y = pamd.PVector.undef(rows, dtype)
    pamd.mul_(y, A, x, alpha, 0.0)
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    oa = O.Cx(np.float64(alpha.real), np.float64(alpha.imag)) if isinstance(alpha, complex) else alpha
    if np.dtype(dtype) == np.float32:
        oa = np.float32(alpha)
    O.mul_(oy, OA, ox, oa, 0.0)
    got, gx = y.to_host(), x.to_host()
    for p in parts.part_ids:
        own = rows.partition.local(p).oid_to_lid - 1
        assert _eq(O, got.local(p)[own], _sel(O, oy.values[p], own)), p
        assert _eq(O, gx.local(p), ox.values[p]), p


@pytest.mark.parametrize("exact", [1, 0])
def test_csr_long_rows_alpha(be, pamd, exact):
    """Long rows (row-length histogram) of a CSR parent with α != 1: the
    long-row kernels scale each product, (v*x)*α — exact mode bit-exact
    against SparseUtils.jl:242-250 restated here, chunked mode within 1e-12."""
    parts = be.get_part_ids((2, 1, 1))
    _, part = pamd.drivers.stencil_partition(parts, (20, 18, 16), 27)
    rng = np.random.default_rng(29)
    csr, ref = {}, {}
    for p in parts.part_ids:
        s = part.partition.local(p)
        I, J = [], []
        longs = set(int(v) for v in rng.choice(s.oid_to_lid, size=3, replace=False))
        for li in s.oid_to_lid:
            k = 3000 if int(li) in longs else 9
            I += [int(li)] * k
            J += list(rng.integers(1, s.num_lids + 1, size=k))
        V = rng.uniform(-1, 1, len(I))
        csr[p] = pamd.sparsecsr(1, I, J, V, s.num_lids, s.num_lids)
    A = pamd.PSparseMatrix.from_csr(pamd.PData(parts.backend, parts.part_ids, [csr[p] for p in parts.part_ids],
                                               parts.shape), part, part)
    for p in parts.part_ids:
        assert A.values.local(p).info()["long_rows"] == 3
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), part.partition), part)
    alpha = 0.3
    prev = pamd._lib.tune("long_rows_exact", exact)
    try:
        y = pamd.PVector.undef(part)
        pamd.mul_(y, A, x, alpha, 0.0)
    finally:
        pamd._lib.tune("long_rows_exact", prev)
    xh = x.to_host()
    for p in parts.part_ids:
        s, M, xl = part.partition.local(p), csr[p], xh.local(p)
        l2o = np.asarray(s.lid_to_ohid)
        want = np.zeros(s.num_lids)
        for li in s.oid_to_lid - 1:
            acc = 0.0
            rng_ = range(M.rowptr[li] - 1, M.rowptr[li + 1] - 1)
            for ghost in (False, True):
                for q in rng_:
                    j = M.colval[q] - 1
                    if (l2o[j] < 0) == ghost:
                        acc = acc + (M.nzval[q] * xl[j]) * alpha
            want[li] = acc
        own = s.oid_to_lid - 1
        got = y.to_host().local(p)[own]
        if exact:
            assert np.array_equal(got, want[own])
        else:
            np.testing.assert_allclose(got, want[own], rtol=1e-12, atol=1e-12 * np.abs(want).max())


@pytest.mark.parametrize("Bi", [0, 1])
@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_csr_fem_sa_device_cg(be, pamd, O, nparts, Bi):
    """test_fem_sa.jl with SparseMatrixCSR{Bi} parents, assembled on the
    device end to end (device COO → assemble!(I,J,V,rows) → sparsecsr on the
    device, pa_mat_from_dcoo_csr): nonzeros(A) == the oracle's CSR, equal to
    the host-compressed build, and the CG history follows the oracle's."""
    parts = be.get_part_ids(nparts)
    A, b, x0, xh = pamd.drivers.fem_sa_problem(parts, 10, init=pamd.csr_init(Bi))
    OA, ob, ox0, oxh = O.fem_sa_problem(O.get_part_ids(nparts), 10, init=_csr_init(O, Bi))
    for M, OM in zip(A.values.parts, OA.values.parts):
        assert np.array_equal(M.get_values(), OM.nzval)
    rows, cols, I, J, V, _, _, _ = pamd.drivers.fem_sa_host(parts, 10)
    H = pamd.PSparseMatrix.from_csr(
        pamd.map_parts(lambda i, j, v, r, c: pamd.sparsecsr(Bi, r.to_lids(i), c.to_lids(j), v, r.num_lids, c.num_lids),
                       I, J, V, rows.partition, cols.partition), rows, cols)
    for M, MH in zip(A.values.parts, H.values.parts):
        assert np.array_equal(M.get_values(), MH.get_values())
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist)
    ox = O.PVector(O.map_parts(lambda v: v.copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist)
    np.testing.assert_allclose(hist, ohist, rtol=1e-8)


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32])
def test_csr_device_compress_duplicates_bitexact(be, pamd, O, dtype):
    """sparsecsr on the device (pa_mat_from_coo_csr) of shuffled triplets with
    many duplicates == the oracle's sparse_csr (input-order sums), and mul!
    with α != 1 == the oracle's CSR mul!."""
    parts = be.get_part_ids((2, 1, 1))
    _, part = pamd.drivers.stencil_partition(parts, (12, 10, 9), 27)
    rng = np.random.default_rng(41)
    trip = {}
    for p in parts.part_ids:
        s = part.partition.local(p)
        n = 40 * len(s.oid_to_lid)
        I = rng.choice(s.oid_to_lid, size=n)
        J = rng.integers(1, s.num_lids + 1, size=n)
        V = _rand(rng, n, dtype)
        trip[p] = (I, J, V)
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [trip[p][k] for p in parts.part_ids], parts.shape)
    A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), part, part, ids="local", init=pamd.csr_init(0))
    xs = {p: _rand(rng, part.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], part.partition), part)
    y = pamd.PVector.undef(part, dtype)
    alpha = 0.37
    pamd.mul_(y, A, x, alpha, 0.0)
    for p in parts.part_ids:
        s = part.partition.local(p)
        I, J, V = trip[p]
        OM = O.sparse_csr(0, I, J, _ox(O, V), s.num_lids, s.num_lids)
        got = A.values.local(p).get_values()
        assert _eq(O, got, OM.nzval)
    # mul! of each part: SparseUtils.jl:242-250 over its owned rows (owned
    # columns, then ghost columns, storage order), α on each product
    got = y.to_host()
    for p in parts.part_ids:
        s = part.partition.local(p)
        I, J, V = trip[p]
        M = pamd.sparsecsr(0, I, J, V, s.num_lids, s.num_lids)
        xl = x.to_host().local(p)
        l2o = np.asarray(s.lid_to_ohid)
        want = np.zeros(s.num_lids, dtype)
        a = np.dtype(dtype).type(alpha)
        for li in s.oid_to_lid - 1:
            acc = np.dtype(dtype).type(0)
            for ghost in (False, True):
                for q in range(M.rowptr[li], M.rowptr[li + 1]):
                    j = M.colval[q]
                    if (l2o[j] < 0) == ghost:
                        acc = acc + (M.nzval[q] * xl[j]) * a
            want[li] = acc
        own = s.oid_to_lid - 1
        if np.dtype(dtype).kind == "c":
            # Julia's complex product, not numpy's (which may fuse differently): compare to 1 ulp-ish
            np.testing.assert_allclose(got.local(p)[own], want[own], rtol=1e-13)
        else:
            assert np.array_equal(got.local(p)[own], want[own])


@pytest.mark.parametrize("fmt", [1, 0], ids=["pattern", "int32"])
@pytest.mark.parametrize("parent", ["csc", "csr"])
def test_fillstored_on_device(be, pamd, O, fmt, parent):
    """fillstored!(A, v) (Interfaces.jl:2127-2132) on the device
    (pa_mat_fillstored): nonzeros(A) all v (ghost rows included), and mul!
    then equals the oracle's mul! with every stored value = v; test_fem_sa's
    matrix (stored ghost rows, side rows)."""
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids((2, 2))
        init = pamd.csr_init(1) if parent == "csr" else None
        A, _, _, _ = pamd.drivers.fem_sa_problem(parts, 10, init=init)
        OA, _, _, _ = O.fem_sa_problem(O.get_part_ids((2, 2)), 10,
                                       init=_csr_init(O, 1) if parent == "csr" else None)
        v = -0.625
        pamd.fillstored_(A, v)
        for M, OM in zip(A.values.parts, OA.values.parts):
            got = M.get_values()
            assert got.shape == OM.nzval.shape and np.all(got == v)
            OM.nzval[:] = v
        rng = np.random.default_rng(8)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
        ox = O.PVector(O.PData([t.copy() for t in x.to_host().parts], OA.cols.partition.shape), OA.cols)
        y = pamd.PVector.undef(A.rows)
        oy = O.pvector_undef(OA.rows)
        pamd.mul_(y, A, x)
        O.mul_(oy, OA, ox)
        for p in parts.part_ids:
            own = A.rows.partition.local(p).oid_to_lid - 1
            assert np.array_equal(y.to_host().local(p)[own], oy.values[p][own])
    finally:
        pamd._lib.tune("spmv_format", prev)
