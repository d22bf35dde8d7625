"""The reference's driver problems on the device: test_fem_sa.jl (2D Q1 FE,
COO assembly with ghost rows, assemble! of the rhs, CG) against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_fem_sa_cg(be, pamd, O, nparts):
    parts = be.get_part_ids(nparts)
    A, b, x0, xh = pamd.drivers.fem_sa_problem(parts, 10)
    OA, ob, ox0, oxh = O.fem_sa_problem(O.get_part_ids(nparts), 10)
    # assemble!(b) on the device == the oracle's (ghost contributions added in order, ghosts zeroed)
    bh = b.to_host()
    for p in parts.part_ids:
        assert np.array_equal(bh.local(p), ob.values[p])
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist)
    d = pamd.map_parts(lambda u, v, s: u[s.oid_to_lid - 1] - v[s.oid_to_lid - 1], x.to_host(), xh.to_host(),
                       x.rows.partition)
    err = sum(float(np.sum(t ** 2)) for t in d.parts) ** 0.5
    assert err < 1e-5  # test_fem_sa.jl:137
    ox = O.PVector(O.map_parts(lambda v: v.copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist)
    np.testing.assert_allclose(hist, ohist, rtol=1e-8)


@pytest.mark.parametrize("fmt", [1, 0])
@pytest.mark.parametrize("shape,N,dtype", [((2, 2, 1), (12, 10, 9), np.float64), ((1, 1, 1), (9, 8, 7), np.float64),
                                           ((2, 1, 2), (10, 7, 9), np.complex128), ((2, 1, 1), (9, 9, 9), np.float32)])
def test_fused_cg_kernels(be, pamd, O, fmt, shape, N, dtype):
    """pa_spmv_dot_all: c bit-exact, dot(u,c) to 1e-12; pa_cg_update_all:
    x, r bit-exact against the broadcasts, norm(r) to 1e-12."""
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27, dtype)
        cols = A.cols
        rng = np.random.default_rng(9)

        def rnd(s):
            v = rng.uniform(-1, 1, s.num_lids)
            if np.dtype(dtype).kind == "c":
                v = v + 1j * rng.uniform(-1, 1, s.num_lids)
            return v.astype(dtype)
        vals = {k: {p: rnd(cols.partition.local(p)) for p in parts.part_ids} for k in "xruc"}
        mk = lambda k: pamd.PVector.from_host(pamd.map_parts(lambda s: vals[k][s.part], cols.partition), cols)
        u, c = mk("u"), mk("c")
        d = pamd.mul_dot_(c, A, u)
        c2 = mk("c")
        pamd.mul_(c2, A, u)
        d2 = pamd.dot(u, c2)
        for p in parts.part_ids:
            assert np.array_equal(c.to_host().local(p), c2.to_host().local(p))
        tol = 1e-5 if dtype == np.float32 else 1e-12
        assert abs(d - d2) <= tol * abs(d2)
        x, r = mk("x"), mk("r")
        x2, r2 = mk("x"), mk("r")
        alpha = np.asarray(0.37 + (0.11j if np.dtype(dtype).kind == "c" else 0), dtype=dtype).item()
        nr = pamd.cg_update_(x, r, u, c, alpha)
        pamd.axpy_(x2, alpha, u)
        pamd.axmy_(r2, alpha, c)
        nr2 = pamd.norm(r2)
        for p in parts.part_ids:
            assert np.array_equal(x.to_host().local(p), x2.to_host().local(p))
            assert np.array_equal(r.to_host().local(p), r2.to_host().local(p))
        assert abs(nr - nr2) <= tol * nr2
    finally:
        pamd._lib.tune("spmv_format", prev)


@pytest.mark.parametrize("fused", [True, False])
def test_fdm_cg_fused_and_unfused(be, pamd, O, fused):
    parts = be.get_part_ids((2, 2, 2))
    A, b, x0, xh = pamd.drivers.fdm_problem(parts, 10)
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist, fused=fused)
    OA, ob, ox0, oxh = O.fdm_problem(O.get_part_ids((2, 2, 2)), 10)
    ox = O.PVector(O.map_parts(lambda v: v.copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist)
    np.testing.assert_allclose(hist, ohist, rtol=1e-8)


def test_interfaces_diag_matvec_kat(be, pamd):
    """test_interfaces.jl:646-680 on the irregular IndexSet partition (non
    contiguous owned lids on some parts): A = 2I, x = 3 → 6 (owned, then all
    lids after exchange!); values set to 1 → 3."""
    import json
    import os
    k = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "interfaces_kats.json")))["exchanger"]
    parts = be.get_part_ids(4)
    part = pamd.PData(parts.backend, parts.part_ids,
                      [pamd.IndexSet(p + 1, k["lid_to_gid"][p], k["lid_to_part"][p]) for p in range(4)], parts.shape)
    ids = pamd.prange_from_partition(10, part)
    csc = pamd.map_parts(lambda s: pamd.compresscoo(np.arange(1, s.num_lids + 1), np.arange(1, s.num_lids + 1),
                                                    np.full(s.num_lids, 2.0), s.num_lids, s.num_lids), ids.partition)
    A = pamd.PSparseMatrix.from_csc(csc, ids, ids)
    x = pamd.PVector.undef(ids).fill_(3.0)
    b = pamd.PVector.undef(ids)
    pamd.mul_(b, A, x)
    for v, s in zip(b.to_host().parts, ids.partition.parts):
        assert (v[s.oid_to_lid - 1] == 6.0).all()
    pamd.exchange_(b)
    assert all((v == 6.0).all() for v in b.to_host().parts)
    for M, C in zip(A.values.parts, csc.parts):  # fillstored!(A, 1.0)
        M.set_values(np.ones(C.nnz))
    pamd.mul_(b, A, x)
    pamd.exchange_(b)
    assert all((v == 3.0).all() for v in b.to_host().parts)
    # exchange! of 10*part values (test_interfaces.jl:623-641) through a PVector
    v = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.where(s.lid_to_part == s.part, 10.0 * s.part, 0.0), ids.partition), ids)
    pamd.exchange_(v)
    for vv, s in zip(v.to_host().parts, ids.partition.parts):
        assert (vv == 10.0 * s.lid_to_part).all()


def _nz_eq(M, OM):
    return np.array_equal(M.get_values(), OM.nzval)


@pytest.mark.parametrize("fmt", [1, 0])
@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_fem_sa_matrix_exchange_assemble(be, pamd, O, nparts, fmt):
    """exchange!(A) / assemble!(A) (Interfaces.jl:2375-2404) on test_fem_sa's
    matrix (ghost rows stored by the COO assembly): nonzeros(A) bit-exact
    against the oracle after each, and mul! with the assembled values."""
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids(nparts)
        A, b, x0, _ = pamd.drivers.fem_sa_problem(parts, 10)
        OA, ob, ox0, _ = O.fem_sa_problem(O.get_part_ids(nparts), 10)
        for M, OM in zip(A.values.parts, OA.values.parts):
            assert _nz_eq(M, OM)
        # give the ghost rows values so both directions move data
        rng = np.random.default_rng(11)
        for M, OM in zip(A.values.parts, OA.values.parts):
            v = rng.uniform(-1, 1, len(OM.nzval))
            M.set_values(v)
            OM.nzval[:] = v
        pamd.assemble_(A)
        O.assemble_matrix_(OA)
        for M, OM in zip(A.values.parts, OA.values.parts):
            assert _nz_eq(M, OM)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), A.cols.partition),
                                   A.cols)
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
            assert _nz_eq(M, OM)
    finally:
        pamd._lib.tune("spmv_format", prev)


def test_interfaces_matrix_exchange_kat(be, pamd, O):
    """test_interfaces.jl:676-683: fillstored!(A, 1) then exchange!(A) and
    assemble!(A) on the irregular IndexSet partition's diagonal matrix: each
    owned diagonal ends as 1 + (number of parts ghosting it), ghosts 0."""
    import json
    import os
    k = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "interfaces_kats.json")))["exchanger"]
    parts = be.get_part_ids(4)
    sets = [pamd.IndexSet(p + 1, k["lid_to_gid"][p], k["lid_to_part"][p]) for p in range(4)]
    ids = pamd.prange_from_partition(10, pamd.PData(parts.backend, parts.part_ids, sets, parts.shape))
    csc = pamd.map_parts(lambda s: pamd.compresscoo(np.arange(1, s.num_lids + 1), np.arange(1, s.num_lids + 1),
                                                    np.full(s.num_lids, 2.0), s.num_lids, s.num_lids), ids.partition)
    A = pamd.PSparseMatrix.from_csc(csc, ids, ids)
    for M, C in zip(A.values.parts, csc.parts):
        M.set_values(np.ones(C.nnz))
    pamd.exchange_(A)
    assert all((M.get_values() == 1.0).all() for M in A.values.parts)
    pamd.assemble_(A)
    nghost = {}
    for s in sets:
        for g, o in zip(s.lid_to_gid, s.lid_to_part):
            if o != s.part:
                nghost[int(g)] = nghost.get(int(g), 0) + 1
    for M, s in zip(A.values.parts, sets):
        want = np.where(s.lid_to_part == s.part, 1.0 + np.array([nghost.get(int(g), 0) for g in s.lid_to_gid]), 0.0)
        assert np.array_equal(M.get_values(), want)


def _stencil_rhs(pamd, A, dtype, seed):
    cols = A.cols

    def rnd(s):
        r = np.random.default_rng(seed + s.part)
        v = r.uniform(-1, 1, s.num_lids)
        if np.dtype(dtype).kind == "c":
            v = v + 1j * r.uniform(-1, 1, s.num_lids)
        return v.astype(dtype)
    return pamd.PVector.from_host(pamd.map_parts(rnd, cols.partition), cols)


@pytest.fixture(params=[0, 1, 2], ids=["u_sweep", "u_in_spmv", "u_auto"])
def cgfuse(request, pamd, be):
    """Every device recurrence (pa_tune cg_fuse): u .= r .+ β.*u as its own
    sweep (default), evaluated inside the SpMV, or auto (one batch of each,
    then the faster: the switch between batches changes no value)."""
    prev = pamd._lib.tune("cg_fuse", request.param)
    yield request.param
    pamd._lib.tune("cg_fuse", prev)


@pytest.mark.parametrize("shape,N,dtype,batch,maxiter", [
    ((2, 2, 1), (12, 10, 9), np.float64, 8, 40),    # 4 local parts: device gather kernel
    ((1, 1, 1), (9, 8, 7), np.float64, 3, 25),      # batch not dividing maxiter
    ((2, 1, 2), (10, 7, 9), np.complex128, 5, 30),
    ((2, 1, 1), (9, 9, 9), np.float32, 4, 20),
    ((2, 2, 2), (8, 8, 8), np.complex64, 7, 20),
])
def test_device_cg_equals_host_cg(be, pamd, O, cgfuse, shape, N, dtype, batch, maxiter):
    """pa_cg_solve_all (scalars on the device, batched enqueue) reproduces the
    host-driven fused CG bit for bit: x, the residual history, and the
    iteration count (reltol = 0 → exactly maxiter iterations)."""
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27, dtype)
    b = _stencil_rhs(pamd, A, dtype, 31)
    xs = []
    hs = []
    for device in (False, True):
        x = pamd.PVector.undef(A.cols, dtype).fill_(0)
        h = []
        pamd.cg_(x, A, b, reltol=0.0, maxiter=maxiter, history=h, fused=True, device=device, batch=batch)
        xs.append(x.to_host())
        hs.append(h)
    assert len(hs[0]) == len(hs[1]) == maxiter
    assert hs[0] == hs[1]
    for p in parts.part_ids:
        assert np.array_equal(xs[0].local(p), xs[1].local(p))


@pytest.mark.parametrize("shape,batch", [((2, 2, 2), 1), ((2, 2, 2), 4), ((2, 2, 2), 64), ((1, 1, 1), 5),
                                         ((1, 1, 1), 64)])
def test_device_cg_converges_like_test_fdm(be, pamd, O, shape, batch):
    """test_fdm.jl's CG with the device recurrence: same iteration count and
    history as the host-driven loop (convergence stops mid-batch), and
    norm(x - x̂) < 1e-5 (test_fdm.jl:118).  One part: the folds end in the
    scalar updates (no gather kernels)."""
    parts = be.get_part_ids(shape)
    A, b, x0, xh = pamd.drivers.fdm_problem(parts, 10)
    x1 = x0.copy()
    h1 = []
    pamd.cg_(x1, A, b, history=h1, fused=True)
    x2 = x0.copy()
    h2 = []
    pamd.cg_(x2, A, b, history=h2, device=True, batch=batch)
    assert h1 == h2 and 0 < len(h2) < 1000
    d = pamd.map_parts(lambda u, v, s: u[s.oid_to_lid - 1] - v[s.oid_to_lid - 1], x2.to_host(), xh.to_host(),
                       x2.rows.partition)
    assert sum(float(np.sum(t ** 2)) for t in d.parts) ** 0.5 < 1e-5
    for p in parts.part_ids:
        assert np.array_equal(x1.to_host().local(p), x2.to_host().local(p))


def test_device_cg_fem_sa(be, pamd, O):
    """test_fem_sa.jl's CG (COO-assembled matrix with stored ghost rows) on
    the device recurrence, against the oracle's residual history."""
    parts = be.get_part_ids(4)
    A, b, x0, xh = pamd.drivers.fem_sa_problem(parts, 10)
    if not all(s.num_oids == 0 or (s.oid_to_lid[0] == 1 and s.oid_to_lid[-1] == s.num_oids)
               for s in A.cols.partition.parts):
        pytest.skip("non-contiguous owned lids")
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist, device=True)
    OA, ob, ox0, oxh = O.fem_sa_problem(O.get_part_ids(4), 10)
    ox = O.PVector(O.map_parts(lambda v: v.copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist)
    np.testing.assert_allclose(hist, ohist, rtol=1e-8)


@pytest.mark.parametrize("device", [False, True])
def test_fdm_cg_float32_julia_scalars(be, pamd, O, device):
    """test_fdm.jl in Float32: IterativeSolvers' residual, β and α are
    Float64 (norm of a PVector is Float64, Interfaces.jl:1771), so the
    broadcasts evaluate in Float64 and round to Float32, and dot/norm add the
    parts' Float32 values in Float32.  The device CG (host-driven and device
    recurrence) follows the oracle's Float32 cg! with those semantics: the
    first three residuals bit for bit (Float32 scalars would differ from the
    first iteration on: tools/cg32_probe.py), then within 5e-6 relative (the
    local dot/norm summation order is BLAS's in the reference: unpinned),
    same iteration count."""
    shape = (2, 2, 2)
    parts = be.get_part_ids(shape)
    A, b, x0, _ = pamd.drivers.fdm_problem(parts, 10, np.float32)
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist, device=device)
    OA, ob, ox0, _ = O.fdm_problem(O.get_part_ids(shape), 10)
    vals = O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, O._convert_values(M.nzval, np.float32)),
                       OA.values)
    OA32 = O.PSparseMatrix(vals, OA.rows, OA.cols)
    ob32 = O.PVector(O.map_parts(lambda v: np.asarray(v, np.float32).copy(), ob.values), ob.rows)
    ox = O.PVector(O.map_parts(lambda v: np.asarray(v, np.float32).copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA32, ob32, log=ohist)
    assert len(hist) == len(ohist) and len(hist) > 5
    rel = max(abs(a - b) / abs(b) for a, b in zip(hist, ohist))
    print(f"Float32 CG: {len(hist)} iterations, max relative history difference {rel:.3e}")
    assert hist[:3] == ohist[:3]
    assert rel <= 5e-6
