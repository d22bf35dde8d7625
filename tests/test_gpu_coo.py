"""Device sparse(I, J, V) + SELL build (pa_mat_from_coo)
against the host restatement (compresscoo → pa_mat_from_csc): the CSC
pattern, nonzeros(A) in CSC order (duplicates summed in input order) and the
SpMV are bit-identical."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


def _random_coo(rng, rows, cols, p, n_per_row, dtype, dup=3, ghost_rows=True):
    """local-id COO over owned rows (plus one entry per ghost row), with duplicates."""
    r, c = rows.partition.local(p), cols.partition.local(p)
    I, J = [], []
    for li in range(1, r.num_lids + 1):
        k = n_per_row if r.lid_to_part[li - 1] == p else int(ghost_rows)
        js = rng.integers(1, c.num_lids + 1, size=k)
        I += [li] * k
        J += list(js)
    I, J = np.array(I), np.array(J)
    d = rng.integers(0, len(I), size=len(I) // dup)  # duplicates of existing entries
    I, J = np.concatenate([I, I[d]]), np.concatenate([J, J[d]])
    o = rng.permutation(len(I))
    I, J = I[o], J[o]
    V = rng.uniform(-1, 1, len(I))
    if np.dtype(dtype).kind == "c":
        V = V + 1j * rng.uniform(-1, 1, len(I))
    return I, J, V.astype(dtype)


def _csc_equal(O, got_colptr, got_rowval, got_nzval, ref):
    """device CSC pattern/values == the oracle's sparse(I, J, V) (SparseUtils.jl:80-94)"""
    if not (np.array_equal(got_colptr, ref.colptr) and np.array_equal(got_rowval, ref.rowval)):
        return False
    if isinstance(ref.nzval, O.Cx):
        return np.array_equal(got_nzval.real, ref.nzval.re) and np.array_equal(got_nzval.imag, ref.nzval.im)
    return np.array_equal(got_nzval, ref.nzval)


def _oracle_coo(O, I, J, V):
    if np.iscomplexobj(V):
        return I.copy(), J.copy(), O.Cx(V.real.copy(), V.imag.copy())
    return I.copy(), J.copy(), V.copy()


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128, np.complex64])
@pytest.mark.parametrize("shape,N", [((2, 2, 1), (12, 10, 9)), ((1, 1, 1), (9, 8, 7))])
def test_device_sparse_equals_oracle(be, pamd, O, shape, N, dtype):
    """pa_mat_from_coo (rocPRIM sorts, duplicates summed in input order) ==
    the oracle's sparse_csc: the CSC pattern and nonzeros(A) bit for bit; the
    host compresscoo → pa_mat_from_csc path builds the same device layout."""
    parts = be.get_part_ids(shape)
    _, part = pamd.drivers.stencil_partition(parts, N, 27)
    rows = cols = part  # ghost lids as rows too: stored ghost rows (FE assembly)
    rng = np.random.default_rng(5)
    for p in parts.part_ids:
        I, J, V = _random_coo(rng, rows, cols, p, 9, dtype)
        r, s = rows.partition.local(p), cols.partition.local(p)
        ctx = be.context(p)
        ri, ci = pamd.device_index(ctx, r), pamd.device_index(ctx, s)
        M, colptr, rowval = pamd.DeviceMatrix.from_coo(ctx, I, J, V, ri, ci, r.num_lids, s.num_lids)
        ref = O.sparse_csc(*_oracle_coo(O, I, J, V), r.num_lids, s.num_lids)
        assert _csc_equal(O, colptr, rowval, M.get_values(), ref)
        H = pamd.compresscoo(I, J, V, r.num_lids, s.num_lids)
        M2 = pamd.DeviceMatrix.from_csc(ctx, H, ri, ci, r.num_lids, s.num_lids)
        assert M.info() == M2.info()
        assert np.array_equal(M2.get_values(), M.get_values())


@pytest.mark.parametrize("dtype", [np.float64, np.complex128])
def test_device_sparse_spmv(be, pamd, O, dtype):
    """PSparseMatrix.from_coo (device sparse) then mul! equals the oracle's
    psparse_from_coo + mul! bit for bit (4 parts, halo included)."""
    parts = be.get_part_ids((2, 2, 1))
    N = (11, 9, 8)
    _, part = pamd.drivers.stencil_partition(parts, N, 27)
    OA = O.stencil_problem(O.get_part_ids((2, 2, 1)), N, 27)
    opart = OA.cols  # the same lids, ghosts and Exchanger as `part`
    rng = np.random.default_rng(17)
    # no ghost-row entries: a random ghost layer is not a consistent pattern for matrix_exchanger
    coo = {p: _random_coo(rng, part, part, p, 7, dtype, ghost_rows=False) for p in parts.part_ids}
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [coo[p][k] for p in parts.part_ids], parts.shape)
    A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), part, part, ids="local")
    oc = {p: _oracle_coo(O, *coo[p]) for p in parts.part_ids}
    omk = lambda k: O.PData([oc[p][k] for p in parts.part_ids], (2, 2, 1))
    OM = O.psparse_from_coo(omk(0), omk(1), omk(2), opart, opart, ids="local")
    xs = {p: _rand_vec(rng, part.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], part.partition), part)
    y = pamd.PVector.undef(part, dtype)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: _oracle_vec(O, xs[s.part]), opart.partition), opart)
    oy = O.pvector_undef(opart, dtype)
    O.mul_(oy, OM, ox)
    got = y.to_host()
    for p in parts.part_ids:
        own = part.partition.local(p).oid_to_lid - 1
        ref = oy.values[p]
        g = got.local(p)[own]
        if isinstance(ref, O.Cx):
            assert np.array_equal(g.real, ref.re[own]) and np.array_equal(g.imag, ref.im[own])
        else:
            assert np.array_equal(g, ref[own])


def _rand_vec(rng, n, dtype):
    v = rng.uniform(-1, 1, n)
    if np.dtype(dtype).kind == "c":
        v = v + 1j * rng.uniform(-1, 1, n)
    return v.astype(dtype)


def _oracle_vec(O, a):
    return O.Cx(a.real.copy(), a.imag.copy()) if np.iscomplexobj(a) else a.copy()


def test_device_sparse_int32_and_bounds(be, pamd):
    """index_bytes = 4 (Int32 I, J) gives the same matrix; an out-of-range
    index raises (BoundsError), an empty COO builds an all-zero matrix."""
    L = pamd._lib
    parts = be.get_part_ids((1, 1, 1))
    _, part = pamd.drivers.stencil_partition(parts, (6, 5, 4), 7)
    s = part.partition.local(1)
    ctx = be.context(1)
    idx = pamd.device_index(ctx, s)
    rng = np.random.default_rng(3)
    I = rng.integers(1, s.num_lids + 1, 200)
    J = rng.integers(1, s.num_lids + 1, 200)
    V = rng.uniform(-1, 1, 200)
    # from_coo sends local ids as Int32 (index_bytes 4); the Int64 call must agree
    M4, cp4, rv4 = pamd.DeviceMatrix.from_coo(ctx, I, J, V, idx, idx, s.num_lids, s.num_lids)
    I8, J8 = I.astype(np.int64), J.astype(np.int64)
    colptr = np.empty(s.num_lids + 1, np.int64)
    rowval = np.empty(200, np.int64)
    nnz = C.c_int64()
    h = C.c_void_p()
    L.call("pa_mat_from_coo", ctx.h, L.PA_F64, 8, 0, s.num_lids, s.num_lids, 200, I8.ctypes.data_as(C.c_void_p),
           J8.ctypes.data_as(C.c_void_p), V.ctypes.data_as(C.c_void_p), idx.h, idx.h, C.byref(nnz),
           colptr.ctypes.data_as(C.POINTER(C.c_int64)), rowval.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(h))
    M8 = pamd.DeviceMatrix(h, ctx, np.float64)
    M8.csc_nnz = nnz.value
    assert np.array_equal(colptr, cp4) and np.array_equal(rowval[:nnz.value], rv4)
    assert np.array_equal(M4.get_values(), M8.get_values())
    # a lid beyond Int32 in an Int64 array still fails as BoundsError (no wrap-around)
    Iw = I.copy()
    Iw[3] = 2 ** 32 + 1
    with pytest.raises(L.PAError, match="BoundsError"):
        pamd.DeviceMatrix.from_coo(ctx, Iw, J, V, idx, idx, s.num_lids, s.num_lids)
    Ib = I.copy()
    Ib[7] = s.num_lids + 1
    with pytest.raises(L.PAError, match="BoundsError"):
        pamd.DeviceMatrix.from_coo(ctx, Ib, J, V, idx, idx, s.num_lids, s.num_lids)
    M0, cp0, rv0 = pamd.DeviceMatrix.from_coo(ctx, I[:0], J[:0], V[:0], idx, idx, s.num_lids, s.num_lids)
    assert len(rv0) == 0 and np.all(cp0 == 1)
    x = pamd.PVector.from_host(pamd.map_parts(lambda t: np.ones(t.num_lids), part.partition), part)
    A0 = pamd.PSparseMatrix(pamd.PData(parts.backend, [1], [M0], parts.shape), part, part)
    y = pamd.PVector.undef(part)
    y.fill_(5.0)
    pamd.mul_(y, A0, x)
    assert np.all(y.to_host().local(1)[s.oid_to_lid - 1] == 0.0)


@pytest.mark.parametrize("N,nparts", [((24, 22, 20), 8), ((13, 11, 9), 3)])
def test_device_add_gids_and_to_lids(be, pamd, O, N, nparts):
    """add_gids!(rows, J) with the first-touch discovery on the device
    (pa_add_gids) gives the oracle's ghost layer (gids, owners, order) and
    Exchanger (irregular_problem: add_gids!, Exchanger(ids),
    Interfaces.jl:579-627, 723-786); PSparseMatrix(...; ids=:global) with
    to_lids! on the device holds the oracle's nonzeros(A) in CSC order."""
    drv = pamd.drivers
    owners = drv.voronoi_owners(N, nparts)
    parts = be.get_part_ids(nparts)
    rows, cols, I, J, V = drv.irregular_partition(parts, N, 27, owners)
    OA = O.irregular_problem(O.get_part_ids(nparts), N, 27, np.float64, owners)
    for i, p in enumerate(parts.part_ids):
        a, b = cols.partition.local(p), OA.cols.partition.parts[i]
        assert np.array_equal(a.lid_to_gid, np.asarray(b.lid_to_gid))
        assert np.array_equal(a.lid_to_part, np.asarray(b.lid_to_part))
        assert np.array_equal(a.hid_to_lid, np.asarray(b.hid_to_lid))
        for t in ("lids_rcv", "lids_snd"):
            ta, tb = getattr(cols.exchanger, t).local(p), getattr(OA.cols.exchanger, t).parts[i]
            assert np.array_equal(ta.data, np.asarray(tb.data)) and np.array_equal(ta.ptrs, np.asarray(tb.ptrs))
        assert list(cols.exchanger.parts_rcv.local(p)) == list(OA.cols.exchanger.parts_rcv.parts[i])
        assert list(cols.exchanger.parts_snd.local(p)) == list(OA.cols.exchanger.parts_snd.parts[i])
    A = pamd.PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global")
    for i, p in enumerate(parts.part_ids):
        assert np.array_equal(A.values.local(p).get_values(), OA.values.parts[i].nzval)


def test_device_index_to_lids(be, pamd):
    """pa_index_to_lids (to_lids!, the Exchanger's lids_snd) equals the host
    IndexSet lookup on owned and ghost gids, and an absent gid is a KeyError."""
    parts = be.get_part_ids(3)
    rows, cols, _, _, _ = pamd.drivers.irregular_partition(parts, (9, 8, 7), 27)
    rng = np.random.default_rng(3)
    for p in parts.part_ids:
        s = cols.partition.local(p)
        g = rng.choice(s.lid_to_gid, size=min(500, s.num_lids))
        got = pamd.device.device_to_lids(be.context(p), s, g)
        assert np.array_equal(got, s.to_lids(g))
        missing = np.setdiff1d(np.arange(1, rows.ngids + 1), s.lid_to_gid)
        if len(missing):
            with pytest.raises(pamd.PAError, match="KeyError"):
                pamd.device.device_to_lids(be.context(p), s, np.append(g, missing[:1]))


def test_device_to_lids_unknown_gid(be, pamd):
    parts = be.get_part_ids(1)
    rows = pamd.prange_linear(parts, 10)
    s = rows.partition.local(1)
    ctx = be.context(1)
    I = np.array([1, 2, 11])
    with pytest.raises(pamd.PAError, match="KeyError"):
        pamd.DeviceMatrix.from_coo(ctx, I, I, np.ones(3), pamd.device.device_index_gids(ctx, s),
                                   pamd.device.device_index_gids(ctx, s), 10, 10, ids_global=True)


def _long_row_coo(rng, part, p, dtype, long_lens):
    """owned rows with ~9 entries, a few rows with long_lens entries (over all
    local columns, ghosts included), in random order with duplicates."""
    s = part.partition.local(p)
    own = s.oid_to_lid
    I, J = [], []
    longs = rng.choice(own, size=min(len(long_lens), len(own)), replace=False)
    for li in own:
        k = 9
        if li in longs:
            k = long_lens[list(longs).index(li)]
        I += [li] * k
        J += list(rng.integers(1, s.num_lids + 1, size=k))
    I, J = np.array(I), np.array(J)
    o = rng.permutation(len(I))
    V = rng.uniform(-1, 1, len(I))
    if np.dtype(dtype).kind == "c":
        V = V + 1j * rng.uniform(-1, 1, len(I))
    return I[o], J[o], V[o].astype(dtype), sorted(int(v) for v in longs)


def _ref_spmv(H, s, xl, yl, alpha, beta, dtype):
    """SparseUtils.jl:157-187 on the host CSC: rmul!(c, β) (or fill!(c, 0)),
    then the column loop over owned columns (oid order), then ghost columns."""
    want = (yl * dtype(beta)) if beta != 0 else np.zeros_like(yl)
    if beta == 1:
        want = yl.copy()
    l2o = np.zeros(s.num_lids, dtype=bool)
    l2o[s.oid_to_lid - 1] = True
    for j in list(s.oid_to_lid - 1) + list(s.hid_to_lid - 1):
        axj = xl[j] * dtype(alpha) if alpha != 1 else xl[j]
        for q in range(H.colptr[j] - 1, H.colptr[j + 1] - 1):
            i = H.rowval[q] - 1
            if l2o[i]:
                want[i] = want[i] + H.nzval[q] * axj
    return want


@pytest.mark.parametrize("dtype", [np.float64, np.complex128, np.float32])
@pytest.mark.parametrize("build", ["coo", "csc"])
def test_long_rows_bitexact(be, pamd, dtype, build):
    """Rows far longer than the rest (row-length histogram) run in the
    long-row kernel: mul! with α/β, both column encodings, the halo, and
    set_values all stay bit-exact against the reference's loop."""
    parts = be.get_part_ids((2, 2, 1))
    _, part = pamd.drivers.stencil_partition(parts, (20, 18, 16), 27)
    rng = np.random.default_rng(23)
    coo = {p: _long_row_coo(rng, part, p, dtype, [600, 1000, 4000, 70]) for p in parts.part_ids}
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [coo[p][k] for p in parts.part_ids], parts.shape)
    if build == "coo":
        A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), part, part, ids="local")
    else:
        csc = pamd.map_parts(lambda i, j, v, s: pamd.compresscoo(i, j, v, s.num_lids, s.num_lids),
                             mk(0), mk(1), mk(2), part.partition)
        A = pamd.PSparseMatrix.from_csc(csc, part, part)
    for p in parts.part_ids:
        assert A.values.local(p).info()["long_rows"] == 3  # 600, 1000, 4000 (less duplicates) > max(256, 8*p90)
    xs = {p: (rng.uniform(-1, 1, part.partition.local(p).num_lids) + (1j * rng.uniform(-1, 1, part.partition.local(p).num_lids) if np.dtype(dtype).kind == "c" else 0)).astype(dtype) for p in parts.part_ids}
    ys = {p: rng.uniform(-1, 1, part.partition.local(p).num_lids).astype(dtype) for p in parts.part_ids}
    Hs = {p: pamd.compresscoo(*coo[p][:3], part.partition.local(p).num_lids, part.partition.local(p).num_lids)
          for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], part.partition), part)
    for fmt in (1, 0):
        prev = pamd._lib.tune("spmv_format", fmt)
        try:
            for alpha, beta in ((1.0, 0.0), (2.5, 0.5), (1.0, 1.0)):
                y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], part.partition), part)
                pamd.mul_(y, A, x, alpha, beta)
                xh = x.to_host()
                for p in parts.part_ids:
                    s = part.partition.local(p)
                    want = _ref_spmv(Hs[p], s, xh.local(p), ys[p], alpha, beta, np.dtype(dtype).type)
                    own = s.oid_to_lid - 1
                    assert np.array_equal(y.to_host().local(p)[own], want[own]), (fmt, alpha, beta, p)
        finally:
            pamd._lib.tune("spmv_format", prev)
    # new values into the same pattern (long-row values included)
    for p in parts.part_ids:
        M = A.values.local(p)
        v2 = (M.get_values() * dtype(0.5)).astype(dtype)
        M.set_values(v2)
        assert np.array_equal(M.get_values(), v2)
        Hs[p].nzval = v2
    y = pamd.PVector.undef(part, dtype)
    pamd.mul_(y, A, x)
    for p in parts.part_ids:
        s = part.partition.local(p)
        want = _ref_spmv(Hs[p], s, x.to_host().local(p), np.zeros(s.num_lids, dtype), 1.0, 0.0, np.dtype(dtype).type)
        own = s.oid_to_lid - 1
        assert np.array_equal(y.to_host().local(p)[own], want[own])


def test_long_rows_fast_mode_and_fused_dot(be, pamd):
    """long_rows_exact = 0 (lane-strided tree) stays within 1e-12 of the
    exact order; the fused SpMV+dot includes the long rows."""
    parts = be.get_part_ids((2, 1, 1))
    _, part = pamd.drivers.stencil_partition(parts, (20, 18, 16), 27)
    rng = np.random.default_rng(5)
    coo = {p: _long_row_coo(rng, part, p, np.float64, [5000, 2000]) for p in parts.part_ids}
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [coo[p][k] for p in parts.part_ids], parts.shape)
    A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), part, part, ids="local")
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), part.partition), part)
    y1, y2, y3 = (pamd.PVector.undef(part) for _ in range(3))
    pamd.mul_(y1, A, x)
    prev = pamd._lib.tune("long_rows_exact", 0)
    try:
        pamd.mul_(y2, A, x)
    finally:
        pamd._lib.tune("long_rows_exact", prev)
    for p in parts.part_ids:
        a, b = y1.to_host().local(p), y2.to_host().local(p)
        assert np.allclose(a, b, rtol=1e-12, atol=1e-12 * np.abs(a).max())
    d = pamd.mul_dot_(y3, A, x)
    assert abs(d - pamd.dot(x, y1)) <= 1e-12 * abs(d)
