"""Edge cases of the device path against the oracle: parts that own no ids
(PRange(parts, n) with n < nparts, test_interfaces.jl's linear PRange rule),
parts without neighbours, an empty COO, and the CG on such partitions."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


def _tridiag(n, part_rows):
    """global-id COO of the owned rows of a 1-D Laplacian-like matrix."""
    I, J, V = [], [], []
    for g in part_rows:
        for d, v in ((-1, -1.0), (0, 4.0), (1, -1.5)):
            if 1 <= g + d <= n:
                I.append(g)
                J.append(g + d)
                V.append(v + 0.01 * g)
    return np.array(I, np.int64), np.array(J, np.int64), np.array(V)


def _build(pamd, O, parts, n, nparts):
    rows = pamd.prange_linear(parts, n)
    coo = {p: _tridiag(n, rows.partition.local(p).lid_to_gid[rows.partition.local(p).oid_to_lid - 1])
           for p in parts.part_ids}
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [coo[p][k] for p in parts.part_ids], parts.shape)
    cols = pamd.add_gids(rows, mk(1))
    A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), rows, cols, ids="global")
    oparts = O.get_part_ids(nparts)
    orows = O.prange_linear(oparts, n)
    oI = O.PData([list(coo[p][0]) for p in parts.part_ids])
    oJ = O.PData([list(coo[p][1]) for p in parts.part_ids])
    oV = O.PData([coo[p][2].copy() for p in parts.part_ids])
    ocols = O.add_gids(orows, oJ)
    OA = O.psparse_from_coo(oI, oJ, oV, orows, ocols, ids="global")
    return A, OA


@pytest.mark.parametrize("n,nparts", [(3, 4), (2, 4), (5, 8), (1, 3)])
def test_empty_parts_spmv_exchange_reductions(be, pamd, O, n, nparts):
    parts = be.get_part_ids(nparts)
    A, OA = _build(pamd, O, parts, n, nparts)
    assert any(s.num_oids == 0 for s in A.rows.partition.parts)  # at least one empty part
    rng = np.random.default_rng(2)
    xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        s = A.rows.partition.local(p)
        own = s.oid_to_lid - 1
        assert np.array_equal(y.to_host().local(p)[own], oy.values[p][own])
        assert np.array_equal(x.to_host().local(p), ox.values[p])  # ghosts after the halo
    # exchange! / assemble! on the column partition
    v = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    ov = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    pamd.assemble_(v)
    O.assemble_(ov)
    for p in parts.part_ids:
        assert np.array_equal(v.to_host().local(p), ov.values[p])
    assert abs(pamd.dot(x, x) - O.dot(ox, ox)) <= 1e-12 * abs(O.dot(ox, ox))
    assert abs(pamd.norm(y) - O.norm(oy)) <= 1e-12 * max(1e-300, O.norm(oy))


@pytest.mark.parametrize("device", [False, True])
def test_empty_parts_cg(be, pamd, O, device):
    """CG on a partition with empty parts: host-driven == device-driven, and
    the residual history follows the oracle's."""
    n, nparts = 6, 8
    parts = be.get_part_ids(nparts)
    A, OA = _build(pamd, O, parts, n, nparts)
    bh = {p: np.ones(A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    b = pamd.PVector.from_host(pamd.map_parts(lambda s: bh[s.part], A.cols.partition), A.cols)
    x = pamd.PVector.undef(A.cols).fill_(0)
    hist = []
    pamd.cg_(x, A, b, history=hist, device=device, batch=2)
    ob = O.PVector(O.map_parts(lambda s: bh[s.part].copy(), OA.cols.partition), OA.cols)
    ox = O.pvector_undef(OA.cols)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist) > 0
    np.testing.assert_allclose(hist, ohist, rtol=1e-8, atol=1e-14)


def test_single_part_no_halo_and_empty_matrix(be, pamd):
    """One part (no exchanger traffic) and a matrix with no stored entries:
    mul! writes β*y = 0 on owned values, ghost values untouched."""
    parts = be.get_part_ids(1)
    rows = pamd.prange_linear(parts, 10)
    e = pamd.PData(parts.backend, [1], [np.zeros(0, np.int64)], parts.shape)
    A = pamd.PSparseMatrix.from_coo(e, e, pamd.PData(parts.backend, [1], [np.zeros(0)], parts.shape),
                                    rows, rows, ids="global")
    x = pamd.PVector.full(1.0, rows)
    y = pamd.PVector.full(7.0, rows)
    pamd.mul_(y, A, x)
    assert np.all(y.to_host().local(1) == 0.0)
    pamd.mul_(y, A, x, 2.0, 1.0)
    assert np.all(y.to_host().local(1) == 0.0)


def test_hbm_probe_rates_and_arguments(be, pamd):
    """pa_hbm_probe (bench.py's HBM calibration): plausible read/copy rates on
    a 256 MiB buffer, and its argument check fails loudly."""
    r, c = pamd._lib.hbm_probe(0, 256 << 20, 3)
    assert 500.0 < r < 20000.0 and 500.0 < c < 20000.0
    with pytest.raises(pamd._lib.PAError, match="pa_hbm_probe"):
        pamd._lib.hbm_probe(0, 1024, 1)


def test_mul_with_equal_copies_of_the_ranges(be, pamd, O):
    """mul!(c, a, b) with c.rows / b.rows equal copies (not the same objects)
    of a.rows / a.cols (Interfaces.jl:2253-2255 @checks pass on equal ids):
    the result equals the oracle's, and the checks are answered from the
    per-pair cache after the first call (no per-call O(n) host compare)."""
    import time
    shape, N = (2, 2, 1), (12, 10, 9)
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    rows2, cols2 = A.rows.copy(), A.cols.copy()
    rng = np.random.default_rng(12)
    xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], cols2.partition), cols2)
    y = pamd.PVector.undef(rows2)
    pamd.mul_(y, A, x)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        own = A.rows.partition.local(p).oid_to_lid - 1
        assert np.array_equal(y.to_host().local(p)[own], oy.values[p][own])
    assert "_eq_cache" in A.cols.__dict__ and any(k[0] == "layout" for k in A.cols._eq_cache)


def test_spmv_rejects_partial_exchanger_arrays(be, pamd):
    """pa_spmv_all with an exchanger array whose entries are partly null is
    an error ('exchanger missing'), not a host crash."""
    import ctypes as C
    parts = be.get_part_ids((2, 1, 1))
    A = pamd.drivers.stencil_operator(parts, (8, 6, 5), 7)
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.ones(s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    args = list(pamd.pvector._spmv_args(y, A, x, 1.0, 0.0))
    xg = [pamd.device.device_exchanger(be.context(p), A.cols.exchanger, p) for p in parts.part_ids]
    args[6] = pamd._lib.ptr_array([xg[0].h, None])
    with pytest.raises(pamd._lib.PAError, match="exchanger missing"):
        pamd._lib.call("pa_spmv_all", *args)


def test_rccl_backend_leaves_global_transport_knob(pamd):
    """HIPBackend(rccl=True) marks its own contexts (pa_comm_init_all) instead
    of switching the process-wide halo_transport knob: a backend
    made afterwards without RCCL keeps the device-read transport."""
    before = pamd._lib.tune("halo_transport", 0)
    pamd._lib.tune("halo_transport", before)
    pamd.HIPBackend(devices=[0], rccl=True).get_part_ids((2, 1, 1))
    after = pamd._lib.tune("halo_transport", before)
    assert after == before


def test_mul_argument_cache_follows_objects(be, pamd, O):
    """mul_'s cached C-ABI arguments (per c, b, α, β on the matrix): repeated
    calls, a new α, and a new y allocated after the old one died (possibly
    at the same address) all give the oracle's values."""
    import gc
    nparts, n = 4, 37
    parts = be.get_part_ids(nparts)
    A, OA = _build(pamd, O, parts, n, nparts)
    rng = np.random.default_rng(5)
    xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)

    def check(y, alpha):
        oy = O.pvector_undef(OA.rows)
        O.mul_(oy, OA, ox, alpha, 0.0)
        got = y.to_host()
        for p in parts.part_ids:
            own = A.rows.partition.local(p).oid_to_lid - 1
            assert np.array_equal(got.local(p)[own], oy.values[p][own])

    for alpha in (1.0, 1.0, 0.5, 1.0):
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, x, alpha, 0.0)
        pamd.mul_(y, A, x, alpha, 0.0)
        check(y, alpha)
        del y
        gc.collect()
    assert len(A.__dict__["_args_cache"]) <= 8


def test_context_knobs_override_process_defaults(pamd):
    """pa_ctx_tune: a context's knob applies to the calls its parts lead and
    to nothing else; None (PA_TUNE_DROP) drops it.  spmv_format 0 on one backend's contexts
    shows in its matrix's streamed bytes (int32 ids), not in another
    backend's, and the products stay bit-identical."""
    mk = lambda be: (be, be.get_part_ids((2, 1, 1)))
    (b1, p1), (b2, p2) = mk(pamd.HIPBackend(devices=[0])), mk(pamd.HIPBackend(devices=[0]))
    N = (16, 12, 10)
    A1 = pamd.drivers.stencil_operator(p1, N, 27)
    A2 = pamd.drivers.stencil_operator(p2, N, 27)
    t1 = A1.values.local(1).traffic()["index_bytes"]
    for p in p1.part_ids:
        assert b1.context(p).tune("spmv_format", 0) is None
    assert A1.values.local(1).traffic()["index_bytes"] > t1, "override not applied to the context's calls"
    assert A2.values.local(1).traffic()["index_bytes"] == t1, "override leaked to another context"
    xs = {p: np.random.default_rng(p).uniform(-1, 1, A1.cols.partition.local(p).num_lids) for p in p1.part_ids}
    x1 = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A1.cols.partition), A1.cols)
    x2 = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A2.cols.partition), A2.cols)
    y1, y2 = pamd.PVector.undef(A1.rows), pamd.PVector.undef(A2.rows)
    pamd.mul_(y1, A1, x1)
    pamd.mul_(y2, A2, x2)
    h1, h2 = y1.to_host(), y2.to_host()
    for p in p1.part_ids:
        assert np.array_equal(h1.local(p), h2.local(p))
    for p in p1.part_ids:
        assert b1.context(p).tune("spmv_format", None) == 0
    assert A1.values.local(1).traffic()["index_bytes"] == t1
    # -1 is a value (spmv_xcd_chunk's auto), not a drop: a
    # context can override a fixed process default back to auto
    prev = pamd._lib.tune("spmv_xcd_chunk", 4)
    try:
        assert b1.context(1).tune("spmv_xcd_chunk", -1) is None
        assert b1.context(1).tune("spmv_xcd_chunk", None) == -1
        assert b1.context(1).tune("spmv_xcd_chunk", None) is None
    finally:
        pamd._lib.tune("spmv_xcd_chunk", prev)
    with pytest.raises(pamd._lib.PAError):
        b1.context(1).tune("spmv_format", 5)
    with pytest.raises(pamd._lib.PAError):
        b1.context(1).tune("no_such_knob", 0)
