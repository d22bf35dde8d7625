"""assemble!(I, J, V, rows) on the device (Interfaces.jl:2406-2492,
pa_coo_assemble_all): triplets of rows owned by another part go to that
owner (segments in rows.exchanger.parts_rcv order, input order inside), the
sender keeps the entry with value zero(v), the owner appends what it
receives in parts_snd order.  Compared bit for bit against the oracle's
literal restatement (oracle/pa_oracle.py assemble_coo_) on random COO lists
with ghost rows, linear and Cartesian parts, four element types."""
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


def _problem(pamd, O, be, nparts, ngids, m, dtype, seed, remote_frac=0.25, nan=False, empty_part=None):
    """rows (product and oracle, ghost layer from add_gids!(rows, I)) and a
    random COO per part: rows mostly owned, remote_frac of them owned by any
    other part, columns anywhere."""
    parts = be.get_part_ids(nparts)
    oparts = O.get_part_ids(nparts)
    if isinstance(ngids, tuple):
        rows, orows = pamd.prange_cartesian(parts, ngids), O.prange_cartesian(oparts, ngids)
        ntot = int(np.prod(ngids))
    else:
        rows, orows = pamd.prange_linear(parts, ngids), O.prange_linear(oparts, ngids)
        ntot = ngids
    rng = np.random.default_rng(seed)
    I, J, V = {}, {}, {}
    for p in parts.part_ids:
        s = rows.partition.local(p)
        own = s.lid_to_gid[s.oid_to_lid - 1]
        k = 0 if p == empty_part else m
        nrem = int(k * remote_frac)
        i = np.concatenate([rng.choice(own, k - nrem), rng.integers(1, ntot + 1, nrem)])
        rng.shuffle(i)
        I[p] = i.astype(np.int64)
        J[p] = rng.integers(1, ntot + 1, k).astype(np.int64)
        V[p] = _rand(rng, k, dtype)
        if nan and k:
            V[p][rng.integers(0, k, 8)] = np.nan
            V[p][rng.integers(0, k, 4)] = np.inf
    mk = lambda d: pamd.PData(parts.backend, parts.part_ids, [d[p].copy() for p in parts.part_ids], parts.shape)
    pamd.add_gids_(rows, mk(I))
    O.add_gids_(orows, O.PData([list(map(int, I[p])) for p in parts.part_ids], oparts.shape))
    return parts, oparts, rows, orows, I, J, V, mk


def _check(pamd, O, parts, oparts, rows, orows, I, J, V, mk):
    coo = pamd.COO.from_host(mk(I), mk(J), mk(V), rows)
    pamd.assemble_(coo, rows)
    gI, gJ, gV = coo.to_host()
    oI = O.PData([list(map(int, I[p])) for p in parts.part_ids], oparts.shape)
    oJ = O.PData([list(map(int, J[p])) for p in parts.part_ids], oparts.shape)
    oV = O.PData([V[p].copy() for p in parts.part_ids], oparts.shape)
    rI, rJ, rV = O.assemble_coo_(oI, oJ, oV, orows)
    moved = 0
    for p in parts.part_ids:
        assert gI.local(p).tolist() == list(rI[p]), f"part {p}: I differs"
        assert gJ.local(p).tolist() == list(rJ[p]), f"part {p}: J differs"
        ref = np.asarray(rV[p], dtype=gV.local(p).dtype)
        assert gV.local(p).tobytes() == ref.tobytes(), f"part {p}: V differs"
        moved += len(gI.local(p)) - len(I[p])
    return moved


@pytest.mark.parametrize("nparts,ngids,dtype", [
    (4, 20000, np.float64), (4, 20000, np.complex128), ((2, 2), (150, 140), np.float64),
    ((2, 2), (150, 140), np.float32), (6, 9000, np.complex64), ((2, 2, 2), (30, 28, 26), np.float64)])
def test_coo_assemble_bitexact(be, pamd, O, nparts, ngids, dtype):
    parts, oparts, rows, orows, I, J, V, mk = _problem(pamd, O, be, nparts, ngids, 12000, dtype, SEED)
    moved = _check(pamd, O, parts, oparts, rows, orows, I, J, V, mk)
    assert moved > 0


def test_coo_assemble_nan_inf_and_empty_part(be, pamd, O):
    """a sent NaN/Inf leaves a +0 behind (k_v[k] = zero(v), Interfaces.jl:2446)
    and arrives unchanged; a part with no triplets still receives."""
    parts, oparts, rows, orows, I, J, V, mk = _problem(pamd, O, be, 4, 8000, 3000, np.float64, SEED + 1,
                                                       nan=True, empty_part=3)
    moved = _check(pamd, O, parts, oparts, rows, orows, I, J, V, mk)
    assert moved > 0


def test_coo_assemble_unknown_row_gid(be, pamd):
    parts = be.get_part_ids(2)
    rows = pamd.prange_linear(parts, 10)
    I = pamd.PData(parts.backend, parts.part_ids, [np.array([1, 2, 7]), np.array([6, 7])], parts.shape)
    pamd.add_gids_(rows, I)
    bad = pamd.PData(parts.backend, parts.part_ids, [np.array([1, 2, 9]), np.array([6, 7])], parts.shape)
    J = pamd.PData(parts.backend, parts.part_ids, [np.array([1, 1, 1]), np.array([1, 1])], parts.shape)
    V = pamd.PData(parts.backend, parts.part_ids, [np.ones(3), np.ones(2)], parts.shape)
    coo = pamd.COO.from_host(bad, J, V, rows)
    with pytest.raises(pamd.PAError, match="KeyError"):
        pamd.assemble_(coo, rows)


def test_coo_assemble_then_sparse_equals_oracle(be, pamd, O):
    """the device-assembled COO → PSparseMatrix(…; ids=:global) → mul! equals
    the oracle's assemble_coo_ → psparse_from_coo → mul! (owned rows)."""
    parts, oparts, rows, orows, I, J, V, mk = _problem(pamd, O, be, (2, 2), (90, 80), 6000, np.float64, SEED + 2)
    coo = pamd.COO.from_host(mk(I), mk(J), mk(V), rows)
    pamd.assemble_(coo, rows)
    n = int(np.prod((90, 80)))
    cols = pamd.prange_cartesian(parts, (90, 80))
    ocols = O.prange_cartesian(oparts, (90, 80))
    pamd.add_gids_(cols, coo.global_cols())
    A = pamd.PSparseMatrix.from_coo(coo, None, None, rows, cols, ids="global")
    oI = O.PData([list(map(int, I[p])) for p in parts.part_ids], oparts.shape)
    oJ = O.PData([list(map(int, J[p])) for p in parts.part_ids], oparts.shape)
    oV = O.PData([V[p].copy() for p in parts.part_ids], oparts.shape)
    rI, rJ, rV = O.assemble_coo_(oI, oJ, oV, orows)
    O.add_gids_(ocols, rJ)
    OA = O.psparse_from_coo(rI, rJ, rV, orows, ocols, ids="global")
    rng = np.random.default_rng(SEED + 3)
    xs = {p: rng.uniform(-1, 1, cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], cols.partition), cols)
    y = pamd.PVector.undef(rows)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows)
    O.mul_(oy, OA, ox)
    got = y.to_host()
    assert n > 0
    for p in parts.part_ids:
        own = rows.partition.local(p).oid_to_lid - 1
        assert np.array_equal(got.local(p)[own], oy.values[p][own]), f"part {p}: mul! differs"


def test_coo_assemble_exchanger_missing_owner(be, pamd, O):
    """A ghost row whose owner the rows exchanger does not list is the
    reference's KeyError (owner_to_i, Interfaces.jl:2428-2430), not a
    triplet silently kept local."""
    parts, oparts, rows, orows, I, J, V, mk = _problem(pamd, O, be, 4, 4000, 2000, np.float64, SEED + 7)
    coo = pamd.COO.from_host(mk(I), mk(J), mk(V), rows)
    ctxs = pamd.device.contexts(rows.partition)
    idx = [pamd.device.device_index_gids(c, rows.partition.local(p)) for c, p in zip(ctxs, parts.part_ids)]
    xg = [pamd.device.device_exchanger(c, rows.exchanger, p) for c, p in zip(ctxs, parts.part_ids)]
    ex = rows.exchanger
    empty = pamd.Table(np.zeros(0, np.int32), np.ones(1, np.int32))
    xg[0] = pamd.device.DeviceExchanger(ctxs[0], [], empty, ex.parts_snd.local(1), ex.lids_snd.local(1))
    with pytest.raises(pamd.PAError, match="parts_rcv"):
        pamd._lib.call("pa_coo_assemble_all", len(ctxs), pamd._lib.ptr_array([c.h for c in coo.values.parts]),
                       pamd._lib.ptr_array([d.h for d in idx]), pamd._lib.ptr_array([d.h for d in xg]))
