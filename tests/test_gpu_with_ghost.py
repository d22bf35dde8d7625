"""PRange(parts, ngids, with_ghost[, isperiodic]) on the device
(Interfaces.jl:1166-1223): owned and ghost lids interleave, so the index
sets carry oid/hid tables (no contiguous fast path, no pattern slices) and
the SpMV writes y through its oid → lid map.  A 7-point operator with
random coefficients assembled over each part's owned rows (neighbours wrap
around periodic dimensions), mul!, exchange! and assemble! bit-exact against
the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250114


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


def _coo(rows, parts, ngids, periodic, rng):
    D = len(ngids)
    per = periodic or (False,) * D
    I, J, V = {}, {}, {}
    for p in parts.part_ids:
        s = rows.partition.local(p)
        own = s.lid_to_gid[s.oid_to_lid - 1]
        ci = [(own - 1) // int(np.prod(ngids[:d])) % ngids[d] for d in range(D)]
        ii, jj = [own], [own]
        for d in range(D):
            for step in (-1, 1):
                c = ci[d] + step
                ok = np.ones(len(own), bool) if per[d] else (c >= 0) & (c < ngids[d])
                c = c % ngids[d]
                nb = own + (c - ci[d]) * int(np.prod(ngids[:d]))
                ii.append(own[ok])
                jj.append(nb[ok])
        I[p] = np.concatenate(ii)
        J[p] = np.concatenate(jj)
        V[p] = rng.uniform(-1, 1, len(I[p]))
    return I, J, V


@pytest.mark.parametrize("shape,ngids,periodic", [((2, 2, 2), (12, 10, 9), None), ((2, 2, 1), (16, 14, 6), (True, False, True)),
                                                   ((3, 2, 2), (13, 9, 10), (True, True, True))])
def test_with_ghost_spmv_exchange_assemble(be, pamd, O, shape, ngids, periodic):
    parts = be.get_part_ids(shape)
    oparts = O.get_part_ids(shape)
    rows = pamd.prange_cartesian(parts, ngids, with_ghost=True, isperiodic=periodic)
    orows = O.prange_cartesian(oparts, ngids, with_ghost=True, isperiodic=periodic)
    rng = np.random.default_rng(SEED)
    I, J, V = _coo(rows, parts, ngids, periodic, rng)
    mk = lambda d: pamd.PData(parts.backend, parts.part_ids, [d[p] for p in parts.part_ids], parts.shape)
    A = pamd.PSparseMatrix.from_coo(mk(I), mk(J), mk(V), rows, rows, ids="global")
    omk = lambda d, f: O.PData([f(d[p]) for p in parts.part_ids], oparts.shape)
    OA = O.psparse_from_coo(omk(I, lambda a: [int(v) for v in a]), omk(J, lambda a: [int(v) for v in a]),
                            omk(V, lambda a: a.copy()), orows, orows, ids="global")
    assert not all(np.array_equal(rows.partition.local(p).oid_to_lid, np.arange(1, rows.partition.local(p).num_oids + 1))
                   for p in parts.part_ids)  # interleaved lids
    xs = {p: rng.uniform(-1, 1, rows.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], rows.partition), rows)
    y = pamd.PVector.from_host(pamd.map_parts(lambda s: np.full(s.num_lids, 7.0), rows.partition), rows)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), orows.partition), orows)
    oy = O.PVector(O.map_parts(lambda s: np.full(s.num_lids, 7.0), orows.partition), orows)
    O.mul_(oy, OA, ox)
    got, gx = y.to_host(), x.to_host()
    for p in parts.part_ids:
        s = rows.partition.local(p)
        own = s.oid_to_lid - 1
        assert np.array_equal(got.local(p)[own], oy.values[p][own]), f"part {p}: SpMV differs"
        hid = s.hid_to_lid - 1
        assert np.array_equal(got.local(p)[hid], np.full(len(hid), 7.0)), f"part {p}: mul! wrote a ghost of y"
        assert np.array_equal(gx.local(p), ox.values[p]), f"part {p}: exchanged ghosts of x differ"
    ws = {p: rng.uniform(-1, 1, rows.partition.local(p).num_lids) for p in parts.part_ids}
    w = pamd.PVector.from_host(pamd.map_parts(lambda s: ws[s.part], rows.partition), rows)
    ow = O.PVector(O.map_parts(lambda s: ws[s.part].copy(), orows.partition), orows)
    pamd.assemble_(w)
    O.assemble_(ow)
    for p in parts.part_ids:
        assert np.array_equal(w.to_host().local(p), ow.values[p]), f"part {p}: assemble! differs"
