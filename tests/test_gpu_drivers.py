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
