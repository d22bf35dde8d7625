"""CPU tests of the product's host layer (backends, PRange, Exchanger, COO
compression, drivers) against the reference's KATs and the oracle."""
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "interfaces_kats.json")))


def _pd(pamd, parts, vals):
    return pamd.PData(parts.backend, parts.part_ids, vals, parts.shape)


def test_sequential_exchange_kat(pamd):
    k = GOLD["exchange_scalar"]
    parts = pamd.sequential.get_part_ids(4)
    prcv = _pd(pamd, parts, k["parts_rcv"])
    psnd = _pd(pamd, parts, k["parts_snd"])
    data = pamd.map_parts(lambda p: [10 * i for i in p], psnd)
    got = pamd.exchange(data, prcv, psnd)
    assert got.parts == k["expected_rcv"]
    assert pamd.preduce(lambda a, b: a + b, parts, 0) == 10
    assert pamd.xscan_all(lambda a, b: a + b, _pd(pamd, parts, [4, 2, 6, 3]), 1).parts[0] == [1, 5, 7, 13]
    got = pamd.discover_parts_snd(prcv)
    assert [list(x) for x in got.parts] == k["parts_snd"]


def test_discover_alltoall_equals_gather(pamd):
    """discover_parts_snd without neighbours: the default P-int all-to-all
    (no part holds the whole graph) equals the reference's gather-based
    fallback (Interfaces.jl:515-552) on the KAT and on random graphs."""
    k = GOLD["exchange_scalar"]
    parts = pamd.sequential.get_part_ids(4)
    prcv = _pd(pamd, parts, k["parts_rcv"])
    assert [list(x) for x in pamd.discover_parts_snd(prcv).parts] == k["parts_snd"]
    assert [list(x) for x in pamd.discover_parts_snd(prcv, method="gather").parts] == k["parts_snd"]
    rng = np.random.default_rng(11)
    for P in (1, 2, 5, 9, 16):
        parts = pamd.sequential.get_part_ids(P)
        graph = [sorted(set(int(q) for q in rng.integers(1, P + 1, rng.integers(0, P + 1))) - {p})
                 for p in range(1, P + 1)]
        prcv = _pd(pamd, parts, graph)
        a = pamd.discover_parts_snd(prcv)
        g = pamd.discover_parts_snd(prcv, method="gather")
        assert [list(x) for x in a.parts] == [list(x) for x in g.parts], P
    with pytest.raises(ValueError):
        pamd.discover_parts_snd(_pd(pamd, pamd.sequential.get_part_ids(2), [[3], []]))


def test_irregular_setup_discovers_without_gather(pamd, O, monkeypatch):
    """BASELINE config 5's Voronoi partition: add_gids! finds parts_snd by
    the all-to-all (no gather on MAIN) and yields the
    oracle's (gather-based) Exchanger."""
    P = pamd.prange
    N, nparts = (14, 12, 10), 6
    parts = pamd.sequential.get_part_ids(nparts)
    ref_cols = pamd.drivers.irregular_partition(parts, N, 27)[1]

    def no_gather(*a, **k):
        raise AssertionError("gather-based discover_parts_snd used")
    monkeypatch.setattr(P, "gather", no_gather)
    rows, cols = pamd.drivers.irregular_partition(parts, N, 27)[:2]
    monkeypatch.undo()
    gex = pamd.exchanger_from_ids(ref_cols.partition, discover="gather")
    for p in parts.part_ids:
        assert list(cols.exchanger.parts_snd.local(p)) == list(gex.parts_snd.local(p))
        assert cols.exchanger.lids_snd.local(p).tolist() == gex.lids_snd.local(p).tolist()
        assert cols.exchanger.lids_rcv.local(p).tolist() == gex.lids_rcv.local(p).tolist()
    OA = O.irregular_problem(O.get_part_ids(nparts), N, 27)
    for p in parts.part_ids:
        assert list(cols.exchanger.parts_snd.local(p)) == list(OA.cols.exchanger.parts_snd[p])
        assert cols.exchanger.lids_snd.local(p).tolist() == OA.cols.exchanger.lids_snd[p].tolist()


def _kat_partition(pamd, parts):
    k = GOLD["exchanger"]
    return _pd(pamd, parts, [pamd.IndexSet(p + 1, k["lid_to_gid"][p], k["lid_to_part"][p]) for p in range(4)])


def test_exchanger_kat(pamd):
    k = GOLD["exchanger"]
    parts = pamd.sequential.get_part_ids(4)
    ex = pamd.exchanger_from_ids(_kat_partition(pamd, parts))
    assert [list(x) for x in ex.parts_snd.parts] == k["expected_parts_snd"]
    assert [t.tolist() for t in ex.lids_snd.parts] == k["expected_lids_snd"]
    # neighbour-assisted discover gives the same plan
    nb = _pd(pamd, parts, [[2, 3, 4], [1, 3, 4], [1, 2, 4], [1, 2, 3]])
    ex2 = pamd.exchanger_from_ids(_kat_partition(pamd, parts), neighbors=nb)
    assert [t.tolist() for t in ex2.lids_snd.parts] == k["expected_lids_snd"]


def test_exchanger_matches_oracle_random(pamd, O):
    rng = np.random.default_rng(7)
    n = 60
    owner = rng.integers(1, 5, n)
    for trial in range(3):
        lists = []
        for p in range(1, 5):
            own = [g for g in range(1, n + 1) if owner[g - 1] == p]
            gh = [int(g) for g in rng.choice(np.arange(1, n + 1), 15, replace=False) if owner[g - 1] != p]
            lid_to_gid = list(rng.permutation(own + gh))
            lists.append((lid_to_gid, [int(owner[g - 1]) for g in lid_to_gid]))
        parts = pamd.sequential.get_part_ids(4)
        ex = pamd.exchanger_from_ids(_pd(pamd, parts, [pamd.IndexSet(p + 1, *lists[p]) for p in range(4)]))
        oex = O.exchanger_from_ids(O.PData([O.IndexSet(p + 1, *lists[p]) for p in range(4)]))
        for p in range(4):
            assert list(ex.parts_rcv.parts[p]) == list(oex.parts_rcv.parts[p])
            assert list(ex.parts_snd.parts[p]) == list(oex.parts_snd.parts[p])
            assert ex.lids_rcv.parts[p].tolist() == oex.lids_rcv.parts[p].tolist()
            assert ex.lids_snd.parts[p].tolist() == oex.lids_snd.parts[p].tolist()


def test_prange_kats(pamd):
    k = GOLD["prange_noids"]
    parts = pamd.sequential.get_part_ids(4)
    r = pamd.prange_noids(parts, _pd(pamd, parts, k["noids"]))
    assert [s.lid_to_gid.tolist() for s in r.partition.parts] == k["lid_to_gid"]
    assert r.gid_to_part.parts[0](np.arange(1, 16)).tolist() == k["gid_to_part"]
    k = GOLD["prange_cartesian"]
    parts = pamd.sequential.get_part_ids((2, 2))
    r = pamd.prange_cartesian(parts, (5, 4))
    assert [s.lid_to_gid.tolist() for s in r.partition.parts] == k["lid_to_gid"]
    assert r.gid_to_part.parts[0](np.arange(1, 21)).tolist() == k["gid_to_part"]
    r1 = pamd.prange_linear(pamd.sequential.get_part_ids(3), 10)
    assert [s.lid_to_gid.tolist() for s in r1.partition.parts] == [[1, 2, 3], [4, 5, 6], [7, 8, 9, 10]]


def test_add_gids_first_touch_matches_oracle(pamd, O):
    rng = np.random.default_rng(3)
    n = 50
    parts = pamd.sequential.get_part_ids(4)
    oparts = O.get_part_ids(4)
    gids = [list(rng.integers(1, n + 1, 30)) for _ in range(4)]
    r = pamd.add_gids(pamd.prange_linear(parts, n), _pd(pamd, parts, [np.array(g) for g in gids]))
    o = O.add_gids(O.prange_linear(oparts, n), O.PData([list(g) for g in gids]))
    for p in range(4):
        assert r.partition.parts[p].lid_to_gid.tolist() == o.partition.parts[p].lid_to_gid
        assert r.partition.parts[p].lid_to_part.tolist() == o.partition.parts[p].lid_to_part
        assert r.exchanger.lids_snd.parts[p].tolist() == o.exchanger.lids_snd.parts[p].tolist()


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
def test_compresscoo_matches_sparse(pamd, O, dtype):
    rng = np.random.default_rng(5)
    m, n, k = 30, 25, 400
    I = rng.integers(1, m + 1, k)
    J = rng.integers(1, n + 1, k)
    V = rng.uniform(-1, 1, k).astype(dtype)
    if np.dtype(dtype).kind == "c":
        V = V + 1j * rng.uniform(-1, 1, k)
    A = pamd.compresscoo(I, J, V, m, n)
    OV = O.Cx(V.real.copy(), V.imag.copy()) if np.iscomplexobj(V) else V
    B = O.sparse_csc(I, J, OV, m, n)
    assert np.array_equal(A.colptr, B.colptr) and np.array_equal(A.rowval, B.rowval)
    if np.iscomplexobj(V):
        assert np.array_equal(A.nzval.real, B.nzval.re) and np.array_equal(A.nzval.imag, B.nzval.im)
    else:
        assert np.array_equal(A.nzval, B.nzval)
    k2 = GOLD["sparse_utils"]
    S = pamd.compresscoo(k2["I"], k2["J"], np.array(k2["V"], float), k2["m"], k2["n"])
    assert S.nnz == len(k2["dense_nonzeros"])


@pytest.mark.parametrize("shape,N,kind", [((2, 2, 1), (12, 10, 9), 27), ((2, 1, 2), (9, 8, 11), 7),
                                          ((2, 2, 2), (8, 8, 8), 27), ((3, 1, 1), (13, 4, 5), 27)])
def test_stencil_partition_matches_oracle(pamd, O, shape, N, kind):
    parts = pamd.sequential.get_part_ids(shape)
    rows, cols = pamd.drivers.stencil_partition(parts, N, kind)
    OA = O.stencil_problem(O.get_part_ids(shape), N, kind)
    for p in parts.part_ids:
        s, os_ = cols.partition.local(p), OA.cols.partition[p]
        assert s.lid_to_gid.tolist() == os_.lid_to_gid
        assert s.lid_to_part.tolist() == os_.lid_to_part
        ex, oex = cols.exchanger, OA.cols.exchanger
        assert list(ex.parts_rcv.local(p)) == list(oex.parts_rcv[p])
        assert list(ex.parts_snd.local(p)) == list(oex.parts_snd[p])
        assert ex.lids_rcv.local(p).tolist() == oex.lids_rcv[p].tolist()
        assert ex.lids_snd.local(p).tolist() == oex.lids_snd[p].tolist()


@pytest.mark.parametrize("nparts", [4, (2, 2, 2)])
def test_fdm_host_matches_oracle(pamd, O, nparts):
    parts = pamd.sequential.get_part_ids(nparts)
    rows, cols, I, J, V, bh, xh, x0h = pamd.drivers.fdm_host(parts, 10)
    OA, ob, ox0, oxh = O.fdm_problem(O.get_part_ids(nparts), 10)
    for p in parts.part_ids:
        A = pamd.compresscoo(I.local(p), J.local(p), V.local(p), rows.partition.local(p).num_lids,
                             cols.partition.local(p).num_lids)
        M = OA.values[p]
        assert np.array_equal(A.colptr, M.colptr) and np.array_equal(A.rowval, M.rowval)
        assert np.array_equal(A.nzval, M.nzval)
        assert np.array_equal(bh.local(p), ob.values[p])
        assert np.array_equal(xh.local(p), oxh.values[p])
        assert np.array_equal(x0h.local(p), ox0.values[p])


@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_fem_sa_host_matches_oracle(pamd, O, nparts):
    """test_fem_sa.jl setup: COO assembly (async_assemble!), rows/cols ghost
    layers and the local CSCs equal the oracle's."""
    parts = pamd.sequential.get_part_ids(nparts)
    rows, cols, I, J, V, bh, x0h, xh = pamd.drivers.fem_sa_host(parts, 10)
    oparts = O.get_part_ids(nparts)
    OA, ob, ox0, oxh = O.fem_sa_problem(oparts, 10)
    for p in parts.part_ids:
        r, c = rows.partition.local(p), cols.partition.local(p)
        assert r.lid_to_gid.tolist() == OA.rows.partition[p].lid_to_gid
        assert c.lid_to_gid.tolist() == OA.cols.partition[p].lid_to_gid
        M = pamd.compresscoo(r.to_lids(I.local(p)), c.to_lids(J.local(p)), V.local(p), r.num_lids, c.num_lids)
        OM = OA.values[p]
        assert np.array_equal(M.colptr, OM.colptr) and np.array_equal(M.rowval, OM.rowval)
        assert np.array_equal(M.nzval, OM.nzval)
        assert np.array_equal(x0h.local(p)[c.oid_to_lid - 1], ox0.values[p][c.oid_to_lid - 1])


@pytest.mark.parametrize("kind,N", [(7, (7, 6, 5)), (27, (7, 6, 5)), (27, (5, 9, 4))])
def test_stencil_entries_vectorised(pamd, O, kind, N):
    """The vectorised row generators (product and oracle) == the oracle's
    scalar stencil_row_entries, row by row, entry by entry."""
    coef = O.fd7_coeffs(N[0]) if kind == 7 else O.q1_hex_ke(2.0 / (N[0] - 1)).ravel()
    gids = np.random.default_rng(5).permutation(int(np.prod(N))) + 1
    ref = []
    for g in gids:
        c = tuple(x - 1 for x in O.cartesian_index(N, int(g)))
        for nb, v in O.stencil_row_entries(kind, N, c, coef):
            ref.append((int(g), O.linear_index(N, tuple(x + 1 for x in nb)), v))
    R = np.array(ref)
    for I, J, V in (O.stencil_rows_vec(kind, N, gids, coef), pamd.drivers.stencil_entries(kind, N, gids)):
        assert np.array_equal(gids[I], R[:, 0]) and np.array_equal(J, R[:, 1])
        assert np.array_equal(V, R[:, 2])


def test_oracle_vectorised_add_gids(O):
    rng = np.random.default_rng(3)
    owners = rng.integers(1, 4, 200)
    g2p = lambda g: int(owners[g - 1])
    mk = lambda: O.IndexSet(1, [3, 9, 27], [1, 1, 1], [1, 2, 3], [])
    gids = rng.integers(1, 201, 500)
    a, b = mk(), mk()
    O.add_gids_owner_(g2p, a, gids)
    O.add_gids_owner_vec_(g2p, b, gids)
    assert a.lid_to_gid == b.lid_to_gid and a.lid_to_part == b.lid_to_part and a.hid_to_lid == b.hid_to_lid
    assert O.to_lids_vec(np.array(gids), a).tolist() == O.to_lids_(list(gids), a)


@pytest.mark.parametrize("nparts,N,kind", [(4, (14, 12, 10), 27), (7, (11, 9, 13), 7), (3, (9, 9, 9), 27)])
def test_irregular_partition_matches_oracle(pamd, O, nparts, N, kind):
    """C5 setup: Voronoi owners, first-touch ghosts, gather-discovered
    Exchanger and local CSCs equal the oracle's."""
    parts = pamd.sequential.get_part_ids(nparts)
    rows, cols, I, J, V = pamd.drivers.irregular_partition(parts, N, kind)
    OA = O.irregular_problem(O.get_part_ids(nparts), N, kind)
    assert np.array_equal(pamd.drivers.voronoi_owners(N, nparts), O.voronoi_owners(N, nparts))
    ex, oex = cols.exchanger, OA.cols.exchanger
    for p in parts.part_ids:
        r, c = rows.partition.local(p), cols.partition.local(p)
        oc = OA.cols.partition[p]
        assert c.lid_to_gid.tolist() == oc.lid_to_gid and c.lid_to_part.tolist() == oc.lid_to_part
        assert list(ex.parts_rcv.local(p)) == list(oex.parts_rcv[p])
        assert list(ex.parts_snd.local(p)) == list(oex.parts_snd[p])
        assert ex.lids_rcv.local(p).tolist() == oex.lids_rcv[p].tolist()
        assert ex.lids_snd.local(p).tolist() == oex.lids_snd[p].tolist()
        M = pamd.compresscoo(r.to_lids(I.local(p)), c.to_lids(J.local(p)), V.local(p), r.num_lids, c.num_lids)
        OM = OA.values[p]
        assert np.array_equal(M.colptr, OM.colptr) and np.array_equal(M.rowval, OM.rowval)
        assert np.array_equal(M.nzval, OM.nzval)


@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_matrix_exchanger_matches_oracle(pamd, O, nparts):
    """matrix_exchanger (Interfaces.jl:2300-2372) of test_fem_sa's matrix, whose
    local CSCs store ghost rows: the product's vectorised restatement equals
    the oracle's literal one (parts, nz ids k in both directions)."""
    parts = pamd.sequential.get_part_ids(nparts)
    rows, cols, I, J, V, _, _, _ = pamd.drivers.fem_sa_host(parts, 10)
    csc = pamd.map_parts(lambda i, j, v, r, c: pamd.compresscoo(r.to_lids(i), c.to_lids(j), v, r.num_lids,
                                                                c.num_lids), I, J, V, rows.partition, cols.partition)
    ex = pamd.pvector.matrix_exchanger(csc, rows, cols)
    OA, _, _, _ = O.fem_sa_problem(O.get_part_ids(nparts), 10)
    oex = OA.exchanger
    assert sum(len(oex.lids_rcv[p].data) for p in parts.part_ids) > 0
    for p in parts.part_ids:
        assert list(ex.parts_rcv.local(p)) == list(oex.parts_rcv[p])
        assert list(ex.parts_snd.local(p)) == list(oex.parts_snd[p])
        for a, b in ((ex.lids_rcv.local(p), oex.lids_rcv[p]), (ex.lids_snd.local(p), oex.lids_snd[p])):
            assert a.data.tolist() == list(b.data) and a.ptrs.tolist() == list(b.ptrs)


def test_matrix_exchanger_inconsistent_pattern(pamd):
    """setup_snd's @check (Interfaces.jl:2360): a ghost-row nonzero the owner
    does not store raises."""
    parts = pamd.sequential.get_part_ids(2)
    rows = pamd.prange_linear(parts, 4)
    rows = pamd.add_gids(rows, pamd.PData(parts.backend, parts.part_ids, [np.array([3]), np.array([2])],
                                          parts.shape))
    cols = rows
    # part 1 stores (3,3) in its ghost row 3, part 2 owns row 3 but stores only (3,4)
    c1 = pamd.compresscoo(rows.partition.local(1).to_lids([1, 3]), rows.partition.local(1).to_lids([1, 3]),
                          [1.0, 1.0], 3, 3)
    c2 = pamd.compresscoo(rows.partition.local(2).to_lids([3]), rows.partition.local(2).to_lids([4]), [1.0], 3, 3)
    csc = pamd.PData(parts.backend, parts.part_ids, [c1, c2], parts.shape)
    with pytest.raises(AssertionError):
        pamd.pvector.matrix_exchanger(csc, rows, cols)


@pytest.mark.parametrize("shape,N,kind", [((2, 2, 2), (9, 8, 7), 27), ((3, 2, 1), (10, 9, 4), 7),
                                          ((4, 1, 1), (12, 5, 5), 27)])
def test_grid_neighbor_discovery(pamd, O, shape, N, kind, monkeypatch):
    """Cartesian add_gids! discovers parts_snd from the grid neighbours
    (Interfaces.jl:471-496) — no gather on MAIN — and yields the oracle's
    Exchanger (gather-based, Interfaces.jl:515-521); a ghost owned by a part
    outside the grid neighbourhood falls back to the all-to-all discover."""
    P = pamd.prange
    parts = pamd.sequential.get_part_ids(shape)
    rows = pamd.prange_cartesian(parts, N)
    _, J, _ = pamd.backends.unzip(pamd.map_parts(
        lambda s: pamd.drivers.stencil_entries(kind, N, s.lid_to_gid[s.oid_to_lid - 1]), rows.partition), 3)
    orows = O.prange_cartesian(O.get_part_ids(shape), N)
    ocols = O.add_gids(orows, O.PData([list(map(int, J.local(p))) for p in parts.part_ids]))

    def no_gather(*a, **k):
        raise AssertionError("gather-based discover_parts_snd used")
    monkeypatch.setattr(P, "gather", no_gather)
    cols = pamd.add_gids(rows, J)
    oex = ocols.exchanger
    for p in parts.part_ids:
        assert list(cols.exchanger.parts_snd.local(p)) == list(oex.parts_snd[p])
        assert cols.exchanger.lids_snd.local(p).tolist() == oex.lids_snd[p].tolist()
        assert cols.exchanger.lids_rcv.local(p).tolist() == oex.lids_rcv[p].tolist()
    # a far ghost (part 1 touches the last gid, owned by the last part)
    far = pamd.map_parts(lambda s, j: np.append(j, rows.ngids) if s.part == 1 else j, rows.partition, J)
    nbr_last = pamd.prange.grid_neighbors(shape, parts.num_parts)
    if 1 in nbr_last:
        return
    cols = pamd.add_gids(rows, far)  # outside the grid neighbourhood: the all-to-all discover, still no gather
    monkeypatch.undo()
    ocols = O.add_gids(orows, O.PData([list(map(int, far.local(p))) for p in parts.part_ids]))
    for p in parts.part_ids:
        assert list(cols.exchanger.parts_snd.local(p)) == list(ocols.exchanger.parts_snd[p])
        assert cols.exchanger.lids_snd.local(p).tolist() == ocols.exchanger.lids_snd[p].tolist()


@pytest.mark.parametrize("shape,ngids,periodic", [((2, 2), (5, 4), None), ((2, 2), (4, 4), (True, True)),
                                                   ((2, 2), (4, 4), (False, True)), ((3, 1, 2), (7, 3, 5), None),
                                                   ((2, 3, 2), (6, 7, 5), (True, False, True)), ((4,), (11,), (True,))])
def test_prange_with_ghost_matches_oracle(pamd, O, shape, ngids, periodic):
    """PRange(parts, ngids, with_ghost[, isperiodic]) (Interfaces.jl:1166-1223):
    interleaved owned/ghost lids, owners, and the reuse_parts_rcv Exchanger
    equal the oracle's (pinned by test_interfaces.jl:383-497)."""
    parts = pamd.sequential.get_part_ids(shape)
    r = pamd.prange_cartesian(parts, ngids, with_ghost=True, isperiodic=periodic)
    o = O.prange_cartesian(O.get_part_ids(shape), ngids, with_ghost=True, isperiodic=periodic)
    for p in parts.part_ids:
        s, os_ = r.partition.local(p), o.partition[p]
        assert s.lid_to_gid.tolist() == list(os_.lid_to_gid)
        assert s.lid_to_part.tolist() == list(os_.lid_to_part)
        assert s.oid_to_lid.tolist() == list(os_.oid_to_lid) and s.hid_to_lid.tolist() == list(os_.hid_to_lid)
        ex, oex = r.exchanger, o.exchanger
        assert list(ex.parts_rcv.local(p)) == list(oex.parts_rcv[p])
        assert list(ex.parts_snd.local(p)) == list(oex.parts_snd[p])
        assert ex.lids_rcv.local(p).tolist() == oex.lids_rcv[p].tolist()
        assert ex.lids_snd.local(p).tolist() == oex.lids_snd[p].tolist()


@pytest.mark.parametrize("Bi", [0, 1])
@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
def test_sparsecsr_matches_oracle(pamd, O, Bi, dtype):
    """sparsecsr(Val(Bi), I, J, V, m, n, +) (SparseUtils.jl:193-208): the
    host compress equals the oracle's (duplicates in input order, columns
    ascending in each row, indices in base Bi)."""
    rng = np.random.default_rng(17)
    m, n, k = 40, 33, 600
    I, J = rng.integers(1, m + 1, k), rng.integers(1, n + 1, k)
    V = rng.uniform(-1, 1, k) + (1j * rng.uniform(-1, 1, k) if np.dtype(dtype).kind == "c" else 0)
    V = V.astype(dtype)
    M = pamd.sparsecsr(Bi, I, J, V, m, n)
    OV = O.Cx(V.real.copy(), V.imag.copy()) if np.iscomplexobj(V) else V.copy()
    OM = O.sparse_csr(Bi, I, J, OV, m, n)
    assert M.Bi == Bi and M.rowptr[0] == Bi
    assert np.array_equal(M.rowptr, OM.rowptr) and np.array_equal(M.colval, OM.colval)
    if np.iscomplexobj(V):
        assert np.array_equal(M.nzval.real, OM.nzval.re) and np.array_equal(M.nzval.imag, OM.nzval.im)
    else:
        assert np.array_equal(M.nzval, OM.nzval)


@pytest.mark.parametrize("Bi", [0, 1])
@pytest.mark.parametrize("nparts", [4, (2, 2)])
def test_matrix_exchanger_csr_matches_oracle(pamd, O, nparts, Bi):
    """matrix_exchanger over SparseMatrixCSR parts (nzindex of
    SparseUtils.jl:210-220, CSR storage order): equals the oracle's literal
    matrix_exchanger on the same CSRs."""
    parts = pamd.sequential.get_part_ids(nparts)
    rows, cols, I, J, V, _, _, _ = pamd.drivers.fem_sa_host(parts, 10)
    csr = pamd.map_parts(lambda i, j, v, r, c: pamd.sparsecsr(Bi, r.to_lids(i), c.to_lids(j), v, r.num_lids,
                                                              c.num_lids), I, J, V, rows.partition, cols.partition)
    ex = pamd.pvector.matrix_exchanger(csr, rows, cols)
    OA, _, _, _ = O.fem_sa_problem(O.get_part_ids(nparts), 10, init=lambda i, j, v, m, n: O.sparse_csr(Bi, i, j, v, m, n))
    oex = OA.exchanger
    assert sum(len(oex.lids_rcv[p].data) for p in parts.part_ids) > 0
    for p in parts.part_ids:
        M, OM = csr.local(p), OA.values[p]
        assert np.array_equal(M.rowptr, OM.rowptr) and np.array_equal(M.colval, OM.colval)
        assert list(ex.parts_rcv.local(p)) == list(oex.parts_rcv[p])
        assert list(ex.parts_snd.local(p)) == list(oex.parts_snd[p])
        for a, b in ((ex.lids_rcv.local(p), oex.lids_rcv[p]), (ex.lids_snd.local(p), oex.lids_snd[p])):
            assert a.data.tolist() == list(b.data) and a.ptrs.tolist() == list(b.ptrs)
