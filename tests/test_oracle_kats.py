"""Pin the CPU oracle against the reference's own known-answer tests
(tests/golden/interfaces_kats.json, transcribed from test/test_interfaces.jl
and test/SparseUtilsTests.jl by tests/golden/make_golden.py)."""
import json
import os

import numpy as np
import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "interfaces_kats.json")))


def test_exchange_scalar(O):
    k = GOLD["exchange_scalar"]
    parts = O.get_part_ids(4)
    prcv = O.PData(k["parts_rcv"])
    psnd = O.PData(k["parts_snd"])
    data = O.map_parts(lambda p: [10 * i for i in p], psnd)
    got = O.exchange_scalars(data, prcv, psnd)
    assert got.parts == k["expected_rcv"]
    assert O.num_parts(parts) == 4


def test_reduce_and_scan(O):
    parts = O.get_part_ids(4)
    assert O.preduce(lambda a, b: a + b, parts, 0) == GOLD["reduce"]["expected"]
    assert O.reduce_all(lambda a, b: a + b, parts, 0).parts == [10] * 4
    assert O.psum(parts) == 10
    k = GOLD["scan"]
    a = O.PData(k["a"])
    assert O.iscan(lambda x, y: x + y, a, 0).parts == k["iscan_init0"]
    assert O.iscan_all(lambda x, y: x + y, a, 0).parts[0] == k["iscan_init0"]
    assert O.xscan(lambda x, y: x + y, a, 1).parts == k["xscan_init1"]


def test_discover_parts_snd(O):
    k = GOLD["discover"]
    got = O.discover_parts_snd(O.PData(k["parts_rcv"]))
    assert got.parts == k["expected_parts_snd"]
    O.ERROR_DISCOVER_PARTS_SND[0] = True
    try:
        with pytest.raises(RuntimeError):
            O.discover_parts_snd(O.PData(k["parts_rcv"]))
    finally:
        O.ERROR_DISCOVER_PARTS_SND[0] = False
    # neighbour-assisted form (Interfaces.jl:471-496) with a superset graph
    nb = O.PData([[2, 3, 4], [1, 3, 4], [1, 2, 4], [1, 2, 3]])
    got2 = O.discover_parts_snd(O.PData(k["parts_rcv"]), nb)
    assert got2.parts == k["expected_parts_snd"]


def _kat_partition(O):
    k = GOLD["exchanger"]
    return O.PData([O.IndexSet(p + 1, k["lid_to_gid"][p], k["lid_to_part"][p]) for p in range(4)])


def test_exchanger_kat(O):
    k = GOLD["exchanger"]
    ex = O.exchanger_from_ids(_kat_partition(O))
    assert [list(x) for x in ex.parts_snd.parts] == k["expected_parts_snd"]
    assert [t.tolist() for t in ex.lids_snd.parts] == k["expected_lids_snd"]


def test_exchange_values_kats(O):
    part = _kat_partition(O)
    ex = O.exchanger_from_ids(part)
    vals = O.map_parts(lambda s: np.array([10.0 * s.part if o == s.part else 0.0 for o in s.lid_to_part]), part)
    O.exchange_(vals, ex)
    for s, v in zip(part.parts, vals.parts):
        assert list(v) == [10.0 * o for o in s.lid_to_part]
    # two buffers (test_interfaces.jl:229-251)
    vr = O.map_parts(lambda s: np.full(s.num_lids, 10.0), part)
    vs = O.map_parts(lambda s: np.full(s.num_lids, 20.0), part)
    O.exchange_values_(O._replace, vr, vs, ex)
    for s, v in zip(part.parts, vr.parts):
        assert list(v) == [10.0 if o == s.part else 20.0 for o in s.lid_to_part]
    assert all((v == 20.0).all() for v in vs.parts)


def test_exchange_table_kat(O):
    part = _kat_partition(O)
    ex = O.exchanger_from_ids(part)

    def mk(s):
        vv = [[0, 0, 0] for _ in range(s.num_lids)]
        for lid in s.oid_to_lid:
            gid = s.lid_to_gid[lid - 1]
            vv[lid - 1] = [100 * s.part + 10 * gid + i for i in (1, 2, 3)]
        return O.table_from(vv)
    vals = O.map_parts(mk, part)
    O.exchange_table_values_(vals, ex)
    for s, t in zip(part.parts, vals.parts):
        for lid in range(1, s.num_lids + 1):
            gid, owner = s.lid_to_gid[lid - 1], s.lid_to_part[lid - 1]
            assert list(t[lid]) == [100 * owner + 10 * gid + i for i in (1, 2, 3)]


def test_reverse_add_then_exchange(O):
    """test_interfaces.jl:276-287: exchange!(+, values, reverse) then exchange!"""
    part = _kat_partition(O)
    ex = O.exchanger_from_ids(part)
    vals = O.map_parts(lambda s: np.full(s.num_lids, 10.0 * s.part), part)
    O.exchange_values_(lambda a, b: a + b, vals, vals, O.reverse_exchanger(ex))
    O.exchange_(vals, ex)
    # every copy of a gid now holds the owner's assembled value
    tot = {}
    for s, v in zip(part.parts, vals.parts):
        for lid in s.oid_to_lid:
            tot[s.lid_to_gid[lid - 1]] = v[lid - 1]
    for s, v in zip(part.parts, vals.parts):
        for lid in range(1, s.num_lids + 1):
            assert v[lid - 1] == tot[s.lid_to_gid[lid - 1]]


def test_prange_noids(O):
    k = GOLD["prange_noids"]
    parts = O.get_part_ids(4)
    r = O.prange_noids(parts, O.PData(k["noids"]))
    assert [s.lid_to_gid for s in r.partition.parts] == k["lid_to_gid"]
    assert [r.gid_to_part[1](g) for g in range(1, 16)] == k["gid_to_part"]


def test_prange_cartesian_family(O):
    parts = O.get_part_ids((2, 2))
    k = GOLD["prange_cartesian"]
    r = O.prange_cartesian(parts, (5, 4))
    assert [s.lid_to_gid for s in r.partition.parts] == k["lid_to_gid"]
    assert [r.gid_to_part[1](g) for g in range(1, 21)] == k["gid_to_part"]
    pc = GOLD["pcartesian_indices"]
    assert [[list(x) for x in t] for t in O.pcartesian_indices(parts, (5, 4)).parts] == pc["no_ghost"]
    assert [[list(x) for x in t] for t in O.pcartesian_indices(parts, (5, 4), True).parts] == pc["with_ghost"]
    r = O.prange_cartesian(parts, (5, 4), with_ghost=True)
    assert [s.lid_to_gid for s in r.partition.parts] == GOLD["prange_with_ghost"]["lid_to_gid"]
    r = O.prange_cartesian(parts, (4, 4), with_ghost=True, isperiodic=(True, True))
    assert [s.lid_to_gid for s in r.partition.parts] == GOLD["prange_periodic_tt"]["lid_to_gid"]
    r = O.prange_cartesian(parts, (4, 4), with_ghost=True, isperiodic=(False, True))
    assert [s.lid_to_gid for s in r.partition.parts] == GOLD["prange_periodic_ft"]["lid_to_gid"]


def test_diag_matvec_kat(O):
    """test_interfaces.jl:646-680 on the irregular IndexSet partition"""
    k = GOLD["diag_matvec"]
    ids = O.prange(10, _kat_partition(O))
    vals = O.map_parts(lambda s: O.sparse_csc(range(1, s.num_lids + 1), range(1, s.num_lids + 1),
                                              np.full(s.num_lids, k["diag"]), s.num_lids, s.num_lids),
                       ids.partition)
    A = O.PSparseMatrix(vals, ids, ids)
    x = O.pvector_undef(ids)
    O.map_parts(lambda v: v.fill(k["x"]), x.values)
    b = O.pvector_undef(ids)
    for literal in (True, False):
        O.mul_(b, A, x, literal=literal)
        for v, s in zip(b.values.parts, ids.partition.parts):
            assert (v[np.asarray(s.oid_to_lid) - 1] == k["expected"]).all()
    O.exchange_pvector_(b)
    assert all((v == k["expected"]).all() for v in b.values.parts)
    for M in A.values.parts:
        M.nzval[:] = 1.0
    O.mul_(b, A, x)
    O.exchange_pvector_(b)
    assert all((v == k["expected_after_fillstored_1"]).all() for v in b.values.parts)


def test_irregular_coo_kat(O):
    """test_interfaces.jl:686-717: PSparseMatrix(I,J,V,n,n; ids=:global), A*x
    and a direct solve with residual < 1e-9."""
    k = GOLD["irregular_coo"]
    parts = O.get_part_ids(4)
    I = O.PData([list(v) for v in k["I"]])
    J = O.PData([list(v) for v in k["J"]])
    V = O.PData([np.array(v) for v in k["V"]])
    rows = O.prange_linear(parts, k["n"])
    O.add_gids_(rows, I)
    cols = O.prange_linear(parts, k["n"])
    O.add_gids_(cols, J)
    A = O.psparse_from_coo(I, J, V, rows, cols, ids="global")
    # dense global matrix from the owned rows
    D = np.zeros((k["n"], k["n"]))
    for M, r, c in zip(A.values.parts, rows.partition.parts, cols.partition.parts):
        for j in range(M.n):
            for p in range(M.colptr[j] - 1, M.colptr[j + 1] - 1):
                i = M.rowval[p]
                if r.lid_to_part[i - 1] == r.part:
                    D[r.lid_to_gid[i - 1] - 1, c.lid_to_gid[j] - 1] += M.nzval[p]
    x = O.pvector_undef(cols)
    O.map_parts(lambda v: v.fill(1.0), x.values)
    y = O.pvector_undef(rows)
    O.mul_(y, A, x)
    for v, s in zip(y.values.parts, rows.partition.parts):
        for lid in s.oid_to_lid:
            assert v[lid - 1] == pytest.approx(D[s.lid_to_gid[lid - 1] - 1].sum())
    xs = np.linalg.solve(D, np.ones(k["n"]))
    assert np.linalg.norm(D @ xs - 1.0) < k["residual_tol"]


def test_sparse_utils_kat(O):
    k = GOLD["sparse_utils"]
    A = O.sparse_csc(k["I"], k["J"], np.array(k["V"], dtype=float), k["m"], k["n"])
    D = np.zeros((k["m"], k["n"]))
    for j in range(A.n):
        for p in range(A.colptr[j] - 1, A.colptr[j + 1] - 1):
            D[A.rowval[p] - 1, j] = A.nzval[p]
    for key, v in k["dense_nonzeros"].items():
        i, j = map(int, key.split(","))
        assert D[i - 1, j - 1] == v
    assert np.count_nonzero(D) == len(k["dense_nonzeros"])
    rows, cols = k["rows"], k["cols"]
    inv_rows = [0] * k["m"]
    for i, r in enumerate(rows):
        inv_rows[r - 1] = i + 1
    x = np.random.default_rng(0).uniform(size=len(cols))
    y = np.zeros(len(rows))
    O.csc_mul_sub_(y, A, inv_rows, cols, 1, 1, x, 1.0, 0.0)
    np.testing.assert_allclose(y, D[np.array(rows) - 1][:, np.array(cols) - 1] @ x)


def test_fdm_cg(O):
    k = GOLD["solvers"]
    for nparts in (4, (2, 2, 2)):
        parts = O.get_part_ids(nparts)
        A, b, x0, xh = O.fdm_problem(parts, k["fdm_nx"])
        assert sum(int(M.colptr[-1] - 1) for M in A.values.parts) == k["fdm_nnz"]
        x = O.PVector(O.map_parts(lambda v: v.copy(), x0.values), x0.rows)
        O.cg_(x, A, b)
        err = 0.0
        for xv, hv, sx, sh in zip(x.values.parts, xh.values.parts, x.rows.partition.parts, xh.rows.partition.parts):
            err += float(np.sum((xv[np.asarray(sx.oid_to_lid) - 1] - hv[np.asarray(sh.oid_to_lid) - 1]) ** 2))
        assert err ** 0.5 < k["err_tol"]


def test_stencil_nnz_formulas(O):
    """SURVEY.md §8 size table: FD7 nnz = 7(N−2)³ + (N³−(N−2)³), FE27 27(N−2)³ + …"""
    for kind in (7, 27):
        N = 6
        A = O.stencil_problem(O.get_part_ids((1, 1, 1)), (N, N, N), kind)
        nnz = int(A.values.parts[0].colptr[-1] - 1)
        assert nnz == kind * (N - 2) ** 3 + (N ** 3 - (N - 2) ** 3)


def test_mul_literal_equals_vectorised(O):
    """The literal CSC column loop and the vectorised restatement agree bit-for-bit."""
    for shape, N, kind, dt in [((2, 2, 1), (7, 6, 5), 27, np.float64), ((2, 1, 1), (6, 5, 5), 7, np.float32),
                               ((1, 2, 1), (5, 6, 4), 27, np.complex128)]:
        A = O.stencil_problem(O.get_part_ids(shape), N, kind, dt)
        rng = np.random.default_rng(1)

        def mkx(s):
            if dt == np.complex128:
                return O.Cx(rng.uniform(-1, 1, s.num_lids), rng.uniform(-1, 1, s.num_lids))
            return rng.uniform(-1, 1, s.num_lids).astype(dt)
        xv = O.map_parts(mkx, A.cols.partition)
        outs = []
        for literal in (True, False):
            x = O.PVector(O.map_parts(lambda v: O._copyvals(v), xv), A.cols)
            y = O.pvector_undef(A.rows, dt)
            O.mul_(y, A, x, literal=literal)
            outs.append(y)
        for a, b in zip(outs[0].values.parts, outs[1].values.parts):
            if isinstance(a, O.Cx):
                assert np.array_equal(a.re, b.re) and np.array_equal(a.im, b.im)
            else:
                assert np.array_equal(a, b)


@pytest.mark.parametrize("Bi,tv", [(1, np.float64), (1, np.float32), (0, np.float64), (0, np.float32)])
def test_sparse_utils_csr_kat(O, Bi, tv):
    """SparseUtilsTests.jl:62-65: test_mat(SparseMatrixCSR{Bi,Tv,Ti})"""
    k = GOLD["sparse_utils"]
    kc = GOLD["sparse_utils_csr"]
    B = O.sparse_csr(Bi, k["I"], k["J"], np.array(k["V"], dtype=tv), k["m"], k["n"])
    assert B.nzval.dtype == tv
    ents = O.nz_entries(B)
    assert [[i, j, float(B.nzval[p - 1])] for p, i, j in ents] == kc["findnz_order"]
    for p, i, j in ents:
        assert O.nzindex(B, i, j) == p
    assert O.nzindex(B, 3, 3) == -1 and O.nzindex(B, 1, 6) == -1
    D = np.zeros((k["m"], k["n"]), dtype=tv)
    for i, j, v in kc["findnz_order"]:
        D[i - 1, j - 1] = v
    rows, cols = k["rows"], k["cols"]
    inv_cols = [0] * k["n"]
    for j, c in enumerate(cols):
        inv_cols[c - 1] = j + 1
    x = np.random.default_rng(0).uniform(size=len(cols)).astype(tv)
    y = np.zeros(len(rows), dtype=tv)
    O.csr_mul_sub_(y, B, rows, inv_cols, 1, 1, x, tv(1), tv(0))
    np.testing.assert_allclose(y, D[np.array(rows) - 1][:, np.array(cols) - 1] @ x, rtol=1e-6)


def test_csr_partitioned_mul_literal_equals_vectorised(O):
    """PSparseMatrix(sparsecsr, I, J, V, rows, cols): the vectorised mul!
    equals the literal SparseUtils.jl:222-252 loop bit for bit, α = 1 equals
    the CSC parent's result, α != 1 scales the product (SparseUtils.jl:247)."""
    rng = np.random.default_rng(5)
    for Bi in (0, 1):
        for alpha, beta in ((1.0, 0.0), (0.7, 0.0), (-1.3, 0.5)):
            outs = {}
            for fmt in ("csc", "csr", "csr_lit"):
                parts = O.get_part_ids((2, 2, 1))
                init = None if fmt == "csc" else (lambda i, j, v, m, n: O.sparse_csr(Bi, i, j, v, m, n))
                A = O.stencil_problem(parts, (7, 6, 5), 27, init=init)
                xs = O.PVector(O.map_parts(lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids),
                                           A.cols.partition), A.cols)
                y = O.PVector(O.map_parts(lambda s: np.random.default_rng(9 + s.part).uniform(-1, 1, s.num_lids),
                                          A.rows.partition), A.rows)
                O.mul_(y, A, xs, alpha, beta, literal=fmt == "csr_lit")
                outs[fmt] = [v[np.asarray(s.oid_to_lid) - 1] for v, s in zip(y.values.parts, y.rows.partition.parts)]
            for a, b in zip(outs["csr"], outs["csr_lit"]):
                assert np.array_equal(a, b)
            if alpha == 1.0:
                for a, b in zip(outs["csr"], outs["csc"]):
                    assert np.array_equal(a, b)
            else:
                for a, b in zip(outs["csr"], outs["csc"]):
                    np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12)
    del rng
