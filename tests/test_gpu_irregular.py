"""BASELINE config 5 on the device: the 27-pt FE operator on an irregular
Voronoi ("METIS-like") partition — non-box owned sets, first-touch ghosts,
an Exchanger from the all-to-all discover (prange.discover_parts_snd) — for Float64, Float32,
ComplexF64 (and ComplexF32).  SpMV, exchange! and assemble! bit-exact
against the oracle at 128³; dot/norm to 1e-12."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250114
BIG = ((128, 128, 128), 4)


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


_ORACLE = {}


def _oracle(O, N, nparts, dtype):
    key = (N, nparts)
    if key not in _ORACLE:
        _ORACLE[key] = O.irregular_problem(O.get_part_ids(nparts), N, 27)
    A = _ORACLE[key]
    if np.dtype(dtype) == np.float64:
        return A
    vals = O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, O._convert_values(M.nzval, dtype)), A.values)
    return O.PSparseMatrix(vals, A.rows, A.cols)


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


@pytest.mark.parametrize("N,nparts,dtype,fmt", [
    (BIG[0], BIG[1], np.float64, 1), (BIG[0], BIG[1], np.float64, 0),
    (BIG[0], BIG[1], np.float32, 1), (BIG[0], BIG[1], np.complex128, 1),
    ((24, 22, 20), 8, np.complex64, 1), ((24, 22, 20), 8, np.float64, 0),
    (BIG[0], 8, np.float64, 1), (BIG[0], 8, np.float32, 1),       # C5 as benched: 8 parts of one device
    ((24, 22, 20), 12, np.float64, 1), ((24, 22, 20), 12, np.complex128, 0)])  # > PA_GROUP_MAX parts
@pytest.mark.parametrize("tri16", [1, 0, 3])  # 3: the triple SELL with its other rows first (spmv_tri_order 1)
def test_irregular_spmv_bitexact(be, pamd, O, N, nparts, dtype, fmt, tri16):
    if fmt == 0 and tri16 != 1:
        pytest.skip("spmv_format 0 runs every slice as int32 ids: the triple SELL is not used")
    prev = pamd._lib.tune("spmv_format", fmt)
    prev_tri = pamd._lib.tune("spmv_tri16", min(tri16, 1))
    prev_ord = pamd._lib.tune("spmv_tri_order", 1 if tri16 == 3 else 0)
    # pattern slices from 40 % regular rows (default 70): the side SELL gets
    # the rest, so both the pattern and the side-row paths run
    prev_pct = pamd._lib.tune("pattern_min_regular", 40)
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        OA = _oracle(O, N, nparts, dtype)
        rng = np.random.default_rng(SEED)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        # ghost entries of x are garbage until mul!'s exchange! replaces them
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y, A, x)
        ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows, dtype)
        O.mul_(oy, OA, ox)
        got, gx = y.to_host(), x.to_host()
        for p in parts.part_ids:
            assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
            assert _eq(O, gx.local(p), ox.values[p]), f"part {p}: ghost values of x differ"
        info = A.info()
        if fmt == 1:  # the irregular boxes leave rows off any slice pattern: both paths used
            assert any(i["side_rows"] > 0 for i in info.parts)
    finally:
        pamd._lib.tune("spmv_format", prev)
        pamd._lib.tune("spmv_tri16", prev_tri)
        pamd._lib.tune("spmv_tri_order", prev_ord)
        pamd._lib.tune("pattern_min_regular", prev_pct)


@pytest.mark.parametrize("pull", [1, 0])
def test_irregular_exchange_assemble_dot(be, pamd, O, pull):
    prev = pamd._lib.tune("halo_pull", pull)
    try:
        _irregular_exchange_assemble_dot(be, pamd, O)
    finally:
        pamd._lib.tune("halo_pull", prev)


def _irregular_exchange_assemble_dot(be, pamd, O):
    N, nparts = BIG
    parts = be.get_part_ids(nparts)
    rows, cols, _, _, _ = pamd.drivers.irregular_partition(parts, N, 27)
    OA = _oracle(O, N, nparts, np.float64)
    rng = np.random.default_rng(SEED + 1)
    vs = {p: rng.uniform(-1, 1, cols.partition.local(p).num_lids) for p in parts.part_ids}
    ws = {p: rng.uniform(-1, 1, cols.partition.local(p).num_lids) for p in parts.part_ids}
    v = pamd.PVector.from_host(pamd.map_parts(lambda s: vs[s.part], cols.partition), cols)
    w = pamd.PVector.from_host(pamd.map_parts(lambda s: ws[s.part], cols.partition), cols)
    ov = O.PVector(O.map_parts(lambda s: vs[s.part].copy(), OA.cols.partition), OA.cols)
    ow = O.PVector(O.map_parts(lambda s: ws[s.part].copy(), OA.cols.partition), OA.cols)
    pamd.exchange_(v)
    O.exchange_pvector_(ov)
    pamd.assemble_(w)
    O.assemble_(ow)
    for p in parts.part_ids:
        assert np.array_equal(v.to_host().local(p), ov.values[p])
        assert np.array_equal(w.to_host().local(p), ow.values[p])
    d, od = pamd.dot(v, w), O.dot(ov, ow)
    assert abs(d - od) <= 1e-12 * abs(od)
    assert abs(pamd.norm(w) - O.norm(ow)) <= 1e-12 * O.norm(ow)


@pytest.mark.parametrize("N,nparts,dtype", [
    (BIG[0], BIG[1], np.float64), (BIG[0], BIG[1], np.float32), (BIG[0], BIG[1], np.complex128),
    ((24, 22, 20), 8, np.complex64), ((24, 22, 20), 8, np.float64)])
def test_irregular_big_bitexact(be, pamd, O, N, nparts, dtype):
    """Voronoi parts keep their rows in gid order, so a slice spans several
    x-runs with different y/z offsets (pattern slices with side rows,
    delta16 and int32 slices mixed): the product stays bit-exact."""
    parts = be.get_part_ids(nparts)
    A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
    OA = _oracle(O, N, nparts, dtype)
    rng = np.random.default_rng(SEED + 7)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    got = y.to_host()
    for p in parts.part_ids:
        assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"


@pytest.mark.parametrize("dtype,fmt", [(np.float64, 1), (np.float64, 0), (np.complex128, 1), (np.float32, 1)])
def test_grouped_launches_equal_per_part(be, pamd, dtype, fmt):
    """pa_tune("spmv_group"): the parts sharing a stream pair as one launch
    per phase (default) give the same bits as the per-part launches, the
    fused SpMV+dot included (C5: 8 Voronoi parts of 128³)."""
    N, nparts = BIG[0], 8
    prev = pamd._lib.tune("spmv_format", fmt)
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        rng = np.random.default_rng(SEED + 3)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        out = {}
        for grp in (1, 0):
            g0 = pamd._lib.tune("spmv_group", grp)
            try:
                x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
                y = pamd.PVector.undef(A.rows, dtype)
                pamd.mul_(y, A, x, 2.0, 0.0)
                d = pamd.mul_dot_(y, A, x)
                out[grp] = ([v.copy() for v in y.to_host().parts], [v.copy() for v in x.to_host().parts], d)
            finally:
                pamd._lib.tune("spmv_group", g0)
        for a, b in zip(out[0][0], out[1][0]):
            assert np.array_equal(a, b)
        for a, b in zip(out[0][1], out[1][1]):
            assert np.array_equal(a, b)
        assert out[0][2] == out[1][2]
    finally:
        pamd._lib.tune("spmv_format", prev)


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128, np.complex64])
def test_delta16_slices_equal_int32(be, pamd, O, dtype):
    """C5 Voronoi parts: most int32-column slices become delta16 slices (2 B
    column codes, pa_tune spmv_delta16), re-sliced into the triple SELL (one
    code per consecutive column triple, spmv_tri16: slices of 1-2 rows per
    lane); mul! is
    bit-identical with and without them and equals the oracle."""
    N, nparts = (40, 36, 32), 8
    parts = be.get_part_ids(nparts)
    OA = _oracle(O, N, nparts, dtype)
    rng = np.random.default_rng(SEED + 11)
    out = []
    for d16 in (1, 0):
        prev = pamd._lib.tune("spmv_delta16", d16)
        try:
            A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        finally:
            pamd._lib.tune("spmv_delta16", prev)
        nd = sum(i["delta16_slices"] + i["triple_sell_slices"] for i in A.info().parts)
        assert (nd > 0) == bool(d16)
        if d16:
            xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y, A, x)
        out.append(y.to_host())
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        assert _eq(O, out[0].local(p), oy.values[p]), f"part {p}: delta16 SpMV differs from the oracle"
        assert _eq(O, out[1].local(p), oy.values[p]), f"part {p}: int32 SpMV differs from the oracle"


@pytest.mark.parametrize("merge,direct,d16", [(1, 1, 1), (0, 1, 1), (1, 0, 1), (0, 0, 0), (1, 1, 0)])
def test_launch_paths_equal_oracle(be, pamd, O, merge, direct, d16):
    """Every launch path of mul! over the parts of one GPU gives the oracle's
    bits: merged launch or one launch per slice kind (spmv_merge), direct
    pull or pack + pull on the comm stream (halo_direct), delta16 or int32
    column ids (spmv_delta16); Voronoi parts, F64, 8 parts."""
    N, nparts = (30, 28, 26), 8
    knobs = {"spmv_merge": merge, "halo_direct": direct, "spmv_delta16": d16}
    prev = {k: pamd._lib.tune(k, v) for k, v in knobs.items()}
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, np.float64)
        OA = _oracle(O, N, nparts, np.float64)
        rng = np.random.default_rng(SEED + 21)
        xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        for _ in range(2):  # the second call reuses the cached tables
            pamd.mul_(y, A, x)
        ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows)
        O.mul_(oy, OA, ox)
        got, gx = y.to_host(), x.to_host()
        for p in parts.part_ids:
            assert np.array_equal(got.local(p), oy.values[p]), f"part {p}: SpMV differs"
            assert np.array_equal(gx.local(p), ox.values[p]), f"part {p}: ghost values of x differ"
    finally:
        for k, v in prev.items():
            pamd._lib.tune(k, v)



@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex64, np.complex128])
@pytest.mark.parametrize("d16,tri16", [(1, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("tail", [8, 0])
def test_voronoi_column_loops_equal_oracle(be, pamd, O, dtype, d16, tri16, tail):
    """The int32 / delta16 / triple-SELL column loops (Float64: ids one
    batch ahead; Float32: interleaved delta16 rows; the triple SELL: one
    code and one x run per consecutive column triple), with and without the
    masked tail batch, α != 1: the Voronoi parts' SpMV gives the oracle's
    bits for every column encoding and element type."""
    N, nparts = (30, 28, 26), 8
    prev = {"spmv_delta16": pamd._lib.tune("spmv_delta16", d16),
            "spmv_tri16": pamd._lib.tune("spmv_tri16", tri16),
            "spmv_flags": pamd._lib.tune("spmv_flags", 1 | 4 | 16 | 64 | tail)}
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        info = [A.values.local(p).info() for p in parts.part_ids]
        if tri16:  # the encoding is on and used: triple slices exist; a part with them has no delta16 slice left
            assert sum(i["tri_rows"] for i in info) > 0
            assert all(i["delta16_slices"] == 0 for i in info if i["triple_sell_rows"] > 0)
        else:
            assert all(i["triple_sell_rows"] == 0 for i in info)
        OA = _oracle(O, N, nparts, dtype)
        rng = np.random.default_rng(SEED + 23)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y, A, x, 0.5, 0.0)
        ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows, dtype)
        half = np.float32(0.5) if np.dtype(dtype) in (np.float32, np.complex64) else 0.5
        O.mul_(oy, OA, ox, half, 0.0)
        got = y.to_host()
        for p in parts.part_ids:
            assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
    finally:
        for k, v in prev.items():
            pamd._lib.tune(k, v)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_voronoi_values_round_trip_through_moved_slots(be, pamd, O, dtype):
    """Float32 delta16 slices move their values to interleaved rows at
    build time and the CSC nz → slot map follows, and the triple SELL's
    copies are refreshed from those slots: get_values returns the
    oracle's nzval in CSC order, set_values writes new values to the right
    slots (mul! with them equals the oracle's), for both element types."""
    N, nparts = (30, 28, 26), 8
    parts = be.get_part_ids(nparts)
    A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
    OA = _oracle(O, N, nparts, dtype)
    if np.dtype(dtype) == np.float32:
        assert any(A.values.local(p).info()["delta16_slices"] + A.values.local(p).info()["tri_rows"] > 0
                   for p in parts.part_ids)
    for i, p in enumerate(parts.part_ids):
        assert np.array_equal(A.values.local(p).get_values(), OA.values.parts[i].nzval), p
    rng = np.random.default_rng(SEED + 31)
    new = []
    for i, p in enumerate(parts.part_ids):
        v2 = rng.uniform(-1, 1, len(OA.values.parts[i].nzval)).astype(dtype)
        A.values.local(p).set_values(v2)
        assert np.array_equal(A.values.local(p).get_values(), v2)
        new.append(v2)
    it = iter(new)  # the oracle with the same new values (a copy: _oracle caches its matrices)
    OA = O.PSparseMatrix(O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, next(it).copy()), OA.values),
                         OA.rows, OA.cols)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    pamd.mul_(y, A, x)
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    got = y.to_host()
    for p in parts.part_ids:
        assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV with the new values differs"



@pytest.mark.parametrize("rows,tri16", [(0, 1), (2, 1), (2, 0), (4, 1)])
def test_float32_rows_per_lane_equal_oracle(be, pamd, O, rows, tri16):
    """pa_tune("f32_rows"): Float32 SELL with 4 rows per lane (16 B packs,
    256-row slices), 2 (8 B packs, 128-row slices: the delta16 rows take the
    triple SELL) or auto (0, the default: 2 for a matrix made mostly of
    non-pattern slices, i.e. these Voronoi parts).  The layout never changes
    the terms or their order per row (SparseUtils.jl:176-185): bit-exact
    against the oracle; y and the ghosts of x compared per part."""
    N, nparts, dtype = BIG[0], 8, np.float32
    prev = {k: pamd._lib.tune(k, v) for k, v in {"f32_rows": rows, "spmv_tri16": tri16}.items()}
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        OA = _oracle(O, N, nparts, dtype)
        rng = np.random.default_rng(SEED + rows)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y, A, x)
        ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows, dtype)
        O.mul_(oy, OA, ox)
        got, gx = y.to_host(), x.to_host()
        for p in parts.part_ids:
            assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
            assert _eq(O, gx.local(p), ox.values[p]), f"part {p}: ghost values of x differ"
        want = {p: 256 if rows == 4 else 128 for p in parts.part_ids}
        if rows == 0:  # auto: 128-row slices where the 256-row build has < 80 % pattern slices
            pamd._lib.tune("f32_rows", 4)
            A4 = pamd.drivers.irregular_problem(parts, N, 27, dtype)
            for p in parts.part_ids:
                i4 = A4.values.local(p).info()
                want[p] = 128 if 5 * i4["pattern_slices"] < 4 * i4["nslices"] else 256
            pamd._lib.tune("f32_rows", 0)
        for p in parts.part_ids:
            i = A.values.local(p).info()
            assert i["nslices"] == (i["nrows"] + want[p] - 1) // want[p], (p, i)
            if want[p] == 128 and tri16 and i["tri_rows"] > 0:
                assert i["delta16_slices"] == 0, (p, i)
    finally:
        for k, v in prev.items():
            pamd._lib.tune(k, v)


@pytest.mark.parametrize("dtype,pack", [(np.float32, 7), (np.float32, 4), (np.float32, 1), (np.float32, 0),
                                        (np.float64, 7), (np.float64, 0), (np.complex64, 7), (np.complex64, 0)])
def test_triple_sell_packs_and_pairs_equal_oracle(be, pamd, O, dtype, pack):
    """pa_tune("spmv_tri_pack"): pair slices of the triple SELL (bit 2: rows
    a, a + 1 whose columns differ by one share a lane, one code and one x
    run per triple; Float32, Float64, ComplexF32), Float32 pair slices with
    a triple's values as one 16 B pack (entries 0 and 1 of both rows) and
    one 8 B pack (entry 2) per lane or one 8 B pack per entry (bit 0).  The layout never changes the terms or their order per row
    (SparseUtils.jl:176-185): mul! with alpha != 1 and beta != 0, and mul!
    after set_values (the copies refreshed into the packed layout), give the
    oracle's bits."""
    N, nparts = BIG[0], 8
    prev = {k: pamd._lib.tune(k, v) for k, v in {"f32_rows": 2, "spmv_tri16": 1, "spmv_tri_pack": pack}.items()}
    try:
        parts = be.get_part_ids(nparts)
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        info = [A.values.local(p).info() for p in parts.part_ids]
        assert sum(i["tri_rows"] for i in info) > 0
        # pairs hold most triple rows of these parts (x-neighbours inside a part)
        assert (sum(i["pair_rows"] for i in info) * 2 > sum(i["tri_rows"] for i in info)) == bool(pack & 4)
        OA = _oracle(O, N, nparts, dtype)
        rng = np.random.default_rng(SEED + 41 + pack)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        ys = {p: _rand(rng, A.rows.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], A.rows.partition), A.rows)
        a, b = (np.float32(0.5), np.float32(-1.25)) if np.dtype(dtype) in (np.float32, np.complex64) else (0.5, -1.25)
        pamd.mul_(y, A, x, a, b)
        ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
        oy = O.PVector(O.map_parts(lambda s: _ox(O, ys[s.part]), OA.rows.partition), OA.rows)
        O.mul_(oy, OA, ox, a, b)
        got = y.to_host()
        for p in parts.part_ids:
            assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV (alpha, beta) differs"
        new = []
        for i, p in enumerate(parts.part_ids):
            v2 = _rand(rng, len(A.values.local(p).get_values()), dtype)
            A.values.local(p).set_values(v2)
            new.append(v2)
        it = iter(new)
        OA = O.PSparseMatrix(O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, _ox(O, next(it))),
                                         OA.values), OA.rows, OA.cols)
        y = pamd.PVector.undef(A.rows, dtype)
        pamd.mul_(y, A, x)
        oy = O.pvector_undef(OA.rows, dtype)
        O.mul_(oy, OA, ox)
        got = y.to_host()
        for p in parts.part_ids:
            assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV after set_values differs"
    finally:
        for k, v in prev.items():
            pamd._lib.tune(k, v)


def test_float32_rows_auto_keeps_pattern_matrices(be, pamd):
    """f32_rows auto keeps 4 rows per lane for a matrix of pattern slices
    (the FE27 stencil: 2 would cost +14 %, profiles/r05/af/)."""
    parts = be.get_part_ids((1, 1, 1))
    N = (48, 40, 32)
    A = pamd.drivers.stencil_operator(parts, N, 27, np.float32)
    i = A.info().parts[0]
    assert i["pattern_slices"] * 2 >= i["nslices"], i
    assert i["nslices"] == (i["nrows"] + 255) // 256, i


@pytest.mark.parametrize("merge", [1, 0])
def test_float32_mixed_rows_per_lane_parts_equal_oracle(pamd, O, merge):
    """Parts of one Float32 matrix with different SELL layouts (pa_ctx_tune
    "f32_rows" 2 on even parts, 4 on odd ones: what auto gives when some
    parts are stencil-like): the merged launch runs one launch per layout,
    the per-kind launches runs of equal layout; bit-exact against the oracle."""
    be = pamd.HIPBackend(devices=[0])
    N, nparts, dtype = (30, 28, 26), 8, np.float32
    parts = be.get_part_ids(nparts)
    for p in parts.part_ids:
        be.context(p).tune("f32_rows", 2 if p % 2 == 0 else 4)
    prev = pamd._lib.tune("spmv_merge", merge)
    try:
        A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
        hs = {p: A.values.local(p).info() for p in parts.part_ids}
        for p, i in hs.items():
            h = 128 if p % 2 == 0 else 256
            assert i["nslices"] == (i["nrows"] + h - 1) // h, (p, i)
        OA = _oracle(O, N, nparts, dtype)
        rng = np.random.default_rng(SEED + 31)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
        for alpha in (1.0, 0.5):
            y = pamd.PVector.undef(A.rows, dtype)
            oy = O.pvector_undef(OA.rows, dtype)
            pamd.mul_(y, A, x, alpha, 0.0)
            O.mul_(oy, OA, ox, np.float32(alpha), 0.0)
            got = y.to_host()
            for p in parts.part_ids:
                assert _eq(O, got.local(p), oy.values[p]), f"part {p}, alpha {alpha}: SpMV differs"
    finally:
        pamd._lib.tune("spmv_merge", prev)
