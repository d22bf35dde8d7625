"""GPU parity tests: the HIP path (through the C-ABI) against the CPU oracle on
the same seeded inputs.  Bit-exact for SpMV (the device kernel reproduces the
reference's per-row summation order), exchange! and assemble!; 1e-12
relative for dot/norm (local BLAS order is not pinned by the reference)."""
import subprocess
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 20250114


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    return pamd.HIPBackend(devices=[0])


@pytest.fixture(params=[1, 0], ids=["pattern", "int32"])
def fmt(request, pamd, be):
    """Run a test with both column encodings (pa_tune spmv_format)."""
    prev = pamd._lib.tune("spmv_format", request.param)
    yield request.param
    pamd._lib.tune("spmv_format", prev)


@pytest.fixture(params=[1, 0], ids=["pull", "copies"])
def halo(request, pamd, be):
    """Run a test with both in-process halo transports (pa_tune halo_pull):
    receivers read the senders' buffers in one kernel, or staging copies."""
    prev = pamd._lib.tune("halo_pull", request.param)
    yield request.param
    pamd._lib.tune("halo_pull", prev)


def _rand(rng, n, dtype):
    dtype = np.dtype(dtype)
    if dtype.kind == "c":
        return (rng.uniform(-1, 1, n) + 1j * rng.uniform(-1, 1, n)).astype(dtype)
    return rng.uniform(-1, 1, n).astype(dtype)


def _to_oracle(O, a):
    if np.iscomplexobj(a):
        return O.Cx(a.real.copy(), a.imag.copy())
    return a.copy()


def _eq(O, got, ref):
    if isinstance(ref, O.Cx):
        return np.array_equal(got.real, ref.re) and np.array_equal(got.imag, ref.im)
    return np.array_equal(got, ref)


def _sel(O, ref, idx):
    return O.Cx(ref.re[idx], ref.im[idx]) if isinstance(ref, O.Cx) else ref[idx]


CASES = [
    ((1, 1, 1), (7, 6, 5), 27, np.float64),
    ((2, 2, 1), (12, 10, 9), 27, np.float64),
    ((2, 2, 2), (9, 9, 9), 27, np.float64),
    ((2, 1, 2), (11, 8, 10), 7, np.float64),
    ((2, 2, 2), (10, 10, 10), 7, np.float64),
    ((2, 2, 1), (12, 10, 9), 27, np.float32),
    ((2, 1, 1), (12, 10, 9), 27, np.complex128),
    ((1, 2, 2), (8, 12, 10), 27, np.complex64),
    ((3, 1, 1), (40, 5, 4), 27, np.float64),   # many slices, ragged last slice
]


@pytest.mark.parametrize("shape,N,kind,dtype", CASES)
def test_stencil_spmv_bitexact(be, pamd, O, fmt, halo, shape, N, kind, dtype):
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, kind, dtype)
    rng = np.random.default_rng(SEED)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    pamd.mul_(y, A, x)
    got = y.to_host()
    gx = x.to_host()
    oparts = O.get_part_ids(shape)
    OA = O.stencil_problem(oparts, N, kind, dtype)
    ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
        assert _eq(O, gx.local(p), ox.values[p]), f"part {p}: exchanged ghost values of b differ"


def test_csc_path_equals_stencil_generator(be, pamd, O, fmt):
    """pa_mat_from_csc of the oracle-assembled CSC == pa_mat_stencil."""
    shape, N, kind = (2, 2, 1), (12, 11, 7), 27
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, kind)
    OA = O.stencil_problem(O.get_part_ids(shape), N, kind)
    csc = pamd.PData(parts.backend, parts.part_ids,
                     [pamd.CSC(M.m, M.n, M.colptr, M.rowval, M.nzval) for M in OA.values.parts], parts.shape)
    B = pamd.PSparseMatrix.from_csc(csc, A.rows, A.cols)
    rng = np.random.default_rng(SEED)
    xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y1, y2 = pamd.PVector.undef(A.rows), pamd.PVector.undef(A.rows)
    pamd.mul_(y1, A, x)
    pamd.mul_(y2, B, x)
    for p in parts.part_ids:
        assert np.array_equal(y1.to_host().local(p), y2.to_host().local(p))
    i1, i2 = A.info(), B.info()
    for p in parts.part_ids:
        assert i1.local(p) == i2.local(p)


@pytest.mark.parametrize("alpha,beta", [(1.0, 1.0), (2.5, 0.5), (-1.0, 0.0), (0.75, -2.0)])
def test_alpha_beta(be, pamd, O, fmt, alpha, beta):
    shape, N = (2, 1, 2), (9, 7, 10)
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    rng = np.random.default_rng(SEED + 1)
    xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    ys = {p: rng.uniform(-1, 1, A.rows.partition.local(p).num_lids) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], A.rows.partition), A.rows)
    pamd.mul_(y, A, x, alpha, beta)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
    oy = O.PVector(O.map_parts(lambda s: ys[s.part].copy(), OA.rows.partition), OA.rows)
    O.mul_(oy, OA, ox, alpha, beta, literal=True)
    for p in parts.part_ids:
        assert np.array_equal(y.to_host().local(p), oy.values[p])


def test_exchange_assemble_bitexact(be, pamd, O, halo):
    shape, N = (2, 2, 2), (9, 8, 10)
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    rng = np.random.default_rng(SEED + 2)
    vs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    v = pamd.PVector.from_host(pamd.map_parts(lambda s: vs[s.part], A.cols.partition), A.cols)
    ov = O.PVector(O.map_parts(lambda s: vs[s.part].copy(), OA.cols.partition), OA.cols)
    pamd.exchange_(v)
    O.exchange_pvector_(ov)
    for p in parts.part_ids:
        assert np.array_equal(v.to_host().local(p), ov.values[p])
    vs2 = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
    w = pamd.PVector.from_host(pamd.map_parts(lambda s: vs2[s.part], A.cols.partition), A.cols)
    ow = O.PVector(O.map_parts(lambda s: vs2[s.part].copy(), OA.cols.partition), OA.cols)
    pamd.assemble_(w)
    O.assemble_(ow)
    for p in parts.part_ids:
        assert np.array_equal(w.to_host().local(p), ow.values[p])


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
def test_dot_norm_sum(be, pamd, O, dtype):
    shape, N = (2, 2, 1), (10, 9, 8)
    parts = be.get_part_ids(shape)
    rows, cols = pamd.drivers.stencil_partition(parts, N, 27)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    rng = np.random.default_rng(SEED + 3)
    a_ = {p: _rand(rng, cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    b_ = {p: _rand(rng, cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    a = pamd.PVector.from_host(pamd.map_parts(lambda s: a_[s.part], cols.partition), cols)
    b = pamd.PVector.from_host(pamd.map_parts(lambda s: b_[s.part], cols.partition), cols)
    oa = O.PVector(O.map_parts(lambda s: _to_oracle(O, a_[s.part]), OA.cols.partition), OA.cols)
    ob = O.PVector(O.map_parts(lambda s: _to_oracle(O, b_[s.part]), OA.cols.partition), OA.cols)
    tol = 1e-12 if np.dtype(dtype) in (np.float64, np.complex128) else 1e-6
    assert abs(pamd.dot(a, b) - O.dot(oa, ob)) <= tol * abs(O.dot(oa, ob)) + 1e-300
    assert abs(pamd.norm(a) - O.norm(oa)) <= tol * O.norm(oa)
    assert abs(pamd.psum(a) - O.psum_vector(oa)) <= tol * max(1.0, abs(O.psum_vector(oa)))


@pytest.mark.parametrize("nparts", [4, (2, 2, 2)])
def test_fdm_cg(be, pamd, O, fmt, nparts):
    """test_fdm.jl end to end on the device: CG converges to x̂ (test_fdm.jl:118)
    and follows the oracle's residual history."""
    parts = be.get_part_ids(nparts)
    A, b, x0, xh = pamd.drivers.fdm_problem(parts, 10)
    x = x0.copy()
    hist = []
    pamd.cg_(x, A, b, history=hist)
    d = pamd.map_parts(lambda u, v, s1, s2: u[s1.oid_to_lid - 1] - v[s2.oid_to_lid - 1],
                       x.to_host(), xh.to_host(), x.rows.partition, xh.rows.partition)
    err = sum(float(np.sum(t ** 2)) for t in d.parts) ** 0.5
    assert err < 1e-5
    oparts = O.get_part_ids(nparts)
    OA, ob, ox0, oxh = O.fdm_problem(oparts, 10)
    ox = O.PVector(O.map_parts(lambda v: v.copy(), ox0.values), ox0.rows)
    ohist = []
    O.cg_(ox, OA, ob, log=ohist)
    assert len(hist) == len(ohist)
    np.testing.assert_allclose(hist, ohist, rtol=1e-8)


def test_large_fe27_vs_c_oracle(be, pamd, O, fmt, tmp_path):
    """One part, 48³ FE27 (2.8 M nnz): bit-exact against oracle/build/spmv_ref."""
    ref = os.path.join(ROOT, "oracle", "build", "spmv_ref")
    if not os.path.exists(ref):
        pytest.skip("oracle/build/spmv_ref not built")
    n = 48
    parts = be.get_part_ids((1, 1, 1))
    A = pamd.drivers.stencil_operator(parts, (n, n, n), 27)
    x_ = np.random.default_rng(SEED + 4).uniform(-1, 1, n ** 3)
    x_.tofile(tmp_path / "x.bin")
    subprocess.run([ref, "--kind", "27", "--n", str(n), "--reps", "1", "--xin", str(tmp_path / "x.bin"),
                    "--yout", str(tmp_path / "y.bin")], check=True, capture_output=True)
    yref = np.fromfile(tmp_path / "y.bin")
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: x_, A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    pamd.mul_(y, A, x)
    assert np.array_equal(y.to_host().local(1), yref)


def test_shared_stream_parts(pamd, O):
    """HIPBackend(share_streams=True): the parts on one device share one
    stream pair; mul!, exchange!/assemble! and the device CG give the same
    bits as with a stream pair per part."""
    shape, N = (2, 2, 1), (12, 10, 9)
    out = {}
    for share in (False, True):
        be = pamd.HIPBackend(devices=[0], share_streams=share)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27)
        rng = np.random.default_rng(SEED + 4)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, x)
        w = x.copy()
        pamd.assemble_(w)
        b = x.copy()
        xs = pamd.PVector.undef(A.cols).fill_(0)
        h = []
        pamd.cg_(xs, A, b, reltol=0.0, maxiter=15, history=h, device=True)
        out[share] = ([v.copy() for v in y.to_host().parts], [v.copy() for v in w.to_host().parts],
                      [v.copy() for v in xs.to_host().parts], h)
    for k in range(3):
        for a, b in zip(out[False][k], out[True][k]):
            assert np.array_equal(a, b), k
    assert out[False][3] == out[True][3]


@pytest.mark.parametrize("alpha", [1.0, -2.5])
def test_beta_zero_overwrites_nan_inf(be, pamd, O, fmt, alpha):
    """β = 0 is fill!(c, 0), not c*0 (SparseUtils.jl:167-168, Interfaces.jl:
    2262-2263): NaN / ±Inf in the prior c do not leak, and rows without
    entries become +0.0 even where c held a negative value (c*0 = -0.0).
    Bitwise against the oracle (literal and vectorised), both encodings."""
    shape, N = (2, 1, 1), (9, 8, 7)
    parts = be.get_part_ids(shape)
    _, part = pamd.drivers.stencil_partition(parts, N, 27)
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    opart = OA.cols
    coo, empty = {}, {}
    for i, p in enumerate(parts.part_ids):
        M = OA.values.parts[i]
        s = part.partition.local(p)
        cols_of = np.repeat(np.arange(1, M.n + 1), np.diff(M.colptr))
        oid = np.zeros(s.num_lids, np.int64)
        oid[s.oid_to_lid - 1] = np.arange(1, s.num_oids + 1)
        keep = (oid[M.rowval - 1] % 5) != 0  # every 5th owned row (and all ghost rows) left empty
        coo[p] = (M.rowval[keep].copy(), cols_of[keep].copy(), np.asarray(M.nzval)[keep].copy())
        empty[p] = s.oid_to_lid[np.arange(1, s.num_oids + 1) % 5 == 0] - 1
    mk = lambda k: pamd.PData(parts.backend, parts.part_ids, [coo[p][k] for p in parts.part_ids], parts.shape)
    A = pamd.PSparseMatrix.from_coo(mk(0), mk(1), mk(2), part, part, ids="local")
    omk = lambda k: O.PData([coo[p][k].copy() for p in parts.part_ids], shape)
    OM = O.psparse_from_coo(omk(0), omk(1), omk(2), opart, opart, ids="local")
    rng = np.random.default_rng(SEED + 9)
    xs = {p: rng.uniform(-1, 1, part.partition.local(p).num_lids) for p in parts.part_ids}
    ys = {}
    for p in parts.part_ids:
        v = rng.uniform(-1, 1, part.partition.local(p).num_lids)
        v[0::4], v[1::4], v[2::4] = np.nan, np.inf, -np.inf
        v[empty[p]] = -1.0
        ys[p] = v
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], part.partition), part)
    y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], part.partition), part)
    pamd.mul_(y, A, x, alpha, 0.0)
    got = y.to_host()
    for literal in (True, False):
        ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), opart.partition), opart)
        oy = O.PVector(O.map_parts(lambda s: ys[s.part].copy(), opart.partition), opart)
        O.mul_(oy, OM, ox, alpha, 0.0, literal=literal)
        for p in parts.part_ids:
            own = part.partition.local(p).oid_to_lid - 1
            g, r = got.local(p)[own], oy.values[p][own]
            assert np.isfinite(g).all(), f"part {p}: NaN/Inf of the prior c leaked through β = 0"
            assert np.array_equal(g.view(np.uint64), r.view(np.uint64)), (p, literal)
            e = got.local(p)[empty[p]]
            assert np.array_equal(e.view(np.uint64), np.zeros(len(e), np.uint64)), "empty rows must be +0.0"


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128, np.complex64])
@pytest.mark.parametrize("flags", [1 | 8 | 16 | 32 | 64, 4 | 16, 1 | 4 | 8, 1 | 4 | 16 | 64])
def test_spmv_flag_variants_bitexact(be, pamd, O, dtype, flags):
    """spmv_flags variants (pattern rows' 16 B x runs off, non-temporal y
    stores on, tail batch / short-row kernels off, the tail batch off under
    Float64's ids-ahead loop): the same terms in the same order, so
    bit-exact against the oracle, alpha != 1 included."""
    prev = pamd._lib.tune("spmv_flags", flags)
    try:
        shape, N = (2, 1, 2), (13, 9, 10)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27, dtype)
        rng = np.random.default_rng(SEED + 9)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 27, dtype)
        for alpha in (1.0, 0.75):
            y = pamd.PVector.undef(A.rows, dtype)
            pamd.mul_(y, A, x, alpha, 0.0)
            ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xs[s.part]), OA.cols.partition), OA.cols)
            oy = O.pvector_undef(OA.rows, dtype)
            oa = np.float32(alpha) if np.dtype(dtype) in (np.float32, np.complex64) else alpha
            O.mul_(oy, OA, ox, oa, 0.0)
            got = y.to_host()
            for p in parts.part_ids:
                own = A.rows.partition.local(p).oid_to_lid - 1
                assert _eq(O, got.local(p)[own], _sel(O, oy.values[p], own)), (alpha, p)
    finally:
        pamd._lib.tune("spmv_flags", prev)


def test_threaded_issue_matches_sequential(pamd, O):
    """Parts with their own stream pairs issued from host threads (pa_tune
    issue_threads=2: always; the default 1 does so only across devices):
    mul! with α/β, the fused mul!+dot of the device CG and back-to-back
    calls on alternating x give the same bits as issue_threads=0 (one part
    after the other) and as the oracle."""
    shape, N = (2, 2, 2), (14, 11, 9)
    rng = np.random.default_rng(SEED + 9)
    vals = [rng.uniform(-1, 1, 3000) for _ in range(2)]
    out = {}
    for threads in (0, 2):
        prev = pamd._lib.tune("issue_threads", threads)
        try:
            be = pamd.HIPBackend(devices=[0], share_streams=False)
            parts = be.get_part_ids(shape)
            A = pamd.drivers.stencil_operator(parts, N, 27)
            xs = [pamd.PVector.from_host(pamd.map_parts(lambda s, v=v: v[:s.num_lids].copy(), A.cols.partition),
                                         A.cols) for v in vals]
            y = pamd.PVector.undef(A.rows).fill_(0.5)
            res = []
            for it in range(12):
                pamd.mul_(y, A, xs[it % 2], 1.0 if it % 3 else -2.0, 0.0 if it % 4 else 0.75)
                if it % 4 == 3:
                    res.append([v.copy() for v in y.to_host().parts])
            res.append([v.copy() for v in y.to_host().parts])
            xc = pamd.PVector.undef(A.cols).fill_(0)
            h = []
            pamd.cg_(xc, A, xs[0], reltol=0.0, maxiter=12, history=h, device=True)
            out[threads] = (res, [v.copy() for v in xc.to_host().parts], h)
            if threads == 2:
                y0 = pamd.PVector.undef(A.rows)
                pamd.mul_(y0, A, xs[0])
                OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
                ox = O.PVector(O.map_parts(lambda s: vals[0][:s.num_lids].copy(), OA.cols.partition), OA.cols)
                oy = O.pvector_undef(OA.rows, np.float64)
                O.mul_(oy, OA, ox)
                for p in parts.part_ids:
                    assert np.array_equal(y0.to_host().local(p), oy.values[p]), p
        finally:
            pamd._lib.tune("issue_threads", prev)
    for r0, r1 in zip(out[0][0], out[2][0]):
        for a, b in zip(r0, r1):
            assert np.array_equal(a, b)
    for a, b in zip(out[0][1], out[2][1]):
        assert np.array_equal(a, b)
    assert out[0][2] == out[2][2]


@pytest.mark.parametrize("threads", [0, 2])
def test_barrier_issue_chain_equals_oracle(pamd, O, threads):
    """Stream-pair mul! calls issued back to back without a host sync (the
    one-process-drives-several-GPUs path): with the pack
    barrier and double-buffered send buffers (halo_barrier 1) every call sees
    the x that was copied in just before it, as with per-neighbour waits
    (halo_barrier 0), with the pull on each part's compute stream
    (halo_barrier 2) and the oracle; an exchange! inside the sequence
    restarts the buffer chain; the device CG is bit-identical across all."""
    shape, N = (2, 2, 2), (14, 11, 9)
    rng = np.random.default_rng(SEED + 13)
    K = 9
    vals = [rng.uniform(-1, 1, 3000) for _ in range(K)]
    OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
    want = []
    for v in vals:
        ox = O.PVector(O.map_parts(lambda s, v=v: v[:s.num_lids].copy(), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows, np.float64)
        O.mul_(oy, OA, ox)
        want.append(oy)
    hist = {}
    for barrier in (1, 2, 0):
        p0 = pamd._lib.tune("issue_threads", threads)
        p1 = pamd._lib.tune("halo_barrier", barrier)
        try:
            be = pamd.HIPBackend(devices=[0], share_streams=False)
            parts = be.get_part_ids(shape)
            A = pamd.drivers.stencil_operator(parts, N, 27)
            xs = [pamd.PVector.from_host(pamd.map_parts(lambda s, v=v: v[:s.num_lids].copy(), A.cols.partition),
                                         A.cols) for v in vals]
            x = pamd.PVector.undef(A.cols).fill_(0)
            ys = [pamd.PVector.undef(A.rows).fill_(0) for _ in range(K)]
            for k in range(K):  # no host sync in between
                pamd.copyto_(x, xs[k])
                if k == 4:
                    pamd.exchange_(x)
                pamd.mul_(ys[k], A, x)
            for k in range(K):
                got = ys[k].to_host()
                for p in parts.part_ids:
                    own = A.rows.partition.local(p).oid_to_lid - 1
                    assert np.array_equal(got.local(p)[own], want[k].values[p][own]), (barrier, k, p)
            xc = pamd.PVector.undef(A.cols).fill_(0)
            h = []
            pamd.cg_(xc, A, xs[0], reltol=0.0, maxiter=10, history=h, device=True)
            hist[barrier] = (h, [v.copy() for v in xc.to_host().parts])
        finally:
            pamd._lib.tune("halo_barrier", p1)
            pamd._lib.tune("issue_threads", p0)
    for k in (1, 2):
        assert hist[0][0] == hist[k][0]
        for a, b in zip(hist[0][1], hist[k][1]):
            assert np.array_equal(a, b)


def test_threaded_issue_reports_launch_failures(pamd, O):
    """A kernel launch that fails inside a threaded-issue job (pa_tune
    fault_inject: each job also issues a launch the runtime rejects) makes
    mul! raise instead of returning with y unwritten, whichever thread ran
    the job (HIP keeps the last error per thread); the next
    call without the fault is correct (no sticky error on the workers)."""
    shape, N = (2, 2, 1), (10, 9, 8)
    prev = pamd._lib.tune("issue_threads", 2)
    try:
        be = pamd.HIPBackend(devices=[0], share_streams=False)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27)
        rng = np.random.default_rng(SEED + 11)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: rng.uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows).fill_(0.0)
        pamd._lib.tune("fault_inject", 1)
        try:
            with pytest.raises(pamd.PAError, match="issue job failed"):
                pamd.mul_(y, A, x)
        finally:
            pamd._lib.tune("fault_inject", 0)
        pamd.mul_(y, A, x)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
        ox = O.PVector(O.map_parts(lambda s: x.to_host().local(s.part).copy(), OA.cols.partition), OA.cols)
        oy = O.pvector_undef(OA.rows, np.float64)
        O.mul_(oy, OA, ox)
        for p in parts.part_ids:
            own = A.rows.partition.local(p).oid_to_lid - 1
            assert np.array_equal(y.to_host().local(p)[own], oy.values[p][own]), p
    finally:
        pamd._lib.tune("issue_threads", prev)


@pytest.mark.parametrize("kind,N,dtype", [(27, (40, 33, 9), np.float64), (7, (36, 30, 8), np.float64),
                                          (27, (34, 12, 10), np.float32), (27, (40, 9, 8), np.complex128)])
def test_dirichlet_side_rows_equal_oracle(be, pamd, O, kind, N, dtype):
    """Dirichlet rows (one entry, column == row) of pattern slices run as
    side rows (computing them inside their slice lost,
    profiles/r05/i/, and was removed in r06): mul! with α/β, the fused dot of
    the CG (mul_dot_) and β = 1 all give the oracle's bits."""
    if True:
        shape = (2, 1, 1)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, kind, dtype)
        OA = O.stencil_problem(O.get_part_ids(shape), N, kind, dtype)
        info = [A.values.local(p).info() for p in parts.part_ids]
        assert all(i["side_rows"] > 0 for i in info), info
        rng = np.random.default_rng(SEED + 41)
        xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        ys = {p: _rand(rng, A.rows.partition.local(p).num_lids, dtype) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xs[s.part]), OA.cols.partition), OA.cols)
        sc = np.float32 if np.dtype(dtype) in (np.float32, np.complex64) else np.float64
        for alpha, beta in ((1.0, 0.0), (0.7, 0.0), (1.0, 1.0), (-1.3, 0.5)):
            y = pamd.PVector.from_host(pamd.map_parts(lambda s: ys[s.part], A.rows.partition), A.rows)
            oy = O.PVector(O.map_parts(lambda s: _to_oracle(O, ys[s.part]), OA.rows.partition), OA.rows)
            pamd.mul_(y, A, x, alpha, beta)
            O.mul_(oy, OA, ox, sc(alpha), sc(beta))
            got = y.to_host()
            for p in parts.part_ids:
                own = A.rows.partition.local(p).oid_to_lid - 1
                assert _eq(O, got.local(p)[own], _sel(O, oy.values[p], own)), (alpha, beta, p)
        if np.dtype(dtype) == np.float64 and kind == 27:  # the CG's fused dot(x, A*x) over the owned rows
            xc = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part][:s.num_lids], A.cols.partition), A.cols)
            yc = pamd.PVector.undef(A.cols)
            d = pamd.mul_dot_(yc, A, xc)
            oyc = O.pvector_undef(OA.cols, np.float64)
            O.mul_(oyc, OA, ox)
            ref = 0.0
            for p in parts.part_ids:
                own = np.asarray(OA.cols.partition[p].oid_to_lid) - 1
                ref += float(np.dot(xs[p][own], oyc.values[p][own]))
            assert abs(d - ref) <= 1e-12 * max(1.0, abs(ref)), (d, ref)


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128])
@pytest.mark.parametrize("tail", [0, 1])
def test_side_rows_per_kind_launches_equal_oracle(be, pamd, O, dtype, tail):
    """Per-kind launches of one part (spmv_merge_max below its slice count:
    the headline's path) with the side rows as the pattern launch's trailing
    waves (spmv_side_tail 1) or as a launch after it (0): mul! with α/β, back
    to back on changing x without a host sync, and the fused dot give the
    oracle's bits; the side rows exist (the domain-face Dirichlet rows)."""
    p2 = pamd._lib.tune("spmv_side_tail", tail)
    p1 = pamd._lib.tune("spmv_merge_max", 4)
    try:
        shape, N = (1, 1, 1), (40, 21, 12)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27, dtype)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 27, dtype)
        assert A.values.local(1).info()["side_rows"] > 0
        rng = np.random.default_rng(SEED + 43)
        n = A.cols.partition.local(1).num_lids
        xs = [_rand(rng, n, dtype) for _ in range(3)]
        y0 = _rand(rng, A.rows.partition.local(1).num_lids, dtype)
        sc = np.float32 if np.dtype(dtype) in (np.float32, np.complex64) else np.float64
        cases = [(1.0, 0.0), (0.7, 0.0), (-1.3, 0.5)]
        xd = [pamd.PVector.from_host(pamd.map_parts(lambda s, v=v: v, A.cols.partition), A.cols) for v in xs]
        ys = [pamd.PVector.from_host(pamd.map_parts(lambda s: y0, A.rows.partition), A.rows) for _ in cases]
        for k, (alpha, beta) in enumerate(cases):  # no host sync in between
            pamd.mul_(ys[k], A, xd[k % 3], alpha, beta)
        for k, (alpha, beta) in enumerate(cases):
            ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xs[k % 3]), OA.cols.partition), OA.cols)
            oy = O.PVector(O.map_parts(lambda s: _to_oracle(O, y0), OA.rows.partition), OA.rows)
            O.mul_(oy, OA, ox, sc(alpha), sc(beta))
            own = A.rows.partition.local(1).oid_to_lid - 1
            assert _eq(O, ys[k].to_host().local(1)[own], _sel(O, oy.values[1], own)), (alpha, beta)
        if np.dtype(dtype) == np.float64:
            yc = pamd.PVector.undef(A.cols)
            d = pamd.mul_dot_(yc, A, xd[0])
            oyc = O.pvector_undef(OA.cols, np.float64)
            O.mul_(oyc, OA, O.PVector(O.map_parts(lambda s: xs[0].copy(), OA.cols.partition), OA.cols))
            ref = float(np.dot(xs[0], oyc.values[1]))
            assert abs(d - ref) <= 1e-12 * max(1.0, abs(ref)), (d, ref)
    finally:
        pamd._lib.tune("spmv_merge_max", p1)
        pamd._lib.tune("spmv_side_tail", p2)


@pytest.mark.parametrize("chunk", [1, 3, 5, 16, 64, -1])
def test_xcd_chunked_block_order_equals_round_robin(be, pamd, chunk):
    """spmv_xcd_chunk maps runs of C consecutive 4-slice blocks to one XCD
    (xcd_block, a bijection of the grid: blocks past the last full group of
    8C keep their order); per-kind launches (spmv_merge_max below the slice
    count) with any C, including ones that leave partial groups, and the auto
    value compute every slice exactly once: y equals the round robin's bit
    for bit, with α/β and the side rows as trailing waves."""
    p0 = pamd._lib.tune("spmv_merge_max", 4)
    try:
        shape, N = (1, 1, 1), (64, 60, 37)
        parts = be.get_part_ids(shape)
        rng = np.random.default_rng(SEED + 47)
        outs = {}
        for c in (0, chunk):
            p1 = pamd._lib.tune("spmv_xcd_chunk", c)
            try:
                A = pamd.drivers.stencil_operator(parts, N, 27)
                n = A.cols.partition.local(1).num_lids
                if c == 0:
                    xv = rng.uniform(-1, 1, n)
                    yv = rng.uniform(-1, 1, A.rows.partition.local(1).num_lids)
                x = pamd.PVector.from_host(pamd.map_parts(lambda s: xv.copy(), A.cols.partition), A.cols)
                res = []
                for alpha, beta in ((1.0, 0.0), (-0.7, 0.5)):
                    y = pamd.PVector.from_host(pamd.map_parts(lambda s: yv.copy(), A.rows.partition), A.rows)
                    pamd.mul_(y, A, x, alpha, beta)
                    res.append(y.to_host().local(1).copy())
                outs[c] = res
            finally:
                pamd._lib.tune("spmv_xcd_chunk", p1)
        for a, b in zip(outs[0], outs[chunk]):
            assert np.array_equal(a, b)
    finally:
        pamd._lib.tune("spmv_merge_max", p0)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_short_row_side_tail_equals_oracle(be, pamd, O, dtype):
    """The short-row kernels with the side rows as trailing waves: FD7
    (test_fdm's operator: 7-entry rows, the domain-face identity rows as side
    rows) in one-launch-per-kind mode (spmv_merge 0) runs its pattern slices
    and side rows as ONE short-row launch (k_spmv_sell_group SH + TAIL): mul!
    with α/β gives the oracle's bits."""
    p0 = pamd._lib.tune("spmv_merge", 0)
    try:
        shape, N = (1, 1, 1), (40, 33, 21)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 7, dtype)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 7, dtype)
        assert A.values.local(1).info()["side_rows"] > 0
        rng = np.random.default_rng(SEED + 49)
        xv = _rand(rng, A.cols.partition.local(1).num_lids, dtype)
        yv = _rand(rng, A.rows.partition.local(1).num_lids, dtype)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xv, A.cols.partition), A.cols)
        ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xv), OA.cols.partition), OA.cols)
        sc = np.float32 if np.dtype(dtype) == np.float32 else np.float64
        for alpha, beta in ((1.0, 0.0), (-1.3, 0.5)):
            y = pamd.PVector.from_host(pamd.map_parts(lambda s: yv, A.rows.partition), A.rows)
            oy = O.PVector(O.map_parts(lambda s: _to_oracle(O, yv), OA.rows.partition), OA.rows)
            pamd.mul_(y, A, x, alpha, beta)
            O.mul_(oy, OA, ox, sc(alpha), sc(beta))
            own = A.rows.partition.local(1).oid_to_lid - 1
            assert _eq(O, y.to_host().local(1)[own], _sel(O, oy.values[1], own)), (alpha, beta)
    finally:
        pamd._lib.tune("spmv_merge", p0)


@pytest.mark.parametrize("flags", [93, 221, 223])
@pytest.mark.parametrize("N", [(40, 33, 21), (128, 20, 9)])
def test_fd7_short_row_tail_launch_equals_oracle(be, pamd, O, flags, N):
    """One FD7 part (C2's path: the pattern slices and the side rows in ONE
    short-row tail launch, spmv_flags bit 7 = its Float64 batch-of-7 kernel
    at 7 waves per SIMD): mul! back to back on changing x, with α/β (those
    fall back to the 8-entry kernel), gives the oracle's bits."""
    prev = pamd._lib.tune("spmv_flags", flags)
    try:
        shape = (1, 1, 1)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 7)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 7)
        assert A.values.local(1).info()["side_rows"] > 0
        rng = np.random.default_rng(SEED + 53)
        n = A.cols.partition.local(1).num_lids
        xs = [rng.uniform(-1, 1, n) for _ in range(3)]
        y0 = rng.uniform(-1, 1, A.rows.partition.local(1).num_lids)
        cases = [(1.0, 0.0), (1.0, 0.0), (-1.3, 0.5)]
        xd = [pamd.PVector.from_host(pamd.map_parts(lambda s, v=v: v, A.cols.partition), A.cols) for v in xs]
        ys = [pamd.PVector.from_host(pamd.map_parts(lambda s: y0, A.rows.partition), A.rows) for _ in cases]
        for k, (alpha, beta) in enumerate(cases):  # no host sync in between
            pamd.mul_(ys[k], A, xd[k], alpha, beta)
        own = A.rows.partition.local(1).oid_to_lid - 1
        for k, (alpha, beta) in enumerate(cases):
            ox = O.PVector(O.map_parts(lambda s: xs[k].copy(), OA.cols.partition), OA.cols)
            oy = O.PVector(O.map_parts(lambda s: y0.copy(), OA.rows.partition), OA.rows)
            O.mul_(oy, OA, ox, alpha, beta)
            assert np.array_equal(ys[k].to_host().local(1)[own], oy.values[1][own]), (flags, alpha, beta)
    finally:
        pamd._lib.tune("spmv_flags", prev)


@pytest.mark.parametrize("uniform,flags", [(1, 223), (1, 255), (0, 223)])
@pytest.mark.parametrize("N", [(40, 33, 21), (128, 20, 9)])
def test_fd7_uniform_layout_equals_oracle(be, pamd, O, uniform, flags, N):
    """pa_tune("spmv_uniform"): an FD7 part's pattern slices (patterns of 5-7
    entries, all subsequences of the 7-point union) also stored at slice ·
    H · 7 in the union's entry order, so C2's short-row tail launch issues
    its value and x loads from the slice index alone.  mul! gives the
    oracle's bits with the layout on and off, and again after set_values
    (the copy refreshed); spmv_flags 255 adds the non-temporal y stores."""
    prev = pamd._lib.tune("spmv_uniform", uniform)
    prevf = pamd._lib.tune("spmv_flags", flags)
    try:
        shape = (1, 1, 1)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 7)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 7)
        rng = np.random.default_rng(SEED + 57)
        n = A.cols.partition.local(1).num_lids
        own = A.rows.partition.local(1).oid_to_lid - 1
        for rnd in range(2):
            if rnd == 1:  # test_fdm's operator (built from COO): new values through set_values
                A, _, _, _ = pamd.drivers.fdm_problem(parts, 24)
                OA, _, _, _ = O.fdm_problem(O.get_part_ids(shape), 24)
                assert A.values.local(1).info()["pattern_slices"] > 0
                v2 = rng.uniform(-1, 1, len(OA.values.parts[0].nzval))
                A.values.local(1).set_values(v2)
                OA = O.PSparseMatrix(O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, v2.copy()),
                                                 OA.values), OA.rows, OA.cols)
                n = A.cols.partition.local(1).num_lids
                own = A.rows.partition.local(1).oid_to_lid - 1
            xv = rng.uniform(-1, 1, n)
            x = pamd.PVector.from_host(pamd.map_parts(lambda s: xv, A.cols.partition), A.cols)
            y = pamd.PVector.undef(A.rows)
            pamd.mul_(y, A, x)
            ox = O.PVector(O.map_parts(lambda s: xv.copy(), OA.cols.partition), OA.cols)
            oy = O.pvector_undef(OA.rows)
            O.mul_(oy, OA, ox)
            assert np.array_equal(y.to_host().local(1)[own], oy.values[1][own]), (uniform, flags, rnd)
    finally:
        pamd._lib.tune("spmv_uniform", prev)
        pamd._lib.tune("spmv_flags", prevf)


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.complex128, np.complex64])
@pytest.mark.parametrize("flags", [221, 223])
def test_pattern_slice_descriptor_equals_oracle(be, pamd, O, dtype, flags):
    """One FE27 part (per-kind launches): the pattern slices' metadata read
    as one descriptor (spmv_flags bit 1: offset / H, length word and mask
    words, 32 B for 1-2 rows per lane, 64 B for Float32's 4) or from the
    three arrays gives the oracle's bits, on a grid whose boundary planes
    make several patterns and partial masks."""
    prev = pamd._lib.tune("spmv_flags", flags)
    try:
        shape, N = (1, 1, 1), (70, 19, 11)
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27, dtype)
        info = A.values.local(1).info()
        assert info["pattern_slices"] > 0 and info["side_rows"] > 0
        rng = np.random.default_rng(SEED + 61)
        xs = _rand(rng, A.cols.partition.local(1).num_lids, dtype)
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs, A.cols.partition), A.cols)
        OA = O.stencil_problem(O.get_part_ids(shape), N, 27, dtype)
        own = A.rows.partition.local(1).oid_to_lid - 1
        for alpha in (1.0, 0.75):
            y = pamd.PVector.undef(A.rows, dtype)
            pamd.mul_(y, A, x, alpha, 0.0)
            ox = O.PVector(O.map_parts(lambda s: _to_oracle(O, xs), OA.cols.partition), OA.cols)
            oy = O.pvector_undef(OA.rows, dtype)
            oa = np.float32(alpha) if np.dtype(dtype) in (np.float32, np.complex64) else alpha
            O.mul_(oy, OA, ox, oa, 0.0)
            assert _eq(O, y.to_host().local(1)[own], _sel(O, oy.values[1], own)), (flags, alpha)
    finally:
        pamd._lib.tune("spmv_flags", prev)
