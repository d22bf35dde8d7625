"""The RCCL halo transport (the MPIBackend role, MPIBackend.jl:261-309: one
ncclGroupStart/End of per-neighbour ncclSend/ncclRecv) exercised on ONE GPU.

HIPBackend(rccl=True) makes one RCCL rank per device (pa_comm_init_all); the
parts of a device share that rank, so every halo segment between them is a
grouped send to self, posted in (sender part, receiver part) order — the
same code that carries segments between GPUs or processes.  Results must be
bit-exact against the oracle and bit-identical to the device-read transport,
and pa_comm_stats must show that every ghost value crossed RCCL."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20250114


@pytest.fixture(scope="module")
def be(pamd):
    if pamd.device_count() == 0:
        pytest.fail("no HIP device visible: the GPU tests need the MI355X")
    prev = pamd._lib.tune("halo_transport", 0)
    yield pamd.HIPBackend(devices=[0], rccl=True)
    pamd._lib.tune("halo_transport", prev)


@pytest.fixture(scope="module")
def be_pull(pamd):
    return pamd.HIPBackend(devices=[0])


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


def _stats(pamd, parts):
    return {p: parts.backend.context(p).comm_stats() for p in parts.part_ids}


def _moved(before, after):
    sent = sum(after[p][0] - before[p][0] for p in after)
    recv = sum(after[p][1] - before[p][1] for p in after)
    return sent, recv


@pytest.mark.parametrize("shape,N,kind,dtype", [
    ((2, 2, 2), (9, 9, 9), 27, np.float64),
    ((2, 2, 1), (12, 10, 9), 27, np.float32),
    ((2, 1, 1), (12, 10, 9), 27, np.complex128),
    ((1, 2, 2), (8, 12, 10), 27, np.complex64),
    ((3, 1, 1), (40, 5, 4), 7, np.float64),
])
def test_rccl_spmv_bitexact(be, pamd, O, shape, N, kind, dtype):
    parts = be.get_part_ids(shape)
    A = pamd.drivers.stencil_operator(parts, N, kind, dtype)
    rng = np.random.default_rng(SEED)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    s0 = _stats(pamd, parts)
    pamd.mul_(y, A, x)
    got, gx = y.to_host(), x.to_host()
    sent, recv = _moved(s0, _stats(pamd, parts))
    # every ghost value of x arrived through RCCL, once
    nh = sum(A.cols.partition.local(p).num_hids for p in parts.part_ids)
    assert nh > 0 and recv == nh * np.dtype(dtype).itemsize and sent == recv
    OA = O.stencil_problem(O.get_part_ids(shape), N, kind, dtype)
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    for p in parts.part_ids:
        assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
        assert _eq(O, gx.local(p), ox.values[p]), f"part {p}: ghost values of x differ"


def test_rccl_exchange_assemble_bitexact(be, pamd, O):
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
    s0 = _stats(pamd, parts)
    pamd.assemble_(w)
    O.assemble_(ow)
    sent, recv = _moved(s0, _stats(pamd, parts))
    nh = sum(A.cols.partition.local(p).num_hids for p in parts.part_ids)
    assert sent == recv == nh * 8  # the reverse exchange sends every ghost back to its owner
    for p in parts.part_ids:
        assert np.array_equal(w.to_host().local(p), ow.values[p])


@pytest.mark.parametrize("N,nparts,dtype", [((24, 22, 20), 8, np.complex128), ((24, 22, 20), 12, np.float64),
                                            ((128, 128, 128), 8, np.float64)])
def test_rccl_irregular_bitexact(be, pamd, O, N, nparts, dtype):
    """C5 (Voronoi parts, irregular neighbour graph) through RCCL."""
    parts = be.get_part_ids(nparts)
    A = pamd.drivers.irregular_problem(parts, N, 27, dtype)
    OA = O.irregular_problem(O.get_part_ids(nparts), N, 27)
    if np.dtype(dtype) != np.float64:
        vals = O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, O._convert_values(M.nzval, dtype)),
                           OA.values)
        OA = O.PSparseMatrix(vals, OA.rows, OA.cols)
    rng = np.random.default_rng(SEED)
    xs = {p: _rand(rng, A.cols.partition.local(p).num_lids, dtype) for p in parts.part_ids}
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    s0 = _stats(pamd, parts)
    pamd.mul_(y, A, x)
    sent, recv = _moved(s0, _stats(pamd, parts))
    nh = sum(A.cols.partition.local(p).num_hids for p in parts.part_ids)
    assert recv == sent == nh * np.dtype(dtype).itemsize
    ox = O.PVector(O.map_parts(lambda s: _ox(O, xs[s.part]), OA.cols.partition), OA.cols)
    oy = O.pvector_undef(OA.rows, dtype)
    O.mul_(oy, OA, ox)
    got, gx = y.to_host(), x.to_host()
    for p in parts.part_ids:
        assert _eq(O, got.local(p), oy.values[p]), f"part {p}: SpMV differs"
        assert _eq(O, gx.local(p), ox.values[p]), f"part {p}: ghost values of x differ"


def test_rccl_equals_device_reads_c3(be, be_pull, pamd):
    """C3's (2,2,2) split of FE27 at 128³ per part (256³ total): the RCCL
    transport and the device-read transport give bit-identical y and x."""
    shape, N = (2, 2, 2), (256, 256, 256)
    out = []
    for b in (be, be_pull):
        parts = b.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, N, 27)
        rng = np.random.default_rng(SEED + 5)
        xs = {p: rng.uniform(-1, 1, A.cols.partition.local(p).num_lids) for p in parts.part_ids}
        x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        pamd.mul_(y, A, x)
        out.append((y.to_host(), x.to_host(), parts.part_ids))
        del A, x, y
    (y1, x1, ids), (y2, x2, _) = out
    for p in ids:
        assert np.array_equal(y1.local(p), y2.local(p)), f"part {p}: y differs between transports"
        assert np.array_equal(x1.local(p), x2.local(p)), f"part {p}: x differs between transports"


def test_rccl_device_cg_equals_device_reads(be, be_pull, pamd):
    """pa_cg_solve_all with every halo over RCCL == the device-read transport
    (same residual history bit for bit, same x)."""
    res = []
    for b in (be, be_pull):
        parts = b.get_part_ids((2, 2, 2))
        A, rhs, x0, _ = pamd.drivers.fdm_problem(parts, 12)
        x = x0.copy()
        h = []
        pamd.cg_(x, A, rhs, reltol=0.0, maxiter=12, history=h, fused=True, device=True)
        res.append((h, x.to_host(), parts.part_ids))
    (h1, x1, ids), (h2, x2, _) = res
    assert h1 == h2
    for p in ids:
        assert np.array_equal(x1.local(p), x2.local(p))


def test_rccl_needs_shared_streams(pamd):
    b = pamd.HIPBackend(devices=[0], share_streams=False, rccl=True)
    with pytest.raises(pamd.PAError):
        b.get_part_ids((2, 1, 1))


def test_one_part_per_process_rccl_reductions(be_pull, pamd):
    """HIPDistributedBackend (one part per process, pa_comm_init_rank) in a
    one-process world: dot/norm and the device CG take the RCCL all-gather
    path of the multi-process mode, and must equal HIPBackend's local fold
    bit for bit."""
    import socket
    import torch.distributed as dist
    own = not dist.is_initialized()
    if own:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        res = []
        for b in (pamd.HIPDistributedBackend(device=0), be_pull):
            parts = b.get_part_ids(1)
            A, rhs, x0, _ = pamd.drivers.fdm_problem(parts, 14)
            x = x0.copy()
            h = []
            pamd.cg_(x, A, rhs, reltol=0.0, maxiter=10, history=h, fused=True, device=True)
            h2 = []
            x2 = x0.copy()
            pamd.cg_(x2, A, rhs, reltol=0.0, maxiter=6, history=h2, fused=True)
            res.append((h, h2, pamd.dot(rhs, x), pamd.norm(x), x.to_host().local(1)))
        (a1, a2, d1, n1, x1), (b1, b2, d2, n2, xx) = res
        assert a1 == b1 and a2 == b2 and d1 == d2 and n1 == n2
        assert np.array_equal(x1, xx)
        # what the N > 1 bench line reports (config.rccl_halo): the
        # communicator's size and rank, the device, the librccl resolved
        bd = pamd.HIPDistributedBackend(device=0)
        bd.get_part_ids(1)
        info = bd.context(1).comm_info()
        assert info["ranks"] == 1 and info["rank"] == 0 and info["device"] == 0, info
        assert info["pci"] and bd.device_keys == [info["pci"]], (info, bd.device_keys)
        assert info["rccl_version"] > 0 and "rccl" in info["librccl"], info
    finally:
        if own:
            dist.destroy_process_group()


@pytest.mark.parametrize("nparts,ngids", [(4, 20000), ((2, 2, 2), (30, 28, 26))])
def test_rccl_coo_assemble_bitexact(be, pamd, O, nparts, ngids):
    """assemble!(I, J, V, rows) with every count and every (I, J, V) segment
    through RCCL (pa_coo_assemble_all's cross-process path), bit-exact
    against the oracle."""
    from test_gpu_coo_assemble import _check, _problem
    args = _problem(pamd, O, be, nparts, ngids, 12000, np.float64, SEED + 7)
    s0 = _stats(pamd, args[0])
    assert _check(pamd, O, *args) > 0
    sent, recv = _moved(s0, _stats(pamd, args[0]))
    assert sent == 0 and recv == 0  # the halo counters count mul!/exchange! segments only
