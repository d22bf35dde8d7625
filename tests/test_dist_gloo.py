"""The one-part-per-process path (MPIBackend's role) on CPU: world_size 2 and 4
over torch.distributed gloo.  Host collectives and the distributed setup of
the halo plan must give exactly what the in-process (Sequential) backend and
the oracle give.  (Device transport over RCCL needs GPUs)"""
import json
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "interfaces_kats.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, N, kind, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import pamd
        be = pamd.DistributedBackend()
        out = {}
        # collectives (test_interfaces.jl:65-123)
        parts = be.get_part_ids(world)
        out["sum"] = pamd.preduce(lambda a, b: a + b, parts, 0)
        a = pamd.map_parts(lambda p: [4, 2, 6, 3][p - 1], parts) if world == 4 else None
        if a is not None:
            out["xscan"] = pamd.xscan_all(lambda x, y: x + y, a, 1).parts[0]
            k = GOLD["exchange_scalar"]
            prcv = pamd.map_parts(lambda p: k["parts_rcv"][p - 1], parts)
            psnd = pamd.map_parts(lambda p: k["parts_snd"][p - 1], parts)
            data = pamd.map_parts(lambda s: [10 * i for i in s], psnd)
            out["exchange"] = pamd.exchange(data, prcv, psnd).parts[0]
            out["discover"] = [int(v) for v in pamd.discover_parts_snd(prcv).parts[0]]
            out["discover_gather"] = [int(v) for v in pamd.discover_parts_snd(prcv, method="gather").parts[0]]
            # a non-gloo host group (nccl): alltoall falls back to the object all-gather
            real = dist.get_backend
            dist.get_backend = lambda group=None: "nccl"
            try:
                out["discover_obj"] = [int(v) for v in pamd.discover_parts_snd(prcv).parts[0]]
            finally:
                dist.get_backend = real
        g = pamd.gather(pamd.map_parts(lambda p: 10 * p, parts))
        out["gather"] = g.parts[0]
        out["scatter"] = pamd.scatter(pamd.map_parts(lambda p: [p * 100 for p in range(1, world + 1)] if p == 1 else [], parts)).parts[0]
        # distributed setup of the stencil partition and its Exchanger
        parts = be.get_part_ids(shape)
        rows, cols = pamd.drivers.stencil_partition(parts, N, kind)
        p = parts.part_ids[0]
        s = cols.partition.local(p)
        ex = cols.exchanger
        out["part"] = p
        out["lid_to_gid"] = s.lid_to_gid.tolist()
        out["parts_rcv"] = ex.parts_rcv.local(p).tolist()
        out["parts_snd"] = ex.parts_snd.local(p).tolist()
        out["lids_rcv"] = ex.lids_rcv.local(p).tolist()
        out["lids_snd"] = ex.lids_snd.local(p).tolist()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


def _run(world, shape, N, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, shape, N, kind, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=240)
        res[r] = out
    for p in ps:
        p.join(timeout=60)
    for r, out in res.items():
        assert "error" not in out, out.get("error")
    return res


@pytest.mark.parametrize("world,shape,N,kind", [(2, (2, 1, 1), (10, 7, 6), 27), (4, (2, 2, 1), (9, 8, 7), 27),
                                                (4, (1, 2, 2), (6, 9, 8), 7)])
def test_distributed_setup_matches_sequential(pamd, O, world, shape, N, kind):
    res = _run(world, shape, N, kind)
    seq = pamd.sequential.get_part_ids(shape)
    rows, cols = pamd.drivers.stencil_partition(seq, N, kind)
    OA = O.stencil_problem(O.get_part_ids(shape), N, kind)
    for r in range(world):
        out = res[r]
        p = out["part"]
        assert p == r + 1
        assert out["sum"] == world * (world + 1) // 2
        assert out["gather"] == ([10 * q for q in range(1, world + 1)] if p == 1 else [])
        assert out["scatter"] == 100 * p
        if world == 4:
            assert out["xscan"] == GOLD["scan"]["xscan_init1"]
            assert out["exchange"] == GOLD["exchange_scalar"]["expected_rcv"][r]
            assert out["discover"] == GOLD["discover"]["expected_parts_snd"][r]
            assert out["discover_gather"] == GOLD["discover"]["expected_parts_snd"][r]
            assert out["discover_obj"] == GOLD["discover"]["expected_parts_snd"][r]
        s = cols.partition.local(p)
        assert out["lid_to_gid"] == s.lid_to_gid.tolist() == OA.cols.partition[p].lid_to_gid
        assert out["parts_rcv"] == cols.exchanger.parts_rcv.local(p).tolist()
        assert out["parts_snd"] == cols.exchanger.parts_snd.local(p).tolist() == list(OA.cols.exchanger.parts_snd[p])
        assert out["lids_rcv"] == cols.exchanger.lids_rcv.local(p).tolist()
        assert out["lids_snd"] == cols.exchanger.lids_snd.local(p).tolist() == OA.cols.exchanger.lids_snd[p].tolist()


def _fail_if(p, fail_part):
    if p == fail_part:
        raise AssertionError("boom")  # test_exception.jl: one part's @assert fails
    return p


def _worker_timer_abort(rank, world, port, fail_part, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import time
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pamd

    def driver(parts):
        t = pamd.PTimer(parts)
        t.tic_(barrier=True)
        time.sleep(0.01 * parts.part_ids[0])
        t.toc_("sleep")
        q.put((rank, "timer", t.data))
        if fail_part:
            pamd.map_parts(lambda p: _fail_if(p, fail_part), parts)
            pamd.preduce(lambda a, b: a + b, parts, 0)
        return True
    pamd.prun(driver, pamd.DistributedBackend(), world)
    q.put((rank, "done", None))
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_part", [0, 2])
def test_ptimer_and_prun_abort(fail_part):
    """PTimer min/max/avg over 4 processes on MAIN (PTimers.jl:40-59); with a
    failing part every process exits (non-zero) instead of hanging
    (MPIBackend.jl:21-36, test_exception.jl)."""
    world = 4
    ctx = mp.get_context("spawn")
    # SimpleQueue: put() writes to the pipe before returning, so a rank that
    # aborts (os._exit) right after sending still delivers its message
    q = ctx.SimpleQueue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_timer_abort, args=(r, world, port, fail_part, q)) for r in range(world)]
    for p in ps:
        p.start()
    msgs = []
    import time
    t_end = time.time() + 120
    while time.time() < t_end and any(p.is_alive() for p in ps):
        while not q.empty():
            msgs.append(q.get())
        time.sleep(0.1)
    for p in ps:
        p.join(timeout=10)
    while not q.empty():
        msgs.append(q.get())
    assert all(p.exitcode is not None for p in ps), "a rank hung"
    timers = {r: d for r, k, d in msgs if k == "timer"}
    assert set(timers) == set(range(world))
    d = timers[0]["sleep"]
    assert d["min"] >= 0.009 and d["max"] >= 0.039 and d["min"] <= d["avg"] <= d["max"]
    assert all(timers[r] == {} for r in range(1, world))
    if fail_part:
        assert all(p.exitcode != 0 for p in ps)
    else:
        assert all(p.exitcode == 0 for p in ps)
        assert sorted(r for r, k, _ in msgs if k == "done") == list(range(world))


def test_ptimer_sequential(pamd):
    parts = pamd.sequential.get_part_ids(3)
    t = pamd.PTimer(parts)
    t.tic_()
    t.toc_("a")
    t.toc_("b")
    d = t.data
    assert set(d) == {"a", "b"} and all(v["min"] == v["max"] == v["avg"] for v in d.values())
    assert "Section" in t.report()


def _worker_segments(rank, world, port, shape, N, kind, q):
    """one part per process: the halo messages its RCCL group would post
    (pa_api.cpp transport(): forward = exchange!, reverse = assemble!), as
    (peer part, element count, gids in buffer order) per send and receive"""
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import pamd
        be = pamd.DistributedBackend()
        parts = be.get_part_ids(shape)
        _, cols = pamd.drivers.stencil_partition(parts, N, kind)
        p = parts.part_ids[0]
        s = cols.partition.local(p)
        ex = cols.exchanger

        def segs(part_list, table):
            out = []
            for k, peer in enumerate(part_list.local(p)):
                lids = table.local(p)[k + 1]  # Table segment k (1-based), Helpers.jl:63-94
                out.append((int(peer), len(lids), s.lid_to_gid[np.asarray(lids) - 1].tolist()))
            return out
        fwd_snd, fwd_rcv = segs(ex.parts_snd, ex.lids_snd), segs(ex.parts_rcv, ex.lids_rcv)
        # reverse(exchanger) (Interfaces.jl:796-798): rcv and snd swap
        msgs = {"fwd": (fwd_snd, fwd_rcv), "rev": (fwd_rcv, fwd_snd)}
        allm = [None] * world
        dist.all_gather_object(allm, (p, msgs))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, allm))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


@pytest.mark.parametrize("world,shape", [(2, (2, 1, 1)), (4, (2, 2, 1)), (8, (2, 2, 2))])
def test_rccl_segment_pairing(world, shape):
    """The grouped ncclSend/ncclRecv of the halo (pa_api.cpp transport(),
    MPIBackend.jl:261-309) relies on every message being posted on both
    sides with the same length — SequentialBackend.jl:187's check — and on
    the sender's packed values being the receiver's ghosts in the same
    order.  Every ordered pair of ranks of the (2,1,1), (2,2,1), (2,2,2)
    partitions, forward (exchange!) and reverse (assemble!), over gloo."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    N, kind = (11, 9, 8), 27
    ps = [ctx.Process(target=_worker_segments, args=(r, world, port, shape, N, kind, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, out = q.get(timeout=300)
        res[r] = out
    for p in ps:
        p.join(timeout=60)
    for r, out in res.items():
        assert not isinstance(out, dict), out.get("error")
    allm = dict(res[0])  # part -> messages, identical on every rank
    assert all(dict(res[r]) == allm for r in res)
    npairs = 0
    for direction in ("fwd", "rev"):
        for a, msgs in allm.items():
            for peer, cnt, gids in msgs[direction][0]:
                rcv_b = [m for m in allm[peer][direction][1] if m[0] == a]
                assert len(rcv_b) == 1, f"{direction}: part {peer} posts {len(rcv_b)} receives from part {a}"
                _, cnt_b, gids_b = rcv_b[0]
                assert cnt == cnt_b, f"{direction}: {a}->{peer} sends {cnt}, receiver expects {cnt_b}"
                assert gids == gids_b, f"{direction}: {a}->{peer} packs other gids than the receiver unpacks"
                npairs += cnt > 0
        for b, msgs in allm.items():  # no receive without its send
            for peer, cnt, _ in msgs[direction][1]:
                assert any(m[0] == b for m in allm[peer][direction][0]), f"{direction}: {b} waits on {peer}"
    n_nbrs = {2: 1, 4: 3, 8: 7}[world]
    assert npairs == 2 * world * n_nbrs  # every part talks to all others, both directions


def _worker_cg_agree(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import pamd

        def allreduce_max(v):
            t = torch.tensor(v, dtype=torch.float32)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return t.tolist()
        # rank-local batch times (ms per iteration: sweep, fused) whose local
        # choices disagree: rank 0 alone would keep the sweep, rank 1 the
        # fused update; the max over the ranks is (3.0, 2.5): fused for all
        local = [[1.0, 2.0], [3.0, 2.5], [2.0, 2.2], [0.5, 0.4]][rank]
        out = {"local": pamd._lib.cg_variant_agree(local),
               "agreed": pamd._lib.cg_variant_agree(local, allreduce_max),
               "invalid": pamd._lib.cg_variant_agree([0.0, 1.0], allreduce_max),
               # rank 0's part cannot fuse (e.g. its Voronoi part took the
               # triple SELL): no rank may
               "fuse_local": pamd._lib.cg_fuse_agree(rank != 0),
               "fuse_agreed": pamd._lib.cg_fuse_agree(rank != 0, allreduce_max),
               "fuse_all": pamd._lib.cg_fuse_agree(True, allreduce_max)}
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 4])
def test_cg_variant_agreement_over_ranks(world):
    """The device CG's auto u-update choice with one part per process
    (VERDICT r04 item 7): each rank times its own two batches, the library
    reduces them with max over the ranks (RCCL in pa_cg_solve_all; here the
    same decision through pa_cg_variant_agree with a gloo all-reduce), and
    every rank keeps the same variant even where its local times disagree;
    without a valid time on any rank there is no choice (-1) on all.  The
    fused variant runs at all only if every rank's part allows it
    (pa_cg_fuse_agree): one rank with long rows or a triple
    SELL keeps every rank on the sweep."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_cg_agree, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r, out in res.items():
        assert "error" not in out, out.get("error")
    assert res[0]["local"] == 0 and res[1]["local"] == 1
    assert {res[r]["agreed"] for r in range(world)} == {1}
    assert {res[r]["invalid"] for r in range(world)} == {-1}
    assert res[0]["fuse_local"] is False and all(res[r]["fuse_local"] for r in range(1, world))
    assert {res[r]["fuse_agreed"] for r in range(world)} == {False}
    assert {res[r]["fuse_all"] for r in range(world)} == {True}


def _worker_device_guard(rank, world, port, q):
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        import pamd
        be = pamd.backends.DistributedBackend()
        out = {"distinct": be.assert_distinct_devices(f"0000:{rank + 1:02x}:00.0")}
        try:  # ranks 0 and 1 on the same device: every rank raises
            be.assert_distinct_devices("0000:01:00.0" if rank < 2 else f"0000:{rank + 1:02x}:00.0")
            out["folded"] = "no error"
        except RuntimeError as e:
            out["folded"] = str(e)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, out))
    except Exception as e:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, {"error": repr(e) + traceback.format_exc()}))


@pytest.mark.parametrize("world", [2, 3])
def test_one_device_per_rank_guard(world):
    """One GPU per process: HIPDistributedBackend
    gathers every rank's device key (PCI bus id) and raises on every rank
    when two ranks share a device (LOCAL_RANK wrapped onto fewer visible
    GPUs), instead of timing a folded run; distinct keys come back in rank
    order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_device_guard, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for r, out in res.items():
        assert "error" not in out, out.get("error")
        assert out["distinct"] == [f"0000:{k + 1:02x}:00.0" for k in range(world)]
        assert "one GPU per process" in out["folded"], out["folded"]
