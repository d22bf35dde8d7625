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
