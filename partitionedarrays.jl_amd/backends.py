"""Backends and partitioned data (the reference's L1/L2 plugin layer).

`AbstractBackend` / `AbstractPData` (Interfaces.jl:12, 50) with the two
process models of the reference:

* `SequentialBackend` (SequentialBackend.jl): every part in this process.
  With HIP parts this is "one process drives several parts/GPUs"; halo
  traffic between its parts is device-to-device copies.
* `MPIBackend` role → `DistributedBackend` (MPIBackend.jl): one part per
  process (`torch.distributed` rank = part-1).  Host-side collectives of the
  setup phase go over a gloo group; device halo traffic goes over RCCL
  (libpa_hip.so, pa_comm_init_rank).

Only host data (ids, ptrs, small scalars) flows through these collectives;
vector/matrix values stay on the device (pvector.py).
"""
from __future__ import annotations

import numpy as np

MAIN = 1  # Interfaces.jl:104


class PData:
    """An AbstractPData{T,N}: `parts` are the values of the parts held by this
    process (`part_ids`, 1-based), `shape` the Cartesian shape of the whole
    partition."""

    __slots__ = ("backend", "part_ids", "parts", "shape")

    def __init__(self, backend, part_ids, parts, shape):
        self.backend = backend
        self.part_ids = list(part_ids)
        self.parts = list(parts)
        self.shape = tuple(shape)
        assert len(self.parts) == len(self.part_ids)

    def __len__(self):  # Base.length(::AbstractPData) = prod(size)
        return int(np.prod(self.shape))

    @property
    def num_parts(self):
        return int(np.prod(self.shape))

    def __iter__(self):  # Base.iterate over parts (tuple destructuring)
        return iter(self.parts)

    def local(self, part):
        return self.parts[self.part_ids.index(part)]

    def __repr__(self):
        return f"PData({dict(zip(self.part_ids, self.parts))})"


def num_parts(a: PData) -> int:
    return a.num_parts


def map_parts(task, *args: PData) -> PData:
    """map_parts (SequentialBackend.jl:52-58, MPIBackend.jl): apply per local part."""
    a0 = args[0]
    for a in args[1:]:
        if a.part_ids != a0.part_ids:
            raise ValueError("map_parts: partitioned data over different parts")
    return PData(a0.backend, a0.part_ids, [task(*xs) for xs in zip(*[a.parts for a in args])], a0.shape)


def unzip(a: PData, k: int):
    return tuple(PData(a.backend, a.part_ids, [p[i] for p in a.parts], a.shape) for i in range(k))


def get_part_ids(a) -> PData:
    """get_part_ids(b, nparts) or get_part_ids(::AbstractPData) (Interfaces.jl:84)"""
    if isinstance(a, PData):
        return PData(a.backend, a.part_ids, list(a.part_ids), a.shape)
    raise TypeError("use backend.get_part_ids(nparts)")


class AbstractBackend:
    def get_part_ids(self, nparts) -> PData:
        raise NotImplementedError

    # -- host collectives (Interfaces.jl:127-219) ---------------------------
    def gather(self, snd: PData) -> PData:
        raise NotImplementedError

    def gather_all(self, snd: PData) -> PData:
        raise NotImplementedError

    def scatter(self, snd: PData) -> PData:
        raise NotImplementedError

    def exchange(self, data_snd: PData, parts_rcv: PData, parts_snd: PData) -> PData:
        """Allocating point-to-point exchange: part p sends data_snd[p][j] to
        parts_snd[p][j] and receives, in parts_rcv[p] order, the messages sent
        to it (Interfaces.jl:377-450; delivery rule SequentialBackend.jl:126-200)."""
        raise NotImplementedError

    def alltoall(self, snd: PData) -> PData:
        """Part p holds one int per part (snd[p][q-1] is for part q); part q
        receives the column [snd[p][q-1] for p = 1..P] (MPI_Alltoall of one
        int: the scalable discovery of parts_snd, prange.discover_parts_snd)."""
        raise NotImplementedError

    def i_am_main(self, a: PData) -> bool:
        return MAIN in a.part_ids

    def barrier(self):
        pass


def _shape_of(nparts):
    if isinstance(nparts, tuple):
        return nparts, int(np.prod(nparts))
    return (int(nparts),), int(nparts)


class SequentialBackend(AbstractBackend):
    """SequentialBackend.jl:1-200 — all parts in this process."""

    def get_part_ids(self, nparts) -> PData:
        shape, n = _shape_of(nparts)
        ids = list(range(1, n + 1))
        return PData(self, ids, ids, shape)

    def gather(self, snd):
        return PData(self, snd.part_ids,
                     [list(snd.parts) if p == MAIN else [] for p in snd.part_ids], snd.shape)

    def gather_all(self, snd):
        return PData(self, snd.part_ids, [list(snd.parts) for _ in snd.parts], snd.shape)

    def scatter(self, snd):
        v = snd.local(MAIN)
        if len(v) != snd.num_parts:
            raise ValueError("scatter: MAIN must hold one value per part")
        return PData(self, snd.part_ids, list(v), snd.shape)

    def alltoall(self, snd):
        P = snd.num_parts
        rows = [np.asarray(snd.local(p), dtype=np.int64) for p in range(1, P + 1)]
        if any(len(r) != P for r in rows):
            raise ValueError("alltoall: every part must hold one value per part")
        return PData(self, snd.part_ids, [np.array([r[q - 1] for r in rows], dtype=np.int64)
                                          for q in snd.part_ids], snd.shape)

    def exchange(self, data_snd, parts_rcv, parts_snd):
        out = []
        for p, prcv in zip(parts_rcv.part_ids, parts_rcv.parts):
            r = []
            for q in prcv:
                lst = list(parts_snd.local(q))
                if lst.count(p) != 1:  # _check_rcv_and_snd_match, SequentialBackend.jl:154-165
                    raise ValueError(f"exchange: part {q} does not send exactly once to part {p}")
                r.append(data_snd.local(q)[lst.index(p)])
            out.append(r)
        return PData(self, parts_rcv.part_ids, out, parts_rcv.shape)


class DistributedBackend(AbstractBackend):
    """MPIBackend.jl's role: one part per process over torch.distributed.

    The process group must be initialised (gloo, or nccl with a gloo
    side-group for host objects); part = rank+1, nparts = world size.
    """

    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("DistributedBackend needs torch.distributed initialised")
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)

    def get_part_ids(self, nparts) -> PData:
        shape, n = _shape_of(nparts)
        if n != self.size:  # MPIBackend.jl:11,17: Comm_size == prod(nparts)
            raise ValueError(f"nparts={n} must equal the number of processes ({self.size})")
        return PData(self, [self.rank + 1], [self.rank + 1], shape)

    def assert_distinct_devices(self, device_key):
        """One GPU per process: every rank's device key (the PCI bus id of its
        context's device) must differ from the others'.  A LOCAL_RANK wrapped
        onto fewer visible devices would fold several ranks onto one GPU and
        time another machine than the one reported (the
        reference's Comm_size == prod(nparts) check, MPIBackend.jl:11,17,61,
        has the same purpose).  Returns every rank's key, in rank order."""
        keys = self._all_gather(device_key)
        if len(set(keys)) < self.size:
            raise RuntimeError(f"{self.size} ranks run on {len(set(keys))} distinct device(s) "
                               f"{sorted(set(keys))}: one GPU per process is required")
        return keys

    def _all_gather(self, obj):
        out = [None] * self.size
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def gather(self, snd):
        allv = self._all_gather(snd.parts[0])
        return PData(self, snd.part_ids, [allv if self.rank + 1 == MAIN else []], snd.shape)

    def gather_all(self, snd):
        return PData(self, snd.part_ids, [self._all_gather(snd.parts[0])], snd.shape)

    def scatter(self, snd):
        v = snd.parts[0] if self.rank + 1 == MAIN else None
        objs = [v]
        self.dist.broadcast_object_list(objs, src=0, group=self.group)
        return PData(self, snd.part_ids, [objs[0][self.rank]], snd.shape)

    def alltoall(self, snd):
        import torch
        v = np.asarray(snd.parts[0], dtype=np.int64)
        if len(v) != self.size:
            raise ValueError("alltoall: every part must hold one value per part")
        if self.dist.get_backend(self.group) != "gloo":
            # nccl (or another device backend) as the host group: CPU tensors
            # cannot go through its all_to_all, so take the column from the
            # object all-gather (P ints from each part)
            allv = self._all_gather(v.tolist())
            return PData(self, snd.part_ids, [np.array([r[self.rank] for r in allv], dtype=np.int64)],
                         snd.shape)
        out = torch.empty(self.size, dtype=torch.int64)
        self.dist.all_to_all_single(out, torch.from_numpy(v.copy()), group=self.group)
        return PData(self, snd.part_ids, [out.numpy().astype(np.int64)], snd.shape)

    def exchange(self, data_snd, parts_rcv, parts_snd):
        me = self.rank + 1
        msgs = {int(q): d for q, d in zip(parts_snd.parts[0], data_snd.parts[0])}
        allm = self._all_gather(msgs)
        r = []
        for q in parts_rcv.parts[0]:
            m = allm[int(q) - 1]
            if me not in m:
                raise ValueError(f"exchange: part {q} does not send to part {me}")
            r.append(m[me])
        return PData(self, parts_rcv.part_ids, [r], parts_rcv.shape)

    def barrier(self):
        self.dist.barrier(group=self.group)


sequential = SequentialBackend()


def prun(driver, backend: AbstractBackend, nparts):
    """prun(driver, b, nparts) Interfaces.jl:33-36.  With one part per
    process an exception ends the whole job, as MPIBackend's prun does with
    MPI.Abort (MPIBackend.jl:21-36): this process exits at once, and the
    other ranks' pending collectives fail instead of waiting for it."""
    if not isinstance(backend, DistributedBackend):
        return driver(backend.get_part_ids(nparts))
    try:
        return driver(backend.get_part_ids(nparts))
    except BaseException:
        import os
        import sys
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(1)


# -- collectives over PData (Interfaces.jl:127-340) ---------------------------

def gather(a: PData) -> PData:
    return a.backend.gather(a)


def gather_all(a: PData) -> PData:
    return a.backend.gather_all(a)


def scatter(a: PData) -> PData:
    return a.backend.scatter(a)


def emit(a: PData) -> PData:
    """Interfaces.jl:205-219"""
    g = a.backend.gather_all(a)
    v = g.parts[0][MAIN - 1]
    return PData(a.backend, a.part_ids, [v for _ in a.parts], a.shape)


def _fold(op, v, init):
    acc = init
    for x in v:
        acc = op(acc, x)
    return acc


def reduce_main(op, a: PData, init) -> PData:
    """Interfaces.jl:221-224"""
    return map_parts(lambda v: _fold(op, v, init), gather(a))


def reduce_all(op, a: PData, init) -> PData:
    """Interfaces.jl:226-229"""
    return map_parts(lambda v: _fold(op, v, init), gather_all(a))


def preduce(op, a: PData, init):
    """Base.reduce(op, ::AbstractPData; init) Interfaces.jl:231-234 (get_main_part)"""
    return reduce_all(op, a, init).parts[0]


def psum(a: PData):
    return preduce(lambda x, y: x + y, a, 0)


def xscan_all(op, a: PData, init) -> PData:
    """Interfaces.jl:301-304, 330-340"""
    def scan(v):
        out, acc = [], init
        for x in v:
            out.append(acc)
            acc = op(acc, x)
        return out
    return map_parts(scan, gather_all(a))


def exchange(data_snd: PData, parts_rcv: PData, parts_snd: PData) -> PData:
    return data_snd.backend.exchange(data_snd, parts_rcv, parts_snd)


def alltoall(a: PData) -> PData:
    return a.backend.alltoall(a)


def i_am_main(a: PData) -> bool:
    return a.backend.i_am_main(a)
