"""CPU oracle for the SpMV + halo hot path of PartitionedArrays.jl (v0.2.9).

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker
(or the CPU baseline timed beside the GPU).  The product path
(partitionedarrays.jl_amd/) never imports it.

This is a restatement of the reference's algorithms in Python/numpy, each
function citing the file:line of /root/reference it follows.  The reference
is pure Julia and no `julia` exists on this image, so it can
not be run; parity is pinned instead by the reference's own known-answer
tests (test/test_interfaces.jl, test/SparseUtilsTests.jl, test/test_fdm.jl,
test/test_fem_sa.jl), transcribed in tests/golden/ and checked by
tests/test_oracle_kats.py.

Conventions: ids are 1-based (Julia's), part ids 1..P, Tables keep Julia's
1-based `ptrs`.  Backend semantics are SequentialBackend's (all parts of a
partitioned datum in one Python list, in part order).

Arithmetic: float64/float32 numpy ops are IEEE single ops (no FMA), as
Julia's scalar loops.  Complex numbers are carried as (re, im) real arrays so
that products follow Julia's formula (re*re - im*im, re*im + im*re) exactly.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, List, Sequence

import numpy as np

MAIN = 1  # Interfaces.jl:104


# ---------------------------------------------------------------------------
# Helpers.jl:63-156 — Table (CSR of vectors) and ptr utilities

@dataclass
class Table:
    data: np.ndarray
    ptrs: np.ndarray  # int32, 1-based, length n+1

    def __len__(self):
        return len(self.ptrs) - 1

    def __getitem__(self, i):  # 1-based, Helpers.jl:73-82
        return self.data[self.ptrs[i - 1] - 1: self.ptrs[i] - 1]

    def tolist(self):
        return [list(self[i]) for i in range(1, len(self) + 1)]

    def copy(self):
        return Table(self.data.copy(), self.ptrs.copy())


def table_from(vv, dtype=np.int64) -> Table:
    """Table(a::AbstractArray{<:AbstractArray}) Helpers.jl:85-124"""
    counts = [len(v) for v in vv]
    ptrs = counts_to_ptrs(counts)
    data = np.zeros(int(ptrs[-1] - 1), dtype=dtype)
    k = 0
    for v in vv:
        for x in v:
            data[k] = x
            k += 1
    return Table(data, ptrs)


def length_to_ptrs_(ptrs):
    """Helpers.jl:126-131"""
    ptrs[0] = 1
    for i in range(len(ptrs) - 1):
        ptrs[i + 1] += ptrs[i]
    return ptrs


def counts_to_ptrs(counts):
    """Helpers.jl:133-141"""
    n = len(counts)
    ptrs = np.zeros(n + 1, dtype=np.int32)
    ptrs[1:] = counts
    return length_to_ptrs_(ptrs)


def ptrs_to_counts(ptrs):
    """Helpers.jl:143-149"""
    return np.diff(np.asarray(ptrs))


def rewind_ptrs_(ptrs):
    """Helpers.jl:151-156"""
    for i in range(len(ptrs) - 2, -1, -1):
        ptrs[i + 1] = ptrs[i]
    ptrs[0] = 1
    return ptrs


# ---------------------------------------------------------------------------
# SequentialBackend.jl + Interfaces.jl:1-340 — partitioned data and collectives

class PData:
    """SequentialData{T,N} (SequentialBackend.jl:20-22): all parts in a list."""

    def __init__(self, parts, shape=None):
        self.parts = list(parts)
        self.shape = tuple(shape) if shape is not None else (len(self.parts),)
        assert int(np.prod(self.shape)) == len(self.parts)

    def __len__(self):
        return len(self.parts)

    def __getitem__(self, part):  # get_part(a, part), 1-based
        return self.parts[part - 1]


def num_parts(a: PData) -> int:
    return len(a.parts)


def get_part_ids(nparts) -> PData:
    """get_part_ids(::SequentialBackend, nparts) SequentialBackend.jl:6-14"""
    if isinstance(nparts, tuple):
        return PData(list(range(1, int(np.prod(nparts)) + 1)), nparts)
    return PData(list(range(1, nparts + 1)))


def map_parts(task: Callable, *args: PData) -> PData:
    """SequentialBackend.jl:52-58"""
    assert len(args) > 0
    n = len(args[0].parts)
    assert all(len(a.parts) == n for a in args)
    return PData([task(*xs) for xs in zip(*[a.parts for a in args])], args[0].shape)


def unzip(a: PData, k: int):
    return tuple(PData([p[i] for p in a.parts], a.shape) for i in range(k))


def gather(snd: PData) -> PData:
    """gather (Interfaces.jl:131-168 + SequentialBackend.jl:73-92)"""
    np_ = num_parts(snd)
    return PData([list(snd.parts) if p == MAIN else [] for p in range(1, np_ + 1)], snd.shape)


def gather_all(snd: PData) -> PData:
    """Interfaces.jl:170-196 + SequentialBackend.jl:94-117"""
    return PData([list(snd.parts) for _ in snd.parts], snd.shape)


def scatter(snd: PData) -> PData:
    """SequentialBackend.jl:119-124"""
    v = snd.parts[MAIN - 1]
    assert len(v) == num_parts(snd)
    return PData(list(v), snd.shape)


def emit(snd: PData) -> PData:
    """Interfaces.jl:205-219"""
    v = snd.parts[MAIN - 1]
    return PData([v for _ in snd.parts], snd.shape)


def _julia_reduce(op, v, init):
    # Base.reduce with init: left fold ((init ⊕ v1) ⊕ v2) ⊕ …
    acc = init
    for x in v:
        acc = op(acc, x)
    return acc


def reduce_main(op, snd: PData, init) -> PData:
    """Interfaces.jl:221-224"""
    a = gather(snd)
    return map_parts(lambda i: _julia_reduce(op, i, init), a)


def reduce_all(op, snd: PData, init) -> PData:
    """Interfaces.jl:226-229"""
    return emit(reduce_main(op, snd, init))


def preduce(op, a: PData, init):
    """Base.reduce(op, ::AbstractPData; init) Interfaces.jl:231-234"""
    return reduce_main(op, a, init).parts[MAIN - 1]


def psum(a: PData):
    """Interfaces.jl:236-238"""
    return preduce(lambda x, y: x + y, a, 0)


def _iscan_local(op, b, init):
    """Interfaces.jl:280-288"""
    b = list(b)
    if len(b) != 0:
        b[0] = op(init, b[0])
    for i in range(len(b) - 1):
        b[i + 1] = op(b[i], b[i + 1])
    return b


def _xscan_local(op, b, init):
    """Interfaces.jl:330-340"""
    b = list(b)
    for i in range(len(b) - 1, 0, -1):
        b[i] = b[i - 1]
    if len(b) != 0:
        b[0] = init
    for i in range(len(b) - 1):
        b[i + 1] = op(b[i], b[i + 1])
    return b


def iscan(op, a: PData, init) -> PData:
    """Interfaces.jl:241-244"""
    b = map_parts(lambda b: _iscan_local(op, b, init), gather(a))
    return scatter(b)


def iscan_all(op, a: PData, init) -> PData:
    return emit(map_parts(lambda b: _iscan_local(op, b, init), gather(a)))


def xscan(op, a: PData, init) -> PData:
    """Interfaces.jl:291-294"""
    return scatter(map_parts(lambda b: _xscan_local(op, b, init), gather(a)))


def xscan_all(op, a: PData, init) -> PData:
    return emit(map_parts(lambda b: _xscan_local(op, b, init), gather(a)))


def _check_rcv_and_snd_match(parts_rcv: PData, parts_snd: PData):
    """SequentialBackend.jl:154-165"""
    for part in range(1, num_parts(parts_rcv) + 1):
        for i in parts_rcv[part]:
            assert sum(1 for k in parts_snd[i] if k == part) == 1
        for i in parts_snd[part]:
            assert sum(1 for k in parts_rcv[i] if k == part) == 1


def exchange_scalars(data_snd: PData, parts_rcv: PData, parts_snd: PData) -> PData:
    """Allocating exchange of one value per neighbour (Interfaces.jl:377-390 with
    the Sequential delivery rule SequentialBackend.jl:126-152)."""
    _check_rcv_and_snd_match(parts_rcv, parts_snd)
    out = []
    for part_rcv in range(1, num_parts(parts_rcv) + 1):
        r = []
        for part_snd in parts_rcv[part_rcv]:
            j = list(parts_snd[part_snd]).index(part_rcv)
            r.append(data_snd[part_snd][j])
        out.append(r)
    return PData(out, parts_rcv.shape)


def exchange_tables(data_snd: PData, parts_rcv: PData, parts_snd: PData) -> PData:
    """Allocating Table exchange (Interfaces.jl:404-450 → SequentialBackend.jl:167-200)."""
    n_snd = map_parts(lambda t: [int(x) for x in ptrs_to_counts(t.ptrs)], data_snd)
    n_rcv = exchange_scalars(n_snd, parts_rcv, parts_snd)
    out = []
    for part_rcv in range(1, num_parts(parts_rcv) + 1):
        ptrs = counts_to_ptrs(n_rcv[part_rcv])
        dt = data_snd[part_rcv].data.dtype
        data = np.zeros(int(ptrs[-1] - 1), dtype=dt)
        for i, part_snd in enumerate(parts_rcv[part_rcv]):
            j = list(parts_snd[part_snd]).index(part_rcv)
            src = data_snd[part_snd]
            assert ptrs[i + 1] - ptrs[i] == src.ptrs[j + 1] - src.ptrs[j]  # :187
            data[ptrs[i] - 1: ptrs[i + 1] - 1] = src.data[src.ptrs[j] - 1: src.ptrs[j + 1] - 1]
        out.append(Table(data, ptrs))
    return PData(out, parts_rcv.shape)


ERROR_DISCOVER_PARTS_SND = [False]  # Interfaces.jl:498


def _parts_rcv_to_parts_snd(parts_rcv: List[List[int]]):
    """Interfaces.jl:525-552: transpose the receive graph; sender j lists its
    receivers ascending (column-major nziterator over sparse(I,J,I))."""
    np_ = len(parts_rcv)
    snd = [set() for _ in range(np_)]
    for p in range(1, np_ + 1):
        for q in parts_rcv[p - 1]:
            snd[q - 1].add(p)
    return [sorted(s) for s in snd]


def discover_parts_snd(parts_rcv: PData, neighbors_snd: PData = None,
                       neighbors_rcv: PData = None) -> PData:
    """Interfaces.jl:471-496 (with neighbours) / 515-521 (gather based)."""
    if neighbors_snd is None:
        if ERROR_DISCOVER_PARTS_SND[0]:
            raise RuntimeError("[PartitionedArrays.jl] Using a non-scalable implementation"
                               " to discover reciprocal parts")  # :500-512
        main = gather(parts_rcv)
        snd_main = map_parts(lambda v: _parts_rcv_to_parts_snd(v) if v else [], main)
        return scatter(snd_main)
    if neighbors_rcv is None:
        neighbors_rcv = neighbors_snd
    parts = get_part_ids(parts_rcv.shape if len(parts_rcv.shape) > 1 else num_parts(parts_rcv))

    def tell(part, nrcv, prcv):
        d = {n: -1 for n in nrcv}
        for i in prcv:
            d[i] = part
        return [d[n] for n in nrcv]
    data_rcv = map_parts(tell, parts, neighbors_rcv, parts_rcv)
    data_snd = exchange_scalars(data_rcv, neighbors_snd, neighbors_rcv)
    return map_parts(lambda d: [x for x in d if x > 0], data_snd)


# ---------------------------------------------------------------------------
# Index sets: IndexSets.jl:215-421 and Interfaces.jl:566-696

class IndexSet:
    """IndexSet (IndexSets.jl:215-291).  IndexRange / ExtendedIndexRange share
    the same observable fields and are represented by this class too."""

    def __init__(self, part, lid_to_gid, lid_to_part, oid_to_lid=None, hid_to_lid=None):
        self.part = int(part)
        self.lid_to_gid = [int(g) for g in lid_to_gid]
        self.lid_to_part = [int(p) for p in lid_to_part]
        if oid_to_lid is None:  # IndexSets.jl:267-280
            oid_to_lid = [l + 1 for l, o in enumerate(self.lid_to_part) if o == self.part]
            hid_to_lid = [l + 1 for l, o in enumerate(self.lid_to_part) if o != self.part]
        self.oid_to_lid = [int(x) for x in oid_to_lid]
        self.hid_to_lid = [int(x) for x in hid_to_lid]
        # IndexSets.jl:254-256
        self.lid_to_ohid = [0] * len(self.lid_to_gid)
        for i, l in enumerate(self.oid_to_lid):
            self.lid_to_ohid[l - 1] = i + 1
        for i, l in enumerate(self.hid_to_lid):
            self.lid_to_ohid[l - 1] = -(i + 1)
        self.gid_to_lid = {g: l + 1 for l, g in enumerate(self.lid_to_gid)}  # :233-236

    def copy(self):
        return IndexSet(self.part, self.lid_to_gid, self.lid_to_part, self.oid_to_lid, self.hid_to_lid)

    num_lids = property(lambda s: len(s.lid_to_part))   # Interfaces.jl:568
    num_oids = property(lambda s: len(s.oid_to_lid))
    num_hids = property(lambda s: len(s.hid_to_lid))


def index_range(part, noids, firstgid, hid_to_gid=(), hid_to_part=()):
    """IndexRange(part, noids, firstgid[, hid_to_gid, hid_to_part]) IndexSets.jl:364-421"""
    lid_to_gid = list(range(firstgid, firstgid + noids)) + list(hid_to_gid)
    lid_to_part = [part] * noids + list(hid_to_part)
    oid_to_lid = list(range(1, noids + 1))
    hid_to_lid = list(range(noids + 1, noids + len(hid_to_gid) + 1))
    return IndexSet(part, lid_to_gid, lid_to_part, oid_to_lid, hid_to_lid)


def _add_gid_ghost(a: IndexSet, gid, part):
    """Interfaces.jl:595-603"""
    lid = a.num_lids + 1
    hid = a.num_hids + 1
    a.lid_to_gid.append(int(gid))
    a.lid_to_part.append(int(part))
    a.hid_to_lid.append(lid)
    a.lid_to_ohid.append(-hid)
    a.gid_to_lid[int(gid)] = lid


def add_gid_(a: IndexSet, gid, part):
    """add_gid!(a, gid, part) Interfaces.jl:579-584"""
    if part != a.part and gid not in a.gid_to_lid:
        _add_gid_ghost(a, gid, part)
    return a


def add_gids_parts_(a: IndexSet, i_to_gid, i_to_part):
    """Interfaces.jl:605-616"""
    for g, p in zip(i_to_gid, i_to_part):
        add_gid_(a, int(g), int(p))
    return a


def add_gids_owner_(gid_to_part, a: IndexSet, gids):
    """add_gids!(gid_to_part, a, gids) Interfaces.jl:586-592, 618-627: first touch"""
    for g in gids:
        g = int(g)
        if g not in a.gid_to_lid:
            _add_gid_ghost(a, g, gid_to_part(g))
    return a


def to_lids_(ids, a: IndexSet):
    """Interfaces.jl:629-636"""
    for i in range(len(ids)):
        ids[i] = a.gid_to_lid[int(ids[i])]
    return ids


def to_gids_(ids, a: IndexSet):
    """Interfaces.jl:638-645"""
    for i in range(len(ids)):
        ids[i] = a.lid_to_gid[int(ids[i]) - 1]
    return ids


def oids_are_equal_is(a: IndexSet, b: IndexSet):
    """Interfaces.jl:647-649"""
    return [a.lid_to_gid[l - 1] for l in a.oid_to_lid] == [b.lid_to_gid[l - 1] for l in b.oid_to_lid]


def hids_are_equal_is(a: IndexSet, b: IndexSet):
    """Interfaces.jl:651-653"""
    return [a.lid_to_gid[l - 1] for l in a.hid_to_lid] == [b.lid_to_gid[l - 1] for l in b.hid_to_lid]


def touched_hids(a: IndexSet, gids):
    """Interfaces.jl:670-696"""
    seen = set()
    out = []
    for g in gids:
        lid = a.gid_to_lid[int(g)]
        ohid = a.lid_to_ohid[lid - 1]
        if ohid < 0 and -ohid not in seen:
            seen.add(-ohid)
            out.append(-ohid)
    return out


# ---------------------------------------------------------------------------
# Exchanger (Interfaces.jl:698-961)

@dataclass
class Exchanger:
    parts_rcv: PData
    parts_snd: PData
    lids_rcv: PData  # of Table
    lids_snd: PData


def exchanger_from_ids(ids: PData, neighbors_snd=None, neighbors_rcv=None,
                       reuse_parts_rcv=False) -> Exchanger:
    """Exchanger(ids; reuse_parts_rcv) Interfaces.jl:723-786"""
    parts = get_part_ids(ids.shape if len(ids.shape) > 1 else num_parts(ids))
    parts_rcv = map_parts(lambda part, s: sorted({o for o in s.lid_to_part if o != part}), parts, ids)

    def rcv(part, s, prcv):
        owner_to_i = {o: i for i, o in enumerate(prcv)}
        counts = [0] * len(prcv)
        for o in s.lid_to_part:
            if o != part:
                counts[owner_to_i[o]] += 1
        ptrs = counts_to_ptrs(counts)
        dl = np.zeros(int(ptrs[-1] - 1), dtype=np.int32)
        dg = np.zeros(int(ptrs[-1] - 1), dtype=np.int64)
        cur = ptrs.copy()
        for lid0, o in enumerate(s.lid_to_part):
            if o != part:
                i = owner_to_i[o]
                p = cur[i] - 1
                dl[p] = lid0 + 1
                dg[p] = s.lid_to_gid[lid0]
                cur[i] += 1
        return Table(dl, ptrs.copy()), Table(dg, ptrs.copy())
    lids_rcv, gids_rcv = unzip(map_parts(rcv, parts, ids, parts_rcv), 2)
    if reuse_parts_rcv:
        parts_snd = parts_rcv
    else:
        parts_snd = discover_parts_snd(parts_rcv, neighbors_snd, neighbors_rcv)
    gids_snd = exchange_tables(gids_rcv, parts_snd, parts_rcv)

    def snd(s, g):
        return Table(np.array([s.gid_to_lid[int(x)] for x in g.data], dtype=np.int32), g.ptrs.copy())
    lids_snd = map_parts(snd, ids, gids_snd)
    return Exchanger(parts_rcv, parts_snd, lids_rcv, lids_snd)


def empty_exchanger(a: PData) -> Exchanger:
    """Interfaces.jl:788-794"""
    e = lambda _: []
    t = lambda _: Table(np.zeros(0, np.int32), np.ones(1, np.int32))
    return Exchanger(map_parts(e, a), map_parts(e, a), map_parts(t, a), map_parts(t, a))


def reverse_exchanger(a: Exchanger) -> Exchanger:
    """Base.reverse(::Exchanger) Interfaces.jl:796-798"""
    return Exchanger(a.parts_snd, a.parts_rcv, a.lids_snd, a.lids_rcv)


def _replace(x, y):  # Interfaces.jl:835
    return y


def exchange_values_(combine_op, values_rcv: PData, values_snd: PData, ex: Exchanger):
    """async_exchange!(combine_op, values_rcv, values_snd, exchanger) +
    blocking wait: Interfaces.jl:846-889 (buffers 800-816, delivery
    SequentialBackend.jl:167-200).  values_* hold numpy arrays or lists."""
    def pack(vs, lids):
        return Table(np.array([vs[l - 1] for l in lids.data], dtype=object), lids.ptrs.copy())
    data_snd = map_parts(pack, values_snd, ex.lids_snd)
    data_rcv = exchange_tables(data_snd, ex.parts_rcv, ex.parts_snd)

    def unpack(vs, d, lids):
        for p in range(len(lids.data)):
            lid = int(lids.data[p])
            vs[lid - 1] = combine_op(vs[lid - 1], d.data[p])
    map_parts(unpack, values_rcv, data_rcv, ex.lids_rcv)
    return values_rcv


def exchange_(values: PData, ex: Exchanger, combine_op=_replace):
    """exchange!(values, exchanger) (Interfaces.jl:453-458 → 818-844)"""
    return exchange_values_(combine_op, values, values, ex)


def _table_lids(lids_snd: Table, tptrs) -> Table:
    """_table_lids_snd Interfaces.jl:928-961"""
    np_ = len(lids_snd)
    counts = [0] * np_
    for p in range(np_):
        for i in range(lids_snd.ptrs[p] - 1, lids_snd.ptrs[p + 1] - 1):
            d = int(lids_snd.data[i])
            counts[p] += int(tptrs[d] - tptrs[d - 1])
    ptrs = counts_to_ptrs(counts)
    data = []
    for p in range(np_):
        for i in range(lids_snd.ptrs[p] - 1, lids_snd.ptrs[p + 1] - 1):
            d = int(lids_snd.data[i])
            data.extend(range(int(tptrs[d - 1]), int(tptrs[d])))
    return Table(np.array(data, dtype=np.int32), ptrs)


def exchange_table_values_(values: PData, ex: Exchanger, combine_op=_replace):
    """async_exchange!(combine_op, values::AbstractPData{<:Table}, exchanger)
    Interfaces.jl:899-926"""
    t_ex = Exchanger(ex.parts_rcv, ex.parts_snd,
                     map_parts(lambda l, t: _table_lids(l, t.ptrs), ex.lids_rcv, values),
                     map_parts(lambda l, t: _table_lids(l, t.ptrs), ex.lids_snd, values))
    data = map_parts(lambda t: t.data, values)
    exchange_values_(combine_op, data, data, t_ex)
    return values


# ---------------------------------------------------------------------------
# PRange and partition math (Interfaces.jl:963-1573)

@dataclass
class PRange:
    ngids: int
    partition: PData
    exchanger: Exchanger
    gid_to_part: object = None  # PData of callables gid -> part, or None
    ghost: bool = True


def prange(ngids, partition: PData, gid_to_part=None, ghost=True) -> PRange:
    """PRange(ngids, partition[, gid_to_part, ghost]) Interfaces.jl:998-1006"""
    ex = exchanger_from_ids(partition) if ghost else empty_exchanger(partition)
    return PRange(ngids, partition, ex, gid_to_part, ghost)


def _oid_to_gid(ngids, np_, p):
    """Interfaces.jl:1307-1319 → (first, last) inclusive"""
    _olength = ngids // np_
    _offset = _olength * (p - 1)
    _rem = ngids % np_
    if _rem < (np_ - p + 1):
        olength, offset = _olength, _offset
    else:
        olength = _olength + 1
        offset = _offset + p - (np_ - _rem) - 1
    return list(range(1 + offset, olength + offset + 1))


def _lid_to_gid_1d(ngids, np_, p, isperiodic=None):
    """Interfaces.jl:1321-1335 (isperiodic=None) and 1353-1373"""
    o = _oid_to_gid(ngids, np_, p)
    gini, gend = o[0], o[-1]
    if np_ == 1:
        return list(o)
    if p == 1:
        r = list(range(gini, gend + 2))
        if isperiodic:
            r = [ngids] + r
        return r
    if p != np_:
        return list(range(gini - 1, gend + 2))
    r = list(range(gini - 1, gend + 1))
    if isperiodic:
        r.append(1)
    return r


def _lid_to_gid_out_of_bounds(ngids, np_, p, isperiodic):
    """Interfaces.jl:1337-1351 → (first, last)"""
    o = _oid_to_gid(ngids, np_, p)
    if isperiodic:
        return (o[0], o[-1]) if np_ == 1 else (o[0] - 1, o[-1] + 1)
    r = _lid_to_gid_1d(ngids, np_, p)
    return (r[0], r[-1])


def _lid_to_part_1d(nlids, np_, p, isperiodic=None):
    """Interfaces.jl:1375-1411"""
    r = [p] * nlids
    if np_ == 1:
        return r
    if p == 1:
        r[-1] = p + 1
        if isperiodic:
            r[0] = np_
    elif p != np_:
        r[0] = p - 1
        r[-1] = p + 1
    else:
        r[0] = p - 1
        if isperiodic:
            r[-1] = 1
    return r


def cartesian_index(shape, lin):
    """CartesianIndices(shape)[lin] (1-based, first index fastest)"""
    out = []
    lin -= 1
    for s in shape:
        out.append(lin % s + 1)
        lin //= s
    return tuple(out)


def linear_index(shape, ci):
    lin = 0
    stride = 1
    for s, c in zip(shape, ci):
        lin += (c - 1) * stride
        stride *= s
    return lin + 1


def _id_tensor_product(d_to_dlid_to_gdid, d_to_ngdids):
    """Interfaces.jl:1473-1491: local Cartesian order (first dim fastest)."""
    import itertools
    dims = [len(x) for x in d_to_dlid_to_gdid]
    out = []
    for tup in itertools.product(*[range(n) for n in reversed(dims)]):
        lci = tuple(reversed(tup))
        gci = tuple(d_to_dlid_to_gdid[d][lci[d]] for d in range(len(dims)))
        out.append(linear_index(d_to_ngdids, gci))
    return out


def _oid_first(ngids, np_, p):
    """first(_oid_to_gid(ngids, np, p)): Julia's `first` of a UnitRange is its
    start, also for an empty range (a part that owns no ids)."""
    _olength = ngids // np_
    _offset = _olength * (p - 1)
    _rem = ngids % np_
    offset = _offset if _rem < (np_ - p + 1) else _offset + p - (np_ - _rem) - 1
    return 1 + offset


def _part_to_firstgid(ngids, np_):
    """Interfaces.jl:1493-1495"""
    return [_oid_first(ngids, np_, p) for p in range(1, np_ + 1)]


def linear_gid_to_part(part_to_firstgid):
    """LinearGidToPart (IndexSets.jl:174-193): searchsortedlast"""
    import bisect
    return lambda gid: bisect.bisect_right(part_to_firstgid, gid)


def cartesian_gid_to_part(ngids, np_):
    """CartesianGidToPart (IndexSets.jl:195-213)"""
    import bisect
    firsts = [_part_to_firstgid(n, p) for n, p in zip(ngids, np_)]

    def f(gid):
        cg = cartesian_index(ngids, gid)
        cp = tuple(bisect.bisect_right(fs, g) for fs, g in zip(firsts, cg))
        return linear_index(np_, cp)
    return f


def prange_linear(parts: PData, ngids: int) -> PRange:
    """PRange(parts, ngids) Interfaces.jl:1014-1030 (no ghost layer)"""
    np_ = num_parts(parts)
    p2f = _part_to_firstgid(ngids, np_)

    def mk(part):
        o = _oid_to_gid(ngids, np_, part)
        return index_range(part, len(o), _oid_first(ngids, np_, part))
    partition = map_parts(mk, parts)
    g2p = map_parts(lambda _: linear_gid_to_part(p2f), parts)
    return prange(ngids, partition, g2p, ghost=False)


def prange_noids(parts: PData, noids: PData) -> PRange:
    """PRange(parts, noids) Interfaces.jl:1038-1068"""
    ngids = preduce(lambda a, b: a + b, noids, 0)
    firsts = xscan_all(lambda a, b: a + b, noids, 1)
    partition = map_parts(lambda part, n, f: index_range(part, n, f[part - 1]), parts, noids, firsts)
    g2p = map_parts(lambda f: linear_gid_to_part(list(f)), firsts)
    return prange(ngids, partition, g2p, ghost=False)


def prange_cartesian(parts: PData, ngids: tuple, with_ghost=False, isperiodic=None) -> PRange:
    """PRange(parts, ngids::NTuple) Interfaces.jl:1114-1137, with_ghost
    1166-1193, periodic 1195-1223."""
    np_ = parts.shape
    D = len(ngids)

    def mk(part):
        cp = cartesian_index(np_, part)
        if not with_ghost:
            ranges = [_oid_to_gid(ngids[d], np_[d], cp[d]) for d in range(D)]
            lid_to_gid = _id_tensor_product(ranges, ngids)
            n = len(lid_to_gid)
            return IndexSet(part, lid_to_gid, [part] * n, list(range(1, n + 1)), [])
        per = isperiodic if isperiodic is not None else (None,) * D
        ranges = [_lid_to_gid_1d(ngids[d], np_[d], cp[d], per[d]) for d in range(D)]
        lid_to_gid = _id_tensor_product(ranges, ngids)
        dparts = [_lid_to_part_1d(len(ranges[d]), np_[d], cp[d], per[d]) for d in range(D)]
        lid_to_part = _id_tensor_product(dparts, np_)
        oid = [l + 1 for l, o in enumerate(lid_to_part) if o == part]
        hid = [l + 1 for l, o in enumerate(lid_to_part) if o != part]
        return IndexSet(part, lid_to_gid, lid_to_part, oid, hid)
    partition = map_parts(mk, parts)
    g2p = map_parts(lambda _: cartesian_gid_to_part(ngids, np_), parts)
    ng = int(np.prod(ngids))
    if not with_ghost:
        return prange(ng, partition, g2p, ghost=False)
    ex = exchanger_from_ids(partition, reuse_parts_rcv=True)
    return PRange(ng, partition, ex, g2p, True)


def pcartesian_indices(parts: PData, ngids: tuple, with_ghost=False):
    """PCartesianIndices(parts, ngids[, with_ghost]) Interfaces.jl:1146-1158, 1233-1246:
    per part, the (first,last) global range per dim."""
    np_ = parts.shape

    def mk(part):
        cp = cartesian_index(np_, part)
        out = []
        for d in range(len(ngids)):
            r = (_lid_to_gid_1d(ngids[d], np_[d], cp[d]) if with_ghost
                 else _oid_to_gid(ngids[d], np_[d], cp[d]))
            out.append((r[0], r[-1]))
        return tuple(out)
    return map_parts(mk, parts)


def add_gids_(a: PRange, gids: PData, i_to_part: PData = None) -> PRange:
    """add_gids!(a::PRange, gids[, i_to_part]) Interfaces.jl:1501-1533"""
    if i_to_part is not None:
        map_parts(add_gids_parts_, a.partition, gids, i_to_part)
    else:
        if a.gid_to_part is None:
            raise ValueError("DomainError: PRange without gid_to_part")  # :1522-1528
        map_parts(add_gids_owner_, a.gid_to_part, a.partition, gids)
    a.exchanger = exchanger_from_ids(a.partition)
    a.ghost = True
    return a


def copy_prange(a: PRange) -> PRange:
    return PRange(a.ngids, map_parts(lambda s: s.copy(), a.partition),
                  Exchanger(*(PData([x.copy() if hasattr(x, "copy") else list(x) for x in f.parts], f.shape)
                              for f in (a.exchanger.parts_rcv, a.exchanger.parts_snd,
                                        a.exchanger.lids_rcv, a.exchanger.lids_snd))),
                  a.gid_to_part, a.ghost)


def add_gids(a: PRange, gids: PData, i_to_part: PData = None) -> PRange:
    """Interfaces.jl:1535-1539"""
    return add_gids_(copy_prange(a), gids, i_to_part)


def to_lids_pr_(ids: PData, a: PRange):
    return map_parts(to_lids_, ids, a.partition)


def oids_are_equal(a: PRange, b: PRange):
    """Interfaces.jl:1549-1556"""
    if a.partition is b.partition:
        return True
    return preduce(lambda x, y: x and y, map_parts(oids_are_equal_is, a.partition, b.partition), True)


def hids_are_equal(a: PRange, b: PRange):
    if a.partition is b.partition:
        return True
    return preduce(lambda x, y: x and y, map_parts(hids_are_equal_is, a.partition, b.partition), True)


# ---------------------------------------------------------------------------
# Scalars: Julia arithmetic on (re, im) for complex, numpy scalars for reals

class Cx:
    """A complex scalar/array carried as (re, im) with Julia's formulas."""

    def __init__(self, re, im):
        self.re, self.im = re, im

    def __add__(self, o):
        o = _as_cx(o, self.re)
        return Cx(self.re + o.re, self.im + o.im)

    def __sub__(self, o):
        o = _as_cx(o, self.re)
        return Cx(self.re - o.re, self.im - o.im)

    def __mul__(self, o):
        if not isinstance(o, Cx):  # complex * real: Complex(re*x, im*x)
            return Cx(self.re * o, self.im * o)
        return Cx(self.re * o.re - self.im * o.im, self.re * o.im + self.im * o.re)

    def __rmul__(self, o):  # real * complex: Complex(x*re, x*im)
        return Cx(o * self.re, o * self.im)

    def conj(self):
        return Cx(self.re, -self.im)

    def __repr__(self):
        return f"Cx({self.re!r}, {self.im!r})"


def _as_cx(o, like):
    if isinstance(o, Cx):
        return o
    z = like * 0 if isinstance(like, np.ndarray) else type(like)(0)
    return Cx(o, z)


# ---------------------------------------------------------------------------
# PVector (Interfaces.jl:1576-2106): values are per-part numpy arrays
# (real dtypes) or Cx of two arrays (complex).

@dataclass
class PVector:
    values: PData
    rows: PRange


def pvector_undef(rows: PRange, dtype=np.float64) -> PVector:
    """PVector{T}(undef, rows) Interfaces.jl:1869-1878 (zero-filled here)"""
    return PVector(map_parts(lambda s: _zeros(s.num_lids, dtype), rows.partition), rows)


def _zeros(n, dtype):
    if dtype in (np.complex64, np.complex128):
        rt = np.float32 if dtype == np.complex64 else np.float64
        return Cx(np.zeros(n, rt), np.zeros(n, rt))
    return np.zeros(n, dtype)


def _zero_like(vs):
    """zero(eltype(vs)) (+0.0, not x*0 which keeps the sign)"""
    if isinstance(vs, Cx):
        z = np.zeros((), dtype=vs.re.dtype)[()]
        return Cx(z, z)
    return np.zeros((), dtype=vs.dtype)[()] if isinstance(vs, np.ndarray) else 0.0


def _get(vs, i):
    return Cx(vs.re[i], vs.im[i]) if isinstance(vs, Cx) else vs[i]


def _set(vs, i, v):
    if isinstance(vs, Cx):
        vs.re[i], vs.im[i] = v.re, v.im
    else:
        vs[i] = v


def _copyvals(vs):
    return Cx(vs.re.copy(), vs.im.copy()) if isinstance(vs, Cx) else vs.copy()


class _CxList:
    """list-like view of a Cx array pair (element access as Cx scalars)."""

    def __init__(self, c):
        self.c = c

    def __getitem__(self, i):
        return Cx(self.c.re[i], self.c.im[i])

    def __setitem__(self, i, v):
        self.c.re[i] = v.re
        self.c.im[i] = v.im

    def __len__(self):
        return len(self.c.re)


def exchange_pvector_(v: PVector, combine_op=_replace, reverse=False):
    """exchange!(v::PVector) = async_exchange!(v.values, v.rows.exchanger)
    (Interfaces.jl:2071-2075); reverse for assemble."""
    ex = reverse_exchanger(v.rows.exchanger) if reverse else v.rows.exchanger
    vals = map_parts(lambda x: _CxList(x) if isinstance(x, Cx) else x, v.values)
    exchange_values_(combine_op, vals, vals, ex)
    return v


def assemble_(v: PVector):
    """assemble!(v) Interfaces.jl:2084-2106: reverse exchange with +, then
    values[hid_to_lid] .= 0"""
    exchange_pvector_(v, lambda a, b: a + b, reverse=True)

    def zero(vs, s):
        for l in s.hid_to_lid:
            _set(vs, l - 1, _zero_like(vs))
    map_parts(zero, v.values, v.rows.partition)
    return v


def _owned(vs, s: IndexSet):
    idx = np.asarray(s.oid_to_lid, dtype=np.int64) - 1
    return Cx(vs.re[idx], vs.im[idx]) if isinstance(vs, Cx) else vs[idx]


def dot(a: PVector, b: PVector):
    """dot(a,b) Interfaces.jl:1985-1992: per-part local dot over owned values,
    then sum(c) = reduce(+, c; init=0), folded in part order (221-238).  The
    local dot is BLAS (order not pinned); here a sequential
    sum in float64 (float32 inputs accumulate in float64 too)."""
    def local(x, y, sa, sb):
        xo, yo = _owned(x, sa), _owned(y, sb)
        if isinstance(xo, Cx):
            re = np.sum(xo.re.astype(np.float64) * yo.re + xo.im.astype(np.float64) * yo.im)
            im = np.sum(xo.re.astype(np.float64) * yo.im - xo.im.astype(np.float64) * yo.re)
            return complex(re, im)
        return float(np.sum(xo.astype(np.float64) * yo.astype(np.float64)))
    c = map_parts(local, a.values, b.values, a.rows.partition, b.rows.partition)
    if _is_single(a):  # the local dot returns T; sum(c) adds the T values in T
        if isinstance(c.parts[0], complex):
            re = _julia_reduce(lambda x, y: x + y, [np.float32(v.real) for v in c.parts], np.float32(0))
            im = _julia_reduce(lambda x, y: x + y, [np.float32(v.imag) for v in c.parts], np.float32(0))
            return complex(float(re), float(im))
        return _julia_reduce(lambda x, y: x + y, [np.float32(v) for v in c.parts], np.float32(0))
    return _julia_reduce(lambda x, y: x + y, c.parts, 0.0)


def _is_single(a: PVector):
    v = a.values.parts[0]
    return (v.re.dtype if isinstance(v, Cx) else np.asarray(v).dtype) == np.float32


def norm(a: PVector, p=2):
    """norm(a, p) Interfaces.jl:1767-1772: (Σ_parts norm(owned)^p)^(1/p)"""
    def local(x, s):
        xo = _owned(x, s)
        if isinstance(xo, Cx):
            return float(np.sum(xo.re.astype(np.float64) ** 2 + xo.im.astype(np.float64) ** 2))
        return float(np.sum(xo.astype(np.float64) ** 2))
    c = map_parts(local, a.values, a.rows.partition)
    if _is_single(a):  # norm(v)^p is a Float32, reduced in Float32, then ^(1/p) in Float64
        s = _julia_reduce(lambda x, y: x + y, [np.float32(v) for v in c.parts], np.float32(0))
        return float(s) ** (1.0 / p)
    return _julia_reduce(lambda x, y: x + y, c.parts, 0.0) ** (1.0 / p)


def psum_vector(a: PVector):
    """sum(a) Interfaces.jl:1973-1983"""
    def local(x, s):
        xo = _owned(x, s)
        if isinstance(xo, Cx):
            return complex(float(np.sum(xo.re, dtype=np.float64)), float(np.sum(xo.im, dtype=np.float64)))
        return float(np.sum(xo, dtype=np.float64))
    return _julia_reduce(lambda x, y: x + y, map_parts(local, a.values, a.rows.partition).parts, 0.0)


# ---------------------------------------------------------------------------
# Local sparse matrices: SparseArrays `sparse` semantics + SparseUtils.jl

@dataclass
class CSC:
    """SparseMatrixCSC: 1-based colptr/rowval, nzval (ndarray or Cx)."""
    m: int
    n: int
    colptr: np.ndarray
    rowval: np.ndarray
    nzval: object


def sparse_csc(I, J, V, m, n) -> CSC:
    """sparse(I, J, V, m, n, +) — SparseUtils.jl:80-94 (compresscoo) via
    SparseArrays.sparse!: duplicates combined with `+` in input order (a left
    fold starting at the first occurrence), rows sorted within columns."""
    I = np.asarray(I, dtype=np.int64)
    J = np.asarray(J, dtype=np.int64)
    cx = isinstance(V, Cx)
    k = len(I)
    if k:
        assert I.min() >= 1 and I.max() <= m and J.min() >= 1 and J.max() <= n
    order = np.lexsort((np.arange(k), I, J))  # by col, then row, then input position
    Is, Js = I[order], J[order]
    newgrp = np.ones(k, dtype=bool)
    if k:
        newgrp[1:] = (Is[1:] != Is[:-1]) | (Js[1:] != Js[:-1])
    starts = np.flatnonzero(newgrp)
    sizes = np.diff(np.append(starts, k))

    def fold(vals):
        vs = vals[order]
        acc = vs[starts].copy()
        for t in range(1, int(sizes.max()) if k else 1):
            sel = sizes > t
            acc[sel] = acc[sel] + vs[starts[sel] + t]
        return acc
    nzval = Cx(fold(V.re), fold(V.im)) if cx else fold(np.asarray(V))
    rowval = Is[starts]
    cols = Js[starts]
    colptr = np.concatenate([[1], 1 + np.cumsum(np.bincount(cols - 1, minlength=n))]).astype(np.int64)
    return CSC(m, n, colptr, rowval.astype(np.int64), nzval)


def csc_mul_sub_(C, A: CSC, rows_inv, cols_list, rflag, cflag, B, alpha, beta):
    """mul!(C, A::SubSparseMatrix{<:SparseMatrixCSC}, B, α, β)
    SparseUtils.jl:157-187, literally (pure Python; small sizes).
    C, B: list-like of scalars (numpy scalar or Cx); cols_list = A.indices[2]
    (1-based parent col ids, in view order); rows_inv = invrows (lid_to_ohid)."""
    if not (beta == 1):
        # β != 0 ? rmul!(C, β) : fill!(C, zero(eltype(C)))  (SparseUtils.jl:167-168):
        # β = 0 overwrites, so NaN/Inf or a negative value in C does not leak
        for i in range(len(C)):
            C[i] = C[i] * beta if beta != 0 else _zero_elem(C[i])
    nzv = A.nzval
    for j, Jc in enumerate(cols_list, start=1):
        axj = B[j - 1] * alpha if not _is_one(alpha) else B[j - 1]
        for p in range(int(A.colptr[Jc - 1]) - 1, int(A.colptr[Jc]) - 1):
            Ir = int(A.rowval[p])
            i = rows_inv[Ir - 1] * rflag
            if i > 0:
                C[i - 1] = C[i - 1] + _get(nzv, p) * axj
    return C


@dataclass
class CSR:
    """SparseMatrixCSR{Bi} (SparseMatricesCSR.jl, a dependency not vendored
    in /root/reference): rowptr and colval hold Bi-based indices (Bi = 0 or
    1), getoffset(A) = 1 - Bi (SparseUtils.jl:212), nzval in row order."""
    Bi: int
    m: int
    n: int
    rowptr: np.ndarray
    colval: np.ndarray
    nzval: object


def sparse_csr(Bi, I, J, V, m, n) -> CSR:
    """compresscoo(SparseMatrixCSR{Bi}, I, J, V, m, n) SparseUtils.jl:193-208
    → sparsecsr(Val(Bi), I, J, V, m, n, +).  SparseMatricesCSR's published
    algorithm: the CSC of the transpose, sparse(J, I, V, n, m, +), read as
    rows — duplicates combined with + in input order, columns sorted within
    each row — with its 1-based indices shifted to base Bi.  Pinned by
    SparseUtilsTests.jl:62-65 (compresscoo(T,…) == sparse(I,J,V), nziterator
    order = findnz order, nzindex, the sub-matrix mul! against the dense
    product)."""
    assert Bi in (0, 1)
    t = sparse_csc(J, I, V, n, m)
    return CSR(Bi, m, n, (t.colptr - 1 + Bi).astype(np.int64), (t.rowval - 1 + Bi).astype(np.int64), t.nzval)


def csr_nzrange(A: CSR, I):
    """nzrange(A, I) for SparseMatrixCSR{Bi}: rowptr[I]+o : rowptr[I+1]-Bi
    (1-based positions; SparseUtils.jl:214-215)"""
    o = 1 - A.Bi
    return range(int(A.rowptr[I - 1]) + o, int(A.rowptr[I]) - A.Bi + 1)


def csr_mul_sub_(C, A: CSR, rows_list, cols_inv, rflag, cflag, B, alpha, beta):
    """mul!(C, A::SubSparseMatrix{<:SparseMatrixCSR}, B, α, β)
    SparseUtils.jl:222-252, literally: rows in view order, each row's entries
    in storage order, `C[i] += nzv[p]*B[j]*α` — the product first, then α
    (the CSC twin scales x first, :177).  rows_list = A.indices[1] (1-based
    parent row ids), cols_inv = invcols (lid_to_ohid)."""
    if not (beta == 1):
        for i in range(len(C)):
            C[i] = C[i] * beta if beta != 0 else _zero_elem(C[i])
    nzv = A.nzval
    o = 1 - A.Bi
    for i, Ir in enumerate(rows_list, start=1):
        for p in csr_nzrange(A, Ir):
            Jc = int(A.colval[p - 1]) + o
            j = cols_inv[Jc - 1] * cflag
            if j > 0:
                t = _get(nzv, p - 1) * B[j - 1]
                C[i - 1] = C[i - 1] + (t if _is_one(alpha) else t * alpha)
    return C


def _zero_elem(v):
    """zero(eltype(C)) for one element (numpy scalar or Cx)"""
    if isinstance(v, Cx):
        return Cx(type(v.re)(0), type(v.im)(0))
    return type(v)(0)


def _is_one(a):
    return (not isinstance(a, Cx)) and a == 1


@dataclass
class PSparseMatrix:
    values: PData   # CSC per part
    rows: PRange
    cols: PRange
    exchanger: Exchanger = None


def psparse_from_coo(I: PData, J: PData, V: PData, rows: PRange, cols: PRange, ids="local", init=None):
    """PSparseMatrix(init,I,J,V,rows,cols; ids) Interfaces.jl:2194-2215;
    init = sparse by default (2237-2244), or e.g.
    `lambda i, j, v, m, n: sparse_csr(Bi, i, j, v, m, n)` (sparsecsr)."""
    if ids == "global":
        to_lids_pr_(I, rows)
        to_lids_pr_(J, cols)
    init = init or sparse_csc
    vals = map_parts(lambda i, j, v, r, c: init(i, j, v, r.num_lids, c.num_lids), I, J, V,
                     rows.partition, cols.partition)
    return PSparseMatrix(vals, rows, cols, matrix_exchanger(vals, rows, cols))  # Interfaces.jl:2117


def mul_(c: PVector, a: PSparseMatrix, b: PVector, alpha=1.0, beta=0.0, literal=False):
    """mul!(c, a, b, α, β) Interfaces.jl:2246-2275: exchange!(b), owned block
    (after β scaling), then ghost block, each via SparseUtils.jl:157-187."""
    assert oids_are_equal(c.rows, a.rows)
    assert oids_are_equal(a.cols, b.rows) and hids_are_equal(a.cols, b.rows)
    exchange_pvector_(b)
    if literal:
        def part(cv, A, bv, r, ac, bc, cr):
            C = _OwnedView(cv, cr.oid_to_lid)
            if isinstance(A, CSR):  # owned_owned then owned_ghost views (Interfaces.jl:2142-2156)
                csr_mul_sub_(C, A, r.oid_to_lid, ac.lid_to_ohid, 1, 1, _OwnedView(bv, bc.oid_to_lid), alpha, beta)
                csr_mul_sub_(C, A, r.oid_to_lid, ac.lid_to_ohid, 1, -1, _OwnedView(bv, bc.hid_to_lid), alpha, 1)
                return
            csc_mul_sub_(C, A, r.lid_to_ohid, ac.oid_to_lid, 1, 1, _OwnedView(bv, bc.oid_to_lid), alpha, beta)
            csc_mul_sub_(C, A, r.lid_to_ohid, ac.hid_to_lid, 1, -1, _OwnedView(bv, bc.hid_to_lid), alpha, 1)
        map_parts(part, c.values, a.values, b.values, a.rows.partition, a.cols.partition,
                  b.rows.partition, c.rows.partition)
    else:
        map_parts(lambda cv, A, bv, r, ac, bc, cr: _spmv_part_vec(cv, A, bv, r, ac, bc, cr, alpha, beta),
                  c.values, a.values, b.values, a.rows.partition, a.cols.partition,
                  b.rows.partition, c.rows.partition)
    return c


class _OwnedView:
    def __init__(self, vs, lids):
        self.vs, self.lids = vs, lids

    def __getitem__(self, i):
        return _get(self.vs, self.lids[i] - 1)

    def __setitem__(self, i, v):
        _set(self.vs, self.lids[i] - 1, v)

    def __len__(self):
        return len(self.lids)


def split_rows_csr(A: CSR, rows: IndexSet, cols: IndexSet):
    """split_rows for a CSR parent (SparseUtils.jl:242-250 over owned_owned,
    then owned_ghost): each owned row's owned-column entries in storage
    order, then its ghost-column entries in storage order."""
    oid = np.asarray(rows.oid_to_lid, dtype=np.int64)
    if len(oid) == 0:
        z = np.zeros(0, np.int64)
        return z, z, z
    o = 1 - A.Bi
    starts = A.rowptr[oid - 1] + o - 1          # 0-based first position of each owned row
    cnt = A.rowptr[oid] - A.Bi - (A.rowptr[oid - 1] + o) + 1
    rep = np.repeat(np.arange(len(oid)), cnt)
    pos = np.repeat(starts, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
    lid = A.colval[pos] + o
    ohid = np.asarray(cols.lid_to_ohid, dtype=np.int64)[lid - 1]
    ghost = (ohid < 0).astype(np.int64)
    k = np.lexsort((np.arange(len(pos)), ghost, rep))
    return (rep + 1)[k], lid[k], pos[k]


def split_rows(A: CSC, rows: IndexSet, cols: IndexSet):
    """Owned rows of the local CSC as per-row entry lists in the reference's
    summation order (SparseUtils.jl:176-185 applied to owned_owned then
    owned_ghost, Interfaces.jl:2142-2156): returns (row_oid, col_lid, nz_pos)
    sorted by (row, order) where order = own cols by oid, then ghost cols by hid."""
    if isinstance(A, CSR):
        return split_rows_csr(A, rows, cols)
    row_ohid = np.asarray(rows.lid_to_ohid, dtype=np.int64)
    cols_seq = [(cols.oid_to_lid, 0), (cols.hid_to_lid, len(cols.oid_to_lid))]
    R, Cc, P, K = [], [], [], []
    colptr = A.colptr
    for lids, base in cols_seq:
        lids = np.asarray(lids, dtype=np.int64)
        if len(lids) == 0:
            continue
        starts = colptr[lids - 1] - 1
        ends = colptr[lids] - 1
        cnt = ends - starts
        rep = np.repeat(np.arange(len(lids)), cnt)
        pos = np.repeat(starts, cnt) + (np.arange(cnt.sum()) - np.repeat(np.cumsum(cnt) - cnt, cnt))
        r = row_ohid[A.rowval[pos] - 1]
        keep = r > 0
        R.append(r[keep])
        Cc.append(lids[rep[keep]])
        P.append(pos[keep])
        K.append(base + rep[keep])
    if not R:
        z = np.zeros(0, np.int64)
        return z, z, z
    R, Cc, P, K = map(np.concatenate, (R, Cc, P, K))
    o = np.lexsort((K, R))
    return R[o], Cc[o], P[o]


def _spmv_part_vec(cv, A, bv, rows, acols, bcols, crows, alpha, beta):
    """Vectorised restatement of the same per-row left fold (exact order)."""
    r_oid, c_lid, pos = split_rows(A, rows, acols)
    # b is indexed through b.rows (oids/hids equal as gids to a.cols)
    ohid = np.asarray(acols.lid_to_ohid, dtype=np.int64)[c_lid - 1]
    b_oid = np.asarray(bcols.oid_to_lid, dtype=np.int64)
    b_hid = np.asarray(bcols.hid_to_lid, dtype=np.int64)
    xl = np.where(ohid > 0, b_oid[np.maximum(ohid, 1) - 1] if len(b_oid) else 0,
                  b_hid[np.maximum(-ohid, 1) - 1] if len(b_hid) else 0) - 1
    nrows = len(rows.oid_to_lid)
    ylid = np.asarray(crows.oid_to_lid, dtype=np.int64) - 1
    cx = isinstance(cv, Cx)
    counts = np.bincount(r_oid - 1, minlength=nrows) if len(r_oid) else np.zeros(nrows, np.int64)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]) if nrows else np.zeros(0, np.int64)

    def init(vals):
        y = vals[ylid]
        if beta == 0:  # fill!(co, zero(eltype(co))) (Interfaces.jl:2262-2263), not y*0
            return np.zeros_like(y)
        return y if beta == 1 else y * beta
    if cx:
        if isinstance(beta, Cx):  # a complex β: rmul!(co, β) with Julia's complex product
            yr, yi = cv.re[ylid], cv.im[ylid]
            if beta.re == 0 and beta.im == 0:
                acc = Cx(np.zeros_like(yr), np.zeros_like(yi))
            elif beta.re == 1 and beta.im == 0:
                acc = Cx(yr, yi)
            else:
                acc = Cx(yr * beta.re - yi * beta.im, yr * beta.im + yi * beta.re)
        else:
            acc = Cx(init(cv.re), init(cv.im))
        xr, xi = bv.re[xl], bv.im[xl]
        csr = isinstance(A, CSR)  # CSR: (v*x)*α (SparseUtils.jl:247); CSC: v*(x*α) (:177, 182)
        if not _is_one(alpha):
            a = alpha if isinstance(alpha, Cx) else Cx(alpha, 0 * alpha)
            if not csr:
                xr, xi = xr * a.re - xi * a.im, xr * a.im + xi * a.re
        vr, vi = A.nzval.re[pos], A.nzval.im[pos]
        pr, pi = vr * xr - vi * xi, vr * xi + vi * xr
        if csr and not _is_one(alpha):
            pr, pi = pr * a.re - pi * a.im, pr * a.im + pi * a.re
    else:
        acc = init(cv)
        xv = bv[xl]
        csr = isinstance(A, CSR)
        if not _is_one(alpha) and not csr:
            xv = xv * alpha
        pr = A.nzval[pos] * xv
        if not _is_one(alpha) and csr:
            pr = pr * alpha
    maxlen = int(counts.max()) if nrows and len(r_oid) else 0
    for t in range(maxlen):
        sel = np.flatnonzero(counts > t)
        if cx:
            acc.re[sel] = acc.re[sel] + pr[starts[sel] + t]
            acc.im[sel] = acc.im[sel] + pi[starts[sel] + t]
        else:
            acc[sel] = acc[sel] + pr[starts[sel] + t]
    if cx:
        cv.re[ylid], cv.im[ylid] = acc.re, acc.im
    else:
        cv[ylid] = acc


def matvec(a: PSparseMatrix, b: PVector, dtype=None) -> PVector:
    """Base.:*(a, b) Interfaces.jl:2605-2610"""
    c = pvector_undef(a.rows, dtype or b.values.parts[0].dtype)
    return mul_(c, a, b)


# ---------------------------------------------------------------------------
# Vector broadcasts of the CG loop (Interfaces.jl:1688-1765)

def _owned_or_all(v: PVector, other: PVector):
    same = v.rows is other.rows
    return same


def bcast_(y: PVector, x: PVector, a, mode):
    """y .= x .+ a.*y (0); y .+= a.*x (1); y .-= a.*x (2); y .-= x (3)
    — materialize! (Interfaces.jl:1710-1720): owned values, and ghost values
    when both share the PRange object."""
    same = y.rows is x.rows

    def part(yv, xv, sy, sx):
        iy = np.arange(sy.num_lids) if same else np.asarray(sy.oid_to_lid) - 1
        ix = np.arange(sx.num_lids) if same else np.asarray(sx.oid_to_lid) - 1
        if mode == 0:
            yv[iy] = xv[ix] + a * yv[iy]
        elif mode == 1:
            yv[iy] = yv[iy] + a * xv[ix]
        elif mode == 2:
            yv[iy] = yv[iy] - a * xv[ix]
        elif mode == 3:
            yv[iy] = yv[iy] - xv[ix]
    map_parts(part, y.values, x.values, y.rows.partition, x.rows.partition)
    return y


def copyto_(a: PVector, b: PVector):
    """copyto!(a,b) Interfaces.jl:1659-1667"""
    if a.rows.partition is b.rows.partition:
        map_parts(lambda x, y: x.__setitem__(slice(None), y), a.values, b.values)
    else:
        def part(x, y, sa, sb):
            x[np.asarray(sa.oid_to_lid) - 1] = y[np.asarray(sb.oid_to_lid) - 1]
        map_parts(part, a.values, b.values, a.rows.partition, b.rows.partition)
    return a


def cg_(x: PVector, A: PSparseMatrix, b: PVector, reltol=None, abstol=0.0, maxiter=None,
        log=None):
    """IterativeSolvers.cg! v0.9 (not vendored), restated:
    u = zero(x); r, c = similar(x); copyto!(r,b); mul!(c,A,x); r .-= c;
    residual = norm(r); tol = max(reltol*norm(b), abstol); prev = 1;
    loop: β = res²/prev²; u .= r .+ β.*u; mul!(c,A,u); α = res²/dot(u,c);
    x .+= α.*u; r .-= α.*c; prev = res; res = norm(r)."""
    dt = x.values.parts[0].dtype
    if reltol is None:  # sqrt(eps(T)) in T
        reltol = float(np.sqrt(np.finfo(dt).eps))
    if maxiter is None:
        maxiter = A.cols.ngids
    mk = lambda: PVector(map_parts(lambda v: np.zeros_like(v), x.values), x.rows)
    u, r, c = mk(), mk(), mk()
    copyto_(r, b)
    mul_(c, A, x)
    bcast_(r, c, None, 3)
    residual = norm(r)
    tol = max(reltol * norm(b), abstol)
    prev = 1.0
    it = 0
    hist = []
    while not (it >= maxiter or residual <= tol):
        # residual is a Float64 (norm of a PVector), so are β and α; the
        # broadcasts evaluate in Float64 and round to T (np.float64 scalars
        # are strong under NumPy's promotion)
        beta = np.float64(residual * residual / (prev * prev))
        bcast_(u, r, beta, 0)
        mul_(c, A, u)
        alpha = np.float64(residual * residual / float(dot(u, c)))
        bcast_(x, u, alpha, 1)
        bcast_(r, c, alpha, 2)
        prev = residual
        residual = norm(r)
        hist.append(residual)
        it += 1
    if log is not None:
        log.extend(hist)
    return x


# ---------------------------------------------------------------------------
# Drivers: the reference's test problems

def fdm_problem(parts: PData, nx=10):
    """test_fdm.jl:8-110 (3D 7-point FD Poisson).  Returns (A, b, x0, x̂)."""
    lx = 2.0
    ns = (nx, nx, nx)
    n = nx ** 3
    h = lx / (nx - 1)
    points = [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)]
    coeffs = [c / (h * h) for c in [-6, 1, 1, 1, 1, 1, 1]]  # literal_pow: h^2 = h*h
    if len(parts.shape) == 3:
        rows = prange_cartesian(parts, ns)
    else:
        rows = prange_linear(parts, n)
    u = lambda xi: xi[0] + xi[1]
    b = pvector_undef(rows)
    xh = pvector_undef(rows)

    def coo(s, bv, xv):
        I, J, V = [], [], []
        for lid in s.oid_to_lid:
            i = s.lid_to_gid[lid - 1]
            ci = cartesian_index(ns, i)
            xi = tuple((c - 1) * h for c in ci)
            xv[lid - 1] = u(xi)
            if any(c == 1 or c == nx for c in ci):
                I.append(lid); J.append(i); V.append(1.0)
                bv[lid - 1] = u(xi)
            else:
                for v, d in zip(coeffs, points):
                    cj = tuple(a + b_ for a, b_ in zip(ci, d))
                    I.append(lid); J.append(linear_index(ns, cj)); V.append(-v)
                bv[lid - 1] = 0.0
        return I, J, np.array(V)
    I, J, V = unzip(map_parts(coo, rows.partition, b.values, xh.values), 3)
    cols = add_gids(rows, J)
    to_lids_pr_(J, cols)
    A = psparse_from_coo(I, J, V, rows, cols, ids="local")
    x0 = pvector_undef(cols)

    def bnd(xv, s):
        for lid in s.oid_to_lid:
            ci = cartesian_index(ns, s.lid_to_gid[lid - 1])
            if any(c == 1 or c == nx for c in ci):
                xv[lid - 1] = u(tuple((c - 1) * h for c in ci))
    map_parts(bnd, x0.values, x0.rows.partition)
    return A, b, x0, xh


def assemble_coo_(I: PData, J: PData, V: PData, rows: PRange):
    """async_assemble!(I, J, V, rows) + wait, Interfaces.jl:2406-2492: COO
    triplets whose row is owned elsewhere are sent to the owner (their local
    value set to zero, kept in the list) and appended there; I, J stay global."""
    to_lids_pr_(I, rows)
    parts = get_part_ids(rows.partition.shape if len(rows.partition.shape) > 1 else num_parts(rows.partition))

    vdt = np.asarray(V.parts[0] if V.parts else []).dtype
    vdt = vdt if vdt.kind in "fc" else np.dtype(np.float64)

    def setup_rcv(part, prcv, s, i, j, v):
        owner_to_i = {o: k for k, o in enumerate(prcv)}
        segs = [[[], [], []] for _ in prcv]
        for k in range(len(i)):
            li = i[k]
            owner = s.lid_to_part[li - 1]
            if owner != part:
                seg = segs[owner_to_i[owner]]
                seg[0].append(s.lid_to_gid[li - 1])
                seg[1].append(j[k])
                seg[2].append(v[k])
                v[k] = vdt.type(0)  # k_v[k] = zero(v) (2446): not v*0, a NaN/Inf does not stay
        return segs
    segs = map_parts(setup_rcv, parts, rows.exchanger.parts_rcv, rows.partition, I, J, V)
    ex = rows.exchanger
    got = []
    for t in range(3):
        data = map_parts(lambda sg: table_from([x[t] for x in sg], dtype=vdt if t == 2 else np.int64), segs)
        got.append(exchange_tables(data, ex.parts_snd, ex.parts_rcv))

    def setup_snd(s, i, j, v, gi, gj, gv):
        to_gids_(i, s)
        i.extend(int(x) for x in gi.data)
        j.extend(int(x) for x in gj.data)
        return np.concatenate([np.asarray(v, dtype=vdt), gv.data.astype(vdt)])
    V2 = map_parts(setup_snd, rows.partition, I, J, V, *got)
    return I, J, V2


def fem_sa_problem(parts: PData, nx=10, init=None):
    """test_fem_sa.jl:7-132 (2D Q1 FE, Dirichlet u = 1): returns (A, b, x0, x̂).
    init: the local matrix constructor (sparse by default, or sparse_csr)."""
    lx = 2.0
    ns = (nx, nx)
    h = lx / nx
    Ae = np.array([[4.0, -1.0, -1.0, -2.0], [-1.0, 4.0, -2.0, -1.0],
                   [-1.0, -2.0, 4.0, -1.0], [-2.0, -1.0, -1.0, 4.0]])
    Ae = (h / 6) * Ae
    nsn = (nx + 1, nx + 1)
    cart = len(parts.shape) == 2
    cells = prange_cartesian(parts, ns) if cart else prange_linear(parts, nx * nx)
    enodes = [(1, 1), (2, 1), (1, 2), (2, 2)]  # CartesianIndices((2,2)), first index fastest

    def coo(s):
        I, J, V = [], [], []
        for ocell in s.oid_to_lid:
            gcell = s.lid_to_gid[ocell - 1]
            cc = cartesian_index(ns, gcell)
            for erow, ce in enumerate(enodes):
                cg = (cc[0] + ce[0] - 1, cc[1] + ce[1] - 1)
                grow = linear_index(nsn, cg)
                if any(c == 1 or c == nx + 1 for c in cg):
                    I.append(grow); J.append(grow); V.append(1.0)
                else:
                    for ecol, cf in enumerate(enodes):
                        cgc = (cc[0] + cf[0] - 1, cc[1] + cf[1] - 1)
                        I.append(grow); J.append(linear_index(nsn, cgc)); V.append(Ae[erow, ecol])
        return I, J, V
    I, J, V = unzip(map_parts(coo, cells.partition), 3)
    rows = prange_cartesian(parts, nsn) if cart else prange_linear(parts, nsn[0] * nsn[1])
    cols = prange_cartesian(parts, nsn) if cart else prange_linear(parts, nsn[0] * nsn[1])
    add_gids_(rows, I)
    I, J, V = assemble_coo_(I, J, V, rows)
    b = pvector_undef(rows)

    def fill_b(bv, s, sc):
        for ocell in sc.oid_to_lid:
            cc = cartesian_index(ns, sc.lid_to_gid[ocell - 1])
            for ce in enodes:
                cg = (cc[0] + ce[0] - 1, cc[1] + ce[1] - 1)
                if any(c == 1 or c == nx + 1 for c in cg):
                    lid = s.gid_to_lid[linear_index(nsn, cg)]
                    bv[lid - 1] += 1.0
    map_parts(fill_b, b.values, rows.partition, cells.partition)
    add_gids_(cols, J)
    A = psparse_from_coo(I, J, V, rows, cols, ids="global", init=init)
    assemble_(b)
    x0 = pvector_undef(cols)
    xh = pvector_undef(cols)

    def init(xv, hv, s):
        for lid in s.oid_to_lid:
            cg = cartesian_index(nsn, s.lid_to_gid[lid - 1])
            hv[lid - 1] = 1.0
            if any(c == 1 or c == nx + 1 for c in cg):
                xv[lid - 1] = 1.0
    map_parts(init, x0.values, xh.values, cols.partition)
    return A, b, x0, xh


def q1_hex_ke(h):
    """3D Q1 stiffness h*(K1⊗M1⊗M1 + M1⊗K1⊗M1 + M1⊗M1⊗K1) (SURVEY.md §8d,
    the 3D analogue of test_fem_sa.jl:17-22's element matrix), Julia's kron
    index order (first factor slowest: z, y, x), evaluated as h*((T1+T2)+T3).
    Element node e = ex + 2ey + 4ez.  Returns 8×8 float64 (row-major)."""
    K1 = [[1.0, -1.0], [-1.0, 1.0]]
    M1 = [[1.0 / 3.0, 1.0 / 6.0], [1.0 / 6.0, 1.0 / 3.0]]
    Ke = np.zeros((8, 8))
    for a in range(8):
        ax, ay, az = a & 1, (a >> 1) & 1, a >> 2
        for b in range(8):
            bx, by, bz = b & 1, (b >> 1) & 1, b >> 2
            t1 = (K1[az][bz] * M1[ay][by]) * M1[ax][bx]
            t2 = (M1[az][bz] * K1[ay][by]) * M1[ax][bx]
            t3 = (M1[az][bz] * M1[ay][by]) * K1[ax][bx]
            Ke[a, b] = h * ((t1 + t2) + t3)
    return Ke


def fd7_coeffs(N, lx=2.0):
    """test_fdm.jl:18-20,75: interior row values -(c/h²), diag 6/h²"""
    h = lx / (N - 1)
    return np.array([-((-6) / (h * h)), -(1 / (h * h))])


def stencil_row_entries(kind, N, g, coef):
    """Entries (global neighbour coords, value) of the row of node g (0-based
    global coords) of the Cartesian stencil operators, in neighbour
    lexicographic (dz,dy,dx) order.  kind 7: test_fdm.jl:63-78 (Dirichlet
    rows identity).  kind 27: Q1 FE with test_fem_sa.jl:47-60's Dirichlet
    rows (diagonal only, 1 per touching cell) and entry values summed over
    the cells holding both nodes in ascending cell gid (COO order of the
    cell loop + sparse()'s in-order combine)."""
    gx, gy, gz = g
    Nx, Ny, Nz = N
    dir_ = gx in (0, Nx - 1) or gy in (0, Ny - 1) or gz in (0, Nz - 1)
    if dir_:
        if kind == 7:
            return [((gx, gy, gz), 1.0)]
        acc = None
        for cz in (-1, 0):
            if not 0 <= gz + cz <= Nz - 2:
                continue
            for cy in (-1, 0):
                if not 0 <= gy + cy <= Ny - 2:
                    continue
                for cx in (-1, 0):
                    if not 0 <= gx + cx <= Nx - 2:
                        continue
                    acc = 1.0 if acc is None else acc + 1.0
        return [((gx, gy, gz), acc)]
    out = []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                nz = (dx != 0) + (dy != 0) + (dz != 0)
                if kind == 7:
                    if nz > 1:
                        continue
                    out.append(((gx + dx, gy + dy, gz + dz), coef[0] if nz == 0 else coef[1]))
                    continue
                acc = None
                for cz in (-1, 0):
                    czg = gz + cz
                    bz = gz + dz - czg
                    if not (0 <= czg <= Nz - 2 and 0 <= bz <= 1):
                        continue
                    for cy in (-1, 0):
                        cyg = gy + cy
                        by = gy + dy - cyg
                        if not (0 <= cyg <= Ny - 2 and 0 <= by <= 1):
                            continue
                        for cx in (-1, 0):
                            cxg = gx + cx
                            bx = gx + dx - cxg
                            if not (0 <= cxg <= Nx - 2 and 0 <= bx <= 1):
                                continue
                            a = (gx - cxg) + 2 * (gy - cyg) + 4 * (gz - czg)
                            b = bx + 2 * by + 4 * bz
                            v = coef[a * 8 + b]
                            acc = v if acc is None else acc + v
                out.append(((gx + dx, gy + dy, gz + dz), acc))
    return out


def stencil_problem(parts: PData, N: tuple, kind: int, dtype=np.float64, init=None):
    """Row-wise assembly of the Cartesian stencil operator (FD7 or FE27) on a
    Cartesian PRange (test_fdm.jl's driver structure: each part pushes the
    COO entries of its owned rows, J in row order then stencil order; cols =
    add_gids(rows, J) gives the first-touch ghost order; local CSC via
    sparse).  Small sizes only (pure Python)."""
    rows = prange_cartesian(parts, N)
    coef = fd7_coeffs(N[0]) if kind == 7 else q1_hex_ke(2.0 / (N[0] - 1)).ravel()

    def coo(s):
        I, J, V = [], [], []
        for lid in s.oid_to_lid:
            gid = s.lid_to_gid[lid - 1]
            g = tuple(c - 1 for c in cartesian_index(N, gid))
            for (nb, v) in stencil_row_entries(kind, N, g, coef):
                I.append(lid)
                J.append(linear_index(N, tuple(c + 1 for c in nb)))
                V.append(v)
        return I, J, np.array(V, dtype=np.float64)
    I, J, V = unzip(map_parts(coo, rows.partition), 3)
    cols = add_gids(rows, J)
    to_lids_pr_(J, cols)
    V = map_parts(lambda v: _convert_values(v, dtype), V)
    A = psparse_from_coo(I, J, V, rows, cols, ids="local", init=init)
    return A


def _convert_values(v, dtype):
    """Float32.(A) / A .* (1+0.5im) of BASELINE config 5."""
    if dtype == np.float64:
        return v
    if dtype == np.float32:
        return v.astype(np.float32)
    if dtype == np.complex128:
        return Cx(v * 1.0, v * 0.5)
    if dtype == np.complex64:
        f = v.astype(np.float32)
        return Cx(f * np.float32(1.0), f * np.float32(0.5))
    raise ValueError(dtype)


# ---------------------------------------------------------------------------
# BASELINE config 5: stencil operators on an irregular (Voronoi, "METIS-like")
# owner map.  Vectorised restatements for the 128³ size,
# each checked against the scalar functions above by tests/test_host_setup.py.

def voronoi_owners(N, nparts, seed=20250114):
    """Owner (1-based) of every gid: nearest of nparts points uniform in the
    node box [0, N-1]³, ties to the lowest part (the C5 synthetic input)."""
    rng = np.random.default_rng(seed)
    pts = rng.uniform(0.0, 1.0, (nparts, 3)) * (np.asarray(N, dtype=np.float64) - 1.0)
    ng = int(np.prod(N))
    g = np.arange(ng, dtype=np.int64)
    x = (g % N[0]).astype(np.float64)
    y = ((g // N[0]) % N[1]).astype(np.float64)
    z = (g // (N[0] * N[1])).astype(np.float64)
    d = np.stack([((x - p[0]) ** 2 + (y - p[1]) ** 2) + (z - p[2]) ** 2 for p in pts], 0)
    return (np.argmin(d, axis=0) + 1).astype(np.int32)  # argmin: first minimum


def stencil_rows_vec(kind, N, gids, coef):
    """stencil_row_entries for many rows at once: (row position, column gid,
    value) in row order then neighbour order.  Interior rows all carry the
    entries of one interior node (taken from stencil_row_entries); Dirichlet
    rows come from stencil_row_entries row by row."""
    gids = np.asarray(gids, dtype=np.int64)
    Nx, Ny, Nz = N
    g0 = gids - 1
    gx, gy, gz = g0 % Nx, (g0 // Nx) % Ny, g0 // (Nx * Ny)
    dirm = (gx == 0) | (gx == Nx - 1) | (gy == 0) | (gy == Ny - 1) | (gz == 0) | (gz == Nz - 1)
    I, J, V = [], [], []
    inner = None
    if (~dirm).any():
        c = (1, 1, 1)
        ent = stencil_row_entries(kind, N, c, coef)
        inner = (np.array([(nb[0] - 1) + Nx * ((nb[1] - 1) + Ny * (nb[2] - 1)) for nb, _ in ent], np.int64),
                 np.array([v for _, v in ent], np.float64))
    # rows grouped into runs so the output keeps row order
    cnt = np.where(dirm, 1, len(inner[0]) if inner is not None else 0)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
    nnz = int(cnt.sum())
    I = np.repeat(np.arange(len(gids), dtype=np.int64), cnt)
    J = np.zeros(nnz, np.int64)
    V = np.zeros(nnz, np.float64)
    for r in np.flatnonzero(dirm):
        (nb, v), = stencil_row_entries(kind, N, (int(gx[r]), int(gy[r]), int(gz[r])), coef)
        J[start[r]] = 1 + nb[0] + Nx * (nb[1] + Ny * nb[2])
        V[start[r]] = v
    ii = np.flatnonzero(~dirm)
    if len(ii):
        k = len(inner[0])
        pos = start[ii][:, None] + np.arange(k)[None, :]
        J[pos] = gids[ii][:, None] + inner[0][None, :]
        V[pos] = inner[1][None, :]
    return I, J, V


def add_gids_owner_vec_(gid_to_part, a: IndexSet, gids):
    """add_gids_owner_ (first touch, Interfaces.jl:586-592, 618-627) for
    large gid lists: the unknown gids in order of first occurrence."""
    gids = np.asarray(gids, dtype=np.int64)
    known = np.asarray(a.lid_to_gid, dtype=np.int64)
    new = gids[~np.isin(gids, known)]
    u, first = np.unique(new, return_index=True)
    for g in u[np.argsort(first, kind="stable")]:
        _add_gid_ghost(a, int(g), gid_to_part(int(g)))
    return a


def to_lids_vec(ids, a: IndexSet):
    """to_lids_ for large id lists (every id must be a local gid)."""
    keys = np.asarray(a.lid_to_gid, dtype=np.int64)
    o = np.argsort(keys)
    i = np.searchsorted(keys[o], ids)
    assert np.array_equal(keys[o][i], ids)
    return o[i] + 1


def irregular_problem(parts: PData, N: tuple, kind=27, dtype=np.float64, owners=None, init=None):
    """C5 on the oracle: rows = IndexSets of the owned gids in gid order
    (IndexSets.jl:215-291), gid_to_part = owner map; COO of owned rows with
    global ids; cols = add_gids(rows, J) (first touch); psparse with
    ids=:global (Interfaces.jl:2194-2215)."""
    if owners is None:
        owners = voronoi_owners(N, num_parts(parts))
    coef = fd7_coeffs(N[0]) if kind == 7 else q1_hex_ke(2.0 / (N[0] - 1)).ravel()
    ngids = int(np.prod(N))
    g2p = lambda g: int(owners[g - 1])

    def mk(part):
        gids = np.flatnonzero(owners == part) + 1
        return IndexSet(part, gids, [part] * len(gids), list(range(1, len(gids) + 1)), [])
    rows = PRange(ngids, map_parts(mk, parts), None, map_parts(lambda _: g2p, parts), False)
    rows.exchanger = empty_exchanger(rows.partition)

    def coo(s):
        gids = np.asarray(s.lid_to_gid, np.int64)
        i, j, v = stencil_rows_vec(kind, N, gids, coef)
        return gids[i], j, v
    I, J, V = unzip(map_parts(coo, rows.partition), 3)
    cols = copy_prange(rows)
    map_parts(add_gids_owner_vec_, cols.gid_to_part, cols.partition, J)
    cols.exchanger = exchanger_from_ids(cols.partition)
    cols.ghost = True
    Il = map_parts(to_lids_vec, I, rows.partition)
    Jl = map_parts(to_lids_vec, J, cols.partition)
    V = map_parts(lambda v: _convert_values(v, dtype), V)
    return psparse_from_coo(Il, Jl, V, rows, cols, ids="local", init=init)


# ---------------------------------------------------------------------------
# Matrix nonzero exchange

def nzindex(A, i0, i1):
    """nzindex(A::SparseMatrixCSC, i0, i1) SparseUtils.jl:96-104 (-1 if absent);
    for a CSR parent SparseUtils.jl:210-220"""
    if isinstance(A, CSR):
        o = 1 - A.Bi
        r1, r2 = int(A.rowptr[i0 - 1]) + o, int(A.rowptr[i0]) - A.Bi
        if r1 > r2:
            return -1
        key = i1 - o
        lo, hi = r1, r2 + 1  # searchsortedfirst(colvals(A), i1-o, r1, r2)
        while lo < hi:
            mid = (lo + hi) // 2
            if A.colval[mid - 1] < key:
                lo = mid + 1
            else:
                hi = mid
        return lo if lo <= r2 and A.colval[lo - 1] == key else -1
    r1, r2 = int(A.colptr[i1 - 1]), int(A.colptr[i1]) - 1
    if r1 > r2:
        return -1
    lo, hi = r1, r2 + 1  # searchsortedfirst over rowval[r1:r2] (1-based positions)
    while lo < hi:
        mid = (lo + hi) // 2
        if A.rowval[mid - 1] < i0:
            lo = mid + 1
        else:
            hi = mid
    return lo if lo <= r2 and A.rowval[lo - 1] == i0 else -1


def nz_entries(A):
    """nziterator(A) for CSC (SparseUtils.jl:106-150), or for CSR
    (SparseUtils.jl:254-300, row by row): (k, li, lj) in storage order"""
    out = []
    if isinstance(A, CSR):
        for i in range(1, A.m + 1):
            for k in csr_nzrange(A, i):
                out.append((k, i, int(A.colval[k - 1]) + 1 - A.Bi))
        return out
    for j in range(1, A.n + 1):
        for k in range(int(A.colptr[j - 1]), int(A.colptr[j])):
            out.append((k, int(A.rowval[k - 1]), j))
    return out


def matrix_exchanger(values: PData, rows: PRange, cols: PRange) -> Exchanger:
    """matrix_exchanger(values, rows, cols) Interfaces.jl:2300-2372, literally."""
    if not rows.ghost:
        return empty_exchanger(rows.partition)
    parts_rcv = rows.exchanger.parts_rcv
    parts_snd = rows.exchanger.parts_snd
    parts = get_part_ids(rows.partition.shape if len(rows.partition.shape) > 1 else num_parts(rows.partition))

    def setup_rcv(part, prcv, rl, cl, A):
        owner_to_i = {o: i for i, o in enumerate(prcv)}
        counts = [0] * len(prcv)
        ents = nz_entries(A)
        for k, li, lj in ents:
            owner = rl.lid_to_part[li - 1]
            if owner != part:
                counts[owner_to_i[owner]] += 1
        ptrs = counts_to_ptrs(counts)
        n = int(ptrs[-1] - 1)
        kd, gi, gj = np.zeros(n, np.int64), np.zeros(n, np.int64), np.zeros(n, np.int64)
        cur = ptrs.copy()
        for k, li, lj in ents:
            owner = rl.lid_to_part[li - 1]
            if owner != part:
                i = owner_to_i[owner]
                p = int(cur[i]) - 1
                kd[p], gi[p], gj[p] = k, rl.lid_to_gid[li - 1], cl.lid_to_gid[lj - 1]
                cur[i] += 1
        return Table(kd, ptrs.copy()), Table(gi, ptrs.copy()), Table(gj, ptrs.copy())
    k_rcv, gi_rcv, gj_rcv = unzip(map_parts(setup_rcv, parts, parts_rcv, rows.partition, cols.partition,
                                            values), 3)
    gi_snd = exchange_tables(gi_rcv, parts_snd, parts_rcv)
    gj_snd = exchange_tables(gj_rcv, parts_snd, parts_rcv)

    def setup_snd(rl, cl, gi, gj, A):
        kd = np.zeros(len(gi.data), np.int64)
        for p in range(len(gi.data)):
            k = nzindex(A, rl.gid_to_lid[int(gi.data[p])], cl.gid_to_lid[int(gj.data[p])])
            assert k > 0, "The sparsity pattern of the ghost layer is inconsistent"
            kd[p] = k
        return Table(kd, gi.ptrs.copy())
    k_snd = map_parts(setup_snd, rows.partition, cols.partition, gi_snd, gj_snd, values)
    return Exchanger(parts_rcv, parts_snd, k_rcv, k_snd)


def exchange_matrix_(A: PSparseMatrix):
    """exchange!(A) Interfaces.jl:2375-2381"""
    nz = map_parts(lambda M: _CxList(M.nzval) if isinstance(M.nzval, Cx) else M.nzval, A.values)
    exchange_values_(_replace, nz, nz, A.exchanger)
    return A


def assemble_matrix_(A: PSparseMatrix):
    """assemble!(A) Interfaces.jl:2383-2404: reverse exchange with +, then
    nzval[lids_snd.data] .= 0 (lids_snd of the reversed exchanger)."""
    ex = reverse_exchanger(A.exchanger)
    nz = map_parts(lambda M: _CxList(M.nzval) if isinstance(M.nzval, Cx) else M.nzval, A.values)
    exchange_values_(lambda a, b: a + b, nz, nz, ex)

    def zero(M, lids):
        for k in lids.data:
            _set(M.nzval, int(k) - 1, _zero_like(M.nzval))
    map_parts(zero, A.values, ex.lids_snd)
    return A
