"""Index sets, PRange and the Exchanger (halo plan): the setup layer.

Host-side numpy restatement of IndexSets.jl:215-421 and Interfaces.jl:566-1573
(the partition the hot path is driven by).  Ids are 1-based like Julia's.
Everything here runs once per partition; nothing here touches vector or
matrix values.
"""
from __future__ import annotations

import numpy as np

from .backends import (MAIN, PData, alltoall, exchange, gather, map_parts, preduce, reduce_all, scatter, unzip,
                       xscan_all)
from .helpers import Table, counts_to_ptrs, trace_setup


# ---------------------------------------------------------------------------
# gid → lid lookup

class _SortedMap:
    def __init__(self, keys, vals):
        keys = np.asarray(keys, dtype=np.int64)
        o = np.argsort(keys, kind="stable")
        self.k = keys[o]
        self.v = np.asarray(vals, dtype=np.int64)[o]

    def get(self, q):
        q = np.asarray(q, dtype=np.int64)
        if len(self.k) == 0:
            return np.full(q.shape, -1, dtype=np.int64)
        i = np.searchsorted(self.k, q)
        i = np.minimum(i, len(self.k) - 1)
        hit = self.k[i] == q
        return np.where(hit, self.v[i], -1)


class IndexSet:
    """AbstractIndexSet (Interfaces.jl:566-577) with the fields of IndexSet
    (IndexSets.jl:215-291); IndexRange (343-421) is the special case built by
    `index_range`.  `owned_lookup(gids) -> lids or -1` is an optional fast
    path for structured owned ranges (Cartesian boxes, linear ranges)."""

    def __init__(self, part, lid_to_gid, lid_to_part, oid_to_lid=None, hid_to_lid=None,
                 owned_lookup=None):
        self.part = int(part)
        self.lid_to_gid = np.asarray(lid_to_gid, dtype=np.int64)
        self.lid_to_part = np.asarray(lid_to_part, dtype=np.int32)
        if oid_to_lid is None:  # IndexSets.jl:267-280
            own = self.lid_to_part == self.part
            oid_to_lid = np.flatnonzero(own) + 1
            hid_to_lid = np.flatnonzero(~own) + 1
        self.oid_to_lid = np.asarray(oid_to_lid, dtype=np.int32)
        self.hid_to_lid = np.asarray(hid_to_lid, dtype=np.int32)
        self._owned_lookup = owned_lookup
        self._map = None
        self._device = {}   # ctx id -> device index handle (device.py)

    # IndexSets.jl:254-256
    @property
    def lid_to_ohid(self):
        o = np.zeros(self.num_lids, dtype=np.int32)
        o[self.oid_to_lid - 1] = np.arange(1, self.num_oids + 1, dtype=np.int32)
        o[self.hid_to_lid - 1] = -np.arange(1, self.num_hids + 1, dtype=np.int32)
        return o

    num_lids = property(lambda s: len(s.lid_to_part))
    num_oids = property(lambda s: len(s.oid_to_lid))
    num_hids = property(lambda s: len(s.hid_to_lid))

    def copy(self):
        return IndexSet(self.part, self.lid_to_gid.copy(), self.lid_to_part.copy(),
                        self.oid_to_lid.copy(), self.hid_to_lid.copy(), self._owned_lookup)

    def lids_of(self, gids):
        """gid_to_lid[gids] (vectorised); -1 where absent."""
        gids = np.asarray(gids, dtype=np.int64)
        if self._owned_lookup is not None:
            lids = self._owned_lookup(gids)
            miss = lids < 0
            if miss.any() and self.num_hids:
                if self._map is None:
                    h = self.hid_to_lid.astype(np.int64)
                    self._map = _SortedMap(self.lid_to_gid[h - 1], h)
                lids = lids.copy()
                lids[miss] = self._map.get(gids[miss])
            return lids
        if self._map is None:
            self._map = _SortedMap(self.lid_to_gid, np.arange(1, self.num_lids + 1))
        return self._map.get(gids)

    def to_lids(self, gids):
        lids = self.lids_of(gids)
        if (lids < 0).any():
            bad = np.asarray(gids)[lids < 0][0]
            raise KeyError(f"gid {bad} is not a local id of part {self.part}")
        return lids

    def _append_ghosts(self, gids, parts):
        """_add_gid_ghost! for a batch (Interfaces.jl:595-603)"""
        n0 = self.num_lids
        k = len(gids)
        self.lid_to_gid = np.concatenate([self.lid_to_gid, np.asarray(gids, np.int64)])
        self.lid_to_part = np.concatenate([self.lid_to_part, np.asarray(parts, np.int32)])
        self.hid_to_lid = np.concatenate([self.hid_to_lid, np.arange(n0 + 1, n0 + k + 1, dtype=np.int32)])
        self._map = None
        self._device = {}

    def add_gids_owner(self, gid_to_part, gids):
        """add_gids!(gid_to_part, a, gids) (Interfaces.jl:586-592, 618-627):
        unknown gids become ghosts in first-touch order."""
        gids = np.asarray(gids, dtype=np.int64).ravel()
        new = gids[self.lids_of(gids) < 0]
        if len(new) == 0:
            return self
        u, first = np.unique(new, return_index=True)
        new = u[np.argsort(first, kind="stable")]
        self._append_ghosts(new, gid_to_part(new))
        return self

    def add_gids_parts(self, gids, parts):
        """add_gids!(a, i_to_gid, i_to_part) (Interfaces.jl:579-584, 605-616)"""
        gids = np.asarray(gids, dtype=np.int64).ravel()
        parts = np.asarray(parts, dtype=np.int32).ravel()
        keep = (parts != self.part) & (self.lids_of(gids) < 0)
        g, p = gids[keep], parts[keep]
        if len(g) == 0:
            return self
        u, first = np.unique(g, return_index=True)
        o = np.sort(first)
        self._append_ghosts(g[o], p[o])
        return self


def index_range(part, noids, firstgid, hid_to_gid=(), hid_to_part=()):
    """IndexRange(part, noids, firstgid[, hid_to_gid, hid_to_part]) IndexSets.jl:364-421"""
    noids = int(noids)
    lid_to_gid = np.concatenate([np.arange(firstgid, firstgid + noids, dtype=np.int64),
                                 np.asarray(hid_to_gid, np.int64)])
    lid_to_part = np.concatenate([np.full(noids, part, np.int32), np.asarray(hid_to_part, np.int32)])
    nh = len(hid_to_gid)

    def owned(g, f=int(firstgid), n=noids):
        inside = (g >= f) & (g < f + n)
        return np.where(inside, g - f + 1, -1)
    return IndexSet(part, lid_to_gid, lid_to_part, np.arange(1, noids + 1),
                    np.arange(noids + 1, noids + nh + 1), owned_lookup=owned)


# ---------------------------------------------------------------------------
# Partition math (Interfaces.jl:1307-1319, 1473-1499)

def oid_range(ngids, np_, p):
    """_oid_to_gid → (first, last) inclusive, Interfaces.jl:1307-1319"""
    _olength = ngids // np_
    _offset = _olength * (p - 1)
    _rem = ngids % np_
    if _rem < (np_ - p + 1):
        olength, offset = _olength, _offset
    else:
        olength = _olength + 1
        offset = _offset + p - (np_ - _rem) - 1
    return 1 + offset, olength + offset


def cartesian_index(shape, lin):
    lin = np.asarray(lin, dtype=np.int64) - 1
    out = []
    for s in shape:
        out.append(lin % s + 1)
        lin = lin // s
    return tuple(out)


def linear_index(shape, ci):
    lin = np.zeros_like(np.asarray(ci[0], dtype=np.int64))
    stride = 1
    for s, c in zip(shape, ci):
        lin = lin + (np.asarray(c, dtype=np.int64) - 1) * stride
        stride *= s
    return lin + 1


def part_to_firstgid(ngids, np_):
    """Interfaces.jl:1493-1495"""
    return np.array([oid_range(ngids, np_, p)[0] for p in range(1, np_ + 1)], dtype=np.int64)


def linear_gid_to_part(firsts):
    """LinearGidToPart (IndexSets.jl:174-193)"""
    firsts = np.asarray(firsts, dtype=np.int64)
    return lambda g: np.searchsorted(firsts, np.asarray(g, np.int64), side="right").astype(np.int32)


def cartesian_gid_to_part(ngids, np_):
    """CartesianGidToPart (IndexSets.jl:195-213)"""
    firsts = [part_to_firstgid(n, p) for n, p in zip(ngids, np_)]

    def f(g):
        cg = cartesian_index(ngids, g)
        cp = [np.searchsorted(fs, c, side="right") for fs, c in zip(firsts, cg)]
        return linear_index(np_, cp).astype(np.int32)
    return f


def box_of_part(ngids, np_, part):
    """Owned box (lo 1-based, n) per dim of Cartesian part `part`."""
    cp = [int(c) for c in cartesian_index(np_, part)]
    lo, n = [], []
    for d in range(len(ngids)):
        a, b = oid_range(ngids[d], np_[d], cp[d])
        lo.append(a)
        n.append(b - a + 1)
    return tuple(lo), tuple(n)


def box_gids(ngids, lo, n):
    """_id_tensor_product of the owned box (Interfaces.jl:1473-1491):
    local order first dim fastest."""
    axes = [np.arange(l, l + k, dtype=np.int64) for l, k in zip(lo, n)]
    grids = np.meshgrid(*axes[::-1], indexing="ij")[::-1]
    return linear_index(ngids, [g.ravel() for g in grids])


def box_lookup(ngids, lo, n):
    def f(g):
        ci = cartesian_index(ngids, g)
        inside = np.ones(np.shape(g), dtype=bool)
        loc = []
        for d in range(len(ngids)):
            c = ci[d] - lo[d]
            inside &= (c >= 0) & (c < n[d])
            loc.append(c + 1)
        return np.where(inside, linear_index(n, loc), -1)
    return f


# ---------------------------------------------------------------------------
# Exchanger (Interfaces.jl:698-961)

class Exchanger:
    """Exchanger{parts_rcv,parts_snd,lids_rcv,lids_snd} (Interfaces.jl:698-713)."""

    def __init__(self, parts_rcv, parts_snd, lids_rcv, lids_snd):
        self.parts_rcv = parts_rcv
        self.parts_snd = parts_snd
        self.lids_rcv = lids_rcv
        self.lids_snd = lids_snd
        self._device = {}

    def reverse(self):
        """Base.reverse (Interfaces.jl:796-798)"""
        return Exchanger(self.parts_snd, self.parts_rcv, self.lids_snd, self.lids_rcv)


def _parts_rcv_to_parts_snd(parts_rcv_all):
    """Interfaces.jl:525-552: transpose the receive graph (senders list their
    receivers ascending)."""
    np_ = len(parts_rcv_all)
    snd = [[] for _ in range(np_)]
    for p in range(1, np_ + 1):
        for q in sorted(set(int(x) for x in parts_rcv_all[p - 1])):
            snd[q - 1].append(p)
    return [np.array(sorted(s), dtype=np.int32) for s in snd]


def discover_parts_snd(parts_rcv: PData, neighbors=None, method="alltoall") -> PData:
    """discover_parts_snd (Interfaces.jl:471-521).  With `neighbors` (a
    superset of both the senders and the receivers): each part tells its
    neighbours whether it receives from them (Interfaces.jl:471-496).
    Without: method "alltoall" (default) — each part marks the parts it
    receives from in a P-int vector and one all-to-all of those vectors
    tells every part who receives from it (part q learns p iff p receives
    from q; P ints per part, no part holds the whole graph); method
    "gather" — the reference's fallback (Interfaces.jl:515-521, flagged
    there as non-scalable, :500-510): gather the graph on MAIN, transpose
    (:525-552), scatter.  All give parts_snd ascending."""
    if neighbors is None:
        if method == "gather":
            main = gather(parts_rcv)
            snd = map_parts(lambda v: _parts_rcv_to_parts_snd(v) if len(v) else [], main)
            return scatter(snd)
        if method != "alltoall":
            raise ValueError(f"discover_parts_snd: unknown method {method!r}")
        P = parts_rcv.num_parts

        def marks(prcv):
            m = np.zeros(P, dtype=np.int64)
            for q in prcv:
                if not 1 <= int(q) <= P:
                    raise ValueError(f"discover_parts_snd: part {int(q)} out of 1..{P}")
                m[int(q) - 1] = 1
            return m
        col = alltoall(map_parts(marks, parts_rcv))
        return map_parts(lambda c: (np.flatnonzero(c) + 1).astype(np.int32), col)
    parts = PData(parts_rcv.backend, parts_rcv.part_ids, parts_rcv.part_ids, parts_rcv.shape)

    def tell(part, nb, prcv):
        s = set(int(x) for x in prcv)
        return [part if int(n) in s else -1 for n in nb]
    data = map_parts(tell, parts, neighbors, parts_rcv)
    got = exchange(data, neighbors, neighbors)
    return map_parts(lambda d: np.array([x for x in d if x > 0], dtype=np.int32), got)


def grid_neighbors(part_shape, part):
    """The parts of a Cartesian part grid within one step of `part` in every
    direction (3^d - 1 at most), ascending: the neighbour superset of a
    one-layer ghost (IndexSets.jl:195-213 geometry)."""
    cp = [int(c) for c in cartesian_index(part_shape, part)]
    rng = [range(max(1, c - 1), min(n, c + 1) + 1) for c, n in zip(cp, part_shape)]
    mesh = np.meshgrid(*[np.array(list(r)) for r in rng], indexing="ij")
    nb = np.sort(linear_index(part_shape, [m.ravel() for m in mesh]))
    return nb[nb != part].astype(np.int32)


def grid_neighbors_if_superset(ids: PData, part_shape):
    """Neighbours for discover_parts_snd(parts_rcv, neighbors)
    (Interfaces.jl:471-496) when every part's ghost owners are grid
    neighbours: the grid relation is symmetric, so it is then a superset of
    both the receivers and the senders.  Each part checks its own ghosts; one
    reduce_all AND decides for all (None: the caller falls back to the
    gather-based discovery, Interfaces.jl:515-521)."""
    nbrs = map_parts(lambda s: grid_neighbors(part_shape, s.part), ids)

    def ok(s, nb):
        ghost = s.lid_to_part[s.lid_to_part != s.part]
        return bool(np.all(np.isin(ghost, nb)))
    good = reduce_all(lambda a, b: a and b, map_parts(ok, ids, nbrs), True)
    return nbrs if all(good.parts) else None


def exchanger_from_ids(ids: PData, neighbors=None, reuse_parts_rcv=False, discover="alltoall") -> Exchanger:
    """Exchanger(ids; reuse_parts_rcv) Interfaces.jl:723-786, vectorised
    (parts_snd by discover_parts_snd(..., method=discover) without
    neighbours)."""
    def rcv(s: IndexSet):
        ghost = np.flatnonzero(s.lid_to_part != s.part)
        owners = s.lid_to_part[ghost]
        prcv = np.unique(owners).astype(np.int32)
        o = np.argsort(owners, kind="stable")  # group by owner, ascending lid inside
        lids = (ghost[o] + 1).astype(np.int32)
        counts = np.bincount(np.searchsorted(prcv, owners), minlength=len(prcv)) if len(prcv) else []
        ptrs = counts_to_ptrs(counts)
        return prcv, Table(lids, ptrs), Table(s.lid_to_gid[lids - 1], ptrs.copy())
    parts_rcv, lids_rcv, gids_rcv = unzip(map_parts(rcv, ids), 3)
    if reuse_parts_rcv:
        parts_snd = parts_rcv
    else:
        parts_snd = discover_parts_snd(parts_rcv, neighbors, discover)
    # exchange(gids_rcv, parts_snd, parts_rcv): segment i goes to parts_rcv[i]
    segs = map_parts(lambda t: [t[i] for i in range(1, len(t) + 1)], gids_rcv)
    got = exchange(segs, parts_snd, parts_rcv)

    backend = ids.backend
    if hasattr(backend, "context"):  # HIP parts: to_lids! through the device gid table
        from .device import device_to_lids
        to_lids = lambda s, g: device_to_lids(backend.context(s.part), s, g)
    else:
        to_lids = lambda s, g: s.to_lids(g)

    def snd(s: IndexSet, g):
        ptrs = counts_to_ptrs([len(x) for x in g])
        data = np.concatenate(g).astype(np.int64) if g else np.zeros(0, np.int64)
        return Table(to_lids(s, data).astype(np.int32), ptrs)
    lids_snd = map_parts(snd, ids, got)
    parts_rcv = map_parts(lambda p: np.asarray(p, np.int32), parts_rcv)
    parts_snd = map_parts(lambda p: np.asarray(p, np.int32), parts_snd)
    return Exchanger(parts_rcv, parts_snd, lids_rcv, lids_snd)


def empty_exchanger(a: PData) -> Exchanger:
    """Interfaces.jl:788-794"""
    e = map_parts(lambda _: np.zeros(0, np.int32), a)
    t = lambda _: Table(np.zeros(0, np.int32), np.ones(1, np.int32))
    return Exchanger(e, map_parts(lambda _: np.zeros(0, np.int32), a), map_parts(t, a), map_parts(t, a))


# ---------------------------------------------------------------------------
# PRange (Interfaces.jl:963-1573)

class PRange:
    """Partitioned range of global ids (Interfaces.jl:964-987)."""

    def __init__(self, ngids, partition: PData, exchanger: Exchanger, gid_to_part=None, ghost=True,
                 part_shape=None):
        self.ngids = int(ngids)
        self.partition = partition
        self.exchanger = exchanger
        self.gid_to_part = gid_to_part
        self.ghost = ghost
        # Cartesian part grid (prange_cartesian): lets add_gids! discover
        # parts_snd from grid neighbours instead of a gather on MAIN
        self.part_shape = part_shape

    def __len__(self):
        return self.ngids

    @property
    def num_parts(self):
        return self.partition.num_parts

    def copy(self):
        part = map_parts(lambda s: s.copy(), self.partition)
        return PRange(self.ngids, part, self.exchanger, self.gid_to_part, self.ghost, self.part_shape)


def prange_from_partition(ngids, partition: PData, gid_to_part=None, ghost=True) -> PRange:
    """PRange(ngids, partition[, gid_to_part, ghost]) Interfaces.jl:998-1006"""
    ex = exchanger_from_ids(partition) if ghost else empty_exchanger(partition)
    return PRange(ngids, partition, ex, gid_to_part, ghost)


def prange_linear(parts: PData, ngids: int) -> PRange:
    """PRange(parts, ngids) Interfaces.jl:1014-1030"""
    np_ = parts.num_parts
    firsts = part_to_firstgid(ngids, np_)

    def mk(part):
        a, b = oid_range(ngids, np_, part)
        return index_range(part, b - a + 1, a)
    partition = map_parts(mk, parts)
    g2p = map_parts(lambda _: linear_gid_to_part(firsts), parts)
    return PRange(ngids, partition, empty_exchanger(partition), g2p, False)


def prange_noids(parts: PData, noids: PData, ngids=None) -> PRange:
    """PRange(parts, noids) Interfaces.jl:1038-1068"""
    if ngids is None:
        ngids = preduce(lambda a, b: a + b, noids, 0)
    firsts = xscan_all(lambda a, b: a + b, noids, 1)
    partition = map_parts(lambda part, n, f: index_range(part, n, f[part - 1]), parts, noids, firsts)
    g2p = map_parts(lambda f: linear_gid_to_part(np.asarray(f)), firsts)
    return PRange(ngids, partition, empty_exchanger(partition), g2p, False)


def _lids_1d(ngids, np_, p, periodic):
    """One dimension of a Cartesian part with its ghost layer (Interfaces.jl:
    1321-1335 / 1353-1373 and 1375-1411): the gids of the local ids and the
    part coordinate owning each — the owned range, one ghost id before it
    (from part p-1, or wrapped around from the last part when periodic) and
    one after it (part p+1, or wrapped to the first); a single part in the
    dimension has no ghost layer there."""
    a, b = oid_range(ngids, np_, p)
    g = np.arange(a, b + 1, dtype=np.int64)
    c = np.full(len(g), p, dtype=np.int64)
    if np_ == 1:
        return g, c
    if p > 1 or periodic:
        g = np.concatenate([[a - 1 if p > 1 else ngids], g])
        c = np.concatenate([[p - 1 if p > 1 else np_], c])
    if p < np_ or periodic:
        g = np.concatenate([g, [b + 1 if p < np_ else 1]])
        c = np.concatenate([c, [p + 1 if p < np_ else 1]])
    return g, c


def _tensor(axes, shape):
    """_id_tensor_product (Interfaces.jl:1473-1491): linear ids in `shape` of
    the per-dimension ids, first dimension fastest."""
    grids = np.meshgrid(*[np.asarray(a) for a in axes[::-1]], indexing="ij")[::-1]
    return linear_index(shape, [g.ravel() for g in grids])


def prange_cartesian(parts: PData, ngids: tuple, with_ghost=False, isperiodic=None) -> PRange:
    """PRange(parts, ngids::NTuple) Interfaces.jl:1114-1137 (no ghost layer);
    with_ghost (1166-1193): every part also holds the one-wide layer of its
    neighbours' ids, in the local Cartesian order, so owned and ghost lids
    interleave (oid_to_lid / hid_to_lid = findall of the owner), and the
    Exchanger reuses parts_rcv as parts_snd; isperiodic (1195-1223) wraps the
    layer around the global boundary."""
    np_ = parts.shape
    if len(np_) != len(ngids):
        raise ValueError("Cartesian PRange needs len(parts.shape) == len(ngids)")
    if with_ghost:
        per = tuple(isperiodic) if isperiodic is not None else (False,) * len(ngids)

        def mk_ghost(part):
            cp = [int(c) for c in cartesian_index(np_, part)]
            gs, cs = zip(*[_lids_1d(ngids[d], np_[d], cp[d], per[d]) for d in range(len(ngids))])
            return IndexSet(part, _tensor(gs, ngids), _tensor(cs, np_))  # oid/hid = findall (IndexSets.jl:267-280)
        partition = map_parts(mk_ghost, parts)
        g2p = map_parts(lambda _: cartesian_gid_to_part(ngids, np_), parts)
        ex = exchanger_from_ids(partition, reuse_parts_rcv=True)
        return PRange(int(np.prod(ngids)), partition, ex, g2p, True, tuple(np_))

    def mk(part):
        lo, n = box_of_part(ngids, np_, part)
        gids = box_gids(ngids, lo, n)
        k = len(gids)
        return IndexSet(part, gids, np.full(k, part, np.int32), np.arange(1, k + 1),
                        np.zeros(0, np.int32), owned_lookup=box_lookup(ngids, lo, n))
    partition = map_parts(mk, parts)
    g2p = map_parts(lambda _: cartesian_gid_to_part(ngids, np_), parts)
    return PRange(int(np.prod(ngids)), partition, empty_exchanger(partition), g2p, False, tuple(np_))


def add_gids_(a: PRange, gids: PData, i_to_part: PData = None, neighbors=None) -> PRange:
    """add_gids!(a::PRange, gids[, i_to_part]) Interfaces.jl:1501-1533"""
    trace = trace_setup()
    t0 = trace()
    if i_to_part is not None:
        map_parts(lambda s, g, p: s.add_gids_parts(g, p), a.partition, gids, i_to_part)
    else:
        if a.gid_to_part is None:
            raise ValueError("DomainError: the PRange has no gid_to_part; pass the owners")
        backend = a.partition.backend
        if hasattr(backend, "context"):  # HIP parts: first-touch discovery on the device
            from .device import device_first_touch

            def dev(f, s, g):
                new = device_first_touch(backend.context(s.part), s, g)
                if len(new):
                    s._append_ghosts(new, f(new))
                return s
            map_parts(dev, a.gid_to_part, a.partition, gids)
        else:
            map_parts(lambda f, s, g: s.add_gids_owner(f, g), a.gid_to_part, a.partition, gids)
    t1 = trace("add_gids! first touch", t0)
    if neighbors is None and a.part_shape is not None:
        neighbors = grid_neighbors_if_superset(a.partition, a.part_shape)
    a.exchanger = exchanger_from_ids(a.partition, neighbors)
    trace("exchanger_from_ids", t1)
    a.ghost = True
    return a


def add_gids(a: PRange, gids: PData, i_to_part: PData = None, neighbors=None) -> PRange:
    """Interfaces.jl:1535-1539"""
    return add_gids_(a.copy(), gids, i_to_part, neighbors)


def assemble_coo_(I: PData, J: PData, V: PData, rows: PRange):
    """async_assemble!(I, J, V, rows) + wait (Interfaces.jl:2406-2492), host
    setup: triplets whose row (global id, present in rows) is owned by another
    part are sent to that owner — segments in rows.exchanger.parts_rcv order,
    input order inside — their local value is set to zero and kept; received
    triplets are appended in the receive order.  I, J stay global ids."""
    def setup(s, prcv, i, j, v):
        i = np.asarray(i, np.int64)
        j = np.asarray(j, np.int64)
        v = np.asarray(v).copy()
        owner = s.lid_to_part[s.to_lids(i) - 1]
        remote = owner != s.part
        seg = np.searchsorted(prcv, owner[remote])
        o = np.argsort(seg, kind="stable")
        gi, gj, gv = i[remote][o], j[remote][o], v[remote][o]
        bounds = np.concatenate([[0], np.cumsum(np.bincount(seg, minlength=len(prcv)))]).astype(np.int64)
        msgs = [(gi[a:b], gj[a:b], gv[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]
        v[remote] = 0
        return (i, j, v), msgs
    local, msgs = unzip(map_parts(setup, rows.partition, rows.exchanger.parts_rcv, I, J, V), 2)
    got = exchange(msgs, rows.exchanger.parts_snd, rows.exchanger.parts_rcv)

    def append(loc, g):
        i, j, v = loc
        if g:
            i = np.concatenate([i] + [m[0] for m in g])
            j = np.concatenate([j] + [m[1] for m in g])
            v = np.concatenate([v] + [m[2] for m in g])
        return i, j, v
    return unzip(map_parts(append, local, got), 3)


def to_lids_(ids: PData, a: PRange) -> PData:
    """to_lids! (Interfaces.jl:1541-1543)"""
    def f(g, s):
        g[...] = s.to_lids(g)
        return g
    return map_parts(f, ids, a.partition)


def _cached_eq(kind, a: PRange, b: PRange, f):
    # the @check of mul!/copyto!/broadcasts (Interfaces.jl:1550-1554) is a
    # gather+bcast per call in the reference; the partitions are immutable
    # between add_gids! calls, so the answer is cached per (a, b, sizes)
    key = (kind, id(b.partition), tuple(s.num_lids for s in b.partition.parts),
           tuple(s.num_lids for s in a.partition.parts))
    cache = a.__dict__.setdefault("_eq_cache", {})
    hit = cache.get(key)
    if hit is None or hit[0] is not b.partition:  # keep b alive: no id reuse
        c = map_parts(f, a.partition, b.partition)
        hit = (b.partition, bool(preduce(lambda u, v: u and v, c, True)))
        cache[key] = hit
    return hit[1]


def oids_are_equal(a: PRange, b: PRange) -> bool:
    """Interfaces.jl:1549-1556"""
    if a.partition is b.partition:
        return True
    return _cached_eq("oids", a, b, lambda x, y: bool(np.array_equal(x.lid_to_gid[x.oid_to_lid - 1],
                                                                     y.lid_to_gid[y.oid_to_lid - 1])))


def hids_are_equal(a: PRange, b: PRange) -> bool:
    """Interfaces.jl:1558-1565"""
    if a.partition is b.partition:
        return True
    return _cached_eq("hids", a, b, lambda x, y: bool(np.array_equal(x.lid_to_gid[x.hid_to_lid - 1],
                                                                     y.lid_to_gid[y.hid_to_lid - 1])))


def lids_are_equal(a: PRange, b: PRange) -> bool:
    if a.partition is b.partition:
        return True
    c = map_parts(lambda x, y: bool(np.array_equal(x.lid_to_gid, y.lid_to_gid)), a.partition, b.partition)
    return bool(preduce(lambda u, v: u and v, c, True))
