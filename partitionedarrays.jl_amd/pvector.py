"""PVector / PSparseMatrix on HIP parts and the hot path (Interfaces.jl:1576-2757).

Values live in HBM (one pa_vec / pa_mat per part); every operation below is
a libpa_hip.so call — there is no host fallback.  Host arrays appear only at
construction (upload of the reference's local CSC / initial values) and when
the caller asks for them (`to_host`).
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict
import math
import sys
import weakref

import numpy as np

from . import _lib
from .backends import PData, exchange, map_parts, unzip
from .device import (DeviceCOO, DeviceMatrix, DeviceMatrixExchanger, DeviceVector, contexts, device_exchanger,
                     device_index, device_index_gids)
from .helpers import Table, counts_to_ptrs, trace_setup
from .prange import Exchanger, PRange, _cached_eq, empty_exchanger, hids_are_equal, oids_are_equal


# ---------------------------------------------------------------------------
# Local CSC (setup): SparseArrays.sparse semantics, SparseUtils.jl:80-94

class CSC:
    """SparseMatrixCSC{T,Int64}: 1-based colptr/rowval."""

    def __init__(self, m, n, colptr, rowval, nzval):
        self.m, self.n = int(m), int(n)
        self.colptr = np.asarray(colptr, dtype=np.int64)
        self.rowval = np.asarray(rowval, dtype=np.int64)
        self.nzval = np.asarray(nzval)

    @property
    def nnz(self):
        return int(self.colptr[-1] - 1)


def compresscoo(I, J, V, m, n) -> CSC:
    """sparse(I, J, V, m, n, +): duplicates combined with `+` in input order
    (left fold from the first occurrence), rows ascending within columns."""
    I = np.asarray(I, dtype=np.int64).ravel()
    J = np.asarray(J, dtype=np.int64).ravel()
    V = np.asarray(V).ravel()
    k = len(I)
    if k and (I.min() < 1 or I.max() > m or J.min() < 1 or J.max() > n):
        raise IndexError("compresscoo: index out of bounds")
    order = np.lexsort((np.arange(k), I, J))
    Is, Js, Vs = I[order], J[order], V[order]
    new = np.ones(k, dtype=bool)
    new[1:] = (Is[1:] != Is[:-1]) | (Js[1:] != Js[:-1])
    starts = np.flatnonzero(new)
    sizes = np.diff(np.append(starts, k))
    acc = Vs[starts].copy()
    for t in range(1, int(sizes.max()) if k else 1):
        sel = sizes > t
        acc[sel] = acc[sel] + Vs[starts[sel] + t]
    cols = Js[starts]
    colptr = np.concatenate([[1], 1 + np.cumsum(np.bincount(cols - 1, minlength=n))]).astype(np.int64)
    return CSC(m, n, colptr, Is[starts], acc)


class CSR:
    """SparseMatrixCSR{Bi,T,Int64} (SparseUtils.jl:189-300): rowptr and
    colval hold Bi-based indices (Bi = 0 or 1), nzval in row order."""

    def __init__(self, Bi, m, n, rowptr, colval, nzval):
        if Bi not in (0, 1):
            raise ValueError("SparseMatrixCSR: Bi must be 0 or 1")
        self.Bi, self.m, self.n = int(Bi), int(m), int(n)
        self.rowptr = np.asarray(rowptr, dtype=np.int64)
        self.colval = np.asarray(colval, dtype=np.int64)
        self.nzval = np.asarray(nzval)

    @property
    def nnz(self):
        return int(self.rowptr[-1] - self.Bi)


def sparsecsr(Bi, I, J, V, m, n) -> CSR:
    """compresscoo(SparseMatrixCSR{Bi}, I, J, V, m, n) (SparseUtils.jl:
    193-208) → sparsecsr(Val(Bi), I, J, V, m, n, +): the CSC of the
    transposed triplets read as rows (duplicates combined with + in input
    order, columns ascending within rows), indices shifted to base Bi."""
    t = compresscoo(J, I, V, n, m)
    return CSR(Bi, m, n, t.colptr - 1 + Bi, t.rowval - 1 + Bi, t.nzval)


class csr_init:
    """init for PSparseMatrix.from_coo: sparsecsr with index base Bi (the
    compress then runs on the device, pa_mat_from_coo_csr); called as
    init(I, J, V, m, n) it is the host sparsecsr."""

    def __init__(self, Bi):
        if Bi not in (0, 1):
            raise ValueError("SparseMatrixCSR: Bi must be 0 or 1")
        self.Bi = int(Bi)

    def __call__(self, I, J, V, m, n):
        return sparsecsr(self.Bi, I, J, V, m, n)


# ---------------------------------------------------------------------------
# PVector

class PVector:
    """PVector{T}(values, rows) (Interfaces.jl:1576-1587): values = PData of
    DeviceVector (num_lids(rows) entries per part)."""

    def __init__(self, values: PData, rows: PRange):
        self.values = values
        self.rows = rows

    @property
    def dtype(self):
        return self.values.parts[0].dtype if self.values.parts else np.dtype(np.float64)

    def __len__(self):
        return len(self.rows)

    @staticmethod
    def undef(rows: PRange, dtype=np.float64) -> "PVector":
        """PVector{T}(undef, rows) (Interfaces.jl:1869-1878); zero-initialised."""
        ctxs = contexts(rows.partition)
        vals = [DeviceVector(c, dtype, s.num_lids) for c, s in zip(ctxs, rows.partition.parts)]
        return PVector(PData(rows.partition.backend, rows.partition.part_ids, vals, rows.partition.shape), rows)

    @staticmethod
    def full(v, rows: PRange, dtype=None) -> "PVector":
        """PVector(v::Number, rows) (Interfaces.jl:1880-1884)"""
        dtype = dtype or np.asarray(v).dtype
        a = PVector.undef(rows, dtype)
        a.fill_(v)
        return a

    @staticmethod
    def from_host(host: PData, rows: PRange, dtype=None) -> "PVector":
        dtype = dtype or np.asarray(host.parts[0]).dtype
        a = PVector.undef(rows, dtype)
        for dv, h in zip(a.values.parts, host.parts):
            dv.upload(h)
        return a

    def to_host(self) -> PData:
        return map_parts(lambda v: v.download(), self.values)

    def owned_values(self) -> PData:
        """owned_values view (Interfaces.jl:1589-1593), as host copies"""
        return map_parts(lambda v, s: v.download()[s.oid_to_lid - 1], self.values, self.rows.partition)

    def ghost_values(self) -> PData:
        return map_parts(lambda v, s: v.download()[s.hid_to_lid - 1], self.values, self.rows.partition)

    def similar(self, dtype=None, rows=None) -> "PVector":
        """similar(a[, T][, axes]) (Interfaces.jl:1615-1633)"""
        return PVector.undef(rows or self.rows, dtype or self.dtype)

    def fill_(self, v):
        """fill!(a, v) (Interfaces.jl:1966-1971)"""
        for dv in self.values.parts:
            dv.fill(v)
        return self

    def copy(self) -> "PVector":
        """copy(b) (Interfaces.jl:1669-1673)"""
        a = self.similar()
        copyto_(a, self)
        return a


def _idx(v: PVector):
    return [device_index(c, s).h for c, s in zip(contexts(v.rows.partition), v.rows.partition.parts)]


def copyto_(a: PVector, b: PVector) -> PVector:
    """copyto!(a, b) (Interfaces.jl:1659-1667): all lids when both share the
    partition, owned values otherwise."""
    same = a.rows.partition is b.rows.partition
    if not same and not oids_are_equal(a.rows, b.rows):
        raise AssertionError("copyto!: owned ids differ")
    ia, ib = _idx(a), _idx(b)
    for da, db, xa, xb in zip(a.values.parts, b.values.parts, ia, ib):
        _lib.call("pa_vec_copy", da.h, xa, db.h, xb, 1 if same else 0)
    return a


def _scalar_kind(a, dtype):
    """the scalar of a broadcast as Julia types it: a Python float is a
    Float64 and a Python complex a ComplexF64 (np.float64 / np.complex128
    likewise) — the elements are then evaluated in Float64 / ComplexF64 and
    rounded once (pa_vec_axpby PA_BCAST_*); ints and scalars of narrower or
    equal type are converted to the element type."""
    cplx = np.dtype(dtype).kind == "c"
    if isinstance(a, (complex, np.complex128)) and not isinstance(a, (float, np.floating)):
        if not cplx:
            if complex(a).imag != 0:
                raise TypeError("broadcast: a complex scalar into a real vector (InexactError)")
            return np.float64(complex(a).real), _lib.PA_BCAST_F64
        return np.complex128(a), _lib.PA_BCAST_C128
    if isinstance(a, (float, np.float64)):
        return np.float64(a), _lib.PA_BCAST_F64
    return a, 0


def _bcast(y: PVector, x: PVector, a, mode):
    all_lids = 1 if (x is None or y.rows is x.rows) else 0
    if x is not None and not all_lids and not oids_are_equal(y.rows, x.rows):
        raise AssertionError("broadcast: owned ids differ")
    iy = _idx(y)
    a, kind = _scalar_kind(a if a is not None else 0, y.dtype)
    mode |= kind
    buf, bp = _lib.scalar_buf(a, a.dtype if kind else y.dtype)
    xs = x.values.parts if x is not None else [None] * len(y.values.parts)
    for dy, dx, i in zip(y.values.parts, xs, iy):
        _lib.call("pa_vec_axpby", dy.h, dx.h if dx is not None else None, i, bp, mode, all_lids)
    return y


def xpby_(u: PVector, r: PVector, beta):
    """u .= r .+ β .* u"""
    return _bcast(u, r, beta, 0)


def axpy_(x: PVector, alpha, u: PVector):
    """x .+= α .* u"""
    return _bcast(x, u, alpha, 1)


def axmy_(r: PVector, alpha, c: PVector):
    """r .-= α .* c"""
    return _bcast(r, c, alpha, 2)


def sub_(r: PVector, c: PVector):
    """r .-= c"""
    return _bcast(r, c, None, 3)


def rmul_(a: PVector, v):
    """rmul!(a, v) (Interfaces.jl:1675-1680)"""
    return _bcast(a, None, v, 4)


def _hs(objs):
    return _lib.ptr_array([o.h if o is not None else None for o in objs])


def exchange_(v):
    """exchange!(v) (Interfaces.jl:453-458, 2071-2075): owner → ghost values.
    For a PSparseMatrix: exchange!(A) over nonzeros(A) (2375-2381)."""
    if isinstance(v, PSparseMatrix):
        return _mat_exchange(v, _lib.PA_REPLACE, 0, 0)
    ctxs = contexts(v.values)
    xg = [device_exchanger(c, v.rows.exchanger, p) for c, p in zip(ctxs, v.values.part_ids)]
    n = len(ctxs)
    _lib.call("pa_exchange_all", n, _hs(v.values.parts), _hs(xg), _lib.ptr_array(_idx(v)),
              _lib.PA_REPLACE, 0, 0)
    return v


class COO:
    """The (I, J, V) triplets of a PSparseMatrix before `sparse`, on the
    device: one pa_coo per part, I and J global ids (test_fem_sa.jl:60-131,
    ids=:global)."""

    def __init__(self, values: PData):
        self.values = values

    @staticmethod
    def from_host(I: PData, J: PData, V: PData, rows: PRange) -> "COO":
        ctxs = contexts(rows.partition)
        parts = [DeviceCOO(c, i, j, v) for c, i, j, v in zip(ctxs, I.parts, J.parts, V.parts)]
        p = rows.partition
        return COO(PData(p.backend, p.part_ids, parts, p.shape))

    def to_host(self):
        """(I, J, V) as PData of host arrays"""
        return unzip(map_parts(lambda c: c.download(), self.values), 3)

    def global_cols(self) -> PData:
        """J of every part (host), e.g. for add_gids!(cols, J)"""
        return map_parts(lambda c: c.download()[1], self.values)


def _assemble_coo(coo: COO, rows: PRange) -> COO:
    """async_assemble!(I, J, V, rows) + wait (Interfaces.jl:2406-2492) on the
    device (pa_coo_assemble_all): triplets of rows owned elsewhere go to the
    owner (local value set to zero, entry kept), received ones are appended
    in rows.exchanger.parts_snd order."""
    ctxs = contexts(rows.partition)
    pids = rows.partition.part_ids
    idx = [device_index_gids(c, rows.partition.local(p)) for c, p in zip(ctxs, pids)]
    xg = [device_exchanger(c, rows.exchanger, p) for c, p in zip(ctxs, pids)]
    _lib.call("pa_coo_assemble_all", len(ctxs), _hs(coo.values.parts), _hs(idx), _hs(xg))
    return coo


def assemble_(v, rows: PRange = None):
    """assemble!(v) (Interfaces.jl:2084-2106): ghost values added to their
    owners (reverse exchanger, `+`), then ghost values set to zero.  For a
    PSparseMatrix: assemble!(A) (2383-2404), the ghost rows' nonzeros added
    to the owners' and then zeroed.  For a COO and its rows:
    assemble!(I, J, V, rows) (2406-2492) on the device."""
    if isinstance(v, COO):
        if rows is None:
            raise TypeError("assemble!(I, J, V, rows): the rows PRange is required")
        return _assemble_coo(v, rows)
    if isinstance(v, PSparseMatrix):
        return _mat_exchange(v, _lib.PA_ADD, 1, 1)
    ctxs = contexts(v.values)
    xg = [device_exchanger(c, v.rows.exchanger, p) for c, p in zip(ctxs, v.values.part_ids)]
    _lib.call("pa_exchange_all", len(ctxs), _hs(v.values.parts), _hs(xg), _lib.ptr_array(_idx(v)),
              _lib.PA_ADD, 1, 1)
    return v


def _scalar_out(dtype):
    return np.zeros(1, dtype=dtype)


def dot(a: PVector, b: PVector):
    """dot(a, b) (Interfaces.jl:1985-1992)"""
    out = _scalar_out(a.dtype)
    n = len(a.values.parts)
    _lib.call("pa_dot_all", n, _hs(a.values.parts), _lib.ptr_array(_idx(a)), _hs(b.values.parts),
              _lib.ptr_array(_idx(b)), out.ctypes.data_as(C.c_void_p))
    return out[0].item()


def norm(a: PVector, p=2):
    """norm(a, 2) (Interfaces.jl:1767-1772)"""
    if p != 2:
        raise NotImplementedError("norm(a, p) on HIP parts: p = 2 only")
    out = np.zeros(1, dtype=np.float64)
    _lib.call("pa_norm2_all", len(a.values.parts), _hs(a.values.parts), _lib.ptr_array(_idx(a)),
              out.ctypes.data_as(C.c_void_p))
    return float(out[0])


def psum(a: PVector):
    """sum(a) (Interfaces.jl:1981-1983)"""
    out = _scalar_out(a.dtype)
    _lib.call("pa_sum_all", len(a.values.parts), _hs(a.values.parts), _lib.ptr_array(_idx(a)),
              out.ctypes.data_as(C.c_void_p))
    return out[0].item()


# ---------------------------------------------------------------------------
# PSparseMatrix

class PSparseMatrix:
    """PSparseMatrix(values, rows, cols) (Interfaces.jl:2108-2125): values =
    PData of DeviceMatrix (owned rows in the SELL layout)."""

    def __init__(self, values: PData, rows: PRange, cols: PRange, exchanger=None):
        self.values = values
        self.rows = rows
        self.cols = cols
        # matrix_exchanger(values, rows, cols) (Interfaces.jl:2117): nz ids
        self.exchanger = exchanger if exchanger is not None else empty_exchanger(rows.partition)
        self._dev_xchg = None

    @property
    def dtype(self):
        return self.values.parts[0].dtype

    @property
    def shape(self):
        return (len(self.rows), len(self.cols))

    @staticmethod
    def from_csc(csc: PData, rows: PRange, cols: PRange) -> "PSparseMatrix":
        """From each part's local SparseMatrixCSC (num_lids(rows) × num_lids(cols))."""
        ctxs = contexts(rows.partition)
        mats = []
        for c, A, r, s in zip(ctxs, csc.parts, rows.partition.parts, cols.partition.parts):
            mats.append(DeviceMatrix.from_csc(c, A, device_index(c, r), device_index(c, s),
                                              r.num_lids, s.num_lids))
        ex = matrix_exchanger(csc, rows, cols)
        return PSparseMatrix(PData(rows.partition.backend, rows.partition.part_ids, mats,
                                   rows.partition.shape), rows, cols, ex)

    @staticmethod
    def from_csr(csr: PData, rows: PRange, cols: PRange) -> "PSparseMatrix":
        """From each part's local SparseMatrixCSR{Bi} (num_lids(rows) ×
        num_lids(cols)); mul! then follows SparseUtils.jl:222-252."""
        ctxs = contexts(rows.partition)
        mats = []
        for c, A, r, s in zip(ctxs, csr.parts, rows.partition.parts, cols.partition.parts):
            mats.append(DeviceMatrix.from_csr(c, A, device_index(c, r), device_index(c, s),
                                              r.num_lids, s.num_lids))
        ex = matrix_exchanger(csr, rows, cols)
        return PSparseMatrix(PData(rows.partition.backend, rows.partition.part_ids, mats,
                                   rows.partition.shape), rows, cols, ex)

    @staticmethod
    def from_coo(I, J, V, rows: PRange, cols: PRange, ids="local", init=None):
        """PSparseMatrix(init, I, J, V, rows, cols; ids) (Interfaces.jl:
        2194-2215).  init None = sparse (2237-2244), on the device; I, J, V:
        PData of host arrays, or I a device COO (then J and V are None).
        init = csr_init(Bi) (sparsecsr): the same compress on the device into
        SparseMatrixCSR{Bi} parents (pa_mat_from_coo_csr).  Another callable
        init compresses each part's host triplets and uploads the result
        (pa_mat_from_csc / pa_mat_from_csr)."""
        if isinstance(init, csr_init):  # sparsecsr on the device
            return PSparseMatrix._from_coo_device(I, J, V, rows, cols, ids, csr_bi=init.Bi)
        if init is not None:
            if isinstance(I, COO):
                raise NotImplementedError("from_coo: a custom init needs host triplets")
            if ids == "global":
                I = map_parts(lambda i, r: r.to_lids(np.asarray(i, dtype=np.int64)), I, rows.partition)
                J = map_parts(lambda j, c: c.to_lids(np.asarray(j, dtype=np.int64)), J, cols.partition)
            loc = map_parts(lambda i, j, v, r, c: init(i, j, v, r.num_lids, c.num_lids), I, J, V,
                            rows.partition, cols.partition)
            if all(isinstance(m, CSR) for m in loc.parts):
                return PSparseMatrix.from_csr(loc, rows, cols)
            if all(isinstance(m, CSC) for m in loc.parts):
                return PSparseMatrix.from_csc(loc, rows, cols)
            raise TypeError("from_coo: init must return CSC or CSR local matrices")
        return PSparseMatrix._from_coo_device(I, J, V, rows, cols, ids)

    @staticmethod
    def _from_coo_device(I, J, V, rows: PRange, cols: PRange, ids="local", csr_bi=None):
        # to_lids! (ids=:global) and sparse(I, J, V) (or sparsecsr) on the
        # device (pa_mat_from_coo[_csr]); the host keeps the pattern only, for
        # matrix_exchanger
        glob = ids == "global"
        idx = device_index_gids if glob else device_index
        ctxs = contexts(rows.partition)
        dev = isinstance(I, COO)  # device triplets: from_coo(coo, None, None, rows, cols; ids)
        if dev:
            I, J, V = I.values, I.values, I.values
        mats, pats = [], []
        # the host needs the CSC pattern only for matrix_exchanger, i.e. when
        # rows have ghosts (stored ghost rows of FE assembly)
        want_pattern = bool(rows.ghost)
        trace = trace_setup()
        t0 = trace()
        for c, i, j, v, r, s in zip(ctxs, I.parts, J.parts, V.parts, rows.partition.parts, cols.partition.parts):
            if dev:
                M, colptr, rowval = DeviceMatrix.from_dcoo(i, idx(c, r), idx(c, s), r.num_lids, s.num_lids,
                                                           ids_global=glob, pattern=want_pattern, csr_bi=csr_bi)
            else:
                M, colptr, rowval = DeviceMatrix.from_coo(c, i, j, v, idx(c, r), idx(c, s), r.num_lids,
                                                          s.num_lids, ids_global=glob, pattern=want_pattern,
                                                          csr_bi=csr_bi)
            mats.append(M)
            if not want_pattern:
                pats.append(None)
            elif csr_bi is None:
                pats.append(CSC(r.num_lids, s.num_lids, colptr, rowval, np.zeros(0)))
            else:
                pats.append(CSR(csr_bi, r.num_lids, s.num_lids, colptr, rowval, np.zeros(0)))
        t1 = trace("device sparse + SELL, all parts", t0)
        backend, pids, shape = rows.partition.backend, rows.partition.part_ids, rows.partition.shape
        ex = (matrix_exchanger(PData(backend, pids, pats, shape), rows, cols) if want_pattern
              else empty_exchanger(rows.partition))
        trace("matrix_exchanger", t1)
        return PSparseMatrix(PData(backend, pids, mats, shape), rows, cols, ex)

    def info(self):
        return map_parts(lambda m: m.info(), self.values)


def fillstored_(a: "PSparseMatrix", v) -> "PSparseMatrix":
    """LinearAlgebra.fillstored!(a, v) (Interfaces.jl:2127-2132): every
    stored value of every part becomes v (on the device)."""
    for M in a.values.parts:
        M.fillstored(v)
    return a


def matrix_exchanger(values: PData, rows: PRange, cols: PRange) -> Exchanger:
    """matrix_exchanger(values, rows, cols) (Interfaces.jl:2300-2372),
    vectorised: the nonzeros of ghost rows (CSC order k) grouped by the row
    owner in rows.exchanger.parts_rcv order; their (gi, gj) are sent to the
    owner, which answers with nzindex of (gi, gj) in its local matrix."""
    if not rows.ghost:
        return empty_exchanger(rows.partition)
    parts_rcv = rows.exchanger.parts_rcv
    parts_snd = rows.exchanger.parts_snd

    def nz_lids(A):
        """0-based (row, col) lids of the nonzeros in storage order
        (nziterator, SparseUtils.jl:106-150 for CSC, 254-300 for CSR)"""
        if isinstance(A, CSR):
            return np.repeat(np.arange(A.m), np.diff(A.rowptr)), A.colval - A.Bi
        return A.rowval - 1, np.repeat(np.arange(A.n), np.diff(A.colptr))

    def setup_rcv(prcv, r, c, A):
        prcv = np.asarray(prcv, dtype=np.int64)
        li, lj = nz_lids(A)
        owner = r.lid_to_part[li].astype(np.int64)
        k = np.flatnonzero(owner != r.part)
        seg = np.searchsorted(prcv, owner[k])
        if len(k) and (seg.max() >= len(prcv) or not np.array_equal(prcv[seg], owner[k])):
            raise KeyError("matrix_exchanger: a ghost row's owner is not in parts_rcv")
        o = np.argsort(seg, kind="stable")
        k = k[o]
        ptrs = counts_to_ptrs(np.bincount(seg, minlength=len(prcv)))
        gi = r.lid_to_gid[li[k]]
        gj = c.lid_to_gid[lj[k]]
        return (Table((k + 1).astype(np.int64), ptrs), Table(gi, ptrs.copy()), Table(gj, ptrs.copy()))
    k_rcv, gi_rcv, gj_rcv = unzip(map_parts(setup_rcv, parts_rcv, rows.partition, cols.partition, values), 3)
    segs = lambda t: [t[i] for i in range(1, len(t) + 1)]
    gi_snd = exchange(map_parts(segs, gi_rcv), parts_snd, parts_rcv)
    gj_snd = exchange(map_parts(segs, gj_rcv), parts_snd, parts_rcv)

    def setup_snd(r, c, gi, gj, A):
        ptrs = counts_to_ptrs([len(x) for x in gi])
        gi = np.concatenate(gi).astype(np.int64) if gi else np.zeros(0, np.int64)
        gj = np.concatenate(gj).astype(np.int64) if gj else np.zeros(0, np.int64)
        li = r.to_lids(gi) - 1
        lj = c.to_lids(gj) - 1
        # nzindex(A, li, lj): CSC order is sorted by (col, row) (SparseUtils.jl:
        # 96-104), CSR order by (row, col) (210-220)
        ri, rj = nz_lids(A)
        if isinstance(A, CSR):
            key, q = ri.astype(np.int64) * A.n + rj, li * A.n + lj
        else:
            key, q = rj.astype(np.int64) * A.m + ri, lj * A.m + li
        pos = np.searchsorted(key, q)
        ok = (pos < len(key)) & (key[np.minimum(pos, max(len(key) - 1, 0))] == q) if len(key) else pos < 0
        if not np.all(ok):
            raise AssertionError("The sparsity pattern of the ghost layer is inconsistent")
        return Table((pos + 1).astype(np.int64), ptrs)
    k_snd = map_parts(setup_snd, rows.partition, cols.partition, gi_snd, gj_snd, values)
    return Exchanger(parts_rcv, parts_snd, k_rcv, k_snd)


def _mat_exchange(A: "PSparseMatrix", op, reverse, zero_sent):
    if A._dev_xchg is None:
        ex = A.exchanger
        A._dev_xchg = [DeviceMatrixExchanger(M, ex.parts_rcv.local(p), ex.lids_rcv.local(p),
                                             ex.parts_snd.local(p), ex.lids_snd.local(p))
                       for M, p in zip(A.values.parts, A.values.part_ids)]
    _lib.call("pa_mat_exchange_all", len(A._dev_xchg), _hs(A.values.parts), _hs(A._dev_xchg), op, reverse,
              zero_sent)
    return A


def mul_(c: PVector, a: PSparseMatrix, b: PVector, alpha=1.0, beta=0.0) -> PVector:
    """mul!(c, a, b, α, β) (Interfaces.jl:2246-2275): halo exchange of b
    overlapped with the interior slices, then the slices reading ghosts."""
    _spmv(c, a, b, alpha, beta, None)
    return c


def mul_dot_(c: PVector, a: PSparseMatrix, b: PVector, alpha=1.0, beta=0.0):
    """mul!(c, a, b, α, β) then dot(b, c), the dot accumulated by the SpMV
    kernel (pa_spmv_dot_all).  Returns the dot."""
    out = _scalar_out(a.dtype)
    _spmv(c, a, b, alpha, beta, out)
    return out[0].item()


def _spmv(c, a, b, alpha, beta, dot_out):
    args = _spmv_args(c, a, b, alpha, beta)
    if dot_out is None:
        _lib.call("pa_spmv_all", *args)
    else:
        _lib.call("pa_spmv_dot_all", *args, dot_out.ctypes.data_as(C.c_void_p))


_ARGS_CACHE_MAX = 8


def _spmv_args(c, a, b, alpha, beta):
    """The C-ABI arguments of mul!(c, a, b, α, β), cached on `a` per (c, b,
    α, β): the layout checks and the handle arrays are built on the first
    call only (the Python side of a mul! costs about as much as a small
    SpMV's kernels otherwise).  An entry is reused only while c and b are the
    same live objects with the same values and ranges (the entry holds no
    strong reference to them: their device memory is freed as usual)."""
    cache = a.__dict__.get("_args_cache")
    if cache is None:
        cache = a.__dict__["_args_cache"] = OrderedDict()
    key = (id(c), id(b), type(alpha), alpha, type(beta), beta)
    try:
        e = cache.get(key)
    except TypeError:  # unhashable scalars (0-d arrays): no caching
        return _spmv_args_build(c, a, b, alpha, beta)
    now = (id(c.values), id(b.values), id(c.rows), id(b.rows))
    if e is not None and e[0]() is c and e[1]() is b and e[2] == now:
        cache.move_to_end(key)
        return e[3]
    args = _spmv_args_build(c, a, b, alpha, beta)
    cache[key] = (weakref.ref(c), weakref.ref(b), now, args)
    while len(cache) > _ARGS_CACHE_MAX:
        cache.popitem(last=False)
    return args


def _spmv_args_build(c, a, b, alpha, beta):
    if not (c.rows is a.rows or oids_are_equal(c.rows, a.rows)):
        raise AssertionError("mul!: c.rows and a.rows own different ids")
    if not (b.rows is a.cols or (oids_are_equal(a.cols, b.rows) and hids_are_equal(a.cols, b.rows))):
        raise AssertionError("mul!: b.rows differs from a.cols")
    if b.rows is not a.cols and not _cached_eq(
            "layout", a.cols, b.rows,
            lambda s, t: bool(np.array_equal(s.oid_to_lid, t.oid_to_lid) and np.array_equal(s.hid_to_lid, t.hid_to_lid))):
        raise NotImplementedError("mul!: b.rows must have a.cols' local layout")
    ctxs = contexts(a.values)
    n = len(ctxs)
    ex = b.rows.exchanger
    has_x = any(len(ex.parts_rcv.local(p)) or len(ex.parts_snd.local(p)) for p in b.values.part_ids)
    xg = [device_exchanger(cx, ex, p) for cx, p in zip(ctxs, b.values.part_ids)] if has_x else None
    al, alp = _lib.scalar_buf(alpha, a.dtype)
    be, bep = _lib.scalar_buf(beta, a.dtype)
    # the scalar buffers ride along (the C side reads them during the call)
    return (n, _hs(a.values.parts), _hs(c.values.parts), _lib.ptr_array(_idx(c)),
            _hs(b.values.parts), _lib.ptr_array(_idx(b)), _hs(xg) if xg else None, alp, bep)


def cg_update_(x: PVector, r: PVector, u: PVector, c: PVector, alpha) -> float:
    """x .+= α.*u; r .-= α.*c; norm(r) in one pass (pa_cg_update_all); α is
    a Float64 (ComplexF64 for complex vectors) as in IterativeSolvers."""
    if not (x.rows is r.rows is u.rows is c.rows):
        raise ValueError("cg_update_: the four vectors must share one PRange")
    al, alp = _lib.scalar_buf(alpha, np.complex128 if np.dtype(x.dtype).kind == "c" else np.float64)
    out = C.c_double(0.0)
    _lib.call("pa_cg_update_all", len(x.values.parts), _hs(x.values.parts), _hs(r.values.parts),
              _hs(u.values.parts), _hs(c.values.parts), _lib.ptr_array(_idx(x)), alp, C.byref(out))
    return out.value


def _julia_inv(w: complex) -> complex:
    """Julia's inv(::ComplexF64) (base/complex.jl, scaled Smith): Float64 /
    ComplexF64 is a * inv(z) componentwise (Julia Base arithmetic, restated;
    the device CG's julia_inv is the same)."""
    c, d = w.real, w.imag
    if math.isinf(c) or math.isinf(d):
        return complex(math.copysign(0.0, c), 0.0 if math.copysign(1.0, d) < 0 else -0.0)
    half, two = 0.5, 2.0
    cd = max(abs(c), abs(d))
    ov, un, eps = sys.float_info.max, sys.float_info.min, sys.float_info.epsilon
    bs = two / (eps * eps)
    s = 1.0
    if cd >= half * ov:
        c, d, s = half * c, half * d, s * half
    if cd <= un * two / eps:
        c, d, s = c * bs, d * bs, s * bs
    if abs(d) <= abs(c):
        r = d / c
        t = 1.0 / (c + d * r)
        p, q = t, -r * t
    else:
        c, d = d, c
        r = d / c
        t = 1.0 / (c + d * r)
        p, q = r * t, -t
    return complex(p * s, q * s)


def _rdiv(a: float, z):
    """a::Float64 / z::T (Julia: Float64 for real T, a*inv(ComplexF64(z)) for complex)"""
    if isinstance(z, complex):
        w = _julia_inv(z)
        return complex(a * w.real, a * w.imag)
    return a / float(z)


def matvec(a: PSparseMatrix, b: PVector) -> PVector:
    """Base.:*(a, b) (Interfaces.jl:2605-2610)"""
    c = PVector.undef(a.rows, a.dtype)
    return mul_(c, a, b)


def _own_contig(v: PVector) -> bool:
    return all(s.num_oids == 0 or (s.oid_to_lid[0] == 1 and s.oid_to_lid[-1] == s.num_oids)
               for s in v.rows.partition.parts)


def cg_(x: PVector, A: PSparseMatrix, b: PVector, reltol=None, abstol=0.0, maxiter=None,
        history=None, fused=True, device=False, batch=8):
    """IterativeSolvers.cg! (v0.9; caller of the hot path at test_fdm.jl:115,
    test_fem_sa.jl:135), restated over the device operations:
    u = zero(x); r, c = similar(x); copyto!(r, b); mul!(c, A, x); r .-= c;
    residual = norm(r); tol = max(reltol*norm(b), abstol); prev = 1; then per
    iteration β = res²/prev²; u .= r .+ β.*u; mul!(c, A, u);
    α = res²/dot(u, c); x .+= α.*u; r .-= α.*c; prev = res; res = norm(r).

    device=True runs the same recurrence with its scalars on the device
    (pa_cg_solve_all): the host enqueues `batch` iterations between reads of
    the done flag; results equal the host-driven fused loop bit for bit."""
    real = np.float32 if x.dtype in (np.float32, np.complex64) else np.float64
    if reltol is None:  # sqrt(eps(real(eltype(b)))), in that type
        reltol = float(np.sqrt(np.finfo(real).eps))
    if maxiter is None:
        maxiter = len(A.cols)
    if device:
        return _cg_device(x, A, b, reltol, abstol, maxiter, history, batch)
    u = x.similar().fill_(0)
    r = x.similar()
    c = x.similar()
    copyto_(r, b)
    mul_(c, A, x)
    sub_(r, c)
    residual = norm(r)
    tol = max(reltol * norm(b), abstol)
    prev = 1.0
    it = 0
    # fusions (same arithmetic per element; reduction orders are this
    # library's deterministic ones): dot(u,c) inside the SpMV, and
    # x/r updates + norm(r) in one pass
    fuse = fused and _own_contig(u) and (x.rows is r.rows is u.rows is c.rows)
    while not (it >= maxiter or residual <= tol):
        beta = (residual * residual) / (prev * prev)  # residual^2 (literal_pow: x*x)
        xpby_(u, r, beta)
        if fuse:
            alpha = _rdiv(residual * residual, mul_dot_(c, A, u))
            new = cg_update_(x, r, u, c, alpha)
        else:
            mul_(c, A, u)
            alpha = _rdiv(residual * residual, dot(u, c))
            axpy_(x, alpha, u)
            axmy_(r, alpha, c)
            new = norm(r)
        prev = residual
        residual = new
        it += 1
        if history is not None:
            history.append(residual)
    return x


def _cg_device(x: PVector, A: PSparseMatrix, b: PVector, reltol, abstol, maxiter, history, batch):
    if not _own_contig(x):
        raise ValueError("cg_(device=True): x needs contiguous owned lids")
    if b.rows is not x.rows:  # copyto!(r, b) across partitions copies the owned values
        bb = x.similar()
        copyto_(bb, b)
        b = bb
    u, r, c = x.similar(), x.similar(), x.similar()
    ctxs = contexts(A.values)
    n = len(ctxs)
    ex = x.rows.exchanger
    has_x = any(len(ex.parts_rcv.local(p)) or len(ex.parts_snd.local(p)) for p in x.values.part_ids)
    xg = [device_exchanger(cx, ex, p) for cx, p in zip(ctxs, x.values.part_ids)] if has_x else None
    its = C.c_int64(0)
    res = C.c_double(0.0)
    hist = np.zeros(max(1, int(maxiter)), dtype=np.float64) if history is not None else None
    _lib.call("pa_cg_solve_all", n, _hs(A.values.parts), _hs(x.values.parts), _hs(b.values.parts),
              _hs(u.values.parts), _hs(r.values.parts), _hs(c.values.parts), _lib.ptr_array(_idx(x)),
              _hs(xg) if xg else None, float(reltol), float(abstol), int(maxiter), int(batch),
              C.byref(its), C.byref(res),
              hist.ctypes.data_as(C.POINTER(C.c_double)) if hist is not None else None)
    if history is not None:
        history.extend(float(v) for v in hist[:its.value])
    return x
