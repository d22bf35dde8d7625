"""Device objects of the HIP backend: one `PartContext` per part, and cached
device copies of index sets / exchangers (created once, on first use).

This module is what a Julia `HIPBackend` keeps next to its `AbstractPData`:
`get_part_ids(HIPBackend(...), nparts)` creates the part contexts.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib
from .backends import DistributedBackend, PData, SequentialBackend


class PartContext:
    """pa_ctx: device, streams and scratch of one part."""

    def __init__(self, device: int, part: int, nparts: int, share_with=None):
        h = C.c_void_p()
        if share_with is not None:  # same device: one stream pair for both parts
            _lib.call("pa_ctx_create_shared", part, nparts, share_with.h, C.byref(h))
        else:
            _lib.call("pa_ctx_create", device, part, nparts, C.byref(h))
        self.h = h
        self.device = device
        self.part = part
        self.nparts = nparts

    def sync(self):
        _lib.call("pa_ctx_sync", self.h)

    def tune(self, key: str, value):
        """pa_ctx_tune: this part's value of a knob for the calls it leads
        (None drops it: the process default again); returns the former
        override (None: none)."""
        prev = C.c_int(0)
        v = _lib.TUNE_DROP if value is None else int(value)
        _lib.call("pa_ctx_tune", self.h, key.encode(), v, C.byref(prev))
        return None if prev.value == _lib.TUNE_DROP else prev.value

    def comm_stats(self):
        """(bytes sent, bytes received) this part has posted to RCCL so far"""
        a, b = C.c_int64(), C.c_int64()
        _lib.call("pa_comm_stats", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def comm_info(self):
        """pa_comm_info: the communicator's rank count and this rank (0 / -1
        without one), the device ordinal and PCI bus id, the RCCL version and
        the librccl path the process resolved"""
        ranks, rank, dev, ver = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        pci, lib = C.create_string_buffer(64), C.create_string_buffer(1024)
        _lib.call("pa_comm_info", self.h, C.byref(ranks), C.byref(rank), C.byref(dev), pci, 64, C.byref(ver),
                  lib, 1024)
        return {"ranks": ranks.value, "rank": rank.value, "device": dev.value, "pci": pci.value.decode(),
                "rccl_version": ver.value, "librccl": lib.value.decode()}

    def set_timing(self, on: bool):
        _lib.call("pa_ctx_set_timing", self.h, 1 if on else 0)

    def last_kernel_ms(self):
        """(interior, boundary) ms, means over the mul! calls since set_timing(True)"""
        a, b = C.c_float(), C.c_float()
        _lib.call("pa_ctx_last_kernel_ms", self.h, C.byref(a), C.byref(b))
        return a.value, b.value

    def span_start(self):
        """pa_ctx_span(0): mark the start of a region on the compute stream"""
        _lib.call("pa_ctx_span", self.h, 0)

    def span_stop(self):
        _lib.call("pa_ctx_span", self.h, 1)

    def span_ms(self):
        """device ms between span_start() and span_stop() (waits for the end)"""
        v = C.c_float()
        _lib.call("pa_ctx_span_ms", self.h, C.byref(v))
        return v.value

    def kernel_times(self):
        """dict of mean interior / halo (wait + unpack) / boundary ms and the
        number of mul! calls recorded since set_timing(True); clears the record"""
        a, h, b, n = C.c_float(), C.c_float(), C.c_float(), C.c_int()
        _lib.call("pa_ctx_kernel_times", self.h, C.byref(a), C.byref(h), C.byref(b), C.byref(n))
        return {"interior_ms": a.value, "halo_wait_ms": h.value, "boundary_ms": b.value, "calls": n.value}

    def close(self):
        """pa_ctx_destroy; every vector/matrix of the part must be gone."""
        if getattr(self, "h", None) and _lib._lib is not None:
            _lib._lib.pa_ctx_destroy(self.h)
            self.h = None


class HIPBackend(SequentialBackend):
    """All parts in this process, part p on device devices[(p-1) % len(devices)]
    (SequentialBackend semantics, HIP parts)."""

    def __init__(self, devices=None, share_streams=True, rccl=False):
        """share_streams (default): parts on the same device share one stream
        pair, and mul! runs them as one grouped launch per phase (pack,
        pull-unpack, interior and boundary slices of every part together;
        pa_tune("spmv_group")).  False: a stream pair per part and per-part
        launches.
        rccl: the halo moves by RCCL grouped ncclSend/ncclRecv between the
        parts of this process (pa_comm_init_all, which marks these contexts),
        the MPIBackend transport without processes: one RCCL rank per
        device, parts of one device send to self.  Default: the parts read
        each other's packed buffers."""
        ndev = _lib.device_count()
        if ndev == 0:
            raise _lib.PAError("HIPBackend: no HIP device visible")
        self.devices = list(devices) if devices is not None else list(range(ndev))
        self.share_streams = share_streams
        self.rccl = rccl
        self.ctx = {}
        self._sets = {}  # number of parts -> {part: PartContext}

    def get_part_ids(self, nparts):
        """With share_streams, parts on the same device share one stream pair
        (pa_ctx_create_shared): one in-order chain, and mul! launches each
        phase once for all of them (the grouped path of pa_spmv_all).
        The contexts of a number of parts are created once per backend and
        reused by later calls (streams and RCCL communicators are not
        re-created; objects built on an earlier call stay on their streams)."""
        ids = super().get_part_ids(nparts)
        n = ids.num_parts
        if n in self._sets:
            self.ctx = self._sets[n]
            return ids
        first = {}
        ctx = {}
        for p in ids.part_ids:
            d = self.devices[(p - 1) % len(self.devices)]
            share = first.get(d) if self.share_streams else None
            ctx[p] = PartContext(d, p, n, share_with=share)
            first.setdefault(d, ctx[p])
        if self.rccl and n > 1:
            if not self.share_streams and len({c.device for c in ctx.values()}) != n:
                raise _lib.PAError("HIPBackend(rccl=True): parts of one device share one RCCL rank and "
                                   "must share their stream pair (share_streams=True)")
            # the contexts of this call exchange over RCCL (a per-context flag
            # set by pa_comm_init_all; other backends of the process are unaffected)
            _lib.call("pa_comm_init_all", n, _lib.ptr_array([ctx[p].h for p in ids.part_ids]))
        self._sets[n] = self.ctx = ctx
        return ids

    def context(self, part, nparts=None) -> PartContext:
        """the context of `part` in the partition into `nparts` parts (default:
        the latest get_part_ids)"""
        return (self._sets[nparts] if nparts in self._sets else self.ctx)[part]


class HIPDistributedBackend(DistributedBackend):
    """One part per process (MPIBackend's role); device = local rank; halo over
    RCCL.  torch.distributed must be initialised (gloo is enough: it carries
    the host setup objects and the RCCL unique id)."""

    def __init__(self, device=None, group=None):
        super().__init__(group)
        import os
        if device is None:  # local rank, wrapped onto the visible devices
            device = int(os.environ.get("LOCAL_RANK", self.rank)) % max(1, _lib.device_count())
        self.device = device
        self.ctx = {}

    def get_part_ids(self, nparts):
        ids = super().get_part_ids(nparts)
        n = ids.num_parts
        part = ids.part_ids[0]
        if part in self.ctx:  # created by an earlier call (RCCL communicator included)
            return ids
        c = PartContext(self.device, part, n)
        # RCCL for every world size (with one process, its reductions take the
        # same one-rank all-gather path as with eight)
        buf = C.create_string_buffer(128)
        if part == 1:
            _lib.call("pa_comm_unique_id", buf)
        obj = [bytes(buf.raw) if part == 1 else None]
        self.dist.broadcast_object_list(obj, src=0, group=self.group)
        _lib.call("pa_comm_init_rank", c.h, C.c_char_p(obj[0]))
        self.ctx = {part: c}
        # one GPU per rank, or fail here (not a silently folded timing)
        self.device_keys = self.assert_distinct_devices(c.comm_info()["pci"])
        return ids

    def context(self, part, nparts=None) -> PartContext:
        return self.ctx[part]


def contexts(a: PData):
    return [a.backend.context(p, a.num_parts) for p in a.part_ids]


class DeviceIndex:
    def __init__(self, ctx: PartContext, s):
        o, op = _lib.i32(s.oid_to_lid)
        hh, hp = _lib.i32(s.hid_to_lid)
        h = C.c_void_p()
        _lib.call("pa_index_create", ctx.h, s.num_lids, s.num_oids, op, s.num_hids, hp, C.byref(h))
        self.h = h

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None and not sys.is_finalizing():
                _lib._lib.pa_index_destroy(self.h)
        except Exception:
            pass


def device_index(ctx: PartContext, s):
    """cached device copy of IndexSet s on ctx"""
    key = id(ctx)
    d = s._device.get(key)
    if d is None:
        d = DeviceIndex(ctx, s)
        s._device[key] = d
    return d


def device_index_gids(ctx: PartContext, s):
    """device_index with its gid → lid table attached (pa_index_set_gids)."""
    d = device_index(ctx, s)
    if not getattr(d, "has_gids", False):
        g = np.ascontiguousarray(s.lid_to_gid, dtype=np.int64)
        _lib.call("pa_index_set_gids", d.h, g.ctypes.data_as(C.POINTER(C.c_int64)))
        d.has_gids = True
    return d


def device_first_touch(ctx: PartContext, s, gids):
    """add_gids! discovery on the device (pa_add_gids): the gids that are not
    local ids of s, each once, in first-touch order."""
    d = device_index_gids(ctx, s)
    gids = np.ascontiguousarray(gids, dtype=np.int64).ravel()
    L = _lib.lib()
    cap = min(len(gids), max(4096, len(gids) // 16))
    while True:
        out = np.empty(max(1, cap), dtype=np.int64)
        n_new = C.c_int64(0)
        rc = L.pa_add_gids(d.h, len(gids), gids.ctypes.data_as(C.POINTER(C.c_int64)), cap,
                           out.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(n_new))
        if rc == 0:
            return out[:n_new.value].copy()
        if n_new.value > cap:
            cap = n_new.value
            continue
        raise _lib.PAError(f"pa_add_gids: {L.pa_last_error().decode(errors='replace')}")


def device_to_lids(ctx: PartContext, s, gids):
    """to_lids!(gids, s) through the device gid table (pa_index_to_lids)."""
    d = device_index_gids(ctx, s)
    ids = np.array(gids, dtype=np.int64).ravel()
    _lib.call("pa_index_to_lids", d.h, len(ids), ids.ctypes.data_as(C.POINTER(C.c_int64)))
    return ids


class DeviceExchanger:
    def __init__(self, ctx: PartContext, parts_rcv, lids_rcv, parts_snd, lids_snd):
        pr, prp = _lib.i32(parts_rcv)
        rp, rpp = _lib.i32(lids_rcv.ptrs)
        rl, rlp = _lib.i32(lids_rcv.data)
        ps, psp = _lib.i32(parts_snd)
        sp, spp = _lib.i32(lids_snd.ptrs)
        sl, slp = _lib.i32(lids_snd.data)
        h = C.c_void_p()
        _lib.call("pa_xchg_create", ctx.h, len(pr), prp, rpp, rlp, len(ps), psp, spp, slp, C.byref(h))
        self.h = h

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None and not sys.is_finalizing():
                _lib._lib.pa_xchg_destroy(self.h)
        except Exception:
            pass


def device_exchanger(ctx: PartContext, ex, part):
    key = (id(ctx), part)
    d = ex._device.get(key)
    if d is None:
        d = DeviceExchanger(ctx, ex.parts_rcv.local(part), ex.lids_rcv.local(part),
                            ex.parts_snd.local(part), ex.lids_snd.local(part))
        ex._device[key] = d
    return d


class DeviceMatrixExchanger(DeviceExchanger):
    """pa_mat_xchg_create: an Exchanger over nonzeros(A) (lids = CSC nz k)."""

    def __init__(self, mat, parts_rcv, k_rcv, parts_snd, k_snd):
        pr, prp = _lib.i32(parts_rcv)
        rp, rpp = _lib.i32(k_rcv.ptrs)
        rk = np.ascontiguousarray(k_rcv.data, dtype=np.int64)
        ps, psp = _lib.i32(parts_snd)
        sp, spp = _lib.i32(k_snd.ptrs)
        sk = np.ascontiguousarray(k_snd.data, dtype=np.int64)
        h = C.c_void_p()
        _lib.call("pa_mat_xchg_create", mat.h, len(pr), prp, rpp, rk.ctypes.data_as(C.POINTER(C.c_int64)),
                  len(ps), psp, spp, sk.ctypes.data_as(C.POINTER(C.c_int64)), C.byref(h))
        self.h = h
        self.mat = mat  # the exchanger addresses this matrix's value store


class DeviceVector:
    """pa_vec: the values of one part of a PVector, in HBM."""

    def __init__(self, ctx: PartContext, dtype, n: int):
        self.ctx = ctx
        self.dtype = np.dtype(dtype)
        self.n = int(n)
        h = C.c_void_p()
        _lib.call("pa_vec_create", ctx.h, _lib.DTYPES[self.dtype], self.n, C.byref(h))
        self.h = h

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.shape != (self.n,):
            raise ValueError(f"upload: expected {self.n} values, got {a.shape}")
        _lib.call("pa_vec_upload", self.h, a.ctypes.data_as(C.c_void_p), self.n)

    def download(self):
        a = np.empty(self.n, dtype=self.dtype)
        _lib.call("pa_vec_download", self.h, a.ctypes.data_as(C.c_void_p), self.n)
        return a

    def device_ptr(self) -> int:
        """device address of the values (pa_vec_device_ptr)"""
        p = C.c_void_p()
        _lib.call("pa_vec_device_ptr", self.h, C.byref(p))
        return p.value or 0

    def fill(self, v):
        b, bp = _lib.scalar_buf(v, self.dtype)
        _lib.call("pa_vec_fill", self.h, bp)

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None and not sys.is_finalizing():
                _lib._lib.pa_vec_destroy(self.h)
        except Exception:
            pass


class DeviceCOO:
    """pa_coo: the COO triplets (I, J global ids, V) of one part in HBM."""

    def __init__(self, ctx: PartContext, I, J, V):
        V = np.ascontiguousarray(V).ravel()
        I = np.ascontiguousarray(I, dtype=np.int64).ravel()
        J = np.ascontiguousarray(J, dtype=np.int64).ravel()
        if not (len(I) == len(J) == len(V)):
            raise ValueError("COO: I, J and V must have the same length")
        self.ctx = ctx
        self.dtype = V.dtype
        h = C.c_void_p()
        _lib.call("pa_coo_create", ctx.h, _lib.DTYPES[V.dtype], len(I), I.ctypes.data_as(C.POINTER(C.c_int64)),
                  J.ctypes.data_as(C.POINTER(C.c_int64)), V.ctypes.data_as(C.c_void_p), C.byref(h))
        self.h = h

    def __len__(self):
        n = C.c_int64()
        _lib.call("pa_coo_size", self.h, C.byref(n))
        return n.value

    def download(self):
        n = len(self)
        I, J = np.empty(n, np.int64), np.empty(n, np.int64)
        V = np.empty(n, self.dtype)
        _lib.call("pa_coo_download", self.h, I.ctypes.data_as(C.POINTER(C.c_int64)),
                  J.ctypes.data_as(C.POINTER(C.c_int64)), V.ctypes.data_as(C.c_void_p))
        return I, J, V

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None and not sys.is_finalizing():
                _lib._lib.pa_coo_destroy(self.h)
        except Exception:
            pass


class DeviceMatrix:
    """pa_mat: one part of a PSparseMatrix in the owned-row SELL layout."""

    def __init__(self, h, ctx: PartContext, dtype):
        self.h = h
        self.ctx = ctx
        self.dtype = np.dtype(dtype)

    @staticmethod
    def from_csc(ctx: PartContext, csc, rows_idx: DeviceIndex, cols_idx: DeviceIndex, nrows_lids, ncols_lids):
        colptr = np.ascontiguousarray(csc.colptr, dtype=np.int64)
        rowval = np.ascontiguousarray(csc.rowval, dtype=np.int64)
        nzval = np.ascontiguousarray(csc.nzval)
        h = C.c_void_p()
        _lib.call("pa_mat_from_csc", ctx.h, _lib.DTYPES[nzval.dtype], 8, nrows_lids, ncols_lids,
                  colptr.ctypes.data_as(C.c_void_p), rowval.ctypes.data_as(C.c_void_p),
                  nzval.ctypes.data_as(C.c_void_p), rows_idx.h, cols_idx.h, C.byref(h))
        M = DeviceMatrix(h, ctx, nzval.dtype)
        M.csc_nnz = len(nzval)
        return M

    @staticmethod
    def from_csr(ctx: PartContext, csr, rows_idx: DeviceIndex, cols_idx: DeviceIndex, nrows_lids, ncols_lids):
        """From a local SparseMatrixCSR{Bi} (pa_mat_from_csr): its nonzero
        order (set/get values, nz exchange) is the CSR storage order."""
        rowptr = np.ascontiguousarray(csr.rowptr, dtype=np.int64)
        colval = np.ascontiguousarray(csr.colval, dtype=np.int64)
        nzval = np.ascontiguousarray(csr.nzval)
        h = C.c_void_p()
        _lib.call("pa_mat_from_csr", ctx.h, _lib.DTYPES[nzval.dtype], 8, int(csr.Bi), nrows_lids, ncols_lids,
                  rowptr.ctypes.data_as(C.c_void_p), colval.ctypes.data_as(C.c_void_p),
                  nzval.ctypes.data_as(C.c_void_p), rows_idx.h, cols_idx.h, C.byref(h))
        M = DeviceMatrix(h, ctx, nzval.dtype)
        M.csc_nnz = len(nzval)
        return M

    @staticmethod
    def from_coo(ctx: PartContext, I, J, V, rows_idx: DeviceIndex, cols_idx: DeviceIndex, nrows_lids, ncols_lids,
                 ids_global=False, pattern=True, csr_bi=None):
        """sparse(I, J, V, m, n, +) and the SELL build on the device
        (pa_mat_from_coo; ids_global: I, J are gids mapped by to_lids! on the
        device, the indices need their gid tables).  Returns (matrix, colptr,
        rowval): the CSC pattern (1-based lids) for the host setup that needs
        it (matrix_exchanger); pattern=False returns (matrix, None, None) and
        downloads nothing.  Local ids cross PCIe as Int32 when they fit.
        csr_bi = 0 / 1: sparsecsr instead (pa_mat_from_coo_csr); the pattern
        returned is then (rowptr, colval) in base Bi."""
        V = np.ascontiguousarray(V).ravel()
        ib = 4 if not ids_global and max(nrows_lids, ncols_lids) < 2 ** 31 - 1 else 8
        idt = np.int32 if ib == 4 else np.int64
        I = np.asarray(I).ravel()
        J = np.asarray(J).ravel()
        if ib == 4 and len(I) and I.dtype != np.int32:
            # out-of-range lids must still raise BoundsError, not wrap around
            if min(I.min(), J.min()) < 1 or max(I.max(), J.max()) > 2 ** 31 - 1:
                ib, idt = 8, np.int64
        I = np.ascontiguousarray(I, dtype=idt)
        J = np.ascontiguousarray(J, dtype=idt)
        if not (len(I) == len(J) == len(V)):
            raise ValueError("sparse: I, J and V must have the same length")
        colptr = np.empty((nrows_lids if csr_bi is not None else ncols_lids) + 1, dtype=np.int64) if pattern else None
        rowval = np.empty(max(1, len(I)), dtype=np.int64) if pattern else None
        nnz = C.c_int64(0)
        h = C.c_void_p()
        ptrs = (colptr.ctypes.data_as(C.POINTER(C.c_int64)) if pattern else None,
                rowval.ctypes.data_as(C.POINTER(C.c_int64)) if pattern else None)
        if csr_bi is None:
            _lib.call("pa_mat_from_coo", ctx.h, _lib.DTYPES[V.dtype], ib, 1 if ids_global else 0, nrows_lids,
                      ncols_lids, len(I), I.ctypes.data_as(C.c_void_p), J.ctypes.data_as(C.c_void_p),
                      V.ctypes.data_as(C.c_void_p), rows_idx.h, cols_idx.h, C.byref(nnz), *ptrs, C.byref(h))
        else:
            _lib.call("pa_mat_from_coo_csr", ctx.h, _lib.DTYPES[V.dtype], ib, 1 if ids_global else 0, int(csr_bi),
                      nrows_lids, ncols_lids, len(I), I.ctypes.data_as(C.c_void_p), J.ctypes.data_as(C.c_void_p),
                      V.ctypes.data_as(C.c_void_p), rows_idx.h, cols_idx.h, C.byref(nnz), *ptrs, C.byref(h))
        M = DeviceMatrix(h, ctx, V.dtype)
        M.csc_nnz = nnz.value
        if not pattern:
            return M, None, None
        return M, colptr, rowval[:nnz.value].copy()

    @staticmethod
    def from_dcoo(coo: DeviceCOO, rows_idx: DeviceIndex, cols_idx: DeviceIndex, nrows_lids, ncols_lids,
                  ids_global=True, pattern=True, csr_bi=None):
        """DeviceMatrix.from_coo over device triplets (pa_mat_from_dcoo, or
        pa_mat_from_dcoo_csr with csr_bi = 0 / 1)."""
        n = len(coo)
        colptr = np.empty((nrows_lids if csr_bi is not None else ncols_lids) + 1, dtype=np.int64) if pattern else None
        rowval = np.empty(max(1, n), dtype=np.int64) if pattern else None
        nnz = C.c_int64(0)
        h = C.c_void_p()
        ptrs = (colptr.ctypes.data_as(C.POINTER(C.c_int64)) if pattern else None,
                rowval.ctypes.data_as(C.POINTER(C.c_int64)) if pattern else None)
        if csr_bi is None:
            _lib.call("pa_mat_from_dcoo", coo.h, 1 if ids_global else 0, nrows_lids, ncols_lids, rows_idx.h,
                      cols_idx.h, C.byref(nnz), *ptrs, C.byref(h))
        else:
            _lib.call("pa_mat_from_dcoo_csr", coo.h, 1 if ids_global else 0, int(csr_bi), nrows_lids, ncols_lids,
                      rows_idx.h, cols_idx.h, C.byref(nnz), *ptrs, C.byref(h))
        M = DeviceMatrix(h, coo.ctx, coo.dtype)
        M.csc_nnz = nnz.value
        if not pattern:
            return M, None, None
        return M, colptr, rowval[:nnz.value].copy()

    def set_values(self, nzval):
        nzval = np.ascontiguousarray(nzval, dtype=self.dtype)
        _lib.call("pa_mat_set_values", self.h, nzval.ctypes.data_as(C.c_void_p))

    def fillstored(self, v):
        """fillstored!(A, v) on the device (pa_mat_fillstored)."""
        buf, ptr = _lib.scalar_buf(v, self.dtype)
        _lib.call("pa_mat_fillstored", self.h, ptr)
        del buf

    def get_values(self):
        """nonzeros(A) in the parent's order (CSC, or CSR for a SparseMatrixCSR
        parent), ghost rows included."""
        n = getattr(self, "csc_nnz", None)
        if n is None:
            raise _lib.PAError("matrix was not built from a CSC pattern")
        a = np.empty(n, dtype=self.dtype)
        _lib.call("pa_mat_get_values", self.h, a.ctypes.data_as(C.c_void_p))
        return a

    def cg_choice(self) -> int:
        """the device CG's remembered u-update variant (pa_mat_cg_choice:
        1 fused, 0 sweep, -1 none yet)"""
        v = C.c_int(-1)
        _lib.call("pa_mat_cg_choice", self.h, C.byref(v))
        return v.value

    def info(self):
        v = [C.c_int64() for _ in range(5)]
        _lib.call("pa_mat_info", self.h, *[C.byref(x) for x in v])
        d = dict(zip(["nrows", "nnz", "slots", "nslices", "nslices_interior"], [x.value for x in v]))
        f = [C.c_int64() for _ in range(4)]
        _lib.call("pa_mat_format_info", self.h, *[C.byref(x) for x in f])
        d.update(zip(["pattern_slices", "regular_rows", "side_rows", "side_slots"], [x.value for x in f]))
        dd = C.c_int64()
        _lib.call("pa_mat_delta16_info", self.h, C.byref(dd))
        d["delta16_slices"] = dd.value
        t = [C.c_int64() for _ in range(4)]
        _lib.call("pa_mat_triple_info", self.h, *[C.byref(x) for x in t])
        d.update(zip(["triple_sell_slices", "triple_sell_rows", "tri_slices", "tri_rows"], [x.value for x in t]))
        pr = [C.c_int64() for _ in range(2)]
        if hasattr(_lib.lib(), "pa_mat_pair_info"):  # (an older build under PA_HIP_LIB lacks it: A/B tooling)
            _lib.call("pa_mat_pair_info", self.h, *[C.byref(x) for x in pr])
        d.update(zip(["pair_slices", "pair_rows"], [x.value for x in pr]))
        lr = [C.c_int64() for _ in range(2)]
        _lib.call("pa_mat_long_rows", self.h, *[C.byref(x) for x in lr])
        d.update(zip(["long_rows", "long_nnz"], [x.value for x in lr]))
        d.update(self.traffic())
        return d

    def device_ptrs(self):
        """pa_mat_device_ptrs: addresses of the main arrays (diagnostics)"""
        out = (C.c_uint64 * 8)()
        _lib.call("pa_mat_device_ptrs", self.h, out)
        return dict(zip(["val", "col", "slice_off", "plen", "pat", "mask", "s_val", "s_col"], list(out)))

    def traffic(self):
        """bytes one mul! streams from the matrix (current encoding)"""
        t = [C.c_int64() for _ in range(3)]
        _lib.call("pa_mat_traffic", self.h, *[C.byref(x) for x in t])
        return dict(zip(["value_bytes", "index_bytes", "meta_bytes"], [x.value for x in t]))

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None and not sys.is_finalizing():
                _lib._lib.pa_mat_destroy(self.h)
        except Exception:
            pass
