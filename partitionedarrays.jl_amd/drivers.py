"""Problem drivers: the reference's test problems and the benchmark operators.

* `fdm_problem`  — test_fdm.jl:8-110 (3D 7-point FD Poisson, COO assembly,
  add_gids, PSparseMatrix(I,J,V,rows,cols; ids=:local)), vectorised.
* `stencil_partition` / `stencil_operator` — Cartesian part boxes of the 7-pt
  FD operator and of the 27-pt Q1-hex FE operator (test_fem_sa.jl's pattern
  in 3D), assembled row-wise as test_fdm.jl does (each part
  pushes the COO entries of its owned rows, neighbours in lexicographic
  (z,y,x) order; cols = add_gids(rows, J)).  The partition is computed on the
  host from the part's face rows; the matrix is generated directly on the
  device (pa_mat_stencil) in the layout pa_mat_from_csc produces for the
  assembled CSC — tests/test_gpu_parity.py checks the two are identical.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .backends import PData, map_parts, unzip
from .device import DeviceMatrix, contexts
from .prange import (PRange, add_gids, box_of_part, cartesian_gid_to_part, exchanger_from_ids,
                     grid_neighbors_if_superset, linear_index, prange_cartesian, prange_linear, to_lids_)
from .pvector import PSparseMatrix, PVector


# ---------------------------------------------------------------------------
# test_fdm.jl

FDM_POINTS = [(0, 0, 0), (-1, 0, 0), (1, 0, 0), (0, -1, 0), (0, 1, 0), (0, 0, -1), (0, 0, 1)]


def fdm_problem(parts: PData, nx=10, dtype=np.float64):
    """test_fdm.jl:8-110 on HIP parts: returns (A, b, x0, x̂) as device objects."""
    rows, cols, I, J, V, bh, xh, x0h = fdm_host(parts, nx)
    V = map_parts(lambda v: v.astype(dtype), V)
    A = PSparseMatrix.from_coo(I, J, V, rows, cols, ids="local")
    b = PVector.from_host(map_parts(lambda v: v.astype(dtype), bh), rows)
    x_hat = PVector.from_host(map_parts(lambda v: v.astype(dtype), xh), rows)
    x0 = PVector.from_host(map_parts(lambda v: v.astype(dtype), x0h), cols)
    return A, b, x0, x_hat


def fdm_host(parts: PData, nx=10):
    """Host setup of test_fdm.jl:8-110: rows, cols (= add_gids(rows, J)), the
    COO vectors (I in local row ids, J converted to local col ids) and the
    host values of b, x̂ (on rows) and x0 (on cols).  u(x) = x₁+x₂, f = 0."""
    lx = 2.0
    ns = (nx, nx, nx)
    n = nx ** 3
    h = lx / (nx - 1)
    coeffs = [c / (h * h) for c in (-6, 1, 1, 1, 1, 1, 1)]  # test_fdm.jl:20 (h^2 = h*h)
    rows = prange_cartesian(parts, ns) if len(parts.shape) == 3 else prange_linear(parts, n)

    def coo(s):
        gids = s.lid_to_gid[s.oid_to_lid - 1]
        ci = np.stack([(gids - 1) % nx, ((gids - 1) // nx) % nx, (gids - 1) // (nx * nx)], 1)
        xi = ci * h
        uval = xi[:, 0] + xi[:, 1]
        bnd = np.any((ci == 0) | (ci == nx - 1), axis=1)
        k = len(gids)
        Im = np.repeat(s.oid_to_lid.astype(np.int64)[:, None], 7, 1)
        Jm = np.zeros((k, 7), np.int64)
        Vm = np.zeros((k, 7))
        mask = np.zeros((k, 7), bool)
        Jm[:, 0] = gids
        Vm[:, 0] = 1.0
        mask[bnd, 0] = True
        inner = ~bnd
        for t, (d, c) in enumerate(zip(FDM_POINTS, coeffs)):
            cj = ci + np.array(d)
            Jm[inner, t] = 1 + cj[inner, 0] + nx * cj[inner, 1] + nx * nx * cj[inner, 2]
            Vm[inner, t] = -c
            mask[inner, t] = True
        bv = np.zeros(s.num_lids)
        xv = np.zeros(s.num_lids)
        xv[s.oid_to_lid - 1] = uval
        bv[s.oid_to_lid - 1] = np.where(bnd, uval, 0.0)
        return Im[mask], Jm[mask], Vm[mask], bv, xv
    I, J, V, bh, xh = (PData(rows.partition.backend, rows.partition.part_ids, list(t), rows.partition.shape)
                       for t in zip(*map_parts(coo, rows.partition).parts))
    cols = add_gids(rows, J)
    J = to_lids_(J, cols)

    def x0v(s):
        g = s.lid_to_gid - 1
        ci = np.stack([g % nx, (g // nx) % nx, g // (nx * nx)], 1)
        bnd = np.any((ci == 0) | (ci == nx - 1), axis=1)
        own = s.lid_to_part == s.part
        xi = ci * h
        return np.where(bnd & own, xi[:, 0] + xi[:, 1], 0.0)
    x0h = map_parts(x0v, cols.partition)
    return rows, cols, I, J, V, bh, xh, x0h


# ---------------------------------------------------------------------------
# test_fem_sa.jl

def fem_sa_cells(parts: PData, nx=10):
    """test_fem_sa.jl:7-103 (2D Q1 FE, u = 1) up to the COO assembly: cells,
    COO of the owned cells (I, J global ids), add_gids!(rows, I), the rhs b
    filled through global ids (ghost rows included, before assemble!).
    Returns rows, cols (no ghosts yet), I, J, V, b (host, not yet assembled)
    and init(cols) → (x0, x̂) host values."""
    from .prange import add_gids_, prange_cartesian, prange_linear
    lx = 2.0
    ns = (nx, nx)
    h = lx / nx
    Ae = (h / 6) * np.array([[4.0, -1.0, -1.0, -2.0], [-1.0, 4.0, -2.0, -1.0],
                             [-1.0, -2.0, 4.0, -1.0], [-2.0, -1.0, -1.0, 4.0]])
    nsn = (nx + 1, nx + 1)
    cart = len(parts.shape) == 2
    cells = prange_cartesian(parts, ns) if cart else prange_linear(parts, nx * nx)
    enodes = [(0, 0), (1, 0), (0, 1), (1, 1)]  # CartesianIndices((2,2)), x fastest

    def node_gid(cx, cy):
        return 1 + cx + nsn[0] * cy

    def cell_nodes(gcell):
        cx, cy = (gcell - 1) % nx, (gcell - 1) // nx
        return [(cx + ex, cy + ey) for ex, ey in enodes]

    def on_boundary(c):
        return c[0] in (0, nx) or c[1] in (0, nx)

    def coo(s):
        I, J, V = [], [], []
        for ocell in s.oid_to_lid:
            nodes = cell_nodes(int(s.lid_to_gid[ocell - 1]))
            for erow, nr in enumerate(nodes):
                grow = node_gid(*nr)
                if on_boundary(nr):
                    I.append(grow); J.append(grow); V.append(1.0)
                else:
                    for ecol, nc in enumerate(nodes):
                        I.append(grow); J.append(node_gid(*nc)); V.append(Ae[erow, ecol])
        return np.array(I, np.int64), np.array(J, np.int64), np.array(V)
    I, J, V = unzip(map_parts(coo, cells.partition), 3)
    mk = (lambda: prange_cartesian(parts, nsn)) if cart else (lambda: prange_linear(parts, nsn[0] * nsn[1]))
    rows, cols = mk(), mk()
    add_gids_(rows, I)

    def fill_b(s, sc):
        bv = np.zeros(s.num_lids)
        for ocell in sc.oid_to_lid:
            for nr in cell_nodes(int(sc.lid_to_gid[ocell - 1])):
                if on_boundary(nr):
                    bv[s.to_lids([node_gid(*nr)])[0] - 1] += 1.0  # u(x) = 1
        return bv
    bh = map_parts(fill_b, rows.partition, cells.partition)

    def init(cols):
        def f(s):
            g = s.lid_to_gid - 1
            bnd = (g % nsn[0] == 0) | (g % nsn[0] == nx) | (g // nsn[0] == 0) | (g // nsn[0] == nx)
            own = s.lid_to_part == s.part
            return np.where(own & bnd, 1.0, 0.0), np.where(own, 1.0, 0.0)
        return unzip(map_parts(f, cols.partition), 2)
    return rows, cols, I, J, V, bh, init


def fem_sa_host(parts: PData, nx=10):
    """fem_sa_cells + async_assemble!(I, J, V, rows) restated on the host
    (prange.assemble_coo_; CPU setup tests only — the product path,
    fem_sa_problem, assembles on the device) + add_gids!(cols, J).  Returns
    rows, cols, I, J, V (global ids), b (host, not yet assembled), x0, x̂."""
    from .prange import add_gids_, assemble_coo_
    rows, cols, I, J, V, bh, init = fem_sa_cells(parts, nx)
    I, J, V = assemble_coo_(I, J, V, rows)
    add_gids_(cols, J)
    x0h, xh = init(cols)
    return rows, cols, I, J, V, bh, x0h, xh


def fem_sa_problem(parts: PData, nx=10, init=None):
    """test_fem_sa.jl on HIP parts: the COO triplets go to the device,
    assemble!(I, J, V, rows) moves the ghost rows' triplets to their owners
    there (pa_coo_assemble_all), add_gids!(cols, J), then the PSparseMatrix
    from the device COO (ids=:global; init = csr_init(Bi) for
    SparseMatrixCSR{Bi} parents) and b assembled on the device (assemble!,
    Interfaces.jl:2101)."""
    from .prange import add_gids_
    from .pvector import COO, assemble_
    mat_init = init  # the local matrix constructor (fem_sa_cells returns the x0/x̂ initializer as `init`)
    rows, cols, I, J, V, bh, init = fem_sa_cells(parts, nx)
    coo = COO.from_host(I, J, V, rows)
    assemble_(coo, rows)
    add_gids_(cols, coo.global_cols())
    x0h, xh = init(cols)
    A = PSparseMatrix.from_coo(coo, None, None, rows, cols, ids="global", init=mat_init)
    b = PVector.from_host(bh, rows)
    assemble_(b)
    return A, b, PVector.from_host(x0h, cols), PVector.from_host(xh, cols)


# ---------------------------------------------------------------------------
# Cartesian stencil operators (benchmark)

def fd7_coeffs(N, lx=2.0):
    """test_fdm.jl:18-20,75: stored values −(c/h²): {6/h², −1/h²}"""
    h = lx / (N - 1)
    return np.array([-((-6) / (h * h)), -(1 / (h * h))], dtype=np.float64)


def q1_hex_ke(h):
    """h·(K₁⊗M₁⊗M₁ + M₁⊗K₁⊗M₁ + M₁⊗M₁⊗K₁) with K₁=[1 -1;-1 1], M₁=[1/3 1/6;1/6 1/3]
    (3D analogue of test_fem_sa.jl:17-22), Julia kron order
    (first factor slowest), evaluated h*((T1+T2)+T3); node e = ex+2ey+4ez."""
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


def stencil_coeffs(kind, N):
    if kind == 7:
        return fd7_coeffs(N[0])
    return q1_hex_ke(2.0 / (N[0] - 1)).ravel()


def _offsets(kind):
    out = []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if kind == 7 and (dx != 0) + (dy != 0) + (dz != 0) > 1:
                    continue
                out.append((dx, dy, dz))
    return np.array(out, dtype=np.int64)


def _face_ghosts(N, lo, n, kind):
    """Ghost gids of one part box in first-touch order of the row-wise COO
    traversal (owned rows in oid order, neighbours lexicographic), i.e. what
    add_gids!(rows, J) (Interfaces.jl:1515-1533) gives.  Only rows on the box
    faces can touch ghosts, so only they are traversed."""
    lo0 = np.array(lo) - 1  # 0-based box origin
    nn = np.array(n)
    Nn = np.array(N)
    axes = [np.arange(k) for k in n]
    # face rows in ascending oid
    onface = []
    for d in range(3):
        for v in ({0, n[d] - 1}):
            sl = [slice(None)] * 3
            sl[2 - d] = v  # meshgrid axes are (z, y, x)
            onface.append(tuple(sl))
    mask = np.zeros((n[2], n[1], n[0]), dtype=bool)
    for sl in onface:
        mask[sl] = True
    oids = np.flatnonzero(mask.ravel())  # 0-based oid = x + nx*(y + ny*z)
    lx = oids % n[0]
    ly = (oids // n[0]) % n[1]
    lz = oids // (n[0] * n[1])
    g = np.stack([lx, ly, lz], 1) + lo0
    dirichlet = np.any((g == 0) | (g == Nn - 1), axis=1)
    g = g[~dirichlet]
    loc = np.stack([lx, ly, lz], 1)[~dirichlet]
    off = _offsets(kind)
    nb = g[:, None, :] + off[None, :, :]            # global coords
    nbl = loc[:, None, :] + off[None, :, :]          # box-local coords
    outside = np.any((nbl < 0) | (nbl >= nn), axis=2)
    nbg = nb[outside]                                # row-major = touch order
    gids = 1 + nbg[:, 0] + N[0] * (nbg[:, 1] + N[1] * nbg[:, 2])
    u, first = np.unique(gids, return_index=True)
    return u[np.argsort(first, kind="stable")]


def stencil_partition(parts: PData, N: tuple, kind: int):
    """rows = PRange(parts, N) (Cartesian, Interfaces.jl:1114-1137); cols =
    rows + ghost layer touched by the stencil rows (first-touch order), with
    its Exchanger (Interfaces.jl:723-786)."""
    rows = prange_cartesian(parts, N)
    cols = rows.copy()
    g2p = cartesian_gid_to_part(N, parts.shape)

    def add(s):
        lo, n = box_of_part(N, parts.shape, s.part)
        gh = _face_ghosts(N, lo, n, kind)
        s._append_ghosts(gh, g2p(gh))
        return s
    map_parts(add, cols.partition)
    cols.exchanger = exchanger_from_ids(cols.partition, grid_neighbors_if_superset(cols.partition, parts.shape))
    cols.ghost = True
    return rows, cols


def _shell_table(N, lo, n, s):
    """lid (0-based) of each node of the extended box (one-node shell) that is
    a ghost of index set s; -1 elsewhere."""
    if s.num_hids == 0:
        return None
    tab = np.full((n[2] + 2) * (n[1] + 2) * (n[0] + 2), -1, dtype=np.int32)
    gl = s.hid_to_lid.astype(np.int64)
    g = s.lid_to_gid[gl - 1] - 1
    gx, gy, gz = g % N[0], (g // N[0]) % N[1], g // (N[0] * N[1])
    ex = gx - (lo[0] - 1) + 1
    ey = gy - (lo[1] - 1) + 1
    ez = gz - (lo[2] - 1) + 1
    tab[ex + (n[0] + 2) * (ey + (n[1] + 2) * ez)] = (gl - 1).astype(np.int32)
    return tab


def stencil_operator(parts: PData, N: tuple, kind: int, dtype=np.float64, partition=None):
    """The part-local operators generated on the device (pa_mat_stencil)."""
    rows, cols = partition if partition is not None else stencil_partition(parts, N, kind)
    coef = np.ascontiguousarray(stencil_coeffs(kind, N), dtype=np.float64)
    ctxs = contexts(rows.partition)
    mats = []
    for c, s in zip(ctxs, cols.partition.parts):
        lo, n = box_of_part(N, parts.shape, s.part)
        tab = _shell_table(N, lo, n, s)
        gd = (C.c_int64 * 3)(*N)
        bl = (C.c_int64 * 3)(*[l - 1 for l in lo])
        bn = (C.c_int64 * 3)(*n)
        h = C.c_void_p()
        tp = tab.ctypes.data_as(C.POINTER(C.c_int32)) if tab is not None else None
        _lib.call("pa_mat_stencil", c.h, _lib.DTYPES[np.dtype(dtype)], kind, gd, bl, bn, s.num_lids, tp,
                  coef.ctypes.data_as(C.POINTER(C.c_double)), len(coef), C.byref(h))
        mats.append(DeviceMatrix(h, c, dtype))
    A = PSparseMatrix(PData(rows.partition.backend, rows.partition.part_ids, mats, rows.partition.shape),
                      rows, cols)
    return A


# ---------------------------------------------------------------------------
# BASELINE config 5: the stencil operators on an irregular ("METIS-like")
# partition — owners from the nearest of P seeded points,
# rows in gid order, ghosts in first-touch order (add_gids!), the Exchanger
# (Interfaces.jl:723-786) with parts_snd from a P-int all-to-all instead of
# the gather on MAIN (Interfaces.jl:515-552).

def _row_constants(kind, N):
    """Values of an interior row (all neighbours present), neighbour order
    (dz,dy,dx) lexicographic.  kind 27: for each neighbour the Ke entries of
    the cells holding both nodes, summed in ascending cell gid (the cell
    loop's COO order combined by sparse, test_fem_sa.jl:40-62)."""
    coef = stencil_coeffs(kind, N)
    off = _offsets(kind)
    if kind == 7:
        return off, np.array([coef[0] if not d.any() else coef[1] for d in off])
    vals = []
    for dx, dy, dz in off:
        acc = None
        for cz in (-1, 0):
            for cy in (-1, 0):
                for cx in (-1, 0):
                    bx, by, bz = dx - cx, dy - cy, dz - cz
                    if not (0 <= bx <= 1 and 0 <= by <= 1 and 0 <= bz <= 1):
                        continue
                    a = -cx + 2 * -cy + 4 * -cz
                    v = coef[a * 8 + bx + 2 * by + 4 * bz]
                    acc = v if acc is None else acc + v
        vals.append(acc)
    return off, np.array(vals, dtype=np.float64)


def stencil_entries(kind, N, gids):
    """COO entries of the rows `gids` (1-based) of the Cartesian stencil
    operator: (row position, column gid, value), rows in the given order,
    each row's neighbours in (dz,dy,dx) order.  Dirichlet rows (any
    coordinate on the boundary) keep the diagonal only: 1 for kind 7
    (test_fdm.jl:63-69), the number of touching cells for kind 27
    (test_fem_sa.jl:47-52, one 1.0 per cell)."""
    gids = np.asarray(gids, dtype=np.int64)
    g0 = gids - 1
    Nx, Ny, Nz = N
    gx, gy, gz = g0 % Nx, (g0 // Nx) % Ny, g0 // (Nx * Ny)
    dirichlet = ((gx == 0) | (gx == Nx - 1) | (gy == 0) | (gy == Ny - 1) | (gz == 0) | (gz == Nz - 1))
    off, vals = _row_constants(kind, N)
    K = len(off)
    cnt = np.where(dirichlet, 1, K)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
    nnz = int(cnt.sum())
    I = np.repeat(np.arange(len(gids), dtype=np.int64), cnt)
    J = np.empty(nnz, dtype=np.int64)
    V = np.empty(nnz, dtype=np.float64)
    di = np.flatnonzero(dirichlet)
    J[start[di]] = gids[di]
    if kind == 7:
        V[start[di]] = 1.0
    else:
        ncell = lambda c, n: np.where((c == 0) | (c == n - 1), 1, 2)
        V[start[di]] = (ncell(gx[di], Nx) * ncell(gy[di], Ny) * ncell(gz[di], Nz)).astype(np.float64)
    ii = np.flatnonzero(~dirichlet)
    lin = off[:, 0] + Nx * (off[:, 1] + Ny * off[:, 2])
    pos = start[ii][:, None] + np.arange(K)[None, :]
    J[pos] = gids[ii][:, None] + lin[None, :]
    V[pos] = vals[None, :]
    return I, J, V


def voronoi_owners(N, nparts, seed=20250114):
    """gid → part (1-based, int32 array over gids 1..prod(N)): the nearest of
    `nparts` points drawn uniformly in the node box (ties: lowest part)."""
    rng = np.random.default_rng(seed)
    pts = rng.uniform(0.0, 1.0, (nparts, 3)) * (np.array(N, dtype=np.float64) - 1.0)
    g0 = np.arange(int(np.prod(N)), dtype=np.int64)
    c = np.stack([g0 % N[0], (g0 // N[0]) % N[1], g0 // (N[0] * N[1])], 1).astype(np.float64)
    best = np.zeros(len(g0), dtype=np.int32)
    bd = np.full(len(g0), np.inf)
    for p in range(nparts):
        d = ((c[:, 0] - pts[p, 0]) ** 2 + (c[:, 1] - pts[p, 1]) ** 2) + (c[:, 2] - pts[p, 2]) ** 2
        closer = d < bd
        best[closer] = p
        bd[closer] = d[closer]
    return best + 1


def convert_values(v, dtype):
    """Float32.(A) / A .* (1+0.5im) of BASELINE config 5 (Complex(v*1, v*0.5))."""
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return v
    if dtype == np.float32:
        return v.astype(np.float32)
    if dtype == np.complex128:
        out = np.empty(len(v), np.complex128)
        out.real, out.imag = v * 1.0, v * 0.5
        return out
    if dtype == np.complex64:
        f = v.astype(np.float32)
        out = np.empty(len(v), np.complex64)
        out.real, out.imag = f * np.float32(1.0), f * np.float32(0.5)
        return out
    raise ValueError(dtype)


def irregular_partition(parts: PData, N: tuple, kind: int = 27, owners=None):
    """C5 setup on the host: rows = PRange(ngids, IndexSets of the owned gids
    in gid order, gid_to_part); each part's COO of its owned rows (global
    ids, Float64 values); cols = add_gids(rows, J) (first touch, Exchanger
    with parts_snd from the all-to-all discover, prange.discover_parts_snd).
    Returns rows, cols, I, J, V."""
    from .prange import IndexSet, prange_from_partition
    if owners is None:
        owners = voronoi_owners(N, parts.num_parts)
    ngids = int(np.prod(N))
    g2p = lambda g: owners[np.asarray(g, np.int64) - 1]

    def mk(part):
        gids = np.flatnonzero(owners == part).astype(np.int64) + 1
        return IndexSet(part, gids, np.full(len(gids), part, np.int32), np.arange(1, len(gids) + 1),
                        np.zeros(0, np.int32))
    rows = prange_from_partition(ngids, map_parts(mk, parts), map_parts(lambda _: g2p, parts), ghost=False)

    def coo(s):
        i, j, v = stencil_entries(kind, N, s.lid_to_gid[s.oid_to_lid - 1])
        return s.lid_to_gid[s.oid_to_lid[i] - 1], j, v
    I, J, V = unzip(map_parts(coo, rows.partition), 3)
    cols = add_gids(rows, J)
    return rows, cols, I, J, V


def irregular_problem(parts: PData, N: tuple, kind: int = 27, dtype=np.float64, owners=None):
    """C5: PSparseMatrix(I, J, V, rows, cols; ids=:global) on the irregular
    partition, values converted as BASELINE config 5 says."""
    rows, cols, I, J, V = irregular_partition(parts, N, kind, owners)
    V = map_parts(lambda v: convert_values(v, dtype), V)
    return PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global")
