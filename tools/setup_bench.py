"""Setup time of BASELINE config 5 (FE27 on an irregular Voronoi partition):
add_gids!(rows, J) + Exchanger + PSparseMatrix(I, J, V; ids=:global), with
the heavy steps on the device (pa_add_gids, pa_mat_from_coo with to_lids!)
against the host restatement (numpy first-touch + to_lids + compresscoo,
then pa_mat_from_csc).  Prints one JSON line.

    python tools/setup_bench.py [--n 128] [--parts 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pamd  # noqa: E402
from pamd import drivers  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=128)
ap.add_argument("--parts", type=int, default=8)
args = ap.parse_args()
N = (args.n,) * 3
owners = drivers.voronoi_owners(N, args.parts)
be = pamd.HIPBackend(devices=[0])
out = {"workload": f"FE27 {args.n}^3 nodes, Voronoi partition into {args.parts} parts, F64, 1 GPU"}


def stencil_coo(parts):
    from pamd.prange import IndexSet, prange_from_partition
    ngids = int(np.prod(N))
    g2p = lambda g: owners[np.asarray(g, np.int64) - 1]

    def mk(part):
        gids = np.flatnonzero(owners == part).astype(np.int64) + 1
        return IndexSet(part, gids, np.full(len(gids), part, np.int32), np.arange(1, len(gids) + 1),
                        np.zeros(0, np.int32))
    rows = prange_from_partition(ngids, pamd.map_parts(mk, parts), pamd.map_parts(lambda _: g2p, parts), ghost=False)

    def coo(s):
        i, j, v = drivers.stencil_entries(27, N, s.lid_to_gid[s.oid_to_lid - 1])
        return s.lid_to_gid[s.oid_to_lid[i] - 1], j, v
    I, J, V = pamd.backends.unzip(pamd.map_parts(coo, rows.partition), 3)
    return rows, I, J, V


parts = be.get_part_ids(args.parts)
rows, I, J, V = stencil_coo(parts)
out["coo_entries"] = int(sum(len(j) for j in J.parts))

for _ in range(2):  # second round is the timed one (first pays lazy init)
    t0 = time.perf_counter()
    cols = pamd.add_gids(rows, J)            # device first-touch (HIP backend)
    t1 = time.perf_counter()
    A = pamd.PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global")
    for p in parts.part_ids:
        be.context(p).sync()
    t2 = time.perf_counter()
dev = {"add_gids_exchanger_s": round(t1 - t0, 3), "psparse_from_coo_s": round(t2 - t1, 3)}

# host restatement of the same steps (numpy), then the one-time CSC upload
hrows = pamd.PRange(rows.ngids, rows.partition, rows.exchanger, rows.gid_to_part, False)
hrows.partition = pamd.PData(pamd.sequential, parts.part_ids, rows.partition.parts, parts.shape)
hJ = pamd.PData(pamd.sequential, parts.part_ids, J.parts, parts.shape)
t0 = time.perf_counter()
hcols = pamd.add_gids(hrows, hJ)
t1 = time.perf_counter()
csc = []
for p in parts.part_ids:
    r, c = rows.partition.local(p), hcols.partition.local(p)
    csc.append(pamd.compresscoo(r.to_lids(I.local(p)), c.to_lids(J.local(p)), V.local(p), r.num_lids, c.num_lids))
t2 = time.perf_counter()
host = {"add_gids_exchanger_s": round(t1 - t0, 3), "to_lids_compresscoo_s": round(t2 - t1, 3)}
same = all(np.array_equal(cols.partition.local(p).lid_to_gid, hcols.partition.local(p).lid_to_gid)
           for p in parts.part_ids)
out.update({"device": dev, "host_numpy": host, "same_ghost_layer": same,
            "speedup_total": round((host["add_gids_exchanger_s"] + host["to_lids_compresscoo_s"]) /
                                   (dev["add_gids_exchanger_s"] + dev["psparse_from_coo_s"]), 2)})
print(json.dumps(out), flush=True)
