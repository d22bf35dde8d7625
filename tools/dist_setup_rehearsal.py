"""Rehearsal of bench.py's N>1 host setup at full size on the CPU: one
process per part (gloo), the Cartesian PRange of 256³ nodes per part and its
27-pt ghost layer + Exchanger (Interfaces.jl:1114-1137, 723-786), exactly as
bench.py builds them before the device operators.  Checks the halo plan's
segment lengths agree between every pair of neighbours (what RCCL's paired
send/recv needs) and reports the setup time per rank.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29555 tools/dist_setup_rehearsal.py [--n 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pamd  # noqa: E402

SHAPES = {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--kind", type=int, default=27)
a = ap.parse_args()
dist.init_process_group("gloo")
world, rank = dist.get_world_size(), dist.get_rank()
shape = SHAPES[world]
N = tuple(a.n * s for s in shape)
be = pamd.DistributedBackend()
t0 = time.perf_counter()
parts = be.get_part_ids(shape)
rows, cols = pamd.drivers.stencil_partition(parts, N, a.kind)
t = time.perf_counter() - t0
p = parts.part_ids[0]
ex = cols.exchanger
s = cols.partition.local(p)
seg_snd = {int(q): int(ex.lids_snd.local(p).ptrs[k + 1] - ex.lids_snd.local(p).ptrs[k])
           for k, q in enumerate(ex.parts_snd.local(p))}
seg_rcv = {int(q): int(ex.lids_rcv.local(p).ptrs[k + 1] - ex.lids_rcv.local(p).ptrs[k])
           for k, q in enumerate(ex.parts_rcv.local(p))}
allsnd = [None] * world
dist.all_gather_object(allsnd, seg_snd)
# what q sends to me must be what I receive from q
for q, n_r in seg_rcv.items():
    assert allsnd[q - 1].get(p) == n_r, f"part {p}: receives {n_r} from {q}, which sends {allsnd[q - 1].get(p)}"
tmax = [0.0] * world
dist.all_gather_object(tmax, t)
if rank == 0:
    print(json.dumps({"parts": shape, "global_nodes": N, "rows_per_part": s.num_oids, "ghosts_part1": s.num_hids,
                      "neighbours_part1": len(seg_rcv), "setup_s_max_over_ranks": round(max(tmax), 2),
                      "segments_paired": True}), flush=True)
dist.destroy_process_group()
