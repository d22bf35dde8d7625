"""Multi-process (RCCL) check: every rank builds its part of a small FE27
problem, runs mul! with the halo over RCCL and compares its owned result with
the oracle (computed by each rank on the CPU).  Launch with torchrun."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch.distributed as dist  # noqa: E402

import pamd  # noqa: E402
import pa_oracle as O  # noqa: E402

dist.init_process_group("gloo")
world = dist.get_world_size()
shape = {2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}[world]
N = tuple(int(v) for v in os.environ.get("PA_CHECK_N", "12,10,9").split(","))
be = pamd.HIPDistributedBackend()
parts = be.get_part_ids(shape)
A = pamd.drivers.stencil_operator(parts, N, 27)
rng = np.random.default_rng(11)
OA = O.stencil_problem(O.get_part_ids(shape), N, 27)
xs = {q: rng.uniform(-1, 1, OA.cols.partition[q].num_lids) for q in range(1, world + 1)}
x = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
y = pamd.PVector.undef(A.rows)
for it in range(3):
    pamd.mul_(y, A, x)
ox = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
oy = O.pvector_undef(OA.rows)
O.mul_(oy, OA, ox)
p = parts.part_ids[0]
ok_y = np.array_equal(y.to_host().local(p), oy.values[p])
ok_x = np.array_equal(x.to_host().local(p), ox.values[p])
d = pamd.dot(x, x)
od = O.dot(ox, ox)
ok_d = abs(d - od) <= 1e-12 * abs(od)
v = pamd.PVector.from_host(pamd.map_parts(lambda s: xs[s.part], A.cols.partition), A.cols)
pamd.assemble_(v)
ov = O.PVector(O.map_parts(lambda s: xs[s.part].copy(), OA.cols.partition), OA.cols)
O.assemble_(ov)
ok_a = np.array_equal(v.to_host().local(p), ov.values[p])
print(f"rank {dist.get_rank()} part {p}: spmv {ok_y} halo {ok_x} dot {ok_d} assemble {ok_a}", flush=True)
t = __import__("torch").tensor([int(ok_y and ok_x and ok_d and ok_a)])
dist.all_reduce(t, op=dist.ReduceOp.MIN)
dist.destroy_process_group()
sys.exit(0 if int(t.item()) == 1 else 1)
