import sys, time
sys.path.insert(0, "/root/repo")
import numpy as np, pamd
be = pamd.HIPBackend(devices=[0])
for shape in ((1,1,1), (2,2,2)):
    parts = be.get_part_ids(shape)
    N = tuple(32 * s for s in shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.ones(s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    for _ in range(10): pamd.mul_(y, A, x)
    for p in parts.part_ids: be.context(p).sync()
    t0 = time.perf_counter(); K = 200
    for _ in range(K): pamd.mul_(y, A, x)
    t1 = time.perf_counter()
    for p in parts.part_ids: be.context(p).sync()
    t2 = time.perf_counter()
    print(shape, "host us per mul!:", round(1e6*(t1-t0)/K, 1), "wall us per mul!:", round(1e6*(t2-t0)/K, 1))
    t0 = time.perf_counter()
    for _ in range(K): pamd.dot(x, x)
    print(shape, "dot us:", round(1e6*(time.perf_counter()-t0)/K, 1))
