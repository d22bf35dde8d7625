"""partitionedarrays.jl_amd — MI355X-native backend for PartitionedArrays.jl's
SpMV + halo hot path.

Python host mirror of the reference's interface (names follow
src/PartitionedArrays.jl:10-99 exports; Julia's `f!` is `f_` here) over the
C-ABI library libpa_hip.so (include/pa_hip.h).  Import it as `pamd`
(repository root module pamd.py) — the directory name is not a Python
identifier.
"""
from ._lib import PAError, device_count, LIB_PATH  # noqa: F401
from .backends import (MAIN, AbstractBackend, DistributedBackend, PData, SequentialBackend,  # noqa: F401
                       alltoall, emit, exchange, gather, gather_all, get_part_ids, i_am_main, map_parts,
                       num_parts, preduce, prun, psum as psum_parts, reduce_all, reduce_main,
                       scatter, sequential, xscan_all)
from .helpers import Table, counts_to_ptrs, ptrs_to_counts  # noqa: F401
from .prange import (Exchanger, IndexSet, PRange, add_gids, add_gids_, discover_parts_snd,  # noqa: F401
                     empty_exchanger, exchanger_from_ids, hids_are_equal, index_range,
                     lids_are_equal, oids_are_equal, prange_cartesian, prange_from_partition,
                     prange_linear, prange_noids, to_lids_)
from .device import DeviceMatrix, HIPBackend, HIPDistributedBackend, device_index  # noqa: F401
from .pvector import (COO, CSC, CSR, PSparseMatrix, PVector, assemble_, axmy_, axpy_, cg_, cg_update_,  # noqa: F401
                      compresscoo, copyto_, csr_init, sparsecsr, fillstored_, dot, exchange_, matvec, mul_, mul_dot_, norm, psum, rmul_,
                      sub_, xpby_)
from .ptimers import PTimer  # noqa: F401
from . import drivers  # noqa: F401
