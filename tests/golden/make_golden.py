"""Writes tests/golden/interfaces_kats.json: the known-answer data of the
reference's own tests, transcribed (inputs and expected outputs only) from
/root/reference/test/test_interfaces.jl and test/SparseUtilsTests.jl.

The reference is Julia and cannot run on this image, so these
inline KATs are the fixtures that pin the oracle.  Each entry cites the lines
it comes from.  Run: python tests/golden/make_golden.py
"""
import json
import os

K = {}

# test_interfaces.jl:19-63 (and 126-163): scalar exchange on a fixed graph
K["exchange_scalar"] = {
    "src": "test/test_interfaces.jl:19-63",
    "parts_rcv": [[2, 3], [4], [1, 2], [1, 3]],
    "parts_snd": [[3, 4], [1, 3], [1, 4], [2]],
    "data_snd": "10 .* parts_snd",
    "expected_rcv": [[10, 10], [20], [30, 30], [40, 40]],
}
# :65-72 reduce_main / reduce_all / reduce / sum of part ids
K["reduce"] = {"src": "test/test_interfaces.jl:65-72", "expected": 10}
# :74-123 scans of a = [4,2,6,3]
K["scan"] = {
    "src": "test/test_interfaces.jl:74-123",
    "a": [4, 2, 6, 3],
    "iscan_init0": [4, 6, 12, 15], "iscan_total": 15,
    "xscan_init1": [1, 5, 7, 13], "xscan_total": 16,
}
# :166-173 discover_parts_snd recovers parts_snd; the error flag throws
K["discover"] = {"src": "test/test_interfaces.jl:166-173",
                 "parts_rcv": [[2, 3], [4], [1, 2], [1, 3]],
                 "expected_parts_snd": [[3, 4], [1, 3], [1, 4], [2]]}
# :175-207 Exchanger of an irregular 4-part IndexSet partition, n = 10
K["exchanger"] = {
    "src": "test/test_interfaces.jl:175-207",
    "n": 10,
    "lid_to_gid": [[1, 2, 3, 5, 7, 8], [2, 4, 5, 10], [6, 7, 8, 5, 4, 10], [1, 3, 7, 9, 10]],
    "lid_to_part": [[1, 1, 1, 2, 3, 3], [1, 2, 2, 4], [3, 3, 3, 2, 2, 4], [1, 1, 3, 4, 4]],
    "expected_parts_snd": [[2, 4], [1, 3], [1, 4], [2, 3]],
    "expected_lids_snd": [[[2], [1, 3]], [[3], [3, 2]], [[2, 3], [2]], [[5], [5]]],
}
# :209-227 exchange! of values 10*part at owned lids → every lid holds 10*owner
K["exchange_values"] = {"src": "test/test_interfaces.jl:209-227", "rule": "values[lid] == 10*owner"}
# :229-251 two-buffer exchange: owned keep 10.0, ghosts get 20.0
K["exchange_two_buffers"] = {"src": "test/test_interfaces.jl:229-251", "owned": 10.0, "ghost": 20.0}
# :253-274 Table exchange: values[lid][i] == 100*owner + 10*gid + i
K["exchange_table"] = {"src": "test/test_interfaces.jl:253-274", "rule": "100*owner + 10*gid + i", "width": 3}
# :360-372 PRange(parts, noids = [4,2,6,3])
K["prange_noids"] = {
    "src": "test/test_interfaces.jl:349-372",
    "noids": [4, 2, 6, 3],
    "lid_to_gid": [[1, 2, 3, 4], [5, 6], [7, 8, 9, 10, 11, 12], [13, 14, 15]],
    "gid_to_part": [1, 1, 1, 1, 2, 2, 3, 3, 3, 3, 3, 3, 4, 4, 4],
}
# :383-397 Cartesian PRange(parts (2,2), (5,4))
K["prange_cartesian"] = {
    "src": "test/test_interfaces.jl:383-397",
    "parts": [2, 2], "ngids": [5, 4],
    "lid_to_gid": [[1, 2, 6, 7], [3, 4, 5, 8, 9, 10], [11, 12, 16, 17], [13, 14, 15, 18, 19, 20]],
    "gid_to_part": [1, 1, 2, 2, 2, 1, 1, 2, 2, 2, 3, 3, 4, 4, 4, 3, 3, 4, 4, 4],
}
# :399-424 PCartesianIndices without / with ghost, as (first,last) per dim
K["pcartesian_indices"] = {
    "src": "test/test_interfaces.jl:399-424",
    "no_ghost": [[[1, 2], [1, 2]], [[3, 5], [1, 2]], [[1, 2], [3, 4]], [[3, 5], [3, 4]]],
    "with_ghost": [[[1, 3], [1, 3]], [[2, 5], [1, 3]], [[1, 3], [2, 4]], [[2, 5], [2, 4]]],
}
# :453-467 with_ghost Cartesian PRange (5,4)
K["prange_with_ghost"] = {
    "src": "test/test_interfaces.jl:453-467",
    "lid_to_gid": [[1, 2, 3, 6, 7, 8, 11, 12, 13], [2, 3, 4, 5, 7, 8, 9, 10, 12, 13, 14, 15],
                   [6, 7, 8, 11, 12, 13, 16, 17, 18], [7, 8, 9, 10, 12, 13, 14, 15, 17, 18, 19, 20]],
}
# :469-481 periodic (true,true), (4,4)
K["prange_periodic_tt"] = {
    "src": "test/test_interfaces.jl:469-481",
    "lid_to_gid": [[16, 13, 14, 15, 4, 1, 2, 3, 8, 5, 6, 7, 12, 9, 10, 11],
                   [14, 15, 16, 13, 2, 3, 4, 1, 6, 7, 8, 5, 10, 11, 12, 9],
                   [8, 5, 6, 7, 12, 9, 10, 11, 16, 13, 14, 15, 4, 1, 2, 3],
                   [6, 7, 8, 5, 10, 11, 12, 9, 14, 15, 16, 13, 2, 3, 4, 1]],
}
# :484-496 periodic (false,true), (4,4)
K["prange_periodic_ft"] = {
    "src": "test/test_interfaces.jl:484-496",
    "lid_to_gid": [[13, 14, 15, 1, 2, 3, 5, 6, 7, 9, 10, 11],
                   [14, 15, 16, 2, 3, 4, 6, 7, 8, 10, 11, 12],
                   [5, 6, 7, 9, 10, 11, 13, 14, 15, 1, 2, 3],
                   [6, 7, 8, 10, 11, 12, 14, 15, 16, 2, 3, 4]],
}
# :646-680 diagonal-2 matrix × 3 → 6 (owned; all lids after exchange!);
# fillstored!(A,1) → 3
K["diag_matvec"] = {"src": "test/test_interfaces.jl:646-680", "diag": 2.0, "x": 3.0,
                    "expected": 6.0, "expected_after_fillstored_1": 3.0}
# :686-717 irregular COO matrix; A*x, cg, \ with residual < 1e-9
K["irregular_coo"] = {
    "src": "test/test_interfaces.jl:686-717",
    "n": 10,
    "I": [[1, 2, 1, 2], [3, 3, 4], [5, 5, 6, 7], [9, 9, 8, 10]],
    "J": [[2, 6, 1, 2], [3, 8, 4], [5, 6, 6, 7], [9, 2, 8, 10]],
    "V": [[1.0, 2.0, 30.0, 10.0], [10.0, 2.0, 30.0], [10.0, 2.0, 30.0, 1.0], [10.0, 2.0, 30.0, 50.0]],
    "residual_tol": 1e-9,
}
# SparseUtilsTests.jl:14-56: sparse with duplicates, sub-matrix mul vs dense
K["sparse_utils"] = {
    "src": "test/SparseUtilsTests.jl:14-56",
    "I": [1, 2, 5, 4, 1], "J": [3, 6, 1, 1, 3], "V": [4, 5, 3, 2, 5], "m": 7, "n": 6,
    "rows": [4, 2, 3], "cols": [6, 2, 5, 1],
    "dense_nonzeros": {"1,3": 9, "2,6": 5, "5,1": 3, "4,1": 2},
}
# SparseUtilsTests.jl:62-65: the same test_mat for SparseMatrixCSR{1} and
# {0} (Float64/Int, Float32/Int32): compresscoo(T, I, J, V, m, n) == A, the
# nziterator order equals findnz's (row by row for CSR: the sparsity of A
# above listed row-major), nzindex(B, i, j) == k, the sub-matrix mul! ≈ dense
K["sparse_utils_csr"] = {
    "src": "test/SparseUtilsTests.jl:9-65 (test_mat on SparseMatrixCSR{Bi})",
    "types": [[1, "f64", "i64"], [1, "f32", "i32"], [0, "f64", "i64"], [0, "f32", "i32"]],
    "findnz_order": [[1, 3, 9], [2, 6, 5], [4, 1, 2], [5, 1, 3]],
}
# test_fdm.jl:118 / test_fem_sa.jl:137
K["solvers"] = {"src": "test/test_fdm.jl:118, test/test_fem_sa.jl:137", "err_tol": 1e-5,
                "fdm_nx": 10, "fdm_nnz": 4072}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "interfaces_kats.json")
    with open(out, "w") as f:
        json.dump(K, f, indent=1)
    print("wrote", out)
