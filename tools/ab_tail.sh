# A/B of the masked tail batch (spmv_flags bit 3) and the unroll over stencil
# kinds, sizes and dtypes (tools/ab_spmv.py: one process per workload,
# interleaved rounds, bits checked equal across variants)
set -o pipefail
V=5:8:1,13:8:1,13:4:1,5:8:0,13:8:0
run() { tag=$1; shift; timeout -k 10 240 python3 tools/ab_spmv.py --rounds 4 --reps 10 --variants $V "$@" > gpurun_out/ab_tail_$tag.txt 2>&1 || exit 1; }
run fd7_128_f64 --n 128 --kind 7
run fd7_256_f64 --n 256 --kind 7
run fd7_256_f32 --n 256 --kind 7 --dtype f32
run fe27_256_f64 --n 256 --kind 27
run fe27_128_f64 --n 128 --kind 27
run fe27_256_f32 --n 256 --kind 27 --dtype f32
run fe27_128_c128 --n 128 --kind 27 --dtype c128
run fd7_128_c128 --n 128 --kind 7 --dtype c128
