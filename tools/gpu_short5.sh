# after k_spmv_merged_short: C2 (F64, F32) and headline timings, then the GPU suite
set -o pipefail
out=gpurun_out/short5; mkdir -p $out
timeout -k 10 120 python3 tools/ab_spmv.py --n 128 --kind 7 --copies 5 --variants 93:8:1 --rounds 5 > $out/c2_f64.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/ab_spmv.py --n 128 --kind 7 --dtype f32 --copies 5 --variants 93:8:1 --rounds 5 > $out/c2_f32.txt 2>&1 || exit 2
timeout -k 10 120 python3 tools/ab_spmv.py --n 256 --kind 27 --variants 93:8:1 --rounds 3 > $out/fe27.txt 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || exit 4
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || exit 5
