set -o pipefail
out=gpurun_out/r02f; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_spmv.py --n 128 --kind 7 --copies 5 --variants 93:8:1,29:8:1,93:8:0,29:8:0 --rounds 5 --reps 20 > $out/ab_c2_f64.txt 2>&1 || exit 2
timeout -k 10 300 python3 tools/ab_spmv.py --n 128 --kind 7 --copies 5 --dtype f32 --variants 93:8:1,29:8:1 --rounds 5 --reps 20 > $out/ab_c2_f32.txt 2>&1 || exit 3
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || exit 4
