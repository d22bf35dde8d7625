# Global-typed merged-launch arguments (global_load / s_load instead of flat_load) + triple x sharing A/B.
set -o pipefail
out=gpurun_out/glb; mkdir -p $out
for dt in f64 f32 c128 c64; do
  timeout -k 10 240 python3 tools/ab_spmv.py --dtype $dt --rounds 5 --variants 605:8:1,93:8:1 > $out/ab_fe27_$dt.txt 2>&1 || exit 2
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > $out/bench_default.json 2> $out/bench_default.err || exit 3
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline --no-pmc > $out/bench_c2.json 2> $out/bench_c2.err || exit 4
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 > $out/c5.jsonl 2> $out/c5.err || exit 5
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu.log 2>&1 || exit 1
