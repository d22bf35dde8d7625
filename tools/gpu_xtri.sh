# Lane-shared x runs for triple-pattern slices (spmv_flags bit 9): full GPU suite, interleaved A/B on/off, bench lines.
set -o pipefail
out=gpurun_out/xtri; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu.log 2>&1 || exit 1
for dt in f64 f32 c128 c64; do
  timeout -k 10 240 python3 tools/ab_spmv.py --dtype $dt --rounds 5 --variants 605:8:1,93:8:1 > $out/ab_fe27_$dt.txt 2>&1 || exit 2
done
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $out/bench_default.json 2> $out/bench_default.err || exit 3
