# One GPU call: the GPU test suite, then the C2 (FD7 128^3) and default
# (FE27 256^3) bench lines and the C5 line (8 Voronoi parts of 128^3 on one
# GPU).  Every step has its own time limit; the first failure ends the call.
#   usage: bash tools/gpu_check.sh TAG
set -o pipefail
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
  > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline \
  > $out/bench_c2.json 2> $out/bench_c2.err || exit 2
timeout -k 10 400 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 3
timeout -k 10 400 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128 --graph \
  > $out/c5.jsonl 2> $out/c5.err || exit 4
timeout -k 10 400 python3 tools/c5_bench.py --patterns 1 --dtypes f64 --group 0 \
  >> $out/c5.jsonl 2>> $out/c5.err || exit 5
