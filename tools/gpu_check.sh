# One GPU call: the GPU test suite, then the C2 (FD7 128^3) and default
# (FE27 256^3) bench lines.  Every step has its own time limit; the first
# failure ends the call.   usage: bash tools/gpu_check.sh TAG
set -o pipefail
tag=${1:-check}
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$tag.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline \
  > gpurun_out/bench_c2_$tag.json 2> gpurun_out/bench_c2_$tag.err || exit 2
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default_$tag.json 2> gpurun_out/bench_default_$tag.err || exit 3
