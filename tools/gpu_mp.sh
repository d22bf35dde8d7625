set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s4_gpu_all.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/s4_bench_default.json 2> gpurun_out/s4_bench_default.err || exit 2
bash scripts/profile.sh gpurun_out/prof_s4 || exit 3
