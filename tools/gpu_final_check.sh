# One GPU call: the whole GPU suite, smoke() and the default bench line, each under its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gpu.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 3
