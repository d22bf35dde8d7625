# Session-3 check of the rebuilt tree: GPU suite, smoke, default bench, stream probe.
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s3/gpu.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s3/smoke.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err || exit 3
timeout -k 10 120 ./tools/probe_stream 131072 10 > gpurun_out/s3/probe_stream.jsonl 2>&1 || exit 4
