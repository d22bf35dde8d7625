# RCCL transport on one GPU: its tests, then C5 timed with the halo over RCCL
# (self-sends between the parts of the device) next to the device-read pull.
set -o pipefail
out=gpurun_out/${1:-rccl}; mkdir -p $out
NCCL_DEBUG=WARN timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64 --rccl > $out/c5_rccl.jsonl 2> $out/c5_rccl.err || exit 2
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64 > $out/c5_pull.jsonl 2> $out/c5_pull.err || exit 3
