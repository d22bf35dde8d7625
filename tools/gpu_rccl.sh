set -o pipefail
out=gpurun_out/rccl1; mkdir -p $out
NCCL_DEBUG=WARN timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
