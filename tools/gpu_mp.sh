set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread > gpurun_out/fullsize.log 2>&1 || exit 1
