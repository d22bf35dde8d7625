# device COO assembly: its tests, the RCCL variant, and the fem_sa drivers
set -o pipefail
out=gpurun_out/${1:-coo}; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coo_assemble.py tests/test_gpu_rccl.py tests/test_gpu_drivers.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
