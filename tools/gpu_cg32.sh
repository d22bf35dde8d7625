# CG scalar semantics (Float64 scalars over Float32 vectors), the drivers and parity suites
set -o pipefail
out=gpurun_out/${1:-cg32}; mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_drivers.py tests/test_gpu_parity.py tests/test_gpu_rccl.py -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || exit 1
