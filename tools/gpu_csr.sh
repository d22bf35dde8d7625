# CSR parents on the device: the new tests, then the parity/COO/driver suites as a regression check.
set -o pipefail
mkdir -p gpurun_out/csr
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_csr.py -x -v --timeout 120 --timeout-method thread > gpurun_out/csr/csr.log 2>&1 || exit 1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coo.py tests/test_gpu_drivers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/csr/regress.log 2>&1 || exit 2
