# Session-3 final state: full GPU suite, smoke, then the profile set (tools/profile_final.sh) into gpurun_out/fin4.
set -o pipefail
mkdir -p gpurun_out/fin4
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin4/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin4/smoke.log 2>&1 || exit 2
bash tools/profile_final.sh fin4 || exit 3
