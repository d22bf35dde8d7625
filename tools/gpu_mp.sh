set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/ab_spmv.py --n 256 --kind 27 --variants 13:8:1,29:8:1 --rounds 6 > gpurun_out/ab_idlist_fe27.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_spmv.py --n 256 --kind 7 --variants 13:8:1,29:8:1 --rounds 6 > gpurun_out/ab_idlist_fd7.txt 2>&1 || exit 2
