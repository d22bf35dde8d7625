# phase-merged per-part path: GPU suite, C5 + overlap traces (pull and RCCL modes), bench lines
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-merge2}; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/ov_rccl -o ov -- \
  python3 tools/halo_overlap.py run --n 128 --mode rccl > $out/ov_rccl.out 2>&1 || exit 2
python3 tools/halo_overlap.py analyze $out/ov_rccl > $out/overlap_rccl.json || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/ov_pull -o ov -- \
  python3 tools/halo_overlap.py run --n 128 --mode pull > $out/ov_pull.out 2>&1 || exit 4
python3 tools/halo_overlap.py analyze $out/ov_pull > $out/overlap_pull.json || exit 5
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 --graph > $out/c5.jsonl 2> $out/c5.err || exit 6
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64 --rccl > $out/c5_rccl.jsonl 2> $out/c5_rccl.err || exit 7
timeout -k 10 400 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 8
