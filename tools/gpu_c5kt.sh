# C5 kernel-trace (per-launch timeline of one mul!) for the slice-phase analysis
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-c5kt}; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o kt -- \
  python3 tools/c5_bench.py --patterns 1 --dtypes f64 --steps 20 > $out/c5.jsonl 2> $out/c5.err || exit 1
