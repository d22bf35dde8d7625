# CG (BASELINE config 4, FE27 256^3 one part): bench line, then a kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/cgprof; mkdir -p $out
timeout -k 10 300 python3 bench.py --cg 20 --warmup 3 --no-pmc --no-cpu-baseline > $out/bench_cg.json 2> $out/bench_cg.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_cg -o kt -- \
  python3 bench.py --cg 20 --warmup 3 --no-pmc --no-cpu-baseline > $out/bench_cg_under_kt.json 2> $out/kt_cg.err || exit 2
