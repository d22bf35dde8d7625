# Final-state profile set of the round: bench lines (default FE27 256^3 with
# PMC, C2 FD7 128^3 with PMC, CG), rocprofv3 --kernel-trace --stats of the
# same commands, C5 line + trace.  Each step has its own limit; the first
# failure ends the call.   usage: bash tools/profile_final.sh TAG
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-final}; mkdir -p $out
timeout -k 10 400 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_default -o kt -- \
  python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $out/bench_default_under_kt.json 2> $out/kt_default.err || exit 2
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_c2 -o kt -- \
  python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > $out/bench_c2_under_kt.json 2> $out/kt_c2.err || exit 4
timeout -k 10 400 python3 bench.py --cg 20 --warmup 3 --no-pmc --no-cpu-baseline > $out/bench_cg.json 2> $out/bench_cg.err || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_c5 -o kt -- \
  python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32 > $out/c5_under_kt.jsonl 2> $out/kt_c5.err || exit 6
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 > $out/c5.jsonl 2> $out/c5.err || exit 7
