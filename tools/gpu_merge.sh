# merged launch: GPU suite, C5 A/B (spmv_merge), C2 and default bench lines, C5 kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-merge}; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
for r in 1 2; do
for t in spmv_merge=1 spmv_merge=0; do
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128 --tune $t >> $out/c5_ab.jsonl 2>> $out/c5.err || exit 2
done
done
timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --warmup 5 --no-cpu-baseline > $out/bench_c2.json 2> $out/bench_c2.err || exit 3
timeout -k 10 400 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o kt -- \
  python3 tools/c5_bench.py --patterns 1 --dtypes f64 --steps 20 > $out/c5_kt.jsonl 2> $out/c5_kt.err || exit 5
