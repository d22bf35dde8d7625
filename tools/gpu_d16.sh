# delta16 slices + direct pull: GPU suite, C5 A/B (delta16 x halo_direct), kernel trace
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-d16}; mkdir -p $out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1 || exit 1
for r in 1 2; do
for t in spmv_delta16=1,halo_direct=1 spmv_delta16=0,halo_direct=1 spmv_delta16=1,halo_direct=0 spmv_delta16=0,halo_direct=0; do
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32 --tune $t >> $out/c5_ab.jsonl 2>> $out/c5.err || exit 2
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o kt -- \
  python3 tools/c5_bench.py --patterns 1 --dtypes f64 --steps 20 > $out/c5_kt.jsonl 2> $out/c5_kt.err || exit 3
