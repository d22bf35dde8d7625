# C5 with 16 B x runs in int32/delta16 slices (spmv_flags bit 7: 93 -> 221), interleaved 3 times, all dtypes.
set -o pipefail
out=gpurun_out/xrunc5; mkdir -p $out
for rnd in 1 2 3; do
  for fl in 93 221; do
    timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 --tune spmv_flags=$fl > $out/c5_${fl}_$rnd.jsonl 2> $out/c5_${fl}_$rnd.err || exit 1
  done
done
