# XRUN (16 B x runs in int32/delta16 slices) A/B: C5 all dtypes, FE27 int32 encoding; bit-exactness in ab_spmv
set -o pipefail
out=gpurun_out/${1:-xrun}; mkdir -p $out
for r in 1 2; do for f in 93 221; do
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 --tune spmv_flags=$f >> $out/c5.jsonl 2>> $out/c5.err || exit 1
done; done
timeout -k 10 300 python3 tools/ab_spmv.py --variants 93:8:0,221:8:0,93:8:1,221:8:1 --rounds 4 --reps 8 > $out/ab_fe27.txt 2>&1 || exit 2
timeout -k 10 300 python3 tools/ab_spmv.py --dtype f32 --variants 93:8:0,221:8:0 --rounds 4 --reps 8 > $out/ab_fe27_f32.txt 2>&1 || exit 3
