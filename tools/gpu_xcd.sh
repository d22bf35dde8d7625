# XCD remap A/B on the merged kernel: FE27 256^3, C2 FD7 128^3 (5 copies), C5
set -o pipefail
out=gpurun_out/${1:-xcd}; mkdir -p $out
timeout -k 10 300 python3 tools/ab_spmv.py --variants 93:8:1,95:8:1 --rounds 6 --reps 10 > $out/ab_fe27.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_spmv.py --n 128 --kind 7 --copies 5 --variants 93:8:1,95:8:1 --rounds 6 --reps 20 > $out/ab_c2.txt 2>&1 || exit 2
for r in 1 2; do for f in 93 95; do
timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32 --tune spmv_flags=$f >> $out/c5.jsonl 2>> $out/c5.err || exit 3
done; done
timeout -k 10 120 python3 -c "import sys; sys.path.insert(0,'.'); import pamd; print(pamd._lib.hbm_probe(0, 2<<30, 10))" > $out/probe.txt 2>&1 || exit 4
