set -o pipefail
out=gpurun_out/var1; mkdir -p $out
for r in 1 2; do
timeout -k 10 300 python3 bench.py --no-pmc --no-cpu-baseline > $out/b_default_$r.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-pmc --no-cpu-baseline --steps 400 --warmup 200 > $out/b_long_$r.json 2>/dev/null || exit 2
done
rocm-smi --showclocks --showpower --showtemp > $out/smi.txt 2>&1 || true
