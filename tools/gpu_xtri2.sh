# Triple-pattern x sharing with the per-slice flag precomputed: A/B on/off first (quick), then the GPU suite.
set -o pipefail
out=gpurun_out/xtri2; mkdir -p $out
for dt in f64 f32; do
  timeout -k 10 240 python3 tools/ab_spmv.py --dtype $dt --rounds 5 --variants 605:8:1,93:8:1 > $out/ab_fe27_$dt.txt 2>&1 || exit 2
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu.log 2>&1 || exit 1
