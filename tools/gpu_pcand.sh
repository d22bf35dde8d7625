# pattern candidates: C2 per dtype (format stats + time), then the GPU suite
set -e
mkdir -p gpurun_out/pcand
for d in f32 f64 c64 c128; do
  timeout -k 10 120 python -u tools/ab_spmv.py --n 128 --kind 7 --dtype $d --copies 5 --variants 93:8:1 > gpurun_out/pcand/c2_$d.txt 2>&1
done
timeout -k 10 120 python -u tools/ab_spmv.py --n 256 --kind 27 --dtype f32 --copies 1 --variants 93:8:1 > gpurun_out/pcand/fe27_f32.txt 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pcand/tests.log 2>&1
