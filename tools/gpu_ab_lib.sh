# Same-box A/B of two library builds (PA_HIP_LIB): tools/ab_libs/base.so (the committed tree) vs the working tree's
# libpa_hip.so, interleaved three times (order alternating): FE27 256^3 F64 and F32 bench lines, C2, C5 (4 dtypes).
set -o pipefail
out=gpurun_out/ablib; mkdir -p $out
for rnd in 1 2 3; do
  order="base new"; [ $rnd = 2 ] && order="new base"   # alternate the order against the box's drift
  for lib in $order; do
    if [ $lib = base ]; then L=$PWD/tools/ab_libs/base.so; else L=$PWD/partitionedarrays.jl_amd/libpa_hip.so; fi
    PA_HIP_LIB=$L timeout -k 10 300 python3 bench.py --steps 50 --no-cpu-baseline --no-pmc > $out/fe27_${lib}_$rnd.json 2> $out/fe27_${lib}_$rnd.err || exit 1
    PA_HIP_LIB=$L timeout -k 10 300 python3 bench.py --dtype f32 --steps 50 --no-cpu-baseline --no-pmc > $out/fe27f32_${lib}_$rnd.json 2> $out/fe27f32_${lib}_$rnd.err || exit 1
    PA_HIP_LIB=$L timeout -k 10 300 python3 bench.py --n 128 --kind 7 --steps 50 --no-cpu-baseline --no-pmc > $out/c2_${lib}_$rnd.json 2> $out/c2_${lib}_$rnd.err || exit 2
    PA_HIP_LIB=$L timeout -k 10 300 python3 tools/c5_bench.py --patterns 1 --dtypes f64,f32,c128,c64 > $out/c5_${lib}_$rnd.jsonl 2> $out/c5_${lib}_$rnd.err || exit 3
  done
done
