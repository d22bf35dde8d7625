# A/B of the merged kernel's occupancy hint (PA_MERGED_WAVES builds), C2 and
# the headline operator, alternating libraries; each step has its own limit
set -o pipefail
out=gpurun_out/waves; mkdir -p $out
L=partitionedarrays.jl_amd
for r in 1 2; do
  for v in def w5 w6; do
    lib=$L/libpa_hip.so; [ $v != def ] && lib=$L/libpa_hip_$v.so
    PA_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 tools/ab_spmv.py --n 128 --kind 7 --copies 5 --variants 93:8:1 --rounds 3 > $out/c2_${v}_$r.txt 2>&1 || exit 1
    PA_HIP_LIB=$PWD/$lib timeout -k 10 120 python3 tools/ab_spmv.py --n 256 --kind 27 --variants 93:8:1 --rounds 3 > $out/fe27_${v}_$r.txt 2>&1 || exit 2
  done
done
