#!/bin/bash
# Profiling recipe run on the GPU box (rocprofv3; separate --pmc passes, no
# trace domains beside --pmc).  bench.py's own PMC child passes are switched
# off under the profiler (--no-pmc).
set -o pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--steps 20 --warmup 3 --no-cpu-baseline --no-pmc"}
SHORT="--steps 5 --warmup 1 --no-cpu-baseline --no-pmc"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py $ARGS > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py $SHORT > $OUT/fetch.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py $SHORT > $OUT/write.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum -d $OUT/sq -o sq --output-format csv -- python3 bench.py $SHORT > $OUT/sq.log 2>&1 || exit 4
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/cg -o cg --output-format csv -- python3 bench.py --cg 30 --warmup 3 > $OUT/cg.log 2>&1 || exit 5
