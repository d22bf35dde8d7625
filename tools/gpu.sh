#!/bin/bash
# One gpurun call's recipe, run on the GPU box from the repo root:
#
#   tools/gpu.sh OUT STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failure ends
# the call (no GPU step after a fault, a timeout or an abort).  A step is
# "name" or "name:arguments":
#   tests[:pytest args]   python -m pytest tests -m gpu (e.g. "tests:-k fullsize", "tests:-k 'cg or dot'")
#   smoke                 __graft_entry__.smoke()
#   bench[:bench args]    python bench.py ARGS            > OUT/bench<i>.json
#   kt[:bench args]       rocprofv3 --kernel-trace --stats  -d OUT/kt<i>
#   ktpy:script args      rocprofv3 --kernel-trace --stats of python3 script args  -d OUT/kt<i>
#   pmc:CTR[,CTR..][:bench args]  rocprofv3 --pmc CTR..     -d OUT/pmc<i>
#   pmcpy:CTR[,CTR..]:script args  rocprofv3 --kernel-trace --pmc CTR.. of python3 script args
#   py:script args        python script args              > OUT/py<i>.log
#   cmd:program args      a host program (no GPU), e.g. the C port   > OUT/cmd<i>.log
# Profiled runs default to "--steps 10 --warmup 2 --no-cpu-baseline --no-pmc".
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PROF_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pmc"
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%:*}
  args=""
  [[ "$step" == *:* ]] && args=${step#*:}
  echo "== step $i: $name $args" | tee -a "$OUT/steps.log"
  t0=$(date +%s)
  case $name in
    tests)
      # eval: a quoted -k expression ("tests:-k 'cg or dot'") stays one argument
      eval "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $args" \
        > "$OUT/tests$i.log" 2>&1
      rc=$?; tail -3 "$OUT/tests$i.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke$i.log" 2>&1
      rc=$?; tail -2 "$OUT/smoke$i.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py $args > "$OUT/bench$i.json" 2> "$OUT/bench$i.err"
      rc=$?; cat "$OUT/bench$i.json" | cut -c1-400 ;;
    kt)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt$i" -o kt --output-format csv \
        -- python3 bench.py ${args:-$PROF_ARGS} > "$OUT/kt$i.log" 2>&1
      rc=$? ;;
    ktpy)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/kt$i" -o kt --output-format csv \
        -- python3 $args > "$OUT/kt$i.log" 2>&1
      rc=$? ;;
    pmc)
      ctr=${args%%:*}
      bargs=""
      [[ "$args" == *:* ]] && bargs=${args#*:}
      timeout -s KILL 240 rocprofv3 --pmc ${ctr//,/ } -d "$OUT/pmc$i" -o pmc --output-format csv \
        -- python3 bench.py ${bargs:-$PROF_ARGS} > "$OUT/pmc$i.log" 2>&1
      rc=$? ;;
    pmcpy)
      ctr=${args%%:*}
      sargs=${args#*:}
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc ${ctr//,/ } -d "$OUT/pmc$i" -o pmc --output-format csv \
        -- python3 $sargs > "$OUT/pmc$i.log" 2>&1
      rc=$? ;;
    py)
      timeout -k 10 600 python -u $args > "$OUT/py$i.log" 2>&1
      rc=$?; tail -5 "$OUT/py$i.log" ;;
    cmd)
      timeout -k 10 600 $args > "$OUT/cmd$i.log" 2>&1
      rc=$?; tail -c 600 "$OUT/cmd$i.log" ;;
    *)
      echo "unknown step $name"; exit 2 ;;
  esac
  case $name in kt|ktpy|pmc|pmcpy) python3 tools/prune_prof.py "$OUT/kt$i" "$OUT/pmc$i" ;; esac
  echo "   rc $rc, $(( $(date +%s) - t0 )) s" | tee -a "$OUT/steps.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
