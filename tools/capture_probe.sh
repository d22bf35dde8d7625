# One GPU call: build tools/capture_probe.cpp and run its variants, one process
# each, the ones expected to pass first; a crash ends the chain (the variants
# after it are run by a later call).   usage: bash tools/capture_probe.sh [variants...]
set -o pipefail
out=gpurun_out/capture; mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o /tmp/capture_probe tools/capture_probe.cpp || exit 1
for v in ${@:-0 5 2 3 4 1}; do
  timeout -k 10 60 /tmp/capture_probe $v >> $out/probe.jsonl 2>> $out/probe.err
  rc=$?
  echo "variant $v rc $rc" >> $out/probe.rc
  [ $rc -eq 0 ] || exit 10
done
