#!/bin/bash
# round-4 evidence run (one gpurun call): the -m gpu suite, then the per-slab kernel trace of
# tools/slab_probe.py (512^3, balanced cuts for 1/2/4/8 slabs) summarised by tools/slab_trace.py.
#   usage: tools/r04_run.sh <tag> [tests|trace|all]
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
tag=${1:?tag}
what=${2:-all}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
if [ "$what" = tests ] || [ "$what" = all ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1
  cp "$out/tests.log" profiles/${tag}_gpu_tests.log
fi
if [ "$what" = trace ] || [ "$what" = all ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/$out/slab" -o run -- \
      python3 tools/slab_probe.py 512 10 1,2,4,8 balanced > "$out/slab_probe.json" 2> "$out/slab_probe.err"
  python3 tools/slab_trace.py "$out/slab/run_kernel_trace.csv" 10 1,2,4,8 > "$out/slab_trace_summary.txt"
  cp "$out/slab_trace_summary.txt" profiles/${tag}_slab_trace_summary.txt
  cp "$out/slab_probe.json" profiles/${tag}_slab_probe_512.json
fi
echo done
