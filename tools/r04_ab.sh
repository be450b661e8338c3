#!/bin/bash
# Same-box A/B of the current library against variants (tools/build_variant.sh): for each, the
# config-4 bench headline (512^3, no side legs) twice, alternating, and the per-slab kernel trace of
# tools/slab_probe.py 512 at 1 and 8 balanced slabs (tools/slab_trace.py).
#   usage: tools/r04_ab.sh <tag> variant ...
set -euo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --skip-concurrent"
for rep in 1 2; do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=$root/variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 200 $B > "$out/ab_${v}_$rep.json" 2> "$out/ab_${v}_$rep.err"
    python3 -c "import json;d=json.loads(open('$out/ab_${v}_$rep.json').read().splitlines()[-1]);print('$v', $rep, d['ms_per_step'], d['kernel_ms_each'])" >> "$out/ab_summary.txt"
  done
done
for v in main "$@"; do
  lib=""
  [ "$v" != main ] && lib=$root/variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
  IMPLISOLID_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$root/$out/slab_$v" -o run -- \
      python3 tools/slab_probe.py 512 10 1,8 balanced > "$out/slab_probe_$v.json" 2> "$out/slab_probe_$v.err"
  python3 tools/slab_trace.py "$out/slab_$v/run_kernel_trace.csv" 10 1,8 > "$out/slab_trace_$v.txt"
done
cat "$out/ab_summary.txt"
echo done
