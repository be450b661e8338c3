#!/bin/bash
# Same-box A/B, bench headline only (512^3, no side legs): the current library and each variant
# (tools/build_variant.sh), three rounds alternating.   usage: tools/r04_ab_fast.sh <tag> variant ...
set -euo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --skip-concurrent"
for rep in 1 2 3; do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=$root/variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 200 $B > "$out/ab_${v}_$rep.json" 2> "$out/ab_${v}_$rep.err"
    python3 -c "import json;d=json.loads(open('$out/ab_${v}_$rep.json').read().splitlines()[-1]);print('$v', $rep, d['ms_per_step'], d['kernel_ms_each'])" >> "$out/ab_summary.txt"
  done
done
cat "$out/ab_summary.txt"
echo done
