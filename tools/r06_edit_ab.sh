#!/bin/bash
# Same-box A/B of a new object's builds (tools/first_build_probe.py: first build, edits on the
# unbaked modules, steady state) for the in-tree library ("main") and variants under ab/, rounds
# alternating.   usage: tools/r06_edit_ab.sh <tag> <rounds> variant ...
set -euo pipefail
tag=${1:?tag}; rounds=${2:?rounds}; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for rep in $(seq 1 "$rounds"); do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=$root/ab/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 240 python3 tools/first_build_probe.py > "$out/edit_${v}_$rep.json" 2> "$out/edit_${v}_$rep.err"
    python3 -c "import json;d=json.loads(open('$out/edit_${v}_$rep.json').read().splitlines()[-1]);print('$v', $rep, {k: d.get(k) for k in ('first_build_ms','edit_build_ms','profiled_first_build_ms','steady_ms')}, 'project', d['profiled_first_stats']['stage_ms']['project'])" >> "$out/edit_summary.txt"
  done
done
cat "$out/edit_summary.txt"
