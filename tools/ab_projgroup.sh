#!/bin/bash
# A/B of the searches' lanes per face (IMPLISOLID_PROJ_GROUP 2 / 4 / 8) on baked point modules: kernel
# traces of tools/ob02_r512_probe.py and tools/ob02_probe.py, two alternating rounds, fresh JIT caches.
#   usage: tools/ab_projgroup.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for g in 4 2 8; do
    c=/tmp/jc_${tag}_$g
    mkdir -p "$c"
    IMPLISOLID_JIT_BAKE=1 IMPLISOLID_PROJ_GROUP=$g IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/g${g}r${round}_512" -o run -- python3 tools/ob02_r512_probe.py 3 > "$out/g${g}r${round}_512.log" 2>&1
    IMPLISOLID_JIT_BAKE=1 IMPLISOLID_PROJ_GROUP=$g IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/g${g}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/g${g}r$round.log" 2>&1
    echo "variant $g round $round done"
  done
done
echo done
