#!/bin/bash
# A/B of baked point modules (IMPLISOLID_JIT_BAKE=1: every module with its matrices as literals)
# against unbaked ones (0): kernel traces of tools/ob02_probe.py and tools/ob02_r512_probe.py, two
# alternating rounds, fresh JIT caches.   usage: tools/ab_ptbake.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for b in 0 1; do
    c=/tmp/jc_${tag}_$b
    mkdir -p "$c"
    IMPLISOLID_JIT_BAKE=$b IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/b${b}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/b${b}r$round.log" 2>&1
    IMPLISOLID_JIT_BAKE=$b IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/b${b}r${round}_512" -o run -- python3 tools/ob02_r512_probe.py 3 > "$out/b${b}r${round}_512.log" 2>&1
    echo "variant $b round $round done"
  done
done
echo done
