#!/bin/bash
# the search passes' occupancy request (IMPLISOLID_PT_WAVES 0 / 4 / 5) on baked point modules
# (IMPLISOLID_JIT_BAKE=1): kernel traces of tools/ob02_r512_probe.py and tools/ob02_probe.py, two
# alternating rounds, fresh JIT caches.   usage: tools/ab_ptwaves_baked.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for w in 0 4 5; do
    c=/tmp/jc_${tag}_$w
    mkdir -p "$c"
    IMPLISOLID_JIT_BAKE=1 IMPLISOLID_PT_WAVES=$w IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/w${w}r${round}_512" -o run -- python3 tools/ob02_r512_probe.py 3 > "$out/w${w}r${round}_512.log" 2>&1
    IMPLISOLID_JIT_BAKE=1 IMPLISOLID_PT_WAVES=$w IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/w${w}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/w${w}r$round.log" 2>&1
    echo "variant $w round $round done"
  done
done
echo done
