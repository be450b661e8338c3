#!/bin/bash
# the search passes' occupancy request, each variant compiled into its own fresh JIT cache (its
# sources and code objects kept): kernel traces of tools/ob02_probe.py.   usage: tools/ab_ptwaves2.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for w in 0 3; do
    mkdir -p "$out/dump_w$w" "/tmp/jc_${tag}_$w"
    IMPLISOLID_PT_WAVES=$w IMPLISOLID_JIT=1 IMPLISOLID_JIT_CACHE=/tmp/jc_${tag}_$w IMPLISOLID_JIT_DUMP="$root/$out/dump_w$w" \
        timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/w${w}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/w${w}r$round.log" 2>&1
    echo "variant $w round $round done"
  done
done
echo done
