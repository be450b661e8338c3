#!/bin/bash
# A/B of the early projection pass: the two-loop form (IMPLISOLID_EARLY_SM=0) against the single
# loop with chunks of 64 and 32 faces per wave; kernel traces of tools/ob02_probe.py and
# tools/ob02_r512_probe.py, two alternating rounds, each variant in its own fresh JIT cache.
#   usage: tools/ab_early.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for v in 0:64 1:64 1:32; do
    sm=${v%:*}; ch=${v#*:}
    c=/tmp/jc_${tag}_${sm}_$ch
    mkdir -p "$c"
    IMPLISOLID_EARLY_SM=$sm IMPLISOLID_EARLY_CHUNK=$ch IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/s${sm}c${ch}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/s${sm}c${ch}r$round.log" 2>&1
    IMPLISOLID_EARLY_SM=$sm IMPLISOLID_EARLY_CHUNK=$ch IMPLISOLID_JIT_CACHE=$c timeout -k 10 200 rocprofv3 --kernel-trace \
        --output-format csv -d "$root/$out/s${sm}c${ch}r${round}_512" -o run -- python3 tools/ob02_r512_probe.py 3 > "$out/s${sm}c${ch}r${round}_512.log" 2>&1
    echo "variant $v round $round done"
  done
done
echo done
