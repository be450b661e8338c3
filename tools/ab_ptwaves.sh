#!/bin/bash
# A/B of the search passes' occupancy request (IMPLISOLID_PT_WAVES): each variant's kernel trace of
# tools/ob02_probe.py plus tools/proj_stats_probe.py's 512^3 build, two alternating rounds.
#   usage: tools/ab_ptwaves.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for w in 0 3 4; do
    IMPLISOLID_PT_WAVES=$w IMPLISOLID_JIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/w${w}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/w${w}r$round.log" 2>&1
    echo "variant $w round $round done"
  done
done
echo done
