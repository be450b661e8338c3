#!/bin/bash
# A/B of the late projection pass's group widths (IMPLISOLID_LATE_WMAX, IMPLISOLID_LATE_FLAT): each
# variant's kernel trace of tools/ob02_probe.py, two alternating rounds.   usage: tools/ab_late.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
for round in 1 2; do
  for v in 4:0 16:1 64:1 64:0; do
    w=${v%:*}; f=${v#*:}
    IMPLISOLID_LATE_WMAX=$w IMPLISOLID_LATE_FLAT=$f timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/w${w}f${f}r$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/w${w}f${f}r$round.log" 2>&1
    echo "variant $v round $round done"
  done
done
echo done
