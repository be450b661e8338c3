#!/bin/bash
# config-5 merged pass: the deep class's stream at the lowest priority (default) against the default
# priority (IMPLISOLID_BATCH_DEEP_PRIO=0), three alternating rounds.   usage: tools/c5_prio_ab.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
for rep in 1 2 3; do
  for v in 1 0; do
    echo -n "prio_low=$v $rep " >> "$out/c5_prio.txt"
    IMPLISOLID_BATCH_DEEP_PRIO=$v timeout -k 10 120 python3 tools/config5_merged_probe.py 64 128 20 2>/dev/null | grep merged >> "$out/c5_prio.txt"
  done
done
cat "$out/c5_prio.txt"
