#!/bin/bash
# Same-box A/B of config 4s's steady OB02 build at 512^3 (tools/ob02_r512_probe.py 9 --baked: min and
# median of 9 builds of a hot object; AB_RES="256 512" for more resolutions) for the in-tree library ("main") and variants under ab/, rounds
# alternating.   usage: tools/r06_ob02_ab.sh <tag> <rounds> variant ...
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
    for R in ${AB_RES:-512}; do
      IMPLISOLID_LIB=$lib timeout -k 10 240 python3 tools/ob02_r512_probe.py 9 --baked --R $R > "$out/ob02ab_${v}_${R}_$rep.log" 2>&1
      echo "$v $rep $(grep config4s "$out/ob02ab_${v}_${R}_$rep.log")" >> "$out/ob02ab_summary.txt"
    done
  done
done
cat "$out/ob02ab_summary.txt"
