#!/bin/bash
# config-5 merged pass: the current library against variants (tools/build_variant.sh), three rounds
# alternating: tools/c5_ab.sh <tag> variant ...
set -euo pipefail
tag=${1:?tag}; shift
out=gpurun_out/$tag
mkdir -p "$out"
root=$(pwd)
for rep in 1 2 3; do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=$root/variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    echo -n "$v $rep " >> "$out/c5_ab.txt"
    IMPLISOLID_LIB=$lib timeout -k 10 120 python3 tools/config5_merged_probe.py 64 128 20 2>/dev/null | grep merged >> "$out/c5_ab.txt"
  done
done
cat "$out/c5_ab.txt"
