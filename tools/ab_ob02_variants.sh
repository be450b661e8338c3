#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the OB02 probe, two alternating rounds, then
# the OB02 GPU tests on each variant: usage tools/ab_ob02_variants.sh <tag> v1 v2 ...
set -euo pipefail
out=gpurun_out/${1:?tag}; shift
mkdir -p "$out"
for rep in 1 2; do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 200 python3 tools/ob02_probe.py 5 > "$out/probe_${v}_$rep.log" 2>&1
    echo "$v rep=$rep"; grep "MC+3xOB02" "$out/probe_${v}_$rep.log" | grep build_geometry
  done
done
for v in "$@"; do
  IMPLISOLID_LIB=variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q \
      --timeout 240 --timeout-method thread -k "ob02 or projection or config3 or config2 or point" > "$out/tests_$v.log" 2>&1
  echo "$v tests: $(tail -1 "$out/tests_$v.log")"
done
