#!/bin/bash
# A/B of OB02 build times: the current library vs variants/<name> (tools/build_variant.sh or a git
# archive), alternating, on one box: tools/ab_ob02.sh <tag> <variant>
set -uo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
for rep in 1 2; do
  for v in main "$2"; do
    lib=""
    [ "$v" != main ] && lib=variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 200 python3 tools/ob02_probe.py 7 > "$out/ob02_$v.log" 2>&1 || exit 1
    echo "== $v"; grep "build_geometry" "$out/ob02_$v.log"
  done
done
