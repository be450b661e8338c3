#!/bin/bash
# config-5 merged pass under interpreter knobs (pair / stack-depth floor): tools/c5_knobs.sh <tag>
set -uo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
for v in "" "IMPLISOLID_INTERP_PAIR=0" "IMPLISOLID_EVAL_DEPTH=8" "IMPLISOLID_EVAL_DEPTH=8 IMPLISOLID_INTERP_PAIR=0" "IMPLISOLID_EVAL_DEPTH=16"; do
  echo "== $v" >> "$out/c5_knobs.log"
  env $v timeout -k 10 120 python3 tools/config5_merged_probe.py 64 128 20 >> "$out/c5_knobs.log" 2>&1 || exit 1
done
cat "$out/c5_knobs.log"
