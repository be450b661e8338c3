#!/bin/bash
# Same-box A/B of the headline (512^3, no side legs): the in-tree library ("main") and each variant,
# rounds alternating.  A variant is either a library built by VARIANTS=ab tools/build_variant.sh
# (ab/<name>/...) or "env:NAME=VALUE" (the in-tree library with that environment variable set).
#   usage: tools/r06_ab.sh <tag> <rounds> variant ...
set -euo pipefail
tag=${1:?tag}; rounds=${2:?rounds}; shift 2
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
root=$(pwd)
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02 --skip-concurrent"
for rep in $(seq 1 "$rounds"); do
  for v in main "$@"; do
    lib=""; envs=""; name=$v
    case "$v" in
      main) ;;
      env:*) envs=${v#env:}; name=$(echo "$envs" | tr '=' '_') ;;
      *) lib=$root/ab/$v/implisolid_amd/lib/libimplisolid_mi355x.so ;;
    esac
    env IMPLISOLID_LIB=$lib $envs timeout -k 10 200 $B > "$out/ab_${name}_$rep.json" 2> "$out/ab_${name}_$rep.err"
    python3 -c "import json;d=json.loads(open('$out/ab_${name}_$rep.json').read().splitlines()[-1]);print('$name', $rep, d['ms_per_step'], json.dumps({k: round(x * 1e3, 1) for k, x in d['kernel_ms_each'].items()}))" >> "$out/ab_summary.txt"
  done
done
cat "$out/ab_summary.txt"
echo done
