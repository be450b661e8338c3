#!/bin/bash
# A/B of library variants (tools/build_variant.sh) on the config-4 bench: usage tools/ab_variants.sh v1 v2 ...
set -e
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --skip-256 --skip-config5 --skip-ob02"
for rep in 1 2; do
  for v in main "$@"; do
    lib=""
    [ "$v" != main ] && lib=variants/$v/implisolid_amd/lib/libimplisolid_mi355x.so
    IMPLISOLID_LIB=$lib timeout -k 10 120 $B > gpurun_out/ab_$v.json 2>/dev/null
    python3 -c "import json;d=json.loads(open('gpurun_out/ab_$v.json').read().splitlines()[-1]);print('$v', d['ms_per_step'], d['kernel_ms'])"
  done
done
