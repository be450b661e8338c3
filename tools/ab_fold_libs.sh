#!/bin/bash
# A/B of library builds on the edge-length fold alone: kernel traces of tools/fold_mesh_probe.py, two
# alternating rounds, then the default build's walk statistics (IMPLISOLID_FOLD_STATS).  A variant
# <v> is implisolid_amd/lib/v_<v>.so (make OBJDIR=build_<v> LIB=lib/v_<v>.so ...); "main" is the default build.
#   usage: tools/ab_fold_libs.sh <tag> [variants...]
set -euo pipefail
export TMPDIR=/tmp
root=$(pwd)
tag=${1:?tag}; shift; vs=${*:-old main}; out=gpurun_out/$tag
mkdir -p $out
for round in 1 2; do
  for v in $vs; do
    if [ "$v" = main ]; then lib=; else lib=$root/implisolid_amd/lib/v_$v.so; fi
    IMPLISOLID_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
        -d "$root/$out/w${v}r$round" -o run -- python3 tools/fold_mesh_probe.py 10 > "$out/w${v}r$round.log" 2>&1
    echo "variant $v round $round done"
  done
done
IMPLISOLID_FOLD_STATS=1 timeout -k 10 200 python3 tools/fold_mesh_probe.py 3 > $out/stats.log 2>&1
