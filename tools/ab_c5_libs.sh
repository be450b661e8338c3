#!/bin/bash
# A/B of library builds on config 5's merged pass (tools/config5_merged_probe.py, 64 objects at
# 128^3, 50 passes), three alternating rounds, then a kernel trace of each.  A variant <v> is
# implisolid_amd/lib/v_<v>.so; "main" is the default build.   usage: tools/ab_c5_libs.sh <tag> [variants...]
set -euo pipefail
export TMPDIR=/tmp
root=$(pwd)
tag=${1:?tag}; shift; vs=${*:-old main}; out=gpurun_out/$tag
mkdir -p $out
for round in 1 2 3; do
  for v in $vs; do
    if [ "$v" = main ]; then lib=; else lib=$root/implisolid_amd/lib/v_$v.so; fi
    IMPLISOLID_LIB=$lib timeout -k 10 200 python3 tools/config5_merged_probe.py 64 128 50 > "$out/c5_${v}_r$round.log" 2>&1
    echo "variant $v round $round: $(tail -1 $out/c5_${v}_r$round.log)"
  done
done
for v in $vs; do
  if [ "$v" = main ]; then lib=; else lib=$root/implisolid_amd/lib/v_$v.so; fi
  IMPLISOLID_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/$out/t_$v" -o run -- \
      python3 tools/config5_merged_probe.py 64 128 20 > "$out/t_$v.log" 2>&1
done
echo done
