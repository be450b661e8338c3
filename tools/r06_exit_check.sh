#!/bin/bash
# The exit-with-compiles-in-flight test, repeated (a process that exits right after its first build,
# its tree modules compiling on the JIT workers, must exit promptly): each run under its own limit,
# the first failure ends it.   usage: tools/r06_exit_check.sh <tag> <runs>
set -euo pipefail
tag=${1:?tag}; runs=${2:?runs}
out=gpurun_out/$tag
mkdir -p "$out"
for i in $(seq 1 "$runs"); do
  t0=$(date +%s.%N)
  timeout -k 10 200 python3 -u -m pytest tests -m gpu -x -q --timeout 180 -k test_exit_with_compiles_in_flight \
      > "$out/exit_check_$i.log" 2>&1
  echo "run $i ok $(python3 -c "print(round($(date +%s.%N) - $t0, 1))") s" >> "$out/exit_check.txt"
done
cat "$out/exit_check.txt"
