#!/bin/bash
# Does a JIT cache populated by the GPU tests give slower point kernels than a fresh compile?
# (1) the OB02 tests into cache A, (2) tools/ob02_probe.py on cache A and on an empty cache B under
# a kernel trace, twice each; cache A's code objects and B's dumps are kept for comparison.
#   usage: tools/jit_cache_ab.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out/cacheA" "$out/dumpB"
export TMPDIR=/tmp
root=$(pwd)
A=/tmp/jcA_$tag
mkdir -p "$A"
IMPLISOLID_JIT_CACHE=$A timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "ob02 or projection" > "$out/tests.log" 2>&1
cp -r "$A"/. "$out/cacheA/"
for round in 1 2; do
  IMPLISOLID_JIT=1 IMPLISOLID_JIT_CACHE=$A timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
      -d "$root/$out/A$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/A$round.log" 2>&1
  B=/tmp/jcB_${tag}_$round
  mkdir -p "$B"
  IMPLISOLID_JIT=1 IMPLISOLID_JIT_CACHE=$B IMPLISOLID_JIT_DUMP="$root/$out/dumpB" timeout -k 10 200 rocprofv3 --kernel-trace \
      --output-format csv -d "$root/$out/B$round" -o run -- python3 tools/ob02_probe.py 3 > "$out/B$round.log" 2>&1
  echo "round $round done"
done
echo done
