#!/bin/bash
# Which compiles give the LDS-promoted point modules?  C: tools/ob02_probe.py with the default
# background JIT into a fresh cache; D: the OB02 GPU tests into a fresh cache; both dumped.
#   usage: tools/jit_cache_ab2.sh <tag>
set -euo pipefail
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out/dumpC" "$out/dumpD"
export TMPDIR=/tmp
root=$(pwd)
C=/tmp/jcC_$tag; D=/tmp/jcD_$tag
mkdir -p "$C" "$D"
IMPLISOLID_JIT_CACHE=$C IMPLISOLID_JIT_DUMP="$root/$out/dumpC" timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv \
    -d "$root/$out/C" -o run -- python3 tools/ob02_probe.py 3 > "$out/C.log" 2>&1
echo "C done"
IMPLISOLID_JIT_CACHE=$D IMPLISOLID_JIT_DUMP="$root/$out/dumpD" timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "ob02_point_jit or config3_shifted_projection_live" > "$out/testsD.log" 2>&1
echo "D done"
