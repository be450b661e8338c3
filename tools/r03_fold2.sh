#!/bin/bash
set -euo pipefail
out=gpurun_out/${1:?tag}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fold or ob02 or headline or sharded" > "$out/tests.log" 2>&1
tail -1 "$out/tests.log"
IMPLISOLID_FOLD_STATS=1 timeout -k 10 120 python3 tools/fold_probe.py > "$out/fold.log" 2>&1
grep "^fold n=340000\|^fold n=1000000" "$out/fold.log" | head -2
timeout -k 10 200 python3 tools/ob02_probe.py 5 > "$out/ob02.log" 2>&1
grep -v amdgpu.ids "$out/ob02.log" | head -6
